# Q4_1 prompt matmul variants: 13B Q4_1 512-token prompt per build (equal hashes = same bits)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prompt_speed.py 512 13b > gpurun_out/pd41.log 2>&1 || { tail -20 gpurun_out/pd41.log; exit 2; }
for v in mm41_3_2_0_6 mm41_3_2_0_10 mm41_3_2_1_10; do
  echo "$v" >> gpurun_out/pd41.log
  LVK_LIB=$PWD/llama.vk_amd/lib/$v/libllama_vk_amd.so timeout -k 10 200 python -u tools/prompt_speed.py 512 13b >> gpurun_out/pd41.log 2>&1 || { tail -20 gpurun_out/pd41.log; exit 3; }
done
grep -v "^llama\|kv self" gpurun_out/pd41.log
