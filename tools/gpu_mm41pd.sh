# Q4_1 prompt matmul ring depth: 13B Q4_1 512-token prompt per LVK_MM41_PD build (equal hashes = same bits)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prompt_speed.py 512 13b > gpurun_out/pd41.log 2>&1 || { tail -20 gpurun_out/pd41.log; exit 2; }
for pd in 1 3 4; do
  LVK_LIB=$PWD/llama.vk_amd/lib/mm41pd$pd/libllama_vk_amd.so timeout -k 10 200 python -u tools/prompt_speed.py 512 13b >> gpurun_out/pd41.log 2>&1 || { tail -20 gpurun_out/pd41.log; exit 3; }
done
grep model gpurun_out/pd41.log
