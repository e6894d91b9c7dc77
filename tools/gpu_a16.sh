# prompt-matmul A16 check: MFMA op + model parity (both A sources), then the 7B 512-token
# prompt time with and without the f16 A images (and the mmprobe build: 4 B blocks in flight)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py -k "mfma" > gpurun_out/t_a16.log 2>&1 || { tail -30 gpurun_out/t_a16.log; exit 1; }
tail -3 gpurun_out/t_a16.log
timeout -k 10 300 python -u tools/prompt_speed.py > gpurun_out/p_a16.log 2>&1 || { tail -20 gpurun_out/p_a16.log; exit 2; }
LVK_PROMPT_A16=0 timeout -k 10 300 python -u tools/prompt_speed.py >> gpurun_out/p_a16.log 2>&1 || { tail -20 gpurun_out/p_a16.log; exit 3; }
LVK_LIB=$PWD/llama.vk_amd/lib/mmprobe/libllama_vk_amd.so timeout -k 10 300 python -u tools/prompt_speed.py >> gpurun_out/p_a16.log 2>&1 || { tail -20 gpurun_out/p_a16.log; exit 4; }
grep -v "^llama" gpurun_out/p_a16.log | tail -20
