# Q4_1 / Q4_0 decode matvec check: parity subset, then 13B Q4_1 decode speed per launch
# shape (sweep build, LVK_CFG41) and the 7B Q4_0 decode speed
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "q4_1 or mul_mat" tests/test_gpu_model.py::test_q4_1_shaped_decode_vs_oracle > gpurun_out/t_q41.log 2>&1 || { tail -30 gpurun_out/t_q41.log; exit 1; }
tail -3 gpurun_out/t_q41.log
timeout -k 10 300 python -u tools/decode_speed.py 13b 64 > gpurun_out/sp13.log 2>&1 || exit 2
for c in 1 2 3; do LVK_LIB=$PWD/llama.vk_amd/lib/sweep/libllama_vk_amd.so LVK_CFG41=$c timeout -k 10 200 python -u tools/decode_speed.py 13b 64 >> gpurun_out/sp13.log 2>&1 || exit 3; done
timeout -k 10 300 python -u tools/decode_speed.py 7b 128 >> gpurun_out/sp13.log 2>&1 || exit 4
cat gpurun_out/sp13.log | grep model
