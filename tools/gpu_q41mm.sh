# Q4_1 MFMA prompt path: op + model parity, then 13B Q4_1 512-token prompt speed on the
# MFMA path and on the VALU path (LVK_PROMPT_A16=0); equal logits hashes = identical bits
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "mfma" \
  tests/test_gpu_model.py -k "mfma or q4_1" > gpurun_out/t_q41mm.log 2>&1 || { tail -40 gpurun_out/t_q41mm.log; exit 1; }
tail -3 gpurun_out/t_q41mm.log
timeout -k 10 300 python -u tools/prompt_speed.py 512 13b > gpurun_out/ps13.log 2>&1 || { tail -20 gpurun_out/ps13.log; exit 2; }
LVK_PROMPT_A16=0 timeout -k 10 300 python -u tools/prompt_speed.py 512 13b >> gpurun_out/ps13.log 2>&1 || { tail -20 gpurun_out/ps13.log; exit 3; }
cat gpurun_out/ps13.log
