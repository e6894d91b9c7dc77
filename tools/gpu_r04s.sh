# round 4, GPU call S: prompt attention scores, a lane per position (LVK_ATTN_P_SV=1, default)
# against the quad layout (0): parity tests, logits hash and time of the 7B 512-token prompt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py tests/test_gpu_kvtypes.py -k "attn or attention or mfma or prompt512 or golden or prompt" > gpurun_out/r04s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04s_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    LVK_ATTN_P_SV=$v timeout -k 10 180 python3 tools/prompt_speed.py 512 7b 2>/dev/null | sed "s/^{/{\"sv\": $v, /" | tee -a gpurun_out/r04s_prompt.jsonl || exit 4
  done
done
