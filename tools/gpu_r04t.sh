# round 4, GPU call S: prompt attention scores, a lane per position (LVK_ATTN_P_SV=1, default)
# round 4, GPU call T: prompt P.V with v_fma_mix and butterfly quad reduces (parity, hash, time)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py tests/test_gpu_kvtypes.py -k "attn or attention or mfma or prompt512 or golden or prompt" > gpurun_out/r04t_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04t_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    LVK_ATTN_P_SV=$v timeout -k 10 180 python3 tools/prompt_speed.py 512 7b 2>/dev/null | sed "s/^{/{\"sv\": $v, \"pv\": \"fma_mix\", /" | tee -a gpurun_out/r04t_prompt.jsonl || exit 4
  done
done
