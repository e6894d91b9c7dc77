# round 4, GPU call L: QKV + decode attention in one launch (LVK_QKV_ATTN=1) and beside QKV
# (LVK_ATTN_BESIDE=1): parity (tests/test_gpu_attn_beside.py, and the attention-path / model /
# seq-wrap / full-context tests with the merged launch), then the 7B decode A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_attn_beside.py > gpurun_out/r04l_beside.log 2>&1
rc=$?; tail -14 gpurun_out/r04l_beside.log; [ $rc -eq 0 ] || exit $rc
export LVK_QKV_ATTN=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_attn_paths.py tests/test_gpu_seq_wrap.py -k "decode or golden or agree or wrap" > gpurun_out/r04l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_7b_full.py -k "full_context or prompt16" > gpurun_out/r04l_7b.log 2>&1
rc=$?; tail -3 gpurun_out/r04l_7b.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    LVK_QKV_ATTN=$v timeout -k 10 180 python3 tools/decode_speed.py 7b 96 2>/dev/null | sed "s/^{/{\"merged\": $v, /" | tee -a gpurun_out/r04l_speed.jsonl || exit 4
  done
done
