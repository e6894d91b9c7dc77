# round 4, GPU call C: LDS-DMA decode matvecs (static chunk loop, no redundant refills) --
# parity, decode A/B; prompt matmul variants (LVK_MM_VARIANT) A/B with logits hashes; the
# decode attention phase trace (tools/probe/mv_probe_T)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py tests/test_gpu_model.py -k "decode" > gpurun_out/r04c_tests.log 2>&1
rc=$?; tail -12 gpurun_out/r04c_tests.log; [ $rc -eq 0 ] || exit $rc
LVK_MV_DMA_QKV=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_7b_full.py tests/test_gpu_model.py -k "7b_full_prompt16 or 7b_shaped_decode" > gpurun_out/r04c_tests_qkv.log 2>&1
rc=$?; tail -5 gpurun_out/r04c_tests_qkv.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in 0 1 Q; do
    if [ $v = Q ]; then e="LVK_MV_DMA=1 LVK_MV_DMA_QKV=1"; else e="LVK_MV_DMA=$v"; fi
    env $e timeout -k 10 180 python3 tools/decode_speed.py 7b 96 2>/dev/null | sed "s/^{/{\"cfg\": \"$v\", /" | tee -a gpurun_out/r04c_ab.jsonl || exit 3
  done
done
for k in 1 2; do
  for v in 0 1; do
    LVK_MV_DMA=$v timeout -k 10 180 python3 tools/decode_speed.py 13b 64 2>/dev/null | sed "s/^{/{\"cfg\": \"$v\", /" | tee -a gpurun_out/r04c_ab.jsonl || exit 3
  done
done
for k in 1 2; do
  for v in 0 1 2 4 5 6; do
    LVK_MM_VARIANT=$v timeout -k 10 180 python3 tools/prompt_speed.py 512 7b 2>/dev/null | sed "s/^{/{\"variant\": $v, /" | tee -a gpurun_out/r04c_prompt.jsonl || exit 4
  done
done
for np in 32 264 500; do
  LVK_TRACE_KIND=1 timeout -k 10 120 ./tools/probe/mv_probe_T $np > gpurun_out/r04c_attn_trace_$np.log 2>&1 || exit 5
done
tail -2 gpurun_out/r04c_attn_trace_*.log
