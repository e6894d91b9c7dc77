# round 4, GPU call B: the LDS-DMA decode matvecs (matvec_dma.hip: Q4_0 Wo / W2, opt-in QKV,
# Q4_1 Wo / W2) -- parity through the model-level tests, then the decode speed A/B against
# matvec_cu / matvec_cu41 (LVK_MV_DMA=0), alternating; then the prompt PMC record
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_decode_chain.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py tests/test_gpu_kvtypes.py > gpurun_out/r04b_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r04b_tests.log; [ $rc -eq 0 ] || exit $rc
LVK_MV_DMA_QKV=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_7b_full.py -k "7b_full_prompt16 or 4096 or w4096 or 7b" > gpurun_out/r04b_tests_qkv.log 2>&1
rc=$?; tail -8 gpurun_out/r04b_tests_qkv.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in 0 1 Q; do
    if [ $v = Q ]; then e="LVK_MV_DMA=1 LVK_MV_DMA_QKV=1"; else e="LVK_MV_DMA=$v"; fi
    env $e timeout -k 10 180 python3 tools/decode_speed.py 7b 96 2>/dev/null | sed "s/^{/{\"cfg\": \"$v\", /" | tee -a gpurun_out/r04b_ab.jsonl || exit 3
  done
done
for k in 1 2; do
  for v in 0 1; do
    LVK_MV_DMA=$v timeout -k 10 180 python3 tools/decode_speed.py 13b 64 2>/dev/null | sed "s/^{/{\"cfg\": \"$v\", /" | tee -a gpurun_out/r04b_ab.jsonl || exit 3
  done
done
bash tools/gpu_pmc_prompt.sh 7b gpurun_out/pmc_prompt_7b || exit 4
