# round 4, GPU call B: the LDS-DMA Wo / W2 decode matvecs (matvec_dma.hip, Q4_0 and Q4_1) --
# parity through the model-level tests, then the decode speed A/B against matvec_cu /
# matvec_cu41 (LVK_MV_DMA=0), alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_decode_chain.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py tests/test_gpu_kvtypes.py > gpurun_out/r04b_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r04b_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 7b 13b; do
  for k in 1 2; do
    for v in 0 1; do
      LVK_MV_DMA=$v timeout -k 10 180 python3 tools/decode_speed.py $m 96 2>/dev/null | tee -a gpurun_out/r04b_ab.jsonl || exit 3
    done
  done
done
bash tools/gpu_pmc_prompt.sh 7b gpurun_out/pmc_prompt_7b || exit 4
