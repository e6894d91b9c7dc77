# round 4, GPU call H: parity of the LDS-staged B prompt matmul (default now) and of the
# attention V-DMA order 2 (LVK_ATTN_VORDER=2), and the nibble-A path with B in LDS (mm_probe
# MM_A16=0, hashes must equal the f16-A path's)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_ops.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py -k "mfma or prompt512 or golden or matmul or mm" > gpurun_out/r04h_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04h_tests.log; [ $rc -eq 0 ] || exit $rc
LVK_ATTN_VORDER=2 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_attn_paths.py tests/test_gpu_7b_full.py -k "agree or full_context" > gpurun_out/r04h_vorder2.log 2>&1
rc=$?; tail -4 gpurun_out/r04h_vorder2.log; [ $rc -eq 0 ] || exit $rc
for a in 1 0 1 0; do
  echo "== MM_A16=$a" >> gpurun_out/r04h_mm.log
  MM_A16=$a timeout -k 10 120 ./tools/probe/mm_probe 512 10 >> gpurun_out/r04h_mm.log 2>&1 || exit 3
done
grep -E "==|layer total|hash" gpurun_out/r04h_mm.log
