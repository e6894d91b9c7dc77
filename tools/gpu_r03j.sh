# decode attention: step block through the scalar cache, phase trace at three context lengths, parity
set -o pipefail
o=$PWD/gpurun_out/r03_o; mkdir -p $o
export PYTHONUNBUFFERED=1
cd tools/probe || exit 1
for np in 32 264 500; do
  LVK_TRACE_KIND=1 timeout -k 10 120 ./mv_probe_T $np > $o/attn_$np.log 2>&1 || exit $?
  timeout -k 10 120 ./mv_probe $np > $o/base_$np.log 2>&1 || exit $?
done
cd ../.. || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_attn_paths.py tests/test_gpu_model.py tests/test_gpu_faults.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py tests/test_gpu_kvtypes.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
echo done
