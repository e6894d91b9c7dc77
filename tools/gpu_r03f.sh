set -o pipefail
o=$PWD/gpurun_out/r03_f; mkdir -p $o
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ops.py tests/test_gpu_ggml_graph.py tests/test_gpu_model.py > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $o/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd tools/probe || exit 1
for np in 32 200; do
  timeout -k 10 120 ./mv_probe $np > $o/mv_probe_$np.log 2>&1 || exit $?
done
LVK_TRACE_KIND=1 timeout -k 10 120 ./mv_probe_T 32 > $o/trace_1.log 2>&1 || exit $?
echo done
