set -o pipefail
o=gpurun_out/r03_b; mkdir -p $o
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_stagelink.py tests/test_gpu_ggml_graph.py \
  "tests/test_dropin.py::test_dropin_embedding_matches_reference_cpu" \
  "tests/test_dropin.py::test_dropin_quantize_stats_matches_reference_cpu" > $o/pytest_new.log 2>&1
rc=$?
echo "pytest rc $rc" >> $o/pytest_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd tools/probe || exit 1
for k in 0 2 3 4; do
  LVK_TRACE_KIND=$k timeout -k 10 120 ./mv_probe_T 32 > ../../$o/trace_$k.log 2>&1 || exit $?
done
echo done
