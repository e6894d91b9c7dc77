set -o pipefail
o=$PWD/gpurun_out/r03_g; mkdir -p $o
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ggml_graph.py > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $o/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd tools/probe || exit 1
timeout -k 10 120 ./mv_probe 32 > $o/base.log 2>&1 || exit $?
for pf in 32 128; do for k in 0 1 4; do
  LVK_PROBE_PF=$pf LVK_PROBE_PFK=$k timeout -k 10 120 ./mv_probe 32 > $o/pf${pf}_k$k.log 2>&1 || exit $?
done; done
for sm in 0 128; do
  LVK_ATTN_SHORT=$sm timeout -k 10 120 ./mv_probe 32 > $o/short${sm}_32.log 2>&1 || exit $?
  LVK_ATTN_SHORT=$sm timeout -k 10 120 ./mv_probe 100 > $o/short${sm}_100.log 2>&1 || exit $?
done
echo done
