# r03 mid-round batch: full -m gpu suite on the product library, the parked kernels' tests on
# the dev library, the stream floor, the matvec trace with per-workgroup end statistics, the
# default bench line.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
o=$PWD/gpurun_out/r03_h; mkdir -p $o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > $o/gputests.log 2>&1 || { tail -30 $o/gputests.log; exit 1; }
tail -2 $o/gputests.log
LVK_LIB=$PWD/llama.vk_amd/lib/dev/libllama_vk_amd.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_persistent.py tests/test_gpu_model.py::test_7b_shaped_fused_attention_wo_matches tests/test_gpu_faults.py > $o/devtests.log 2>&1 || { tail -30 $o/devtests.log; exit 2; }
tail -2 $o/devtests.log
(cd tools/probe && timeout -k 10 120 ./bw_probe > $o/bw.log 2>&1) || exit 3
(cd tools/probe && timeout -k 10 120 ./mv_probe_T 32 > $o/trace.log 2>&1) || exit 4
timeout -k 10 900 python3 -u bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 5; }
cat $o/bench.json
echo r03h-ok
