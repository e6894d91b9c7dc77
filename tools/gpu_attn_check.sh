#!/bin/bash
# decode attention: parity tests (both schedules, every exp mode, the fault probe) and probe
# timings at n_past 32 / 100 / 264 / 500.  usage: tools/gpu_attn_check.sh <tag>
set -o pipefail
o=$PWD/gpurun_out/$1; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_attn_paths.py tests/test_gpu_ops.py tests/test_gpu_decode_chain.py tests/test_gpu_faults.py tests/test_gpu_7b_full.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
cd tools/probe || exit 1
for np in 32 100 264 500; do
  timeout -k 10 120 ./mv_probe $np > $o/mv_probe_$np.log 2>&1 || exit $?
  echo "$np $(grep -E '^n_past' $o/mv_probe_$np.log) $(grep -E '^  attn' $o/mv_probe_$np.log)"
done | tee $o/summary.txt
