# Round-5 GPU runs, one or more steps per call (gpurun -- bash tools/gpu_r05.sh STEP...); every GPU
# step runs under its own time limit and the first failure ends the call.
#   suite       the whole -m gpu test suite                          -> gpurun_out/gputests.log
#   l2          L2 retention across launches (tools/probe/l2_probe)   -> gpurun_out/r05_l2/
#   diag65      the 65B decode under rocprofv3 --kernel-trace with LVK_SEGV_TRACE=1 (native frames
#               and /proc/self/maps on a fault)                      -> gpurun_out/r05_diag65/
#   prof65      the same trace, expected to complete                 -> gpurun_out/r05_prof65/
#   ab13        13B Q4_1 decode with and without half-group work units -> gpurun_out/r05_ab13/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"

for step in "$@"; do
  echo "== step $step"
  case "$step" in
  suite)
    timeout -k 10 900 $T tests/ > gpurun_out/gputests.log 2>&1
    rc=$?; grep -E "passed|failed" gpurun_out/gputests.log | tail -2; [ $rc -eq 0 ] || exit $rc ;;
  l2)
    O=gpurun_out/r05_l2; mkdir -p $O
    timeout -k 10 60 ./tools/probe/l2_probe xcc > $O/xcc.log 2>&1 || exit 11
    for kind in wo w13 qkv w2; do
      for mode in "cold 0" "hot 0" "hot 1" "pf 0" "pf 1"; do
        set -- $mode
        d=$O/${kind}_$1_$2
        timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
          ./tools/probe/l2_probe $1 $kind $2 > $d.log 2>&1 || exit 12
      done
    done
    cat $O/xcc.log; grep -h mode $O/*.log ;;
  ab13)
    # 13B Q4_1 decode: half-group work units (LVK_MV41_HALF) A/B, twice each
    O=gpurun_out/r05_ab13; mkdir -p $O
    for r in 1 2; do
      for h in 0 1; do
        LVK_MV41_HALF=$h timeout -k 10 300 python3 tools/decode_speed.py 13b 64 2>/dev/null \
          | sed "s/^{/{\"half\": $h, /" | tee -a $O/ab.jsonl || exit 41
      done
    done ;;
  diag65)
    O=gpurun_out/r05_diag65; mkdir -p $O
    timeout -k 10 600 python3 tools/decode_speed.py 65b 4 > $O/gen.log 2>&1 || exit 21
    LVK_SEGV_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
      python3 tools/decode_speed.py 65b 16 > $O/kt65.log 2>&1
    rc=$?; tail -5 $O/kt65.log; exit $rc ;;
  prof65)
    O=gpurun_out/r05_prof65; mkdir -p $O
    timeout -k 10 600 python3 tools/decode_speed.py 65b 4 > $O/gen.log 2>&1 || exit 31
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
      python3 tools/decode_speed.py 65b 16 > $O/kt65.log 2>&1 || exit 32
    find $O -name '*kernel_stats.csv' ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
