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
R=${GRAFT_REPO_ROOT:-$(pwd)}
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
  pc)
    # the producer / consumer decode matvec (Wo, W2): parity of the 7B-shaped / full 7B decode, then
    # A/B speed and per-wave phase stamps
    O=gpurun_out/r05_pc; mkdir -p $O
    timeout -k 10 900 $T tests/test_gpu_model.py tests/test_gpu_decode_chain.py tests/test_gpu_7b_full.py \
      > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 51; }
    tail -2 $O/tests.log
    for r in 1 2; do
      for k in 0 1 2; do
        LVK_MV_PC=$k timeout -k 10 300 python3 tools/decode_speed.py 7b 96 2>/dev/null \
          | sed "s/^{/{\"pc\": $k, /" | tee -a $O/ab.jsonl || exit 52
      done
    done
    for k in 2 4; do
      for v in 1 2; do
        LVK_MV_PC=$v LVK_TRACE_RAW=1 LVK_TRACE_KIND=$k timeout -k 10 120 ./tools/probe/mv_probe_T 256 > $O/raw_${k}_pc$v.log 2>&1 || exit 53
      done
    done
    cat $O/raw_*.log | grep -v "^exp check" ;;
  ks)
    # the K-split decode matvec (Wo, W2): parity of the 7B-shaped / full 7B decode, then A/B speed
    O=gpurun_out/r05_ks; mkdir -p $O
    timeout -k 10 900 $T tests/test_gpu_model.py tests/test_gpu_decode_chain.py tests/test_gpu_7b_full.py \
      > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 51; }
    tail -2 $O/tests.log
    for r in 1 2; do
      for k in 0 1; do
        LVK_MV_KS=$k timeout -k 10 300 python3 tools/decode_speed.py 7b 96 2>/dev/null \
          | sed "s/^{/{\"ks\": $k, /" | tee -a $O/ab.jsonl || exit 52
      done
    done ;;
  trace)
    # per-wave phase stamps of the decode matvecs (tools/probe/mv_probe_T, LVK_TRACE_RAW: events per
    # wave index), kinds 2 wo, 4 w2, with and without the K-split kernel
    O=gpurun_out/r05_trace; mkdir -p $O
    for k in 2 4; do
      for ks in 0 1; do
        LVK_MV_KS=$ks LVK_TRACE_RAW=1 LVK_TRACE_KIND=$k timeout -k 10 120 ./tools/probe/mv_probe_T 256 \
          > $O/raw_${k}_ks$ks.log 2>&1 || exit 61
      done
    done
    cat $O/raw_*.log | grep -v "^exp check" ;;
  diag04)
    # the round-4 library (lib/r04diag, built from commit 7eefa8d + the maps dump) under the
    # kernel trace that crashed in round 4
    O=gpurun_out/r05_diag04; mkdir -p $O
    timeout -k 10 600 python3 tools/decode_speed.py 65b 4 > $O/gen.log 2>&1 || exit 71
    LVK_SEGV_TRACE=1 LVK_LIB=$R/llama.vk_amd/lib/r04diag/libllama_vk_amd.so timeout -k 10 600 rocprofv3 --kernel-trace \
      --stats -d $O/kt -o run --output-format csv -- python3 tools/r04diag/decode_speed.py 65b 16 > $O/kt65.log 2>&1
    rc=$?; grep -v "^[EW]2026" $O/kt65.log | head -20; exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
