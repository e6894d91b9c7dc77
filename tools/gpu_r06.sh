# Round-6 GPU runs, one or more steps per call (gpurun -- bash tools/gpu_r06.sh STEP...); every GPU
# step runs under its own time limit and the first failure ends the call.
#   suite       the whole -m gpu test suite                          -> gpurun_out/gputests.log
#   smoke       __graft_entry__.smoke()                               -> gpurun_out/r06_smoke.log
#   bench       bench.py as the driver runs it (--steps 20 --warmup 5) -> gpurun_out/r06_bench.json
#   kt          kernel-trace summaries: 7B bench legs, 13B Q4_1 decode, 7B 512-token prompt
#                                                                     -> gpurun_out/r06_kt/
#   pmc         FETCH_SIZE / WRITE_SIZE per decode kernel, 7B and 13B -> gpurun_out/r06_traffic.json
#   sq          SQ issue / wait counters per decode kernel (SQMODEL, 7b) -> gpurun_out/r06_sq_<m>/sq_decode_<m>.json
#   prof65      the 65B decode under rocprofv3 --kernel-trace         -> gpurun_out/r06_prof65/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
# profiled runs: HIP's graph packet capture off.  rocprofv3's dispatch interception reads a
# captured graph's packet batch past the end of the AQL ring when the batch wraps it (SIGSEGV
# at the ring's end: profiles/r05/rocprof_graph_fault/README.md); unprofiled runs keep it on
NOCAP=DEBUG_CLR_GRAPH_PACKET_CAPTURE=0

for step in "$@"; do
  echo "== step $step"
  case "$step" in
  suite)
    timeout -k 10 1100 $T tests/ > gpurun_out/gputests.log 2>&1
    rc=$?; grep -E "passed|failed" gpurun_out/gputests.log | tail -2; [ $rc -eq 0 ] || exit $rc ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > gpurun_out/r06_smoke.log 2>&1 \
      || { tail -20 gpurun_out/r06_smoke.log; exit 25; }
    tail -2 gpurun_out/r06_smoke.log ;;
  bench)
    timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err \
      || { tail -20 gpurun_out/r06_bench.err; exit 21; }
    tail -c 600 gpurun_out/r06_bench.json ;;
  kt)
    O=gpurun_out/r06_kt; mkdir -p $O
    timeout -k 10 300 python3 tools/decode_speed.py 7b 8 > $O/gen.log 2>&1 || exit 31
    env $NOCAP timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt7 -o run --output-format csv -- \
      python3 bench.py --steps 96 --warmup 8 --no-13b --no-65b --no-cpu-baseline --prompt-evals 1 > $O/kt7.log 2>&1 || exit 32
    env $NOCAP timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt13 -o run --output-format csv -- \
      python3 tools/decode_speed.py 13b 64 > $O/kt13.log 2>&1 || exit 33
    env $NOCAP timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ktp -o run --output-format csv -- \
      python3 tools/prompt_once.py > $O/ktp.log 2>&1 || exit 34
    find $O -name '*kernel_stats.csv' ;;
  pmc)
    timeout -k 10 1000 bash tools/gpu_pmc_decode.sh gpurun_out/r06_traffic.json || exit 41 ;;
  sq)
    # one pass of 8 SQ counters over a short 7B decode: issue cycles of the five decode kernels
    M=${SQMODEL:-7b}
    O=gpurun_out/r06_sq_$M; mkdir -p $O
    timeout -k 10 300 python3 tools/decode_speed.py $M 8 > $O/gen.log 2>&1 || exit 51
    env $NOCAP timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
      SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/sqA -o run --output-format csv -- \
      python3 tools/decode_speed.py $M 8 > $O/sqA.log 2>&1 || exit 52
    env $NOCAP timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS \
      -d $O/sqB -o run --output-format csv -- python3 tools/decode_speed.py $M 8 > $O/sqB.log 2>&1 || exit 53
    python3 tools/pmc_reduce.py $O/sq_decode_$M.json $(find $O/sqA $O/sqB -name '*counter_collection.csv') || exit 54
    echo sq-ok ;;
  prof65)
    O=gpurun_out/r06_prof65; mkdir -p $O
    timeout -k 10 600 python3 tools/decode_speed.py 65b 4 > $O/gen.log 2>&1 || exit 81
    env $NOCAP timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
      python3 tools/decode_speed.py 65b 16 > $O/kt65.log 2>&1 || exit 82
    find $O -name '*kernel_stats.csv' ;;
  split)
    # the N > 1 bench path rehearsed on one GPU: two ranks (7B replicas + the 65B split leg, one
    # 40-layer stage per rank over the shm stage link; RCCL needs two devices)
    timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --split-transport shm --no-13b --no-cpu-baseline \
      > gpurun_out/r06_bench_split_shm_s2.json 2> gpurun_out/r06_split.err \
      || { tail -30 gpurun_out/r06_split.err; exit 62; }
    tail -c 800 gpurun_out/r06_bench_split_shm_s2.json ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
