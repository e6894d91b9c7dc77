# Round-5 GPU runs, one or more steps per call (gpurun -- bash tools/gpu_r05.sh STEP...); every GPU
# step runs under its own time limit and the first failure ends the call.
#   suite       the whole -m gpu test suite                          -> gpurun_out/gputests.log
#   bench       bench.py at its defaults (N = 1)                      -> gpurun_out/r05_bench.json
#   kt          kernel-trace summaries: 7B bench legs, 13B Q4_1 decode, 7B 512-token prompt
#                                                                     -> gpurun_out/r05_kt/
#   pmc         FETCH_SIZE / WRITE_SIZE per decode kernel, 7B and 13B -> gpurun_out/r05_traffic.json
#   sq          SQ issue / wait counters per decode kernel (SQMODEL, 7b) -> gpurun_out/r05_sq_<m>/sq_decode_<m>.json
#   split       65B layer split over 2 ranks on the one GPU through the shm stage link
#                                                                     -> gpurun_out/r05_bench_split_shm_s2.json
#   l2          L2 retention across launches (tools/probe/l2_probe)   -> gpurun_out/r05_l2/
#   trace       per-wave phase stamps of the Wo / W2 decode matvecs   -> gpurun_out/r05_trace/
#   prof65      the 65B decode under rocprofv3 --kernel-trace         -> gpurun_out/r05_prof65/
#   ab13        13B Q4_1 decode with and without half-group work units -> gpurun_out/r05_ab13/
#   smoke       __graft_entry__.smoke()                               -> gpurun_out/r05_smoke.log
#   diag7       the 7B bench under rocprofv3 with the fault dump (DIAG_ENV: extra environment)
#   x / mmx     decode / prompt matmul knockout probes                -> gpurun_out/r05_x/, r05_mmx/
#   mmab        prompt matmul probe builds A/B (MMB)                  -> gpurun_out/r05_mmab/
#   envab       one environment switch A/B on the 7B bench legs (ABVAR, ABVALS, ABTESTS)
#   libab       library A/B (lib/ab_base vs the tree) on decode_speed (ABMODEL, ABTESTS)
#   ab41        Q4_1 in-kernel weight sums A/B (LVK_MV41_WSI; the variant is removed since)
# Probe steps run binaries built beforehand in this container (never on the box):
#   x: make -C tools/probe mv_probe mv_probe_x;  mmx: make -C tools/probe mm_probe MM_EXPS="...";
#   trace: make -C tools/probe mv_probe_T;  l2: make -C tools/probe l2_probe;  libab: a library in
#   llama.vk_amd/lib/ab_base.
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
    timeout -k 10 900 $T tests/ > gpurun_out/gputests.log 2>&1
    rc=$?; grep -E "passed|failed" gpurun_out/gputests.log | tail -2; [ $rc -eq 0 ] || exit $rc ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > gpurun_out/r05_smoke.log 2>&1 \
      || { tail -20 gpurun_out/r05_smoke.log; exit 25; }
    tail -2 gpurun_out/r05_smoke.log ;;
  bench)
    timeout -k 10 900 python3 -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err \
      || { tail -20 gpurun_out/r05_bench.err; exit 21; }
    tail -c 600 gpurun_out/r05_bench.json ;;
  kt)
    O=gpurun_out/r05_kt; mkdir -p $O
    timeout -k 10 300 python3 tools/decode_speed.py 7b 8 > $O/gen.log 2>&1 || exit 31
    env $NOCAP timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt7 -o run --output-format csv -- \
      python3 bench.py --steps 96 --warmup 8 --no-13b --no-65b --no-cpu-baseline --prompt-evals 1 > $O/kt7.log 2>&1 || exit 32
    env $NOCAP timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt13 -o run --output-format csv -- \
      python3 tools/decode_speed.py 13b 64 > $O/kt13.log 2>&1 || exit 33
    env $NOCAP timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ktp -o run --output-format csv -- \
      python3 tools/prompt_once.py > $O/ktp.log 2>&1 || exit 34
    find $O -name '*kernel_stats.csv' ;;
  pmc)
    timeout -k 10 1000 bash tools/gpu_pmc_decode.sh gpurun_out/r05_traffic.json || exit 41 ;;
  sq)
    # one pass of 8 SQ counters over a short 7B decode: issue cycles of the five decode kernels
    M=${SQMODEL:-7b}
    O=gpurun_out/r05_sq_$M; mkdir -p $O
    timeout -k 10 300 python3 tools/decode_speed.py $M 8 > $O/gen.log 2>&1 || exit 51
    env $NOCAP timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
      SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/sqA -o run --output-format csv -- \
      python3 tools/decode_speed.py $M 8 > $O/sqA.log 2>&1 || exit 52
    env $NOCAP timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS \
      -d $O/sqB -o run --output-format csv -- python3 tools/decode_speed.py $M 8 > $O/sqB.log 2>&1 || exit 53
    python3 tools/pmc_reduce.py $O/sq_decode_$M.json $(find $O/sqA $O/sqB -name '*counter_collection.csv') || exit 54
    echo sq-ok ;;
  split)
    # the N > 1 65B leg rehearsed on one GPU: two ranks, one 40-layer stage each, shm stage link
    timeout -k 10 600 python3 tools/decode_speed.py 65b 2 > gpurun_out/r05_split_gen.log 2>&1 || exit 61
    timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --split-transport shm --no-13b --no-cpu-baseline \
      > gpurun_out/r05_bench_split_shm_s2.json 2> gpurun_out/r05_split.err \
      || { tail -30 gpurun_out/r05_split.err; exit 62; }
    tail -c 800 gpurun_out/r05_bench_split_shm_s2.json ;;
  diag7)
    # the 7B bench under the kernel trace with the fault dump (LVK_SEGV_TRACE: frames + maps)
    O=gpurun_out/r05_diag7; mkdir -p $O
    timeout -k 10 300 python3 tools/decode_speed.py 7b 4 > $O/gen.log 2>&1 || exit 101
    # DIAG_ENV: extra environment of the profiled run (e.g. HSA_ENABLE_SDMA=0)
    env LVK_SEGV_TRACE=1 $DIAG_ENV timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
      python3 bench.py --steps 96 --warmup 8 --no-13b --no-65b --no-cpu-baseline --prompt-evals 1 > $O/kt7.log 2>&1
    rc=$?; grep -v "^[EW]2026" $O/kt7.log | head -30; exit $rc ;;
  x)
    # chain-part costs (tools/probe mv_probe_xN, LVK_PROBE_EXP; not bit-exact) beside the product kernels
    O=gpurun_out/r05_x; mkdir -p $O
    for e in 0 1 2 4 7 0; do
      b=./tools/probe/mv_probe_x$e; [ $e = 0 ] && b=./tools/probe/mv_probe
      timeout -k 10 120 $b 256 > $O/x$e.log 2>&1 || exit 111
      echo "exp $e: $(grep -E '^  (wo|w2|qkv|w13) ' $O/x$e.log | tr -s ' ' | tr '\n' ';')"
    done ;;
  l2)
    O=gpurun_out/r05_l2; mkdir -p $O
    timeout -k 10 60 ./tools/probe/l2_probe xcc > $O/xcc.log 2>&1 || exit 11
    for kind in wo w13 qkv w2; do
      for mode in "cold 0" "hot 0" "hot 1" "pf 0" "pf 1"; do
        set -- $mode
        d=$O/${kind}_$1_$2
        env $NOCAP timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
          ./tools/probe/l2_probe $1 $kind $2 > $d.log 2>&1 || exit 12
      done
    done
    cat $O/xcc.log; grep -h mode $O/*.log ;;
  trace)
    # per-wave phase stamps (tools/probe/mv_probe_T, LVK_TRACE_RAW: events per wave index), kinds 2 wo, 4 w2
    O=gpurun_out/r05_trace; mkdir -p $O
    for k in 2 4; do
      LVK_TRACE_RAW=1 LVK_TRACE_KIND=$k timeout -k 10 120 ./tools/probe/mv_probe_T 256 > $O/raw_$k.log 2>&1 || exit 71
    done
    cat $O/raw_*.log | grep -v "^exp check" ;;
  prof65)
    O=gpurun_out/r05_prof65; mkdir -p $O
    timeout -k 10 600 python3 tools/decode_speed.py 65b 4 > $O/gen.log 2>&1 || exit 81
    env $NOCAP timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
      python3 tools/decode_speed.py 65b 16 > $O/kt65.log 2>&1 || exit 82
    find $O -name '*kernel_stats.csv' ;;
  ab41)
    # 13B Q4_1 decode: even-chain weight sums in the kernel (LVK_MV41_WSI=1) vs the weight-sum
    # image; the Q4_1 parity tests with the in-kernel sums first
    O=gpurun_out/r05_ab41; mkdir -p $O
    LVK_MV41_WSI=1 timeout -k 10 600 $T tests/test_gpu_13b_full.py tests/test_gpu_model.py -k "q4_1 or 13b" \
      > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 121; }
    tail -2 $O/tests.log
    for r in 1 2; do
      for w in 0 1; do
        LVK_MV41_WSI=$w timeout -k 10 300 python3 tools/decode_speed.py 13b 64 2>/dev/null \
          | sed "s/^{/{\"wsi\": $w, /" | tee -a $O/ab.jsonl || exit 122
      done
    done ;;
  mmx)
    # prompt matmul knockouts on the 7B shapes, N = 512, f16 A image (tools/probe/mm_probe_expN,
    # LVK_MM_EXP bits: 1 no fp32 chains, 2 no MFMA, 8 no A loads; timing only)
    O=gpurun_out/r05_mmx; mkdir -p $O
    for e in ${MMX:-0 1 2 3 8 9 10 11}; do
      b=./tools/probe/mm_probe_exp$e; [ $e = 0 ] && b=./tools/probe/mm_probe
      MM_A16=1 timeout -k 10 120 $b 512 20 > $O/x$e.log 2>&1 || exit 141
      echo "exp $e: $(tr -s ' ' < $O/x$e.log | tr '\n' ';')"
    done ;;
  mmab)
    # prompt matmul A/B: probe builds named in MMB (tools/probe/<name>), twice each; hashes must match
    O=gpurun_out/r05_mmab; mkdir -p $O
    for r in 1 2; do
      for b in ${MMB:-mm_probe}; do
        MM_A16=1 timeout -k 10 120 ./tools/probe/$b 512 20 > $O/${b}_$r.log 2>&1 || exit 161
        echo "$b: $(grep -o 'hash [0-9a-f]*\|[0-9.]* us [0-9]\|32 layers [0-9.]* ms' $O/${b}_$r.log | tr '\n' ' ')"
      done
    done ;;
  envab)
    # A/B of one environment switch (ABVAR, values ABVALS, default 0 1) on the 7B bench legs, twice;
    # with ABTESTS set, those GPU tests run first with the last value
    O=gpurun_out/r05_envab_$ABVAR; mkdir -p $O
    vals=${ABVALS:-0 1}
    if [ -n "$ABTESTS" ]; then
      env $ABVAR=${vals##* } timeout -k 10 900 $T $ABTESTS > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 171; }
      tail -2 $O/tests.log
    fi
    for r in 1 2; do
      for v in $vals; do
        env $ABVAR=$v timeout -k 10 400 python3 bench.py --no-13b --no-65b --no-cpu-baseline --prompt-evals 1 \
          > $O/b_${v}_${r}.json 2> $O/b_${v}_${r}.err || exit 172
        python3 -c "import json,sys; d=json.loads(open('$O/b_${v}_${r}.json').read().splitlines()[-1]); g=d['decode_greedy_device']; print(json.dumps({'$ABVAR': '$v', 'eval_loop': round(d['value'],1), 'greedy': round(g['value'],1), 'chained': round(g['chained']['value'],1), 'sampled_dev': round(g['sampled_decode_tok_s']['device_sampler'],1)}))" | tee -a $O/ab.jsonl
      done
    done ;;
  libab)
    # library A/B: llama.vk_amd/lib/ab_base (the previous build) vs the tree's library, decode_speed on
    # ABMODEL (default 13b), twice each; with ABTESTS set those GPU tests run first on the tree's library
    O=gpurun_out/r05_libab; mkdir -p $O
    if [ -n "$ABTESTS" ]; then
      timeout -k 10 900 $T $ABTESTS > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 181; }
      tail -2 $O/tests.log
    fi
    for r in 1 2; do
      for l in base tree; do
        if [ $l = base ]; then LIBV=$R/llama.vk_amd/lib/ab_base/libllama_vk_amd.so; else LIBV=; fi
        env ${LIBV:+LVK_LIB=$LIBV} timeout -k 10 300 python3 tools/decode_speed.py ${ABMODEL:-13b} 64 2>/dev/null \
          | sed "s/^{/{\"lib_ab\": \"$l\", /" | tee -a $O/ab.jsonl || exit 182
      done
    done ;;
  pfsweep)
    # prologue orders (LVK_MV_PF 0..5) of the Q4_0 decode matvecs on the current kernels, sweep probe
    # build (tools/probe/mv_probe_S, make -C tools/probe mv_probe_S), n_past 256, twice
    O=gpurun_out/r05_pfsweep; mkdir -p $O
    for r in 1 2; do
      for pf in 0 1 2 3 4 5; do
        LVK_MV_PF=$pf LVK_CFG=0 timeout -k 10 120 ./tools/probe/mv_probe_S 256 > $O/pf${pf}_$r.log 2>&1 || exit 191
        echo "pf $pf: $(grep -E '^  (qkv|wo|w13|w2|lm_head) ' $O/pf${pf}_$r.log | tr -s ' ' | cut -d' ' -f2,3 | tr '\n' ' ')"
      done
    done ;;
  ab13)
    # 13B Q4_1 decode: half-group work units (LVK_MV41_HALF) A/B, twice each
    O=gpurun_out/r05_ab13; mkdir -p $O
    for r in 1 2; do
      for h in 0 1; do
        LVK_MV41_HALF=$h timeout -k 10 300 python3 tools/decode_speed.py 13b 64 2>/dev/null \
          | sed "s/^{/{\"half\": $h, /" | tee -a $O/ab.jsonl || exit 91
      done
    done ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
