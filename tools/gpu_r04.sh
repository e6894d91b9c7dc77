# Round-4 GPU runs, one step per call (gpurun -- bash tools/gpu_r04.sh STEP); every GPU step
# runs under its own time limit and the first failure ends the call.  The records under
# profiles/ name the step that produced them (profiles/r04_README.md).
#   suite        the whole -m gpu test suite                        -> gputests.log
#   parity       full-size / full-context / graph / stage-link tests
#   pmc-decode   FETCH_SIZE / WRITE_SIZE of the 7B and 13B decode    -> r04_traffic.json
#   pmc-prompt   PMC record of the 7B prompt matmuls                 -> pmc_prompt_7b/
#   split-shm    the 65B layer-split bench leg, 2 ranks on one GPU   -> r04_bench_split_shm_s2.json
#   prompt-ab    prompt A/B: super-tile width, prompt scores layout  -> r04_prompt_*.jsonl
#   mm-probe     prompt matmul probes: knockouts, MFMA / f32 FMA issue costs
#   attn-ab      decode attention: QKV overlap modes (parity + speed), V-slice order trace
#   sweep13      13B Q4_1 W2 / Wo launch shapes (lib/sweep, LVK_CFG41)  -> r04_sweep13.jsonl
#   apko         prompt attention knockouts (lib/apko_<KO>: make -C llama.vk_amd apko first) + table exp
#   attn-p       prompt attention parity (ops, paths, model, 7B full) + speed + kernel stats
#   attn-d       decode attention parity (ops, paths, beside, seq wrap, 7B full) + 7B decode speed
#   bench        the default bench (N = 1) and rocprofv3 kernel statistics
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"

case "$1" in
suite)
  timeout -k 10 1080 $T tests/ > gpurun_out/gputests.log 2>&1
  rc=$?; grep -E "passed|failed" gpurun_out/gputests.log | tail -2; exit $rc ;;
parity)
  timeout -k 10 900 $T tests/test_gpu_ggml_graph.py tests/test_gpu_stagelink.py tests/test_gpu_seq_wrap.py \
    tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py tests/test_gpu_attn_beside.py > gpurun_out/parity.log 2>&1
  rc=$?; tail -3 gpurun_out/parity.log; exit $rc ;;
pmc-decode)
  bash tools/gpu_pmc_decode.sh gpurun_out/r04_traffic.json ;;
pmc-prompt)
  bash tools/gpu_pmc_prompt.sh 7b gpurun_out/pmc_prompt_7b ;;
split-shm)
  timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --no-13b --no-cpu-baseline --split-transport shm \
    > gpurun_out/r04_bench_split_shm_s2.json 2> gpurun_out/split_shm.err
  rc=$?; tail -3 gpurun_out/split_shm.err; exit $rc ;;
prompt-ab)
  for r in 1 2; do
    for v in 0 1; do
      LVK_MM_SUPERTILE=$v timeout -k 10 180 python3 tools/prompt_speed.py 512 7b 2>/dev/null \
        | sed "s/^{/{\"supertile\": $v, /" | tee -a gpurun_out/r04_prompt_supertile.jsonl || exit 4
      LVK_ATTN_P_SV=$v timeout -k 10 180 python3 tools/prompt_speed.py 512 7b 2>/dev/null \
        | sed "s/^{/{\"sv\": $v, /" | tee -a gpurun_out/r04_prompt_scores.jsonl || exit 4
    done
  done ;;
mm-probe)
  make -C tools/probe mm_probe mfma_cycles valu_cycles > /dev/null || exit 2
  for st in 0 1 2 8; do
    echo "== supertile $st" >> gpurun_out/mm_probe.log
    LVK_MM_SUPERTILE=$st MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe 512 10 >> gpurun_out/mm_probe.log 2>&1 || exit 3
  done
  for e in 16 32 48; do
    echo "== exp$e" >> gpurun_out/mm_probe.log
    MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe_exp$e 512 10 >> gpurun_out/mm_probe.log 2>&1 || exit 3
  done
  timeout -k 10 60 ./tools/probe/mfma_cycles > gpurun_out/mfma_cycles.log 2>&1 || exit 3
  timeout -k 10 60 ./tools/probe/valu_cycles > gpurun_out/valu_cycles.log 2>&1 || exit 3
  grep -E "==|layer total" gpurun_out/mm_probe.log ;;
attn-ab)
  timeout -k 10 600 $T tests/test_gpu_attn_beside.py tests/test_gpu_attn_paths.py > gpurun_out/attn_ab.log 2>&1
  rc=$?; tail -2 gpurun_out/attn_ab.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do
    for m in 0 B Q; do
      case $m in 0) e="";; B) e="LVK_ATTN_BESIDE=1";; Q) e="LVK_QKV_ATTN=1";; esac
      env $e timeout -k 10 180 python3 tools/decode_speed.py 7b 96 2>/dev/null \
        | sed "s/^{/{\"mode\": \"$m\", /" | tee -a gpurun_out/r04_attn_modes.jsonl || exit 4
    done
  done
  make -C tools/probe mv_probe_T > /dev/null || exit 5
  for np in 32 264 500; do
    LVK_TRACE_KIND=1 timeout -k 10 120 ./tools/probe/mv_probe_T $np > gpurun_out/attn_trace_$np.log 2>&1 || exit 5
  done ;;
sweep13)
  for r in 1 2; do
    for c in 0 4 5 8 9 10 11; do
      LVK_LIB=llama.vk_amd/lib/sweep/libllama_vk_amd.so LVK_CFG41=$c timeout -k 10 180 python3 tools/decode_speed.py 13b 64 \
        2>/dev/null | sed "s/^{/{\"cfg41\": $c, /" | tee -a gpurun_out/r04_sweep13.jsonl || exit 4
    done
  done ;;
apko)
  mkdir -p gpurun_out/apko
  cd /tmp && export TMPDIR=/tmp
  for v in base table 1 2 4 8; do
    case $v in base) e="LVK_NONE=1";; table) e="LVK_EXP_TABLE=1";; *) e="LVK_LIB=$R/llama.vk_amd/lib/apko_$v/libllama_vk_amd.so";; esac
    export $e
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/apko -o $v \
      -- python3 $R/tools/prompt_speed.py 512 7b > $R/gpurun_out/apko/$v.log 2>&1 || exit 5
    unset ${e%%=*}
    grep -h "k_attn_p\|k_rope_kv" $R/gpurun_out/apko/${v}_kernel_stats.csv | cut -c1-60,150-230 | sed "s/^/$v /" || true
  done ;;
attn-p)
  timeout -k 10 300 $T tests/test_gpu_ops.py > gpurun_out/attn_p.log 2>&1 && \
  timeout -k 10 600 $T tests/test_gpu_attn_paths.py tests/test_gpu_model.py tests/test_gpu_7b_full.py >> gpurun_out/attn_p.log 2>&1
  rc=$?; grep -E "passed|failed" gpurun_out/attn_p.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do timeout -k 10 180 python3 tools/prompt_speed.py 512 7b 2>/dev/null | tee -a gpurun_out/attn_p.jsonl || exit 4; done
  mkdir -p gpurun_out/attn_p
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/attn_p -o p7b \
    -- python3 $R/tools/prompt_speed.py 512 7b > $R/gpurun_out/attn_p/p7b.log 2>&1 || exit 5 ;;
attn-d)
  timeout -k 10 300 $T tests/test_gpu_ops.py > gpurun_out/attn_d.log 2>&1 && \
  timeout -k 10 700 $T tests/test_gpu_attn_paths.py tests/test_gpu_attn_beside.py tests/test_gpu_seq_wrap.py \
    tests/test_gpu_7b_full.py tests/test_gpu_decode_chain.py >> gpurun_out/attn_d.log 2>&1
  rc=$?; grep -E "passed|failed" gpurun_out/attn_d.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do timeout -k 10 180 python3 tools/decode_speed.py 7b 96 2>/dev/null | tee -a gpurun_out/attn_d.jsonl || exit 4; done ;;
bench)
  timeout -k 10 840 python3 bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
  rc=$?; tail -2 gpurun_out/r04_bench.err; [ $rc -eq 0 ] || exit $rc
  mkdir -p gpurun_out/prof
  cd /tmp && export TMPDIR=/tmp
  for m in 7b 13b; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o $m \
      -- python3 $R/tools/decode_speed.py $m 64 > $R/gpurun_out/prof/$m.log 2>&1 || exit 5
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o p7b \
    -- python3 $R/tools/prompt_speed.py 512 7b > $R/gpurun_out/prof/p7b.log 2>&1 || exit 5 ;;
*)
  echo "usage: bash tools/gpu_r04.sh suite|parity|pmc-decode|pmc-prompt|split-shm|prompt-ab|mm-probe|attn-ab|sweep13|apko|attn-p|attn-d|bench"; exit 2 ;;
esac
