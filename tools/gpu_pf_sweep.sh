#!/bin/bash
# Decode matvec prologue-order sweep (LVK_MV_PF overrides every shape) and a W13 / lm_head phase
# trace.  usage: tools/gpu_pf_sweep.sh <tag> [n_past]
set -o pipefail
tag=${1:-pf}; np=${2:-256}
out=$PWD/gpurun_out/$tag; mkdir -p $out
cd tools/probe || exit 1
for rep in 1 2; do
  timeout -k 10 120 ./mv_probe $np > $out/mv_probe_def_$rep.log 2>&1 || exit $?
  for pf in 0 1 2; do
    LVK_MV_PF=$pf timeout -k 10 120 ./mv_probe $np > $out/mv_probe_pf${pf}_$rep.log 2>&1 || exit $?
  done
done
for k in 0 2 3 4 5; do
  LVK_TRACE_KIND=$k timeout -k 10 120 ./mv_probe_T $np > $out/trace_$k.log 2>&1 || exit $?
done
grep -H -E "token|qkv|wo |w13|w2 |lm_head" $out/mv_probe_*.log
