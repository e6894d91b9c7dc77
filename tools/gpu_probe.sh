#!/bin/bash
# Decode-kernel probes on the GPU box: per-kind launch times and per-wave phase traces.
# usage: tools/gpu_probe.sh <tag> [n_past] [sweep]
set -o pipefail
tag=${1:-probe}; np=${2:-32}; sweep=${3:-0}
out=$PWD/gpurun_out/$tag; mkdir -p $out
cd tools/probe || exit 1
timeout -k 10 120 ./mv_probe $np > $out/mv_probe.log 2>&1 || exit $?
LVK_MV_PF=0 timeout -k 10 120 ./mv_probe $np > $out/mv_probe_pf0.log 2>&1 || exit $?
LVK_PROBE_HOT=1 timeout -k 10 120 ./mv_probe $np > $out/mv_probe_hot.log 2>&1 || exit $?
for k in 0 1 2 3 4 5; do
  LVK_TRACE_KIND=$k timeout -k 10 120 ./mv_probe_T $np > $out/trace_$k.log 2>&1 || exit $?
done
if [ "$sweep" != 0 ] && [ -x ./mv_probe_S ]; then
  for c in 0 1 2 3; do
    LVK_CFG=$c timeout -k 10 120 ./mv_probe_S $np > $out/sweep_$c.log 2>&1 || exit $?
  done
fi
echo done
