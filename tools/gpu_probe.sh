#!/bin/bash
# Decode-kernel probes on the GPU box: per-kind launch times and per-wave phase traces.
# usage: tools/gpu_probe.sh <tag> [n_past]
set -o pipefail
tag=${1:-probe}; np=${2:-32}
out=gpurun_out/$tag; mkdir -p $out
cd tools/probe || exit 1
timeout -k 10 120 ./mv_probe $np > ../../$out/mv_probe.log 2>&1 || exit $?
LVK_PROBE_HOT=1 timeout -k 10 120 ./mv_probe $np > ../../$out/mv_probe_hot.log 2>&1 || exit $?
for k in 0 1 2 3 4 5; do
  LVK_TRACE_KIND=$k timeout -k 10 120 ./mv_probe_T $np > ../../$out/trace_$k.log 2>&1 || exit $?
done
if [ -x ./bw_probe ]; then timeout -k 10 120 ./bw_probe > ../../$out/bw_probe.log 2>&1 || exit $?; fi
echo done
