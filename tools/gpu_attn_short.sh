#!/bin/bash
# decode attention: the no-exchange schedule past n_kv 128 (LVK_ATTN_SHORT) against the exchange
set -o pipefail
o=$PWD/gpurun_out/$1; mkdir -p $o
cd tools/probe || exit 1
for rep in 1 2; do for np in 160 200 264 400 500; do for sm in 128 192 320 512; do
  LVK_ATTN_SHORT=$sm timeout -k 10 120 ./mv_probe $np > $o/s${sm}_$np.log 2>&1 || exit $?
  echo "short_max $sm n_past $np $(grep -E '^  attn' $o/s${sm}_$np.log)"
done; done; done | tee $o/summary.txt
