# traces: decode attention phases at three context lengths, per-workgroup end statistics of every matvec kind
set -o pipefail
o=$PWD/gpurun_out/r03_i; mkdir -p $o
cd tools/probe || exit 1
for np in 32 264 500; do
  LVK_TRACE_KIND=1 timeout -k 10 120 ./mv_probe_T $np > $o/attn_$np.log 2>&1 || exit $?
  LVK_TRACE_KIND=1 LVK_ATTN_SHORT=100000 timeout -k 10 120 ./mv_probe_T $np > $o/attn_noex_$np.log 2>&1 || exit $?
done
for k in 0 2 3 4; do LVK_TRACE_KIND=$k timeout -k 10 120 ./mv_probe_T 32 > $o/kind$k.log 2>&1 || exit $?; done
timeout -k 10 120 ./mv_probe 264 > $o/base264.log 2>&1 || exit $?
timeout -k 10 120 ./mv_probe 500 > $o/base500.log 2>&1 || exit $?
echo done
