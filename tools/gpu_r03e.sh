set -o pipefail
o=$PWD/gpurun_out/r03_e; mkdir -p $o
cd tools/probe || exit 1
for pf in 1 2 3; do
  for c in 0 1 2 3; do
    LVK_MV_PF=$pf LVK_CFG=$c timeout -k 10 120 ./mv_probe_S 32 > $o/sweep_pf${pf}_c$c.log 2>&1 || exit $?
  done
done
for k in 0 2 3 4 5; do
  LVK_MV_PF=3 LVK_TRACE_KIND=$k timeout -k 10 120 ./mv_probe_T 32 > $o/trace_$k.log 2>&1 || exit $?
done
echo done
