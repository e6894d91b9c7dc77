set -o pipefail
o=$PWD/gpurun_out/r03_d; mkdir -p $o
R=$PWD
# 1. the ggml graph compute fault: per-node sync names the failing node
(cd /tmp && LVK_GGML_SYNC=1 timeout -k 5 60 $R/tools/ggml_graph/bin/graph_test_lvk /tmp/l.bin 0 1 > $o/ggml_sync.log 2>&1; echo "rc $?" >> $o/ggml_sync.log)
if grep -q "failed\|rc 134\|rc 1[0-9][0-9]" $o/ggml_sync.log; then echo "ggml fault, stopping"; exit 0; fi
cd tools/probe || exit 1
# 2. prologue order x launch shape
for pf in 0 1 2; do
  for c in 0 1 2 3; do
    LVK_MV_PF=$pf LVK_CFG=$c timeout -k 10 120 ./mv_probe_S 32 > $o/sweep_pf${pf}_c$c.log 2>&1 || exit $?
  done
done
for k in 0 2 3 4; do
  LVK_TRACE_KIND=$k timeout -k 10 120 ./mv_probe_T 32 > $o/trace_$k.log 2>&1 || exit $?
done
echo done
