# prologue-wave sweep (LVK_CFG 0..3 per kind; see matvec_cu.hip LVK_PROBE_SWEEP), PF 2 and 1
set -o pipefail
o=$PWD/gpurun_out/$1; mkdir -p $o
cd tools/probe || exit 1
for pf in 2 1; do for cfg in 0 1 2 3; do
  LVK_MV_PF=$pf LVK_CFG=$cfg timeout -k 10 120 ./mv_probe_S 264 > $o/pf${pf}_cfg$cfg.log 2>&1 || exit $?
  echo "pf $pf cfg $cfg $(grep -E '^n_past' $o/pf${pf}_cfg$cfg.log) | $(grep -E '^  (qkv|w13|lm_head)' $o/pf${pf}_cfg$cfg.log | awk '{print $1, $2}' | tr '\n' ' ')"
done; done | tee $o/summary.txt
