# launch-shape sweep (LVK_CFG 0..3 per kind; see matvec_cu.hip LVK_PROBE_SWEEP) over prologue
# orders (LVK_MV_PF).  usage: tools/gpu_sweep_np.sh <tag> [n_past] [pf list]
set -o pipefail
o=$PWD/gpurun_out/$1; np=${2:-256}; pfs=${3:-"0 1 2"}; mkdir -p $o
cd tools/probe || exit 1
for pf in $pfs; do for cfg in 0 1 2 3; do
  LVK_MV_PF=$pf LVK_CFG=$cfg timeout -k 10 120 ./mv_probe_S $np > $o/pf${pf}_cfg$cfg.log 2>&1 || exit $?
  echo "pf $pf cfg $cfg $(grep -E '^n_past' $o/pf${pf}_cfg$cfg.log) | $(grep -E '^  (qkv|wo|w13|w2|lm_head)' $o/pf${pf}_cfg$cfg.log | awk '{print $1, $2}' | tr '\n' ' ')"
done; done | tee $o/summary.txt
