# round 4, GPU call G: prompt matmul L2 locality -- super-tile width R (LVK_MM_SUPERTILE) and
# the L2-hot knockouts (mm_probe_exp16: weights of 4 row tiles only, exp32: activations of 2
# token tiles only, exp48: both; timing only)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for st in 0 1 2 8 16; do
    echo "== supertile $st round $r" >> gpurun_out/r04g_mm.log
    LVK_MM_SUPERTILE=$st MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe 512 10 >> gpurun_out/r04g_mm.log 2>&1 || exit 3
  done
  for e in 16 32 48; do
    echo "== exp$e round $r" >> gpurun_out/r04g_mm.log
    MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe_exp$e 512 10 >> gpurun_out/r04g_mm.log 2>&1 || exit 3
  done
done
grep -E "==|layer total" gpurun_out/r04g_mm.log
