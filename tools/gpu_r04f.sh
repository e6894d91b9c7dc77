# round 4, GPU call F: software-pipelined prompt matmul variants (k_mm_q40_pipe, LVK_MM_PIPE =
# PCR*100 + QA*10 + SCV; 0 = the two-slot kernel with B in LDS), output hashes must agree
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 241 321 341 421 240; do
    echo "== pipe $v round $r" >> gpurun_out/r04f_mm.log
    LVK_MM_PIPE=$v MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe 512 10 >> gpurun_out/r04f_mm.log 2>&1 || exit 3
  done
  for v in 241 321; do
    echo "== sb0 pipe $v round $r" >> gpurun_out/r04f_mm.log
    LVK_MM_PIPE=$v MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe_sb0 512 10 >> gpurun_out/r04f_mm.log 2>&1 || exit 3
  done
done
grep -E "==|layer total|hash" gpurun_out/r04f_mm.log
