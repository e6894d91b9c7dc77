# round 4, GPU call E: prompt matmul A/B (B staged in LDS, scalar fp32 chains) with output
# hashes, and the decode attention V-DMA order A/B (LVK_ATTN_VORDER 0/1/2)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in b0 b1 b0ns b1ns; do
    echo "== mm_probe_$v round $r" >> gpurun_out/r04e_mm.log
    MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe_$v 512 10 >> gpurun_out/r04e_mm.log 2>&1 || exit 3
  done
done
grep -E "==|layer total|hash" gpurun_out/r04e_mm.log | head -60
for r in 1 2; do
  for v in 0 1 2; do
    LVK_ATTN_VORDER=$v timeout -k 10 180 python3 tools/decode_speed.py 7b 96 2>/dev/null | sed "s/^{/{\"vorder\": $v, /" | tee -a gpurun_out/r04e_vorder.jsonl || exit 4
  done
done
