# round 4, GPU call O: where the merged QKV + attention launch loses time (probe bits)
set -o pipefail
mkdir -p gpurun_out
for v in "0 0" "1 0" "1 1" "1 2" "1 3"; do
  set -- $v
  LVK_QKV_ATTN=$1 LVK_QKV_ATTN_EXP=$2 timeout -k 10 180 python3 tools/decode_speed.py 7b 64 2>/dev/null | sed "s/^{/{\"merged\": $1, \"exp\": $2, /" | tee -a gpurun_out/r04o_speed.jsonl || exit 4
done
