# round 4, GPU call M: why the merged QKV + attention launch is slow -- the QKV role alone
# (LVK_QKV_ATTN_EXP=1, attention workgroups exit; timing only) and a kernel trace
set -o pipefail
mkdir -p gpurun_out
for v in "0 0" "1 0" "1 1"; do
  set -- $v
  LVK_QKV_ATTN=$1 LVK_QKV_ATTN_EXP=$2 timeout -k 10 180 python3 tools/decode_speed.py 7b 64 2>/dev/null | sed "s/^{/{\"merged\": $1, \"exp\": $2, /" | tee -a gpurun_out/r04m_speed.jsonl || exit 4
done
cd /tmp && export TMPDIR=/tmp
LVK_QKV_ATTN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04m_prof -o merged -- python3 $GRAFT_REPO_ROOT/tools/decode_speed.py 7b 32 > $GRAFT_REPO_ROOT/gpurun_out/r04m_prof.log 2>&1 || exit 5
find $GRAFT_REPO_ROOT/gpurun_out/r04m_prof -name "*stats*"
