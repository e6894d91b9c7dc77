# round 4, GPU call Q: the full default bench (N = 1), then rocprofv3 kernel-trace statistics of
# the 7B / 13B Q4_1 / 65B decode (tools/decode_speed.py on the bench's model files) as CSV
set -o pipefail
mkdir -p gpurun_out/r04q_prof
R=$GRAFT_REPO_ROOT
timeout -k 10 840 python3 bench.py > gpurun_out/r04q_bench.json 2> gpurun_out/r04q_bench.err
rc=$?; tail -2 gpurun_out/r04q_bench.err; head -c 300 gpurun_out/r04q_bench.json; echo; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for m in 7b 13b 65b; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04q_prof -o $m -- python3 $R/tools/decode_speed.py $m 64 > $R/gpurun_out/r04q_prof/$m.log 2>&1 || exit 5
done
find $R/gpurun_out/r04q_prof -name "*kernel_stats*"
