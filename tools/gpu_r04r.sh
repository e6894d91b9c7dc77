# round 4, GPU call R: rocprofv3 kernel statistics of the 512-token 7B prompt (tools/prompt_speed.py)
set -o pipefail
mkdir -p gpurun_out/r04r_prof
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04r_prof -o p7b -- python3 $R/tools/prompt_speed.py 512 7b > $R/gpurun_out/r04r_prof/p7b.log 2>&1 || exit 5
tail -2 $R/gpurun_out/r04r_prof/p7b.log | cut -c1-300
