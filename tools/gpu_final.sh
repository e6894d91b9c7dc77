# round-end measurement batch: -m gpu suite, default bench line, kernel-trace summaries of
# the 7B bench (short, under the rocprofiler's ~11k traced graph-dispatch limit) and of the
# 13B Q4_1 decode.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
O=gpurun_out/final
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt7 -o run --output-format csv -- python3 bench.py --steps 16 --warmup 4 --no-13b --no-65b --no-cpu-baseline --prompt-evals 1 > $O/kt7.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt13 -o run --output-format csv -- python3 tools/decode_speed.py 13b 16 > $O/kt13.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt13p -o run --output-format csv -- python3 tools/prompt_speed.py 512 13b > $O/kt13p.log 2>&1 || exit 5
find $O -name '*kernel_stats.csv'
echo final-ok
