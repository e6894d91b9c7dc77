# round-3 measurement batch: -m gpu suite, smoke, default bench line, kernel-trace summaries of
# the 7B bench and the 13B Q4_1 decode.  Each GPU step has its own limit; the chain stops at
# the first failure.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt7 -o run --output-format csv -- python3 bench.py --steps 16 --warmup 4 --no-13b --no-65b --no-cpu-baseline --prompt-evals 1 > $O/kt7.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt13 -o run --output-format csv -- python3 tools/decode_speed.py 13b 16 > $O/kt13.log 2>&1 || exit 5
find $O -name '*kernel_stats.csv'
echo final-ok
