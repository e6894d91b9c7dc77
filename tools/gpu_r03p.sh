# per-token decode timeline: kernel + memory-copy traces of a short 7B decode (no counters)
set -o pipefail
o=$PWD/gpurun_out/r03_p; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $o/tl -o run --output-format csv -- python3 tools/decode_speed.py 7b 32 > $o/tl.log 2>&1 || exit 1
python3 tools/timeline.py $o/tl > $o/timeline.txt 2>&1; cat $o/timeline.txt
