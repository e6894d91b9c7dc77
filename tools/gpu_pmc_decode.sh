# HBM traffic of the 7B and 13B decode kernels (bench.py --traffic-json): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes over a short decode (tools/decode_speed.py),
# each under its own time limit, reduced by tools/pmc_traffic.py (gfx950 FETCH_SIZE x2).
# usage: bash tools/gpu_pmc_decode.sh OUT.json
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_decode
mkdir -p $O
OUT=${1:-gpurun_out/pmc_decode/traffic.json}
for m in 7b 13b; do
  timeout -k 10 300 python3 tools/decode_speed.py $m 8 > $O/gen_$m.log 2>&1 || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${m}_$c -o run --output-format csv -- python3 tools/decode_speed.py $m 8 > $O/${m}_$c.log 2>&1 || exit 2
    echo "pmc $m $c done"
  done
done
f() { find $O/$1 -name '*counter_collection.csv' | head -1; }
python3 tools/pmc_traffic.py $OUT 7b:$(f 7b_FETCH_SIZE):$(f 7b_WRITE_SIZE) 13b:$(f 13b_FETCH_SIZE):$(f 13b_WRITE_SIZE) || exit 3
echo pmc-ok
