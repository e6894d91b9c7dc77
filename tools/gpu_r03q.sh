# chained greedy decode + step-counter epochs: parity suites touching the decode graph, then the bench
set -o pipefail
o=$PWD/gpurun_out/r03_q; mkdir -p $o
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_decode_chain.py tests/test_gpu_attn_paths.py tests/test_gpu_model.py tests/test_gpu_faults.py \
  tests/test_gpu_sampling.py tests/test_gpu_kvstate.py tests/test_gpu_split.py tests/test_gpu_7b_full.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 900 python3 -u bench.py --no-13b --no-65b --no-cpu-baseline > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 5; }
python3 -c "
import json; d=json.load(open('$o/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step']); g=d.get('decode_greedy_device') or {}
print('greedy', g.get('value'), 'chained', g.get('chained'))"
