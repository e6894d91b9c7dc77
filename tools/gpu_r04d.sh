# round 4, GPU call D: super-tile prompt order parity, the prompt matmul knockout probe
# (tools/probe/mm_probe_expN with the f16 A image), and one full default bench run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py -k "mfma or prompt512 or golden" > gpurun_out/r04d_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r04d_tests.log; [ $rc -eq 0 ] || exit $rc
for e in "" _exp1 _exp2 _exp3 _exp4 _exp8 _exp12 _exp15; do
  echo "== mm_probe$e" >> gpurun_out/r04d_mmprobe.log
  MM_A16=1 timeout -k 10 120 ./tools/probe/mm_probe$e 512 10 >> gpurun_out/r04d_mmprobe.log 2>&1 || exit 3
done
cat gpurun_out/r04d_mmprobe.log | grep -E "==|layer total"
for v in 0 1; do
  for m in 7b 13b; do
    LVK_MM_SUPERTILE=$v timeout -k 10 180 python3 tools/prompt_speed.py 512 $m 2>/dev/null | sed "s/^{/{\"supertile\": $v, /" | tee -a gpurun_out/r04d_prompt.jsonl || exit 4
  done
done
timeout -k 10 900 python3 bench.py > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err
rc=$?; tail -3 gpurun_out/r04d_bench.err; head -c 600 gpurun_out/r04d_bench.json; exit $rc
