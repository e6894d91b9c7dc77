set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ggml_graph.py tests/test_gpu_stagelink.py tests/test_gpu_seq_wrap.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r04a_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc_decode.sh gpurun_out/r04_traffic.json
