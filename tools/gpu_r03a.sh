set -o pipefail
mkdir -p gpurun_out/r03_a
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "mul_mat or quantize" -p no:cacheprovider > gpurun_out/r03_a/pytest_ops.log 2>&1 || { echo OPSFAIL; tail -30 gpurun_out/r03_a/pytest_ops.log; exit 1; }
tools/gpu_probe.sh r03_a 32 1
