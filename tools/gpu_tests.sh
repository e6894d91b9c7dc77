# GPU test run: argv = pytest selection (default: the whole -m gpu suite)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${T:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > gpurun_out/gputests.log 2>&1
rc=$?; tail -25 gpurun_out/gputests.log; exit $rc
