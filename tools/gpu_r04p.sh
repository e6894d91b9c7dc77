# round 4, GPU call P: the whole -m gpu suite on the round-4 tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04p_gputests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04p_gputests.log | tail -3; grep -E "FAILED|ERROR" gpurun_out/r04p_gputests.log | head -20; exit $rc
