# round 4, GPU call A: the new parity tests, the decode PMC traffic record, and the one-GPU
# rehearsal of the 65B layer-split bench leg (2 ranks, shm stage link)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ggml_graph.py tests/test_gpu_stagelink.py tests/test_gpu_seq_wrap.py tests/test_gpu_7b_full.py tests/test_gpu_13b_full.py > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r04a_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc_decode.sh gpurun_out/r04_traffic.json || exit 2
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-13b --no-cpu-baseline --split-transport shm \
  > gpurun_out/r04_bench_split_shm_s2.json 2> gpurun_out/r04_split_shm.err
rc=$?; tail -5 gpurun_out/r04_split_shm.err; cat gpurun_out/r04_bench_split_shm_s2.json | head -c 3000; exit $rc
