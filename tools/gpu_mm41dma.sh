# Q4_1 prompt matmul: LDS-DMA ring vs register ring -- op parity, model parity, 13B prompt speed
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "mfma_q4_1" > gpurun_out/t_dma.log 2>&1 || { tail -40 gpurun_out/t_dma.log; exit 1; }
tail -2 gpurun_out/t_dma.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_model.py -k "q4_1" >> gpurun_out/t_dma.log 2>&1 || { tail -40 gpurun_out/t_dma.log; exit 2; }
tail -2 gpurun_out/t_dma.log
timeout -k 10 300 python -u tools/prompt_speed.py 512 13b > gpurun_out/dma41.log 2>&1 || { tail -20 gpurun_out/dma41.log; exit 3; }
LVK_MM41_DMA=0 timeout -k 10 300 python -u tools/prompt_speed.py 512 13b >> gpurun_out/dma41.log 2>&1 || { tail -20 gpurun_out/dma41.log; exit 4; }
grep model gpurun_out/dma41.log
