# W2 split-chain kernel (LVK_W2_SPLIT=1) ring variants: parity with it on, 7B decode speed
set -o pipefail
mkdir -p gpurun_out
LVK_W2_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "w2_split" > gpurun_out/t_w2s.log 2>&1 || { tail -30 gpurun_out/t_w2s.log; exit 1; }
for v in w2h26 w2h30; do LVK_LIB=$PWD/llama.vk_amd/lib/$v/libllama_vk_amd.so LVK_W2_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "w2_split" >> gpurun_out/t_w2s.log 2>&1 || { tail -30 gpurun_out/t_w2s.log; exit 1; }; done
grep passed gpurun_out/t_w2s.log
timeout -k 10 300 python -u tools/decode_speed.py 7b 256 > gpurun_out/w2s.log 2>&1 || exit 2
LVK_W2_SPLIT=1 timeout -k 10 300 python -u tools/decode_speed.py 7b 256 >> gpurun_out/w2s.log 2>&1 || exit 3
for v in w2h26 w2h30; do LVK_LIB=$PWD/llama.vk_amd/lib/$v/libllama_vk_amd.so LVK_W2_SPLIT=1 timeout -k 10 300 python -u tools/decode_speed.py 7b 256 >> gpurun_out/w2s.log 2>&1 || exit 4; done
grep model gpurun_out/w2s.log | cut -c1-230
