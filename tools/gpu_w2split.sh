# W2 split-chain kernel (LVK_W2_SPLIT=1): 7B-shaped and full-7B parity with it on, 7B decode speed on/off
set -o pipefail
mkdir -p gpurun_out
LVK_W2_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_7b_full.py -k "7b_shaped_decode or 7b_full_prompt16" > gpurun_out/t_w2s.log 2>&1 || { tail -30 gpurun_out/t_w2s.log; exit 1; }
tail -2 gpurun_out/t_w2s.log
timeout -k 10 300 python -u tools/decode_speed.py 7b 256 > gpurun_out/w2s.log 2>&1 || { tail -20 gpurun_out/w2s.log; exit 2; }
LVK_W2_SPLIT=1 timeout -k 10 300 python -u tools/decode_speed.py 7b 256 >> gpurun_out/w2s.log 2>&1 || { tail -20 gpurun_out/w2s.log; exit 3; }
timeout -k 10 300 python -u tools/decode_speed.py 7b 256 >> gpurun_out/w2s.log 2>&1 || { tail -20 gpurun_out/w2s.log; exit 4; }
LVK_W2_SPLIT=1 timeout -k 10 300 python -u tools/decode_speed.py 7b 256 >> gpurun_out/w2s.log 2>&1 || { tail -20 gpurun_out/w2s.log; exit 5; }
grep model gpurun_out/w2s.log
