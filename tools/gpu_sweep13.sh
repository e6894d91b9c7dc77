#!/bin/bash
# 13B Q4_1 decode launch-shape sweep (lib/sweep, LVK_CFG41 0..3).  usage: tools/gpu_sweep13.sh <tag>
set -o pipefail
o=$PWD/gpurun_out/$1; mkdir -p $o
timeout -k 10 300 python3 tools/decode_speed.py 13b 4 > $o/gen.log 2>&1 || exit $?
for cfg in 0 1 2 3; do
  echo "cfg $cfg $(LVK_LIB=$PWD/llama.vk_amd/lib/sweep/libllama_vk_amd.so LVK_CFG41=$cfg timeout -k 10 200 python3 tools/decode_speed.py 13b 64)" | tee -a $o/summary.txt || exit $?
done
