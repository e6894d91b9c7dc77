#!/bin/bash
# 65B decode W2 launch-shape sweep (lib/sweep, LVK_CFG 0..3 selects the K = 22016 shape; the
# other 65B shapes keep their defaults).  usage: tools/gpu_sweep65.sh <tag>
set -o pipefail
o=$PWD/gpurun_out/$1; mkdir -p $o
timeout -k 10 400 python3 tools/decode_speed.py 65b 4 > $o/gen.log 2>&1 || exit $?
for cfg in 0 1 2 3; do
  echo "cfg $cfg $(LVK_LIB=$PWD/llama.vk_amd/lib/sweep/libllama_vk_amd.so LVK_CFG=$cfg timeout -k 10 200 python3 tools/decode_speed.py 65b 24)" | tee -a $o/summary.txt || exit $?
done
