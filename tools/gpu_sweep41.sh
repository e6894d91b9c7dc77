# 13B Q4_1 decode launch-shape sweep (lib/sweep, LVK_CFG41 0..3)
set -o pipefail
o=$PWD/gpurun_out/$1; mkdir -p $o
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 tools/decode_speed.py 13b 8 > $o/gen.log 2>&1 || exit 1
for cfg in 0 1 2 3; do
  LVK_LIB=$PWD/llama.vk_amd/lib/sweep/libllama_vk_amd.so LVK_CFG41=$cfg timeout -k 10 300 python3 tools/decode_speed.py 13b 32 > $o/cfg$cfg.log 2>&1 || exit 2
  tail -1 $o/cfg$cfg.log
done
