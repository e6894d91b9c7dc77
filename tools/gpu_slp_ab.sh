#!/bin/bash
# Prompt matmul A/B on one box: the product build against the no-SLP build (scalar v_fma_f32
# chain FMAs instead of v_pk_fma_f32 beside the MFMAs); same logits hash = identical bits.
# usage: tools/gpu_slp_ab.sh <tag> [7b|13b ...]
set -o pipefail
o=$PWD/gpurun_out/$1; shift; mkdir -p $o
for m in "${@:-7b}"; do for rep in 1 2; do
  timeout -k 10 300 python3 tools/prompt_speed.py 512 $m >> $o/prompt_${m}.jsonl 2>>$o/err.log || exit $?
  LVK_LIB=$PWD/llama.vk_amd/lib/mmprobe/libllama_vk_amd.so timeout -k 10 300 python3 tools/prompt_speed.py 512 $m \
      | sed 's/^{/{"build": "noslp", /' >> $o/prompt_${m}.jsonl 2>>$o/err.log || exit $?
done; done
cat $o/prompt_*.jsonl
