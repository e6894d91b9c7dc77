#!/bin/bash
# 65B decode: prologue order override (LVK_MV_PF applies to every Q4_0 decode shape)
set -o pipefail
o=$PWD/gpurun_out/$1; mkdir -p $o
timeout -k 10 400 python3 tools/decode_speed.py 65b 4 > $o/gen.log 2>&1 || exit $?
for pf in def 5 1 0; do
  if [ $pf = def ]; then r=$(timeout -k 10 200 python3 tools/decode_speed.py 65b 24) || exit 1
  else r=$(LVK_MV_PF=$pf timeout -k 10 200 python3 tools/decode_speed.py 65b 24) || exit 1; fi
  echo "pf $pf $r" | tee -a $o/summary.txt
done
