# same-box A/B of probe builds: argv = out dir, then binaries; n_past 32 100 264 500, two rounds
set -o pipefail
o=$PWD/gpurun_out/$1; shift; mkdir -p $o
cd tools/probe || exit 1
for rep in 1 2; do for np in 32 100 264 500; do for b in "$@"; do
  timeout -k 10 120 ./$b $np > $o/${b}_${np}_$rep.log 2>&1 || exit $?
  echo "$b $np $rep $(grep -E '^n_past' $o/${b}_${np}_$rep.log) $(grep -E '^  attn' $o/${b}_${np}_$rep.log)"
done; done; done | tee $o/summary.txt
