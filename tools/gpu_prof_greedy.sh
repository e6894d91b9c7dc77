# rocprofv3 kernel-trace crash in the greedy graph launch: does it depend on the number of
# traced dispatches before it?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp LVK_SEGV_TRACE=1
[ -f /tmp/lvk_bench/llama-7b-q4_0.bin ] || timeout -k 10 300 python3 tools/decode_speed.py 7b 8 > /dev/null
for n in 32 64 128; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pg_$n -o run -- python3 tools/diag_prof_greedy.py graph /tmp/lvk_bench/llama-7b-q4_0.bin 512 $n > gpurun_out/pg_$n.log 2>&1
  rc=$?; echo "steps $n rc=$rc"; grep -E "ok|step 3|done|signal" gpurun_out/pg_$n.log | head -8
  [ $rc -eq 0 ] || exit $rc
done
