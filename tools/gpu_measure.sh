# round-2 measurement batch: kernel-trace summaries (7B bench, 13B and 65B decode) and PMC passes
# (prompt-eval VALU/MFMA issue, decode attention traffic).  Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out/meas
export TMPDIR=/tmp
O=gpurun_out/meas
timeout -k 10 300 python3 tools/decode_speed.py 7b 8 > $O/gen7.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt7 -o run --output-format csv -- python3 bench.py --steps 16 --warmup 4 --no-13b --no-65b --no-cpu-baseline --prompt-evals 1 > $O/kt7.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt13 -o run --output-format csv -- python3 tools/decode_speed.py 13b 16 > $O/kt13.log 2>&1 || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt65 -o run --output-format csv -- python3 tools/decode_speed.py 65b 16 > $O/kt65.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/pmcA -o run --output-format csv -- python3 tools/prompt_once.py > $O/pmcA.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY -d $O/pmcB -o run --output-format csv -- python3 tools/prompt_once.py > $O/pmcB.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcF -o run --output-format csv -- python3 tools/attn_traffic.py 255 > $O/pmcF.log 2>&1 || exit 7
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcW -o run --output-format csv -- python3 tools/attn_traffic.py 255 > $O/pmcW.log 2>&1 || exit 8
python3 tools/pmc_reduce.py $O/pmc_prompt.json $(find $O/pmcA $O/pmcB -name '*counter_collection.csv')
python3 tools/pmc_reduce.py $O/pmc_attn.json $(find $O/pmcF $O/pmcW -name '*counter_collection.csv')
find $O -name '*kernel_stats.csv' | head
echo measure-ok
