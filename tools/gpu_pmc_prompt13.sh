# PMC passes over two 13B Q4_1 512-token prompt evals (the Q4_1 MFMA path): VALU / MFMA issue
# and busy cycles, LDS and wait counts of k_mm_q41_dma.  Each pass has its own time limit.
set -o pipefail
mkdir -p gpurun_out/pp13
export TMPDIR=/tmp
O=gpurun_out/pp13
timeout -k 10 300 python3 tools/prompt_once.py 512 13b > $O/gen.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/A -o run --output-format csv -- python3 tools/prompt_once.py 512 13b > $O/A.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY -d $O/B -o run --output-format csv -- python3 tools/prompt_once.py 512 13b > $O/B.log 2>&1 || exit 3
python3 tools/pmc_reduce.py $O/pmc_prompt13.json $(find $O/A $O/B -name '*counter_collection.csv')
echo pmc-ok
