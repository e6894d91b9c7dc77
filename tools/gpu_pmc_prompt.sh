# PMC passes over two 512-token prompt evals (the MFMA prompt path, tools/prompt_once.py):
# VALU / MFMA issue and busy cycles and wait counts (pass A), L2 hits / misses and L1 -> L2
# read requests (pass B), HBM fetch (pass C) of the prompt kernels.  Each pass has its own
# time limit.  usage: bash tools/gpu_pmc_prompt.sh [7b|13b] OUTDIR
set -o pipefail
M=${1:-7b}
O=${2:-gpurun_out/pmc_prompt_$M}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/prompt_once.py 512 $M > $O/gen.log 2>&1 || exit 1
env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/A -o run --output-format csv -- python3 tools/prompt_once.py 512 $M > $O/A.log 2>&1 || exit 2
echo "pass A done"
env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD -d $O/B -o run --output-format csv -- python3 tools/prompt_once.py 512 $M > $O/B.log 2>&1 || exit 3
echo "pass B done"
env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/C -o run --output-format csv -- python3 tools/prompt_once.py 512 $M > $O/C.log 2>&1 || exit 4
python3 tools/pmc_reduce.py $O/pmc_prompt_$M.json $(find $O/A $O/B $O/C -name '*counter_collection.csv')
echo pmc-ok
