# PMC passes over a short 13B Q4_1 decode (tools/decode_speed.py 13b 8): VALU / LDS / wait
# cycles and HBM bytes of the Q4_1 decode kernels.  Each pass has its own time limit.
set -o pipefail
mkdir -p gpurun_out/p13
export TMPDIR=/tmp
O=gpurun_out/p13
timeout -k 10 300 python3 tools/decode_speed.py 13b 8 > $O/gen.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS -d $O/A -o run --output-format csv -- python3 tools/decode_speed.py 13b 8 > $O/A.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $O/B -o run --output-format csv -- python3 tools/decode_speed.py 13b 8 > $O/B.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/F -o run --output-format csv -- python3 tools/decode_speed.py 13b 8 > $O/F.log 2>&1 || exit 4
python3 tools/pmc_reduce.py $O/pmc13.json $(find $O/A $O/B $O/F -name '*counter_collection.csv')
echo pmc-ok
