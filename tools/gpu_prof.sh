#!/bin/bash
# Profiling session for one workload (run on the GPU box via gpurun).
# usage: tools/gpu_prof.sh <config> <outdir> [extra run_kernel args]
set -o pipefail
CFG=${1:-c1}; OUT=${2:-gpurun_out/prof_$CFG}; shift 2; EXTRA="$@"
export TMPDIR=/tmp
mkdir -p $OUT
R="python3 tools/run_kernel.py --config $CFG --reps 3 $EXTRA"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $R > $OUT/trace.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc1 -o run -- $R > $OUT/pmc1.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL --output-format csv -d $OUT/pmc2 -o run -- $R > $OUT/pmc2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- $R > $OUT/pmc3.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc4 -o run -- $R > $OUT/pmc4.log 2>&1 &&
python3 tools/pmc_summary.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 > $OUT/pmc_summary.json
