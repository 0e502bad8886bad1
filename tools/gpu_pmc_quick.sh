#!/bin/bash
# quick clock + LDS utilisation counters for a command: tools/gpu_pmc_quick.sh <outdir> <cmd...>
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc -o run -- "$@" > $OUT/pmc.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1 &&
python3 tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.json
