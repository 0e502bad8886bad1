#!/bin/bash
# Counter comparison of kernel variants (run on the GPU box): for each
# "name:knob args" pair, one rocprofv3 pass with clock, VALU and LDS counters.
# usage: tools/gpu_clock_cmp.sh <outdir> <config> "name:--knob 11=200 ..." ...
set -o pipefail
OUT=$1; CFG=$2; shift 2
export TMPDIR=/tmp
mkdir -p $OUT
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/$name -o run -- python3 tools/run_kernel.py --config $CFG --reps 3 $args > $OUT/$name.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${name}_t -o run -- python3 tools/run_kernel.py --config $CFG --reps 3 $args > $OUT/${name}_t.log 2>&1 || exit 1
done
for spec in "$@"; do name=${spec%%:*}; python3 tools/pmc_summary.py $OUT/$name > $OUT/${name}_pmc.json; done
