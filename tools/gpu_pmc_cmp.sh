#!/bin/bash
# Counter comparison of kernel variants (run on the GPU box).  For each
# "name:run_kernel args" spec: a kernel-trace pass and three counter passes
# (SQ timing/LDS/VALU; FETCH_SIZE; WRITE_SIZE), each its own rocprofv3 run.
# usage: tools/gpu_pmc_cmp.sh <outdir> <config> "name:--knob 7=13" ...
set -o pipefail
OUT=$1; CFG=$2; shift 2
export TMPDIR=/tmp
mkdir -p $OUT
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  R="python3 tools/run_kernel.py --config $CFG --reps 3 $args"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name/t -o run -- $R > $OUT/$name.t.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/$name/sq -o run -- $R > $OUT/$name.sq.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$name/f -o run -- $R > $OUT/$name.f.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$name/w -o run -- $R > $OUT/$name.w.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $OUT/$name/sq $OUT/$name/f $OUT/$name/w > $OUT/${name}_pmc.json || exit 1
done
