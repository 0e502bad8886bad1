#!/bin/bash
# Round profiling on the GPU box: for each bench config, a rocprofv3
# kernel-trace summary of the bench command itself, plus FETCH_SIZE and
# WRITE_SIZE passes (separate runs, as the MI355X guide prescribes).
# usage: tools/make_profiles.sh <outdir> [configs...]
set -o pipefail
OUT=${1:-gpurun_out/profiles}; shift
CFGS=${@:-c1 c2 c3 c4}
export TMPDIR=/tmp
mkdir -p $OUT
for c in $CFGS; do
  mkdir -p $OUT/$c
  # the driver's protocol (W = 5, K = 20, after the settle phase); no e2e / copy-probe legs
  B="python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-copy-peak --no-anchor"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c/trace -o run -- $B > $OUT/$c/bench.json 2> $OUT/$c/trace.err || exit 1
  R="python3 tools/run_kernel.py --config $c --reps 5"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$c/fetch -o run -- $R > $OUT/$c/fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$c/write -o run -- $R > $OUT/$c/write.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/$c/sq -o run -- $R > $OUT/$c/sq.log 2>&1 || exit 1
  # request-size counters (round 6): DRAM read bytes = 32 x TCC_EA0_RDREQ_DRAM_32B_sum (64-byte requests
  # counted twice, 128-byte four times), so gathers need no calibration; writes by request size
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/$c/rdreq -o run -- $R > $OUT/$c/rdreq.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $OUT/$c/wrreq -o run -- $R > $OUT/$c/wrreq.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $OUT/$c/fetch $OUT/$c/write $OUT/$c/sq $OUT/$c/rdreq $OUT/$c/wrreq > $OUT/$c/pmc_summary.json || exit 1
done
if [ -x tools/fetch_calib ]; then
  mkdir -p $OUT/calib
  for w in stream gather16 gather4; do
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib/$w -o run -- tools/fetch_calib $w 3 > $OUT/calib/$w.log 2>&1 || exit 1
  done
  python3 tools/pmc_summary.py $OUT/calib/stream $OUT/calib/gather16 $OUT/calib/gather4 > $OUT/calib/fetch_calib.json || exit 1
fi
