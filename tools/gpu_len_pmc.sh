#!/bin/bash
# The metric's 16-64 B range: per key length, a kernel-trace pass and counter
# passes (SQ LDS/waits + GRBM clock; FETCH_SIZE; WRITE_SIZE) over
# tools/len_sweep.py restricted to that length (100M keys, default kernel
# shape), each its own rocprofv3 run.  usage: tools/gpu_len_pmc.sh <outdir> "16 24 32 48 64"
set -o pipefail
O=$1; LENS=${2:-16 24 32 48 64}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
for L in $LENS; do
  R="python3 tools/len_sweep.py 100000000 $L default"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$L -o run -- $R > $O/t$L.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p$L -o run -- $R > $O/p$L.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$L -o run -- $R > $O/f$L.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$L -o run -- $R > $O/w$L.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/p$L $O/f$L $O/w$L > $O/pmc$L.json || exit 1
done
