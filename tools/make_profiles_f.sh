#!/bin/bash
# Round profiling of the f rows on the GPU box: a rocprofv3 kernel-trace
# summary of the bench command (the driver's protocol) and FETCH_SIZE /
# WRITE_SIZE passes over a short bench run (separate runs, as the MI355X
# guide prescribes).  usage: tools/make_profiles_f.sh <outdir> [configs...]
set -o pipefail
OUT=${1:-gpurun_out/profiles_f}; shift
CFGS=${@:-f1 f1p f2 f3 f4 f4v}
export TMPDIR=/tmp
mkdir -p $OUT
for c in $CFGS; do
  mkdir -p $OUT/$c
  B="python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-copy-peak"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c/trace -o run -- $B > $OUT/$c/bench.json 2> $OUT/$c/trace.err || exit 1
  R="python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-copy-peak --settle-ms 0"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$c/fetch -o run -- $R > $OUT/$c/fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$c/write -o run -- $R > $OUT/$c/write.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $OUT/$c/fetch $OUT/$c/write > $OUT/$c/pmc_summary.json || exit 1
  echo "== $c"; cut -c1-200 $OUT/$c/bench.json
done
