#!/bin/bash
# One GPU-box session: the given pytest selection, then bench.py runs.
# usage: tools/gpu_session.sh <tag> "<pytest args>" "<bench config list>"
set -o pipefail
TAG=$1; PT=$2; CFGS=$3
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$PT" ]; then
  timeout -k 10 900 python -u -m pytest $PT -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.txt 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -3 $O/tests.txt
  [ $rc -ne 0 ] && exit $rc
fi
for c in $CFGS; do
  timeout -k 10 400 python3 bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  echo "== $c"; cut -c1-400 $O/bench_$c.json
done
