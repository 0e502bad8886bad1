#!/bin/bash
# Round-5 session 6: full gpu suite on the current tree (stable window sort,
# padded span constants, bucket-sort successor by shuffle); C2 and C1 bench
# lines (driver protocol).
set -o pipefail
O=${1:-gpurun_out/r5s6}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -3 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
for c in c2 c1; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-e2e --cpu-seconds 4 > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],round(d['ms_per_step'],4),r['kernel_ms'],r['frac'],d['parity']['mismatches'],d['parity']['full_compare'])"
done
