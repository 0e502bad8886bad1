#!/bin/bash
# Round-4 session 8: the new defaults (wave tickets up to 32 B, C2 windows in
# address order) -- full gpu suite, per-length order A/B incl. C3, bench
# driver protocol on c1 c2 c3 c4 c64.
set -o pipefail
O=${1:-gpurun_out/r4s8}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
ORDERS=1,2 timeout -k 10 500 python3 tools/order_ab.py > $O/order_ab.jsonl 2> $O/order_ab.log || exit 1
cat $O/order_ab.jsonl
for c in c1 c2 c3 c4 c64; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-e2e --cpu-seconds 4 > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],r['kernel_ms'],r['frac'],r.get('frac_vs_achievable'),d['parity']['mismatches'])"
done
