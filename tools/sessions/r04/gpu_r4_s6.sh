#!/bin/bash
# Round-4 session 6: in-order ticket k_fixed_q -- parity tests, A/B vs the
# static order on C1/C4/C64, the driver protocol on c1/c4/c64, sort tests
# with k_bk_sortr as the default.
set -o pipefail
O=${1:-gpurun_out/r4s6}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sort.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/order_ab.py > $O/order_ab.jsonl 2> $O/order_ab.log || exit 1
cat $O/order_ab.jsonl
for c in c1 c4 c64; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-e2e > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['roofline'].get('frac_vs_achievable'),d['parity']['mismatches'])"
done
