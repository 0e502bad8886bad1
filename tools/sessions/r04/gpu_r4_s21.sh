#!/bin/bash
# Round-4 session 21: k_spans with its chunks through wave tickets -- ingest
# and order-knob tests, f3 A/B under a kernel trace, bench f3.
set -o pipefail
O=${1:-gpurun_out/r4s21}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ingest.py tests/test_gpu_parity.py -k "ingest or spans or token or frag or order_knob or tickets" > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
ORDERS=1,2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/order_ab.py f3 > $O/f3_ab.jsonl 2> $O/f3_ab.log || exit 1
cat $O/f3_ab.jsonl
grep -h "k_spans\|k_tok" $O/trace/run_kernel_stats.csv | cut -d, -f1-8
timeout -k 10 300 python3 bench.py --config f3 --steps 20 --warmup 5 --no-e2e --cpu-seconds 4 > $O/bench_f3.json 2> $O/bench_f3.log || exit 1
python3 -c "import json;d=json.load(open('$O/bench_f3.json'));r=d['roofline'];print('f3',d['value'],r['kernel_ms'],r['frac'],d['parity']['mismatches'])"
