#!/bin/bash
# Round-4 session 7: ticket sizes for k_fixed_q (tests + A/B), copy_peak in the ticket form.
set -o pipefail
O=${1:-gpurun_out/r4s7}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tickets or golden or every" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
ORDERS=0,1,2,3 timeout -k 10 400 python3 tools/order_ab.py > $O/order_ab.jsonl 2> $O/order_ab.log || exit 1
cat $O/order_ab.jsonl
timeout -k 10 120 tools/copy_peak 100000000 500 50 > $O/copy_peak.json 2> $O/copy_peak.log || exit 1
cat $O/copy_peak.json
