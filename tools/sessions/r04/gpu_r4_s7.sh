#!/bin/bash
# Round-4 session 7: in-order tickets -- k_fixed_q (1/4/16 rounds per ticket)
# and the barrier-free k_fixed_qw (tests + A/B vs the static order), C2 with
# windows in address order (knob 7 = 46), copy_peak in the ticket form.
set -o pipefail
O=${1:-gpurun_out/r4s7}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tickets or golden or every or variants" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
ORDERS=0,1,2,3,4 timeout -k 10 400 python3 tools/order_ab.py > $O/order_ab.jsonl 2> $O/order_ab.log || exit 1
cat $O/order_ab.jsonl
KVH_LIB=raikv_amd/libkvh.so timeout -k 10 300 python3 tools/c2_ab.py --variants 23,46 --rounds 5 > $O/c2_q_ab.jsonl 2> $O/c2_q_ab.log || exit 1
cat $O/c2_q_ab.jsonl
timeout -k 10 120 tools/copy_peak 100000000 500 50 > $O/copy_peak.json 2> $O/copy_peak.log || exit 1
cat $O/copy_peak.json
