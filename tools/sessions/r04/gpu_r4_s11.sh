#!/bin/bash
# Round-4 session 11: wave tickets in k_fixed_rt and k_crc_var_sorted --
# their tests, then the order A/B on the runtime lengths and f4v.
set -o pipefail
O=${1:-gpurun_out/r4s11}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_crc.py tests/test_gpu_positions.py > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
ORDERS=1,2 timeout -k 10 400 python3 tools/order_ab.py 20,33,50,f4v,f1p > $O/order_ab.jsonl 2> $O/order_ab.log || exit 1
cat $O/order_ab.jsonl
