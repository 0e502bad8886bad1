#!/bin/bash
# Round-5 session 3: exact-order sort after the wave-register chains: GPU sort
# tests + timing.
set -o pipefail
O=${1:-gpurun_out/r5s3}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -x -v --timeout 300 --timeout-method thread -k "ref_order or drop_in" > $O/gpu_sort.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_sort.txt; tail -3 $O/gpu_sort.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/refsort_time.py > $O/refsort_time.jsonl 2> $O/refsort_time.err || exit 1
cat $O/refsort_time.jsonl
