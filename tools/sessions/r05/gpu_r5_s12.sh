#!/bin/bash
# Round-5 session 12: kvh_ht_sort_batched (ctest's batch loop in one launch,
# each batch in the reference's exact order): the sort tests and the timing
# of 1 / 64 / 1024 batches of 16K against the reference on one core.
set -o pipefail
O=${1:-gpurun_out/r5s12}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -x -v --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; tail -3 $O/gpu_sort.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_sort.txt | head -20; exit $rc; }
timeout -k 10 300 python3 tools/refsort_time.py > $O/refsort_time.jsonl 2> $O/refsort_time.log || { tail $O/refsort_time.log; exit 1; }
cat $O/refsort_time.jsonl
