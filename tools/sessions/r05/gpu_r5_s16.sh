#!/bin/bash
# Round-5 session 16: the 128-thread exact-order form (eight sorts per CU)
# against the 256-thread form beyond four batches per CU; the sort tests.
set -o pipefail
O=${1:-gpurun_out/r5s16}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; tail -2 $O/gpu_sort.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_sort.txt | head; exit $rc; }
KVH_LIB=$PWD/tools/libkvh_exp.so timeout -k 10 400 python3 tools/refsort_forms_ab.py > $O/forms_ab.jsonl 2> $O/forms_ab.log || { tail $O/forms_ab.log; exit 1; }
cat $O/forms_ab.jsonl
