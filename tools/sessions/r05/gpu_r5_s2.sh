#!/bin/bash
# Round-5 session 2: the exact-order sort (KVH_REF_ORDER): GPU sort tests,
# timing at ctest batch sizes beside the reference CPU sort; smoke.
set -o pipefail
O=${1:-gpurun_out/r5s2}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -x -v --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_sort.txt; tail -3 $O/gpu_sort.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/refsort_time.py > $O/refsort_time.jsonl 2> $O/refsort_time.err || exit 1
cat $O/refsort_time.jsonl
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; cat $O/smoke.txt; exit $rc
