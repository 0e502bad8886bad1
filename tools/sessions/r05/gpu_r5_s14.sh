#!/bin/bash
# Round-5 session 14: kvh_ht_sort_segments (batches of any sizes) and ctest's
# whole ingest pipeline on the device (tokenize_hash -> ctest's batches in the
# reference's exact order with duplicate marking); the sort and ingest tests.
set -o pipefail
O=${1:-gpurun_out/r5s14}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_ingest.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -3 $O/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_tests.txt | head -20; exit $rc; }
grep -E "segments|ctest_pipeline" $O/gpu_tests.txt
