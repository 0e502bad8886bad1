#!/bin/bash
# Round 6, session c: where the wrong bytes of the first probe come from (tools/heap_reuse_probe2.py),
# the bounds-checked build on the sort / ingest tests, then the full GPU suite on the default copy path.
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 python -u tools/heap_reuse_probe2.py 150 > $O/probe2.jsonl 2> $O/probe2.err || { echo "probe2 rc=$?"; tail -5 $O/probe2.err; exit 1; }
KVH_LIB=tools/libkvh_checked.so KVH_ASSERT_CHECKS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_sort.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/checked_tests.txt 2>&1 || { echo "checked rc=$?"; tail -30 $O/checked_tests.txt; exit 1; }
tail -2 $O/checked_tests.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "suite rc=$?"; tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
