#!/bin/bash
# Round 6, session a: heap-reuse probe of the runtime's locked-user-page copy path, the bounds-checked
# build on the sort / ingest tests, then the full GPU suite on the runtime's default copy path.
set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 300 python -u tools/heap_reuse_probe.py 300 > $O/heap_probe.jsonl 2> $O/heap_probe.err || { echo "probe rc=$?"; exit 1; }
AMD_LOG_LEVEL=4 timeout -k 10 180 python -u tools/heap_reuse_probe.py 2 > $O/heap_probe_log4.jsonl 2> $O/heap_probe_log4.raw || { echo "probe log rc=$?"; exit 1; }
grep -E "PROBE|Locking|nlock|Pinned resource|Staging resource|rror" $O/heap_probe_log4.raw > $O/heap_probe_log4.txt; rm -f $O/heap_probe_log4.raw
KVH_LIB=tools/libkvh_checked.so KVH_ASSERT_CHECKS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_sort.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/checked_tests.txt 2>&1 || { echo "checked rc=$?"; tail -30 $O/checked_tests.txt; exit 1; }
tail -3 $O/checked_tests.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "suite rc=$?"; tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
