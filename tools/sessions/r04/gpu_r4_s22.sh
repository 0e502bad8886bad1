#!/bin/bash
# Round-4 session 22: tokenizer chunk per wave 16 / 32 / 64 KiB (knob 19 = 1 / 2 / 3):
# ingest tests, f3 A/B under a kernel trace.
# (Ran against a temporary knob 19 = 2 / 3 path, removed after the A/B.)
set -o pipefail
O=${1:-gpurun_out/r4s22}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ingest.py > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
VARY=19:1,2,3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/order_ab.py f3 > $O/f3_tok_ab.jsonl 2> $O/f3_tok_ab.log || exit 1
cut -c1-200 $O/f3_tok_ab.jsonl
python3 - $O/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_tok2" in r["Name"] or "k_spans" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), "ms")
PY
