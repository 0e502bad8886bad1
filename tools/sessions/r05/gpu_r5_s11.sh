#!/bin/bash
# Round-5 session 11: the fused tokenize + hash kernel (knob 19 = 2): the
# ingest tests (both kvh_tokenize_hash forms), the A/B on f3's text, and a
# kernel trace of the fused form.
set -o pipefail
O=${1:-gpurun_out/r5s11}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -x -v --timeout 300 --timeout-method thread > $O/gpu_ingest.txt 2>&1
rc=$?; tail -3 $O/gpu_ingest.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_ingest.txt | head -20; exit $rc; }
timeout -k 10 300 python3 tools/th_ab.py 1,2 > $O/th_ab.json 2> $O/th_ab.log || { tail $O/th_ab.log; exit 1; }
cat $O/th_ab.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/th_ab.py 2 > $O/trace.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_stats.csv")))[:8]:
    print("%-50s %5s %9.1f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
