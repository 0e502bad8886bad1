#!/bin/bash
# Round-4 session 19: k_bk_sortr with buckets from a ticket counter (knob 23 = 3, buckets in address order):
# sort tests, f2 A/B (1 vs 3), kernel trace of the A/B.
# (Knob 23 = 3 named that temporary variant then; it was removed after the A/B, and 23 = 3 now
# selects the half-size buckets of session 23.)
set -o pipefail
O=${1:-gpurun_out/r4s19}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sort.py > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
TUNE_KNOB=23 timeout -k 10 300 python3 tools/tune_sort.py 1,3 > $O/f2_q_ab.jsonl 2> $O/f2_q_ab.log || exit 1
cat $O/f2_q_ab.jsonl
TUNE_KNOB=23 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/tune_sort.py 1,3 > $O/trace.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
by = {}
for r in rows:
    if "k_bk_sort" in r["Kernel_Name"]:
        by.setdefault(r["Kernel_Name"][:60], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in by.items():
    print(k, len(v), "avg ms", sum(v) / len(v) / 1e6, "min ms", min(v) / 1e6)
PY
