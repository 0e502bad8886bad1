#!/bin/bash
# Round-4 session 3: bucket sorts 0/1/2 (tests + per-kernel times), streaming
# forms with dynamic chunk assignment.
set -o pipefail
O=${1:-gpurun_out/r4s3}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread > $O/sort_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/sort_tests.txt; tail -2 $O/sort_tests.txt; [ $rc -ne 0 ] && exit $rc
TUNE_KNOB=23 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f2_trace -o run -- python3 tools/tune_sort.py 0,1,2 > $O/f2_trace.log 2>&1 || exit 1
grep median $O/f2_trace.log
python3 -c "
import csv
for r in csv.DictReader(open('$O/f2_trace/run_kernel_stats.csv')):
    n=r['Name']
    if 'k_bk_sort' in n or 'scatter' in n: print(n[:48], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
timeout -k 10 240 tools/stream_forms 100000000 500 5 20 > $O/stream_forms.json 2> $O/stream_forms.log || exit 1
python3 -c "import json;[print(f) for f in json.load(open('$O/stream_forms.json'))['forms']]"
