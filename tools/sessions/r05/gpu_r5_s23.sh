#!/bin/bash
# Round-5 session 23: f2 with 12 counting-sort bits as the default: the sort
# tests, the driver-protocol f2 line, f2's profile (kernel trace + PMC).
set -o pipefail
O=${1:-gpurun_out/r5s23}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; tail -2 $O/gpu_sort.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config f2 --steps 20 --warmup 5 > $O/bench_f2.json 2> $O/bench_f2.log || exit 1
python3 -c "import json;d=json.load(open('$O/bench_f2.json'));r=d['roofline'];print('f2',d['value'],r['kernel_ms'],r['frac'],d['parity']['mismatches'],d['parity'].get('full_compare'))"
tools/make_profiles.sh $O/prof f2 || exit 1
python3 tools/timed_avg.py $O/prof/f2/trace 20 > $O/prof/f2/timed_avg.json || exit 1
