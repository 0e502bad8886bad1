#!/bin/bash
# Round-4 session 2: sort tests with scatter2's nt loads (the product now),
# the f2 bench, per-kernel times of both bucket sorts, the extended
# streaming forms and the scatter2 modes incl. 6.
set -o pipefail
O=${1:-gpurun_out/r4s2}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread > $O/sort_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/sort_tests.txt; tail -2 $O/sort_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config f2 --steps 20 --warmup 5 > $O/bench_f2.json 2> $O/bench_f2.log || exit 1
python3 -c "import json;d=json.load(open('$O/bench_f2.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity'])"
TUNE_KNOB=23 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f2_trace -o run -- python3 tools/tune_sort.py 0,1 > $O/f2_trace.log 2>&1 || exit 1
grep median $O/f2_trace.log
timeout -k 10 240 tools/stream_forms 100000000 500 5 20 > $O/stream_forms.json 2> $O/stream_forms.log || exit 1
python3 -c "import json;[print(f) for f in json.load(open('$O/stream_forms.json'))['forms']]"
timeout -k 10 120 tools/scatter2_real 100000000 5 > $O/s2real.json 2> $O/s2real.log || exit 1
cat $O/s2real.json
