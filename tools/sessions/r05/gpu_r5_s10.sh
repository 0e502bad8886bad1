#!/bin/bash
# Round-5 session 10: f2 bucket sort with the rank kept from the histogram
# atomic (RK, knob 23 = 3) vs the W2 form before it (knob 23 = 6,
# experiments build, outputs asserted equal); the sort tests; the f2
# kernel breakdown and counters.
set -o pipefail
O=${1:-gpurun_out/r5s10}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
KVH_LIB=$PWD/tools/libkvh_exp.so TUNE_KNOB=23 timeout -k 10 400 python3 tools/tune_sort.py 3,6 > $O/f2_rk_ab.json 2> $O/f2_rk_ab.log || { tail $O/f2_rk_ab.log; exit 1; }
cat $O/f2_rk_ab.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; tail -2 $O/gpu_sort.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_f2_prof.sh $O/f2prof || exit 1
