#!/bin/bash
# Round-5 session 22: the bucket sort with the pairs in LDS through the sort
# (k_bk_sortx, knob 23 = 3) against k_bk_sortr (knob 23 = 11, experiments
# build), outputs asserted equal; the sort tests; f2 kernel breakdown.
set -o pipefail
O=${1:-gpurun_out/r5s22}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; tail -2 $O/gpu_sort.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_sort.txt | head; exit $rc; }
KVH_LIB=$PWD/tools/libkvh_exp.so TUNE_KNOB=23 timeout -k 10 400 python3 tools/tune_sort.py 3,11 > $O/f2_ab.json 2> $O/f2_ab.log || { tail $O/f2_ab.log; exit 1; }
cat $O/f2_ab.json
bash tools/gpu_f2_prof.sh $O/f2prof || exit 1
