#!/bin/bash
# Round 3: the whole gpu test suite on the box, plus one research-library
# call (tools/libkvh_exp.so answers the research knobs through the hooks).
# usage: tools/gpu_r3_tests.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/r3/tests}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.txt
tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
KVH_LIB=$PWD/tools/libkvh_exp.so timeout -k 10 200 python3 tools/tune_var.py --variants 23,13,26 --rounds 2 > $O/exp_var_ab.json 2> $O/exp_var_ab.log
echo "exp rc=$?"; tail -3 $O/exp_var_ab.json
