#!/bin/bash
# Round-4 session 24: C2 under wave tickets with the next block in flight (49: 16 waves; 50: 12 waves)
# against the default (46).
set -o pipefail
O=${1:-gpurun_out/r4s24}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "var" > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
KVH_LIB=raikv_amd/libkvh.so timeout -k 10 300 python3 tools/c2_ab.py --variants 46,49,50 --rounds 8 > $O/c2_ab.jsonl 2> $O/c2_ab.log || exit 1
cat $O/c2_ab.jsonl
