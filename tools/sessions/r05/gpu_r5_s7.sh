#!/bin/bash
# Round-5 session 7: C2 quad-coalescing ablation (70) against 46, 68, 67.
set -o pipefail
O=${1:-gpurun_out/r5s7}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
KVH_LIB=$PWD/tools/libkvh_exp.so timeout -k 10 400 python3 tools/c2_ab.py --variants 46 --ablations 70,68,67 --rounds 6 > $O/c2_ab.json 2> $O/c2_ab.log || { tail $O/c2_ab.log; exit 1; }
cat $O/c2_ab.json
