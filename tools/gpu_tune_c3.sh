#!/bin/bash
# C3 lanes-kernel layout A/B (product knobs 0 = tables, 3 = keys per lane)
O=${1:-gpurun_out/c3ab}; cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O
KVH_LIB=$PWD/raikv_amd/libkvh.so timeout -k 10 300 python3 tools/tune.py --n 50000000 --L 32 --arity 4 --rounds 5 --variants "nt=2,4;kpl=1,2,4" > $O/c3_ab.txt 2>&1 || exit 1
cat $O/c3_ab.txt
