#!/bin/bash
# C3 layout A/B + the kv compat GPU test + the C++ paths program
O=${1:-gpurun_out/misc}; cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "kv_compat or cpp_paths" > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
KVH_LIB=$PWD/raikv_amd/libkvh.so timeout -k 10 300 python3 tools/tune.py --n 50000000 --L 32 --arity 4 --rounds 5 --variants "nt=2,4;kpl=1,2,4" > $O/c3_ab.txt 2>&1 || exit 1
cat $O/c3_ab.txt
