#!/bin/bash
# End-of-session check on the GPU box: C2 kernel A/B (more rounds), the whole
# gpu test suite, smoke, the driver's bench protocol c1-c4, the 2-rank bench.
# usage: tools/gpu_final.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/final}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
KVH_LIB=$PWD/raikv_amd/libkvh.so timeout -k 10 300 python3 tools/tune_var.py --variants 13,23,25 --rounds 8 > $O/var_ab.json 2> $O/var_ab.log || exit 1
cat $O/var_ab.json
tools/gpu_round_check.sh $O "c1 c2 c3 c4"
