#!/bin/bash
# Round-5 session 4: C2 counter ablations of k_var9:
# per variant time (in-process A/B) + SQ_INSTS_VALU / LDS / waits; the sort
# ablation (61) against the product (46) on input pre-sorted by class.
set -o pipefail
O=${1:-gpurun_out/r5s4}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_c2_pmc.sh $O/mix 46 62,63,64,65,66 || exit 1
export KVH_LIB=$PWD/tools/libkvh_exp.so
timeout -k 10 300 python3 tools/c2_ab.py --variants 46 --ablations 61 --presorted > $O/presorted_ab.json 2> $O/presorted_ab.log || exit 1
cat $O/presorted_ab.json
for v in 46 61; do
  R="python3 tools/run_kernel.py --config c2 --reps 3 --var $v --presorted"
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/ps_q$v -o run -- $R > $O/ps_q$v.log 2>&1 || exit 1
done
