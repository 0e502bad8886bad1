#!/bin/bash
# C2 variants: in-process A/B (tools/c2_ab.py), then per variant a kernel-trace
# pass and counter passes (LDS / waits; FETCH_SIZE; WRITE_SIZE), each its own
# rocprofv3 run.  usage: tools/gpu_c2_pmc.sh <outdir> "<hash variants>" "<ablation variants>" [lib]
set -o pipefail
O=$1; V=$2; A=$3; LIB=${4:-tools/libkvh_exp.so}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
export KVH_LIB=$PWD/$LIB
timeout -k 10 300 python3 tools/c2_ab.py --variants "$V" --ablations "$A" > $O/ab.json 2> $O/ab.log || { tail -5 $O/ab.log; exit 1; }
cat $O/ab.json
for v in ${V//,/ } ${A//,/ }; do
  R="python3 tools/run_kernel.py --config c2 --reps 3 --var $v"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o run -- $R > $O/t$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p$v -o run -- $R > $O/p$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/q$v -o run -- $R > $O/q$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$v -o run -- $R > $O/f$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$v -o run -- $R > $O/w$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/p$v $O/q$v $O/f$v $O/w$v > $O/pmc$v.json || exit 1
done
python3 tools/pmc_table.py $O ${V//,/ } ${A//,/ } > $O/table.txt; cat $O/table.txt
