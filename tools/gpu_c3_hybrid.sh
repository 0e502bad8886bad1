#!/bin/bash
# C3 bitsliced-share A/B (tools/c3_hybrid.py) + LDS/VALU/clock counters per variant.
# usage: tools/gpu_c3_hybrid.sh <outdir> "<variants>"
set -o pipefail
O=$1; V=${2:-prod,0:4:2,125:4:2,250:4:2}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
export KVH_LIB=$PWD/tools/libkvh_exp.so
timeout -k 10 300 python3 tools/c3_hybrid.py --variants "$V" > $O/ab.json 2> $O/ab.log || { tail -5 $O/ab.log; exit 1; }
cat $O/ab.json
for v in ${V//,/ }; do
  tag=${v//:/_}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$tag -o run -- python3 tools/c3_hybrid.py --profile $v > $O/t$tag.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p$tag -o run -- python3 tools/c3_hybrid.py --profile $v > $O/p$tag.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/q$tag -o run -- python3 tools/c3_hybrid.py --profile $v > $O/q$tag.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/p$tag $O/q$tag > $O/pmc$tag.json || exit 1
done
