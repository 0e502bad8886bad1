#!/bin/bash
# C2 kernel A/B + counters (GPU box). usage: tools/gpu_var_ab.sh <outdir> "<variants>" [pytest -k expr]
set -o pipefail
O=${1:-gpurun_out/var_ab}; V=${2:-13,14}; K=${3:-}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.txt 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
fi
KVH_LIB=${KVH_LIB:-$PWD/raikv_amd/libkvh.so} timeout -k 10 300 python3 tools/tune_var.py --variants $V --rounds 5 > $O/ab.json 2> $O/ab.log || exit 1
cat $O/ab.json
for v in ${V//,/ }; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o run -- python3 tools/run_kernel.py --config c2 --reps 3 --var $v > $O/t$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p$v -o run -- python3 tools/run_kernel.py --config c2 --reps 3 --var $v > $O/p$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/q$v -o run -- python3 tools/run_kernel.py --config c2 --reps 3 --var $v > $O/q$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/p$v $O/q$v > $O/pmc$v.json
done
