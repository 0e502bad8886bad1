#!/bin/bash
# Memory-side counters (L1->L2 latency, TLB, vmem levels) for C1 and C2 (GPU box).
# usage: tools/gpu_mem_pmc.sh <outdir> "<c2 var knobs>"
set -o pipefail
O=${1:-gpurun_out/mempmc}; VARS=${2:-13}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
P1="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum"
P2="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY"
P3="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
run() {  # name, run_kernel args
  local n=$1; shift
  local i=1
  for P in "$P1" "$P2" "$P3"; do
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/$n/p$i -o run -- python3 tools/run_kernel.py --reps 2 "$@" > $O/$n.p$i.log 2>&1 || return 1
    i=$((i+1))
  done
}
run c1 --config c1 || exit 1
for v in ${VARS//,/ }; do run c2v$v --config c2 --var $v || exit 1; done
echo done
