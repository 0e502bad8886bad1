#!/bin/bash
# Round 3, session 2 start: whole gpu suite + smoke + bench (c1 c2 c64 f2)
# + 2-rank c4g, then the f2 kernel breakdown.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
tools/gpu_round_check.sh gpurun_out/r3s2/check "c1 c2 c64 f2" || exit 1
tools/gpu_f2_prof.sh gpurun_out/r3s2/f2prof
