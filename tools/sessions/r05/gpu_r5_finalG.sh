#!/bin/bash
# Round-5 final validation after the load-order changes (f2 tile kernels and
# bucket sort, k_spans, f4v): the whole gpu suite, smoke, every bench line under
# the driver's protocol, the 2-rank path, then f2 / f3 / f4v profiles
# (kernel trace + PMC passes) refreshed.
set -o pipefail
O=${1:-gpurun_out/r5finalG}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
bash tools/sessions/r05/gpu_r5_finalC.sh $O || exit 1
tools/make_profiles.sh $O/prof f2 f3 f4v || exit 1
for c in f2 f3 f4v; do python3 tools/timed_avg.py $O/prof/$c/trace 20 > $O/prof/$c/timed_avg.json || exit 1; done
