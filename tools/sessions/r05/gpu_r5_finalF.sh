#!/bin/bash
# Round-5 final validation after the DPP tokenizer: the whole gpu suite, smoke,
# every bench line under the driver's protocol, the 2-rank path, then f3's
# profile (kernel trace + PMC passes) refreshed.
set -o pipefail
O=${1:-gpurun_out/r5finalF}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
bash tools/sessions/r05/gpu_r5_finalC.sh $O || exit 1
tools/make_profiles.sh $O/prof f3 || exit 1
python3 tools/timed_avg.py $O/prof/f3/trace 20 > $O/prof/f3/timed_avg.json || exit 1
