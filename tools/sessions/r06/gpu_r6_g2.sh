#!/bin/bash
# Round 6 final, part 2: rocprofv3 kernel-trace summaries of the bench commands and the PMC passes per config
# (tools/make_profiles.sh), and the timed-dispatch averages.
set -o pipefail
O=${1:-gpurun_out/r6g2}; PCFGS=${2:-"c1 c2 c3 c4 c64 f1 f2 f3 f4 f4v"}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
tools/make_profiles.sh $O/prof $PCFGS || exit 1
for c in $PCFGS; do python3 tools/timed_avg.py $O/prof/$c/trace 20 > $O/prof/$c/timed_avg.json || exit 1; done
for c in $PCFGS; do python3 -c "import json;d=json.load(open('$O/prof/$c/timed_avg.json'));[print('$c',k[:60],round(v['avg_ns']/1e6,4)) for k,v in d.items() if v['timed']>=20]"; done
