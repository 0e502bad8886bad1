#!/bin/bash
# Round-4 session 20: f2 counters per kernel (where the bucket sort spends its time).
set -o pipefail
O=${1:-gpurun_out/r4s20}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
tools/make_profiles.sh $O/prof f2 || exit 1
python3 - $O/prof/f2/pmc_summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "k_bk" in k or "k_tw" in k:
        g = v.get("GRBM_GUI_ACTIVE", 0)
        print(k[:60], {c: round(x / 1e6, 2) for c, x in v.items() if c != "_dispatches"})
PY
