#!/bin/bash
# Round-4 session 26: f1 (fused hash + positions) tables x keys per lane under wave tickets
# (interleaved rounds, outputs asserted equal within each run).  Ran against a temporary
# knob 0 / 3 path in launch_fused (ht_pos.hip), removed after it measured no gain.
set -o pipefail
O=${1:-gpurun_out/r4s26}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
ROUNDS=8 VARY=3:2,1,4 KNOBS=0=2 timeout -k 10 200 python3 tools/order_ab.py f1 >> $O/f1_sweep.jsonl 2>> $O/f1_sweep.log || exit 1
ROUNDS=8 VARY=3:2,1,4 KNOBS=0=4 timeout -k 10 200 python3 tools/order_ab.py f1 >> $O/f1_sweep.jsonl 2>> $O/f1_sweep.log || exit 1
ROUNDS=8 VARY=0:2,4 timeout -k 10 200 python3 tools/order_ab.py f1 >> $O/f1_sweep.jsonl 2>> $O/f1_sweep.log || exit 1
cut -c1-180 $O/f1_sweep.jsonl
