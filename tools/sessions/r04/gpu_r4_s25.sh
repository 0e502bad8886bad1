#!/bin/bash
# Round-4 session 25: counting-sort bits of the half-size bucket sort (knob 25 = 10 / 11 / 12).
set -o pipefail
O=${1:-gpurun_out/r4s25}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
TUNE_KNOB=25 timeout -k 10 300 python3 tools/tune_sort.py 11,10,12 > $O/f2_hd_ab.jsonl 2> $O/f2_hd_ab.log || exit 1
cat $O/f2_hd_ab.jsonl
