#!/bin/bash
# Round-4 session 16: close A/Bs of the near ties in the s14/s15b sweeps
# (12 interleaved rounds): keys per lane 2 vs 4 at C3 and 32 B; tables 2 vs 4 at 8 B.
set -o pipefail
O=${1:-gpurun_out/r4s16}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
ROUNDS=12 VARY=3:2,4 timeout -k 10 300 python3 tools/order_ab.py c3,32 >> $O/ab.jsonl 2>> $O/ab.log || exit 1
ROUNDS=12 VARY=0:2,4 timeout -k 10 300 python3 tools/order_ab.py 8 >> $O/ab.jsonl 2>> $O/ab.log || exit 1
cut -c1-200 $O/ab.jsonl
