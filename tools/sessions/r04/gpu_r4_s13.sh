#!/bin/bash
# Round-4 session 13: chunk order x keys per lane at 40 and 64 B (the two
# lengths where wave tickets lost at the default keys per lane).
set -o pipefail
O=${1:-gpurun_out/r4s13}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
for k in 1 2 3 4; do
  KNOBS=3=$k ORDERS=1,2 timeout -k 10 200 python3 tools/order_ab.py 40,64 >> $O/order_kpl.jsonl 2>> $O/order_kpl.log || exit 1
done
cat $O/order_kpl.jsonl
