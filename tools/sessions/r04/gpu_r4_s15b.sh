#!/bin/bash
# Round-4 session 15b: s15's sweep after the C3 knob fallback fix: (tables,
# keys per lane) under wave tickets for the runtime-length kernel and C3.
set -o pipefail
O=${1:-gpurun_out/r4s15b}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
for nt in 4 2; do for k in 1 2 4 8; do
  KNOBS=0=$nt,3=$k ORDERS=2 timeout -k 10 300 python3 tools/order_ab.py 12,20,33,50,c3 >> $O/sweep.jsonl 2>> $O/sweep.log || exit 1
done; done
ORDERS=1,2 timeout -k 10 300 python3 tools/order_ab.py 12,20,33,50,c3 >> $O/sweep.jsonl 2>> $O/sweep.log || exit 1
python3 - $O/sweep.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for sh in dict.fromkeys(r["shape"] for r in rows):
    rs = sorted((r["median_ms"], r["knobs"] or "default", r["order"]) for r in rows if r["shape"] == sh)
    print(sh, " | ".join(f"{k}/{o[:4]} {m:.3f}" for m, k, o in rs[:6]))
PY
