#!/bin/bash
# Round-4 session 14: (tables, keys per lane) re-swept under wave tickets for
# every fixed length 8-64 B, static-order defaults alongside.
set -o pipefail
O=${1:-gpurun_out/r4s14}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
S=8,16,24,32,40,48,56,64
ORDERS=1,2 timeout -k 10 300 python3 tools/order_ab.py $S >> $O/sweep.jsonl 2>> $O/sweep.log || exit 1
for nt in 4 2; do for k in 1 2 3 4 8; do
  KNOBS=0=$nt,3=$k ORDERS=2 timeout -k 10 300 python3 tools/order_ab.py $S >> $O/sweep.jsonl 2>> $O/sweep.log || exit 1
done; done
python3 - $O/sweep.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for L in sorted({r["key_len"] for r in rows}):
    rs = sorted((r["median_ms"], r["knobs"] or "default", r["order"]) for r in rows if r["key_len"] == L)
    print(L, " | ".join(f"{k}/{o[:4]} {m:.3f}" for m, k, o in rs[:5]))
PY
