#!/bin/bash
# Round-4 session 15: the new fixed-length defaults (all lengths on wave
# tickets; 40/48 B U3, 56/64 B U1) -- parity tests, A/B against the old ones;
# (tables, keys per lane) under tickets for the runtime-length kernel and C3.
set -o pipefail
O=${1:-gpurun_out/r4s15}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
ORDERS=1,0 timeout -k 10 300 python3 tools/order_ab.py 40,48,56,64 > $O/newdef.jsonl 2>> $O/sweep.log || exit 1
for nt in 4 2; do for k in 1 2 4 8; do
  KNOBS=0=$nt,3=$k ORDERS=2 timeout -k 10 300 python3 tools/order_ab.py 12,20,33,50,c3 >> $O/sweep.jsonl 2>> $O/sweep.log || exit 1
done; done
ORDERS=1,2 timeout -k 10 300 python3 tools/order_ab.py 12,20,33,50,c3 >> $O/sweep.jsonl 2>> $O/sweep.log || exit 1
cat $O/newdef.jsonl | cut -c1-200
python3 - $O/sweep.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for sh in dict.fromkeys(r["shape"] for r in rows):
    rs = sorted((r["median_ms"], r["knobs"] or "default", r["order"]) for r in rows if r["shape"] == sh)
    print(sh, " | ".join(f"{k}/{o[:4]} {m:.3f}" for m, k, o in rs[:6]))
PY
