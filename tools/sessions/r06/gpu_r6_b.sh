#!/bin/bash
# Round 6, session b: the box's counter list (for the gather traffic calibration), the default bench line
# (c1 + the 1-GPU c4g scaling anchor) and the self-launched two-rank line (c4g + efficiency vs anchor).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 120 rocprofv3 --list-avail > $O/counters.txt 2>&1 || echo "list-avail rc=$?"
timeout -k 10 600 python -u bench.py > $O/bench_c1.json 2> $O/bench_c1.err || { echo "bench rc=$?"; tail -20 $O/bench_c1.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { echo "bench2 rc=$?"; tail -20 $O/bench_gpus2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_c1", "bench_gpus2"):
    d = json.loads(open(f"gpurun_out/r6b/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], json.dumps(d.get("scaling_anchor"))[:300], d.get("efficiency_vs_anchor"))
PY
