#!/bin/bash
# Round 6 re-entry, session 5: the default N > 1 line is now C1 per GPU (weak scaling). The self-launched
# two-rank default line (both ranks on the box's one GPU), and the c4g two-rank line with its anchors.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s5; mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { echo "bench2 rc=$?"; tail -20 $O/bench_gpus2.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 --config c4g > $O/bench_gpus2_c4g.json 2> $O/bench_gpus2_c4g.err || { echo "bench2 c4g rc=$?"; tail -20 $O/bench_gpus2_c4g.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_gpus2", "bench_gpus2_c4g"):
    d = json.loads(open(f"gpurun_out/r6s5/{f}.json").read().strip().splitlines()[-1])
    print(f, d["config"]["config"], d["scaling"], d["value"], d["ms_per_step"], d["parity"]["mismatches"], d.get("efficiency_vs_anchor"))
PY
