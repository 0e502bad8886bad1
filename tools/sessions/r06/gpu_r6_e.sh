#!/bin/bash
# Round 6, session e: the stress with registrations on never-unmapped pages (expected clean), the full GPU
# suite and smoke on the runtime's default copy path (no GPU_PINNED_MIN_XFER_SIZE; the registering tests now
# use never-unmapped mappings), then the counter list, the default bench line (c1 + scaling anchor) and the
# self-launched two-rank line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 200 python -u tools/copy_fault_stress.py torch 1200 regmap > $O/stress_torch_regmap.jsonl 2>&1 || { echo "regmap rc=$?"; tail -3 $O/stress_torch_regmap.jsonl; exit 1; }
tail -1 $O/stress_torch_regmap.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "suite rc=$?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -3 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.txt; exit 1; }
timeout -k 10 120 rocprofv3 --list-avail > $O/counters.txt 2>&1 || echo "list-avail rc=$?"
timeout -k 10 600 python -u bench.py > $O/bench_c1.json 2> $O/bench_c1.err || { echo "bench rc=$?"; tail -20 $O/bench_c1.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { echo "bench2 rc=$?"; tail -20 $O/bench_gpus2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_c1", "bench_gpus2"):
    d = json.loads(open(f"gpurun_out/r6e/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], json.dumps(d.get("scaling_anchor"))[:400], d.get("efficiency_vs_anchor"))
PY
