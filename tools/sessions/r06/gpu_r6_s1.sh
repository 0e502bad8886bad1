#!/bin/bash
# Round 6, re-entry session: the rebuilt tree (C64/C56 lane pairs, table fills eight at a time) through the
# whole GPU suite on the default copy path, smoke, and the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "suite rc=$?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -3 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench_c1.json 2> $O/bench_c1.err || { echo "bench rc=$?"; tail -20 $O/bench_c1.err; exit 1; }
timeout -k 10 600 python -u bench.py --config c64 > $O/bench_c64.json 2> $O/bench_c64.err || { echo "bench c64 rc=$?"; tail -20 $O/bench_c64.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_c1", "bench_c64"):
    d = json.loads(open(f"gpurun_out/r6s1/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"])
PY
