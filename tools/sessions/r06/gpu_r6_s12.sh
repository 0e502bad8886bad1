#!/bin/bash
# Round 6 last session, the committed final tree: the whole GPU suite and smoke once more (k_spans' product
# kernels were recompiled with the experiments-only template arms: same instructions, other registers), and
# the f3 and default bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s12; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "suite rc=$?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -3 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for c in f3 c1; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.log || { echo "bench $c rc=$?"; tail -5 $O/bench_$c.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],r['kernel_ms'],r['frac'],d['parity']['mismatches'],d['parity']['full_compare'])"
done
