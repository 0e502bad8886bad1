#!/bin/bash
# Round 6 last session: the bench exactly as the driver's default invocation runs it (no flags: C1, K = W = 100,
# cpu_baseline, e2e_pcie, copy peak, scaling anchor), on the committed final tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s13; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench rc=$?"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);r=d['roofline'];c=d['cpu_baseline'];print(d['value'],d['ms_per_step'],r['frac'],r.get('frac_vs_achievable'),c['value'],c['cores'],c['kind'],d['parity']['mismatches'],d['parity']['full_compare'],(d.get('scaling_anchor') or {}).get('hashes_per_s'))"
