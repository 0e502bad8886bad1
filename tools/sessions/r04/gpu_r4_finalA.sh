#!/bin/bash
# Round-4 measurement, part A: whole gpu suite, smoke, the driver's bench
# protocol per config, the self-launched 2-rank path.
set -o pipefail
O=${1:-gpurun_out/r4finalA}; CFGS=${2:-"c1 c2 c3 c4 c64 c4g f1 f2 f3 f4 f4v"}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
for c in $CFGS; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],r['kernel_ms'],r['frac'],r.get('frac_vs_achievable'),d['parity']['mismatches'])"
done
timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.log || exit 1
cut -c1-300 $O/bench_gpus2.json
