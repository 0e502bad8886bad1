#!/bin/bash
# Round 6 final, part 1: every bench line under the driver's protocol (W = 5, K = 20, after the settle),
# the default line (c1, with the scaling anchor) and the self-launched two-rank line.
set -o pipefail
O=${1:-gpurun_out/r6g1}; CFGS=${2:-"c1 c2 c3 c4 c64 c4g f1 f2 f3 f4 f4v"}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.log || { echo "bench $c rc=$?"; tail -5 $O/bench_$c.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],r['kernel_ms'],r['frac'],r.get('frac_vs_achievable'),d['parity']['mismatches'],d['parity']['full_compare'])"
done
timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.log || { echo "gpus2 rc=$?"; tail -5 $O/bench_gpus2.log; exit 1; }
cut -c1-300 $O/bench_gpus2.json
