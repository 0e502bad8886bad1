#!/bin/bash
# Round-4 session 17: the re-swept fixed-length defaults (40/48 B U3, 56/64 B
# U1, 32 B and C3 U4, 8 B NT4, wave tickets everywhere): whole gpu suite,
# driver-protocol bench lines and profiles of the configs whose kernel changed.
set -o pipefail
O=${1:-gpurun_out/r4s17}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
for c in c1 c3 c4 c4g c64; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c',d['value'],r['kernel_ms'],r['frac'],r.get('frac_vs_achievable'),d['parity']['mismatches'])"
done
tools/make_profiles.sh $O/prof c3 c4 c64 || exit 1
for c in c3 c4 c64; do python3 tools/timed_avg.py $O/prof/$c/trace 20 > $O/prof/$c/timed_avg.json || exit 1; done
