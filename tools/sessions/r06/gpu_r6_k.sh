#!/bin/bash
# Round-6: 64-byte keys by lane pairs in the product kernels -- the fixed-length
# parity tests, the C64 bench line, and keys per lane under the new loads
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config c64 --steps 20 --warmup 5 --no-anchor > $O/bench_c64.json 2> $O/bench_c64.err || exit 1
python -c "import json;d=json.load(open('$O/bench_c64.json'));print(d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d.get('parity'))"
timeout -k 10 300 python -u tools/c64_kpl.py > $O/kpl.jsonl 2> $O/kpl.err; rc=$?; cat $O/kpl.jsonl; exit $rc
