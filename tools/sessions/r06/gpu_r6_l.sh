#!/bin/bash
# Round-6: C64 at 3 keys per lane (lane-pair loads) under the driver protocol,
# and the load-pattern ablation at 48 B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --config c64 --steps 20 --warmup 5 --no-anchor > $O/bench_c64.json 2> $O/bench_c64.err || exit 1
python -c "import json;d=json.load(open('$O/bench_c64.json'));print(d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['parity']['mismatches'], d['parity']['full_compare'])"
timeout -k 10 300 python -u tools/load_ab.py l48 > $O/load_ab48.jsonl 2> $O/load_ab48.err; rc=$?; cat $O/load_ab48.jsonl; exit $rc
