#!/bin/bash
# Round 6 last session: rehearsal of the driver's multi-rank default line with four ranks (self-launched,
# all on the box's one GPU; the N = 8 case is the driver's alone).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s9; mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_gpus4.json 2> $O/bench_gpus4.err || { echo "bench4 rc=$?"; tail -20 $O/bench_gpus4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_gpus4.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['scaling'], d['config']['config'], d['value'], d['ms_per_step'], d['parity']['checked'], d['parity']['mismatches'], [round(p['hashes_per_s']/1e9,1) for p in d.get('per_gpu', [])])"
