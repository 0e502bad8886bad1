#!/bin/bash
# Round-4 rehearsal of the self-launched multi-rank path at N = 4 on the box's one GPU
# (c4g: one global 1B x 32 B batch, four index-range shards sharing cuda:0).
set -o pipefail
O=${1:-gpurun_out/r4ranks4}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python3 bench.py --gpus 4 --steps 10 --warmup 3 > $O/bench_gpus4.json 2> $O/bench_gpus4.log || exit 1
python3 -c "import json;d=json.load(open('$O/bench_gpus4.json'));print(d['n_gpus'],d['value'],d['scaling'],d['config']['config'],[round(p['hashes_per_s']/1e9,1) for p in d['per_gpu']],d['parity'])"
