#!/bin/bash
# Round-5 session 8: f2 bucket sort with two field rounds (16-byte h1/h2
# records) vs the round-4 three rounds (knob 23 = 3 vs 5, experiments build,
# outputs asserted equal); the f2 kernel breakdown; the sort tests; a
# two-rank bench on the one GPU (the N > 1 path).
set -o pipefail
O=${1:-gpurun_out/r5s8}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
KVH_LIB=$PWD/tools/libkvh_exp.so TUNE_KNOB=23 timeout -k 10 400 python3 tools/tune_sort.py 3,5 > $O/f2_w2_ab.json 2> $O/f2_w2_ab.log || { tail $O/f2_w2_ab.log; exit 1; }
cat $O/f2_w2_ab.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; tail -2 $O/gpu_sort.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_f2_prof.sh $O/f2prof || exit 1
timeout -k 10 600 python3 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_gpus2.json 2> $O/bench_gpus2.log || { tail $O/bench_gpus2.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_gpus2.json'));print('gpus2',d['n_gpus'],d['value'],d['config']['config'],d['parity']['mismatches'],d['parity']['full_compare'])"
