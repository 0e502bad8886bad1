#!/bin/bash
# Round-3 final check on the GPU box: whole gpu suite, smoke, the driver's
# bench protocol per config, the 2-rank path, then kernel-trace summaries of
# the bench commands (timed-dispatch averages) and PMC passes.
# usage: tools/gpu_r3_final.sh <outdir> "<bench configs>" "<profile configs>"
set -o pipefail
O=${1:-gpurun_out/r3final}; CFGS=${2:-"c1 c2 c3 c4 c64 c4g f2"}; PCFGS=${3:-"c1 c2 c64"}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
for c in $CFGS; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.log || exit 1
  echo "== $c"; cut -c1-200 $O/bench_$c.json
done
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_c4g_2ranks.json 2> $O/bench_c4g_2ranks.log || exit 1
cut -c1-200 $O/bench_c4g_2ranks.json
tools/make_profiles.sh $O/prof $PCFGS || exit 1
for c in $PCFGS; do python3 tools/timed_avg.py $O/prof/$c/trace 20 > $O/prof/$c/timed_avg.json || exit 1; done
