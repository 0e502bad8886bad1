#!/bin/bash
# Round-5 session 29: f2 pass-2 tiles found by a binary search in LDS (was ~8
# dependent global loads per workgroup) and the histogram atomics on every lane
# (no load sinks into a branch): the sort and full-size tests, then f2 with the new and the previous
# library (tools/libkvh_prev.so) on one box, twice each, and a kernel trace.
set -o pipefail
O=${1:-gpurun_out/r5s29}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/gpu_sort.txt 2>&1
rc=$?; tail -2 $O/gpu_sort.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_sort.txt | head; exit $rc; }
BF="--steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-copy-peak"
for r in 1 2; do
  for lib in prev new; do
    L=$PWD/raikv_amd/libkvh.so; [ $lib = prev ] && L=$PWD/tools/libkvh_prev.so
    KVH_LIB=$L timeout -k 10 300 python3 bench.py --config f2 $BF > $O/bench_f2_${lib}_$r.json 2> $O/bench_f2_${lib}_$r.log || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_f2_${lib}_$r.json'));print('f2 $lib $r', round(d['ms_per_step'],4), d['roofline']['kernel_ms'], d['parity'].get('mismatches'), d['parity'].get('full_compare'))"
  done
done
for lib in prev new; do
  L=$PWD/raikv_amd/libkvh.so; [ $lib = prev ] && L=$PWD/tools/libkvh_prev.so
  KVH_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$lib -o run -- python3 bench.py --config f2 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-copy-peak > $O/trace_$lib.json 2> $O/trace_$lib.err || exit 1
done
