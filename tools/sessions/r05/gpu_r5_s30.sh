#!/bin/bash
# Round-5 session 30: f4v's per-key loop reads the group two ahead clamped to
# the key's last group (one unconditional load: the compiler's wait no longer
# covers the load just issued): the CRC tests, then f4v with the new and the
# previous library (tools/libkvh_prev.so) on one box, twice each.
set -o pipefail
O=${1:-gpurun_out/r5s30}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_crc.py -x -q --timeout 300 --timeout-method thread > $O/gpu_crc.txt 2>&1
rc=$?; tail -2 $O/gpu_crc.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_crc.txt | head; exit $rc; }
BF="--steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-copy-peak"
for r in 1 2; do
  for lib in prev new; do
    L=$PWD/raikv_amd/libkvh.so; [ $lib = prev ] && L=$PWD/tools/libkvh_prev.so
    KVH_LIB=$L timeout -k 10 300 python3 bench.py --config f4v $BF > $O/bench_f4v_${lib}_$r.json 2> $O/bench_f4v_${lib}_$r.log || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_f4v_${lib}_$r.json'));print('f4v $lib $r', round(d['ms_per_step'],4), d['roofline']['kernel_ms'], d['parity'].get('mismatches'), d['parity'].get('full_compare'))"
  done
done
