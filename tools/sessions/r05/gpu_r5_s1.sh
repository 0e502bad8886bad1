#!/bin/bash
# Round-5 session 1: ordered ticket fetches, per-stream ticket words, pruned
# product, poisoned outputs.  Pin-reuse probe, the full
# gpu suite without the registration keep-alive, the unordered-fetch demo
# (probe library vs product, once), the default bench line.
set -o pipefail
O=${1:-gpurun_out/r5s1}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 ./tools/pin_reuse_probe 40 > $O/pin_reuse.txt 2>&1; rc=$?; cat $O/pin_reuse.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -3 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
KVH_LIB=tools/libkvh_unordered.so timeout -k 10 300 python3 tools/unordered_demo.py > $O/unordered.jsonl 2> $O/unordered.err || exit 1
timeout -k 10 300 python3 tools/unordered_demo.py >> $O/unordered.jsonl 2>> $O/unordered.err || exit 1
cat $O/unordered.jsonl
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c1.json 2> $O/bench_c1.log || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c1.json'));r=d['roofline'];print('c1',d['value'],r['kernel_ms'],r['frac'],d['parity'])"
