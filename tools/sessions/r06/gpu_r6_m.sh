#!/bin/bash
# Round-6: the batched table fill A/B (tools/fill_ab.py), each library in its own process, alternating
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6m; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  KVH_LIB=tools/ab/libkvh_before.so timeout -k 10 200 python -u tools/fill_ab.py before >> $O/fill_ab.jsonl 2>> $O/fill_ab.err || exit 1
  timeout -k 10 200 python -u tools/fill_ab.py after >> $O/fill_ab.jsonl 2>> $O/fill_ab.err || exit 1
done
cat $O/fill_ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_crc.py tests/test_gpu_ingest.py tests/test_gpu_positions.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; tail -3 $O/tests.txt; exit $rc
