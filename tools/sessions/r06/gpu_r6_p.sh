#!/bin/bash
# Round-6: 56-byte keys by lane pairs -- parity, before/after A/B at 56 and 64 B, tables x keys per lane at 56 B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  KVH_LIB=tools/ab/libkvh_before.so timeout -k 10 120 python -u tools/len_ab.py before 56 64 >> $O/len_ab.jsonl 2>> $O/len_ab.err || exit 1
  timeout -k 10 120 python -u tools/len_ab.py after 56 64 >> $O/len_ab.jsonl 2>> $O/len_ab.err || exit 1
done
cat $O/len_ab.jsonl
timeout -k 10 400 python -u tools/c64_kpl.py 56 > $O/kpl56.jsonl 2> $O/kpl56.err; rc=$?; cat $O/kpl56.jsonl; exit $rc
