#!/bin/bash
# Round-6: f4v windows staged in LDS (knob 14 = 7) -- CRC tests, then the A/B against knob 14 = 6
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/crc_stg_ab.py > $O/ab.jsonl 2> $O/ab.err; rc=$?; cat $O/ab.jsonl; tail -3 $O/ab.err; exit $rc
