#!/bin/bash
# Round-6: tables x keys per lane at 64 B under the lane-pair loads (tools/c64_kpl.py)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/c64_kpl.py > $O/kpl.jsonl 2> $O/kpl.err; rc=$?; cat $O/kpl.jsonl; tail -3 $O/kpl.err; exit $rc
