#!/bin/bash
# Round-6 load-pattern ablation at 32 / 64 B (tools/load_ab.py, experiments build)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/r6j; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/load_ab.py ${1:-all} > gpurun_out/r6j/load_ab.jsonl 2> gpurun_out/r6j/load_ab.err
rc=$?; cat gpurun_out/r6j/load_ab.jsonl; tail -5 gpurun_out/r6j/load_ab.err; exit $rc
