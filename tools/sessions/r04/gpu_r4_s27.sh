#!/bin/bash
# Round-4 session 27: after the capture check in stream_tickets -- the ticket, host-pipeline
# and multi-rank tests (streams created per pipeline and per rank).
set -o pipefail
O=${1:-gpurun_out/r4s27}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_host.py tests/test_gpu_multirank.py tests/test_gpu_parity.py -k "host or multi or rank or tickets or order_knob or pipeline or device" > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; exit $rc
