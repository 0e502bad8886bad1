#!/bin/bash
# Host-pipeline latency at raikv's batch sizes (tests/cpp/host_latency), the
# host-pipeline tests, and the 50M-key PCIe-inclusive rate (tests/cpp/e2e_host).
# usage: tools/gpu_host_latency.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/r3/host}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tests/cpp/host_latency 16 pinned > $O/lat_16_pinned.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 16 pageable > $O/lat_16_pageable.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 0 pinned > $O/lat_zipf_pinned.jsonl || exit 1
timeout -k 10 200 tests/cpp/e2e_host 50000000 16 5 > $O/e2e_16.json || exit 1
timeout -k 10 200 tests/cpp/e2e_host 50000000 0 5 > $O/e2e_zipf.json || exit 1
cat $O/lat_16_pinned.jsonl $O/e2e_16.json $O/e2e_zipf.json
