#!/bin/bash
# Round-5 session 9: the extended streams test (every ticketed entry point
# on hipStreamPerThread threads, in captured graphs, through release).
set -o pipefail
O=${1:-gpurun_out/r5s9}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 ./tests/cpp/streams_gpu > $O/streams.txt 2>&1; rc=$?; cat $O/streams.txt; exit $rc
