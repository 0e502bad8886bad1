#!/bin/bash
# Round-3 batch: fixed-length kernel shapes incl. the pipelined kernel over
# 16-64 B, host-pipeline tests + latency curves (tiny path), the sort tests
# (two-pass engine), the C2 constant-layout change with counters.
set -o pipefail
O=${1:-gpurun_out/r3/batch}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/len_sweep.py 100000000 16,24,32,40,48,56,64 44,42,41,44p,42p,41p,24p,22p > $O/len_sweep_pl.jsonl 2> $O/len_sweep_pl.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -q --timeout 120 --timeout-method thread > $O/host_tests.txt 2>&1 || { tail -20 $O/host_tests.txt; exit 1; }
timeout -k 10 300 tests/cpp/host_latency 16 pinned 8,64,1024,4096,8192,16384,32768,65536,131072,262144 > $O/lat16_pinned.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 16 pageable 8,64,1024,4096,16384,65536,262144 > $O/lat16_pageable.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 0 pinned 8,64,1024,4096,16384,65536,262144 > $O/latzipf_pinned.jsonl || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort.py -x -v --timeout 300 --timeout-method thread > $O/sort_tests.txt 2>&1 || { tail -30 $O/sort_tests.txt; exit 1; }
tail -2 $O/sort_tests.txt
tools/gpu_c2_pmc.sh $O/c2 "23" "29" || exit 1
