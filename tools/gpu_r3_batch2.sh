#!/bin/bash
# Round-3 batch 2: host-pipeline tests + latency curves with the LDS-staged
# tiny kernel (limit 16384 vs off), the sort tests (hot-key three-way
# partition), the C2 constant-layout change with counters.
set -o pipefail
O=${1:-gpurun_out/r3/batch2}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -q --timeout 120 --timeout-method thread > $O/host_tests.txt 2>&1 || { tail -20 $O/host_tests.txt; exit 1; }
tail -1 $O/host_tests.txt
S=8,64,1024,4096,8192,16384,32768,65536,262144
timeout -k 10 300 tests/cpp/host_latency 16 pinned $S > $O/lat16_pinned.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 16 pinned $S 0 > $O/lat16_pinned_notiny.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 0 pinned $S > $O/latzipf_pinned.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 0 pinned $S 0 > $O/latzipf_pinned_notiny.jsonl || exit 1
timeout -k 10 300 tests/cpp/host_latency 16 pageable 8,64,1024,4096,16384,65536,262144 > $O/lat16_pageable.jsonl || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort.py -x -v --timeout 300 --timeout-method thread > $O/sort_tests.txt 2>&1 || { tail -30 $O/sort_tests.txt; exit 1; }
tail -2 $O/sort_tests.txt
tools/gpu_c2_pmc.sh $O/c2 "23" "29" || exit 1
