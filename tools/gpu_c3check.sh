#!/bin/bash
O=${1:-gpurun_out/c3check}; cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k "multiseed or c3 or all_lengths or drop_ins" > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config c3 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.log || exit 1
cut -c1-250 $O/bench_c3.json
