#!/bin/bash
# Round 6 re-entry, session 2: k_bk_sortx ranks the PER runs of a thread in one interleaved loop (default)
# against the round-5 serial walk (experiments knob 23 = 16) and pass 2 reading bA (17), f2 workload, outputs asserted equal; then the
# sort tests on the product library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s2; mkdir -p $O
KVH_LIB=tools/libkvh_exp.so TUNE_KNOB=23 timeout -k 10 300 python -u tools/tune_sort.py 3,16,17 > $O/sortx_il_ab.jsonl 2> $O/sortx_il_ab.err || { echo "ab rc=$?"; tail -20 $O/sortx_il_ab.err; exit 1; }
cat $O/sortx_il_ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/sort_tests.txt 2>&1 || { echo "tests rc=$?"; grep -E "^E |FAILED" $O/sort_tests.txt | head; tail -3 $O/sort_tests.txt; exit 1; }
tail -1 $O/sort_tests.txt
timeout -k 10 600 python -u bench.py --config f2 > $O/bench_f2.json 2> $O/bench_f2.err || { echo "bench rc=$?"; tail -20 $O/bench_f2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_f2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'])"
