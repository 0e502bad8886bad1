#!/bin/bash
# Round 6 re-entry, session 3: f2 A/B in one process, outputs asserted equal (experiments build, knob 23):
#   3  the new defaults: four tiles per histogram workgroup, persistent pass-1/pass-2 scatters with the
#      next tile's loads issued ahead, pass 2's digit from h1, k_bk_sortx
#   4  as 3 with k_bk_sortp (one 1024-thread workgroup per CU, the next bucket prefetched)
#   18 as 3 with the one-tile histogram;  19 as 3 with the one-shot scatter grids
# then the sort tests and the f2 bench line on the product library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s3; mkdir -p $O
KVH_LIB=tools/libkvh_exp.so TUNE_KNOB=23 timeout -k 10 300 python -u tools/tune_sort.py 3,4,18,19 > $O/f2_ab.jsonl 2> $O/f2_ab.err || { echo "ab rc=$?"; tail -20 $O/f2_ab.err; exit 1; }
cat $O/f2_ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/sort_tests.txt 2>&1 || { echo "tests rc=$?"; grep -E "^E |FAILED" $O/sort_tests.txt | head; tail -3 $O/sort_tests.txt; exit 1; }
tail -1 $O/sort_tests.txt
timeout -k 10 600 python -u bench.py --config f2 > $O/bench_f2.json 2> $O/bench_f2.err || { echo "bench rc=$?"; tail -20 $O/bench_f2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_f2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'])"
