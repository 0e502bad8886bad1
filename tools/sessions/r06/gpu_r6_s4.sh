#!/bin/bash
# Round 6 re-entry, session 4: after pass 2's digit-from-h1 change, the sort/ingest tests, the f2 bench line
# under the driver's protocol, and f2's rocprofv3 kernel trace + PMC passes (tools/make_profiles.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/sort_tests.txt 2>&1 || { echo "tests rc=$?"; grep -E "^E |FAILED" $O/sort_tests.txt | head; tail -3 $O/sort_tests.txt; exit 1; }
tail -1 $O/sort_tests.txt
timeout -k 10 600 python -u bench.py --config f2 --steps 20 --warmup 5 > $O/bench_f2.json 2> $O/bench_f2.err || { echo "bench rc=$?"; tail -20 $O/bench_f2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_f2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['mismatches'], d['parity']['full_compare'])"
bash tools/sessions/r06/gpu_r6_g2.sh $O/g2 "f2" || { echo "profiles rc=$?"; exit 1; }
