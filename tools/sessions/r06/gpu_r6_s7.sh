#!/bin/bash
# Round 6 final tree (last session): the whole GPU suite and smoke on the runtime's default copy paths, then
# every bench line under the driver's protocol and the self-launched two-rank default line (gpu_r6_g1.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "suite rc=$?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -3 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
bash tools/sessions/r06/gpu_r6_g1.sh $O/final || exit 1
