#!/bin/bash
# Round 6: the full GPU suite and smoke again on a fresh box (default copy path), as the driver runs them.
set -o pipefail
O=${1:-gpurun_out/r6h}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "suite rc=$?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -3 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
