# fixed-length checks: parity tests for the fixed-length entry, then the length sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/fixed}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fixed or lengths or unaligned or multiseed" > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.txt; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/len_sweep.py > $O/len_sweep.json 2> $O/len_sweep.err || exit 1
cat $O/len_sweep.json
