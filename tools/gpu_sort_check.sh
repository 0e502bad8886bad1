# f2 check: the sort GPU tests, the C++ host-API paths test and the f2 bench.
# usage: tools/gpu_sort_check.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/sort}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -x -v --timeout 120 --timeout-method thread > $O/sort_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/sort_tests.txt; tail -3 $O/sort_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tests/cpp/paths_gpu > $O/paths_gpu.txt 2>&1 || exit $?
tail -1 $O/paths_gpu.txt
timeout -k 10 300 python -u bench.py --config f2 --steps 20 --warmup 5 --no-e2e --no-copy-peak > $O/f2_bench.json 2> $O/f2_bench.err || exit $?
cat $O/f2_bench.json
