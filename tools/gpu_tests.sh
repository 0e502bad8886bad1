cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02/gpu_tests.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/r02/gpu_tests.txt
tail -5 gpurun_out/r02/gpu_tests.txt
