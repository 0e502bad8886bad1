cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r02
KVH_LIB=$PWD/gpurun_old_libkvh.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 250 --timeout-method thread -k "windows" > gpurun_out/r02/wide_old_lib.txt 2>&1
echo "old-lib rc=$?" >> gpurun_out/r02/wide_old_lib.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 250 --timeout-method thread -k "windows" > gpurun_out/r02/wide_new_lib.txt 2>&1
echo "new-lib rc=$?" >> gpurun_out/r02/wide_new_lib.txt
tail -3 gpurun_out/r02/wide_old_lib.txt gpurun_out/r02/wide_new_lib.txt
