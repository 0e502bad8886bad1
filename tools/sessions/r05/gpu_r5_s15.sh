#!/bin/bash
# Round-5 session 15: ctest's ingest on the device at f3 size (tokenize_hash,
# then ctest's ~8K-frag batches in the reference's exact order), timed; the
# ingest tests after moving the batch-boundary helper.
set -o pipefail
O=${1:-gpurun_out/r5s15}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 300 --timeout-method thread > $O/gpu_ingest.txt 2>&1
rc=$?; tail -2 $O/gpu_ingest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 tools/ctest_pipeline_time.py > $O/ctest_pipeline.json 2> $O/ctest_pipeline.log || { tail $O/ctest_pipeline.log; exit 1; }
cat $O/ctest_pipeline.json
