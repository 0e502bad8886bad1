#!/bin/bash
# Round-5 session 13: the tokenizer emit pass with int32 staging (16 KiB of
# LDS, 8 workgroups per CU) against the u64 staging; the ingest tests; an f3
# kernel trace.
set -o pipefail
O=${1:-gpurun_out/r5s13}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 300 --timeout-method thread > $O/gpu_ingest.txt 2>&1
rc=$?; tail -2 $O/gpu_ingest.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_ingest.txt | head; exit $rc; }
timeout -k 10 300 python3 tools/tok_stage_ab.py > $O/stage_ab.json 2> $O/stage_ab.log || { tail $O/stage_ab.log; exit 1; }
cat $O/stage_ab.json
