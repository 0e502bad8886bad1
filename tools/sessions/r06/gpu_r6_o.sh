#!/bin/bash
# Round-6: C64 with the lane-pair loads -- the driver-protocol bench line and the rocprofv3 passes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
bash tools/sessions/r06/gpu_r6_g1.sh gpurun_out/r6o/g1 "c64" && bash tools/sessions/r06/gpu_r6_g2.sh gpurun_out/r6o/g2 "c64"
