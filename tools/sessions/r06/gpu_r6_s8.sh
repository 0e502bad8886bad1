#!/bin/bash
# Round 6 final tree (last session), profiles part A/B: rocprofv3 kernel traces and PMC passes per config
# (tools/make_profiles.sh via gpu_r6_g2.sh), in two calls of four configs (f2 and c64 have their own).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/sessions/r06/gpu_r6_g2.sh gpurun_out/r6s8${1} "${2}" || exit 1
