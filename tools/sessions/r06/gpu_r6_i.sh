#!/bin/bash
# Round-6 host sanitizer rerun over the round's new host code (the ticket
# pool's event-ordered reuse and thread-exit return, the exact-order batch
# front end): the round-5 ASan/UBSan and TSan sessions on the round-6 tree
# (`make asan tsan` in the container; take ./tools/asan and ./tools/tsan out
# of .gpurunignore for the call).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/sessions/r05/gpu_r5_asan.sh gpurun_out/r6asan && \
bash tools/sessions/r05/gpu_r5_tsan.sh gpurun_out/r6tsan
