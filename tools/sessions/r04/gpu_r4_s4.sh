#!/bin/bash
# Round-4 session 4: streaming forms (scrambled one-shot).
set -o pipefail
O=${1:-gpurun_out/r4s4}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 240 tools/stream_forms 100000000 500 5 20 > $O/stream_forms.json 2> $O/stream_forms.log || exit 1
python3 -c "import json;[print(f) for f in json.load(open('$O/stream_forms.json'))['forms']]"
