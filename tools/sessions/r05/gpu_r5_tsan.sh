#!/bin/bash
# Round-5 ThreadSanitizer run on the host code (`make tsan`): the streams
# program (4 host threads on hipStreamPerThread over every ticketed entry
# point, graphs, stream release) and two host pipelines on one device.
# Reports are kept whole; the summary counts them by the module they name.
set -o pipefail
O=${1:-gpurun_out/r5tsan}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
export TSAN_OPTIONS=halt_on_error=0:report_signal_unsafe=0:second_deadlock_stack=1:history_size=4
timeout -k 10 400 stdbuf -oL -eL tools/tsan/streams_gpu > $O/streams.txt 2>&1; echo "streams rc=$?"
timeout -k 10 300 stdbuf -oL -eL tools/tsan/e2e_host 3000001 24 1 0,0 > $O/e2e_multi.txt 2>&1; echo "e2e_multi rc=$?"
for f in streams e2e_multi; do
  echo "== $f: $(grep -c 'WARNING: ThreadSanitizer' $O/$f.txt) reports; success line: $(grep -c '^OK$\|hash_per_s' $O/$f.txt)"
  grep -A14 "WARNING: ThreadSanitizer" $O/$f.txt | grep -o "raikv_amd/csrc/[a-z_]*\.[a-z]*:[0-9]*\|libamdhip64\|libhsa-runtime64\|tests/cpp/[a-z_]*\.cpp:[0-9]*" | sort | uniq -c | sort -rn | head -12
done
