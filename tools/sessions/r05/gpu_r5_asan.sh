#!/bin/bash
# Round-5 host sanitizer run: the library's host code under AddressSanitizer
# + UndefinedBehaviorSanitizer (device code as usual; `make asan`), driven by
# the C++ programs: the streams program (threads, graphs, ticket pool,
# release), the PCIe host pipelines (fixed and variable length, one and two
# pipelines), the C++ API of the f1-f4 paths and the hash_test harness.
# A program passes when it prints its own success line and the sanitizers
# report nothing ("ERROR: AddressSanitizer", "runtime error").  One thing is
# let through, after the success line: ASan's device-allocator CHECK that the
# device runtime is still loaded, hit at process exit (the HIP runtime's
# __cxa_finalize, or a worker thread's quarantine flushed after it) -- an
# interaction of the ASan runtime with ROCm's unloading, outside this code.
set -o pipefail
O=${1:-gpurun_out/r5asan}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:print_summary=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
A=tools/asan
run() {  # name, success pattern, limit, command...
  local name=$1 ok=$2 lim=$3; shift 3
  timeout -k 10 $lim stdbuf -oL -eL "$@" > $O/$name.txt 2>&1; local rc=$?
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && { echo "$name: time limit"; return 1; }
  if grep -q "ERROR: AddressSanitizer\|runtime error" $O/$name.txt; then echo "$name: SANITIZER REPORT"; grep -m3 -A12 "ERROR: AddressSanitizer\|runtime error" $O/$name.txt; return 1; fi
  grep -q "$ok" $O/$name.txt || { echo "$name: no success line (rc $rc)"; tail -30 $O/$name.txt; return 1; }
  if [ $rc -ne 0 ]; then
    grep -q 'CHECK failed: sanitizer_allocator_device.h:125 "((!dev_runtime_unloaded_))' $O/$name.txt \
      || { echo "$name: rc $rc"; tail -30 $O/$name.txt; return 1; }
    echo "$name: clean (after main: ASan's device-allocator CHECK, device runtime already unloaded)"
  else
    echo "$name: clean"
  fi
}
run streams "^OK$" 300 $A/streams_gpu || exit 1
run paths "0 failures" 200 $A/paths_gpu || exit 1
run hash_test "0 failures" 200 $A/hash_test_gpu || exit 1
run e2e_16 "hash_per_s" 200 $A/e2e_host 5000000 16 2 || exit 1
run e2e_var "hash_per_s" 200 $A/e2e_host 2000000 0 2 || exit 1
run e2e_multi "hash_per_s" 200 $A/e2e_host 3000001 24 2 0,0 || exit 1
echo "ASAN/UBSAN: all host programs clean"
