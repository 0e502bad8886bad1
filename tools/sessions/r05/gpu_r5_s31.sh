#!/bin/bash
# Round-5 session 31: f4v HBM traffic (FETCH_SIZE, WRITE_SIZE) of the clamped
# group loads against the zero-filled ones, same box, one PMC pass each.
set -o pipefail
O=${1:-gpurun_out/r5s31}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
for lib in prev new; do
  L=$PWD/raikv_amd/libkvh.so; [ $lib = prev ] && L=$PWD/tools/libkvh_prev.so
  KVH_LIB=$L timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$lib -o run -- python3 tools/run_kernel.py --config f4v --reps 5 > $O/fetch_$lib.log 2>&1 || exit 1
  KVH_LIB=$L timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$lib -o run -- python3 tools/run_kernel.py --config f4v --reps 5 > $O/write_$lib.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/fetch_$lib $O/write_$lib > $O/pmc_$lib.json || exit 1
  python3 -c "
import json;d=json.load(open('$O/pmc_$lib.json'))
for k,v in d.items():
  if 'k_crc_var' in k: print('$lib', k[:60], v)"
done
