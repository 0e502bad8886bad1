#!/bin/bash
# Round-5 session 21: f2 bucket-sort phase ablations (experiments build,
# knob 23 = 7 no run insertion sort, 8 no output field rounds, 9 no counting
# sort, 10 no record loads; 3 = the product) -- f2 call time, and the bucket
# sort kernel's own time from a kernel trace.
set -o pipefail
O=${1:-gpurun_out/r5s21}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
KVH_LIB=$PWD/tools/libkvh_exp.so TUNE_KNOB=23 timeout -k 10 400 python3 tools/tune_sort.py 3,7,8,9,10 > $O/f2_ab.json 2> $O/f2_ab.log || { tail $O/f2_ab.log; exit 1; }
cat $O/f2_ab.json
KVH_LIB=$PWD/tools/libkvh_exp.so TUNE_KNOB=23 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/tune_sort.py 3,7,8,9,10 > $O/trace.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_trace.csv")))
c = collections.defaultdict(list)
for r in rows:
    if "k_bk_sortr" in r["Kernel_Name"]:
        name = r["Kernel_Name"]
        c[name[name.index("k_bk_sortr"):name.index("(")]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in c.items():
    v.sort()
    print("%-50s n %3d median %.3f ms" % (k, len(v), v[len(v) // 2] / 1e6))
PY
