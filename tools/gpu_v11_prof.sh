#!/bin/bash
# k_var11 / k_var11_q kernel times and memory counters on C2 (knob 7 = $1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
V=${1:-40}; O=gpurun_out/v11p_$V; mkdir -p $O
B="python3 tools/check_var11.py --variants $V --rounds 1 --skip-cases"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/run.jsonl 2> $O/trace.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE SQ_WAVES --output-format csv -d $O/mem -o run -- $B > $O/mem.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- $B > $O/wr.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O/mem $O/wr $O/sq > $O/pmc.json || exit 1
python3 - $O <<'PY'
import csv, json, sys
o = sys.argv[1]
pm = json.load(open(o + "/pmc.json"))
for r in csv.DictReader(open(o + "/trace/run_kernel_stats.csv")):
    if "k_var" in r["Name"]:
        k = [v for n, v in pm.items() if n[:40] == r["Name"][:40]]
        x = k[0] if k else {}
        print(r["Name"][:60], r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1),
              {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in x.items()})
PY
