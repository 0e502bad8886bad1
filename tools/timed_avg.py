#!/usr/bin/env python3
"""Per-kernel average duration over the TIMED dispatches only: rocprofv3's
--stats summary averages every dispatch of a kernel, including bench.py's
500 ms settle phase and warm-up.  This takes the last
`steps` dispatches of each named kernel from run_kernel_trace.csv (bench.py
launches the timed steps last).

    python tools/timed_avg.py <trace_dir> <steps> [name_substring ...]
"""
import csv
import glob
import json
import sys

d, steps = sys.argv[1], int(sys.argv[2])
subs = sys.argv[3:] or ["k_"]
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    if any(s in r["Kernel_Name"] for s in subs):
        by.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for k, v in by.items():
    t = v[-steps:]
    out[k[:120]] = {"dispatches_total": len(v), "timed": len(t), "avg_ns": sum(t) / len(t),
                    "min_ns": min(t), "max_ns": max(t), "avg_ns_all_dispatches": sum(v) / len(v)}
print(json.dumps(out, indent=1))
