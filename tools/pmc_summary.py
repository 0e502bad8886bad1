#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs: per-kernel mean of each counter."""
import collections
import csv
import glob
import json
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")
            rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in rows.items():
    out[k[:120]] = {c: sum(v) / len(v) for c, v in cs.items()}
    # dispatches of this kernel in the profiled run (rows of its first counter;
    # one row per dispatch per counter)
    out[k[:120]]["_dispatches"] = max(len(v) for v in cs.values())
print(json.dumps(out, indent=1))
