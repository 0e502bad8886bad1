#!/bin/bash
# Round 6 re-entry, session 6: f3's span hash reads 2.1x its text bytes from DRAM (profiles/r06/final/
# f3_pmc_summary.json). A/B of the short path's second text block (experiments knob 18: 2 product, 3 only
# where the span crosses a 16-byte boundary), outputs equal; DRAM read requests per arm (one rocprofv3 pass
# each).  (A first version's arm 4, "always the next block", read past the text buffer's end and faulted.)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s6; mkdir -p $O
export KVH_LIB=tools/libkvh_exp.so
timeout -k 10 300 python -u tools/tune_spans.py 2,3 > $O/spans_ab.jsonl 2> $O/spans_ab.err || { echo "ab rc=$?"; tail -20 $O/spans_ab.err; exit 1; }
cat $O/spans_ab.jsonl
for a in 2 3; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc$a -o run -- python3 tools/tune_spans.py $a --once > $O/pmc$a.log 2>&1 || { echo "pmc $a rc=$?"; tail -5 $O/pmc$a.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, json
for a in (2, 3):
    f = glob.glob(f"gpurun_out/r6s6/pmc{a}/**/run_counter_collection.csv", recursive=True)
    rows = [r for r in csv.DictReader(open(f[0])) if "k_spans" in r["Kernel_Name"]]
    agg = {}
    for r in rows:
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(a, {k: round(sum(v) / len(v) * (32 if "32B" in k else 1) / 1e9, 3) for k, v in agg.items()}, len(rows))
PY
