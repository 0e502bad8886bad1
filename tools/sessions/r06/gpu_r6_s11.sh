#!/bin/bash
# Round 6 last session: k_spans with each queued span's (offset, length) parked in its own output slot
# (experiments knob 18 = 6) against the product (2): outputs asserted equal over 3 rounds, DRAM reads per arm.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s11; mkdir -p $O
KVH_LIB=tools/libkvh_exp.so timeout -k 10 300 python -u tools/tune_spans.py 2,6 > $O/spans_ab.jsonl 2> $O/spans_ab.err || { echo "ab rc=$?"; tail -20 $O/spans_ab.err; exit 1; }
cat $O/spans_ab.jsonl
for a in 2 6; do
  KVH_LIB=tools/libkvh_exp.so timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $O/pmc$a -o run -- python3 tools/tune_spans.py $a --once > $O/pmc$a.log 2>&1 || { echo "pmc $a rc=$?"; tail -5 $O/pmc$a.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for a in (2, 6):
    f = glob.glob(f"gpurun_out/r6s11/pmc{a}/**/run_counter_collection.csv", recursive=True)
    rows = [r for r in csv.DictReader(open(f[0])) if "k_spans" in r["Kernel_Name"]]
    agg = {}
    for r in rows:
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    v = {k: sum(x) / len(x) for k, x in agg.items()}
    rd = 32 * v["TCC_EA0_RDREQ_DRAM_32B_sum"]; wr = 64 * v["TCC_EA0_WRREQ_64B_sum"] + 32 * (v["TCC_EA0_WRREQ_sum"] - v["TCC_EA0_WRREQ_64B_sum"])
    print(a, "read GB %.3f write GB %.3f" % (rd / 1e9, wr / 1e9), len(rows))
PY
