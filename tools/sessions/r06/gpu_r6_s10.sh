#!/bin/bash
# Round 6 last session: (1) where k_spans' excess DRAM reads come from (4.65 GB read for 3.5 GB of
# offsets, lengths and text): traffic ablations of the short path's text loads (experiments knob 18: 2
# product, 4 first block only, 5 no text loads; 4 and 5 do not produce hashes), one rocprofv3 pass each;
# (2) rehearsal of the driver's multi-rank default line with four ranks on the box's one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s10; mkdir -p $O
KVH_LIB=tools/libkvh_exp.so timeout -k 10 300 python -u tools/tune_spans.py 2,4,5 > $O/spans_ab.jsonl 2> $O/spans_ab.err || { echo "ab rc=$?"; tail -20 $O/spans_ab.err; exit 1; }
cat $O/spans_ab.jsonl
for a in 2 4 5; do
  KVH_LIB=tools/libkvh_exp.so timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc$a -o run -- python3 tools/tune_spans.py $a --once > $O/pmc$a.log 2>&1 || { echo "pmc $a rc=$?"; tail -5 $O/pmc$a.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for a in (2, 4, 5):
    f = glob.glob(f"gpurun_out/r6s10/pmc{a}/**/run_counter_collection.csv", recursive=True)
    rows = [r for r in csv.DictReader(open(f[0])) if "k_spans" in r["Kernel_Name"]]
    agg = {}
    for r in rows:
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(a, {k: round(sum(v) / len(v) * (32 if "32B" in k else 1) / 1e9, 3) for k, v in agg.items()}, len(rows))
PY
bash tools/sessions/r06/gpu_r6_s9.sh || exit 1
