#!/usr/bin/env python3
"""Compact per-variant table from tools/gpu_c2_pmc.sh output: kernel time
(rocprofv3 kernel-trace stats), LDS bank-conflict share of LDS-array cycles,
LDS busy (LDS-array cycles / (GUI-active cycles x CUs)), share of wave time
waiting, LDS and VALU instructions, FETCH/WRITE bytes (FETCH_SIZE and
WRITE_SIZE are KiB; FETCH as counted, i.e. NOT the x2 streaming correction).
usage: pmc_table.py <dir> <variant>..."""
import csv, glob, json, sys

d = sys.argv[1]
CUS = 256
print(f"{'var':>4} {'kern_ms':>8} {'confl/idx':>9} {'lds_busy':>8} {'wait/wave':>9} {'INSTS_LDS':>10} "
      f"{'INSTS_VALU':>11} {'FETCH_GB':>8} {'WRITE_GB':>8}")
for v in sys.argv[2:]:
    ms = None
    for f in glob.glob(f"{d}/t{v}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_var" in r["Name"] or "k_generic" in r["Name"]:
                ms = float(r["AverageNs"]) / 1e6
    try:
        p = json.load(open(f"{d}/pmc{v}.json"))
    except Exception:
        print(f"{v:>4} (no counters)")
        continue
    k = [x for x in p if "k_var" in x or "k_generic" in x]
    c = p[k[0]] if k else {}
    g = lambda n: c.get(n, float("nan"))
    conf = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    busy = g("SQ_LDS_IDX_ACTIVE") / (g("GRBM_GUI_ACTIVE") * CUS / 8) if g("GRBM_GUI_ACTIVE") else float("nan")
    wait = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
    print(f"{v:>4} {ms if ms else float('nan'):8.3f} {conf:9.3f} {busy:8.3f} {wait:9.3f} {g('SQ_INSTS_LDS'):10.3g} "
          f"{g('SQ_INSTS_VALU'):11.3g} {g('FETCH_SIZE') * 1024 / 1e9:8.3f} {g('WRITE_SIZE') * 1024 / 1e9:8.3f}")
