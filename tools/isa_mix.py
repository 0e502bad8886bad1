#!/usr/bin/env python3
"""Static instruction mix of product kernels, by class (the C2 attribution of
DESIGN.md §3.3): compiles a product source for gfx950 with --save-temps into
a scratch directory and counts, per kernel whose name matches, the VALU
instructions of the AES round (v_perm address, v_bitop3 / v_xor combine,
v_alignbit rotate) against the rest (register moves, selects, 64-bit
address math, funnel shifts, masks, compares).  Static counts: each
instruction once, whatever its dynamic weight.

    python tools/isa_mix.py raikv_amd/csrc/kvh_varlen.hip k_var9
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROUND = {"v_perm_b32": "round: lookup address", "v_bitop3_b32": "round: 3-way XOR", "v_xor_b32_e32": "round/xor",
         "v_xor_b32_e64": "round/xor", "v_alignbit_b32": "round: rotate (NT=2)"}
CLASSES = [("v_mov", "register moves"), ("v_cndmask", "selects"), ("v_cmp", "compares"),
           ("v_lshl_add_u64", "64-bit address math"), ("v_add_co", "64-bit address math"),
           ("v_addc", "64-bit address math"), ("v_alignbyte", "piece funnels"), ("v_and", "masks/shifts"),
           ("v_or", "masks/shifts"), ("v_lsh", "masks/shifts"), ("v_bfe", "masks/shifts"), ("v_add_u32", "int add"),
           ("v_sub", "int add"), ("v_readfirstlane", "uniform moves"), ("v_mbcnt", "ranks"), ("v_mul", "mul")]


def classify(op):
    if op in ROUND:
        return ROUND[op]
    for p, c in CLASSES:
        if op.startswith(p):
            return c
    return "other VALU"


def main():
    src, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-pass-failed",
                        "-I" + os.path.join(ROOT, "include"), "--save-temps", "-c", os.path.abspath(src), "-o",
                        os.path.join(d, "x.o")], cwd=d, check=True, capture_output=True)
        asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
        lines = open(os.path.join(d, asm)).read().splitlines()
    out = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):\s", l)
        if not m or pat not in m.group(1):
            continue
        j = next(k for k in range(i, len(lines)) if "s_endpgm" in lines[k])
        ops = [x.strip().split()[0] for x in lines[i + 1:j]
               if x.strip() and not x.strip().startswith((".", ";")) and not x.strip().endswith(":")]
        valu = [o for o in ops if o.startswith("v_")]
        cls = collections.Counter(classify(o) for o in valu)
        out[m.group(1)[:90]] = {"instructions": len(ops), "valu": len(valu),
                                "ds": sum(o.startswith("ds_") for o in ops),
                                "valu_by_class": dict(cls.most_common())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
