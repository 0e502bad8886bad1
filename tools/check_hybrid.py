#!/usr/bin/env python3
"""Research check (GPU): the hybrid T-table + bitsliced kernel of the
experiments build (KVH_LIB=tools/libkvh_exp.so, kvh_set_tuning knob 11) is
bit-exact against the oracle, tails included.  Not part of the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("KVH_LIB", os.path.join(ROOT, "tools", "libkvh_exp.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import raikv_amd as kvh  # noqa: E402
from oracle_lib import load_oracle, orc_fixed  # noqa: E402

orc = load_oracle()
for n in (512, 1000, 4099, 1 << 20):
    for share in (200, 1000):
        rng = np.random.default_rng(n + share)
        kb = rng.integers(0, 256, n * 16, dtype=np.uint8)
        seed = (int(rng.integers(0, 2**63)), int(rng.integers(0, 2**63)))
        dk = torch.from_numpy(kb).cuda()
        prev = kvh.lib.kvh_set_tuning(11, share)
        assert prev >= 0
        try:
            for fix in (False, True):
                got = kvh.meow128_fixed(dk, 16, seed, fixup=fix)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64),
                                              orc_fixed(orc, kb, 16, seed, fixup=fix))
        finally:
            kvh.lib.kvh_set_tuning(11, prev)
print("hybrid kernel bit-exact")
