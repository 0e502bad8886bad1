"""PROBE, run once: the round-4 unordered ticket fetches
(tools/libkvh_unordered.so, tickets.hpp built with KVH_TICKETS_UNORDERED)
against the product's ordered fetches (raikv_amd/libkvh.so), both with the
knob-26 fetch delay, on ragged sizes into poisoned outputs: counts the
launches whose output differs from the static-order kernel (knob 24 = 1),
i.e. chunks no wave hashed.  One JSON line per library.

  KVH_LIB=tools/libkvh_unordered.so python3 tools/unordered_demo.py
  python3 tools/unordered_demo.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KVH_POISON_OUTPUTS"] = "1"
import raikv_amd as kvh  # noqa: E402

SEED = (0xA8E0BCC94D1855F5, 0xAD3BEC1E8DE4A1A3)
delay = int(os.environ.get("DELAY", "6"))
g = torch.Generator(device="cuda")
g.manual_seed(5)
keys = torch.randint(0, 256, (3_000_000 * 16,), dtype=torch.uint8, device="cuda", generator=g)
rng = np.random.default_rng(1)
sizes = sorted(set(int(x) for x in rng.integers(4096, 3_000_000, 60)))
bad_launches, bad_keys, launches = 0, 0, 0
for n in sizes:
    prev = kvh.lib.kvh_set_tuning(24, 1)
    want = kvh.meow128_fixed(keys[:n * 16], 16, SEED)
    kvh.lib.kvh_set_tuning(24, prev)
    pd = kvh.lib.kvh_set_tuning(26, delay)
    for _ in range(5):
        got = kvh.meow128_fixed(keys[:n * 16], 16, SEED)
        torch.cuda.synchronize()
        d = int((got != want).any(1).sum())
        launches += 1
        bad_launches += d > 0
        bad_keys += d
    kvh.lib.kvh_set_tuning(26, pd)
print(json.dumps({"lib": os.path.basename(kvh.binding.lib_path), "delay_knob": delay, "launches": launches,
                  "sizes": len(sizes), "launches_with_unhashed_keys": bad_launches, "unhashed_keys": bad_keys}))
