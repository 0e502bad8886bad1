"""CPU, world_size 2 over gloo (127.0.0.1): the sharded batch hash.

Each rank hashes its shard (here with the oracle: there is no GPU in this
container; the product kernel is exercised by the gpu tests), the shards are
gathered, and the union must equal the unsharded batch bit-for-bit; the
control-plane helpers bench.py uses (barrier, max-over-ranks) are exercised
on the same group."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_lib import load_oracle, orc_fixed, orc_var
    from raikv_amd import dist as kdist
    from raikv_amd.workload import random_keys, shard_range, shard_var, var_keys, STATIC_SEED
    r, w, _ = kdist.env_ranks()
    kdist.init(w)
    orc = load_oracle()
    # fixed-length shard
    n, L = 10_001, 16
    keys = random_keys(n, L, seed=9)
    lo, hi = shard_range(n, r, w)
    mine = orc_fixed(orc, keys[lo * L:hi * L].copy(), L, STATIC_SEED)
    parts = [None] * w
    dist.all_gather_object(parts, (lo, hi, mine))
    # variable-length shard, byte balanced
    kb, offs, lens = var_keys(5000, 8, 256, seed=4)
    vlo, vhi = shard_var(offs, r, w)
    sub_off = (offs[vlo:vhi + 1] - offs[vlo]).astype(np.uint64)
    vm = orc_var(orc, kb[int(offs[vlo]):int(offs[vhi])].copy(), sub_off, STATIC_SEED)
    vparts = [None] * w
    dist.all_gather_object(vparts, (vlo, vhi, vm))
    kdist.barrier(w)
    mx = kdist.reduce_max(float(r + 1) * 0.5, w)
    if r == 0:
        full = orc_fixed(orc, keys, L, STATIC_SEED)
        got = np.concatenate([p[2] for p in sorted(parts, key=lambda p: p[0])])
        vfull = orc_var(orc, kb, offs, STATIC_SEED)
        vgot = np.concatenate([p[2] for p in sorted(vparts, key=lambda p: p[0])])
        result_q.put((bool(np.array_equal(full, got)), bool(np.array_equal(vfull, vgot)), mx))
    kdist.finalize(w)


def test_world2_gloo_shards_cover_batch_exactly():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] and res[1]
    assert res[2] == 1.0  # max over ranks of (r+1)/2
