"""GPU, world_size 2 over gloo (127.0.0.1): the sharded batch hash through
the product kernels, the way bench.py runs N > 1 (one process per GPU, no
data-path collective).  On the one-GPU box both ranks share cuda:0.

Each rank hashes its index-range shard (fixed length) and its byte-balanced
shard (variable length) of one global batch with libkvh.so; rank 0 gathers
the shards and checks that they are disjoint, cover the batch, and equal the
unsharded batch hashed in one call -- i.e. per-rank outputs are slices of a
single global layout."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    import raikv_amd as kvh
    from raikv_amd import dist as kdist
    from raikv_amd.workload import STATIC_SEED, random_keys, shard_range, shard_var, var_keys
    r, w, local = kdist.env_ranks()
    kdist.init(w)
    torch.cuda.set_device(local % torch.cuda.device_count())
    n, L = 1_000_003, 32
    keys = random_keys(n, L, seed=9)
    lo, hi = shard_range(n, r, w)
    mine = kvh.meow128_fixed(torch.from_numpy(keys[lo * L:hi * L].copy()).cuda(), L, STATIC_SEED).cpu()
    parts = [None] * w
    dist.all_gather_object(parts, (lo, hi, mine.numpy()))
    kb, offs, _ = var_keys(300_007, 8, 256, seed=4)
    vlo, vhi = shard_var(offs, r, w)
    sub = torch.from_numpy(kb[int(offs[vlo]):int(offs[vhi])].copy()).cuda()
    so = torch.from_numpy((offs[vlo:vhi + 1] - offs[vlo]).astype(np.uint64).view(np.int64)).cuda()
    vm = kvh.meow128_var(sub, so, STATIC_SEED).cpu()
    vparts = [None] * w
    dist.all_gather_object(vparts, (vlo, vhi, vm.numpy()))
    kdist.barrier(w)
    mx = kdist.reduce_max(float(r + 1), w)
    if r == 0:
        full = kvh.meow128_fixed(torch.from_numpy(keys).cuda(), L, STATIC_SEED).cpu().numpy()
        ps = sorted(parts, key=lambda p: p[0])
        cover = ps[0][0] == 0 and ps[-1][1] == n and all(a[1] == b[0] for a, b in zip(ps, ps[1:]))
        got = np.concatenate([p[2] for p in ps])
        vfull = kvh.meow128_var(torch.from_numpy(kb).cuda(), torch.from_numpy(offs.view(np.int64)).cuda(),
                                STATIC_SEED).cpu().numpy()
        vps = sorted(vparts, key=lambda p: p[0])
        vcover = vps[0][0] == 0 and vps[-1][1] == len(offs) - 1 and all(a[1] == b[0] for a, b in zip(vps, vps[1:]))
        vgot = np.concatenate([p[2] for p in vps])
        result_q.put((cover and bool(np.array_equal(full, got)), vcover and bool(np.array_equal(vfull, vgot)), mx))
    kdist.finalize(w)


def test_two_ranks_shards_are_slices_of_one_layout():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res == (True, True, 2.0)
