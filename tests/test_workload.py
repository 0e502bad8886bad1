"""CPU: synthetic workload generators and the multi-GPU sharding rules."""
import numpy as np

from raikv_amd.workload import (ZipfConst, int_content_keys, offsets_from_lengths, shard_range, shard_var,
                                var_keys, zipf_lengths)


def test_zipf_lengths_shape_of_c2():
    lens = zipf_lengths(200_000, 8, 256, seed=5)
    assert lens.min() == 8 and lens.max() <= 256
    # SURVEY §8 d: P(8 B) ~ 16 %, median ~ 19 B, mean ~ 48.7 B
    assert 0.13 < np.mean(lens == 8) < 0.19
    assert 14 <= np.median(lens) <= 24
    assert 42 < lens.mean() < 55


def test_zipf_rank_formula_edges():
    zc = ZipfConst(99, 100, 249)
    r = zc.ranks(np.array([0.0, 1e-9, 0.999999]))
    assert r[0] == 0 and r[1] == 0 and r[2] <= 249


def test_offsets_and_var_keys():
    kb, offs, lens = var_keys(1000, 8, 256, seed=1)
    assert offs[0] == 0 and offs[-1] == kb.size and np.all(np.diff(offs.astype(np.int64)) == lens)
    assert offsets_from_lengths(np.array([], dtype=np.uint32)).tolist() == [0]


def test_int_content_keys_match_hash_test_layout():
    k = int_content_keys(3, 16, counter0=10).reshape(3, 16)
    assert k[0, :8].view(np.uint64)[0] == 10 and k[0, 8:].view(np.uint64)[0] == 11
    assert k[2, :8].view(np.uint64)[0] == 14


def test_shards_partition_exactly():
    for n in (0, 1, 7, 1000, 10**9):
        for w in (1, 2, 3, 8):
            ranges = [shard_range(n, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))


def test_var_shards_balance_bytes():
    kb, offs, lens = var_keys(20000, 8, 256, seed=3)
    w = 4
    rs = [shard_var(offs, r, w) for r in range(w)]
    assert rs[0][0] == 0 and rs[-1][1] == 20000
    assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
    b = [int(offs[hi] - offs[lo]) for lo, hi in rs]
    assert max(b) - min(b) < 3 * 256 + 0.02 * sum(b)


def test_c_abi_shard_bounds_match_workload_rules():
    """kvh_shard_bounds (the shard arithmetic of kvh_meow128_*_host_multi,
    host-only) equals workload.shard_range / shard_var, also with a nonzero
    first offset, empty keys, one huge key and more shards than keys."""
    import raikv_amd as kvh
    for n in (0, 1, 2, 7, 1000, 100_003):
        for w in (1, 2, 3, 8):
            b = kvh.shard_bounds(n, w)
            assert [int(x) for x in b] == [shard_range(n, r, w)[0] for r in range(w)] + [n]
    rng = np.random.default_rng(0)
    for n in (1, 5, 999, 50_000):
        lens = rng.integers(0, 300, n)
        if n > 10:
            lens[n // 3] = 10_000_000
            lens[: n // 10] = 0
        offs = offsets_from_lengths(lens)
        for w in (1, 2, 3, 8, 16):
            b = [int(x) for x in kvh.shard_bounds(n, w, offs)]
            assert b == [shard_var(offs, r, w)[0] for r in range(w)] + [n], (n, w)
            assert all(b[i] <= b[i + 1] for i in range(w))
            # a nonzero first offset (a slice of a bigger buffer) shifts nothing
            b2 = [int(x) for x in kvh.shard_bounds(n, w, offs + np.uint64(12345))]
            assert b2 == b
