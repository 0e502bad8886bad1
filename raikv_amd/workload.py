"""Synthetic key sets for the benchmark configs (BASELINE.json `configs`).

All generators are deterministic (numpy PCG64 with a recorded seed).  They
produce host arrays; callers move them to HBM.

* fixed-length keys: uniform random bytes, packed at stride ``key_len``
  (configs C1, C3, C4);
* zipf key lengths: ``len = lo + ZipfianGen<99,100>(hi - lo + 1)``, i.e. the
  YCSB zipfian generator with theta = 0.99 that the reference ports in
  /root/reference/include/raikv/zipf.h:8-81 (rank 0 -> shortest key);
  keys are packed back to back with u64 offsets (config C2);
* ``hash_test`` IntContent keys: consecutive little-endian u64 counters
  (/root/reference/test/hash_test.cpp:54-68).

The default hash seed is raikv's db-0 seed under ``RAIKV_STATIC_RANDOM``
(README.md:130-137), which yields the README's known-answer vector.
"""
from __future__ import annotations

import numpy as np

STATIC_SEED = (0xA8E0BCC94D1855F5, 0xAD3BEC1E8DE4A1A3)
C3_SEEDS = ((1, 2), (3, 4), (5, 6), (7, 8))


def random_keys(n: int, key_len: int, seed: int = 1) -> np.ndarray:
    """n * key_len uniform random bytes (flat uint8)."""
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=n * key_len, dtype=np.uint8)


class ZipfConst:
    """zipf.h:8-33 ZipfianConst, theta = zipf / zipd."""

    def __init__(self, zipf: int, zipd: int, cnt: int):
        self.theta = zipf / zipd
        self.alpha = 1.0 / (1.0 - self.theta)
        self.baseplus1 = 1.0 + 0.5 ** self.theta
        self.item_cnt = cnt
        zeta2 = sum(1.0 / (i + 1) ** self.theta for i in range(2))
        i = np.arange(1, cnt + 1, dtype=np.float64)
        self.zetan = float(np.sum(1.0 / i ** self.theta))
        self.eta = (1 - (2.0 / cnt) ** (1 - self.theta)) / (1 - zeta2 / self.zetan)

    def ranks(self, u: np.ndarray) -> np.ndarray:
        """zipf.h:44-58 ZipfianBuf::gen applied to uniforms u in [0,1)."""
        uz = u * self.zetan
        v = (self.item_cnt * np.power(self.eta * u - self.eta + 1.0, self.alpha)).astype(np.uint64)
        v = np.where(uz < self.baseplus1, np.uint64(1), v)
        v = np.where(uz < 1.0, np.uint64(0), v)
        return v


def zipf_lengths(n: int, lo: int = 8, hi: int = 256, seed: int = 2) -> np.ndarray:
    """Key lengths lo + zipf rank over (hi - lo + 1) items, theta 0.99."""
    zc = ZipfConst(99, 100, hi - lo + 1)
    rng = np.random.default_rng(seed)
    out = np.empty(n, dtype=np.uint32)
    step = 1 << 22
    for s in range(0, n, step):
        e = min(n, s + step)
        r = zc.ranks(rng.random(e - s))
        out[s:e] = np.minimum(r, hi - lo).astype(np.uint32) + lo
    return out


def offsets_from_lengths(lens: np.ndarray) -> np.ndarray:
    offs = np.zeros(len(lens) + 1, dtype=np.uint64)
    np.cumsum(lens, dtype=np.uint64, out=offs[1:])
    return offs


def var_keys(n: int, lo: int = 8, hi: int = 256, seed: int = 3):
    """(flat key bytes, u64 offsets[n+1], lengths) for a zipf-length set."""
    lens = zipf_lengths(n, lo, hi, seed)
    offs = offsets_from_lengths(lens)
    rng = np.random.default_rng(seed + 1000)
    keys = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    return keys, offs, lens


def int_content_keys(n: int, key_len: int = 16, counter0: int = 0) -> np.ndarray:
    """hash_test IntContent: key i = u64 counters counter0 + (key_len//8)*i + j."""
    per = max(1, (key_len + 7) // 8)
    ctr = (np.uint64(counter0) + np.arange(n * per, dtype=np.uint64)).reshape(n, per)
    return ctr.view(np.uint8).reshape(n, per * 8)[:, :key_len].copy().reshape(-1)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous index range of rank `rank` (SURVEY.md §8 e)."""
    return n * rank // world, n * (rank + 1) // world


def shard_var(offs: np.ndarray, rank: int, world: int) -> tuple[int, int]:
    """Key-index range for `rank` that balances key BYTES across ranks."""
    total = int(offs[-1])
    n = len(offs) - 1
    lo = int(np.searchsorted(offs, total * rank // world, side="left")) if rank else 0
    hi = int(np.searchsorted(offs, total * (rank + 1) // world, side="left")) if rank + 1 < world else n
    return min(lo, n), min(hi, n)
