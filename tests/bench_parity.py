"""The checker behind bench.py's `parity` field -- TEST INFRASTRUCTURE ONLY.

bench.py calls these after its timed region, on a bounded sample of the
timed launch's own output (default 20 000 keys plus the first and the last),
so that every bench line certifies the bytes it timed.  The expected values
come from the compiled reference (oracle/_ref/libkvref.so: the unmodified
src/key_hash.c, `kv_hash_meow128` key_hash.c:1413-1429, `kv_crc_c_array`
key_hash.c:129-150) when it is present, else from the clean-room oracle port
(oracle/liboracle.so, pinned to the reference's vectors by
tests/test_oracle_golden.py).  The product never imports this module.

Every function takes host numpy arrays and returns
    {"checked": k, "mismatches": m, "against": "reference" | "oracle port" | ...}
so a CPU test can feed it deliberately wrong hashes (tests/test_bench_parity.py).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle_lib import load_oracle, load_ref, orc_positions, crc_sigs

U64 = C.c_uint64


def sample_indices(n: int, k: int = 20_000, seed: int = 0) -> np.ndarray:
    """k distinct indices of [0, n) (all of them when n <= k), always with
    the first and the last key, sorted."""
    if n <= 0:
        return np.zeros(0, np.int64)
    if n <= k + 2:
        return np.arange(n, dtype=np.int64)
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, k, dtype=np.int64)]))
    return idx.astype(np.int64)


def fixup_h1(h1: np.ndarray) -> np.ndarray:
    """KeyCtx::set_key_hash's fixup (key_ctx.cpp:97-105): clear bit 63; 0 and
    1 become 2 (as oracle/ref_cuckoo.cpp:93-94 applies it)."""
    h = np.asarray(h1, dtype=np.uint64) & np.uint64((1 << 63) - 1)
    return np.where(h <= np.uint64(1), np.uint64(2), h)


def _result(exp: np.ndarray, got: np.ndarray, against: str, rows: int) -> dict:
    exp = np.asarray(exp).reshape(rows, -1)
    got = np.asarray(got).reshape(rows, -1)
    bad = ~np.all(exp == got, axis=1) if rows else np.zeros(0, bool)
    res = {"checked": int(rows), "mismatches": int(bad.sum()), "against": against}
    if bad.any():
        res["first_bad_sample_row"] = int(np.argmax(bad))
    return res


def meow_fixed(keys: np.ndarray, key_len: int, out: np.ndarray, seeds, fixup: bool = False) -> dict:
    """keys: (m, key_len) u8, the sampled keys; out: (m, arity, 2) or (m, 2)
    u64, what the device wrote for them; seeds: one (s1, s2) per arity slot
    (kv_hash_meow128_4_same_length_4_seed gives each slot exactly
    kv_hash_meow128 under that slot's seed, key_hash.c:1891-1937)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
    m = keys.size // key_len if key_len else int(np.asarray(out).reshape(-1, 2).shape[0] // max(1, len(seeds)))
    exp = np.zeros((m, len(seeds), 2), np.uint64)
    ref = load_ref()
    kb = keys if keys.size else np.zeros(1, np.uint8)
    for a, (s1, s2) in enumerate(seeds):
        e = np.zeros((m, 2), np.uint64)
        if ref is not None:
            ref.ref_batch_fixed(kb.ctypes.data, key_len, m, U64(s1), U64(s2), e.ctypes.data)
        else:
            load_oracle().orc_batch_fixed(kb.ctypes.data, key_len, m, U64(s1), U64(s2), e.ctypes.data, 0)
        if fixup:
            e[:, 0] = fixup_h1(e[:, 0])
        exp[:, a] = e
    return _result(exp, np.asarray(out, np.uint64), "reference" if ref is not None else "oracle port", m)


def meow_var(key_bytes: np.ndarray, offs: np.ndarray, out: np.ndarray, seed, fixup: bool = False) -> dict:
    """key_bytes + offs (m + 1, local): the sampled keys packed back to back."""
    kb = np.ascontiguousarray(key_bytes, dtype=np.uint8)
    kb = kb if kb.size else np.zeros(1, np.uint8)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    m = o.size - 1
    e = np.zeros((m, 2), np.uint64)
    ref = load_ref()
    if ref is not None:
        ref.ref_batch_var(kb.ctypes.data, o.ctypes.data, m, U64(seed[0]), U64(seed[1]), e.ctypes.data)
    else:
        load_oracle().orc_batch_var(kb.ctypes.data, o.ctypes.data, m, U64(seed[0]), U64(seed[1]), e.ctypes.data, 0)
    if fixup:
        e[:, 0] = fixup_h1(e[:, 0])
    return _result(e, np.asarray(out, np.uint64), "reference" if ref is not None else "oracle port", m)


def crc_var(key_bytes: np.ndarray, offs: np.ndarray, out: np.ndarray, seed: int = 0) -> dict:
    """kv_crc_c of each sampled key (the reference's kv_crc_c_array)."""
    kb = np.ascontiguousarray(key_bytes, dtype=np.uint8)
    kb = kb if kb.size else np.zeros(1, np.uint8)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    m = o.size - 1
    ref = load_ref()
    if ref is not None:
        ref.kv_crc_c_array.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        ptrs = (np.uint64(kb.ctypes.data) + o[:-1]).astype(np.uint64)
        szs = np.diff(o).astype(np.uint64)
        e = np.full(m, seed, dtype=np.uint32)
        if m:
            ref.kv_crc_c_array(ptrs.ctypes.data, szs.ctypes.data, e.ctypes.data, m)
        against = "reference"
    else:
        lib = crc_sigs(load_oracle())
        e = np.zeros(m, np.uint32)
        lib.orc_crc_batch_var(kb.ctypes.data, o.ctypes.data, m, None, seed, e.ctypes.data)
        against = "oracle port"
    return _result(e, np.asarray(out).astype(np.uint32), against, m)


def positions(hashes: np.ndarray, pos: np.ndarray, geom_args) -> dict:
    """cuckoo positions of sampled fixed-up (h1, h2): the oracle's
    CuckooAltHash::calc_hash restatement, pinned to the reference's own
    calc_hash on 11 geometries (tests/golden/cuckoo_*.npz); the reference's
    ref_cuckoo_positions allocates the whole map, which a 64 GiB geometry
    rules out here."""
    from oracle_lib import orc_geom
    lib = load_oracle()
    g = orc_geom(lib, *geom_args)
    h = np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1, 2)
    e = orc_positions(lib, g, h)
    return _result(e, np.asarray(pos, np.uint64), "oracle port (pinned: cuckoo_*.npz)", len(h))


SEPARATORS = (32, 10, 9)  # ' ', '\n', '\t' (ctest.c:202-233)


def spans(tokens, before, after, out: np.ndarray, seed, max_token: int = 256) -> dict:
    """f3: `tokens` are the sampled tokens' bytes, `before` / `after` the text
    byte just outside each one (-1 at the text's ends).  Each must be a
    maximal run of non-separator bytes shorter than max_token (ctest.c:202-233)
    and its hash kv_hash_meow128 over the token and its NUL with the fixup
    (kv_hash_key_frag, key_ctx.cpp:1774-1783)."""
    m = len(tokens)
    sep = np.zeros(256, bool)
    sep[list(SEPARATORS)] = True
    bad_tok = np.zeros(m, bool)
    for k, tok in enumerate(tokens):
        tk = np.asarray(tok, dtype=np.uint8)
        bad_tok[k] = (tk.size == 0 or tk.size >= max_token or sep[tk].any()
                      or (before[k] >= 0 and not sep[before[k]]) or (after[k] >= 0 and not sep[after[k]]))
    kb = (np.concatenate([np.append(np.asarray(t, np.uint8), np.uint8(0)) for t in tokens])
          if m else np.zeros(1, np.uint8))
    lo = np.concatenate([[0], np.cumsum([len(t) + 1 for t in tokens])]).astype(np.uint64)
    r = meow_var(kb, lo, out, seed, fixup=True)
    r["mismatches"] += int(bad_tok.sum())
    r["against"] += " + token boundaries"
    return r


def ht_order(descents: int, perm_ok: bool, pairs_in: np.ndarray, pairs_out: np.ndarray, dups: int,
             zeroed: int, geom_np=None, slots_out: np.ndarray = None) -> dict:
    """f2 by size-independent properties (the serial reference sort of 100M
    pairs is outside a bench line's budget, and its tie order is not the
    device's).  Counted on the device over the whole output:
    `descents` (adjacent slots that decrease), `perm_ok` (items are a
    permutation of 0..n-1), `zeroed` (h1 == 0 entries); here, on a sample:
    each output pair equals the input pair its item names (h1 zeroed for a
    marked duplicate), and, with `geom_np` = (mask, fraction, shift), the
    device's slots equal ht_mod (shm_ht.h:181-184) of the input h1."""
    pi, po = np.asarray(pairs_in, np.uint64).reshape(-1, 2), np.asarray(pairs_out, np.uint64).reshape(-1, 2)
    ok = (pi[:, 1] == po[:, 1]) & ((pi[:, 0] == po[:, 0]) | (po[:, 0] == 0))
    if geom_np is not None and slots_out is not None:
        mask, frac, shift = (np.uint64(x) for x in geom_np)
        with np.errstate(over="ignore"):
            exp = ((pi[:, 0] & mask) * frac) >> shift
        ok &= exp == np.asarray(slots_out, np.uint64)
    bad = int((~ok).sum()) + int(descents) + int(not perm_ok) + int(dups != zeroed)
    return {"checked": int(len(pi)), "mismatches": bad,
            "against": "properties: slot order, item permutation, pair identity, ht_mod, duplicate count"}
