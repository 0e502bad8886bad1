#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container (where /root/reference exists) after
`make -C oracle` has compiled the unmodified reference src/key_hash.c into
oracle/_ref/libkvref.so.  Every expected output below is produced by the
reference's own functions (kv_hash_meow128 and its batched / streaming /
vec variants, key_hash.c:1413-2020); the inputs are our own seeded random
data.  The fixtures are data only (inputs + expected outputs).

    python tests/golden/make_golden.py [--only-cuckoo | --only-crc | --only-ingest | --only-sort |
                                        --only-partition4]

The table-position fixtures (cuckoo_*.npz) come from the reference's
ht_init.cpp + ht_cuckoo.cpp compiled where they lie into
oracle/_ref/libkvref_ht.so (oracle/ref_cuckoo.cpp drives
CuckooAltHash::calc_hash).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from raikv_amd.workload import STATIC_SEED, C3_SEEDS, int_content_keys, var_keys  # noqa: E402

U64 = C.c_uint64
P = C.c_void_p


def load_ref():
    path = os.path.join(ROOT, "oracle", "_ref", "libkvref.so")
    lib = C.CDLL(path)
    lib.kv_hash_meow128.argtypes = [P, C.c_size_t, C.POINTER(U64), C.POINTER(U64)]
    lib.kv_hash_meow64.argtypes = [P, C.c_size_t, U64]
    lib.kv_hash_meow64.restype = U64
    lib.ref_batch_fixed.argtypes = [P, C.c_size_t, C.c_size_t, U64, U64, P]
    lib.ref_batch_var.argtypes = [P, P, C.c_size_t, U64, U64, P]
    lib.ref_batch_4seed.argtypes = [P, C.c_size_t, C.c_size_t, P, P]
    S = C.c_size_t
    lib.kv_hash_meow128_2_same_length.argtypes = [P, P, S, P]
    lib.kv_hash_meow128_2_diff_length.argtypes = [P, S, P, S, P]
    lib.kv_hash_meow128_4_same_length.argtypes = [P, P, P, P, S, P]
    lib.kv_hash_meow128_4_diff_length.argtypes = [P, S, P, S, P, S, P, S, P]
    lib.kv_hash_meow128_8_same_length_a.argtypes = [P, S, P]
    lib.kv_hash_meow128_4_same_length_4_seed.argtypes = [P, P, P, P, S, P]
    lib.kv_hash_meow128_vec.argtypes = [P, S, C.POINTER(U64), C.POINTER(U64)]
    lib.kv_meow_test.argtypes = [P, S, C.POINTER(U64), C.POINTER(U64)]
    return lib


def addr(obj, off=0):
    return P(C.addressof(obj) + off)


def ptr(a: np.ndarray):
    return a.ctypes.data_as(P)


def meow(lib, b: bytes, s1: int, s2: int):
    h1, h2 = U64(s1), U64(s2)
    buf = C.create_string_buffer(b, max(1, len(b)))
    lib.kv_hash_meow128(buf, len(b), C.byref(h1), C.byref(h2))
    return h1.value, h2.value


def hexpair(h):
    return "%016x:%016x" % h


def main():
    lib = load_ref()
    out = {}

    # ---- known answers (SURVEY.md §8 c, README.md:130-137)
    kat = []
    ramp = bytes(range(256))
    for L, s in [(0, (0, 0)), (16, (0, 0)), (16, (1010, 2020)), (32, (0, 0)), (64, (0, 0)),
                 (65, (0, 0)), (256, (0, 0))]:
        kat.append({"key_hex": ramp[:L].hex(), "seed": list(s), "h": hexpair(meow(lib, ramp[:L], *s))})
    for text, s in [(b"security is for the messaging la", (1010, 2020)), (b"hello\0", STATIC_SEED)]:
        kat.append({"key_hex": text.hex(), "seed": list(s), "h": hexpair(meow(lib, text, *s))})
    out["kat"] = kat

    # ---- hash_test.cpp:319-403 cross-variant set, computed by each reference variant
    ar = [b"security is for the messaging la", b"authenticate the publisher to th",
          b"subscribers must be able to trus", b"uniquely serialized, and authent"]
    L = len(ar[0])
    bufs = [C.create_string_buffer(a, L) for a in ar]
    seed = (1010, 2020)
    variants = {}
    variants["single"] = [list(meow(lib, a, *seed)) for a in ar]
    x = (U64 * 8)(*([seed[0], seed[1]] * 4))
    lib.kv_hash_meow128_2_same_length(bufs[0], bufs[1], C.c_size_t(L), x)
    lib.kv_hash_meow128_2_same_length(bufs[2], bufs[3], C.c_size_t(L), addr(x, 32))
    variants["2_same"] = list(x)
    x = (U64 * 8)(*([seed[0], seed[1]] * 4))
    lib.kv_hash_meow128_2_diff_length(bufs[0], C.c_size_t(L), bufs[1], C.c_size_t(L), x)
    lib.kv_hash_meow128_2_diff_length(bufs[2], C.c_size_t(L), bufs[3], C.c_size_t(L), addr(x, 32))
    variants["2_diff"] = list(x)
    x = (U64 * 8)(*([seed[0], seed[1]] * 4))
    lib.kv_hash_meow128_4_same_length(bufs[0], bufs[1], bufs[2], bufs[3], C.c_size_t(L), x)
    variants["4_same"] = list(x)
    x = (U64 * 8)(*([seed[0], seed[1]] * 4))
    lib.kv_hash_meow128_4_diff_length(bufs[0], C.c_size_t(L), bufs[1], C.c_size_t(L), bufs[2],
                                      C.c_size_t(L), bufs[3], C.c_size_t(L), x)
    variants["4_diff"] = list(x)
    x = (U64 * 16)(*([seed[0], seed[1]] * 8))
    pa = (P * 8)(*[C.cast(b, P) for b in bufs + bufs])
    lib.kv_hash_meow128_8_same_length_a(pa, C.c_size_t(L), x)
    variants["8_same"] = list(x)
    seeds4 = [1, 2, 3, 4, 5, 6, 7, 8]
    x = (U64 * 8)(*seeds4)
    lib.kv_hash_meow128_4_same_length_4_seed(bufs[0], bufs[1], bufs[2], bufs[3], C.c_size_t(L), x)
    variants["4_same_4_seed"] = {"seeds": seeds4, "x": list(x)}

    class Vec(C.Structure):
        _fields_ = [("p", P), ("sz", C.c_size_t)]
    vec_out = []
    for b in bufs:
        n = L // 2
        v = (Vec * 2)(Vec(C.cast(b, P), n), Vec(C.cast(b, P).value + n, L - n))
        h1, h2 = U64(seed[0]), U64(seed[1])
        lib.kv_hash_meow128_vec(v, C.c_size_t(2), C.byref(h1), C.byref(h2))
        vec_out.append([h1.value, h2.value])
    variants["vec_split_half"] = vec_out
    strm = []
    for b in bufs:
        h1, h2 = U64(seed[0]), U64(seed[1])
        lib.kv_meow_test(b, C.c_size_t(L), C.byref(h1), C.byref(h2))
        strm.append([h1.value, h2.value])
    variants["stream"] = strm
    out["variants"] = {"keys": [a.decode() for a in ar], "seed": list(seed), "results": variants}

    # ---- kv_hash_meow64 (key_hash.c:1485-1491)
    out["meow64"] = [{"key_hex": ramp[:l].hex(), "seed": s, "h": int(lib.kv_hash_meow64(
        C.create_string_buffer(ramp[:l], max(1, l)), C.c_size_t(l), U64(s)))}
        for l, s in [(0, 0), (7, 12345), (16, 2 ** 64 - 1), (100, 42)]]

    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)

    rng = np.random.default_rng(20260101)
    # ---- every length 0..300 x 4 seed pairs (incl. wrap cases)
    seeds = np.array([[0, 0], [1010, 2020], [2 ** 64 - 1, 2 ** 64 - 1], list(STATIC_SEED)], dtype=np.uint64)
    maxl = 300
    keys = rng.integers(0, 256, size=(maxl + 1, maxl), dtype=np.uint8)
    res = np.zeros((maxl + 1, len(seeds), 2), dtype=np.uint64)
    for L in range(maxl + 1):
        kb = keys[L, :L].tobytes()
        for si, (a, b) in enumerate(seeds):
            res[L, si] = meow(lib, kb, int(a), int(b))
    np.savez_compressed(os.path.join(HERE, "lengths.npz"), keys=keys, seeds=seeds, out=res)

    # ---- fixed-length batches (fast kernels L%8==0 and generic lengths)
    for L in (8, 16, 24, 32, 40, 48, 56, 64, 1, 13, 100, 255):
        n = 1000
        kb = rng.integers(0, 256, size=n * L, dtype=np.uint8)
        o = np.zeros(2 * n, dtype=np.uint64)
        lib.ref_batch_fixed(ptr(kb), L, n, U64(STATIC_SEED[0]), U64(STATIC_SEED[1]), ptr(o))
        np.savez_compressed(os.path.join(HERE, f"fixed_{L}.npz"), keys=kb, out=o.reshape(n, 2),
                            seed=np.array(STATIC_SEED, dtype=np.uint64))

    # ---- zipf variable-length batch (config C2 shape)
    kb, offs, lens = var_keys(4000, 8, 256, seed=77)
    o = np.zeros(2 * len(lens), dtype=np.uint64)
    lib.ref_batch_var(ptr(kb), ptr(offs), len(lens), U64(STATIC_SEED[0]), U64(STATIC_SEED[1]), ptr(o))
    np.savez_compressed(os.path.join(HERE, "var_zipf.npz"), keys=kb, offsets=offs,
                        out=o.reshape(-1, 2), seed=np.array(STATIC_SEED, dtype=np.uint64))

    # ---- arity-4 multi-seed through the reference's 4-seed function (config C3 shape)
    n = 1000
    kb = rng.integers(0, 256, size=n * 32, dtype=np.uint8)
    s4 = np.array(C3_SEEDS, dtype=np.uint64).reshape(-1)
    o = np.zeros(8 * n, dtype=np.uint64)
    lib.ref_batch_4seed(ptr(kb), 32, n, ptr(s4), ptr(o))
    np.savez_compressed(os.path.join(HERE, "multiseed4_32.npz"), keys=kb, seeds=s4, out=o.reshape(n, 4, 2))

    # ---- hash_test int meow 16 keys (config C0): the 1M pass starts at counter 2,097,120
    n = 4096
    c0 = 2 * sum(16 << k for k in range(16))  # 16+32+..+524288 keys, 2 counters each
    kb = int_content_keys(n, 16, c0)
    o = np.zeros(2 * n, dtype=np.uint64)
    lib.ref_batch_fixed(ptr(kb), 16, n, U64(0), U64(0), ptr(o))
    np.savez_compressed(os.path.join(HERE, "hash_test_int16.npz"), keys=kb, out=o.reshape(n, 2),
                        counter0=np.array([c0], dtype=np.uint64))

    # ---- hash_test.cpp:404-442 partition vectors on bytes 0..127, seed (10101, 20202)
    buf = np.arange(128, dtype=np.uint8)
    p2 = np.zeros((129, 4), dtype=np.uint64)
    cb = C.create_string_buffer(buf.tobytes(), 128)
    for n in range(129):
        x = (U64 * 4)(10101, 20202, 10101, 20202)
        lib.kv_hash_meow128_2_diff_length(cb, C.c_size_t(n), addr(cb, n), C.c_size_t(128 - n), x)
        p2[n] = list(x)
    np.savez_compressed(os.path.join(HERE, "partition2.npz"), out=p2)
    print("golden fixtures written to", HERE)


# geometries for the table-position fixtures:
# (name, map_size, hash_entry_size, hash_value_ratio, cuckoo_buckets, cuckoo_arity)
CUCKOO_GEOMS = [
    ("kat64m_4x4", 64 << 20, 64, 1.0, 4, 4),        # SURVEY §8c "hello" KAT geometry
    ("srv64m_2p4", 64 << 20, 64, 0.5, 4, 2),        # server default "2+4" (server.cpp:49)
    ("tiny600_8x8", (448 << 10) + 64 * 600, 64, 1.0, 8, 8),  # tiny table: heavy rejection
    ("tiny5000_2x5", (448 << 10) + 64 * 5000, 64, 1.0, 2, 5),
    ("mid16m_3x1", 16 << 20, 128, 0.75, 1, 3),      # buckets 1 = linear probe (key_ctx.cpp:130)
    ("mid32m_6x2", 32 << 20, 64, 0.9, 2, 6),
    ("mid24m_7x3", 24 << 20, 64, 0.6, 3, 7),
    ("lin64m_1", 64 << 20, 64, 1.0, 1, 1),          # linear table: home slot only
    ("c2x2_8m", 8 << 20, 64, 1.0, 2, 2),            # smallest cuckoo shape
    ("ar1b4_8m", 8 << 20, 64, 1.0, 4, 1),           # arity 1: start slot only
    ("big4g_4x4", 4 << 30, 64, 1.0, 4, 4),          # 2^26-entry table (mask bits > 26)
]


def load_ref_ht():
    lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libkvref_ht.so"))
    lib.ref_cuckoo_positions.argtypes = [U64, C.c_uint32, C.c_float, C.c_uint16, C.c_uint8, P, C.c_size_t,
                                         P, P]
    return lib


def make_cuckoo():
    """CuckooAltHash::calc_hash positions (ht_cuckoo.cpp:38-79) from the
    reference's own ht_init.cpp + ht_cuckoo.cpp (oracle/ref_cuckoo.cpp)."""
    ref = load_ref_ht()
    lib = load_ref()
    rng = np.random.default_rng(20261015)
    # inputs: fixed-up meow hashes of real keys, raw random pairs, and pairs
    # built to collide (h2 = h1, h2 near h1's slot) so both alt1 branches run
    n_real, n_rand = 3000, 3000
    kb = rng.integers(0, 256, size=n_real * 16, dtype=np.uint8)
    hh = np.zeros(2 * n_real, dtype=np.uint64)
    lib.ref_batch_fixed(ptr(kb), 16, n_real, U64(STATIC_SEED[0]), U64(STATIC_SEED[1]), ptr(hh))
    hh = hh.reshape(-1, 2)
    hh[:, 0] &= np.uint64((1 << 63) - 1)
    hh[hh[:, 0] <= 1, 0] = 2
    hello = meow(lib, b"hello\0", *STATIC_SEED)
    hello = ((hello[0] & ((1 << 63) - 1)) or 2, hello[1])
    rand = rng.integers(0, 2 ** 64, size=(n_rand, 2), dtype=np.uint64)
    same = rand[:200].copy(); same[:, 1] = same[:, 0]
    near = rand[200:400].copy(); near[:, 1] = near[:, 0] + np.uint64(1)
    edge = np.array([[0, 0], [1, 2], [2 ** 64 - 1, 2 ** 64 - 1], [2 ** 63, 0], [0, 2 ** 63]], dtype=np.uint64)
    hashes = np.ascontiguousarray(np.concatenate([np.array([hello], dtype=np.uint64), hh, rand, same, near,
                                                  edge]))
    for name, ms, es, ratio, buckets, arity in CUCKOO_GEOMS:
        a = arity if (buckets > 1 and arity > 1) else 1  # linear tables: start slot only
        pos = np.zeros(len(hashes) * a, dtype=np.uint64)
        geom = np.zeros(4, dtype=np.uint64)
        rc = ref.ref_cuckoo_positions(ms, es, ratio, buckets, arity, ptr(hashes), len(hashes), ptr(pos),
                                      ptr(geom))
        assert rc == 0, name
        np.savez_compressed(os.path.join(HERE, f"cuckoo_{name}.npz"), hashes=hashes, pos=pos.reshape(-1, a),
                            params=np.array([ms, es, buckets, arity], dtype=np.uint64),
                            ratio=np.array([ratio], dtype=np.float32),
                            geom=geom,  # ht_mod_mask, ht_mod_fraction, ht_mod_shift, ht_size
                            keys16=kb, seed=np.array(STATIC_SEED, dtype=np.uint64))  # hashes[1:1+len(kb)//16]
        print(name, "ht_size", int(geom[3]), "pos[0]", pos[:a])


def make_crc():
    """kv_crc_c family (key_hash.c:27-179) outputs of the reference itself."""
    lib = load_ref()
    S = C.c_size_t
    lib.kv_crc_c.argtypes = [P, S, C.c_uint32]
    lib.kv_crc_c.restype = C.c_uint32
    lib.kv_hash_uint.argtypes = [C.c_uint32]
    lib.kv_hash_uint.restype = C.c_uint32
    lib.kv_hash_uint2.argtypes = [C.c_uint32, C.c_uint32]
    lib.kv_hash_uint2.restype = C.c_uint32
    lib.kv_crc_c_array.argtypes = [P, P, P, S]
    lib.kv_crc_c_key_array.argtypes = [P, P, P, S]
    rng = np.random.default_rng(20261016)
    # every length 0..300 x 3 seeds, one random buffer per length
    maxl = 300
    keys = rng.integers(0, 256, size=(maxl + 1, maxl), dtype=np.uint8)
    seeds = np.array([0, 0xFFFFFFFF, 0x9E3779B9], dtype=np.uint32)
    lens = np.zeros((maxl + 1, len(seeds)), dtype=np.uint32)
    for L in range(maxl + 1):
        b = np.ascontiguousarray(keys[L, :L])
        buf = C.create_string_buffer(b.tobytes(), max(1, L))
        for si, sd in enumerate(seeds):
            lens[L, si] = lib.kv_crc_c(buf, L, int(sd))
    # zipf variable-length batch with per-key seeds through kv_crc_c_array
    kb, offs, ln = var_keys(3000, 1, 256, seed=91)
    n = len(ln)
    ps = (P * n)(*[kb.ctypes.data + int(offs[i]) for i in range(n)])
    psz = (C.c_size_t * n)(*[int(x) for x in ln])
    sd = rng.integers(0, 2 ** 32, n, dtype=np.uint32)
    arr = sd.copy()
    lib.kv_crc_c_array(ps, psz, arr.ctypes.data, n)
    # kv_crc_c_key_array: prefixes of one 200-byte buffer
    one = rng.integers(0, 256, 200, dtype=np.uint8)
    pl = np.array([0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 199, 200], dtype=np.uint64)
    pseed = rng.integers(0, 2 ** 32, len(pl), dtype=np.uint32)
    pout = pseed.copy()
    psz2 = (C.c_size_t * len(pl))(*[int(x) for x in pl])
    lib.kv_crc_c_key_array(one.ctypes.data, psz2, pout.ctypes.data, len(pl))
    ui = rng.integers(0, 2 ** 32, 64, dtype=np.uint32)
    uo = np.array([lib.kv_hash_uint(int(x)) for x in ui], dtype=np.uint32)
    uo2 = np.array([lib.kv_hash_uint2(int(x), int(y)) for x, y in zip(ui, ui[::-1])], dtype=np.uint32)
    np.savez_compressed(os.path.join(HERE, "crc32c.npz"), len_keys=keys, len_seeds=seeds, len_out=lens,
                        var_keys=kb, var_offsets=offs, var_seeds=sd, var_out=arr,
                        prefix_buf=one, prefix_lens=pl, prefix_seeds=pseed, prefix_out=pout,
                        uint_in=ui, uint_out=uo, uint2_out=uo2)
    print("crc32c fixtures: len", lens.shape, "var", n)


def make_ingest():
    """ctest.c ingest: tokens -> kv_make_key_frag/kv_set_key_frag_string
    records -> kv_hash_key_frag, all by the reference's own functions."""
    ref = load_ref_ht()
    ref.ref_ctest_frags.argtypes = [P, C.c_size_t, C.c_uint32, P, C.c_size_t, P, P, C.c_size_t, P]
    ref.ref_ctest_frags.restype = C.c_long
    rng = np.random.default_rng(20261017)
    # words of zipf-ish lengths 1..300 (some >= 256: dropped), runs of 1-3
    # separators from ' ', '\n', '\t', printable + high bytes, spanning
    # several 64 KiB device chunks; starts and ends without a separator
    parts = []
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789._-:/", dtype=np.uint8)
    total = 0
    while total < 300_000:
        r = rng.random()
        L = int(rng.integers(1, 12)) if r < 0.8 else (int(rng.integers(12, 255)) if r < 0.97 else int(rng.integers(255, 300)))
        w = rng.choice(alpha, L)
        if rng.random() < 0.05:
            w[rng.integers(0, L)] = rng.integers(128, 256)
        parts.append(w.astype(np.uint8))
        sep = rng.choice(np.frombuffer(b" \n\t", dtype=np.uint8), int(rng.integers(1, 4)))
        parts.append(sep.astype(np.uint8))
        total += L + len(sep)
    parts.append(np.frombuffer(b"last_token_no_separator", dtype=np.uint8))
    text = np.concatenate(parts)
    n = len(text)
    tbuf = C.create_string_buffer(text.tobytes(), n + 2)
    cap_tok = n // 2 + 1
    frag = np.zeros(n * 2 + 64, dtype=np.uint8)
    roffs = np.zeros(cap_tok, dtype=np.uint64)
    hashes = np.zeros(2 * cap_tok, dtype=np.uint64)
    seed = np.zeros(2, dtype=np.uint64)
    cnt = ref.ref_ctest_frags(tbuf, n, 256, ptr(frag), frag.size, ptr(roffs), ptr(hashes), cap_tok, ptr(seed))
    assert cnt > 0
    used = int(roffs[cnt - 1]) + 2 + int(frag[int(roffs[cnt - 1])] | (frag[int(roffs[cnt - 1]) + 1] << 8))
    used = (used + 1) & ~1
    np.savez_compressed(os.path.join(HERE, "ingest.npz"), text=text, max_token=np.array([256], np.uint32),
                        frags=frag[:used], rec_offs=roffs[:cnt], hashes=hashes[:2 * cnt].reshape(-1, 2), seed=seed)
    print("ingest fixtures:", n, "bytes,", cnt, "tokens, seed", [hex(int(x)) for x in seed])


SORT_GEOMS = [  # (name, map_size, entry_size, ratio, buckets, arity, n, dup_fraction)
    ("kat64m", 64 << 20, 64, 1.0, 4, 4, 20000, 0.05),
    ("tiny600", (448 << 10) + 64 * 600, 64, 1.0, 8, 8, 5000, 0.10),   # many equal slots
    ("big4g", 4 << 30, 64, 1.0, 4, 4, 50000, 0.02),
]


def make_sort():
    """kv_ht_radix_sort (radix_sort.cpp:31-41) + ctest.c:96-104 dedup by the
    reference itself (oracle/ref_cuckoo.cpp ref_ht_sort)."""
    ref = load_ref_ht()
    ref.ref_ht_sort.argtypes = [U64, C.c_uint32, C.c_float, C.c_uint16, C.c_uint8, P, C.c_size_t, P, P, P]
    ref.ref_ht_sort.restype = C.c_int
    lib = load_ref()
    rng = np.random.default_rng(20261018)
    for name, ms, es, ratio, b, a, n, dupf in SORT_GEOMS:
        kb = rng.integers(0, 256, size=n * 16, dtype=np.uint8)
        hh = np.zeros(2 * n, dtype=np.uint64)
        lib.ref_batch_fixed(ptr(kb), 16, n, U64(STATIC_SEED[0]), U64(STATIC_SEED[1]), ptr(hh))
        hh = hh.reshape(n, 2)
        hh[:, 0] &= np.uint64((1 << 63) - 1)
        hh[hh[:, 0] <= 1, 0] = 2
        nd = int(n * dupf)  # duplicated keys (copies of earlier rows), scattered
        src = rng.integers(0, n - nd, nd)
        dst = rng.choice(np.arange(n - nd, n), nd, replace=False)
        hh[dst] = hh[src]
        hh = np.ascontiguousarray(hh)
        oh = np.zeros(2 * n, dtype=np.uint64)
        oi = np.zeros(n, dtype=np.uint64)
        dups = np.zeros(1, dtype=np.uint64)
        assert ref.ref_ht_sort(ms, es, ratio, b, a, ptr(hh), n, ptr(oh), ptr(oi), ptr(dups)) == 0
        np.savez_compressed(os.path.join(HERE, f"sort_{name}.npz"), hashes=hh, out_hashes=oh.reshape(n, 2),
                            out_items=oi, dups=dups, params=np.array([ms, es, b, a], dtype=np.uint64),
                            ratio=np.array([ratio], dtype=np.float32))
        print("sort", name, n, "ref dups", int(dups[0]))


def partition_digest(d: np.ndarray) -> int:
    """Order-dependent digest of u64 words: sum of w_i * (2i + 1) mod 2^64."""
    w = d.reshape(-1).astype(np.uint64)
    k = (2 * np.arange(w.size, dtype=np.uint64) + np.uint64(1))
    with np.errstate(over="ignore"):
        return int(np.sum(w * k, dtype=np.uint64))


def make_partition4():
    """hash_test.cpp:418-442: bytes 0..127 cut at every n <= m <= o < 128
    into four keys hashed by the reference's kv_hash_meow128_4_diff_length
    (seed 10101, 20202).  Every key is a substring buf[a:b], so the fixture
    is the reference's kv_hash_meow128 of all 8385 substrings (the table the
    device paths are checked against) plus the digest of the reference's own
    357,760 x 4-diff outputs in loop order; the generator asserts that each
    4-diff output equals the four substring hashes, which is the reference
    test's own assertion."""
    lib = load_ref()
    buf = bytes(range(128))
    cb = C.create_string_buffer(buf, 128)
    idx = np.full((129, 129), -1, dtype=np.int64)
    subs = []
    for a in range(129):
        for b in range(a, 129):
            idx[a, b] = len(subs)
            subs.append((a, b))
    sub = np.array(subs, dtype=np.uint32)
    h = np.zeros((len(subs), 2), dtype=np.uint64)
    for i, (a, b) in enumerate(subs):
        h[i] = meow(lib, buf[a:b], 10101, 20202)
    trip = [(n, m, o) for n in range(128) for m in range(n, 128) for o in range(m, 128)]
    d = np.zeros((len(trip), 8), dtype=np.uint64)
    x = (U64 * 8)()
    for t, (n, m, o) in enumerate(trip):
        for q in range(0, 8, 2):
            x[q], x[q + 1] = 10101, 20202
        lib.kv_hash_meow128_4_diff_length(cb, C.c_size_t(n), addr(cb, n), C.c_size_t(m - n), addr(cb, m),
                                          C.c_size_t(o - m), addr(cb, o), C.c_size_t(128 - o), x)
        d[t] = list(x)
    tr = np.array(trip, dtype=np.int64)
    want = np.concatenate([h[idx[0, tr[:, 0]]], h[idx[tr[:, 0], tr[:, 1]]], h[idx[tr[:, 1], tr[:, 2]]],
                           h[idx[tr[:, 2], 128]]], axis=1)
    assert np.array_equal(d, want), "reference 4-diff != single hashes"
    np.savez_compressed(os.path.join(HERE, "partition4.npz"), sub=sub, out=h, ntrip=np.array([len(trip)]),
                        digest4=np.array([partition_digest(d)], dtype=np.uint64))
    print("partition4.npz:", len(subs), "substrings,", len(trip), "triples")


if __name__ == "__main__":
    only = [a for a in sys.argv[1:] if a.startswith("--only-")]
    if not only:
        main()
    if not only or "--only-cuckoo" in only:
        make_cuckoo()
    if not only or "--only-crc" in only:
        make_crc()
    if not only or "--only-ingest" in only:
        make_ingest()
    if not only or "--only-sort" in only:
        make_sort()
    if not only or "--only-partition4" in only:
        make_partition4()
