"""Test-side loader for the oracle (oracle/liboracle.so) and, when present,
the compiled reference (oracle/_ref/libkvref.so).  Only tests/, smoke() and
bench.py's cpu_baseline use these; the product never does."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "liboracle.so")
REF = os.path.join(ROOT, "oracle", "_ref", "libkvref.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")
U64, P, SZ = C.c_uint64, C.c_void_p, C.c_size_t


def load_oracle():
    if not os.path.exists(ORACLE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"], check=True)
    lib = C.CDLL(ORACLE)
    lib.orc_meow128.argtypes = [P, SZ, C.POINTER(U64), C.POINTER(U64)]
    lib.orc_meow64.argtypes = [P, SZ, U64]
    lib.orc_meow64.restype = U64
    lib.orc_fixup.argtypes = [U64]
    lib.orc_fixup.restype = U64
    lib.orc_batch_fixed.argtypes = [P, SZ, SZ, U64, U64, P, C.c_int]
    lib.orc_batch_var.argtypes = [P, P, SZ, U64, U64, P, C.c_int]
    lib.orc_batch_multiseed.argtypes = [P, SZ, SZ, P, SZ, P, C.c_int]
    lib.orc_stream_size.restype = SZ
    lib.orc_stream_init.argtypes = [P, U64, U64, SZ]
    lib.orc_stream_update.argtypes = [P, P, SZ]
    lib.orc_stream_final.argtypes = [P, C.POINTER(U64), C.POINTER(U64)]
    lib.orc_aesdec.argtypes = [P, P, P]
    return lib


def load_ref():
    if not os.path.exists(REF):
        return None
    lib = C.CDLL(REF)
    lib.kv_hash_meow128.argtypes = [P, SZ, C.POINTER(U64), C.POINTER(U64)]
    lib.ref_batch_fixed.argtypes = [P, SZ, SZ, U64, U64, P]
    lib.ref_batch_var.argtypes = [P, P, SZ, U64, U64, P]
    lib.ref_bench_fixed.argtypes = [P, SZ, SZ, U64, U64, P, C.c_int]
    lib.ref_bench_fixed.restype = C.c_double
    lib.ref_hash_test_int.argtypes = [SZ, C.c_uint16, U64, U64]
    lib.ref_hash_test_int.restype = C.c_double
    return lib


def orc_meow(lib, data: bytes, s1: int, s2: int):
    h1, h2 = U64(s1), U64(s2)
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    lib.orc_meow128(buf, len(data), C.byref(h1), C.byref(h2))
    return h1.value, h2.value


def orc_fixed(lib, keys: np.ndarray, key_len: int, seed, fixup=False) -> np.ndarray:
    n = keys.size // key_len if key_len else 0
    out = np.zeros((n, 2), dtype=np.uint64)
    lib.orc_batch_fixed(keys.ctypes.data, key_len, n, U64(seed[0]), U64(seed[1]), out.ctypes.data, int(fixup))
    return out


def orc_var(lib, keys: np.ndarray, offs: np.ndarray, seed, fixup=False) -> np.ndarray:
    n = offs.size - 1
    out = np.zeros((n, 2), dtype=np.uint64)
    kb = keys if keys.size else np.zeros(1, np.uint8)
    lib.orc_batch_var(kb.ctypes.data, offs.ctypes.data, n, U64(seed[0]), U64(seed[1]), out.ctypes.data,
                      int(fixup))
    return out


def orc_multiseed(lib, keys: np.ndarray, key_len: int, seeds, fixup=False) -> np.ndarray:
    n = keys.size // key_len
    s = np.array(seeds, dtype=np.uint64).reshape(-1)
    out = np.zeros((n, len(seeds), 2), dtype=np.uint64)
    lib.orc_batch_multiseed(keys.ctypes.data, key_len, n, s.ctypes.data, len(seeds), out.ctypes.data,
                            int(fixup))
    return out


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


# ------------------------------------------------------------ table positions (§8 f1)
class OrcGeom(C.Structure):
    _fields_ = [("ht_size", U64), ("ht_mod_mask", U64), ("ht_mod_fraction", U64), ("ht_mod_shift", C.c_uint32),
                ("cuckoo_buckets", C.c_uint16), ("cuckoo_arity", C.c_uint8), ("pad", C.c_uint8)]


def _orc_pos_sigs(lib):
    lib.orc_ht_geom.argtypes = [U64, C.c_uint32, C.c_float, C.c_uint16, C.c_uint8, C.POINTER(OrcGeom)]
    lib.orc_ht_geom.restype = C.c_int
    lib.orc_ht_mod.argtypes = [C.POINTER(OrcGeom), U64]
    lib.orc_ht_mod.restype = U64
    lib.orc_positions_per_key.argtypes = [C.POINTER(OrcGeom)]
    lib.orc_positions_per_key.restype = C.c_uint
    lib.orc_cuckoo_positions.argtypes = [C.POINTER(OrcGeom), P, SZ, P]


def orc_geom(lib, map_size, entry_size, ratio, buckets, arity) -> OrcGeom:
    _orc_pos_sigs(lib)
    g = OrcGeom()
    assert lib.orc_ht_geom(map_size, entry_size, ratio, buckets, arity, C.byref(g)) == 0
    return g


def orc_positions(lib, g: OrcGeom, hashes: np.ndarray) -> np.ndarray:
    _orc_pos_sigs(lib)
    h = np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1, 2)
    a = lib.orc_positions_per_key(C.byref(g))
    pos = np.zeros((len(h), a), dtype=np.uint64)
    lib.orc_cuckoo_positions(C.byref(g), h.ctypes.data, len(h), pos.ctypes.data)
    return pos


def cuckoo_fixtures():
    import glob
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "cuckoo_*.npz"))):
        d = np.load(f)
        ms, es, b, a = (int(x) for x in d["params"])
        out.append(dict(name=os.path.basename(f)[7:-4], map_size=ms, entry_size=es, buckets=b, arity=a,
                        ratio=float(d["ratio"][0]), geom=d["geom"], hashes=d["hashes"], pos=d["pos"],
                        keys16=d["keys16"], seed=tuple(int(x) for x in d["seed"])))
    return out


def load_ref_ht():
    p = os.path.join(ROOT, "oracle", "_ref", "libkvref_ht.so")
    if not os.path.exists(p):
        return None
    lib = C.CDLL(p)
    lib.ref_cuckoo_positions.argtypes = [U64, C.c_uint32, C.c_float, C.c_uint16, C.c_uint8, P, SZ, P, P]
    lib.ref_cuckoo_bench.argtypes = [U64, U64, U64, C.c_uint32, C.c_uint16, C.c_uint8, P, SZ, SZ, U64, U64, P, P,
                                     C.c_int]
    lib.ref_cuckoo_bench.restype = C.c_double
    lib.ref_ht_sort_bench.argtypes = [U64, U64, U64, C.c_uint32, P, SZ, P]
    lib.ref_ht_sort_bench.restype = C.c_double
    lib.ref_ht_sort.argtypes = [U64, C.c_uint32, C.c_float, C.c_uint16, C.c_uint8, P, SZ, P, P, P]
    lib.ref_ht_sort.restype = C.c_int
    return lib


def ref_ht_sort(lib, map_size, hashes):
    """The compiled reference's kv_ht_radix_sort + ctest marking
    (oracle/ref_cuckoo.cpp ref_ht_sort) on a 64-byte-entry 4x4 table of
    map_size bytes -> (hashes, items, dup_count)."""
    h = np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1, 2)
    n = len(h)
    oh = np.zeros((n, 2), np.uint64)
    oi = np.zeros(n, np.uint64)
    d = np.zeros(1, np.uint64)
    assert lib.ref_ht_sort(map_size, 64, 1.0, 4, 4, h.ctypes.data, n, oh.ctypes.data, oi.ctypes.data,
                           d.ctypes.data) == 0
    return oh, oi, int(d[0])


def ref_order_cases(seed=0):
    """Inputs for the exact-order sort (KVH_REF_ORDER): table geometries whose
    slot bit counts (1 + floor(log2 ht_size): 10, 17, 20, 25, 26) reach every
    step of RadixSort::sort -- 8-bit passes, 2-5-bit last passes, the 1-bit
    Hoare pass (17, 25) -- and batches with duplicates, a hot slot (one node
    of equal slots, re-pushed down to no bits), slots clustered in one
    top-level bucket, and sizes around the 32-element tail and 2048-element
    wave thresholds."""
    rng = np.random.default_rng(seed)
    out = []
    for ms in (497152, 5 << 20, 64 << 20, 1200 << 20, 4 << 30):
        for n in (2, 3, 4, 5, 31, 32, 33, 100, 2048, 2049, 5000, 16384):
            h = rng.integers(0, 2**64, (n, 2), dtype=np.uint64)
            kind = rng.integers(0, 4)
            if kind == 1 and n > 8:  # exact duplicates
                src = rng.integers(0, n, n // 8)
                h[rng.integers(0, n, n // 8)] = h[src]
            elif kind == 2 and n > 8:  # a hot h1 (one slot), distinct h2
                h[rng.integers(0, n, n // 3), 0] = h[0, 0]
            elif kind == 3:  # h1 clustered: few distinct high slot bits
                h[:, 0] = (h[:, 0] & np.uint64(0xffff)) | (h[0, 0] & ~np.uint64(0xffff))
            out.append((ms, h))
    return out


# ------------------------------------------------------------ CRC32C (§8 f4)
def crc_sigs(lib):
    lib.orc_crc_c.argtypes = [P, SZ, C.c_uint32]
    lib.orc_crc_c.restype = C.c_uint32
    lib.orc_hash_uint2.argtypes = [C.c_uint32, C.c_uint32]
    lib.orc_hash_uint2.restype = C.c_uint32
    lib.orc_crc_batch_var.argtypes = [P, P, SZ, P, C.c_uint32, P]
    lib.orc_crc_batch_fixed.argtypes = [P, SZ, SZ, P, C.c_uint32, P]
    return lib


def orc_crc(lib, data: bytes, seed: int) -> int:
    crc_sigs(lib)
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    return int(lib.orc_crc_c(buf, len(data), seed))


def orc_crc_var(lib, keys: np.ndarray, offs: np.ndarray, seeds=None, seed: int = 0) -> np.ndarray:
    crc_sigs(lib)
    n = offs.size - 1
    out = np.zeros(n, dtype=np.uint32)
    kb = keys if keys.size else np.zeros(1, np.uint8)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    lib.orc_crc_batch_var(kb.ctypes.data, np.ascontiguousarray(offs, dtype=np.uint64).ctypes.data, n,
                          None if sd is None else sd.ctypes.data, seed, out.ctypes.data)
    return out


def orc_crc_fixed(lib, keys: np.ndarray, key_len: int, seeds=None, seed: int = 0) -> np.ndarray:
    crc_sigs(lib)
    n = keys.size // key_len if key_len else 0
    out = np.zeros(n, dtype=np.uint32)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    lib.orc_crc_batch_fixed(keys.ctypes.data, key_len, n, None if sd is None else sd.ctypes.data, seed,
                            out.ctypes.data)
    return out


# ------------------------------------------------------------ ingest (§8 f3)
def ingest_sigs(lib):
    lib.orc_tokenize.argtypes = [P, SZ, C.c_uint32, P, P, SZ]
    lib.orc_tokenize.restype = SZ
    lib.orc_hash_spans.argtypes = [P, P, P, SZ, U64, U64, C.c_int, C.c_int, P]
    return lib


def orc_tokenize(lib, text: np.ndarray, max_token: int = 256):
    ingest_sigs(lib)
    n = text.size
    cap = n // 2 + 1
    offs = np.zeros(cap, dtype=np.uint64)
    lens = np.zeros(cap, dtype=np.uint32)
    tb = text if n else np.zeros(1, np.uint8)
    cnt = lib.orc_tokenize(tb.ctypes.data, n, max_token, offs.ctypes.data, lens.ctypes.data, cap)
    return offs[:cnt], lens[:cnt]


def orc_hash_spans(lib, buf: np.ndarray, offs, lens, seed, nul=True, fix=True) -> np.ndarray:
    ingest_sigs(lib)
    n = len(offs)
    out = np.zeros((n, 2), dtype=np.uint64)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    l = np.ascontiguousarray(lens, dtype=np.uint32)
    bb = buf if buf.size else np.zeros(1, np.uint8)
    lib.orc_hash_spans(bb.ctypes.data, o.ctypes.data, l.ctypes.data, n, U64(seed[0]), U64(seed[1]), int(nul),
                       int(fix), out.ctypes.data)
    return out


# ------------------------------------------------------------ table order (§8 f2)
def np_ht_mod(geom, h1: np.ndarray) -> np.ndarray:
    """FileHdr::ht_mod (shm_ht.h:181-184) in u64 numpy arithmetic (wraps)."""
    x = h1 & np.uint64(geom.ht_mod_mask)
    with np.errstate(over="ignore"):
        return (x * np.uint64(geom.ht_mod_fraction)) >> np.uint64(geom.ht_mod_shift)


def np_ht_sort(geom, hashes: np.ndarray, items=None, dedup=False):
    """Restatement of kv_ht_radix_sort's order (radix_sort.cpp:31-41: by
    ht_mod(key)) with the device's deterministic tie order (h1 << 1, h1,
    h2), plus ctest.c:96-104's marking (earlier of an equal adjacent pair
    gets h1 = 0).  Returns (hashes, items, dup_count)."""
    h = np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1, 2)
    n = len(h)
    it = np.arange(n, dtype=np.uint64) if items is None else np.asarray(items, dtype=np.uint64)
    slot = np_ht_mod(geom, h[:, 0])
    order = np.lexsort((h[:, 1], h[:, 0], h[:, 0] << np.uint64(1), slot))
    oh = h[order].copy()
    oi = it[order].copy()
    dups = 0
    if dedup and n > 1:
        eq = (oh[:-1, 0] == oh[1:, 0]) & (oh[:-1, 1] == oh[1:, 1])
        oh[:-1, 0][eq] = 0
        dups = int(eq.sum())
    return oh, oi, dups


def orc_ht_radix_sort_ref(lib, geom, hashes: np.ndarray, items=None, dedup=False):
    """oracle/sort_oracle.c: kv_ht_radix_sort's exact element order
    (radix_sort.h:89-298 via radix_sort.cpp:31-41) + ctest.c:96-104's marking.
    Returns (hashes, items, dup_count)."""
    lib.orc_ht_radix_sort_ref.argtypes = [C.POINTER(OrcGeom), P, C.c_uint32]
    lib.orc_ht_radix_sort_ref.restype = None
    lib.orc_ht_mark_dups.argtypes = [P, C.c_uint32]
    lib.orc_ht_mark_dups.restype = U64
    h = np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1, 2)
    n = len(h)
    el = np.empty((n, 3), dtype=np.uint64)
    el[:, :2] = h
    el[:, 2] = np.arange(n, dtype=np.uint64) if items is None else np.asarray(items, dtype=np.uint64)
    lib.orc_ht_radix_sort_ref(C.byref(geom), el.ctypes.data, n)
    d = int(lib.orc_ht_mark_dups(el.ctypes.data, n)) if dedup else 0
    return el[:, :2].copy(), el[:, 2].copy(), d


def sort_fixtures():
    import glob
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "sort_*.npz"))):
        d = np.load(f)
        ms, es, b, a = (int(x) for x in d["params"])
        out.append(dict(name=os.path.basename(f)[5:-4], map_size=ms, entry_size=es, buckets=b, arity=a,
                        ratio=float(d["ratio"][0]), hashes=d["hashes"], out_hashes=d["out_hashes"],
                        out_items=d["out_items"], dups=int(d["dups"][0])))
    return out
