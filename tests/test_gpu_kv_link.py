"""GPU: the reference's own KV core, linked against libkvh_kv.so instead of
src/key_hash.c (oracle/_ref/libkvref_ht_kvh.so, built in the container by
oracle/Makefile with -Wl,--no-undefined; tests/test_kv_link.py), computes on
the device what the reference computes on the CPU:

  - ctest's ingest (ctest.c:202-233) through the reference's kv_make_key_frag /
    kv_set_key_frag_string / kv_hash_key_frag (key_ctx.cpp:1737-1783), whose
    kv_hash_meow128 is now libkvh_kv.so's: the records equal the reference's
    own (tests/golden/ingest.npz, made with key_hash.c) and the hashes the
    pinned oracle's under the table seed this run drew;
  - kv_hash_meow128 + KeyCtx::set_hash + CuckooAltHash::calc_hash for 16-byte
    keys (oracle/ref_cuckoo.cpp ref_cuckoo_bench) equal the same driver linked
    with key_hash.c (oracle/_ref/libkvref_ht.so).
Every kv_hash_meow128 here is one GPU call of the single-key drop-in."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle_lib import load_oracle, orc_hash_spans

pytestmark = pytest.mark.gpu
ORC = load_oracle()

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(ROOT, "oracle", "_ref", "libkvref_ht_kvh.so")
P = C.c_void_p


@pytest.fixture(scope="module")
def kvcore():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: build it in the container (make -C oracle _ref/libkvref_ht_kvh.so)")
    lib = C.CDLL(LIB)
    lib.ref_ctest_frags.argtypes = [P, C.c_size_t, C.c_uint32, P, C.c_size_t, P, P, C.c_size_t, P]
    lib.ref_ctest_frags.restype = C.c_long
    lib.ref_cuckoo_bench.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint16, C.c_uint8, P,
                                     C.c_size_t, C.c_size_t, C.c_uint64, C.c_uint64, P, P, C.c_int]
    lib.ref_cuckoo_bench.restype = C.c_double
    return lib


def test_reference_ctest_ingest_on_libkvh_kv(kvcore):
    G = np.load(os.path.join(HERE, "golden", "ingest.npz"))
    text = np.ascontiguousarray(G["text"])
    n = text.size
    cap = n // 2 + 1
    frag = np.zeros(n * 2 + 64, np.uint8)
    ro = np.zeros(cap, np.uint64)
    hh = np.zeros(2 * cap, np.uint64)
    seed = np.zeros(2, np.uint64)
    cnt = kvcore.ref_ctest_frags(text.ctypes.data, n, 256, frag.ctypes.data, frag.size, ro.ctypes.data,
                                 hh.ctypes.data, cap, seed.ctypes.data)
    # the records are the reference's own (ingest.npz); the table's seed is drawn per HashTab
    # (HashTab::alloc_map), so the hashes are checked against the pinned oracle under this run's seed
    assert cnt == len(G["rec_offs"])
    np.testing.assert_array_equal(ro[:cnt], G["rec_offs"].astype(np.uint64))
    np.testing.assert_array_equal(frag[:G["frags"].size], G["frags"])
    ro = ro[:cnt]
    lens = (frag[ro.astype(np.int64)].astype(np.uint32) | (frag[ro.astype(np.int64) + 1].astype(np.uint32) << 8))
    want = orc_hash_spans(ORC, frag, ro + np.uint64(2), lens, (int(seed[0]), int(seed[1])), nul=False, fix=True)
    np.testing.assert_array_equal(hh[:2 * cnt].reshape(-1, 2), want)
    assert not np.array_equal(hh[:2 * cnt].reshape(-1, 2), G["hashes"]) or np.array_equal(seed, G["seed"])


def test_reference_cuckoo_path_on_libkvh_kv(kvcore):
    import sys
    sys.path.insert(0, HERE)
    from oracle_lib import load_ref_ht
    import raikv_amd as kvh
    ref = load_ref_ht()
    if ref is None:
        pytest.fail("oracle/_ref/libkvref_ht.so missing")
    g = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
    n, L = 3000, 16
    keys = np.random.default_rng(77).integers(0, 256, n * L, dtype=np.uint8)
    out = []
    for lib in (kvcore, ref):
        h = np.zeros(2 * n, np.uint64)
        pos = np.zeros(n * g.per_key, np.uint64)
        t = lib.ref_cuckoo_bench(g.ht_size, g.ht_mod_mask, g.ht_mod_fraction, g.ht_mod_shift, g.cuckoo_buckets,
                                 g.cuckoo_arity, keys.ctypes.data, L, n, 0x1234567890ABCDEF, 0xFEDCBA0987654321,
                                 h.ctypes.data, pos.ctypes.data, 1)
        assert t >= 0
        out.append((h, pos))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert np.count_nonzero(out[0][1]) > n
