"""GPU parity for SURVEY.md §8 row f2 (batch order by table position +
duplicate marking): kvh_ht_sort and the kvh_ht_radix_sort drop-in vs the
oracle order (oracle_lib.np_ht_sort, itself checked against the
reference's kv_ht_radix_sort in test_sort_oracle.py) on the golden inputs,
plus edge cases and a full-size property test.  Bit-exact."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle_lib import (load_oracle, np_ht_mod, np_ht_sort, orc_geom, orc_ht_radix_sort_ref,  # noqa: E402
                        ref_order_cases, sort_fixtures)

FIX = sort_fixtures()
ORC = load_oracle()


@pytest.fixture(scope="module")
def kvh():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    import raikv_amd
    return raikv_amd


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


ENGINES = [(0, 0, 0), (0, 0, 3), (0, 2, None), (0, 1, None), (33, 0, None)]
ENGINE_IDS = ["bucketed2", "bucketed2_half", "bucketed1", "radix_u32", "radix_u64"]


class _engine:
    """knob 20 = 0 two-pass bucketed (the default), 2 one-pass bucketed, 1
    radix; knob 17 = 33 forces the radix engine on u64 keys over slot + 33 h1
    bits (0: u32 keys when the prefix fits 31 bits); knob 23 picks the
    two-pass path's bucket sort (0 k_bk_sort, 3 -- the default -- half-size
    buckets: up to 15 bucket bits, the second pass on 8-bit digits, the
    register-resident k_bk_sortr at two 512-thread workgroups per CU; 1 / 2
    only in the experiments build)."""

    def __init__(self, kvh, sort_bits, engine, b3=None):
        self.kvh, self.v, self.b3 = kvh, (sort_bits, engine), b3

    def __enter__(self):
        self.prev = (self.kvh.lib.kvh_set_tuning(17, self.v[0]), self.kvh.lib.kvh_set_tuning(20, self.v[1]))
        if self.b3 is not None:
            self.prev_b3 = self.kvh.lib.kvh_set_tuning(23, self.b3)

    def __exit__(self, *a):
        self.kvh.lib.kvh_set_tuning(17, self.prev[0])
        self.kvh.lib.kvh_set_tuning(20, self.prev[1])
        if self.b3 is not None:
            self.kvh.lib.kvh_set_tuning(23, self.prev_b3)


@pytest.mark.parametrize("eng", ENGINES, ids=ENGINE_IDS)
@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_sort_golden(kvh, f, eng):
    """Golden sets on each engine: bucketed, radix on u32 keys, radix on u64 keys."""
    with _engine(kvh, *eng):
        _sort_golden(kvh, f)


def _sort_golden(kvh, f):
    g = kvh.HtGeom.from_map(f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    og = orc_geom(ORC, f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    h = f["hashes"]
    srt = kvh.HtSorter(g, len(h))
    for dedup in (False, True):
        oh, oi = srt.sort(dev(h), dedup=dedup)
        wh, wi, wd = np_ht_sort(og, h, dedup=dedup)
        np.testing.assert_array_equal(host(oh), wh)
        np.testing.assert_array_equal(host(oi), wi)
        if dedup:
            assert int(srt.dups.item()) == wd >= f["dups"]
    # items carried through
    items = np.arange(len(h), dtype=np.uint64) * np.uint64(7919) + np.uint64(3)
    oh, oi = srt.sort(dev(h), items=dev(items))
    np.testing.assert_array_equal(host(oi), np_ht_sort(og, h, items=items)[1])


class SortT(C.Structure):  # kv_ht_sort_t (radix_sort.h:8-11)
    _fields_ = [("key", C.c_uint64), ("key2", C.c_uint64), ("item", C.c_void_p)]


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_radix_sort_drop_in_is_the_reference_order(kvh, f):
    """kvh_ht_radix_sort (the kv_ht_radix_sort drop-in, radix_sort.h:19-20)
    sorts a kv_ht_sort_t array in place in the reference's EXACT order for
    batches of <= 64K (ctest's): the fixture's element order word for word,
    items (pointers) carried."""
    g = kvh.HtGeom.from_map(f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    h = f["hashes"]
    ar = (SortT * len(h))(*[SortT(int(a), int(b), i + 1) for i, (a, b) in enumerate(h)])
    assert kvh.lib.kvh_ht_radix_sort(ar, len(h), C.byref(g)) == 0
    got = np.array([x.item for x in ar], dtype=np.uint64) - np.uint64(1)
    np.testing.assert_array_equal(got, f["out_items"])
    keys = np.array([[x.key, x.key2] for x in ar], dtype=np.uint64)
    np.testing.assert_array_equal(keys, h[f["out_items"].astype(np.int64)])


def test_radix_sort_batch_front_end(kvh):
    """kvh_ht_radix_sort_batch: many host kv_ht_sort_t
    arrays -- ctest's batch shapes (empty, 1, 2, 31, 32, a full 16K, ~8K
    ones) and the reference's own fixtures -- sorted in place in ONE launch,
    each in kv_ht_radix_sort's exact order (the pinned restatement, and the
    fixtures' own element order word for word), items carried; again with a
    larger second call (the staging buffers grow)."""
    rng = np.random.default_rng(8)
    f = FIX[0]
    g = kvh.HtGeom.from_map(f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    og = orc_geom(ORC, f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    for sizes in ([0, 1, 2, 31, 32, 16384] + [int(x) for x in rng.integers(6000, 10000, 10)],
                  [int(x) for x in rng.integers(1, 16385, 48)]):
        hs = [rng.integers(0, 2 ** 64, size=(k, 2), dtype=np.uint64) for k in sizes]
        for h in hs[6:9]:
            if len(h) > 100:
                h[rng.integers(0, len(h), len(h) // 30)] = h[rng.integers(0, len(h), len(h) // 30)]
        hs.append(f["hashes"])  # the fixture, with its own expected order
        arrs, views = [], []
        for b, h in enumerate(hs):
            ar = (SortT * max(len(h), 1))()
            v = np.frombuffer(ar, dtype=np.uint64).reshape(-1, 3)[:len(h)]
            v[:, :2] = h
            v[:, 2] = (np.uint64(b) << np.uint64(32)) + np.arange(len(h), dtype=np.uint64)
            arrs.append(ar)
            views.append(v)
        ptrs = (C.c_void_p * len(arrs))(*[C.addressof(a) for a in arrs])
        szs = (C.c_uint32 * len(arrs))(*[len(h) for h in hs])
        assert kvh.lib.kvh_ht_radix_sort_batch(ptrs, szs, len(arrs), C.byref(g)) == 0
        for b, (h, v) in enumerate(zip(hs, views)):
            items = v[:, 2] - (np.uint64(b) << np.uint64(32))
            if b == len(hs) - 1:
                np.testing.assert_array_equal(items, f["out_items"])
            wh, wi, _ = orc_ht_radix_sort_ref(ORC, og, h)
            np.testing.assert_array_equal(items, wi, err_msg=f"batch {b} of {len(hs)}")
            np.testing.assert_array_equal(v[:, :2], wh, err_msg=f"batch {b}")
    assert kvh.lib.kvh_ht_radix_sort_batch(None, None, 0, C.byref(g)) == 0
    bad = (C.c_uint32 * 1)(65537)
    assert kvh.lib.kvh_ht_radix_sort_batch(ptrs, bad, 1, C.byref(g)) == -22


def test_radix_sort_drop_in_above_64k(kvh):
    """Above 64K elements the drop-in takes the engine's total order (same
    slot order; ties by (h1 << 1, h1, h2))."""
    f = FIX[0]
    g = kvh.HtGeom.from_map(f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    og = orc_geom(ORC, f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    rng = np.random.default_rng(3)
    h = rng.integers(0, 2 ** 64, size=(65537, 2), dtype=np.uint64)
    ar = (SortT * len(h))()
    arr = np.frombuffer(ar, dtype=np.uint64).reshape(-1, 3)
    arr[:, :2] = h
    arr[:, 2] = np.arange(1, len(h) + 1, dtype=np.uint64)
    assert kvh.lib.kvh_ht_radix_sort(ar, len(h), C.byref(g)) == 0
    wh, wi, _ = np_ht_sort(og, h, items=np.arange(1, len(h) + 1, dtype=np.uint64))
    np.testing.assert_array_equal(arr[:, :2], wh)
    np.testing.assert_array_equal(arr[:, 2], wi)


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_ref_order_fixtures_word_for_word(kvh, f):
    """kvh_ht_sort with KVH_REF_ORDER reproduces the
    reference's kv_ht_radix_sort + ctest marking on its own fixtures word for
    word: element order (ties included), zeroed duplicates, and the count
    (99 on the 600-slot table, 992 and 1000 on the others)."""
    g = kvh.HtGeom.from_map(f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    h = f["hashes"]
    srt = kvh.HtSorter(g, len(h))
    oh, oi = srt.sort(dev(h), dedup=True, ref_order=True)
    np.testing.assert_array_equal(host(oi), f["out_items"])
    np.testing.assert_array_equal(host(oh), f["out_hashes"])
    assert int(srt.dups.item()) == f["dups"]
    # a 16K slice (ctest's batch, ctest.c:34) against the pinned restatement
    og = orc_geom(ORC, f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    part = h[:16384]
    oh, oi = srt.sort(dev(part), dedup=True, ref_order=True)
    wh, wi, wd = orc_ht_radix_sort_ref(ORC, og, part, dedup=True)
    np.testing.assert_array_equal(host(oi), wi)
    np.testing.assert_array_equal(host(oh), wh)
    assert int(srt.dups.item()) == wd


def test_ref_order_every_step_vs_oracle(kvh):
    """KVH_REF_ORDER against the pinned restatement (oracle/sort_oracle.c) on
    batches that reach every step of RadixSort::sort: 8-bit and short last
    passes, the 1-bit pass (17- and 25-bit slot counts), tails of 2-31,
    nodes around the 2048-element wave threshold, duplicates, a hot slot,
    clustered slots; plus 65536 elements, items carried."""
    cases = ref_order_cases(seed=7)
    rng = np.random.default_rng(8)
    cases.append((64 << 20, rng.integers(0, 2 ** 64, size=(65536, 2), dtype=np.uint64)))
    sorters = {}
    for ms, h in cases:
        if ms not in sorters:
            sorters[ms] = (kvh.HtSorter(kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4), 65536),
                           orc_geom(ORC, ms, 64, 1.0, 4, 4))
        srt, og = sorters[ms]
        items = rng.integers(0, 2 ** 63, len(h), dtype=np.uint64)
        oh, oi = srt.sort(dev(h), items=dev(items), dedup=True, ref_order=True)
        wh, wi, wd = orc_ht_radix_sort_ref(ORC, og, h, items=items, dedup=True)
        np.testing.assert_array_equal(host(oi), wi, err_msg=f"map {ms} n {len(h)}")
        np.testing.assert_array_equal(host(oh), wh, err_msg=f"map {ms} n {len(h)}")
        assert int(srt.dups.item()) == wd


@pytest.mark.parametrize("batch,nb", [(16384, 3), (5000, 3), (32, 3), (65536, 3), (64, 301), (4096, 300),
                                      (64, 1100), (2048, 1030)])
def test_batched_ref_order_vs_oracle(kvh, batch, nb):
    """kvh_ht_sort_batched: ctest's batch loop (ctest.c:34, :90, :96-104) in
    one launch -- every batch equals a separate exact-order sort of it (the
    pinned restatement), duplicate counts per batch, global input indices as
    items, a short last batch; poisoned outputs.  Up to one batch per CU runs
    the 1024-thread form, up to four per CU (nb = 300, 301) the 256-thread
    form, more (1030, 1100) the 128-thread form."""
    rng = np.random.default_rng(batch + nb)
    ms = 5 << 20
    g = kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4)
    og = orc_geom(ORC, ms, 64, 1.0, 4, 4)
    n = nb * batch + batch // 3 + 7
    h = rng.integers(0, 2 ** 64, size=(n, 2), dtype=np.uint64)
    h[rng.integers(0, n, n // 50)] = h[rng.integers(0, n, n // 50)]  # duplicates, some across batches
    oh, oi, dc = kvh.ht_sort_batched(dev(h), g, batch=batch, dedup=True)
    oh, oi, dc = host(oh), host(oi), host(dc)
    assert dc.size == (n + batch - 1) // batch
    check = range(dc.size) if dc.size < 20 or batch <= 64 else \
        sorted(set([0, 1, dc.size - 2, dc.size - 1] + list(rng.integers(0, dc.size, 12))))
    for b in check:
        lo, hi = b * batch, min(n, (b + 1) * batch)
        wh, wi, wd = orc_ht_radix_sort_ref(ORC, og, h[lo:hi], dedup=True)
        np.testing.assert_array_equal(oi[lo:hi], wi + np.uint64(lo), err_msg=f"batch {b}")
        np.testing.assert_array_equal(oh[lo:hi], wh, err_msg=f"batch {b}")
        assert int(dc[b]) == wd
    # items carried, no dedup
    items = rng.integers(0, 2 ** 63, n, dtype=np.uint64)
    oh, oi, _ = kvh.ht_sort_batched(dev(h), g, batch=batch, items=dev(items))
    oh, oi = host(oh), host(oi)
    lo, hi = batch, min(n, 2 * batch)
    wh, wi, _ = orc_ht_radix_sort_ref(ORC, og, h[lo:hi], items=items[lo:hi])
    np.testing.assert_array_equal(oi[lo:hi], wi)
    np.testing.assert_array_equal(oh[lo:hi], wh)


@pytest.mark.parametrize("nseg", [40, 300, 1100])
def test_segments_vs_oracle(kvh, nseg):
    """kvh_ht_sort_segments: batches of any sizes (0, 1, 2, 31, 32, 2049,
    16384 and random ones), each equal to a separate exact-order sort of it,
    per-batch duplicate counts; a batch longer than max_seg is flagged ~0 and
    the others are unaffected.  nseg 40 runs the 1024-thread form, 300 the
    256-thread form, 1100 the 128-thread form."""
    rng = np.random.default_rng(nseg)
    ms = 64 << 20
    g = kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4)
    og = orc_geom(ORC, ms, 64, 1.0, 4, 4)
    sizes = list(rng.integers(0, 3000, nseg))
    sizes[:8] = [0, 1, 2, 31, 32, 2049, 16384, 0]
    big = 5
    sizes[big] = 16385  # longer than max_seg
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    n = int(offs[-1])
    h = rng.integers(0, 2 ** 64, size=(n, 2), dtype=np.uint64)
    h[rng.integers(0, n, n // 40)] = h[rng.integers(0, n, n // 40)]
    oh, oi, dc = kvh.ht_sort_segments(dev(h), g, dev(offs), max_seg=16384, dedup=True)
    oh, oi, dc = host(oh), host(oi), host(dc)
    assert dc.size == nseg and int(dc[big]) == 2 ** 64 - 1
    for b in range(nseg):
        lo, hi = int(offs[b]), int(offs[b + 1])
        if b == big:  # copied through in input order, unmarked
            np.testing.assert_array_equal(oh[lo:hi], h[lo:hi])
            np.testing.assert_array_equal(oi[lo:hi], np.arange(lo, hi, dtype=np.uint64))
            continue
        wh, wi, wd = orc_ht_radix_sort_ref(ORC, og, h[lo:hi], dedup=True)
        np.testing.assert_array_equal(oi[lo:hi], wi + np.uint64(lo), err_msg=f"segment {b}")
        np.testing.assert_array_equal(oh[lo:hi], wh, err_msg=f"segment {b}")
        assert int(dc[b]) == wd, b


def test_segments_bad_offsets_are_flagged_not_followed(kvh):
    """the offsets are device memory, so the kernel checks them
    against n itself.  A segment that ends past n or runs backwards is
    flagged ~0 and nothing of it is written (its range may not exist); the
    valid segments around it are sorted as usual.  The binding rejects
    offsets that are not an int64 device tensor."""
    rng = np.random.default_rng(5)
    ms = 64 << 20
    g = kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4)
    og = orc_geom(ORC, ms, 64, 1.0, 4, 4)
    n = 5000
    h = rng.integers(0, 2 ** 64, size=(n, 2), dtype=np.uint64)
    offs = np.array([0, 1000, 2500, 1500, 1 << 40, 3000, 5000, 5001], dtype=np.uint64)
    oh, oi, dc = kvh.ht_sort_segments(dev(h), g, dev(offs), max_seg=16384, dedup=True)
    oh, oi, dc = host(oh), host(oi), host(dc)
    flagged = {2, 3, 4, 6}  # 2500 -> 1500 reversed, 1500 -> 2^40 past n, 2^40 -> 3000 reversed, 5000 -> 5001 past n
    for b in range(len(offs) - 1):
        if b in flagged:
            assert int(dc[b]) == 2 ** 64 - 1, b
            continue
        lo, hi = int(offs[b]), int(offs[b + 1])
        wh, wi, wd = orc_ht_radix_sort_ref(ORC, og, h[lo:hi], dedup=True)
        np.testing.assert_array_equal(oi[lo:hi], wi + np.uint64(lo), err_msg=f"segment {b}")
        np.testing.assert_array_equal(oh[lo:hi], wh, err_msg=f"segment {b}")
        assert int(dc[b]) == wd
    with pytest.raises(kvh.KvhError):
        kvh.ht_sort_segments(dev(h), g, dev(offs).to(torch.int32), max_seg=16384)
    with pytest.raises(kvh.KvhError):
        kvh.ht_sort_segments(dev(h), g, torch.from_numpy(offs.view(np.int64)), max_seg=16384)


def test_segments_every_step_many_batch_form(kvh):
    """The many-batch form (more batches than CUs: 256 threads, wave nodes
    <= 512, fin in global memory) on the batches that reach every step of
    RadixSort::sort -- hot slots re-pushed down to no bits, clustered slots,
    duplicates, the 1-bit pass, tails -- for each geometry, padded with small
    batches past the CU count; against the pinned restatement."""
    rng = np.random.default_rng(21)
    cases = ref_order_cases(seed=21)
    for ms in sorted(set(m for m, _ in cases)):
        g = kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4)
        og = orc_geom(ORC, ms, 64, 1.0, 4, 4)
        segs = [h for m, h in cases if m == ms]
        segs += [rng.integers(0, 2 ** 64, (int(k), 2), dtype=np.uint64) for k in rng.integers(0, 40, 400)]
        sizes = [len(x) for x in segs]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        h = np.concatenate(segs).astype(np.uint64)
        oh, oi, dc = kvh.ht_sort_segments(dev(h), g, dev(offs), max_seg=16384, dedup=True)
        oh, oi, dc = host(oh), host(oi), host(dc)
        for b in range(len(segs)):
            lo, hi = int(offs[b]), int(offs[b + 1])
            wh, wi, wd = orc_ht_radix_sort_ref(ORC, og, h[lo:hi], dedup=True)
            np.testing.assert_array_equal(oi[lo:hi], wi + np.uint64(lo), err_msg=f"map {ms} segment {b}")
            np.testing.assert_array_equal(oh[lo:hi], wh, err_msg=f"map {ms} segment {b}")
            assert int(dc[b]) == wd


def test_batched_on_a_callers_stream_keeps_its_scratch(kvh):
    """kvh_ht_sort_batched / _segments on a caller's stream return before the
    sort has run, dropping the scratch slices that hold its element indices.
    The binding records them (and the outputs) on that stream, so torch's
    caching allocator does not hand them to work on the current stream while
    the sort still reads them: here the current stream at once fills fresh
    blocks of the same sizes with 0xFF (indices far out of range) while the
    side stream sorts; the results equal the current-stream sort."""
    rng = np.random.default_rng(5)
    ms = 64 << 20
    g = kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4)
    batch, nb = 16384, 600
    n = batch * nb
    h = dev(rng.integers(0, 2 ** 64, size=(n, 2), dtype=np.uint64))
    sizes = rng.integers(0, 16385, 700)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    offs = dev(offs[offs <= n])
    want_b = [host(x) for x in kvh.ht_sort_batched(h, g, batch=batch, dedup=True)]
    want_s = [host(x) for x in kvh.ht_sort_segments(h, g, offs, max_seg=16384, dedup=True)]
    sb = kvh.lib.kvh_ht_sort_batched_scratch_bytes(n, batch)
    ss = kvh.lib.kvh_ht_sort_segments_scratch_bytes(offs.numel() - 1, 16384)
    side = torch.cuda.Stream()
    for _ in range(3):
        got_b = kvh.ht_sort_batched(h, g, batch=batch, dedup=True, stream=side)
        got_s = kvh.ht_sort_segments(h, g, offs, max_seg=16384, dedup=True, stream=side)
        junk = [torch.empty((b + 7) // 8, dtype=torch.int64, device="cuda") for b in (sb, ss)]
        for j in junk:
            j.fill_(-1)
        del junk
        side.synchronize()
        for w, x in zip(want_b, got_b):
            np.testing.assert_array_equal(host(x), w)
        for w, x in zip(want_s, got_s):
            np.testing.assert_array_equal(host(x), w)


def test_batched_bounds(kvh):
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    assert kvh.lib.kvh_ht_sort_batched_scratch_bytes(1000, 0) == 0
    assert kvh.lib.kvh_ht_sort_batched_scratch_bytes(1000, 65537) == 0
    with pytest.raises(kvh.KvhError):
        kvh.ht_sort_batched(dev(np.ones((10, 2), dtype=np.uint64)), g, batch=65537)
    oh, oi, dc = kvh.ht_sort_batched(dev(np.zeros((0, 2), dtype=np.uint64)), g, batch=16384, dedup=True)
    assert oh.shape[0] == 0 and dc.numel() == 0


def test_ref_order_bounds(kvh):
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    srt = kvh.HtSorter(g, 65537)
    h = dev(np.ones((65537, 2), dtype=np.uint64))
    with pytest.raises(kvh.KvhError):
        srt.sort(h, ref_order=True)
    # 0 and 1 elements: nothing to order
    for n in (0, 1):
        oh, oi = srt.sort(dev(np.full((n, 2), 5, dtype=np.uint64)), dedup=True, ref_order=True)
        assert oh.shape[0] == n and int(srt.dups.item()) == 0


def test_edges(kvh):
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    og = orc_geom(ORC, 64 << 20, 64, 1.0, 4, 4)
    srt = kvh.HtSorter(g, 5000)
    rng = np.random.default_rng(2)
    for n in (1, 2, 3, 255, 256, 257, 4999):
        h = rng.integers(0, 2 ** 63, size=(n, 2), dtype=np.uint64)
        oh, oi = srt.sort(dev(h), dedup=True)
        wh, wi, wd = np_ht_sort(og, h, dedup=True)
        np.testing.assert_array_equal(host(oh), wh)
        np.testing.assert_array_equal(host(oi), wi)
    # all identical: one run, n-1 duplicates
    h = np.tile(np.array([[12345, 678]], dtype=np.uint64), (3000, 1))
    oh, oi = srt.sort(dev(h), dedup=True)
    assert int(srt.dups.item()) == 2999
    assert np.all(host(oh)[:-1, 0] == 0) and host(oh)[-1, 0] == 12345


@pytest.mark.parametrize("eng", ENGINES, ids=ENGINE_IDS)
def test_long_runs(kvh, eng):
    """Runs of equal sort prefix longer than k_sort_fixup's insertion-sort
    limit (64) go to k_sort_long's bitonic network: one 30000-element run
    (one h1, random h2 with duplicates), 60 runs of ~500 (60 h1 values), a
    run already in order (skips the network), mixed with random pairs; items
    carried, stable among exact duplicates, dedup counted -- against the
    oracle order."""
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    og = orc_geom(ORC, 64 << 20, 64, 1.0, 4, 4)
    rng = np.random.default_rng(11)
    one = np.stack([np.full(30000, 0x1234_5678_9abc_def0, dtype=np.uint64),
                    rng.integers(0, 8000, 30000, dtype=np.uint64)], axis=1)
    many = np.stack([rng.integers(0, 2 ** 63, 60, dtype=np.uint64)[rng.integers(0, 60, 30000)],
                     rng.integers(0, 2 ** 20, 30000, dtype=np.uint64)], axis=1)
    ordered = np.stack([np.full(3000, 0x0fed_cba9_8765_4321, dtype=np.uint64),
                        np.arange(3000, dtype=np.uint64)], axis=1)
    rand = rng.integers(0, 2 ** 63, size=(20000, 2), dtype=np.uint64)
    h = np.concatenate([one, many, ordered, rand])
    h = h[rng.permutation(len(h))]
    items = rng.integers(0, 2 ** 63, len(h), dtype=np.uint64)
    with _engine(kvh, *eng):
        srt = kvh.HtSorter(g, len(h))
        for dedup in (False, True):
            oh, oi = srt.sort(dev(h), items=dev(items), dedup=dedup)
            wh, wi, wd = np_ht_sort(og, h, items=items, dedup=dedup)
            np.testing.assert_array_equal(host(oh), wh)
            np.testing.assert_array_equal(host(oi), wi)
            if dedup:
                assert int(srt.dups.item()) == wd > 20000
        oh, oi = srt.sort(dev(h), dedup=True)  # items = input index
        wh, wi, wd = np_ht_sort(og, h, dedup=True)
        np.testing.assert_array_equal(host(oh), wh)
        np.testing.assert_array_equal(host(oi), wi)


@pytest.mark.parametrize("n,map_size", [(1, 1 << 30), (2, 1 << 30), (6144, 1 << 30), (6145, 1 << 30),
                                        (12289, 1 << 30), (24577, 1 << 30), (2048, 1 << 30), (2049, 1 << 30),
                                        (65536, 1 << 30), (65537, 1 << 30), (1_000_003, 1 << 30),
                                        (1_000_003, (3 << 28) + 64 * 1000), (30_000_001, (96 << 30) + 64 * 7),
                                        (20_000_000, 1 << 30), (65537, (448 << 10) + 64 * 600), (1_000_003, (448 << 10) + 64 * 600),
                                        (65537, 1 << 40), (1_000_003, 1 << 40)])
def test_engines_agree(kvh, n, map_size):
    """The bucketed engine against the radix engine, word for word, across
    bucket counts (1 .. 4096 buckets, ragged last tiles) and table sizes (a
    600-entry table: most elements share a slot; a 1 TiB table: 35 slot
    bits, past the radix engine's u32 keys), with items and dedup; the
    oracle on the smaller sizes."""
    gen = torch.Generator(device="cuda")
    gen.manual_seed(n)
    h = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device="cuda", generator=gen)
    if n > 100:
        k = n // 100  # 1 % duplicates
        h[torch.randint(0, n, (k,), device="cuda", generator=gen)] = h[torch.randint(0, n, (k,), device="cuda", generator=gen)]
    items = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=gen)
    g = kvh.HtGeom.from_map(map_size, 64, 1.0, 4, 4)
    srt = kvh.HtSorter(g, n)
    res = {}
    for e in (0, 2, 1):
        with _engine(kvh, 0, e):
            oh, oi = srt.sort(h, items=items, dedup=True)
            res[e] = (oh.clone(), oi.clone(), int(srt.dups.item()))
    # the one-workgroup-per-CU bucket sort (knob 22 = 1) on the default engine
    prev = kvh.lib.kvh_set_tuning(22, 1)
    try:
        oh, oi = srt.sort(h, items=items, dedup=True)
        res["cap"] = (oh.clone(), oi.clone(), int(srt.dups.item()))
    finally:
        kvh.lib.kvh_set_tuning(22, prev)
    # the other bucket sort of the product (knob 23 = 0; 3 is the default above)
    for b3 in (0,):
        prev = kvh.lib.kvh_set_tuning(23, b3)
        try:
            oh, oi = srt.sort(h, items=items, dedup=True)
            res[f"sortr{b3}"] = (oh.clone(), oi.clone(), int(srt.dups.item()))
        finally:
            kvh.lib.kvh_set_tuning(23, prev)
    for e in (2, 1, "cap", "sortr0"):
        assert torch.equal(res[0][0], res[e][0]) and torch.equal(res[0][1], res[e][1]) and res[0][2] == res[e][2], e
    if n <= 65537:
        og = orc_geom(ORC, map_size, 64, 1.0, 4, 4)
        wh, wi, wd = np_ht_sort(og, host(h), items=host(items), dedup=True)
        np.testing.assert_array_equal(host(res[0][0]), wh)
        np.testing.assert_array_equal(host(res[0][1]), wi)
        assert res[0][2] == wd


def test_long_run_bound(kvh):
    """A 2M-element batch with one h1 (a single run of distinct h2 in
    reverse order): O(R log^2 R) on one workgroup, well under the test
    timeout, where the insertion sort it replaces is O(R^2)."""
    import time
    n = 2_000_000
    h = np.stack([np.full(n, 77, dtype=np.uint64), np.arange(n, 0, -1, dtype=np.uint64)], axis=1)
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    srt = kvh.HtSorter(g, n)
    d = dev(h)
    t0 = time.time()
    oh, oi = srt.sort(d, dedup=True)
    out = host(oh)
    dt = time.time() - t0
    assert np.array_equal(out[:, 1], np.arange(1, n + 1, dtype=np.uint64))
    assert np.array_equal(host(oi), np.arange(n - 1, -1, -1, dtype=np.uint64))
    assert int(srt.dups.item()) == 0
    assert dt < 30, dt


def test_hot_key_bound(kvh):
    """~20M copies of one (h1, h2) (the KVH_DEDUP hot key) in a
    25M batch on the default engine.  The hot key's bucket overflows the LDS
    sort; the two-pass scatter delivers its records in input order, so
    k_bk_long finds it ordered and emits it in one pass (it took seconds
    through the bitonic network).  Output: the hot key's rows contiguous,
    all but the last marked duplicate, items the input indices in order;
    the rest against the radix engine."""
    import time
    n, hot = 25_000_000, 20_000_000
    gen = torch.Generator(device="cuda")
    gen.manual_seed(9)
    h = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device="cuda", generator=gen)
    sel = torch.randperm(n, device="cuda", generator=gen)[:hot]
    h[sel, 0] = 0x0123_4567_89ab_cdef
    h[sel, 1] = 0x7777
    g = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
    srt = kvh.HtSorter(g, n)
    srt.sort(h, dedup=True)  # warm
    torch.cuda.synchronize()
    t0 = time.time()
    oh, oi = srt.sort(h, dedup=True)
    torch.cuda.synchronize()
    dt = time.time() - t0
    dups = int(srt.dups.item())
    with _engine(kvh, 0, 1):
        rh, ri = srt.sort(h, dedup=True)
        rd = int(srt.dups.item())
    assert torch.equal(oh, rh) and torch.equal(oi, ri) and dups == rd >= hot - 1
    is_hot = (h[oi, 1] == 0x7777) & (h[oi, 0] == 0x0123_4567_89ab_cdef)
    idx = torch.nonzero(is_hot).flatten()
    assert idx.numel() == hot and int(idx[-1] - idx[0]) == hot - 1  # contiguous
    hi = oi[idx]
    assert bool((hi[1:] > hi[:-1]).all())  # input order
    assert dt < 0.5, dt


@pytest.mark.parametrize("inb,hots", [(1_100_000, (900_000,)), (900_000, (600_000, 500_000)),
                                      (1_000_000, (1_000_000,)), (800_000, (400_000, 400_000, 400_000))],
                         ids=["one_hot_45pct", "two_hot_30_25pct", "one_hot_50pct", "three_hot_20pct"])
def test_hot_keys_minority_of_bucket(kvh, inb, hots):
    """hot keys that are NOT the majority of their bucket, and
    several hot keys in one bucket.  `inb` distinct pairs whose h1 share the
    hot keys' top bits (one oversized bucket), the hot keys (`hots` copies
    each, 20-50 % of that bucket), 4M ordinary pairs elsewhere.  Each
    partition of the bucket takes the sampled-mode pivot, so every hot key
    lands in an equal part (already ordered) whatever its share, and the
    ordinary records are partitioned down to LDS-sized parts.  Output
    identical to the radix engine; every hot key contiguous, in input order,
    all but its last copy marked; well under a second."""
    import time
    n = 4_000_000 + inb + sum(hots)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(17)
    base = 0x0123_4567_89ab_0000
    h = torch.randint(0, 2**62, (n, 2), dtype=torch.int64, device="cuda", generator=gen)
    perm = torch.randperm(n, device="cuda", generator=gen)
    sel = perm[:inb]
    h[sel, 0] = base + torch.randint(0, 1 << 16, (inb,), dtype=torch.int64, device="cuda", generator=gen)
    hot, at = [], inb
    for k, m in enumerate(hots):
        sel = perm[at:at + m]
        at += m
        h[sel, 0] = base + 0x1000 * (k + 1)
        h[sel, 1] = 0x7777 + k
        hot.append((base + 0x1000 * (k + 1), 0x7777 + k, m))
    g = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
    srt = kvh.HtSorter(g, n)
    srt.sort(h, dedup=True)  # warm
    torch.cuda.synchronize()
    t0 = time.time()
    oh, oi = srt.sort(h, dedup=True)
    torch.cuda.synchronize()
    dt = time.time() - t0
    dups = int(srt.dups.item())
    with _engine(kvh, 0, 1):
        rh, ri = srt.sort(h, dedup=True)
        rd = int(srt.dups.item())
    assert torch.equal(oh, rh) and torch.equal(oi, ri) and dups == rd >= sum(m - 1 for _, _, m in hot)
    for h1, h2, m in hot:
        idx = torch.nonzero((h[oi, 0] == h1) & (h[oi, 1] == h2)).flatten()
        assert idx.numel() == m and int(idx[-1] - idx[0]) == m - 1  # contiguous
        assert bool((oi[idx][1:] > oi[idx][:-1]).all())  # input order
        assert int((oh[idx, 0] == 0).sum()) == m - 1  # all but the last marked
    assert dt < 0.5, dt


def test_full_size_properties(kvh):
    """100M fixed-up hashes of C1 keys with 1% duplicates into a 64 GiB
    table: output slots non-decreasing, items a permutation, rows equal the
    gathered inputs, duplicate count = n - unique, oracle on a window."""
    n = 100_000_000
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    keys = torch.randint(0, 256, (n * 16,), dtype=torch.uint8, device="cuda", generator=gen)
    h = kvh.meow128_fixed(keys, 16, kvh.STATIC_SEED, fixup=True)
    del keys
    nd = n // 100
    dst = torch.randperm(n, device="cuda", generator=gen)[:nd]
    src = torch.randint(0, n, (nd,), device="cuda", generator=gen)
    h[dst] = h[src]
    g = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
    srt = kvh.HtSorter(g, n)
    oh, oi = srt.sort(h, dedup=False)
    mask, frac, shift = int(g.ht_mod_mask), int(g.ht_mod_fraction), int(g.ht_mod_shift)
    slot = ((oh[:, 0] & mask) * frac) >> shift  # < 2^62: no int64 overflow for this geometry
    assert bool((slot[1:] >= slot[:-1]).all())
    assert bool(torch.equal(torch.sort(oi).values, torch.arange(n, device="cuda")))
    for a in range(0, n, 1 << 23):  # chunked gather (one 100M-row advanced index misreads past 2^26 rows here)
        assert bool(torch.equal(oh[a:a + (1 << 23)], h.index_select(0, oi[a:a + (1 << 23)])))
    uniq = torch.unique(h, dim=0).shape[0]
    _, _ = srt.sort(h, dedup=True)
    assert int(srt.dups.item()) == n - uniq
    # knob 23 = 0 at this size (the default 3 runs 15 bucket bits with an 8-bit second pass): word for word
    prev = kvh.lib.kvh_set_tuning(23, 0)
    try:
        oh3, oi3 = srt.sort(h, dedup=False)
        assert torch.equal(oh3, oh) and torch.equal(oi3, oi)
        _, _ = srt.sort(h, dedup=True)
        assert int(srt.dups.item()) == n - uniq
    finally:
        kvh.lib.kvh_set_tuning(23, prev)
    og = orc_geom(ORC, 64 << 30, 64, 1.0, 4, 4)
    hs = host(h)
    w = np.flatnonzero(np.isin(host(oi), np.arange(0, n, 997)))  # a spread-out sample of rows
    assert np.all(np.diff(np_ht_mod(og, hs[host(oi)[w].astype(np.int64), 0]).astype(np.int64)) >= 0)
