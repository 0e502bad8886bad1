"""GPU parity for SURVEY.md §8 row f3 (key ingest): the device tokenizer,
span hashing with the appended NUL, and packed kv_key_frag_t records vs
the reference's own ctest-style ingest (tests/golden/ingest.npz) and the
oracle (oracle/ingest_oracle.c).  Bit-exact."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle_lib import GOLDEN, load_oracle, orc_hash_spans, orc_tokenize  # noqa: E402

G = np.load(os.path.join(GOLDEN, "ingest.npz"))
ORC = load_oracle()
SEED = tuple(int(x) for x in G["seed"])


@pytest.fixture(scope="module")
def kvh():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    import raikv_amd
    return raikv_amd


def host(t):
    torch.cuda.synchronize()
    a = t.cpu().numpy()
    return a.view(np.uint64) if a.dtype == np.int64 else a.view(np.uint32)


def test_tokenize_and_hash_golden(kvh):
    text = torch.from_numpy(G["text"]).cuda()
    offs, lens = kvh.tokenize(text, 256)
    want_o, want_l = orc_tokenize(ORC, G["text"], 256)
    np.testing.assert_array_equal(host(offs), want_o)
    np.testing.assert_array_equal(host(lens), want_l)
    h = kvh.meow128_spans(text, offs, lens, SEED)
    np.testing.assert_array_equal(host(h), G["hashes"])


def test_frag_records_golden(kvh):
    frags = torch.from_numpy(G["frags"]).cuda()
    ro = torch.from_numpy(G["rec_offs"].view(np.int64)).cuda()
    np.testing.assert_array_equal(host(kvh.meow128_frags(frags, ro, SEED)), G["hashes"])


@pytest.fixture(params=[1, 0], ids=["tok_wave", "tok_wg"])
def tok_kernel(kvh, request):
    """Both tokenizers (kvh_set_tuning(19, v): 1 wave-chunked, 0 workgroup-chunked)."""
    prev = kvh.lib.kvh_set_tuning(19, request.param)
    yield request.param
    kvh.lib.kvh_set_tuning(19, prev)


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 5, 15])
def test_tokenize_unaligned_and_edges(kvh, tok_kernel, shift):
    rng = np.random.default_rng(shift)
    cases = [b"", b"   ", b"a", b" a", b"a ", b"x" * 255 + b" y", b"x" * 256 + b"\ty", b"\n\n\tq\t\n",
             bytes(rng.choice(np.frombuffer(b"ab \n\t", dtype=np.uint8), 70000))]
    for s in cases:
        arr = np.frombuffer(b"#" * shift + s, dtype=np.uint8).copy()
        dev = torch.from_numpy(arr).cuda()[shift:] if arr.size else torch.zeros(0, dtype=torch.uint8, device="cuda")
        offs, lens = kvh.tokenize(dev, 256)
        wo, wl = orc_tokenize(ORC, np.frombuffer(s, dtype=np.uint8).copy(), 256)
        np.testing.assert_array_equal(host(offs), wo)
        np.testing.assert_array_equal(host(lens), wl)
        if len(wo):
            h = kvh.meow128_spans(dev, offs, lens, SEED)
            np.testing.assert_array_equal(host(h), orc_hash_spans(ORC, np.frombuffer(s, np.uint8).copy(), wo, wl,
                                                                   SEED))


def _mixed_text(rng, n):
    """Tokens of 1..8 bytes, runs of separators, and some of 200..40000
    bytes so that tokens cross 16 KiB / 64 KiB chunk seams and the backward
    carry search needs several 256-byte windows."""
    parts, size = [], 0
    while size < n:
        u = rng.random()
        if u < 0.02:
            k = int(rng.integers(200, 40000))
        elif u < 0.1:
            k = int(rng.integers(9, 40))
        else:
            k = int(rng.integers(1, 9))
        parts.append(bytes(rng.integers(33, 127, k, dtype=np.uint8)))
        parts.append(bytes(rng.choice(np.frombuffer(b" \n\t", dtype=np.uint8), int(rng.integers(1, 4)))))
        size += k + 3
    return np.frombuffer(b"".join(parts)[:n], dtype=np.uint8).copy()


@pytest.mark.parametrize("max_token", [1, 5, 16, 17, 256, 5000, 100000])
def test_tokenize_kernels_vs_oracle(kvh, tok_kernel, max_token):
    rng = np.random.default_rng(max_token)
    for shift, n in ((0, 1 << 20), (3, 300001), (13, 16384 * 3 + 5)):
        arr = np.concatenate([np.full(shift, 35, np.uint8), _mixed_text(rng, n)])
        dev = torch.from_numpy(arr).cuda()[shift:]
        offs, lens = kvh.tokenize(dev, max_token)
        wo, wl = orc_tokenize(ORC, arr[shift:], max_token)
        np.testing.assert_array_equal(host(offs), wo)
        np.testing.assert_array_equal(host(lens), wl)


def test_spans_without_nul_match_var(kvh):
    rng = np.random.default_rng(4)
    buf = rng.integers(0, 256, 100000, dtype=np.uint8)
    lens = rng.integers(0, 300, 2000).astype(np.uint32)
    offs = rng.integers(0, 100000 - 300, 2000).astype(np.uint64)
    d = torch.from_numpy(buf).cuda()
    h = kvh.meow128_spans(d, torch.from_numpy(offs.view(np.int64)).cuda(), torch.from_numpy(lens.view(np.int32)).cuda(),
                          SEED, fixup=False, nulterm=False)
    np.testing.assert_array_equal(host(h), orc_hash_spans(ORC, buf, offs, lens, SEED, nul=False, fix=False))


def test_evkey_nul_format(kvh):
    """EvKeyCtx keys (ev_key.h:105-114 copy_key): the string then a '\\0',
    keylen = strlen + 1, hashed by HashSeed::hash.  The expected values come
    from explicit "string\\0" buffers hashed with no appended NUL.  The device
    hashes (offset, strlen) spans inside unterminated text with KVH_NULTERM."""
    rng = np.random.default_rng(11)
    n = 5000
    strl = rng.integers(0, 300, n).astype(np.uint32)
    strl[:40] = np.arange(40)                          # every short length, strlen 0 included
    parts, offs, kb, kb_offs = [], [], [], []
    pos = kpos = 0
    for L in strl:
        s = bytes(rng.integers(1, 256, int(L), dtype=np.uint8))    # no NUL inside a key string
        gap = bytes(rng.integers(1, 256, int(rng.integers(0, 5)), dtype=np.uint8))
        offs.append(pos)
        parts += [s, gap]
        pos += len(s) + len(gap)
        kb_offs.append(kpos)
        kb.append(s + b"\0")
        kpos += len(s) + 1
    text = np.frombuffer(b"".join(parts) + b"x", dtype=np.uint8).copy()
    kbuf = np.frombuffer(b"".join(kb), dtype=np.uint8).copy()
    want = orc_hash_spans(ORC, kbuf, np.array(kb_offs, np.uint64), strl + 1, SEED, nul=False, fix=True)
    h = kvh.meow128_spans(torch.from_numpy(text).cuda(), torch.from_numpy(np.array(offs, np.int64)).cuda(),
                          torch.from_numpy(strl.view(np.int32)).cuda(), SEED)
    np.testing.assert_array_equal(host(h), want)


def test_cap_truncates_but_counts(kvh, tok_kernel):
    text = torch.from_numpy(G["text"]).cuda()
    offs, lens = kvh.tokenize(text, 256, cap=100)
    want_o, _ = orc_tokenize(ORC, G["text"], 256)
    assert offs.numel() == 100
    np.testing.assert_array_equal(host(offs), want_o[:100])


def test_large_text_property(kvh, tok_kernel):
    """1 GiB of synthetic text (≈ 180M tokens): device tokens equal the
    oracle on sampled 64 KiB windows away from chunk seams, counts are
    consistent, and spans hash == packed-record hash on a sample."""
    n = 1 << 30
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=gen)
    # ~25% separators
    text = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
    del r
    offs, lens = kvh.tokenize(text, 256)
    o, l = host(offs), host(lens)
    assert np.all(np.diff(o.astype(np.int64)) > 0) and np.all(l > 0) and np.all(l < 256)
    th = text.cpu().numpy()
    for start in (0, 12345678, (1 << 29) + 77, n - 70000):
        seg = th[start:start + 65536]
        wo, wl = orc_tokenize(ORC, seg, 256)
        # compare tokens strictly inside the window (first/last may be cut)
        inner = (wo > 0) & (wo + wl < len(seg))
        a = np.searchsorted(o, start + wo[inner])
        np.testing.assert_array_equal(o[a], start + wo[inner])
        np.testing.assert_array_equal(l[a], wl[inner])


@pytest.mark.parametrize("kernel", [0, 1, 2])
@pytest.mark.parametrize("nulterm", [True, False])
def test_spans_kernels_vs_oracle(kvh, kernel, nulterm):
    """Both span kernels (lane per span; short spans in place with the long
    ones queued per wave, knob 18) on spans of 0..40 bytes with a long one
    every so often, so that chunks are all short, all long and mixed; odd
    counts for the chunk tails; 600001 mostly-long spans so that each wave
    walks several chunks and its queue overflows 64 and carries over."""
    rng = np.random.default_rng(17 + kernel + 2 * nulterm)
    buf = rng.integers(0, 256, 400000, dtype=np.uint8)
    for n in (1, 63, 129, 4097, 50001, 600001):
        lens = rng.integers(0, 16 if n not in (4097, 600001) else 41, n).astype(np.uint32)
        if n > 1000:
            lens[rng.integers(0, n, n // 500)] = rng.integers(16, 300, n // 500).astype(np.uint32)
        offs = rng.integers(0, 400000 - 300, n).astype(np.uint64)
        prev = kvh.lib.kvh_set_tuning(18, kernel)
        try:
            h = kvh.meow128_spans(torch.from_numpy(buf).cuda(), torch.from_numpy(offs.view(np.int64)).cuda(),
                                  torch.from_numpy(lens.view(np.int32)).cuda(), SEED, nulterm=nulterm)
            np.testing.assert_array_equal(host(h), orc_hash_spans(ORC, buf, offs, lens, SEED, nul=nulterm))
        finally:
            kvh.lib.kvh_set_tuning(18, prev)


@pytest.mark.parametrize("max_token", [1, 5, 16, 17, 256, 5000, 40000])
def test_tokenize_hash_fused_vs_oracle(kvh, max_token):
    """kvh_tokenize_hash (tokenizer, then the span hash reading the token count
    on the device) against the oracle's tokens and span hashes, with and
    without the NUL, at three text misalignments; the golden text against the
    reference's own kv_hash_key_frag hashes, also with cap below the count."""
    rng = np.random.default_rng(max_token + 1)
    for shift, n, nul in ((0, 1 << 20, True), (3, 300001, False), (13, 16384 * 3 + 5, True)):
        arr = np.concatenate([np.full(shift, 35, np.uint8), _mixed_text(rng, n)])
        dev = torch.from_numpy(arr).cuda()[shift:]
        o, l, h = kvh.tokenize_hash(dev, SEED, max_token, nulterm=nul)
        wo, wl = orc_tokenize(ORC, arr[shift:], max_token)
        np.testing.assert_array_equal(host(o), wo)
        np.testing.assert_array_equal(host(l), wl)
        np.testing.assert_array_equal(host(h), orc_hash_spans(ORC, arr[shift:], wo, wl, SEED, nul=nul))
    if max_token == 256:
        o, l, h = kvh.tokenize_hash(torch.from_numpy(G["text"]).cuda(), SEED, 256)
        np.testing.assert_array_equal(host(h), G["hashes"])
        _, _, hc = kvh.tokenize_hash(torch.from_numpy(G["text"]).cuda(), SEED, 256, cap=100)
        np.testing.assert_array_equal(host(hc), G["hashes"][:100])


def _token_text(rng, n, lo, hi):
    """Tokens of lo..hi-1 bytes separated by single separators."""
    parts, size = [], 0
    while size < n:
        k = int(rng.integers(lo, hi))
        parts.append(bytes(rng.integers(33, 127, k, dtype=np.uint8)))
        parts.append(bytes(rng.choice(np.frombuffer(b" \n\t", dtype=np.uint8), 1)))
        size += k + 1
    return np.frombuffer(b"".join(parts)[:n], dtype=np.uint8).copy()


@pytest.mark.parametrize("lo,hi", [(1, 2), (14, 18), (15, 32), (28, 36), (30, 300), (1, 40)])
def test_tokenize_hash_length_mixes(kvh, lo, hi):
    """Token-length mixes that load each path of the span hash: one-byte
    tokens (512 per tokenizer pass), all-medium tokens (the medium queue
    flushing every chunk), the short/medium seam at 15/16 and the
    medium/long seam at 31/32 hashed bytes, mostly long tokens, and a cap
    that cuts the tokens mid-chunk.  Poisoned outputs, against the oracle."""
    rng = np.random.default_rng(lo * 1000 + hi)
    for shift, n, nul in ((0, 1 << 19, True), (7, 200003, False)):
        arr = np.concatenate([np.full(shift, 35, np.uint8), _token_text(rng, n, lo, hi)])
        dev = torch.from_numpy(arr).cuda()[shift:]
        wo, wl = orc_tokenize(ORC, arr[shift:], 256)
        want = orc_hash_spans(ORC, arr[shift:], wo, wl, SEED, nul=nul)
        o, l, h = kvh.tokenize_hash(dev, SEED, 256, nulterm=nul)
        np.testing.assert_array_equal(host(o), wo)
        np.testing.assert_array_equal(host(l), wl)
        np.testing.assert_array_equal(host(h), want)
        cap = int(wo.size * 0.6) + 7
        o, l, h = kvh.tokenize_hash(dev, SEED, 256, cap=cap, nulterm=nul)
        np.testing.assert_array_equal(host(o), wo[:cap])
        np.testing.assert_array_equal(host(h), want[:cap])


def test_tokenize_hash_large_text(kvh):
    """1 GiB of f3 text: one-call hashes equal tokenize + span hash, bit for bit."""
    n = 1 << 30
    gen = torch.Generator(device="cuda")
    gen.manual_seed(12)
    r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=gen)
    text = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
    del r
    o, l, h = kvh.tokenize_hash(text, SEED, 256)
    o2, l2 = kvh.tokenize(text, 256)
    assert torch.equal(o, o2) and torch.equal(l, l2)
    del o2
    h2 = kvh.meow128_spans(text, o, l2, SEED)
    assert torch.equal(h, h2)


def test_ctest_pipeline_on_device(kvh):
    """ctest's whole ingest on the device, as raikv's test program runs it
    (ctest.c:73-104, :195-237, :316-340): the input read in 256 KiB blocks,
    each block tokenized on its own (its end is a separator) into
    NUL-terminated frag hashes with the table's seed (kvh_tokenize_hash), the
    batches cut per block (16K frags or a full 64 KiB frag buffer; count and
    buffer restart at each block, tests/ctest_batches.py), then every batch in
    kv_ht_radix_sort's exact order with its adjacent-duplicate marking (one
    kvh_ht_sort_segments call).  Every batch equals the pinned restatement of
    the reference sort, some also the reference compiled from its sources, and
    the total is ctest's dup_count."""
    from ctest_batches import ctest_block_batches, ctest_blocks
    from oracle_lib import load_ref_ht, orc_geom, orc_ht_radix_sort_ref, ref_ht_sort
    rng = np.random.default_rng(11)
    ms = 64 << 20
    og = orc_geom(ORC, ms, 64, 1.0, 4, 4)
    g = kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4)
    ref = load_ref_ht()
    # the golden text (the reference's own hashes pinned above) and 3 MB of words, many repeated
    words = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(1, 14, 4000)]
    parts = [words[int(i)] + (b" " if j % 9 else b"\n") for j, i in enumerate(rng.integers(0, 4000, 400000))]
    for text in (G["text"], np.frombuffer(b"".join(parts), dtype=np.uint8).copy()):
        dt = torch.from_numpy(text).cuda()
        hb, lb = [], []
        for s0, e0 in ctest_blocks(text.size):  # one ctest read() block each
            o, l, h = kvh.tokenize_hash(dt[s0:e0], SEED, 256)
            hb.append(h)
            lb.append(host(l))
        h = torch.cat(hb)
        cuts = ctest_block_batches(lb)
        assert len(lb) > 1 and int(cuts[-1]) == h.shape[0]
        segs = dev64(cuts)
        hs, oi, dc = kvh.ht_sort_segments(h, g, segs, max_seg=16 * 1024, dedup=True)
        hs, oi, dc, hh = host(hs).reshape(-1, 2), host(oi), host(dc), host(h).reshape(-1, 2)
        total = 0
        for b in range(len(cuts) - 1):
            lo, hi = int(cuts[b]), int(cuts[b + 1])
            wh, wi, wd = orc_ht_radix_sort_ref(ORC, og, hh[lo:hi], dedup=True)
            np.testing.assert_array_equal(oi[lo:hi], wi + np.uint64(lo), err_msg=f"batch {b}")
            np.testing.assert_array_equal(hs[lo:hi], wh, err_msg=f"batch {b}")
            assert int(dc[b]) == wd
            if ref is not None and b < 3:  # the reference's own kv_ht_radix_sort + ctest marking
                rh, ri, rd = ref_ht_sort(ref, ms, hh[lo:hi])
                np.testing.assert_array_equal(hs[lo:hi], rh)
                np.testing.assert_array_equal(oi[lo:hi], ri + np.uint64(lo))
                assert int(dc[b]) == rd
            total += wd
        assert int(dc.sum()) == total
    assert total > 0 and len(cuts) > 10


def dev64(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def _pack_frags(rng, lens, truncate=0):
    """kv_key_frag_t records {u16 keylen, bytes, pad to 2} back to back."""
    parts, offs, o = [], [], 0
    for L in lens:
        rec = int(L).to_bytes(2, "little") + bytes(rng.integers(0, 256, int(L), dtype=np.uint8))
        if len(rec) & 1:
            rec += b"\0"
        parts.append(rec)
        offs.append(o)
        o += len(rec)
    buf = b"".join(parts)
    if truncate:
        buf = buf[:-truncate]
    return np.frombuffer(buf, dtype=np.uint8).copy(), np.array(offs, dtype=np.uint64)


def test_frag_stream_golden(kvh):
    """The reference's own packed frag records (ctest's buffer) parse on the
    device to its record offsets and hash to its kv_hash_key_frag hashes."""
    frags = torch.from_numpy(G["frags"]).cuda()
    np.testing.assert_array_equal(host(kvh.frag_offsets(frags)), G["rec_offs"].astype(np.uint64))
    o, h = kvh.frags_hash(frags, SEED)
    np.testing.assert_array_equal(host(o), G["rec_offs"].astype(np.uint64))
    np.testing.assert_array_equal(host(h), G["hashes"])
    _, h100 = kvh.frags_hash(frags, SEED, cap=100)
    np.testing.assert_array_equal(host(h100), G["hashes"][:100])


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 100003])
def test_frag_stream_random(kvh, n):
    """Random streams (keylen 0..300, odd and even), the last record cut
    short (it must end the stream), against the host packer's offsets and
    the oracle's hash of each record's bytes."""
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 301, n)
    lens[rng.integers(0, n, max(1, n // 10))] = rng.integers(0, 3, max(1, n // 10))
    buf, offs = _pack_frags(rng, lens)
    np.testing.assert_array_equal(host(kvh.frag_offsets(torch.from_numpy(buf).cuda())), offs)
    o, h = kvh.frags_hash(torch.from_numpy(buf).cuda(), SEED)
    np.testing.assert_array_equal(host(o), offs)
    sp_off = offs + 2
    want = orc_hash_spans(ORC, buf, sp_off, lens.astype(np.uint32), SEED, nul=False)
    np.testing.assert_array_equal(host(h), want)
    if n > 1 and lens[-1] > 1:
        bt, _ = _pack_frags(np.random.default_rng(n), lens, truncate=1 + (lens[-1] & 1))
        np.testing.assert_array_equal(host(kvh.frag_offsets(torch.from_numpy(bt).cuda())), offs[:-1])


def test_frag_stream_tiny(kvh):
    for b in (b"", b"\x00", b"\x00\x00", b"\x01\x00a", b"\x01\x00a\x00", b"\x05\x00ab"):
        arr = np.frombuffer(b, dtype=np.uint8).copy()
        dev = torch.from_numpy(arr).cuda() if arr.size else torch.zeros(0, dtype=torch.uint8, device="cuda")
        got = host(kvh.frag_offsets(dev))
        want = {b"": [], b"\x00": [], b"\x00\x00": [0], b"\x01\x00a": [0], b"\x01\x00a\x00": [0], b"\x05\x00ab": []}[b]
        np.testing.assert_array_equal(got, np.array(want, dtype=np.uint64), err_msg=repr(b))


def test_side_stream_counts(kvh):
    """the count-returning calls on a caller's own non-blocking
    stream (torch.cuda.Stream and a raw stream handle) read the count only
    after their kernels ran, and order after the current stream's zero fill
    of it: the same results as on the current stream, repeatedly."""
    text = torch.from_numpy(G["text"]).cuda()
    frags = torch.from_numpy(G["frags"]).cuda()
    want_o, want_l = orc_tokenize(ORC, G["text"], 256)
    side = torch.cuda.Stream()
    for st in (side, side.cuda_stream):
        for _ in range(3):
            o, l = kvh.tokenize(text, 256, stream=st)
            np.testing.assert_array_equal(host(o), want_o)
            np.testing.assert_array_equal(host(l), want_l)
            o2, l2, h2 = kvh.tokenize_hash(text, SEED, 256, stream=st)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(host(h2), G["hashes"])
            ro = kvh.frag_offsets(frags, stream=st)
            np.testing.assert_array_equal(host(ro), G["rec_offs"])
            ro2, hh = kvh.frags_hash(frags, SEED, stream=st)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(host(hh), G["hashes"])
