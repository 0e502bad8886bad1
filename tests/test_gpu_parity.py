"""GPU parity: every device path through the C-ABI vs the oracle and the
reference's golden vectors.  Bit-exact (integer/byte work).

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle_lib import (GOLDEN, ROOT, golden, load_oracle, orc_fixed, orc_meow, orc_multiseed,  # noqa: E402
                        orc_var)

ORC = load_oracle()
VEC = json.load(open(os.path.join(GOLDEN, "reference_vectors.json")))
STATIC = (0xA8E0BCC94D1855F5, 0xAD3BEC1E8DE4A1A3)


# pinned host buffers of these tests, kept to the end of the process
_PINNED = []


@pytest.fixture(scope="module")
def kvh():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    import raikv_amd
    return raikv_amd


def dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def dev_u64(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def u64(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("L", [8, 16, 24, 32, 40, 48, 56, 64, 1, 13, 100, 255])
def test_fixed_golden(kvh, L):
    g = golden(f"fixed_{L}.npz")
    out = kvh.meow128_fixed(dev(g["keys"]), L, STATIC)
    np.testing.assert_array_equal(u64(out), g["out"])
    # KeyFragment::hash epilogue fused
    fx = kvh.meow128_fixed(dev(g["keys"]), L, STATIC, fixup=True)
    np.testing.assert_array_equal(u64(fx), orc_fixed(ORC, g["keys"], L, STATIC, fixup=True))


def poisoned_like(t):
    o = torch.empty_like(t)
    o.view(torch.uint8).fill_(0xA5)
    return o


@pytest.mark.parametrize("order,delay", [(0, 0), (2, 0), (0, 6)])
def test_fixed_in_order_tickets(kvh, order, delay):
    """Knob 24: 0 the per-length default, 2 k_fixed_qw (wave tickets): chunks
    taken in address order from a per-stream ticket counter that the last
    workgroup resets.  Equal to the static-order kernel (knob 24 = 1) and the
    oracle over ragged sizes (one key, under one workgroup-iteration, ragged
    last chunks), over many launches in a row on one stream (the reset), and
    with launches on two streams in flight at once (separate counters).
    Every output starts as 0xA5 bytes (conftest: the binding poisons what it
    allocates), so a chunk no wave hashed fails the comparison.  delay: knob 26
    makes the fetchers of every other ticket sleep ~25 us first, which
    reordered the round-4 fetches (tickets.hpp)."""
    rng = np.random.default_rng(24)
    prev_order = kvh.lib.kvh_set_tuning(24, order)
    prev_delay = kvh.lib.kvh_set_tuning(26, delay)
    try:
        _tickets_cases(kvh, rng)
    finally:
        kvh.lib.kvh_set_tuning(24, prev_order)
        kvh.lib.kvh_set_tuning(26, prev_delay)


def _tickets_cases(kvh, rng):
    for L in (16, 32, 64, 24, 8, 40, 48, 56):
        for n in (1, 63, 4095, 4097, 65536 * 3 + 5, 1_000_003):
            kb = rng.integers(0, 256, n * L, dtype=np.uint8)
            t = dev(kb)
            got = u64(kvh.meow128_fixed(t, L, STATIC))
            prev = kvh.lib.kvh_set_tuning(24, 1)
            try:
                stat = u64(kvh.meow128_fixed(t, L, STATIC))
            finally:
                kvh.lib.kvh_set_tuning(24, prev)
            np.testing.assert_array_equal(got, stat, err_msg=f"L={L} n={n}")
            m = min(n, 3000)
            np.testing.assert_array_equal(got[:m], orc_fixed(ORC, kb[:m * L], L, STATIC))
            np.testing.assert_array_equal(got[-m:], orc_fixed(ORC, kb[(n - m) * L:], L, STATIC))
    # many launches in a row: every one must start from a zero counter
    n = 2_000_003
    t = torch.randint(0, 256, (n * 16,), dtype=torch.uint8, device="cuda")
    want = kvh.meow128_fixed(t, 16, STATIC)
    outs = [poisoned_like(want) for _ in range(50)]
    for o in outs:
        kvh.meow128_fixed(t, 16, STATIC, out=o)
    torch.cuda.synchronize()
    assert all(torch.equal(o, want) for o in outs)
    # two streams at once
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1, o2 = poisoned_like(want), poisoned_like(want)
    torch.cuda.synchronize()
    for _ in range(10):
        kvh.meow128_fixed(t, 16, STATIC, out=o1, stream=s1)
        kvh.meow128_fixed(t, 16, STATIC, out=o2, stream=s2)
    torch.cuda.synchronize()
    assert torch.equal(o1, want) and torch.equal(o2, want)


@pytest.mark.parametrize("delay", [0, 6])
@pytest.mark.parametrize("n", [1, 4097, 1_000_003])
def test_order_knob_every_streaming_kernel(kvh, n, delay):
    """Every kernel that takes its chunks through wave tickets by default
    (runtime-length k_fixed_rt, k_fixed_lanes (C3), the fused hash+positions
    kernel, CRC32C of fixed and of variable-length keys, the variable-length
    kernel, the span hash alone and behind the tokenizer) equals its
    static-order form (knob 24 = 1) on the same input, twice in a row (the
    counter reset), into poisoned outputs; delay = knob 26 (fetches of every
    other ticket delayed, tickets.hpp)."""
    from raikv_amd.workload import C3_SEEDS
    rng = np.random.default_rng(n)
    geom = kvh.HtGeom.from_map(map_size=1 << 30, hash_entry_size=64, hash_value_ratio=1.0, cuckoo_buckets=4,
                               cuckoo_arity=4)
    k16 = dev(rng.integers(0, 256, n * 16, dtype=np.uint8))
    k32 = dev(rng.integers(0, 256, n * 32, dtype=np.uint8))
    k20 = dev(rng.integers(0, 256, n * 20, dtype=np.uint8))
    k50 = dev(rng.integers(0, 256, n * 50, dtype=np.uint8))
    lens = rng.integers(0, 300, n).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    kv, dof = dev(rng.integers(0, 256, int(offs[-1]) + 1, dtype=np.uint8)), dev(offs.view(np.int64))
    dlen = dev(np.minimum(lens, 40).astype(np.int32))  # spans of 0-40 bytes at the var keys' offsets
    tb = rng.choice(np.frombuffer(b"abcdefgh \n\t", dtype=np.uint8), size=max(16, n * 4))
    text = dev(tb)
    runs = {
        "rt20": lambda: kvh.meow128_fixed(k20, 20, STATIC),
        "rt50": lambda: kvh.meow128_fixed(k50, 50, STATIC),
        "c3": lambda: kvh.meow128_multiseed(k32, 32, list(C3_SEEDS)),
        "fused": lambda: torch.cat([t.view(torch.int64).reshape(n, -1) for t in
                                    kvh.meow128_fixed_positions(k16, 16, STATIC, geom)], 1),
        "crc16": lambda: kvh.crc_c_fixed(k16, 16, 7),
        "crc_var": lambda: kvh.crc_c_var(kv, dof, 7),
        "var": lambda: kvh.meow128_var(kv, dof, STATIC),
        # spans with a long / medium / short mix (k_spans' three paths and queues)
        "spans": lambda: kvh.meow128_spans(kv, dof[:-1], dlen, STATIC),
        "tokenize_hash": lambda: kvh.tokenize_hash(text, STATIC)[2],
    }
    for name, run in runs.items():
        prev = kvh.lib.kvh_set_tuning(24, 1)
        try:
            want = run().cpu()
        finally:
            kvh.lib.kvh_set_tuning(24, prev)
        prev_delay = kvh.lib.kvh_set_tuning(26, delay)
        try:
            for _ in range(2):
                got = run().cpu()
                assert torch.equal(got, want), f"{name} n={n}"
        finally:
            kvh.lib.kvh_set_tuning(26, prev_delay)


def test_all_lengths_0_300_all_paths(kvh):
    g = golden("lengths.npz")
    keys, seeds, out = g["keys"], g["seeds"], g["out"]
    maxl = keys.shape[0] - 1
    lens = np.arange(maxl + 1, dtype=np.uint32)
    offs = np.zeros(maxl + 2, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    flat = np.concatenate([keys[L, :L] for L in range(maxl + 1)])
    dk, doff = dev(flat), dev_u64(offs)
    for si in range(seeds.shape[0]):
        s = (int(seeds[si, 0]), int(seeds[si, 1]))
        # variable-length kernel, every length in one batch
        np.testing.assert_array_equal(u64(kvh.meow128_var(dk, doff, s)), out[:, si], err_msg=f"var seed {si}")
        # straight-line kernel with per-key seeds
        sd = dev_u64(np.tile(np.array(s, dtype=np.uint64), (maxl + 1, 1)))
        np.testing.assert_array_equal(u64(kvh.meow128_var_seeded(dk, doff, sd)), out[:, si])
    # fixed-length entry for every length (fast kernels for L%8==0, generic otherwise),
    # all four seeds at once through the multi-seed entry
    sl = [(int(a), int(b)) for a, b in seeds]
    for L in range(1, maxl + 1):
        got = u64(kvh.meow128_multiseed(dev(keys[L, :L].copy()), L, sl))
        np.testing.assert_array_equal(got[0], out[L], err_msg=f"L={L}")
        got1 = u64(kvh.meow128_fixed(dev(keys[L, :L].copy()), L, sl[3]))
        np.testing.assert_array_equal(got1[0], out[L, 3], err_msg=f"fixed L={L}")


def test_fixed_every_length_batched(kvh):
    """Every length 1..70 as a batch of a few thousand keys (the runtime-length
    kernel for 1..63 outside the multiples of 8, its byte-exact last chunk, the
    specialised kernels, k_generic past 63), at a 16-byte aligned, an 8-byte
    aligned (the per-key loads where 64-byte keys otherwise go by lane pairs)
    and an odd base, against the oracle."""
    rng = np.random.default_rng(70)
    for L in range(1, 71):
        n = 2000 + 37 * L
        for shift in (0, 8, 3):
            raw = rng.integers(0, 256, n * L + shift, dtype=np.uint8)
            t = dev(raw)
            got = u64(kvh.meow128_fixed(t[shift:], L, STATIC, n=n))
            np.testing.assert_array_equal(got, orc_fixed(ORC, raw[shift:].copy(), L, STATIC),
                                          err_msg=f"L={L} shift={shift}")


def test_var_zipf_golden(kvh):
    g = golden("var_zipf.npz")
    out = kvh.meow128_var(dev(g["keys"]), dev_u64(g["offsets"]), STATIC)
    np.testing.assert_array_equal(u64(out), g["out"])
    fx = kvh.meow128_var(dev(g["keys"]), dev_u64(g["offsets"]), STATIC, fixup=True)
    np.testing.assert_array_equal(u64(fx), orc_var(ORC, g["keys"], g["offsets"], STATIC, fixup=True))


def test_multiseed_golden_and_arities(kvh):
    g = golden("multiseed4_32.npz")
    seeds = [tuple(int(x) for x in s) for s in g["seeds"].reshape(-1, 2)]
    np.testing.assert_array_equal(u64(kvh.meow128_multiseed(dev(g["keys"]), 32, seeds)), g["out"])
    rng = np.random.default_rng(4)
    for L in (16, 32, 64, 24, 20):
        kb = rng.integers(0, 256, 3000 * L, dtype=np.uint8)
        for a in range(1, 9):
            ss = [(int(rng.integers(0, 2**63)) * 2 + 1, int(rng.integers(0, 2**63))) for _ in range(a)]
            got = u64(kvh.meow128_multiseed(dev(kb), L, ss))
            np.testing.assert_array_equal(got.reshape(-1, a, 2), orc_multiseed(ORC, kb, L, ss), err_msg=f"{L} {a}")


def test_hash_test_int_keys(kvh):
    g = golden("hash_test_int16.npz")
    np.testing.assert_array_equal(u64(kvh.meow128_fixed(dev(g["keys"]), 16, (0, 0))), g["out"])


def test_unaligned_bases_and_allocation_end(kvh):
    rng = np.random.default_rng(5)
    for L in (16, 32, 13, 8, 64, 3):
        n = 5000
        for shift in (1, 3, 4, 8):
            raw = rng.integers(0, 256, n * L + shift, dtype=np.uint8)
            t = dev(raw)
            view = t[shift:]  # device pointer at base + shift
            got = u64(kvh.meow128_fixed(view, L, STATIC, n=n))
            np.testing.assert_array_equal(got, orc_fixed(ORC, raw[shift:].copy(), L, STATIC), err_msg=f"{L}+{shift}")
    # keys ending exactly at the end of a fresh allocation (odd sizes)
    for L in (1, 7, 13, 31, 33, 255):
        n = 777
        kb = rng.integers(0, 256, n * L, dtype=np.uint8)
        t = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        t.copy_(torch.from_numpy(kb))
        np.testing.assert_array_equal(u64(kvh.meow128_fixed(t, L, STATIC)), orc_fixed(ORC, kb, L, STATIC))


def test_empty_single_and_zero_length(kvh):
    z = torch.empty(0, dtype=torch.uint8, device="cuda")
    assert kvh.meow128_fixed(z, 16, STATIC).shape == (0, 2)
    one = np.frombuffer(b"hello\0", dtype=np.uint8).copy()
    got = u64(kvh.meow128_var(dev(one), dev_u64(np.array([0, 6], dtype=np.uint64)), STATIC))
    assert "%016x:%016x" % tuple(int(v) for v in got[0]) == "2aa73a1eeb0b2d45:fd102121185ce157"
    # all-empty keys through the var kernel
    offs = np.zeros(1001, dtype=np.uint64)
    got = u64(kvh.meow128_var(dev(one), dev_u64(offs), (7, 9)))
    assert np.all(got == np.array(orc_meow(ORC, b"", 7, 9), dtype=np.uint64))


def test_drop_ins_against_reference_vectors(kvh):
    for k in VEC["kat"]:
        assert "%016x:%016x" % kvh.kv_hash_meow128(bytes.fromhex(k["key_hex"]), *k["seed"]) == k["h"]
    for m in VEC["meow64"]:
        assert kvh.kv_hash_meow64(bytes.fromhex(m["key_hex"]), m["seed"]) == m["h"]
    r = VEC["variants"]["results"]
    keys = [k.encode() for k in VEC["variants"]["keys"]]
    s1, s2 = VEC["variants"]["seed"]
    L = len(keys[0])
    bufs = [C.create_string_buffer(k, L) for k in keys]
    lib = kvh.lib
    x = (C.c_uint64 * 8)(*([s1, s2] * 4))
    assert lib.kvh_hash_meow128_2_same_length(bufs[0], bufs[1], L, x) == 0
    assert lib.kvh_hash_meow128_2_same_length(bufs[2], bufs[3], L, C.c_void_p(C.addressof(x) + 32)) == 0
    assert list(x) == r["2_same"]
    x = (C.c_uint64 * 8)(*([s1, s2] * 4))
    assert lib.kvh_hash_meow128_4_diff_length(bufs[0], L, bufs[1], L, bufs[2], L, bufs[3], L, x) == 0
    assert list(x) == r["4_diff"]
    x = (C.c_uint64 * 8)(*([s1, s2] * 4))
    assert lib.kvh_hash_meow128_4_same_length(bufs[0], bufs[1], bufs[2], bufs[3], L, x) == 0
    assert list(x) == r["4_same"]
    x = (C.c_uint64 * 16)(*([s1, s2] * 8))
    pa = (C.c_void_p * 8)(*[C.cast(b, C.c_void_p) for b in bufs + bufs])
    assert lib.kvh_hash_meow128_8_same_length_a(pa, L, x) == 0
    assert list(x) == r["8_same"]
    x = (C.c_uint64 * 8)(*r["4_same_4_seed"]["seeds"])
    assert lib.kvh_hash_meow128_4_same_length_4_seed(bufs[0], bufs[1], bufs[2], bufs[3], L, x) == 0
    assert list(x) == r["4_same_4_seed"]["x"]
    for i, k in enumerate(keys):
        a, b = C.c_uint64(s1), C.c_uint64(s2)
        assert lib.kvh_meow_test(bufs[i], L, C.byref(a), C.byref(b)) == 0
        assert [a.value, b.value] == r["stream"][i]
    # KeyFragment / HashSeed mirrors with the fixup
    hs = kvh.HashSeed(*STATIC)
    kf = kvh.KeyFragment.from_string("hello")
    assert hs.hash(kf) == (0x2AA73A1EEB0B2D45 & ~(1 << 63), 0xFD102121185CE157)
    frags = [kvh.KeyFragment(bytes([i]) * i) for i in range(40)]
    got = hs.hash_batch(frags)
    for i, f in enumerate(frags):
        h1, h2 = orc_meow(ORC, f.data, *STATIC)
        assert int(got[i, 0]) == int(ORC.orc_fixup(h1)) and int(got[i, 1]) == h2


def test_streaming_uneven_updates(kvh):
    lib = kvh.lib
    data = bytes(range(256)) * 4
    for total in (0, 1, 15, 16, 63, 64, 65, 127, 128, 300, 1000):
        m = C.create_string_buffer(64 + 64)
        b = C.create_string_buffer(128)
        # 64-byte alignment of the ctx struct is not needed by the GPU path
        assert lib.kvh_meow128_init(m, b, 11, 22, total) == 0
        pos = 0
        for piece in (3, 64, 1, 70, 200, 1000):
            take = min(piece, total - pos)
            if take <= 0:
                break
            assert lib.kvh_meow128_update(m, b, C.create_string_buffer(data[pos:pos + take], take), take) == 0
            pos += take
        h1, h2 = C.c_uint64(11), C.c_uint64(22)
        assert lib.kvh_meow128_final(m, b, C.byref(h1), C.byref(h2)) == 0
        assert (h1.value, h2.value) == orc_meow(ORC, data[:total], 11, 22), total


def test_host_pipeline_pinned_and_pageable(kvh):
    rng = np.random.default_rng(6)
    n, L = 3_000_001, 16
    kb = rng.integers(0, 256, n * L, dtype=np.uint8)
    want = u64(kvh.meow128_fixed(dev(kb), L, STATIC))
    got = kvh.meow128_fixed_host(kb, L, STATIC)
    np.testing.assert_array_equal(got, want)
    pk = torch.from_numpy(kb).pin_memory()
    po = torch.empty((n, 2), dtype=torch.int64).pin_memory()
    got2 = kvh.meow128_fixed_host(pk.numpy(), L, STATIC, out=po.numpy().view(np.uint64))
    np.testing.assert_array_equal(got2, want)
    # kvh_host_alloc buffers; chunk sizes that leave a ragged last chunk; slot
    # reuse (more chunks than slots) and one chunk only
    hk = kvh.host_empty((n * L,), np.uint8)
    hk[:] = kb
    ho = kvh.host_empty((n, 2), np.uint64)
    _PINNED.extend((hk, ho))  # never handed back during the session
    for mib, slots in ((1, 2), (4, 4), (64, 16)):
        pm, ps = kvh.lib.kvh_set_tuning(15, mib), kvh.lib.kvh_set_tuning(16, slots)
        try:
            ho[:] = 0
            kvh.meow128_fixed_host(hk, L, STATIC, out=ho, fixup=(mib == 4))
            np.testing.assert_array_equal(ho, want if mib != 4 else u64(kvh.meow128_fixed(dev(kb), L, STATIC,
                                                                                           fixup=True)))
        finally:
            kvh.lib.kvh_set_tuning(15, pm)
            kvh.lib.kvh_set_tuning(16, ps)
    # mixed: pinned keys, pageable output
    got3 = kvh.meow128_fixed_host(hk, L, STATIC)
    np.testing.assert_array_equal(got3, want)


def test_full_size_c1_properties(kvh):
    """BASELINE config C1 at full size (100M x 16 B): sampled oracle parity,
    agreement of three independent kernels, determinism."""
    n, L = 100_000_000, 16
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    out = kvh.meow128_fixed(keys, L, STATIC)
    out2 = kvh.meow128_fixed(keys, L, STATIC)
    assert torch.equal(out, out2)
    h = u64(out)
    idx = np.random.default_rng(7).choice(n, 20000, replace=False)
    idx.sort()
    kb = keys.view(n, L)[torch.from_numpy(idx).cuda()].cpu().numpy().reshape(-1)
    np.testing.assert_array_equal(h[idx], orc_fixed(ORC, kb, L, STATIC))
    # generic (runtime-length) kernel and variable-length kernel on a 10M prefix
    m = 10_000_000
    prev = kvh.lib.kvh_set_tuning(2, 1)
    try:
        gen = u64(kvh.meow128_fixed(keys[: m * L], L, STATIC))
    finally:
        kvh.lib.kvh_set_tuning(2, prev)
    np.testing.assert_array_equal(gen, h[:m])
    offs = torch.arange(0, (m + 1) * L, L, dtype=torch.int64, device="cuda")
    np.testing.assert_array_equal(u64(kvh.meow128_var(keys, offs, STATIC)), h[:m])
    assert len(np.unique(h[:1_000_000, 0])) > 999_000  # no degenerate collisions


def test_var_10m_zipf_vs_literal_kernel(kvh):
    from raikv_amd.workload import zipf_lengths, offsets_from_lengths
    m = 10_000_000
    lens = zipf_lengths(m, 8, 256, seed=11)
    offs = offsets_from_lengths(lens)
    g = torch.Generator(device="cuda")
    g.manual_seed(99)
    keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda", generator=g)
    doff = dev_u64(offs)
    a = kvh.meow128_var(keys, doff, STATIC)
    sd = dev_u64(np.tile(np.array(STATIC, dtype=np.uint64), (m, 1)))
    b = kvh.meow128_var_seeded(keys, doff, sd)
    assert torch.equal(a, b)
    idx = np.random.default_rng(8).choice(m, 3000, replace=False)
    kh = keys.cpu().numpy()
    ha = u64(a)
    for i in idx:
        o0, o1 = int(offs[i]), int(offs[i + 1])
        assert orc_meow(ORC, kh[o0:o1].tobytes(), *STATIC) == (int(ha[i, 0]), int(ha[i, 1]))


def test_cpp_hash_test_program(kvh):
    exe = os.path.join(ROOT, "tests", "cpp", "hash_test_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "cpptests"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("variant", [0, 23, 46])
def test_var_kernel_variants_vs_oracle(kvh, variant):
    """The variable-length kernels of the product (kvh_set_tuning(7, v): 0
    unsorted, 23 windows sorted by 16-byte length class in the static order,
    46 the same taken in address order through wave tickets) against
    the oracle: zipf 8-256 B plus 0..300-byte and 70 000-byte keys, odd counts
    for ragged last windows, at an unaligned base."""
    from raikv_amd.workload import zipf_lengths
    rng = np.random.default_rng(variant)
    for n in (1, 255, 257, 4099, 100003):
        lens = zipf_lengths(n, 8, 256, seed=n).astype(np.int64)
        if n > 300:
            lens[rng.integers(0, n, 300)] = rng.integers(0, 301, 300)
            lens[rng.integers(0, n)] = 70000
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + 3
        keys = rng.integers(0, 256, int(offs[-1]) + 5, dtype=np.uint8)
        want = orc_var(ORC, keys, offs, STATIC)
        prev = kvh.lib.kvh_set_tuning(7, variant)
        try:
            got = u64(kvh.meow128_var(dev(keys), dev_u64(offs), STATIC))
        finally:
            kvh.lib.kvh_set_tuning(7, prev)
        np.testing.assert_array_equal(got, want, err_msg=f"n={n}")


def test_streams_program(kvh):
    """tests/cpp/streams_gpu -- four host threads on
    hipStreamPerThread at once (with and without the knob-26 fetch delay),
    graphs captured on one stream and replayed on two others while direct
    launches run on the capture stream, kvh_stream_release before a stream is
    destroyed; every output poisoned first and checked word for word against
    the oracle."""
    exe = os.path.join(ROOT, "tests", "cpp", "streams_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "tests/cpp/streams_gpu"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_cpp_paths_program(kvh):
    """The C++ API of the f1-f4 paths (include/raikv_amd/key_hash.hpp) on the GPU."""
    exe = os.path.join(ROOT, "tests", "cpp", "paths_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "cpptests"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def _digest(d: np.ndarray) -> int:
    """tests/golden/make_golden.py partition_digest: sum w_i * (2i + 1) mod 2^64."""
    w = d.reshape(-1).astype(np.uint64)
    with np.errstate(over="ignore"):
        return int(np.sum(w * (2 * np.arange(w.size, dtype=np.uint64) + np.uint64(1)), dtype=np.uint64))


@pytest.mark.parametrize("variant", [46, 0, 23])
def test_partition_vectors_against_reference(kvh, variant):
    """hash_test.cpp:404-442 on the device, pinned to the REFERENCE's outputs
    (tests/golden/partition2.npz, partition4.npz; make_golden.py): bytes
    0..127 cut at every n (part2) and at every n <= m <= o < 128 (part4,
    357,760 cuts).  Every piece is a substring buf[a:b]; all 8385 substrings
    are hashed by the device kernels and must equal the reference's
    kv_hash_meow128; the part4 cuts composed from them must reproduce the
    digest of the reference's own kv_hash_meow128_4_diff_length outputs."""
    seed = (10101, 20202)
    buf = np.arange(128, dtype=np.uint8)
    p2 = golden("partition2.npz")["out"]
    g4 = golden("partition4.npz")
    sub, want = g4["sub"].astype(np.int64), g4["out"]
    lens = sub[:, 1] - sub[:, 0]
    offs = np.zeros(len(sub) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    flat = np.concatenate([buf[a:b] for a, b in sub])
    prev = kvh.lib.kvh_set_tuning(7, variant)
    try:
        h = u64(kvh.meow128_var(dev(flat), dev_u64(offs), seed))
        # part2 as 258 keys in cut order
        k2 = [buf[:n] if j == 0 else buf[n:] for n in range(129) for j in (0, 1)]
        o2 = np.zeros(259, dtype=np.uint64)
        o2[1:] = np.cumsum([len(k) for k in k2])
        h2 = u64(kvh.meow128_var(dev(np.concatenate(k2)), dev_u64(o2), seed))
    finally:
        kvh.lib.kvh_set_tuning(7, prev)
    np.testing.assert_array_equal(h, want)
    np.testing.assert_array_equal(h2.reshape(129, 4), p2)
    if variant != 46:
        return
    # the other device paths over the same substrings: straight-line kernel,
    # (offset, length) spans, and the synchronous drop-ins
    sd = dev_u64(np.tile(np.array(seed, dtype=np.uint64), (len(sub), 1)))
    np.testing.assert_array_equal(u64(kvh.meow128_var_seeded(dev(flat), dev_u64(offs), sd)), want)
    sp = kvh.meow128_spans(dev(buf), dev_u64(sub[:, 0].astype(np.uint64)),
                           torch.from_numpy(lens.astype(np.int32)).cuda(), seed, fixup=False, nulterm=False)
    np.testing.assert_array_equal(u64(sp), want)
    idx = np.full((129, 129), -1, dtype=np.int64)
    idx[sub[:, 0], sub[:, 1]] = np.arange(len(sub))
    tr = np.array([(n, m, o) for n in range(128) for m in range(n, 128) for o in range(m, 128)], dtype=np.int64)
    assert len(tr) == int(g4["ntrip"][0])
    d = np.concatenate([h[idx[0, tr[:, 0]]], h[idx[tr[:, 0], tr[:, 1]]], h[idx[tr[:, 1], tr[:, 2]]],
                        h[idx[tr[:, 2], 128]]], axis=1)
    assert _digest(d) == int(g4["digest4"][0])
    cb = C.create_string_buffer(buf.tobytes(), 128)
    base = C.addressof(cb)
    lib = kvh.lib
    for n in range(129):
        x = (C.c_uint64 * 4)(*seed, *seed)
        assert lib.kvh_hash_meow128_2_diff_length(cb, n, C.c_void_p(base + n), 128 - n, x) == 0
        assert list(x) == [int(v) for v in p2[n]], n
    for t in np.random.default_rng(9).choice(len(tr), 200, replace=False):
        n, m, o = (int(v) for v in tr[t])
        x = (C.c_uint64 * 8)(*(seed * 4))
        assert lib.kvh_hash_meow128_4_diff_length(cb, n, C.c_void_p(base + n), m - n, C.c_void_p(base + m), o - m,
                                                  C.c_void_p(base + o), 128 - o, x) == 0
        assert list(x) == [int(v) for v in d[t]], (n, m, o)


def test_kv_compat_symbols_against_reference_vectors(kvh):
    """libkvh_kv.so's kv_* symbols (same names and signatures as
    include/raikv/key_hash.h) reproduce the reference's vectors on the GPU."""
    lib = C.CDLL(os.path.join(ROOT, "raikv_amd", "libkvh_kv.so"))
    U = C.c_uint64
    lib.kv_hash_meow128.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(U), C.POINTER(U)]
    lib.kv_hash_meow128.restype = None
    lib.kv_hash_meow64.argtypes = [C.c_void_p, C.c_size_t, U]
    lib.kv_hash_meow64.restype = U
    for k in VEC["kat"]:
        key = bytes.fromhex(k["key_hex"])
        a, b = U(k["seed"][0]), U(k["seed"][1])
        lib.kv_hash_meow128(C.create_string_buffer(key, max(1, len(key))), len(key), C.byref(a), C.byref(b))
        assert "%016x:%016x" % (a.value, b.value) == k["h"]
    for m in VEC["meow64"]:
        key = bytes.fromhex(m["key_hex"])
        assert lib.kv_hash_meow64(C.create_string_buffer(key, max(1, len(key))), len(key), U(m["seed"])) == m["h"]
    r = VEC["variants"]["results"]
    keys = [k.encode() for k in VEC["variants"]["keys"]]
    s1, s2 = VEC["variants"]["seed"]
    L = len(keys[0])
    bufs = [C.create_string_buffer(k, L) for k in keys]
    x = (U * 8)(*([s1, s2] * 4))
    lib.kv_hash_meow128_4_diff_length(bufs[0], C.c_size_t(L), bufs[1], C.c_size_t(L), bufs[2], C.c_size_t(L),
                                      bufs[3], C.c_size_t(L), x)
    assert list(x) == r["4_diff"]
    x = (U * 8)(*r["4_same_4_seed"]["seeds"])
    lib.kv_hash_meow128_4_same_length_4_seed(bufs[0], bufs[1], bufs[2], bufs[3], C.c_size_t(L), x)
    assert list(x) == r["4_same_4_seed"]["x"]
    for i in range(4):
        a, b = U(s1), U(s2)
        lib.kv_meow_test(bufs[i], C.c_size_t(L), C.byref(a), C.byref(b))
        assert [a.value, b.value] == r["stream"][i]
