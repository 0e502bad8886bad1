"""GPU parity for SURVEY.md §8 row f4 (batched CRC32C): kvh_crc_c_fixed /
kvh_crc_c_var and the host drop-ins vs the reference's own outputs
(tests/golden/crc32c.npz) and the oracle (oracle/crc_oracle.c).  Bit-exact.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle_lib import GOLDEN, ROOT, load_oracle, orc_crc_fixed, orc_crc_var  # noqa: E402

G = np.load(os.path.join(GOLDEN, "crc32c.npz"))
ORC = load_oracle()


@pytest.fixture(scope="module")
def kvh():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    import raikv_amd
    return raikv_amd


def u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_every_length_fixed_and_var(kvh):
    keys, seeds, want = G["len_keys"], G["len_seeds"], G["len_out"]
    for si, s in enumerate(seeds):
        # var: every length 0..300 in one batch
        lens = np.arange(keys.shape[0], dtype=np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        flat = np.concatenate([keys[L, :L] for L in range(keys.shape[0])])
        got = u32(kvh.crc_c_var(dev(flat), dev(offs.view(np.int64)), seed=int(s)))
        np.testing.assert_array_equal(got, want[:, si])
    # fixed: each length as a batch of one key (and 7 copies)
    for L in range(1, keys.shape[0], 7):
        k = np.tile(keys[L, :L], 7)
        got = u32(kvh.crc_c_fixed(dev(k), L, seed=int(seeds[1])))
        assert np.all(got == want[L, 1]), L


def test_array_per_key_seeds(kvh):
    seeds = dev(G["var_seeds"].view(np.int32))
    got = u32(kvh.crc_c_var(dev(G["var_keys"]), dev(G["var_offsets"].view(np.int64)), seeds=seeds))
    np.testing.assert_array_equal(got, G["var_out"])
    # in/out seeds in one buffer, like kv_crc_c_array
    io = seeds.clone()
    kvh.crc_c_var(dev(G["var_keys"]), dev(G["var_offsets"].view(np.int64)), seeds=io, out=io)
    np.testing.assert_array_equal(u32(io), G["var_out"])


@pytest.mark.parametrize("L", [1, 3, 4, 7, 8, 16, 24, 32, 33, 64, 100])
def test_fixed_batches_vs_oracle(kvh, L):
    rng = np.random.default_rng(L)
    n = 4099
    kb = rng.integers(0, 256, n * L, dtype=np.uint8)
    sd = rng.integers(0, 2 ** 32, n, dtype=np.uint32)
    np.testing.assert_array_equal(u32(kvh.crc_c_fixed(dev(kb), L, seed=0x12345678)),
                                  orc_crc_fixed(ORC, kb, L, seed=0x12345678))
    np.testing.assert_array_equal(u32(kvh.crc_c_fixed(dev(kb), L, seeds=dev(sd.view(np.int32)))),
                                  orc_crc_fixed(ORC, kb, L, seeds=sd))
    # unaligned base
    buf = dev(np.concatenate([np.zeros(3, np.uint8), kb]))
    np.testing.assert_array_equal(u32(kvh.crc_c_fixed(buf[3:], L, seed=7)), orc_crc_fixed(ORC, kb, L, seed=7))


def test_drop_ins(kvh):
    lib = kvh.lib
    buf = G["prefix_buf"]
    for L, s, w in zip(G["prefix_lens"], G["prefix_seeds"], G["prefix_out"]):
        assert kvh.kv_crc_c(buf[:int(L)].tobytes(), int(s)) == int(w)
    n = len(G["prefix_lens"])
    sz = (C.c_size_t * n)(*[int(x) for x in G["prefix_lens"]])
    io = G["prefix_seeds"].copy()
    assert lib.kvh_crc_c_key_array(buf.ctypes.data, sz, io.ctypes.data, n) == 0
    np.testing.assert_array_equal(io, G["prefix_out"])
    for i, w, w2, r in zip(G["uint_in"][:8], G["uint_out"], G["uint2_out"], G["uint_in"][::-1]):
        assert lib.kvh_hash_uint(int(i)) == int(w)
        assert lib.kvh_hash_uint2(int(i), int(r)) == int(w2)
    keys, offs, sd, want = G["var_keys"], G["var_offsets"], G["var_seeds"], G["var_out"]
    m = 37
    ps = (C.c_void_p * m)(*[keys.ctypes.data + int(offs[i]) for i in range(m)])
    psz = (C.c_size_t * m)(*[int(offs[i + 1] - offs[i]) for i in range(m)])
    io = sd[:m].copy()
    assert lib.kvh_crc_c_array(ps, psz, io.ctypes.data, m) == 0
    np.testing.assert_array_equal(io, want[:m])
    a, b = C.c_uint32(int(sd[0])), C.c_uint32(int(sd[1]))
    assert lib.kvh_crc_c_2_diff(ps[0], psz[0], C.byref(a), ps[1], psz[1], C.byref(b)) == 0
    assert (a.value, b.value) == (int(want[0]), int(want[1]))


def test_full_size_var_property(kvh):
    """100M zipf 8-256 B keys (the C2 shape): CRC of each key equals the
    fixed-length kernel on the same bytes where lengths agree, and a sample
    matches the oracle; crc(A||B) composes (linearity of CRC)."""
    from raikv_amd.workload import zipf_lengths, offsets_from_lengths
    n = 100_000_000
    lens = zipf_lengths(n, 8, 256, seed=3)
    offs = offsets_from_lengths(lens)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda", generator=gen)
    doff = torch.from_numpy(offs.view(np.int64)).cuda()
    out = kvh.crc_c_var(keys, doff, seed=0xFFFFFFFF)
    idx = np.random.default_rng(1).integers(0, n, 20000)
    kh = keys.cpu().numpy()
    sub_offs = np.zeros(len(idx) + 1, np.uint64)
    parts = []
    for k, i in enumerate(idx):
        a, e = int(offs[i]), int(offs[i + 1])
        parts.append(kh[a:e])
        sub_offs[k + 1] = sub_offs[k] + (e - a)
    want = orc_crc_var(ORC, np.concatenate(parts), sub_offs, seed=0xFFFFFFFF)
    np.testing.assert_array_equal(u32(out)[idx], want)
    # chaining: crc(key_i from seed) used as seed of key_{i+1} == crc of the concatenation
    c = kvh.kv_crc_c(kh[int(offs[0]):int(offs[3])].tobytes(), 99)
    s = 99
    for i in range(3):
        s = kvh.kv_crc_c(kh[int(offs[i]):int(offs[i + 1])].tobytes(), s)
    assert c == s


@pytest.mark.parametrize("kernel", [0, 6])
@pytest.mark.parametrize("n", [1, 255, 257, 2561])
def test_var_kernels_vs_oracle(kvh, kernel, n):
    """Both variable-length kernels (input order; length-sorted windows, knob
    14), window tails, keys of 0 bytes and of >= 65535 bytes (the sorted
    kernel's record saturates and re-reads the offsets), per-key seeds."""
    rng = np.random.default_rng(n * 3 + kernel)
    lens = rng.integers(0, 300, n).astype(np.uint64)
    if n > 2:
        lens[1] = 0
        lens[n // 2] = 70001
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    flat = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    prev = kvh.lib.kvh_set_tuning(14, kernel)
    try:
        got = u32(kvh.crc_c_var(dev(flat), dev(offs.view(np.int64)), seed=0x1234567))
        np.testing.assert_array_equal(got, orc_crc_var(ORC, flat, offs, seed=0x1234567))
        got = u32(kvh.crc_c_var(dev(flat), dev(offs.view(np.int64)), seeds=dev(seeds.view(np.int32))))
        np.testing.assert_array_equal(got, orc_crc_var(ORC, flat, offs, seeds))
    finally:
        kvh.lib.kvh_set_tuning(14, prev)


def test_kv_compat_c_program_links_only_libkvh_kv(kvh, tmp_path):
    """a C program that includes only include/kvh_kv.h and
    links only libkvh_kv.so calls every CRC32C symbol of
    include/raikv/key_hash.h:8-20 (kv_crc_c over every length 0..300 under
    three seeds, kv_crc_c_array / _2_diff / _4_diff over 3000 variable-length
    keys with per-key seeds, kv_crc_c_key_array over prefixes, kv_hash_uint /
    kv_hash_uint2) against the reference's own outputs (crc32c.npz)."""
    import struct
    exe = os.path.join(ROOT, "tests", "cpp", "kv_compat_crc")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "tests/cpp/kv_compat_crc"], check=True)
    lk, ls, lo = G["len_keys"], G["len_seeds"], G["len_out"]
    parts = [struct.pack("<III", lk.shape[0], lk.shape[1], ls.shape[0]), lk.astype(np.uint8).tobytes(),
             ls.astype("<u4").tobytes(), lo.astype("<u4").tobytes()]
    vo, vk = G["var_offsets"].astype("<u8"), G["var_keys"].astype(np.uint8)
    parts += [struct.pack("<I", len(vo) - 1), vo.tobytes(), G["var_seeds"].astype("<u4").tobytes(),
              G["var_out"].astype("<u4").tobytes(), struct.pack("<Q", vk.size), vk.tobytes()]
    pb = G["prefix_buf"].astype(np.uint8)
    parts += [struct.pack("<II", len(G["prefix_lens"]), pb.size), pb.tobytes(),
              G["prefix_lens"].astype("<u4").tobytes(), G["prefix_seeds"].astype("<u4").tobytes(),
              G["prefix_out"].astype("<u4").tobytes()]
    parts += [struct.pack("<I", len(G["uint_in"])), G["uint_in"].astype("<u4").tobytes(),
              G["uint_out"].astype("<u4").tobytes(), G["uint2_out"].astype("<u4").tobytes()]
    f = tmp_path / "crc_cases.bin"
    f.write_bytes(b"".join(parts))
    r = subprocess.run([exe, str(f)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0" in r.stdout

