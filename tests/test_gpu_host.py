"""GPU: the PCIe-inclusive host pipelines (keys and hashes in host memory)
and their one-process multi-device sharding, through the C-ABI.

kvh_meow128_var_host is the path socket / shm-segment keys take
(include/raikv/ev_key.h:83-114, test/ctest.c:202-233): variable-length keys
in host memory.  Each result must equal the device-resident kernel on
device copies of the same buffers (which test_gpu_parity.py and
test_gpu_fullsize.py pin to the oracle), plus an oracle sample here.
kvh_meow128_{fixed,var}_host_multi shard one host batch over a device list
(one host thread per entry); on the one-GPU box the list repeats device 0,
which runs the shards concurrently on separate pipelines of that device.
"""
import ctypes as C
import mmap

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle_lib import load_oracle, orc_var  # noqa: E402

ORC = load_oracle()
STATIC = (0xA8E0BCC94D1855F5, 0xAD3BEC1E8DE4A1A3)


@pytest.fixture(scope="module")
def kvh():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    import raikv_amd
    return raikv_amd


def dev_hash_var(kvh, keys: np.ndarray, offs: np.ndarray, seed, fixup=False):
    base = int(offs[0])
    k = torch.from_numpy(keys[base:int(offs[-1])].copy() if offs[-1] > base else np.zeros(1, np.uint8)).cuda()
    o = torch.from_numpy((offs - np.uint64(base)).view(np.int64)).cuda()
    out = kvh.meow128_var(k, o, seed, fixup=fixup)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint64)


# Host memory these tests page-lock with kvh_host_register: fresh anonymous
# mappings, kept mapped to the end of the process.  On this ROCm stack pages
# that were registered and unregistered and then come back from the heap as
# the buffer of a later pageable copy of more than ~1 MiB can make that copy
# raise hipErrorIllegalAddress (reproduced with torch and hipHostRegister
# alone, no code of this repository: tools/copy_fault_stress.py, DESIGN.md
# §4.4, include/kvh.h above kvh_host_register).  Registered pages that are
# never handed back to the allocator cannot become such a buffer; the suite's
# own pageable copies then run on the runtime's default path.
_LOCKED = []


def locked_pages(nbytes: int) -> np.ndarray:
    """A page-aligned uint8 array of nbytes on its own anonymous mapping,
    never unmapped (the memory a caller registers: raikv's shm segment)."""
    m = mmap.mmap(-1, max(nbytes, 1))
    _LOCKED.append(m)
    return np.frombuffer(m, dtype=np.uint8)[:nbytes]


def zipf_batch(n, seed, lead=0, long_keys=()):
    from raikv_amd.workload import zipf_lengths
    lens = zipf_lengths(n, 8, 256, seed=seed).astype(np.uint64)
    for i, L in long_keys:
        lens[i] = L
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += np.uint64(lead)
    keys = np.random.default_rng(seed).integers(0, 256, int(offs[-1]) + 7, dtype=np.uint8)
    return keys, offs


@pytest.mark.parametrize("mib,slots", [(16, 4), (1, 2), (1, 16)])
def test_var_host_pipeline(kvh, mib, slots):
    """Zipf keys with a nonzero first offset, keys longer than the chunk
    budget (3 MiB with 1 MiB chunks: a chunk of their own) and runs of empty
    keys; pageable, kvh_host_alloc-pinned and kvh_host_register'ed buffers;
    ragged last chunk and slot reuse."""
    n = 400_003
    keys, offs = zipf_batch(n, 7, lead=5, long_keys=[(10, 3 << 20), (200_000, 3 << 20), (200_001, 1 << 20),
                                                       (n - 1, 2 << 20)])
    lens = np.diff(offs)
    lens[5000:5100] = 0
    offs[1:] = offs[0] + np.cumsum(lens)
    want = dev_hash_var(kvh, keys, offs, STATIC)
    pm, ps = kvh.lib.kvh_set_tuning(15, mib), kvh.lib.kvh_set_tuning(16, slots)
    try:
        got = kvh.meow128_var_host(keys, offs, STATIC)
        np.testing.assert_array_equal(got, want)
        # pinned (kvh_host_alloc) keys, offsets and output
        hk = kvh.host_empty(keys.shape, np.uint8)
        hk[:] = keys
        hf = kvh.host_empty(offs.shape, np.uint64)
        hf[:] = offs
        ho = kvh.host_empty((n, 2), np.uint64)
        _LOCKED.extend((hk, hf, ho))  # pinned pages are never handed back during the session either
        kvh.meow128_var_host(hk, hf, STATIC, out=ho, fixup=True)
        np.testing.assert_array_equal(ho, dev_hash_var(kvh, keys, offs, STATIC, fixup=True))
        # a caller's own buffer page-locked in place (raikv's shm segment)
        reg = locked_pages(keys.size + 4096)
        view = reg[:keys.size]
        view[:] = keys
        assert kvh.lib.kvh_host_register(view.ctypes.data, view.nbytes) == 0
        try:
            np.testing.assert_array_equal(kvh.meow128_var_host(view, offs, STATIC), want)
        finally:
            assert kvh.lib.kvh_host_unregister(view.ctypes.data) == 0
    finally:
        kvh.lib.kvh_set_tuning(15, pm)
        kvh.lib.kvh_set_tuning(16, ps)
    # oracle sample (short keys and a 3 MiB one)
    idx = np.sort(np.concatenate([np.random.default_rng(1).choice(n, 3000, replace=False), [10]]))
    sub = np.concatenate([keys[int(offs[i]):int(offs[i + 1])] for i in idx])
    so = np.zeros(len(idx) + 1, dtype=np.uint64)
    so[1:] = np.cumsum(lens[idx])
    np.testing.assert_array_equal(want[idx], orc_var(ORC, sub, so, STATIC))


def test_var_host_edges(kvh):
    keys = np.frombuffer(b"hello\0", dtype=np.uint8).copy()
    got = kvh.meow128_var_host(keys, np.array([0, 6], dtype=np.uint64), STATIC)
    assert "%016x:%016x" % (int(got[0, 0]), int(got[0, 1])) == "2aa73a1eeb0b2d45:fd102121185ce157"
    empty = kvh.meow128_var_host(keys, np.zeros(1001, dtype=np.uint64), (7, 9))
    np.testing.assert_array_equal(empty, dev_hash_var(kvh, keys, np.zeros(1001, dtype=np.uint64), (7, 9)))
    assert kvh.meow128_var_host(keys, np.zeros(1, dtype=np.uint64), STATIC).shape == (0, 2)
    assert kvh.lib.kvh_meow128_var_host(None, None, 5, 0, 0, None, 0) == -22


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_fixed_and_var(kvh, devices):
    """One host batch over a device list: the output equals the one-device
    call (the same global layout); ragged shard sizes; more shards than keys."""
    rng = np.random.default_rng(len(devices))
    for n, L in ((1_000_003, 16), (777, 32), (2, 16)):
        kb = rng.integers(0, 256, n * L, dtype=np.uint8)
        want = kvh.meow128_fixed_host(kb, L, STATIC)
        np.testing.assert_array_equal(kvh.meow128_host_multi(kb, STATIC, devices, key_len=L), want)
        np.testing.assert_array_equal(kvh.meow128_host_multi(kb, STATIC, devices, key_len=L, fixup=True),
                                      kvh.meow128_fixed_host(kb, L, STATIC, fixup=True))
    for n in (300_001, 3, 1):
        keys, offs = zipf_batch(n, 11 + n, lead=3)
        want = dev_hash_var(kvh, keys, offs, STATIC)
        np.testing.assert_array_equal(kvh.meow128_host_multi(keys, STATIC, devices, offsets=offs), want)


def test_multi_device_rejects_bad_device_lists(kvh):
    kb = np.zeros(1600, np.uint8)
    out = np.zeros((100, 2), np.uint64)
    bad = (C.c_int * 2)(0, 9999)
    assert kvh.lib.kvh_meow128_fixed_host_multi(kb.ctypes.data, 16, 100, 0, 0, out.ctypes.data, 0, bad, 2) == -22
    assert kvh.lib.kvh_meow128_fixed_host_multi(kb.ctypes.data, 16, 100, 0, 0, out.ctypes.data, 0, bad, 0) == -22
    neg = (C.c_int * 1)(-1)
    assert kvh.lib.kvh_meow128_fixed_host_multi(kb.ctypes.data, 16, 100, 0, 0, out.ctypes.data, 0, neg, 1) == -22


def test_partially_registered_buffers_take_the_bounce_path(kvh):
    """a buffer page-locked only in part (its first pages
    registered, the rest pageable) must not be DMA'd past the registered
    extent; the pipeline checks the range's first and last byte and bounces
    it otherwise.  Keys, offsets and output each registered at the front only,
    one chunk and several chunks."""
    n = 300_001
    keys, offs = zipf_batch(n, 21, lead=1)
    want = dev_hash_var(kvh, keys, offs, STATIC)
    page = 4096
    bufs = {}
    for name, arr in (("keys", keys), ("offs", offs)):
        raw = locked_pages(arr.nbytes + 2 * page)
        start = (-raw.ctypes.data) % page
        view = raw[start:start + arr.nbytes].view(arr.dtype)
        view[:] = arr
        bufs[name] = (raw, view)
    out_raw = locked_pages(n * 16 + 2 * page)
    ostart = (-out_raw.ctypes.data) % page
    out = out_raw[ostart:ostart + n * 16].view(np.uint64).reshape(n, 2)
    regs = [bufs["keys"][1], bufs["offs"][1], out]
    for r in regs:  # the first 2 pages only
        assert kvh.lib.kvh_host_register(r.ctypes.data, 2 * page) == 0
    pm = kvh.lib.kvh_set_tuning(15, 1)
    try:
        for mib in (1, 64):  # several chunks, then one chunk
            kvh.lib.kvh_set_tuning(15, mib)
            out[:] = 0
            rc = kvh.lib.kvh_meow128_var_host(bufs["keys"][1].ctypes.data, bufs["offs"][1].ctypes.data, n,
                                              C.c_uint64(STATIC[0]), C.c_uint64(STATIC[1]), out.ctypes.data, 0)
            assert rc == 0
            np.testing.assert_array_equal(out, want)
    finally:
        kvh.lib.kvh_set_tuning(15, pm)
        for r in regs:
            assert kvh.lib.kvh_host_unregister(r.ctypes.data) == 0


def test_two_registrations_with_a_pageable_gap_bounce(kvh):
    """a buffer made of two separate kvh_host_register ranges with
    a pageable page between them has both ends page-locked, but must not be
    DMA'd as one range (the DMA would run through the gap's missing mapping):
    the pipeline's own registry sees two registrations and bounces it.  One
    chunk and several chunks, keys and output split the same way."""
    n = 200_003
    keys, offs = zipf_batch(n, 23, lead=1)
    want = dev_hash_var(kvh, keys, offs, STATIC)
    page = 4096
    raw = locked_pages(keys.nbytes + 4 * page)
    start = (-raw.ctypes.data) % page
    kv = raw[start:start + keys.nbytes]
    kv[:] = keys
    out_raw = locked_pages(n * 16 + 4 * page)
    ostart = (-out_raw.ctypes.data) % page
    out = out_raw[ostart:ostart + n * 16].view(np.uint64).reshape(n, 2)
    regs = []
    for a in (kv, out.reshape(-1).view(np.uint8)):
        base = a.ctypes.data
        tail = (a.nbytes // page - 2) * page  # pages [3, end) registered, page 2 left pageable
        assert tail > page
        assert kvh.lib.kvh_host_register(base, 2 * page) == 0
        assert kvh.lib.kvh_host_register(base + 3 * page, a.nbytes - 3 * page) == 0
        regs += [base, base + 3 * page]
    pm = kvh.lib.kvh_set_tuning(15, 1)
    try:
        for mib in (1, 64):
            kvh.lib.kvh_set_tuning(15, mib)
            out[:] = 0
            rc = kvh.lib.kvh_meow128_var_host(kv.ctypes.data, offs.ctypes.data, n, C.c_uint64(STATIC[0]),
                                              C.c_uint64(STATIC[1]), out.ctypes.data, 0)
            assert rc == 0
            np.testing.assert_array_equal(out, want)
    finally:
        kvh.lib.kvh_set_tuning(15, pm)
        for r in regs:
            assert kvh.lib.kvh_host_unregister(r) == 0


@pytest.mark.parametrize("tiny", ["default", 0], ids=["tiny_path", "one_chunk_dma"])
@pytest.mark.parametrize("n", [1, 8, 64, 1024, 16384])
def test_one_chunk_batches_at_raikv_sizes(kvh, n, tiny):
    """raikv's own batch sizes (8 keys per prefetch pipe, ev_net.h:442; 16K
    frags per ctest batch, ctest.c:34): with knob 21 at its default these
    take the zero-copy k_tiny path, with knob 21 = 0 the one-chunk DMA path
    (same-stream H2D, kernel, D2H).  Pinned and pageable, fixed
    and variable length, against the device-resident kernel and the oracle."""
    prev = kvh.lib.kvh_set_tuning(21, 16384 if tiny == "default" else 0)
    try:
        rng = np.random.default_rng(n)
        kb = rng.integers(0, 256, n * 16, dtype=np.uint8)
        want = kvh.meow128_fixed(torch.from_numpy(kb).cuda(), 16, STATIC).cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(kvh.meow128_fixed_host(kb, 16, STATIC), want)
        hk = kvh.host_empty(kb.shape, np.uint8)
        hk[:] = kb
        ho = kvh.host_empty((n, 2), np.uint64)
        _LOCKED.extend((hk, ho))
        kvh.meow128_fixed_host(hk, 16, STATIC, out=ho)
        np.testing.assert_array_equal(ho, want)
        keys, offs = zipf_batch(n, 100 + n, lead=2)
        got = kvh.meow128_var_host(keys, offs, STATIC)
        np.testing.assert_array_equal(got, dev_hash_var(kvh, keys, offs, STATIC))
        m = min(n, 500)
        sub = keys[int(offs[0]):int(offs[m])]
        np.testing.assert_array_equal(got[:m], orc_var(ORC, sub, offs[:m + 1] - offs[0], STATIC))
    finally:
        kvh.lib.kvh_set_tuning(21, prev)


def test_multi_device_pool_reused(kvh):
    """The _multi entries run on persistent workers: many calls in a row
    (and device lists of growing length) all equal the one-device call."""
    rng = np.random.default_rng(5)
    kb = rng.integers(0, 256, 4096 * 16, dtype=np.uint8)
    want = kvh.meow128_fixed_host(kb, 16, STATIC)
    for it in range(40):
        devs = [0] * (1 + it % 4)
        np.testing.assert_array_equal(kvh.meow128_host_multi(kb, STATIC, devs, key_len=16), want)
