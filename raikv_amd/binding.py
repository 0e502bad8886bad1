"""ctypes binding of libkvh.so (include/kvh.h) + small Python mirrors of
raikv's key-fragment API (hash_entry.h:56-112, shm_ht.h:333-351).

Device buffers are torch tensors on a ROCm device; the kernels run on the
caller's current torch stream (or an explicit `stream`).  torch is imported
before libkvh.so is loaded so that one HIP runtime serves both.
"""
from __future__ import annotations

import ctypes as C
import weakref
import os
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

try:  # torch first: one HIP runtime per process
    import torch
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

KVH_FIXUP = 0x1
KVH_POS32 = 0x2
KVH_NULTERM = 0x4
KVH_DEDUP = 0x8
KVH_REF_ORDER = 0x10
KVH_MAX_ARITY = 8

_HERE = os.path.dirname(os.path.abspath(__file__))
# KVH_LIB: research tools (tools/*.py) point this at the experiments build
# tools/libkvh_exp.so; the product path and its tests load libkvh.so.
lib_path = os.environ.get("KVH_LIB") or os.path.join(_HERE, "libkvh.so")

U64 = C.c_uint64
U32 = C.c_uint32
SZ = C.c_size_t
P = C.c_void_p
I = C.c_int


class KvhError(RuntimeError):
    pass


class HtGeom(C.Structure):
    """kvh_ht_geom_t: the FileHdr fields ht_mod / calc_hash read
    (include/raikv/shm_ht.h:143-157)."""
    _fields_ = [("ht_size", C.c_uint64), ("ht_mod_mask", C.c_uint64), ("ht_mod_fraction", C.c_uint64),
                ("ht_mod_shift", C.c_uint32), ("cuckoo_buckets", C.c_uint16), ("cuckoo_arity", C.c_uint8),
                ("pad", C.c_uint8)]

    @classmethod
    def from_map(cls, map_size: int, hash_entry_size: int = 64, hash_value_ratio: float = 1.0,
                 cuckoo_buckets: int = 4, cuckoo_arity: int = 2) -> "HtGeom":
        """HashTab::initialize's geometry (ht_init.cpp:117-156); default
        cuckoo shape "2+4" as the reference server (arity 2, 4 buckets)."""
        g = cls()
        check(lib.kvh_ht_geom_init(map_size, hash_entry_size, hash_value_ratio, cuckoo_buckets, cuckoo_arity,
                                   C.byref(g)), "kvh_ht_geom_init")
        return g

    @property
    def per_key(self) -> int:
        return int(lib.kvh_positions_per_key(C.byref(self)))

    def ht_mod(self, k: int) -> int:
        """FileHdr::ht_mod (shm_ht.h:181-184), host side."""
        return (((k & self.ht_mod_mask) * self.ht_mod_fraction) & (2**64 - 1)) >> self.ht_mod_shift


def _load():
    if not os.path.exists(lib_path):
        raise ImportError(
            f"raikv_amd: HIP library {lib_path} is missing; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` or `make`")
    lib = C.CDLL(lib_path)
    sig = {
        "kvh_meow128_fixed": (I, [P, U32, SZ, U64, U64, P, U32, P]),
        "kvh_meow128_var": (I, [P, P, SZ, U64, U64, P, U32, P]),
        "kvh_meow128_multiseed": (I, [P, U32, SZ, P, U32, P, U32, P]),
        "kvh_meow128_batch": (I, [P, P, U32, SZ, P, U32, P, U32, P]),
        "kvh_meow128_var_seeded": (I, [P, P, SZ, P, P, U32, P]),
        "kvh_meow128_fixed_host": (I, [P, U32, SZ, U64, U64, P, U32]),
        "kvh_meow128_var_host": (I, [P, P, SZ, U64, U64, P, U32]),
        "kvh_meow128_fixed_host_multi": (I, [P, U32, SZ, U64, U64, P, U32, P, I]),
        "kvh_meow128_var_host_multi": (I, [P, P, SZ, U64, U64, P, U32, P, I]),
        "kvh_host_register": (I, [P, SZ]),
        "kvh_shard_bounds": (I, [P, SZ, I, P]),
        "kvh_host_unregister": (I, [P]),
        "kvh_host_alloc": (I, [C.POINTER(P), SZ]),
        "kvh_host_free": (I, [P]),
        "kvh_device_alloc": (I, [C.POINTER(P), SZ]),
        "kvh_device_free": (I, [P]),
        "kvh_hash_meow128": (I, [P, SZ, C.POINTER(U64), C.POINTER(U64)]),
        "kvh_hash_meow64": (U64, [P, SZ, U64]),
        "kvh_hash_meow128_2_same_length": (I, [P, P, SZ, P]),
        "kvh_hash_meow128_2_diff_length": (I, [P, SZ, P, SZ, P]),
        "kvh_hash_meow128_4_same_length": (I, [P, P, P, P, SZ, P]),
        "kvh_hash_meow128_4_same_length_a": (I, [P, SZ, P]),
        "kvh_hash_meow128_4_same_length_4_seed": (I, [P, P, P, P, SZ, P]),
        "kvh_hash_meow128_4_diff_length": (I, [P, SZ, P, SZ, P, SZ, P, SZ, P]),
        "kvh_hash_meow128_8_same_length": (I, [P, P, P, P, P, P, P, P, SZ, P]),
        "kvh_hash_meow128_8_same_length_a": (I, [P, SZ, P]),
        "kvh_hash_meow128_vec": (I, [P, SZ, C.POINTER(U64), C.POINTER(U64)]),
        "kvh_meow128_init": (I, [P, P, U64, U64, SZ]),
        "kvh_meow128_update": (I, [P, P, P, SZ]),
        "kvh_meow128_final": (I, [P, P, C.POINTER(U64), C.POINTER(U64)]),
        "kvh_meow_test": (I, [P, SZ, C.POINTER(U64), C.POINTER(U64)]),
        "kvh_hash_key_frag": (I, [P, P, C.POINTER(U64), C.POINTER(U64)]),
        "kvh_hash_key_frags": (I, [P, P, SZ, P]),
        "kvh_ht_geom_init": (I, [U64, U32, C.c_float, C.c_uint16, C.c_uint8, P]),
        "kvh_positions_per_key": (U32, [P]),
        "kvh_ht_positions": (I, [P, SZ, P, P, U32, P]),
        "kvh_meow128_fixed_positions": (I, [P, U32, SZ, U64, U64, P, P, P, U32, P]),
        "kvh_crc_c_fixed": (I, [P, U32, SZ, P, U32, P, P]),
        "kvh_crc_c_var": (I, [P, P, SZ, P, U32, P, P]),
        "kvh_crc_c": (U32, [P, SZ, U32]),
        "kvh_hash_uint": (U32, [U32]),
        "kvh_hash_uint2": (U32, [U32, U32]),
        "kvh_crc_c_2_diff": (I, [P, SZ, P, P, SZ, P]),
        "kvh_crc_c_4_diff": (I, [P, SZ, P, P, SZ, P, P, SZ, P, P, SZ, P]),
        "kvh_crc_c_array": (I, [P, P, P, SZ]),
        "kvh_crc_c_key_array": (I, [P, P, P, SZ]),
        "kvh_tokenize_scratch_bytes": (SZ, [SZ]),
        "kvh_tokenize": (I, [P, SZ, U32, P, P, SZ, P, P, SZ, P]),
        "kvh_tokenize_hash": (I, [P, SZ, U32, U64, U64, U32, P, P, P, SZ, P, P, SZ, P]),
        "kvh_meow128_spans": (I, [P, P, P, SZ, U64, U64, P, U32, P]),
        "kvh_meow128_frags": (I, [P, P, SZ, U64, U64, P, U32, P]),
        "kvh_frag_offsets_scratch_bytes": (SZ, [SZ]),
        "kvh_frag_offsets": (I, [P, SZ, P, SZ, P, P, SZ, P]),
        "kvh_frags_hash": (I, [P, SZ, U64, U64, U32, P, P, SZ, P, P, SZ, P]),
        "kvh_ht_sort_scratch_bytes": (SZ, [SZ]),
        "kvh_ht_sort": (I, [P, P, SZ, P, P, P, P, U32, P, SZ, P]),
        "kvh_ht_sort_batched_scratch_bytes": (SZ, [SZ, U32]),
        "kvh_ht_sort_batched": (I, [P, P, SZ, U32, P, P, P, P, U32, P, SZ, P]),
        "kvh_ht_sort_segments_scratch_bytes": (SZ, [SZ, U32]),
        "kvh_ht_sort_segments": (I, [P, P, SZ, P, SZ, U32, P, P, P, P, U32, P, SZ, P]),
        "kvh_ht_radix_sort": (I, [P, U32, P]),
        "kvh_ht_radix_sort_batch": (I, [P, P, U32, P]),
        "kvh_last_error": (I, []),
        "kvh_strerror": (C.c_char_p, [I]),
        "kvh_version": (C.c_char_p, []),
        "kvh_device_synchronize": (I, []),
        "kvh_debug_checks": (I, [P]),
        "kvh_set_tuning": (I, [I, I]),
        "kvh_stream_release": (I, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def check(rc: int, what: str = "kvh") -> None:
    if rc != 0:
        msg = lib.kvh_strerror(rc)
        raise KvhError(f"{what} failed: {rc} ({msg.decode() if msg else '?'})")


# Test hook: with poisoning on, every output this module
# allocates -- device tensors and host arrays -- is filled with 0xA5 bytes
# before the call, so an element the kernel never wrote shows up as a
# mismatch instead of as whatever the caching allocator left there.  Off by
# default (the product allocates outputs uninitialised); tests/conftest.py
# turns it on for the GPU suite, or KVH_POISON_OUTPUTS=1.
_POISON = os.environ.get("KVH_POISON_OUTPUTS", "") == "1"
POISON_BYTE = 0xA5


def set_poison_outputs(on: bool) -> bool:
    """Turn output poisoning on or off; returns the previous setting."""
    global _POISON
    prev, _POISON = _POISON, bool(on)
    return prev


def _empty(shape, dtype, device):
    t = torch.empty(shape, dtype=dtype, device=device)
    if _POISON and t.numel():
        t.view(torch.uint8).fill_(POISON_BYTE)  # on the current stream; _stream_ptr orders a caller's stream after it
    return t


def _np_empty(shape, dtype=np.uint64):
    a = np.empty(shape, dtype=dtype)
    if _POISON:
        a.view(np.uint8).fill(POISON_BYTE)
    return a


def _stream_ptr(stream, *keep) -> Optional[int]:
    """The launch stream.  A caller's own stream first waits for torch's
    current stream: this call's outputs and scratch were just allocated (and
    poisoned) there, and the caching allocator may have handed out a block
    that work still queued on the current stream was using.  Tensors in
    `keep` (scratch dropped on return) are recorded on the caller's stream, so
    the allocator does not reuse them before the launch reading them is done."""
    if stream is not None:
        ptr = int(getattr(stream, "cuda_stream", stream))
        if torch is not None and torch.cuda.is_available():
            cur = torch.cuda.current_stream()
            if ptr != int(cur.cuda_stream):
                ts = _as_torch_stream(stream)
                ts.wait_stream(cur)
                for t in keep:
                    if t is not None and t.is_cuda:
                        t.record_stream(ts)
        return ptr
    if torch is not None and torch.cuda.is_available():
        return int(torch.cuda.current_stream().cuda_stream)
    return None


def _as_torch_stream(stream):
    if hasattr(stream, "wait_stream"):
        return stream
    return torch.cuda.ExternalStream(int(getattr(stream, "cuda_stream", stream)))


def _after_current(stream) -> None:
    """A caller's stream first waits for torch's current stream, on which
    the count / scratch / output tensors of the call were just allocated and
    zeroed."""
    if stream is not None:
        _as_torch_stream(stream).wait_stream(torch.cuda.current_stream())


def _count(cnt, stream) -> int:
    """Read a device count written by kernels on `stream`.  Tensor.item()
    waits only for torch's current stream; a caller's own (non-blocking)
    stream is synchronised first, or the zero-initialised count could be
    read before the kernels that write it have run."""
    if stream is not None:
        _as_torch_stream(stream).synchronize()
    return int(cnt.item())


def _dev_ptr(t) -> int:
    if not t.is_cuda:
        raise KvhError("expected a device tensor")
    if not t.is_contiguous():
        raise KvhError("expected a contiguous tensor")
    return int(t.data_ptr())


def _new_out(shape, like):
    return _empty(shape, torch.int64, like.device)


# --------------------------------------------------------------- batches
def meow128_fixed(keys, key_len: int, seed: Tuple[int, int], out=None, fixup: bool = False,
                  stream=None, n: Optional[int] = None):
    """keys: uint8 device tensor of n*key_len bytes -> int64 [n, 2] (h1, h2 bits)."""
    if n is None:
        n = keys.numel() // key_len if key_len else 0
    if out is None:
        out = _new_out((n, 2), keys)
    check(lib.kvh_meow128_fixed(_dev_ptr(keys) if keys.numel() else None, key_len, n,
                                U64(seed[0] & (2**64 - 1)), U64(seed[1] & (2**64 - 1)),
                                _dev_ptr(out) if n else None, KVH_FIXUP if fixup else 0,
                                _stream_ptr(stream)), "kvh_meow128_fixed")
    return out


def ht_positions(hashes, geom: "HtGeom", out=None, pos32: bool = False, stream=None):
    """hashes: int64 device tensor [n, 2] of fixed-up (h1, h2) -> table
    positions [n, geom.per_key] (int64, or int32 bit patterns with pos32):
    ht_mod(h1) and CuckooAltHash::calc_hash (ht_cuckoo.cpp:38-79)."""
    n = hashes.numel() // 2
    a = geom.per_key
    if out is None:
        out = _empty((n, a), torch.int32 if pos32 else torch.int64, hashes.device)
    check(lib.kvh_ht_positions(_dev_ptr(hashes) if n else None, n, C.byref(geom), _dev_ptr(out) if n else None,
                               KVH_POS32 if pos32 else 0, _stream_ptr(stream)), "kvh_ht_positions")
    return out


def meow128_fixed_positions(keys, key_len: int, seed: Tuple[int, int], geom: "HtGeom", hashes=None,
                            keep_hashes: bool = True, out=None, pos32: bool = False, stream=None):
    """Fused fixed-length hash -> fixup -> table positions.  Returns
    (hashes [n, 2] or None, positions [n, geom.per_key])."""
    n = keys.numel() // key_len if key_len else 0
    a = geom.per_key
    if hashes is None and keep_hashes:
        hashes = _new_out((n, 2), keys)
    if out is None:
        out = _empty((n, a), torch.int32 if pos32 else torch.int64, keys.device)
    check(lib.kvh_meow128_fixed_positions(_dev_ptr(keys) if n else None, key_len, n, U64(seed[0] & (2**64 - 1)),
                                          U64(seed[1] & (2**64 - 1)), C.byref(geom),
                                          _dev_ptr(hashes) if (hashes is not None and n) else None,
                                          _dev_ptr(out) if n else None, KVH_POS32 if pos32 else 0,
                                          _stream_ptr(stream)), "kvh_meow128_fixed_positions")
    return hashes, out


class HtSorter:
    """Device order-by-table-position of hash batches up to `cap` elements
    (kv_ht_radix_sort + ctest dedup); holds its scratch buffer."""

    def __init__(self, geom: "HtGeom", cap: int, device="cuda"):
        self.geom, self.cap = geom, cap
        nb = lib.kvh_ht_sort_scratch_bytes(cap)
        if nb == 0:
            raise KvhError("kvh_ht_sort_scratch_bytes failed")
        self.scratch = torch.empty((nb + 7) // 8, dtype=torch.int64, device=device)
        self.dups = torch.zeros((1,), dtype=torch.int64, device=device)

    def sort(self, hashes, items=None, dedup: bool = False, out=None, items_out=None, stream=None,
             ref_order: bool = False):
        """ref_order: the reference's exact element order (KVH_REF_ORDER,
        kv_ht_radix_sort step for step; n <= 65536); else the engine's total
        order (the same slot order, ties by (h1 << 1, h1, h2))."""
        n = hashes.numel() // 2
        if n > self.cap:
            raise KvhError(f"batch {n} > sorter capacity {self.cap}")
        if out is None:
            out = _new_out((n, 2), hashes)
        if items_out is None:
            items_out = _empty((n,), torch.int64, hashes.device)
        check(lib.kvh_ht_sort(_dev_ptr(hashes) if n else None, _dev_ptr(items) if items is not None else None, n,
                              C.byref(self.geom), _dev_ptr(out) if n else None, _dev_ptr(items_out) if n else None,
                              _dev_ptr(self.dups), (KVH_DEDUP if dedup else 0) | (KVH_REF_ORDER if ref_order else 0),
                              _dev_ptr(self.scratch),
                              self.scratch.numel() * 8,
                              _stream_ptr(stream, self.scratch, self.dups, out, items_out, hashes, items)),
              "kvh_ht_sort")
        return out, items_out


def ht_sort_batched(hashes, geom: "HtGeom", batch: int = 16384, items=None, dedup: bool = False, stream=None):
    """kvh_ht_sort_batched: the (n, 2) device pairs cut into batches of
    `batch` (<= 65536), each in kv_ht_radix_sort's exact order (ctest's batch
    loop, ctest.c:34, :90, :96-104) -> (hashes_out, items_out, dup_counts per
    batch)."""
    n = hashes.numel() // 2
    nb = (n + batch - 1) // batch
    sb = lib.kvh_ht_sort_batched_scratch_bytes(n, batch)
    if sb == 0:
        raise KvhError(f"kvh_ht_sort_batched: batch {batch} out of range")
    scratch = torch.empty((sb + 7) // 8, dtype=torch.int64, device=hashes.device)
    out = _new_out((n, 2), hashes)
    items_out = _empty((n,), torch.int64, hashes.device)
    dups = _empty((max(nb, 1),), torch.int64, hashes.device)
    check(lib.kvh_ht_sort_batched(_dev_ptr(hashes) if n else None, _dev_ptr(items) if items is not None else None, n,
                                  batch, C.byref(geom), _dev_ptr(out) if n else None,
                                  _dev_ptr(items_out) if n else None, _dev_ptr(dups),
                                  KVH_DEDUP if dedup else 0, _dev_ptr(scratch), scratch.numel() * 8,
                                  _stream_ptr(stream, scratch, out, items_out, dups, hashes, items)),
          "kvh_ht_sort_batched")
    return out, items_out, dups[:nb]


def ht_sort_segments(hashes, geom: "HtGeom", seg_offs, max_seg: int = 16384, items=None, dedup: bool = False,
                     stream=None):
    """kvh_ht_sort_segments: batches of any sizes, batch b = pairs
    [seg_offs[b], seg_offs[b+1]) (int64 device tensor, nseg + 1 entries), each
    in kv_ht_radix_sort's exact order -> (hashes_out, items_out, dup_counts;
    ~0 flags a batch longer than max_seg)."""
    n = hashes.numel() // 2
    if not seg_offs.is_cuda or seg_offs.dtype not in (torch.int64, torch.uint64) or not seg_offs.is_contiguous():
        raise KvhError("seg_offs: a contiguous int64/uint64 device tensor of nseg + 1 offsets")
    nseg = max(seg_offs.numel() - 1, 0)
    sb = lib.kvh_ht_sort_segments_scratch_bytes(nseg, max_seg)
    if sb == 0:
        raise KvhError(f"kvh_ht_sort_segments: max_seg {max_seg} out of range")
    scratch = torch.empty((sb + 7) // 8, dtype=torch.int64, device=hashes.device)
    out = _new_out((n, 2), hashes)
    items_out = _empty((n,), torch.int64, hashes.device)
    dups = _empty((max(nseg, 1),), torch.int64, hashes.device)
    check(lib.kvh_ht_sort_segments(_dev_ptr(hashes) if n else None, _dev_ptr(items) if items is not None else None,
                                   n, _dev_ptr(seg_offs) if nseg else None, nseg, max_seg, C.byref(geom),
                                   _dev_ptr(out) if n else None, _dev_ptr(items_out) if n else None, _dev_ptr(dups),
                                   KVH_DEDUP if dedup else 0, _dev_ptr(scratch), scratch.numel() * 8,
                                   _stream_ptr(stream, scratch, out, items_out, dups, hashes, items, seg_offs)),
          "kvh_ht_sort_segments")
    return out, items_out, dups[:nseg]


def tokenize(text, max_token: int = 256, cap: Optional[int] = None, stream=None):
    """ctest.c:202-233 whitespace tokenizer on a uint8 device tensor ->
    (offsets int64 [k], lengths int32 [k]) of the kept tokens in order."""
    n = text.numel()
    cnt = torch.zeros((1,), dtype=torch.int64, device=text.device)
    scratch = torch.empty((max(1, lib.kvh_tokenize_scratch_bytes(n) // 8),), dtype=torch.int64, device=text.device)
    if cap is None:
        cap = n // 2 + 1
    offs = _empty((max(cap, 1),), torch.int64, text.device)
    lens = _empty((max(cap, 1),), torch.int32, text.device)
    _after_current(stream)
    check(lib.kvh_tokenize(_dev_ptr(text) if n else None, n, max_token, _dev_ptr(offs), _dev_ptr(lens), cap,
                           _dev_ptr(cnt), _dev_ptr(scratch), scratch.numel() * 8, _stream_ptr(stream)), "kvh_tokenize")
    k = _count(cnt, stream)
    return offs[:min(k, cap)], lens[:min(k, cap)]


def tokenize_hash(text, seed: Tuple[int, int], max_token: int = 256, cap: Optional[int] = None, fixup: bool = True,
                  nulterm: bool = True, stream=None):
    """kvh_tokenize + kvh_meow128_spans in one asynchronous call (ctest.c:202-233
    with a kv_hash_key_frag per token; the count stays on the device) ->
    (offsets int64 [k], lengths int32 [k], hashes int64 [k, 2])."""
    n = text.numel()
    cnt = torch.zeros((1,), dtype=torch.int64, device=text.device)
    scratch = torch.empty((max(1, lib.kvh_tokenize_scratch_bytes(n) // 8),), dtype=torch.int64, device=text.device)
    if cap is None:
        cap = n // 2 + 1
    offs = _empty((max(cap, 1),), torch.int64, text.device)
    lens = _empty((max(cap, 1),), torch.int32, text.device)
    out = _empty((max(cap, 1), 2), torch.int64, text.device)
    _after_current(stream)
    check(lib.kvh_tokenize_hash(_dev_ptr(text) if n else None, n, max_token, U64(seed[0] & (2**64 - 1)),
                                U64(seed[1] & (2**64 - 1)),
                                (KVH_FIXUP if fixup else 0) | (KVH_NULTERM if nulterm else 0), _dev_ptr(offs),
                                _dev_ptr(lens), _dev_ptr(out), cap, _dev_ptr(cnt), _dev_ptr(scratch),
                                scratch.numel() * 8, _stream_ptr(stream)), "kvh_tokenize_hash")
    k = min(_count(cnt, stream), cap)
    return offs[:k], lens[:k], out[:k]


def meow128_spans(buf, offs, lens, seed: Tuple[int, int], out=None, fixup: bool = True, nulterm: bool = True,
                  stream=None):
    """Meow128 of (offset, length) spans of a device buffer; nulterm hashes
    each span + one 0 byte (the kv_key_frag_t of a token)."""
    n = offs.numel()
    if out is None:
        out = _new_out((n, 2), offs)
    check(lib.kvh_meow128_spans(_dev_ptr(buf), _dev_ptr(offs) if n else None, _dev_ptr(lens) if n else None, n,
                                U64(seed[0] & (2**64 - 1)), U64(seed[1] & (2**64 - 1)), _dev_ptr(out) if n else None,
                                (KVH_FIXUP if fixup else 0) | (KVH_NULTERM if nulterm else 0), _stream_ptr(stream)),
          "kvh_meow128_spans")
    return out


def frag_offsets(buf, cap: Optional[int] = None, stream=None):
    """Record offsets of a packed kv_key_frag_t stream, found on the device
    (list ranking) -> int64 [count]."""
    n = buf.numel()
    cnt = torch.zeros((1,), dtype=torch.int64, device=buf.device)
    scratch = torch.empty((max(1, lib.kvh_frag_offsets_scratch_bytes(n) // 8 + 1),), dtype=torch.int64,
                          device=buf.device)
    if cap is None:
        cap = n // 2 + 1
    offs = _empty((max(cap, 1),), torch.int64, buf.device)
    _after_current(stream)
    check(lib.kvh_frag_offsets(_dev_ptr(buf) if n else None, n, _dev_ptr(offs), cap, _dev_ptr(cnt), _dev_ptr(scratch),
                               scratch.numel() * 8, _stream_ptr(stream)), "kvh_frag_offsets")
    return offs[:min(_count(cnt, stream), cap)]


def frags_hash(buf, seed: Tuple[int, int], cap: Optional[int] = None, fixup: bool = True, stream=None):
    """Hashes of every record of a packed kv_key_frag_t stream in one call
    (offsets found on the device) -> (offsets int64 [k], hashes int64 [k, 2])."""
    n = buf.numel()
    cnt = torch.zeros((1,), dtype=torch.int64, device=buf.device)
    scratch = torch.empty((max(1, lib.kvh_frag_offsets_scratch_bytes(n) // 8 + 1),), dtype=torch.int64,
                          device=buf.device)
    if cap is None:
        cap = n // 2 + 1
    offs = _empty((max(cap, 1),), torch.int64, buf.device)
    out = _empty((max(cap, 1), 2), torch.int64, buf.device)
    _after_current(stream)
    check(lib.kvh_frags_hash(_dev_ptr(buf) if n else None, n, U64(seed[0] & (2**64 - 1)), U64(seed[1] & (2**64 - 1)),
                             KVH_FIXUP if fixup else 0, _dev_ptr(offs), _dev_ptr(out), cap, _dev_ptr(cnt),
                             _dev_ptr(scratch), scratch.numel() * 8, _stream_ptr(stream)), "kvh_frags_hash")
    k = min(_count(cnt, stream), cap)
    return offs[:k], out[:k]


def meow128_frags(buf, rec_offs, seed: Tuple[int, int], out=None, fixup: bool = True, stream=None):
    """Meow128 of packed kv_key_frag_t records at byte offsets rec_offs."""
    n = rec_offs.numel()
    if out is None:
        out = _new_out((n, 2), rec_offs)
    check(lib.kvh_meow128_frags(_dev_ptr(buf), _dev_ptr(rec_offs) if n else None, n, U64(seed[0] & (2**64 - 1)),
                                U64(seed[1] & (2**64 - 1)), _dev_ptr(out) if n else None,
                                KVH_FIXUP if fixup else 0, _stream_ptr(stream)), "kvh_meow128_frags")
    return out


def crc_c_fixed(keys, key_len: int, seed: int = 0, seeds=None, out=None, stream=None):
    """kv_crc_c over n fixed-length keys (key_hash.c:53-63) -> uint32 bit
    patterns in an int32 device tensor [n]; seeds: optional int32 [n]."""
    n = keys.numel() // key_len if key_len else 0
    if out is None:
        out = _empty((n,), torch.int32, keys.device)
    check(lib.kvh_crc_c_fixed(_dev_ptr(keys) if keys.numel() else None, key_len, n,
                              _dev_ptr(seeds) if seeds is not None else None, seed & 0xFFFFFFFF,
                              _dev_ptr(out) if n else None, _stream_ptr(stream)), "kvh_crc_c_fixed")
    return out


def crc_c_var(keys, offsets, seed: int = 0, seeds=None, out=None, stream=None):
    """kv_crc_c over n variable-length keys (u64 offsets [n+1])."""
    n = offsets.numel() - 1
    if out is None:
        out = _empty((n,), torch.int32, offsets.device)
    check(lib.kvh_crc_c_var(_dev_ptr(keys) if keys.numel() else _dev_ptr(offsets), _dev_ptr(offsets), n,
                            _dev_ptr(seeds) if seeds is not None else None, seed & 0xFFFFFFFF,
                            _dev_ptr(out) if n else None, _stream_ptr(stream)), "kvh_crc_c_var")
    return out


def kv_crc_c(data: bytes, seed: int = 0) -> int:
    """Drop-in kv_crc_c (executes on the GPU)."""
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    r = lib.kvh_crc_c(buf, len(data), seed & 0xFFFFFFFF)
    rc = lib.kvh_last_error()
    if rc:
        check(rc, "kvh_crc_c")
    return int(r)


def meow128_var(keys, offsets, seed: Tuple[int, int], out=None, fixup: bool = False, stream=None):
    """keys: uint8 device tensor; offsets: int64 device tensor [n+1] -> int64 [n, 2]."""
    n = offsets.numel() - 1
    if out is None:
        out = _new_out((n, 2), offsets)
    check(lib.kvh_meow128_var(_dev_ptr(keys) if keys.numel() else _dev_ptr(offsets),
                              _dev_ptr(offsets), n, U64(seed[0] & (2**64 - 1)),
                              U64(seed[1] & (2**64 - 1)), _dev_ptr(out) if n else None,
                              KVH_FIXUP if fixup else 0, _stream_ptr(stream)), "kvh_meow128_var")
    return out


def meow128_multiseed(keys, key_len: int, seeds: Sequence[Tuple[int, int]], out=None,
                      fixup: bool = False, stream=None):
    """Each key hashed under every seed -> int64 [n, arity, 2]."""
    n = keys.numel() // key_len
    a = len(seeds)
    sv = (U64 * (2 * a))(*[int(x) & (2**64 - 1) for s in seeds for x in s])
    if out is None:
        out = _new_out((n, a, 2), keys)
    check(lib.kvh_meow128_multiseed(_dev_ptr(keys), key_len, n, sv, a, _dev_ptr(out),
                                    KVH_FIXUP if fixup else 0, _stream_ptr(stream)),
          "kvh_meow128_multiseed")
    return out


def meow128_var_seeded(keys, offsets, seeds, out=None, fixup: bool = False, stream=None):
    """Per-key seeds (int64 device tensor [n, 2]) through the straight-line kernel."""
    n = offsets.numel() - 1
    if out is None:
        out = _new_out((n, 2), offsets)
    check(lib.kvh_meow128_var_seeded(_dev_ptr(keys), _dev_ptr(offsets), n, _dev_ptr(seeds),
                                     _dev_ptr(out), KVH_FIXUP if fixup else 0,
                                     _stream_ptr(stream)), "kvh_meow128_var_seeded")
    return out


def meow128_fixed_host(keys: np.ndarray, key_len: int, seed: Tuple[int, int],
                       out: Optional[np.ndarray] = None, fixup: bool = False) -> np.ndarray:
    """Host keys -> host hashes through the chunked H2D/kernel/D2H pipeline."""
    n = keys.size // key_len
    if out is None:
        out = _np_empty((n, 2))
    check(lib.kvh_meow128_fixed_host(keys.ctypes.data, key_len, n, U64(seed[0]), U64(seed[1]),
                                     out.ctypes.data, KVH_FIXUP if fixup else 0),
          "kvh_meow128_fixed_host")
    return out


def meow128_var_host(keys: np.ndarray, offsets: np.ndarray, seed: Tuple[int, int],
                     out: Optional[np.ndarray] = None, fixup: bool = False) -> np.ndarray:
    """Host keys + host u64 offsets [n+1] -> host hashes [n, 2] through the
    byte-budgeted H2D/kernel/D2H pipeline (kvh_meow128_var_host)."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    if out is None:
        out = _np_empty((n, 2))
    kb = keys if keys.size else np.zeros(1, np.uint8)
    check(lib.kvh_meow128_var_host(kb.ctypes.data, offsets.ctypes.data, n, U64(seed[0]), U64(seed[1]),
                                   out.ctypes.data, KVH_FIXUP if fixup else 0), "kvh_meow128_var_host")
    return out


def meow128_host_multi(keys: np.ndarray, seed: Tuple[int, int], devices: Sequence[int], key_len: int = 0,
                       offsets: Optional[np.ndarray] = None, out: Optional[np.ndarray] = None,
                       fixup: bool = False) -> np.ndarray:
    """One host batch sharded over `devices` (one host thread each):
    kvh_meow128_fixed_host_multi (key_len) or kvh_meow128_var_host_multi
    (offsets)."""
    dv = (C.c_int * len(devices))(*devices)
    fl = KVH_FIXUP if fixup else 0
    kb = keys if keys.size else np.zeros(1, np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        out = _np_empty((n, 2)) if out is None else out
        check(lib.kvh_meow128_var_host_multi(kb.ctypes.data, offsets.ctypes.data, n, U64(seed[0]), U64(seed[1]),
                                             out.ctypes.data, fl, dv, len(devices)), "kvh_meow128_var_host_multi")
    else:
        n = keys.size // key_len
        out = _np_empty((n, 2)) if out is None else out
        check(lib.kvh_meow128_fixed_host_multi(kb.ctypes.data, key_len, n, U64(seed[0]), U64(seed[1]),
                                               out.ctypes.data, fl, dv, len(devices)),
              "kvh_meow128_fixed_host_multi")
    return out


def shard_bounds(n: int, nshards: int, offsets: Optional[np.ndarray] = None) -> np.ndarray:
    """kvh_shard_bounds: the shard arithmetic of the _host_multi entries."""
    b = np.zeros(nshards + 1, dtype=np.uint64)
    op = None
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        op = offsets.ctypes.data
    check(lib.kvh_shard_bounds(op, n, nshards, b.ctypes.data), "kvh_shard_bounds")
    return b


def host_empty(shape, dtype=np.uint8) -> np.ndarray:
    """A numpy array over pinned host memory from kvh_host_alloc (freed with
    the array): the buffers kvh_meow128_fixed_host DMAs at full PCIe rate."""
    dt = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dt.itemsize
    ptr = P()
    check(lib.kvh_host_alloc(C.byref(ptr), max(nbytes, 1)), "kvh_host_alloc")
    buf = (C.c_uint8 * max(nbytes, 1)).from_address(ptr.value)
    arr = np.frombuffer(buf, dtype=np.uint8, count=nbytes).view(dt).reshape(shape)
    weakref.finalize(buf, lib.kvh_host_free, ptr.value)
    return arr


# ------------------------------------------------------------- drop-ins
def kv_hash_meow128(data: bytes, h1: int, h2: int) -> Tuple[int, int]:
    """key_hash.h:61 semantics: (h1, h2) are the seed in and the hash out."""
    a, b = U64(h1 & (2**64 - 1)), U64(h2 & (2**64 - 1))
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    check(lib.kvh_hash_meow128(buf, len(data), C.byref(a), C.byref(b)), "kvh_hash_meow128")
    return a.value, b.value


def kv_hash_meow64(data: bytes, seed: int) -> int:
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    return int(lib.kvh_hash_meow64(buf, len(data), U64(seed & (2**64 - 1))))


class HashSeed:
    """shm_ht.h:333-351 HashSeed: a per-db 128-bit seed."""

    def __init__(self, hash1: int, hash2: int):
        self.hash1, self.hash2 = hash1 & (2**64 - 1), hash2 & (2**64 - 1)

    def hash(self, kb: "KeyFragment") -> Tuple[int, int]:
        return kb.hash(self.hash1, self.hash2)

    def hash_batch(self, frags: Iterable["KeyFragment"]) -> np.ndarray:
        frags = list(frags)
        return KeyFragment.hash_many(frags, self.hash1, self.hash2)


class KeyFragment:
    """hash_entry.h:56-112 KeyFragment: u16 keylen + bytes."""

    def __init__(self, data: bytes):
        if len(data) > 0xFFFF:
            raise ValueError("keylen is a u16")
        self.data = bytes(data)

    @classmethod
    def from_string(cls, s: str) -> "KeyFragment":
        """KeyBufT::set_string / kv_set_key_frag_string: includes the NUL."""
        return cls(s.encode() + b"\0")

    def _raw(self):
        raw = C.create_string_buffer(2 + len(self.data) + 4)
        C.memmove(raw, len(self.data).to_bytes(2, "little") + self.data, 2 + len(self.data))
        return raw

    def hash(self, seed: int, seed2: int) -> Tuple[int, int]:
        """KeyFragment::hash: Meow128 then the ZOMBIE/reserved fixup on h1."""
        sv = (U64 * 2)(seed & (2**64 - 1), seed2 & (2**64 - 1))
        k, k2 = U64(), U64()
        check(lib.kvh_hash_key_frag(sv, self._raw(), C.byref(k), C.byref(k2)), "kvh_hash_key_frag")
        return k.value, k2.value

    @staticmethod
    def hash_many(frags: Sequence["KeyFragment"], seed: int, seed2: int) -> np.ndarray:
        sv = (U64 * 2)(seed & (2**64 - 1), seed2 & (2**64 - 1))
        raws = [f._raw() for f in frags]
        arr = (P * max(1, len(raws)))(*[C.cast(r, P) for r in raws])
        out = _np_empty((len(frags), 2))
        check(lib.kvh_hash_key_frags(sv, arr, len(frags), out.ctypes.data), "kvh_hash_key_frags")
        return out


def as_u64(t) -> np.ndarray:
    """int64 device/host tensor -> numpy uint64 view."""
    if torch is not None and isinstance(t, torch.Tensor):
        t = t.detach().cpu().numpy()
    return np.ascontiguousarray(t).view(np.uint64)
