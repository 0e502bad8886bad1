"""raikv_amd -- MI355X (gfx950) batched 128-bit Meow key hash for raikv.

Python plumbing over the C-ABI in include/kvh.h (libkvh.so, built in-tree
by `make` / __graft_entry__.build()).  The product path is the HIP library;
there is no CPU fallback: if libkvh.so is missing, importing the binding
raises.  Torch is only used for device memory and streams.
"""
from __future__ import annotations

from .binding import (  # noqa: F401
    KVH_FIXUP,
    KVH_POS32,
    HtGeom,
    crc_c_fixed,
    tokenize,
    tokenize_hash,
    frag_offsets,
    frags_hash,
    HtSorter,
    ht_sort_batched,
    ht_sort_segments,
    KVH_DEDUP,
    KVH_REF_ORDER,
    set_poison_outputs,
    meow128_spans,
    meow128_frags,
    KVH_NULTERM,
    crc_c_var,
    kv_crc_c,
    ht_positions,
    meow128_fixed_positions,
    KvhError,
    lib,
    lib_path,
    meow128_fixed,
    meow128_var,
    meow128_multiseed,
    meow128_var_seeded,
    meow128_fixed_host,
    meow128_var_host,
    meow128_host_multi,
    shard_bounds,
    host_empty,
    kv_hash_meow128,
    kv_hash_meow64,
    HashSeed,
    KeyFragment,
)
from .workload import STATIC_SEED  # noqa: F401

__all__ = [
    "KVH_FIXUP", "KvhError", "lib", "lib_path", "meow128_fixed", "meow128_var",
    "meow128_multiseed", "meow128_var_seeded", "meow128_fixed_host", "meow128_var_host", "meow128_host_multi", "shard_bounds", "host_empty", "kv_hash_meow128",
    "kv_hash_meow64", "HashSeed", "KeyFragment", "STATIC_SEED", "KVH_POS32", "HtGeom", "ht_positions",
    "meow128_fixed_positions", "crc_c_fixed", "crc_c_var", "kv_crc_c",
    "tokenize", "tokenize_hash", "frag_offsets", "frags_hash", "meow128_spans", "meow128_frags", "KVH_NULTERM", "HtSorter", "ht_sort_batched", "ht_sort_segments", "KVH_DEDUP", "KVH_REF_ORDER", "set_poison_outputs",
]
