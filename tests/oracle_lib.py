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
