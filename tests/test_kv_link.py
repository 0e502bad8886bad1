"""CPU (container): raikv links against libkvh_kv.so unchanged (VERDICT r5
item 7).

The reference's library objects (GNUmakefile:137-158, libraikv_files) are
compiled from their sources where they lie (oracle/Makefile `kvcore`), with
src/key_hash.c left out.  Then:
  - every kv_* symbol those objects leave undefined is defined by another of
    them or exported by libkvh_kv.so: nothing of key_hash.c is missing (the
    ones the library uses are kv_hash_meow128, kv_crc_c, kv_crc_c_key_array and
    kv_hash_uint2: key_ctx.cpp:1774-1783, ht_init.cpp, route_db.cpp);
  - the KV-core subset (ht_init, ht_cuckoo, key_ctx, ... radix_sort) plus the
    golden-vector driver links with -Wl,--no-undefined against libkvh_kv.so
    (oracle/_ref/libkvref_ht_kvh.so), and does not without it.
tests/test_gpu_kv_link.py runs that library on the GPU box against the reference.
ev_tcp / ev_udp / ev_cares include c-ares' ares.h, absent from this image; their
sources name none of key_hash.c's functions (checked as text below).
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(ROOT, "oracle", "_ref")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "key_hash.c")),
                                reason="the reference tree is only in the build container")


def _syms(args, path):
    r = subprocess.run(["nm"] + args + [path], capture_output=True, text=True, check=True)
    out = set()
    for line in r.stdout.splitlines():
        parts = line.split()
        if len(parts) >= 2:
            out.add((parts[-2], parts[-1]))
    return out


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", ROOT, "raikv_amd/libkvh_kv.so"], check=True, capture_output=True)
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-j8", "kvcore", "_ref/libkvref_ht_kvh.so"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(OUT, "kvcore")


def test_library_objects_need_nothing_kvh_kv_lacks(built):
    objs = sorted(os.path.join(built, f) for f in os.listdir(built) if f.endswith(".o"))
    assert len(objs) == 22
    undef, defined = set(), set()
    for o in objs:
        for t, name in _syms([], o):
            if t == "U":
                undef.add(name)
            elif t in "TDBRVW":
                defined.add(name)
    exported = {name for t, name in _syms(["-D", "--defined-only"], os.path.join(ROOT, "raikv_amd", "libkvh_kv.so"))}
    need = {s for s in undef if s.startswith("kv_")} - defined
    assert need == {"kv_hash_meow128", "kv_crc_c", "kv_crc_c_key_array", "kv_hash_uint2"}, need
    assert need <= exported, need - exported
    # the three objects this image cannot compile name none of key_hash.c's functions
    kobj = os.path.join(OUT, "key_hash_syms.o")  # compiled only to list what it defines; linked nowhere
    subprocess.run(["gcc", "-c", "-O0", "-mavx", "-maes", "-I" + os.path.join(REF, "include"), "-o", kobj,
                    os.path.join(REF, "src", "key_hash.c")], check=True)
    kh = {name for t, name in _syms(["--defined-only"], kobj) if t == "T"}
    assert {"kv_hash_meow128", "kv_crc_c", "kv_hash_murmur64"} <= kh and need <= kh
    for f in ("ev_tcp.cpp", "ev_udp.cpp", "ev_cares.cpp"):
        src = open(os.path.join(REF, "src", f), encoding="latin-1").read()
        assert not (set(re.findall(r"\b(kv_\w+)\s*\(", src)) & kh), f


def test_kv_core_links_with_no_undefined_against_kvh_kv(built):
    lib = os.path.join(OUT, "libkvref_ht_kvh.so")
    assert os.path.exists(lib)
    und = {name for t, name in _syms(["-D", "--undefined-only"], lib)}
    assert {"kv_hash_meow128", "kv_crc_c"} <= und  # resolved from libkvh_kv.so at load time
    r = subprocess.run(["ldd", lib], capture_output=True, text=True)
    assert "libkvh_kv.so" in r.stdout and "not found" not in r.stdout.split("libkvh_kv.so")[1].splitlines()[0]
    # control: without libkvh_kv.so the same link fails on exactly key_hash.c's symbols
    ht = ["ht_init", "ht_cuckoo", "key_ctx", "ht_linear", "msg_ctx", "ht_stats", "scratch_mem", "rela_ts", "util",
          "print", "radix_sort"]
    r = subprocess.run(["g++", "-shared", "-o", "/dev/null"] + [os.path.join(built, f + ".o") for f in ht] +
                       ["-Wl,--no-undefined", "-lpthread", "-lrt"], capture_output=True, text=True)
    assert r.returncode != 0
    missing = set(re.findall(r"undefined reference to `(\w+)'", r.stderr))
    assert missing and missing <= {"kv_hash_meow128", "kv_crc_c", "kv_crc_c_key_array", "kv_hash_uint2"}, missing
