"""Bitsliced AESDEC / Meow chain (raikv_amd/csrc/bs_aes.hpp, bs_meow.hpp).

CPU: the generated circuits are reproducible from tools/gen_bitslice.py (which
checks every circuit bit-exactly against a direct AESDEC before writing), and
the bitsliced Meow chain, run on the host with the gfx950 primitives emulated
(tests/cpp/bs_host_test.cpp), equals the oracle's kv_hash_meow128
(key_hash.c:1413-1429) for 16/32/48-byte keys under random and edge seeds.
The hybrid kernel that runs this chain beside the T-table waves (+1-2 % on
C1) lost its A/B and lives only in the experiments build
(tools/libkvh_exp.so); tools/check_hybrid.py checks it on a GPU.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def test_generator_reproduces_committed_header(tmp_path):
    out = tmp_path / "bs_aes.hpp"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_bitslice.py"), "--out", str(out)],
                   check=True, capture_output=True, timeout=300)
    with open(os.path.join(ROOT, "raikv_amd", "csrc", "bs_aes.hpp")) as fh:
        assert out.read_text() == fh.read()


def test_bitsliced_chain_matches_oracle_on_host():
    exe = os.path.join(ROOT, "tests", "cpp", "bs_host_test")
    assert os.path.exists(exe), "run `make` (or __graft_entry__.build()) first"
    r = subprocess.run([exe, "48"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("bs_host_test ok 1152")
