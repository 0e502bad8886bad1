"""CPU: the CRC32C oracle (oracle/crc_oracle.c) against
the reference's own kv_crc_c / kv_crc_c_array / kv_crc_c_key_array /
kv_hash_uint outputs (tests/golden/crc32c.npz), and the C-ABI's argument
checks (no device calls)."""
import os

import numpy as np

from oracle_lib import GOLDEN, load_oracle, orc_crc, orc_crc_var

G = np.load(os.path.join(GOLDEN, "crc32c.npz"))
ORC = load_oracle()


def test_known_answer():
    # CRC32C check value for "123456789" is 0xE3069283 with the usual
    # ~0 init / ~ final; kv_crc_c has neither, so apply them around it
    assert orc_crc(ORC, b"123456789", 0xFFFFFFFF) ^ 0xFFFFFFFF == 0xE3069283
    assert orc_crc(ORC, b"", 1234) == 1234


def test_every_length_and_seed():
    keys, seeds, want = G["len_keys"], G["len_seeds"], G["len_out"]
    for L in range(want.shape[0]):
        for si, s in enumerate(seeds):
            assert orc_crc(ORC, keys[L, :L].tobytes(), int(s)) == int(want[L, si]), (L, int(s))


def test_array_with_per_key_seeds():
    got = orc_crc_var(ORC, G["var_keys"], G["var_offsets"], seeds=G["var_seeds"])
    np.testing.assert_array_equal(got, G["var_out"])


def test_key_array_prefixes():
    buf = G["prefix_buf"].tobytes()
    for L, s, w in zip(G["prefix_lens"], G["prefix_seeds"], G["prefix_out"]):
        assert orc_crc(ORC, buf[:int(L)], int(s)) == int(w)


def test_hash_uint():
    for i, w, w2, r in zip(G["uint_in"], G["uint_out"], G["uint2_out"], G["uint_in"][::-1]):
        assert orc_crc(ORC, int(i).to_bytes(4, "little"), 0) == int(w)
        assert orc_crc(ORC, int(r).to_bytes(4, "little"), int(i)) == int(w2)


def test_capi_crc_argument_checks_without_device():
    import raikv_amd as kvh
    lib = kvh.lib
    assert lib.kvh_crc_c_fixed(None, 16, 0, None, 0, None, None) == 0
    assert lib.kvh_crc_c_fixed(None, 16, 10, None, 0, None, None) == -22
    assert lib.kvh_crc_c_var(None, None, 10, None, 0, None, None) == -22
    assert lib.kvh_crc_c_array(None, None, None, 0) == 0
