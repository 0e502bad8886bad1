"""CPU: the ingest oracle (oracle/ingest_oracle.c) against
the reference's own ctest-style ingest (tests/golden/ingest.npz:
kv_make_key_frag + kv_set_key_frag_string records and kv_hash_key_frag
hashes), plus tokenizer edge cases and C-ABI argument checks."""
import os

import numpy as np

from oracle_lib import GOLDEN, load_oracle, orc_hash_spans, orc_tokenize

G = np.load(os.path.join(GOLDEN, "ingest.npz"))
ORC = load_oracle()


def frag_records(frags, rec_offs):
    out = []
    for o in rec_offs:
        o = int(o)
        kl = int(frags[o]) | (int(frags[o + 1]) << 8)
        out.append(frags[o + 2:o + 2 + kl].tobytes())
    return out


def test_tokens_match_reference_records():
    text = G["text"]
    offs, lens = orc_tokenize(ORC, text, int(G["max_token"][0]))
    recs = frag_records(G["frags"], G["rec_offs"])
    assert len(recs) == len(offs)
    for (o, l), r in zip(zip(offs, lens), recs):
        assert r == text[int(o):int(o) + int(l)].tobytes() + b"\0"
    # records are packed back to back, 2-byte aligned (kv_make_key_frag)
    ro = G["rec_offs"].astype(np.int64)
    sizes = np.array([(len(r) + 2 + 1) & ~1 for r in recs], dtype=np.int64)
    np.testing.assert_array_equal(ro[1:], ro[:-1] + sizes[:-1])


def test_hashes_match_kv_hash_key_frag():
    text = G["text"]
    offs, lens = orc_tokenize(ORC, text, 256)
    got = orc_hash_spans(ORC, text, offs, lens, tuple(int(x) for x in G["seed"]), nul=True, fix=True)
    np.testing.assert_array_equal(got, G["hashes"])


def test_tokenizer_edges():
    def tok(s, m=256):
        o, l = orc_tokenize(ORC, np.frombuffer(s, dtype=np.uint8).copy(), m)
        return [s[int(a):int(a) + int(b)] for a, b in zip(o, l)]
    assert tok(b"") == []
    assert tok(b"   \n\t ") == []
    assert tok(b"a") == [b"a"]
    assert tok(b" a  bb\tccc\n") == [b"a", b"bb", b"ccc"]
    assert tok(b"x" * 255 + b" y") == [b"x" * 255, b"y"]
    assert tok(b"x" * 256 + b" y") == [b"y"]          # i < MAX_TOKEN_SIZE
    assert tok(b"ab\rcd\x00ef") == [b"ab\rcd\x00ef"]  # only ' ', '\n', '\t' separate
    assert tok(b"abc de", 3) == [b"de"]                # max_token 3 keeps tokens of < 3 bytes


def test_capi_ingest_argument_checks_without_device():
    import raikv_amd as kvh
    lib = kvh.lib
    for n in (0, 1, 65536, 65536 * 3 + 17, 1 << 30):
        assert lib.kvh_tokenize_scratch_bytes(n) >= 8 * ((n + 31) // 65536 + 1)
    assert lib.kvh_tokenize(None, 100, 256, None, None, 0, None, None, 0, None) == -22  # no count
    assert lib.kvh_meow128_spans(None, None, None, 0, 0, 0, None, 0, None) == 0
    assert lib.kvh_meow128_spans(None, None, None, 5, 0, 0, None, 0, None) == -22
    assert lib.kvh_meow128_frags(None, None, 5, 0, 0, None, 0, None) == -22
