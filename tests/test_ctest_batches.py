"""CPU: the one-step-per-batch form of ctest's batch boundaries equals the
token-by-token loop (tests/ctest_batches.py)."""
import numpy as np

from ctest_batches import (CTEST_BLOCK, ctest_batches, ctest_batches_loop, ctest_block_batches, ctest_blocks,
                           ctest_loop_text)
from oracle_lib import load_oracle, orc_tokenize


def test_ctest_batches_forms_agree():
    rng = np.random.default_rng(5)
    for lo, hi, n in ((1, 2, 70000), (1, 14, 200000), (1, 256, 50000), (200, 256, 3000), (1, 8, 1)):
        lens = rng.integers(lo, hi, n)
        a, b = ctest_batches_loop(lens), ctest_batches(lens)
        np.testing.assert_array_equal(a, b)
        assert a[0] == 0 and a[-1] == n
        assert np.all(np.diff(a.astype(np.int64)) > 0) and np.all(np.diff(a.astype(np.int64)) <= 16384)
    assert ctest_batches_loop(np.zeros(0, np.int64)).tolist() == [0]
    assert ctest_batches(np.zeros(0, np.int64)).tolist() == [0]


def test_block_batches_follow_ctests_read_blocks():
    """over several 256 KiB read blocks, tokenizing each block on
    its own (oracle tokenizer) and cutting batches per block gives exactly
    ctest's byte-by-byte loop: tokens cut at block ends, batches never span a
    block, every block flushes its last batch."""
    rng = np.random.default_rng(9)
    words = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(1, 14, 3000)]
    seps = [b" ", b"\n", b"\t", b"  "]
    parts = [words[int(i)] + seps[int(j)] for i, j in zip(rng.integers(0, 3000, 120000), rng.integers(0, 4, 120000))]
    parts.insert(5000, b"x" * 300)  # a token too long to keep
    text = b"".join(parts)[:3 * CTEST_BLOCK + 12345]
    toks, cuts = ctest_loop_text(text)
    orc = load_oracle()
    arr = np.frombuffer(text, np.uint8)
    offs, lens = [], []
    for s, e in ctest_blocks(len(text)):
        o, l = orc_tokenize(orc, arr[s:e].copy(), 256)
        offs.append(o.astype(np.int64) + s)
        lens.append(l)
    np.testing.assert_array_equal(np.concatenate(offs), np.array([t[0] for t in toks], np.int64))
    np.testing.assert_array_equal(np.concatenate(lens), np.array([t[1] for t in toks], np.int64))
    np.testing.assert_array_equal(ctest_block_batches(lens), cuts)
    assert len(ctest_blocks(len(text))) == 4
