"""CPU: the one-step-per-batch form of ctest's batch boundaries equals the
token-by-token loop (tests/ctest_batches.py)."""
import numpy as np

from ctest_batches import ctest_batches, ctest_batches_loop


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
