"""C2 lengths reordered so that each 256-key window is already sorted by
16-byte length class (stable): k_var9's window sort then leaves the order as
it is, and the no-sort ablation (knob 7 = 61, experiments build) hashes the
same chunks -- their time difference is the sort's cost."""
import numpy as np


def presort_windows(lens: np.ndarray, win: int = 256) -> np.ndarray:
    lens = np.asarray(lens)
    out = lens.copy()
    n = len(lens)
    m = n // win * win
    cls = np.minimum(lens >> 4, 63)
    if m:
        idx = np.argsort(cls[:m].reshape(-1, win), axis=1, kind="stable")
        out[:m] = np.take_along_axis(lens[:m].reshape(-1, win), idx, axis=1).reshape(-1)
    if m < n:
        out[m:] = lens[m:][np.argsort(cls[m:], kind="stable")]
    return out
