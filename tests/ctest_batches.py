"""ctest's batch boundaries over its kept tokens (test/ctest.c:31-34,
:214-222): a batch is processed when 16K frags are queued (the frag buffer
carries on), or when the next kv_make_key_frag record -- align(keylen + 2, 2)
bytes, keylen = token + NUL (src/key_ctx.cpp:1738-1745) -- does not fit the
64 KiB frag buffer (buffer and count restart).  Host-side test helper: the
boundaries kvh_ht_sort_segments takes to sort ctest's batches."""
import numpy as np

MAX_FRAGS = 16 * 1024
BUF_BYTES = 64 * 1024


def ctest_batches_loop(lens, max_frags=MAX_FRAGS, buf_bytes=BUF_BYTES):
    """Token by token, as ctest's loop runs."""
    cuts, count, used = [0], 0, 0
    for k, L in enumerate(lens):
        rec = (int(L) + 1 + 2 + 1) & ~1
        if count == max_frags:
            cuts.append(k)
            count = 0
        if used + rec > buf_bytes:
            if count:
                cuts.append(k)
            count, used = 0, 0
        used += rec
        count += 1
    if count:
        cuts.append(len(lens))
    return np.array(cuts, dtype=np.uint64)


def ctest_batches(lens, max_frags=MAX_FRAGS, buf_bytes=BUF_BYTES):
    """The same, one step per batch: prefix sums of the record sizes and a
    search for where the buffer overflows (for 200M tokens)."""
    lens = np.asarray(lens, dtype=np.int64)
    n = len(lens)
    cum = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((lens + 1 + 2 + 1) & ~1, out=cum[1:])
    cuts = [0]
    s = c = 0  # buffer epoch start, count epoch start
    while c < n:
        kc = c + max_frags  # the count cut
        kb = int(np.searchsorted(cum, cum[s] + buf_bytes, side="right")) - 1  # first token that does not fit
        if kc < kb and kc < n:
            cuts.append(kc)
            c = kc
        elif kb < n:
            cuts.append(kb)
            s = c = kb
        else:
            cuts.append(n)
            break
    return np.array(cuts, dtype=np.uint64)
