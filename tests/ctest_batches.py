"""ctest's batch boundaries over its kept tokens (test/ctest.c:31-34,
:214-222): a batch is processed when 16K frags are queued (the frag buffer
carries on), or when the next kv_make_key_frag record -- align(keylen + 2, 2)
bytes, keylen = token + NUL (src/key_ctx.cpp:1738-1745) -- does not fit the
64 KiB frag buffer (buffer and count restart).  Host-side test helper: the
boundaries kvh_ht_sort_segments takes to sort ctest's batches.

ctest reads its input in blocks of 256 KiB (ctest.c:31 `str[256 * 1024]`,
one read() per block, :316-340) and tokenizes each block on its own: the
block end acts as a separator (:206, `p == ens`), the frag count and the frag
buffer restart at each block (:198-201) and a block's last batch is flushed
at its end (:236-237).  ctest_blocks / ctest_block_batches follow that; the
single-block forms above are exact for one block of at most 256 KiB."""
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


CTEST_BLOCK = 256 * 1024  # ctest.c:31: the read buffer, one read() per block


def ctest_blocks(nbytes: int, block: int = CTEST_BLOCK):
    """(start, end) byte ranges of ctest's read blocks over an input of
    nbytes, read() returning full blocks (a file)."""
    return [(s, min(s + block, nbytes)) for s in range(0, nbytes, block)]


def ctest_block_batches(block_lens, max_frags=MAX_FRAGS, buf_bytes=BUF_BYTES):
    """ctest's batches over several read blocks: block_lens[b] = the kept
    token lengths of block b tokenized on its own.  Count and buffer restart
    per block, and every block flushes its last batch -> cuts over the
    blocks' tokens concatenated in order."""
    cuts, base = [0], 0
    for lens in block_lens:
        c = ctest_batches(lens, max_frags, buf_bytes)
        cuts.extend(int(x) + base for x in c[1:])
        base += len(lens)
    return np.array(cuts, dtype=np.uint64)


def ctest_loop_text(text: bytes, max_token: int = 256, block: int = CTEST_BLOCK, max_frags=MAX_FRAGS,
                    buf_bytes=BUF_BYTES):
    """ctest's reader + tokenizer + batching loop (ctest.c:195-237, :316-340)
    byte by byte in pure Python (small inputs only): -> (token (offset,
    length) pairs in input order, batch cuts)."""
    toks, cuts = [], [0]
    ws = b" \n\t"
    for s, e in ctest_blocks(len(text), block):
        count = used = 0
        i = 0
        for p in range(s, e + 1):
            if p < e and text[p] not in ws:
                i += 1
                continue
            if 0 < i < max_token:
                rec = (i + 1 + 2 + 1) & ~1
                if count == max_frags:
                    cuts.append(len(toks))
                    count = 0
                if used + rec > buf_bytes:
                    if count:  # an empty process_key_frags is no batch
                        cuts.append(len(toks))
                    count, used = 0, 0
                used += rec
                toks.append((p - i, i))
                count += 1
            i = 0
        if count:
            cuts.append(len(toks))
    return toks, np.array(cuts, dtype=np.uint64)
