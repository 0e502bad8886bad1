/*
 * oracle/ingest_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker
 * for SURVEY.md §8 row f3, key ingest).  Linked into liboracle.so; nothing
 * in the product links, loads or calls it.
 *
 * Clean-room restatement of ctest.c's tokenizer (test/ctest.c:202-233):
 * scan the text once; a token is a maximal run of bytes other than ' ',
 * '\n', '\t'; a token of i bytes is kept when 0 < i < max_token
 * (MAX_TOKEN_SIZE, ctest.c:23).  Each kept token becomes the key
 * "token\0" (kv_set_key_frag_string, src/key_ctx.cpp:1764-1772), hashed by
 * kv_hash_key_frag (key_ctx.cpp:1774-1783) = orc_meow128 + the
 * KeyFragment fixup (meow_oracle.c).
 *
 * Pinning: tests/golden/ingest.npz holds the reference's own frag records,
 * offsets and hashes (oracle/ref_cuckoo.cpp ref_ctest_frags, generator
 * tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

void orc_meow128(const void *p, size_t sz, uint64_t *x1, uint64_t *x2);
uint64_t orc_fixup(uint64_t h1);

static int ws(uint8_t c) { return c == ' ' || c == '\n' || c == '\t'; }

/* kept tokens' (offset, length) in text order; returns the kept count
 * (offsets/lengths written for the first `cap`) */
size_t orc_tokenize(const uint8_t *text, size_t n, uint32_t max_token, uint64_t *offs, uint32_t *lens, size_t cap)
{
  size_t cnt = 0, i = 0;
  for (size_t p = 0; p <= n; p++) {
    if (p < n && !ws(text[p])) { i++; continue; }
    if (i > 0 && i < max_token) {
      if (cnt < cap) { offs[cnt] = p - i; lens[cnt] = (uint32_t) i; }
      cnt++;
    }
    i = 0;
  }
  return cnt;
}

/* hash of span + optional NUL (fixup optional), per span */
void orc_hash_spans(const uint8_t *buf, const uint64_t *offs, const uint32_t *lens, size_t n, uint64_t s1,
                    uint64_t s2, int nul, int fix, uint64_t *out)
{
  uint8_t tmp[65536 + 1];
  for (size_t k = 0; k < n; k++) {
    const size_t L = lens[k];
    memcpy(tmp, buf + offs[k], L);
    tmp[L] = 0;
    uint64_t h1 = s1, h2 = s2;
    orc_meow128(tmp, L + (nul ? 1 : 0), &h1, &h2);
    out[2 * k] = fix ? orc_fixup(h1) : h1;
    out[2 * k + 1] = h2;
  }
}
