/*
 * oracle/ref_cuckoo.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Driver compiled together with the unmodified reference KV-core sources
 * (oracle/Makefile) into oracle/_ref/libkvref_ht.so.  It builds a malloc()
 * HashTab (HashTab::alloc_map, src/ht_init.cpp:252-261) of the requested
 * geometry and asks the reference's CuckooAltHash::calc_hash
 * (src/ht_cuckoo.cpp:38-79) for the arity table positions of given
 * (h1, h2) pairs, exactly as KeyCtx::acquire_cuckoo does
 * (src/ht_cuckoo.cpp:374-398) after KeyCtx::set_hash (src/key_ctx.cpp:89-94:
 * start = ht_mod(h1)).  A linear table (cuckoo_buckets <= 1 selects
 * acquire_linear_probe, src/key_ctx.cpp:130) has only the start slot; so
 * does arity <= 1.  Used only to produce golden vectors; no reference
 * source is copied here.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <new>
#include <raikv/shm_ht.h>
#include <raikv/key_ctx.h>
#include <raikv/ht_cuckoo.h>

using namespace rai::kv;

extern "C" int ref_cuckoo_positions(uint64_t map_size, uint32_t entry_size, float ratio, uint16_t buckets,
                                    uint8_t arity, const uint64_t *h, size_t n, uint64_t *pos,
                                    uint64_t *geom_out) {
  HashTabGeom g;
  memset(&g, 0, sizeof(g));
  g.map_size = map_size;
  g.max_value_size = 0;
  g.hash_entry_size = entry_size;
  g.hash_value_ratio = ratio;
  g.cuckoo_buckets = buckets;
  g.cuckoo_arity = arity;
  HashTab *ht = HashTab::alloc_map(g);
  if (ht == NULL) return -1;
  {
    KeyCtx kctx(*ht, 0);
    alignas(64) char buf[sizeof(CuckooAltHash) + 3 * 8 * 256];
    CuckooAltHash *c = new (buf) CuckooAltHash(arity);
    const bool cuckoo = buckets > 1 && arity > 1;
    for (size_t i = 0; i < n; i++) {
      kctx.set_hash(h[2 * i], h[2 * i + 1]);
      if (!cuckoo) {
        pos[i] = kctx.start;
        continue;
      }
      c->calc_hash(kctx, kctx.key, kctx.key2, kctx.start);
      for (uint8_t a = 0; a < arity; a++) pos[i * arity + a] = c->pos[a];
    }
  }
  geom_out[0] = ht->hdr.ht_mod_mask;
  geom_out[1] = ht->hdr.ht_mod_fraction;
  geom_out[2] = ht->hdr.ht_mod_shift;
  geom_out[3] = ht->hdr.ht_size;
  ::free(ht);
  return 0;
}

/* CPU baseline for bench.py's f1/f1p configs: the reference's per-key path
 * (kv_hash_meow128 + KeyFragment fixup as in KeyCtx::set_key_hash,
 * key_ctx.cpp:97-105, then CuckooAltHash::calc_hash) on `threads` pthreads.
 * The table geometry is written into a header-only HashTab (hdr + ctx +
 * stats regions, zeroed): calc_hash and KeyCtx read only header fields, so
 * a 64 GiB map's geometry needs no 64 GiB allocation.  keys == NULL times
 * calc_hash alone on the given hashes (f1p).  Returns elapsed seconds. */
#include <pthread.h>
#include <time.h>
extern "C" void kv_hash_meow128(const void *p, size_t sz, uint64_t *h1, uint64_t *h2);

namespace {
struct BenchArg {
  HashTab *ht;
  const uint8_t *keys;
  size_t len, lo, hi;
  uint64_t s1, s2;
  uint64_t *hashes, *pos;
};

void *bench_thr(void *vp) {
  BenchArg *a = (BenchArg *) vp;
  KeyCtx kctx(*a->ht, 0);
  const uint8_t ar = a->ht->hdr.cuckoo_arity;
  alignas(64) char buf[sizeof(CuckooAltHash) + 3 * 8 * 256];
  CuckooAltHash *c = new (buf) CuckooAltHash(ar);
  for (size_t i = a->lo; i < a->hi; i++) {
    uint64_t k, k2;
    if (a->keys != NULL) {
      k = a->s1; k2 = a->s2;
      kv_hash_meow128(a->keys + i * a->len, a->len, &k, &k2);
      k &= ~((uint64_t) 1 << 63);
      if (k <= 1) k = 2;
      a->hashes[2 * i] = k; a->hashes[2 * i + 1] = k2;
    } else {
      k = a->hashes[2 * i]; k2 = a->hashes[2 * i + 1];
    }
    kctx.set_hash(k, k2);
    c->calc_hash(kctx, kctx.key, kctx.key2, kctx.start);
    for (uint8_t j = 0; j < ar; j++) a->pos[i * ar + j] = c->pos[j];
  }
  return NULL;
}
}  // namespace

extern "C" double ref_cuckoo_bench(uint64_t ht_size, uint64_t mask, uint64_t frac, uint32_t shift,
                                   uint16_t buckets, uint8_t arity, const uint8_t *keys, size_t len, size_t n,
                                   uint64_t s1, uint64_t s2, uint64_t *hashes, uint64_t *pos, int threads) {
  const size_t hdr_bytes = KV_HT_HDR_SIZE + KV_HT_CTX_SIZE + KV_HT_STATS_SIZE;
  HashTab *ht = (HashTab *) ::aligned_alloc(4096, hdr_bytes);
  if (ht == NULL || arity < 2 || buckets < 2) return -1.0;
  ::memset((void *) ht, 0, hdr_bytes);
  ht->hdr.ht_size = ht_size;
  ht->hdr.ht_mod_mask = mask;
  ht->hdr.ht_mod_fraction = frac;
  ht->hdr.ht_mod_shift = (uint8_t) shift;
  ht->hdr.cuckoo_buckets = buckets;
  ht->hdr.cuckoo_arity = arity;
  ht->hdr.hash_entry_size = 64;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  BenchArg args[256];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; t++) {
    args[t] = BenchArg{ht, keys, len, n * t / threads, n * (t + 1) / threads, s1, s2, hashes, pos};
    pthread_create(&tid[t], NULL, bench_thr, &args[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  ::free(ht);
  return (double) (t1.tv_sec - t0.tv_sec) + 1e-9 * (double) (t1.tv_nsec - t0.tv_nsec);
}

/* f3 golden vectors: ctest.c's ingest (ctest.c:202-233) through the
 * reference's own key-fragment functions.  Tokens (maximal runs of bytes
 * other than ' ', '\n', '\t', kept when shorter than max_token) are packed
 * with kv_make_key_frag + kv_set_key_frag_string (key_ctx.cpp:1737-1772)
 * into `frag_buf` (record offsets -> rec_offs) and hashed with
 * kv_hash_key_frag (key_ctx.cpp:1774-1783) against a malloc'd HashTab whose
 * db-0 seed is returned in seed_out.  Returns the token count or -1. */
extern "C" long ref_ctest_frags(const char *text, size_t n, uint32_t max_token, uint8_t *frag_buf, size_t frag_cap,
                                uint64_t *rec_offs, uint64_t *hashes, size_t max_tok, uint64_t *seed_out) {
  HashTabGeom g;
  memset(&g, 0, sizeof(g));
  g.map_size = 8 << 20;
  g.hash_entry_size = 64;
  g.hash_value_ratio = 1.0f;
  g.cuckoo_buckets = 4;
  g.cuckoo_arity = 2;
  HashTab *ht = HashTab::alloc_map(g);
  if (ht == NULL) return -1;
  HashSeed hs;
  ht->hdr.get_hash_seed(0, hs);
  seed_out[0] = hs.hash1;
  seed_out[1] = hs.hash2;
  uint8_t *in = frag_buf, *end = frag_buf + frag_cap;
  long cnt = 0;
  size_t i = 0;
  for (size_t p = 0;; p++) {
    const bool tok = p < n && !(text[p] == ' ' || text[p] == '\n' || text[p] == '\t');
    if (tok) {
      i++;
      continue;
    }
    if (i > 0 && i < max_token) {
      void *out = NULL;
      kv_key_frag_t *frag = kv_make_key_frag((uint16_t)(i + 1), (size_t)(end - in), in, &out);
      if (frag == NULL || (size_t)cnt >= max_tok) { ::free(ht); return -1; }
      kv_set_key_frag_string(frag, &text[p - i], (uint16_t)i);
      rec_offs[cnt] = (uint64_t)((uint8_t *)frag - frag_buf);
      kv_hash_key_frag((kv_hash_tab_t *)ht, frag, &hashes[2 * cnt], &hashes[2 * cnt + 1]);
      cnt++;
      in = (uint8_t *)out;
    }
    i = 0;
    if (p >= n) break;
  }
  ::free(ht);
  return cnt;
}

/* f2 golden vectors: the reference's kv_ht_radix_sort (radix_sort.cpp:31-41)
 * on a malloc'd HashTab of the given geometry; items carry input indices.
 * Then ctest.c:96-104's adjacent-duplicate marking on that order (dup_out
 * = count; the zeroed hashes are written to out_h). */
#include <raikv/radix_sort.h>
extern "C" int ref_ht_sort(uint64_t map_size, uint32_t entry_size, float ratio, uint16_t buckets, uint8_t arity,
                           const uint64_t *h, size_t n, uint64_t *out_h, uint64_t *out_item, uint64_t *dup_out) {
  HashTabGeom g;
  memset(&g, 0, sizeof(g));
  g.map_size = map_size;
  g.hash_entry_size = entry_size;
  g.hash_value_ratio = ratio;
  g.cuckoo_buckets = buckets;
  g.cuckoo_arity = arity;
  HashTab *ht = HashTab::alloc_map(g);
  if (ht == NULL) return -1;
  kv_ht_sort_t *ar = (kv_ht_sort_t *) ::malloc(sizeof(kv_ht_sort_t) * (n ? n : 1));
  for (size_t i = 0; i < n; i++) {
    ar[i].key = h[2 * i];
    ar[i].key2 = h[2 * i + 1];
    ar[i].item = (void *) (uintptr_t) i;
  }
  kv_ht_radix_sort(ar, (uint32_t) n, (kv_hash_tab_t *) ht);
  uint64_t dups = 0;
  for (size_t k = 1; k < n; k++)
    if (ar[k - 1].key == ar[k].key && ar[k - 1].key2 == ar[k].key2) {
      ar[k - 1].key = 0;
      dups++;
    }
  for (size_t i = 0; i < n; i++) {
    out_h[2 * i] = ar[i].key;
    out_h[2 * i + 1] = ar[i].key2;
    out_item[i] = (uint64_t) (uintptr_t) ar[i].item;
  }
  *dup_out = dups;
  ::free(ar);
  ::free(ht);
  return 0;
}

/* f2 CPU baseline: the reference's kv_ht_radix_sort (radix_sort.cpp:31-41)
 * + ctest.c:96-104's adjacent-duplicate marking over n (h1, h2) pairs with
 * their indices as items, against a header that carries only the table
 * geometry (as ref_cuckoo_bench).  The reference sort is single-threaded;
 * the array fill is not timed.  Returns seconds (or -1); *dup_out = count. */
extern "C" double ref_ht_sort_bench(uint64_t ht_size, uint64_t mask, uint64_t frac, uint32_t shift,
                                    const uint64_t *h, size_t n, uint64_t *dup_out) {
  const size_t hdr_bytes = KV_HT_HDR_SIZE + KV_HT_CTX_SIZE + KV_HT_STATS_SIZE;
  HashTab *ht = (HashTab *) ::aligned_alloc(4096, hdr_bytes);
  kv_ht_sort_t *ar = (kv_ht_sort_t *) ::malloc(sizeof(kv_ht_sort_t) * (n ? n : 1));
  if (ht == NULL || ar == NULL) { ::free(ht); ::free(ar); return -1.0; }
  ::memset((void *) ht, 0, hdr_bytes);
  ht->hdr.ht_size = ht_size;
  ht->hdr.ht_mod_mask = mask;
  ht->hdr.ht_mod_fraction = frac;
  ht->hdr.ht_mod_shift = (uint8_t) shift;
  for (size_t i = 0; i < n; i++) {
    ar[i].key = h[2 * i];
    ar[i].key2 = h[2 * i + 1];
    ar[i].item = (void *) (uintptr_t) i;
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  kv_ht_radix_sort(ar, (uint32_t) n, (kv_hash_tab_t *) ht);
  uint64_t dups = 0;
  for (size_t k = 1; k < n; k++)
    if (ar[k - 1].key == ar[k].key && ar[k - 1].key2 == ar[k].key2) {
      ar[k - 1].key = 0;
      dups++;
    }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  *dup_out = dups;
  ::free(ar);
  ::free(ht);
  return (double) (t1.tv_sec - t0.tv_sec) + 1e-9 * (double) (t1.tv_nsec - t0.tv_nsec);
}
