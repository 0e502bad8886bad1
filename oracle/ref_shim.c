/*
 * oracle/ref_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin batch drivers compiled TOGETHER WITH the unmodified reference
 * /root/reference/src/key_hash.c (see oracle/Makefile) into
 * oracle/_ref/libkvref.so.  They only loop over the reference's own entry
 * points so that Python (ctypes) can produce golden vectors and time the
 * reference CPU path on the GPU box's host cores.  No reference source is
 * copied here; the reference functions are declared from its header.
 *
 *   kv_hash_meow128                       key_hash.c:1413-1429
 *   kv_hash_meow128_4_same_length_4_seed  key_hash.c:1891-1937
 *   hash_test IntContent / KeyBufAligned  test/hash_test.cpp:54-68, :447-457,
 *                                         include/raikv/key_buf.h:69-110
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>
#include <time.h>
#include <raikv/key_hash.h>

void ref_batch_fixed(const uint8_t *keys, size_t len, size_t n, uint64_t s1,
                     uint64_t s2, uint64_t *out)
{
  for (size_t i = 0; i < n; i++) {
    uint64_t h1 = s1, h2 = s2;
    kv_hash_meow128(keys + i * len, len, &h1, &h2);
    out[2 * i] = h1;
    out[2 * i + 1] = h2;
  }
}

void ref_batch_var(const uint8_t *keys, const uint64_t *offs, size_t n,
                   uint64_t s1, uint64_t s2, uint64_t *out)
{
  for (size_t i = 0; i < n; i++) {
    uint64_t h1 = s1, h2 = s2;
    kv_hash_meow128(keys + offs[i], (size_t)(offs[i + 1] - offs[i]), &h1, &h2);
    out[2 * i] = h1;
    out[2 * i + 1] = h2;
  }
}

/* arity-4 multi-seed via the reference's own 4-seed entry point with the
 * same key in all four slots */
void ref_batch_4seed(const uint8_t *keys, size_t len, size_t n,
                     const uint64_t *seeds, uint64_t *out)
{
  for (size_t i = 0; i < n; i++) {
    uint64_t *x = out + 8 * i;
    const uint8_t *p = keys + i * len;
    memcpy(x, seeds, 8 * sizeof(uint64_t));
    kv_hash_meow128_4_same_length_4_seed(p, p, p, p, len, x);
  }
}

/* ---- multi-threaded CPU baselines (the reference's own entry points) ----
 * kind 0: packed fixed-length keys, kv_hash_meow128 per key;
 * kind 1: packed keys + u64 offsets (C2 shape), kv_hash_meow128 per key;
 * kind 2: packed fixed-length keys, kv_hash_meow128_4_same_length_4_seed
 *         with the key in all four slots (C3 shape), out 8 words per key. */
typedef struct {
  int kind;
  const uint8_t *keys; const uint64_t *offs; size_t len, lo, hi;
  uint64_t s1, s2; const uint64_t *seeds; uint64_t *out;
} ref_job;

static void *ref_worker(void *arg)
{
  ref_job *j = (ref_job *)arg;
  for (size_t i = j->lo; i < j->hi; i++) {
    if (j->kind == 2) {
      uint64_t *x = j->out + 8 * i;
      const uint8_t *p = j->keys + i * j->len;
      memcpy(x, j->seeds, 8 * sizeof(uint64_t));
      kv_hash_meow128_4_same_length_4_seed(p, p, p, p, j->len, x);
      continue;
    }
    uint64_t h1 = j->s1, h2 = j->s2;
    if (j->kind == 1)
      kv_hash_meow128(j->keys + j->offs[i], (size_t)(j->offs[i + 1] - j->offs[i]), &h1, &h2);
    else
      kv_hash_meow128(j->keys + i * j->len, j->len, &h1, &h2);
    j->out[2 * i] = h1;
    j->out[2 * i + 1] = h2;
  }
  return NULL;
}

static double ref_bench(int kind, const uint8_t *keys, const uint64_t *offs, size_t len, size_t n,
                        uint64_t s1, uint64_t s2, const uint64_t *seeds, uint64_t *out, int threads)
{
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  ref_job job[256];
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int t = 0; t < threads; t++) {
    job[t].kind = kind; job[t].keys = keys; job[t].offs = offs; job[t].len = len;
    job[t].s1 = s1; job[t].s2 = s2; job[t].seeds = seeds; job[t].out = out;
    job[t].lo = n * (size_t)t / (size_t)threads;
    job[t].hi = n * (size_t)(t + 1) / (size_t)threads;
    pthread_create(&tid[t], NULL, ref_worker, &job[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* returns elapsed seconds (monotonic) for hashing n keys on `threads`
 * POSIX threads */
double ref_bench_fixed(const uint8_t *keys, size_t len, size_t n, uint64_t s1,
                       uint64_t s2, uint64_t *out, int threads)
{
  return ref_bench(0, keys, NULL, len, n, s1, s2, NULL, out, threads);
}

double ref_bench_var(const uint8_t *keys, const uint64_t *offs, size_t n, uint64_t s1,
                     uint64_t s2, uint64_t *out, int threads)
{
  return ref_bench(1, keys, offs, 0, n, s1, s2, NULL, out, threads);
}

double ref_bench_4seed(const uint8_t *keys, size_t len, size_t n, const uint64_t *seeds,
                       uint64_t *out, int threads)
{
  return ref_bench(2, keys, NULL, len, n, 0, 0, seeds, out, threads);
}

/* hash_test "int meow <keylen>" protocol (test/hash_test.cpp:447-460,
 * :730-737): keycount keys in a 134-byte-stride KeyBufAligned-shaped array,
 * IntContent counters starting at `counter0`, `calls` timed calls with seeds
 * (0,0) cycling j = (j+1) & (keycount-1).  Returns ns per hash. */
double ref_hash_test_int(size_t keycount, uint16_t keylen, uint64_t counter0,
                         uint64_t calls)
{
  const size_t stride = 134, buf_off = 8; /* pad[3] u16 + keylen u16 */
  uint8_t *arr = (uint8_t *)calloc(keycount, stride);
  if (!arr) return -1.0;
  uint64_t counter = counter0;
  for (size_t i = 0; i < keycount; i++) {
    uint8_t *kb = arr + i * stride;
    memcpy(kb + 6, &keylen, 2);
    uint8_t j = 0;
    do {
      memcpy(kb + buf_off + j, &counter, 8);
      counter++;
      j += 8;
    } while (j < keylen);
  }
  struct timespec a, b;
  volatile uint64_t sink = 0;
  size_t j = 0;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (uint64_t i = 0; i < calls; i++) {
    uint64_t h1 = 0, h2 = 0;
    kv_hash_meow128(arr + j * stride + buf_off, keylen, &h1, &h2);
    sink += h1;
    j = (j + 1) & (keycount - 1);
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  free(arr);
  (void)sink;
  double s = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  return s / (double)calls * 1e9;
}
