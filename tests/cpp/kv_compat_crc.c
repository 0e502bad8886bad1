/* kv_compat_crc.c -- TEST: a plain C program that includes only
 * include/kvh_kv.h and links only libkvh_kv.so (as a raikv build that drops
 * src/key_hash.c would), calling every CRC32C symbol of
 * include/raikv/key_hash.h:8-20 against the reference's own outputs
 * (tests/golden/crc32c.npz, unpacked by tests/test_gpu_crc.py into the flat
 * little-endian file named by argv[1]).  Prints one line per family and
 * exits 0 only when every value matches. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "kvh_kv.h"

static unsigned char *g_buf;
static size_t g_len, g_pos;

static void *take(size_t n) {
  if (g_pos + n > g_len) { fprintf(stderr, "short input\n"); exit(2); }
  void *p = g_buf + g_pos;
  g_pos += n;
  return p;
}
static uint32_t u32(void) { uint32_t v; memcpy(&v, take(4), 4); return v; }

int main(int argc, char **argv) {
  if (argc != 2) { fprintf(stderr, "usage: %s crc_cases.bin\n", argv[0]); return 2; }
  FILE *f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 2; }
  fseek(f, 0, SEEK_END);
  g_len = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  g_buf = (unsigned char *)malloc(g_len);
  if (fread(g_buf, 1, g_len, f) != g_len) { perror("read"); return 2; }
  fclose(f);
  long bad = 0, checked = 0;

  /* every length 0..maxL under each seed: kv_crc_c (key_hash.c:39-63) */
  const uint32_t nl = u32(), maxl = u32(), ns = u32();
  const unsigned char *lk = (const unsigned char *)take((size_t)nl * maxl);
  uint32_t *ls = (uint32_t *)malloc(4 * ns), *lo = (uint32_t *)malloc(4 * (size_t)nl * ns);
  memcpy(ls, take(4 * ns), 4 * ns);
  memcpy(lo, take(4 * (size_t)nl * ns), 4 * (size_t)nl * ns);
  for (uint32_t L = 0; L < nl; L++)
    for (uint32_t s = 0; s < ns; s++, checked++)
      if (kv_crc_c(lk + (size_t)L * maxl, L, ls[s]) != lo[(size_t)L * ns + s]) bad++;
  printf("kv_crc_c: %u lengths x %u seeds, %ld bad\n", nl, ns, bad);

  /* variable-length keys with per-key seeds: kv_crc_c_array (:149-166),
   * kv_crc_c_2_diff (:65-84), kv_crc_c_4_diff (:86-120) */
  const uint32_t nv = u32();
  uint64_t *vo = (uint64_t *)malloc(8 * ((size_t)nv + 1));
  uint32_t *vs = (uint32_t *)malloc(4 * (size_t)nv), *vw = (uint32_t *)malloc(4 * (size_t)nv);
  memcpy(vo, take(8 * ((size_t)nv + 1)), 8 * ((size_t)nv + 1));
  memcpy(vs, take(4 * (size_t)nv), 4 * (size_t)nv);
  memcpy(vw, take(4 * (size_t)nv), 4 * (size_t)nv);
  uint64_t kb;
  memcpy(&kb, take(8), 8);
  const unsigned char *vk = (const unsigned char *)take(kb);
  const void **pp = (const void **)malloc(sizeof(void *) * nv);
  size_t *psz = (size_t *)malloc(sizeof(size_t) * nv);
  uint32_t *io = (uint32_t *)malloc(4 * (size_t)nv);
  for (uint32_t i = 0; i < nv; i++) {
    pp[i] = vk + vo[i];
    psz[i] = (size_t)(vo[i + 1] - vo[i]);
    io[i] = vs[i];
  }
  long b0 = bad;
  kv_crc_c_array(pp, psz, io, nv);
  for (uint32_t i = 0; i < nv; i++, checked++) if (io[i] != vw[i]) bad++;
  printf("kv_crc_c_array: %u keys, %ld bad\n", nv, bad - b0);
  b0 = bad;
  for (uint32_t i = 0; i + 1 < nv; i += 2) {
    uint32_t a = vs[i], b = vs[i + 1];
    kv_crc_c_2_diff(pp[i], psz[i], &a, pp[i + 1], psz[i + 1], &b);
    bad += (a != vw[i]) + (b != vw[i + 1]);
    checked += 2;
  }
  for (uint32_t i = 0; i + 3 < nv; i += 4) {
    uint32_t a = vs[i], b = vs[i + 1], c = vs[i + 2], d = vs[i + 3];
    kv_crc_c_4_diff(pp[i], psz[i], &a, pp[i + 1], psz[i + 1], &b, pp[i + 2], psz[i + 2], &c, pp[i + 3], psz[i + 3],
                    &d);
    bad += (a != vw[i]) + (b != vw[i + 1]) + (c != vw[i + 2]) + (d != vw[i + 3]);
    checked += 4;
  }
  printf("kv_crc_c_2_diff / kv_crc_c_4_diff: %ld bad\n", bad - b0);

  /* prefixes of one buffer: kv_crc_c_key_array (:168-179) */
  const uint32_t np = u32(), pbl = u32();
  const unsigned char *pb = (const unsigned char *)take(pbl);
  size_t *pl = (size_t *)malloc(sizeof(size_t) * np);
  uint32_t *pio = (uint32_t *)malloc(4 * (size_t)np), *pw = (uint32_t *)malloc(4 * (size_t)np);
  for (uint32_t i = 0; i < np; i++) pl[i] = u32();
  memcpy(pio, take(4 * (size_t)np), 4 * (size_t)np);
  memcpy(pw, take(4 * (size_t)np), 4 * (size_t)np);
  b0 = bad;
  kv_crc_c_key_array(pb, pl, pio, np);
  for (uint32_t i = 0; i < np; i++, checked++) if (pio[i] != pw[i]) bad++;
  printf("kv_crc_c_key_array: %u prefixes, %ld bad\n", np, bad - b0);

  /* kv_hash_uint / kv_hash_uint2 (:27-37) */
  const uint32_t nu = u32();
  uint32_t *ui = (uint32_t *)malloc(4 * (size_t)nu), *uo = (uint32_t *)malloc(4 * (size_t)nu),
           *u2 = (uint32_t *)malloc(4 * (size_t)nu);
  memcpy(ui, take(4 * (size_t)nu), 4 * (size_t)nu);
  memcpy(uo, take(4 * (size_t)nu), 4 * (size_t)nu);
  memcpy(u2, take(4 * (size_t)nu), 4 * (size_t)nu);
  b0 = bad;
  for (uint32_t i = 0; i < nu; i++, checked += 2) {
    bad += kv_hash_uint(ui[i]) != uo[i];
    bad += kv_hash_uint2(ui[i], ui[nu - 1 - i]) != u2[i];
  }
  printf("kv_hash_uint / kv_hash_uint2: %u inputs, %ld bad\n", nu, bad - b0);
  printf("checked %ld, bad %ld\n", checked, bad);
  return bad ? 1 : 0;
}
