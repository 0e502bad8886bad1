// tests/cpp/hash_test_gpu.cpp -- the reference's hash_test self-consistency
// checks (/root/reference/test/hash_test.cpp:319-442) re-expressed against
// the GPU engine through the C++ mirror (include/raikv_amd/key_hash.hpp) and
// the C-ABI (include/kvh.h).  Known answers come from the README
// (README.md:130-137) and tests/golden (produced by the reference).
//
// Exit status 0 = all checks passed.  Prints one line per failed check.
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <inttypes.h>
#include <vector>
#include <hip/hip_runtime_api.h>
#include "raikv_amd/key_hash.hpp"

static int failures = 0, checks = 0;
#define EXPECT(c, ...) do { checks++; if (!(c)) { failures++; printf("FAIL: " __VA_ARGS__); printf("\n"); } } while (0)
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("FAIL: %s -> hip error %d\n", #x, (int)e_); exit(2); } } while (0)

int main() {
  using namespace kvh;
  // ---- README KAT: "hello\0" with the RAIKV_STATIC_RANDOM db-0 seed
  {
    KeyBuf kb("hello");
    HashSeed hs{0xa8e0bcc94d1855f5ULL, 0xad3bec1e8de4a1a3ULL};
    uint64_t h1 = hs.hash1, h2 = hs.hash2;
    check(kvh_hash_meow128(kb.u.buf, kb.keylen, &h1, &h2), "meow128");
    EXPECT(h1 == 0x2aa73a1eeb0b2d45ULL && h2 == 0xfd102121185ce157ULL, "README KAT %016" PRIx64 ":%016" PRIx64, h1, h2);
    uint64_t k1, k2;
    hs.hash(kb, k1, k2);  // KeyFragment::hash + fixup: bit 63 already clear here
    EXPECT(k1 == (0x2aa73a1eeb0b2d45ULL & ~ZOMBIE64) && k2 == 0xfd102121185ce157ULL, "HashSeed::hash");
  }
  // ---- cross-variant block (hash_test.cpp:319-403)
  const char* ar[] = {"security is for the messaging la", "authenticate the publisher to th",
                      "subscribers must be able to trus", "uniquely serialized, and authent"};
  uint64_t x[8], y[8], d[8], e[8], z[8], u[8], v[8], w[16];
  for (int n = 0; n < 8; n += 2) {
    x[n] = y[n] = d[n] = e[n] = z[n] = u[n] = v[n] = 1010;
    x[n + 1] = y[n + 1] = d[n + 1] = e[n + 1] = z[n + 1] = u[n + 1] = v[n + 1] = 2020;
  }
  for (int n = 0; n < 16; n += 2) { w[n] = 1010; w[n + 1] = 2020; }
  const size_t len = strlen(ar[0]);
  for (int i = 0; i < 4; i++) check(kvh_hash_meow128(ar[i], len, &x[2 * i], &x[2 * i + 1]), "meow128");
  check(kvh_hash_meow128_2_same_length(ar[0], ar[1], len, y), "2same");
  check(kvh_hash_meow128_2_same_length(ar[2], ar[3], len, &y[4]), "2same");
  check(kvh_hash_meow128_2_diff_length(ar[0], len, ar[1], len, d), "2diff");
  check(kvh_hash_meow128_2_diff_length(ar[2], len, ar[3], len, &d[4]), "2diff");
  check(kvh_hash_meow128_4_same_length(ar[0], ar[1], ar[2], ar[3], len, z), "4same");
  check(kvh_hash_meow128_4_diff_length(ar[0], len, ar[1], len, ar[2], len, ar[3], len, e), "4diff");
  for (int i = 0; i < 4; i++) {
    kvh_meow_ctx_t m; kvh_meow_block_t b;
    check(kvh_meow128_init(&m, &b, u[2 * i], u[2 * i + 1], len), "init");
    check(kvh_meow128_update(&m, &b, ar[i], len), "update");
    check(kvh_meow128_final(&m, &b, &u[2 * i], &u[2 * i + 1]), "final");
    const size_t h = len / 2;
    kvh_meow_vec_t vec[2] = {{ar[i], h}, {ar[i] + h, len - h}};
    check(kvh_hash_meow128_vec(vec, 2, &v[2 * i], &v[2 * i + 1]), "vec");
  }
  const void* par[8] = {ar[0], ar[1], ar[2], ar[3], ar[0], ar[1], ar[2], ar[3]};
  check(kvh_hash_meow128_8_same_length_a(par, len, w), "8same");
  for (int n = 0; n < 8; n++) {
    EXPECT(x[n] == y[n], "2 same failed %d", n);
    EXPECT(x[n] == d[n], "2 diff failed %d", n);
    EXPECT(x[n] == z[n], "4 same failed %d", n);
    EXPECT(x[n] == e[n], "4 diff failed %d", n);
    EXPECT(x[n] == u[n], "upd same failed %d", n);
    EXPECT(x[n] == v[n], "vec same failed %d", n);
    EXPECT(x[n] == w[n], "lrg same failed %d", n);
    EXPECT(x[n] == w[n + 8], "lrg same failed 1 %d", n);
  }
  // golden value of the first string (tests/golden/reference_vectors.json)
  EXPECT(x[0] == 10896601673284352656ULL && x[1] == 3059145504078390846ULL, "golden string 0");

  // ---- partition tests (hash_test.cpp:404-442) on bytes 0..127, seed (10101,20202)
  char buf[128];
  for (int n = 0; n < 128; n++) buf[n] = (char)n;
  for (size_t n = 0; n < 128; n++) {
    uint64_t a[2] = {10101, 20202}, b[2] = {10101, 20202}, dd[4] = {10101, 20202, 10101, 20202};
    check(kvh_hash_meow128(buf, n, &a[0], &a[1]), "p2");
    check(kvh_hash_meow128(&buf[n], 128 - n, &b[0], &b[1]), "p2");
    check(kvh_hash_meow128_2_diff_length(&buf[0], n, &buf[n], 128 - n, dd), "p2");
    EXPECT(a[0] == dd[0] && a[1] == dd[1] && b[0] == dd[2] && b[1] == dd[3], "part2 diff %zu", n);
  }
  // part4: all n<=m<=o<128 as ONE device batch through the folded kernel,
  // compared with the straight-line kernel over the same segments.
  {
    std::vector<uint64_t> offs;
    for (size_t n = 0; n < 128; n++)
      for (size_t m = n; m < 128; m++)
        for (size_t o = m; o < 128; o++) {
          // 4 keys as offsets into a repeated copy of buf: use absolute segments
          offs.push_back(n); offs.push_back(m); offs.push_back(o);
        }
    const size_t T = offs.size() / 3, nk = 4 * T;
    // lay each quadruple's 128 bytes out contiguously so segment ends == next start
    std::vector<uint8_t> keys(T * 128);
    std::vector<uint64_t> koff(nk + 1), seeds(2 * nk);
    for (size_t t = 0; t < T; t++) {
      memcpy(&keys[t * 128], buf, 128);
      const uint64_t base = t * 128;
      koff[4 * t + 0] = base;
      koff[4 * t + 1] = base + offs[3 * t];
      koff[4 * t + 2] = base + offs[3 * t + 1];
      koff[4 * t + 3] = base + offs[3 * t + 2];
    }
    koff[nk] = T * 128;
    for (size_t i = 0; i < nk; i++) { seeds[2 * i] = 10101; seeds[2 * i + 1] = 20202; }
    void *dk, *doff, *dseed, *do1, *do2;
    HC(hipMalloc(&dk, keys.size())); HC(hipMalloc(&doff, 8 * koff.size())); HC(hipMalloc(&dseed, 8 * seeds.size()));
    HC(hipMalloc(&do1, 16 * nk)); HC(hipMalloc(&do2, 16 * nk));
    HC(hipMemcpy(dk, keys.data(), keys.size(), hipMemcpyHostToDevice));
    HC(hipMemcpy(doff, koff.data(), 8 * koff.size(), hipMemcpyHostToDevice));
    HC(hipMemcpy(dseed, seeds.data(), 8 * seeds.size(), hipMemcpyHostToDevice));
    check(kvh_meow128_var(dk, (const uint64_t*)doff, nk, 10101, 20202, (uint64_t*)do1, 0, nullptr), "var");
    check(kvh_meow128_var_seeded(dk, (const uint64_t*)doff, nk, (const uint64_t*)dseed, (uint64_t*)do2, 0,
                                 nullptr), "seeded");
    std::vector<uint64_t> r1(2 * nk), r2(2 * nk);
    HC(hipMemcpy(r1.data(), do1, 16 * nk, hipMemcpyDeviceToHost));
    HC(hipMemcpy(r2.data(), do2, 16 * nk, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < 2 * nk; i++) bad += r1[i] != r2[i];
    EXPECT(bad == 0, "part4 folded vs literal: %zu mismatching words of %zu", bad, 2 * nk);
    // and against 4-diff drop-ins for a sample of triples
    for (size_t t = 0; t < T; t += 997) {
      uint64_t dd[8] = {10101, 20202, 10101, 20202, 10101, 20202, 10101, 20202};
      const size_t n = offs[3 * t], m = offs[3 * t + 1], o = offs[3 * t + 2];
      check(kvh_hash_meow128_4_diff_length(&buf[0], n, &buf[n], m - n, &buf[m], o - m, &buf[o], 128 - o, dd),
            "4diff");
      EXPECT(memcmp(dd, &r1[8 * t], 64) == 0, "part4 diff %zu %zu %zu", n, m, o);
    }
    HC(hipFree(dk)); HC(hipFree(doff)); HC(hipFree(dseed)); HC(hipFree(do1)); HC(hipFree(do2));
  }
  printf("hash_test_gpu: %d checks, %d failures\n", checks, failures);
  return failures ? 1 : 0;
}
