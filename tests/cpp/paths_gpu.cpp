// tests/cpp/paths_gpu.cpp -- the C++ host API for the calls either side of
// the hash (include/raikv_amd/key_hash.hpp: ht_geom, hash_fixed_positions,
// ht_positions, ht_sort, ingest_text, crc_var) on the GPU, each checked
// against an independent path through the C-ABI or the host drop-ins.
// Exit status 0 = all checks passed.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <random>
#include <vector>
#include "raikv_amd/key_hash.hpp"

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fails++; printf("FAIL %s:%d ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); } } while (0)

template <class T> T* dalloc(size_t n) {
  void* p = nullptr;
  if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) { printf("hipMalloc failed\n"); exit(2); }
  return (T*)p;
}
template <class T> void h2d(T* d, const std::vector<T>& h) { (void)hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice); }
template <class T> std::vector<T> d2h(const T* d, size_t n) {
  std::vector<T> h(n);
  (void)hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost);
  return h;
}

int main() {
  std::mt19937_64 rng(7);
  const kvh::HashSeed hs{0xa8e0bcc94d1855f5ull, 0xad3bec1e8de4a1a3ull};
  const kvh_ht_geom_t g = kvh::ht_geom(1ull << 30, 64, 1.0f, 4, 4);
  const uint32_t pk = kvh::positions_per_key(g);
  CHECK(pk >= 1, "positions per key %u", pk);

  // f1: fused hash + positions == hash, then positions
  const size_t n = 100003, L = 16;
  std::vector<uint8_t> keys(n * L);
  for (auto& b : keys) b = (uint8_t)rng();
  uint8_t* dk = dalloc<uint8_t>(keys.size());
  h2d(dk, keys);
  uint64_t *h1 = dalloc<uint64_t>(2 * n), *h2 = dalloc<uint64_t>(2 * n);
  uint64_t *p1 = dalloc<uint64_t>(pk * n), *p2 = dalloc<uint64_t>(pk * n);
  kvh::hash_fixed_positions(dk, L, n, hs, g, h1, p1);
  kvh::hash_fixed(dk, L, n, hs, h2, true);
  kvh::ht_positions(h2, n, g, p2);
  (void)hipDeviceSynchronize();
  CHECK(d2h(h1, 2 * n) == d2h(h2, 2 * n), "fused hashes differ");
  CHECK(d2h(p1, pk * n) == d2h(p2, pk * n), "fused positions differ");

  // host-memory pipelines (kvh::hash_*_host, one device and a repeated
  // device list) == the device-resident kernels
  {
    std::vector<uint64_t> hh(2 * n), hm(2 * n);
    kvh::hash_fixed_host(keys.data(), L, n, hs, hh.data(), true);
    kvh::hash_fixed_host(keys.data(), L, n, hs, hm.data(), true, {0, 0, 0});
    const std::vector<uint64_t> dh = d2h(h2, 2 * n);
    CHECK(hh == dh, "hash_fixed_host differs from hash_fixed");
    CHECK(hm == dh, "hash_fixed_host over {0,0,0} differs");
    const size_t nv = 50001;
    std::vector<uint64_t> off(nv + 1, 0);
    for (size_t i = 0; i < nv; i++) off[i + 1] = off[i] + 8 + rng() % 249;
    std::vector<uint8_t> vk(off[nv]);
    for (auto& b : vk) b = (uint8_t)rng();
    uint8_t* dvk = dalloc<uint8_t>(vk.size());
    uint64_t* doff = dalloc<uint64_t>(nv + 1);
    uint64_t* dvh = dalloc<uint64_t>(2 * nv);
    h2d(dvk, vk);
    h2d(doff, off);
    kvh::hash_var(dvk, doff, nv, hs, dvh, true);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> vh(2 * nv), vm(2 * nv);
    kvh::hash_var_host(vk.data(), off.data(), nv, hs, vh.data(), true);
    kvh::hash_var_host(vk.data(), off.data(), nv, hs, vm.data(), true, {0, 0});
    const std::vector<uint64_t> want = d2h(dvh, 2 * nv);
    CHECK(vh == want, "hash_var_host differs from hash_var");
    CHECK(vm == want, "hash_var_host over {0,0} differs");
    (void)hipFree(dvk); (void)hipFree(doff); (void)hipFree(dvh);
  }

  // f2: table order by home slot, duplicates adjacent and counted
  std::vector<uint64_t> hh = d2h(h2, 2 * n);
  for (size_t i = 0; i < 100; i++) {  // 100 duplicated pairs
    const size_t a = rng() % n, b = rng() % n;
    hh[2 * a] = hh[2 * b];
    hh[2 * a + 1] = hh[2 * b + 1];
  }
  h2d(h1, hh);
  uint64_t *so = dalloc<uint64_t>(2 * n), *io = dalloc<uint64_t>(n), *dc = dalloc<uint64_t>(1);
  kvh::Scratch sc;
  kvh::ht_sort(h1, nullptr, n, g, so, io, dc, false, sc);
  (void)hipDeviceSynchronize();
  std::vector<uint64_t> sh = d2h(so, 2 * n), si = d2h(io, n);
  std::vector<uint64_t> home(n);
  kvh::ht_positions(so, n, g, p1);
  (void)hipDeviceSynchronize();
  std::vector<uint64_t> ps = d2h(p1, pk * n);
  bool ordered = true, perm = true;
  for (size_t i = 0; i + 1 < n; i++) ordered &= ps[pk * i] <= ps[pk * (i + 1)];
  std::vector<uint64_t> sorted_idx = si;
  std::sort(sorted_idx.begin(), sorted_idx.end());
  for (size_t i = 0; i < n; i++) perm &= sorted_idx[i] == i;
  for (size_t i = 0; i < n && perm; i++) perm &= sh[2 * i] == hh[2 * si[i]] && sh[2 * i + 1] == hh[2 * si[i] + 1];
  CHECK(ordered, "not in home-slot order");
  CHECK(perm, "items are not the permutation of the hashes");
  kvh::ht_sort(h1, nullptr, n, g, so, io, dc, true, sc);
  (void)hipDeviceSynchronize();
  const uint64_t dups = d2h(dc, 1)[0];
  std::vector<std::pair<uint64_t, uint64_t>> pairs(n);
  for (size_t i = 0; i < n; i++) pairs[i] = {hh[2 * i], hh[2 * i + 1]};
  std::sort(pairs.begin(), pairs.end());
  uint64_t want = 0;
  for (size_t i = 0; i + 1 < n; i++) want += pairs[i] == pairs[i + 1];
  CHECK(dups == want, "duplicates %llu, want %llu", (unsigned long long)dups, (unsigned long long)want);
  {  // the exact-order drop-in: three batches in one call == each batch through kvh_ht_radix_sort
    const uint32_t sz[3] = {10000, 5000, 3};
    std::vector<std::vector<kvh_ht_sort_t>> one(3), many(3);
    size_t o = 0;
    for (int b = 0; b < 3; b++) {
      for (uint32_t i = 0; i < sz[b]; i++, o++)
        one[b].push_back({hh[2 * o], hh[2 * o + 1], (void*)(uintptr_t)(o + 1)});
      many[b] = one[b];
      CHECK(kvh_ht_radix_sort(one[b].data(), sz[b], &g) == 0, "kvh_ht_radix_sort");
    }
    kvh_ht_sort_t* ptrs[3] = {many[0].data(), many[1].data(), many[2].data()};
    kvh::ht_radix_sort_batch(ptrs, sz, 3, g);
    bool same = true;
    for (int b = 0; b < 3; b++)
      for (uint32_t i = 0; i < sz[b]; i++)
        same &= one[b][i].key == many[b][i].key && one[b][i].key2 == many[b][i].key2 &&
                one[b][i].item == many[b][i].item;
    CHECK(same, "ht_radix_sort_batch differs from kvh_ht_radix_sort per batch");
  }

  // f3: one-call ingest == tokenize + span hash
  std::string text;
  while (text.size() < 300000) {
    const size_t k = 1 + rng() % 12;
    for (size_t i = 0; i < k; i++) text.push_back((char)('a' + rng() % 26));
    text.push_back(" \n\t"[rng() % 3]);
  }
  uint8_t* dt = dalloc<uint8_t>(text.size());
  (void)hipMemcpy(dt, text.data(), text.size(), hipMemcpyHostToDevice);
  const size_t cap = text.size() / 2 + 1;
  uint64_t *to = dalloc<uint64_t>(cap), *th = dalloc<uint64_t>(2 * cap), *cnt = dalloc<uint64_t>(1);
  uint32_t* tl = dalloc<uint32_t>(cap);
  kvh::ingest_text(dt, text.size(), hs, to, tl, th, cap, cnt, sc);
  (void)hipDeviceSynchronize();
  const uint64_t k = d2h(cnt, 1)[0];
  uint64_t* th2 = dalloc<uint64_t>(2 * cap);
  kvh::check(kvh_meow128_spans(dt, to, tl, k, hs.hash1, hs.hash2, th2, KVH_FIXUP | KVH_NULTERM, nullptr), "spans");
  (void)hipDeviceSynchronize();
  CHECK(k > 1000, "token count %llu", (unsigned long long)k);
  CHECK(d2h(th, 2 * k) == d2h(th2, 2 * k), "ingest hashes differ from the span hash");

  // f4: variable-length CRC32C == the host drop-in kv_crc_c
  std::vector<uint64_t> offs(1001);
  for (size_t i = 1; i <= 1000; i++) offs[i] = offs[i - 1] + (rng() % 300);
  std::vector<uint8_t> ck(offs[1000] + 1);
  for (auto& b : ck) b = (uint8_t)rng();
  uint8_t* dck = dalloc<uint8_t>(ck.size());
  uint64_t* dof = dalloc<uint64_t>(offs.size());
  uint32_t* dcrc = dalloc<uint32_t>(1000);
  h2d(dck, ck);
  h2d(dof, offs);
  kvh::crc_var(dck, dof, 1000, nullptr, 0x1234u, dcrc);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> crc = d2h(dcrc, 1000);
  for (size_t i = 0; i < 1000; i += 37)
    CHECK(crc[i] == kvh_crc_c(ck.data() + offs[i], offs[i + 1] - offs[i], 0x1234u), "crc %zu", i);

  printf("paths_gpu: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
