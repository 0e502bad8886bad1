// raikv_amd/key_hash.hpp -- C++ host mirror of raikv's key-fragment hashing
// API over the C-ABI in kvh.h.  Same names and argument meaning as the
// reference (/root/reference/include/raikv/hash_entry.h:56-112,
// key_buf.h:14-110, shm_ht.h:333-351) so existing call sites port by
// changing the namespace; every hash executes on the GPU.
//
// Error behaviour: the reference functions are void and total; here a
// device/runtime failure throws kvh::Error (the product has no CPU path to
// fall back to).
#pragma once
#include <stdint.h>
#include <string.h>
#include <stdexcept>
#include <string>
#include <vector>
#include "../kvh.h"

namespace kvh {

struct Error : std::runtime_error {
  int code;
  Error(const char* what, int rc)
      : std::runtime_error(std::string(what) + ": " + kvh_strerror(rc)), code(rc) {}
};

inline void check(int rc, const char* what) {
  if (rc != 0) throw Error(what, rc);
}

// hash_entry.h:46-50
static const uint64_t ZOMBIE64 = (uint64_t)0x80000000 << 32, DROPPED_HASH = 1;
static const size_t KEY_FRAG_SIZE = 6;

// hash_entry.h:28-36 kv_key_frag_t: u16 keylen + bytes (layout-identical)
struct KeyFragment {
  uint16_t keylen;
  union {
    char buf[4];
    struct { uint16_t b1, b2; } x;
  } u;

  // KeyFragment::hash (hash_entry.h:80-86): Meow128 with (seed, seed2) in,
  // hash out, then h1 &= ~ZOMBIE64, h1 <= 1 -> 2.
  void hash(uint64_t& seed, uint64_t& seed2) const {
    const uint64_t s[2] = {seed, seed2};
    check(kvh_hash_key_frag(s, reinterpret_cast<const kvh_key_frag_t*>(this), &seed, &seed2),
          "KeyFragment::hash");
  }
  // hash_entry.h:87-96: two keys, one seed in seed[0..1], out seed[0..3]
  static void hash2(KeyFragment& kb, KeyFragment& kb2, uint64_t* seed) {
    const kvh_key_frag_t* f[2] = {reinterpret_cast<const kvh_key_frag_t*>(&kb),
                                  reinterpret_cast<const kvh_key_frag_t*>(&kb2)};
    const uint64_t s[2] = {seed[0], seed[1]};
    check(kvh_hash_key_frags(s, f, 2, seed), "KeyFragment::hash2");
  }
  // hash_entry.h:97-111: four keys
  static void hash4(KeyFragment& kb, KeyFragment& kb2, KeyFragment& kb3, KeyFragment& kb4,
                    uint64_t* seed) {
    const kvh_key_frag_t* f[4] = {
        reinterpret_cast<const kvh_key_frag_t*>(&kb), reinterpret_cast<const kvh_key_frag_t*>(&kb2),
        reinterpret_cast<const kvh_key_frag_t*>(&kb3), reinterpret_cast<const kvh_key_frag_t*>(&kb4)};
    const uint64_t s[2] = {seed[0], seed[1]};
    check(kvh_hash_key_frags(s, f, 4, seed), "KeyFragment::hash4");
  }
};

// key_buf.h:14-60 KeyBufT<N>: a KeyFragment with room for N-2 key bytes
template <uint16_t KEY_SIZE>
struct KeyBufT : public KeyFragment {
  static const uint16_t MAX_BUF_SIZE = KEY_SIZE - 2;
  char morebuf[KEY_SIZE - KEY_FRAG_SIZE];

  KeyBufT() { this->keylen = 0; }
  KeyBufT(const char* s) { this->set_string(s); }
  // includes the trailing NUL, like the reference (key_buf.h:29-31)
  void set_string(const char* s) { this->copy(s, ::strnlen(s, MAX_BUF_SIZE) + 1); }
  template <class T> void set(T arg) { this->copy((const void*)&arg, sizeof(T)); }
  uint16_t copy(const void* p, size_t len) {
    if (len > MAX_BUF_SIZE) len = MAX_BUF_SIZE;
    ::memcpy(this->u.buf, p, len);
    this->keylen = (uint16_t)len;
    return (uint16_t)len;
  }
  void zero(void) { ::memset((void*)this, 0, sizeof(*this)); }
};
typedef KeyBufT<128> KeyBuf;

// shm_ht.h:333-351 HashSeed
struct HashSeed {
  uint64_t hash1, hash2;
  void get(uint64_t& h1, uint64_t& h2) const { h1 = this->hash1; h2 = this->hash2; }
  void hash(KeyFragment& kb, uint64_t& h1, uint64_t& h2) const {
    h1 = this->hash1; h2 = this->hash2;
    kb.hash(h1, h2);
  }
  void hash(KeyFragment& kb, KeyFragment& kb2, uint64_t* h) const {
    h[0] = this->hash1; h[1] = this->hash2;
    KeyFragment::hash2(kb, kb2, h);
  }
  void hash(KeyFragment& kb, KeyFragment& kb2, KeyFragment& kb3, KeyFragment& kb4, uint64_t* h) const {
    h[0] = this->hash1; h[1] = this->hash2;
    KeyFragment::hash4(kb, kb2, kb3, kb4, h);
  }
};

// ---- batched device API (the hot path), C++ shape over kvh.h
// Fixed-length keys packed at stride key_len, device pointers, async on stream.
inline void hash_fixed(const void* keys, uint32_t key_len, size_t n, const HashSeed& hs, uint64_t* out,
                       bool fixup = true, void* stream = nullptr) {
  check(kvh_meow128_fixed(keys, key_len, n, hs.hash1, hs.hash2, out, fixup ? KVH_FIXUP : 0u, stream),
        "kvh::hash_fixed");
}
inline void hash_var(const void* keys, const uint64_t* offsets, size_t n, const HashSeed& hs, uint64_t* out,
                     bool fixup = true, void* stream = nullptr) {
  check(kvh_meow128_var(keys, offsets, n, hs.hash1, hs.hash2, out, fixup ? KVH_FIXUP : 0u, stream),
        "kvh::hash_var");
}
inline void hash_multiseed(const void* keys, uint32_t key_len, size_t n, const std::vector<HashSeed>& seeds,
                           uint64_t* out, bool fixup = false, void* stream = nullptr) {
  std::vector<uint64_t> s;
  for (const HashSeed& h : seeds) { s.push_back(h.hash1); s.push_back(h.hash2); }
  check(kvh_meow128_multiseed(keys, key_len, n, s.data(), (uint32_t)seeds.size(), out,
                              fixup ? KVH_FIXUP : 0u, stream),
        "kvh::hash_multiseed");
}

// ---- keys and hashes in HOST memory (socket / shm batches): the PCIe-inclusive
// pipelines, synchronous.  devices empty: the current device; else one host
// thread per listed device, each writing its disjoint slice of out.
inline void hash_fixed_host(const void* keys, uint32_t key_len, size_t n, const HashSeed& hs, uint64_t* out,
                            bool fixup = true, const std::vector<int>& devices = {}) {
  const uint32_t f = fixup ? KVH_FIXUP : 0u;
  check(devices.empty() ? kvh_meow128_fixed_host(keys, key_len, n, hs.hash1, hs.hash2, out, f)
                        : kvh_meow128_fixed_host_multi(keys, key_len, n, hs.hash1, hs.hash2, out, f, devices.data(),
                                                       (int)devices.size()),
        "kvh::hash_fixed_host");
}
inline void hash_var_host(const void* keys, const uint64_t* offsets, size_t n, const HashSeed& hs, uint64_t* out,
                          bool fixup = true, const std::vector<int>& devices = {}) {
  const uint32_t f = fixup ? KVH_FIXUP : 0u;
  check(devices.empty() ? kvh_meow128_var_host(keys, offsets, n, hs.hash1, hs.hash2, out, f)
                        : kvh_meow128_var_host_multi(keys, offsets, n, hs.hash1, hs.hash2, out, f, devices.data(),
                                                     (int)devices.size()),
        "kvh::hash_var_host");
}

// ---- the calls either side of the hash, same shape

// Table geometry from the map's header fields (shm_ht.h:143-157, ht_init.cpp:117-156).
inline kvh_ht_geom_t ht_geom(uint64_t map_size, uint32_t hash_entry_size, float hash_value_ratio,
                             uint16_t cuckoo_buckets, uint8_t cuckoo_arity) {
  kvh_ht_geom_t g;
  check(kvh_ht_geom_init(map_size, hash_entry_size, hash_value_ratio, cuckoo_buckets, cuckoo_arity, &g),
        "kvh::ht_geom");
  return g;
}
// f1: hash pairs -> ht_mod(h1) and the cuckoo alternates, positions_per_key(g) per key.
inline uint32_t positions_per_key(const kvh_ht_geom_t& g) { return kvh_positions_per_key(&g); }
inline void ht_positions(const uint64_t* hashes, size_t n, const kvh_ht_geom_t& g, uint64_t* pos,
                         void* stream = nullptr) {
  check(kvh_ht_positions(hashes, n, &g, pos, 0u, stream), "kvh::ht_positions");
}
// f1 fused: fixed-length keys -> fixed-up hash pairs + positions in one pass.
inline void hash_fixed_positions(const void* keys, uint32_t key_len, size_t n, const HashSeed& hs,
                                 const kvh_ht_geom_t& g, uint64_t* hashes, uint64_t* pos, void* stream = nullptr) {
  check(kvh_meow128_fixed_positions(keys, key_len, n, hs.hash1, hs.hash2, &g, hashes, pos, 0u, stream),
        "kvh::hash_fixed_positions");
}

// Device scratch owned by the caller-side helpers below (grown on demand,
// reused across calls; not thread-safe, one per stream).
struct Scratch {
  void* p = nullptr;
  size_t bytes = 0;
  void* need(size_t b) {
    if (b > bytes) {
      check(kvh_device_free(p), "kvh::Scratch");
      p = nullptr;
      bytes = 0;
      check(kvh_device_alloc(&p, b), "kvh::Scratch");
      bytes = b;
    }
    return p;
  }
  Scratch() = default;
  Scratch(const Scratch&) = delete;
  Scratch& operator=(const Scratch&) = delete;
  ~Scratch() { (void)kvh_device_free(p); }
};

// f2: kv_ht_radix_sort + ctest's duplicate loop (ctest.c:89-104) on the device:
// hash pairs (+ items, or nullptr to carry the input index) -> table order.
inline void ht_sort(const uint64_t* hashes, const uint64_t* items, size_t n, const kvh_ht_geom_t& g,
                    uint64_t* hashes_out, uint64_t* items_out, uint64_t* dup_count, bool dedup, Scratch& sc,
                    void* stream = nullptr) {
  const size_t b = kvh_ht_sort_scratch_bytes(n);
  check(kvh_ht_sort(hashes, items, n, &g, hashes_out, items_out, dup_count, dedup ? KVH_DEDUP : 0u, sc.need(b), b,
                    stream),
        "kvh::ht_sort");
}

// f2 at ctest's call shape (ctest.c:89-104, :395): several threads' kv_ht_sort_t batches (<= 64K
// elements each) sorted in place in kv_ht_radix_sort's exact order, all in one launch.
inline void ht_radix_sort_batch(kvh_ht_sort_t* const* ars, const uint32_t* sizes, uint32_t nbatch,
                                const kvh_ht_geom_t& g) {
  check(kvh_ht_radix_sort_batch(ars, sizes, nbatch, &g), "kvh::ht_radix_sort_batch");
}

// f3: ctest's ingest loop (tokenize + kv_hash_key_frag of "token\0") in one
// asynchronous call; *count (device) receives the kept token count.
inline void ingest_text(const void* text, size_t nbytes, const HashSeed& hs, uint64_t* tok_offs, uint32_t* tok_lens,
                        uint64_t* hashes, size_t cap, uint64_t* count, Scratch& sc, uint32_t max_token = 256,
                        void* stream = nullptr) {
  const size_t b = kvh_tokenize_scratch_bytes(nbytes);
  check(kvh_tokenize_hash(text, nbytes, max_token, hs.hash1, hs.hash2, KVH_FIXUP | KVH_NULTERM, tok_offs, tok_lens,
                          hashes, cap, count, sc.need(b), b, stream),
        "kvh::ingest_text");
}

// f4: kv_crc_c of n packed variable-length keys (seeds nullptr: one seed for all).
inline void crc_var(const void* keys, const uint64_t* offsets, size_t n, const uint32_t* seeds, uint32_t seed,
                    uint32_t* out, void* stream = nullptr) {
  check(kvh_crc_c_var(keys, offsets, n, seeds, seed, out, stream), "kvh::crc_var");
}

}  // namespace kvh
