// kv_compat.cpp -- link-compatible kv_* symbols over the C-ABI
// (libkvh_kv.so).  A raikv build that drops src/key_hash.c's Meow and CRC32C
// families and links this library instead keeps every call site of
// include/raikv/key_hash.h:8-20 and :59-130 unchanged: same names, same
// argument meaning, same x[] / seed[] layouts, void returns.  Each call runs on the current
// GPU through libkvh.so's host drop-ins (one device round trip per call: the
// latency trap include/kvh.h documents above them -- this library is for
// link compatibility and tests; batches belong on kvh_meow128_*_host /
// KeyCtx::set_hash).
//
// The reference functions have no error path.  A device error here cannot be
// returned, and a silently wrong hash would corrupt a table, so it aborts the
// process with the HIP error string.  HMAC-Meow (key_hash.h:100-109) is a
// different function and out of scope.
#include <stdio.h>
#include <stdlib.h>
#include "kvh_kv.h"
#include "kvh.h"

static void must(int rc, const char* what) {
  if (rc != 0) {
    fprintf(stderr, "libkvh_kv: %s failed: %d (%s)\n", what, rc, kvh_strerror(rc));
    abort();
  }
}

extern "C" {

void kv_hash_meow128(const void* p, size_t sz, uint64_t* h1, uint64_t* h2) {
  must(kvh_hash_meow128(p, sz, h1, h2), "kv_hash_meow128");
}

uint64_t kv_hash_meow64(const void* p, size_t sz, uint64_t seed) {
  const uint64_t h = kvh_hash_meow64(p, sz, seed);
  must(kvh_last_error(), "kv_hash_meow64");
  return h;
}

void kv_hash_meow128_vec(const meow_vec_t* vec, size_t vec_sz, uint64_t* h1, uint64_t* h2) {
  // meow_vec_t and kvh_meow_vec_t are both {const void *p; size_t sz;}
  must(kvh_hash_meow128_vec((const kvh_meow_vec_t*)vec, vec_sz, h1, h2), "kv_hash_meow128_vec");
}

void kv_meow128_init(meow_ctx_t* m, meow_block_t* b, uint64_t k1, uint64_t k2, size_t total_update_sz) {
  must(kvh_meow128_init((kvh_meow_ctx_t*)m, (kvh_meow_block_t*)b, k1, k2, total_update_sz), "kv_meow128_init");
}

void kv_meow128_update(meow_ctx_t* m, meow_block_t* b, const void* p, size_t sz) {
  must(kvh_meow128_update((kvh_meow_ctx_t*)m, (kvh_meow_block_t*)b, p, sz), "kv_meow128_update");
}

void kv_meow128_final(meow_ctx_t* m, meow_block_t* b, uint64_t* k1, uint64_t* k2) {
  must(kvh_meow128_final((kvh_meow_ctx_t*)m, (kvh_meow_block_t*)b, k1, k2), "kv_meow128_final");
}

void kv_meow_test(const void* p, size_t sz, uint64_t* k1, uint64_t* k2) {
  must(kvh_meow_test(p, sz, k1, k2), "kv_meow_test");
}

void kv_hash_meow128_2_same_length(const void* p, const void* p2, size_t sz, uint64_t* x4) {
  must(kvh_hash_meow128_2_same_length(p, p2, sz, x4), "kv_hash_meow128_2_same_length");
}

void kv_hash_meow128_4_same_length_a(const void** p, size_t sz, uint64_t* x) {
  must(kvh_hash_meow128_4_same_length_a(p, sz, x), "kv_hash_meow128_4_same_length_a");
}

void kv_hash_meow128_8_same_length_a(const void** p, size_t sz, uint64_t* x) {
  must(kvh_hash_meow128_8_same_length_a(p, sz, x), "kv_hash_meow128_8_same_length_a");
}

void kv_hash_meow128_4_same_length(const void* p, const void* p2, const void* p3, const void* p4, size_t sz,
                                   uint64_t* x) {
  must(kvh_hash_meow128_4_same_length(p, p2, p3, p4, sz, x), "kv_hash_meow128_4_same_length");
}

void kv_hash_meow128_4_same_length_4_seed(const void* p, const void* p2, const void* p3, const void* p4, size_t sz,
                                          uint64_t* x) {
  must(kvh_hash_meow128_4_same_length_4_seed(p, p2, p3, p4, sz, x), "kv_hash_meow128_4_same_length_4_seed");
}

void kv_hash_meow128_8_same_length(const void* p, const void* p2, const void* p3, const void* p4, const void* p5,
                                   const void* p6, const void* p7, const void* p8, size_t sz, uint64_t* x) {
  must(kvh_hash_meow128_8_same_length(p, p2, p3, p4, p5, p6, p7, p8, sz, x), "kv_hash_meow128_8_same_length");
}

void kv_hash_meow128_2_diff_length(const void* p, size_t sz, const void* p2, size_t sz2, uint64_t* x) {
  must(kvh_hash_meow128_2_diff_length(p, sz, p2, sz2, x), "kv_hash_meow128_2_diff_length");
}

void kv_hash_meow128_4_diff_length(const void* p, size_t sz, const void* p2, size_t sz2, const void* p3,
                                   size_t s3, const void* p4, size_t s4, uint64_t* x) {
  must(kvh_hash_meow128_4_diff_length(p, sz, p2, sz2, p3, s3, p4, s4, x), "kv_hash_meow128_4_diff_length");
}

// CRC32C family (key_hash.h:8-20, key_hash.c:27-179): the kvh_crc_c drop-ins
uint32_t kv_hash_uint(uint32_t i) {
  const uint32_t h = kvh_hash_uint(i);
  must(kvh_last_error(), "kv_hash_uint");
  return h;
}

uint32_t kv_hash_uint2(uint32_t r, uint32_t i) {
  const uint32_t h = kvh_hash_uint2(r, i);
  must(kvh_last_error(), "kv_hash_uint2");
  return h;
}

uint32_t kv_crc_c(const void* p, size_t sz, uint32_t seed) {
  const uint32_t h = kvh_crc_c(p, sz, seed);
  must(kvh_last_error(), "kv_crc_c");
  return h;
}

void kv_crc_c_2_diff(const void* p, size_t sz, uint32_t* seed, const void* p2, size_t sz2, uint32_t* seed2) {
  must(kvh_crc_c_2_diff(p, sz, seed, p2, sz2, seed2), "kv_crc_c_2_diff");
}

void kv_crc_c_4_diff(const void* p, size_t sz, uint32_t* seed, const void* p2, size_t sz2, uint32_t* seed2,
                     const void* p3, size_t sz3, uint32_t* seed3, const void* p4, size_t sz4, uint32_t* seed4) {
  must(kvh_crc_c_4_diff(p, sz, seed, p2, sz2, seed2, p3, sz3, seed3, p4, sz4, seed4), "kv_crc_c_4_diff");
}

void kv_crc_c_array(const void** p, size_t* psz, uint32_t* seed, size_t count) {
  must(kvh_crc_c_array(p, psz, seed, count), "kv_crc_c_array");
}

void kv_crc_c_key_array(const void* p, size_t* psz, uint32_t* seed, size_t count) {
  must(kvh_crc_c_key_array(p, psz, seed, count), "kv_crc_c_key_array");
}

}  // extern "C"
