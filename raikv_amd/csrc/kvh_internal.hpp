// kvh_internal.hpp -- shared by the translation units of libkvh.so
// (kvh.hip: hash kernels + C-ABI; ht_pos.hip: table positions, SURVEY.md
// §8 f1): the fixed-length key loaders/stores and the host runtime helpers
// (error state, device properties).  Not installed, not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "meow_dev.hpp"

namespace kvh {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));


// Key i of a fixed-length batch as NC 16-byte chunks (zero padded past L).
// NTM: non-temporal (streamed-once) loads.
template <int L, bool A16, bool NTM = false>
__device__ __forceinline__ void load_fixed(const uint8_t* __restrict__ p, Blk* D) {
  constexpr int NC = Plan<L>::NC;
  if constexpr (A16 && (L % 16) == 0) {
#pragma unroll
    for (int j = 0; j < NC; j++) {
      const v4u* q = (const v4u*)(p + 16 * j);
      const v4u v = NTM ? __builtin_nontemporal_load(q) : *q;
      D[j].w[0] = v.x; D[j].w[1] = v.y; D[j].w[2] = v.z; D[j].w[3] = v.w;
    }
  } else {
    // L % 8 == 0 and 8-byte aligned rows
#pragma unroll
    for (int j = 0; j < L / 8; j++) {
      const v2u* q = (const v2u*)(p + 8 * j);
      const v2u v = NTM ? __builtin_nontemporal_load(q) : *q;
      D[j / 2].w[(j & 1) * 2 + 0] = v.x;
      D[j / 2].w[(j & 1) * 2 + 1] = v.y;
    }
    if constexpr ((L % 16) == 8) { D[NC - 1].w[2] = 0; D[NC - 1].w[3] = 0; }
  }
}

template <bool NTM = false>
__device__ __forceinline__ void store_h(uint64_t* __restrict__ out, uint64_t idx, Blk h, bool fix) {
  if (fix) h = fixup(h);
  v4u v;
  v.x = h.w[0]; v.y = h.w[1]; v.z = h.w[2]; v.w = h.w[3];
  v4u* q = (v4u*)(out + 2 * idx);
  if constexpr (NTM) __builtin_nontemporal_store(v, q); else *q = v;
}

constexpr int kLT = 64;   // full per-length constant records (L < 64)
constexpr int kNF = 256;  // F-only records for 64 <= L < 64 + kNF

// Per-length folding constants of a variable-length batch from LDS tables
// (k_generic, k_keysrc): full records for L < kLT, first-absorb folds for
// kLT <= L < kLT + kNF, in-lane folds beyond.
template <class Tab>
struct LdsK {
  const MeowConst* full;   // [kLT]
  const Blk* ftab;         // [kNF][4]
  uint32_t L;
  Blk m;
  const Tab& T;
  __device__ __forceinline__ LdsK(const MeowConst* f, const Blk* ft, uint32_t len, uint64_t s1,
                                  uint64_t s2, const Tab& t)
      : full(f), ftab(ft), L(len), m(mixer(s1, s2, len)), T(t) {}
  __device__ __forceinline__ uint32_t li() const { return L < (uint32_t)kLT ? L : (uint32_t)kLT - 1; }
  __device__ __forceinline__ Blk M() const { return m; }
  __device__ __forceinline__ Blk F(int i) const {
    if (L < (uint32_t)kLT) return full[L].F[i];
    if (L < (uint32_t)(kLT + kNF)) return ftab[(L - kLT) * 4 + i];
    return aesT(bxor(ramp(i), m), T);
  }
  __device__ __forceinline__ Blk G(int i) const { return full[li()].G[i]; }
  __device__ __forceinline__ Blk TG2() const { return full[li()].TG2; }
  __device__ __forceinline__ Blk CS2b() const { return full[li()].CS2b; }
  __device__ __forceinline__ Blk TCS0a() const { return full[li()].TCS0a; }
};

namespace rt {
// thread-local last error (kvh_last_error); returns e
int set_err(int e);
// HIP error -> KVH_EHIP_BASE - e, recorded
int hip_err(hipError_t e);
// compute units of the current device (cached)
int device_cus(int* cus);
// hipGetLastError after a launch -> 0 or the recorded error
int launch_done();
}  // namespace rt

}  // namespace kvh
