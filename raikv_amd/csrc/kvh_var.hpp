// kvh_var.hpp -- pieces shared by the variable-length Meow kernels (kvh.hip:
// k_var6, k_var9) and the research kernels of the experiments build
// (tools/exp/kvh_exp.hip): per-length constant records read from LDS, the
// 4-GiB-window fallback, the per-wave window layout and the wave-local LDS
// ordering.  Not installed, not part of the ABI.
#pragma once
#include "kvh_internal.hpp"

namespace kvh {

struct VConst {  // MeowConst minus the Mixer (recomputed in-lane)
  Blk F[4], G[4], TG2, CS2b, TCS0a;
};

template <class Tab, class LenT = uint32_t>
struct LdsKV5 {
  const VConst* full;
  LenT L;
  Blk m;
  const Tab& T;
  const Blk* ftab;  // first-absorb folds F[0..3] for kLT <= L < kLT + kNF, or null
  __device__ __forceinline__ LdsKV5(const VConst* f, LenT len, uint64_t s1, uint64_t s2, const Tab& t,
                                    const Blk* ft = nullptr)
      : full(f), L(len), m(mixer(s1, s2, len)), T(t), ftab(ft) {}
  __device__ __forceinline__ uint32_t li() const { return L < (LenT)kLT ? (uint32_t)L : (uint32_t)kLT - 1; }
  __device__ __forceinline__ Blk M() const { return m; }
  __device__ __forceinline__ Blk F(int i) const {
    if (L < (LenT)kLT) return full[L].F[i];
    if (ftab && L < (LenT)(kLT + kNF)) return ftab[(L - kLT) * 4 + i];
    return aesT(bxor(ramp(i), m), T);
  }
  __device__ __forceinline__ Blk G(int i) const { return full[li()].G[i]; }
  __device__ __forceinline__ Blk TG2() const { return full[li()].TG2; }
  __device__ __forceinline__ Blk CS2b() const { return full[li()].CS2b; }
  __device__ __forceinline__ Blk TCS0a() const { return full[li()].TCS0a; }
};

// The keys [i0, i0 + k) of a window whose bytes span 4 GiB or more, hashed
// in input order with u64 offsets and lengths (k_var6 / k_var7 keep u32
// window-relative records).  Out of line and without the LDS constant
// records (every key of such a window is folded in-lane): the hot kernels'
// register allocation does not see it.
template <int NT>
__device__ __attribute__((noinline)) void wide_window(const uint8_t* __restrict__ keys,
                                                      const uint64_t* __restrict__ offs, uint64_t i0, uint32_t k,
                                                      int nchunks, uint64_t s1, uint64_t s2,
                                                      uint64_t* __restrict__ out, bool fix, const uint32_t* lds) {
  const LdsTab<NT> T(lds);
  const uint32_t lane = threadIdx.x & 63;
  for (int c = 0; c < nchunks; c++) {
    const uint32_t j = 64 * c + lane;
    if (j < k) {
      const uint64_t a = offs[i0 + j], len = offs[i0 + j + 1] - a;
      const MeowConst K = make_const(s1, s2, len, T);
      const RegK R{K};
      store_h(out, i0 + j, meow_rt(keys + a, len, R, T), fix);
    }
  }
}

template <int WIN, int NW = kBlock / 64>
struct Var6Cfg {
  static constexpr int kWaves = NW;
  static constexpr int kHist = 256 * 4;                       // u32[256]
  static constexpr int kRec = WIN * 12;                       // u32 off, u32 len, u32 idx
  static constexpr int kPerWave = kHist + kRec > WIN * 16 ? kHist + kRec : WIN * 16;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct VConst9 {  // VConst minus CS2b (meow_a never needs it), padded to 13 blocks:
  Blk F[4], G[4], TG2, TCS0a, pad;  // a 52-dword stride puts the 16 lengths of a class on distinct banks
};
// Block index of first-absorb fold F[i] of length L (kLT <= L) in the k_var9
// fold table: 4 blocks per length, the block order XOR-swizzled by bits 2-3
// of L - kLT, so that 16 consecutive lengths (a 16-byte class of long keys)
// read any one F[i] from 16 distinct 16-byte bank slots (ds_read_b128: 16
// lanes per LDS cycle over a 256-byte bank row); unswizzled, lengths 4
// apart share a slot (4-way conflicts in a chunk of long keys).
__device__ __forceinline__ uint32_t kf_index(uint32_t L, int i) {
  const uint32_t r = L - (uint32_t)kLT;
  return (r << 2) + ((uint32_t)i ^ ((r >> 2) & 3u));
}
template <class Tab, int NF>
struct LdsKV9 {
  const VConst9* full;
  const Blk* ftab;  // first-absorb folds F[0..3] for kLT <= L < kLT + NF
  uint32_t L;
  Blk m;
  const Tab& T;
  __device__ __forceinline__ LdsKV9(const VConst9* f, const Blk* ft, uint32_t len, uint64_t s1, uint64_t s2,
                                    const Tab& t)
      : full(f), ftab(ft), L(len), m(mixer(s1, s2, len)), T(t) {}
  __device__ __forceinline__ uint32_t li() const { return L < (uint32_t)kLT ? L : (uint32_t)kLT - 1; }
  __device__ __forceinline__ Blk M() const { return m; }
  __device__ __forceinline__ Blk F(int i) const {
    if (L < (uint32_t)kLT) return full[L].F[i];
    if (L < (uint32_t)(kLT + NF)) return ftab[kf_index(L, i)];
    return aesT(bxor(ramp(i), m), T);
  }
  // F of a key shorter than kLT, read branch-free; the lanes that do not use
  // it (keys of kLT bytes or more) all read record 0: one broadcast address
  // instead of scattered records that conflict with the short keys' reads
  __device__ __forceinline__ Blk F0(int i) const { return full[L < (uint32_t)kLT ? L : 0u].F[i]; }
  // the same for meow_a's chunks without a full block (every key under kLT bytes)
  __device__ __forceinline__ Blk Fs(int i) const { return full[L < (uint32_t)kLT ? L : 0u].F[i]; }
  __device__ __forceinline__ Blk G(int i) const { return full[li()].G[i]; }
  __device__ __forceinline__ Blk TG2() const { return full[li()].TG2; }
  __device__ __forceinline__ Blk TCS0a() const { return full[li()].TCS0a; }
};
}  // namespace kvh
