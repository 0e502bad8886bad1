// kvh_exp.hip -- the RESEARCH kernels of the Meow engine: variants that lost
// their A/B and ablation builds whose outputs are not hashes.  Not part of
// libkvh.so.  `make experiments` links the product objects plus this file
// into tools/libkvh_exp.so; a static initialiser fills rt::g_exp, so the
// research kernels answer the same C-ABI calls under extra kvh_set_tuning
// values (tools/*.py select the library with KVH_LIB).  Their measured
// results are in DESIGN.md (§3.3, §3.8, §4.3, §6).
//
//   k_fixed_x   k_fixed with ablation MODEs (knob 5) and a register prefetch
//               of the next chunk (knob 10)
//   k_fixed_dma LDS-DMA ring streaming (knob 6)
//   k_hybrid    T-table and bitsliced waves side by side (knobs 11-13)
//   k_var, k_var3, k_var5, k_var7, k_var8  variable-length experiments
//   k_var6x     k_var6 with next-chunk prefetches (knob 7 = 9, 10, 20, 22)
//   k_var9x     k_var9 with long keys two lanes per key (knob 7 = 26, 27)
//   k_var11, k_var11_q, k_var12  long keys deferred to class-uniform queues
//               (knob 7 = 40-43, round 3): fewer LDS instructions, slower
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <atomic>
#include <algorithm>
#include <mutex>
#include "../../raikv_amd/csrc/meow_dev.hpp"
#include "../../raikv_amd/csrc/bs_prelude.hpp"
#include "../../raikv_amd/csrc/kvh_internal.hpp"
#include "../../raikv_amd/csrc/kvh_var.hpp"
#include "meow_exp.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

// ------------------------------------------------------------ k_fixed_x
// Wave-chunked streaming: wave w owns chunks of 64*U consecutive keys
// (chunk c = keys [64U(w + c*W), 64U(w + c*W + 1)), W = waves in the grid);
// lane l takes keys base + 64u + l, so every load/store instruction moves
// one contiguous 64*L-byte (64*16-byte) run.  The U loads of a chunk are all
// issued before the first round (U independent AES chains per lane hide LDS
// latency; U loads per lane in flight hide HBM latency), loads and stores are
// non-temporal (each byte is touched once).  Measured on MI355X this access
// shape streams 6.2 TB/s where a grid-stride loop with a one-step register
// prefetch tops out near 5.1 TB/s (tools/mem_probe.hip).
// Indices past the end are clamped to n-1: those lanes recompute key n-1 and
// store the identical hash to out[n-1] (benign duplicate), which keeps the
// chunk body one basic block.
// MODE (ablation builds, kvh_set_tuning(5, m)): 0 = the product path;
// 1 = copy keys to out without hashing (memory-only); 2 = no key loads (keys
// synthesised from the index: LDS + stores); 3 = no stores (hashes folded
// into one value per lane: LDS + loads).
template <int L, int NT, bool A16, int U, int MODE = 0, bool PF = false>
__global__ void __launch_bounds__(kBlock)
k_fixed_x(const uint8_t* __restrict__ keys, uint64_t n, uint64_t s1, uint64_t s2,
        uint64_t* __restrict__ out, uint32_t flags) {
  constexpr int NC = Plan<L>::NC;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  const uint64_t last = n - 1;
  Blk acc = bzero();
  auto load_chunk = [&](uint64_t b, Blk (&D)[U][NC]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      if constexpr (MODE == 2) {
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
          for (int w = 0; w < 4; w++) D[u][c].w[w] = (uint32_t)j * 2654435761u + (uint32_t)(4 * c + w);
      } else if constexpr (MODE == 4) {
        // the same 64L bytes of the group, read as NC fully coalesced 1 KiB
        // runs (lane l takes 16 bytes at 1024c + 16l): the load pattern a
        // lane transpose would allow, with the keys scrambled
        static_assert(L % 16 == 0, "MODE 4: whole 16-byte pieces");
        const uint64_t cb = (b + 64 * u) * (uint64_t)L, tot = n * (uint64_t)L;
#pragma unroll
        for (int c = 0; c < NC; c++) {
          uint64_t off = cb + 1024 * (uint64_t)c + 16 * lane;
          off = off + 16 <= tot ? off : tot - 16;
          const v4u v = __builtin_nontemporal_load((const v4u*)(keys + off));
          D[u][c].w[0] = v.x; D[u][c].w[1] = v.y; D[u][c].w[2] = v.z; D[u][c].w[3] = v.w;
        }
      } else if constexpr (MODE == 6 || MODE == 8) {
        // 64-byte keys, lanes in pairs (2i, 2i+1) owning keys i and 32 + i
        // of the group: each load instruction reads 32 bytes of each of 32
        // keys (16 lines, half of each), and the pair swaps the two pieces
        // each lane loaded for the other (two DPP moves per dword: lane
        // parity picks which registers are sent; MODE 8 skips the exchange,
        // the load pattern alone, keys scrambled)
        static_assert(L == 64, "MODE 6/8: 64-byte keys");
        const uint64_t g = b + 64 * u, i = lane >> 1;
        const bool odd = (lane & 1) != 0;
        const uint64_t klo = g + i < last ? g + i : last, khi = g + 32 + i < last ? g + 32 + i : last;
        const uint32_t o = odd ? 16u : 0u, e = odd ? 0u : 16u;
        const uint8_t* src[4] = {keys + klo * 64 + o, keys + klo * 64 + 32 + o, keys + khi * 64 + e,
                                 keys + khi * 64 + 32 + e};
        Blk R[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const v4u v = __builtin_nontemporal_load((const v4u*)src[c]);
          R[c].w[0] = v.x; R[c].w[1] = v.y; R[c].w[2] = v.z; R[c].w[3] = v.w;
        }
        if constexpr (MODE == 8) {
#pragma unroll
          for (int c = 0; c < 4; c++) D[u][c] = R[c];
        } else {
#pragma unroll
          for (int w = 0; w < 4; w++) {
            const uint32_t X = odd ? R[0].w[w] : R[2].w[w], Y = odd ? R[1].w[w] : R[3].w[w];
            D[u][0].w[w] = odd ? R[2].w[w] : R[0].w[w];
            D[u][1].w[w] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)X, 0xB1, 0xF, 0xF, false);
            D[u][2].w[w] = odd ? R[3].w[w] : R[1].w[w];
            D[u][3].w[w] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)Y, 0xB1, 0xF, 0xF, false);
          }
        }
      } else {
        load_fixed<L, A16, true>(keys + (j < last ? j : last) * L, D[u]);
      }
    }
  };
  // the key a lane hashes: lane l, except under MODE 6/8 (lane pairs own i and 32 + i)
  auto key_of = [&](uint64_t b, int u) -> uint64_t {
    if constexpr (MODE == 6 || MODE == 8) return b + 64 * u + ((lane & 1) ? 32 + (lane >> 1) : (lane >> 1));
    else return b + 64 * u + lane;
  };
  // PF: the next chunk's loads are issued before this chunk's rounds, so
  // each wave keeps its HBM reads in flight across its whole compute phase
  // (U*NC*4 more VGPRs; the past-the-end prefetch of the last trip reads the
  // clamped key n-1 and is dropped)
  Blk Dn[U][NC];
  if constexpr (PF) load_chunk(wave * 64 * U, Dn);
  for (uint64_t b = wave * 64 * U; b < n; b += step) {  // wave-uniform trip count
    Blk D[U][NC];
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int c = 0; c < NC; c++) D[u][c] = Dn[u][c];
      load_chunk(b + step, Dn);
    } else {
      load_chunk(b, D);
    }
    Blk h[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      if constexpr (MODE == 1) h[u] = D[u][0];
      else h[u] = meow_ct<L>(D[u], K, T);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = key_of(b, u);
      if constexpr (MODE == 3) acc = bxor(acc, h[u]);
      else store_h<true>(out, j < last ? j : last, h[u], fix);
    }
  }
  if constexpr (MODE == 3) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g < n) store_h(out, g, acc, false);
  }
}

// ---------------------------------------------------------------------
// LDS-DMA streaming (opt-in, knob 6; the register path k_fixed is C1/C4's
// default: 153.9 vs 130-139 G hash/s at ring depths 2-6, tools/tune.py).
// One 1024-thread workgroup per CU:
// NT replicated tables plus, per wave, a ring of R chunk slots in the SAME
// __shared__ array (one LDS object: no compiler-inserted vmcnt(0) before the
// ring reads).  A chunk is 64 consecutive keys (64*L contiguous bytes); the
// wave streams them into its ring with global_load_lds_dwordx4 (no VGPRs,
// non-temporal), R-1 chunks ahead of the one it hashes, so the HBM latency is
// covered by DMA in flight instead of by registers.  Each wave waits for its
// own chunk with a counted `s_waitcnt vmcnt(N)` (N = DMA and store
// instructions issued after it), reads its key from LDS, hashes, and stores
// 16 B per key non-temporally.  Only full chunks take this path; the < 64
// trailing keys are hashed by the last wave with direct loads.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int L, int NT, int R>
struct DmaCfg {
  static constexpr int kWaves = kBlock / 64;
  static constexpr int CH = 64 * L;                 // chunk bytes
  static constexpr int D = (CH + 1023) / 1024;      // DMA instructions per chunk
  static constexpr int S = 1;                       // store instructions per chunk
  static constexpr int kTabBytes = NT * 8192 * 4;
  static constexpr int kBytes = kTabBytes + kWaves * R * CH;
  static constexpr bool kFits = kBytes <= 163840 && L % 16 == 0;
};

template <int L, int NT, int R>
__device__ __forceinline__ void dma_chunk(const uint8_t* __restrict__ src, uint32_t* slot, uint32_t lane) {
  using C = DmaCfg<L, NT, R>;
#pragma unroll
  for (int q = 0; q < C::D; q++) {
    __builtin_amdgcn_global_load_lds((const void*)(src + 1024 * q + 16 * lane),
                                     (void __attribute__((address_space(3)))*)((char*)slot + 1024 * q),
                                     16, 0, 2 /* nt */);
  }
}

// wait until DMA(k) has landed: after it were issued (R-1) chunk DMAs and
// min(k, R-1) iterations' stores
template <int L, int NT, int R>
__device__ __forceinline__ void wait_chunk(uint64_t k) {
  using C = DmaCfg<L, NT, R>;
  constexpr int base = (R - 1) * C::D;
  if (k >= (uint64_t)(R - 1)) { wait_vmcnt<base + (R - 1) * C::S>(); return; }
  if constexpr (R > 1) if (k == 0) { wait_vmcnt<base>(); return; }
  if constexpr (R > 2) if (k == 1) { wait_vmcnt<base + C::S>(); return; }
  if constexpr (R > 3) if (k == 2) { wait_vmcnt<base + 2 * C::S>(); return; }
  if constexpr (R > 4) if (k == 3) { wait_vmcnt<base + 3 * C::S>(); return; }
  if constexpr (R > 5) if (k == 4) { wait_vmcnt<base + 4 * C::S>(); return; }
  if constexpr (R > 6) if (k == 5) { wait_vmcnt<base + 5 * C::S>(); return; }
  if constexpr (R > 7) if (k == 6) { wait_vmcnt<base + 6 * C::S>(); return; }
  wait_vmcnt<0>();
}

template <int L, int NT, int R>
__global__ void __launch_bounds__(kBlock)
k_fixed_dma(const uint8_t* __restrict__ keys, uint64_t n, uint64_t s1, uint64_t s2,
            uint64_t* __restrict__ out, uint32_t flags) {
  using C = DmaCfg<L, NT, R>;
  static_assert(C::kFits, "LDS budget / 16-byte key pieces");
  constexpr int NC = Plan<L>::NC;
  __shared__ __attribute__((aligned(16))) uint32_t lds[C::kBytes / 4];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * C::kWaves + wv;
  const uint64_t NW = (uint64_t)gridDim.x * C::kWaves;
  const uint64_t nchunks = n / 64;
  uint32_t* ring = lds + C::kTabBytes / 4 + wv * (R * C::CH / 4);
  const uint64_t nk = gw < nchunks ? (nchunks - 1 - gw) / NW + 1 : 0;  // wave-uniform
  if (nk) {
    const uint64_t lastc = nchunks - 1;
    auto src_of = [&](uint64_t k) {
      const uint64_t c = gw + k * NW;
      return keys + (c < lastc ? c : lastc) * (uint64_t)C::CH;
    };
#pragma unroll
    for (int k = 0; k < R - 1; k++) dma_chunk<L, NT, R>(src_of(k), ring + k * (C::CH / 4), lane);
    for (uint64_t k = 0; k < nk; k++) {
      const uint64_t kn = k + R - 1;
      dma_chunk<L, NT, R>(src_of(kn), ring + (kn % R) * (C::CH / 4), lane);
      wait_chunk<L, NT, R>(k);
      const uint32_t* slot = ring + (k % R) * (C::CH / 4);
      Blk D[NC];
#pragma unroll
      for (int j = 0; j < NC; j++) {
        const v4u v = *(const v4u*)((const char*)slot + lane * L + 16 * j);
        D[j].w[0] = v.x; D[j].w[1] = v.y; D[j].w[2] = v.z; D[j].w[3] = v.w;
      }
      const Blk h = meow_ct<L>(D, K, T);
      store_h<true>(out, (gw + k * NW) * 64 + lane, h, fix);
    }
    wait_vmcnt<0>();  // drain the trailing dummy DMAs before the wave exits
  }
  // keys past the last full chunk
  if (gw == NW - 1) {
    const uint64_t j = nchunks * 64 + lane;
    if (j < n) {
      Blk D[NC];
      load_fixed<L, true>(keys + j * L, D);
      store_h(out, j, meow_ct<L>(D, K, T), fix);
    }
  }
}

// ---------------------------------------------------------------------
// Variable-length batches (config C2).  One lane per key, but NOT in input
// order: each workgroup takes a window of 1024 consecutive keys, counting-
// sorts them by length in LDS (LDS atomics + one wave-wide scan), and every
// wave then hashes 64 keys of (nearly) equal length, so the absorb loop trip
// count and every trail/finalisation branch are (nearly) wave-uniform.  The
// window's key bytes (~50 KB for C2) stay L2-resident while its waves gather
// their keys with dword-aligned dwordx4 loads; hashes are scattered back to
// the keys' original slots.  Per-length constants live in LDS: the full
// folding record for L < 64 and the first-absorb folds F[i] for
// 64 <= L < 64 + NF; longer keys fold in-lane.
template <int NT>
struct VarCfg {
  static constexpr int kNF = NT == 4 ? 32 : 256;
  static constexpr int kTab = NT * 8192 * 4;
  static constexpr int kFull = kTab;                                 // MeowConst[kLT]
  static constexpr int kFOff = kFull + kLT * (int)sizeof(MeowConst); // Blk[kNF][4]
  static constexpr int kCnt = kFOff + kNF * 4 * 16;                  // u32[320] counts / starts
  static constexpr int kRecO = kCnt + 320 * 4;                       // u64[1024] sorted key start
  static constexpr int kRecL = kRecO + kBlock * 8;                   // u32[1024] sorted key length
  static constexpr int kRecI = kRecL + kBlock * 4;                   // u16[1024] sorted -> window slot
  static constexpr int kBytes = kRecI + kBlock * 2;
  static_assert(kBytes <= 163840, "LDS budget");
};

template <class Tab, int NF>
struct LdsKV {
  const MeowConst* full;
  const Blk* ftab;
  uint32_t L;
  Blk m;
  const Tab& T;
  __device__ __forceinline__ LdsKV(const MeowConst* f, const Blk* ft, uint32_t len, uint64_t s1, uint64_t s2,
                                   const Tab& t)
      : full(f), ftab(ft), L(len), m(mixer(s1, s2, len)), T(t) {}
  __device__ __forceinline__ uint32_t li() const { return L < (uint32_t)kLT ? L : (uint32_t)kLT - 1; }
  __device__ __forceinline__ Blk M() const { return m; }
  __device__ __forceinline__ Blk F(int i) const {
    if (L < (uint32_t)kLT) return full[L].F[i];
    if (L < (uint32_t)(kLT + NF)) return ftab[(L - kLT) * 4 + i];
    return aesT(bxor(ramp(i), m), T);
  }
  __device__ __forceinline__ Blk G(int i) const { return full[li()].G[i]; }
  __device__ __forceinline__ Blk TG2() const { return full[li()].TG2; }
  __device__ __forceinline__ Blk CS2b() const { return full[li()].CS2b; }
  __device__ __forceinline__ Blk TCS0a() const { return full[li()].TCS0a; }
};

template <int NT>
__global__ void __launch_bounds__(kBlock)
k_var(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
      uint64_t* __restrict__ out, uint32_t flags) {
  using C = VarCfg<NT>;
  __shared__ __attribute__((aligned(16))) uint32_t lds[C::kBytes / 4];
  MeowConst* kfull = (MeowConst*)((char*)lds + C::kFull);
  Blk* kf = (Blk*)((char*)lds + C::kFOff);
  uint32_t* cnt = (uint32_t*)((char*)lds + C::kCnt);
  uint64_t* rec_o = (uint64_t*)((char*)lds + C::kRecO);
  uint32_t* rec_l = (uint32_t*)((char*)lds + C::kRecL);
  uint16_t* rec_i = (uint16_t*)((char*)lds + C::kRecI);
  fill_tables<NT>(lds);
  for (uint32_t b = threadIdx.x; b < 320; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + C::kNF); l += blockDim.x) {
    if (l < (uint32_t)kLT) {
      kfull[l] = make_const(s1, s2, l, T);
    } else {
      const Blk M = mixer(s1, s2, l);
#pragma unroll
      for (int q = 0; q < 4; q++) kf[(l - kLT) * 4 + q] = aesT(bxor(ramp(q), M), T);
    }
  }
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t t = threadIdx.x, lane = t & 63;
  const uint64_t wstep = (uint64_t)gridDim.x * kBlock;
  uint64_t base = (uint64_t)blockIdx.x * kBlock;
  // offsets of this thread's key in the first window (prefetched one window ahead)
  uint64_t p0 = 0, p1 = 0;
  if (base + t < n) { p0 = offs[base + t]; p1 = offs[base + t + 1]; }
  for (; base < n; base += wstep) {
    const uint64_t o0 = p0, o1 = p1;
    const uint64_t nxt = base + wstep + t;
    if (nxt < n) { p0 = offs[nxt]; p1 = offs[nxt + 1]; }
    const bool valid = base + t < n;
    const uint32_t L = (uint32_t)(o1 - o0);
    const uint32_t bucket = valid ? (L < 255u ? L : 255u) : 300u;  // past-the-end keys sort last
    atomicAdd(&cnt[bucket], 1u);
    __syncthreads();
    if (t < 64) {  // exclusive scan of 320 counts by one wave: 5 per lane
      uint32_t v[5], sum = 0;
#pragma unroll
      for (int k = 0; k < 5; k++) { v[k] = cnt[lane * 5 + k]; sum += v[k]; }
      uint32_t incl = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
      }
      uint32_t run = incl - sum;
#pragma unroll
      for (int k = 0; k < 5; k++) { cnt[lane * 5 + k] = run; run += v[k]; }
    }
    __syncthreads();
    const uint32_t pos = atomicAdd(&cnt[bucket], 1u);
    rec_o[pos] = o0;
    rec_l[pos] = L;
    rec_i[pos] = (uint16_t)t;
    __syncthreads();
    const uint64_t ko = rec_o[t];
    const uint32_t kl = rec_l[t];
    const uint64_t j = base + rec_i[t];
    cnt[t < 320 ? t : 319] = 0;  // ready for the next window (read only before the barrier above)
    if (j < n) {
      const LdsKV<LdsTab<NT>, C::kNF> K(kfull, kf, kl, s1, s2, T);
      store_h(out, j, meow_var(keys + ko, kl, K, T), fix);
    }
    __syncthreads();  // rec_* / cnt reuse by the next window
  }
}

// k_var3: windows of KPT*1024 keys per workgroup.
//  [A] each thread loads the offsets of its KPT window keys (kept in VGPRs)
//      and counts them into 256 length buckets (LDS atomics);
//  [B] one wave scans the counts; threads scatter records {u64 start,
//      u32 length, u16 window slot} in length order;
//  [C] thread t reads its sorted records t, t+1024, ... and hashes them with
//      the first pieces of the next key already in flight (prefetch_first):
//      the keys of a wave have (nearly) one length, so trip counts and
//      trail/finalisation branches are (nearly) uniform;
//  [D] hashes are staged in LDS by window slot (the record area, free after
//      [C] has read it) and written back as contiguous 16-byte runs -- a
//      scattered 16-byte store per key doubled the HBM write traffic.
template <int NT, int KPT>
struct Var3Cfg {
  static constexpr int W = KPT * kBlock;
  static constexpr int kTab = NT * 8192 * 4;
  static constexpr int kFull = kTab;                                   // MeowConst[kLT]
  static constexpr int kCnt = kFull + kLT * (int)sizeof(MeowConst);    // u32[320]
  static constexpr int kU = kCnt + 320 * 4;                            // union area
  static constexpr int kRecO = kU;                                     // u64[W]
  static constexpr int kRecL = kRecO + W * 8;                          // u32[W]
  static constexpr int kRecI = kRecL + W * 4;                          // u16[W]
  static constexpr int kRecEnd = kRecI + W * 2;
  static constexpr int kOutEnd = kU + W * 16;                          // Blk[W] staged hashes
  static constexpr int kBytes = kRecEnd > kOutEnd ? kRecEnd : kOutEnd;
  static_assert(kBytes <= 163840, "LDS budget");
};

template <int NT, int KPT, int MODE = 0>
__global__ void __launch_bounds__(kBlock)
k_var3(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
       uint64_t* __restrict__ out, uint32_t flags) {
  using C = Var3Cfg<NT, KPT>;
  constexpr uint32_t W = C::W;
  __shared__ __attribute__((aligned(16))) uint32_t lds[C::kBytes / 4];
  MeowConst* kfull = (MeowConst*)((char*)lds + C::kFull);
  uint32_t* cnt = (uint32_t*)((char*)lds + C::kCnt);
  uint64_t* rec_o = (uint64_t*)((char*)lds + C::kRecO);
  uint32_t* rec_l = (uint32_t*)((char*)lds + C::kRecL);
  uint16_t* rec_i = (uint16_t*)((char*)lds + C::kRecI);
  Blk* hout = (Blk*)((char*)lds + C::kU);
  fill_tables<NT>(lds);
  for (uint32_t b = threadIdx.x; b < 320; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)kLT; l += blockDim.x) kfull[l] = make_const(s1, s2, l, T);
  const Blk* nofold = nullptr;
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t t = threadIdx.x, lane = t & 63;
  for (uint64_t base = (uint64_t)blockIdx.x * W; base < n; base += (uint64_t)gridDim.x * W) {
    const uint64_t wend = base + W < n ? base + W : n;
    const uint32_t nw = (uint32_t)(wend - base);
    // [A]
    uint64_t o0[KPT], o1[KPT];
    uint32_t bk[KPT];
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const uint32_t s = t + k * kBlock;
      o0[k] = o1[k] = 0;
      if (s < nw) { o0[k] = offs[base + s]; o1[k] = offs[base + s + 1]; }
    }
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const uint64_t L = o1[k] - o0[k];
      bk[k] = (t + k * kBlock < nw) ? (L < 255 ? (uint32_t)L : 255u) : 300u;
      atomicAdd(&cnt[bk[k]], 1u);
    }
    __syncthreads();
    // [B]
    if (t < 64) {
      uint32_t v[5], sum = 0;
#pragma unroll
      for (int k = 0; k < 5; k++) { v[k] = cnt[lane * 5 + k]; sum += v[k]; }
      uint32_t incl = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
      }
      uint32_t run = incl - sum;
#pragma unroll
      for (int k = 0; k < 5; k++) { cnt[lane * 5 + k] = run; run += v[k]; }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const uint32_t pos = MODE == 3 ? t + k * kBlock : atomicAdd(&cnt[bk[k]], 1u);
      rec_o[pos] = o0[k];
      rec_l[pos] = (uint32_t)(o1[k] - o0[k]);
      rec_i[pos] = (uint16_t)(t + k * kBlock);
    }
    __syncthreads();
    // [C]
    uint64_t ko[KPT];
    uint32_t kl[KPT], ki[KPT];
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const uint32_t s = t + k * kBlock;
      ko[k] = rec_o[s]; kl[k] = rec_l[s]; ki[k] = rec_i[s];
    }
    for (uint32_t b = t; b < 320; b += blockDim.x) cnt[b] = 0;
    __syncthreads();  // records consumed: the area now stages hashes
    Blk pre[4] = {bzero(), bzero(), bzero(), bzero()};
    if (MODE != 2 && t < nw) prefetch_first(keys + ko[0], kl[0], pre);
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const uint32_t s = t + k * kBlock;
      Blk npre[4] = {bzero(), bzero(), bzero(), bzero()};
      if (MODE != 2 && k + 1 < KPT && s + kBlock < nw) prefetch_first(keys + ko[k + 1], kl[k + 1], npre);
      if (s < nw) {
        const LdsKV<LdsTab<NT>, 0> K(kfull, nofold, kl[k], s1, s2, T);
        Blk h;
        if constexpr (MODE == 1) h = bxor(bxor(pre[0], pre[1]), bxor(pre[2], pre[3]));
        else if constexpr (MODE == 2) {
          Blk sy[4];
          for (int q = 0; q < 4; q++) for (int w = 0; w < 4; w++) sy[q].w[w] = (uint32_t)ko[k] * 2654435761u + q * 4 + w;
          h = meow_var_pre(keys, kl[k] < 64 ? kl[k] : (kl[k] & 63), sy, K, T);
        } else h = meow_var_pre(keys + ko[k], kl[k], pre, K, T);
        if (fix) h = fixup(h);
        hout[ki[k]] = h;
      }
      if (k + 1 < KPT) {
#pragma unroll
        for (int q = 0; q < 4; q++) pre[q] = npre[q];
      }
    }
    __syncthreads();
    // [D]
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const uint32_t s = t + k * kBlock;
      if (s < nw) store_h<true>(out, base + s, hout[s], false);
    }
    __syncthreads();  // staging area reuse
  }
}

// k_var5: windows of 1024 keys; the window's contiguous key bytes are
// streamed into an LDS staging buffer by LDS-DMA (coalesced 1 KiB pieces)
// while the window is counting-sorted by length.  The sorted list is then
// cut into 16 WORK-BALANCED contiguous ranges, one per wave (work of a key ~
// its table rounds), and each wave hashes its range 64 lanes at a time:
// lanes of a step hold (nearly) equal lengths, and no wave idles at the
// window barrier while another hashes the longest keys.  Key bytes are read
// from LDS; hashes are staged in LDS in sorted order and written back
// through the inverse permutation as contiguous 16-byte runs.  (Gathering
// keys straight from HBM/L2 ran at ~2.4 TB/s; equal-size per-wave slices of
// the sorted list left 3/4 of the waves idle at the barrier.)  A window
// whose bytes exceed the staging buffer (~0.2 % for zipf 8-256 B keys)
// gathers from global memory instead.
template <int NT>
struct Var5Cfg {
  static constexpr int kTab = NT * 8192 * 4;
  static constexpr int kFull = kTab;                                 // VConst[kLT]
  static constexpr int kCnt = kFull + kLT * (int)sizeof(VConst);     // u32[320] counts -> bucket ends
  static constexpr int kWpre = kCnt + 320 * 4;                       // u32[321] work prefix per bucket
  static constexpr int kRecO = kWpre + 324 * 4;                      // u32[1024] offset in window
  static constexpr int kRecL = kRecO + kBlock * 4;                   // u16[1024]
  static constexpr int kRecI = kRecL + kBlock * 2;                   // u16[1024] sorted -> slot
  static constexpr int kInv = kRecI + kBlock * 2;                    // u16[1024] slot -> sorted
  static constexpr int kHout = kInv + kBlock * 2;                    // Blk[1024] hashes, sorted order
  static constexpr int kStage = kHout + kBlock * 16;                 // staging buffer
  static constexpr int S = ((163840 - kStage) / 1024) * 1024;
  static constexpr int kBytes = kStage + S;
  static_assert(kHout % 16 == 0 && kStage % 16 == 0, "alignment");
  static_assert(S >= 32768 && kBytes <= 163840, "LDS budget");
};

// work estimate of a length bucket: table rounds + load/store overhead
__device__ __forceinline__ uint32_t bucket_work(uint32_t b) {
  return b >= 300 ? 0u : 2u * ((b + 15u) >> 4) + 11u;
}

__device__ uint64_t g_dbg[4096 * 8];  // diagnostic stamps (STAMP builds only)

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int NT, bool STAMP = false>
__global__ void __launch_bounds__(kBlock)
k_var5(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
       uint64_t* __restrict__ out, uint32_t flags) {
  using C = Var5Cfg<NT>;
  __shared__ __attribute__((aligned(16))) uint32_t lds[C::kBytes / 4];
  VConst* kfull = (VConst*)((char*)lds + C::kFull);
  uint32_t* cnt = (uint32_t*)((char*)lds + C::kCnt);
  uint32_t* wpre = (uint32_t*)((char*)lds + C::kWpre);
  uint32_t* rec_o = (uint32_t*)((char*)lds + C::kRecO);
  uint16_t* rec_l = (uint16_t*)((char*)lds + C::kRecL);
  uint16_t* rec_i = (uint16_t*)((char*)lds + C::kRecI);
  uint16_t* inv = (uint16_t*)((char*)lds + C::kInv);
  Blk* hout = (Blk*)((char*)lds + C::kHout);
  uint8_t* stage = (uint8_t*)lds + C::kStage;
  fill_tables<NT>(lds);
  for (uint32_t b = threadIdx.x; b < 320; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)kLT; l += blockDim.x) {
    const MeowConst k = make_const(s1, s2, l, T);
    VConst v;
#pragma unroll
    for (int q = 0; q < 4; q++) { v.F[q] = k.F[q]; v.G[q] = k.G[q]; }
    v.TG2 = k.TG2; v.CS2b = k.CS2b; v.TCS0a = k.TCS0a;
    kfull[l] = v;
  }
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  constexpr uint32_t NWV = kBlock / 64;
  const uint64_t wstep = (uint64_t)gridDim.x * kBlock;
  uint64_t base = (uint64_t)blockIdx.x * kBlock;
  uint64_t po0 = 0, po1 = 0, pws = 0, pwe = 0;
  if (base < n) {
    const uint64_t wend = base + kBlock < n ? base + kBlock : n;
    if (base + t < n) { po0 = offs[base + t]; po1 = offs[base + t + 1]; }
    pws = offs[base]; pwe = offs[wend];
  }
  uint64_t acc[6] = {0, 0, 0, 0, 0, 0}, tp = 0;
  auto mark = [&](int ph) {
    if constexpr (STAMP) { const uint64_t x = stamp(); if (ph >= 0) acc[ph] += x - tp; tp = x; }
  };
  mark(-1);
  for (; base < n; base += wstep) {
    const uint64_t wend = base + kBlock < n ? base + kBlock : n;
    const uint32_t nw = (uint32_t)(wend - base);
    const uint64_t o0 = po0, o1 = po1, ws = pws, we = pwe;
    const uint64_t astart = ws & ~(uint64_t)15;
    const uint64_t span = we - astart;
    const bool staged = span <= (uint64_t)C::S;
    if (staged) {  // DMA the window bytes [astart, we) in 1 KiB pieces, wave-strided
      const uint32_t np = (uint32_t)((span + 1023) >> 10);
      for (uint32_t pc = wv; pc < np; pc += NWV) {
        const uint64_t src = astart + (uint64_t)pc * 1024 + 16 * lane;
        uint8_t* dst = stage + pc * 1024;
        if (src + 16 <= we) {
          __builtin_amdgcn_global_load_lds((const void*)(keys + src), (void __attribute__((address_space(3)))*)dst,
                                           16, 0, 2 /* nt */);
        } else if (src < we) {  // the piece holding the window's last byte: never read past it
          const uint32_t* q = (const uint32_t*)(keys + src);
          uint32_t* d = (uint32_t*)(dst + 16 * lane);
          for (uint32_t j = 0; j < 4; j++)
            if (src + 4 * j < we) d[j] = q[j];
        }
      }
    }
    mark(0);
    const uint64_t L = o1 - o0;
    const uint32_t bk = t < nw ? (L < 255 ? (uint32_t)L : 255u) : 300u;
    atomicAdd(&cnt[bk], 1u);
    __syncthreads();
    if (t < 64) {  // bucket starts and work prefix, one wave, 5 buckets per lane
      uint32_t v[5], sum = 0, wsum = 0;
#pragma unroll
      for (int k = 0; k < 5; k++) {
        v[k] = cnt[lane * 5 + k];
        sum += v[k];
        wsum += v[k] * bucket_work(lane * 5 + k);
      }
      uint32_t incl = sum, wincl = wsum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64), wy = __shfl_up(wincl, d, 64);
        if (lane >= (uint32_t)d) { incl += y; wincl += wy; }
      }
      uint32_t run = incl - sum, wrun = wincl - wsum;
#pragma unroll
      for (int k = 0; k < 5; k++) {
        cnt[lane * 5 + k] = run;
        wpre[lane * 5 + k] = wrun;
        run += v[k];
        wrun += v[k] * bucket_work(lane * 5 + k);
      }
      if (lane == 63) wpre[320] = wrun;
    }
    __syncthreads();
    {
      const uint32_t pos = atomicAdd(&cnt[bk], 1u);  // cnt[b] ends as the end of bucket b
      rec_o[pos] = (uint32_t)(o0 - astart);
      rec_l[pos] = (uint16_t)(L < 65535 ? L : 65535);
      rec_i[pos] = (uint16_t)t;
      inv[t] = (uint16_t)pos;
    }
    mark(1);
    wait_vmcnt<0>();  // this wave's DMA pieces have landed ...
    __syncthreads();  // ... and everyone's; records are complete
    mark(2);
    {  // prefetch the next window's offsets (lands while this window hashes)
      const uint64_t nb = base + wstep;
      if (nb < n) {
        const uint64_t nwend = nb + kBlock < n ? nb + kBlock : n;
        if (nb + t < n) { po0 = offs[nb + t]; po1 = offs[nb + t + 1]; }
        pws = offs[nb]; pwe = offs[nwend];
      }
    }
    // this wave's work-balanced range [lo, hi) of sorted positions
    const uint32_t TW = wpre[320];
    auto pos_of = [&](uint32_t x) -> uint32_t {  // first sorted position with work prefix >= x
      if (x >= TW) return nw;
      uint32_t lo = 0, hi = 319;                  // largest bucket b with wpre[b] <= x
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (wpre[mid] <= x) lo = mid; else hi = mid - 1;
      }
      const uint32_t b = lo, st = b ? cnt[b - 1] : 0u, en = cnt[b];
      const uint32_t w = bucket_work(b);
      uint32_t p = st + (w ? (x - wpre[b] + w - 1) / w : 0u);
      return p < en ? p : en;
    };
    const uint32_t lo = pos_of((uint32_t)(((uint64_t)TW * wv) / NWV));
    const uint32_t hi = wv + 1 == NWV ? nw : pos_of((uint32_t)(((uint64_t)TW * (wv + 1)) / NWV));
    for (uint32_t p0 = lo; p0 < hi; p0 += 64) {
      const uint32_t pos = p0 + lane;
      if (pos < hi) {
        const uint32_t ko = rec_o[pos], ki = rec_i[pos];
        uint32_t kl = rec_l[pos];
        Blk h;
        if (staged) {
          const LdsKV5<LdsTab<NT>> K(kfull, kl, s1, s2, T);
          h = meow_rt<LdsTab<NT>, LdsKV5<LdsTab<NT>>, LdsLd>(stage + ko, kl, K, T);
        } else {
          const uint64_t g0 = offs[base + ki];
          kl = (uint32_t)(offs[base + ki + 1] - g0);
          const LdsKV5<LdsTab<NT>> K(kfull, kl, s1, s2, T);
          h = meow_rt(keys + g0, kl, K, T);
        }
        if (fix) h = fixup(h);
        hout[pos] = h;
      }
    }
    mark(3);
    __syncthreads();
    mark(4);
    if (t < nw) store_h<true>(out, base + t, hout[inv[t]], false);
    for (uint32_t b = t; b < 320; b += blockDim.x) cnt[b] = 0;
    __syncthreads();  // staging areas reuse
    mark(5);
  }
  if constexpr (STAMP) {
    const uint32_t gw = blockIdx.x * (kBlock / 64) + wv;
    if (lane == 0 && gw < 4096)
      for (int q = 0; q < 6; q++) g_dbg[gw * 8 + q] = acc[q];
  }
}

// ------------------------------------------------------------ k_var6x
template <int NT, int WIN, bool PF = false, int NW = kBlock / 64, int SH = 0, bool PFS = false>
__global__ void __launch_bounds__(NW * 64)
k_var6x(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
       uint64_t* __restrict__ out, uint32_t flags) {
  using C = Var6Cfg<WIN, NW>;
  constexpr int M = WIN / 64;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ VConst kfull[kLT];
  __shared__ Blk kf[C::kWaves * C::kPerWave + LdsTab<NT>::kWords * 4 + kLT * sizeof(VConst) + kNF * 64 <= 163840
                    ? kNF * 4 : 1];  // F folds for 64 <= L < 320 when the LDS has room
  constexpr bool kHaveF = sizeof(kf) == kNF * 4 * sizeof(Blk);
  __shared__ __attribute__((aligned(16))) uint8_t wavemem[C::kWaves * C::kPerWave];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + (kHaveF ? kNF : 0)); l += blockDim.x) {
    if (l >= (uint32_t)kLT) {
      const Blk M = mixer(s1, s2, l);
#pragma unroll
      for (int q = 0; q < 4; q++) kf[(l - kLT) * 4 + q] = aesT(bxor(ramp(q), M), T);
      continue;
    }
    const MeowConst k = make_const(s1, s2, l, T);
    VConst v;
#pragma unroll
    for (int q = 0; q < 4; q++) { v.F[q] = k.F[q]; v.G[q] = k.G[q]; }
    v.TG2 = k.TG2; v.CS2b = k.CS2b; v.TCS0a = k.TCS0a;
    kfull[l] = v;
  }
  const Blk* ftab = kHaveF ? kf : nullptr;
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* hist = (uint32_t*)(wavemem + wv * C::kPerWave);
  uint32_t* r_off = hist + 256;
  uint32_t* r_len = r_off + WIN;
  uint32_t* r_idx = r_len + WIN;
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t gw = (uint64_t)blockIdx.x * C::kWaves + wv, tw = (uint64_t)gridDim.x * C::kWaves;
  for (uint64_t w = gw; w < nwin; w += tw) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const uint64_t ws = offs[i0];
    uint64_t o[M];
    uint32_t L[M], b[M], r[M];
    bool wide = false;
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      const uint64_t a = offs[i0 + (j < k ? j : k)], e = offs[i0 + (j < k ? j + 1 : k)];
      o[m] = a - ws;
      L[m] = (uint32_t)(e - a);
      wide |= e - ws >= (1ull << 32);
    }
    // A window spanning 4 GiB or more (some key of >= 16 MiB; a key of
    // >= 4 GiB): the records below hold u32 window offsets and lengths, so
    // this window is hashed in input order with u64 offsets and lengths
    // instead (wave-uniform), through the same hash call site.
    const bool wwin = __ballot(wide) != 0;
    if constexpr (PF || PFS) {
      if (wwin) { wide_window<NT>(keys, offs, i0, k, M, s1, s2, out, fix, lds); continue; }
    }
    if (!wwin) {
#pragma unroll
      for (int q = 0; q < 4; q++) hist[lane * 4 + q] = 0;
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        b[m] = (L[m] >> SH) < 255u ? (L[m] >> SH) : 255u;  // SH: see wave_sort_from
        r[m] = j < k ? atomicAdd(&hist[b[m]], 1u) : 0u;
      }
      wave_sync();
      {  // exclusive scan of the 256 bucket counts, 4 per lane
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) { v[q] = hist[lane * 4 + q]; sum += v[q]; }
        uint32_t inc = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(inc, d, 64);
          if (lane >= (uint32_t)d) inc += y;
        }
        uint32_t run = inc - sum;
#pragma unroll
        for (int q = 0; q < 4; q++) { hist[lane * 4 + q] = run; run += v[q]; }
      }
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        if (j < k) {
          const uint32_t pos = hist[b[m]] + r[m];
          r_off[pos] = (uint32_t)o[m];
          r_len[pos] = L[m];
          r_idx[pos] = j;
        }
      }
      wave_sync();
    }
    const uint8_t* base = keys + ws;
    if constexpr (PF) {
      // first 64 bytes of the next chunk's key are in flight while this
      // chunk hashes (meow_var_pre fetches later blocks one block ahead)
      Blk pre[4];
      {
        const uint32_t p0 = lane < k ? lane : k - 1;
        prefetch_first(base + r_off[p0], r_len[p0], pre);
      }
#pragma unroll
      for (int c = 0; c < M; c++) {
        const uint32_t pos = 64 * c + lane;
        const uint32_t pc = pos < k ? pos : k - 1;
        Blk nxt[4];
        if (c + 1 < M) {
          const uint32_t pn = pos + 64 < k ? pos + 64 : k - 1;
          prefetch_first(base + r_off[pn], r_len[pn], nxt);
        }
        const uint32_t kl = r_len[pc];
        const LdsKV5<LdsTab<NT>> K(kfull, kl, s1, s2, T);
        const Blk h = meow_var_pre(base + r_off[pc], kl, pre, K, T);
        if (pos < k) store_h<true>(out, i0 + r_idx[pos], h, fix);
        if (c + 1 < M) {
#pragma unroll
          for (int q = 0; q < 4; q++) pre[q] = nxt[q];
        }
      }
    } else {
      // hashes stay in registers until the window is done, then go through
      // the wave's (now free) record area to leave as one contiguous run:
      // scattered 16-byte stores in sorted order inflated HBM writes 1.76x
      Blk hs[M];
      uint32_t ix[M];
      Blk pre[4];
      if constexpr (PFS) {  // experiments: the first 64 bytes of the next chunk's key one chunk ahead
        const uint32_t p0 = lane < k ? lane : k - 1;
        prefetch_first(base + r_off[p0], r_len[p0], pre);
      }
#pragma unroll
      for (int c = 0; c < M; c++) {
        const uint32_t pos = 64 * c + lane;
        ix[c] = WIN;
        if constexpr (PFS) {
          Blk nxt[4];
          if (c + 1 < M) {
            const uint32_t pn = pos + 64 < k ? pos + 64 : k - 1;
            prefetch_first(base + r_off[pn], r_len[pn], nxt);
          }
          if (pos < k) {
            const uint32_t kl = r_len[pos];
            ix[c] = r_idx[pos];
            const LdsKV5<LdsTab<NT>> K(kfull, kl, s1, s2, T, ftab);
            hs[c] = meow_var_pre(base + r_off[pos], kl, pre, K, T);
            if (fix) hs[c] = fixup(hs[c]);
          }
          if (c + 1 < M) {
#pragma unroll
            for (int q = 0; q < 4; q++) pre[q] = nxt[q];
          }
          continue;
        }
        if (pos < k) {
          const uint8_t* p;
          uint64_t kl;
          if (!wwin) {
            p = base + r_off[pos];
            kl = r_len[pos];
            ix[c] = r_idx[pos];
          } else {
            const uint64_t a = offs[i0 + pos];
            p = keys + a;
            kl = offs[i0 + pos + 1] - a;
            ix[c] = pos;
          }
          const LdsKV5<LdsTab<NT>, uint64_t> K(kfull, kl, s1, s2, T, ftab);
          hs[c] = meow_rt(p, kl, K, T);
          if (fix) hs[c] = fixup(hs[c]);
        }
      }
      wave_sync();
      static_assert(C::kPerWave >= WIN * 16, "output staging fits the wave's area");
      Blk* stage = (Blk*)hist;
#pragma unroll
      for (int c = 0; c < M; c++)
        if (ix[c] < (uint32_t)WIN) stage[ix[c]] = hs[c];
      wave_sync();
#pragma unroll
      for (int c = 0; c < M; c++) {
        const uint32_t j = 64 * c + lane;
        if (j < k) store_h<true>(out, i0 + j, stage[j], false);
      }
    }
    wave_sync();  // records reused by the next window
  }
}

// ------------------------------------------------------------ k_var9x
// ABL (counter-only builds, outputs are not hashes): 1 = hash stage written
// in sorted order (no slot scatter), 3 = per-length constants read for the
// wave's first lane's length (no lane-divergent constant reads), 4 = window
// ranks by 6 ballots "match any" + one atomic per distinct class (no
// same-address atomics; outputs ARE hashes).  ST: 0 = LDS hash stage, 1 =
// hashes stored straight to their slots (normal stores), 2 = the same
// non-temporal.
template <int NT, int NW, int KF, bool PF = false, bool PR = false, int ABL = 0, int ST = 0, int SB = 4>
__global__ void __launch_bounds__(NW * 64)
k_var9x(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
       uint64_t* __restrict__ out, uint32_t flags) {
  // per wave: the hash stage (4 KiB); while sorting it holds the bucket counts
  // (first KiB) and the sorted records (last 2 KiB), which each lane then
  // takes into registers (its four sorted positions) before hashes land
  constexpr int WIN = 256, M = WIN / 64, AREA = WIN * 16;
  // one LDS object, tables first: a lookup address is then the v_perm result
  // itself (a table at a nonzero base costs one v_add per lookup)
  constexpr int kTabB = LdsTab<NT>::kWords * 4, kFullB = kLT * (int)sizeof(VConst9), kKfB = KF * 64;
  constexpr int kBytes = kTabB + kFullB + kKfB + NW * AREA;
  static_assert(kBytes <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint32_t smem[kBytes / 4];
  uint32_t* lds = smem;
  VConst9* kfull = (VConst9*)((uint8_t*)smem + kTabB);
  Blk* kf = (Blk*)((uint8_t*)smem + kTabB + kFullB);
  uint8_t* wavemem = (uint8_t*)smem + kTabB + kFullB + kKfB;
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + KF); l += blockDim.x) {
    if (l >= (uint32_t)kLT) {
      const Blk Mx = mixer(s1, s2, l);
#pragma unroll
      for (int q = 0; q < 4; q++) kf[kf_index(l, q)] = aesT(bxor(ramp(q), Mx), T);
      continue;
    }
    const MeowConst k = make_const(s1, s2, l, T);
    VConst9 v;
#pragma unroll
    for (int q = 0; q < 4; q++) { v.F[q] = k.F[q]; v.G[q] = k.G[q]; }
    v.TG2 = k.TG2; v.TCS0a = k.TCS0a;
    kfull[l] = v;
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Blk* stage = (Blk*)(wavemem + wv * AREA);
  uint32_t* hist = (uint32_t*)stage;
  uint2* rec = (uint2*)(wavemem + wv * AREA + WIN * 8);
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + wv, tw = (uint64_t)gridDim.x * NW;
  const uint64_t kend = offs[n];  // the buffer holds every byte up to the last key's end
  for (uint64_t w = gw; w < nwin; w += tw) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const uint64_t ws = offs[i0];
    const uint64_t wend = kend - ws;  // window-relative
    uint32_t o[M], L[M], r[M], b[M];
    bool wide = false;
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      const uint64_t a = offs[i0 + (j < k ? j : k)], e = offs[i0 + (j < k ? j + 1 : k)];
      o[m] = (uint32_t)(a - ws);
      L[m] = (uint32_t)(e - a);
      wide |= e - ws >= (1ull << 32) || e - a >= (1ull << 24);
    }
    if (__ballot(wide) != 0) {  // wave-uniform
      wide_window<NT>(keys, offs, i0, k, M, s1, s2, out, fix, lds);
      continue;
    }
    // counting sort of the window by 16-byte length class
#pragma unroll
    for (int q = 0; q < SB; q++) hist[lane * SB + q] = 0;
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      if constexpr (ABL == 4) {  // ranks by ballots; counters at class * 4 (sub-counter 0)
        const bool v = j < k;
        const uint32_t cls = (L[m] >> 4) < 63u ? (L[m] >> 4) : 63u;
        b[m] = cls * 4u;
        uint64_t eq = __ballot(v);
#pragma unroll
        for (int bit = 0; bit < 6; bit++) {
          const uint64_t B = __ballot((cls >> bit) & 1u);
          eq &= ((cls >> bit) & 1u) ? B : ~B;
        }
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(eq >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)eq, 0u));
        uint32_t bs = 0;
        if (v && below == 0) bs = atomicAdd(&hist[b[m]], (uint32_t)__popcll(eq));
        const uint32_t lead = v ? (uint32_t)__builtin_ctzll(eq) : lane;
        bs = __shfl(bs, lead, 64);
        r[m] = bs + below;
        continue;
      }
      // 64 length classes x 4 sub-counters by lane & 3: a quarter of the
      // same-address atomics (a class's keys in one instruction serialise)
      b[m] = ((L[m] >> 4) < 63u ? (L[m] >> 4) : 63u) * (uint32_t)SB + (lane & (uint32_t)(SB - 1));
      r[m] = j < k ? atomicAdd(&hist[b[m]], 1u) : 0u;
    }
    wave_sync();
    {
      uint32_t v[SB], sum = 0;
#pragma unroll
      for (int q = 0; q < SB; q++) { v[q] = hist[lane * SB + q]; sum += v[q]; }
      uint32_t inc = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
      uint32_t run = inc - sum;
#pragma unroll
      for (int q = 0; q < SB; q++) { hist[lane * SB + q] = run; run += v[q]; }
    }
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      if (j < k) rec[hist[b[m]] + r[m]] = make_uint2(o[m], (L[m] << 8) | j);
    }
    wave_sync();
    // this lane's sorted positions lane, 64 + lane, ... (rotated through
    // scalars below: a register array indexed in a rolled loop is scratch)
    uint2 rc0 = rec[lane], rc1 = rec[64 + lane], rc2 = rec[128 + lane], rc3 = rec[192 + lane];
    wave_sync();  // the stage takes hashes from here on
    const uint8_t* base = keys + ws;
#pragma unroll 1
    for (int c = 0; c < M; c++) {
      const uint32_t pos = 64 * c + lane;
      const bool valid = pos < k;
      const uint2 rc = rc0;
      rc0 = rc1; rc1 = rc2; rc2 = rc3;
      const uint32_t kl = valid ? rc.y >> 8 : 0u;
      const bool al = __ballot(kl >= 64u) != 0;
      const int cm = __ballot((kl & 48u) == 48u) ? 48 : __ballot((kl & 48u) >= 32u) ? 32
                   : __ballot((kl & 48u) >= 16u) ? 16 : 0;
      if constexpr (PR) {  // experiments: long keys two lanes per key (meow_pair), the chunk as two 32-key halves
      if (al) {
        const auto sx = __builtin_amdgcn_permlane32_swap(rc.x, rc.x, false, false);
        const auto sy = __builtin_amdgcn_permlane32_swap(rc.y, rc.y, false, false);
        const uint32_t hh = lane >> 5;
#pragma unroll 1
        for (int ps = 0; ps < 2; ps++) {
          const uint32_t px = ps ? sx[1] : sx[0], py = ps ? sy[1] : sy[0];
          const bool v2 = 64 * c + 32 * ps + (lane & 31) < k;
          const uint32_t o2 = v2 ? px : 0u, kl2 = v2 ? py >> 8 : 0u;
          const LdsKV9<LdsTab<NT>, KF> K2(kfull, kf, kl2, s1, s2, T);
          const Blk h2 = meow_pair(base + o2, kl2, hh, (uint64_t)o2 + kl2 + 16 <= wend, K2, T);
          if (v2 && hh == 0) stage[py & 255u] = fix ? fixup(h2) : h2;
        }
        continue;
      }
      }
      if (valid) {
        const uint8_t* p = base + rc.x;
        const bool safe = (uint64_t)rc.x + kl + 16 <= wend;  // whole dwordx4 groups stay in the buffer
        const LdsKV9<LdsTab<NT>, KF> K(kfull, kf, ABL == 3 ? rfl(kl) : kl, s1, s2, T);
        Blk h;
        if (al) h = meow_a<true, 48, PF>(p, kl, safe, K, T);
        else if (cm == 48) h = meow_a<false, 48, PF>(p, kl, safe, K, T);
        else if (cm == 32) h = meow_a<false, 32, PF>(p, kl, safe, K, T);
        else if (cm == 16) h = meow_a<false, 16, PF>(p, kl, safe, K, T);
        else h = meow_a<false, 0, PF>(p, kl, safe, K, T);
        if constexpr (ST == 1) store_h<false>(out, i0 + (rc.y & 255u), h, fix);
        else if constexpr (ST == 2) store_h<true>(out, i0 + (rc.y & 255u), h, fix);
        else stage[ABL == 1 ? pos : (rc.y & 255u)] = fix ? fixup(h) : h;
      }
    }
    if constexpr (ST == 0) {
      wave_sync();
#pragma unroll
      for (int c = 0; c < M; c++) {
        const uint32_t j = 64 * c + lane;
        if (j < k) store_h<true>(out, i0 + j, stage[j], false);
      }
    }
    wave_sync();  // stage and records reused by the next window
  }
}


// ---------------------------------------------------------------------
// k_var10: k_var9 with larger per-wave windows (WIN = 512 or 1024 keys).
// A divergence model over the C2 lengths (one chunk of 64 sorted keys runs
// as long as the meow_a variant its longest / widest key needs) gives 1.59x
// the ideal lane-rounds at 256-key windows, 1.29x at 512, 1.16x at 1024.
// LDS per wave is the sorted records only (8 B per key; the class counters
// live in the same area while sorting): hashes are stored straight to their
// slots (NTS: non-temporal) instead of through a 16 B/key LDS stage.  Record
// = (window byte offset, length << LB | slot), LB = log2(WIN); a window
// spanning 4 GiB or holding a key of 2^(32-LB) bytes or more takes
// wide_window.  Offsets: one u64 per key per lane (the end offset of key j
// is the start of key j+1: a lane shuffle).
template <int NT, int NW, int KF, int WIN, bool NTS>
__global__ void __launch_bounds__(NW * 64)
k_var10(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
        uint64_t* __restrict__ out, uint32_t flags) {
  constexpr int M = WIN / 64, AREA = WIN * 8;
  constexpr int LB = WIN == 256 ? 8 : WIN == 512 ? 9 : 10;
  static_assert((1 << LB) == WIN, "window size");
  static_assert(AREA >= 1024, "class counters fit the record area");
  constexpr int kTabB = LdsTab<NT>::kWords * 4, kFullB = kLT * (int)sizeof(VConst9), kKfB = KF * 64;
  constexpr int kBytes = kTabB + kFullB + kKfB + NW * AREA;
  static_assert(kBytes <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint32_t smem[kBytes / 4];
  uint32_t* lds = smem;
  VConst9* kfull = (VConst9*)((uint8_t*)smem + kTabB);
  Blk* kf = (Blk*)((uint8_t*)smem + kTabB + kFullB);
  uint8_t* wavemem = (uint8_t*)smem + kTabB + kFullB + kKfB;
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + KF); l += blockDim.x) {
    if (l >= (uint32_t)kLT) {
      const Blk Mx = mixer(s1, s2, l);
#pragma unroll
      for (int q = 0; q < 4; q++) kf[kf_index(l, q)] = aesT(bxor(ramp(q), Mx), T);
      continue;
    }
    const MeowConst kc = make_const(s1, s2, l, T);
    VConst9 v;
#pragma unroll
    for (int q = 0; q < 4; q++) { v.F[q] = kc.F[q]; v.G[q] = kc.G[q]; }
    v.TG2 = kc.TG2; v.TCS0a = kc.TCS0a;
    kfull[l] = v;
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint2* rec = (uint2*)(wavemem + wv * AREA);
  uint32_t* hist = (uint32_t*)rec;
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + wv, tw = (uint64_t)gridDim.x * NW;
  const uint64_t kend = offs[n];
  for (uint64_t w = gw; w < nwin; w += tw) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const uint64_t ws = offs[i0];
    const uint64_t wend = kend - ws;
    uint32_t o[M], L[M], b[M], r[M];
    bool wide = false;
    {
      uint64_t a[M];
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        a[m] = offs[i0 + (j < k ? j : k)];
      }
      const uint64_t last = offs[i0 + k];
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        uint64_t e = __shfl_down(a[m], 1, 64);
        const uint64_t nx = m + 1 < M ? __shfl(a[m + 1 < M ? m + 1 : m], 0, 64) : last;
        if (lane == 63) e = nx;
        if (j >= k) e = a[m];
        o[m] = (uint32_t)(a[m] - ws);
        L[m] = (uint32_t)(e - a[m]);
        wide |= e - ws >= (1ull << 32) || e - a[m] >= (1ull << (32 - LB));
      }
    }
    if (__ballot(wide) != 0) {
      wide_window<NT>(keys, offs, i0, k, M, s1, s2, out, fix, lds);
      continue;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) hist[lane * 4 + q] = 0;
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      b[m] = ((L[m] >> 4) < 63u ? (L[m] >> 4) : 63u) * 4u + (lane & 3u);
      r[m] = j < k ? atomicAdd(&hist[b[m]], 1u) : 0u;
    }
    wave_sync();
    {
      uint32_t v[4], sum = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) { v[q] = hist[lane * 4 + q]; sum += v[q]; }
      uint32_t inc = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
      uint32_t run = inc - sum;
#pragma unroll
      for (int q = 0; q < 4; q++) { hist[lane * 4 + q] = run; run += v[q]; }
    }
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) r[m] += hist[b[m]];  // final sorted positions
    wave_sync();  // the counters are overwritten by records below
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      if (j < k) rec[r[m]] = make_uint2(o[m], (L[m] << LB) | j);
    }
    wave_sync();
    const uint8_t* base = keys + ws;
#pragma unroll 1
    for (int c = 0; c < M; c++) {
      const uint32_t pos = 64 * c + lane;
      if (64u * c >= k) break;  // wave-uniform
      const bool valid = pos < k;
      const uint2 rc = rec[valid ? pos : 0];
      const uint32_t kl = valid ? rc.y >> LB : 0u;
      const bool al = __ballot(kl >= 64u) != 0;
      const int cm = __ballot((kl & 48u) == 48u) ? 48 : __ballot((kl & 48u) >= 32u) ? 32
                   : __ballot((kl & 48u) >= 16u) ? 16 : 0;
      if (valid) {
        const uint8_t* p = base + rc.x;
        const bool safe = (uint64_t)rc.x + kl + 16 <= wend;
        const LdsKV9<LdsTab<NT>, KF> K(kfull, kf, kl, s1, s2, T);
        Blk h;
        if (al) h = meow_a<true, 48, false>(p, kl, safe, K, T);
        else if (cm == 48) h = meow_a<false, 48, false>(p, kl, safe, K, T);
        else if (cm == 32) h = meow_a<false, 32, false>(p, kl, safe, K, T);
        else if (cm == 16) h = meow_a<false, 16, false>(p, kl, safe, K, T);
        else h = meow_a<false, 0, false>(p, kl, safe, K, T);
        store_h<NTS>(out, i0 + (rc.y & (WIN - 1)), h, fix);
      }
    }
    wave_sync();  // records reused by the next window
  }
}

// ---------------------------------------------------------------------
// k_var8: k_var6's length-sorted per-wave windows, hashed as balanced
// per-state CHAINS.  Until Compress, Meow's four states never meet: state s
// absorbs its own 16-byte column of every 64-byte block, its own trail chunk
// and its own Mix round (key_hash.c:1155-1160, 1200-1226).  Per (key, state)
// that is a chain of nch = nb + (trail chunk of s ? 1 : 0) units over the
// chain's chunks c_0..c_{nch-1}:
//   X = F_s ^ c_0 (the folded first absorb), then for u < nch
//   X = AESDEC(AESDEC(X, c_u), u + 1 < nch ? c_{u+1} : M)
// (the round-key sequence c_0 | c_1 c_1 | ... | c_last c_last | M paired up).
// A lane runs four chains back to back -- state 0 of key l, 1 of key 63-l,
// 2 of key l^32, 3 of key (63-l)^32 in the chunk's length order -- so its
// work is a sum over a short and a long key, not one key's trip count and
// trail branches: a chunk of 64 sorted zipf 8-256 B keys costs 1.23x the
// ideal lane-rounds (simulated), k_var6's one key per lane 1.68x.  The four
// states of key l then return to lane l by lane shuffles for Compress and
// the final round (per key, in-lane).
// MEASURED AND REJECTED (experiments build, knob 7 = 18/19; C2 on one
// MI355X, outputs equal to k_var6): 4.92 ms (one unit per step, loads at
// use), 4.88 ms (loads one unit ahead, conditional), 9.85 ms (this version:
// unconditional buffer loads, double-buffered) against k_var6's 3.02 ms.
// LDS instructions fell only 10 % (F folds at every chain start, the state
// exchange and the tail add back most of the saved lookups), VALU rose
// 44-80 % (slot bookkeeping, chunk extraction) and the per-unit gathers
// doubled the wait time.
__device__ __forceinline__ uint32_t chain_deal(uint32_t l, int s) {
  return s == 0 ? l : s == 1 ? 63u - l : s == 2 ? l ^ 32u : (63u - l) ^ 32u;
}
// units of state s's chain for a key of L bytes: one per full block, plus
// its trail chunk (s < 3: the full chunk at 16 s when L & 48 > 16 s; s = 3:
// the partial tail)
__device__ __forceinline__ uint32_t chain_units(uint32_t L, int s) {
  const uint32_t C = L & 48u, t = L & 15u;
  return (L >> 6) + (s < 3 ? (C > 16u * (uint32_t)s ? 1u : 0u) : (t ? 1u : 0u));
}
// A chain chunk as loaded: the 5 dwords from the dword-aligned address at or
// below it (a buffer load off the window's base), with its byte shift and
// valid byte count; extracted only where it is used, so the load stays in
// flight until then.  Chunk u of state s's chain: the state's column of block
// u, or its trail chunk (s = 3: the t-byte tail at 64 nb + C, zero padded).
struct RawChunk {
  uint32_t d[5], sn;  // sn = byte shift | valid bytes << 8
};
__device__ __forceinline__ RawChunk chain_ld(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t L, uint32_t s,
                                             uint32_t u) {
  const bool tail3 = s == 3 && u == (L >> 6);
  const uint32_t a = off + 64u * u + (tail3 ? (L & 48u) : 16u * s);
  const uint32_t q = a & ~3u;
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, q, 0, 0);
  RawChunk c;
  c.d[0] = v[0]; c.d[1] = v[1]; c.d[2] = v[2]; c.d[3] = v[3];
  c.d[4] = __builtin_amdgcn_raw_buffer_load_b32(r, q + 16, 0, 0);
  c.sn = (a & 3u) | ((tail3 ? (L & 15u) : 16u) << 8);
  return c;
}
__device__ __forceinline__ Blk chain_fix(const RawChunk& c) {
  const uint32_t sh = c.sn & 3u, nbytes = c.sn >> 8;
  // bytes [nbytes, 16) are zero: 64-bit masks of the low and high halves
  const uint64_t mlo = nbytes >= 8 ? ~0ull : (1ull << (8 * nbytes)) - 1;
  const uint64_t mhi = nbytes >= 16 ? ~0ull : nbytes <= 8 ? 0ull : (1ull << (8 * (nbytes - 8))) - 1;
  Blk x;
  x.w[0] = __builtin_amdgcn_alignbyte(c.d[1], c.d[0], sh) & (uint32_t)mlo;
  x.w[1] = __builtin_amdgcn_alignbyte(c.d[2], c.d[1], sh) & (uint32_t)(mlo >> 32);
  x.w[2] = __builtin_amdgcn_alignbyte(c.d[3], c.d[2], sh) & (uint32_t)mhi;
  x.w[3] = __builtin_amdgcn_alignbyte(c.d[4], c.d[3], sh) & (uint32_t)(mhi >> 32);
  return x;
}

// A lane's chains, compacted: slot 0 is the running chain, slot 1 the next.
struct ChainSlot {
  uint32_t off, len, st, nu;  // key offset in the window, key length, state, units
};
__device__ __forceinline__ void slot_shift(ChainSlot (&q)[4], bool go) {
#pragma unroll
  for (int i = 0; i < 3; i++) {
    q[i].off = go ? q[i + 1].off : q[i].off;
    q[i].len = go ? q[i + 1].len : q[i].len;
    q[i].st = go ? q[i + 1].st : q[i].st;
    q[i].nu = go ? q[i + 1].nu : q[i].nu;
  }
  q[3].nu = go ? 0u : q[3].nu;
}

// The chunks of the lane's next unit, requested one unit ahead: chunk 0 of
// the next chain (used when the running chain ends with this unit) and the
// next unit's second-round chunk.  Unconditional loads (addresses clamped to
// the chain's own chunks): no branch splits the wait counters.
struct UnitLoads {
  RawChunk c0, c1;
};
__device__ __forceinline__ UnitLoads chain_prefetch(__amdgpu_buffer_rsrc_t r, const ChainSlot (&q)[4], uint32_t u,
                                                    bool last) {
  const uint32_t o2 = last ? q[1].off : q[0].off, L2 = last ? q[1].len : q[0].len,
                 s2 = last ? q[1].st : q[0].st, n2 = last ? q[1].nu : q[0].nu, u2 = last ? 0u : u + 1;
  UnitLoads n;  // chunk 0 of the chain after the one the next unit runs
  n.c0 = chain_ld(r, last ? q[2].off : q[1].off, last ? q[2].len : q[1].len, last ? q[2].st : q[1].st, 0);
  n.c1 = chain_ld(r, o2, L2, s2, u2 + 1 < n2 ? u2 + 1 : 0u);
  return n;
}

// One unit of the lane's running chain (slot 0, unit u): two rounds, with
// the chunks loaded one unit earlier (cur); then the lane advances.
template <int NT>
__device__ __forceinline__ void chain_unit(ChainSlot (&q)[4], uint32_t& u, bool act, Blk& X, Blk& K1,
                                           const UnitLoads& cur, Blk (&Q)[4], uint64_t s1, uint64_t s2,
                                           const LdsTab<NT>& T, const VConst* kfull, const Blk* ftab) {
  const uint32_t L = q[0].len, st = q[0].st;
  const bool last = u + 1 >= q[0].nu;
  const Blk Mx = mixer(s1, s2, L);
  if (u == 0) {  // chain start: the folded first absorb
    Blk F;
    if (L < (uint32_t)kLT) F = kfull[L].F[st];
    else if (ftab && L < (uint32_t)(kLT + kNF)) F = ftab[(L - kLT) * 4 + st];
    else F = aesT(bxor(ramp((int)st), Mx), T);
    X = bxor(F, K1);
  }
  const Blk D = last ? Mx : chain_fix(cur.c1);
  X = aesdec(aesdec(X, K1, T), D, T);
  if (act && last) {
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (st == (uint32_t)i) Q[i] = X;
  }
  K1 = last ? chain_fix(cur.c0) : D;
  slot_shift(q, act && last);
  u = last ? 0u : u + 1;
}

// One chunk of 64 length-sorted keys (records [c0, c0 + 64) of the wave's
// window, k valid): returns the hash of key c0 + lane (garbage past k).
template <int NT>
__device__ __forceinline__ Blk chain_hash_chunk(__amdgpu_buffer_rsrc_t rs, const uint32_t* r_off,
                                                const uint32_t* r_len, uint32_t c0, uint32_t k, uint64_t s1,
                                                uint64_t s2, const LdsTab<NT>& T, const VConst* kfull,
                                                const Blk* ftab) {
  const uint32_t lane = threadIdx.x & 63;
  ChainSlot q[4];
  uint32_t total = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = ChainSlot{0u, 0u, 0u, 0u};
#pragma unroll
  for (int s = 3; s >= 0; s--) {  // push the non-empty chains to the front, state order
    const uint32_t pos = c0 + chain_deal(lane, s);
    const bool v = pos < k;
    const uint32_t L = v ? r_len[pos] : 0u, o = v ? r_off[pos] : 0u;
    const uint32_t nu = v ? chain_units(L, s) : 0u;
    total += nu;
    const bool push = nu != 0;
#pragma unroll
    for (int i = 3; i > 0; i--) {
      q[i].off = push ? q[i - 1].off : q[i].off;
      q[i].len = push ? q[i - 1].len : q[i].len;
      q[i].st = push ? q[i - 1].st : q[i].st;
      q[i].nu = push ? q[i - 1].nu : q[i].nu;
    }
    q[0].off = push ? o : q[0].off;
    q[0].len = push ? L : q[0].len;
    q[0].st = push ? (uint32_t)s : q[0].st;
    q[0].nu = push ? nu : q[0].nu;
  }
  uint32_t umax = total;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) umax = max(umax, (uint32_t)__shfl_xor((int)umax, o, 64));
  Blk Q[4], X = bzero();
#pragma unroll
  for (int i = 0; i < 4; i++) Q[i] = bzero();
  // the first unit's chunks: chunk 0 (K1) and chunk 1 of the first chain
  Blk K1 = chain_fix(chain_ld(rs, q[0].off, q[0].len, q[0].st, 0));
  UnitLoads A, B;
  A.c0 = chain_ld(rs, q[1].off, q[1].len, q[1].st, 0);
  A.c1 = chain_ld(rs, q[0].off, q[0].len, q[0].st, q[0].nu > 1 ? 1u : 0u);
  uint32_t u = 0;
  // two units per trip with alternating load sets: the loads for unit i + 1
  // are issued before unit i's rounds and consumed after them
  for (uint32_t step = 0; step < umax; step += 2) {
    B = chain_prefetch(rs, q, u, u + 1 >= q[0].nu);
    chain_unit<NT>(q, u, step < total, X, K1, A, Q, s1, s2, T, kfull, ftab);
    if (step + 1 < umax) {
      A = chain_prefetch(rs, q, u, u + 1 >= q[0].nu);
      chain_unit<NT>(q, u, step + 1 < total, X, K1, B, Q, s1, s2, T, kfull, ftab);
    }
  }
  // key c0 + lane: its states from the lanes that ran them
  Blk S[4];
  S[0] = Q[0];
#pragma unroll
  for (int s = 1; s < 4; s++) {
    const int src = (int)chain_deal(lane, s);
#pragma unroll
    for (int w = 0; w < 4; w++) S[s].w[w] = (uint32_t)__shfl((int)Q[s].w[w], src, 64);
  }
  const uint32_t pos = c0 + lane;
  const uint32_t L = pos < k ? r_len[pos] : 0u;
  const Blk M = mixer(s1, s2, L);
  const VConst& kc = kfull[L < (uint32_t)kLT ? L : (uint32_t)kLT - 1];
  const bool T0 = chain_units(L, 0) != 0, T1 = chain_units(L, 1) != 0, T2 = chain_units(L, 2) != 0,
             T3 = chain_units(L, 3) != 0;
  const Blk S0 = T0 ? S[0] : kc.G[0], S1 = T1 ? S[1] : kc.G[1], S2 = T2 ? S[2] : kc.G[2],
            S3 = T3 ? S[3] : kc.G[3];
  Blk S2b;
  if (T2) S2b = aesdec(aesdec(S2, S3, T), M, T);
  else if (T3) S2b = aesdec(bxor(kc.TG2, S3), M, T);
  else S2b = kc.CS2b;
  Blk S0b;
  if (T0) S0b = aesdec(aesdec(S0, S1, T), S2b, T);
  else S0b = bxor(kc.TCS0a, S2b);
  return aesdec(S0b, M, T);
}

template <int NT, int WIN, int SH = 4>
__global__ void __launch_bounds__(kBlock)
k_var8(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
       uint64_t* __restrict__ out, uint32_t flags) {
  using C = Var6Cfg<WIN>;
  constexpr int M = WIN / 64;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ VConst kfull[kLT];
  __shared__ Blk kf[C::kWaves * C::kPerWave + LdsTab<NT>::kWords * 4 + kLT * sizeof(VConst) + kNF * 64 <= 163840
                    ? kNF * 4 : 1];
  constexpr bool kHaveF = sizeof(kf) == kNF * 4 * sizeof(Blk);
  __shared__ __attribute__((aligned(16))) uint8_t wavemem[C::kWaves * C::kPerWave];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + (kHaveF ? kNF : 0)); l += blockDim.x) {
    if (l >= (uint32_t)kLT) {
      const Blk Mx = mixer(s1, s2, l);
#pragma unroll
      for (int q = 0; q < 4; q++) kf[kf_index(l, q)] = aesT(bxor(ramp(q), Mx), T);
      continue;
    }
    const MeowConst kc = make_const(s1, s2, l, T);
    VConst v;
#pragma unroll
    for (int q = 0; q < 4; q++) { v.F[q] = kc.F[q]; v.G[q] = kc.G[q]; }
    v.TG2 = kc.TG2; v.CS2b = kc.CS2b; v.TCS0a = kc.TCS0a;
    kfull[l] = v;
  }
  const Blk* ftab = kHaveF ? kf : nullptr;
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* hist = (uint32_t*)(wavemem + wv * C::kPerWave);
  uint32_t* r_off = hist + 256;
  uint32_t* r_len = r_off + WIN;
  uint32_t* r_idx = r_len + WIN;
  const uint64_t kend_off = offs[n];
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t gw = (uint64_t)blockIdx.x * C::kWaves + wv, tw = (uint64_t)gridDim.x * C::kWaves;
  for (uint64_t w = gw; w < nwin; w += tw) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const uint64_t ws = offs[i0];
    uint64_t o[M];
    uint32_t L[M], b[M], r[M];
    bool wide = false;
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      const uint64_t a = offs[i0 + (j < k ? j : k)], e = offs[i0 + (j < k ? j + 1 : k)];
      o[m] = a - ws;
      L[m] = (uint32_t)(e - a);
      wide |= e - ws >= (1ull << 32);
    }
    // a window of >= 4 GiB (u32 records), or one within 64 bytes of the
    // batch's last key byte (the chunk loads read whole dwords past a key's
    // end): u64 offsets, input order, byte-exact loads (see k_var6)
    const uint64_t we = offs[i0 + k];
    if (__ballot(wide) != 0 || we + 64 > kend_off) {
      wide_window<NT>(keys, offs, i0, k, M, s1, s2, out, fix, lds);
      continue;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) hist[lane * 4 + q] = 0;
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      b[m] = (L[m] >> SH) < 255u ? (L[m] >> SH) : 255u;
      r[m] = j < k ? atomicAdd(&hist[b[m]], 1u) : 0u;
    }
    wave_sync();
    {
      uint32_t v[4], sum = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) { v[q] = hist[lane * 4 + q]; sum += v[q]; }
      uint32_t inc = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
      uint32_t run = inc - sum;
#pragma unroll
      for (int q = 0; q < 4; q++) { hist[lane * 4 + q] = run; run += v[q]; }
    }
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      if (j < k) {
        const uint32_t pos = hist[b[m]] + r[m];
        r_off[pos] = (uint32_t)o[m];
        r_len[pos] = L[m];
        r_idx[pos] = j;
      }
    }
    wave_sync();
    // the window's bytes as a buffer: 32-bit offsets, no 64-bit address math
    const uint64_t span = kend_off - ws;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(keys + ws), (short)0, (int)(span < 0xffffffffull ? span : 0xffffffffull), 0x00020000);
    Blk hs[M];
    uint32_t ix[M];
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t pos = 64 * c + lane;
      hs[c] = chain_hash_chunk<NT>(rs, r_off, r_len, 64 * c, k, s1, s2, T, kfull, ftab);
      if (fix) hs[c] = fixup(hs[c]);
      ix[c] = pos < k ? r_idx[pos] : (uint32_t)WIN;
    }
    wave_sync();
    Blk* stage = (Blk*)hist;
#pragma unroll
    for (int c = 0; c < M; c++)
      if (ix[c] < (uint32_t)WIN) stage[ix[c]] = hs[c];
    wave_sync();
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t j = 64 * c + lane;
      if (j < k) store_h<true>(out, i0 + j, stage[j], false);
    }
    wave_sync();
  }
}


// ---------------------------------------------------------------------
// k_var7: k_var6's per-wave length-class windows with the LDS traffic that
// the round-1 counters charged to it removed:
//  * ranking without LDS atomics on shared addresses: a key's class c =
//    min(len >> 4, 63) (16-byte length class: same full-block count, so the
//    same trip counts; the stable counting sort keeps a class in address
//    order).  The lanes of one 64-key sub-chunk that share c are found with
//    6 ballots (one per bit of c, "match any"); the lowest of them adds the
//    group's size to hist[c] (one LDS atomic per distinct class, at distinct
//    addresses) and broadcasts the old count; each lane's rank is that plus
//    its mbcnt in the group.  64 buckets: one per lane, one-wave scan.
//    (k_var6: 256 buckets, one same-address atomic per key: 8-15 B keys,
//    16 % of them 8 B, all land in bucket 0.)
//  * per-length constants as one 16-byte array per field (F0..F3, G0..G3,
//    TG2, CS2b, TCS0a for L < 64; F0..F3 for 64 <= L < 320) instead of
//    176-byte / 64-byte records: lanes of a sorted chunk read lengths that
//    differ by less than 8, which map to disjoint 4-bank groups.
//  * the 4 GiB check from the lanes' offsets (one ballot), no extra load.
template <class Tab, class LenT = uint32_t>
struct LdsKV7 {
  const Blk* c;  // field-major constant arrays, see k_var7
  LenT L;
  Blk m;
  const Tab& T;
  static constexpr int kF = 0, kG = 4 * kLT, kTG2 = 8 * kLT, kCS2b = 9 * kLT, kTCS0a = 10 * kLT, kFF = 11 * kLT;
  static constexpr int kWords = 11 * kLT + 4 * kNF;  // Blk entries
  __device__ __forceinline__ LdsKV7(const Blk* cc, LenT len, uint64_t s1, uint64_t s2, const Tab& t)
      : c(cc), L(len), m(mixer(s1, s2, len)), T(t) {}
  __device__ __forceinline__ uint32_t li() const { return L < (LenT)kLT ? (uint32_t)L : (uint32_t)kLT - 1; }
  __device__ __forceinline__ Blk M() const { return m; }
  __device__ __forceinline__ Blk F(int i) const {
    if (L < (LenT)kLT) return c[kF + i * kLT + (uint32_t)L];
    if (L < (LenT)(kLT + kNF)) return c[kFF + i * kNF + (uint32_t)(L - kLT)];
    return aesT(bxor(ramp(i), m), T);
  }
  __device__ __forceinline__ Blk G(int i) const { return c[kG + i * kLT + li()]; }
  __device__ __forceinline__ Blk TG2() const { return c[kTG2 + li()]; }
  __device__ __forceinline__ Blk CS2b() const { return c[kCS2b + li()]; }
  __device__ __forceinline__ Blk TCS0a() const { return c[kTCS0a + li()]; }
};

template <int NT, int WIN = 256, int NW = kBlock / 64, int HV = 0>
__global__ void __launch_bounds__(NW * 64)
k_var7(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
       uint64_t* __restrict__ out, uint32_t flags) {
  using KC = LdsKV7<LdsTab<NT>>;
  constexpr int M = WIN / 64;
  constexpr int kNB = 64;                          // length classes
  constexpr int kRec = kNB * 4 + WIN * 12;         // hist + u32 off, len, idx
  constexpr int kPerWave = kRec > WIN * 16 ? kRec : WIN * 16;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ Blk kc[KC::kWords];
  __shared__ __attribute__((aligned(16))) uint8_t wavemem[NW * kPerWave];
  static_assert(sizeof(lds) + sizeof(kc) + sizeof(wavemem) <= 163840, "LDS budget");
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + kNF); l += blockDim.x) {
    if (l >= (uint32_t)kLT) {
      const Blk Mx = mixer(s1, s2, l);
#pragma unroll
      for (int q = 0; q < 4; q++) kc[KC::kFF + q * kNF + (l - kLT)] = aesT(bxor(ramp(q), Mx), T);
      continue;
    }
    const MeowConst k = make_const(s1, s2, l, T);
#pragma unroll
    for (int q = 0; q < 4; q++) { kc[KC::kF + q * kLT + l] = k.F[q]; kc[KC::kG + q * kLT + l] = k.G[q]; }
    kc[KC::kTG2 + l] = k.TG2; kc[KC::kCS2b + l] = k.CS2b; kc[KC::kTCS0a + l] = k.TCS0a;
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* hist = (uint32_t*)(wavemem + wv * kPerWave);
  uint32_t* r_off = hist + kNB;
  uint32_t* r_len = r_off + WIN;
  uint32_t* r_idx = r_len + WIN;
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + wv, tw = (uint64_t)gridDim.x * NW;
  for (uint64_t w = gw; w < nwin; w += tw) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const uint64_t ws = offs[i0];
    uint32_t o[M], L[M], b[M], r[M];
    bool wide = false;
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      const uint64_t a = offs[i0 + (j < k ? j : k)], e = offs[i0 + (j < k ? j + 1 : k)];
      o[m] = (uint32_t)(a - ws);
      L[m] = (uint32_t)(e - a);
      wide |= e - ws >= (1ull << 32);
    }
    // A window spanning 4 GiB or more (a key of >= 16 MiB) cannot use the
    // u32 window-relative records: it is hashed in input order with u64
    // offsets and lengths through the same hash call site (no second copy
    // of the round code: k_var6's inlined u64 path cost 32 VGPR spills).
    const bool wwin = __ballot(wide) != 0;
    if (!wwin) {
      hist[lane] = 0;
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        const bool v = j < k;
        b[m] = (L[m] >> 4) < (uint32_t)(kNB - 1) ? (L[m] >> 4) : (uint32_t)(kNB - 1);
        uint64_t eq = __ballot(v);
#pragma unroll
        for (int bit = 0; bit < 6; bit++) {
          const uint64_t B = __ballot((b[m] >> bit) & 1u);
          eq &= ((b[m] >> bit) & 1u) ? B : ~B;
        }
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(eq >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)eq, 0u));
        uint32_t base = 0;
        if (v && below == 0) base = atomicAdd(&hist[b[m]], (uint32_t)__popcll(eq));
        const uint32_t lead = v ? (uint32_t)__builtin_ctzll(eq) : lane;
        base = __shfl(base, lead, 64);
        r[m] = base + below;
      }
      wave_sync();
      {  // exclusive scan of the 64 class counts, one per lane
        const uint32_t cnt = hist[lane];
        uint32_t inc = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(inc, d, 64);
          if (lane >= (uint32_t)d) inc += y;
        }
        hist[lane] = inc - cnt;
      }
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        if (j < k) {
          const uint32_t pos = hist[b[m]] + r[m];
          r_off[pos] = o[m];
          r_len[pos] = L[m];
          r_idx[pos] = j;
        }
      }
      wave_sync();
    }
    Blk hs[M];
    uint32_t ix[M];
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t pos = 64 * c + lane;
      ix[c] = WIN;
      if (pos < k) {
        const uint8_t* p;
        uint64_t kl;
        if (!wwin) {
          p = keys + ws + r_off[pos];
          kl = r_len[pos];
          ix[c] = r_idx[pos];
        } else {
          const uint64_t a = offs[i0 + pos];
          p = keys + a;
          kl = offs[i0 + pos + 1] - a;
          ix[c] = pos;
        }
        const LdsKV7<LdsTab<NT>, uint64_t> K(kc, kl, s1, s2, T);
        // HV 1: every load of the key issued before its rounds (meow_var)
        if constexpr (HV == 1) hs[c] = meow_var(p, kl, K, T);
        else hs[c] = meow_rt(p, kl, K, T);
        if (fix) hs[c] = fixup(hs[c]);
      }
    }
    wave_sync();
    Blk* stage = (Blk*)hist;  // records consumed: the wave's area stages the hashes in input order
#pragma unroll
    for (int c = 0; c < M; c++)
      if (ix[c] < (uint32_t)WIN) stage[ix[c]] = hs[c];
    wave_sync();
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t j = 64 * c + lane;
      if (j < k) store_h<true>(out, i0 + j, stage[j], false);
    }
    wave_sync();  // staging read before the next window's histogram
  }
}

// ---------------------------------------------------------------------
// k_hybrid: the LDS T-table round and the bitsliced VALU round (bs_meow.hpp)
// side by side in one workgroup per CU.  The T-table keys are bound by the
// LDS lookup rate (16 ds_read_b32 per key-round) with the VALU about a third
// busy; the bitsliced keys need no LDS at all.  Waves [0, 16-NBW) hash keys
// [nB, n) exactly like k_fixed (wave-chunked, U keys per lane); waves
// [16-NBW, 16) hash keys [0, nB) in batches of 512 (lane l takes keys
// b + 64j + l, j < 8: every load/store instruction moves a contiguous 1 KiB
// run).  nB is a multiple of 512 chosen by the host (kvh_set_tuning knob 11:
// the bitsliced share in per mille).
template <int L, int NT, int U, int NBW, int PRIO = 2>
__global__ void __launch_bounds__(kBlock)
k_hybrid(const uint8_t* __restrict__ keys, uint64_t n, uint64_t nB, uint64_t s1, uint64_t s2,
         uint64_t* __restrict__ out, uint32_t flags) {
  static_assert(L == 16 || L == 32 || L == 48, "hybrid: 16, 32 or 48-byte keys");
  constexpr int NC = L / 16;
  constexpr int NTW = kBlock / 64 - NBW;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t wv = threadIdx.x >> 6;
  const uint64_t lane = threadIdx.x & 63;
  if (wv < (uint32_t)NTW) {
    // the LDS-bound waves win VALU issue arbitration; the bitsliced waves
    // fill the VALU slots they leave
    if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
    const uint64_t gw = (uint64_t)blockIdx.x * NTW + wv, tw = (uint64_t)gridDim.x * NTW;
    const uint64_t last = n - 1;
    for (uint64_t b = nB + gw * 64 * U; b < n; b += tw * 64 * U) {
      Blk D[U][NC];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t j = b + 64 * u + lane;
        load_fixed<L, true, true>(keys + (j < last ? j : last) * L, D[u]);
      }
      Blk h[U];
#pragma unroll
      for (int u = 0; u < U; u++) h[u] = meow_ct<L>(D[u], K, T);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t j = b + 64 * u + lane;
        store_h<true>(out, j < last ? j : last, h[u], fix);
      }
    }
  } else {
    // constant masks, lane t < 32 holds register t's (bs_meow.hpp KeySrc)
    bs::KeySrc ks;
    {
      const uint32_t t = (uint32_t)lane & 31u;
      const uint32_t zero[4] = {0, 0, 0, 0};
      auto mk = [&](const Blk& z, int kind) {
        const uint32_t zz[4] = {z.w[0], z.w[1], z.w[2], z.w[3]};
        return bs::mask_of(zz, t, kind);
      };
      ks.lv[bs::KeySrc::kZero] = bs::mask_of(zero, t, bs::kKap);
      ks.lv[bs::KeySrc::kA0] = mk(K.F[0], bs::kKapX);
      ks.lv[bs::KeySrc::kA1] = mk(K.F[1], bs::kKapX);
      ks.lv[bs::KeySrc::kA2] = mk(K.F[2], bs::kKapX);
      ks.lv[bs::KeySrc::kM] = mk(K.M, bs::kKap);
      ks.lv[bs::KeySrc::kG1] = mk(K.G[1], bs::kKap);
      ks.lv[bs::KeySrc::kG3] = mk(K.G[3], bs::kKap);
      ks.lv[bs::KeySrc::kCS2b] = mk(K.CS2b, bs::kKap);
      ks.lv[bs::KeySrc::kMstd] = mk(K.M, bs::kStd);
    }
    const uint64_t gw = (uint64_t)blockIdx.x * NBW + (wv - NTW), tw = (uint64_t)gridDim.x * NBW;
    for (uint64_t b = gw * 512; b < nB; b += tw * 512) {
      uint32_t w[NC][8][4];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint8_t* p = keys + (b + 64 * j + lane) * L;
#pragma unroll
        for (int c = 0; c < NC; c++) {
          const v4u v = __builtin_nontemporal_load((const v4u*)(p + 16 * c));
          w[c][j][0] = v.x; w[c][j][1] = v.y; w[c][j][2] = v.z; w[c][j][3] = v.w;
        }
      }
      uint32_t h[8][4];
      bs::meow_bs<L>(w, ks, h);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        Blk x;
        x.w[0] = h[j][0]; x.w[1] = h[j][1]; x.w[2] = h[j][2]; x.w[3] = h[j][3];
        store_h<true>(out, b + 64 * j + lane, x, fix);
      }
    }
  }
}


// ---------------------------------------------------------------------
// k_hybrid_lanes (round 3): config C3 (32-byte keys, 4 seeds per key,
// kv_hash_meow128_4_same_length_4_seed with one key in all slots) with NBW
// of the 16 waves running the bitsliced VALU round (bs_meow.hpp) on keys
// [0, nB) and the others k_fixed_lanes' T-table code (LA = 4 lanes per key)
// on the hash slots [4 nB, 4 n).  The bitsliced constant masks are
// wave-uniform, so a bitsliced wave hashes each batch of 512 keys under
// the four seeds in turn (the keys re-read from L2), storing slot 4 i + a
// with normal stores (the four passes fill each line in L2).
template <int NT, int U, int NBW, int PRIO>
__global__ void __launch_bounds__(kBlock)
k_hybrid_lanes(const uint8_t* __restrict__ keys, uint64_t n, uint64_t nB, uint64_t* __restrict__ out, uint32_t flags,
               uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1, uint64_t a2, uint64_t b2, uint64_t a3,
               uint64_t b3) {
  constexpr int L = 32, NC = 2, SH = 2, NTW = kBlock / 64 - NBW;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ uint32_t bmask[4][bs::KeySrc::kN][32];  // per seed: register t's constant mask
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t wv = threadIdx.x >> 6;
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t sa[4] = {a0, a1, a2, a3}, sb[4] = {b0, b1, b2, b3};
  if (wv == (uint32_t)NTW) {
    const uint32_t t = (uint32_t)lane & 31u;
    const uint32_t zero[4] = {0, 0, 0, 0};
    auto mk = [&](const Blk& z, int kind) {
      const uint32_t zz[4] = {z.w[0], z.w[1], z.w[2], z.w[3]};
      return bs::mask_of(zz, t, kind);
    };
#pragma unroll 1
    for (int a = 0; a < 4; a++) {
      const MeowConst K = uniform(make_const(sa[a], sb[a], (uint64_t)L, T));
      uint32_t v[bs::KeySrc::kN];
      v[bs::KeySrc::kZero] = bs::mask_of(zero, t, bs::kKap);
      v[bs::KeySrc::kA0] = mk(K.F[0], bs::kKapX);
      v[bs::KeySrc::kA1] = mk(K.F[1], bs::kKapX);
      v[bs::KeySrc::kA2] = mk(K.F[2], bs::kKapX);
      v[bs::KeySrc::kM] = mk(K.M, bs::kKap);
      v[bs::KeySrc::kG1] = mk(K.G[1], bs::kKap);
      v[bs::KeySrc::kG3] = mk(K.G[3], bs::kKap);
      v[bs::KeySrc::kCS2b] = mk(K.CS2b, bs::kKap);
      v[bs::KeySrc::kMstd] = mk(K.M, bs::kStd);
      if (lane < 32)
#pragma unroll
        for (int q = 0; q < bs::KeySrc::kN; q++) bmask[a][q][t] = v[q];
    }
  }
  __syncthreads();
  if (wv < (uint32_t)NTW) {
    if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
    const uint32_t sl = threadIdx.x & 3;
    uint64_t s1 = sa[0], s2 = sb[0];
#pragma unroll
    for (int q = 1; q < 4; q++)
      if (sl == (uint32_t)q) { s1 = sa[q]; s2 = sb[q]; }
    const MeowConst K = make_const(s1, s2, (uint64_t)L, T);
    const uint64_t gw = (uint64_t)blockIdx.x * NTW + wv, tw = (uint64_t)gridDim.x * NTW;
    const uint64_t ns = n << SH, lastk = n - 1;
    for (uint64_t b = (nB << SH) + gw * 64 * U; b < ns; b += tw * 64 * U) {
      Blk D[U][NC];
      uint64_t slot[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t kk = (b + 64 * u + lane) >> SH;
        kk = kk < lastk ? kk : lastk;
        slot[u] = (kk << SH) | sl;
        load_fixed<L, true, true>(keys + kk * L, D[u]);
      }
      Blk h[U];
#pragma unroll
      for (int u = 0; u < U; u++) h[u] = meow_ct<L>(D[u], K, T);
#pragma unroll
      for (int u = 0; u < U; u++) store_h<true>(out, slot[u], h[u], fix);
    }
  } else {
    const uint64_t gw = (uint64_t)blockIdx.x * NBW + (wv - NTW), tw = (uint64_t)gridDim.x * NBW;
    for (uint64_t b = gw * 512; b < nB; b += tw * 512) {
#pragma unroll 1
      for (int a = 0; a < 4; a++) {
        bs::KeySrc cur;
#pragma unroll
        for (int q = 0; q < bs::KeySrc::kN; q++) cur.lv[q] = bmask[a][q][lane & 31];
        uint32_t w[NC][8][4];
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const uint8_t* p = keys + (b + 64 * j + lane) * L;
#pragma unroll
          for (int c = 0; c < NC; c++) {
            const v4u v = *(const v4u*)(p + 16 * c);
            w[c][j][0] = v.x; w[c][j][1] = v.y; w[c][j][2] = v.z; w[c][j][3] = v.w;
          }
        }
        uint32_t h[8][4];
        bs::meow_bs<L>(w, cur, h);
#pragma unroll
        for (int j = 0; j < 8; j++) {
          Blk x;
          x.w[0] = h[j][0]; x.w[1] = h[j][1]; x.w[2] = h[j][2]; x.w[3] = h[j][3];
          store_h<false>(out, ((b + 64 * j + lane) << SH) | (uint64_t)a, x, fix);
        }
      }
    }
  }
}

// ------------------------------------------------------------ host side
using Knob = std::atomic<int>;
Knob g_tune_pf{0};        // k_fixed: 1 = register prefetch of the next chunk
Knob g_tune_bs{0};        // hybrid kernel: bitsliced share of the keys in per mille (0 = k_fixed)
Knob g_tune_bsw{4};       // hybrid kernel: bitsliced waves per 16-wave workgroup
Knob g_tune_prio{2};      // hybrid kernel: s_setprio of the T-table waves (0, 2, 3)
Knob g_tune_ablate{0};    // ablation build of k_fixed (0 = product path)
Knob g_tune_dma{0};       // LDS-DMA ring depth for L in {16, 32} (0 = register path)
Knob g_tune_var_mode{0};  // ablation of k_var3: 1 no-hash, 2 no-gather, 3 no-sort

// knob() and grid_for() are the product's (kvh_internal.hpp)

template <int L, int NT, int U, int MODE = 0, bool PF = false>
int launch_k(const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out, uint32_t flags,
             hipStream_t st, int cus) {
  const bool a16 = ((uintptr_t)keys & 15) == 0;
  const uint32_t grid = grid_for(n, cus, NT == 4 ? 1 : 2);
  if (a16)
    hipLaunchKernelGGL((k_fixed_x<L, NT, true, U, MODE, PF>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out,
                       flags);
  else
    hipLaunchKernelGGL((k_fixed_x<L, NT, false, U, MODE, PF>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2,
                       out, flags);
  return launch_done();
}

// ---------------------------------------------------------------------
// k_var11 + k_var11_q: k_var9 with the divergence of its sorted chunks cut
// by DEFERRAL.  A chunk of 64 class-sorted keys runs as long as its longest
// key, and in a 256-key window the 4th chunk holds the ~61 keys of 64 B or
// more (24 % of C2's keys, lengths 64..256): it costs the longest key's
// rounds for all of them.  A divergence model over the C2 lengths
//  gives 16.3 lane-rounds per key for k_var9 against 10.2
// ideal; with the keys of 64..319 B, and each window's remainder chunk of at
// most REM short keys, sent to per-class queues and hashed there in
// class-uniform chunks (every lane of a chunk has the same block count and
// trail shape), 11.9.
//  * k_var11 (windows): a wave pushes its window's long keys to ITS OWN
//    queue region (no global atomics: one region per wave of the grid),
//    counting-sorts the rest by class as k_var9 does, pushes the partial last
//    chunk (<= REM keys) too, and hashes only full chunks.  A region is a
//    bump-allocated array of 64-record blocks; each class has one open block
//    whose (block, fill) lives in lane `class` of one VGPR.  A record is
//    16 B {offset lo, offset hi, length, index}.  A key whose push finds the
//    region full is hashed in the window as before.  The window's hash run
//    is stored whole (deferred slots carry stale stage words), so its stores
//    stay full lines;
//  * k_var11_q (queues): one wave per region, one block at a time, every
//    lane of a block the same class, so the straight-line meow_a variant is
//    exact for all of them; each hash overwrites its slot in `out`.
// Reference semantics are unchanged (key_hash.c:1155-1226): both kernels
// hash with meow_a and the same folded constants.
constexpr int kQCls = 20;  // deferred classes 0..19 (keys of 0..319 bytes)

struct VarQ {
  uint4* rec;       // [regions][rb][64]: {offset lo, offset hi, length, index}
  uint32_t* meta;   // [regions][rb]: class << 8 | count
  uint32_t* nblk;   // [regions]: blocks used
  uint32_t rb;      // blocks per region
};

// Window sort buckets: the short classes first, then the classes hashed in
// the window whatever happens (keys of 320 B and more), then the deferrable
// long classes 4..19 -- so the keys hashed in the window are one prefix of
// the sorted order and the deferred ones one suffix.
__device__ __forceinline__ uint32_t v11_bucket(uint32_t c) {
  return c < 4u ? c : c >= (uint32_t)kQCls ? 4u + (c - kQCls < 27u ? c - kQCls : 27u) : 32u + (c - 4u);
}

template <int NT, int NW, int REM>
__global__ void __launch_bounds__(NW * 64)
k_var11(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
        uint64_t* __restrict__ out, uint32_t flags, VarQ q) {
  constexpr int WIN = 256, M = WIN / 64, AREA = WIN * 16;
  // no first-absorb fold table: keys of 64 B or more are hashed here only
  // when their region is full (or they are 320 B and longer): folds in-lane
  constexpr int kTabB = LdsTab<NT>::kWords * 4, kFullB = kLT * (int)sizeof(VConst9);
  constexpr int kBytes = kTabB + kFullB + NW * AREA;
  static_assert(kBytes <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint32_t smem[kBytes / 4];
  uint32_t* lds = smem;
  VConst9* kfull = (VConst9*)((uint8_t*)smem + kTabB);
  uint8_t* wavemem = (uint8_t*)smem + kTabB + kFullB;
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)kLT; l += blockDim.x) {
    const MeowConst k = make_const(s1, s2, l, T);
    VConst9 v;
#pragma unroll
    for (int i = 0; i < 4; i++) { v.F[i] = k.F[i]; v.G[i] = k.G[i]; }
    v.TG2 = k.TG2; v.TCS0a = k.TCS0a;
    kfull[l] = v;
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Blk* stage = (Blk*)(wavemem + wv * AREA);
  uint32_t* hist = (uint32_t*)stage;
  uint2* rec = (uint2*)(wavemem + wv * AREA + WIN * 8);
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + wv, tw = (uint64_t)gridDim.x * NW;
  const uint64_t kend = offs[n];
  uint4* const qrec = q.rec + gw * q.rb * 64;
  uint32_t* const qmeta = q.meta + gw * q.rb;
  // lane c < kQCls: class c's open block << 16 | its fill (64: none open)
  uint32_t qs = 0xffffu << 16 | 64u, nb = 0;
  for (uint64_t w = gw; w < nwin; w += tw) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const uint64_t ws = offs[i0];
    const uint64_t wend = kend - ws;
    uint32_t kk, d0;  // keys of the window; the sorted positions [d0, kk) go to the queues
    {
      uint32_t o[M], L[M], r[M], b[M];
      bool wide = false;
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        const uint64_t a = offs[i0 + (j < k ? j : k)], e = offs[i0 + (j < k ? j + 1 : k)];
        o[m] = (uint32_t)(a - ws);
        L[m] = (uint32_t)(e - a);
        wide |= e - ws >= (1ull << 32) || e - a >= (1ull << 24);
      }
      if (__ballot(wide) != 0) {
        wide_window<NT>(keys, offs, i0, k, M, s1, s2, out, fix, lds);
        continue;
      }
#pragma unroll
      for (int i = 0; i < 4; i++) hist[lane * 4 + i] = 0;
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        b[m] = v11_bucket(L[m] >> 4) * 4u + (lane & 3u);
        r[m] = j < k ? atomicAdd(&hist[b[m]], 1u) : 0u;
      }
      wave_sync();
      {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) { v[i] = hist[lane * 4 + i]; sum += v[i]; }
        uint32_t inc = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(inc, d, 64);
          if (lane >= (uint32_t)d) inc += y;
        }
        uint32_t run = inc - sum;
#pragma unroll
        for (int i = 0; i < 4; i++) { hist[lane * 4 + i] = run; run += v[i]; }
        kk = __builtin_amdgcn_readlane(inc, 63);
      }
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        if (j < k) rec[hist[b[m]] + r[m]] = make_uint2(o[m], (L[m] << 8) | j);
      }
      wave_sync();
    }
    // the split: long classes, plus the partial last chunk of short keys
    // when it is small and holds no key that must stay
    const uint32_t x = __builtin_amdgcn_readfirstlane(hist[32 * 4]);    // start of the deferrable buckets
    const uint32_t xs = __builtin_amdgcn_readfirstlane(hist[4 * 4]);    // end of the short classes
    const uint32_t rem = x & 63u;
    d0 = rem != 0 && rem <= (uint32_t)REM && xs == x ? x - rem : x;
    if (nb + kQCls + M > q.rb) d0 = kk;  // region nearly full: this window keeps its keys
    if (d0 < kk) {
      // per class c (lane c): its run [cb, ce) of the deferred suffix
      uint32_t cb = 0, cnt = 0;
      if (lane < (uint32_t)kQCls) {
        const uint32_t bk = v11_bucket(lane);
        const uint32_t s0 = hist[bk * 4], e0 = hist[bk * 4 + 4];
        cb = s0 > d0 ? s0 : d0;
        cnt = e0 > cb ? e0 - cb : 0u;
      }
      // block placement, one class at a time (wave-uniform): fill the open
      // block, then consecutive new blocks from the region's bump pointer
      uint32_t pl = 0, pb = 0;  // lane c: open block << 16 | fill before, first new block
      uint64_t cm = __ballot(cnt != 0);
      while (cm) {
        const uint32_t c = (uint32_t)__builtin_ctzll(cm);
        cm &= cm - 1;
        const uint32_t cc = __builtin_amdgcn_readlane(cnt, c);
        const uint32_t st = __builtin_amdgcn_readlane(qs, c);
        const uint32_t blk = st >> 16, fill = st & 0xffffu;
        const uint32_t n1 = cc < 64u - fill ? cc : 64u - fill;
        const uint32_t nnew = (cc - n1 + 63u) >> 6, nbase = nb;
        nb += nnew;
        const uint32_t lastfill = nnew ? cc - n1 - 64u * (nnew - 1u) : fill + n1;
        const uint32_t lastblk = nnew ? nbase + nnew - 1u : blk;
        if (lane == 0 && n1 != 0 && fill + n1 == 64u) qmeta[blk] = c << 8 | 64u;
        if (lane < nnew && (lane + 1u < nnew || lastfill == 64u)) qmeta[nbase + lane] = c << 8 | 64u;
        if (lane == c) { pl = st; pb = nbase; qs = lastblk << 16 | lastfill; }
      }
      // records of the deferred suffix to their blocks (the shuffles run in
      // every lane: ds_bpermute reads nothing from a lane that is off)
#pragma unroll
      for (int m = 0; m < M; m++) {
        if (d0 + 64u * m >= kk) break;  // wave-uniform
        const uint32_t p = d0 + lane + 64 * m;
        const bool v = p < kk;
        const uint2 rr = rec[v ? p : d0];
        const uint32_t kl = rr.y >> 8, c = kl >> 4;
        const uint32_t rank = p - (uint32_t)__shfl((int)cb, (int)c, 64);
        const uint32_t st = (uint32_t)__shfl((int)pl, (int)c, 64), fill = st & 0xffffu;
        const uint32_t nbc = (uint32_t)__shfl((int)pb, (int)c, 64);
        uint32_t blk, pos;
        if (rank < 64u - fill) { blk = st >> 16; pos = fill + rank; }
        else {
          const uint32_t r2 = rank - (64u - fill);
          blk = nbc + (r2 >> 6);
          pos = r2 & 63u;
        }
        const uint64_t off = ws + rr.x;
        if (v) qrec[blk * 64 + pos] = make_uint4((uint32_t)off, (uint32_t)(off >> 32), kl, (uint32_t)(i0 + (rr.y & 255u)));
      }
    }
    wave_sync();
    uint2 rc0 = rec[lane], rc1 = rec[64 + lane], rc2 = rec[128 + lane], rc3 = rec[192 + lane];
    wave_sync();  // the stage takes hashes from here on
    const uint8_t* base = keys + ws;
    const uint32_t nch = (d0 + 63) >> 6;
#pragma unroll 1
    for (uint32_t c = 0; c < nch; c++) {
      const uint32_t pos = 64 * c + lane;
      const bool valid = pos < d0;
      const uint2 rc = rc0;
      rc0 = rc1; rc1 = rc2; rc2 = rc3;
      const uint32_t kl = valid ? rc.y >> 8 : 0u;
      const bool al = __ballot(kl >= 64u) != 0;
      const int cm = __ballot((kl & 48u) == 48u) ? 48 : __ballot((kl & 48u) >= 32u) ? 32
                   : __ballot((kl & 48u) >= 16u) ? 16 : 0;
      if (valid) {
        const uint8_t* p = base + rc.x;
        const bool safe = (uint64_t)rc.x + kl + 16 <= wend;
        const LdsKV9<LdsTab<NT>, 0> K(kfull, nullptr, kl, s1, s2, T);
        Blk h;
        if (al) h = meow_a<true, 48, false>(p, kl, safe, K, T);
        else if (cm == 48) h = meow_a<false, 48, false>(p, kl, safe, K, T);
        else if (cm == 32) h = meow_a<false, 32, false>(p, kl, safe, K, T);
        else if (cm == 16) h = meow_a<false, 16, false>(p, kl, safe, K, T);
        else h = meow_a<false, 0, false>(p, kl, safe, K, T);
        stage[rc.y & 255u] = fix ? fixup(h) : h;
      }
    }
    wave_sync();
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t j = 64 * c + lane;
      if (j < k) store_h<true>(out, i0 + j, stage[j], false);
    }
    wave_sync();
  }
  // close the open blocks; the region's block count
  if (lane < (uint32_t)kQCls) {
    const uint32_t blk = qs >> 16, fill = qs & 0xffffu;
    if (fill < 64u) qmeta[blk] = lane << 8 | fill;
  }
  if (lane == 0) q.nblk[gw] = nb;
}

// Per-length constants for k_var11_q: full records for L < kLT, the
// swizzled first-absorb folds for kLT <= L < kLT + KF, in-lane beyond.  F0
// (the folded first trail round of a key without a full block) is only
// selected when nb == 0, which a chunk of a long class never has.
template <class Tab, int KF>
struct LdsKQ {
  const VConst9* full;
  const Blk* ftab;
  uint32_t L;
  Blk m;
  const Tab& T;
  __device__ __forceinline__ LdsKQ(const VConst9* f, const Blk* ft, uint32_t len, uint64_t s1, uint64_t s2,
                                   const Tab& t)
      : full(f), ftab(ft), L(len), m(mixer(s1, s2, len)), T(t) {}
  __device__ __forceinline__ uint32_t li() const { return L < (uint32_t)kLT ? L : (uint32_t)kLT - 1; }
  __device__ __forceinline__ Blk M() const { return m; }
  __device__ __forceinline__ Blk F(int i) const {
    if (L < (uint32_t)kLT) return full[L].F[i];
    if (L < (uint32_t)(kLT + KF)) return ftab[kf_index(L, i)];
    return aesT(bxor(ramp(i), m), T);
  }
  __device__ __forceinline__ Blk F0(int) const { return bzero(); }
  __device__ __forceinline__ Blk G(int i) const { return full[li()].G[i]; }
  __device__ __forceinline__ Blk TG2() const { return full[li()].TG2; }
  __device__ __forceinline__ Blk TCS0a() const { return full[li()].TCS0a; }
};

template <int NT, int NW, bool PF>
__global__ void __launch_bounds__(NW * 64)
k_var11_q(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ kendp, uint64_t s1, uint64_t s2, uint64_t* __restrict__ out,
          uint32_t flags, VarQ q, uint64_t regions) {
  constexpr int KF = 16 * kQCls - kLT;
  constexpr int kTabB = LdsTab<NT>::kWords * 4, kFullB = kLT * (int)sizeof(VConst9), kKfB = KF * 64;
  constexpr int kBytes = kTabB + kFullB + kKfB;
  static_assert(kBytes <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint32_t smem[kBytes / 4];
  uint32_t* lds = smem;
  VConst9* kfull = (VConst9*)((uint8_t*)smem + kTabB);
  Blk* kf = (Blk*)((uint8_t*)smem + kTabB + kFullB);
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + KF); l += blockDim.x) {
    if (l >= (uint32_t)kLT) {
      const Blk Mx = mixer(s1, s2, l);
#pragma unroll
      for (int i = 0; i < 4; i++) kf[kf_index(l, i)] = aesT(bxor(ramp(i), Mx), T);
      continue;
    }
    const MeowConst k = make_const(s1, s2, l, T);
    VConst9 v;
#pragma unroll
    for (int i = 0; i < 4; i++) { v.F[i] = k.F[i]; v.G[i] = k.G[i]; }
    v.TG2 = k.TG2; v.TCS0a = k.TCS0a;
    kfull[l] = v;
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + wv, tw = (uint64_t)gridDim.x * NW;
  const uint64_t kend = *kendp;  // offsets[n]: the buffer holds every byte up to the last key's end
  for (uint64_t rg = gw; rg < regions; rg += tw) {
    const uint32_t nb = q.nblk[rg];
    const uint4* rb = q.rec + rg * q.rb * 64;
    uint4 nx = nb ? rb[lane] : make_uint4(0, 0, 0, 0);  // next block's record, one block ahead
#pragma unroll 1
    for (uint32_t b = 0; b < nb; b++) {
      const uint32_t meta = __builtin_amdgcn_readfirstlane(q.meta[rg * q.rb + b]);
      const uint4 rc = nx;
      if (b + 1 < nb) nx = rb[(b + 1) * 64 + lane];
      const uint32_t c = meta >> 8, cnt = meta & 255u;
      if (lane < cnt) {
        const uint64_t off = (uint64_t)rc.y << 32 | rc.x;
        const uint32_t kl = rc.z;
        const uint8_t* p = keys + off;
        const bool safe = off + kl + 16 <= kend;
        const LdsKQ<LdsTab<NT>, KF> K(kfull, kf, kl, s1, s2, T);
        Blk h;
        switch (c & 3u | (c >= 4u ? 4u : 0u)) {  // class-uniform: the exact variant of every lane
          case 0: h = meow_a<false, 0, false>(p, kl, safe, K, T); break;
          case 1: h = meow_a<false, 16, false>(p, kl, safe, K, T); break;
          case 2: h = meow_a<false, 32, false>(p, kl, safe, K, T); break;
          case 3: h = meow_a<false, 48, false>(p, kl, safe, K, T); break;
          case 4: h = meow_a<true, 0, PF>(p, kl, safe, K, T); break;
          case 5: h = meow_a<true, 16, PF>(p, kl, safe, K, T); break;
          case 6: h = meow_a<true, 32, PF>(p, kl, safe, K, T); break;
          default: h = meow_a<true, 48, PF>(p, kl, safe, K, T); break;
        }
        store_h(out, rc.w, h, fix);
      }
    }
  }
}

// ---------------------------------------------------------------------
// k_var12: k_var11's deferral in ONE kernel, each wave its own consumer.
// k_var11 + k_var11_q cut the LDS instructions by 22 % and still lost (4.5
// vs 3.0 ms): the queue kernel found the long keys' lines cold and had no
// short-key work to hide the waits behind (53 % of its wave time waiting).
// Here a wave hashes a class block as soon as it is full -- right after the
// window that filled it, while those keys' lines are recent -- so every wave
// keeps k_var9's mix of short-key chunks and (now class-uniform) long-key
// chunks.  A wave's queue is 64 blocks of 64 records in its own slice of a
// scratch buffer (<= 20 open blocks + <= 24 filled per window, so it never
// runs out); free blocks are a 64-bit mask.  The window's hash run is stored
// first (deferred slots carry stale stage words), then, after a fence, the
// filled blocks overwrite their slots; at the end the open blocks are hashed.
template <int NT, class K2, int KF>
__device__ __forceinline__ void v12_block(const uint8_t* __restrict__ keys, uint64_t kend, const uint4* blk,
                                          uint32_t c, uint32_t cnt, uint64_t s1, uint64_t s2,
                                          uint64_t* __restrict__ out, bool fix, const VConst9* kfull,
                                          const Blk* kf, const LdsTab<NT>& T) {
  const uint32_t lane = threadIdx.x & 63;
  if (lane < cnt) {
    const uint4 rc = blk[lane];
    const uint64_t off = (uint64_t)rc.y << 32 | rc.x;
    const uint32_t kl = rc.z;
    const uint8_t* p = keys + off;
    const bool safe = off + kl + 16 <= kend;
    const LdsKQ<LdsTab<NT>, KF> K(kfull, kf, kl, s1, s2, T);
    Blk h;
    switch (c & 3u | (c >= 4u ? 4u : 0u)) {  // class-uniform: the exact variant of every lane
      case 0: h = meow_a<false, 0, false>(p, kl, safe, K, T); break;
      case 1: h = meow_a<false, 16, false>(p, kl, safe, K, T); break;
      case 2: h = meow_a<false, 32, false>(p, kl, safe, K, T); break;
      case 3: h = meow_a<false, 48, false>(p, kl, safe, K, T); break;
      case 4: h = meow_a<true, 0, false>(p, kl, safe, K, T); break;
      case 5: h = meow_a<true, 16, false>(p, kl, safe, K, T); break;
      case 6: h = meow_a<true, 32, false>(p, kl, safe, K, T); break;
      default: h = meow_a<true, 48, false>(p, kl, safe, K, T); break;
    }
    store_h(out, rc.w, h, fix);
  }
}

template <int NT, int NW, int REM>
__global__ void __launch_bounds__(NW * 64)
k_var12(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
        uint64_t* __restrict__ out, uint32_t flags, uint4* __restrict__ qbuf) {
  constexpr int WIN = 256, M = WIN / 64, AREA = WIN * 16, QB = 64;  // blocks per wave
  constexpr int KF = 16 * kQCls - kLT;
  constexpr int kTabB = LdsTab<NT>::kWords * 4, kFullB = kLT * (int)sizeof(VConst9), kKfB = KF * 64;
  constexpr int kBytes = kTabB + kFullB + kKfB + NW * AREA;
  static_assert(kBytes <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint32_t smem[kBytes / 4];
  uint32_t* lds = smem;
  VConst9* kfull = (VConst9*)((uint8_t*)smem + kTabB);
  Blk* kf = (Blk*)((uint8_t*)smem + kTabB + kFullB);
  uint8_t* wavemem = (uint8_t*)smem + kTabB + kFullB + kKfB;
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + KF); l += blockDim.x) {
    if (l >= (uint32_t)kLT) {
      const Blk Mx = mixer(s1, s2, l);
#pragma unroll
      for (int i = 0; i < 4; i++) kf[kf_index(l, i)] = aesT(bxor(ramp(i), Mx), T);
      continue;
    }
    const MeowConst k = make_const(s1, s2, l, T);
    VConst9 v;
#pragma unroll
    for (int i = 0; i < 4; i++) { v.F[i] = k.F[i]; v.G[i] = k.G[i]; }
    v.TG2 = k.TG2; v.TCS0a = k.TCS0a;
    kfull[l] = v;
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Blk* stage = (Blk*)(wavemem + wv * AREA);
  uint32_t* hist = (uint32_t*)stage;
  uint2* rec = (uint2*)(wavemem + wv * AREA + WIN * 8);
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + wv, tw = (uint64_t)gridDim.x * NW;
  const uint64_t kend = offs[n];
  uint4* const qrec = qbuf + gw * QB * 64;
  uint32_t qs = 0xffffu << 16 | 64u;  // lane c < kQCls: class c's open block << 16 | fill (64: none)
  uint64_t freem = ~0ull;              // free blocks (wave-uniform)
  for (uint64_t w = gw; w < nwin; w += tw) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const uint64_t ws = offs[i0];
    const uint64_t wend = kend - ws;
    uint32_t kk, d0;
    {
      uint32_t o[M], L[M], r[M], b[M];
      bool wide = false;
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        const uint64_t a = offs[i0 + (j < k ? j : k)], e = offs[i0 + (j < k ? j + 1 : k)];
        o[m] = (uint32_t)(a - ws);
        L[m] = (uint32_t)(e - a);
        wide |= e - ws >= (1ull << 32) || e - a >= (1ull << 24);
      }
      if (__ballot(wide) != 0) {
        wide_window<NT>(keys, offs, i0, k, M, s1, s2, out, fix, lds);
        continue;
      }
#pragma unroll
      for (int i = 0; i < 4; i++) hist[lane * 4 + i] = 0;
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        b[m] = v11_bucket(L[m] >> 4) * 4u + (lane & 3u);
        r[m] = j < k ? atomicAdd(&hist[b[m]], 1u) : 0u;
      }
      wave_sync();
      {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) { v[i] = hist[lane * 4 + i]; sum += v[i]; }
        uint32_t inc = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(inc, d, 64);
          if (lane >= (uint32_t)d) inc += y;
        }
        uint32_t run = inc - sum;
#pragma unroll
        for (int i = 0; i < 4; i++) { hist[lane * 4 + i] = run; run += v[i]; }
        kk = __builtin_amdgcn_readlane(inc, 63);
      }
      wave_sync();
#pragma unroll
      for (int m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        if (j < k) rec[hist[b[m]] + r[m]] = make_uint2(o[m], (L[m] << 8) | j);
      }
      wave_sync();
    }
    const uint32_t x = __builtin_amdgcn_readfirstlane(hist[32 * 4]);
    const uint32_t xs = __builtin_amdgcn_readfirstlane(hist[4 * 4]);
    const uint32_t rem = x & 63u;
    d0 = rem != 0 && rem <= (uint32_t)REM && xs == x ? x - rem : x;
    uint32_t fb = 0, nfb = 0;  // lane i < nfb: class << 8 | block of the i-th block filled in this window
    if (d0 < kk) {
      uint32_t cb = 0, cnt = 0;
      if (lane < (uint32_t)kQCls) {
        const uint32_t bk = v11_bucket(lane);
        const uint32_t s0 = hist[bk * 4], e0 = hist[bk * 4 + 4];
        cb = s0 > d0 ? s0 : d0;
        cnt = e0 > cb ? e0 - cb : 0u;
      }
      uint32_t pl = 0, pb = 0;  // lane c: open block << 16 | fill before; its new blocks, 8 bits each
      uint64_t cm = __ballot(cnt != 0);
      while (cm) {
        const uint32_t c = (uint32_t)__builtin_ctzll(cm);
        cm &= cm - 1;
        const uint32_t cc = __builtin_amdgcn_readlane(cnt, c);
        const uint32_t st = __builtin_amdgcn_readlane(qs, c);
        const uint32_t blk = st >> 16, fill = st & 0xffffu;
        const uint32_t n1 = cc < 64u - fill ? cc : 64u - fill;
        const uint32_t nnew = (cc - n1 + 63u) >> 6;
        uint32_t nbs = 0, last = blk;
        if (n1 != 0 && fill + n1 == 64u) {  // the open block is full
          if (lane == nfb) fb = c << 8 | blk;
          nfb++;
        }
        for (uint32_t t = 0; t < nnew; t++) {
          const uint32_t nbk = (uint32_t)__builtin_ctzll(freem);
          freem &= freem - 1;
          nbs |= nbk << (8 * t);
          last = nbk;
          if (t + 1 < nnew) {  // a full new block
            if (lane == nfb) fb = c << 8 | nbk;
            nfb++;
          }
        }
        uint32_t lastfill = nnew ? cc - n1 - 64u * (nnew - 1u) : fill + n1;
        if (nnew && lastfill == 64u) {
          if (lane == nfb) fb = c << 8 | last;
          nfb++;
        }
        if (lastfill == 64u) { last = 0xffffu; }  // nothing open
        if (lane == c) { pl = st; pb = nbs; qs = last << 16 | lastfill; }
      }
#pragma unroll
      for (int m = 0; m < M; m++) {
        if (d0 + 64u * m >= kk) break;  // wave-uniform
        const uint32_t p = d0 + lane + 64 * m;
        const bool v = p < kk;
        const uint2 rr = rec[v ? p : d0];
        const uint32_t kl = rr.y >> 8, c = kl >> 4;
        const uint32_t rank = p - (uint32_t)__shfl((int)cb, (int)c, 64);
        const uint32_t st = (uint32_t)__shfl((int)pl, (int)c, 64), fill = st & 0xffffu;
        const uint32_t nbc = (uint32_t)__shfl((int)pb, (int)c, 64);
        uint32_t blk, pos;
        if (rank < 64u - fill) { blk = st >> 16; pos = fill + rank; }
        else {
          const uint32_t r2 = rank - (64u - fill);
          blk = (nbc >> (8 * (r2 >> 6))) & 255u;
          pos = r2 & 63u;
        }
        const uint64_t off = ws + rr.x;
        if (v) qrec[blk * 64 + pos] = make_uint4((uint32_t)off, (uint32_t)(off >> 32), kl, (uint32_t)(i0 + (rr.y & 255u)));
      }
    }
    wave_sync();
    uint2 rc0 = rec[lane], rc1 = rec[64 + lane], rc2 = rec[128 + lane], rc3 = rec[192 + lane];
    wave_sync();
    const uint8_t* base = keys + ws;
    const uint32_t nch = (d0 + 63) >> 6;
#pragma unroll 1
    for (uint32_t c = 0; c < nch; c++) {
      const uint32_t pos = 64 * c + lane;
      const bool valid = pos < d0;
      const uint2 rc = rc0;
      rc0 = rc1; rc1 = rc2; rc2 = rc3;
      const uint32_t kl = valid ? rc.y >> 8 : 0u;
      const bool al = __ballot(kl >= 64u) != 0;
      const int cmx = __ballot((kl & 48u) == 48u) ? 48 : __ballot((kl & 48u) >= 32u) ? 32
                    : __ballot((kl & 48u) >= 16u) ? 16 : 0;
      if (valid) {
        const uint8_t* p = base + rc.x;
        const bool safe = (uint64_t)rc.x + kl + 16 <= wend;
        const LdsKV9<LdsTab<NT>, KF> K(kfull, kf, kl, s1, s2, T);
        Blk h;
        if (al) h = meow_a<true, 48, false>(p, kl, safe, K, T);
        else if (cmx == 48) h = meow_a<false, 48, false>(p, kl, safe, K, T);
        else if (cmx == 32) h = meow_a<false, 32, false>(p, kl, safe, K, T);
        else if (cmx == 16) h = meow_a<false, 16, false>(p, kl, safe, K, T);
        else h = meow_a<false, 0, false>(p, kl, safe, K, T);
        stage[rc.y & 255u] = fix ? fixup(h) : h;
      }
    }
    wave_sync();
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t j = 64 * c + lane;
      if (j < k) store_h<true>(out, i0 + j, stage[j], false);
    }
    wave_sync();
    if (nfb) {
      // the run's stores (stale words in deferred slots) before the blocks'
      // hashes for those slots; the blocks' records visible to every lane
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
      for (uint32_t i = 0; i < nfb; i++) {
        const uint32_t e = __builtin_amdgcn_readlane(fb, i);
        const uint32_t blk = e & 255u;
        v12_block<NT, void, KF>(keys, kend, qrec + blk * 64, e >> 8, 64u, s1, s2, out, fix, kfull, kf, T);
        freem |= 1ull << blk;
      }
    }
  }
  // the open blocks
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  uint64_t om = __ballot(lane < (uint32_t)kQCls && (qs & 0xffffu) < 64u);
  while (om) {
    const uint32_t c = (uint32_t)__builtin_ctzll(om);
    om &= om - 1;
    const uint32_t st = __builtin_amdgcn_readlane(qs, c);
    v12_block<NT, void, KF>(keys, kend, qrec + (st >> 16) * 64, c, st & 0xffffu, s1, s2, out, fix, kfull, kf, T);
  }
}

// Per-stream scratch for the deferral queues: a private stream-ordered pool
// per device (allocations are cached by the pool, so a call does not pay for
// a fresh hipMalloc, and concurrent calls on different streams get disjoint
// buffers).
std::mutex g_qpool_mu;
hipMemPool_t g_qpool[64] = {};

int qpool_get(hipMemPool_t* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  if (dev < 0 || dev >= 64) return set_err(KVH_EINVAL);
  std::lock_guard<std::mutex> g(g_qpool_mu);
  if (!g_qpool[dev]) {
    hipMemPoolProps p = {};
    p.allocType = hipMemAllocationTypePinned;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = dev;
    e = hipMemPoolCreate(&g_qpool[dev], &p);
    if (e != hipSuccess) { g_qpool[dev] = nullptr; return hip_err(e); }
    uint64_t keep = ~0ull;  // never release cached memory on synchronisation
    (void)hipMemPoolSetAttribute(g_qpool[dev], hipMemPoolAttrReleaseThreshold, &keep);
  }
  *out = g_qpool[dev];
  return 0;
}

// k_var12: one kernel; scratch = 64 blocks of 64 records per wave.
template <int REM>
int var12_launch(const uint8_t* kp, const uint64_t* offsets, uint64_t n, uint64_t seed1, uint64_t seed2,
                 uint64_t* out, uint32_t flags, hipStream_t st, int cus) {
  if (n >= (1ull << 32) || n < 4096) return 1;
  const uint32_t grid = grid_for(n / 4 + 1, cus, 1);
  const size_t bytes = (size_t)grid * 16 * 64 * 64 * sizeof(uint4);
  hipMemPool_t pool;
  if (qpool_get(&pool) != 0) return 1;
  void* mem = nullptr;
  if (hipMallocFromPoolAsync(&mem, bytes, pool, st) != hipSuccess) { (void)hipGetLastError(); return 1; }
  hipLaunchKernelGGL((k_var12<2, 16, REM>), dim3(grid), dim3(1024), 0, st, kp, offsets, n, seed1, seed2, out, flags,
                     (uint4*)mem);
  int rc = launch_done();
  const hipError_t e = hipFreeAsync(mem, st);
  if (rc == 0 && e != hipSuccess) rc = hip_err(e);
  return rc;
}

// Windows, then queues.  Returns 1 when the batch does not take this path
// (the caller runs k_var9), 0 or an error otherwise.
template <int REM>
int var11_launch(const uint8_t* kp, const uint64_t* offsets, uint64_t n, uint64_t seed1, uint64_t seed2,
                 uint64_t* out, uint32_t flags, hipStream_t st, int cus) {
  if (n >= (1ull << 32) || n < 4096) return 1;  // u32 record indices; small batches gain nothing
  const uint32_t grid = grid_for(n / 4 + 1, cus, 1);
  const uint64_t regions = (uint64_t)grid * 16;
  const uint64_t nwin = (n + 255) / 256;
  const uint64_t keys_per_wave = (nwin + regions - 1) / regions * 256;
  // blocks for 3/8 of a wave's keys (C2 defers ~1/4) plus one open block per class
  const uint64_t rb = (keys_per_wave * 3 / 8 + 63) / 64 + 2 * kQCls + 4;
  const size_t rec_b = (size_t)(regions * rb * 64 * sizeof(uint4));
  const size_t meta_b = (size_t)(regions * rb * 4), bytes = rec_b + meta_b + regions * 4;
  hipMemPool_t pool;
  if (qpool_get(&pool) != 0) return 1;
  void* mem = nullptr;
  if (hipMallocFromPoolAsync(&mem, bytes, pool, st) != hipSuccess) { (void)hipGetLastError(); return 1; }
  VarQ q{(uint4*)mem, (uint32_t*)((uint8_t*)mem + rec_b), (uint32_t*)((uint8_t*)mem + rec_b + meta_b),
         (uint32_t)rb};
  hipLaunchKernelGGL((k_var11<2, 16, REM>), dim3(grid), dim3(1024), 0, st, kp, offsets, n, seed1, seed2, out,
                     flags, q);
  int rc = launch_done();
  if (rc == 0) {
    hipLaunchKernelGGL((k_var11_q<4, 16, false>), dim3(grid), dim3(1024), 0, st, kp, offsets + n, seed1,
                       seed2, out, flags, q, regions);
    rc = launch_done();
  }
  const hipError_t e = hipFreeAsync(mem, st);
  if (rc == 0 && e != hipSuccess) rc = hip_err(e);
  return rc;
}


constexpr int kNotMine = 1;  // the knob value belongs to the product path

// fixed length: the research kernels for L = 16 / 32 (the product knobs 0
// and 3 pick NT and keys per lane: tnt, tkpl)
template <int L>
int exp_fixed_L(const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out, uint32_t flags,
                hipStream_t st, int cus, int tnt, int tkpl) {
  const int nt = tnt ? tnt : 4;
  const int kpl = tkpl ? tkpl : (L == 16 ? 4 : 2);
    if (const int ab = knob(g_tune_ablate)) {
      switch (ab) {
        case 1: return launch_k<L, 2, 4, 1>(keys, n, s1, s2, out, flags, st, cus);
        case 2: return launch_k<L, 2, 4, 2>(keys, n, s1, s2, out, flags, st, cus);
        case 3: return launch_k<L, 2, 4, 3>(keys, n, s1, s2, out, flags, st, cus);
        default: return set_err(KVH_EINVAL);
      }
    }
    if (knob(g_tune_dma) && ((uintptr_t)keys & 15) == 0) {
      const int dk = (tnt ? tnt : 2) * 10 + knob(g_tune_dma);
      const uint32_t grid = grid_for(n, cus, 1);
      switch (dk) {
#define KVH_DMA(NTv, Rv)                                                                              \
  case NTv * 10 + Rv:                                                                                 \
    if constexpr (DmaCfg<L, NTv, Rv>::kFits) {                                                        \
      hipLaunchKernelGGL((k_fixed_dma<L, NTv, Rv>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out, \
                         flags);                                                                       \
      return launch_done();                                                                           \
    }                                                                                                 \
    break;
        KVH_DMA(2, 2) KVH_DMA(2, 3) KVH_DMA(2, 4) KVH_DMA(2, 6) KVH_DMA(4, 2)
#undef KVH_DMA
        default: break;
      }
    }
    if (L == 16 && knob(g_tune_bs) > 0 && ((uintptr_t)keys & 15) == 0) {
      const uint64_t nB = (uint64_t)((double)n * knob(g_tune_bs) / 1000.0) / 512 * 512;
      const uint32_t grid = grid_for(n, cus, 1);
      const int hk = knob(g_tune_prio) * 1000 + nt * 100 + kpl * 10 + knob(g_tune_bsw);
      switch (hk) {
#define KVH_HY(Pv, NTv, Uv, Wv)                                                                               \
  case Pv * 1000 + NTv * 100 + Uv * 10 + Wv:                                                                 \
    hipLaunchKernelGGL((k_hybrid<16, NTv, Uv, Wv, Pv>), dim3(grid), dim3(kBlock), 0, st, keys, n, nB, s1, s2, \
                       out, flags);                                                                          \
    return launch_done();
        KVH_HY(0, 4, 4, 4) KVH_HY(2, 4, 4, 4) KVH_HY(2, 4, 2, 4) KVH_HY(2, 4, 4, 8) KVH_HY(2, 4, 4, 2)
#undef KVH_HY
        default: return set_err(KVH_EINVAL);
      }
    }
    if (knob(g_tune_pf)) {
      switch (nt * 100 + kpl) {
        case 201: return launch_k<L, 2, 1, 0, true>(keys, n, s1, s2, out, flags, st, cus);
        case 202: return launch_k<L, 2, 2, 0, true>(keys, n, s1, s2, out, flags, st, cus);
        case 204: return launch_k<L, 2, 4, 0, true>(keys, n, s1, s2, out, flags, st, cus);
        case 402: return launch_k<L, 4, 2, 0, true>(keys, n, s1, s2, out, flags, st, cus);
        default: return set_err(KVH_EINVAL);
      }
    }
  return kNotMine;
}

// the load-pattern ablation at 32 and 64 B (round 6, knob 5 = 4..8): the
// product's (NT, U) in k_fixed_x's static order, with the keys' 16-byte
// pieces loaded per key (5, the product's pattern: a 16-byte piece of each of
// 64 keys per instruction, 2L-byte lane stride), as coalesced 1 KiB runs (4,
// keys scrambled), or (64 B) 32 bytes of each of 32 keys per instruction with
// a lane-pair exchange (6; 8 without the exchange, keys scrambled)
template <int L, int U>
int exp_fixed_load_ab(const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out, uint32_t flags,
                      hipStream_t st, int cus) {
  if (((uintptr_t)keys & 15) != 0) return set_err(KVH_EINVAL);
  switch (knob(g_tune_ablate)) {
    case 1: return launch_k<L, 4, U, 1>(keys, n, s1, s2, out, flags, st, cus);
    case 2: return launch_k<L, 4, U, 2>(keys, n, s1, s2, out, flags, st, cus);
    case 3: return launch_k<L, 4, U, 3>(keys, n, s1, s2, out, flags, st, cus);
    case 4: return launch_k<L, 4, U, 4>(keys, n, s1, s2, out, flags, st, cus);
    case 5: return launch_k<L, 4, U, 0>(keys, n, s1, s2, out, flags, st, cus);
    case 6: if constexpr (L == 64) return launch_k<L, 4, U, 6>(keys, n, s1, s2, out, flags, st, cus); break;
    case 8: if constexpr (L == 64) return launch_k<L, 4, U, 8>(keys, n, s1, s2, out, flags, st, cus); break;
    default: break;
  }
  return set_err(KVH_EINVAL);
}

bool exp_fixed(int L, const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out, uint32_t flags,
               hipStream_t st, int cus, int tnt, int tkpl, int* rc) {
  int r = kNotMine;
  if (knob(g_tune_ablate) && (L == 64 || ((L == 32 || L == 48) && knob(g_tune_ablate) >= 4))) {
    *rc = L == 64   ? exp_fixed_load_ab<64, 1>(keys, n, s1, s2, out, flags, st, cus)
          : L == 48 ? exp_fixed_load_ab<48, 3>(keys, n, s1, s2, out, flags, st, cus)
                    : exp_fixed_load_ab<32, 4>(keys, n, s1, s2, out, flags, st, cus);
    return true;
  }
  if (L == 16) r = exp_fixed_L<16>(keys, n, s1, s2, out, flags, st, cus, tnt, tkpl);
  if (L == 32) r = exp_fixed_L<32>(keys, n, s1, s2, out, flags, st, cus, tnt, tkpl);
  if (r == kNotMine) return false;
  *rc = r;
  return true;
}

int exp_var_int(int var, const uint8_t* kp, const uint64_t* offsets, uint64_t n, uint64_t seed1, uint64_t seed2,
                uint64_t* out, uint32_t flags, hipStream_t st, int cus) {
  const uint32_t grid = grid_for(n / 4 + 1, cus, 1);
  switch (var) {
    case 40: case 41: case 42: case 43: {  // deferral (round 3); batches they do not take: the generic kernel
      int r = var == 40 ? var11_launch<32>(kp, offsets, n, seed1, seed2, out, flags, st, cus)
            : var == 41 ? var11_launch<0>(kp, offsets, n, seed1, seed2, out, flags, st, cus)
            : var == 42 ? var12_launch<32>(kp, offsets, n, seed1, seed2, out, flags, st, cus)
                        : var12_launch<0>(kp, offsets, n, seed1, seed2, out, flags, st, cus);
      if (r == 1) {
        uint64_t sd[16] = {seed1, seed2};
        r = generic_launch(true, kp, offsets, 0, n, sd, 1, out, flags, st, cus);
      }
      return r;
    }
    // conflict attribution (counter-only except 31) and store modes of k_var9 (round 3)
    case 28: hipLaunchKernelGGL((k_var9x<2, 16, 256, false, false, 1>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 29: hipLaunchKernelGGL((k_var9x<2, 16, 256, false, false, 3>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 30: hipLaunchKernelGGL((k_var9x<2, 16, 256, false, false, 4>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 31: hipLaunchKernelGGL((k_var9x<2, 16, 256, false, false, 0, 1>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 32: hipLaunchKernelGGL((k_var9x<2, 16, 256, false, false, 0, 2>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 38: hipLaunchKernelGGL((k_var9x<2, 16, 256, false, false, 0, 0, 8>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 39: hipLaunchKernelGGL((k_var9x<2, 16, 256, false, false, 3, 0, 8>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    // k_var10: larger windows, records-only LDS, hashes stored straight to their slots
    case 33: hipLaunchKernelGGL((k_var10<2, 16, 256, 512, false>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 34: hipLaunchKernelGGL((k_var10<2, 16, 256, 512, true>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 35: hipLaunchKernelGGL((k_var10<2, 8, 256, 1024, false>), dim3(grid), dim3(512), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 36: hipLaunchKernelGGL((k_var10<2, 12, 192, 512, false>), dim3(grid), dim3(768), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 37: hipLaunchKernelGGL((k_var10<2, 16, 256, 256, false>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 26:  // k_var9 with long keys two lanes per key (meow_pair), 16 waves: spills, 3.75 ms
      hipLaunchKernelGGL((k_var9x<2, 16, 256, false, true>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n,
                         seed1, seed2, out, flags);
      return launch_done();
    case 27:  // the same at 12 waves: 10 % fewer LDS instructions, 3.14 vs 3.03 ms (two serial passes)
      hipLaunchKernelGGL((k_var9x<2, 12, 192, true, true>), dim3(grid), dim3(768), 0, st, kp, offsets, (uint64_t)n,
                         seed1, seed2, out, flags);
      return launch_done();
    case 18:
      hipLaunchKernelGGL((k_var8<2, 256, 4>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1,
                         seed2, out, flags);
      return launch_done();
    case 19:
      hipLaunchKernelGGL((k_var8<2, 256, 0>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1,
                         seed2, out, flags);
      return launch_done();
    case 14:
      hipLaunchKernelGGL((k_var7<2>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out,
                         flags);
      return launch_done();
    case 15:
      hipLaunchKernelGGL((k_var7<2, 256, kBlock / 64, 1>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n,
                         seed1, seed2, out, flags);
      return launch_done();
    case 16:
      hipLaunchKernelGGL((k_var7<2, 256, 12, 1>), dim3(cus), dim3(768), 0, st, kp, offsets, (uint64_t)n,
                         seed1, seed2, out, flags);
      return launch_done();
    case 17:
      hipLaunchKernelGGL((k_var7<2, 256, 12, 0>), dim3(cus), dim3(768), 0, st, kp, offsets, (uint64_t)n,
                         seed1, seed2, out, flags);
      return launch_done();
    case 11: hipLaunchKernelGGL((k_var6x<2, 384, false, 12>), dim3(cus), dim3(768), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 12: hipLaunchKernelGGL((k_var6x<2, 512, false, 10>), dim3(cus), dim3(640), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 8: hipLaunchKernelGGL((k_var6x<2, 128>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 9: hipLaunchKernelGGL((k_var6x<2, 256, true>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 20: hipLaunchKernelGGL((k_var6x<2, 256, false, 12, 4, true>), dim3(cus), dim3(768), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 21: hipLaunchKernelGGL((k_var6x<2, 256, false, 12, 4>), dim3(cus), dim3(768), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 22: hipLaunchKernelGGL((k_var6x<2, 256, false, kBlock / 64, 4, true>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    case 10: hipLaunchKernelGGL((k_var6x<2, 128, true>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); return launch_done();
    default: break;
  }
  const int vm = knob(g_tune_var_mode);
  if (var == 6) {
    const uint32_t g1 = grid_for(n, cus, 1);
    if (vm == 1)
      hipLaunchKernelGGL((k_var5<2, true>), dim3(g1), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags);
    else
      hipLaunchKernelGGL((k_var5<2>), dim3(g1), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags);
    return launch_done();
  }
  if (var == 3 || var == 5) {
    const uint32_t g4 = grid_for((n + 3) / 4, cus, 1);
    if (vm) {
      switch (vm) {
        case 1: hipLaunchKernelGGL((k_var3<2, 4, 1>), dim3(g4), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); break;
        case 2: hipLaunchKernelGGL((k_var3<2, 4, 2>), dim3(g4), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); break;
        default: hipLaunchKernelGGL((k_var3<2, 4, 3>), dim3(g4), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags); break;
      }
      return launch_done();
    }
    if (var == 5)
      hipLaunchKernelGGL((k_var3<2, 4>), dim3(g4), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags);
    else
      hipLaunchKernelGGL((k_var3<2, 2>), dim3(g4), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags);
    return launch_done();
  }
  if (var == 2 || var == 4) {
    const uint32_t g1 = grid_for(n, cus, 1);
    if (var == 4)
      hipLaunchKernelGGL((k_var<4>), dim3(g1), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags);
    else
      hipLaunchKernelGGL((k_var<2>), dim3(g1), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2, out, flags);
    return launch_done();
  }
  return kNotMine;
}

bool exp_var(int var, const uint8_t* kp, const uint64_t* offsets, uint64_t n, uint64_t seed1, uint64_t seed2,
             uint64_t* out, uint32_t flags, hipStream_t st, int cus, int* rc) {
  const int r = exp_var_int(var, kp, offsets, n, seed1, seed2, out, flags, st, cus);
  if (r == kNotMine) return false;
  *rc = r;
  return true;
}

bool exp_var_knob(int v) { return (v >= 2 && v <= 50) || (v >= 61 && v <= 70); }  // 7, 13, 24, 25, 44, 45, 47-50: var_dispatch under KVH_EXPERIMENTS

int exp_set_tuning(int k, int value) {
  auto set = [](Knob& g, int v) { return g.exchange(v, std::memory_order_relaxed); };
  switch (k) {
    case 5: if (value < 0 || value > 8) return KVH_EINVAL; return set(g_tune_ablate, value);
    case 6: if (value != 0 && value != 2 && value != 3 && value != 4 && value != 6) return KVH_EINVAL;
            return set(g_tune_dma, value);
    case 9: if (value < 0 || value > 3) return KVH_EINVAL; return set(g_tune_var_mode, value);
    case 10: return set(g_tune_pf, value ? 1 : 0);
    case 11: if (value < 0 || value > 1000) return KVH_EINVAL; return set(g_tune_bs, value);
    case 12: if (value != 2 && value != 4 && value != 8) return KVH_EINVAL; return set(g_tune_bsw, value);
    case 13: if (value != 0 && value != 2 && value != 3) return KVH_EINVAL; return set(g_tune_prio, value);
    default: return KVH_EINVAL;
  }
}

struct Register {
  Register() {
    g_exp.set_tuning = exp_set_tuning;
    g_exp.var_knob = exp_var_knob;
    g_exp.fixed = exp_fixed;
    g_exp.var = exp_var;
  }
} g_register;

}  // namespace

extern "C" {

// C3 hybrid (research): `permille` of the keys (rounded down to 512) through
// the bitsliced waves, nbw of 16 waves bitsliced (2, 4 or 8), T-table waves at
// s_setprio(prio) (0 or 2).  32-byte keys at a 16-byte aligned base, 4 seeds
// (seeds[8]), out[n][4][2].  permille = 0 runs the same kernel with no
// bitsliced keys (the waves idle): compare with the product's k_fixed_lanes.
int kvh_exp_multiseed_hybrid(const void* keys, size_t n, const uint64_t* seeds, uint64_t* out, int permille,
                             int nbw, int prio, uint32_t flags, void* stream) {
  if (!keys || !out || !seeds || n == 0 || ((uintptr_t)keys & 15)) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  const uint64_t nB = (uint64_t)((double)n * permille / 1000.0) / 512 * 512;
  const uint64_t* s = seeds;
  const int key = nbw * 10 + prio;
  switch (key) {
#define KVH_HL(NBWv, Pv)                                                                                         \
  case NBWv * 10 + Pv:                                                                                           \
    hipLaunchKernelGGL((k_hybrid_lanes<4, 2, NBWv, Pv>), dim3(cus), dim3(kBlock), 0, (hipStream_t)stream,         \
                       (const uint8_t*)keys, (uint64_t)n, nB, out, flags, s[0], s[1], s[2], s[3], s[4], s[5], s[6], \
                       s[7]);                                                                                    \
    return launch_done();
    KVH_HL(2, 0) KVH_HL(2, 2) KVH_HL(4, 0) KVH_HL(4, 2) KVH_HL(8, 2)
#undef KVH_HL
    default: return set_err(KVH_EINVAL);
  }
}
// diagnostics: copy the per-wave phase stamps of the last STAMP launch
int kvh_debug_stamps(uint64_t* host, size_t count) {
  if (count > 4096 * 8) count = 4096 * 8;
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg), count * 8, 0, hipMemcpyDeviceToHost);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}
}
