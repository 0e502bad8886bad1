// kvh.hip -- gfx950 kernels and the C-ABI (include/kvh.h) of the batched
// Meow128 key-hash engine.  See DESIGN.md for the data layout in HBM, the
// kernels' rooflines and the folding argument; meow_dev.hpp for the round.
//
// Kernels
//   k_fixed<L,NT,A16,U>   fixed length L in {8,16,..,64}, one seed, constants
//                         folded into SGPRs (configs C1, C4)
//   k_fixed_lanes         LA lanes per key, one seed each (config C3)
//   k_fixed_ms            one lane per key, `arity` seeds (C3 fallback)
//   k_fixed_rt            any fixed length below one block (runtime L)
//   k_generic<VAR,NT>     any length: fixed stride or u64 offsets
//   k_var9, k_var6        variable length, per-wave length-sorted windows (C2)
//   k_seeded              straight-line restatement, per-key seeds, constant
//                         memory tables (drop-ins, x2/x4/x8 variants)
//   k_stream_*            streaming init/update/final state transitions
//
// libkvh.so holds only kernels some call of include/kvh.h launches.  The
// research kernels that lost their A/B and the ablation builds whose outputs
// are not hashes live in tools/exp/ (`make experiments` -> tools/libkvh_exp.so,
// which links these objects plus tools/exp/*.o; see rt::g_exp).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <atomic>
#include <mutex>
#include <thread>
#include <condition_variable>
#include <deque>
#include <functional>
#include <vector>
#include <algorithm>
#include "meow_dev.hpp"
#include "kvh_internal.hpp"
#include "kvh_var.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

#ifndef KVH_VERSION
#define KVH_VERSION "raikv_amd-kvh 0.1 (gfx950)"
#endif

namespace {

// ------------------------------------------------------------ kernels
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
template <int L, int NT, bool A16, int U>
__global__ void __launch_bounds__(kBlock)
k_fixed(const uint8_t* __restrict__ keys, uint64_t n, uint64_t s1, uint64_t s2,
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
  for (uint64_t b = wave * 64 * U; b < n; b += step) {  // wave-uniform trip count
    Blk D[U][NC];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      load_fixed<L, A16, true>(keys + (j < last ? j : last) * L, D[u]);
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
}

// k_fixed software-pipelined across chunks: while chunk c+1's key loads are
// in flight, chunk c's TAIL (three serial rounds, meow_tail) runs; then
// chunk c+1's HEAD (the absorb/Mix/Compress rounds whose chains run side by
// side, meow_head) -- so the serial end of one chunk overlaps the loads and
// the parallel start of the next instead of exposing its LDS latency.
// Same chunking, clamping and stores as k_fixed.
template <int L, int NT, bool A16, int U>
__global__ void __launch_bounds__(kBlock)
k_fixed_pl(const uint8_t* __restrict__ keys, uint64_t n, uint64_t s1, uint64_t s2,
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
  uint64_t pb = wave * 64 * U;
  if (pb >= n) return;  // wave-uniform
  Blk X[U], Y[U];
  {
    Blk D[U][NC];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = pb + 64 * u + lane;
      load_fixed<L, A16, true>(keys + (j < last ? j : last) * L, D[u]);
    }
#pragma unroll
    for (int u = 0; u < U; u++) meow_head<L>(D[u], K, T, X[u], Y[u]);
  }
  for (uint64_t b = pb + step; b < n; b += step) {  // wave-uniform trip count
    Blk D[U][NC];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      load_fixed<L, A16, true>(keys + (j < last ? j : last) * L, D[u]);
    }
    Blk h[U];
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = meow_tail<L>(X[u], Y[u], K, T);
#pragma unroll
    for (int u = 0; u < U; u++) meow_head<L>(D[u], K, T, X[u], Y[u]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = pb + 64 * u + lane;
      store_h<true>(out, j < last ? j : last, h[u], fix);
    }
    pb = b;
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t j = pb + 64 * u + lane;
    store_h<true>(out, j < last ? j : last, meow_tail<L>(X[u], Y[u], K, T), fix);
  }
}

// Multi-seed (config C3, kv_hash_meow128_4_same_length_4_seed with one key
// in all slots, key_hash.c:1891-1937): LA = 2, 4 or 8 lanes per key, lane l
// hashes under seed (l & (LA-1)).  The output slot of (key i, seed a) is
// i*LA + a, so lane j of a chunk writes slot j: every store is one contiguous
// 1 KiB run (one lane per key with LA strided 16-byte stores inflated the
// write traffic 1.3x).  The LA lanes of a key load the same 16-byte pieces
// (same cache line, one request).  Constants are per lane (VGPRs), computed
// once in the prologue for the lane's fixed seed.
template <int L, int NT, bool A16, int U, int LA>
__global__ void __launch_bounds__(kBlock)
k_fixed_lanes(const uint8_t* __restrict__ keys, uint64_t n, uint64_t* __restrict__ out, uint32_t flags,
              uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1, uint64_t a2, uint64_t b2, uint64_t a3,
              uint64_t b3, uint64_t a4, uint64_t b4, uint64_t a5, uint64_t b5, uint64_t a6, uint64_t b6,
              uint64_t a7, uint64_t b7) {
  static_assert(LA == 2 || LA == 4 || LA == 8, "lanes per key");
  constexpr int NC = Plan<L>::NC;
  constexpr int SH = LA == 2 ? 1 : LA == 4 ? 2 : 3;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  const uint32_t sl = threadIdx.x & (LA - 1);
  const uint64_t sa[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
  const uint64_t sb[8] = {b0, b1, b2, b3, b4, b5, b6, b7};
  uint64_t s1 = sa[0], s2 = sb[0];
#pragma unroll
  for (int q = 1; q < LA; q++)
    if (sl == (uint32_t)q) { s1 = sa[q]; s2 = sb[q]; }
  const MeowConst K = make_const(s1, s2, (uint64_t)L, T);
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  const uint64_t ns = n << SH, lastk = n - 1;
  for (uint64_t b = wave * 64 * U; b < ns; b += step) {
    Blk D[U][NC];
    uint64_t slot[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t k = (b + 64 * u + lane) >> SH;
      k = k < lastk ? k : lastk;
      slot[u] = (k << SH) | sl;
      load_fixed<L, A16, true>(keys + k * L, D[u]);
    }
    Blk h[U];
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = meow_ct<L>(D[u], K, T);
#pragma unroll
    for (int u = 0; u < U; u++) store_h<true>(out, slot[u], h[u], fix);
  }
}


template <int L, int NT, bool A16>
__global__ void __launch_bounds__(kBlock)
k_fixed_ms(const uint8_t* __restrict__ keys, uint64_t n, const uint64_t* __restrict__ seeds_unused,
           uint64_t* __restrict__ out, uint32_t flags, uint32_t arity,
           uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1, uint64_t a2, uint64_t b2,
           uint64_t a3, uint64_t b3, uint64_t a4, uint64_t b4, uint64_t a5, uint64_t b5,
           uint64_t a6, uint64_t b6, uint64_t a7, uint64_t b7) {
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ MeowConst kc[KVH_MAX_ARITY];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  if (threadIdx.x < KVH_MAX_ARITY && threadIdx.x < arity) {
    const uint64_t sa[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
    const uint64_t sb[8] = {b0, b1, b2, b3, b4, b5, b6, b7};
    kc[threadIdx.x] = make_const(sa[threadIdx.x], sb[threadIdx.x], (uint64_t)L, T);
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    Blk D[Plan<L>::NC];
    load_fixed<L, A16>(keys + i * L, D);
    for (uint32_t a = 0; a < arity; a++) {
      const MeowConst K = uniform(kc[a]);
      store_h(out, i * arity + a, meow_ct<L>(D, K, T), fix);
    }
  }
}

// per-lane constants for variable-length batches, from LDS records

// Any length.  VAR: key i = keys[offs[i], offs[i+1]) with per-lane length;
// !VAR: stride = fixed_len, every lane the same length, `arity` seeds.
template <bool VAR, int NT>
__global__ void __launch_bounds__(kBlock)
k_generic(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint32_t fixed_len,
          uint64_t n, uint64_t* __restrict__ out, uint32_t flags, uint32_t arity,
          uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1, uint64_t a2, uint64_t b2,
          uint64_t a3, uint64_t b3, uint64_t a4, uint64_t b4, uint64_t a5, uint64_t b5,
          uint64_t a6, uint64_t b6, uint64_t a7, uint64_t b7) {
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ MeowConst kfull[VAR ? kLT : KVH_MAX_ARITY];
  __shared__ Blk kf[VAR ? kNF * 4 : 1];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  if constexpr (VAR) {
    for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + kNF); l += blockDim.x) {
      if (l < (uint32_t)kLT) {
        kfull[l] = make_const(a0, b0, l, T);
      } else {
        const Blk M = mixer(a0, b0, l);
#pragma unroll
        for (int s = 0; s < 4; s++) kf[(l - kLT) * 4 + s] = aesT(bxor(ramp(s), M), T);
      }
    }
  } else {
    if (threadIdx.x < arity) {
      const uint64_t sa[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
      const uint64_t sb[8] = {b0, b1, b2, b3, b4, b5, b6, b7};
      kfull[threadIdx.x] = make_const(sa[threadIdx.x], sb[threadIdx.x], fixed_len, T);
    }
  }
  __syncthreads();
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if constexpr (VAR) {
      const uint64_t o0 = offs[i], o1 = offs[i + 1];
      const uint64_t L = o1 - o0;  // any size_t length, as kv_hash_meow128 (key_hash.c:1413)
      const LdsK<LdsTab<NT>, uint64_t> K(kfull, kf, L, a0, b0, T);
      store_h(out, i, meow_rt(keys + o0, L, K, T), fix);
    } else {
      const uint8_t* p = keys + i * (uint64_t)fixed_len;
      for (uint32_t a = 0; a < arity; a++) {
        const MeowConst Kc = uniform(kfull[a]);
        const RegK K{Kc};
        store_h(out, i * arity + a, meow_rt(p, fixed_len, K, T), fix);
      }
    }
  }
}




// ---------------------------------------------------------------------
// k_var6: per-WAVE windows, no workgroup barriers after the prologue.
// Wave w takes windows of WIN consecutive keys (grid-stride over windows),
// counting-sorts the window by length in its own LDS slice (LDS atomics
// give each key its rank inside its length bucket; one wave-wide scan of
// the 256 bucket counts), then hashes the window in WIN/64 chunks of 64
// length-sorted keys: a chunk's lanes run (nearly) the same absorb trip
// count and trail branches, where input order costs 2.7x in divergence for
// zipf 8-256 B keys (simulation: 0.58 vs 0.29 lane-rounds/key at WIN 256).
// A wave never waits for another wave, so the long-key chunk of one window
// no longer stalls the whole workgroup (k_var5's 33 % barrier time).  Keys
// are gathered from global memory (the window's ~12 KiB stay L2-hot across
// its chunks); hashes are stored to their original slots.

template <int NT, int WIN, int NW = kBlock / 64, int SH = 0>
__global__ void __launch_bounds__(NW * 64)
k_var6(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
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
    // hashes stay in registers until the window is done, then go through
    // the wave's (now free) record area to leave as one contiguous run:
    // scattered 16-byte stores in sorted order inflated HBM writes 1.76x
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
    wave_sync();  // records reused by the next window
  }
}

// ---------------------------------------------------------------------
// k_var9: k_var6's per-wave windows, sorted by 16-byte length class, with
// the two costs its counters name removed:
//  * L2 requests.  The L1 does not merge misses of different load
//    instructions, so k_var6's byte-aligned pieces (dwordx4 + dword each)
//    and dword-by-dword tails cost ~7 L2 requests per key, and the L1->L2
//    queue (46 requests in flight per CU at ~430 cycles) sets its time.
//    meow_a reads 16-byte aligned chunks: one request per 16 bytes;
//  * serial latency.  meow_rt's per-lane branches run one after the other
//    in a wave (each trail chunk's load, each Mix state, each Compress half);
//    meow_a runs, per chunk of 64 sorted keys, one straight-line variant
//    chosen by two wave-uniform facts (some key has a full block; the
//    largest trail), so the state chains interleave and every short key's
//    loads are issued before its first round.
// The variants need ~165 VGPRs, so 12 waves per CU; hashes go straight to
// the wave's LDS stage at their input slot, records are 8 bytes
// (window offset, length << 8 | slot), and no per-window value lives in a
// register array.  Windows spanning 4 GiB or holding a key of 16 MiB or
// more take wide_window (input order, u64 offsets and lengths).

template <int NT, int NW, int KF, bool PF = false>
__global__ void __launch_bounds__(NW * 64)
k_var9(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
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
      for (int q = 0; q < 4; q++) kf[(l - kLT) * 4 + q] = aesT(bxor(ramp(q), Mx), T);
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
    for (int q = 0; q < 4; q++) hist[lane * 4 + q] = 0;
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      // 64 length classes x 4 sub-counters by lane & 3: a quarter of the
      // same-address atomics (a class's keys in one instruction serialise)
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
      if (valid) {
        const uint8_t* p = base + rc.x;
        const bool safe = (uint64_t)rc.x + kl + 16 <= wend;  // whole dwordx4 groups stay in the buffer
        const LdsKV9<LdsTab<NT>, KF> K(kfull, kf, kl, s1, s2, T);
        Blk h;
        if (al) h = meow_a<true, 48, PF>(p, kl, safe, K, T);
        else if (cm == 48) h = meow_a<false, 48, PF>(p, kl, safe, K, T);
        else if (cm == 32) h = meow_a<false, 32, PF>(p, kl, safe, K, T);
        else if (cm == 16) h = meow_a<false, 16, PF>(p, kl, safe, K, T);
        else h = meow_a<false, 0, PF>(p, kl, safe, K, T);
        stage[rc.y & 255u] = fix ? fixup(h) : h;
      }
    }
    wave_sync();
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t j = 64 * c + lane;
      if (j < k) store_h<true>(out, i0 + j, stage[j], false);
    }
    wave_sync();  // stage and records reused by the next window
  }
}




// straight-line restatement, one thread per key, per-key seeds
__global__ void __launch_bounds__(256)
k_seeded(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n,
         const uint64_t* __restrict__ seeds, uint64_t* __restrict__ out, uint32_t flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ConstTab T;
  const uint64_t o0 = offs[i], o1 = offs[i + 1];
  const Blk h = meow_literal(keys + o0, o1 - o0, seeds[2 * i], seeds[2 * i + 1], T);
  store_h(out, i, h, (flags & KVH_FIXUP) != 0);
}

// Tiny host batches (raikv's 8-key prefetch pipes, ev_net.h:442; a ctest
// batch of a few thousand frags, ctest.c:34): keys, offsets and hashes stay
// in coherent pinned host memory and the kernel reads and writes them
// across PCIe itself -- one launch and one synchronize, no DMA copies, no
// LDS table fill (constant-memory tables, the literal restatement).  Key i
// is keys[offs[i] - offs[0] ..) (variable length) or keys[i * key_len ..).
__global__ void __launch_bounds__(256)
k_tiny(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint32_t key_len, uint64_t n, uint64_t s1,
       uint64_t s2, uint64_t* __restrict__ out, uint32_t flags) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const ConstTab T;
  uint64_t a, L;
  if (offs) {
    a = offs[i] - offs[0];
    L = offs[i + 1] - offs[i];
  } else {
    a = i * key_len;
    L = key_len;
  }
  store_h(out, i, meow_literal(keys + a, L, s1, s2, T), (flags & KVH_FIXUP) != 0);
}

// streaming: state[16 words] in/out; absorb nblk full 64-byte blocks
__global__ void k_stream_absorb(uint32_t* st, const uint8_t* data, uint64_t nblk) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ConstTab T;
  MeowState s;
  for (int i = 0; i < 4; i++) for (int c = 0; c < 4; c++) s.S[i].w[c] = st[4 * i + c];
  absorb_blocks(s, data, nblk, T);
  for (int i = 0; i < 4; i++) for (int c = 0; c < 4; c++) st[4 * i + c] = s.S[i].w[c];
}

// streaming final: Meow_Loop over the buffered `off` bytes, then finish
// with the Mixer of (k1, k2, total) (key_hash.c:1541-1568)
__global__ void k_stream_final(const uint32_t* st, const uint8_t* block, uint64_t off,
                               uint64_t k1, uint64_t k2, uint64_t total, uint64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ConstTab T;
  MeowState s;
  for (int i = 0; i < 4; i++) for (int c = 0; c < 4; c++) s.S[i].w[c] = st[4 * i + c];
  if (off > 0) absorb_loop(s, block, off, T);
  const Blk h = finish(s, mixer(k1, k2, total), T);
  out[0] = (uint64_t)h.w[0] | ((uint64_t)h.w[1] << 32);
  out[1] = (uint64_t)h.w[2] | ((uint64_t)h.w[3] << 32);
}

}  // namespace

// ------------------------------------------------------------ host runtime (kvh_internal.hpp)
namespace kvh {
namespace rt {

thread_local int t_last_err = 0;
ExpHooks g_exp{};

struct DevInfo {
  int cus = 0;
};
std::mutex g_mu;
std::vector<DevInfo> g_dev;

int set_err(int e) { t_last_err = e; return e; }
int hip_err(hipError_t e) { return set_err(KVH_EHIP_BASE - (int)e); }

int device_cus(int* cus) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  std::lock_guard<std::mutex> g(g_mu);
  if ((int)g_dev.size() <= dev) g_dev.resize(dev + 1);
  if (g_dev[dev].cus == 0) {
    int c = 0;
    e = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return hip_err(e);
    g_dev[dev].cus = c > 0 ? c : 1;
  }
  *cus = g_dev[dev].cus;
  return 0;
}

int launch_done() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(e);
  return set_err(0);
}

}  // namespace rt
}  // namespace kvh

namespace {

// ------------------------------------------------------------ host side
// Tuning knobs (kvh_set_tuning): process-wide, read once per call with
// relaxed atomic loads, so a knob set on one thread never races a launch on
// another (a call in flight keeps the value it read).
using Knob = std::atomic<int>;
Knob g_tune_nt{0};        // tables per LDS: 2 or 4 (0 = per-length default)
Knob g_tune_wgmul{1};     // workgroups per CU multiplier
Knob g_tune_generic{0};   // force the generic kernel
Knob g_tune_kpl{0};       // keys per lane per chunk in k_fixed (1, 2, 4 or 8; 0 = per-length default)
Knob g_tune_ms_lanes{1};  // multi-seed: 1 = lanes-per-key kernel, 0 = one lane per key
Knob g_tune_pl{0};        // fixed-length kernel: 1 = software-pipelined across chunks (k_fixed_pl)
Knob g_tune_var{23};      // var-length kernel: 23 = k_var9 (16 waves; 24 = 12 waves, 25 = 12 waves + block prefetch); 13 = k_var6 windows sorted by 16-byte length class; 7 = by exact length; 0 = unsorted k_generic
inline int knob(const Knob& k) { return k.load(std::memory_order_relaxed); }

uint32_t grid_for(uint64_t n, int cus, int wg_per_cu) {
  const uint64_t need = (n + kBlock - 1) / kBlock;
  uint64_t g = (uint64_t)cus * (uint64_t)std::max(1, wg_per_cu * knob(g_tune_wgmul));
  if (need < g) g = need;
  return (uint32_t)std::max<uint64_t>(g, 1);
}


template <int L, int NT, int U>
int launch_k(const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out, uint32_t flags,
             hipStream_t st, int cus) {
  const bool a16 = ((uintptr_t)keys & 15) == 0;
  const uint32_t grid = grid_for(n, cus, NT == 4 ? 1 : 2);
  if (knob(g_tune_pl)) {
    if (a16)
      hipLaunchKernelGGL((k_fixed_pl<L, NT, true, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out, flags);
    else
      hipLaunchKernelGGL((k_fixed_pl<L, NT, false, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out, flags);
    return launch_done();
  }
  if (a16)
    hipLaunchKernelGGL((k_fixed<L, NT, true, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out, flags);
  else
    hipLaunchKernelGGL((k_fixed<L, NT, false, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out, flags);
  return launch_done();
}

// Fixed-length keys of any length 1-63 (k_fixed<L> covers the multiples of
// 8 at 8-byte aligned bases): the same wave-chunked streaming and U keys per
// lane as k_fixed, with the length a kernel argument.  Every lane of the
// launch has the same length, so every branch of the Meow plan below is
// wave-uniform (scalar branches, each body U independent rounds: the ILP
// k_generic's one key per lane lacks, which ran these lengths at half the
// neighbouring multiples of 8).  NC = ceil(L / 16) 16-byte chunks per key,
// each read as the dword-aligned 16 bytes at or below it plus one dword,
// funnelled by the byte offset (v_alignbyte), then masked past the key.  A
// chunk of keys within 32 bytes of the batch's last byte reads byte-exact
// (load_bytes) instead: wave-uniform, the last chunk only.
template <int NC, int U, class Tab>
__device__ __forceinline__ void meow_small(Blk (&D)[U][NC], uint32_t L, const MeowConst& K, const Tab& T,
                                           Blk (&h)[U]) {
  // nb = 0: the trail only (key_hash.c:1200-1210); every state's first
  // absorb is folded (F_s ^ k, one round)
  const uint32_t C = L & 48u, t = L & 15u;
  const bool T0 = C >= 16, T1 = C >= 32, T2 = C >= 48, T3 = t != 0;
  Blk S0[U], S1[U], S2[U], S3[U];
  if (T3) {  // the partial chunk is the last one
#pragma unroll
    for (int u = 0; u < U; u++) S3[u] = aesdec(aesdec(bxor(K.F[3], D[u][NC - 1]), D[u][NC - 1], T), K.M, T);
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) S3[u] = K.G[3];
  }
  if constexpr (NC >= 3) {
    if (T2) {
#pragma unroll
      for (int u = 0; u < U; u++) S2[u] = aesdec(aesdec(bxor(K.F[2], D[u][2]), D[u][2], T), K.M, T);
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) S2[u] = K.G[2];
    }
  }
  if constexpr (NC >= 2) {
    if (T1) {
#pragma unroll
      for (int u = 0; u < U; u++) S1[u] = aesdec(aesdec(bxor(K.F[1], D[u][1]), D[u][1], T), K.M, T);
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) S1[u] = K.G[1];
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) S1[u] = K.G[1];
  }
  if (T0) {
#pragma unroll
    for (int u = 0; u < U; u++) S0[u] = aesdec(aesdec(bxor(K.F[0], D[u][0]), D[u][0], T), K.M, T);
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) S0[u] = K.G[0];
  }
  // Compress_Meow2 / Compress_Meow and the final round, as meow_ct
  Blk S2b[U];
  if (NC >= 3 && T2) {
    if constexpr (NC >= 3) {
#pragma unroll
      for (int u = 0; u < U; u++) S2b[u] = aesdec(aesdec(S2[u], S3[u], T), K.M, T);
    }
  } else if (T3) {
#pragma unroll
    for (int u = 0; u < U; u++) S2b[u] = aesdec(bxor(K.TG2, S3[u]), K.M, T);
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) S2b[u] = K.CS2b;
  }
  if (T0) {
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = aesdec(aesdec(aesdec(S0[u], S1[u], T), S2b[u], T), K.M, T);
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = aesdec(bxor(K.TCS0a, S2b[u]), K.M, T);
  }
}

template <int NC, int NT, int U>
__global__ void __launch_bounds__(kBlock)
k_fixed_rt(const uint8_t* __restrict__ keys, uint64_t n, uint32_t L, uint64_t s1, uint64_t s2,
           uint64_t* __restrict__ out, uint32_t flags) {
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  const uint64_t last = n - 1, total = n * (uint64_t)L;
  for (uint64_t b = wave * 64 * U; b < n; b += step) {  // wave-uniform trip count
    const bool exact = (b + 64 * U) * (uint64_t)L + 32 > total;  // this chunk reaches the batch's end
    Blk D[U][NC];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      const uint8_t* p = keys + (j < last ? j : last) * (uint64_t)L;
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const int left = (int)L - 16 * c;
        const uint32_t nv = left >= 16 ? 16u : (uint32_t)left;
        if (exact) {
          D[u][c] = load_bytes(p + 16 * c, nv);
        } else {
          D[u][c] = load16_full(p + 16 * c);
          if (c == NC - 1 && nv < 16) {
#pragma unroll
            for (int w = 0; w < 4; w++) {
              const int keep = (int)nv - 4 * w;
              D[u][c].w[w] &= keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
            }
          }
        }
      }
    }
    Blk h[U];
    meow_small<NC, U>(D, L, K, T, h);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      store_h<true>(out, j < last ? j : last, h[u], fix);
    }
  }
}

template <int NC, int NT, int U>
int launch_fixed_rt(const uint8_t* keys, uint64_t n, uint32_t L, uint64_t s1, uint64_t s2, uint64_t* out,
                    uint32_t flags, hipStream_t st, int cus) {
  const uint32_t grid = grid_for(n, cus, NT == 4 ? 1 : 2);
  hipLaunchKernelGGL((k_fixed_rt<NC, NT, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, L, s1, s2, out, flags);
  return launch_done();
}

// Default (NT, U) per length from tools/tune.py and tools/len_sweep.py
// sweeps; knobs 0 and 3 select the others.
template <int L>
int launch_fixed_nt(const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out,
                    uint32_t flags, hipStream_t st, int cus) {
  if (int rc = 0; g_exp.fixed && g_exp.fixed(L, keys, n, s1, s2, out, flags, st, cus, knob(g_tune_nt), knob(g_tune_kpl), &rc))
    return rc;
  if constexpr (L == 16 || L == 32) {
    // per-length defaults from tools/tune.py: Td0..Td3 in LDS
    // (no rotations), 4 keys per lane at 16 B, 2 at 32 B
    const int tnt = knob(g_tune_nt), tkpl = knob(g_tune_kpl);
    const int nt = tnt ? tnt : 4;
    const int kpl = tkpl ? tkpl : (L == 16 ? 4 : 2);
    switch (nt * 100 + kpl) {
      case 401: return launch_k<L, 4, 1>(keys, n, s1, s2, out, flags, st, cus);
      case 402: return launch_k<L, 4, 2>(keys, n, s1, s2, out, flags, st, cus);
      case 404: return launch_k<L, 4, 4>(keys, n, s1, s2, out, flags, st, cus);
      case 408: return launch_k<L, 4, 8>(keys, n, s1, s2, out, flags, st, cus);
      case 201: return launch_k<L, 2, 1>(keys, n, s1, s2, out, flags, st, cus);
      case 202: return launch_k<L, 2, 2>(keys, n, s1, s2, out, flags, st, cus);
      case 204: return launch_k<L, 2, 4>(keys, n, s1, s2, out, flags, st, cus);
      case 208: return launch_k<L, 2, 8>(keys, n, s1, s2, out, flags, st, cus);
      default: return set_err(KVH_EINVAL);
    }
  } else {
    const int tnt = knob(g_tune_nt), tkpl = knob(g_tune_kpl);
    switch ((tnt ? tnt : 2) * 100 + (tkpl ? tkpl : 4)) {
      case 401: return launch_k<L, 4, 1>(keys, n, s1, s2, out, flags, st, cus);
      case 402: return launch_k<L, 4, 2>(keys, n, s1, s2, out, flags, st, cus);
      case 404: return launch_k<L, 4, 4>(keys, n, s1, s2, out, flags, st, cus);
      case 201: return launch_k<L, 2, 1>(keys, n, s1, s2, out, flags, st, cus);
      case 202: return launch_k<L, 2, 2>(keys, n, s1, s2, out, flags, st, cus);
      case 204: return launch_k<L, 2, 4>(keys, n, s1, s2, out, flags, st, cus);
      case 403: if constexpr (L >= 40) return launch_k<L, 4, 3>(keys, n, s1, s2, out, flags, st, cus); break;
      case 203: if constexpr (L >= 40) return launch_k<L, 2, 3>(keys, n, s1, s2, out, flags, st, cus); break;
      default: break;
    }
    return set_err(KVH_EINVAL);
  }
}

template <int L, int NT, int U>
int launch_lanes_v(const uint8_t* keys, uint64_t n, const uint64_t* s, uint32_t arity, uint64_t* out,
                   uint32_t flags, hipStream_t st, int cus) {
  const uint32_t grid = grid_for(n * arity, cus, NT == 4 ? 1 : 2);
#define KVH_LANES_V(LAv)                                                                                \
  hipLaunchKernelGGL((k_fixed_lanes<L, NT, true, U, LAv>), dim3(grid), dim3(kBlock), 0, st, keys, n, out, flags, \
                     s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10], s[11], s[12], s[13],   \
                     s[14], s[15])
  if (arity == 2) KVH_LANES_V(2); else if (arity == 4) KVH_LANES_V(4); else KVH_LANES_V(8);
#undef KVH_LANES_V
  return launch_done();
}

template <int L>
int launch_lanes_L(const uint8_t* keys, uint64_t n, const uint64_t* s, uint32_t arity, uint64_t* out,
                   uint32_t flags, hipStream_t st, int cus) {
  const bool a16 = ((uintptr_t)keys & 15) == 0;
  if constexpr (L == 32) {
    // C3's length: Td0..Td3 in LDS (no rotates, one 16-wave workgroup per CU)
    // and 2 keys per lane by default -- 118 vs 112 G hash/s for Td0/Td1 with
    // two workgroups per CU (tools/tune.py, profiles/r02/c3_layout_ab.txt);
    // knobs 0 / 3 select the others
    const int nt = knob(g_tune_nt), kpl = knob(g_tune_kpl);
    if (a16) {
      switch ((nt ? nt : 4) * 10 + (kpl ? kpl : 2)) {
        case 22: break;
        case 21: return launch_lanes_v<L, 2, 1>(keys, n, s, arity, out, flags, st, cus);
        case 24: return launch_lanes_v<L, 2, 4>(keys, n, s, arity, out, flags, st, cus);
        case 41: return launch_lanes_v<L, 4, 1>(keys, n, s, arity, out, flags, st, cus);
        case 42: return launch_lanes_v<L, 4, 2>(keys, n, s, arity, out, flags, st, cus);
        case 44: return launch_lanes_v<L, 4, 4>(keys, n, s, arity, out, flags, st, cus);
        default: return set_err(KVH_EINVAL);
      }
    }
  }
  const uint32_t grid = grid_for(n * arity, cus, 2);
#define KVH_LANES(A16v, LAv)                                                                            \
  hipLaunchKernelGGL((k_fixed_lanes<L, 2, A16v, 2, LAv>), dim3(grid), dim3(kBlock), 0, st, keys, n, out, flags, \
                     s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10], s[11], s[12], s[13],   \
                     s[14], s[15])
  if (a16) {
    if (arity == 2) KVH_LANES(true, 2); else if (arity == 4) KVH_LANES(true, 4); else KVH_LANES(true, 8);
  } else {
    if (arity == 2) KVH_LANES(false, 2); else if (arity == 4) KVH_LANES(false, 4); else KVH_LANES(false, 8);
  }
#undef KVH_LANES
  return launch_done();
}

template <int L>
int launch_ms_L(const uint8_t* keys, uint64_t n, const uint64_t* s, uint32_t arity, uint64_t* out,
                uint32_t flags, hipStream_t st, int cus) {
  const bool a16 = ((uintptr_t)keys & 15) == 0;
  const uint32_t grid = grid_for(n, cus, 1);
  if (a16)
    hipLaunchKernelGGL((k_fixed_ms<L, 4, true>), dim3(grid), dim3(kBlock), 0, st, keys, n, nullptr, out,
                       flags, arity, s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10],
                       s[11], s[12], s[13], s[14], s[15]);
  else
    hipLaunchKernelGGL((k_fixed_ms<L, 4, false>), dim3(grid), dim3(kBlock), 0, st, keys, n, nullptr, out,
                       flags, arity, s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10],
                       s[11], s[12], s[13], s[14], s[15]);
  return launch_done();
}

int launch_generic(bool var, const uint8_t* keys, const uint64_t* offs, uint32_t fixed_len, uint64_t n,
                   const uint64_t* s, uint32_t arity, uint64_t* out, uint32_t flags, hipStream_t st,
                   int cus) {
  const uint32_t grid = grid_for(n, cus, 1);
  if (var)
    hipLaunchKernelGGL((k_generic<true, 4>), dim3(grid), dim3(kBlock), 0, st, keys, offs, fixed_len, n,
                       out, flags, arity, s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9],
                       s[10], s[11], s[12], s[13], s[14], s[15]);
  else
    hipLaunchKernelGGL((k_generic<false, 4>), dim3(grid), dim3(kBlock), 0, st, keys, offs, fixed_len, n,
                       out, flags, arity, s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9],
                       s[10], s[11], s[12], s[13], s[14], s[15]);
  return launch_done();
}

// Pinned/device staging for the synchronous host drop-ins.
struct Staging {
  std::mutex mu;
  uint8_t* dev = nullptr;
  size_t cap = 0;
  int device = -1;
};
Staging g_stage;

int stage_reserve(size_t bytes) {  // caller holds g_stage.mu
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  if (g_stage.dev && g_stage.device == dev && g_stage.cap >= bytes) return 0;
  if (g_stage.dev) {
    int cur = dev;
    (void)hipSetDevice(g_stage.device);  // best-effort release of the old staging buffer
    (void)hipFree(g_stage.dev);
    (void)hipSetDevice(cur);
    g_stage.dev = nullptr;
  }
  size_t cap = std::max<size_t>(bytes, 1 << 20);
  e = hipMalloc(&g_stage.dev, cap);
  if (e != hipSuccess) { g_stage.dev = nullptr; g_stage.cap = 0; return hip_err(e); }
  g_stage.cap = cap;
  g_stage.device = dev;
  return 0;
}

size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// Hash `n` host keys (pointers + lengths) with per-key seeds on the GPU via
// k_seeded; out gets 2n words.  Synchronous.
int seeded_host(const void* const* ptrs, const size_t* lens, size_t n, const uint64_t* seeds,
                uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  size_t kbytes = 0;
  for (size_t i = 0; i < n; i++) {
    if (lens[i] && !ptrs[i]) return set_err(KVH_EINVAL);
    kbytes += lens[i];
  }
  std::vector<uint8_t> host(al16(kbytes) + al16(8 * (n + 1)) + al16(16 * n));
  std::vector<uint64_t> offs(n + 1);
  size_t o = 0;
  for (size_t i = 0; i < n; i++) {
    offs[i] = o;
    if (lens[i]) memcpy(host.data() + o, ptrs[i], lens[i]);
    o += lens[i];
  }
  offs[n] = o;
  const size_t off_offs = al16(kbytes), off_seeds = off_offs + al16(8 * (n + 1)),
               off_out = off_seeds + al16(16 * n);
  memcpy(host.data() + off_offs, offs.data(), 8 * (n + 1));
  memcpy(host.data() + off_seeds, seeds, 16 * n);
  std::lock_guard<std::mutex> g(g_stage.mu);
  int rc = stage_reserve(off_out + 16 * n);
  if (rc) return rc;
  uint8_t* d = g_stage.dev;
  hipError_t e = hipMemcpy(d, host.data(), off_out, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(e);
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(k_seeded, dim3(grid), dim3(256), 0, 0, d, (const uint64_t*)(d + off_offs), (uint64_t)n,
                     (const uint64_t*)(d + off_seeds), (uint64_t*)(d + off_out), flags);
  rc = launch_done();
  if (rc) return rc;
  e = hipMemcpy(out, d + off_out, 16 * n, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_err(e);
  return set_err(0);
}

int same_len_host(const void* const* ptrs, size_t cnt, size_t sz, const uint64_t* seed_pairs,
                  bool per_key_seed, uint64_t* x) {
  std::vector<size_t> lens(cnt, sz);
  std::vector<uint64_t> seeds(2 * cnt);
  for (size_t i = 0; i < cnt; i++) {
    seeds[2 * i] = per_key_seed ? seed_pairs[2 * i] : seed_pairs[0];
    seeds[2 * i + 1] = per_key_seed ? seed_pairs[2 * i + 1] : seed_pairs[1];
  }
  return seeded_host(ptrs, lens.data(), cnt, seeds.data(), x, 0);
}

// Host pipeline state (kvh_meow128_{fixed,var}_host): streams, events and
// buffer slots, grown on demand and kept for the process lifetime.  Each
// device has kPipesPerDev of them, so that several host threads may drive one
// device at once (kvh_*_host_multi with a device listed twice); a call holds
// one pipeline for its duration.
constexpr int kPipeSlots = 16;  // buffer slots allocated; g_tune_pipe_slots of them used
constexpr int kMaxDev = 64;
constexpr int kPipesPerDev = 4;
Knob g_tune_pipe_mib{16};   // key bytes per pipeline chunk, MiB (knob 15)
Knob g_tune_pipe_slots{4};  // chunks in flight (knob 16)
Knob g_tune_tiny{4096};     // host batches of at most this many keys take the zero-copy tiny path (knob 21; 0 = off)
constexpr size_t kTinyBytes = 256 << 10;  // ... and at most this many key bytes
struct HostPipe {
  std::mutex mu;
  hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
  hipEvent_t ev_in[kPipeSlots] = {}, ev_k[kPipeSlots] = {}, ev_out[kPipeSlots] = {};
  uint8_t* dk[kPipeSlots] = {};      // key bytes (device)
  uint64_t* doff[kPipeSlots] = {};   // key offsets (device, variable length)
  uint64_t* dout[kPipeSlots] = {};   // hashes (device)
  uint8_t* tiny = nullptr;           // coherent pinned keys | offsets | hashes of the tiny path
  size_t tinycap = 0;
  uint8_t* hk[kPipeSlots] = {};      // pinned bounce buffers for pageable callers
  uint64_t* hoff[kPipeSlots] = {};
  uint64_t* ho[kPipeSlots] = {};
  size_t kcap = 0, fcap = 0, ocap = 0, hkcap = 0, hfcap = 0, hocap = 0;
  // slots [0, ns) of buffer array b hold `want` bytes each (grow-only)
  template <class T, class A, class F>
  static hipError_t regrow(T* (&b)[kPipeSlots], size_t& cap, size_t want, int ns, A alloc, F release) {
    if (cap < want) {
      for (int s = 0; s < kPipeSlots; s++) if (b[s]) { (void)release(b[s]); b[s] = nullptr; }
      cap = want;
    }
    for (int s = 0; s < ns; s++) {
      if (b[s]) continue;
      const hipError_t e = alloc((void**)&b[s], cap);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // streams, events and ns slots for chunks of kb key bytes, fb offset bytes
  // (0: fixed length) and ob hash bytes on the current device
  int reserve(int ns, size_t kb, size_t fb, size_t ob, bool need_hk, bool need_hf, bool need_ho) {
    hipError_t e = hipSuccess;
    for (hipStream_t* st : {&s_in, &s_k, &s_out})
      if (e == hipSuccess && !*st) e = hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    for (int s = 0; s < kPipeSlots && e == hipSuccess; s++)
      for (hipEvent_t* ev : {&ev_in[s], &ev_k[s], &ev_out[s]})
        if (e == hipSuccess && !*ev) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    auto dmal = [](void** p, size_t b) { return hipMalloc(p, b); };
    auto dfree = [](void* p) { return hipFree(p); };
    auto hmal = [](void** p, size_t b) { return hipHostMalloc(p, b, 0); };
    auto hfree = [](void* p) { return hipHostFree(p); };
    if (e == hipSuccess) e = regrow(dk, kcap, std::max<size_t>(kb, 16), ns, dmal, dfree);
    if (e == hipSuccess && fb) e = regrow(doff, fcap, fb, ns, dmal, dfree);
    if (e == hipSuccess) e = regrow(dout, ocap, ob, ns, dmal, dfree);
    if (e == hipSuccess && need_hk) e = regrow(hk, hkcap, std::max<size_t>(kb, 16), ns, hmal, hfree);
    if (e == hipSuccess && need_hf) e = regrow(hoff, hfcap, fb, ns, hmal, hfree);
    if (e == hipSuccess && need_ho) e = regrow(ho, hocap, ob, ns, hmal, hfree);
    return e == hipSuccess ? 0 : hip_err(e);
  }
};
HostPipe g_pipe[kMaxDev][kPipesPerDev];

// a free pipeline of the current device (blocks on pipeline 0 when all are busy)
std::unique_lock<std::mutex> pick_pipe(int dev, HostPipe** P) {
  for (int i = 0; i < kPipesPerDev; i++) {
    std::unique_lock<std::mutex> lk(g_pipe[dev][i].mu, std::try_to_lock);
    if (lk.owns_lock()) { *P = &g_pipe[dev][i]; return lk; }
  }
  *P = &g_pipe[dev][0];
  return std::unique_lock<std::mutex>(g_pipe[dev][0].mu);
}

// [p, p + bytes) is page-locked host memory (kvh_host_alloc, hipHostMalloc,
// or kvh_host_register of a range holding it): its first AND last byte are
// (a range registered only in part takes the bounce buffers, never a DMA
// past the registered extent).
bool pinned_byte(const void* p) {
  hipPointerAttribute_t a;
  const bool pin = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  return pin;
}
bool is_pinned(const void* p, size_t bytes) {
  if (!bytes) return true;
  return pinned_byte(p) && (bytes == 1 || pinned_byte((const uint8_t*)p + bytes - 1));
}

// One host batch through H2D -> kernel -> D2H on the current device.
// Chunk c is keys [lo_c, hi_c): fixed length (key_len > 0) in chunks of
// `chunk_keys` keys, variable length (offs != nullptr, n+1 host offsets) in
// chunks of at most `budget` key bytes and `chunk_keys` keys (a longer key
// is a chunk of its own, the buffers grow to hold it).  Three streams (H2D,
// kernel, D2H) linked by per-slot events, `slots` chunks in flight: chunk c
// is copied in on s_in, hashed on s_k once its copy-in event fired, copied
// out on s_out once its kernel event fired; a slot is refilled once its
// previous chunk's copy-out event fired.  One stream per DMA direction lets
// both PCIe directions run at once (full duplex).
int host_pipeline(const uint8_t* keys, uint32_t key_len, const uint64_t* offs, size_t n, uint64_t s1, uint64_t s2,
                  uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  if (dev < 0 || dev >= kMaxDev) return set_err(KVH_EINVAL);
  HostPipe* P = nullptr;
  std::unique_lock<std::mutex> lk = pick_pipe(dev, &P);
  const bool var = offs != nullptr;
  if (n <= (size_t)knob(g_tune_tiny) && (var ? offs[n] - offs[0] : (uint64_t)n * key_len) <= kTinyBytes) {
    // tiny batch: copy into the pipeline's coherent pinned buffer, one
    // kernel reading and writing host memory, one synchronize
    const size_t kb = var ? (size_t)(offs[n] - offs[0]) : n * (size_t)key_len;
    const size_t o_off = al16(kb), o_out = o_off + al16(var ? 8 * (n + 1) : 0), need = o_out + 16 * n;
    if (P->tinycap < need) {
      if (P->tiny) (void)hipHostFree(P->tiny);
      P->tiny = nullptr;
      P->tinycap = 0;
      const size_t cap = std::max<size_t>(need, kTinyBytes + 16 * 4096 + 8 * 4097 + 64);
      if ((e = hipHostMalloc((void**)&P->tiny, cap, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess)
        return hip_err(e);
      P->tinycap = cap;
    }
    if (!P->s_k && (e = hipStreamCreateWithFlags(&P->s_k, hipStreamNonBlocking)) != hipSuccess) return hip_err(e);
    if (kb) memcpy(P->tiny, keys + (var ? offs[0] : 0), kb);
    if (var) memcpy(P->tiny + o_off, offs, 8 * (n + 1));
    hipLaunchKernelGGL(k_tiny, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, P->s_k, (const uint8_t*)P->tiny,
                       var ? (const uint64_t*)(P->tiny + o_off) : (const uint64_t*)nullptr, key_len, (uint64_t)n, s1,
                       s2, (uint64_t*)(P->tiny + o_out), flags);
    int rc = launch_done();
    if ((e = hipStreamSynchronize(P->s_k)) != hipSuccess && !rc) rc = hip_err(e);
    if (rc) return rc;
    memcpy(out, P->tiny + o_out, 16 * n);
    return set_err(0);
  }
  const size_t budget = (size_t)knob(g_tune_pipe_mib) << 20;
  const size_t chunk_keys = var ? std::max<size_t>(1, budget / 8) : std::max<size_t>(1, budget / key_len);
  // chunk boundaries; the largest chunk sizes the buffers
  std::vector<size_t> bounds{0};
  size_t max_bytes = 0, max_keys = 0;
  while (bounds.back() < n) {
    const size_t lo = bounds.back();
    size_t hi = std::min(n, lo + chunk_keys);
    if (var) {  // at most `budget` key bytes, at least one key
      const uint64_t lim = offs[lo] + budget;
      hi = std::max(lo + 1, (size_t)(std::upper_bound(offs + lo, offs + hi + 1, lim) - offs) - 1);
      max_bytes = std::max<size_t>(max_bytes, offs[hi] - offs[lo]);
    } else {
      max_bytes = std::max<size_t>(max_bytes, (hi - lo) * key_len);
    }
    max_keys = std::max(max_keys, hi - lo);
    bounds.push_back(hi);
  }
  const uint64_t kb0 = var ? offs[0] : 0, kb1 = var ? offs[n] : (uint64_t)n * key_len;
  const bool pin_k = is_pinned(keys + kb0, kb1 - kb0), pin_o = is_pinned(out, 16 * n),
             pin_f = var && is_pinned(offs, 8 * (n + 1));
  const int slots = std::min(std::max(knob(g_tune_pipe_slots), 2), kPipeSlots);
  int rc = P->reserve(slots, max_bytes, var ? 8 * (max_keys + 1) : 0, 16 * max_keys, !pin_k, var && !pin_f, !pin_o);
  if (rc) return rc;
  if (bounds.size() == 2) {
    // one chunk (raikv's batches: 8 keys per prefetch pipe, ev_net.h:442; up
    // to 16K frags per ctest batch, ctest.c:34): H2D, kernel and D2H in order
    // on one stream and one synchronize, no cross-stream events
    const uint8_t* src = keys + kb0;
    const size_t nbytes = (size_t)(kb1 - kb0);
    if (!pin_k && nbytes) { memcpy(P->hk[0], src, nbytes); src = P->hk[0]; }
    const uint64_t* fsrc = offs;
    if (var && !pin_f) { memcpy(P->hoff[0], offs, 8 * (n + 1)); fsrc = P->hoff[0]; }
    uint64_t* dst = pin_o ? out : P->ho[0];
    if ((nbytes && (e = hipMemcpyAsync(P->dk[0], src, nbytes, hipMemcpyHostToDevice, P->s_k)) != hipSuccess) ||
        (var && (e = hipMemcpyAsync(P->doff[0], fsrc, 8 * (n + 1), hipMemcpyHostToDevice, P->s_k)) != hipSuccess))
      return hip_err(e);
    rc = var ? kvh_meow128_var((const uint8_t*)((uintptr_t)P->dk[0] - (uintptr_t)kb0), P->doff[0], n, s1, s2,
                               P->dout[0], flags, P->s_k)
             : kvh_meow128_fixed(P->dk[0], key_len, n, s1, s2, P->dout[0], flags, P->s_k);
    if (!rc && (e = hipMemcpyAsync(dst, P->dout[0], 16 * n, hipMemcpyDeviceToHost, P->s_k)) != hipSuccess)
      rc = hip_err(e);
    if ((e = hipStreamSynchronize(P->s_k)) != hipSuccess && !rc) rc = hip_err(e);
    if (rc) return rc;
    if (!pin_o) memcpy(out, P->ho[0], 16 * n);
    return set_err(0);
  }
  size_t pend_lo[kPipeSlots] = {}, pend_cnt[kPipeSlots] = {};
  auto drain = [&](int s) -> int {  // the slot's previous chunk has left the device
    if (!pend_cnt[s]) return 0;
    hipError_t x = hipEventSynchronize(P->ev_out[s]);
    if (x != hipSuccess) return hip_err(x);
    if (!pin_o) memcpy(out + 2 * pend_lo[s], P->ho[s], pend_cnt[s] * 16);
    pend_cnt[s] = 0;
    return 0;
  };
  for (size_t c = 0; !rc && c + 1 < bounds.size(); c++) {
    const int s = (int)(c % slots);
    if ((rc = drain(s))) break;
    const size_t lo = bounds[c], cnt = bounds[c + 1] - lo;
    const uint64_t base = var ? offs[lo] : (uint64_t)lo * key_len;
    const size_t nbytes = var ? (size_t)(offs[lo + cnt] - base) : cnt * key_len;
    const uint8_t* src = keys + base;
    if (!pin_k && nbytes) { memcpy(P->hk[s], src, nbytes); src = P->hk[s]; }
    const uint64_t* fsrc = var ? offs + lo : nullptr;
    if (var && !pin_f) { memcpy(P->hoff[s], fsrc, 8 * (cnt + 1)); fsrc = P->hoff[s]; }
    uint64_t* dst = pin_o ? out + 2 * lo : P->ho[s];
    if ((nbytes && (e = hipMemcpyAsync(P->dk[s], src, nbytes, hipMemcpyHostToDevice, P->s_in)) != hipSuccess) ||
        (var && (e = hipMemcpyAsync(P->doff[s], fsrc, 8 * (cnt + 1), hipMemcpyHostToDevice, P->s_in)) != hipSuccess) ||
        (e = hipEventRecord(P->ev_in[s], P->s_in)) != hipSuccess ||
        (e = hipStreamWaitEvent(P->s_k, P->ev_in[s], 0)) != hipSuccess) {
      rc = hip_err(e); break;
    }
    // variable length: the chunk's offsets stay absolute (offs[lo] .. offs[hi]);
    // the key pointer handed to the kernel is biased by -offs[lo], so every
    // address it forms, keys + offs[i], lies inside this chunk's buffer
    rc = var ? kvh_meow128_var((const uint8_t*)((uintptr_t)P->dk[s] - (uintptr_t)base), P->doff[s], cnt, s1, s2,
                               P->dout[s], flags, P->s_k)
             : kvh_meow128_fixed(P->dk[s], key_len, cnt, s1, s2, P->dout[s], flags, P->s_k);
    if (rc) break;
    if ((e = hipEventRecord(P->ev_k[s], P->s_k)) != hipSuccess ||
        (e = hipStreamWaitEvent(P->s_out, P->ev_k[s], 0)) != hipSuccess ||
        (e = hipMemcpyAsync(dst, P->dout[s], cnt * 16, hipMemcpyDeviceToHost, P->s_out)) != hipSuccess ||
        (e = hipEventRecord(P->ev_out[s], P->s_out)) != hipSuccess) {
      rc = hip_err(e); break;
    }
    pend_lo[s] = lo; pend_cnt[s] = cnt;
  }
  for (int s = 0; s < slots; s++) {
    const int r2 = drain(s);
    if (!rc) rc = r2;
  }
  if (rc) {  // leave the pipeline idle for the next call
    (void)hipStreamSynchronize(P->s_in); (void)hipStreamSynchronize(P->s_k); (void)hipStreamSynchronize(P->s_out);
  }
  return rc ? rc : set_err(0);
}

// Shard d of n keys is [b[d], b[d+1]): equal index ranges (offs == nullptr)
// or, for variable length, ranges holding equal key bytes: b[d] = the first
// key whose start offset is >= offs[0] + total * d / ns (workload.py:
// shard_var).  b[0] = 0, b[ns] = n, non-decreasing.
void shard_bounds(const uint64_t* offs, size_t n, int ns, size_t* b) {
  for (int d = 0; d <= ns; d++) {
    if (!offs || n == 0) {
      b[d] = (size_t)((unsigned __int128)n * d / ns);
    } else {
      const uint64_t tot = offs[n] - offs[0];
      const uint64_t tgt = offs[0] + (uint64_t)((unsigned __int128)tot * d / ns);
      b[d] = d == 0 ? 0 : d == ns ? n : (size_t)(std::lower_bound(offs, offs + n + 1, tgt) - offs);
      if (b[d] > n) b[d] = n;
    }
  }
}

// Shards [lo_d, hi_d) of one host batch over ndev devices, one host thread
// each (SURVEY.md §8 e: independent keys, no collective; each device writes
// its disjoint slice of the caller's output, the same global layout as a
// one-device call).  Fixed length: equal index ranges; variable length:
// ranges of equal key BYTES (raikv_amd/workload.py: shard_var).
// Persistent host workers for the _multi entries: a job queue served by
// threads created on first use and kept for the process lifetime (grown to
// the largest device list seen), instead of one new std::thread per device
// per call.  Jobs are independent (a job never waits for another), so a
// pool smaller than the jobs in flight only serialises them.
struct WorkPool {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  int threads = 0;
  void run(std::vector<std::function<void()>>& jobs) {
    std::mutex dmu;
    std::condition_variable dcv;
    size_t left = jobs.size();
    {
      std::lock_guard<std::mutex> g(mu);
      while (threads < (int)jobs.size()) {
        std::thread([this]() { worker(); }).detach();
        threads++;
      }
      for (auto& j : jobs)
        q.push_back([&dmu, &dcv, &left, &j]() {
          j();
          std::lock_guard<std::mutex> g2(dmu);
          if (--left == 0) dcv.notify_all();
        });
    }
    cv.notify_all();
    std::unique_lock<std::mutex> lk(dmu);
    dcv.wait(lk, [&]() { return left == 0; });
  }
  void worker() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this]() { return !q.empty(); });
        job = std::move(q.front());
        q.pop_front();
      }
      job();
    }
  }
};
WorkPool* g_pool = new WorkPool;  // never destroyed: its detached workers outlive static destructors

int host_multi(const uint8_t* keys, uint32_t key_len, const uint64_t* offs, size_t n, uint64_t s1, uint64_t s2,
               uint64_t* out, uint32_t flags, const int* devices, int ndev) {
  if (ndev < 1 || ndev > kMaxDev || !devices) return set_err(KVH_EINVAL);
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess) return hip_err(e);
  for (int d = 0; d < ndev; d++)
    if (devices[d] < 0 || devices[d] >= count || devices[d] >= kMaxDev) return set_err(KVH_EINVAL);
  std::vector<size_t> lo(ndev + 1);
  shard_bounds(offs, n, ndev, lo.data());
  std::vector<int> rcs(ndev, 0);
  std::vector<std::function<void()>> jobs;
  for (int d = 0; d < ndev; d++) {
    const size_t a = lo[d], b = std::max(lo[d], lo[d + 1]);
    if (b == a) continue;
    jobs.emplace_back([&, d, a, b]() {
      const hipError_t se = hipSetDevice(devices[d]);
      if (se != hipSuccess) { rcs[d] = hip_err(se); return; }
      // variable length: shard offsets stay absolute into `keys`;
      // fixed length: the shard's keys start at a * key_len
      rcs[d] = offs ? host_pipeline(keys, 0, offs + a, b - a, s1, s2, out + 2 * a, flags)
                    : host_pipeline(keys + (uint64_t)a * key_len, key_len, nullptr, b - a, s1, s2, out + 2 * a, flags);
    });
  }
  if (jobs.size() == 1) {  // one shard: on the calling thread, whose current device is restored
    int cur = 0;
    if ((e = hipGetDevice(&cur)) != hipSuccess) return hip_err(e);
    jobs[0]();
    (void)hipSetDevice(cur);
  } else if (!jobs.empty()) {
    g_pool->run(jobs);
  }
  for (int d = 0; d < ndev; d++)
    if (rcs[d]) return set_err(rcs[d]);
  return set_err(0);
}

}  // namespace

// =============================================================== C-ABI
extern "C" {

int kvh_meow128_fixed(const void* keys, uint32_t key_len, size_t n, uint64_t seed1, uint64_t seed2,
                      uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !out) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  const uint8_t* k = (const uint8_t*)keys;
  hipStream_t st = (hipStream_t)stream;
  const bool a8 = ((uintptr_t)k & 7) == 0;
  if (!knob(g_tune_generic) && a8) {
    switch (key_len) {
      case 8: return launch_fixed_nt<8>(k, n, seed1, seed2, out, flags, st, cus);
      case 16: return launch_fixed_nt<16>(k, n, seed1, seed2, out, flags, st, cus);
      case 24: return launch_fixed_nt<24>(k, n, seed1, seed2, out, flags, st, cus);
      case 32: return launch_fixed_nt<32>(k, n, seed1, seed2, out, flags, st, cus);
      case 40: return launch_fixed_nt<40>(k, n, seed1, seed2, out, flags, st, cus);
      case 48: return launch_fixed_nt<48>(k, n, seed1, seed2, out, flags, st, cus);
      case 56: return launch_fixed_nt<56>(k, n, seed1, seed2, out, flags, st, cus);
      case 64: return launch_fixed_nt<64>(k, n, seed1, seed2, out, flags, st, cus);
      default: break;
    }
  }
  if (!knob(g_tune_generic) && key_len >= 1 && key_len < 64) {  // any other length below one block
    const int tnt = knob(g_tune_nt), tkpl = knob(g_tune_kpl);
    const int nc = (int)(key_len + 15) / 16, nt = tnt ? tnt : 4, kpl = tkpl ? tkpl : (nc == 1 ? 4 : 2);
    switch (nc * 1000 + nt * 10 + kpl) {
#define KVH_RT(NCv, NTv, Uv) \
  case NCv * 1000 + NTv * 10 + Uv: return launch_fixed_rt<NCv, NTv, Uv>(k, n, key_len, seed1, seed2, out, flags, st, cus);
      KVH_RT(1, 4, 4) KVH_RT(1, 4, 2) KVH_RT(1, 4, 8) KVH_RT(1, 2, 4) KVH_RT(1, 2, 8)
      KVH_RT(2, 4, 2) KVH_RT(2, 4, 4) KVH_RT(2, 2, 2) KVH_RT(2, 2, 4)
      KVH_RT(3, 4, 2) KVH_RT(3, 4, 4) KVH_RT(3, 2, 2) KVH_RT(3, 2, 4)
      KVH_RT(4, 4, 2) KVH_RT(4, 4, 4) KVH_RT(4, 2, 2) KVH_RT(4, 2, 4)
#undef KVH_RT
      default: break;  // a knob pair without an instance: the generic kernel
    }
  }
  uint64_t s[16] = {seed1, seed2};
  return launch_generic(false, k, nullptr, key_len, n, s, 1, out, flags, st, cus);
}

int kvh_meow128_var(const void* keys, const uint64_t* offsets, size_t n, uint64_t seed1, uint64_t seed2,
                    uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !out) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t* kp = (const uint8_t*)keys;
  const int var = knob(g_tune_var);
  const uint32_t grid = grid_for(n / 4 + 1, cus, 1);
  switch (var) {
    case 0: {
      uint64_t s[16] = {seed1, seed2};
      return launch_generic(true, kp, offsets, 0, n, s, 1, out, flags, st, cus);
    }
    case 13:
      hipLaunchKernelGGL((k_var6<2, 256, kBlock / 64, 4>), dim3(grid), dim3(kBlock), 0, st, kp, offsets,
                         (uint64_t)n, seed1, seed2, out, flags);
      return launch_done();
    case 7:
      hipLaunchKernelGGL((k_var6<2, 256>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2,
                         out, flags);
      return launch_done();
    case 23:
      hipLaunchKernelGGL((k_var9<2, 16, 256>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2,
                         out, flags);
      return launch_done();
    case 24:
      hipLaunchKernelGGL((k_var9<2, 12, 192>), dim3(grid), dim3(768), 0, st, kp, offsets, (uint64_t)n, seed1, seed2,
                         out, flags);
      return launch_done();
    case 25:
      hipLaunchKernelGGL((k_var9<2, 12, 192, true>), dim3(grid), dim3(768), 0, st, kp, offsets, (uint64_t)n, seed1,
                         seed2, out, flags);
      return launch_done();
    default:
      break;
  }
  if (int rc = 0; g_exp.var && g_exp.var(var, kp, offsets, n, seed1, seed2, out, flags, st, cus, &rc)) return rc;
  return set_err(KVH_EINVAL);
}

int kvh_meow128_multiseed(const void* keys, uint32_t key_len, size_t n, const uint64_t* seeds,
                          uint32_t arity, uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !out || !seeds || arity < 1 || arity > KVH_MAX_ARITY) return set_err(KVH_EINVAL);
  if (arity == 1) return kvh_meow128_fixed(keys, key_len, n, seeds[0], seeds[1], out, flags, stream);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  uint64_t s[16] = {0};
  for (uint32_t a = 0; a < arity; a++) { s[2 * a] = seeds[2 * a]; s[2 * a + 1] = seeds[2 * a + 1]; }
  const uint8_t* k = (const uint8_t*)keys;
  hipStream_t st = (hipStream_t)stream;
  const bool a8 = ((uintptr_t)k & 7) == 0;
  if (!knob(g_tune_generic) && a8 && knob(g_tune_ms_lanes) && (arity == 2 || arity == 4 || arity == 8)) {
    switch (key_len) {
      case 8: return launch_lanes_L<8>(k, n, s, arity, out, flags, st, cus);
      case 16: return launch_lanes_L<16>(k, n, s, arity, out, flags, st, cus);
      case 24: return launch_lanes_L<24>(k, n, s, arity, out, flags, st, cus);
      case 32: return launch_lanes_L<32>(k, n, s, arity, out, flags, st, cus);
      case 40: return launch_lanes_L<40>(k, n, s, arity, out, flags, st, cus);
      case 48: return launch_lanes_L<48>(k, n, s, arity, out, flags, st, cus);
      case 56: return launch_lanes_L<56>(k, n, s, arity, out, flags, st, cus);
      case 64: return launch_lanes_L<64>(k, n, s, arity, out, flags, st, cus);
      default: break;
    }
  }
  if (!knob(g_tune_generic) && a8) {
    switch (key_len) {
      case 16: return launch_ms_L<16>(k, n, s, arity, out, flags, st, cus);
      case 32: return launch_ms_L<32>(k, n, s, arity, out, flags, st, cus);
      case 64: return launch_ms_L<64>(k, n, s, arity, out, flags, st, cus);
      default: break;
    }
  }
  return launch_generic(false, k, nullptr, key_len, n, s, arity, out, flags, st, cus);
}

int kvh_meow128_batch(const void* keys, const uint64_t* offsets, uint32_t fixed_len, size_t n,
                      const uint64_t* seeds, uint32_t arity, uint64_t* out, uint32_t flags, void* stream) {
  if (!seeds) return set_err(KVH_EINVAL);
  if (offsets) {
    if (arity != 1) return set_err(KVH_EINVAL);
    return kvh_meow128_var(keys, offsets, n, seeds[0], seeds[1], out, flags, stream);
  }
  return kvh_meow128_multiseed(keys, fixed_len, n, seeds, arity, out, flags, stream);
}

int kvh_meow128_var_seeded(const void* keys, const uint64_t* offsets, size_t n, const uint64_t* seeds,
                           uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !seeds || !out) return set_err(KVH_EINVAL);
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(k_seeded, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)keys, offsets,
                     (uint64_t)n, seeds, out, flags);
  return launch_done();
}

int kvh_meow128_fixed_host(const void* keys, uint32_t key_len, size_t n, uint64_t seed1, uint64_t seed2,
                           uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  if (!keys || !out || key_len == 0) return set_err(KVH_EINVAL);
  return host_pipeline((const uint8_t*)keys, key_len, nullptr, n, seed1, seed2, out, flags);
}

int kvh_meow128_var_host(const void* keys, const uint64_t* offsets, size_t n, uint64_t seed1, uint64_t seed2,
                         uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !out) return set_err(KVH_EINVAL);
  return host_pipeline((const uint8_t*)keys, 0, offsets, n, seed1, seed2, out, flags);
}

int kvh_meow128_fixed_host_multi(const void* keys, uint32_t key_len, size_t n, uint64_t seed1, uint64_t seed2,
                                 uint64_t* out, uint32_t flags, const int* devices, int ndev) {
  if (n == 0) return set_err(0);
  if (!keys || !out || key_len == 0) return set_err(KVH_EINVAL);
  return host_multi((const uint8_t*)keys, key_len, nullptr, n, seed1, seed2, out, flags, devices, ndev);
}

int kvh_meow128_var_host_multi(const void* keys, const uint64_t* offsets, size_t n, uint64_t seed1, uint64_t seed2,
                               uint64_t* out, uint32_t flags, const int* devices, int ndev) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !out) return set_err(KVH_EINVAL);
  return host_multi((const uint8_t*)keys, 0, offsets, n, seed1, seed2, out, flags, devices, ndev);
}

int kvh_shard_bounds(const uint64_t* offsets, size_t n, int nshards, size_t* bounds) {
  if (nshards < 1 || !bounds) return set_err(KVH_EINVAL);
  shard_bounds(offsets, n, nshards, bounds);
  return set_err(0);
}

int kvh_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return set_err(KVH_EINVAL);
  const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterDefault);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_host_unregister(void* p) {
  if (!p) return set_err(KVH_EINVAL);
  const hipError_t e = hipHostUnregister(p);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_host_alloc(void** p, size_t bytes) {
  if (!p) return set_err(KVH_EINVAL);
  *p = nullptr;
  const hipError_t e = hipHostMalloc(p, bytes ? bytes : 1, 0);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_host_free(void* p) {
  if (!p) return set_err(0);
  const hipError_t e = hipHostFree(p);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_device_alloc(void** p, size_t bytes) {
  if (!p) return set_err(KVH_EINVAL);
  *p = nullptr;
  const hipError_t e = hipMalloc(p, bytes ? bytes : 1);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_device_free(void* p) {
  if (!p) return set_err(0);
  const hipError_t e = hipFree(p);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_hash_meow128(const void* p, size_t sz, uint64_t* h1, uint64_t* h2) {
  if (!h1 || !h2) return set_err(KVH_EINVAL);
  uint64_t s[2] = {*h1, *h2}, o[2];
  int rc = seeded_host(&p, &sz, 1, s, o, 0);
  if (rc) return rc;
  *h1 = o[0]; *h2 = o[1];
  return 0;
}

uint64_t kvh_hash_meow64(const void* p, size_t sz, uint64_t seed) {
  uint64_t h1 = seed, h2 = seed;
  kvh_hash_meow128(p, sz, &h1, &h2);
  return h1;
}

int kvh_hash_meow128_2_same_length(const void* p, const void* p2, size_t sz, uint64_t* x) {
  const void* ps[2] = {p, p2};
  return same_len_host(ps, 2, sz, x, false, x);
}
int kvh_hash_meow128_4_same_length(const void* p, const void* p2, const void* p3, const void* p4, size_t sz,
                                   uint64_t* x) {
  const void* ps[4] = {p, p2, p3, p4};
  return same_len_host(ps, 4, sz, x, false, x);
}
int kvh_hash_meow128_4_same_length_a(const void** p, size_t sz, uint64_t* x) {
  return same_len_host(p, 4, sz, x, false, x);
}
int kvh_hash_meow128_4_same_length_4_seed(const void* p, const void* p2, const void* p3, const void* p4,
                                          size_t sz, uint64_t* x) {
  const void* ps[4] = {p, p2, p3, p4};
  return same_len_host(ps, 4, sz, x, true, x);
}
int kvh_hash_meow128_8_same_length(const void* p, const void* p2, const void* p3, const void* p4,
                                   const void* p5, const void* p6, const void* p7, const void* p8, size_t sz,
                                   uint64_t* x) {
  const void* ps[8] = {p, p2, p3, p4, p5, p6, p7, p8};
  return same_len_host(ps, 8, sz, x, false, x);
}
int kvh_hash_meow128_8_same_length_a(const void** p, size_t sz, uint64_t* x) {
  return same_len_host(p, 8, sz, x, false, x);
}
int kvh_hash_meow128_2_diff_length(const void* p, size_t sz, const void* p2, size_t sz2, uint64_t* x) {
  const void* ps[2] = {p, p2};
  size_t ls[2] = {sz, sz2};
  uint64_t seeds[4] = {x[0], x[1], x[0], x[1]};
  return seeded_host(ps, ls, 2, seeds, x, 0);
}
int kvh_hash_meow128_4_diff_length(const void* p, size_t sz, const void* p2, size_t sz2, const void* p3,
                                   size_t sz3, const void* p4, size_t sz4, uint64_t* x) {
  const void* ps[4] = {p, p2, p3, p4};
  size_t ls[4] = {sz, sz2, sz3, sz4};
  uint64_t seeds[8] = {x[0], x[1], x[0], x[1], x[0], x[1], x[0], x[1]};
  return seeded_host(ps, ls, 4, seeds, x, 0);
}

int kvh_hash_meow128_vec(const kvh_meow_vec_t* vec, size_t vec_sz, uint64_t* h1, uint64_t* h2) {
  if (!h1 || !h2 || (vec_sz && !vec)) return set_err(KVH_EINVAL);
  size_t total = 0;
  for (size_t i = 0; i < vec_sz; i++) total += vec[i].sz;
  std::vector<uint8_t> cat(total ? total : 1);
  size_t o = 0;
  for (size_t i = 0; i < vec_sz; i++) {
    if (vec[i].sz) memcpy(cat.data() + o, vec[i].p, vec[i].sz);
    o += vec[i].sz;
  }
  return kvh_hash_meow128(cat.data(), total, h1, h2);
}

// Streaming: the 16-word Meow state lives in m->ctx (layout S0..S3 as
// little-endian 128-bit lanes, same as the reference's Meow_Save_Ctx).
static int stream_absorb_dev(kvh_meow_ctx_t* m, const uint8_t* data, size_t nblk) {
  std::lock_guard<std::mutex> g(g_stage.mu);
  int rc = stage_reserve(64 + nblk * 64);
  if (rc) return rc;
  uint8_t* d = g_stage.dev;
  hipError_t e = hipMemcpy(d, m->ctx, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess && nblk) e = hipMemcpy(d + 64, data, nblk * 64, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(e);
  hipLaunchKernelGGL(k_stream_absorb, dim3(1), dim3(64), 0, 0, (uint32_t*)d, (const uint8_t*)(d + 64),
                     (uint64_t)nblk);
  if ((rc = launch_done())) return rc;
  e = hipMemcpy(m->ctx, d, 64, hipMemcpyDeviceToHost);
  return e == hipSuccess ? 0 : hip_err(e);
}

int kvh_meow128_init(kvh_meow_ctx_t* m, kvh_meow_block_t* b, uint64_t k1, uint64_t k2, size_t total) {
  if (!m || !b) return set_err(KVH_EINVAL);
  // Declare_Meow + Xor_Meow (key_hash.c:1509-1521): byte ramps ^ Mixer
  const uint64_t lo = k1 - total, hi = k2 + total + 1;
  for (int i = 0; i < 4; i++) {
    uint8_t r[16];
    for (int j = 0; j < 16; j++) r[j] = (uint8_t)(16 * i + j);
    uint64_t w0, w1;
    memcpy(&w0, r, 8); memcpy(&w1, r + 8, 8);
    m->ctx[2 * i] = w0 ^ lo;
    m->ctx[2 * i + 1] = w1 ^ hi;
  }
  b->off = 0;
  b->total_update_sz = total;
  return set_err(0);
}

int kvh_meow128_update(kvh_meow_ctx_t* m, kvh_meow_block_t* b, const void* p, size_t sz) {
  if (!m || !b || (sz && !p)) return set_err(KVH_EINVAL);
  const uint8_t* src = (const uint8_t*)p;
  size_t len = sz;
  int rc = 0;
  if (b->off > 0) {
    size_t fill = 64 - b->off;
    if (fill > len) fill = len;
    memcpy(&b->block[b->off], src, fill);
    b->off += fill; len -= fill; src += fill;
    if (b->off == 64) {
      if ((rc = stream_absorb_dev(m, b->block, 1))) return rc;
      b->off = 0;
    }
  }
  if (len > 0) {
    b->off = len & 63;
    if (len > b->off && (rc = stream_absorb_dev(m, src, (len - b->off) / 64))) return rc;
    memcpy(b->block, &src[len - b->off], b->off);
  }
  return set_err(0);
}

int kvh_meow128_final(kvh_meow_ctx_t* m, kvh_meow_block_t* b, uint64_t* k1, uint64_t* k2) {
  if (!m || !b || !k1 || !k2) return set_err(KVH_EINVAL);
  std::lock_guard<std::mutex> g(g_stage.mu);
  int rc = stage_reserve(64 + 64 + 16);
  if (rc) return rc;
  uint8_t* d = g_stage.dev;
  hipError_t e = hipMemcpy(d, m->ctx, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 64, b->block, 64, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(e);
  hipLaunchKernelGGL(k_stream_final, dim3(1), dim3(64), 0, 0, (const uint32_t*)d, (const uint8_t*)(d + 64),
                     (uint64_t)b->off, *k1, *k2, (uint64_t)b->total_update_sz, (uint64_t*)(d + 128));
  if ((rc = launch_done())) return rc;
  uint64_t o[2];
  e = hipMemcpy(o, d + 128, 16, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_err(e);
  *k1 = o[0]; *k2 = o[1];
  return set_err(0);
}

int kvh_meow_test(const void* p, size_t sz, uint64_t* k1, uint64_t* k2) {
  kvh_meow_ctx_t m;
  kvh_meow_block_t b;
  int rc = kvh_meow128_init(&m, &b, *k1, *k2, sz);
  if (!rc) rc = kvh_meow128_update(&m, &b, p, sz);
  if (!rc) rc = kvh_meow128_final(&m, &b, k1, k2);
  return rc;
}

int kvh_hash_key_frag(const uint64_t seed[2], const kvh_key_frag_t* frag, uint64_t* k, uint64_t* k2) {
  if (!seed || !frag || !k || !k2) return set_err(KVH_EINVAL);
  const void* p = frag->buf;
  size_t len = frag->keylen;
  uint64_t o[2];
  int rc = seeded_host(&p, &len, 1, seed, o, KVH_FIXUP);
  if (rc) return rc;
  *k = o[0]; *k2 = o[1];
  return 0;
}

int kvh_hash_key_frags(const uint64_t seed[2], const kvh_key_frag_t* const* frags, size_t n, uint64_t* out) {
  if (!seed || (n && (!frags || !out))) return set_err(KVH_EINVAL);
  std::vector<const void*> ps(n);
  std::vector<size_t> ls(n);
  std::vector<uint64_t> seeds(2 * n);
  for (size_t i = 0; i < n; i++) {
    ps[i] = frags[i]->buf; ls[i] = frags[i]->keylen;
    seeds[2 * i] = seed[0]; seeds[2 * i + 1] = seed[1];
  }
  return seeded_host(ps.data(), ls.data(), n, seeds.data(), out, KVH_FIXUP);
}


int kvh_last_error(void) { return t_last_err; }

const char* kvh_strerror(int err) {
  if (err == 0) return "ok";
  if (err == KVH_EINVAL) return "invalid argument";
  if (err == KVH_ENOMEM) return "out of memory";
  if (err == KVH_ENODEV) return "no device";
  if (err <= KVH_EHIP_BASE) return hipGetErrorString((hipError_t)(KVH_EHIP_BASE - err));
  return "unknown error";
}

const char* kvh_version(void) { return KVH_VERSION; }

int kvh_device_synchronize(void) {
  hipError_t e = hipDeviceSynchronize();
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

// Every knob selects among kernels whose outputs are the same hashes (or
// sizes the host pipeline); the ablation and research knobs exist only in
// the experiments build.  Atomic exchange: safe against concurrent calls.
int kvh_set_tuning(int k, int value) {
  auto set = [](Knob& g, int v) { return g.exchange(v, std::memory_order_relaxed); };
  switch (k) {
    case 0: if (value != 0 && value != 2 && value != 4) return KVH_EINVAL; return set(g_tune_nt, value);
    case 1: if (value < 1 || value > 8) return KVH_EINVAL; return set(g_tune_wgmul, value);
    case 2: return set(g_tune_generic, value ? 1 : 0);
    case 3: if (value < 0 || value > 8 || value == 5 || value == 6 || value == 7) return KVH_EINVAL;
            return set(g_tune_kpl, value);
    case 7: if (value != 0 && value != 7 && value != 13 && (value < 23 || value > 25) &&
                !(g_exp.var_knob && g_exp.var_knob(value)))
              return KVH_EINVAL;
            return set(g_tune_var, value);
    case 8: return set(g_tune_ms_lanes, value ? 1 : 0);
    case 14: if (value < 0 || value > 6) return KVH_EINVAL; return set(g_tune_crc_var, value);
    case 15: if (value < 1 || value > 1024) return KVH_EINVAL; return set(g_tune_pipe_mib, value);
    case 16: if (value < 2 || value > 16) return KVH_EINVAL; return set(g_tune_pipe_slots, value);
    case 17: if (value < 0 || value > 64) return KVH_EINVAL; return set(g_tune_sort_bits, value);
    case 18: if (value < 0 || value > 2) return KVH_EINVAL; return set(g_tune_spans, value);
    case 19: if (value < 0 || value > 1) return KVH_EINVAL; return set(g_tune_tok, value);
    case 20: if (value < 0 || value > 2) return KVH_EINVAL; return set(g_tune_sort_engine, value);
    case 21: if (value < 0 || value > (1 << 20)) return KVH_EINVAL; return set(g_tune_tiny, value);
    case 22: if (value < 0 || value > 1) return KVH_EINVAL; return set(g_tune_pl, value);
    default: return g_exp.set_tuning ? g_exp.set_tuning(k, value) : KVH_EINVAL;
  }
}

}  // extern "C"
