// kvh_varlen.hip -- the variable-length Meow128 kernels (config C2: keys
// packed back to back with u64 offsets) and the runtime-length generic
// kernel; the C-ABI entry points (kvh.hip) call var_dispatch /
// generic_launch after checking their arguments.  See DESIGN.md §3.3.
//   k_var9<NT,NW,KF,PF>   per-wave 256-key windows sorted by 16-byte length
//                         class, keys read as dwordx4 groups, one
//                         straight-line variant per chunk (the C2 default)
//   k_var6<NT,WIN,NW,SH>  the round-2 sorted-window kernel (knob 7 = 13, 7: experiments build only)
//   k_generic<VAR,NT>     any length: fixed stride or u64 offsets, one lane per key
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <atomic>
#include <algorithm>
#include "meow_dev.hpp"
#include "kvh_internal.hpp"
#include "kvh_var.hpp"
#include "tickets.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

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
// Keys used in several rounds (a block's chunks, the Mixer) are prepared
// once for the two-table round (PKY, LdsTab::prep; 2.89 vs 2.93 ms).
// The variants need ~165 VGPRs, so 12 waves per CU; hashes go straight to
// the wave's LDS stage at their input slot, records are 8 bytes
// (window offset, length << 8 | slot), and no per-window value lives in a
// register array.  Windows spanning 4 GiB or holding a key of 16 MiB or
// more take wide_window (input order, u64 offsets and lengths).

// AB (experiments build only, knob 7 = 61-69): counter ablations whose
// outputs are not hashes -- 1 no window sort (records in input order; timed on
// input already sorted by class within each window), 2-4 and 7 meow_a's (see
// there), 5 the table rounds replaced by one XOR per column, 6 no hashing,
// 8 every lane's key read from window base + 48 lane (the chunk's loads as
// coalesced as keys stored contiguously in lane order), 10 the four lanes of
// each quad read the quad's first key (the line count of a quad-per-key
// load).  (9, the stable window sort, became the product's in round 5.)
template <int NT, int NW, int KF, bool PF = false, bool PKY = true, bool CL = false, bool Q = false, int AB = 0>
__global__ void __launch_bounds__(NW * 64)
k_var9(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n, uint64_t s1, uint64_t s2,
       uint64_t* __restrict__ out, uint32_t flags, unsigned long long* __restrict__ tk = nullptr) {
  // per wave: the hash stage (4 KiB); while sorting it holds the bucket counts
  // (first KiB) and the sorted records (last 2 KiB), which each lane then
  // takes into registers (its four sorted positions) before hashes land
  constexpr int WIN = 256, M = WIN / 64, AREA = WIN * 16;
  // one LDS object, tables first: a lookup address is then the v_perm result
  // itself (a table at a nonzero base costs one v_add per lookup)
  constexpr int kTabB = LdsTab<NT>::kWords * 4, kFullB = kLT * (int)sizeof(VConst9), kKfB = KF * 64;
  constexpr int kTkB = Q ? (int)sizeof(WaveTickets) : 0;  // the ticket ring, last
  constexpr int kBytes = kTabB + kFullB + kKfB + NW * AREA + kTkB;
  static_assert(kBytes <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint32_t smem[(kBytes + 3) / 4];
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
  // Q (knob 7 = 46): windows in address order through wave tickets (tickets.hpp)
  WaveTickets& WT = *(WaveTickets*)((uint8_t*)smem + kBytes - kTkB);
  if constexpr (Q) wt_init(WT, tk);
  for (uint64_t w = Q ? wt_next(WT, tk, NW) : gw; w < nwin; w = Q ? wt_next(WT, tk, NW) : w + tw) {
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
    uint2 rc0, rc1, rc2, rc3;
    if constexpr (AB == 1) {
      rc0 = make_uint2(o[0], (L[0] << 8) | lane);
      rc1 = make_uint2(o[1], (L[1] << 8) | (64 + lane));
      rc2 = make_uint2(o[2], (L[2] << 8) | (128 + lane));
      rc3 = make_uint2(o[3], (L[3] << 8) | (192 + lane));
    } else {
    // counting sort of the window by 16-byte length class
#pragma unroll
    for (int q = 0; q < 4; q++) hist[lane * 4 + q] = 0;
    wave_sync();
#pragma unroll
    for (int m = 0; m < M; m++) {
      const uint32_t j = lane + 64 * m;
      // 64 length classes, one counter each (of four slots: the scan below
      // reads them as before): the ranks of one instruction's lanes come back
      // in lane order, so a class's keys keep their input order and a chunk's
      // loads walk the window forward -- 2 % over four sub-counters by
      // lane & 3, which spread a class's keys (round 5, profiles/r05/s5/)
      b[m] = ((L[m] >> 4) < 63u ? (L[m] >> 4) : 63u) * 4u;
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
    rc0 = rec[lane]; rc1 = rec[64 + lane]; rc2 = rec[128 + lane]; rc3 = rec[192 + lane];
    wave_sync();  // the stage takes hashes from here on
    }
    const uint8_t* base = keys + ws;
#pragma unroll 1
    for (int c = 0; c < M; c++) {
      const uint32_t pos = 64 * c + lane;
      const bool valid = pos < k;
      const uint2 rc = rc0;
      rc0 = rc1; rc1 = rc2; rc2 = rc3;
      const uint32_t kl = valid ? rc.y >> 8 : 0u;
      uint32_t lead_x = rc.x;
      if constexpr (AB == 10) {  // the key of the quad's first lane (when it is a valid position)
        const uint32_t lx = (uint32_t)__shfl((int)rc.x, (int)(lane & ~3u), 64);
        if ((64 * c + (lane & ~3u)) < k) lead_x = lx;
      }
      const bool al = __ballot(kl >= 64u) != 0;
      const int cm = __ballot((kl & 48u) == 48u) ? 48 : __ballot((kl & 48u) >= 32u) ? 32
                   : __ballot((kl & 48u) >= 16u) ? 16 : 0;
      if (valid) {
        uint32_t kx = rc.x;
        if constexpr (AB == 8) {  // pretend the chunk's keys lie back to back in lane order
          const uint64_t fake = 48ull * lane;
          if (fake + kl + 16 <= wend) kx = (uint32_t)fake;
        }
        if constexpr (AB == 10) {  // the four lanes of a quad read one key's lines (the access
          // pattern of a quad-per-key load: 16 keys' lines per load instruction instead of 64)
          if ((uint64_t)lead_x + kl + 16 <= wend) kx = lead_x;
        }
        const uint8_t* p = base + kx;
        const bool safe = (uint64_t)kx + kl + 16 <= wend;  // whole dwordx4 groups stay in the buffer
        Blk h;
        if constexpr (AB == 6) {
          h = bzero();
          h.w[0] = kl;
        } else if constexpr (AB == 5) {
          const XorTab X;
          const LdsKV9<XorTab, KF> K(kfull, kf, kl, s1, s2, X);
          if (al) h = meow_a<true, 48, PF, PKY, CL>(p, kl, safe, K, X);
          else if (cm == 48) h = meow_a<false, 48, PF, PKY, CL>(p, kl, safe, K, X);
          else if (cm == 32) h = meow_a<false, 32, PF, PKY, CL>(p, kl, safe, K, X);
          else if (cm == 16) h = meow_a<false, 16, PF, PKY, CL>(p, kl, safe, K, X);
          else h = meow_a<false, 0, PF, PKY, CL>(p, kl, safe, K, X);
        } else {
          constexpr int A2 = (AB >= 2 && AB <= 4) || AB == 7 ? AB : 0;
          const LdsKV9<LdsTab<NT>, KF> K(kfull, kf, kl, s1, s2, T);
          if (al) h = meow_a<true, 48, PF, PKY, CL, A2>(p, kl, safe, K, T);
          else if (cm == 48) h = meow_a<false, 48, PF, PKY, CL, A2>(p, kl, safe, K, T);
          else if (cm == 32) h = meow_a<false, 32, PF, PKY, CL, A2>(p, kl, safe, K, T);
          else if (cm == 16) h = meow_a<false, 16, PF, PKY, CL, A2>(p, kl, safe, K, T);
          else h = meow_a<false, 0, PF, PKY, CL, A2>(p, kl, safe, K, T);
        }
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
  if constexpr (Q) wt_done(tk);
}

}  // namespace

namespace kvh {
namespace rt {

int generic_launch(bool var, const uint8_t* keys, const uint64_t* offs, uint32_t fixed_len, uint64_t n,
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

int var_dispatch(const uint8_t* kp, const uint64_t* offsets, uint64_t n, uint64_t seed1, uint64_t seed2,
                 uint64_t* out, uint32_t flags, hipStream_t st, int cus) {
  const int var = knob(g_tune_var);
  const uint32_t grid = grid_for(n / 4 + 1, cus, 1);
  switch (var) {
    case 0: {
      uint64_t s[16] = {seed1, seed2};
      return generic_launch(true, kp, offsets, 0, n, s, 1, out, flags, st, cus);
    }
    case 46: {  // the default: windows in address order (wave tickets), unless knob 24 = 1 or a captured launch
      unsigned long long* tk = nullptr;
      if (knob(g_tune_order) != 1)
        if (int rc = stream_tickets(st, &tk)) return rc;
      if (tk) {
        hipLaunchKernelGGL((k_var9<2, 16, 256, false, true, false, true>), dim3(grid), dim3(1024), 0, st, kp, offsets,
                           (uint64_t)n, seed1, seed2, out, flags, tk);
        return launch_done();
      }
    }
      [[fallthrough]];
    case 23:  // the static window order
      hipLaunchKernelGGL((k_var9<2, 16, 256>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2,
                         out, flags);
      return launch_done();
#ifdef KVH_EXPERIMENTS  // the variants that lost their A/B (rounds 2-4): experiments build only
    case 13:
      hipLaunchKernelGGL((k_var6<2, 256, kBlock / 64, 4>), dim3(grid), dim3(kBlock), 0, st, kp, offsets,
                         (uint64_t)n, seed1, seed2, out, flags);
      return launch_done();
    case 7:
      hipLaunchKernelGGL((k_var6<2, 256>), dim3(grid), dim3(kBlock), 0, st, kp, offsets, (uint64_t)n, seed1, seed2,
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
    case 47:    // round-4 A/B: 46 with four tables at 16 copies (LdsTab<5>)
    case 48:    // round-4 A/B: 46 with 12 waves per workgroup
    case 49:    // round-4 A/B: 46 with the next block's groups in flight
    case 50: {  // round-4 A/B: 25 (12 waves, next block's groups in flight) in address order
      unsigned long long* tk = nullptr;
      if (int rc = stream_tickets(st, &tk)) return rc;
      if (!tk) return set_err(KVH_EINVAL);
      if (var == 47)
        hipLaunchKernelGGL((k_var9<5, 16, 256, false, true, false, true>), dim3(grid), dim3(1024), 0, st, kp, offsets,
                           (uint64_t)n, seed1, seed2, out, flags, tk);
      else if (var == 49)
        hipLaunchKernelGGL((k_var9<2, 16, 256, true, true, false, true>), dim3(grid), dim3(1024), 0, st, kp, offsets,
                           (uint64_t)n, seed1, seed2, out, flags, tk);
      else if (var == 50)
        hipLaunchKernelGGL((k_var9<2, 12, 192, true, true, false, true>), dim3(grid), dim3(768), 0, st, kp, offsets,
                           (uint64_t)n, seed1, seed2, out, flags, tk);
      else
        hipLaunchKernelGGL((k_var9<2, 12, 192, false, true, false, true>), dim3(grid), dim3(768), 0, st, kp, offsets,
                           (uint64_t)n, seed1, seed2, out, flags, tk);
      return launch_done();
    }
    case 45:  // round-4 A/B: clamped group loads (AChunks::chunk_cl)
      hipLaunchKernelGGL((k_var9<2, 16, 256, false, true, true>), dim3(grid), dim3(1024), 0, st, kp, offsets,
                         (uint64_t)n, seed1, seed2, out, flags);
      return launch_done();
    case 61: case 62: case 63: case 64: case 65: case 66: case 67: case 68: case 70: {  // round-5 ablations (69 hashes)
      unsigned long long* tk = nullptr;
      if (int rc = stream_tickets(st, &tk)) return rc;
      if (!tk) return set_err(KVH_EINVAL);
#define KVH_AB(v) \
  case 60 + v: hipLaunchKernelGGL((k_var9<2, 16, 256, false, true, false, true, v>), dim3(grid), dim3(1024), 0, st, kp, \
                                  offsets, (uint64_t)n, seed1, seed2, out, flags, tk); break;
      switch (var) { KVH_AB(1) KVH_AB(2) KVH_AB(3) KVH_AB(4) KVH_AB(5) KVH_AB(6) KVH_AB(7) KVH_AB(8) KVH_AB(10) }
#undef KVH_AB
      return launch_done();
    }
    case 44:  // round-4 A/B: four tables at 16 copies in the same 64 KiB (LdsTab<5>)
      hipLaunchKernelGGL((k_var9<5, 16, 256>), dim3(grid), dim3(1024), 0, st, kp, offsets, (uint64_t)n, seed1, seed2,
                         out, flags);
      return launch_done();
#endif
    default:
      break;
  }
  if (int rc = 0; g_exp.var && g_exp.var(var, kp, offsets, n, seed1, seed2, out, flags, st, cus, &rc)) return rc;
  return set_err(KVH_EINVAL);
}

}  // namespace rt
}  // namespace kvh
