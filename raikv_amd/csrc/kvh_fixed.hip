// kvh_fixed.hip -- the fixed-length Meow128 kernels of the engine (configs
// C1, C3, C4 and the metric's 16-64 B range) and their launchers; the C-ABI
// entry points (kvh.hip) call fixed_dispatch / multiseed_dispatch after
// checking their arguments.  See DESIGN.md §3.1-3.3 and meow_dev.hpp.
//   k_fixed<L,NT,A16,U>   fixed length L in {8,16,..,64}, one seed, constants
//                         folded into SGPRs (C1, C4)
//   k_fixed_lanes         LA lanes per key, one seed each (C3)
//   k_fixed_ms            one lane per key, `arity` seeds (C3 fallback)
//   k_fixed_rt            any fixed length below one block (runtime L)
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
// chunk body one basic block.  64-byte keys at 16-byte aligned bases and
// 56-byte keys go by lane pairs instead (load_pair64 / load_pair56: lanes 2i,
// 2i+1 own keys i, 32+i of each 64-key group; each load instruction of the
// first two reads 32 contiguous bytes per key).
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
  constexpr bool PAIR = (A16 && L == 64) || L == 56;  // lane pairs (load_pair64 / load_pair56)
  const uint64_t kl = PAIR ? pair64_key((uint32_t)lane) : lane;
  for (uint64_t b = wave * 64 * U; b < n; b += step) {  // wave-uniform trip count
    Blk D[U][NC];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      if constexpr (L == 56) load_pair56(keys, b + 64 * u, last, (uint32_t)lane, D[u]);
      else if constexpr (PAIR) load_pair64(keys, b + 64 * u, last, (uint32_t)lane, D[u]);
      else load_fixed<L, A16, true>(keys + (j < last ? j : last) * L, D[u]);
    }
    Blk h[U];
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = meow_ct<L>(D[u], K, T);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + kl;
      store_h<true>(out, j < last ? j : last, h[u], fix);
    }
  }
}

#ifdef KVH_EXPERIMENTS  // lost its A/B to k_fixed_qw (round 4): experiments build only
// k_fixed with the chunks taken IN ADDRESS ORDER (round 4, knob 24 = 3/4/5;
// k_fixed_qw below is the default form).  A workgroup-iteration (16 waves x 64U keys) is one ticket from a
// per-stream counter (stream_tickets), the next ticket fetched one iteration
// ahead, so the chunks in flight on the whole chip form one compact address
// window, as a one-shot grid's do.  k_fixed's static order lets waves drift
// apart over a launch and the window spreads: on the same 3.2 GB the static
// persistent copy streams 5.2-5.4 TB/s, in-order tickets 6.7 TB/s, and a
// one-shot grid 6.2-6.5 TB/s but only 5.2 with its blocks scrambled
// (tools/stream_forms.hip, profiles/r04/s4-s5/).  The last workgroup to exit
// puts the counter pair back to zero.
template <int L, int NT, bool A16, int U, int R = 1>
__global__ void __launch_bounds__(kBlock)
k_fixed_q(const uint8_t* __restrict__ keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* __restrict__ out,
          uint32_t flags, unsigned long long* __restrict__ tk) {
  constexpr int NC = Plan<L>::NC;
  struct Smem { uint32_t tab[LdsTab<NT>::kWords]; unsigned long long tkl[2]; };  // tables first
  __shared__ Smem sm;
  uint32_t* lds = sm.tab;
  unsigned long long* tkl = sm.tkl;
  fill_tables<NT>(lds);
  if (threadIdx.x == 0) tkl[0] = atomicAdd(tk, 1ull);
  __syncthreads();
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint64_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t per_it = (uint64_t)(blockDim.x >> 6) * 64 * U * R;  // keys per ticket: R rounds of the 16 waves
  const uint64_t last = n - 1;
  for (uint32_t it = 0;; it++) {
    const uint64_t t = tkl[it & 1];
    if (threadIdx.x == 0) tkl[(it + 1) & 1] = atomicAdd(tk, 1ull);
    if (t * per_it >= n) break;  // workgroup-uniform
#pragma unroll 1
    for (int r = 0; r < R; r++) {
      const uint64_t b = t * per_it + ((uint64_t)r * (blockDim.x >> 6) + wv) * 64 * U;
      if (b < n) {  // wave-uniform
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
    __syncthreads();  // tkl[(it + 1) & 1] written before it is read; tkl[it & 1] read before it is rewritten
  }
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(tk + 1, 1ull) == (unsigned long long)gridDim.x - 1) {  // every other workgroup is done with tk
      atomicExch(tk, 0ull);
      atomicExch(tk + 1, 0ull);
    }
  }
}

#endif  // KVH_EXPERIMENTS

// k_fixed_qw: the same in-order tickets without the per-ticket barrier
// (tickets.hpp: each wave takes chunks one at a time through an LDS counter
// and a ring of prefetched workgroup tickets), so each wave runs at its own
// pace -- its loads under the other waves' rounds, as in k_fixed -- while
// the chip's chunks in flight stay one address window.
template <int L, int NT, bool A16, int U>
__global__ void __launch_bounds__(kBlock)
k_fixed_qw(const uint8_t* __restrict__ keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* __restrict__ out,
           uint32_t flags, unsigned long long* __restrict__ tk) {
  constexpr int NC = Plan<L>::NC;
  // one LDS object, tables first (a lookup address is the v_perm result itself)
  struct Smem { uint32_t tab[LdsTab<NT>::kWords]; WaveTickets W; };
  __shared__ Smem sm;
  uint32_t* lds = sm.tab;
  WaveTickets& W = sm.W;
  fill_tables<NT>(lds);
  wt_init(W, tk);
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  const uint64_t last = n - 1;
  constexpr bool PAIR = (A16 && L == 64) || L == 56;  // lane pairs (load_pair64 / load_pair56)
  const uint32_t kl = PAIR ? pair64_key(lane) : lane;
  for (;;) {
    const uint64_t b = wt_next(W, tk, wpb) * (64 * U);
    if (b >= n) break;  // wave-uniform: the wave's later chunks lie further on
    Blk D[U][NC];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      if constexpr (L == 56) load_pair56(keys, b + 64 * u, last, lane, D[u]);
      else if constexpr (PAIR) load_pair64(keys, b + 64 * u, last, lane, D[u]);
      else load_fixed<L, A16, true>(keys + (j < last ? j : last) * L, D[u]);
    }
    Blk h[U];
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = meow_ct<L>(D[u], K, T);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + kl;
      store_h<true>(out, j < last ? j : last, h[u], fix);
    }
  }
  wt_done(tk);
}

// Multi-seed (config C3, kv_hash_meow128_4_same_length_4_seed with one key
// in all slots, key_hash.c:1891-1937): LA = 2, 4 or 8 lanes per key, lane l
// hashes under seed (l & (LA-1)).  The output slot of (key i, seed a) is
// i*LA + a, so lane j of a chunk writes slot j: every store is one contiguous
// 1 KiB run (one lane per key with LA strided 16-byte stores inflated the
// write traffic 1.3x).  The LA lanes of a key load the same 16-byte pieces
// (same cache line, one request).  Constants are per lane (VGPRs), computed
// once in the prologue for the lane's fixed seed.
template <int L, int NT, bool A16, int U, int LA, bool Q = false>
__global__ void __launch_bounds__(kBlock)
k_fixed_lanes(const uint8_t* __restrict__ keys, uint64_t n, uint64_t* __restrict__ out, uint32_t flags,
              uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1, uint64_t a2, uint64_t b2, uint64_t a3,
              uint64_t b3, uint64_t a4, uint64_t b4, uint64_t a5, uint64_t b5, uint64_t a6, uint64_t b6,
              uint64_t a7, uint64_t b7, unsigned long long* __restrict__ tk = nullptr) {
  static_assert(LA == 2 || LA == 4 || LA == 8, "lanes per key");
  constexpr int NC = Plan<L>::NC;
  constexpr int SH = LA == 2 ? 1 : LA == 4 ? 2 : 3;
  // one LDS object, tables first; Q: chunks in address order through wave tickets (knob 24)
  struct Smem { uint32_t tab[LdsTab<NT>::kWords]; WaveTickets W; };
  __shared__ Smem sm;
  uint32_t* lds = sm.tab;
  fill_tables<NT>(lds);
  __syncthreads();
  if constexpr (Q) wt_init(sm.W, tk);
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
  for (uint64_t b = Q ? wt_next(sm.W, tk, blockDim.x >> 6) * (64 * U) : wave * 64 * U; b < ns;
       b = Q ? wt_next(sm.W, tk, blockDim.x >> 6) * (64 * U) : b + step) {
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
  if constexpr (Q) wt_done(tk);
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

template <int L, int NT, int U>
int launch_k(const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out, uint32_t flags,
             hipStream_t st, int cus) {
  const bool a16 = ((uintptr_t)keys & 15) == 0;
  const uint32_t grid = grid_for(n, cus, NT == 4 ? 1 : 2);
  // chunk order (knob 24): wave tickets (in address order)
  // by default, at every length with the keys per lane re-swept under them
  // (profiles/r04/s14/sweep.jsonl); knob 24 = 1, and a launch captured into a
  // graph (stream_tickets gives no words), the static order
  if (knob(g_tune_order) != 1) {
    unsigned long long* tk = nullptr;
    if (int rc = stream_tickets(st, &tk)) return rc;
#ifdef KVH_EXPERIMENTS
    const int ord = knob(g_tune_order);
#define KVH_Q(A, R) hipLaunchKernelGGL((k_fixed_q<L, NT, A, U, R>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, \
                                       out, flags, tk)
    if (tk && ord >= 3) {
      if (a16) { if (ord == 3) KVH_Q(true, 1); else if (ord == 4) KVH_Q(true, 4); else KVH_Q(true, 16); }
      else { if (ord == 3) KVH_Q(false, 1); else if (ord == 4) KVH_Q(false, 4); else KVH_Q(false, 16); }
      return launch_done();
    }
#undef KVH_Q
#endif
    if (tk) {
      if (a16)
        hipLaunchKernelGGL((k_fixed_qw<L, NT, true, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out, flags, tk);
      else
        hipLaunchKernelGGL((k_fixed_qw<L, NT, false, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, s1, s2, out, flags,
                           tk);
      return launch_done();
    }
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

// Q: chunks in address order through wave tickets (tickets.hpp, knob 24)
template <int NC, int NT, int U, bool Q = false>
__global__ void __launch_bounds__(kBlock)
k_fixed_rt(const uint8_t* __restrict__ keys, uint64_t n, uint32_t L, uint64_t s1, uint64_t s2,
           uint64_t* __restrict__ out, uint32_t flags, unsigned long long* __restrict__ tk = nullptr) {
  struct Smem { uint32_t tab[LdsTab<NT>::kWords]; WaveTickets W; };  // tables first
  __shared__ Smem sm;
  uint32_t* lds = sm.tab;
  fill_tables<NT>(lds);
  __syncthreads();
  if constexpr (Q) wt_init(sm.W, tk);
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  const uint64_t last = n - 1, total = n * (uint64_t)L;
  for (uint64_t b = Q ? wt_next(sm.W, tk, blockDim.x >> 6) * (64 * U) : wave * 64 * U; b < n;
       b = Q ? wt_next(sm.W, tk, blockDim.x >> 6) * (64 * U) : b + step) {  // wave-uniform trip count
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
  if constexpr (Q) wt_done(tk);
}

template <int NC, int NT, int U>
int launch_fixed_rt(const uint8_t* keys, uint64_t n, uint32_t L, uint64_t s1, uint64_t s2, uint64_t* out,
                    uint32_t flags, hipStream_t st, int cus) {
  const uint32_t grid = grid_for(n, cus, NT == 4 ? 1 : 2);
  unsigned long long* tk = nullptr;
  if (knob(g_tune_order) != 1)  // chunk order (knob 24): wave tickets unless 1 = static (or captured)
    if (int rc = stream_tickets(st, &tk)) return rc;
  if (tk) {
    hipLaunchKernelGGL((k_fixed_rt<NC, NT, U, true>), dim3(grid), dim3(kBlock), 0, st, keys, n, L, s1, s2, out,
                       flags, tk);
  } else {
    hipLaunchKernelGGL((k_fixed_rt<NC, NT, U>), dim3(grid), dim3(kBlock), 0, st, keys, n, L, s1, s2, out, flags,
                       nullptr);
  }
  return launch_done();
}

// Default (NT, U) per length, from the round-4 sweeps under wave tickets
// over 100M keys (profiles/r04/s14/sweep.jsonl, s16/ab.jsonl): Td0..Td3 in LDS
// (NT4: no rotations; 8 B 6 % over NT2) everywhere; keys per lane 4 at 8, 16,
// 24 and 32 B (32 B: 2.6 % over 2), 3 at 40 / 48 B (7 / 4 % over the round-3
// defaults), 1 at 56 / 64 B (4 / 8 %).  The other (NT, U) instances are the
// sweep's losers and compile only into the experiments build, where knobs 0
// and 3 select them (a pair with no instance runs the default).  56 and
// 64 B since the lane-pair loads (round 6, profiles/r06/c64_pair/): 64 B 3
// keys per lane (1.62 vs 1.69 ms at 1), 56 B 2 (1.585 vs 1.613; 3 spills).
template <int L>
struct FixedDefault {
  static constexpr int NT = 4;
  static constexpr int U = (L == 40 || L == 48 || L == 64) ? 3 : (L == 56 ? 2 : 4);
};

template <int L>
int launch_fixed_nt(const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out,
                    uint32_t flags, hipStream_t st, int cus) {
  if (int rc = 0; g_exp.fixed && g_exp.fixed(L, keys, n, s1, s2, out, flags, st, cus, knob(g_tune_nt), knob(g_tune_kpl), &rc))
    return rc;
  constexpr int dnt = FixedDefault<L>::NT, dkpl = FixedDefault<L>::U;
#ifdef KVH_EXPERIMENTS
  const int tnt = knob(g_tune_nt), tkpl = knob(g_tune_kpl);
  switch ((tnt ? tnt : dnt) * 100 + (tkpl ? tkpl : dkpl)) {
    case 401: return launch_k<L, 4, 1>(keys, n, s1, s2, out, flags, st, cus);
    case 402: return launch_k<L, 4, 2>(keys, n, s1, s2, out, flags, st, cus);
    case 404: return launch_k<L, 4, 4>(keys, n, s1, s2, out, flags, st, cus);
    case 201: return launch_k<L, 2, 1>(keys, n, s1, s2, out, flags, st, cus);
    case 202: return launch_k<L, 2, 2>(keys, n, s1, s2, out, flags, st, cus);
    case 204: return launch_k<L, 2, 4>(keys, n, s1, s2, out, flags, st, cus);
    case 408: if constexpr (L == 16 || L == 32) return launch_k<L, 4, 8>(keys, n, s1, s2, out, flags, st, cus); break;
    case 208: if constexpr (L == 16 || L == 32) return launch_k<L, 2, 8>(keys, n, s1, s2, out, flags, st, cus); break;
    case 403: if constexpr (L >= 40) return launch_k<L, 4, 3>(keys, n, s1, s2, out, flags, st, cus); break;
    case 203: if constexpr (L >= 40) return launch_k<L, 2, 3>(keys, n, s1, s2, out, flags, st, cus); break;
    default: break;  // a knob pair without an instance: this length's default
  }
#endif
  return launch_k<L, dnt, dkpl>(keys, n, s1, s2, out, flags, st, cus);
}

template <int L, int NT, int U>
int launch_lanes_v(const uint8_t* keys, uint64_t n, const uint64_t* s, uint32_t arity, uint64_t* out,
                   uint32_t flags, hipStream_t st, int cus) {
  const uint32_t grid = grid_for(n * arity, cus, NT == 4 ? 1 : 2);
  // chunk order (knob 24): 0 / 2 wave tickets (the default), 1 static (and captured launches)
  const int ord = knob(g_tune_order);
  unsigned long long* tk = nullptr;
  if (ord != 1)
    if (int rc = stream_tickets(st, &tk)) return rc;
#define KVH_LANES_V(LAv, Qv)                                                                                   \
  hipLaunchKernelGGL((k_fixed_lanes<L, NT, true, U, LAv, Qv>), dim3(grid), dim3(kBlock), 0, st, keys, n, out, flags, \
                     s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10], s[11], s[12], s[13],   \
                     s[14], s[15], tk)
  if (tk) {
    if (arity == 2) KVH_LANES_V(2, true); else if (arity == 4) KVH_LANES_V(4, true); else KVH_LANES_V(8, true);
  } else {
    if (arity == 2) KVH_LANES_V(2, false); else if (arity == 4) KVH_LANES_V(4, false); else KVH_LANES_V(8, false);
  }
#undef KVH_LANES_V
  return launch_done();
}

template <int L>
int launch_lanes_L(const uint8_t* keys, uint64_t n, const uint64_t* s, uint32_t arity, uint64_t* out,
                   uint32_t flags, hipStream_t st, int cus) {
  const bool a16 = ((uintptr_t)keys & 15) == 0;
  if constexpr (L == 32) {
    // C3's length: Td0..Td3 in LDS (no rotates, one 16-wave workgroup per CU)
    // -- 118 vs 112 G hash/s for Td0/Td1 with two workgroups per CU
    // (tools/tune.py, profiles/r02/c3_layout_ab.txt) -- and 4 keys per lane
    // under wave tickets (2.7 % over 2: profiles/r04/s16/ab.jsonl); the other
    // pairs in the experiments build (knobs 0 / 3)
    if (a16) {
#ifdef KVH_EXPERIMENTS
      const int nt = knob(g_tune_nt), kpl = knob(g_tune_kpl);
      switch ((nt ? nt : 4) * 10 + (kpl ? kpl : 4)) {
        case 21: return launch_lanes_v<L, 2, 1>(keys, n, s, arity, out, flags, st, cus);
        case 24: return launch_lanes_v<L, 2, 4>(keys, n, s, arity, out, flags, st, cus);
        case 41: return launch_lanes_v<L, 4, 1>(keys, n, s, arity, out, flags, st, cus);
        case 42: return launch_lanes_v<L, 4, 2>(keys, n, s, arity, out, flags, st, cus);
        default: break;
      }
#endif
      return launch_lanes_v<L, 4, 4>(keys, n, s, arity, out, flags, st, cus);
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

}  // namespace

namespace kvh {
namespace rt {

int fixed_dispatch(const uint8_t* k, uint32_t key_len, uint64_t n, uint64_t seed1, uint64_t seed2, uint64_t* out,
                   uint32_t flags, hipStream_t st, int cus) {
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
    // NT4, 4 keys per lane for one 16-byte chunk, 2 above (the experiments
    // build has the other pairs behind knobs 0 / 3)
    const int nc = (int)(key_len + 15) / 16;
#ifdef KVH_EXPERIMENTS
    const int tnt = knob(g_tune_nt), tkpl = knob(g_tune_kpl);
    const int nt = tnt ? tnt : 4, kpl = tkpl ? tkpl : (nc == 1 ? 4 : 2);
    switch (nc * 1000 + nt * 10 + kpl) {
#define KVH_RT(NCv, NTv, Uv) \
  case NCv * 1000 + NTv * 10 + Uv: return launch_fixed_rt<NCv, NTv, Uv>(k, n, key_len, seed1, seed2, out, flags, st, cus);
      KVH_RT(1, 4, 2) KVH_RT(1, 4, 8) KVH_RT(1, 2, 4) KVH_RT(1, 2, 8)
      KVH_RT(2, 4, 4) KVH_RT(2, 2, 2) KVH_RT(2, 2, 4)
      KVH_RT(3, 4, 4) KVH_RT(3, 2, 2) KVH_RT(3, 2, 4)
      KVH_RT(4, 4, 4) KVH_RT(4, 2, 2) KVH_RT(4, 2, 4)
#undef KVH_RT
      default: break;  // a knob pair without an instance: the default
    }
#endif
    switch (nc) {
      case 1: return launch_fixed_rt<1, 4, 4>(k, n, key_len, seed1, seed2, out, flags, st, cus);
      case 2: return launch_fixed_rt<2, 4, 2>(k, n, key_len, seed1, seed2, out, flags, st, cus);
      case 3: return launch_fixed_rt<3, 4, 2>(k, n, key_len, seed1, seed2, out, flags, st, cus);
      default: return launch_fixed_rt<4, 4, 2>(k, n, key_len, seed1, seed2, out, flags, st, cus);
    }
  }
  uint64_t s[16] = {seed1, seed2};
  return generic_launch(false, k, nullptr, key_len, n, s, 1, out, flags, st, cus);
}

int multiseed_dispatch(const uint8_t* k, uint32_t key_len, uint64_t n, const uint64_t* s, uint32_t arity,
                       uint64_t* out, uint32_t flags, hipStream_t st, int cus) {
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
  return generic_launch(false, k, nullptr, key_len, n, s, arity, out, flags, st, cus);
}

}  // namespace rt
}  // namespace kvh
