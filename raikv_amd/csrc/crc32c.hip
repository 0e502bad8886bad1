// crc32c.hip -- SURVEY.md §8 row f4: batched CRC32C (raikv's kv_crc_c
// family, src/key_hash.c:27-179) on gfx950.
//
// kv_crc_c(p, sz, seed) is the SSE4.2 crc32 instruction chain started at
// `seed` with no pre/post inversion (key_hash.c:53-63): 8-byte steps, then
// 4/2/1-byte steps.  CRC is byte-serial, so the chunking does not change
// the value: it is the reflected Castagnoli CRC (polynomial 0x82F63B78) of
// the bytes, register initialised to seed, no final xor.
//
// Device form: slice-by-4.  Per 4 input bytes w, x = r ^ w and
//   r' = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3]
// with T_k[v] = CRC of byte v followed by k zero bytes.  A tail of n < 4
// bytes is the same step on the zero-extended bytes with tables
// T_{n-1} .. T_0 and r shifted right by 8n.  The four tables sit in LDS
// replicated 32 times, lane l reading copy l & 31 (the layout of the Meow
// T-tables, meow_dev.hpp LdsTab<4>): conflict-free random lookups, one
// v_perm_b32 per lookup address.  One LDS lookup per key byte; a 16-byte
// key moves 20 bytes of HBM, so short keys are HBM-bound.
//
//   k_crc_fixed   n keys of key_len bytes at stride key_len
//   k_crc_var     n keys by u64 offsets (lane per key)
// Both take an optional per-key seed array (kv_crc_c_array semantics:
// seed[i] in, crc out) and otherwise one seed for all keys.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <vector>
#include <type_traits>
#include "kvh_internal.hpp"
#include "tickets.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

constexpr uint32_t kPoly = 0x82F63B78u;  // reflected Castagnoli

struct CrcTabs {
  uint32_t t[4][256];
};

constexpr CrcTabs make_crc_tabs() {
  CrcTabs c{};
  for (uint32_t v = 0; v < 256; v++) {
    uint32_t r = v;
    for (int b = 0; b < 8; b++) r = (r >> 1) ^ ((r & 1u) ? kPoly : 0u);
    c.t[0][v] = r;
  }
  for (int k = 1; k < 4; k++)
    for (uint32_t v = 0; v < 256; v++) c.t[k][v] = (c.t[k - 1][v] >> 8) ^ c.t[0][c.t[k - 1][v] & 255u];
  return c;
}
constexpr CrcTabs kCrc = make_crc_tabs();
static_assert(kCrc.t[0][1] == 0xF26B8303u, "CRC32C table");  // standard Castagnoli table entry

__constant__ CrcTabs c_crc = kCrc;

constexpr int kWords = 4 * 8192;  // 4 tables x 256 entries x 32 copies

// LDS slot s holds table T_{3-s}, so slot s is indexed by byte s of x.
// R = 32 copies (conflict-free), byte address of (slot s, value v, copy c):
//   (s >> 1) << 16 | v << 8 | (s & 1) << 7 | c << 2
// R = 16 copies (64 KiB, lanes 16 apart share a bank: 2-way), all four
// slots in one 256-byte row per value:
//   v << 8 | s << 6 | c << 2
// eight words per thread per batch, every load before the first write (as
// fill_tables, meow_dev.hpp)
template <int R = 32>
__device__ __forceinline__ void fill_crc(uint32_t* lds) {
  constexpr uint32_t words = R == 32 ? (uint32_t)kWords : (uint32_t)kWords / 2;
  constexpr int B = 8;
  const uint32_t bd = blockDim.x;
  auto batch = [&](uint32_t i0, auto guarded) {
    uint32_t x[B];
#pragma unroll
    for (int k = 0; k < B; k++) {
      const uint32_t i0k = i0 + (uint32_t)k * bd, i = (guarded && i0k >= words) ? 0u : i0k;
      const uint32_t s = R == 32 ? ((((i >> 14) & 1u) << 1) | ((i >> 5) & 1u)) : ((i >> 4) & 3u);
      x[k] = c_crc.t[3 - s][(i >> 6) & 255u];
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
      const uint32_t i = i0 + (uint32_t)k * bd;
      if (!guarded || i < words) lds[i] = x[k];
    }
  };
  if (words % (B * bd) == 0) {  // workgroup-uniform: whole batches
    for (uint32_t i0 = threadIdx.x; i0 < words; i0 += B * bd) batch(i0, std::false_type{});
  } else {
    for (uint32_t i0 = threadIdx.x; i0 < words; i0 += B * bd) batch(i0, std::true_type{});
  }
}

template <int R = 32>
struct CrcLdsT {
  static_assert(R == 32 || R == 16, "table copies");
  const uint32_t* lds;
  uint32_t lw[4];
  __device__ __forceinline__ explicit CrcLdsT(const uint32_t* p) : lds(p) {
    const uint32_t lane = (threadIdx.x & (uint32_t)(R - 1)) << 2;
#pragma unroll
    for (int s = 0; s < 4; s++)
      lw[s] = R == 32 ? (((uint32_t)(s >> 1) << 16) | ((uint32_t)(s & 1) << 7) | lane) : (((uint32_t)s << 6) | lane);
  }
  __device__ __forceinline__ uint32_t ld(uint32_t a) const { return *(const uint32_t*)((const char*)lds + a); }
  template <int K> static constexpr uint32_t sel() { return 0x03020000u | ((4u + K) << 8); }
  // four bytes: r' = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3]
  __device__ __forceinline__ uint32_t word(uint32_t r, uint32_t w) const {
    const uint32_t x = r ^ w;
    const uint32_t a = ld(__builtin_amdgcn_perm(x, lw[0], sel<0>()));
    const uint32_t b = ld(__builtin_amdgcn_perm(x, lw[1], sel<1>()));
    const uint32_t c = ld(__builtin_amdgcn_perm(x, lw[2], sel<2>()));
    const uint32_t d = ld(__builtin_amdgcn_perm(x, lw[3], sel<3>()));
    return xor3(a, b, c) ^ d;
  }
  // n in 1..3 bytes (zero-extended in w): tables T_{n-1}..T_0 = slots 4-n..3
  __device__ __forceinline__ uint32_t tail(uint32_t r, uint32_t w, uint32_t n) const {
    const uint32_t x = r ^ w;
    uint32_t o = r >> (8 * n);
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t s = 4 - n + i;
      const uint32_t v = (x >> (8 * i)) & 255u, c = (threadIdx.x & (uint32_t)(R - 1)) << 2;
      const uint32_t a = R == 32 ? (((s >> 1) << 16) | (v << 8) | ((s & 1) << 7) | c) : ((v << 8) | (s << 6) | c);
      o ^= ld(a);
    }
    return o;
  }
};

using CrcLds = CrcLdsT<32>;

// kv_crc_c over one key of len bytes; 16-byte pieces through the
// dword-aligned loaders (no over-read past the key).
__device__ __forceinline__ uint32_t crc_key(const uint8_t* p, uint64_t len, uint32_t r, const CrcLds& T) {
  uint64_t o = 0;
  for (; o + 16 <= len; o += 16) {
    const Blk b = load16_full(p + o);
    r = T.word(r, b.w[0]);
    r = T.word(r, b.w[1]);
    r = T.word(r, b.w[2]);
    r = T.word(r, b.w[3]);
  }
  const uint32_t t = (uint32_t)(len - o);
  if (t) {
    const Blk b = load_bytes(p + o, t);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int left = (int)t - 4 * c;
      if (left >= 4) r = T.word(r, b.w[c]);
      else if (left > 0) r = T.tail(r, b.w[c], (uint32_t)left);
    }
  }
  return r;
}

// Compile-time length: every piece of the U keys of a chunk is loaded
// before the first table step (U*ceil(L/16) 16-byte loads per lane in
// flight), then the slice-by-4 chains run.
template <int L, int U, bool Q = false>
__global__ void __launch_bounds__(kBlock)
k_crc_fixed_ct(const uint8_t* __restrict__ keys, uint64_t n, const uint32_t* __restrict__ seeds, uint32_t seed,
               uint32_t* __restrict__ out, unsigned long long* __restrict__ tk = nullptr) {
  constexpr int NP = (L + 15) / 16;
  // one LDS object, tables first; Q: chunks in address order through wave tickets (knob 24, tickets.hpp)
  struct Smem { uint32_t tab[kWords]; WaveTickets W; };
  __shared__ Smem sm;
  uint32_t* lds = sm.tab;
  fill_crc(lds);
  __syncthreads();
  if constexpr (Q) wt_init(sm.W, tk);
  const CrcLds T(lds);
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  for (uint64_t b = Q ? wt_next(sm.W, tk, blockDim.x >> 6) * (64 * U) : wave * 64 * U; b < n;
       b = Q ? wt_next(sm.W, tk, blockDim.x >> 6) * (64 * U) : b + step) {
    Blk D[U][NP];
    uint32_t r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = std::min<uint64_t>(b + 64 * u + lane, n - 1);
      const uint8_t* p = keys + j * L;
#pragma unroll
      for (int c = 0; c < NP; c++) {
        D[u][c] = (16 * c + 16 <= L) ? load16_full(p + 16 * c) : load_bytes(p + 16 * c, L - 16 * c);
      }
      r[u] = seeds ? seeds[j] : seed;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int c = 0; c < NP; c++) {
#pragma unroll
        for (int w = 0; w < 4; w++) {
          const int left = L - 16 * c - 4 * w;
          if (left >= 4) r[u] = T.word(r[u], D[u][c].w[w]);
          else if (left > 0) r[u] = T.tail(r[u], D[u][c].w[w], (uint32_t)left);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      if (j < n) __builtin_nontemporal_store(r[u], out + j);
    }
  }
  if constexpr (Q) wt_done(tk);
}

template <int U>
__global__ void __launch_bounds__(kBlock)
k_crc_fixed(const uint8_t* __restrict__ keys, uint32_t L, uint64_t n, const uint32_t* __restrict__ seeds,
            uint32_t seed, uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[kWords];
  fill_crc(lds);
  __syncthreads();
  const CrcLds T(lds);
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  for (uint64_t b = wave * 64 * U; b < n; b += step) {
    uint32_t r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = std::min<uint64_t>(b + 64 * u + lane, n - 1);
      r[u] = crc_key(keys + j * L, L, seeds ? seeds[j] : seed, T);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      if (j < n) __builtin_nontemporal_store(r[u], out + j);
    }
  }
}

__global__ void __launch_bounds__(kBlock)
k_crc_var(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n,
          const uint32_t* seeds, uint32_t seed, uint32_t* out) {  // seeds may alias out (in/out seeds)
  __shared__ uint32_t lds[kWords];
  fill_crc(lds);
  __syncthreads();
  const CrcLds T(lds);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
    const uint64_t a = offs[j], e = offs[j + 1];
    out[j] = crc_key(keys + a, e - a, seeds ? seeds[j] : seed, T);
  }
}

// kv_crc_c over one key with the next 16-byte piece in flight while the
// current one steps through the tables.
template <class Tab>
__device__ __forceinline__ uint32_t crc_key_pf(const uint8_t* p, uint64_t len, uint32_t r, const Tab& T) {
  uint64_t o = 0;
  if (len >= 16) {
    Blk cur = load16_full(p);
    for (; o + 32 <= len; o += 16) {
      const Blk nxt = load16_full(p + o + 16);
      r = T.word(r, cur.w[0]); r = T.word(r, cur.w[1]);
      r = T.word(r, cur.w[2]); r = T.word(r, cur.w[3]);
      cur = nxt;
    }
    r = T.word(r, cur.w[0]); r = T.word(r, cur.w[1]);
    r = T.word(r, cur.w[2]); r = T.word(r, cur.w[3]);
    o += 16;
  }
  const uint32_t t = (uint32_t)(len - o);
  if (t) {
    const Blk b = load_bytes(p + o, t);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int left = (int)t - 4 * c;
      if (left >= 4) r = T.word(r, b.w[c]);
      else if (left > 0) r = T.tail(r, b.w[c], (uint32_t)left);
    }
  }
  return r;
}

// kv_crc_c over one key read as dwordx4 groups of its dword-aligned span
// (AChunks, meow_dev.hpp): one load instruction, so one L2 request, per 16
// bytes, where crc_key_pf's byte-aligned pieces cost two and its tail up to
// five.  Two groups are in flight ahead of the piece being stepped.
template <class Tab>
__device__ __forceinline__ uint32_t crc_key_g2(const AChunks& A, uint32_t len, uint32_t r, const Tab& T, Blk cur,
                                               Blk nxt) {
  uint32_t k = 0;
  for (; 16 * k + 16 <= len; k++) {
    const Blk nn = A.chunk(k + 2);
    const Blk b = A.piece(cur, nxt);
    r = T.word(r, b.w[0]); r = T.word(r, b.w[1]);
    r = T.word(r, b.w[2]); r = T.word(r, b.w[3]);
    cur = nxt;
    nxt = nn;
  }
  const uint32_t t = len - 16 * k;
  if (t) {
    const Blk b = A.piece(cur, nxt);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int left = (int)t - 4 * c;
      if (left >= 4) r = T.word(r, b.w[c]);
      else if (left > 0) r = T.tail(r, b.w[c], (uint32_t)left);
    }
  }
  return r;
}
template <class Tab>
__device__ __forceinline__ uint32_t crc_key_g(const uint8_t* p, uint32_t len, bool safe, uint32_t r,
                                              const Tab& T) {
  const AChunks A(p, len, safe);
  Blk cur = A.chunk(0), nxt = A.chunk(1);
  uint32_t k = 0;
  for (; 16 * k + 16 <= len; k++) {
    const Blk nn = A.chunk(k + 2);
    const Blk b = A.piece(cur, nxt);
    r = T.word(r, b.w[0]); r = T.word(r, b.w[1]);
    r = T.word(r, b.w[2]); r = T.word(r, b.w[3]);
    cur = nxt;
    nxt = nn;
  }
  const uint32_t t = len - 16 * k;
  if (t) {
    const Blk b = A.piece(cur, nxt);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int left = (int)t - 4 * c;
      if (left >= 4) r = T.word(r, b.w[c]);
      else if (left > 0) r = T.tail(r, b.w[c], (uint32_t)left);
    }
  }
  return r;
}

// Variable length, length-sorted per-wave windows (the k_var6 scheme of
// kvh.hip): one lane per key in input order runs each wave as long as its
// longest key (zipf 8-256 B: ~25 % of the lane-steps do work).  Each wave
// counting-sorts windows of WIN consecutive keys by length
// (wave_sort_window) and takes them 64 at a time in length order; the CRCs
// go through the wave's LDS slice back to input order and leave as one
// contiguous run.  NW waves per workgroup: the 128 KiB of replicated tables
// leave room for NW * 3 KiB of window state.
template <int R>
__device__ __attribute__((noinline)) void crc_wide_window(const uint8_t* __restrict__ keys,
                                                          const uint64_t* __restrict__ offs, uint64_t i0, uint32_t k,
                                                          int nchunks, const uint32_t* seeds, uint32_t seed,
                                                          uint32_t* out, const uint32_t* lds) {
  const CrcLdsT<R> T(lds);
  const uint32_t lane = threadIdx.x & 63;
  for (int c = 0; c < nchunks; c++) {
    const uint32_t j = 64 * c + lane;
    if (j < k) {
      const uint64_t a = offs[i0 + j], e = offs[i0 + j + 1];
      out[i0 + j] = crc_key_pf(keys + a, e - a, seeds ? seeds[i0 + j] : seed, T);
    }
  }
}

// Q: windows taken in address order through wave tickets (tickets.hpp, knob 24)
template <int WIN, int NW, int SH = 0, int R = 32, int G = 0, int SUB = 1, bool Q = false>
__global__ void __launch_bounds__(NW * 64)
k_crc_var_sorted(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n,
                 const uint32_t* seeds, uint32_t seed, uint32_t* out,
                 unsigned long long* __restrict__ tk = nullptr) {  // seeds may alias out
  constexpr int M = WIN / 64;
  static_assert(WIN <= 256 * 4, "hist slice doubles as the CRC staging area");
  __shared__ uint32_t lds[R == 32 ? kWords : kWords / 2];
  __shared__ uint32_t hist_s[NW][(WIN > 256 ? WIN : 256) * SUB];
  __shared__ uint32_t roff_s[NW][WIN];
  __shared__ uint16_t rlen_s[NW][WIN];
  __shared__ uint16_t ridx_s[NW][WIN];
  __shared__ WaveTickets WT;
  fill_crc<R>(lds);
  __syncthreads();
  if constexpr (Q) wt_init(WT, tk);
  const CrcLdsT<R> T(lds);
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* hist = hist_s[wv];
  const uint64_t nwin = (n + WIN - 1) / WIN;
  const uint64_t kend = offs[n];  // the buffer holds every byte up to the last key's end
  for (uint64_t w = Q ? wt_next(WT, tk, NW) : (uint64_t)blockIdx.x * NW + wv; w < nwin;
       w = Q ? wt_next(WT, tk, NW) : w + (uint64_t)gridDim.x * NW) {
    const uint64_t i0 = w * WIN;
    const uint32_t k = (uint32_t)(n - i0 < (uint64_t)WIN ? n - i0 : (uint64_t)WIN);
    const WinOffs<WIN> W = win_load<WIN>(offs, i0, k);
    bool wide = false;
#pragma unroll
    for (int m = 0; m < M; m++) wide |= W.e[m] - W.ws >= (1ull << 32);
    if (__ballot(wide)) {
      // a window spanning 4 GiB or more: its records would hold u32 window
      // offsets, so it runs in input order with u64 offsets (wave-uniform;
      // out of line, off the hot path's register allocation)
      crc_wide_window<R>(keys, offs, i0, k, M, seeds, seed, out, lds);
      continue;
    }
    const uint64_t ws = wave_sort_from<WIN, SH, SUB>(W, k, hist, roff_s[wv], rlen_s[wv], ridx_s[wv]);
    // (running the lane's M keys as interleaved chains was slower: each
    // lane then steps as long as its longest key, chunk M-1's)
    uint32_t crc[M], ix[M];
    // G == 2: the first two groups of the lane's next key are in flight while
    // it steps through the current one (keys of 64 KiB and more re-read theirs)
    Blk pf0 = bzero(), pf1 = bzero();
    auto pre = [&](uint32_t pos, Blk& g0, Blk& g1) {
      g0 = bzero();
      g1 = bzero();
      if (pos < k) {
        const uint32_t ln = rlen_s[wv][pos];
        const uint64_t a = ws + roff_s[wv][pos];
        const AChunks A(keys + a, ln, a + ln + 16 <= kend);
        g0 = A.chunk(0);
        g1 = A.chunk(1);
      }
    };
    if constexpr (G == 2) pre(lane, pf0, pf1);
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t pos = 64 * c + lane;
      ix[c] = 0xffffffffu;
      Blk nf0, nf1;
      if constexpr (G == 2) {
        if (c + 1 < M) pre(pos + 64, nf0, nf1);
      }
      if (pos < k) {
        const uint32_t j = ridx_s[wv][pos];
        uint64_t len = rlen_s[wv][pos];
        if constexpr (G == 2) {
          const uint64_t a = ws + roff_s[wv][pos];
          if (len < 65535u) {
            const AChunks A(keys + a, len, a + len + 16 <= kend);
            crc[c] = crc_key_g2(A, (uint32_t)len, seeds ? seeds[i0 + j] : seed, T, pf0, pf1);
          } else {
            len = offs[i0 + j + 1] - offs[i0 + j];
            if (len < (1u << 31)) crc[c] = crc_key_g(keys + a, (uint32_t)len, a + len + 16 <= kend, seeds ? seeds[i0 + j] : seed, T);
            else crc[c] = crc_key_pf(keys + a, len, seeds ? seeds[i0 + j] : seed, T);
          }
          ix[c] = j;
          if (c + 1 < M) { pf0 = nf0; pf1 = nf1; }
          continue;
        }
        if (len == 65535u) len = offs[i0 + j + 1] - offs[i0 + j];
        if constexpr (G != 0) {
          if (len < (1u << 31)) {  // whole groups stay inside the buffer unless the key ends within 16 bytes of it
            const uint64_t a = ws + roff_s[wv][pos];
            crc[c] = crc_key_g(keys + a, (uint32_t)len, a + len + 16 <= kend, seeds ? seeds[i0 + j] : seed, T);
          } else {
            crc[c] = crc_key_pf(keys + ws + roff_s[wv][pos], len, seeds ? seeds[i0 + j] : seed, T);
          }
        } else {
          crc[c] = crc_key_pf(keys + ws + roff_s[wv][pos], len, seeds ? seeds[i0 + j] : seed, T);
        }
        ix[c] = j;
      }
      if constexpr (G == 2) {
        if (c + 1 < M) { pf0 = nf0; pf1 = nf1; }
      }
    }
    wave_lds_sync();  // the records are read; the hist slice becomes the staging area
#pragma unroll
    for (int c = 0; c < M; c++)
      if (ix[c] != 0xffffffffu) hist[ix[c]] = crc[c];
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < M; c++) {
      const uint32_t j = 64 * c + lane;
      if (j < k) __builtin_nontemporal_store(hist[j], out + i0 + j);
    }
    wave_lds_sync();  // staging read before the next window's histogram
  }
  if constexpr (Q) wt_done(tk);
}

#ifdef KVH_EXPERIMENTS  // lost its A/B (round 6): experiments build only
// kv_crc_c of one key whose bytes sit in an LDS stage at byte `off`: the
// bytes up to the next dword boundary as a short step, then one aligned
// ds_read_b32 and one slice-by-4 step per 4 bytes, then the tail.
template <int R>
__device__ __forceinline__ uint32_t crc_stage(const uint8_t* st, uint32_t off, uint32_t len, uint32_t r,
                                              const CrcLdsT<R>& T) {
  const uint32_t* w32 = (const uint32_t*)st;
  uint32_t p = off, left = len;
  const uint32_t h = p & 3u;
  if (h != 0 && left != 0) {
    const uint32_t nb = 4u - h < left ? 4u - h : left;  // 1..3
    r = T.tail(r, (w32[p >> 2] >> (8 * h)) & ((1u << (8 * nb)) - 1u), nb);
    p += nb;
    left -= nb;
  }
  for (; left >= 4; left -= 4, p += 4) r = T.word(r, w32[p >> 2]);
  if (left) r = T.tail(r, w32[p >> 2] & ((1u << (8 * left)) - 1u), left);
  return r;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
  return ((uint64_t)hi << 32) | lo;
}

// Variable length, windows STAGED IN LDS (round 6, knob 14 = 7; lost its A/B,
// experiments build only: DESIGN.md §3.7).  The sorted
// kernel above gathers each key from global memory in length order: a load
// instruction touches up to 64 lines of its ~12 KiB window, and lines shared
// by keys of two length classes are fetched again once the XCD's L2 dropped
// them (8.3 GB requested for 5.9 GB of unique bytes).  Here each wave cuts its
// keys into windows of at most 256 keys whose bytes fit SB bytes of LDS,
// reads the window's bytes once as coalesced 16-byte groups of the 16-byte
// aligned span (a group that holds one byte of the window lies in that byte's
// page, so nothing past the caller's buffer can fault), sorts the window by
// exact length, and steps each key's CRC from the stage.  Keys too long for a
// stage run one per lane from global memory (crc_key_pf), up to 64 at a time.
// A wave takes SEG consecutive keys per ticket; windows never cross a segment.
template <int NW, int SB, bool Q>
__global__ void __launch_bounds__(NW * 64)
k_crc_var_stg(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n,
              const uint32_t* seeds, uint32_t seed, uint32_t* out,
              unsigned long long* __restrict__ tk = nullptr) {  // seeds may alias out
  constexpr uint32_t SEG = 1024, WIN = 256, M = WIN / 64, NG = SB / 1024;
  static_assert(SB % 1024 == 0 && SB <= 65535, "stage size");
  struct Wave {
    uint8_t stage[SB];
    uint32_t hist[WIN];  // the counting sort's buckets, then the CRC staging area
    uint32_t roff[WIN];
    uint16_t rlen[WIN], ridx[WIN];
  };
  struct Smem {
    uint32_t tab[kWords / 2];  // 16 copies (64 KiB)
    Wave w[NW];
    WaveTickets W;
  };
  __shared__ __attribute__((aligned(16))) Smem sm;
  fill_crc<16>(sm.tab);
  __syncthreads();
  if constexpr (Q) wt_init(sm.W, tk);
  const CrcLdsT<16> T(sm.tab);
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Wave& V = sm.w[wv];
  const uint64_t kend = offs[n];
  const uint64_t nseg = (n + SEG - 1) / SEG;
  const uint64_t kb0 = (uint64_t)(uintptr_t)keys;
  for (uint64_t sg = Q ? wt_next(sm.W, tk, NW) : (uint64_t)blockIdx.x * NW + wv; sg < nseg;
       sg = Q ? wt_next(sm.W, tk, NW) : sg + (uint64_t)gridDim.x * NW) {
    uint64_t i = sg * SEG;
    const uint64_t iend = n - i < SEG ? n : i + SEG;
    while (i < iend) {  // wave-uniform
      const uint32_t cap = (uint32_t)(iend - i < WIN ? iend - i : WIN);
      const WinOffs<WIN> W = win_load<WIN>(offs, i, cap);
      const uint64_t base = (kb0 + W.ws) & ~15ull;  // the stage's first byte (absolute)
      uint32_t k = 0;
#pragma unroll
      for (uint32_t m = 0; m < M; m++) {
        const uint32_t j = lane + 64 * m;
        const bool fit = j < cap && ((kb0 + W.e[m] + 15) & ~15ull) - base <= (uint64_t)SB;
        k += (uint32_t)__popcll(__ballot(fit));  // a prefix: the ends never decrease
      }
      if (k == 0) {
        // key i alone overflows a stage: the run of such keys (up to 64), one per lane from global memory
        const bool big = lane < cap && ((kb0 + W.e[0] + 15) & ~15ull) - ((kb0 + W.a[0]) & ~15ull) > (uint64_t)SB;
        const uint64_t nb = __ballot(!big);
        const uint32_t kb = nb ? (uint32_t)__builtin_ctzll(nb) : (cap < 64 ? cap : 64u);
        if (lane < kb) {
          const uint64_t a = W.a[0];
          out[i + lane] = crc_key_pf(keys + a, W.e[0] - a, seeds ? seeds[i + lane] : seed, T);
        }
        i += kb;
        continue;
      }
      // the window's bytes, [base, end of key k-1 rounded up to 16), as coalesced 16-byte groups
      uint64_t ek = 0;
#pragma unroll
      for (uint32_t m = 0; m < M; m++) {
        const uint64_t v = readlane64(W.e[m], (k - 1) & 63);
        if (((k - 1) >> 6) == m) ek = v;
      }
      const uint32_t G = (uint32_t)((((kb0 + ek + 15) & ~15ull) - base) >> 4);
      v4u g[NG];
#pragma unroll
      for (uint32_t q = 0; q < NG; q++) {
        const uint32_t x = lane + 64 * q, xc = x < G ? x : G - 1;
        g[q] = __builtin_nontemporal_load((const v4u*)(uintptr_t)(base + 16ull * xc));
      }
      const uint32_t mis = (uint32_t)((kb0 + W.ws) - base);
      wave_sort_from<WIN>(W, k, V.hist, V.roff, V.rlen, V.ridx);
#pragma unroll
      for (uint32_t q = 0; q < NG; q++) {
        const uint32_t x = lane + 64 * q;
        if (x < G) *(v4u*)(V.stage + 16 * x) = g[q];
      }
      wave_lds_sync();
      uint32_t crc[M], ix[M];
#pragma unroll
      for (uint32_t c = 0; c < M; c++) {
        const uint32_t pos = 64 * c + lane;
        ix[c] = 0xffffffffu;
        if (64 * c < k && pos < k) {
          const uint32_t j = V.ridx[pos];
          crc[c] = crc_stage(V.stage, V.roff[pos] + mis, V.rlen[pos], seeds ? seeds[i + j] : seed, T);
          ix[c] = j;
        }
      }
      wave_lds_sync();  // the records are read; the hist slice becomes the staging area
#pragma unroll
      for (uint32_t c = 0; c < M; c++)
        if (ix[c] != 0xffffffffu) V.hist[ix[c]] = crc[c];
      wave_lds_sync();
#pragma unroll
      for (uint32_t c = 0; c < M; c++) {
        const uint32_t j = 64 * c + lane;
        if (j < k) __builtin_nontemporal_store(V.hist[j], out + i + j);
      }
      wave_lds_sync();  // stage, records and staging read before the next window's
      i += k;
    }
  }
  if constexpr (Q) wt_done(tk);
  (void)kend;
}
#endif  // KVH_EXPERIMENTS

}  // namespace
namespace kvh { namespace rt { std::atomic<int> g_tune_crc_var{6}; } }
namespace {

uint32_t grid_crc(uint64_t n, int cus) {
  const uint64_t need = (n + kBlock - 1) / kBlock;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(need, (uint64_t)cus));
}

// synchronous host drop-ins: stage keys + offsets + seeds, run k_crc_var
struct CrcStage {
  std::mutex mu;
  uint8_t* dev = nullptr;
  size_t cap = 0;
  int device = -1;
};
CrcStage g_cs;

size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

int crc_host(const void* const* ptrs, const size_t* lens, size_t n, uint32_t* seeds_io) {
  if (n == 0) return set_err(0);
  size_t kb = 0;
  for (size_t i = 0; i < n; i++) {
    if (lens[i] && !ptrs[i]) return set_err(KVH_EINVAL);
    kb += lens[i];
  }
  const size_t off_offs = al16(kb), off_seed = off_offs + al16(8 * (n + 1)), total = off_seed + al16(4 * n);
  std::vector<uint8_t> host(total);
  uint64_t* offs = (uint64_t*)(host.data() + off_offs);
  size_t o = 0;
  for (size_t i = 0; i < n; i++) {
    offs[i] = o;
    if (lens[i]) memcpy(host.data() + o, ptrs[i], lens[i]);
    o += lens[i];
  }
  offs[n] = o;
  memcpy(host.data() + off_seed, seeds_io, 4 * n);
  std::lock_guard<std::mutex> g(g_cs.mu);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  if (!g_cs.dev || g_cs.device != dev || g_cs.cap < total) {
    if (g_cs.dev) {
      int cur = dev;
      (void)hipSetDevice(g_cs.device);
      (void)hipFree(g_cs.dev);
      (void)hipSetDevice(cur);
      g_cs.dev = nullptr;
      g_cs.cap = 0;
    }
    e = hipMalloc(&g_cs.dev, std::max<size_t>(total, 1 << 20));
    if (e != hipSuccess) { g_cs.dev = nullptr; return hip_err(e); }
    g_cs.cap = std::max<size_t>(total, 1 << 20);
    g_cs.device = dev;
  }
  uint8_t* d = g_cs.dev;
  e = hipMemcpy(d, host.data(), total, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(e);
  uint32_t* dseed = (uint32_t*)(d + off_seed);
  hipLaunchKernelGGL(k_crc_var, dim3(1), dim3(kBlock), 0, 0, d, (const uint64_t*)(d + off_offs), (uint64_t)n,
                     dseed, 0u, dseed);
  int rc = launch_done();
  if (rc) return rc;
  e = hipMemcpy(seeds_io, dseed, 4 * n, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_err(e);
  return set_err(0);
}

}  // namespace

extern "C" {

int kvh_crc_c_fixed(const void* keys, uint32_t key_len, size_t n, const uint32_t* seeds, uint32_t seed,
                    uint32_t* out, void* stream) {
  if (n == 0) return set_err(0);
  if (!out || (key_len && !keys)) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t* k = (const uint8_t*)keys;
  // chunk order (knob 24): wave tickets (in address order) unless 1 = static
  unsigned long long* tk = nullptr;
  if (knob(g_tune_order) != 1)
    if ((rc = stream_tickets(st, &tk))) return rc;
  const bool q = tk != nullptr;  // no words for a captured launch: the static order
  switch (key_len) {
#define KVH_CRC_L(Lv, Uv)                                                                                   \
  case Lv:                                                                                                  \
    if (q)                                                                                                  \
      hipLaunchKernelGGL((k_crc_fixed_ct<Lv, Uv, true>), dim3(grid_crc((n + Uv - 1) / Uv, cus)), dim3(kBlock), 0, \
                         st, k, (uint64_t)n, seeds, seed, out, tk);                                          \
    else                                                                                                    \
      hipLaunchKernelGGL((k_crc_fixed_ct<Lv, Uv>), dim3(grid_crc((n + Uv - 1) / Uv, cus)), dim3(kBlock), 0, st, k, \
                         (uint64_t)n, seeds, seed, out, nullptr);                                            \
    return launch_done();
    KVH_CRC_L(4, 8) KVH_CRC_L(8, 8) KVH_CRC_L(12, 8) KVH_CRC_L(16, 8) KVH_CRC_L(24, 4) KVH_CRC_L(32, 4)
    KVH_CRC_L(48, 2) KVH_CRC_L(64, 2)
#undef KVH_CRC_L
    default:
      break;
  }
  hipLaunchKernelGGL((k_crc_fixed<2>), dim3(grid_crc((n + 1) / 2, cus)), dim3(kBlock), 0, st, k, key_len,
                     (uint64_t)n, seeds, seed, out);
  return launch_done();
}

int kvh_crc_c_var(const void* keys, const uint64_t* offsets, size_t n, const uint32_t* seeds, uint32_t seed,
                  uint32_t* out, void* stream) {
  if (n == 0) return set_err(0);
  if (!out || !offsets || !keys) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  const int v = g_tune_crc_var.load(std::memory_order_relaxed);
#ifdef KVH_EXPERIMENTS
  if (v == 7) {  // windows staged in LDS, segments in address order unless knob 24 = 1 (or captured)
    unsigned long long* tk = nullptr;
    if (knob(g_tune_order) != 1)
      if ((rc = stream_tickets((hipStream_t)stream, &tk))) return rc;
    if (tk)
      hipLaunchKernelGGL((k_crc_var_stg<8, 8192, true>), dim3(cus), dim3(512), 0, (hipStream_t)stream,
                         (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out, tk);
    else
      hipLaunchKernelGGL((k_crc_var_stg<8, 8192, false>), dim3(cus), dim3(512), 0, (hipStream_t)stream,
                         (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out, nullptr);
  } else
#endif
  if (v == 6) {  // windows in address order unless knob 24 = 1 (or a captured launch)
    unsigned long long* tk = nullptr;
    if (knob(g_tune_order) != 1)
      if ((rc = stream_tickets((hipStream_t)stream, &tk))) return rc;
    if (tk)
      hipLaunchKernelGGL((k_crc_var_sorted<256, 16, 0, 16, 2, 1, true>), dim3(cus), dim3(1024), 0,
                         (hipStream_t)stream, (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out, tk);
    else
      hipLaunchKernelGGL((k_crc_var_sorted<256, 16, 0, 16, 2>), dim3(cus), dim3(1024), 0, (hipStream_t)stream,
                         (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out, nullptr);
  }
#ifdef KVH_EXPERIMENTS  // the variants that lost their A/B (round 3): experiments build only
  else if (v == 1)
    hipLaunchKernelGGL((k_crc_var_sorted<256, 10>), dim3(cus), dim3(640), 0, (hipStream_t)stream,
                       (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out);
  else if (v == 3)  // tables with 16 copies (64 KiB): 16 waves per CU
    hipLaunchKernelGGL((k_crc_var_sorted<256, 16, 0, 16>), dim3(cus), dim3(1024), 0, (hipStream_t)stream,
                       (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out);
  else if (v == 4)  // as 3, keys read as dwordx4 groups (crc_key_g)
    hipLaunchKernelGGL((k_crc_var_sorted<256, 16, 0, 16, 1>), dim3(cus), dim3(1024), 0, (hipStream_t)stream,
                       (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out);
  else if (v == 5)  // as 4, two sub-counters per length bucket in the window sort
    hipLaunchKernelGGL((k_crc_var_sorted<256, 16, 0, 16, 1, 2>), dim3(cus), dim3(1024), 0, (hipStream_t)stream,
                       (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out);
  else if (v == 2)
    hipLaunchKernelGGL((k_crc_var_sorted<256, 8>), dim3(cus), dim3(512), 0, (hipStream_t)stream,
                       (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out);
#endif
  else
    hipLaunchKernelGGL(k_crc_var, dim3(grid_crc(n, cus)), dim3(kBlock), 0, (hipStream_t)stream,
                       (const uint8_t*)keys, offsets, (uint64_t)n, seeds, seed, out);
  return launch_done();
}

uint32_t kvh_crc_c(const void* p, size_t sz, uint32_t seed) {
  uint32_t s = seed;
  const void* ptrs[1] = {p};
  if (crc_host(ptrs, &sz, 1, &s) != 0) return 0;
  return s;
}

uint32_t kvh_hash_uint(uint32_t i) { return kvh_crc_c(&i, 4, 0); }
uint32_t kvh_hash_uint2(uint32_t r, uint32_t i) { return kvh_crc_c(&i, 4, r); }

int kvh_crc_c_2_diff(const void* p, size_t sz, uint32_t* seed, const void* p2, size_t sz2, uint32_t* seed2) {
  if (!seed || !seed2) return set_err(KVH_EINVAL);
  const void* ptrs[2] = {p, p2};
  const size_t lens[2] = {sz, sz2};
  uint32_t s[2] = {*seed, *seed2};
  const int rc = crc_host(ptrs, lens, 2, s);
  if (rc == 0) { *seed = s[0]; *seed2 = s[1]; }
  return rc;
}

int kvh_crc_c_4_diff(const void* p, size_t sz, uint32_t* seed, const void* p2, size_t sz2, uint32_t* seed2,
                     const void* p3, size_t sz3, uint32_t* seed3, const void* p4, size_t sz4, uint32_t* seed4) {
  if (!seed || !seed2 || !seed3 || !seed4) return set_err(KVH_EINVAL);
  const void* ptrs[4] = {p, p2, p3, p4};
  const size_t lens[4] = {sz, sz2, sz3, sz4};
  uint32_t s[4] = {*seed, *seed2, *seed3, *seed4};
  const int rc = crc_host(ptrs, lens, 4, s);
  if (rc == 0) { *seed = s[0]; *seed2 = s[1]; *seed3 = s[2]; *seed4 = s[3]; }
  return rc;
}

int kvh_crc_c_array(const void** p, size_t* psz, uint32_t* seed, size_t count) {
  if (count && (!p || !psz || !seed)) return set_err(KVH_EINVAL);
  return crc_host(p, psz, count, seed);
}

int kvh_crc_c_key_array(const void* p, size_t* psz, uint32_t* seed, size_t count) {
  if (count && (!psz || !seed)) return set_err(KVH_EINVAL);
  std::vector<const void*> ptrs(count, p);
  return crc_host(ptrs.data(), psz, count, seed);
}

}  // extern "C"
