// ingest.hip -- SURVEY.md §8 row f3: key ingest formats raikv produces,
// hashed on the device without host repacking.
//
//   k_tok<false> / k_tok_scan / k_tok<true>
//       whitespace tokenizer of ctest.c:202-233: a token is a maximal run
//       of bytes other than ' ', '\n', '\t'; a token of i bytes is kept if
//       i < max_token (MAX_TOKEN_SIZE = 256, ctest.c:23) and becomes the key
//       "token\0" (kv_set_key_frag_string, key_ctx.cpp:1764-1772: keylen =
//       i + 1).  Three launches: per-chunk counts, one exclusive scan of the
//       chunk counts, then each chunk re-finds its tokens and writes
//       (offset, length) in text order.  Bit-parallel: 16-byte separator
//       masks per lane, token starts carried across lanes by a max-scan.
//   k_keysrc<SRC>
//       Meow128 of keys named by (offset, length) spans (SRC_SPANS; with
//       KVH_NULTERM the hashed key is the span plus one 0 byte that is not
//       in the buffer) or by offsets of packed kv_key_frag_t records
//       {u16 keylen, keylen bytes, pad to 2} (SRC_FRAGS; kv_make_key_frag,
//       key_ctx.cpp:1737-1745; the xh[].frag pointers of ctest.c:28 as byte
//       offsets).  One lane per key, per-length constants in LDS as
//       k_generic (kvh.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <type_traits>
#include "kvh_internal.hpp"
#include "tickets.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

KVH_CHK_DECL  // checked build: the first failed bounds check of this unit
// check sites (kvh_debug_checks' out[1]; the sort's are 1..8)
enum : unsigned { kChkTokSlot = 17, kChkTokChunk, kChkSpanQueue, kChkSpanIdx, kChkTokOut };

constexpr int kTokBlock = 256;
constexpr uint64_t kTokSeg = 16;                            // bytes per thread per pass
constexpr uint64_t kTokPass = kTokBlock * kTokSeg;          // 4 KiB per pass
constexpr uint64_t kTokChunk = 16 * kTokPass;               // 64 KiB per workgroup
constexpr int kScanBlock = 1024;
constexpr int64_t kNoStart = INT64_MIN / 2;

__device__ __forceinline__ bool is_ws(uint32_t c) { return (c == ' ') | (c == '\n') | (c == '\t'); }

// 4 bytes -> 4-bit mask of separator bytes, branch-free SWAR: for each
// separator c, z = w ^ c*0x01010101 has a zero byte exactly where w holds c,
// and ((z & 0x7f7f7f7f) + 0x7f7f7f7f) | z has that byte's top bit clear
// exactly then (no carry crosses a byte).  The top bits of the bytes that are
// a separator (bits 7, 15, 23, 31) are gathered into bits 0-3 by one
// multiply whose partial products never overlap.
__device__ __forceinline__ uint32_t ws_bits(uint32_t w) {
  const uint32_t z0 = w ^ 0x20202020u, z1 = w ^ 0x0a0a0a0au, z2 = w ^ 0x09090909u;
  const uint32_t n0 = ((z0 & 0x7f7f7f7fu) + 0x7f7f7f7fu) | z0;
  const uint32_t n1 = ((z1 & 0x7f7f7f7fu) + 0x7f7f7f7fu) | z1;
  const uint32_t n2 = ((z2 & 0x7f7f7f7fu) + 0x7f7f7f7fu) | z2;
  const uint32_t t = (~(n0 & n1 & n2) & 0x80808080u) >> 7;  // bits 0, 8, 16, 24
  return (t * 0x00204081u) >> 21 & 15u;
}

// Segments are 16-byte blocks at ABSOLUTE 16-byte alignment, so every load
// is one aligned dwordx4 (it never leaves the 16-byte block, hence never the
// page); bytes outside [0, n) of the text count as separators.  Segment g
// covers text indices [g*16 - lead, g*16 - lead + 16), lead = text & 15.
struct TokGeo {
  const uint8_t* base;  // text rounded down to 16 bytes
  int64_t lead, n;
  uint64_t nseg;
};

__device__ __forceinline__ uint32_t seg_ws(const TokGeo& G, uint64_t g) {
  if (g >= G.nseg) return 0xffffu;
  const v4u v = __builtin_nontemporal_load((const v4u*)(G.base + 16 * g));
  uint32_t m = ws_bits(v.x) | ws_bits(v.y) << 4 | ws_bits(v.z) << 8 | ws_bits(v.w) << 12;
  const int64_t p0 = (int64_t)(16 * g) - G.lead;  // text index of byte 0
  if (p0 < 0) m |= (1u << (uint32_t)(-p0)) - 1u;
  if (p0 + 16 > G.n) m |= 0xffffu & ~((1u << (uint32_t)(G.n - p0 > 0 ? G.n - p0 : 0)) - 1u);
  return m;
}

// separator flag of text index i (outside the text: separator)
__device__ __forceinline__ bool ws_at(const uint8_t* t, int64_t n, int64_t i) {
  return i < 0 || i >= n || is_ws(t[i]);
}

// Start of the token holding text index i (i not a separator), searched
// back at most max_token bytes; kNoStart-ish (i - max_token) if further.
__device__ int64_t token_start_back(const uint8_t* t, int64_t n, int64_t i, uint32_t max_token) {
  int64_t s = i;
  const int64_t lim = i - (int64_t)max_token;
  while (s > 0 && s > lim && !ws_at(t, n, s - 1)) s--;
  return s > lim ? s : lim;
}

// inclusive max-scan over the 64 lanes of a wave
__device__ __forceinline__ int64_t wave_max_scan(int64_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v = v > y ? v : y;
  }
  return v;
}

__device__ __forceinline__ int32_t wave_max_scan32(int32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t y = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v = v > y ? v : y;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += y;
  }
  return v;
}

// The same scans and neighbour moves on DPP (the wave tokenizer, k_tok2):
// row shifts, then row broadcasts 15 and 31 (GFX9 data-parallel primitives),
// instead of ds_bpermute round trips through the LDS crossbar.  Lanes with
// no source keep `fill`.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t v, uint32_t fill) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ uint32_t lane_prev(uint32_t v, uint32_t fill) { return dpp<0x138>(v, fill); }  // wave_shr:1
__device__ __forceinline__ uint32_t lane_next(uint32_t v, uint32_t fill) { return dpp<0x130>(v, fill); }  // wave_shl:1
__device__ __forceinline__ int32_t dpp_max_scan32(int32_t v) {  // inclusive, over the wave's 64 lanes
  constexpr uint32_t id = 0x80000000u;  // INT32_MIN
  auto mx = [](int32_t a, uint32_t b) { return a > (int32_t)b ? a : (int32_t)b; };
  v = mx(v, dpp<0x111>((uint32_t)v, id));  // row_shr:1
  v = mx(v, dpp<0x112>((uint32_t)v, id));  // row_shr:2
  v = mx(v, dpp<0x114>((uint32_t)v, id));  // row_shr:4
  v = mx(v, dpp<0x118>((uint32_t)v, id));  // row_shr:8
  v = mx(v, dpp<0x142, 0xa>((uint32_t)v, id));  // row_bcast:15 into rows 1, 3
  v = mx(v, dpp<0x143, 0xc>((uint32_t)v, id));  // row_bcast:31 into rows 2, 3
  return v;
}
__device__ __forceinline__ uint32_t dpp_sum_scan(uint32_t v) {  // inclusive
  v += dpp<0x111>(v, 0u);
  v += dpp<0x112>(v, 0u);
  v += dpp<0x114>(v, 0u);
  v += dpp<0x118>(v, 0u);
  v += dpp<0x142, 0xa>(v, 0u);
  v += dpp<0x143, 0xc>(v, 0u);
  return v;
}
__device__ __forceinline__ uint32_t lane_get(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

// One kernel for both passes.  Per 16-byte segment: separator mask W,
// token starts S = ~W & (W << 1 | ws before), token ends E = ~W & (W >> 1 |
// ws after << 15).  A token is attributed to its END; its start is the
// highest start bit at or below the end in the same segment, else the
// running (max-scanned) last start of earlier segments.  Length =
// end - start + 1, kept when < max_token (ctest.c: i < MAX_TOKEN_SIZE).
// EMIT = false: per-chunk kept counts; EMIT = true: (offset, length) at
// the chunk's scanned base, in text order.
template <bool EMIT>
__global__ void __launch_bounds__(kTokBlock)
k_tok(const uint8_t* __restrict__ t, TokGeo G, uint32_t max_token, uint64_t* __restrict__ chunk_cnt,
      uint64_t* __restrict__ offs, uint32_t* __restrict__ lens, uint64_t cap) {
  __shared__ int64_t wmax[kTokBlock / 64];
  __shared__ uint32_t wsum[kTokBlock / 64];
  __shared__ int64_t carry_s;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t g0 = (uint64_t)blockIdx.x * (kTokChunk / kTokSeg);
  if (threadIdx.x == 0) {
    // start of a token running into this chunk from the previous one
    const int64_t p = (int64_t)(16 * g0) - G.lead;  // text index of the chunk's first byte
    carry_s = (p > 0 && !ws_at(t, G.n, p - 1)) ? token_start_back(t, G.n, p - 1, max_token) : kNoStart;
  }
  __syncthreads();
  int64_t carry = carry_s;
  uint64_t k0 = EMIT ? chunk_cnt[blockIdx.x] : 0;
  uint32_t cnt = 0;
  for (uint64_t ps = 0; ps < kTokChunk / kTokSeg; ps += kTokBlock) {
    const uint64_t g = g0 + ps + threadIdx.x;
    const int64_t p0 = (int64_t)(16 * g) - G.lead;
    const uint32_t W = seg_ws(G, g);
    // neighbours' separator flags: lanes share W; wave edges read the byte
    const uint32_t Wp = __shfl_up(W, 1, 64), Wn = __shfl_down(W, 1, 64);
    const uint32_t before = lane ? (Wp >> 15) & 1u : (uint32_t)ws_at(t, G.n, p0 - 1);
    const uint32_t after = lane < 63 ? Wn & 1u : (uint32_t)ws_at(t, G.n, p0 + 16);
    const uint32_t S = ~W & ((W << 1) | before) & 0xffffu;
    const uint32_t E = ~W & ((W >> 1) | (after << 15)) & 0xffffu;
    // running last start: exclusive max-scan over segments in text order
    const int64_t mine = S ? p0 + 31 - __builtin_clz(S) : kNoStart;
    const int64_t inc = wave_max_scan(mine, lane);
    if (lane == 63) wmax[wv] = inc;
    __syncthreads();
    int64_t pre = carry;
    for (uint32_t w = 0; w < wv; w++) pre = pre > wmax[w] ? pre : wmax[w];
    int64_t ex = __shfl_up(inc, 1, 64);
    ex = lane ? (ex > pre ? ex : pre) : pre;
    int64_t nc = carry;
    for (uint32_t w = 0; w < kTokBlock / 64; w++) nc = nc > wmax[w] ? nc : wmax[w];
    // ends in this segment
    uint32_t c = 0;
    for (uint32_t e = E; e; e &= e - 1) {
      const uint32_t i = (uint32_t)__builtin_ctz(e);
      const uint32_t sm = S & ((2u << i) - 1u);
      const int64_t st = sm ? p0 + 31 - __builtin_clz(sm) : ex;
      c += (p0 + (int64_t)i - st + 1) < (int64_t)max_token;
    }
    if constexpr (EMIT) {
      const uint32_t ci = wave_sum_scan(c, lane);
      if (lane == 63) wsum[wv] = ci;
      __syncthreads();
      uint32_t before_w = 0, tot = 0;
      for (uint32_t w = 0; w < kTokBlock / 64; w++) {
        before_w += w < wv ? wsum[w] : 0u;
        tot += wsum[w];
      }
      uint64_t k = k0 + before_w + ci - c;
      for (uint32_t e = c ? E : 0u; e; e &= e - 1) {
        const uint32_t i = (uint32_t)__builtin_ctz(e);
        const uint32_t sm = S & ((2u << i) - 1u);
        const int64_t st = sm ? p0 + 31 - __builtin_clz(sm) : ex;
        const int64_t L = p0 + (int64_t)i - st + 1;
        if (L < (int64_t)max_token) {
          if (k < cap) { offs[k] = (uint64_t)st; lens[k] = (uint32_t)L; }
          k++;
        }
      }
      k0 += tot;
    } else {
      cnt += c;
    }
    carry = nc;
    __syncthreads();  // wmax / wsum reuse
  }
  if constexpr (!EMIT) {
    for (int d = 32; d >= 1; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
    if (lane == 0) wsum[wv] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t s = 0;
      for (int w = 0; w < kTokBlock / 64; w++) s += wsum[w];
      chunk_cnt[blockIdx.x] = s;
    }
  }
}

// Wave-chunked tokenizer (default; kvh_set_tuning(19, 0) selects k_tok).
// Each wave owns a 16 KiB chunk (16 passes of 64 segments) and needs no
// workgroup barrier: all 16 segment loads are issued up front; the start of
// a token running into the chunk comes from one 256-byte window per wave
// (ballot over separator bytes) instead of a byte-serial backward walk; the
// pass-to-pass carry (running last start, neighbour separator bits) stays in
// registers.  With max_token > 16 the count is popc(ends) minus the first
// end's token when that one is too long (every later end in a segment has
// its start in the segment, hence length <= 16).  EMIT stages a pass's
// (offset, length) records in LDS and writes them out coalesced.
constexpr uint64_t kTok2Passes = 16;
constexpr uint64_t kTok2Chunk = kTok2Passes * 64 * kTokSeg;  // 16 KiB per wave

__device__ __forceinline__ v4u seg_ld(const TokGeo& G, uint64_t g) {
  return __builtin_nontemporal_load((const v4u*)(G.base + 16 * (g < G.nseg ? g : 0)));
}
__device__ __forceinline__ uint32_t seg_ws2(const TokGeo& G, uint64_t g, const v4u v) {
  const bool in = g < G.nseg;
  uint32_t m = ws_bits(v.x) | ws_bits(v.y) << 4 | ws_bits(v.z) << 8 | ws_bits(v.w) << 12;
  const int64_t p0 = (int64_t)(16 * g) - G.lead;
  if (p0 < 0) m |= (1u << (uint32_t)(-p0)) - 1u;
  if (p0 + 16 > G.n) m |= 0xffffu & ~((1u << (uint32_t)(G.n - p0 > 0 ? G.n - p0 : 0)) - 1u);
  return in ? m : 0xffffu;
}

__device__ __forceinline__ int64_t wave_max64(int64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int64_t y = __shfl_xor(v, d, 64);
    v = v > y ? v : y;
  }
  return v;
}

template <bool EMIT>
__global__ void __launch_bounds__(256)
k_tok2(const uint8_t* __restrict__ t, TokGeo G, uint32_t max_token, uint64_t* __restrict__ chunk_cnt,
       uint64_t nchunks, uint64_t* __restrict__ offs, uint32_t* __restrict__ lens, uint64_t cap) {
  __shared__ uint64_t so[4][512];  // <= 8 token ends per 16-byte segment
  __shared__ uint32_t sl[4][512];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + wv;
  if (w >= nchunks) return;
  const uint64_t g0 = w * (kTok2Chunk / kTokSeg);
  // segment loads run kPf passes ahead of the pass being tokenized
  constexpr uint32_t kPf = 3;
  v4u raw[kPf];
#pragma unroll
  for (uint32_t d = 0; d < kPf; d++) raw[d] = seg_ld(G, g0 + (1 + d) * 64 + lane);
  uint32_t Wc = seg_ws2(G, g0 + lane, seg_ld(G, g0 + lane)), Wnx = 0, prevW = 0;
  const int64_t p = (int64_t)(16 * g0) - G.lead;  // text index of the chunk's first byte
  const uint32_t after_chunk = (uint32_t)ws_at(t, G.n, p + (int64_t)kTok2Chunk);
  // Token running in: the last separator before p, searched back in 256-byte
  // windows (4 bytes per lane, dword aligned since p + lead is); indices < 0
  // are separators, so the search ends at the text start.  A start at or
  // before lim = p-1-max_token only has to make the token too long.
  int64_t carry = kNoStart;
  uint32_t before_chunk = 1;
  if (p > 0) {
    const int64_t lim = p - 1 - (int64_t)max_token;
    int64_t hi = p, ls = INT64_MIN;
    for (;;) {
      const int64_t i0 = hi - 256 + 4 * (int64_t)lane;
      uint32_t bytes = 0;
      if (i0 + 3 >= 0) bytes = *(const uint32_t*)(t + i0);  // the aligned dword holding a text byte stays in its page
      int64_t mine = INT64_MIN;
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (i0 + k < 0 || is_ws((bytes >> (8 * k)) & 255u)) mine = i0 + k;
      if (hi == p) before_chunk = (uint32_t)__shfl(mine == p - 1 ? 1 : 0, 63, 64);
      ls = wave_max64(mine);
      if (ls != INT64_MIN || hi - 256 <= lim) break;
      hi -= 256;
    }
    if (!before_chunk) carry = ls + 1 > lim ? ls + 1 : lim;
  }
  uint32_t total = 0;
  uint64_t k0 = EMIT ? chunk_cnt[w] : 0;
#pragma unroll 1
  for (uint32_t ps = 0; ps < kTok2Passes; ps++) {
    const int64_t p0 = p + (int64_t)(16 * (ps * 64 + lane));
    if (ps + 1 < kTok2Passes) Wnx = seg_ws2(G, g0 + (ps + 1) * 64 + lane, raw[0]);
#pragma unroll
    for (uint32_t d = 0; d + 1 < kPf; d++) raw[d] = raw[d + 1];
    if (ps + 1 + kPf < kTok2Passes) raw[kPf - 1] = seg_ld(G, g0 + (ps + 1 + kPf) * 64 + lane);
    const uint32_t Wp = lane_prev(Wc, 0u), Wn = lane_next(Wc, 0u);
    const uint32_t prev63 = ps ? lane_get(prevW, 63) >> 15 & 1u : before_chunk;
    const uint32_t next0 = ps + 1 < kTok2Passes ? lane_get(Wnx, 0) & 1u : after_chunk;
    const uint32_t before = lane ? (Wp >> 15) & 1u : prev63;
    const uint32_t after = lane < 63 ? Wn & 1u : next0;
    const uint32_t S = ~Wc & ((Wc << 1) | before) & 0xffffu;
    const uint32_t E = ~Wc & ((Wc >> 1) | (after << 15)) & 0xffffu;
    // last start at or before each segment, as an offset into this pass
    // (-1: none in the pass so far, then the carry from earlier passes)
    const int64_t pp = p + (int64_t)(16 * 64 * ps);
    const int32_t mine = S ? (int32_t)(16 * lane + 31 - __builtin_clz(S)) : -1;
    const int32_t inc = dpp_max_scan32(mine);
    const int32_t exr = (int32_t)lane_prev((uint32_t)inc, 0xffffffffu);  // lane 0: -1
    const int64_t ex = exr >= 0 ? pp + exr : carry;
    {
      const int32_t last = (int32_t)lane_get((uint32_t)inc, 63);
      if (last >= 0) carry = pp + last;
    }
    uint32_t c;
    if (max_token > 16) {
      c = (uint32_t)__builtin_popcount(E);
      if (E) {
        const uint32_t i = (uint32_t)__builtin_ctz(E);
        const uint32_t sm = S & ((2u << i) - 1u);
        const int64_t st = sm ? p0 + 31 - __builtin_clz(sm) : ex;
        c -= (p0 + (int64_t)i - st + 1) >= (int64_t)max_token;
      }
    } else {
      c = 0;
      for (uint32_t e = E; e; e &= e - 1) {
        const uint32_t i = (uint32_t)__builtin_ctz(e);
        const uint32_t sm = S & ((2u << i) - 1u);
        const int64_t st = sm ? p0 + 31 - __builtin_clz(sm) : ex;
        c += (p0 + (int64_t)i - st + 1) < (int64_t)max_token;
      }
    }
    if constexpr (EMIT) {
      const uint32_t ci = dpp_sum_scan(c);
      const uint32_t tot = lane_get(ci, 63);
      uint32_t slot = ci - c;
      for (uint32_t e = c ? E : 0u; e; e &= e - 1) {
        const uint32_t i = (uint32_t)__builtin_ctz(e);
        const uint32_t sm = S & ((2u << i) - 1u);
        const int64_t st = sm ? p0 + 31 - __builtin_clz(sm) : ex;
        const int64_t L = p0 + (int64_t)i - st + 1;
        if (L < (int64_t)max_token) {
          KVH_CHK(slot < 512u, kChkTokSlot, slot, 512u);
          so[wv][slot] = (uint64_t)st;
          sl[wv][slot] = (uint32_t)L;
          slot++;
        }
      }
      wave_lds_sync();
      KVH_CHK(tot <= 512u, kChkTokSlot, tot, 512u);
      for (uint32_t j = lane; j < tot; j += 64) {
        const uint64_t k = k0 + j;
        if (k < cap) {
          offs[k] = so[wv][j];
          lens[k] = sl[wv][j];
        }
      }
      wave_lds_sync();
      k0 += tot;
    } else {
      total += c;
    }
    prevW = Wc;
    Wc = Wnx;
  }
  if constexpr (!EMIT) {
    for (int d = 32; d >= 1; d >>= 1) total += __shfl_xor(total, d, 64);
    KVH_CHK(w < nchunks, kChkTokChunk, w, nchunks);
    if (lane == 0) chunk_cnt[w] = total;
  }
}

// exclusive scan of nc chunk counts in place; total -> *total (one workgroup)
__global__ void __launch_bounds__(kScanBlock)
k_tok_scan(uint64_t* __restrict__ cnt, uint64_t nc, uint64_t* __restrict__ total) {
  __shared__ uint64_t part[kScanBlock];
  const uint64_t per = (nc + kScanBlock - 1) / kScanBlock;
  const uint64_t lo = std::min<uint64_t>(nc, threadIdx.x * per), hi = std::min<uint64_t>(nc, lo + per);
  uint64_t s = 0;
  for (uint64_t i = lo; i < hi; i++) s += cnt[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < kScanBlock; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint64_t v = threadIdx.x >= (uint32_t)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint64_t run = part[threadIdx.x] - s;
  for (uint64_t i = lo; i < hi; i++) {
    const uint64_t v = cnt[i];
    cnt[i] = run;
    run += v;
  }
  if (threadIdx.x == kScanBlock - 1) *total = part[kScanBlock - 1];
}

// Exclusive scan of the wave-chunked tokenizer's chunk counts (cnt -> pre,
// total -> *total) over many workgroups with no inter-workgroup hand-off:
// the counts are all in memory, so workgroup b sums every count before its
// block of kScan3 (coalesced 16-byte loads; at most a few hundred KB per
// workgroup for a GiB of text) and scans its own block.
constexpr uint32_t kScan3 = 2 * kScanBlock;
__global__ void __launch_bounds__(kScanBlock)
k_tok_scan3(const uint64_t* __restrict__ cnt, uint64_t nc, uint64_t* __restrict__ pre, uint64_t* __restrict__ total) {
  __shared__ uint64_t wpart[kScanBlock / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t lo = (uint64_t)blockIdx.x * kScan3;
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  uint64_t s = 0;
  for (uint64_t i = 2 * tid; i < lo; i += kScan3) {  // lo is a multiple of kScan3: i + 1 < lo
    const u64x2 v = *(const u64x2*)(cnt + i);
    s += v.x + v.y;
  }
  const uint64_t i0 = lo + 2 * tid;
  const uint64_t x0 = i0 < nc ? cnt[i0] : 0, x1 = i0 + 1 < nc ? cnt[i0 + 1] : 0;
  // block reduce of s and block scan of x0 + x1 together
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  uint64_t inc = x0 + x1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += y;
  }
  __shared__ uint64_t wsum[kScanBlock / 64];
  if (lane == 63) wpart[wv] = inc;
  if (lane == 0) wsum[wv] = s;
  __syncthreads();
  uint64_t base = 0, tot = 0;
  for (uint32_t k = 0; k < kScanBlock / 64; k++) {
    base += wsum[k] + (k < wv ? wpart[k] : 0);
    tot += wsum[k] + wpart[k];
  }
  const uint64_t ex = base + inc - (x0 + x1);
  if (i0 < nc) pre[i0] = ex;
  if (i0 + 1 < nc) pre[i0 + 1] = ex + x0;
  if (lo + kScan3 >= nc && tid == 0) *total = tot;
}

enum { SRC_SPANS = 0, SRC_FRAGS = 1 };

template <int SRC, int NT>
__global__ void __launch_bounds__(1024)
k_keysrc(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
         uint64_t n, uint64_t s1, uint64_t s2, uint64_t* __restrict__ out, uint32_t flags,
         const uint64_t* __restrict__ dcount = nullptr) {  // dcount: n = min(n, *dcount), read on the device
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ MeowConstL kfull[kLT];
  __shared__ Blk kf[kNF * 4];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + kNF); l += blockDim.x) {
    if (l < (uint32_t)kLT) {
      static_cast<MeowConst&>(kfull[l]) = make_const(s1, s2, l, T);
    } else {
      const Blk M = mixer(s1, s2, l);
#pragma unroll
      for (int s = 0; s < 4; s++) kf[(l - kLT) * 4 + s] = aesT(bxor(ramp(s), M), T);
    }
  }
  __syncthreads();
  if (dcount) {  // no barrier follows
    const uint64_t dn = *dcount;
    n = dn < n ? dn : n;
  }
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t nul = (flags & KVH_NULTERM) ? 1u : 0u;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint8_t* p;
    uint32_t D, H;
    if constexpr (SRC == SRC_SPANS) {
      p = buf + offs[i];
      D = lens[i];
      H = D + nul;
    } else {
      const uint8_t* rec = buf + offs[i];
      D = *(const uint16_t*)rec;
      H = D;
      p = rec + 2;
    }
    const LdsK<LdsTab<NT>, uint32_t, MeowConstL> K(kfull, kf, H, s1, s2, T);
    const MaskLd ld{p + D};
    store_h(out, i, meow_rt<LdsTab<NT>, LdsK<LdsTab<NT>, uint32_t, MeowConstL>, MaskLd>(p, H, K, T, ld), fix);
  }
}

// hash the queued spans q[0 .. cnt) (cnt <= 64), lane per entry, runtime length
// STASH: the span's (offset, length) was parked in its own output slot
// out[j] when it was queued (k_spans' short-hash store, by this wave); read
// it there (one slot) instead of offs[j] and lens[j] (two scattered lines).
// The pop waits for the wave's stores (vmcnt(0)) and reads through L2.
template <bool STASH>
__device__ __forceinline__ void span_at(const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
                                        const uint64_t* out, uint64_t j, uint64_t* off, uint32_t* len) {
  if constexpr (STASH) {  // agent-scope atomic loads: served by L2, never by a stale L1 line
    *off = __hip_atomic_load(out + 2 * j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *len = (uint32_t)__hip_atomic_load(out + 2 * j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *off = offs[j];
    *len = lens[j];
  }
}
template <int NT, bool STASH = false>
__device__ __forceinline__ void spans_long(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ offs,
                                           const uint32_t* __restrict__ lens, uint64_t* __restrict__ out,
                                           const uint32_t* q, uint32_t cnt, uint32_t lane, uint64_t qbase,
                                           uint64_t step, uint32_t CH, uint32_t nul, bool fix, const MeowConstL* kfull,
                                           uint64_t s1, uint64_t s2, const LdsTab<NT>& T, uint64_t nchk) {
  if (lane < cnt) {
    const uint32_t e = q[lane];
    const uint64_t j = qbase + (uint64_t)(e / CH) * step + (e % CH);
    KVH_CHK(j < nchk, kChkSpanIdx, j, nchk);
    uint64_t o;
    uint32_t D;
    span_at<STASH>(offs, lens, out, j, &o, &D);
    const uint8_t* p = buf + o;
    const uint32_t H = D + nul;
    const LdsK<LdsTab<NT>, uint32_t, MeowConstL> K(kfull, nullptr, H, s1, s2, T);
    const MaskLd ld{p + D};
    store_h(out, j, meow_rt<LdsTab<NT>, LdsK<LdsTab<NT>, uint32_t, MeowConstL>, MaskLd>(p, H, K, T, ld), fix);
  }
}

// Spans (kvh_meow128_spans): one lane per span in 64-span chunks per wave.
// Text tokens are short (f3: mean 3 bytes), and a span hashing 1..15 bytes
// touches only S3, so kv_hash_meow128 (key_hash.c:1413-1429) folds
//  to four table rounds with no branch:
//   S3 = AESDEC(F3 ^ k, k); S3 = AESDEC(S3, M)          Meow_Loop_Trail + Mix
//   S2 = AESDEC(TG2 ^ S3, M)                            Compress_Meow2
//   h  = AESDEC(TCS0a ^ S2, M)                          Compress_Meow
// But ~1 % of the tokens are longer, which in a lane-per-span kernel puts a
// longer path (8+ rounds) into most chunks.  So each wave hashes its short
// spans in place and appends the others to its own LDS queue (ballot +
// mbcnt compaction, no atomics), and runs the runtime-length path only when
// 64 of them are queued (and once for the remainder at the end): the long
// path then runs on full, mostly same-shape waves.  Loads run ahead of the
// hashing (a span's text load depends on its offset load).  LDS: all four
// tables (no rotates in the round), full constant records for L < 64 (the
// first-absorb folds of longer spans are made in-lane), u32 queue entries.
// A short span's bytes come from two aligned 16-byte blocks, the one holding
// its first byte and the one holding its last (the same block when the span
// does not cross), so no load leaves the span's pages.  The blocks stay raw
// in the load pipeline; when the chunk is hashed, two selects rotate them
// down by (p & 15) >> 2 words and one v_perm per word does the byte shift
// and the zero fill past the span, with selectors from an LDS table indexed
// by (length, p & 3).
struct ShortRaw {
  v4u A, B;
  uint32_t s, D;  // p & 15, span bytes (0: nothing loaded)
};

// a 16-byte aligned target for the lanes with nothing to load: every lane
// issues its two loads, so the load count is the same on every path and the
// compiler's in-order vmcnt waits never cover loads issued after the ones a
// use needs (a branch around the loads made them wait for the next chunk's
// offsets too)
__device__ v4u g_no_span[1];

// SB (experiments A/B): 0 B = the block of the last byte (== A unless the
// span crosses a 16-byte boundary); 1 B loaded only by the lanes whose span
// crosses (the others copy A); traffic ablations, hashes wrong: 2 the A
// block only, 3 no text loads.  (Always loading the next block reads past
// the buffer's last byte: not an option.)
template <int SB = 0>
__device__ __forceinline__ ShortRaw short_issue(const uint8_t* __restrict__ p, uint32_t D, bool load) {
  ShortRaw r;
  const uint8_t* q = load ? p : (const uint8_t*)g_no_span;
  const uint32_t a = (uint32_t)(uintptr_t)q & 15u;
  const uint32_t e = load ? D - 1 : 0u;
  r.s = a;
  r.D = load ? D : 0u;
  // pointer arithmetic (not integer masks) keeps these global loads
  if constexpr (SB == 3) {  // traffic ablation (hashes wrong): no text loads at all
    r.A = v4u{a, e, 0u, 0u};
    r.B = r.A;
    return r;
  }
  r.A = *(const v4u*)(q - a);
  if constexpr (SB == 1) {
    r.B = r.A;
    if (a + e >= 16u) r.B = *(const v4u*)(q - a + 16);  // the last byte's block: in bounds
  } else if constexpr (SB == 2) {  // traffic ablation (hashes wrong): the A block only
    r.B = r.A;
  } else {
    r.B = *(const v4u*)(q + e - ((a + e) & 15u));
  }
  return r;
}

__device__ __forceinline__ Blk short_key(const ShortRaw& r, const uint32_t* __restrict__ psel) {
  uint32_t w[8] = {r.A.x, r.A.y, r.A.z, r.A.w, r.B.x, r.B.y, r.B.z, r.B.w};
  if (r.s & 8) {
#pragma unroll
    for (int i = 0; i < 6; i++) w[i] = w[i + 2];
  }
  if (r.s & 4) {
#pragma unroll
    for (int i = 0; i < 5; i++) w[i] = w[i + 1];
  }
  const v4u sel = *(const v4u*)(psel + 4 * (4 * r.D + (r.s & 3u)));
  Blk k;
  k.w[0] = __builtin_amdgcn_perm(w[1], w[0], sel.x);
  k.w[1] = __builtin_amdgcn_perm(w[2], w[1], sel.y);
  k.w[2] = __builtin_amdgcn_perm(w[3], w[2], sel.z);
  k.w[3] = __builtin_amdgcn_perm(w[4], w[3], sel.w);
  return k;
}

// NH = spans per lane per iteration (NH 64-span halves of a 64*NH-span
// chunk): their four-round chains are independent, so the LDS latency of one
// overlaps the other (the kernel is latency-bound at the 4 waves per SIMD its
// 149 KiB of LDS allow).  The short path is computed for every lane of both
// halves (zero key for the others) so the chains share one branch.
// Medium spans, 16..31 hashed bytes (nb = 0, C = 16, t = H - 16): S0 absorbs
// bytes [0, 16), S3 the trail [16, H) when t != 0, then Mix / Compress2 /
// Compress fold to eight table rounds with no branch (the t = 0 case takes
// CS2b in place of the trail's Compress2).  Bytes from up to three aligned
// 16-byte blocks, each clamped to the block holding the span's last byte
// (never past its pages), funnelled like the short key.
struct MedRaw {
  v4u A, B, C;
  uint32_t s;
};
__device__ __forceinline__ MedRaw med_issue(const uint8_t* __restrict__ p, uint32_t L) {  // L >= 1
  MedRaw r;
  const uint32_t a = (uint32_t)(uintptr_t)p & 15u;
  r.s = a;
  const uint8_t* blk = p - a;                                         // block of the first byte
  const uint32_t lastoff = (a + L - 1) & ~15u;                        // last byte's block, from blk
  r.A = *(const v4u*)blk;
  r.B = *(const v4u*)(blk + (16u < lastoff ? 16u : lastoff));
  r.C = *(const v4u*)(blk + (32u < lastoff ? 32u : lastoff));
  return r;
}
__device__ __forceinline__ Blk funnel(const uint32_t (&w)[8], uint32_t s, uint32_t D, const uint32_t* __restrict__ psel) {
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = w[i];
  if (s & 8) {
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = x[i + 2];
  }
  if (s & 4) {
#pragma unroll
    for (int i = 0; i < 5; i++) x[i] = x[i + 1];
  }
  const v4u sel = *(const v4u*)(psel + 4 * (4 * D + (s & 3u)));
  Blk k;
  k.w[0] = __builtin_amdgcn_perm(x[1], x[0], sel.x);
  k.w[1] = __builtin_amdgcn_perm(x[2], x[1], sel.y);
  k.w[2] = __builtin_amdgcn_perm(x[3], x[2], sel.z);
  k.w[3] = __builtin_amdgcn_perm(x[4], x[3], sel.w);
  return k;
}
template <class Tab>
__device__ __forceinline__ Blk meow_medium(const MedRaw& r, uint32_t L, uint32_t H, const MeowConst& c,
                                           const uint32_t* __restrict__ psel, const Tab& T) {
  const uint32_t wAB[8] = {r.A.x, r.A.y, r.A.z, r.A.w, r.B.x, r.B.y, r.B.z, r.B.w};
  const uint32_t wBC[8] = {r.B.x, r.B.y, r.B.z, r.B.w, r.C.x, r.C.y, r.C.z, r.C.w};
  const Blk k0 = funnel(wAB, r.s, L < 16 ? L : 16u, psel);
  const Blk k3 = funnel(wBC, r.s, L > 16 ? L - 16 : 0u, psel);
  const Blk M = c.M;
  Blk S0 = aesdec(bxor(c.F[0], k0), k0, T);
  S0 = aesdec(S0, M, T);
  Blk S3 = aesdec(bxor(c.F[3], k3), k3, T);
  S3 = aesdec(S3, M, T);
  const Blk S2t = aesdec(bxor(c.TG2, S3), M, T);
  const bool t = H != 16;
  Blk S2b;
#pragma unroll
  for (int i = 0; i < 4; i++) S2b.w[i] = t ? S2t.w[i] : c.CS2b.w[i];
  const Blk S0b = aesdec(aesdec(S0, c.G[1], T), S2b, T);
  return aesdec(S0b, M, T);
}

// hash the queued medium spans q[0 .. cnt) (cnt <= 64), lane per entry
template <int NT, bool STASH = false>
__device__ __forceinline__ void spans_medium(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ offs,
                                             const uint32_t* __restrict__ lens, uint64_t* __restrict__ out,
                                             const uint32_t* q, uint32_t cnt, uint32_t lane, uint64_t qbase,
                                             uint64_t step, uint32_t CH, uint32_t nul, bool fix, const MeowConstL* kfull,
                                             const uint32_t* __restrict__ psel, const LdsTab<NT>& T, uint64_t nchk) {
  if (lane < cnt) {
    const uint32_t e = q[lane];
    const uint64_t j = qbase + (uint64_t)(e / CH) * step + (e % CH);
    KVH_CHK(j < nchk, kChkSpanIdx, j, nchk);
    uint64_t o;
    uint32_t L;
    span_at<STASH>(offs, lens, out, j, &o, &L);
    const uint32_t H = L + nul;
    const MedRaw r = med_issue(buf + o, L);
    store_h(out, j, meow_medium(r, L, H, kfull[H], psel, T), fix);
  }
}

// Q: chunks in address order through wave tickets (tickets.hpp; n < 2^32 - 1,
// the queues then hold span indices themselves)
template <int NT, int NH, int PD = 2, bool Q = false, int SB = 0, bool STASH = false>
__global__ void __launch_bounds__(1024)
k_spans(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
        uint64_t n, uint64_t s1, uint64_t s2, uint64_t* __restrict__ out, uint32_t flags,
        const uint64_t* __restrict__ dcount = nullptr,  // dcount: n = min(n, *dcount), read on the device
        unsigned long long* __restrict__ tk = nullptr) {
  static_assert(!Q || PD == 2, "the ticket form keeps two chunk bases");
  constexpr int NW = 1024 / 64;
  constexpr uint32_t CH = 64 * NH;  // spans per wave per iteration
  // medium spans stack up from 0, longer ones down from QCAP - 1; each holds
  // < 64 after a flush and an iteration adds <= CH to the two together
  constexpr uint32_t QCAP = 2 * 64 + CH;
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ MeowConstL kfull[kLT];
  __shared__ uint32_t queue[NW][QCAP];
  __shared__ uint32_t psel[17 * 4 * 4];  // [D 0..16][p & 3][word] v_perm selectors
  fill_tables<NT>(lds);
  for (uint32_t i = threadIdx.x; i < 17u * 4u * 4u; i += blockDim.x) {
    const uint32_t c = i & 3u, sh = (i >> 2) & 3u, D = i >> 4;
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; k++) v |= (4 * c + k < D ? sh + k : 0x0cu) << (8 * k);
    psel[i] = v;
  }
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)kLT; l += blockDim.x) static_cast<MeowConst&>(kfull[l]) = make_const(s1, s2, l, T);
  __shared__ WaveTickets WT;
  if constexpr (Q) wt_init(WT, tk);  // ends with a barrier
  else __syncthreads();
  if (dcount) {  // no barrier follows
    const uint64_t dn = *dcount;
    n = dn < n ? dn : n;
  }
  if (n == 0) {  // grid-uniform
    if constexpr (Q) wt_done(tk);
    return;
  }
  const bool fix = (flags & KVH_FIXUP) != 0;
  const uint32_t nul = (flags & KVH_NULTERM) ? 1u : 0u;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t* q = queue[threadIdx.x >> 6];
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  // spans per grid iteration (static order); Q: the queues hold span indices
  // (CH_Q = ~0: j = e / CH_Q * step + e % CH_Q = e)
  const uint64_t step = (uint64_t)gridDim.x * NW * CH;
  const uint32_t CHq = Q ? 0xffffffffu : CH;
  // The long-span queue is a stack: entry e = CH * (iteration) + 64 * half + lane
  // -> span wave*CH + (e / CH) * step + e % CH; full sets of 64 pop off the top.
  uint32_t qn = 0, ql = 0;  // wave-uniform: medium (16..31 hashed bytes) and long queue depths
  const uint64_t qbase = Q ? 0 : wave * CH;
  auto is_short = [nul](uint32_t D) { return D + nul - 1u < 15u; };
  // Pipeline, unrolled by PD so that no register is renamed while its load
  // is in flight: iteration c issues the offsets/lengths of chunk c+PD and the
  // text blocks of chunk c+1 (whose offsets arrived during iteration c-PD+1),
  // then hashes chunk c from the blocks issued during iteration c-1.  Offset
  // slots cycle mod PD, text slots mod 2.
  static_assert(PD % 2 == 0, "text slots alternate");
  uint64_t mo[PD][NH];
  uint32_t mD[PD][NH];
  ShortRaw tr[2][NH];
  uint64_t to[2][NH];  // STASH: the text offsets behind tr (dead code otherwise)
  // Q: cb[u] = base of the chunk whose offsets sit in slot u
  uint64_t cb[PD];
  if constexpr (Q) {
#pragma unroll
    for (int d = 0; d < PD; d++) cb[d] = wt_next(WT, tk, NW) * CH;
  } else {
#pragma unroll
    for (int d = 0; d < PD; d++) cb[d] = qbase + d * step;
  }
  const uint64_t b0 = cb[0];
#pragma unroll
  for (int h = 0; h < NH; h++) {
    const uint64_t j0 = std::min<uint64_t>(b0 + 64 * h + lane, n - 1);
    const uint64_t o0 = offs[j0];
    const uint32_t D0 = lens[j0];
#pragma unroll
    for (int d = 1; d < PD; d++) {
      const uint64_t jd = std::min<uint64_t>(cb[d] + 64 * h + lane, n - 1);
      mo[d][h] = __builtin_nontemporal_load(offs + jd);  // read once: streaming
      mD[d][h] = __builtin_nontemporal_load(lens + jd);
    }
    tr[0][h] = short_issue<SB>(buf + o0, D0, b0 + 64 * h + lane < n && D0 && is_short(D0));
    tr[0][h].D = D0;  // the length rides with the blocks (0-byte spans load nothing)
    to[0][h] = o0;
  }
  uint32_t it = 0;
  auto body = [&](uint64_t b, auto uc) {
    constexpr int u = decltype(uc)::value;  // offset slot, a compile-time constant
    constexpr int un = (u + 1) % PD, x = u & 1;  // next chunk's offset slot; this chunk's text slot
    const uint64_t bn = Q ? cb[un] : b + step;  // the next chunk
    cb[u] = Q ? wt_next(WT, tk, NW) * CH : b + PD * step;  // the chunk PD on
#pragma unroll
    for (int h = 0; h < NH; h++) {  // offsets of chunk cb[u] into slot u (chunk b's, consumed)
      const uint64_t jj = std::min<uint64_t>(cb[u] + 64 * h + lane, n - 1);
      mo[u][h] = __builtin_nontemporal_load(offs + jj);
      mD[u][h] = __builtin_nontemporal_load(lens + jj);
    }
#pragma unroll
    for (int h = 0; h < NH; h++) {  // text of the next chunk
      const uint32_t D1 = mD[un][h];
      tr[x ^ 1][h] = short_issue<SB>(buf + mo[un][h], D1, bn + 64 * h + lane < n && D1 && is_short(D1));
      tr[x ^ 1][h].D = D1;
      to[x ^ 1][h] = mo[un][h];
    }
    bool valid[NH], shrt[NH];
    Blk hh[NH];
    uint32_t any = 0;
#pragma unroll
    for (int h = 0; h < NH; h++) {
      valid[h] = b + 64 * h + lane < n;
      shrt[h] = is_short(tr[x][h].D);
      any |= (valid[h] && shrt[h]) ? 1u : 0u;
    }
    if (any) {
#pragma unroll
      for (int h = 0; h < NH; h++) {
        const uint32_t D0 = shrt[h] ? tr[x][h].D : 0u;  // long / invalid lanes hash a zero key, discarded
        ShortRaw r = tr[x][h];
        r.D = D0;
        const Blk k0 = short_key(r, psel);
        const MeowConst& c = kfull[D0 + nul];
        const Blk M = c.M;
        Blk S3 = aesdec(bxor(c.F[3], k0), k0, T);
        S3 = aesdec(S3, M, T);
        const Blk S2 = aesdec(bxor(c.TG2, S3), M, T);
        hh[h] = aesdec(bxor(c.TCS0a, S2), M, T);
      }
      if constexpr (!STASH) {
#pragma unroll
        for (int h = 0; h < NH; h++)
          if (valid[h] && shrt[h]) store_h<true>(out, b + 64 * h + lane, hh[h], fix);  // streaming
      }
    }
    if constexpr (STASH) {  // short lanes their hash, the queued ones their (offset, length): whole lines
#pragma unroll
      for (int h = 0; h < NH; h++)
        if (valid[h]) {
          v4u v;
          if (shrt[h]) {
            const Blk hx = fix ? fixup(hh[h]) : hh[h];
            v.x = hx.w[0]; v.y = hx.w[1]; v.z = hx.w[2]; v.w = hx.w[3];
          } else {
            const uint64_t o = to[x][h];
            v.x = (uint32_t)o; v.y = (uint32_t)(o >> 32); v.z = tr[x][h].D; v.w = 0u;
          }
          *(v4u*)(out + 2 * (b + 64 * h + lane)) = v;
        }
    }
#pragma unroll
    for (int h = 0; h < NH; h++) {
      const uint32_t H = tr[x][h].D + nul;
      const bool med = valid[h] && !shrt[h] && H - 16u < 16u, lng = valid[h] && !shrt[h] && !med;
      const uint64_t mm = __ballot(med), lm = __ballot(lng);
      const uint32_t e = Q ? (uint32_t)(b + 64 * h + lane) : CH * it + 64 * h + lane;
      if (mm) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
        if (med) q[qn + below] = e;
        qn += (uint32_t)__popcll(mm);
      }
      if (lm) {  // the long stack grows down from q[QCAP - 1]
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
        if (lng) q[QCAP - 1 - (ql + below)] = e;
        ql += (uint32_t)__popcll(lm);
      }
    }
    KVH_CHK(qn + ql <= QCAP, kChkSpanQueue, qn + ql, QCAP);
    if (qn >= 64 || ql >= 64) {
      wave_lds_sync();
      if constexpr (STASH) {  // this wave's stash stores before its reads of them
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the stash stores have reached L2
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
      while (qn >= 64) {
        spans_medium<NT, STASH>(buf, offs, lens, out, q + qn - 64, 64, lane, qbase, step, CHq, nul, fix, kfull, psel, T, n);
        qn -= 64;
      }
      while (ql >= 64) {  // its newest 64 entries: q[QCAP - ql .. QCAP - ql + 64)
        spans_long<NT, STASH>(buf, offs, lens, out, q + QCAP - ql, 64, lane, qbase, step, CHq, nul, fix, kfull, s1, s2, T, n);
        ql -= 64;
      }
      wave_lds_sync();
    }
    it++;
  };
  if constexpr (Q) {  // a wave's tickets only grow: past the end once, past it for good
    if (b0 < n) {
      for (;;) {
        body(cb[0], std::integral_constant<int, 0>{});
        if (cb[1] >= n) break;
        body(cb[1], std::integral_constant<int, 1>{});
        if (cb[0] >= n) break;
      }
    }
  } else {
    for (uint64_t b = b0; b < n; b += PD * step) {  // wave-uniform trip count
      body(b, std::integral_constant<int, 0>{});
      if (b + step >= n) break;
      body(b + step, std::integral_constant<int, 1>{});
      if constexpr (PD >= 4) {
        if (b + 2 * step >= n) break;
        body(b + 2 * step, std::integral_constant<int, 2 % PD>{});
        if (b + 3 * step >= n) break;
        body(b + 3 * step, std::integral_constant<int, 3 % PD>{});
      }
    }
  }
  if (qn || ql) {
    wave_lds_sync();
    if constexpr (STASH) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the stash stores have reached L2
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (qn) spans_medium<NT, STASH>(buf, offs, lens, out, q, qn, lane, qbase, step, CHq, nul, fix, kfull, psel, T, n);
    if (ql) spans_long<NT, STASH>(buf, offs, lens, out, q + QCAP - ql, ql, lane, qbase, step, CHq, nul, fix, kfull, s1, s2, T, n);
  }
  if constexpr (Q) wt_done(tk);
}


// ---------------------------------------------------------------------
// Packed kv_key_frag_t stream -> record offsets: records
// {u16 keylen, keylen bytes, pad to 2} back to back (kv_make_key_frag,
// key_ctx.cpp:1737-1745, as ctest packs them), so record starts are 2-byte
// positions and each one names the next: a linked list.  List ranking on the
// device: every position i gets next(i) = i + 1 + (keylen + 1) / 2 (in 2-byte
// units); ceil(log2 M) + 1 pointer-jumping launches mark every position
// reachable from 0 (after step k every record fewer than 2^(k+1) hops from
// the start is marked, which needs the previous step's marks complete: one
// launch per step); a count / scan / emit compacts the marks into offsets.
// A record running past the buffer ends the chain (jump sentinel M + 1).
constexpr uint32_t kFragChunk = 1024;

__global__ void __launch_bounds__(256)
k_frag_next(const uint8_t* __restrict__ b, uint64_t nbytes, uint32_t M, uint32_t* __restrict__ jump,
            uint8_t* __restrict__ mark) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += stride) {
    const uint64_t o = 2 * i;
    const uint32_t len = (uint32_t)b[o] | ((uint32_t)b[o + 1] << 8);  // o + 2 <= nbytes: i < M = nbytes / 2
    const uint64_t end = o + 2 + len;                                // the record's last byte + 1
    const bool valid = end <= nbytes;
    const uint64_t nx = (end + 1) >> 1;                              // past the pad byte, in positions
    jump[i] = valid ? (uint32_t)(nx < M ? nx : M) : M + 1;
    mark[i] = (i == 0 && valid) ? 1 : 0;
  }
}

__global__ void __launch_bounds__(256)
k_frag_jump(const uint32_t* __restrict__ jin, uint32_t* __restrict__ jout, uint8_t* __restrict__ mark, uint32_t M) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += stride) {
    const uint32_t j = jin[i];
    if (j < M) {
      const uint32_t jj = jin[j];
      if (jj != M + 1 && mark[i]) mark[j] = 1;  // j is a valid record reachable from 0
      jout[i] = jj == M + 1 ? M : jj;
    } else {
      jout[i] = j;
    }
  }
}

// marks per chunk of kFragChunk positions
__global__ void __launch_bounds__(kFragChunk)
k_frag_count(const uint8_t* __restrict__ mark, uint32_t M, uint64_t* __restrict__ cnt) {
  __shared__ uint32_t ws[kFragChunk / 64];
  const uint64_t i = (uint64_t)blockIdx.x * kFragChunk + threadIdx.x;
  const uint64_t bm = __ballot(i < M && mark[i]);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = (uint32_t)__popcll(bm);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kFragChunk / 64; w++) t += ws[w];
    cnt[blockIdx.x] = t;
  }
}

// marked positions -> byte offsets, in order, at the chunk's scanned base
__global__ void __launch_bounds__(kFragChunk)
k_frag_emit(const uint8_t* __restrict__ mark, uint32_t M, const uint64_t* __restrict__ pre,
            uint64_t* __restrict__ rec_offs, uint64_t cap) {
  __shared__ uint32_t ws[kFragChunk / 64];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t i = (uint64_t)blockIdx.x * kFragChunk + threadIdx.x;
  const bool m = i < M && mark[i];
  const uint64_t bm = __ballot(m);
  if (lane == 0) ws[wv] = (uint32_t)__popcll(bm);
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < wv; w++) before += ws[w];
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
  const uint64_t k = pre[blockIdx.x] + before + below;
  if (m && k < cap) rec_offs[k] = 2 * i;
}

}  // namespace
namespace kvh { namespace rt { std::atomic<int> g_tune_spans{2}; std::atomic<int> g_tune_tok{1}; } }
namespace {

TokGeo tok_geo(const void* text, size_t nbytes) {
  TokGeo G;
  G.lead = (int64_t)((uintptr_t)text & 15);
  G.base = (const uint8_t*)text - G.lead;
  G.n = (int64_t)nbytes;
  G.nseg = ((uint64_t)G.lead + nbytes + 15) / 16;
  return G;
}

uint64_t tok_chunks(const void* text, size_t nbytes) {
  return (tok_geo(text, nbytes).nseg * kTokSeg + kTokChunk - 1) / kTokChunk;
}

}  // namespace

namespace {
// k_spans<4, 2>, its chunks in address order through wave tickets unless
// knob 24 = 1 (or the spans overflow the queues' u32 span indices)
int launch_spans(const void* buf, const uint64_t* offs, const uint32_t* lens, uint64_t n, uint64_t seed1,
                 uint64_t seed2, uint64_t* out, uint32_t flags, const uint64_t* dcount, uint32_t grid,
                 hipStream_t st) {
  unsigned long long* tk = nullptr;
  if (knob(g_tune_order) != 1 && n < 0xffffffffull)
    if (int rc = stream_tickets(st, &tk)) return rc;
#ifdef KVH_EXPERIMENTS
  const int sk = g_tune_spans.load(std::memory_order_relaxed);
  if (tk && sk == 3)  // A/B: the second text block loaded only where the span crosses
    hipLaunchKernelGGL((k_spans<4, 2, 2, true, 1>), dim3(grid), dim3(1024), 0, st, (const uint8_t*)buf, offs, lens,
                       n, seed1, seed2, out, flags, dcount, tk);
  else if (tk && sk == 6)  // A/B: queued spans' (offset, length) parked in their output slots
    hipLaunchKernelGGL((k_spans<4, 2, 2, true, 0, true>), dim3(grid), dim3(1024), 0, st, (const uint8_t*)buf, offs,
                       lens, n, seed1, seed2, out, flags, dcount, tk);
  else if (tk && sk == 4)  // traffic ablation (hashes wrong): the A block only
    hipLaunchKernelGGL((k_spans<4, 2, 2, true, 2>), dim3(grid), dim3(1024), 0, st, (const uint8_t*)buf, offs, lens,
                       n, seed1, seed2, out, flags, dcount, tk);
  else if (tk && sk == 5)  // traffic ablation (hashes wrong): no text loads on the short path
    hipLaunchKernelGGL((k_spans<4, 2, 2, true, 3>), dim3(grid), dim3(1024), 0, st, (const uint8_t*)buf, offs, lens,
                       n, seed1, seed2, out, flags, dcount, tk);
  else
#endif
  if (tk) {  // (no words for a captured launch: the static order)
    hipLaunchKernelGGL((k_spans<4, 2, 2, true>), dim3(grid), dim3(1024), 0, st, (const uint8_t*)buf, offs, lens, n,
                       seed1, seed2, out, flags, dcount, tk);
  } else {
    hipLaunchKernelGGL((k_spans<4, 2>), dim3(grid), dim3(1024), 0, st, (const uint8_t*)buf, offs, lens, n, seed1,
                       seed2, out, flags, dcount, nullptr);
  }
  return launch_done();
}
}  // namespace

extern "C" {

size_t kvh_tokenize_scratch_bytes(size_t nbytes) {
  return 16 * ((nbytes + 31 + kTok2Chunk - 1) / kTok2Chunk + 1);  // counts + prefixes; either kernel, any alignment
}

int kvh_tokenize(const void* text, size_t nbytes, uint32_t max_token, uint64_t* tok_offs, uint32_t* tok_lens,
                 size_t cap, uint64_t* count, void* scratch, size_t scratch_bytes, void* stream) {
  if (!count || max_token == 0) return set_err(KVH_EINVAL);
  hipStream_t st = (hipStream_t)stream;
  if (nbytes == 0) {
    hipError_t e = hipMemsetAsync(count, 0, 8, st);
    return e == hipSuccess ? set_err(0) : hip_err(e);
  }
  if (!text || !scratch || scratch_bytes < kvh_tokenize_scratch_bytes(nbytes) || (cap && (!tok_offs || !tok_lens)))
    return set_err(KVH_EINVAL);
  const TokGeo G = tok_geo(text, nbytes);
  uint64_t* cc = (uint64_t*)scratch;
  const uint8_t* t = (const uint8_t*)text;
  if (g_tune_tok.load(std::memory_order_relaxed)) {
    const uint64_t nc = (G.nseg * kTokSeg + kTok2Chunk - 1) / kTok2Chunk;
    uint64_t* pre = cc + nc;
    const uint32_t grid = (uint32_t)((nc + 3) / 4);
    hipLaunchKernelGGL(k_tok2<false>, dim3(grid), dim3(256), 0, st, t, G, max_token, cc, nc, (uint64_t*)nullptr,
                       (uint32_t*)nullptr, (uint64_t)0);
    int rc = launch_done();
    if (rc) return rc;
    hipLaunchKernelGGL(k_tok_scan3, dim3((uint32_t)((nc + kScan3 - 1) / kScan3)), dim3(kScanBlock), 0, st, cc, nc,
                       pre, count);
    rc = launch_done();
    if (rc) return rc;
    if (cap == 0) return set_err(0);
    hipLaunchKernelGGL(k_tok2<true>, dim3(grid), dim3(256), 0, st, t, G, max_token, pre, nc, tok_offs, tok_lens,
                       (uint64_t)cap);
    return launch_done();
  }
  const uint64_t nc = tok_chunks(text, nbytes);
  hipLaunchKernelGGL(k_tok<false>, dim3((uint32_t)nc), dim3(kTokBlock), 0, st, t, G, max_token, cc,
                     (uint64_t*)nullptr, (uint32_t*)nullptr, (uint64_t)0);
  int rc = launch_done();
  if (rc) return rc;
  hipLaunchKernelGGL(k_tok_scan, dim3(1), dim3(kScanBlock), 0, st, cc, nc, count);
  rc = launch_done();
  if (rc) return rc;
  if (cap == 0) return set_err(0);
  hipLaunchKernelGGL(k_tok<true>, dim3((uint32_t)nc), dim3(kTokBlock), 0, st, t, G, max_token, cc, tok_offs,
                     tok_lens, (uint64_t)cap);
  return launch_done();
}

int kvh_tokenize_hash(const void* text, size_t nbytes, uint32_t max_token, uint64_t seed1, uint64_t seed2,
                      uint32_t flags, uint64_t* tok_offs, uint32_t* tok_lens, uint64_t* out, size_t cap,
                      uint64_t* count, void* scratch, size_t scratch_bytes, void* stream) {
  if (cap && !out) return set_err(KVH_EINVAL);
  int rc = kvh_tokenize(text, nbytes, max_token, tok_offs, tok_lens, cap, count, scratch, scratch_bytes, stream);
  if (rc || cap == 0 || nbytes == 0) return rc;
  int cus = 0;
  rc = device_cus(&cus);
  if (rc) return rc;
  // the span hash takes its count from the device: no host round trip
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((cap + 1023) / 1024, (uint64_t)cus));
  return launch_spans(text, tok_offs, tok_lens, cap, seed1, seed2, out, flags, (const uint64_t*)count, grid,
                      (hipStream_t)stream);
}

size_t kvh_frag_offsets_scratch_bytes(size_t nbytes) {
  const uint64_t M = nbytes / 2, nc = (M + kFragChunk - 1) / kFragChunk + 1;
  return 2 * 4 * (M + 64) + (M + 64) + 2 * 8 * nc + 256;
}

int kvh_frag_offsets(const void* buf, size_t nbytes, uint64_t* rec_offs, size_t cap, uint64_t* count, void* scratch,
                     size_t scratch_bytes, void* stream) {
  if (!count) return set_err(KVH_EINVAL);
  hipStream_t st = (hipStream_t)stream;
  const uint64_t M = nbytes / 2;
  if (M == 0) {
    hipError_t e = hipMemsetAsync(count, 0, 8, st);
    return e == hipSuccess ? set_err(0) : hip_err(e);
  }
  if (!buf || M >= 0xfffffff0ull || !scratch || scratch_bytes < kvh_frag_offsets_scratch_bytes(nbytes) ||
      (cap && !rec_offs))
    return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  const uint64_t nc = (M + kFragChunk - 1) / kFragChunk;
  uint8_t* sp = (uint8_t*)scratch;
  uint32_t* ja = (uint32_t*)sp;
  uint32_t* jb = ja + (M + 64);
  uint64_t* cnt = (uint64_t*)(((uintptr_t)(jb + (M + 64)) + 15) & ~(uintptr_t)15);
  uint64_t* pre = cnt + nc;
  uint8_t* mark = (uint8_t*)(pre + nc);
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((M + 255) / 256, (uint64_t)cus * 8));
  hipLaunchKernelGGL(k_frag_next, dim3(grid), dim3(256), 0, st, (const uint8_t*)buf, (uint64_t)nbytes, (uint32_t)M,
                     ja, mark);
  if ((rc = launch_done())) return rc;
  uint32_t steps = 1;
  while ((1ull << steps) <= M) steps++;
  for (uint32_t k = 0; k <= steps; k++) {
    hipLaunchKernelGGL(k_frag_jump, dim3(grid), dim3(256), 0, st, (const uint32_t*)ja, jb, mark, (uint32_t)M);
    if ((rc = launch_done())) return rc;
    std::swap(ja, jb);
  }
  hipLaunchKernelGGL(k_frag_count, dim3((uint32_t)nc), dim3(kFragChunk), 0, st, (const uint8_t*)mark, (uint32_t)M,
                     cnt);
  if ((rc = launch_done())) return rc;
  hipLaunchKernelGGL(k_tok_scan3, dim3((uint32_t)((nc + kScan3 - 1) / kScan3)), dim3(kScanBlock), 0, st,
                     (const uint64_t*)cnt, nc, pre, count);
  if ((rc = launch_done())) return rc;
  if (cap == 0) return set_err(0);
  hipLaunchKernelGGL(k_frag_emit, dim3((uint32_t)nc), dim3(kFragChunk), 0, st, (const uint8_t*)mark, (uint32_t)M,
                     (const uint64_t*)pre, rec_offs, (uint64_t)cap);
  return launch_done();
}

int kvh_frags_hash(const void* buf, size_t nbytes, uint64_t seed1, uint64_t seed2, uint32_t flags,
                   uint64_t* rec_offs, uint64_t* out, size_t cap, uint64_t* count, void* scratch,
                   size_t scratch_bytes, void* stream) {
  if (cap && !out) return set_err(KVH_EINVAL);
  int rc = kvh_frag_offsets(buf, nbytes, rec_offs, cap, count, scratch, scratch_bytes, stream);
  if (rc || cap == 0 || nbytes < 2) return rc;
  int cus = 0;
  if ((rc = device_cus(&cus))) return rc;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((cap + 1023) / 1024, (uint64_t)cus));
  hipLaunchKernelGGL((k_keysrc<SRC_FRAGS, 4>), dim3(grid), dim3(1024), 0, (hipStream_t)stream, (const uint8_t*)buf,
                     rec_offs, (const uint32_t*)nullptr, (uint64_t)cap, seed1, seed2, out, flags & ~KVH_NULTERM,
                     (const uint64_t*)count);
  return launch_done();
}

int kvh_meow128_spans(const void* buf, const uint64_t* offs, const uint32_t* lens, size_t n, uint64_t seed1,
                      uint64_t seed2, uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!buf || !offs || !lens || !out) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 1023) / 1024, (uint64_t)cus));
  const int sk = g_tune_spans.load(std::memory_order_relaxed);
  if (sk >= 2)
    return launch_spans(buf, offs, lens, n, seed1, seed2, out, flags, nullptr, grid, (hipStream_t)stream);
  else if (sk == 1)
    hipLaunchKernelGGL((k_spans<4, 1>), dim3(grid), dim3(1024), 0, (hipStream_t)stream, (const uint8_t*)buf, offs,
                       lens, (uint64_t)n, seed1, seed2, out, flags);
  else
    hipLaunchKernelGGL((k_keysrc<SRC_SPANS, 4>), dim3(grid), dim3(1024), 0, (hipStream_t)stream,
                       (const uint8_t*)buf, offs, lens, (uint64_t)n, seed1, seed2, out, flags);
  return launch_done();
}

int kvh_meow128_frags(const void* buf, const uint64_t* rec_offs, size_t n, uint64_t seed1, uint64_t seed2,
                      uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!buf || !rec_offs || !out) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 1023) / 1024, (uint64_t)cus));
  hipLaunchKernelGGL((k_keysrc<SRC_FRAGS, 4>), dim3(grid), dim3(1024), 0, (hipStream_t)stream,
                     (const uint8_t*)buf, rec_offs, (const uint32_t*)nullptr, (uint64_t)n, seed1, seed2, out,
                     flags & ~KVH_NULTERM);
  return launch_done();
}

}  // extern "C"

namespace kvh {
namespace rt {
int chk_take_ingest(unsigned long long out[4]) {
#if KVH_CHECKED_ON
  if (hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chk), 32)) return hip_err(e);
  const unsigned long long z[4] = {0, 0, 0, 0};
  if (hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_chk), z, 32)) return hip_err(e);
#else
  for (int i = 0; i < 4; i++) out[i] = 0;
#endif
  return 0;
}
}  // namespace rt
}  // namespace kvh
