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
#include "kvh_internal.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

constexpr int kTokBlock = 256;
constexpr uint64_t kTokSeg = 16;                            // bytes per thread per pass
constexpr uint64_t kTokPass = kTokBlock * kTokSeg;          // 4 KiB per pass
constexpr uint64_t kTokChunk = 16 * kTokPass;               // 64 KiB per workgroup
constexpr int kScanBlock = 1024;
constexpr int64_t kNoStart = INT64_MIN / 2;

__device__ __forceinline__ bool is_ws(uint32_t c) { return c == ' ' || c == '\n' || c == '\t'; }

// 4 bytes -> 4-bit mask of separator bytes (SWAR: a byte equal to c has
// (x ^ c*0x01010101) == 0 in that lane)
__device__ __forceinline__ uint32_t ws_bits(uint32_t w) {
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) m |= (uint32_t)is_ws((w >> (8 * k)) & 255u) << k;
  return m;
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

__device__ __forceinline__ uint32_t wave_sum_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += y;
  }
  return v;
}

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

enum { SRC_SPANS = 0, SRC_FRAGS = 1 };

template <int SRC, int NT>
__global__ void __launch_bounds__(1024)
k_keysrc(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
         uint64_t n, uint64_t s1, uint64_t s2, uint64_t* __restrict__ out, uint32_t flags) {
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  __shared__ MeowConst kfull[kLT];
  __shared__ Blk kf[kNF * 4];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  for (uint32_t l = threadIdx.x; l < (uint32_t)(kLT + kNF); l += blockDim.x) {
    if (l < (uint32_t)kLT) {
      kfull[l] = make_const(s1, s2, l, T);
    } else {
      const Blk M = mixer(s1, s2, l);
#pragma unroll
      for (int s = 0; s < 4; s++) kf[(l - kLT) * 4 + s] = aesT(bxor(ramp(s), M), T);
    }
  }
  __syncthreads();
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
    const LdsK<LdsTab<NT>> K(kfull, kf, H, s1, s2, T);
    const MaskLd ld{p + D};
    store_h(out, i, meow_rt<LdsTab<NT>, LdsK<LdsTab<NT>>, MaskLd>(p, H, K, T, ld), fix);
  }
}

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

extern "C" {

size_t kvh_tokenize_scratch_bytes(size_t nbytes) {
  return 8 * ((nbytes + 31 + kTokChunk - 1) / kTokChunk + 1);  // any text alignment
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
  const uint64_t nc = tok_chunks(text, nbytes);
  uint64_t* cc = (uint64_t*)scratch;
  const uint8_t* t = (const uint8_t*)text;
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

int kvh_meow128_spans(const void* buf, const uint64_t* offs, const uint32_t* lens, size_t n, uint64_t seed1,
                      uint64_t seed2, uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!buf || !offs || !lens || !out) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 1023) / 1024, (uint64_t)cus));
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
