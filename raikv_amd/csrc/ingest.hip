// ingest.hip -- SURVEY.md §8 row f3: key ingest formats raikv produces,
// hashed on the device without host repacking.
//
//   k_tok_count / k_tok_scan / k_tok_emit
//       whitespace tokenizer of ctest.c:202-233: a token is a maximal run
//       of bytes other than ' ', '\n', '\t'; a token of i bytes is kept if
//       i < max_token (MAX_TOKEN_SIZE = 256, ctest.c:23) and becomes the key
//       "token\0" (kv_set_key_frag_string, key_ctx.cpp:1764-1772: keylen =
//       i + 1).  Three passes: per-chunk counts, one exclusive scan of the
//       chunk counts, then each chunk re-finds its tokens and writes
//       (offset, length) in text order.
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

__device__ __forceinline__ bool is_ws(uint32_t c) { return c == ' ' || c == '\n' || c == '\t'; }

// byte i of the text (0 past the end)
__device__ __forceinline__ uint32_t byte_at(const uint8_t* t, uint64_t n, uint64_t i) { return i < n ? t[i] : 0u; }

// Length of the token starting at s (no whitespace at s), or max_token if
// it is max_token bytes or longer (dropped).  Reads dword-aligned words.
__device__ uint32_t tok_len(const uint8_t* t, uint64_t n, uint64_t s, uint32_t max_token) {
  uint64_t e = s + 1;
  const uint64_t lim = std::min<uint64_t>(n, s + max_token);
  const uint64_t mis = (uintptr_t)t & 3;  // word-align on absolute addresses
  while (e < lim) {
    // text index of the absolutely aligned word holding e (may be -1..-3)
    const int64_t a = (int64_t)((e + mis) & ~(uint64_t)3) - (int64_t)mis;
    const bool whole = a >= 0 && (uint64_t)a + 4 <= n;
    const uint32_t w = whole ? *(const uint32_t*)(t + a)
                             : (byte_at(t, n, a) | byte_at(t, n, a + 1) << 8 | byte_at(t, n, a + 2) << 16 |
                                byte_at(t, n, a + 3) << 24);
    for (uint64_t k = (uint64_t)((int64_t)e - a); k < 4 && e < lim; k++, e++)
      if (is_ws((w >> (8 * k)) & 255u)) return (uint32_t)(e - s);
  }
  return (uint32_t)(e - s) < max_token ? (uint32_t)(e - s) : max_token;
}

// 16 bytes of this thread's segment [q, q + 16) and the byte before it:
// bit i of the returned mask = a kept-or-not token starts at q + i
__device__ __forceinline__ uint32_t seg_starts(const uint8_t* t, uint64_t n, uint64_t q, uint8_t (&b)[16]) {
  if (q + 16 <= n && ((uintptr_t)(t + q) & 15) == 0) {
    const uint4 v = *(const uint4*)(t + q);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; i++) b[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  } else {
#pragma unroll
    for (int i = 0; i < 16; i++) b[i] = (uint8_t)byte_at(t, n, q + i);
  }
  uint32_t prev_ws = q == 0 ? 1u : (uint32_t)is_ws(t[q - 1]);
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t w = (uint32_t)is_ws(b[i]) | (q + i >= n ? 1u : 0u);
    if (!w && prev_ws) m |= 1u << i;
    prev_ws = w;
  }
  return m;
}

// kept tokens starting in [q, q + 16)
__device__ __forceinline__ uint32_t seg_count(const uint8_t* t, uint64_t n, uint64_t q, uint32_t max_token) {
  if (q >= n) return 0;
  uint8_t b[16];
  uint32_t m = seg_starts(t, n, q, b), c = 0;
  while (m) {
    const int i = __builtin_ctz(m);
    m &= m - 1;
    c += tok_len(t, n, q + i, max_token) < max_token;
  }
  return c;
}

__global__ void __launch_bounds__(kTokBlock)
k_tok_count(const uint8_t* __restrict__ t, uint64_t n, uint32_t max_token, uint64_t* __restrict__ chunk_cnt) {
  __shared__ uint32_t red[kTokBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kTokChunk;
  uint32_t c = 0;
  for (uint64_t p = 0; p < kTokChunk; p += kTokPass) c += seg_count(t, n, base + p + threadIdx.x * kTokSeg, max_token);
  // block reduce
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kTokBlock / 64; w++) s += red[w];
    chunk_cnt[blockIdx.x] = s;
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

__global__ void __launch_bounds__(kTokBlock)
k_tok_emit(const uint8_t* __restrict__ t, uint64_t n, uint32_t max_token, const uint64_t* __restrict__ chunk_base,
           uint64_t* __restrict__ offs, uint32_t* __restrict__ lens, uint64_t cap) {
  __shared__ uint32_t wsum[kTokBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kTokChunk;
  uint64_t k0 = chunk_base[blockIdx.x];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint64_t p = 0; p < kTokChunk; p += kTokPass) {
    const uint64_t q = base + p + threadIdx.x * kTokSeg;
    uint8_t b[16];
    const uint32_t m0 = q < n ? seg_starts(t, n, q, b) : 0u;
    uint32_t c = 0;  // kept starts in this segment (counted, then re-walked to write)
    for (uint32_t m = m0; m; m &= m - 1) c += tok_len(t, n, q + __builtin_ctz(m), max_token) < max_token;
    // block exclusive scan of c
    uint32_t inc = c;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (int w = 0; w < kTokBlock / 64; w++) {
      before += w < (int)wv ? wsum[w] : 0u;
      tot += wsum[w];
    }
    uint64_t k = k0 + before + inc - c;
    for (uint32_t m = c ? m0 : 0u; m; m &= m - 1) {
      const uint64_t at = q + __builtin_ctz(m);
      const uint32_t L = tok_len(t, n, at, max_token);
      if (L < max_token) {
        if (k < cap) { offs[k] = at; lens[k] = L; }
        k++;
      }
    }
    k0 += tot;
    __syncthreads();  // wsum reuse
  }
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

uint64_t tok_chunks(size_t nbytes) { return (nbytes + kTokChunk - 1) / kTokChunk; }

}  // namespace

extern "C" {

size_t kvh_tokenize_scratch_bytes(size_t nbytes) { return 8 * (tok_chunks(nbytes) + 1); }

int kvh_tokenize(const void* text, size_t nbytes, uint32_t max_token, uint64_t* tok_offs, uint32_t* tok_lens,
                 size_t cap, uint64_t* count, void* scratch, size_t scratch_bytes, void* stream) {
  if (!count || max_token == 0) return set_err(KVH_EINVAL);
  hipStream_t st = (hipStream_t)stream;
  if (nbytes == 0) {
    hipError_t e = hipMemsetAsync(count, 0, 8, st);
    return e == hipSuccess ? set_err(0) : hip_err(e);
  }
  const uint64_t nc = tok_chunks(nbytes);
  if (!text || !scratch || scratch_bytes < kvh_tokenize_scratch_bytes(nbytes) || (cap && (!tok_offs || !tok_lens)))
    return set_err(KVH_EINVAL);
  uint64_t* cc = (uint64_t*)scratch;
  const uint8_t* t = (const uint8_t*)text;
  hipLaunchKernelGGL(k_tok_count, dim3((uint32_t)nc), dim3(kTokBlock), 0, st, t, (uint64_t)nbytes, max_token, cc);
  int rc = launch_done();
  if (rc) return rc;
  hipLaunchKernelGGL(k_tok_scan, dim3(1), dim3(kScanBlock), 0, st, cc, nc, count);
  rc = launch_done();
  if (rc) return rc;
  if (cap == 0) return set_err(0);
  hipLaunchKernelGGL(k_tok_emit, dim3((uint32_t)nc), dim3(kTokBlock), 0, st, t, (uint64_t)nbytes, max_token, cc,
                     tok_offs, tok_lens, (uint64_t)cap);
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
