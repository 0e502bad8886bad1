// tools/stream_forms.hip -- which streaming form reaches the highest HBM rate
// for the key-hash traffic shape on this box (measurement infrastructure for
// DESIGN.md §4.3; not part of the product).
//
// Every form moves the same bytes: n 16-byte items read and n written (the C1
// traffic, 32 B per key; default n = 100M = 3.2 GB).  After one common settle
// (the k_fixed-shaped copy launched for settle_ms) the forms
// run interleaved, `rounds` times `reps` launches each; per form the median
// rate over rounds is printed, with the engine clock each form ran at,
// measured inside the kernel: one lane of every 64th workgroup reads the
// shader clock (clock64) and the constant wall clock (wall_clock64) at its
// start and end and adds the deltas to two counters (vector atomics).
//
// Forms:
//   chunk<U>/g   wave-chunked (wave w owns runs of 64*U consecutive items, every
//                load/store instruction a contiguous 1 KiB), nt loads and
//                stores, grid = g workgroups of 1024 per CU -- k_fixed's and
//                tools/copy_peak's shape at U=4, g=1
//   f4           the guide's float4 copy: one item per thread, 256-thread
//                workgroups, plain loads/stores (MI355X_MICROARCH.md: 6.29 TB/s)
//   f4nt         the same with nt loads/stores
//   memcpy       hipMemcpyAsync device-to-device
//   chunk_pf     the chunk form with the next chunk's loads issued before
//                this chunk's stores
//   chunk_xi     the chunk form with chunks dealt round-robin over workgroups
//   f4u<U>       one-shot grid, U items per thread, nt
//   chunk_dyn    persistent chunk form taking chunks from a global counter
//                (all of them, or the last 12.5 % after a static share)
//   f4u_scr      f4u with the blocks in a scrambled order
//   chunk_q      persistent workgroups taking workgroup-iterations in address
//                order from one counter per XCD (q8) or one global one (q1)
//
// usage: stream_forms [n_items=100000000] [settle_ms=500] [rounds=5] [reps=20]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

struct Clk {
  unsigned long long dclk, dwall, samples;
};

__device__ inline void clk_begin(uint64_t& c0, uint64_t& w0) {
  c0 = clock64();
  w0 = wall_clock64();
}
__device__ inline void clk_end(Clk* ck, uint64_t c0, uint64_t w0) {
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  atomicAdd(&ck->dclk, (unsigned long long)(c1 - c0));
  atomicAdd(&ck->dwall, (unsigned long long)(w1 - w0));
  atomicAdd(&ck->samples, 1ull);
}

template <int U>
__global__ void __launch_bounds__(1024) chunk(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                              Clk* ck) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6, last = n - 1;
  for (uint64_t b = wave * 64 * U; b < n; b += nw * 64 * U) {
    v4u X[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      X[u] = __builtin_nontemporal_load(in + (j < last ? j : last));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      v4u v = X[u];
      v.x ^= 0x9e3779b9u;
      __builtin_nontemporal_store(v, out + (j < last ? j : last));
    }
  }
  if (probe) clk_end(ck, c0, w0);
}

// chunk form with the next chunk's loads issued before this chunk's stores
// (software-pipelined: the wait for chunk c + 1's data does not sit behind
// chunk c's stores)
template <int U>
__global__ void __launch_bounds__(1024) chunk_pf(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                                 Clk* ck) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6, last = n - 1, step = nw * 64 * U;
  uint64_t b = wave * 64 * U;
  v4u X[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t j = b + 64 * u + lane;
    X[u] = __builtin_nontemporal_load(in + (j < last ? j : last));
  }
  for (; b < n; b += step) {
    v4u Y[U];
    const uint64_t bn = b + step;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = bn + 64 * u + lane;
      Y[u] = __builtin_nontemporal_load(in + (j < last ? j : last));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      v4u v = X[u];
      v.x ^= 0x9e3779b9u;
      __builtin_nontemporal_store(v, out + (j < last ? j : last));
    }
#pragma unroll
    for (int u = 0; u < U; u++) X[u] = Y[u];
  }
  if (probe) clk_end(ck, c0, w0);
}

// chunk form with chunks dealt to workgroups round-robin (chunk k of a pass
// -> workgroup k % G, so consecutive 1 KiB-per-instruction runs go to
// consecutive workgroups, i.e. to different XCDs, as the one-item-per-thread
// grid does)
template <int U>
__global__ void __launch_bounds__(1024) chunk_xi(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                                 Clk* ck) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  const uint64_t G = gridDim.x, wib = threadIdx.x >> 6, lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  const uint64_t chunk0 = wib * G + blockIdx.x, nw = G * wpb, last = n - 1;
  for (uint64_t c = chunk0; c * 64 * U < n; c += nw) {
    const uint64_t b = c * 64 * U;
    v4u X[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      X[u] = __builtin_nontemporal_load(in + (j < last ? j : last));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      v4u v = X[u];
      v.x ^= 0x9e3779b9u;
      __builtin_nontemporal_store(v, out + (j < last ? j : last));
    }
  }
  if (probe) clk_end(ck, c0, w0);
}

// persistent chunk form with dynamic chunk assignment: after its static
// share (the first `stat` chunk rounds), a wave takes G chunks at a time from
// a global counter -- do faster XCDs/CUs absorb the tail, as a one-shot
// grid's dispatcher lets them?
template <int U, int G>
__global__ void __launch_bounds__(1024) chunk_dyn(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                                  Clk* ck, unsigned long long* ctr, uint64_t stat) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6, last = n - 1;
  const uint64_t nch = (n + 64 * U - 1) / (64 * U);
  auto body = [&](uint64_t c) {
    const uint64_t b = c * 64 * U;
    v4u X[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      X[u] = __builtin_nontemporal_load(in + (j < last ? j : last));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      v4u v = X[u];
      v.x ^= 0x9e3779b9u;
      __builtin_nontemporal_store(v, out + (j < last ? j : last));
    }
  };
  const uint64_t sc = stat * nw < nch ? stat * nw : nch;  // chunks dealt statically
  for (uint64_t c = wave; c < sc; c += nw) body(c);
  for (;;) {
    uint64_t g0 = 0;
    if (lane == 0) g0 = atomicAdd(ctr, (unsigned long long)G);
    g0 = __shfl(g0, 0, 64) + sc;
    if (g0 >= nch) break;
    for (uint64_t c = g0; c < g0 + G && c < nch; c++) body(c);
  }
  if (probe) clk_end(ck, c0, w0);
}

// persistent workgroups taking whole workgroup-iterations (one chunk per
// wave) IN ADDRESS ORDER from a counter, the next ticket fetched one
// iteration ahead: the chunks in flight stay one compact window, as in a
// one-shot grid.  NQ = 8: one counter and one contiguous eighth of the array
// per XCD (workgroup b on XCD b % 8); NQ = 1: one global counter.
template <int U, int NQ>
__global__ void __launch_bounds__(1024) chunk_q(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                                Clk* ck, unsigned long long* ctr) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  __shared__ unsigned long long tk[2];
  const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, wpb = blockDim.x >> 6;
  const uint64_t last = n - 1, nch = (n + 64 * U - 1) / (64 * U);
  const uint32_t q = NQ == 1 ? 0u : blockIdx.x % NQ;
  const uint64_t c_lo = nch * q / NQ, c_hi = nch * (q + 1) / NQ;
  if (tid == 0) tk[0] = atomicAdd(ctr + q, 1ull);
  __syncthreads();
  for (uint32_t it = 0;; it++) {
    const uint64_t t = tk[it & 1];
    if (tid == 0) tk[(it + 1) & 1] = atomicAdd(ctr + q, 1ull);
    const uint64_t c = c_lo + t * wpb + wv;
    if (c_lo + t * wpb >= c_hi) break;  // workgroup-uniform
    if (c < c_hi) {
      const uint64_t b = c * 64 * U;
      v4u X[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t j = b + 64 * u + lane;
        X[u] = __builtin_nontemporal_load(in + (j < last ? j : last));
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t j = b + 64 * u + lane;
        v4u v = X[u];
        v.x ^= 0x9e3779b9u;
        __builtin_nontemporal_store(v, out + (j < last ? j : last));
      }
    }
    __syncthreads();
  }
  if (probe) clk_end(ck, c0, w0);
}

// one-shot grid, U items per thread (non-persistent, 256-thread workgroups)
template <int U>
__global__ void __launch_bounds__(256) f4u(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n, Clk* ck) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  const uint64_t b = (uint64_t)blockIdx.x * 256 * U + (threadIdx.x >> 6) * 64 * U + (threadIdx.x & 63);
  v4u X[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t j = b + 64 * u;
    if (j < n) X[u] = __builtin_nontemporal_load(in + j);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t j = b + 64 * u;
    v4u v = X[u];
    v.x ^= 0x9e3779b9u;
    if (j < n) __builtin_nontemporal_store(v, out + j);
  }
  if (probe) clk_end(ck, c0, w0);
}

// f4u with the workgroup -> block mapping scrambled (a bijection): the same
// one-shot dispatch, but the blocks in flight no longer form one compact
// address window
template <int U>
__global__ void __launch_bounds__(256) f4u_scr(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                               Clk* ck) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  const uint64_t G = gridDim.x, blk = ((uint64_t)blockIdx.x * 2654435761ull) % G;  // odd multiplier, G odd
  const uint64_t b = blk * 256 * U + (threadIdx.x >> 6) * 64 * U + (threadIdx.x & 63);
  v4u X[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t j = b + 64 * u;
    if (j < n) X[u] = __builtin_nontemporal_load(in + j);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t j = b + 64 * u;
    v4u v = X[u];
    v.x ^= 0x9e3779b9u;
    if (j < n) __builtin_nontemporal_store(v, out + j);
  }
  if (probe) clk_end(ck, c0, w0);
}

template <bool NT>
__global__ void __launch_bounds__(256) f4copy(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                              Clk* ck) {
  const bool probe = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
  uint64_t c0 = 0, w0 = 0;
  if (probe) clk_begin(c0, w0);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    v4u v = NT ? __builtin_nontemporal_load(in + i) : in[i];
    v.x ^= 0x9e3779b9u;
    if (NT)
      __builtin_nontemporal_store(v, out + i);
    else
      out[i] = v;
  }
  if (probe) clk_end(ck, c0, w0);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Form {
  const char* name;
  int kind;  // 0 chunk, 1 f4, 2 f4nt, 3 memcpy, 4 chunk_pf, 5 chunk_xi, 6 f4u, 7 chunk_dyn (g = static rounds)
  int U, g;
};

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
  const double settle_ms = argc > 2 ? atof(argv[2]) : 500.0;
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  const int reps = argc > 4 ? atoi(argv[4]) : 20;
  int cus = 0, wall_khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  v4u *in = nullptr, *out = nullptr;
  Clk* ck = nullptr;
  CK(hipMalloc(&in, n * 16));
  CK(hipMalloc(&out, n * 16));
  CK(hipMalloc(&ck, sizeof(Clk)));
  unsigned long long* ctr = nullptr;
  CK(hipMalloc(&ctr, 64));
  CK(hipMemset(in, 1, n * 16));
  const std::vector<Form> forms = {
      {"chunk4_g1 (k_fixed/copy_peak shape)", 0, 4, 1}, {"chunk4_g2", 0, 4, 2}, {"chunk8_g1", 0, 8, 1},
      {"chunk2_g2", 0, 2, 2}, {"chunk4_g8", 0, 4, 8},   {"f4 (guide float4 copy)", 1, 0, 0},
      {"f4nt", 2, 0, 0},      {"memcpy_d2d", 3, 0, 0},  {"chunk4_pf_g1 (next chunk's loads before stores)", 4, 4, 1},
      {"chunk2_pf_g1", 4, 2, 1}, {"chunk4_xi_g1 (chunks round-robin over workgroups)", 5, 4, 1},
      {"f4u4nt (one-shot grid, 4 items per thread)", 6, 4, 0}, {"f4u2nt", 6, 2, 0},
      {"chunk4_dyn_all (every chunk from a counter, 4 per grab)", 7, 4, 0},
      {"chunk4_dyn_tail (87.5% static, then the counter)", 7, 4, 83},
      {"f4u4nt_scrambled (one-shot, blocks in a scrambled order)", 8, 4, 0},
      {"chunk4_q8 (in-order tickets, one counter per XCD)", 9, 4, 8},
      {"chunk4_q1 (in-order tickets, one global counter)", 9, 4, 1},
      {"chunk8_q8", 9, 8, 8}};
  auto launch = [&](const Form& f) {
    if (f.kind == 0) {
      const dim3 grid(cus * f.g), block(1024);
      if (f.U == 2) hipLaunchKernelGGL(chunk<2>, grid, block, 0, 0, in, out, n, ck);
      if (f.U == 4) hipLaunchKernelGGL(chunk<4>, grid, block, 0, 0, in, out, n, ck);
      if (f.U == 8) hipLaunchKernelGGL(chunk<8>, grid, block, 0, 0, in, out, n, ck);
    } else if (f.kind == 1 || f.kind == 2) {
      const dim3 grid((unsigned)((n + 255) / 256)), block(256);
      if (f.kind == 1) hipLaunchKernelGGL(f4copy<false>, grid, block, 0, 0, in, out, n, ck);
      else hipLaunchKernelGGL(f4copy<true>, grid, block, 0, 0, in, out, n, ck);
    } else if (f.kind == 4) {
      const dim3 grid(cus * f.g), block(1024);
      if (f.U == 2) hipLaunchKernelGGL(chunk_pf<2>, grid, block, 0, 0, in, out, n, ck);
      else hipLaunchKernelGGL(chunk_pf<4>, grid, block, 0, 0, in, out, n, ck);
    } else if (f.kind == 5) {
      hipLaunchKernelGGL(chunk_xi<4>, dim3(cus * f.g), dim3(1024), 0, 0, in, out, n, ck);
    } else if (f.kind == 9) {
      CK(hipMemsetAsync(ctr, 0, 64, 0));
      if (f.g == 8 && f.U == 4) hipLaunchKernelGGL((chunk_q<4, 8>), dim3(cus), dim3(1024), 0, 0, in, out, n, ck, ctr);
      else if (f.g == 8) hipLaunchKernelGGL((chunk_q<8, 8>), dim3(cus), dim3(1024), 0, 0, in, out, n, ck, ctr);
      else hipLaunchKernelGGL((chunk_q<4, 1>), dim3(cus), dim3(1024), 0, 0, in, out, n, ck, ctr);
    } else if (f.kind == 8) {
      uint32_t G = (uint32_t)((n + 256 * 4 - 1) / (256 * 4));
      G |= 1u;  // odd; gcd(G, 2654435761) = 1 at the default n (a bijection)
      hipLaunchKernelGGL(f4u_scr<4>, dim3(G), dim3(256), 0, 0, in, out, n, ck);
    } else if (f.kind == 7) {
      CK(hipMemsetAsync(ctr, 0, 8, 0));
      hipLaunchKernelGGL((chunk_dyn<4, 4>), dim3(cus), dim3(1024), 0, 0, in, out, n, ck, ctr, (uint64_t)f.g);
    } else if (f.kind == 6) {
      const dim3 grid((unsigned)((n + 256 * f.U - 1) / (256 * f.U))), block(256);
      if (f.U == 2) hipLaunchKernelGGL(f4u<2>, grid, block, 0, 0, in, out, n, ck);
      else hipLaunchKernelGGL(f4u<4>, grid, block, 0, 0, in, out, n, ck);
    } else {
      CK(hipMemcpyAsync(out, in, n * 16, hipMemcpyDeviceToDevice, 0));
    }
  };
  auto t0 = std::chrono::steady_clock::now();
  int settle = 0;
  for (;;) {
    launch(forms[0]);
    CK(hipDeviceSynchronize());
    settle++;
    if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() >= settle_ms) break;
  }
  std::vector<std::vector<double>> rate(forms.size()), ghz(forms.size());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < rounds; r++) {
    for (size_t f = 0; f < forms.size(); f++) {
      launch(forms[f]);  // one untimed launch at this form's load
      CK(hipMemset(ck, 0, sizeof(Clk)));
      CK(hipEventRecord(a, 0));
      for (int k = 0; k < reps; k++) launch(forms[f]);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      Clk h;
      CK(hipMemcpy(&h, ck, sizeof(Clk), hipMemcpyDeviceToHost));
      rate[f].push_back(32.0 * (double)n / (ms / reps * 1e-3) / 1e12);
      ghz[f].push_back(h.dwall ? (double)h.dclk / (double)h.dwall * wall_khz * 1e-6 : 0.0);
    }
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  printf("{\"items\": %llu, \"bytes_per_launch\": %llu, \"settle_launches\": %d, \"rounds\": %d, \"reps\": %d, "
         "\"cus\": %d, \"wall_clock_khz\": %d, \"forms\": [",
         (unsigned long long)n, (unsigned long long)(32 * n), settle, rounds, reps, cus, wall_khz);
  for (size_t f = 0; f < forms.size(); f++) {
    const auto mm = std::minmax_element(rate[f].begin(), rate[f].end());
    printf("%s{\"form\": \"%s\", \"TBps_median\": %.3f, \"TBps_min\": %.3f, \"TBps_max\": %.3f, "
           "\"clock_GHz_median\": %.3f}",
           f ? ", " : "", forms[f].name, med(rate[f]), *mm.first, *mm.second, med(ghz[f]));
  }
  printf("]}\n");
  CK(hipFree(in));
  CK(hipFree(out));
  CK(hipFree(ck));
  return 0;
}
