// scatter2_probe: the write address streams of f2's two record passes,
// replayed alone.  n 24-byte records, tiles of
// 2048, 128 runs of 16 records per tile, one 8-byte word per lane stored:
//   mode 1 (pass-1 shape): run d of tile t -> region d (n/128 records each)
//          at record t*16
//   mode 3: mode 2 with the tile first read from the previous launch's output
//   mode 2 (pass-2 shape): tiles grouped 381 per first-level region; run d2
//          of the k-th tile of region d1 -> sub-region (d1, d2) (n/16384
//          records each) at record k*16
//   mode 4: the pass-2 shape with ragged runs (length uniform in 8..24
//          records, mean 16, as real buckets are), each run placed right after
//          the previous tile's run of the same sub-region, so a 128-byte line
//          at a run boundary is written by two workgroups
//   mode 5: mode 4 with every run's start padded to 16 records (384 B, three
//          whole lines): the same ragged lengths, no line shared by two tiles
// Prints ms per launch; run under rocprofv3 --pmc WRITE_SIZE for the bytes.
// usage: scatter2_probe <mode> [n_millions=100] [reps=10]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

constexpr uint32_t kTile = 2048, kRuns = 128, kRun = kTile / kRuns;

__global__ void __launch_bounds__(512) probe(uint64_t* __restrict__ out, uint64_t n, int mode) {
  const uint64_t ntiles = n / kTile, t = blockIdx.x;
  if (t >= ntiles) return;
  const uint64_t region1 = n / kRuns;                 // pass-1 region size (records)
  const uint64_t tiles_per_d1 = ntiles / kRuns;        // ~381 at 100M
  const uint64_t sub = region1 / kRuns;                // pass-2 sub-region size
  for (uint32_t w = threadIdx.x; w < 3 * kTile; w += 512) {
    const uint32_t p = w / 3, part = w - 3 * p, run = p / kRun, in = p % kRun;
    uint64_t rec;
    if (mode == 1) {
      rec = run * region1 + t * kRun + in;
    } else {
      const uint64_t d1 = t / tiles_per_d1 < kRuns ? t / tiles_per_d1 : kRuns - 1, k = t - d1 * tiles_per_d1;
      rec = d1 * region1 + run * sub + (k * kRun + in) % sub;
    }
    out[rec * 3 + part] = w;
  }
}

// mode 3: the pass-2 stream preceded, in the same kernel, by a coalesced read
// of the tile's 2048 records from `in` (written by the previous launch, as
// f2's pass 2 reads pass 1's output); each read word is folded into the store
__global__ void __launch_bounds__(512) probe_rd(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n) {
  __shared__ uint64_t st[3 * kTile];
  const uint64_t ntiles = n / kTile, t = blockIdx.x;
  if (t >= ntiles) return;
  for (uint32_t w = threadIdx.x; w < 3 * kTile; w += 512) st[w] = in[t * 3 * kTile + w];
  __syncthreads();
  const uint64_t region1 = n / kRuns, tiles_per_d1 = ntiles / kRuns, sub = region1 / kRuns;
  for (uint32_t w = threadIdx.x; w < 3 * kTile; w += 512) {
    const uint32_t p = w / 3, part = w - 3 * p, run = p / kRun, in_ = p % kRun;
    const uint64_t d1 = t / tiles_per_d1 < kRuns ? t / tiles_per_d1 : kRuns - 1, k = t - d1 * tiles_per_d1;
    const uint64_t rec = d1 * region1 + run * sub + (k * kRun + in_) % sub;
    out[rec * 3 + part] = st[(w + 3 * 37) % (3 * kTile)];
  }
}

// modes 4/5: run r of tile t has len[t*kRuns+r] records, written from record dst[t*kRuns+r]
__global__ void __launch_bounds__(512) probe_rag(const uint16_t* __restrict__ len, const uint64_t* __restrict__ dst,
                                                 uint64_t* __restrict__ out, uint64_t ntiles) {
  const uint64_t t = blockIdx.x;
  if (t >= ntiles) return;
  const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  for (uint32_t r = wv; r < kRuns; r += 8) {
    const uint32_t words = 3u * len[t * kRuns + r];
    const uint64_t base = dst[t * kRuns + r] * 3;
    for (uint32_t j = ln; j < words; j += 64) out[base + j] = j;
  }
}

static int run_ragged(int mode, uint64_t n, int reps) {
  const uint64_t ntiles = n / kTile, tiles_per_d1 = ntiles / kRuns;
  uint16_t* hl = (uint16_t*)malloc(ntiles * kRuns * 2);
  uint64_t* hd = (uint64_t*)malloc(ntiles * kRuns * 8);
  uint64_t* tot = (uint64_t*)calloc(kRuns * kRuns, 8);
  uint64_t st = 12345, written = 0;
  for (uint64_t i = 0; i < ntiles * kRuns; i++) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    hl[i] = (uint16_t)(8 + (st >> 33) % 17);
    written += hl[i];
  }
  for (int pass = 0; pass < 2; pass++) {  // pass 0: sub-region totals; pass 1: placement
    uint64_t* cur = (uint64_t*)calloc(kRuns * kRuns, 8);
    if (pass == 1) {
      uint64_t acc = 0;
      for (uint64_t s = 0; s < kRuns * kRuns; s++) { cur[s] = acc; acc += tot[s]; }
      tot[0] = acc;  // total placed records
    }
    for (uint64_t t = 0; t < ntiles; t++) {
      const uint64_t d1 = t / tiles_per_d1 < kRuns ? t / tiles_per_d1 : kRuns - 1;
      for (uint32_t r = 0; r < kRuns; r++) {
        const uint64_t l = hl[t * kRuns + r], pl = mode == 5 ? (l + 15) / 16 * 16 : l;
        if (pass == 0) tot[d1 * kRuns + r] += pl;
        else { hd[t * kRuns + r] = cur[d1 * kRuns + r]; cur[d1 * kRuns + r] += pl; }
      }
    }
    free(cur);
  }
  const uint64_t placed = tot[0];
  uint16_t* dl; uint64_t* dd; uint64_t* out;
  if (hipMalloc(&dl, ntiles * kRuns * 2) != hipSuccess || hipMalloc(&dd, ntiles * kRuns * 8) != hipSuccess ||
      hipMalloc(&out, placed * 24) != hipSuccess) return 1;
  (void)hipMemcpy(dl, hl, ntiles * kRuns * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dd, hd, ntiles * kRuns * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL(probe_rag, dim3((uint32_t)ntiles), dim3(512), 0, 0, dl, dd, out, ntiles);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(probe_rag, dim3((uint32_t)ntiles), dim3(512), 0, 0, dl, dd, out, ntiles);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("{\"mode\": %d, \"records\": %llu, \"placed\": %llu, \"alg_GB\": %.3f, \"ms\": %.4f}\n", mode,
         (unsigned long long)written, (unsigned long long)placed, written * 24e-9, ms / reps);
  return 0;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 1;
  const uint64_t n = (argc > 2 ? atoll(argv[2]) : 100) * 1000000ull;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  if (mode == 4 || mode == 5) return run_ragged(mode, n, reps);
  uint64_t* out;
  if (hipMalloc(&out, n * 24) != hipSuccess) return 1;
  if (mode == 3) {  // in = the previous launch's mode-1 output; out written in the pass-2 shape
    uint64_t* in;
    if (hipMalloc(&in, n * 24) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const uint32_t grid = (uint32_t)(n / kTile);
    float tot = 0;
    for (int r = 0; r < reps; r++) {
      hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, in, n, 1);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(probe_rd, dim3(grid), dim3(512), 0, 0, in, out, n);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      tot += ms;
    }
    printf("{\"mode\": 3, \"n\": %llu, \"ms\": %.4f}\n", (unsigned long long)n, tot / reps);
    return 0;
  }
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const uint32_t grid = (uint32_t)(n / kTile);
  hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, out, n, mode);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, out, n, mode);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  printf("{\"mode\": %d, \"n\": %llu, \"ms\": %.4f, \"GBps_written\": %.1f}\n", mode, (unsigned long long)n, ms / reps,
         n * 24.0 / (ms / reps * 1e6));
  hipFree(out);
  return 0;
}
