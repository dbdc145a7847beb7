// mb_bin.hip -- microbenchmark: what bounds the bin (bucketize + scatter) pass?
// Variants over N samples, S series, tiles of 32 series:
//   read      : read series+values only (8 B/sample), fold into a checksum
//   search    : + LDS binary search over the limits
//   cursor    : + LDS cursor atomic (ds_add_rtn) per sample, no store
//   scatter   : + 4-B store at the cursor position (= production k_bin)
//   seqstore  : search + sequential (coalesced) store, no cursor
//   sorted    : search + LDS counting sort of 16K-sample sub-chunks by tile, run writes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int NL = 1797;
constexpr int LIM_PAD = 2048;
constexpr int WG = 1024;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void gen(uint32_t* series, float* values, size_t n, uint32_t S) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t r = mix64((i + 1) * 0x9E3779B97F4A7C15ull);
    series[i] = (uint32_t)((r >> 32) % S);
    float u = ((r & 0xFFFFFFull) + 1) * (1.0f / 16777216.0f);
    values[i] = expf(4.0f + 1.2f * logf(u) * -0.5f);
  }
}

__device__ __forceinline__ uint32_t search(float f, const int32_t* lim) {
  const int32_t key = (int32_t)(uint32_t)f;
  int idx = 0;
#pragma unroll
  for (int step = 1024; step > 0; step >>= 1)
    if (lim[idx + step - 1] <= key) idx += step;
  return (uint32_t)(idx < NL ? idx : NL);
}

template <int V>
__global__ __launch_bounds__(WG) void kbin(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                           size_t n, size_t per, uint32_t F, const uint32_t* __restrict__ cur0,
                                           const int32_t* __restrict__ limg, uint32_t* __restrict__ out,
                                           uint32_t* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  int32_t* lim = (int32_t*)smem;
  uint32_t* cur = smem + LIM_PAD;
  for (int i = threadIdx.x; i < LIM_PAD; i += WG) lim[i] = limg[i];
  for (uint32_t t = threadIdx.x; t < F; t += WG) cur[t] = cur0 ? cur0[(size_t)blockIdx.x * F + t] : 0;
  __syncthreads();
  const size_t lo = blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  uint32_t acc = 0;
  const uint4* ps = (const uint4*)(series + lo);
  const float4* pv = (const float4*)(values + lo);
  const size_t nv = (hi - lo) / 4;
  for (size_t i = threadIdx.x; i < nv; i += WG) {
    uint4 s = ps[i];
    float4 f = pv[i];
    uint32_t sv[4] = {s.x, s.y, s.z, s.w};
    float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (V == 0) {
        acc += sv[k] ^ __float_as_uint(fv[k]);
      } else {
        uint32_t b = search(fv[k], lim);
        uint32_t rec = ((sv[k] & 31) << 27) | (b << 16);
        if (V == 1) acc += rec;
        if (V == 2 || V == 3) {
          uint32_t pos = atomicAdd(&cur[sv[k] >> 5], 1u);
          if (V == 2) acc += pos ^ rec;
          if (V == 3) out[pos] = rec;
        }
        if (V == 4) out[lo + 4 * i + k] = rec;
      }
    }
  }
  if (acc == 0x12345678) sink[0] = acc;
}

// V5: sorted sub-chunks.  Each WG processes its slab in sub-chunks of CH samples:
// compute rec/tile into LDS, counting sort by tile within the sub-chunk, then
// write each tile's run to its global cursor.
template <int CH>
__global__ __launch_bounds__(WG) void kbin_sorted(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                                  size_t n, size_t per, uint32_t F, const uint32_t* __restrict__ cur0,
                                                  const int32_t* __restrict__ limg, uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  int32_t* lim = (int32_t*)smem;
  uint32_t* cur = smem + LIM_PAD;          // [F] global cursor
  uint32_t* lcnt = cur + F;                // [F] sub-chunk count -> offset
  uint32_t* stage = lcnt + F;              // [CH] records sorted by tile
  uint16_t* ltile = (uint16_t*)(stage + CH);  // unused
  (void)ltile;
  for (int i = threadIdx.x; i < LIM_PAD; i += WG) lim[i] = limg[i];
  for (uint32_t t = threadIdx.x; t < F; t += WG) {
    cur[t] = cur0[(size_t)blockIdx.x * F + t];
    lcnt[t] = 0;
  }
  __syncthreads();
  const size_t lo = blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  constexpr int PER_T = CH / WG;
  for (size_t c0 = lo; c0 < hi; c0 += CH) {
    uint32_t rec[PER_T], tile[PER_T], rank[PER_T];
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
      size_t i = c0 + k * WG + threadIdx.x;
      if (i < hi) {
        uint32_t s = series[i];
        float f = values[i];
        uint32_t b = search(f, lim);
        rec[k] = ((s & 31) << 27) | (b << 16);
        tile[k] = s >> 5;
        rank[k] = atomicAdd(&lcnt[tile[k]], 1u);
      } else {
        tile[k] = 0xFFFFFFFF;
      }
    }
    __syncthreads();
    // exclusive scan of lcnt over F tiles (block-wide), keep counts in cur-space
    // simple: each thread scans a contiguous range
    {
      __shared__ uint32_t part[17];
      const uint32_t per_t = (F + WG - 1) / WG;
      const uint32_t t0 = threadIdx.x * per_t;
      uint32_t s = 0;
      for (uint32_t k = 0; k < per_t && t0 + k < F; ++k) s += lcnt[t0 + k];
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      uint32_t x = s;
      for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
      if (lane == 63) part[w] = x;
      __syncthreads();
      if (threadIdx.x == 0) { uint32_t q = 0; for (int k = 0; k < 16; ++k) { uint32_t v = part[k]; part[k] = q; q += v; } }
      __syncthreads();
      uint32_t a = part[w] + x - s;
      for (uint32_t k = 0; k < per_t && t0 + k < F; ++k) {
        uint32_t v = lcnt[t0 + k];
        lcnt[t0 + k] = a;  // exclusive offset in stage
        a += v;
      }
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < PER_T; ++k)
      if (tile[k] != 0xFFFFFFFF) stage[lcnt[tile[k]] + rank[k]] = rec[k] | (tile[k] & 0);
    __syncthreads();
    // write runs: thread per staged record, need its tile: recompute by binary search over lcnt (offsets)
    const uint32_t total = (uint32_t)((hi - c0) < CH ? (hi - c0) : CH);
    for (uint32_t j = threadIdx.x; j < total; j += WG) {
      // find tile t with lcnt[t] <= j < lcnt[t+1]
      uint32_t a = 0, b = F;
      while (b - a > 1) {
        uint32_t m = (a + b) >> 1;
        if (lcnt[m] <= j) a = m; else b = m;
      }
      out[cur[a] + (j - lcnt[a])] = stage[j];
    }
    __syncthreads();
    // advance cursors, reset counts
    for (uint32_t t = threadIdx.x; t < F; t += WG) {
      uint32_t nxt = (t + 1 < F) ? lcnt[t + 1] : total;
      cur[t] += nxt - lcnt[t];
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < F; t += WG) lcnt[t] = 0;
    __syncthreads();
  }
}

__global__ void count_k(const uint32_t* series, size_t n, size_t per, uint32_t F, uint32_t* table) {
  extern __shared__ uint32_t cnt[];
  for (uint32_t t = threadIdx.x; t < F; t += blockDim.x) cnt[t] = 0;
  __syncthreads();
  size_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (size_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&cnt[series[i] >> 5], 1u);
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < F; t += blockDim.x) table[(size_t)blockIdx.x * F + t] = cnt[t];
}

int main(int argc, char** argv) {
  size_t n = argc > 1 ? atoll(argv[1]) : 100000000ull;
  uint32_t S = argc > 2 ? atoi(argv[2]) : 100000;
  int G = argc > 3 ? atoi(argv[3]) : 256;
  uint32_t F = (S + 31) / 32;
  uint32_t *series, *out, *sink, *table, *cur0;
  float* values;
  int32_t* lim;
  CHK(hipMalloc(&series, n * 4));
  CHK(hipMalloc(&values, n * 4));
  CHK(hipMalloc(&out, n * 4 + 64));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMalloc(&table, (size_t)G * F * 4));
  CHK(hipMalloc(&cur0, (size_t)G * F * 4));
  CHK(hipMalloc(&lim, LIM_PAD * 4));
  std::vector<int32_t> L(LIM_PAD, 2147483647);
  {
    double cur = 1.0;
    int k = 0;
    L[k++] = 1;
    int last = -1;
    for (;;) {
      double nx = cur * 1.01;
      if (nx >= 2147483647.0) break;
      int v = (int)nx + 1;
      if (v != last) L[k++] = last = v;
      cur = nx;
    }
  }
  CHK(hipMemcpy(lim, L.data(), LIM_PAD * 4, hipMemcpyHostToDevice));
  gen<<<2048, 256>>>(series, values, n, S);
  size_t per = ((n + G - 1) / G + 3) & ~(size_t)3;
  for (int kset : {0}) (void)kset;
  CHK(hipFuncSetAttribute((const void*)count_k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  count_k<<<G, 1024, F * 4>>>(series, n, per, F, table);
  CHK(hipDeviceSynchronize());
  // exclusive offsets (host)
  std::vector<uint32_t> tab((size_t)G * F), off((size_t)G * F);
  CHK(hipMemcpy(tab.data(), table, tab.size() * 4, hipMemcpyDeviceToHost));
  uint64_t acc = 0;
  for (uint32_t t = 0; t < F; ++t)
    for (int g = 0; g < G; ++g) {
      off[(size_t)g * F + t] = (uint32_t)acc;
      acc += tab[(size_t)g * F + t];
    }
  CHK(hipMemcpy(cur0, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    launch();
    CHK(hipDeviceSynchronize());
    float best = 1e9, sum = 0;
    const int R = 5;
    for (int r = 0; r < R; ++r) {
      CHK(hipEventRecord(a));
      launch();
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
      sum += ms;
    }
    printf("%-10s best %.3f ms avg %.3f ms  (%.1f Gsamples/s, %.2f TB/s of 8B/sample)\n", name, best, sum / R,
           n / best / 1e6, n * 8.0 / best / 1e9);
  };
  const size_t lds = (LIM_PAD + F) * 4;
  CHK(hipFuncSetAttribute((const void*)kbin<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHK(hipFuncSetAttribute((const void*)kbin<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHK(hipFuncSetAttribute((const void*)kbin<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHK(hipFuncSetAttribute((const void*)kbin<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHK(hipFuncSetAttribute((const void*)kbin<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  printf("n=%zu S=%u F=%u G=%d\n", n, S, F, G);
  run("read", [&] { kbin<0><<<G, WG, lds>>>(series, values, n, per, F, nullptr, lim, out, sink); });
  run("search", [&] { kbin<1><<<G, WG, lds>>>(series, values, n, per, F, nullptr, lim, out, sink); });
  run("cursor", [&] { kbin<2><<<G, WG, lds>>>(series, values, n, per, F, cur0, lim, out, sink); });
  run("scatter", [&] { kbin<3><<<G, WG, lds>>>(series, values, n, per, F, cur0, lim, out, sink); });
  run("seqstore", [&] { kbin<4><<<G, WG, lds>>>(series, values, n, per, F, cur0, lim, out, sink); });
  constexpr int CH = 16384;
  const size_t lds5 = (LIM_PAD + 2 * F + CH) * 4;
  if (lds5 <= 160 * 1024 - 512) {
    CHK(hipFuncSetAttribute((const void*)kbin_sorted<CH>, hipFuncAttributeMaxDynamicSharedMemorySize, lds5));
    run("sorted16k", [&] { kbin_sorted<CH><<<G, WG, lds5>>>(series, values, n, per, F, cur0, lim, out); });
  }
  constexpr int CH2 = 8192;
  const size_t lds6 = (LIM_PAD + 2 * F + CH2) * 4;
  if (lds6 <= 160 * 1024 - 512) {
    CHK(hipFuncSetAttribute((const void*)kbin_sorted<CH2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds6));
    run("sorted8k", [&] { kbin_sorted<CH2><<<G, WG, lds6>>>(series, values, n, per, F, cur0, lim, out); });
  }
  return 0;
}
