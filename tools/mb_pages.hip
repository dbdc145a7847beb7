// mb_pages.hip -- measured prototype of the k_count-free level-1 partition
// (verdict item 5): k_bin1's LDS counting sort with placement
// from CU-private PAGE POOLS instead of the count table, so the separate id
// pass (k_count) and the column/tile scans disappear.
//
// Input: the C3 workload from libl5dsynth (1M series Zipf(s=1), 1e9 samples,
// log-normal values), as bench.py generates it.  Bins as the engine's k_bin1:
// FS super-tiles + two per direct tile (here the 255 Zipf-hottest tiles, the
// set k_stplan picks on C3) + a trash bin.  Each slab (one 1024-thread
// workgroup per CU) owns a pool of P-record pages; a bin's run continues in the
// bin's current page and spills into freshly allocated, consecutive pages (one
// LDS atomic per spilling bin and sub-chunk, no global atomics), logged as
// (page, bin, pages) for the consumer.
//
// Checks: every sample placed exactly once -- per-bin totals (the pages' fills)
// equal an exact count, and a hash of all placed records equals the hash of
// all input records.  Prints per-launch ms (HIP events).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_pages.hip -o tools/mb_pages \
//         -Llinkerd_amd/lib -ll5dsynth -Wl,-rpath,$PWD/linkerd_amd/lib
//   tools/mb_pages [n=1e9] [reps=5] [page=4096]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" int l5ds_gen_zipf(uint32_t* series, float* values, uint64_t n, uint64_t S, const double* cdf, uint64_t seed,
                             double sigma, uint64_t base_index, uint32_t series_base, void* stream);

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int CH1 = 16384, NT = 1024, PT = CH1 / NT;
constexpr int BINS = 1024;
constexpr uint32_t S_C3 = 1000000;
constexpr int ND = 255;  // direct tiles: tiles 0..ND-1 (Zipf ranks are ids)

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if ((int)lane_id() >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ uint32_t bin_of(uint32_t s, uint32_t S, uint32_t FS, uint32_t TB) {
  const uint32_t t = s >> 5;
  return s >= S ? TB : (t < (uint32_t)ND ? FS + 2u * t + ((s >> 4) & 1u) : (s >> 11));
}
__device__ __forceinline__ uint32_t rec_of(uint32_t s, float f) {
  const uint32_t v = (f >= 0.0f && f < 2095104.0f) ? (uint32_t)f : 2095104u;
  return ((s & 2047u) << 21) | v;
}
__device__ __forceinline__ uint64_t rhash(uint32_t r) {
  uint64_t z = (uint64_t)r * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  z ^= z >> 29;
  z *= 0xBF58476D1CE4E5B9ull;
  return z ^ (z >> 32);
}

// LDS: stage[CH1] uint2 | cnt | boff | dA | room | dB | pg | fill [BINS] | pool cursor, log cursor
constexpr size_t LDS_BYTES = (size_t)CH1 * 8 + 7 * BINS * 4 + 16;

__global__ __launch_bounds__(NT, 1) void k_bin1p(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                                 size_t n, size_t per, uint32_t S, uint32_t P, uint32_t pool_pages,
                                                 uint32_t* __restrict__ pool, uint2* __restrict__ plog,
                                                 uint32_t* __restrict__ nlog, uint2* __restrict__ tailpg,
                                                 const uint32_t* __restrict__ dst0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint2* stage = reinterpret_cast<uint2*>(smem);
  uint32_t* cnt = smem + 2 * CH1;
  uint32_t* boff = cnt + BINS;
  uint32_t* dA = boff + BINS;
  uint32_t* room = dA + BINS;
  uint32_t* dB = room + BINS;
  uint32_t* pg = dB + BINS;
  uint32_t* fill = pg + BINS;
  uint32_t* cur = fill + BINS;  // [0] next free page of the pool, [1] log entries
  const uint32_t FS = (S + 2047) / 2048;
  const uint32_t TB = FS + 2 * ND;
  const uint32_t g = blockIdx.x;
  const uint32_t pool0 = g * pool_pages;  // first page of this slab's pool
  // dst0 (comparison layouts): exact per-(slab, bin) start positions, no pages
  for (uint32_t b = threadIdx.x; b < BINS; b += NT) {
    cnt[b] = 0;
    pg[b] = dst0 ? dst0[(size_t)blockIdx.x * BINS + b] : 0u;
    fill[b] = P;  // no page yet: the first run allocates
  }
  if (threadIdx.x == 0) cur[0] = cur[1] = 0;
  __syncthreads();
  const size_t lo = (size_t)g * per;
  const size_t hi = lo + per < n ? lo + per : n;
  const int lane = (int)lane_id(), wv = threadIdx.x >> 6;
  uint2* mylog = plog + (size_t)g * pool_pages;
  for (size_t c0 = lo; c0 < hi; c0 += CH1) {
    uint32_t sv[PT];
    float fv[PT];
    if (c0 + CH1 <= hi) {
#pragma unroll
      for (int k = 0; k < PT / 4; ++k) {
        const size_t base = c0 + 4 * ((size_t)k * NT + threadIdx.x);
        const uint4 s4 = *reinterpret_cast<const uint4*>(series + base);
        const float4 f4 = *reinterpret_cast<const float4*>(values + base);
        sv[4 * k] = s4.x; sv[4 * k + 1] = s4.y; sv[4 * k + 2] = s4.z; sv[4 * k + 3] = s4.w;
        fv[4 * k] = f4.x; fv[4 * k + 1] = f4.y; fv[4 * k + 2] = f4.z; fv[4 * k + 3] = f4.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const size_t i = c0 + 4 * ((size_t)(k >> 2) * NT + threadIdx.x) + (k & 3);
        sv[k] = i < hi ? series[i] : 0xFFFFFFFFu;
        fv[k] = i < hi ? values[i] : 0.0f;
      }
    }
    uint32_t rec[PT], pk[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t b = bin_of(sv[k], S, FS, TB);
      rec[k] = rec_of(sv[k], fv[k]);
      pk[k] = atomicAdd(cnt + b, 1u) | (b << 14);
    }
    __syncthreads();
    if (wv == 0) {  // stage offsets: lane l scans bins [16 l, 16 l + 16)
      uint32_t c[16], tl = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) tl += (c[q] = cnt[16 * lane + q]);
      uint32_t e = wave_incl_scan(tl) - tl;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        boff[16 * lane + q] = e;
        e += c[q];
      }
    }
    // pages: a bin's run fills its current page, then continues in consecutive new pages
    for (uint32_t b = threadIdx.x; b < BINS; b += NT) {
      const uint32_t c = cnt[b];
      if (!c) continue;
      if (dst0) {  // exact placement: the run continues at the bin's cursor
        dA[b] = pg[b];
        room[b] = 0xFFFFFFFFu;
        pg[b] += c;
        continue;
      }
      const uint32_t rm = P - fill[b];
      dA[b] = pg[b] + fill[b];
      room[b] = rm;
      if (c <= rm) {
        fill[b] += c;
      } else {
        const uint32_t need = (c - rm + P - 1) / P;
        const uint32_t np = atomicAdd(&cur[0], need);
        const uint32_t li = atomicAdd(&cur[1], 1u);
        mylog[li] = make_uint2(pool0 + np, b | (need << 16));
        dB[b] = (pool0 + np) * P;
        pg[b] = (pool0 + np + need - 1) * P;
        fill[b] = c - rm - (need - 1) * P;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t b = pk[k] >> 14, r = pk[k] & 16383u;
      const uint32_t rm = room[b];
      stage[boff[b] + r] = make_uint2(rec[k], r < rm ? dA[b] + r : dB[b] + (r - rm));
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += NT) cnt[b] = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint2 e = stage[(uint32_t)wv * (PT * 64) + (uint32_t)k * 64 + (uint32_t)lane];
      pool[e.y] = e.x;
    }
    __syncthreads();
  }
  for (uint32_t b = threadIdx.x; b < BINS; b += NT) tailpg[(size_t)g * BINS + b] = make_uint2(pg[b], fill[b]);
  if (threadIdx.x == 0) nlog[g] = cur[1];
}

// per-(slab, bin) counts of the same slabs (for the exact comparison layouts)
__global__ __launch_bounds__(1024) void k_cnt_slab_bins(const uint32_t* __restrict__ series, size_t n, size_t per,
                                                        uint32_t S, uint32_t* __restrict__ out) {
  __shared__ uint32_t c[BINS];
  const uint32_t FS = (S + 2047) / 2048, TB = FS + 2 * ND;
  for (int b = threadIdx.x; b < BINS; b += 1024) c[b] = 0;
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (size_t i = lo + threadIdx.x; i < hi; i += 1024) atomicAdd(&c[bin_of(series[i], S, FS, TB)], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < BINS; b += 1024) out[(size_t)blockIdx.x * BINS + b] = c[b];
}

// ---- checks ----
__global__ void k_count_bins(const uint32_t* series, const float* values, size_t n, uint32_t S,
                             unsigned long long* bins, unsigned long long* hash) {
  const uint32_t FS = (S + 2047) / 2048, TB = FS + 2 * ND;
  unsigned long long h = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    atomicAdd(&bins[bin_of(series[i], S, FS, TB)], 1ull);
    h += rhash(rec_of(series[i], values[i]));
  }
  atomicAdd(hash, h);
}
// one workgroup per log entry set of a slab: walk its pages, hash the valid records
// (the trash bin -- sample slots past a slab's end -- is not compared)
__global__ void k_hash_pages(const uint32_t* pool, const uint2* plog, const uint32_t* nlog, const uint2* tailpg,
                             uint32_t pool_pages, uint32_t P, uint32_t TB, unsigned long long* bins,
                             unsigned long long* hash) {
  const uint32_t g = blockIdx.x;
  unsigned long long h = 0;
  for (uint32_t li = 0; li < nlog[g]; ++li) {
    const uint2 e = plog[(size_t)g * pool_pages + li];
    const uint32_t b = e.y & 0xFFFFu, np = e.y >> 16;
    if (b == TB) continue;
    const uint2 tp = tailpg[(size_t)g * BINS + b];
    for (uint32_t q = 0; q < np; ++q) {
      const uint32_t page = e.x + q;
      const uint32_t valid = (page * P == tp.x) ? tp.y : P;  // the bin's last page is partial
      for (uint32_t i = threadIdx.x; i < valid; i += blockDim.x) h += rhash(pool[(size_t)page * P + i]);
      if (threadIdx.x == 0) atomicAdd(&bins[b], (unsigned long long)valid);
    }
  }
  atomicAdd(hash, h);
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atof(argv[1]) : 1000000000ull;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const uint32_t P = argc > 3 ? (uint32_t)atoi(argv[3]) : 4096;
  const uint32_t S = S_C3;
  int ncu = 0;
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int G = ncu;
  size_t per = (n + G - 1) / G;
  per = (per + 3) & ~(size_t)3;
  const uint32_t pool_pages = (uint32_t)((per + P - 1) / P + BINS + 1);
  if ((double)G * pool_pages * P >= 4294967296.0) {
    printf("pool of %.3g records: record indices must fit u32 (smaller n or page)\n", (double)G * pool_pages * P);
    return 1;
  }
  printf("n=%zu S=%u G=%d per=%zu page=%u records (%u KB) pool=%u pages/slab (%.2f GB total)\n", n, S, G, per, P,
         P * 4 / 1024, pool_pages, (double)G * pool_pages * P * 4 / 1e9);
  std::vector<double> cdf(S);
  double acc = 0;
  for (uint32_t k = 0; k < S; ++k) cdf[k] = (acc += 1.0 / (k + 1.0));
  for (auto& x : cdf) x /= acc;
  cdf[S - 1] = 1.0;
  double* dcdf;
  uint32_t *series, *pool, *nlog;
  float* values;
  uint2 *plog, *tailpg;
  unsigned long long* chk;
  CHK(hipMalloc(&dcdf, S * 8));
  CHK(hipMemcpy(dcdf, cdf.data(), S * 8, hipMemcpyHostToDevice));
  CHK(hipMalloc(&series, n * 4 + 64));
  CHK(hipMalloc(&values, n * 4 + 64));
  CHK(hipMalloc(&pool, (size_t)G * pool_pages * P * 4));
  CHK(hipMalloc(&plog, (size_t)G * pool_pages * 8));
  CHK(hipMalloc(&nlog, G * 4));
  CHK(hipMalloc(&tailpg, (size_t)G * BINS * 8));
  CHK(hipMalloc(&chk, (2 * BINS + 2) * 8));
  if (l5ds_gen_zipf(series, values, n, S, dcdf, 3, 0.8, 0, 0, nullptr)) return 1;
  CHK(hipDeviceSynchronize());
  CHK(hipFuncSetAttribute((const void*)k_bin1p, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES));
  // comparison layouts with exact placement (the engine's k_count provides it):
  // bin-major = the engine's level-1 layout (a bin's region, slabs in order inside
  // it); slab-major = each slab's own region, bins in order inside it
  uint32_t *cnts, *dbm, *dsm;
  CHK(hipMalloc(&cnts, (size_t)G * BINS * 4));
  CHK(hipMalloc(&dbm, (size_t)G * BINS * 4));
  CHK(hipMalloc(&dsm, (size_t)G * BINS * 4));
  hipLaunchKernelGGL(k_cnt_slab_bins, dim3(G), dim3(1024), 0, 0, series, n, per, S, cnts);
  std::vector<uint32_t> hc((size_t)G * BINS), hb((size_t)G * BINS), hs((size_t)G * BINS);
  CHK(hipMemcpy(hc.data(), cnts, hc.size() * 4, hipMemcpyDeviceToHost));
  {
    uint64_t x = 0;
    for (int bb = 0; bb < BINS; ++bb)
      for (int g = 0; g < G; ++g) {
        hb[(size_t)g * BINS + bb] = (uint32_t)x;
        x += hc[(size_t)g * BINS + bb];
      }
    x = 0;
    for (int g = 0; g < G; ++g)
      for (int bb = 0; bb < BINS; ++bb) {
        hs[(size_t)g * BINS + bb] = (uint32_t)x;
        x += hc[(size_t)g * BINS + bb];
      }
  }
  CHK(hipMemcpy(dbm, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dsm, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  // bin-major with every (slab, bin) segment start aligned to A records (gaps between)
  const uint32_t AL[2] = {16, 1024};
  uint32_t* dal[2];
  for (int q = 0; q < 2; ++q) {
    uint64_t x = 0;
    for (int bb = 0; bb < BINS; ++bb)
      for (int g = 0; g < G; ++g) {
        const uint32_t c = hc[(size_t)g * BINS + bb];
        if (c) x = (x + AL[q] - 1) / AL[q] * AL[q];
        hb[(size_t)g * BINS + bb] = (uint32_t)x;
        x += c;
      }
    if (x + 20000 > (uint64_t)G * pool_pages * P) { printf("aligned layout exceeds the pool\n"); return 1; }
    CHK(hipMalloc(&dal[q], (size_t)G * BINS * 4));
    CHK(hipMemcpy(dal[q], hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int NM = 5;
  const char* names[NM] = {"pages", "bin-major (engine layout)", "slab-major", "bin-major, 64-B aligned", "bin-major, 4-KB aligned"};
  const uint32_t* tabs[NM] = {nullptr, dbm, dsm, dal[0], dal[1]};
  double best[NM], sum[NM];
  for (int m = 0; m < NM; ++m) best[m] = 1e30, sum[m] = 0;
  for (int r = 0; r < reps + 1; ++r)
    for (int m = NM - 1; m >= 0; --m) {  // pages last: its pool is what the checks read
      CHK(hipEventRecord(a));
      hipLaunchKernelGGL(k_bin1p, dim3(G), dim3(NT), LDS_BYTES, 0, series, values, n, per, S, P, pool_pages, pool,
                         plog, nlog, tailpg, tabs[m]);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (r > 0) {  // the first round is a warmup (first touch of the pool)
        best[m] = ms < best[m] ? ms : best[m];
        sum[m] += ms;
      }
    }
  for (int m = 0; m < NM; ++m)
    printf("k_bin1p %-26s mean %.4f ms, best %.4f ms over %d launches (%.1f GB/s of input)\n", names[m], sum[m] / reps,
           best[m], reps, 8.0 * n / (sum[m] / reps) / 1e6);
  // checks
  CHK(hipMemset(chk, 0, (2 * BINS + 2) * 8));
  unsigned long long* bins_in = chk;
  unsigned long long* bins_out = chk + BINS;
  hipLaunchKernelGGL(k_count_bins, dim3(4096), dim3(256), 0, 0, series, values, n, S, bins_in, chk + 2 * BINS);
  hipLaunchKernelGGL(k_hash_pages, dim3(G), dim3(256), 0, 0, pool, plog, nlog, tailpg, pool_pages, P,
                     (S + 2047) / 2048 + 2 * ND, bins_out,
                     chk + 2 * BINS + 1);
  std::vector<unsigned long long> h(2 * BINS + 2);
  CHK(hipMemcpy(h.data(), chk, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<uint32_t> nl(G);
  CHK(hipMemcpy(nl.data(), nlog, G * 4, hipMemcpyDeviceToHost));
  size_t bad = 0, logs = 0, placed = 0;
  for (int k = 0; k < BINS; ++k) {
    bad += h[k] != h[BINS + k];
    placed += h[BINS + k];
  }
  for (int g = 0; g < G; ++g) logs += nl[g];
  const bool ok = bad == 0 && placed == n && h[2 * BINS] == h[2 * BINS + 1];
  printf("check: %s (bins differing %zu, placed %zu of %zu, hash %s); page allocations %zu (%.1f per slab)\n",
         ok ? "ok" : "FAILED", bad, placed, n, h[2 * BINS] == h[2 * BINS + 1] ? "equal" : "DIFFERS", logs,
         (double)logs / G);
  return ok ? 0 : 2;
}
