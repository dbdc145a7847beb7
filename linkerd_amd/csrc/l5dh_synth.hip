// l5dh_synth.hip -- synthetic BASELINE.md workloads generated in HBM (bench and
// test infrastructure; not part of the engine).  Same counter-based recipe as
// linkerd_amd/synth.py: rand(seed, stream, i) = mix64(((seed<<48) ^ (stream<<40)
// ^ i) + 1) * GOLD), Box-Muller normals, float32(exp(mu + sigma*z)) clamped to
// [0, 1e9].  Device libm may differ from numpy in the last ulp, so values are
// recipe-equivalent, not bit-identical to synth.py; parity tests always feed
// the same bytes to the engine and to the oracle.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr uint64_t GOLD = 0x9E3779B97F4A7C15ull;
constexpr uint64_t PERM_A = 2654435761ull;
constexpr uint64_t PERM_B = 40503ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ double uni(uint64_t seed, uint64_t stream, uint64_t i) {
  return (double)(mix64((((seed << 48) ^ (stream << 40) ^ i) + 1ull) * GOLD) >> 11) * 0x1.0p-53;
}

__device__ __forceinline__ double normal(uint64_t seed, uint64_t stream, uint64_t i) {
  const double u1 = uni(seed, stream, 2 * i) + 0x1.0p-53;
  const double u2 = uni(seed, stream, 2 * i + 1);
  return sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
}

__device__ __forceinline__ float lognormal(double mu, double sigma, double z) {
  double v = exp(mu + sigma * z);
  v = v < 0.0 ? 0.0 : (v > 1e9 ? 1e9 : v);
  return (float)v;
}

__device__ __forceinline__ double series_mu(uint64_t seed, uint32_t s) {
  return log(1.0 + 999.0 * uni(seed, 1, s));
}

__global__ void k_gen_c1(float* __restrict__ values, uint32_t* __restrict__ series, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    values[i] = lognormal(log(20.0), 1.0, normal(seed, 2, i));
    series[i] = 0;
  }
}

__global__ void k_gen_c2(uint32_t* __restrict__ series, float* __restrict__ values, uint64_t S, uint64_t K,
                         uint64_t seed, double sigma, uint32_t series_base) {
  const uint64_t N = S * K;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = (i * PERM_A + PERM_B) % N;
    const uint32_t s = (uint32_t)(j / K);
    series[i] = s;  // local id within this shard; series_base only seeds mu
    values[i] = lognormal(series_mu(seed, s + series_base), sigma, normal(seed, 2, j));
  }
}

// Zipf(s=1) series by inverse CDF (cdf[r] = H(r+1)/H(S), device array), values as C2.
__global__ void k_gen_zipf(uint32_t* __restrict__ series, float* __restrict__ values, uint64_t n, uint64_t S,
                           const double* __restrict__ cdf, uint64_t seed, double sigma, uint64_t base_index,
                           uint32_t series_base) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t gi = base_index + i;
    const double u = uni(seed, 3, gi);
    uint64_t lo = 0, hi = S;  // first r with cdf[r] > u
    while (lo < hi) {
      const uint64_t m = (lo + hi) >> 1;
      if (cdf[m] <= u) lo = m + 1; else hi = m;
    }
    const uint32_t s = (uint32_t)(lo < S ? lo : S - 1);
    series[i] = s;  // local id within this shard; series_base only seeds mu
    values[i] = lognormal(series_mu(seed, s + series_base), sigma, normal(seed, 2, gi));
  }
}

}  // namespace

extern "C" {

int l5ds_gen_c1(float* values, uint32_t* series, uint64_t n, uint64_t seed, void* stream) {
  hipLaunchKernelGGL(k_gen_c1, dim3(4096), dim3(256), 0, (hipStream_t)stream, values, series, n, seed);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int l5ds_gen_c2(uint32_t* series, float* values, uint64_t S, uint64_t K, uint64_t seed, double sigma,
                uint32_t series_base, void* stream) {
  hipLaunchKernelGGL(k_gen_c2, dim3(4096), dim3(256), 0, (hipStream_t)stream, series, values, S, K, seed, sigma,
                     series_base);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int l5ds_gen_zipf(uint32_t* series, float* values, uint64_t n, uint64_t S, const double* cdf, uint64_t seed,
                  double sigma, uint64_t base_index, uint32_t series_base, void* stream) {
  hipLaunchKernelGGL(k_gen_zipf, dim3(4096), dim3(256), 0, (hipStream_t)stream, series, values, n, S, cdf, seed,
                     sigma, base_index, series_base);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
