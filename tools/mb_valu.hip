// mb_valu.hip -- microbenchmark: VALU throughput of integer vs float ops (wave64, gfx950).
// Each thread runs ITER iterations of 8 independent dependency chains.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int ITER = 4096;

template <int OP>
__global__ __launch_bounds__(256) void kv(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = threadIdx.x * 7u + j + seed;
    f[j] = (float)a[j];
  }
  const uint32_t c = seed | 1u;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) a[j] = a[j] + c;                       // v_add_u32
      else if (OP == 1) a[j] = (a[j] ^ c) + (a[j] >> 3);  // xor, lshr, add (3 ops)
      else if (OP == 2) f[j] = f[j] * 1.0001f + 0.5f;     // v_fma_f32
      else if (OP == 3) a[j] = a[j] * c;                   // v_mul_lo_u32
      else if (OP == 4) a[j] = (a[j] << 2) + c;            // v_lshl_add_u32
      else if (OP == 5) a[j] = a[j] > c ? a[j] - c : a[j] + 7u;  // cmp + cndmask + 2 add
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= a[j] ^ __float_as_uint(f[j]);
  if (r == 0x9E3779B9u) out[blockIdx.x] = r;
}

template <int OP>
void run(const char* name, int ops_per_iter, int waves_per_simd) {
  const int blocks = 256 * waves_per_simd;  // 256-thread blocks = 4 waves = 1 per SIMD
  uint32_t* d;
  CHK(hipMalloc(&d, blocks * 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(kv<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  CHK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kv<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u + r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  const double winstr = (double)blocks * 4 * ITER * 8 * ops_per_iter;  // wave-instructions
  const double per_simd = winstr / 1024.0;
  printf("%-24s waves/SIMD %d: %7.3f ms  %5.2f cyc per wave-instr per SIMD (at 2.4 GHz)\n", name, waves_per_simd, ms,
         ms * 1e-3 * 2.4e9 / per_simd);
  CHK(hipFree(d));
}

int main() {
  for (int w : {2, 4, 8}) {
    run<0>("v_add_u32", 1, w);
    run<1>("xor+lshr+add", 3, w);
    run<2>("v_fma_f32", 1, w);
    run<3>("v_mul_lo_u32", 1, w);
    run<4>("v_lshl_add_u32", 1, w);
    run<5>("cmp+cndmask+add", 3, w);
  }
  return 0;
}
