// mb_lds.hip -- microbenchmark: LDS atomic / read / write throughput on gfx950.
// Every CU runs one (or two) 1024-thread workgroups; each thread issues ITER
// LDS ops whose addresses follow a pattern:
//   0 conflict-free (addr = lane-linear), 1 random over `span` words,
//   2 same address per wave, 3 random over 32 words (same-address heavy)
// ops: 0 ds_add_u32 (no return), 1 ds_add_rtn_u32, 2 ds_write_b32, 3 ds_read_b32,
//      4 ds_add_u64 (no return), 5 ds_add_rtn_u32 + dependent use
// Prints lane-ops per clock per CU (2.4 GHz assumed for the clock).
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

constexpr int NT = 1024;
constexpr int ITER = 4096;

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

template <int OP, int PAT>
__global__ __launch_bounds__(NT) void kl(uint32_t* out, uint32_t span, uint32_t seed) {
  extern __shared__ uint32_t lds[];
  for (uint32_t i = threadIdx.x; i < span + 64; i += NT) lds[i] = 0;
  __syncthreads();
  uint32_t acc = 0;
  uint32_t h = hsh(threadIdx.x * 7919u + blockIdx.x * 104729u + seed);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t ad[16];  // addresses precomputed: the loop is LDS-only
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint32_t a;
    if (PAT == 0) a = (threadIdx.x + k * 64u) & (span - 1);
    else if (PAT == 1) a = h & (span - 1);
    else if (PAT == 2) a = ((threadIdx.x >> 6) * 97u + k) & (span - 1);
    else a = h & 31u;
    h = h * 1664525u + 1013904223u;
    h ^= h >> 13;
    ad[k] = a;
  }
  for (int it = 0; it < ITER / 16; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t a = ad[k];
      if (OP == 0) atomicAdd(&lds[a], 1u);
      else if (OP == 1) acc += atomicAdd(&lds[a], 1u);
      else if (OP == 2) lds[a] = it;
      else if (OP == 3) acc += lds[a];
      else if (OP == 4) atomicAdd(reinterpret_cast<unsigned long long*>(&lds[a & ~1u]), 1ull);
      else if (OP == 5) acc += atomicAdd(&lds[a], 1u);
    }
    asm volatile("" ::: "memory");
  }
  (void)lane;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc + lds[0] + h;
}

template <int OP, int PAT>
void run(const char* name, int blocks, uint32_t span, uint32_t* d_out) {
  const size_t lds = (span + 64) * 4;
  CHK(hipFuncSetAttribute((const void*)kl<OP, PAT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL((kl<OP, PAT>), dim3(blocks), dim3(NT), lds, 0, d_out, span, 1u);
  CHK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((kl<OP, PAT>), dim3(blocks), dim3(NT), lds, 0, d_out, span, 2u + r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  const double lane_ops = (double)blocks * NT * ITER;
  const double per_cu_clk = lane_ops / 256.0 / (ms * 1e-3 * 2.4e9);
  printf("%-28s span %6u blocks %4d: %8.3f ms  %6.2f lane-ops/clk/CU  (%5.1f clk per wave-instr)\n", name, span, blocks,
         ms, per_cu_clk, 64.0 / per_cu_clk);
}

int main() {
  uint32_t* d_out;
  CHK(hipMalloc(&d_out, 4096 * 4));
  const int B = 256;
  for (uint32_t span : {1024u, 32768u}) {
    run<0, 0>("add_u32 noret linear", B, span, d_out);
    run<0, 1>("add_u32 noret random", B, span, d_out);
    run<0, 2>("add_u32 noret same-addr", B, span, d_out);
    run<0, 3>("add_u32 noret rand32", B, span, d_out);
    run<1, 0>("add_rtn_u32 linear", B, span, d_out);
    run<1, 1>("add_rtn_u32 random", B, span, d_out);
    run<1, 3>("add_rtn_u32 rand32", B, span, d_out);
    run<5, 1>("add_rtn_u32 random dep", B, span, d_out);
    run<2, 0>("write_b32 linear", B, span, d_out);
    run<2, 1>("write_b32 random", B, span, d_out);
    run<3, 0>("read_b32 linear", B, span, d_out);
    run<3, 1>("read_b32 random", B, span, d_out);
    run<4, 1>("add_u64 noret random", B, span, d_out);
  }
  run<0, 1>("add_u32 noret random 2/CU", 2 * B, 16384, d_out);
  run<1, 1>("add_rtn_u32 random 2/CU", 2 * B, 16384, d_out);
  return 0;
}
