// mb_store.hip -- microbenchmark: dense-row store rate on gfx950, shaped like the
// cold accumulate's emission: T tiles of 32 rows x 7192 B (contiguous per tile),
// one persistent 1024-thread workgroup per CU walking tiles; each wave stores its
// rows with 16-B stores in the coalesced lane order (lane l -> groups l + 64 k).
// Variants: 0 stores only; 1 stores + an LDS read per group (u16 source);
// 2 = 1 with a workgroup barrier per tile; 3 the tile as one linear range stored by
// the whole workgroup.  Prints TB/s.
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

constexpr int NB = 1798, NB4 = 450;

template <int V>
__global__ __launch_bounds__(1024, 1) void ks(int32_t* out, uint32_t tiles) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < 32 * 900; i += 1024) lds[i] = i * 0x10001u;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (V == 3) {  // the tile as one linear range of 14384 16-B chunks, the workgroup in lockstep
    for (uint32_t t = blockIdx.x; t < tiles; t += gridDim.x) {
      uint4* o = reinterpret_cast<uint4*>(out + (size_t)t * 32 * NB);
      for (int c = threadIdx.x; c < 14384; c += 1024) {
        const int e = 4 * c;
        const int r0 = e / NB, b0 = e - r0 * NB;
        const int r1 = (e + 2) / NB, b1 = e + 2 - r1 * NB;
        const uint32_t x = lds[r0 * 900 + (b0 >> 1)], y = lds[r1 * 900 + (b1 >> 1)];
        o[c] = make_uint4(x & 0xFFFFu, x >> 16, y & 0xFFFFu, y >> 16);
      }
      __syncthreads();
    }
    return;
  }
  for (uint32_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    for (int loc = w; loc < 32; loc += 16) {
      const size_t oi = (size_t)t * 32 + loc;
      int32_t* orow = out + oi * NB;
      const uint32_t* row = lds + loc * 900;
#pragma unroll 2
      for (int k = 0; k < 8; ++k) {
        const int q = lane + 64 * k;
        if (q < NB4) {
          uint4 v = make_uint4(q, q, q, q);
          if (V >= 1) {
            const uint2 x = *reinterpret_cast<const uint2*>(row + 2 * q);
            v = make_uint4(x.x & 0xFFFFu, x.x >> 16, x.y & 0xFFFFu, x.y >> 16);
          }
          if ((oi & 1) == 0 && q != 449) {
            *reinterpret_cast<uint4*>(orow + 4 * q) = v;
          } else {
            *reinterpret_cast<uint2*>(orow + 4 * q) = make_uint2(v.x, v.y);
            if (q != 449) *reinterpret_cast<uint2*>(orow + 4 * q + 2) = make_uint2(v.z, v.w);
          }
        }
      }
    }
    if (V == 2) __syncthreads();
  }
}

int main(int argc, char** argv) {
  const uint32_t tiles = argc > 1 ? atoi(argv[1]) : 30000;
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  int32_t* out;
  const size_t bytes = (size_t)tiles * 32 * NB * 4;
  CHK(hipMalloc(&out, bytes));
  CHK(hipFuncSetAttribute((const void*)ks<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CHK(hipFuncSetAttribute((const void*)ks<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CHK(hipFuncSetAttribute((const void*)ks<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CHK(hipFuncSetAttribute((const void*)ks<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int v = 0; v < 4; ++v) {
    for (int grid_mul = 1; grid_mul <= 2; ++grid_mul) {
      float best = 1e9f;
      for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(a));
        if (v == 0) hipLaunchKernelGGL(ks<0>, dim3(ncu * grid_mul), dim3(1024), 131072, 0, out, tiles);
        if (v == 1) hipLaunchKernelGGL(ks<1>, dim3(ncu * grid_mul), dim3(1024), 131072, 0, out, tiles);
        if (v == 2) hipLaunchKernelGGL(ks<2>, dim3(ncu * grid_mul), dim3(1024), 131072, 0, out, tiles);
        if (v == 3) hipLaunchKernelGGL(ks<3>, dim3(ncu * grid_mul), dim3(1024), 131072, 0, out, tiles);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      printf("variant %d grid %dx: %.3f ms  %.2f TB/s\n", v, grid_mul, best, bytes / (best * 1e-3) / 1e12);
    }
  }
  // plain copy-like reference: hipMemsetD32 over the same bytes
  float best = 1e9f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(a));
    CHK(hipMemsetD32((hipDeviceptr_t)out, 7, bytes / 4));
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  printf("hipMemsetD32: %.3f ms  %.2f TB/s\n", best, bytes / (best * 1e-3) / 1e12);
  CHK(hipFree(out));
  return 0;
}
