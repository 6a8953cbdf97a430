// Microbenchmark: issue cost of v_mfma_f32_4x4x1_16b_f32 (16 independent 4x4 blocks, k = 1)
// against v_mfma_f32_16x16x4_f32, at 1 and 2 waves per SIMD: ITER iterations of 8
// independent accumulator chains; cycles per MFMA from the shader clock (s_memtime).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_4x4_rate scripts/mfma_4x4_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
#define ITER 4000

template <bool SMALL>
__global__ void __launch_bounds__(512) kern(float *out, long long *cyc, float a, float b) {
  f4 c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = f4{0.f, 0.f, 0.f, (float)k};
  const float A_ = a * threadIdx.x, B_ = b - threadIdx.x;
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (SMALL) c[k] = __builtin_amdgcn_mfma_f32_4x4x1f32(A_, B_, c[k], 0, 0, 0);
      else c[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(A_, B_, c[k], 0, 0, 0);
    }
  }
  long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += c[k][0] + c[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <bool SMALL>
static void run(int waves_per_simd) {
  const int threads = 64 * 4 * waves_per_simd, blocks = 256;
  float *out;
  long long *cyc;
  hipMalloc(&out, sizeof(float) * threads * blocks);
  hipMalloc(&cyc, sizeof(long long) * (threads / 64) * blocks);
  hipLaunchKernelGGL(kern<SMALL>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0001f, 0.9999f);
  hipLaunchKernelGGL(kern<SMALL>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0001f, 0.9999f);
  hipDeviceSynchronize();
  const int n = (threads / 64) * blocks;
  long long *h = (long long *)malloc(sizeof(long long) * n);
  hipMemcpy(h, cyc, sizeof(long long) * n, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < n; ++i) avg += (double)h[i];
  avg /= n;
  printf("%s waves/SIMD %d: %.2f cycles per MFMA per wave (%.2f per SIMD)\n",
         SMALL ? "4x4x1_16b_f32 " : "16x16x4_f32   ", waves_per_simd, avg / (ITER * 8.0),
         avg / (ITER * 8.0) / waves_per_simd);
  free(h);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 2; ++w) {
    run<false>(w);
    run<true>(w);
  }
  return 0;
}
