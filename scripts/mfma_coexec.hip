// Microbenchmark: does independent VALU work hide under v_mfma_f32_16x16x4_f32?
// Each wave runs ITER iterations of: 4 independent MFMAs (4 accumulators) with
// NV independent v_fma_f32 per MFMA placed between them.  Reports cycles per
// MFMA (s_memtime) for NV = 0..12, at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
#ifdef USE_BF16
#define MFMA(A_, B_, C_) __builtin_amdgcn_mfma_f32_16x16x32_bf16(A_, B_, C_, 0, 0, 0)
#else
#define MFMA(A_, B_, C_) __builtin_amdgcn_mfma_f32_16x16x4f32(A_, B_, C_, 0, 0, 0)
#endif
#define ITER 2000

template <int NV>
__global__ void __launch_bounds__(512) kern(float *out, long long *cyc, float a, float b) {
  f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
#ifdef USE_BF16
  bf8 A_, B_;
  for (int i = 0; i < 8; ++i) { A_[i] = (__bf16)(a + i); B_[i] = (__bf16)(b - i); }
#else
  float A_ = a, B_ = b;
#endif
  float v[48];
#pragma unroll
  for (int i = 0; i < 48; ++i) v[i] = a * (threadIdx.x + i);
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
    c0 = MFMA(A_, B_, c0);
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = __builtin_fmaf(v[i], a, b);
    c1 = MFMA(A_, B_, c1);
#pragma unroll
    for (int i = 0; i < NV; ++i) v[12 + i] = __builtin_fmaf(v[12 + i], b, a);
    c2 = MFMA(A_, B_, c2);
#pragma unroll
    for (int i = 0; i < NV; ++i) v[24 + i] = __builtin_fmaf(v[24 + i], a, b);
    c3 = MFMA(A_, B_, c3);
#pragma unroll
    for (int i = 0; i < NV; ++i) v[36 + i] = __builtin_fmaf(v[36 + i], b, a);
  }
  long long t1 = __builtin_readcyclecounter();
  float s = c0[0] + c1[1] + c2[2] + c3[3];
#pragma unroll
  for (int i = 0; i < 48; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

// VALU only (same NV chains, no MFMA): cycles per group of 4*NV fmas
template <int NV>
__global__ void __launch_bounds__(512) kern_valu(float *out, long long *cyc, float a, float b) {
  float v[48];
#pragma unroll
  for (int i = 0; i < 48; ++i) v[i] = a * (threadIdx.x + i);
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < NV; ++i) v[12 * q + i] = __builtin_fmaf(v[12 * q + i], (q & 1) ? b : a, (q & 1) ? a : b);
  }
  long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 48; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int NV>
void run(float *out, long long *cyc, int waves_per_simd) {
  const int threads = 64 * 4 * waves_per_simd;  // one block per CU, 4 SIMDs
  long long h[32];
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kern<NV>, dim3(1), dim3(threads), 0, 0, out, cyc, 1.0001f, 0.9999f);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, cyc, sizeof(long long) * threads / 64, hipMemcpyDeviceToHost);
  long long mx = 0;
  for (int i = 0; i < threads / 64; ++i) mx = h[i] > mx ? h[i] : mx;
  double per_mfma = (double)mx / (ITER * 4.0);
  hipLaunchKernelGGL(kern_valu<NV>, dim3(1), dim3(threads), 0, 0, out, cyc, 1.0001f, 0.9999f);
  hipDeviceSynchronize();
  hipMemcpy(h, cyc, sizeof(long long) * threads / 64, hipMemcpyDeviceToHost);
  long long mv = 0;
  for (int i = 0; i < threads / 64; ++i) mv = h[i] > mv ? h[i] : mv;
  printf("waves/SIMD %d  NV %2d : %.1f cyc per (MFMA + %d fma) per wave; VALU-only %.1f cyc per %d fma\n",
         waves_per_simd, NV, per_mfma, NV, (double)mv / (ITER * 4.0), NV);
}

int main() {
  float *out;
  long long *cyc;
  hipMalloc(&out, 4096 * sizeof(float));
  hipMalloc(&cyc, 64 * sizeof(long long));
  for (int w = 1; w <= 2; ++w) {
    run<0>(out, cyc, w);
    run<2>(out, cyc, w);
    run<4>(out, cyc, w);
    run<6>(out, cyc, w);
    run<8>(out, cyc, w);
    run<12>(out, cyc, w);
  }
  return 0;
}
