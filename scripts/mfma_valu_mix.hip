// Microbenchmark: cost of v_fma_f32 work mixed with MFMAs in one wave, by placement.
// Per iteration: 4 MFMAs on independent accumulators and 48 independent v_fma_f32,
//   mode 0: VALU only (48 fma);  mode 1: MFMA only (4);
//   mode 2: interleaved, 12 fma after each MFMA;
//   mode 3: grouped, the 4 MFMAs back to back then the 48 fma
//           (sched_group_barrier pins the order);
// for v_mfma_f32_16x16x4_f32 and v_mfma_f32_16x16x32_bf16, 1 and 2 waves per SIMD.
// Cycles per iteration per wave from s_memtime.  Build with -fno-slp-vectorize (as the
// library): otherwise the FMAs are packed into v_pk_fma_f32.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
#define ITER 2000

template <bool BF, int MODE>
__global__ void __launch_bounds__(512) kern(float *out, long long *cyc, float a, float b) {
  f4 c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = f4{0.f, 0.f, 0.f, 0.f};
  bf8 A8, B8;
#pragma unroll
  for (int i = 0; i < 8; ++i) { A8[i] = (__bf16)(a + i); B8[i] = (__bf16)(b - i); }
  float v[48];
#pragma unroll
  for (int i = 0; i < 48; ++i) v[i] = a * (threadIdx.x + i);
  auto mf = [&](int q) __attribute__((always_inline)) {
    if (BF) c[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8, B8, c[q], 0, 0, 0);
    else c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[q], 0, 0, 0);
  };
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 48; ++i) v[i] = __builtin_fmaf(v[i], a, b);
    } else if (MODE == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) mf(q);
    } else if (MODE == 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        mf(q);
#pragma unroll
        for (int i = 0; i < 12; ++i) v[12 * q + i] = __builtin_fmaf(v[12 * q + i], a, b);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);  // then 12 VALU
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) mf(q);
#pragma unroll
      for (int i = 0; i < 48; ++i) v[i] = __builtin_fmaf(v[i], a, b);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);    // 4 MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 48, 0);   // then 48 VALU
    }
  }
  long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) s += c[q][q];
#pragma unroll
  for (int i = 0; i < 48; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <bool BF, int MODE>
double run(float *out, long long *cyc, int waves_per_simd) {
  const int threads = 64 * 4 * waves_per_simd;
  long long h[32];
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((kern<BF, MODE>), dim3(1), dim3(threads), 0, 0, out, cyc, 1.0001f, 0.9999f);
    (void)hipDeviceSynchronize();
  }
  (void)hipMemcpy(h, cyc, sizeof(long long) * threads / 64, hipMemcpyDeviceToHost);
  long long mx = 0;
  for (int i = 0; i < threads / 64; ++i) mx = h[i] > mx ? h[i] : mx;
  return (double)mx / ITER;
}

template <bool BF>
void table(float *out, long long *cyc, int w) {
  const double v = run<BF, 0>(out, cyc, w), m = run<BF, 1>(out, cyc, w);
  const double il = run<BF, 2>(out, cyc, w), gr = run<BF, 3>(out, cyc, w);
  printf("%s waves/SIMD %d: 48 fma %.1f | 4 MFMA %.1f | sum %.1f | interleaved %.1f | grouped %.1f\n",
         BF ? "bf16 16x16x32" : "f32 16x16x4  ", w, v, m, v + m, il, gr);
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 4096 * sizeof(float));
  (void)hipMalloc(&cyc, 64 * sizeof(long long));
  for (int w = 1; w <= 2; ++w) {
    table<false>(out, cyc, w);
    table<true>(out, cyc, w);
  }
  return 0;
}
