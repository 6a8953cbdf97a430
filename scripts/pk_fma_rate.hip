// Microbenchmark: issue cost of packed FP32 (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32,
// two floats per lane) against v_fma_f32, alone and between f32 MFMAs.  Each wave runs
// ITER iterations over 24 independent chains; cycles per instruction per wave from
// s_memtime, one block per CU at 1 and 2 waves per SIMD.  Build with -fno-slp-vectorize,
// or the scalar FMA case is packed as well.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define ITER 2000
#define NC 24

enum Op { FMA = 0, PK_FMA = 1, PK_ADD = 2, PK_MUL = 3 };

template <int OP, int WITH_MFMA>
__global__ void __launch_bounds__(512) kern(float *out, long long *cyc, float a, float b) {
  f2 v[NC];
  float s1[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    v[i] = f2{a * (threadIdx.x + i), b * (threadIdx.x - i)};
    s1[i] = a * (threadIdx.x + 2 * i);
  }
  const f2 A2 = {a, b}, B2 = {b, a};
  f4 c0 = {0, 0, 0, 0}, c1 = c0;
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
    if (WITH_MFMA) c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NC / 2; ++i) {
      if (OP == FMA) s1[i] = __builtin_fmaf(s1[i], a, b);
      if (OP == PK_FMA) v[i] = __builtin_elementwise_fma(v[i], A2, B2);
      if (OP == PK_ADD) v[i] = v[i] + A2;
      if (OP == PK_MUL) v[i] = v[i] * A2;
    }
    if (WITH_MFMA) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
#pragma unroll
    for (int i = NC / 2; i < NC; ++i) {
      if (OP == FMA) s1[i] = __builtin_fmaf(s1[i], b, a);
      if (OP == PK_FMA) v[i] = __builtin_elementwise_fma(v[i], B2, A2);
      if (OP == PK_ADD) v[i] = v[i] + B2;
      if (OP == PK_MUL) v[i] = v[i] * B2;
    }
  }
  long long t1 = __builtin_readcyclecounter();
  float s = c0[0] + c1[1];
#pragma unroll
  for (int i = 0; i < NC; ++i) s += v[i].x + v[i].y + s1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP, int M>
void run(float *out, long long *cyc, int waves_per_simd, const char *name) {
  const int threads = 64 * 4 * waves_per_simd;
  long long h[32];
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((kern<OP, M>), dim3(1), dim3(threads), 0, 0, out, cyc, 1.0001f, 0.9999f);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, cyc, sizeof(long long) * threads / 64, hipMemcpyDeviceToHost);
  long long mx = 0;
  for (int i = 0; i < threads / 64; ++i) mx = h[i] > mx ? h[i] : mx;
  const double per_iter = (double)mx / ITER;
  printf("waves/SIMD %d  %-7s %s: %.1f cyc per iteration (%d VALU%s) = %.2f cyc per VALU\n",
         waves_per_simd, name, M ? "+2 MFMA" : "       ", per_iter, NC, M ? " + 2 MFMA" : "",
         (per_iter - (M ? 64.0 : 0.0)) / NC);
}

int main() {
  float *out;
  long long *cyc;
  hipMalloc(&out, 4096 * sizeof(float));
  hipMalloc(&cyc, 64 * sizeof(long long));
  for (int w = 1; w <= 2; ++w) {
    run<FMA, 0>(out, cyc, w, "fma");
    run<PK_FMA, 0>(out, cyc, w, "pk_fma");
    run<PK_ADD, 0>(out, cyc, w, "pk_add");
    run<PK_MUL, 0>(out, cyc, w, "pk_mul");
    run<FMA, 1>(out, cyc, w, "fma");
    run<PK_FMA, 1>(out, cyc, w, "pk_fma");
    run<PK_ADD, 1>(out, cyc, w, "pk_add");
  }
  return 0;
}
