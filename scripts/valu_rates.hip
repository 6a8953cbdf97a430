// Microbenchmark: issue cost per wave instruction of the VALU classes the fused kernel
// uses (24 independent chains per wave, ITER iterations; s_memtime cycles, one block per
// CU at 1 and 2 waves per SIMD).  The ISA of each loop body is checked by counting
// opcodes in the device assembly.  Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize
// -fno-unroll-loops (each loop body is then exactly 24 of the measured instruction).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ITER 2000
#define NC 24

enum Op { FMA, FMA_DEP, ADD_DPP, XOR, MUL_U24, CNDMASK, CVT_PK_BF16, PERMLANE16, EXP, NOPS };
static const char *kName[NOPS] = {"v_fma_f32", "v_fma_f32 (1 chain)", "v_add_f32_dpp",
                                  "v_xor_b32", "v_mul_u32_u24", "v_cndmask_b32",
                                  "v_cvt_pk_bf16_f32", "v_permlane16_swap", "v_exp_f32"};

template <int N>
__device__ __forceinline__ float dpp_b1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), N, 0xF,
                                                            0xF, true));
}

template <int OP>
__global__ void __launch_bounds__(512) kern(float *out, long long *cyc, float a, float b,
                                            uint32_t ka) {
  float v[NC], w[NC];
  uint32_t u[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    v[i] = a * (threadIdx.x + i);
    w[i] = b * (threadIdx.x + 2 * i);
    u[i] = threadIdx.x * 2654435761u + i;
  }
  float dep = a * threadIdx.x;
  bool c[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) c[i] = (threadIdx.x >> (i % 6)) & 1;
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
    if (OP == FMA_DEP) {
#pragma unroll
      for (int i = 0; i < NC; ++i) dep = __builtin_fmaf(dep, a, b);
    }
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      if (OP == FMA) v[i] = __builtin_fmaf(v[i], a, b);
      if (OP == ADD_DPP) v[i] = v[i] + dpp_b1<0xB1>(w[i]);
      if (OP == XOR) u[i] ^= u[(i + 1) % NC];
      if (OP == MUL_U24) u[i] = __umul24(u[i], ka);
      if (OP == CNDMASK) v[i] = c[i] ? -v[i] : w[i];
      if (OP == CVT_PK_BF16) {
        typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
        const bf2 p = {(__bf16)__uint_as_float(u[i]), (__bf16)w[i]};
        u[i] = __builtin_bit_cast(uint32_t, p);
      }
      if (OP == PERMLANE16) {
        const auto r = __builtin_amdgcn_permlane16_swap(u[i], u[(i + 1) % NC], false, false);
        u[i] = r[0];
        u[(i + 1) % NC] = r[1];
      }
      if (OP == EXP) v[i] = __builtin_amdgcn_exp2f(v[i]);
    }
  }
  long long t1 = __builtin_readcyclecounter();
  float s = dep;
#pragma unroll
  for (int i = 0; i < NC; ++i) s += v[i] + w[i] + (float)u[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(float *out, long long *cyc) {
  printf("%-22s", kName[OP]);
  for (int w = 1; w <= 2; ++w) {
    const int threads = 64 * 4 * w;
    long long h[32];
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 0, 0, out, cyc, 1.0001f, 0.9999f,
                         0x9E3779B9u);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, cyc, sizeof(long long) * threads / 64, hipMemcpyDeviceToHost);
    long long mx = 0;
    for (int i = 0; i < threads / 64; ++i) mx = h[i] > mx ? h[i] : mx;
    printf("  %d wave/SIMD: %5.2f cyc per instr per wave (%5.2f per SIMD)", w,
           (double)mx / ITER / NC, (double)mx / ITER / NC / w);
  }
  printf("\n");
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 4096 * sizeof(float));
  (void)hipMalloc(&cyc, 64 * sizeof(long long));
  run<FMA>(out, cyc);
  run<FMA_DEP>(out, cyc);
  run<ADD_DPP>(out, cyc);
  run<XOR>(out, cyc);
  run<MUL_U24>(out, cyc);
  run<CNDMASK>(out, cyc);
  run<CVT_PK_BF16>(out, cyc);
  run<PERMLANE16>(out, cyc);
  run<EXP>(out, cyc);
  return 0;
}
