// LDS instruction cost microbenchmark for gfx950 (design data for sg_fast.hip).
// Each variant: 256 blocks x 512 threads, every wave issues ITERS x 8 LDS ops of
// one kind; reports ns per wave-instruction per CU (= LDS cycles/instr at clk).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 2048

template <int V>
__global__ void __launch_bounds__(512) kern(float *out, int salt) {
  __shared__ __attribute__((aligned(16))) float s[16384];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 16384; i += 512) s[i] = (float)(i ^ salt);
  __syncthreads();
  float acc = 0.f;
  float *ws = s + w * 2048;
  const int g = l >> 4, j = l & 15;
  for (int it = 0; it < ITERS; ++it) {
    const int o = (it * 8) & 255;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (V == 0) acc += ws[(o + l + u * 64) & 1023];                            // b32 per-lane
      if (V == 1) acc += ws[(o + u) & 1023];                                     // b32 broadcast
      if (V == 2) { float4 q = *(float4 *)&ws[((o + u * 4) * 4 + l * 4) & 1020];  // b128 per-lane
                    acc += q.x + q.w; }
      if (V == 3) { float4 q = *(float4 *)&ws[((o + u) * 4) & 1020];             // b128 broadcast
                    acc += q.x + q.w; }
      if (V == 4) ws[(o + l + u * 64) & 1023] = acc + u;                         // write b32
      if (V == 5) atomicAdd(&ws[(j + 16 * (u & 1) + 32 * g * (1 + (it & 3))) & 1023], 1.f);  // add, 4-way same bank
      if (V == 6) atomicAdd(&ws[(l + 64 * u) & 1023], 1.f);                      // add, distinct banks
      if (V == 7) acc += __shfl_xor(acc, 16, 64);                                // ds_bpermute
      if (V == 8) atomicAdd(&ws[(j + 16 * (u & 1) + 32 * (it % 29)) & 1023], 1.f);  // add, 4 lanes same addr
    }
    asm volatile("" ::: "memory");
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int V>
float run(float *d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kern<V>, dim3(256), dim3(512), 0, 0, d, 1);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern<V>, dim3(256), dim3(512), 0, 0, d, r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  // per CU: 8 waves x ITERS x 8 instructions per launch
  return ms * 1e6f / 5.f / (8.f * ITERS * 8.f);
}

int main() {
  float *d;
  hipMalloc(&d, 64);
  const char *names[] = {"b32 per-lane read", "b32 broadcast read", "b128 per-lane read",
                         "b128 broadcast read", "b32 write", "add_f32 4-way same-bank",
                         "add_f32 distinct banks", "bpermute (shfl_xor)", "add_f32 same-addr x4"};
  float t[9] = {run<0>(d), run<1>(d), run<2>(d), run<3>(d), run<4>(d), run<5>(d), run<6>(d),
                run<7>(d), run<8>(d)};
  for (int i = 0; i < 9; ++i) printf("%-26s %7.3f ns/instr/CU  (%5.1f cyc @2.4GHz)\n", names[i], t[i], t[i] * 2.4f);
  return 0;
}
