// Layout probe for v_mfma_f32_4x4x1_16b_f32: A = lane id + 1 (as the lane's A value),
// B = 1000 * (lane id + 1); one MFMA on a zero accumulator.  Output reg r of lane l holds
// A[lane a] * B[lane b] for the lanes (a, b) the hardware pairs there: printed as
// (a, b) = (v mod 1000 ..., v / 1000 ...) after factoring.  Used to fix the block / row /
// column map the fused kernel's Â·Z0 product relies on.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_4x4_layout scripts/mfma_4x4_layout.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void kern(float *out) {
  const int l = threadIdx.x;
  // A value encodes the A lane, B value the B lane: a product (la+1) * 1000 (lb+1) is
  // unique and factorable since la + 1 <= 64 < 1000
  const float a = (float)(l + 1), b = 1000.f * (float)(l + 1);
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

int main() {
  float *d, h[256];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int ok = 1;
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int r = 0; r < 4; ++r) {
      const double v = h[l * 4 + r];
      // find la, lb with (la+1) * 1000 (lb+1) == v
      int fa = -1, fb = -1;
      for (int la = 0; la < 64 && fa < 0; ++la)
        for (int lb = 0; lb < 64; ++lb)
          if ((double)(la + 1) * 1000.0 * (double)(lb + 1) == v) { fa = la; fb = lb; break; }
      printf(" r%d=(A%2d,B%2d)", r, fa, fb);
      // hypothesis: block = l / 4, col j = l % 4, row i = r: A lane 4 block + i, B lane l
      if (fa != 4 * (l / 4) + r || fb != l) ok = 0;
    }
    printf("\n");
  }
  printf("hypothesis (D_b[i][j] at lane 4b + j, reg i; A_b[i] at lane 4b + i; B_b[j] at lane 4b + j): %s\n",
         ok ? "HOLDS" : "FAILS");
  hipFree(d);
  return 0;
}
