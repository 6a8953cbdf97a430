// sg_fast.hip — fused fwd(+bwd) kernel for the reference's default Siamese
// stack (config.py:44-66): GCN(d_in→32, relu, sparse one-hot) → GCN(32→16,
// identity) → Dense(16→1, relu) → Padding(D) → NTN(D, K=10, relu), every layer
// with bias and dropout, Gaussian final act, broadcast or aligned MSE.
//
// One wavefront owns one graph pair at a time.  The pair record is staged in
// LDS; each graph instance is one 16-row MFMA tile whose rows are the nodes.
// All seven GCN products (Â·Z0, D1·W1, Â·Z1 forward; Âᵀ·gH2, D1ᵀ·gZ1, gZ1·W1ᵀ,
// Âᵀ·gP1 backward) run on v_mfma_f32_16x16x4_f32 — exact f32, bit-for-bit a
// k-ordered fmaf chain.  Node n lives in tile row ρ(n) = 4·(n%4) + n/4, so the
// accumulator of one product (lane (g,j) holds rows 4g..4g+3) IS the B operand
// of the next Â product with the K index permuted (k-step κ ↔ rows 4g+κ), and
// rows 4g+3 are empty for n ≤ 12: Â products need 3 k-steps, not 4.  The
// feature-contracting products need one 16×32 / 16×16 transpose through LDS.
// The NTN head runs on VALU (D = K = 10 is too small for MFMA to pay), lanes
// (ag, k) = (l/10, l%10) own NTN weight rows a ∈ {ag, ag+6}.
// Parameter gradients accumulate in registers (gW1 in MFMA accumulators) and a
// per-wave LDS table (gW0 rows, scattered by node type), flushed once per
// launch, wave by wave, into one slab row per workgroup (deterministic).
#include "sg_plan.h"

int sg_num_cus();

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int FH1 = 32, FH2 = 16, FK = 10;
constexpr int TS1 = 36;  // D1 tile row stride (floats)
constexpr int TS2 = 20;  // gZ1 tile row stride

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}

// Sum over the 16 lanes of a DPP row; result in every lane of the row.
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

struct FastArgs {
  const uint8_t *recs;
  int64_t n_pairs;
  int64_t pair_offset;
  const float *params;
  const float *y_stats;
  float *s_out;
  float *slab;
  uint32_t key;
  uint32_t thr0, thr1, thr2, thr4;
  float ik0, ik1, ik2, ik4;
  float yeta;
  float inv_batch;
  int final_act, loss_mode, ntn_mode;
  int d_in, n_params;
  int shared_floats, wave_floats;
  int oW0, ob0, oW1, ob1, oWd, obd, oW, oV, oU, obn;
};

template <int D>
struct FastLds {
  static constexpr int RW = 2 * D * D + 2 * D + 4;  // record words (multiple of 4)
  static constexpr int REC = 0;
  static constexpr int TILE = REC + RW;               // 2 x 16 x TS1 (D1 / gZ1 tiles)
  static constexpr int X = TILE + 2 * 16 * TS1;       // x1[12] | x2[12]
  static constexpr int PM = X + 32;                   // NTN partial m [6][10]
  static constexpr int M = PM + 64;                   // m[10]
  static constexpr int G1 = M + 16;                   // ge1 partials [12][12]
  static constexpr int G2 = G1 + 144;                 // ge2 partials [12][12]
  static constexpr int GE = G2 + 144;                 // ge[2][12]
  static constexpr int GW0 = GE + 32;                 // gW0 accumulator [d_in][32]
  static int wave_floats(int d_in) { return (GW0 + d_in * FH1 + 3) & ~3; }
  static int shared_floats(int d_in) {
    return ((d_in * FH1 + 3) & ~3) + 2 * D * FK * 12 + FK * 24;
  }
};

template <int D, bool BWD>
__global__ void __launch_bounds__(512) sg_fast_kernel(FastArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using L = FastLds<D>;
  constexpr int RW4 = L::RW / 4;
  constexpr int NREC = (RW4 + 63) / 64;
  const int tid = threadIdx.x;
  const int l = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  const int g = l >> 4, j = l & 15;
  const int d_in = A.d_in;
  const float *__restrict__ prm = A.params;

  float *sW0 = smem;
  float *sWa = sW0 + ((d_in * FH1 + 3) & ~3);  // [a][k][12]: W[a][b][k] at b
  float *sWb = sWa + D * FK * 12;               // [b][k][12]: W[a][b][k] at a
  float *sV = sWb + D * FK * 12;                // [k][24]
  float *W = smem + A.shared_floats + wv * A.wave_floats;
  float *sRec = W + L::REC;
  float *sT = W + L::TILE;
  float *sX = W + L::X;
  float *sPM = W + L::PM;
  float *sM = W + L::M;
  float *sG1 = W + L::G1;
  float *sG2 = W + L::G2;
  float *sGE = W + L::GE;
  float *sGW0 = W + L::GW0;

  for (int i = tid; i < d_in * FH1; i += blockDim.x) sW0[i] = prm[A.oW0 + i];
  for (int i = tid; i < D * FK * 12; i += blockDim.x) {
    const int x = i / (FK * 12), rem = i - x * FK * 12, k = rem / 12, y = rem - k * 12;
    sWa[i] = y < D ? prm[A.oW + (x * D + y) * FK + k] : 0.f;
    sWb[i] = y < D ? prm[A.oW + (y * D + x) * FK + k] : 0.f;
  }
  for (int i = tid; i < FK * 24; i += blockDim.x) {
    const int k = i / 24, c = i - k * 24;
    sV[i] = c < 2 * D ? prm[A.oV + k * 2 * D + c] : 0.f;
  }
  for (int i = l; i < 2 * 16 * TS1; i += 64) sT[i] = 0.f;
  if (BWD)
    for (int i = l; i < d_in * FH1; i += 64) sGW0[i] = 0.f;
  __syncthreads();

  // ---- per-lane constants ----
  float w1b[8], w1t[2][4];
#pragma unroll
  for (int q = 0; q < 8; ++q) w1b[q] = prm[A.oW1 + (8 * g + q) * FH2 + j];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) w1t[t][q] = prm[A.oW1 + (16 * t + j) * FH2 + 4 * g + q];
  const float b0v[2] = {prm[A.ob0 + j], prm[A.ob0 + 16 + j]};
  const float b1v = prm[A.ob1 + j];
  const float wdv = prm[A.oWd + j];
  const float bd = prm[A.obd];
  float usum = 0.f;
#pragma unroll
  for (int k = 0; k < FK; ++k) usum += prm[A.oU + k];
  const bool nl = l < 60;             // NTN lane
  const int ag = nl ? l / 10 : 0, kk = nl ? l - ag * 10 : 0;
  const int a0 = ag, a1 = ag + 6;     // own NTN rows (a1 valid if < D)
  const float Uk = prm[A.oU + kk];
  const float bnk = prm[A.obn + (l < FK ? l : 0)];
  const bool ntn_ref = A.ntn_mode == SG_NTN_REFERENCE;
  // A-operand row of this lane: tile row i = j ↔ node ni
  const int ri = j & 3, ni = 4 * ri + (j >> 2);

  // ---- accumulators ----
  f4 gw1[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  float gb0a[2] = {0.f, 0.f}, gb1a = 0.f, gwda = 0.f, gbda = 0.f;
  float gWn[2][D];
#pragma unroll
  for (int b = 0; b < D; ++b) gWn[0][b] = gWn[1][b] = 0.f;
  float gVa[4] = {0.f, 0.f, 0.f, 0.f};
  float gbn = 0.f, gUa = 0.f, lossa = 0.f;
  const float ybar = (BWD && A.loss_mode == SG_LOSS_BROADCAST) ? A.y_stats[0] : 0.f;

  const int64_t stride = (int64_t)gridDim.x * nw;
  int64_t p = (int64_t)blockIdx.x * nw + wv;
  uint4 pre[NREC];
#pragma unroll
  for (int c = 0; c < NREC; ++c) {
    const int w4 = l + 64 * c;
    pre[c] = (p < A.n_pairs && w4 < RW4)
                 ? ((const uint4 *)(A.recs + (size_t)p * (L::RW * 4)))[w4]
                 : uint4{0u, 0u, 0u, 0u};
  }

  for (; p < A.n_pairs; p += stride) {
    sg_wsync();
#pragma unroll
    for (int c = 0; c < NREC; ++c) {
      const int w4 = l + 64 * c;
      if (w4 < RW4) ((uint4 *)sRec)[w4] = pre[c];
    }
    sg_wsync();
    {
      const int64_t pn = p + stride;
#pragma unroll
      for (int c = 0; c < NREC; ++c) {
        const int w4 = l + 64 * c;
        if (pn < A.n_pairs && w4 < RW4)
          pre[c] = ((const uint4 *)(A.recs + (size_t)pn * (L::RW * 4)))[w4];
      }
    }
    const int *ty = (const int *)(sRec + 2 * D * D);
    const int Nn[2] = {((const int *)sRec)[2 * D * D + 2 * D],
                       ((const int *)sRec)[2 * D * D + 2 * D + 1]};
    const float label = sRec[2 * D * D + 2 * D + 2];
    const uint32_t pk = sg_pair_key(A.key, (uint32_t)(A.pair_offset + p));

    // ================= forward =================
    float af[2][3];
    f4 d1[2][2];
    f4 zp2[2];            // zpre rows r<3 (r=3 unused)
    f4 d2[2];
    uint32_t bits[2];     // per instance: r*8 + t*4 + {0:keep0,1:keep1,2:pos1,3:keep2}
    int tyr[2][3];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int Ns = Nn[s];
      const float *As = sRec + s * D * D;
      const bool rowok = ri < 3 && ni < Ns;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int c = 4 * q + g;
        af[s][q] = (rowok && c < Ns) ? As[ni * D + c] : 0.f;
      }
      uint32_t bs = 0u;
      f4 z0[2];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int n = 4 * r + g;
        const bool vr = n < Ns;
        int t_ = vr ? ty[s * D + n] : 0;
        t_ = t_ < 0 ? 0 : (t_ >= d_in ? d_in - 1 : t_);
        tyr[s][r] = t_;
        const bool k0 = vr && sg_keep(pk, 0, s, n, A.thr0);
        bs |= (k0 ? 1u : 0u) << (r * 8);
        z0[0][r] = k0 ? sW0[t_ * FH1 + j] * A.ik0 : 0.f;
        z0[1][r] = k0 ? sW0[t_ * FH1 + 16 + j] * A.ik0 : 0.f;
      }
      z0[0][3] = z0[1][3] = 0.f;
      // P1 = Â Z0 + b0 ; H1 = relu ; D1 = dropout
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f4 acc;
#pragma unroll
        for (int r = 0; r < 3; ++r) acc[r] = (4 * r + g < Ns) ? b0v[t] : 0.f;
        acc[3] = 0.f;
#pragma unroll
        for (int q = 0; q < 3; ++q) acc = mfma4(af[s][q], z0[t][q], acc);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const int n = 4 * r + g;
          const bool vr = n < Ns;
          const float v = acc[r];
          const bool pos = vr && v > 0.f;
          const bool k1 = vr && sg_keep(pk, 1, s, n * FH1 + 16 * t + j, A.thr1);
          d1[s][t][r] = (pos && k1) ? v * A.ik1 : 0.f;
          bs |= ((k1 ? 2u : 0u) | (pos ? 4u : 0u)) << (r * 8 + t * 4);
        }
        d1[s][t][3] = 0.f;
      }
      bits[s] = bs;
      float *T = sT + s * 16 * TS1;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(4 * g + r) * TS1 + 16 * t + j] = d1[s][t][r];
    }
    sg_wsync();
    // Z1 = D1 W1 ; H2 = Â Z1 + b1 ; D2 ; zpre = D2 Wd + bd
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int Ns = Nn[s];
      const float *T = sT + s * 16 * TS1 + j * TS1 + 8 * g;
      const f4 lo = *(const f4 *)T, hi = *(const f4 *)(T + 4);
      f4 z1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) z1 = mfma4(lo[q], w1b[q], z1);
#pragma unroll
      for (int q = 0; q < 4; ++q) z1 = mfma4(hi[q], w1b[4 + q], z1);
      f4 h2;
#pragma unroll
      for (int r = 0; r < 3; ++r) h2[r] = (4 * r + g < Ns) ? b1v : 0.f;
      h2[3] = 0.f;
#pragma unroll
      for (int q = 0; q < 3; ++q) h2 = mfma4(af[s][q], z1[q], h2);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int n = 4 * r + g;
        const bool k2 = n < Ns && sg_keep(pk, 2, s, n * FH2 + j, A.thr2);
        d2[s][r] = k2 ? h2[r] * A.ik2 : 0.f;
        bits[s] |= (k2 ? 8u : 0u) << (r * 8);
        zp2[s][r] = row_sum16(d2[s][r] * wdv) + bd;
      }
      d2[s][3] = 0.f;
      // e = relu(zpre) for real nodes, 0-padded to D (Padding, layers.py:223-227);
      // NTN input dropout (layers.py:287-288)
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int n = 4 * r + g;
        const float e = (n < Ns && zp2[s][r] > 0.f) ? zp2[s][r] : 0.f;
        if (j == 0 && n < D) sX[s * 12 + n] = sg_keep(pk, 4, s, n, A.thr4) ? e * A.ik4 : 0.f;
      }
    }
    sg_wsync();

    // ================= NTN head (layers.py:282-310) =================
    float x1[D], x2[D];
#pragma unroll
    for (int b = 0; b < D; ++b) {
      x1[b] = sX[b];
      x2[b] = sX[12 + b];
    }
    float u0 = 0.f, u1 = 0.f, xv[4] = {0.f, 0.f, 0.f, 0.f}, x1a0 = 0.f, x1a1 = 0.f;
    if (nl) {
      const float *wa0 = sWa + (a0 * FK + kk) * 12;
#pragma unroll
      for (int b = 0; b < D; ++b) u0 = fmaf(wa0[b], x2[b], u0);
      x1a0 = sX[a0];
      float part = x1a0 * u0;
      if (a1 < D) {
        const float *wa1 = sWa + (a1 * FK + kk) * 12;
#pragma unroll
        for (int b = 0; b < D; ++b) u1 = fmaf(wa1[b], x2[b], u1);
        x1a1 = sX[a1];
        part = fmaf(x1a1, u1, part);
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = 4 * ag + ii;
        if (i < 2 * D) {
          xv[ii] = sX[i < D ? i : 12 + i - D];
          part = fmaf(sV[kk * 24 + i], xv[ii], part);
        }
      }
      sPM[ag * 10 + kk] = part;
    }
    sg_wsync();
    if (l < FK) {
      float m = bnk;
#pragma unroll
      for (int q = 0; q < 6; ++q) m += sPM[q * 10 + l];
      sM[l] = m;
    }
    sg_wsync();
    float rsum = 0.f, sdot = 0.f;
#pragma unroll
    for (int k = 0; k < FK; ++k) {
      const float mk = sM[k];
      const float rk = mk > 0.f ? mk : 0.f;
      rsum += rk;
      sdot = fmaf(prm[A.oU + k], rk, sdot);
    }
    const float sv = ntn_ref ? usum * rsum : sdot;
    if (!BWD) {
      if (l == 0) A.s_out[p] = sv;
      continue;
    }
    if (A.s_out && l == 0) A.s_out[p] = sv;
    const float yhat = sg_final(A.final_act, A.yeta, sv);
    float gy;
    if (A.loss_mode == SG_LOSS_BROADCAST) {
      gy = yhat - ybar;
      lossa += 0.5f * gy * gy;
    } else {
      const float dl = yhat - label;
      gy = dl * A.inv_batch;
      lossa += 0.5f * dl * dl * A.inv_batch;
    }
    const float gs = gy * sg_final_grad(A.final_act, A.yeta, sv, yhat);

    // ================= NTN backward =================
    if (nl) {
      const float mk = sM[kk];
      const float gr = ntn_ref ? gs * usum : gs * Uk;
      const float gmk = mk > 0.f ? gr : 0.f;
      if (ag == 0) {
        gbn += gmk;
        gUa += ntn_ref ? gs * rsum : gs * (mk > 0.f ? mk : 0.f);
      }
      const float c0 = gmk * x1a0, c1 = gmk * x1a1;
#pragma unroll
      for (int b = 0; b < D; ++b) {
        gWn[0][b] = fmaf(c0, x2[b], gWn[0][b]);
        gWn[1][b] = fmaf(c1, x2[b], gWn[1][b]);
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) gVa[ii] = fmaf(gmk, xv[ii], gVa[ii]);
      sG1[a0 * 12 + kk] = gmk * (sV[kk * 24 + a0] + u0);
      if (a1 < D) sG1[a1 * 12 + kk] = gmk * (sV[kk * 24 + a1] + u1);
      {
        const float *wb = sWb + (a0 * FK + kk) * 12;   // b0 = ag
        float w = 0.f;
#pragma unroll
        for (int a = 0; a < D; ++a) w = fmaf(x1[a], wb[a], w);
        sG2[a0 * 12 + kk] = gmk * (w + sV[kk * 24 + D + a0]);
      }
      if (a1 < D) {
        const float *wb = sWb + (a1 * FK + kk) * 12;   // b1 = ag + 6
        float w = 0.f;
#pragma unroll
        for (int a = 0; a < D; ++a) w = fmaf(x1[a], wb[a], w);
        sG2[a1 * 12 + kk] = gmk * (w + sV[kk * 24 + D + a1]);
      }
    }
    sg_wsync();
    if (l < 24) {
      const int s = l / 12, q = l - s * 12;
      if (q < D) {
        const float *row = (s ? sG2 : sG1) + q * 12;
        float gx = 0.f;
#pragma unroll
        for (int k = 0; k < FK; ++k) gx += row[k];
        sGE[s * 12 + q] = sg_keep(pk, 4, s, q, A.thr4) ? gx * A.ik4 : 0.f;
      }
    }
    sg_wsync();

    // ================= GCN backward =================
    f4 gz1[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int Ns = Nn[s];
      f4 gh2;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int n = 4 * r + g;
        const float ge = n < D ? sGE[s * 12 + n] : 0.f;
        const float gp = (n < Ns && zp2[s][r] > 0.f) ? ge : 0.f;  // Dense relu'
        gwda = fmaf(d2[s][r], gp, gwda);
        if (j == 0) gbda += gp;
        const float v = ((bits[s] >> (r * 8)) & 8u) ? gp * wdv * A.ik2 : 0.f;
        gb1a += v;
        gh2[r] = v;
      }
      gh2[3] = 0.f;
      f4 z = {0.f, 0.f, 0.f, 0.f};  // gZ1 = Âᵀ gH2  (Â symmetric, checked at pack time)
#pragma unroll
      for (int q = 0; q < 3; ++q) z = mfma4(af[s][q], gh2[q], z);
      gz1[s] = z;
#pragma unroll
      for (int t = 0; t < 2; ++t)    // gW1 += D1ᵀ gZ1
#pragma unroll
        for (int q = 0; q < 3; ++q) gw1[t] = mfma4(d1[s][t][q], z[q], gw1[t]);
      float *T = sT + s * 16 * TS1;
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(4 * g + r) * TS2 + j] = z[r];
    }
    sg_wsync();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int Ns = Nn[s];
      const f4 ga = *(const f4 *)(sT + s * 16 * TS1 + j * TS2 + 4 * g);
      const uint32_t bs = bits[s];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f4 gd = {0.f, 0.f, 0.f, 0.f};  // gD1 = gZ1 W1ᵀ
#pragma unroll
        for (int q = 0; q < 4; ++q) gd = mfma4(ga[q], w1t[t][q], gd);
        f4 gp1;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const uint32_t b = bs >> (r * 8 + t * 4);
          const float v = ((b & 6u) == 6u) ? gd[r] * A.ik1 : 0.f;  // keep1 && pos
          gb0a[t] += v;
          gp1[r] = v;
        }
        gp1[3] = 0.f;
        f4 gz0 = {0.f, 0.f, 0.f, 0.f};  // gZ0 = Âᵀ gP1
#pragma unroll
        for (int q = 0; q < 3; ++q) gz0 = mfma4(af[s][q], gp1[q], gz0);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          if (((bs >> (r * 8)) & 1u) && (4 * r + g) < Ns)
            atomicAdd(&sGW0[tyr[s][r] * FH1 + 16 * t + j], gz0[r] * A.ik0);
        }
      }
    }
  }

  if (!BWD) return;
  // ---- flush: one wave at a time into the workgroup slab row (deterministic) ----
  __syncthreads();
  float *G = smem;  // the weight tables are dead now
  for (int i = tid; i <= A.n_params; i += blockDim.x) G[i] = 0.f;
  __syncthreads();
  for (int w = 0; w < nw; ++w) {
    if (wv == w) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) G[A.oW1 + (16 * t + 4 * g + r) * FH2 + j] += gw1[t][r];
      }
      sg_wsync();
#pragma unroll
      for (int t = 0; t < 2; ++t) atomicAdd(&G[A.ob0 + 16 * t + j], gb0a[t]);
      atomicAdd(&G[A.ob1 + j], gb1a);
      atomicAdd(&G[A.oWd + j], gwda);
      atomicAdd(&G[A.obd], gbda);
      if (nl) {
#pragma unroll
        for (int b = 0; b < D; ++b) {
          G[A.oW + (a0 * D + b) * FK + kk] += gWn[0][b];
          if (a1 < D) G[A.oW + (a1 * D + b) * FK + kk] += gWn[1][b];
        }
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int i = 4 * ag + ii;
          if (i < 2 * D) G[A.oV + kk * 2 * D + i] += gVa[ii];
        }
        if (ag == 0) {
          G[A.obn + kk] += gbn;
          G[A.oU + kk] += gUa;
        }
      }
      for (int i = l; i < d_in * FH1; i += 64) G[A.oW0 + i] += sGW0[i];
      if (l == 0) G[A.n_params] += lossa;
    }
    __syncthreads();
  }
  float *dst = A.slab + (size_t)blockIdx.x * (size_t)(A.n_params + 1);
  for (int i = tid; i <= A.n_params; i += blockDim.x) dst[i] = G[i];
}

struct FastCfg {
  int D;
  int waves;
  int blocks;
  size_t lds;
  int shared_floats, wave_floats;
};

template <int D>
FastCfg fast_cfg_t(int d_in, int64_t n_pairs) {
  FastCfg c;
  c.D = D;
  c.shared_floats = FastLds<D>::shared_floats(d_in);
  c.wave_floats = FastLds<D>::wave_floats(d_in);
  // pick waves/block maximising resident waves per CU under 160 KiB of LDS
  int best = 1, best_res = 0;
  const char *ev = getenv("SG_FAST_WAVES");
  const int force = ev ? atoi(ev) : 0;
  for (int nw = 1; nw <= 8; ++nw) {
    if (force > 0 && nw != force) continue;
    const size_t lds = (size_t)(c.shared_floats + nw * c.wave_floats) * 4u;
    if (lds > 163840u) break;
    int per_cu = (int)(163840u / lds);
    int res = per_cu * nw;
    if (res > 8) res = 8;  // register-limited occupancy (2 waves/SIMD at 250 VGPRs)
    if (res > best_res || (res == best_res && nw > best)) {
      best = nw;
      best_res = res;
    }
  }
  c.waves = best;
  c.lds = (size_t)(c.shared_floats + best * c.wave_floats) * 4u;
  const int per_cu = (int)(163840u / c.lds);
  const int64_t want = (n_pairs + best - 1) / best;
  const int64_t cap = (int64_t)sg_num_cus() * per_cu;
  c.blocks = (int)(want < cap ? (want > 0 ? want : 1) : cap);
  return c;
}

}  // namespace

// --------------------------------------------------------------------------
static bool fast_shape(const sg_model_t *m, const SgGenPlan &P) {
  if (m->num_layers != 5) return false;
  const sg_layer_t *Ly = m->layers;
  if (Ly[0].kind != SG_GCN || !Ly[0].sparse_inputs || Ly[0].output_dim != FH1 ||
      Ly[0].act != SG_ACT_RELU || !Ly[0].bias)
    return false;
  if (Ly[1].kind != SG_GCN || Ly[1].input_dim != FH1 || Ly[1].output_dim != FH2 ||
      Ly[1].act != SG_ACT_IDENTITY || !Ly[1].bias)
    return false;
  if (Ly[2].kind != SG_DENSE || Ly[2].input_dim != FH2 || Ly[2].output_dim != 1 ||
      Ly[2].act != SG_ACT_RELU || !Ly[2].bias)
    return false;
  if (Ly[3].kind != SG_PADDING || Ly[3].padding_value != 0.f) return false;
  const int D = Ly[3].output_dim;
  if (Ly[4].kind != SG_NTN || Ly[4].input_dim != D || Ly[4].output_dim != FK ||
      Ly[4].act != SG_ACT_RELU || !Ly[4].bias)
    return false;
  if (m->n_max != D || D > 12 || D < 4) return false;
  if (m->d_in > 64) return false;
  return P.n_params > 0;
}

int sg_fast_supported(const sg_model_t *m, const SgGenPlan &P) {
  if (getenv("SG_DISABLE_FAST")) return 0;
  return fast_shape(m, P) ? 1 : 0;
}

static FastCfg fast_cfg(int D, int d_in, int64_t n_pairs) {
  switch (D) {
    case 4: return fast_cfg_t<4>(d_in, n_pairs);
    case 5: return fast_cfg_t<5>(d_in, n_pairs);
    case 6: return fast_cfg_t<6>(d_in, n_pairs);
    case 7: return fast_cfg_t<7>(d_in, n_pairs);
    case 8: return fast_cfg_t<8>(d_in, n_pairs);
    case 9: return fast_cfg_t<9>(d_in, n_pairs);
    case 10: return fast_cfg_t<10>(d_in, n_pairs);
    case 11: return fast_cfg_t<11>(d_in, n_pairs);
    default: return fast_cfg_t<12>(d_in, n_pairs);
  }
}

int64_t sg_fast_slab_floats(const SgGenPlan &P, int64_t n_pairs) {
  FastCfg c = fast_cfg(P.n_max, P.d_in, n_pairs);
  return (int64_t)c.blocks * (P.n_params + 1);
}

template <int D>
static void launch_fast(const FastCfg &c, bool bwd, const FastArgs &A, hipStream_t st) {
  if (bwd) {
    if (c.lds > 65536u)
      hipFuncSetAttribute((const void *)sg_fast_kernel<D, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds);
    hipLaunchKernelGGL((sg_fast_kernel<D, true>), dim3(c.blocks), dim3(64 * c.waves), c.lds, st, A);
  } else {
    if (c.lds > 65536u)
      hipFuncSetAttribute((const void *)sg_fast_kernel<D, false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds);
    hipLaunchKernelGGL((sg_fast_kernel<D, false>), dim3(c.blocks), dim3(64 * c.waves), c.lds, st,
                       A);
  }
}

int sg_fast_run(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                int64_t n_pairs, int64_t pair_offset, int64_t batch_total, const float *params,
                uint64_t seed, const float *y_stats, float *s_out, float *slab, int *blocks_out,
                hipStream_t stream) {
  const int D = P.n_max;
  FastCfg c = fast_cfg(D, P.d_in, n_pairs);
  FastArgs A;
  A.recs = (const uint8_t *)recs;
  A.n_pairs = n_pairs;
  A.pair_offset = pair_offset;
  A.params = params;
  A.y_stats = y_stats;
  A.s_out = s_out;
  A.slab = slab;
  A.key = sg_seed_key(seed);
  const float keep = m->keep_prob;
  const float k0 = m->layers[0].dropout ? keep : 1.f, k1 = m->layers[1].dropout ? keep : 1.f;
  const float k2 = m->layers[2].dropout ? keep : 1.f, k4 = m->layers[4].dropout ? keep : 1.f;
  A.thr0 = sg_keep_threshold(k0);
  A.thr1 = sg_keep_threshold(k1);
  A.thr2 = sg_keep_threshold(k2);
  A.thr4 = sg_keep_threshold(k4);
  A.ik0 = 1.f / k0;
  A.ik1 = 1.f / k1;
  A.ik2 = 1.f / k2;
  A.ik4 = 1.f / k4;
  A.yeta = m->yeta;
  A.inv_batch = batch_total > 0 ? 1.f / (float)batch_total : 0.f;
  A.final_act = m->final_act;
  A.loss_mode = m->loss_mode;
  A.ntn_mode = m->ntn_mode;
  A.d_in = P.d_in;
  A.n_params = P.n_params;
  A.shared_floats = c.shared_floats;
  A.wave_floats = c.wave_floats;
  A.oW0 = P.L[0].offW;
  A.ob0 = P.L[0].offB;
  A.oW1 = P.L[1].offW;
  A.ob1 = P.L[1].offB;
  A.oWd = P.L[2].offW;
  A.obd = P.L[2].offB;
  A.oW = P.offW;
  A.oV = P.offV;
  A.oU = P.offU;
  A.obn = P.offB;
  // the flush reuses the shared weight tables as the slab-row buffer
  if ((size_t)c.shared_floats < (size_t)P.n_params + 1) return SG_ERR_UNSUPPORTED;
  switch (D) {
    case 4: launch_fast<4>(c, bwd, A, stream); break;
    case 5: launch_fast<5>(c, bwd, A, stream); break;
    case 6: launch_fast<6>(c, bwd, A, stream); break;
    case 7: launch_fast<7>(c, bwd, A, stream); break;
    case 8: launch_fast<8>(c, bwd, A, stream); break;
    case 9: launch_fast<9>(c, bwd, A, stream); break;
    case 10: launch_fast<10>(c, bwd, A, stream); break;
    case 11: launch_fast<11>(c, bwd, A, stream); break;
    default: launch_fast<12>(c, bwd, A, stream); break;
  }
  if (blocks_out) *blocks_out = c.blocks;
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}
