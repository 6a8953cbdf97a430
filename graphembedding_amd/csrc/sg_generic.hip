// sg_generic.hip — generic Siamese fwd(+bwd) kernel: one wavefront owns one
// graph pair; the pair record, every activation and every gradient tensor of
// the pair live in the wave's LDS slice; lanes sweep each op element-wise.
// Covers every layer stack sg_build_plan accepts (GCN/Dense/Padding/Average/
// Attention → NTN/Dot), all activations, both NTN modes and both loss modes.
// The default AIDS stack has a fused register/MFMA kernel (sg_fast.hip); this
// one is its general fallback and its on-GPU cross-check.
//
// Reference math: layers.py:91-118 (GCN), 136-140 (Average), 154-160
// (Attention), 192-205 (Dense), 223-227 (Padding), 249-252 (Dot), 282-310
// (NTN), 332-338 (sparse dropout); models.py:39-88; model_mse.py:117-151.
#include "sg_plan.h"

namespace {

struct GenArgs {
  const uint8_t *recs;
  const int32_t *order;   // processing order (sg_pair_order) or null
  int64_t n_pairs;
  int64_t pair_offset;
  float inv_batch;      // 1/B for the aligned loss
  const float *params;
  uint32_t key;
  const float *y_stats; // {ybar, ½Σ(y-ȳ)²}
  float *s_out;
  float *slab;          // [gridDim.x][n_params + 1]
};

__device__ __forceinline__ int rows_of(int fixed, int n) { return fixed < 0 ? n : fixed; }

// ---------------------------------------------------------------------------
// Forward of the node-level stack for both graphs of the pair at once.
// Tensors are [2][R][d] row-major; rows >= rows_s are zero.
// ---------------------------------------------------------------------------
__device__ void gen_forward_nodes(const SgGenPlan &P, float *S, const float *__restrict__ prm,
                                  const float *adj, const int *types, int n0, int n1,
                                  uint32_t pk, int lane) {
  const int nmax = P.n_max;
  for (int l = 0; l < P.nl; ++l) {
    const SgGenLayer &L = P.L[l];
    const int r0 = rows_of(L.rin_fixed, n0), r1 = rows_of(L.rin_fixed, n1);
    const float *x = L.l_in >= 0 ? S + L.l_in : nullptr;
    float *out = S + L.l_out;
    if (L.kind == SG_GCN || L.kind == SG_DENSE) {
      float *xd = S + L.l_xd;
      float *pre = S + L.l_pre;
      float *tmp = S + P.l_tmp;
      const int din = L.din, dout = L.dout, R = L.Rin;
      // (1) dropout of the input (layers.py:97-100, 196)
      if (L.sparse) {
        for (int e = lane; e < 2 * nmax; e += SG_WAVE) {
          const int s = e / nmax, n = e - s * nmax;
          const int rs = s ? r1 : r0;
          xd[e] = (n < rs && sg_keep(pk, L.li, s, n, L.thr)) ? L.inv_keep : 0.f;
        }
      } else {
        for (int e = lane; e < 2 * R * din; e += SG_WAVE) {
          const int s = e / (R * din), rem = e - s * R * din, r = rem / din;
          const int rs = s ? r1 : r0;
          float v = 0.f;
          if (r < rs && sg_keep(pk, L.li, s, rem, L.thr)) v = x[e] * L.inv_keep;
          xd[e] = v;
        }
      }
      sg_wsync();
      // (2) xd · W  (row gather of W for the one-hot X, layers.py:106-107)
      float *dst = (L.kind == SG_GCN) ? tmp : pre;
      for (int e = lane; e < 2 * R * dout; e += SG_WAVE) {
        const int s = e / (R * dout), rem = e - s * R * dout, r = rem / dout, j = rem - r * dout;
        const int rs = s ? r1 : r0;
        float acc = 0.f;
        if (r < rs) {
          if (L.sparse) {
            int t = types[s * nmax + r];
            t = t < 0 ? 0 : (t >= din ? din - 1 : t);
            acc = xd[s * nmax + r] * prm[L.offW + t * dout + j];
          } else {
            const float *xr = xd + (s * R + r) * din;
            for (int i = 0; i < din; ++i) acc = fmaf(xr[i], prm[L.offW + i * dout + j], acc);
          }
          if (L.kind == SG_DENSE && L.bias) acc += prm[L.offB + j];
        }
        dst[e] = acc;
      }
      sg_wsync();
      // (3) GCN: Â · (xd W) + b  (layers.py:110-116)
      if (L.kind == SG_GCN) {
        for (int e = lane; e < 2 * R * dout; e += SG_WAVE) {
          const int s = e / (R * dout), rem = e - s * R * dout, n = rem / dout, j = rem - n * dout;
          const int rs = s ? r1 : r0;
          float acc = 0.f;
          if (n < rs) {
            const float *ar = adj + (s * nmax + n) * nmax;
            const float *tc = tmp + s * R * dout + j;
            for (int m = 0; m < rs; ++m) acc = fmaf(ar[m], tc[m * dout], acc);
            if (L.bias) acc += prm[L.offB + j];
          }
          pre[e] = acc;
        }
        sg_wsync();
      }
      for (int e = lane; e < 2 * R * dout; e += SG_WAVE) {
        const int s = e / (R * dout), r = (e - s * R * dout) / dout;
        const int rs = s ? r1 : r0;
        out[e] = r < rs ? sg_act(L.act, pre[e]) : 0.f;
      }
      sg_wsync();
    } else if (L.kind == SG_PADDING) {
      const int d = L.din, Pr = L.Rout, Rin = L.Rin;
      for (int e = lane; e < 2 * Pr * d; e += SG_WAVE) {
        const int s = e / (Pr * d), rem = e - s * Pr * d, r = rem / d, c = rem - r * d;
        const int rs = s ? r1 : r0;
        out[e] = (r < rs && r < Rin) ? x[(s * Rin + r) * d + c] : L.padv;
      }
      sg_wsync();
    } else if (L.kind == SG_AVERAGE) {
      const int d = L.din, Rin = L.Rin;
      for (int e = lane; e < 2 * d; e += SG_WAVE) {
        const int s = e / d, c = e - s * d;
        const int rs = s ? r1 : r0;
        float acc = 0.f;
        for (int r = 0; r < rs; ++r) acc += x[(s * Rin + r) * d + c];
        out[e] = acc / (float)rs;
      }
      sg_wsync();
    } else {  // SG_ATTENTION (layers.py:154-160)
      const int d = L.din, Rin = L.Rin;
      float *temp = S + L.l_temp, *hv = S + L.l_hv, *att = S + L.l_att;
      for (int e = lane; e < 2 * d; e += SG_WAVE) {
        const int s = e / d, c = e - s * d;
        const int rs = s ? r1 : r0;
        float acc = 0.f;
        for (int r = 0; r < rs; ++r) acc += x[(s * Rin + r) * d + c];
        temp[e] = acc / (float)rs;
      }
      sg_wsync();
      for (int e = lane; e < 2 * d; e += SG_WAVE) {
        const int s = e / d, c = e - s * d;
        float acc = 0.f;
        for (int i = 0; i < d; ++i) acc = fmaf(temp[s * d + i], prm[L.offW + i * d + c], acc);
        hv[e] = tanhf(acc);
      }
      sg_wsync();
      for (int e = lane; e < 2 * Rin; e += SG_WAVE) {
        const int s = e / Rin, r = e - s * Rin;
        const int rs = s ? r1 : r0;
        float v = 0.f;
        if (r < rs) {
          float acc = 0.f;
          for (int c = 0; c < d; ++c) acc = fmaf(x[(s * Rin + r) * d + c], hv[s * d + c], acc);
          v = 1.f / (1.f + expf(-acc));
        }
        att[e] = v;
      }
      sg_wsync();
      for (int e = lane; e < 2 * d; e += SG_WAVE) {
        const int s = e / d, c = e - s * d;
        const int rs = s ? r1 : r0;
        float acc = 0.f;
        for (int r = 0; r < rs; ++r) acc = fmaf(att[s * Rin + r], x[(s * Rin + r) * d + c], acc);
        out[e] = acc;
      }
      sg_wsync();
    }
  }
}

// ---------------------------------------------------------------------------
// Backward of the node-level stack; gin = gradient of the last layer's output.
// Parameter gradients go to the workgroup accumulator G with LDS atomics.
// ---------------------------------------------------------------------------
__device__ void gen_backward_nodes(const SgGenPlan &P, float *S, float *G,
                                   const float *__restrict__ prm, const float *adj,
                                   const int *types, int n0, int n1, uint32_t pk, int lane,
                                   float *gcur, float *gnext) {
  const int nmax = P.n_max;
  for (int l = P.nl - 1; l >= 0; --l) {
    const SgGenLayer &L = P.L[l];
    const int r0 = rows_of(L.rin_fixed, n0), r1 = rows_of(L.rin_fixed, n1);
    const float *x = L.l_in >= 0 ? S + L.l_in : nullptr;
    if (L.kind == SG_GCN || L.kind == SG_DENSE) {
      const int din = L.din, dout = L.dout, R = L.Rin;
      const float *xd = S + L.l_xd, *pre = S + L.l_pre, *out = S + L.l_out;
      float *gpre = S + P.l_tmp;
      float *gsup = S + P.l_tmp2;
      for (int e = lane; e < 2 * R * dout; e += SG_WAVE) {
        const int s = e / (R * dout), r = (e - s * R * dout) / dout;
        const int rs = s ? r1 : r0;
        gpre[e] = r < rs ? sg_act_grad(L.act, pre[e], out[e], gcur[e]) : 0.f;
      }
      sg_wsync();
      if (L.bias) {
        for (int j = lane; j < dout; j += SG_WAVE) {
          float acc = 0.f;
          for (int sr = 0; sr < 2 * R; ++sr) acc += gpre[sr * dout + j];
          atomicAdd(&G[L.offB + j], acc);
        }
      }
      const float *gz = gpre;  // gradient w.r.t. (xd · W)
      if (L.kind == SG_GCN) {
        // adjoint of the sparse matmul: gsup = Âᵀ gpre
        for (int e = lane; e < 2 * R * dout; e += SG_WAVE) {
          const int s = e / (R * dout), rem = e - s * R * dout, m = rem / dout, j = rem - m * dout;
          const int rs = s ? r1 : r0;
          float acc = 0.f;
          if (m < rs) {
            const float *ac = adj + s * nmax * nmax + m;
            const float *gc = gpre + s * R * dout + j;
            for (int n = 0; n < rs; ++n) acc = fmaf(ac[n * nmax], gc[n * dout], acc);
          }
          gsup[e] = acc;
        }
        sg_wsync();
        gz = gsup;
      }
      if (L.sparse) {
        // scatter-add into the rows of W0 selected by the node types
        const float *xm = xd;
        for (int e = lane; e < 2 * nmax * dout; e += SG_WAVE) {
          const int s = e / (nmax * dout), rem = e - s * nmax * dout, n = rem / dout, j = rem - n * dout;
          const int rs = s ? r1 : r0;
          const float sc = xm[s * nmax + n];
          if (n < rs && sc != 0.f) {
            int t = types[s * nmax + n];
            t = t < 0 ? 0 : (t >= din ? din - 1 : t);
            atomicAdd(&G[L.offW + t * dout + j], sc * gz[e]);
          }
        }
      } else {
        for (int e = lane; e < din * dout; e += SG_WAVE) {
          const int i = e / dout, j = e - i * dout;
          float acc = 0.f;
          for (int sr = 0; sr < 2 * R; ++sr) acc = fmaf(xd[sr * din + i], gz[sr * dout + j], acc);
          atomicAdd(&G[L.offW + e], acc);
        }
        for (int e = lane; e < 2 * R * din; e += SG_WAVE) {
          const int s = e / (R * din), rem = e - s * R * din, r = rem / din, i = rem - r * din;
          const int rs = s ? r1 : r0;
          float v = 0.f;
          if (r < rs && sg_keep(pk, L.li, s, rem, L.thr)) {
            const float *gr = gz + (s * R + r) * dout;
            float acc = 0.f;
            for (int j = 0; j < dout; ++j) acc = fmaf(gr[j], prm[L.offW + i * dout + j], acc);
            v = acc * L.inv_keep;
          }
          gnext[e] = v;
        }
      }
      sg_wsync();
    } else if (L.kind == SG_PADDING) {
      const int d = L.din, Rin = L.Rin, Pr = L.Rout;
      for (int e = lane; e < 2 * Rin * d; e += SG_WAVE) {
        const int s = e / (Rin * d), rem = e - s * Rin * d, r = rem / d, c = rem - r * d;
        const int rs = s ? r1 : r0;
        gnext[e] = (r < rs && r < Pr) ? gcur[(s * Pr + r) * d + c] : 0.f;
      }
      sg_wsync();
    } else if (L.kind == SG_AVERAGE) {
      const int d = L.din, Rin = L.Rin;
      for (int e = lane; e < 2 * Rin * d; e += SG_WAVE) {
        const int s = e / (Rin * d), rem = e - s * Rin * d, r = rem / d, c = rem - r * d;
        const int rs = s ? r1 : r0;
        gnext[e] = r < rs ? gcur[s * d + c] / (float)rs : 0.f;
      }
      sg_wsync();
    } else {  // SG_ATTENTION
      const int d = L.din, Rin = L.Rin;
      const float *temp = S + L.l_temp, *hv = S + L.l_hv, *att = S + L.l_att;
      float *gzb = S + L.l_gz, *gu = S + L.l_gu, *gt = S + L.l_gt;
      for (int e = lane; e < 2 * Rin; e += SG_WAVE) {
        const int s = e / Rin, r = e - s * Rin;
        const int rs = s ? r1 : r0;
        float v = 0.f;
        if (r < rs) {
          float ga = 0.f;
          for (int c = 0; c < d; ++c) ga = fmaf(gcur[s * d + c], x[(s * Rin + r) * d + c], ga);
          v = ga * att[e] * (1.f - att[e]);
        }
        gzb[e] = v;
      }
      sg_wsync();
      for (int e = lane; e < 2 * d; e += SG_WAVE) {
        const int s = e / d, c = e - s * d;
        const int rs = s ? r1 : r0;
        float gh = 0.f;
        for (int r = 0; r < rs; ++r) gh = fmaf(gzb[s * Rin + r], x[(s * Rin + r) * d + c], gh);
        gu[e] = gh * (1.f - hv[e] * hv[e]);
      }
      sg_wsync();
      for (int e = lane; e < d * d; e += SG_WAVE) {
        const int i = e / d, c = e - i * d;
        atomicAdd(&G[L.offW + e], temp[i] * gu[c] + temp[d + i] * gu[d + c]);
      }
      for (int e = lane; e < 2 * d; e += SG_WAVE) {
        const int s = e / d, i = e - s * d;
        float acc = 0.f;
        for (int c = 0; c < d; ++c) acc = fmaf(gu[s * d + c], prm[L.offW + i * d + c], acc);
        gt[e] = acc;
      }
      sg_wsync();
      for (int e = lane; e < 2 * Rin * d; e += SG_WAVE) {
        const int s = e / (Rin * d), rem = e - s * Rin * d, r = rem / d, c = rem - r * d;
        const int rs = s ? r1 : r0;
        gnext[e] = r < rs ? att[s * Rin + r] * gcur[s * d + c] + gzb[s * Rin + r] * hv[s * d + c] +
                                gt[s * d + c] / (float)rs
                          : 0.f;
      }
      sg_wsync();
    }
    float *t = gcur;
    gcur = gnext;
    gnext = t;
  }
}

template <bool BWD>
__global__ void __launch_bounds__(256) sg_generic_kernel(SgGenPlan P, GenArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int gfl = BWD ? ((P.n_params + 1 + 3) & ~3) : 0;
  float *G = smem;
  float *S = smem + gfl + wave * P.wave_floats;
  const float *__restrict__ prm = A.params;
  if (BWD) {
    for (int i = threadIdx.x; i < gfl; i += blockDim.x) G[i] = 0.f;
  }
  __syncthreads();
  const int nmax = P.n_max;
  const float ybar = (BWD && P.loss_mode == SG_LOSS_BROADCAST) ? A.y_stats[0] : 0.f;
  float loss_acc = 0.f;
  for (int64_t q = (int64_t)blockIdx.x * nw + wave; q < A.n_pairs; q += (int64_t)gridDim.x * nw) {
    int64_t p = q;   // record = batch pair index
    if (A.order) {
      const int v = A.order[q];
      p = v < 0 ? 0 : (v >= A.n_pairs ? A.n_pairs - 1 : v);   // never out of bounds
    }
    const uint32_t *rec = (const uint32_t *)(A.recs + (size_t)p * (size_t)P.hbm_words * 4u);
    uint32_t *R = (uint32_t *)(S + P.l_rec);
    if (P.adj_dtype == SG_DTYPE_BF16) {   // widen Â to the f32 LDS layout
      const int aw = P.hbm_adj_words;
      for (int i = lane; i < P.hbm_words; i += SG_WAVE) {
        const uint32_t v = rec[i];
        if (i < aw) {
          R[2 * i] = v << 16;
          R[2 * i + 1] = v & 0xFFFF0000u;
        } else if (i - aw < P.rec_words - 2 * aw) {
          R[i + aw] = v;
        }
      }
    } else {
      for (int i = lane; i < P.rec_words; i += SG_WAVE) R[i] = rec[i];
    }
    sg_wsync();
    const float *adj = S + P.l_rec;
    const int *types = (const int *)(S + P.l_rec + P.rec_types);
    const int n0 = ((const int *)(S + P.l_rec))[P.rec_nnodes];
    const int n1 = ((const int *)(S + P.l_rec))[P.rec_nnodes + 1];
    const float label = S[P.l_rec + P.rec_label];
    const uint32_t pk = sg_pair_key(A.key, (uint32_t)(A.pair_offset + p));
    gen_forward_nodes(P, S, prm, adj, types, n0, n1, pk, lane);

    // ---- pair head ----
    const SgGenLayer &last = P.L[P.nl - 1];
    const float *e0 = S + last.l_out;
    const float *e1 = e0 + last.Rout * last.dout;
    const int D = P.D, K = P.K;
    float s = 0.f, rsum = 0.f, usum = 0.f;
    float *x12 = S + P.l_x12, *u = S + P.l_u, *m = S + P.l_m;
    if (P.head_kind == SG_NTN) {
      for (int e = lane; e < 2 * D; e += SG_WAVE) {
        const int sd = e / D, q = e - sd * D;
        const float v = (sd ? e1 : e0)[q];
        x12[e] = sg_keep(pk, P.head_li, sd, q, P.head_thr) ? v * P.head_inv_keep : 0.f;
      }
      sg_wsync();
      for (int e = lane; e < D * K; e += SG_WAVE) {  // u[a][k] = Σ_b W[a][b][k] x2[b]
        const int a = e / K, k = e - a * K;
        float acc = 0.f;
        for (int b = 0; b < D; ++b) acc = fmaf(prm[P.offW + (a * D + b) * K + k], x12[D + b], acc);
        u[e] = acc;
      }
      sg_wsync();
      for (int k = lane; k < K; k += SG_WAVE) {
        float acc = 0.f;
        for (int i = 0; i < 2 * D; ++i) acc = fmaf(prm[P.offV + k * 2 * D + i], x12[i], acc);
        for (int a = 0; a < D; ++a) acc = fmaf(x12[a], u[a * K + k], acc);
        if (P.head_bias) acc += prm[P.offB + k];
        m[k] = acc;
      }
      sg_wsync();
      for (int k = 0; k < K; ++k) {
        const float r = sg_act(P.head_act, m[k]);
        const float U = prm[P.offU + k];
        rsum += r;
        usum += U;
        if (P.ntn_mode == SG_NTN_INTENDED) s = fmaf(U, r, s);
      }
      if (P.ntn_mode == SG_NTN_REFERENCE) s = usum * rsum;
    } else {  // Dot
      float part = 0.f;
      for (int q = lane; q < D; q += SG_WAVE) part = fmaf(e0[q], e1[q], part);
      s = sg_wave_sum(part);
    }

    if (!BWD) {
      if (lane == 0) A.s_out[p] = s;
      continue;
    }
    if (A.s_out && lane == 0) A.s_out[p] = s;
    // ---- loss (model_mse.py:145-151) ----
    const float yhat = sg_final(P.final_act, P.yeta, s);
    float gy;
    if (P.loss_mode == SG_LOSS_BROADCAST) {
      gy = yhat - ybar;                     // ∂/∂ŷ_j of l2_loss((B,1)-(B,))/B
      loss_acc += 0.5f * gy * gy;
    } else {
      const float dlt = yhat - label;
      gy = dlt * A.inv_batch;
      loss_acc += 0.5f * dlt * dlt * A.inv_batch;
    }
    const float gs = gy * sg_final_grad(P.final_act, P.yeta, s, yhat);

    // ---- head backward ----
    float *gcur = S + P.l_g0, *gnext = S + P.l_g1;
    const int Rh = last.Rout * last.dout;
    if (P.head_kind == SG_NTN) {
      float *gm = S + P.l_gm;
      for (int k = lane; k < K; k += SG_WAVE) {
        const float r = sg_act(P.head_act, m[k]);
        const float gr = (P.ntn_mode == SG_NTN_REFERENCE) ? gs * usum : gs * prm[P.offU + k];
        const float g = sg_act_grad(P.head_act, m[k], r, gr);
        gm[k] = g;
        if (P.head_bias) atomicAdd(&G[P.offB + k], g);
        atomicAdd(&G[P.offU + k], (P.ntn_mode == SG_NTN_REFERENCE) ? gs * rsum : gs * r);
      }
      sg_wsync();
      for (int e = lane; e < K * 2 * D; e += SG_WAVE) {
        const int k = e / (2 * D), i = e - k * 2 * D;
        atomicAdd(&G[P.offV + e], gm[k] * x12[i]);
      }
      for (int e = lane; e < D * D * K; e += SG_WAVE) {
        const int a = e / (D * K), rem = e - a * D * K, b = rem / K, k = rem - b * K;
        atomicAdd(&G[P.offW + e], gm[k] * x12[a] * x12[D + b]);
      }
      for (int e = lane; e < 2 * D; e += SG_WAVE) {
        const int sd = e / D, q = e - sd * D;
        float acc = 0.f;
        for (int k = 0; k < K; ++k) acc = fmaf(prm[P.offV + k * 2 * D + e], gm[k], acc);
        if (sd == 0) {
          for (int k = 0; k < K; ++k) acc = fmaf(u[q * K + k], gm[k], acc);
        } else {
          for (int k = 0; k < K; ++k) {
            float w = 0.f;
            for (int a = 0; a < D; ++a) w = fmaf(x12[a], prm[P.offW + (a * D + q) * K + k], w);
            acc = fmaf(gm[k], w, acc);
          }
        }
        const float g = sg_keep(pk, P.head_li, sd, q, P.head_thr) ? acc * P.head_inv_keep : 0.f;
        gcur[sd * Rh + q] = g;
      }
    } else {
      for (int e = lane; e < 2 * D; e += SG_WAVE) {
        const int sd = e / D, q = e - sd * D;
        gcur[e] = gs * (sd ? e0[q] : e1[q]);
      }
    }
    sg_wsync();
    gen_backward_nodes(P, S, G, prm, adj, types, n0, n1, pk, lane, gcur, gnext);
  }
  if (BWD) {
    if (lane == 0) atomicAdd(&G[P.n_params], loss_acc);
    __syncthreads();
    float *dst = A.slab + (size_t)blockIdx.x * (size_t)(P.n_params + 1);
    for (int i = threadIdx.x; i <= P.n_params; i += blockDim.x) dst[i] = G[i];
  }
}

}  // namespace

// Launch configuration of the generic kernel (shared with sg_workspace_bytes).
struct SgGenLaunch {
  int waves_per_block;
  int blocks;
  size_t lds_bytes;
};

int sg_num_cus();

static SgGenLaunch sg_generic_launch(const SgGenPlan &P, int64_t n_pairs, bool bwd) {
  SgGenLaunch L;
  const size_t gbytes = bwd ? (size_t)((P.n_params + 1 + 3) & ~3) * 4u : 0u;
  const size_t wbytes = (size_t)P.wave_floats * 4u;
  int nw = 4;
  while (nw > 1 && gbytes + nw * wbytes > 81920u) --nw;
  L.waves_per_block = nw;
  L.lds_bytes = gbytes + nw * wbytes;
  int per_cu = (int)(163840u / (L.lds_bytes ? L.lds_bytes : 1u));
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 8) per_cu = 8;
  int64_t want = (n_pairs + nw - 1) / nw;
  int64_t cap = (int64_t)sg_num_cus() * per_cu;
  L.blocks = (int)(want < cap ? (want > 0 ? want : 1) : cap);
  return L;
}

int sg_generic_lds_ok(const SgGenPlan &P, bool bwd) {
  SgGenLaunch L = sg_generic_launch(P, 1, bwd);
  return L.lds_bytes <= 163840u;
}

int64_t sg_generic_slab_floats(const SgGenPlan &P, int64_t n_pairs) {
  SgGenLaunch L = sg_generic_launch(P, n_pairs, true);
  return (int64_t)L.blocks * (P.n_params + 1);
}

int sg_generic_run(const SgGenPlan &P, bool bwd, const void *recs, const int32_t *order,
                   int64_t n_pairs, int64_t pair_offset, int64_t batch_total, const float *params, uint64_t seed,
                   const float *y_stats, float *s_out, float *slab, int *blocks_out,
                   hipStream_t stream) {
  SgGenLaunch L = sg_generic_launch(P, n_pairs, bwd);
  if (L.lds_bytes > 163840u) return SG_ERR_UNSUPPORTED;
  GenArgs A;
  A.recs = (const uint8_t *)recs;
  A.order = order;
  A.n_pairs = n_pairs;
  A.pair_offset = pair_offset;
  A.inv_batch = batch_total > 0 ? 1.f / (float)batch_total : 0.f;
  A.params = params;
  A.key = sg_seed_key(seed);
  A.y_stats = y_stats;
  A.s_out = s_out;
  A.slab = slab;
  if (L.lds_bytes > 65536u) {
    (void)hipFuncSetAttribute(bwd ? (const void *)sg_generic_kernel<true>
                            : (const void *)sg_generic_kernel<false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_bytes);
  }
  if (bwd)
    hipLaunchKernelGGL(sg_generic_kernel<true>, dim3(L.blocks), dim3(64 * L.waves_per_block),
                       L.lds_bytes, stream, P, A);
  else
    hipLaunchKernelGGL(sg_generic_kernel<false>, dim3(L.blocks), dim3(64 * L.waves_per_block),
                       L.lds_bytes, stream, P, A);
  if (blocks_out) *blocks_out = L.blocks;
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}
