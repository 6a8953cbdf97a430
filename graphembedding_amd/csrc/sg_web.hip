// sg_web.hip — graph-store path for Web-sized graphs (BASELINE config C5; path 3).
//
// The reference's default stack (config.py:44-66) with Padding / NTN widened to
// D in [32, 512] (quirk A9: tf.pad needs N <= max_in_dims):
//   GCN(d_in→32, relu, sparse one-hot) → GCN(32→16, identity) → Dense(16→1, relu)
//   → Padding(D) → NTN(D, K ≤ 16) → final act → broadcast / aligned MSE.
// Dense pair records stop scaling at a few dozen nodes (Â is n_max² per side), so
// this path reads the graphs from a CSR store and a list of pair ids, and splits
// a pair's work in two kinds of kernels:
//
//  * per graph instance (pair, side): one 8-wave workgroup stages the instance's
//    activations in LDS (up to 512 nodes) and runs the GCN / Dense / Padding stack
//    (layers.py:91-118, 192-227).  The sparse products Â·Z run on VALU over the CSR
//    rows; the dense ones (D1·W1, gZ1·W1ᵀ, D1ᵀ·gZ1 and the one-hot Xᵀ·gZ0) on
//    v_mfma_f32_16x16x4_f32 with the instance's nodes as 16-row tiles.  Forward
//    writes the NTN input x (after its dropout) per pair and side; backward
//    recomputes the forward and accumulates the GCN/Dense gradients per workgroup.
//  * NTN (layers.py:282-310) as batched GEMMs over the pairs, 128×128 f32 MFMA
//    tiles: T[p][k][a] = Σ_b W[a][b][k] x2[p][b] (forward), gx2 = (gm ⊗ x1)·W
//    and gW[k] = Σ_p (gm_k x1)ᵀ x2 (backward).  A per-pair head kernel turns T into
//    m_k, s, ŷ, the loss and gm = ∂L/∂m, and gx1 = Σ_k gm_k (T_k + V_k).
//    Tiles whose feature range lies beyond every pair's node count (x is zero
//    there when padding_value = 0) are skipped: callers that order pairs by size
//    (web.py) make the tiles homogeneous.
//
// Dropout keys, masks and loss conventions are those of the pair-record kernels
// (sg_common.h; oracle/siamese_oracle.py): pair i of the list is pair_offset + i.
// Reductions run in a fixed order: results are bitwise reproducible.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <list>
#include <mutex>
#include <type_traits>
#include <vector>

#include "sg_common.h"
#include "sg_mfma.h"

int sg_num_cus();

namespace {
using sgk::f4;
using sgk::mfma4;

constexpr int WH1 = 32, WH2 = 16;   // GCN widths of the default stack
constexpr int WKP = 16;             // NTN K capacity (gm rows, head slab)
constexpr int WMAXD = 512;          // max Padding / NTN width (LDS budget of one instance)
constexpr int TB = 128;             // GEMM tile edge
constexpr int MKS = 20;             // MK LDS tile row stride (16 + 4): conflict-free b128 reads
constexpr int KMS = TB + 4;         // KM LDS tile row stride
constexpr int HSLAB = 1 + 2 * WKP;  // head slab row: loss | gU[16] | gb[16]
constexpr int WSPLIT = 16;   // split-K over pairs of the weight-gradient GEMMs
constexpr int kUnitChunk = 4096;    // instances per block of the size-class sort (web_icls_*)
// XCD partitions of the instance units: instances of graph g go to partition g % kXcdParts,
// and unit slot u runs on the workgroups with blockIdx.x = u (mod kXcdParts), which the
// dispatcher deals to one XCD (observed placement; speed only, never correctness): each
// XCD then gathers the CSR rows of an eighth of the graphs, which fit its 4 MiB L2
constexpr int kXcdParts = 8;
constexpr int kIKeys = 3 * kXcdParts;   // sort keys: size class x partition

struct WebPlan {
  int d_in, D, Dp, K;
  int n_params, n_gcn;
  int ob0, oW1, ob1, oWd, obd, oW, oV, oU, obn;
  uint32_t thr0, thr1, thr2, thr4;
  float ik0, ik1, ik2, ik4;
  float padv;
  int final_act, loss_mode, ntn_mode;
  float yeta;
  int tb;  // 16-row type tiles of the one-hot gW0 product
};

int web_plan(const sg_model_t *m, WebPlan *W) {
  if (!m || !W) return SG_ERR_ARG;
  memset(W, 0, sizeof(*W));
  if (m->num_layers != 5) return SG_ERR_UNSUPPORTED;
  const sg_layer_t *L = m->layers;
  if (L[0].kind != SG_GCN || !L[0].sparse_inputs || L[0].output_dim != WH1 ||
      L[0].act != SG_ACT_RELU || !L[0].bias)
    return SG_ERR_UNSUPPORTED;
  if (L[0].input_dim > 0 && L[0].input_dim != m->d_in) return SG_ERR_ARG;
  if (L[1].kind != SG_GCN || L[1].sparse_inputs || L[1].input_dim != WH1 ||
      L[1].output_dim != WH2 || L[1].act != SG_ACT_IDENTITY || !L[1].bias)
    return SG_ERR_UNSUPPORTED;
  if (L[2].kind != SG_DENSE || L[2].input_dim != WH2 || L[2].output_dim != 1 ||
      L[2].act != SG_ACT_RELU || !L[2].bias)
    return SG_ERR_UNSUPPORTED;
  if (L[3].kind != SG_PADDING) return SG_ERR_UNSUPPORTED;
  const int D = L[3].output_dim;
  if (D < 32 || D > WMAXD) return SG_ERR_UNSUPPORTED;
  if (L[4].kind != SG_NTN || L[4].input_dim != D || L[4].output_dim < 1 ||
      L[4].output_dim > WKP || L[4].act != SG_ACT_RELU)
    return SG_ERR_UNSUPPORTED;
  if (m->d_in <= 0 || m->d_in > 64) return SG_ERR_UNSUPPORTED;
  if (m->n_max <= 0) return SG_ERR_ARG;
  if (m->n_max > D) return SG_ERR_SHAPE;   // tf.pad with N > max_in_dims (A9)
  if (!(m->keep_prob > 0.f && m->keep_prob <= 1.f)) return SG_ERR_ARG;
  if (m->final_act < SG_FINAL_GAUSSIAN || m->final_act > SG_FINAL_TANH) return SG_ERR_ARG;
  if (m->loss_mode != SG_LOSS_BROADCAST && m->loss_mode != SG_LOSS_ALIGNED) return SG_ERR_ARG;
  if (m->ntn_mode != SG_NTN_REFERENCE && m->ntn_mode != SG_NTN_INTENDED) return SG_ERR_ARG;
  W->d_in = m->d_in;
  W->D = D;
  W->Dp = (D + TB - 1) / TB * TB;
  W->K = L[4].output_dim;
  W->tb = (m->d_in + 15) / 16;
  int off = m->d_in * WH1;   // W0 at 0
  W->ob0 = off; off += WH1;
  W->oW1 = off; off += WH1 * WH2;
  W->ob1 = off; off += WH2;
  W->oWd = off; off += WH2;
  W->obd = off; off += 1;
  W->n_gcn = off;
  W->oW = off; off += D * D * W->K;
  W->oV = off; off += W->K * 2 * D;
  W->oU = off; off += W->K;
  W->obn = -1;
  if (L[4].bias) { W->obn = off; off += W->K; }
  W->n_params = off;
  const float keep = m->keep_prob;
  const float k0 = L[0].dropout ? keep : 1.f, k1 = L[1].dropout ? keep : 1.f;
  const float k2 = L[2].dropout ? keep : 1.f, k4 = L[4].dropout ? keep : 1.f;
  W->thr0 = sg_keep_threshold(k0);
  W->thr1 = sg_keep_threshold(k1);
  W->thr2 = sg_keep_threshold(k2);
  W->thr4 = sg_keep_threshold(k4);
  W->ik0 = 1.f / k0;
  W->ik1 = 1.f / k1;
  W->ik2 = 1.f / k2;
  W->ik4 = 1.f / k4;
  W->padv = L[3].padding_value;
  W->final_act = m->final_act;
  W->loss_mode = m->loss_mode;
  W->ntn_mode = m->ntn_mode;
  W->yeta = m->yeta;
  return SG_OK;
}

// ---------------------------------------------------------------------------
// Workspace layout (floats unless noted), for chunks of up to `chunk` pairs.
// ---------------------------------------------------------------------------
struct WebWs {
  int64_t Cp;                                        // chunk rounded up to TB
  // per-chunk buffers, one set per pipeline slot (slot 1 = slot 0 + SLOT): the
  // instance kernels of chunk c + 1 overlap the NTN GEMMs of chunk c (sg_web_run)
  int64_t X, GX, T, GM, EXT, EXT16, EXT128, INST;
  int64_t ISORT, ICNT, ICLS;                         // instance units (web_icls_*)
  int64_t MASK;   // uint16 [2 Cp][Dp][4]: the forward's dropout keep bits per (instance, node, g)
  int64_t D2;     // [2 Cp][Dp][16]: the forward's D2 = dropout(H2) per (instance, node)
  int64_t SLOT;                                      // floats per slot
  int64_t S0;                                        // slot 0 (slot 1 = S0 + SLOT, last)
  int64_t Wg, Wh, GWS, GVS, GSLAB, HSLABo;           // per-call buffers (first)
  int64_t total, total1;   // with both slots; with slot 0 only (calls of one chunk)
  int gcn_blocks, head_blocks;
};

int gcn_blocks_for() { return sg_num_cus(); }
int head_blocks_for() { return 3 * sg_num_cus(); }


// The backward instance kernel reads the dropout keep bits the forward wrote (GcnArgs::masks)
// instead of re-hashing 13 elements per lane and tile; 0: it re-hashes (A/B)
// ... and the forward's D2 = dropout(H2) rows (GcnArgs::d2) instead of recomputing Z1 = D1'·W1
// and the H2 pass, which also drops two of the unit's barriers; 0: it recomputes (A/B)

WebWs web_ws(const WebPlan &W, int64_t chunk) {
  WebWs w;
  if (chunk < 1) chunk = 1;
  w.Cp = (chunk + TB - 1) / TB * TB;
  const int64_t Dp = W.Dp, K = W.K;
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) & ~(int64_t)63; return r; };
  // per-call buffers first, then the pipeline slots, slot 1 last: a call of one chunk
  // (n_pairs <= chunk) never pipelines and needs total1 floats only
  w.Wg = take(K * Dp * Dp);
  w.Wh = take(K * Dp * Dp);
  w.GWS = take((int64_t)WSPLIT * K * Dp * Dp);
  w.GVS = take((int64_t)WSPLIT * WKP * 2 * Dp);
  w.gcn_blocks = gcn_blocks_for();
  w.head_blocks = head_blocks_for();
  w.GSLAB = take((int64_t)w.gcn_blocks * W.n_gcn);
  w.HSLABo = take((int64_t)w.head_blocks * 4 * HSLAB);
  w.S0 = o;
  o = 0;   // slot-relative offsets
  w.X = take(2 * w.Cp * Dp);        // X1 | X2
  w.GX = take(2 * w.Cp * Dp);       // gX1 | gX2
  // T: the a-tile shares MP[p][k][4] of web_t_kernel_b3<true>, or all of T (f32 path)
  w.T = take(w.Cp * WKP * 4);
  w.GM = take(w.Cp * WKP);
  w.EXT = take(2 * w.Cp);           // int2 per pair
  w.EXT16 = take(2 * (w.Cp / 16));
  w.EXT128 = take(2 * (w.Cp / TB));
  w.INST = take(8 * w.Cp);          // int4 per instance
  w.ISORT = take(2 * w.Cp);         // instances sorted by size class
  w.ICNT = take(kIKeys * ((2 * w.Cp + kUnitChunk - 1) / kUnitChunk));
  w.ICLS = take(kIKeys + 8);
  w.MASK = take(4 * w.Cp * Dp);     // 2 Cp x Dp x 4 uint16
  w.D2 = take(32 * w.Cp * Dp);   // 2 Cp x Dp x 16
  w.SLOT = o;
  w.total1 = w.S0 + w.SLOT;
  w.total = w.S0 + 2 * w.SLOT;
  return w;
}

// ---------------------------------------------------------------------------
// Per-pair extents: e = n (padding_value 0: x is zero beyond the graph's nodes)
// or D; per 16- and 128-pair maxima for the GEMM tile skips.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(TB) web_ext_kernel(const int32_t *__restrict__ pairs, int64_t n,
                                                     const int32_t *__restrict__ node_off,
                                                     const int32_t *__restrict__ row_ptr,
                                                     int full, int D, int2 *__restrict__ ext,
                                                     int2 *__restrict__ ext16,
                                                     int2 *__restrict__ ext128,
                                                     int4 *__restrict__ inst) {
  __shared__ int2 red[2];
  const int64_t p = (int64_t)blockIdx.x * TB + threadIdx.x;
  int e1 = 0, e2 = 0;
  if (p < n) {
    const int g1 = pairs[2 * p], g2 = pairs[2 * p + 1];
    const int o1 = node_off[g1], n1 = node_off[g1 + 1] - o1;
    const int o2 = node_off[g2], n2 = node_off[g2 + 1] - o2;
    e1 = full ? D : n1;
    e2 = full ? D : n2;
    // per-instance (first node, nodes, first Â entry, Â entries) for web_gcn_kernel
    const int b1 = row_ptr[o1], b2 = row_ptr[o2];
    inst[2 * p] = make_int4(o1, n1, b1, row_ptr[o1 + n1] - b1);
    inst[2 * p + 1] = make_int4(o2, n2, b2, row_ptr[o2 + n2] - b2);
  }
  ext[p] = make_int2(e1, e2);
  int m1 = e1, m2 = e2;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    m1 = max(m1, __shfl_xor(m1, o, 64));
    m2 = max(m2, __shfl_xor(m2, o, 64));
  }
  if ((threadIdx.x & 15) == 0) ext16[p >> 4] = make_int2(m1, m2);
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    m1 = max(m1, __shfl_xor(m1, o, 64));
    m2 = max(m2, __shfl_xor(m2, o, 64));
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_int2(m1, m2);
  __syncthreads();
  if (threadIdx.x == 0)
    ext128[blockIdx.x] = make_int2(max(red[0].x, red[1].x), max(red[0].y, red[1].y));
}

// ---------------------------------------------------------------------------
// Instance units for the instance kernels (GcnArgs::isorted): a stable counting sort of
// the chunk's instances by key = size class (0: N <= cap4, 1: N <= cap2, 2: the rest;
// cap4 / cap2 = a quarter / half of the instance region) x XCD partition (graph % np,
// np = kXcdParts, or 1 with SG_WEB_XCD=0).  Blocks own contiguous runs of kUnitChunk
// instances; counts are key-major so one exclusive scan gives every (key, run) its base;
// the scatter ranks by ballot: deterministic.  Instance q is side q & 1 of pair q >> 1,
// whose graph is pairs[q].
// ---------------------------------------------------------------------------
__device__ __forceinline__ int web_ikey(const int4 *inst, const int32_t *pairs, int64_t q,
                                        int cap4, int cap2, int np) {
  const int N = inst[q].y;
  const int c = N <= cap4 ? 0 : (N <= cap2 ? 1 : 2);
  return c * kXcdParts + (np > 1 ? (int)((uint32_t)pairs[q] % (uint32_t)np) : 0);
}

__global__ void __launch_bounds__(256) web_icls_count(const int4 *__restrict__ inst,
                                                      const int32_t *__restrict__ pairs, int64_t n,
                                                      int cap4, int cap2, int np, int nb,
                                                      int32_t *__restrict__ cnt) {
  __shared__ int h[kIKeys];
  if (threadIdx.x < kIKeys) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * kUnitChunk;
  for (int i = threadIdx.x; i < kUnitChunk && b0 + i < n; i += blockDim.x)
    atomicAdd(&h[web_ikey(inst, pairs, b0 + i, cap4, cap2, np)], 1);
  __syncthreads();
  if (threadIdx.x < kIKeys) cnt[(size_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of the kIKeys x nb counts (one 1024-thread block: each thread sums a run of
// consecutive counts, a block scan of the run sums, then each thread rewrites its run), the
// key starts icls[0..kIKeys], and the unit-slot layout: class c holds np x R_c unit slots
// from icls[kIKeys + 1 + c] (R_c = the most units of any of its partitions; units of 4, 2
// and 1 instances for classes 0, 1, 2), icls[kIKeys + 4] = all slots, icls[kIKeys + 5] = np.
// (A one-thread scan over the 24 x nb counts took 0.6 ms per 262,144-pair chunk.)
constexpr int kScanT = 1024;
__global__ void __launch_bounds__(kScanT) web_icls_scan(int32_t *__restrict__ cnt, int nb, int64_t n,
                                                        int np, int32_t *__restrict__ icls) {
  __shared__ int part[kScanT];
  const int t = threadIdx.x;
  const int tot = kIKeys * nb, per = (tot + kScanT - 1) / kScanT, b0 = t * per;
  int sum = 0;
  for (int k = 0; k < per; ++k)
    if (b0 + k < tot) sum += cnt[b0 + k];
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < kScanT; o <<= 1) {   // inclusive Hillis-Steele scan of the run sums
    const int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = t ? part[t - 1] : 0;
  for (int k = 0; k < per; ++k) {
    const int x = b0 + k;
    if (x < tot) {
      const int v = cnt[x];
      cnt[x] = run;
      if (x % nb == 0) icls[x / nb] = run;   // key x / nb starts here
      run += v;
    }
  }
  if (tot == 0 && t < kIKeys) icls[t] = 0;
  __syncthreads();   // the block's global writes of icls are visible to thread 0
  if (t != 0) return;
  icls[kIKeys] = (int32_t)n;
  int ub = 0;
  for (int c = 0; c < 3; ++c) {
    const int gsz = c == 0 ? 4 : (c == 1 ? 2 : 1);
    int R = 0;
    for (int p = 0; p < np; ++p) {
      const int k = c * kXcdParts + p;
      const int nu = (icls[k + 1] - icls[k] + gsz - 1) / gsz;
      R = nu > R ? nu : R;
    }
    icls[kIKeys + 1 + c] = ub;
    ub += np * R;
  }
  icls[kIKeys + 4] = ub;
  icls[kIKeys + 5] = np;
}

__global__ void __launch_bounds__(256) web_icls_scatter(const int4 *__restrict__ inst,
                                                        const int32_t *__restrict__ pairs, int64_t n,
                                                        int cap4, int cap2, int np, int nb,
                                                        const int32_t *__restrict__ base,
                                                        int32_t *__restrict__ sorted) {
  __shared__ int run[kIKeys];
  __shared__ int wc[4][kIKeys];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t < kIKeys) run[t] = base[(size_t)t * nb + blockIdx.x];
  const int64_t b0 = (int64_t)blockIdx.x * kUnitChunk;
  const int64_t b1 = b0 + kUnitChunk < n ? b0 + kUnitChunk : n;
  for (int64_t t0 = b0; t0 < b1; t0 += 256) {
    if (t < 4 * kIKeys) (&wc[0][0])[t] = 0;
    __syncthreads();
    const int64_t q = t0 + t;
    const bool valid = q < b1;
    const int key = valid ? web_ikey(inst, pairs, q, cap4, cap2, np) : -1;
    int rank = 0;
    for (int k = 0; k < kIKeys; ++k) {
      const uint64_t m = __ballot(valid && key == k);
      if (m == 0ull) continue;   // wave-uniform
      if (key == k) rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wc[w][k] = __popcll(m);
    }
    __syncthreads();
    if (valid) {
      int off = run[key] + rank;
      for (int v = 0; v < w; ++v) off += wc[v][key];
      sorted[off] = (int32_t)q;
    }
    __syncthreads();
    if (t < kIKeys) run[t] += wc[0][t] + wc[1][t] + wc[2][t] + wc[3][t];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Weight layouts for the GEMMs: Wg[k][a][b] = W[a][b][k] (T: rows a, contraction b)
// and Wh[k][b][a] (gx2: rows b, contraction a); zero beyond D.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) web_wprep_g(const float *__restrict__ Wt, int D, int Dp,
                                                   int K, float *__restrict__ Wg) {
  // block: one row a, 64 b's; reads W[a][b0..b0+63][0..K) (contiguous), writes Wg rows
  __shared__ float t[64 * (WKP + 1)];
  const int a = blockIdx.x, b0 = blockIdx.y * 64;
  const int span = 64 * K;
  for (int i = threadIdx.x; i < span; i += 256) {
    const int b = b0 + i / K, k = i % K;
    t[(i / K) * (WKP + 1) + k] = (a < D && b < D) ? Wt[((size_t)a * D + b) * K + k] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < span; i += 256) {
    const int k = i >> 6, bl = i & 63;
    Wg[((size_t)k * Dp + a) * Dp + b0 + bl] = t[bl * (WKP + 1) + k];
  }
}

__global__ void __launch_bounds__(256) web_wprep_h(const float *__restrict__ Wg, int Dp,
                                                   float *__restrict__ Wh) {
  // 32×32 tiled transpose of each Wg[k]
  __shared__ float t[32][33];
  const int k = blockIdx.z, x0 = blockIdx.x * 32, y0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float *src = Wg + (size_t)k * Dp * Dp;
  float *dst = Wh + (size_t)k * Dp * Dp;
  for (int r = ty; r < 32; r += 8) t[r][tx] = src[(size_t)(y0 + r) * Dp + x0 + tx];
  __syncthreads();
  for (int r = ty; r < 32; r += 8) dst[(size_t)(x0 + r) * Dp + y0 + tx] = t[tx][r];
}

// ---------------------------------------------------------------------------
// Per-instance GCN → Dense → Padding stack (+ backward with recompute).
// One workgroup per instance (pair, side); node tiles of 16 rows, tile t on wave
// t % waves (N <= 512: 32 tiles).  The sparse loops read the instance's CSR rows
// through the caches; LCSR (opt-in) stages them in LDS first.
// ---------------------------------------------------------------------------
// waves per instance workgroup: 8 forward, 16 backward.
// The backward wants more than the 128 VGPRs of a 16-wave block and spills ~32 of them
// there, but twice the waves per instance hide the latency-bound sparse phases better:
// 16 waves measured 411 -> 379 ms per C5 step against 8 (246 VGPRs, no spills).
// forward instance kernel: 8 waves (4 tiles each) measured 3.596 vs 3.571 M pairs/s
// against 16 on C5 (one stream), 3.610 with the chunk pipeline (profiles/r03_c5fw8/)
__host__ __device__ constexpr int gcn_gw(bool bwd) { return bwd ? 16 : 8; }

struct GcnArgs {
  const int32_t *node_off, *types, *row_ptr, *col;
  const float *val;
  const int32_t *pairs;
  const int4 *inst;  // [2 n_pairs] (first node, nodes, first Â entry, Â entries) per instance
  // Units (web_units): the chunk's instances stable-sorted by size class x XCD partition
  // (isorted) with the key starts and unit-slot layout in icls (web_icls_scan; class 0:
  // N <= cap/4, 1: N <= cap/2, 2: larger; cap = the instance region of n_max nodes).  A
  // workgroup takes a unit of 4, 2 or 1 instances of one class and partition and gives
  // each a quarter / half / all of its waves and of its instance region: the
  // latency-bound phases of small instances overlap.
  // isorted == null: units of one instance in list order.
  const int32_t *isorted;
  const int32_t *icls;
  int64_t n_pairs, pair_offset, Cp;
  const float *params;
  float *X;          // [2][Cp][Dp] NTN inputs (forward)
  // [2 n_pairs][Dp][4] dropout keep bits of lane g of node n of instance q (or null): the
  // forward writes them, the backward reads them instead of re-hashing.  Bits 4c + s: layer 1,
  // feature 16c + 4g + s; 8 + s: layer 2, feature 4g + s; 12: layer 4 (the node's NTN input)
  uint16_t *masks;
  // [2 n_pairs][Dp][16] the forward's D2 = dropout(H2) of every node (or null): the backward
  // reads its nodes' rows instead of recomputing Z1 and the H2 pass
  float *d2;
  const float *GX;   // [2][Cp][Dp] ∂L/∂x (backward)
  float *slab;       // [gridDim.x][n_gcn] (backward, accumulated)
  uint32_t key, thr0, thr1, thr2, thr4;
  float ik0, ik1, ik2, ik4, padv;
  int d_in, D, Dp, n_gcn, n_max, max_nnz;
  int ob0, oW1, ob1, oWd, obd;
};

// LDS (4-byte words): tables, then the instance region sized for n_max nodes
//   sW0 [(d_in+1)][32] = W0·ik0 (row d_in zero: dropped one-hot rows), sb0 [32],
//   sW1 [32][16] = W1·ik1, sW1T [16][32] = (W1·ik1)ᵀ, sb1 [16], sWd [16] = Wd·ik2
//   sEt [N16] effective type (d_in when dropped / absent),
//   sZ1 [N16][16]: Z1, then (backward) gZ1,
//   sD1 [N16][32] (backward): D1' = H1·m1, then gP0,
//   sScr [8 waves][16][16] (backward): a wave's gS1 tile, re-read as MFMA B operand,
//   CSR (LCSR): row offsets [N16 + 1], columns [max_nnz], values [max_nnz].
// LDS row strides (words): not multiples of 16, so the random-row b128 gathers of
// the sparse products spread over the banks (stride 16 puts every row on 4 bank groups)
constexpr int W0S = 36, ZS = 20, DS = 36;
// a wave's scratch tile (backward): 16 rows at stride SCS (≡ 20 mod 64 words: the column
// reads (4g + s)·SCS + i of lanes (i, g) hit distinct banks; stride 16 put 4 rows g on one)
constexpr int SCS = 20, SCR = 16 * SCS;
// gS0 = Â·gP0 with one CSR row per lane (node 16t + i, features 16c + 4g + s) and the tile
// transposed through the wave's scratch for the one-hot gW0 MFMA; 0: four rows per lane
// (nodes 16t + 4g + s, features i, 16 + i), the MFMA layout directly
// Backward MFMAs on split-bf16 (round 4): gD1 = gS1·W1ᵀ as three v_mfma_f32_16x16x32_bf16
// per feature half against W1's bf16 parts built once per block (the six leading products
// of (h + m + l)(H + M + L), ≈ f32 accuracy; sg_fast's gD1), and the one-hot gW0 = Xᵀ·gS0 as
// three v_mfma_f32_16x16x16_bf16 per (type tile, feature half) on the h, m and l parts of
// gS0 (one-hot is exact in bf16) — 16-cycle / 8-cycle bf16 MFMAs that co-issue with VALU in
// place of 32-cycle f32 ones that do not.  0: the f32 MFMAs (A/B)

struct GcnLds {
  int w0, b0, w1, w1t, b1, wd, w1b, tables, et, gx, z1, d1, scr, rp, col, val, total;
};

__host__ __device__ inline GcnLds gcn_lds(int d_in, int n16, int max_nnz, bool bwd, bool lcsr) {
  GcnLds L;
  int o = 0;
  L.w0 = o; o += (d_in + 1) * W0S;
  L.b0 = o; o += WH1;
  L.w1 = o; o += WH1 * WH2;
  L.w1t = o; o += WH1 * WH2;
  L.b1 = o; o += WH2;
  L.wd = o; o += WH2;
  o = (o + 3) & ~3;
  // backward: [cb][term][lane] uint4 bf16 B operands of gD1
  L.w1b = o; if (bwd) o += 2 * 3 * 64 * 4;
  L.tables = o;
  L.et = o; o += n16;
  L.gx = o; if (bwd) o += n16;
  L.z1 = o; o += n16 * ZS;
  L.d1 = o; if (bwd) o += n16 * DS;
  L.scr = o; if (bwd) o += gcn_gw(true) * SCR;
  L.rp = o; if (lcsr) o += (n16 + 4) & ~3;
  L.col = o; if (lcsr) o += ((max_nnz + 1) / 2 + 3) & ~3;   // u16 columns
  L.val = o; if (lcsr) o += (max_nnz + 3) & ~3;
  L.total = o;
  return L;
}


// Σ_e val[e] · f(col[e]) over one CSR row: four neighbours' loads in flight at a time,
// then a tail of a pair and a single.  (Measured and dropped on C5, profiles/r03_c5ab/: w
// entries per branch-free step with indices past the row clamped, w = 4 2.97 and w = 8 2.65
// against 3.88 M pairs/s; the padded entries' LDS gathers cost more than the round trips
// they save.)  The CSR row extents of a lane's rows are loaded once per unit.
template <typename CT, typename F>
__device__ __forceinline__ void csr_row(const CT *__restrict__ col, const float *__restrict__ val,
                                        int e0, int e1, F f) {
  int e = e0;
  for (; e + 4 <= e1; e += 4) {
    const int c0 = col[e], c1 = col[e + 1], c2 = col[e + 2], c3 = col[e + 3];
    const float v0 = val[e], v1 = val[e + 1], v2 = val[e + 2], v3 = val[e + 3];
    f(c0, v0);
    f(c1, v1);
    f(c2, v2);
    f(c3, v3);
  }
  // a tail of 2-3 entries as a pair then a single (two dependent round trips, not three)
  if (e + 2 <= e1) {
    const int c0 = col[e], c1 = col[e + 1];
    const float v0 = val[e], v1 = val[e + 1];
    f(c0, v0);
    f(c1, v1);
    e += 2;
  }
  if (e < e1) f(col[e], val[e]);
}

// instance (.x, -1: none) of wave w in unit slot u of the partitioned size-class order
// (web_icls_scan), and the unit size (.y): class c's slots start at ub_c; slot ub_c +
// np r + p is unit r of key (c, p), i.e. instances icls[k] + gsz r .. of the sorted list,
// or empty when partition p has fewer units.  With np = kXcdParts and gridDim.x a multiple
// of it, every unit of partition p runs on the XCD of blocks b = p (mod np).
__device__ __forceinline__ int2 web_unit_q(int u, const int32_t *isorted, const int32_t *icls, int ni,
                                           int ub1, int ub2, int np, int n_units, int w, int gw) {
  if (!isorted) return make_int2(u < ni ? u : -1, 1);
  const bool a0 = u < ub1, a1 = !a0 && u < ub2;
  const int gsz = a0 ? 4 : (a1 ? 2 : 1);
  const int rel = u - (a0 ? 0 : (a1 ? ub1 : ub2));
  const int r = rel / np, k = (a0 ? 0 : (a1 ? 1 : 2)) * kXcdParts + (rel - r * np);
  const int s0 = icls[k] + r * gsz, end = icls[k + 1];
  const int kk = w / (gw / gsz);
  return make_int2((u < n_units && s0 + kk < end) ? isorted[s0 + kk] : -1, gsz);
}

// the forward's keep draws (the backward reads them back)
__device__ __forceinline__ bool web_fkeep(uint32_t pk, uint32_t layer, uint32_t side, uint32_t e,
                                          uint32_t thr) {
  return sg_keep(pk, layer, side, e, thr);
}

template <bool BWD, int NTB, bool LCSR>
__global__ void __launch_bounds__(64 * gcn_gw(BWD)) web_gcn_kernel(GcnArgs A) {
  using ColT = typename std::conditional<LCSR, uint16_t, int>::type;
  constexpr int GW_ = gcn_gw(BWD), NT = 64 * GW_, GCN_TPW = (32 + GW_ - 1) / GW_;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int i = l & 15, g = l >> 4;
  const int d_in = A.d_in;
  const int n16max = (A.n_max + 15) & ~15;
  const GcnLds L = gcn_lds(d_in, n16max, A.max_nnz, BWD, LCSR);
  float *sW0 = sm + L.w0, *sb0 = sm + L.b0, *sW1 = sm + L.w1, *sW1T = sm + L.w1t;
  float *sb1 = sm + L.b1, *sWd = sm + L.wd;
  int *sEt = (int *)(sm + L.et);
  float *sZ1 = sm + L.z1, *sD1 = sm + L.d1, *scr = sm + L.scr + w * SCR;
  int *sRp = (int *)(sm + L.rp);
  uint16_t *sCol = (uint16_t *)(sm + L.col);
  float *sVal = sm + L.val;
  const float *prm = A.params;
  for (int x = tid; x < (d_in + 1) * WH1; x += NT)
    sW0[(x / WH1) * W0S + x % WH1] = x < d_in * WH1 ? prm[x] * A.ik0 : 0.f;
  for (int x = tid; x < WH1 * WH2; x += NT) {
    const float v = prm[A.oW1 + x] * A.ik1;
    sW1[x] = v;
    sW1T[(x % WH2) * WH1 + x / WH2] = v;
  }
  // gD1's B operands: lane (i, g) of feature half cb holds the parts of
  // W1[16cb + i][4g..4g+3]·ik1 as (H | H), (M | H), (L | M) (k-slots 8g..8g+7)
  uint4 *sW1B = (uint4 *)(sm + L.w1b);
  if (BWD)
    for (int x = tid; x < 2 * 3 * 64; x += NT) {
      const int cb = x / 192, term = (x / 64) % 3, ln = x & 63;
      const float *wr = prm + A.oW1 + (16 * cb + (ln & 15)) * WH2 + 4 * (ln >> 4);
      uint32_t h01, m01, l01, h23, m23, l23;
      sgk::split3(wr[0] * A.ik1, wr[1] * A.ik1, h01, m01, l01);
      sgk::split3(wr[2] * A.ik1, wr[3] * A.ik1, h23, m23, l23);
      sW1B[x] = term == 0 ? uint4{h01, h23, h01, h23}
                          : (term == 1 ? uint4{m01, m23, h01, h23} : uint4{l01, l23, m01, m23});
    }
  if (tid < WH1) sb0[tid] = prm[A.ob0 + tid];
  if (tid < WH2) {
    sb1[tid] = prm[A.ob1 + tid];
    sWd[tid] = prm[A.oWd + tid] * A.ik2;
  }
  const float bd = prm[A.obd];

  // gradient accumulators (backward), persistent over the block's instances
  f4 aW0[NTB][2], aW1[2];
  float aB0[2] = {0.f, 0.f}, aB1[4] = {0.f, 0.f, 0.f, 0.f}, aWd[4] = {0.f, 0.f, 0.f, 0.f};
  float aBd = 0.f;
#pragma unroll
  for (int t = 0; t < NTB; ++t) aW0[t][0] = aW0[t][1] = f4{0.f, 0.f, 0.f, 0.f};
  aW1[0] = aW1[1] = f4{0.f, 0.f, 0.f, 0.f};

  // ---- unit schedule (GcnArgs::isorted): unit u -> (instances per unit gsz, first
  // sorted slot, instances present); this thread's instance is number w / (GW_ / gsz)
  const int64_t n_inst = 2 * A.n_pairs;
  // (32-bit: a chunk has < 2^31 instances; selects, not branches, so that no table of
  // the three cases is built in scratch)
  // (the lambdas below capture locals only: a reference to the kernel argument block
  // would make the compiler copy it to scratch)
  const int ni = (int)n_inst;
  const int32_t *const isorted = A.isorted;
  const int4 *const ginst = A.inst;
  const int32_t *const grow_ptr = A.row_ptr, *const gtypes = A.types, *const gcol = A.col;
  const float *const gval = A.val, *const gGX = A.GX;
  const int64_t gCp = A.Cp;
  const int gDp = A.Dp;
  const int32_t *const icls = A.icls;
  int ub1 = ni, ub2 = ni, np = 1, n_units = ni;
  if (isorted) {
    ub1 = __builtin_amdgcn_readfirstlane(icls[kIKeys + 2]);
    ub2 = __builtin_amdgcn_readfirstlane(icls[kIKeys + 3]);
    n_units = __builtin_amdgcn_readfirstlane(icls[kIKeys + 4]);
    np = __builtin_amdgcn_readfirstlane(icls[kIKeys + 5]);
  }
  // this thread's instance of unit u (.x, -1: none) and the unit size (.y): a plain
  // function of values (a lambda's closure got its selects turned into loads from scratch)
  auto unit_q = [&](int u) __attribute__((always_inline)) -> int2 {
    return web_unit_q(u, isorted, icls, ni, ub1, ub2, np, n_units, w, GW_);
  };

  // The next unit's inputs are prefetched into registers while this one computes:
  // its (o, N, eb, nnz) at the top of the iteration, its rows after the first phase.
  // Every thread serves its own instance: node lt = its thread index in the instance's
  // share of the block (NT / gsz threads).
  constexpr int KM = LCSR ? 4096 / NT : 1;   // CSR entries per thread (LCSR: nnz <= 4096)
  int pr_rp = 0, pr_ty = 0, pr_col[KM];
  float pr_val[KM], pr_gx = 0.f;
  auto load_rows = [&](int64_t q, int4 in, int lt) __attribute__((always_inline)) {
    const int o = in.x, N = in.y, eb = in.z, nnz = in.w;
    pr_rp = lt < N ? grow_ptr[o + lt] - eb : 0;
    pr_ty = lt < N ? gtypes[o + lt] : 0;
    if (BWD)
      pr_gx = lt < N ? gGX[((int64_t)(q & 1) * gCp + (q >> 1)) * gDp + lt] : 0.f;
    if (LCSR) {
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int e = tid + k * NT;
        pr_col[k] = e < nnz ? gcol[eb + e] : 0;
        pr_val[k] = e < nnz ? gval[eb + e] : 0.f;
      }
    }
  };
  const int2 u0_ = unit_q(blockIdx.x);
  int64_t q = u0_.x;
  int gsz = u0_.y;
  int4 in = make_int4(0, 0, 0, 0);
  {
    const int nt_ = NT / gsz, lt_ = tid - (w / (GW_ / gsz)) * nt_;
    if (q >= 0) {
      in = ginst[q];
      load_rows(q, in, lt_);
    }
  }
  for (int unit = blockIdx.x; unit < n_units; unit += gridDim.x) {
    __syncthreads();   // the previous unit (or the table build) is done with the LDS
    // this thread's instance of the unit: waves [k WPI, (k+1) WPI), instance region k
    const int WPI = GW_ / gsz, NTL = NT / gsz;
    const int kin = w / WPI, lw = w - kin * WPI, lt = tid - kin * NTL;
    const int cap = (n16max / gsz) & ~15;
    const int kreg = kin * cap;
    int *sEtk = sEt + kreg;
    float *sGxk = sm + L.gx + kreg;
    float *sZ1k = sZ1 + kreg * ZS;
    float *sD1k = sD1 + kreg * DS;
    const int64_t p = q >= 0 ? (q >> 1) : 0;
    const int side = (int)(q & 1);
    const int o = in.x, N = q >= 0 ? in.y : 0;
    const int n16 = (N + 15) & ~15;
    const int ntile = n16 >> 4;
    const uint32_t pk = sg_pair_key(A.key, (uint32_t)(A.pair_offset + p));
    // dropout keep bits of this lane's tiles: the backward loads the forward's (their
    // latency overlaps the staging below), the forward builds them
    uint32_t mw[GCN_TPW];
    constexpr bool use_mw = BWD;   // sg_web_run passes masks then
    constexpr bool use_d2 = BWD;   // ... and the D2 rows
    f4 d2v[GCN_TPW];
#pragma unroll
    for (int u = 0; u < GCN_TPW; ++u) {
      const int n = 16 * (lw + u * WPI) + i;
      mw[u] = (use_mw && n < N) ? (uint32_t)A.masks[((size_t)q * A.Dp + n) * 4 + g] : 0u;
      d2v[u] = (use_d2 && n < N) ? *(const f4 *)(A.d2 + ((size_t)q * A.Dp + n) * 16 + 4 * g)
                                 : f4{0.f, 0.f, 0.f, 0.f};
    }
    const int *rp;
    const ColT *cl;
    const float *vl;
    // stage the prefetched rows; effective one-hot column per node (sparse dropout of
    // X, layer 0, e = node: d_in = the zero row of sW0 for dropped and absent nodes)
    if (lt < n16)
      sEtk[lt] = (lt < N && sg_keep(pk, 0, side, lt, A.thr0)) ? pr_ty : d_in;
    if (BWD && lt < n16) sGxk[lt] = pr_gx;
    if (LCSR) {   // units of one instance only (the host passes no isorted with LCSR)
      if (tid < N) sRp[tid] = pr_rp;
      if (tid == 0) sRp[N] = in.w;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int e = tid + k * NT;
        if (e < in.w) {
          sCol[e] = (uint16_t)pr_col[k];
          sVal[e] = pr_val[k];
        }
      }
      rp = sRp; cl = (const ColT *)(const void *)sCol; vl = sVal;
    } else {
      rp = A.row_ptr + o; cl = (const ColT *)(const void *)A.col; vl = A.val;
    }
    const int2 un_ = unit_q(unit + gridDim.x);
    const int64_t qn = un_.x;
    const int gszn = un_.y;
    const int4 inn = qn >= 0 ? ginst[qn] : make_int4(0, 0, 0, 0);
    __syncthreads();
    // the CSR extents of this lane's rows (node 16t + i of each of its tiles), loaded
    // together once per unit: every one-row-per-lane phase below starts from them
    // instead of a dependent row-pointer load before each row's gather
    int re0[GCN_TPW], re1[GCN_TPW];
#pragma unroll
    for (int u = 0; u < GCN_TPW; ++u) {
      const int n = 16 * (lw + u * WPI) + i;
      const bool in_ = n < N;
      re0[u] = in_ ? rp[n] : 0;
      re1[u] = in_ ? rp[n + 1] : 0;
    }
    auto row0 = [&](int u, int n) __attribute__((always_inline)) -> int {
      return re0[u];
    };
    auto row1 = [&](int u, int n) __attribute__((always_inline)) -> int {
      return re1[u];
    };

    // ---- forward: H1 (lane (i, g): node 16t+i, features 16c + 4g + s), D1', Z1 ----
#pragma unroll
    for (int u = 0; u < GCN_TPW; ++u) {
      const int t = lw + u * WPI;
      if (t >= ntile) break;
      const int n = 16 * t + i;
      float h[8];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float4 b = *(const float4 *)(sb0 + 16 * c + 4 * g);
        h[4 * c] = b.x; h[4 * c + 1] = b.y; h[4 * c + 2] = b.z; h[4 * c + 3] = b.w;
      }
      if (n < N) {
        csr_row(cl, vl, row0(u, n), row1(u, n), [&](int mm, float v) {
          const float *wr = sW0 + sEtk[mm] * W0S + 4 * g;
          const float4 wa = *(const float4 *)wr, wb = *(const float4 *)(wr + 16);
          h[0] = fmaf(v, wa.x, h[0]); h[1] = fmaf(v, wa.y, h[1]);
          h[2] = fmaf(v, wa.z, h[2]); h[3] = fmaf(v, wa.w, h[3]);
          h[4] = fmaf(v, wb.x, h[4]); h[5] = fmaf(v, wb.y, h[5]);
          h[6] = fmaf(v, wb.z, h[6]); h[7] = fmaf(v, wb.w, h[7]);
        });
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int f = 16 * c + 4 * g + s;
            const float hv = sgk::relu_bits(h[4 * c + s]);
            const bool k1 = use_mw ? ((mw[u] >> (4 * c + s)) & 1u) != 0u
                                   : web_fkeep(pk, 1, side, (uint32_t)(n * WH1 + f), A.thr1);
            if (!BWD) mw[u] |= (k1 ? 1u : 0u) << (4 * c + s);
            h[4 * c + s] = k1 ? hv : 0.f;
          }
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) h[s] = 0.f;
      }
      if (!use_d2) {   // Z1 = D1'·W1 (the backward with D2 rows needs no Z1)
        f4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int s = 0; s < 4; ++s) z = mfma4(h[4 * c + s], sW1[(16 * c + 4 * g + s) * WH2 + i], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) sZ1k[(16 * t + 4 * g + r) * ZS + i] = z[r];
      }
      if (BWD) {
        *(float4 *)(sD1k + n * DS + 4 * g) = make_float4(h[0], h[1], h[2], h[3]);
        *(float4 *)(sD1k + n * DS + 16 + 4 * g) = make_float4(h[4], h[5], h[6], h[7]);
      }
    }
    if (!use_d2) __syncthreads();   // Z1 complete before the H2 pass gathers it
    if (qn >= 0) {   // lands during the rest of this unit
      const int ntn = NT / gszn;
      load_rows(qn, inn, tid - (w / (GW_ / gszn)) * ntn);
    }

    // ---- H2 (lane (i, g): node 16t+i, features 4g..4g+3), Dense, Padding, NTN input ----
    float gzr[GCN_TPW][4];
#pragma unroll
    for (int u = 0; u < GCN_TPW; ++u) {
      const int t = lw + u * WPI;
      if (t >= ntile) break;
      const int n = 16 * t + i;
      float h2[4] = {0.f, 0.f, 0.f, 0.f};
      if (use_d2) {   // D2 = dropout(H2) as the forward wrote it (k2 applied: k2 ? h2 : 0)
#pragma unroll
        for (int s = 0; s < 4; ++s) h2[s] = d2v[u][s];
      } else if (n < N) {
        const float4 b = *(const float4 *)(sb1 + 4 * g);
        h2[0] = b.x; h2[1] = b.y; h2[2] = b.z; h2[3] = b.w;
#ifdef SG_WEB_ABL_NOH2   // timing ablation only (results invalid): the backward skips the H2 pass
        if (!BWD)
#endif
        csr_row(cl, vl, row0(u, n), row1(u, n), [&](int mm, float v) {
          const float4 zz = *(const float4 *)(sZ1k + mm * ZS + 4 * g);
          h2[0] = fmaf(v, zz.x, h2[0]); h2[1] = fmaf(v, zz.y, h2[1]);
          h2[2] = fmaf(v, zz.z, h2[2]); h2[3] = fmaf(v, zz.w, h2[3]);
        });
      }
      bool k2[4];
      float part = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        k2[s] = use_mw ? ((mw[u] >> (8 + s)) & 1u) != 0u
                       : web_fkeep(pk, 2, side, (uint32_t)(n * WH2 + 4 * g + s), A.thr2);
        if (!BWD) mw[u] |= (k2[s] ? 1u : 0u) << (8 + s);
        part = fmaf(k2[s] ? h2[s] : 0.f, sWd[4 * g + s], part);
      }
      const float pre = sgk::xsum32(sgk::xsum16(part)) + bd;
      const float z = sgk::relu_bits(pre);
      const bool k4 = n < N && (use_mw ? ((mw[u] >> 12) & 1u) != 0u
                                       : web_fkeep(pk, 4, side, (uint32_t)n, A.thr4));
      if (!BWD) {
        if (g == 0 && n < N)
          A.X[((int64_t)side * A.Cp + p) * A.Dp + n] = k4 ? z * A.ik4 : 0.f;
        if (A.d2 != nullptr && n < N)
          *(f4 *)(A.d2 + ((size_t)q * A.Dp + n) * 16 + 4 * g) =
              f4{k2[0] ? h2[0] : 0.f, k2[1] ? h2[1] : 0.f, k2[2] ? h2[2] : 0.f, k2[3] ? h2[3] : 0.f};
        if (A.masks != nullptr && n < N)
          A.masks[((size_t)q * A.Dp + n) * 4 + g] = (uint16_t)(mw[u] | (k4 ? 1u << 12 : 0u));
      } else {
        // Dense / Padding / NTN-input backward: gZ1 (= gH2, identity act) in registers
        const float gx = k4 ? sGxk[n] * A.ik4 : 0.f;
        const float gp = (n < N && pre > 0.f) ? gx : 0.f;
        if (g == 0) aBd += gp;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          aWd[s] = fmaf(k2[s] ? h2[s] : 0.f, gp, aWd[s]);
          gzr[u][s] = k2[s] ? gp * sWd[4 * g + s] : 0.f;
          aB1[s] += gzr[u][s];
        }
      }
    }
    if (!BWD) {
      // Padding rows [N, Dp): padding_value (zero beyond D), after the NTN-input dropout
      if (q >= 0)
        for (int a = N + lt; a < A.Dp; a += NTL)
          A.X[((int64_t)side * A.Cp + p) * A.Dp + a] =
              (a < A.D && A.padv != 0.f && sg_keep(pk, 4, side, (uint32_t)a, A.thr4))
                  ? A.padv * A.ik4 : 0.f;
      in = inn;
      q = qn;
      gsz = gszn;
      continue;
    }
    if (!use_d2) __syncthreads();   // every wave is done reading Z1: it becomes gZ1
#pragma unroll
    for (int u = 0; u < GCN_TPW; ++u) {
      const int t = lw + u * WPI;
      if (t >= ntile) break;
      *(float4 *)(sZ1k + (16 * t + i) * ZS + 4 * g) =
          make_float4(gzr[u][0], gzr[u][1], gzr[u][2], gzr[u][3]);
    }
    __syncthreads();

    // ---- gS1 = Â·gZ1 (lane (i, g): node 16t+i, j = 4g..4g+3); gD1 = gS1·W1ᵀ; gW1 ----
#pragma unroll
    for (int u = 0; u < GCN_TPW; ++u) {
      const int t = lw + u * WPI;
      if (t >= ntile) break;
      const int n = 16 * t + i;
      float q4[4] = {0.f, 0.f, 0.f, 0.f};
      if (n < N)
        csr_row(cl, vl, row0(u, n), row1(u, n), [&](int mm, float v) {
          const float4 gg = *(const float4 *)(sZ1k + mm * ZS + 4 * g);
          q4[0] = fmaf(v, gg.x, q4[0]); q4[1] = fmaf(v, gg.y, q4[1]);
          q4[2] = fmaf(v, gg.z, q4[2]); q4[3] = fmaf(v, gg.w, q4[3]);
        });
      // gD1·ik1 (rows n = 16t + 4g + r, column f = 16cb + i)
      f4 gd[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
      {   // A k-slots 8g..8g+7 = (h | m) or (h | l) of gS1[n][4g..4g+3]: hH + mH + hM + lH + hL + mM
        uint32_t h01, m01, l01, h23, m23, l23;
        sgk::split3(q4[0], q4[1], h01, m01, l01);
        sgk::split3(q4[2], q4[3], h23, m23, l23);
        const uint4 ahm = {h01, h23, m01, m23}, ahl = {h01, h23, l01, l23};
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const uint4 *wb = sW1B + cb * 192 + l;
          gd[cb] = sgk::mfbf(ahm, wb[0], gd[cb]);
          gd[cb] = sgk::mfbf(ahl, wb[64], gd[cb]);
          gd[cb] = sgk::mfbf(ahm, wb[128], gd[cb]);
        }
      }
      // the tile's gS1 through the wave's scratch, read back as the B operand of gW1
      *(float4 *)(scr + i * SCS + 4 * g) = make_float4(q4[0], q4[1], q4[2], q4[3]);
      sg_wsync();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int nn = 16 * t + 4 * g + s;
        const float b = scr[(4 * g + s) * SCS + i];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) aW1[cb] = mfma4(sD1k[nn * DS + 16 * cb + i], b, aW1[cb]);
      }
      sg_wsync();
      // gP0 = relu'·keep·gD1·ik1 = (D1' > 0) · gD1·ik1, in place of D1'
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float *dp = sD1k + (16 * t + 4 * g + r) * DS + 16 * cb + i;
          const float v = *dp > 0.f ? gd[cb][r] : 0.f;
          aB0[cb] += v;
          *dp = v;
        }
    }
    __syncthreads();

    // ---- gS0 = Â·gP0; gW0 += Xᵀ·(scale0·gS0) ----
#pragma unroll
    for (int u = 0; u < GCN_TPW; ++u) {
      const int t = lw + u * WPI;
      if (t >= ntile) break;
      // one CSR row per lane: node n = 16t + i, features 16c + 4g + s (two b128 reads of
      // the gP0 row per entry); dropped and absent nodes (et = d_in) contribute zero
      float hq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      {
        const int n = 16 * t + i;
        if (n < N && sEtk[n] < d_in)
          csr_row(cl, vl, row0(u, n), row1(u, n), [&](int mm, float v) {
            const float *dr = sD1k + mm * DS + 4 * g;
            const float4 da = *(const float4 *)dr, db = *(const float4 *)(dr + 16);
            hq[0] = fmaf(v, da.x, hq[0]); hq[1] = fmaf(v, da.y, hq[1]);
            hq[2] = fmaf(v, da.z, hq[2]); hq[3] = fmaf(v, da.w, hq[3]);
            hq[4] = fmaf(v, db.x, hq[4]); hq[5] = fmaf(v, db.y, hq[5]);
            hq[6] = fmaf(v, db.z, hq[6]); hq[7] = fmaf(v, db.w, hq[7]);
          });
      }
      int et[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) et[s] = sEtk[16 * t + 4 * g + s];
      // one-hot Xᵀ as a bf16 A operand: row i ↔ type 16tb + i, k-slot 4g + s ↔ node
      // 16t + 4g + s (v_mfma_f32_16x16x16_bf16: 4 k-slots per lane)
      uint2 oh[NTB];
#pragma unroll
      for (int tb = 0; tb < NTB; ++tb) {
        uint32_t o[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) o[s] = et[s] == 16 * tb + i ? 0x3F80u : 0u;   // bf16 1.0
        oh[tb] = uint2{o[0] | (o[1] << 16), o[2] | (o[3] << 16)};
      }
      // per feature half c: the tile through the scratch, read back as the B operand
      // (k-slot g ↔ node 16t + 4g + s, column i ↔ feature 16c + i)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        *(float4 *)(scr + i * SCS + 4 * g) =
            make_float4(hq[4 * c] * A.ik0, hq[4 * c + 1] * A.ik0, hq[4 * c + 2] * A.ik0,
                        hq[4 * c + 3] * A.ik0);
        sg_wsync();
        float bq[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) bq[s] = scr[(4 * g + s) * SCS + i];
        sg_wsync();
        uint32_t h01, m01, l01, h23, m23, l23;
        sgk::split3(bq[0], bq[1], h01, m01, l01);
        sgk::split3(bq[2], bq[3], h23, m23, l23);
#pragma unroll
        for (int tb = 0; tb < NTB; ++tb) {
          aW0[tb][c] = sgk::mfbf16(oh[tb], uint2{l01, l23}, aW0[tb][c]);
          aW0[tb][c] = sgk::mfbf16(oh[tb], uint2{m01, m23}, aW0[tb][c]);
          aW0[tb][c] = sgk::mfbf16(oh[tb], uint2{h01, h23}, aW0[tb][c]);
        }
      }
    }
    in = inn;
    q = qn;
    gsz = gszn;
  }
  if (!BWD) return;
  __syncthreads();

  // ---- flush: waves 0-7 store their gradient contributions into LDS rows 0-7,
  // waves 8-15 add theirs into rows w-8 (every element is owned by one lane of each
  // wave), then the block sums the 8 rows in order into its slab row (deterministic) ----
  const int C = A.n_gcn;
  float *row = sm + L.tables + (w & 7) * C;   // the instance region is dead
  auto put = [&](int x, float v) {
    if (w < 8) row[x] = v;
    else row[x] += v;
  };
  for (int pass = 0; pass < 2; ++pass) {
    if ((w >= 8) == (pass == 1)) {
#pragma unroll
      for (int tb = 0; tb < NTB; ++tb)
#pragma unroll
        for (int fb = 0; fb < 2; ++fb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ty = 16 * tb + 4 * g + r;
            if (ty < d_in) put(ty * WH1 + 16 * fb + i, aW0[tb][fb][r]);
          }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const float v = sgk::xsum32(sgk::xsum16(aB0[cb]));
        if (g == 0) put(A.ob0 + 16 * cb + i, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) put(A.oW1 + (16 * cb + 4 * g + r) * WH2 + i, aW1[cb][r] * A.ik1);
      }
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const float vb = sgk::row_sum16(aB1[s2]);
        const float vd = sgk::row_sum16(aWd[s2]) * A.ik2;
        if (i == 0) {
          put(A.ob1 + 4 * g + s2, vb);
          put(A.oWd + 4 * g + s2, vd);
        }
      }
      const float bsum = sg_wave_sum(aBd);
      if (l == 0) put(A.obd, bsum);
    }
    __syncthreads();
  }
  float *dst = A.slab + (size_t)blockIdx.x * C;
  for (int x = tid; x < C; x += NT) {
    float v = 0.f;
    for (int uu = 0; uu < 8; ++uu) v += sm[L.tables + uu * C + x];
    dst[x] += v;
  }
}

// ---------------------------------------------------------------------------
// 128×128 f32 MFMA GEMM tiles (4 waves as 2×2, 64×64 per wave).
// MK layout: rows m, 16 contraction values + pad (one b128 read per 4 k-steps with
// the k-step order kk = 4g + s); KM layout: 16 contraction rows × 128 (+4).
// ---------------------------------------------------------------------------
struct Tile {
  f4 c[4][4];
  __device__ void zero() {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) c[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  }
};

__device__ __forceinline__ void mma_mk_mk(Tile &T, const float *sA, const float *sB, int wm,
                                          int wn, int i, int g) {
  float4 a[4], b[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    a[x] = *(const float4 *)(sA + (wm * 64 + x * 16 + i) * MKS + 4 * g);
    b[x] = *(const float4 *)(sB + (wn * 64 + x * 16 + i) * MKS + 4 * g);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const float av = s == 0 ? a[mi].x : s == 1 ? a[mi].y : s == 2 ? a[mi].z : a[mi].w;
        const float bv = s == 0 ? b[ni].x : s == 1 ? b[ni].y : s == 2 ? b[ni].z : b[ni].w;
        T.c[mi][ni] = mfma4(av, bv, T.c[mi][ni]);
      }
}

__device__ __forceinline__ void mma_km_km(Tile &T, const float *sA, const float *sB, int wm,
                                          int wn, int i, int g) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float a[4], b[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      a[x] = sA[(4 * g + s) * KMS + wm * 64 + x * 16 + i];
      b[x] = sB[(4 * g + s) * KMS + wn * 64 + x * 16 + i];
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) T.c[mi][ni] = mfma4(a[mi], b[ni], T.c[mi][ni]);
  }
}

// ---- T on bf16 MFMAs: both operands are split on the
// fly into three bf16 parts (x = h + m + l, sgk::split3: |x - h - m - l| < 2^-21 |x|)
// and T accumulates hh + hm + mh + hl + lh + mm in f32 on v_mfma_f32_16x16x32_bf16:
// 6 MFMAs of 16 cycles per 32-deep product instead of 8 f32 MFMAs of 32 cycles.
// LDS: [part][128 rows][40 bf16] per operand (80-byte rows: the b128 fragment reads
// of 8 consecutive rows fall on distinct banks), 60 KiB; 32-deep contraction chunks,
// the next chunk's f32 operands prefetched into registers during the MFMAs.
constexpr int B3K = 32, B3S = 40;   // contraction chunk, LDS row stride (bf16)

// Block order of the pair-block GEMMs.  (Measured and dropped: a 1-D grid where the NT column
// tiles of pair block pb (and, for T, each k, slowest) run on blocks L ≡ pb (mod 8), which
// the dispatcher deals to one XCD, so that the pair block's x rows would come into that
// XCD's L2 once for all its tiles.  Measured 3.82-3.84 against 4.21-4.22 M pairs/s on C5
// (profiles/r03_c5ab/gemm_*).)  The grid is (pair block, tile, k).
__device__ __forceinline__ void web_pb_tile(int NT, int G8, int &pb, int &tile, int &kk) {
  pb = (int)blockIdx.x;
  tile = (int)blockIdx.y;
  kk = (int)blockIdx.z;
}
static dim3 web_pb_grid(int64_t nblk, int NT, int K) {
  return dim3((unsigned)nblk, (unsigned)NT, (unsigned)K);
}
// gX1 / gX2 GEMMs: the contraction runs over (32-deep chunk, k) with k inner, so a chunk's
// x rows are loaded once and rescaled by gm[p][k] for each k (k outer, the chunk reloaded
// per k, measured 4.19-4.20 against 4.21-4.22 M pairs/s on C5)
constexpr int B3PART = TB * B3S;    // bf16 per part plane

__device__ __forceinline__ void b3_split_store(uint16_t *plane, int r, int c, float4 x) {
  uint32_t h01, m01, l01, h23, m23, l23;
  sgk::split3(x.x, x.y, h01, m01, l01);
  sgk::split3(x.z, x.w, h23, m23, l23);
  const int o = r * B3S + c;
  *(uint2 *)(plane + o) = uint2{h01, h23};
  *(uint2 *)(plane + B3PART + o) = uint2{m01, m23};
  *(uint2 *)(plane + 2 * B3PART + o) = uint2{l01, l23};
}

// MFUSE: instead of T, write the tile's share of the bilinear term,
// MP[p][k][a-tile] = Σ_{a in the tile} x1[p][a] T[p][k][a] (T itself never reaches memory:
// the head sums the a-tiles, and gx1's T term is a GEMM of its own, web_gx1_kernel_b3)
template <bool MFUSE>
__global__ void __launch_bounds__(256) web_t_kernel_b3(const float *__restrict__ X2,
                                                       const float *__restrict__ Wg,
                                                       const int2 *__restrict__ ext128, int64_t n,
                                                       int Dp, int K, float *__restrict__ Tout,
                                                       const float *__restrict__ X1) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[3 * B3PART], sB[3 * B3PART];
  __shared__ float mred[2][TB];
  int pbk, at, k;
  web_pb_tile(Dp / TB, (int)((n + TB * 8 - 1) / (TB * 8)), pbk, at, k);
  if ((int64_t)pbk * TB >= n) return;
  const int64_t p0 = (int64_t)pbk * TB;
  const int a0 = at * TB;
  const int2 e = ext128[pbk];
  if (a0 >= e.x) return;
  const int nb = (e.y + B3K - 1) / B3K * B3K;   // x2 is zero past n2 (Dp is a multiple of 128)
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, i = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  const float *pa = X2 + p0 * Dp;
  const float *pb = Wg + ((size_t)k * Dp + a0) * Dp;
  float4 ra[4], rb[4];
  auto load = [&](int b0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 3, c = (q & 7) * 4;
      ra[u] = *(const float4 *)(pa + (size_t)r * Dp + b0 + c);
      rb[u] = *(const float4 *)(pb + (size_t)r * Dp + b0 + c);
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f4{0.f, 0.f, 0.f, 0.f};
  if (nb > 0) load(0);
  for (int b0 = 0; b0 < nb; b0 += B3K) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 3, c = (q & 7) * 4;
      b3_split_store(sA, r, c, ra[u]);
      b3_split_store(sB, r, c, rb[u]);
    }
    __syncthreads();
    if (b0 + B3K < nb) load(b0 + B3K);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int oa = (wm * 64 + mi * 16 + i) * B3S + 8 * g;
      const uint4 ah = *(const uint4 *)(sA + oa), am = *(const uint4 *)(sA + B3PART + oa),
                  al = *(const uint4 *)(sA + 2 * B3PART + oa);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int ob = (wn * 64 + ni * 16 + i) * B3S + 8 * g;
        const uint4 bh = *(const uint4 *)(sB + ob), bm = *(const uint4 *)(sB + B3PART + ob),
                    bl = *(const uint4 *)(sB + 2 * B3PART + ob);
        f4 c = acc[mi][ni];
        c = sgk::mfbf(al, bh, c);
        c = sgk::mfbf(ah, bl, c);
        c = sgk::mfbf(am, bm, c);
        c = sgk::mfbf(am, bh, c);
        c = sgk::mfbf(ah, bm, c);
        c = sgk::mfbf(ah, bh, c);
        acc[mi][ni] = c;
      }
    }
    __syncthreads();
  }
  if (MFUSE) {
    // lane (i, g): rows 4g + r of each 16-row group, columns 16 ni + i of the wave's half
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pl = wm * 64 + mi * 16 + 4 * g + r;
        const float *x1 = X1 + (p0 + pl) * Dp + a0 + wn * 64 + i;
        float part = 0.f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) part = fmaf(x1[ni * 16], acc[mi][ni][r], part);
        part = sgk::row_sum16(part);
        if (i == 0) mred[wn][pl] = part;
      }
    __syncthreads();
    if (tid < TB && p0 + tid < n)
      Tout[((p0 + tid) * WKP + k) * 4 + at] = mred[0][tid] + mred[1][tid];
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t p = p0 + wm * 64 + mi * 16 + 4 * g + r;
      if (p >= n) continue;
      float *dst = Tout + ((size_t)p * K + k) * Dp + a0 + wn * 64 + i;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) dst[ni * 16] = acc[mi][ni][r];
    }
}

// ---- T with TKG feature maps k per block (round 4; SG_WEB_TKG=0 at run time: web_t_kernel_b3): web_t_kernel_b3
// re-fetched a pair block's x2 rows for each of its K x (a-tiles) tiles (18.45 GB per
// 524,288-pair chunk against ≈0.5 GB of x rows, rocprof FETCH_SIZE).  Here one 8-wave block
// stages the x2 chunk once for TKG = 4 feature maps k (the B operands of the four W[k]
// planes beside it: 150 KB of LDS, one block per CU), so x2 is fetched ceil(K / 4) times per
// a-tile instead of K times.  Wave w: k = 4 kg + 2 (w >> 2) + {0, 1}, 64x64 sub-tile
// ((w >> 1) & 1, w & 1).  Per (k, tile) the MFMA order is web_t_kernel_b3's, so MP is bitwise
// the same.
constexpr int TKG = 4;
__global__ void __launch_bounds__(512) web_t_kernel_kg(const float *__restrict__ X2,
                                                       const float *__restrict__ Wg,
                                                       const int2 *__restrict__ ext128, int64_t n,
                                                       int Dp, int K, float *__restrict__ Tout,
                                                       const float *__restrict__ X1) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[3 * B3PART], sB[TKG][3 * B3PART];
  __shared__ float mred[TKG][2][TB];
  const int pbk = (int)blockIdx.x, at = (int)blockIdx.y, kg = (int)blockIdx.z;
  if ((int64_t)pbk * TB >= n) return;
  const int64_t p0 = (int64_t)pbk * TB;
  const int a0 = at * TB;
  const int2 e = ext128[pbk];
  if (a0 >= e.x) return;
  const int nb = (e.y + B3K - 1) / B3K * B3K;   // x2 is zero past n2 (Dp is a multiple of 128)
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, i = l & 15, g = l >> 4;
  const int wk = w >> 2, wm = (w >> 1) & 1, wn = w & 1;
  const int k0 = kg * TKG;
  const int nk = K - k0 < TKG ? K - k0 : TKG;   // feature maps of this block
  const float *pa = X2 + p0 * Dp;
  float4 ra[2], rb[TKG][2];
  auto load = [&](int b0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = tid + 512 * u, r = q >> 3, c = (q & 7) * 4;
      ra[u] = *(const float4 *)(pa + (size_t)r * Dp + b0 + c);
#pragma unroll
      for (int kk = 0; kk < TKG; ++kk)
        if (kk < nk)
          rb[kk][u] = *(const float4 *)(Wg + ((size_t)(k0 + kk) * Dp + a0 + r) * Dp + b0 + c);
    }
  };
  f4 acc[2][4][4];
#pragma unroll
  for (int kx = 0; kx < 2; ++kx)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[kx][mi][ni] = f4{0.f, 0.f, 0.f, 0.f};
  if (nb > 0) load(0);
  for (int b0 = 0; b0 < nb; b0 += B3K) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = tid + 512 * u, r = q >> 3, c = (q & 7) * 4;
      b3_split_store(sA, r, c, ra[u]);
#pragma unroll
      for (int kk = 0; kk < TKG; ++kk)
        if (kk < nk) b3_split_store(sB[kk], r, c, rb[kk][u]);
    }
    __syncthreads();
    if (b0 + B3K < nb) load(b0 + B3K);
    // A fragments of two row groups mi at a time (the registers of all four, beside the
    // accumulators of two k and the next chunk's loads, would spill)
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
    uint4 ah[2], am[2], al[2];
#pragma unroll
    for (int m2 = 0; m2 < 2; ++m2) {
      const int oa = (wm * 64 + (2 * mh + m2) * 16 + i) * B3S + 8 * g;
      ah[m2] = *(const uint4 *)(sA + oa);
      am[m2] = *(const uint4 *)(sA + B3PART + oa);
      al[m2] = *(const uint4 *)(sA + 2 * B3PART + oa);
    }
#pragma unroll
    for (int kx = 0; kx < 2; ++kx) {
      const int kk = 2 * wk + kx;
      if (kk >= nk) continue;
      const uint16_t *sb = sB[kk];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int ob = (wn * 64 + ni * 16 + i) * B3S + 8 * g;
        const uint4 bh = *(const uint4 *)(sb + ob), bm = *(const uint4 *)(sb + B3PART + ob),
                    bl = *(const uint4 *)(sb + 2 * B3PART + ob);
#pragma unroll
        for (int m2 = 0; m2 < 2; ++m2) {
          const int mi = 2 * mh + m2;
          f4 c = acc[kx][mi][ni];
          c = sgk::mfbf(al[m2], bh, c);
          c = sgk::mfbf(ah[m2], bl, c);
          c = sgk::mfbf(am[m2], bm, c);
          c = sgk::mfbf(am[m2], bh, c);
          c = sgk::mfbf(ah[m2], bm, c);
          c = sgk::mfbf(ah[m2], bh, c);
          acc[kx][mi][ni] = c;
        }
      }
    }
    }
    __syncthreads();
  }
  // the tile's share of the bilinear term per k, as web_t_kernel_b3<true>
#pragma unroll
  for (int kx = 0; kx < 2; ++kx) {
    const int kk = 2 * wk + kx;
    if (kk >= nk) continue;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pl = wm * 64 + mi * 16 + 4 * g + r;
        const float *x1 = X1 + (p0 + pl) * Dp + a0 + wn * 64 + i;
        float part = 0.f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) part = fmaf(x1[ni * 16], acc[kx][mi][ni][r], part);
        part = sgk::row_sum16(part);
        if (i == 0) mred[kk][wn][pl] = part;
      }
  }
  __syncthreads();
  {
    const int kk = tid >> 7, pr = tid & 127;
    if (kk < nk && p0 + pr < n)
      Tout[((p0 + pr) * WKP + k0 + kk) * 4 + at] = mred[kk][0][pr] + mred[kk][1][pr];
  }
}

// ---- gX2 on bf16 MFMAs (as web_t_kernel_b3): A = gm[p][k] x1[p][a] scaled while
// staging, B = Wh[k][b][a]; 32-deep chunks of a for each k ----
__global__ void __launch_bounds__(256) web_gx2_kernel_b3(const float *__restrict__ X1,
                                                         const float *__restrict__ GM,
                                                         const float *__restrict__ Wh,
                                                         const int2 *__restrict__ ext128,
                                                         int64_t n, int Dp, int K,
                                                         float *__restrict__ GX2) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[3 * B3PART], sB[3 * B3PART];
  int pb, bt, kk_;
  web_pb_tile(Dp / TB, (int)((n + TB * 8 - 1) / (TB * 8)), pb, bt, kk_);
  if ((int64_t)pb * TB >= n) return;
  const int64_t p0 = (int64_t)pb * TB;
  const int b0 = bt * TB;
  const int2 e = ext128[pb];
  if (b0 >= e.y) return;
  const int na = (e.x + B3K - 1) / B3K * B3K;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, i = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  float4 ra[4], rb[4];
  float gmr[4];
  auto load = [&](int k, int a0, bool xload) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 3, c = (q & 7) * 4;
      const int64_t p = p0 + r;
      gmr[u] = p < n ? GM[p * WKP + k] : 0.f;
      if (xload) ra[u] = *(const float4 *)(X1 + p * Dp + a0 + c);
      rb[u] = *(const float4 *)(Wh + ((size_t)k * Dp + b0 + r) * Dp + a0 + c);
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f4{0.f, 0.f, 0.f, 0.f};
  const int steps = na / B3K, total = K * steps;
  if (total > 0) load(0, 0, true);
  for (int st = 0; st < total; ++st) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 3, c = (q & 7) * 4;
      const float gm = gmr[u];
      b3_split_store(sA, r, c, make_float4(gm * ra[u].x, gm * ra[u].y, gm * ra[u].z, gm * ra[u].w));
      b3_split_store(sB, r, c, rb[u]);
    }
    __syncthreads();
    if (st + 1 < total) {
      const int s1 = st + 1;
      load(s1 % K, (s1 / K) * B3K, s1 % K == 0);
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int oa = (wm * 64 + mi * 16 + i) * B3S + 8 * g;
      const uint4 ah = *(const uint4 *)(sA + oa), am = *(const uint4 *)(sA + B3PART + oa),
                  al = *(const uint4 *)(sA + 2 * B3PART + oa);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int ob = (wn * 64 + ni * 16 + i) * B3S + 8 * g;
        const uint4 bh = *(const uint4 *)(sB + ob), bm = *(const uint4 *)(sB + B3PART + ob),
                    bl = *(const uint4 *)(sB + 2 * B3PART + ob);
        f4 c = acc[mi][ni];
        c = sgk::mfbf(al, bh, c);
        c = sgk::mfbf(ah, bl, c);
        c = sgk::mfbf(am, bm, c);
        c = sgk::mfbf(am, bh, c);
        c = sgk::mfbf(ah, bm, c);
        c = sgk::mfbf(ah, bh, c);
        acc[mi][ni] = c;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t p = p0 + wm * 64 + mi * 16 + 4 * g + r;
      if (p >= n) continue;
      float *dst = GX2 + p * Dp + b0 + wn * 64 + i;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) dst[ni * 16] += acc[mi][ni][r];
    }
}

// ---- the T term of gX1 as a GEMM (with web_t_kernel_b3<true>, T is never stored):
// gX1[p][a] += Σ_{k,b} gm[p][k] x2[p][b] W[a][b][k]; A = gm·x2 scaled while staging,
// B = Wg[k][a][b]; 32-deep chunks of b for each k ----
__global__ void __launch_bounds__(256) web_gx1_kernel_b3(const float *__restrict__ X2,
                                                         const float *__restrict__ GM,
                                                         const float *__restrict__ Wg,
                                                         const int2 *__restrict__ ext128,
                                                         int64_t n, int Dp, int K,
                                                         float *__restrict__ GX1) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[3 * B3PART], sB[3 * B3PART];
  int pb, at, kk_;
  web_pb_tile(Dp / TB, (int)((n + TB * 8 - 1) / (TB * 8)), pb, at, kk_);
  if ((int64_t)pb * TB >= n) return;
  const int64_t p0 = (int64_t)pb * TB;
  const int a0 = at * TB;
  const int2 e = ext128[pb];
  if (a0 >= e.x) return;
  const int nb = (e.y + B3K - 1) / B3K * B3K;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, i = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  float4 ra[4], rb[4];
  float gmr[4];
  auto load = [&](int k, int b0, bool xload) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 3, c = (q & 7) * 4;
      const int64_t p = p0 + r;
      gmr[u] = p < n ? GM[p * WKP + k] : 0.f;
      if (xload) ra[u] = *(const float4 *)(X2 + p * Dp + b0 + c);
      rb[u] = *(const float4 *)(Wg + ((size_t)k * Dp + a0 + r) * Dp + b0 + c);
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f4{0.f, 0.f, 0.f, 0.f};
  const int steps = nb / B3K, total = K * steps;
  if (total > 0) load(0, 0, true);
  for (int st = 0; st < total; ++st) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 3, c = (q & 7) * 4;
      const float gm = gmr[u];
      b3_split_store(sA, r, c, make_float4(gm * ra[u].x, gm * ra[u].y, gm * ra[u].z, gm * ra[u].w));
      b3_split_store(sB, r, c, rb[u]);
    }
    __syncthreads();
    if (st + 1 < total) {
      const int s1 = st + 1;
      load(s1 % K, (s1 / K) * B3K, s1 % K == 0);
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int oa = (wm * 64 + mi * 16 + i) * B3S + 8 * g;
      const uint4 ah = *(const uint4 *)(sA + oa), am = *(const uint4 *)(sA + B3PART + oa),
                  al = *(const uint4 *)(sA + 2 * B3PART + oa);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int ob = (wn * 64 + ni * 16 + i) * B3S + 8 * g;
        const uint4 bh = *(const uint4 *)(sB + ob), bm = *(const uint4 *)(sB + B3PART + ob),
                    bl = *(const uint4 *)(sB + 2 * B3PART + ob);
        f4 c = acc[mi][ni];
        c = sgk::mfbf(al, bh, c);
        c = sgk::mfbf(ah, bl, c);
        c = sgk::mfbf(am, bm, c);
        c = sgk::mfbf(am, bh, c);
        c = sgk::mfbf(ah, bm, c);
        c = sgk::mfbf(ah, bh, c);
        acc[mi][ni] = c;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t p = p0 + wm * 64 + mi * 16 + 4 * g + r;
      if (p >= n) continue;
      float *dst = GX1 + p * Dp + a0 + wn * 64 + i;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) dst[ni * 16] += acc[mi][ni][r];
    }
}

// ---- gWs on bf16 MFMAs: the contraction runs over pairs, so the operands are staged
// transposed ([a][p] and [b][p], pairs contiguous): thread (column c, half h) loads the
// column of 16 pairs of one active 16-pair chunk (two active chunks per 32-deep step,
// any two: the k-slots are only summed), splits them and writes 32 bytes per part ----
// It also forms gV = gmᵀ [x1 | x2] (web_gv_kernel's sums) from the operands it stages:
// the blocks of b-tile 0 sum gm·x1 over their columns a, those of a-tile 0 gm·x2 over b.
__global__ void __launch_bounds__(256) web_wgrad_kernel_b3(const float *__restrict__ X1,
                                                           const float *__restrict__ X2,
                                                           const float *__restrict__ GM,
                                                           const int2 *__restrict__ ext16,
                                                           int64_t n, int Dp, int K,
                                                           float *__restrict__ GWS,
                                                           float *__restrict__ GVS) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[3 * B3PART], sB[3 * B3PART];
  __shared__ int act[1024];
  __shared__ int wcnt[4];
  __shared__ float gvh[2][TB];
  // ≈66.6 KB of static LDS: beyond the 64 KiB of earlier CDNA parts, within gfx950's
  // 160 KB per CU (the library is built for gfx950 only, build.py)
  static_assert(2 * 3 * B3PART * sizeof(uint16_t) + 1024 * sizeof(int) + 4 * sizeof(int) +
                    2 * TB * sizeof(float) <= 160 * 1024,
                "web_wgrad_kernel_b3 exceeds the gfx950 LDS");
  const int nbt = Dp / TB;
  const int a0 = (blockIdx.x / nbt) * TB, b0 = (blockIdx.x % nbt) * TB;
  const int k = blockIdx.y, s = blockIdx.z;
  const int64_t nc = (n + 15) / 16;
  const int64_t c0 = nc * s / WSPLIT, c1 = nc * (s + 1) / WSPLIT;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, i = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int col = tid & 127, half = tid >> 7;
  // raw prefetch registers (the gm scaling happens at the LDS store, so the loads of
  // the next step stay in flight during this step's MFMAs)
  float xg[16], xa[16], xb[16];
  auto stage = [&](int64_t c) {   // c < 0: a zero chunk
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t p = c * 16 + r;
      xg[r] = xa[r] = xb[r] = 0.f;
      if (c >= 0 && p < n) {
        xg[r] = GM[p * WKP + k];
        xa[r] = X1[p * Dp + a0 + col];
        xb[r] = X2[p * Dp + b0 + col];
      }
    }
  };
  const bool gv1 = (blockIdx.x % nbt) == 0, gv2 = (blockIdx.x / nbt) == 0;
  float gva = 0.f, gvb = 0.f;   // Σ gm·x1[a0 + col], Σ gm·x2[b0 + col] over this thread's pairs
  auto put = [&](uint16_t *plane, const float (&x)[16], bool scale) {
    uint32_t h[8], m[8], lo[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float v0 = scale ? xg[2 * q] * x[2 * q] : x[2 * q];
      const float v1 = scale ? xg[2 * q + 1] * x[2 * q + 1] : x[2 * q + 1];
      sgk::split3(v0, v1, h[q], m[q], lo[q]);
    }
    if (scale && gv1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) gva = fmaf(xg[r], x[r], gva);
    }
    if (!scale && gv2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) gvb = fmaf(xg[r], x[r], gvb);
    }
    uint16_t *d = plane + col * B3S + 16 * half;
    *(uint4 *)d = uint4{h[0], h[1], h[2], h[3]};
    *(uint4 *)(d + 8) = uint4{h[4], h[5], h[6], h[7]};
    *(uint4 *)(d + B3PART) = uint4{m[0], m[1], m[2], m[3]};
    *(uint4 *)(d + B3PART + 8) = uint4{m[4], m[5], m[6], m[7]};
    *(uint4 *)(d + 2 * B3PART) = uint4{lo[0], lo[1], lo[2], lo[3]};
    *(uint4 *)(d + 2 * B3PART + 8) = uint4{lo[4], lo[5], lo[6], lo[7]};
  };
  f4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f4{0.f, 0.f, 0.f, 0.f};
  for (int64_t wbase = c0; wbase < c1; wbase += 1024) {
    int na = 0;
    for (int r0 = 0; r0 < 1024 && wbase + r0 < c1; r0 += 256) {
      const int64_t c = wbase + r0 + tid;
      bool on = false;
      if (c < c1) {
        const int2 e = ext16[c];
        on = e.x > a0 && e.y > b0;
      }
      const uint64_t bal = __ballot(on);
      const int before = __popcll(bal & ((1ull << l) - 1ull));
      if (l == 0) wcnt[w] = __popcll(bal);
      __syncthreads();
      int off = na;
      for (int u = 0; u < w; ++u) off += wcnt[u];
      if (on) act[off + before] = (int)(r0 + tid);
      na += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
      __syncthreads();
    }
    if (na == 0) continue;
    const int nsteps = (na + 1) / 2;
    auto chunk_of = [&](int x) -> int64_t {   // this thread's chunk of 32-deep step x
      const int j = 2 * x + half;
      return j < na ? wbase + act[j] : (int64_t)-1;
    };
    stage(chunk_of(0));
    for (int x = 0; x < nsteps; ++x) {
      put(sA, xa, true);
      put(sB, xb, false);
      __syncthreads();
      if (x + 1 < nsteps) stage(chunk_of(x + 1));
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int oa = (wm * 64 + mi * 16 + i) * B3S + 8 * g;
        const uint4 ah = *(const uint4 *)(sA + oa), am = *(const uint4 *)(sA + B3PART + oa),
                    al = *(const uint4 *)(sA + 2 * B3PART + oa);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int ob = (wn * 64 + ni * 16 + i) * B3S + 8 * g;
          const uint4 bh = *(const uint4 *)(sB + ob), bm = *(const uint4 *)(sB + B3PART + ob),
                      bl = *(const uint4 *)(sB + 2 * B3PART + ob);
          f4 c = acc[mi][ni];
          c = sgk::mfbf(al, bh, c);
          c = sgk::mfbf(ah, bl, c);
          c = sgk::mfbf(am, bm, c);
          c = sgk::mfbf(am, bh, c);
          c = sgk::mfbf(ah, bm, c);
          c = sgk::mfbf(ah, bh, c);
          acc[mi][ni] = c;
        }
      }
      __syncthreads();
    }
  }
  float *base = GWS + (((size_t)s * K + k) * Dp) * Dp;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = a0 + wm * 64 + mi * 16 + 4 * g + r;
      float *dst = base + (size_t)a * Dp + b0 + wn * 64 + i;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) dst[ni * 16] += acc[mi][ni][r];
    }
  if (gv1 || gv2) {   // the two halves' sums, half 0 first (fixed order)
    if (half) {
      gvh[0][col] = gva;
      gvh[1][col] = gvb;
    }
    __syncthreads();
    if (!half) {
      float *gv = GVS + ((size_t)s * WKP + k) * 2 * Dp;
      if (gv1) gv[a0 + col] += gva + gvh[0][col];
      if (gv2) gv[Dp + b0 + col] += gvb + gvh[1][col];
    }
  }
}

// ---------------------------------------------------------------------------
// Per-pair NTN head: m_k, s, ŷ, loss, gm; gx1 = Σ_k gm_k (T_k + V_k),
// gx2 := Σ_k gm_k V_k[D + ·] (web_gx2 adds the W term).  One wave per pair.
// ---------------------------------------------------------------------------
struct HeadArgs {
  const float *X, *T, *params, *labels, *y_stats;
  const int2 *ext;
  const int2 *ext128;   // MT: per-128-pair extents (which a-tiles web_t_kernel_b3 computed)
  float *GX, *GM, *s_out, *hslab;
  int64_t n, Cp;
  int D, Dp, K, oV, oU, obn;
  int final_act, loss_mode, ntn_mode;
  float yeta, inv_batch;
};

// MT: T holds web_t_kernel_b3<true>'s a-tile shares MP[p][k][tile] of Σ_a x1[a] T[k][a]
// instead of T, and gx1 gets only its V term here (web_gx1_kernel_b3 adds the T term)
template <bool BWD, bool MT>
__global__ void __launch_bounds__(256) web_head_kernel(HeadArgs A) {
  extern __shared__ __attribute__((aligned(16))) float sV[];   // [K][2Dp]: V[k][a] | V[k][D+b]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int D = A.D, Dp = A.Dp, K = A.K;
  for (int x = tid; x < K * 2 * Dp; x += 256) {
    const int k = x / (2 * Dp), c = x % (2 * Dp);
    const int cc = c < Dp ? c : c - Dp;
    sV[x] = cc < D ? A.params[A.oV + k * 2 * D + (c < Dp ? 0 : D) + cc] : 0.f;
  }
  float U[WKP], bn[WKP];
  float usum = 0.f;
#pragma unroll
  for (int k = 0; k < WKP; ++k) {
    U[k] = k < K ? A.params[A.oU + k] : 0.f;
    bn[k] = (k < K && A.obn >= 0) ? A.params[A.obn + k] : 0.f;
    usum += U[k];
  }
  const float ybar = (A.loss_mode == SG_LOSS_BROADCAST && A.y_stats) ? A.y_stats[0] : 0.f;
  __syncthreads();
  const int nc = Dp / 64;
  float aLoss = 0.f, aU = 0.f, aB = 0.f;   // lane k: gU[k], gb[k]
  const int64_t gw = (int64_t)blockIdx.x * 4 + w, nw = (int64_t)gridDim.x * 4;
  for (int64_t p = gw; p < A.n; p += nw) {
    const int2 ex = A.ext[p];
    const int e1 = ex.x;
    // x1 / x2 are zero past the extents (padding 0) and gx past them is never read (the
    // instance kernels take ∂L/∂x of present nodes only): 64-wide column blocks up to the
    // larger extent
    const int ncp = min(nc, (max(ex.x, ex.y) + 63) >> 6);
    const float *x1 = A.X + p * Dp, *x2 = A.X + (A.Cp + p) * Dp;
    const float *Tp = A.T + (size_t)p * K * Dp;
    float m[WKP];
#pragma unroll
    for (int k = 0; k < WKP; ++k) m[k] = 0.f;
    for (int c = 0; c < ncp; ++c) {
      const int a = 64 * c + l;
      const float xa = x1[a], xb = x2[a];
#pragma unroll
      for (int k = 0; k < WKP; ++k) {
        if (k < K) {
          const float t = (!MT && a < e1) ? Tp[k * Dp + a] : 0.f;
          m[k] = fmaf(xa, t + sV[k * 2 * Dp + a], m[k]);
          m[k] = fmaf(xb, sV[k * 2 * Dp + Dp + a], m[k]);
        }
      }
    }
    float mt[WKP];   // MT: the bilinear term from the a-tile shares, tiles in order
#pragma unroll
    for (int k = 0; k < WKP; ++k) mt[k] = 0.f;
    if (MT) {
      const int ex = A.ext128[p / TB].x;
      const float *mp = A.T + (size_t)p * WKP * 4;
#pragma unroll
      for (int k = 0; k < WKP; ++k)
        if (k < K)
          for (int t = 0; t < 4 && t * TB < ex; ++t) mt[k] += mp[k * 4 + t];
    }
    float rsum = 0.f, s = 0.f;
#pragma unroll
    for (int k = 0; k < WKP; ++k) {
      if (k < K) {
        m[k] = sg_wave_sum(m[k]) + mt[k] + bn[k];
        const float r = m[k] > 0.f ? m[k] : 0.f;
        rsum += r;
        s = fmaf(U[k], r, s);
      }
    }
    if (A.ntn_mode == SG_NTN_REFERENCE) s = usum * rsum;   // quirk A1
    if (!BWD) {
      if (l == 0 && A.s_out) A.s_out[p] = s;
      continue;
    }
    const float yh = sg_final(A.final_act, A.yeta, s);
    float gy;
    if (A.loss_mode == SG_LOSS_BROADCAST) {
      gy = yh - ybar;                       // quirk A2: ∂/∂ŷ_j = ŷ_j - ȳ
      aLoss += 0.5f * gy * gy;
    } else {
      const float y = A.labels[p];
      gy = (yh - y) * A.inv_batch;
      aLoss += 0.5f * (y - yh) * (y - yh) * A.inv_batch;
    }
    const float gs = gy * sg_final_grad(A.final_act, A.yeta, s, yh);
    float gm[WKP];
#pragma unroll
    for (int k = 0; k < WKP; ++k) {
      const float gr = A.ntn_mode == SG_NTN_REFERENCE ? gs * usum : gs * U[k];
      gm[k] = (k < K && m[k] > 0.f) ? gr : 0.f;
      if (l == k) {
        aU += A.ntn_mode == SG_NTN_REFERENCE ? gs * rsum : gs * (m[k] > 0.f ? m[k] : 0.f);
        aB += gm[k];
      }
    }
    if (l < WKP) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < WKP; ++k) v = l == k ? gm[k] : v;
      A.GM[p * WKP + l] = v;
    }
    if (l == 0 && A.s_out) A.s_out[p] = s;
    float *g1 = A.GX + p * Dp, *g2 = A.GX + (A.Cp + p) * Dp;
    for (int c = 0; c < ncp; ++c) {
      const int a = 64 * c + l;
      float v1 = 0.f, v2 = 0.f;
#pragma unroll
      for (int k = 0; k < WKP; ++k) {
        if (k < K) {
          const float t = (!MT && a < e1) ? Tp[k * Dp + a] : 0.f;
          v1 = fmaf(gm[k], t + sV[k * 2 * Dp + a], v1);
          v2 = fmaf(gm[k], sV[k * 2 * Dp + Dp + a], v2);
        }
      }
      g1[a] = v1;
      g2[a] = v2;
    }
  }
  if (!BWD) return;
  float *row = A.hslab + ((size_t)blockIdx.x * 4 + w) * HSLAB;
  if (l == 0) row[0] += aLoss;   // wave-uniform
  if (l < WKP) {
    row[1 + l] += aU;
    row[1 + WKP + l] += aB;
  }
}

// ---------------------------------------------------------------------------
// Final reductions (once per call): column sums in fixed order.
// ---------------------------------------------------------------------------
// dst[c] = Σ_r src[r·stride + c] (+ add[0] on column `addcol`)
__global__ void __launch_bounds__(1024) web_colsum(const float *__restrict__ src, int rows,
                                                   int cols, int stride, float *__restrict__ dst,
                                                   int dstride, const float *__restrict__ add,
                                                   int addcol) {
  __shared__ float red[16][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l;
  float a0 = 0.f, a1 = 0.f;
  if (c < cols)
    for (int r = w; r < rows; r += 32) {
      a0 += src[(size_t)r * stride + c];
      if (r + 16 < rows) a1 += src[(size_t)(r + 16) * stride + c];
    }
  red[w][l] = a0 + a1;
  __syncthreads();
  if (w == 0 && c < cols) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][l];
    if (add && c == addcol) v += add[0];
    dst[(size_t)c * dstride] = v;
  }
}

// grad W[a][b][k] = Σ_s gWs[s][k][a][b]   (block: row a, 64 b's, all k)
__global__ void __launch_bounds__(256) web_wsum(const float *__restrict__ GWS, int D, int Dp, int K,
                                                float *__restrict__ gW) {
  __shared__ float t[64 * (WKP + 1)];
  const int a = blockIdx.x, b0 = blockIdx.y * 64;
  for (int x = threadIdx.x; x < 64 * K; x += 256) {
    const int k = x >> 6, bl = x & 63;
    float v = 0.f;
    for (int s = 0; s < WSPLIT; ++s) v += GWS[(((size_t)s * K + k) * Dp + a) * Dp + b0 + bl];
    t[bl * (WKP + 1) + k] = v;
  }
  __syncthreads();
  const int nb = min(64, D - b0);
  for (int x = threadIdx.x; x < nb * K; x += 256) {
    const int bl = x / K, k = x % K;
    gW[((size_t)a * D + b0 + bl) * K + k] = t[bl * (WKP + 1) + k];
  }
}

// grad V[k][c] = Σ_s gVs[s][k][c'] (c < D: c' = c; else c' = Dp + c - D)
__global__ void __launch_bounds__(256) web_vsum(const float *__restrict__ GVS, int D, int Dp, int K,
                                                float *__restrict__ gV) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= K * 2 * D) return;
  const int k = x / (2 * D), c = x % (2 * D);
  const int cc = c < D ? c : Dp + c - D;
  float v = 0.f;
  for (int s = 0; s < WSPLIT; ++s) v += GVS[((size_t)s * WKP + k) * 2 * Dp + cc];
  gV[x] = v;
}

__global__ void web_copy_scalar(const float *__restrict__ src, float *__restrict__ dst) {
  if (threadIdx.x == 0) dst[0] = src[0];
}

}  // namespace

// ===========================================================================
// Host side
// ===========================================================================
int sg_web_plan_params(const sg_model_t *m, int64_t *n_params) {
  WebPlan W;
  const int rc = web_plan(m, &W);
  if (rc == SG_OK && n_params) *n_params = W.n_params;
  return rc;
}

int64_t sg_web_ws_bytes(const sg_model_t *m, int64_t chunk, int64_t n_pairs) {
  WebPlan W;
  if (web_plan(m, &W) != SG_OK) return -1;
  // chunk <= 0 is one chunk of the whole call, as sg_web_run reads it: sizable only for a
  // known n_pairs
  if (chunk <= 0) {
    if (n_pairs < 0) return -1;
    chunk = n_pairs > 0 ? n_pairs : 1;
  }
  const WebWs ws = web_ws(W, chunk);
  // calls of at most one chunk never pipeline (sg_web_run): slot 0 only
  const bool one = n_pairs >= 0 && n_pairs <= chunk;
  return (one ? ws.total1 : ws.total) * 4 + 256;
}

// A/B: dynamic LDS padding of a GEMM launch (bytes, from the environment), which lowers the
// blocks a CU holds at once (the GEMMs hold ≈61-67 KB of static LDS: 2 blocks per CU)
static size_t web_lds_pad(const char *name, const void *fn) {
  const char *e = getenv(name);
  const int v = e ? atoi(e) : 0;
  if (v <= 0) return 0;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, v);
  return (size_t)v;
}

static int web_status() {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return SG_OK;
  if (getenv("SG_DEBUG")) fprintf(stderr, "sg_web: %s\n", hipGetErrorString(e));
  return SG_ERR_HIP;
}

// LDS of the instance kernel (+ the CSR rows with LCSR)
static size_t gcn_lds_bytes(const WebPlan &W, int n_max, int max_nnz, bool bwd, bool lcsr) {
  const int n16 = (n_max + 15) & ~15;
  const GcnLds L = gcn_lds(W.d_in, n16, max_nnz, bwd, lcsr);
  size_t lds = (size_t)L.total * 4u;
  if (bwd) {
    const size_t fl = ((size_t)L.tables + 8u * (size_t)W.n_gcn) * 4u;
    if (fl > lds) lds = fl;
  }
  return lds;
}

static int gcn_launch(bool bwd, const WebPlan &W, const GcnArgs &A, int64_t n_inst,
                      hipStream_t st) {
  // CSR rows staged in LDS (LCSR) measured slower than reading them through the caches
  // once the instance kernels run 16 waves (forward 14.7 -> 13.1 ms per chunk without),
  // so it is opt-in (SG_WEB_LCSR=1); the backward's LDS no longer fits it at 16 waves
  static const bool want_lcsr = getenv("SG_WEB_LCSR") != nullptr;
  const bool lcsr = want_lcsr && gcn_lds_bytes(W, A.n_max, A.max_nnz, bwd, true) <= 163840u &&
                    A.max_nnz <= 4096;
  const size_t lds = gcn_lds_bytes(W, A.n_max, A.max_nnz, bwd, lcsr);
  if (lds > 163840u) return SG_ERR_UNSUPPORTED;
  GcnArgs A_ = A;
  if (lcsr) A_.isorted = nullptr, A_.icls = nullptr;   // LCSR stages one instance at a time
  int per_cu = (int)(163840u / lds);
  if (per_cu > 2048 / (64 * gcn_gw(bwd))) per_cu = 2048 / (64 * gcn_gw(bwd));
  if (!bwd) {
    // forward blocks per CU: 2 of the 3 that the LDS admits (4.445 vs 4.32 M pairs/s on C5,
    // profiles/r03_c5ab/knob_*: fewer blocks contend for the CU's LDS and issue slots, and
    // leave room for the pipelined GEMMs); SG_WEB_FWD_BPC=n sets it (A/B)
    int want = 2;
    const char *e = getenv("SG_WEB_FWD_BPC");
    if (e && atoi(e) > 0) want = atoi(e);
    if (want < per_cu) per_cu = want;
  }
  int64_t blocks = (int64_t)sg_num_cus() * per_cu;
  if (bwd) blocks = sg_num_cus();   // one slab row per block (web_ws sizes the slab for this)
  if (blocks > n_inst) blocks = n_inst;
  if (blocks < 1) return SG_OK;
#define SG_WEB_GCN(B, NT, LC)                                                                   \
  do {                                                                                        \
    const void *fn = (const void *)web_gcn_kernel<B, NT, LC>;                                 \
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);      \
    hipLaunchKernelGGL((web_gcn_kernel<B, NT, LC>), dim3((unsigned)blocks), dim3(64 * gcn_gw(B)), \
                       lds, st, A_);                                                          \
  } while (0)
#define SG_WEB_GCN_NT(NT)                             \
  do {                                                \
    if (bwd) {                                        \
      if (lcsr) SG_WEB_GCN(true, NT, true);           \
      else SG_WEB_GCN(true, NT, false);               \
    } else {                                          \
      if (lcsr) SG_WEB_GCN(false, NT, true);          \
      else SG_WEB_GCN(false, NT, false);              \
    }                                                 \
  } while (0)
  switch (W.tb) {
    case 1: SG_WEB_GCN_NT(1); break;
    case 2: SG_WEB_GCN_NT(2); break;
    case 3: SG_WEB_GCN_NT(3); break;
    default: SG_WEB_GCN_NT(4); break;
  }
#undef SG_WEB_GCN_NT
#undef SG_WEB_GCN
  return SG_OK;
}

int sg_web_lds_ok(const sg_model_t *m) {
  WebPlan W;
  if (web_plan(m, &W) != SG_OK) return 0;
  return gcn_lds_bytes(W, m->n_max, 0, true, false) <= 163840u;
}

// The chunk pipeline's second stream and its events (sg_web_run: F = a chunk's forward
// instance kernel done, G[slot] = the GEMMs of the chunk in that workspace slot done), one
// set per (device, caller stream): calls on different caller streams do not share a second
// stream (no false dependency between them), and calls from any host thread on the same
// caller stream reuse one set.  A set is leased for the whole sg_web_run call (in_use): the
// registry keeps up to kWebAuxMax sets, and a caller stream without a set recycles the least
// recently used set of its device only when no call holds it (else a new set is created),
// so no call can see its stream and events handed to another caller between its event
// record and the matching wait.  The recycled set's second stream is drained after the
// registry lock is released.  A caller stream whose handle is reused after it was destroyed
// inherits that set, which is harmless: the set only orders the call's own work.
// sg_web_release() destroys them all (teardown, no call in flight).
struct WebAux {
  int dev;
  hipStream_t caller, aux;
  hipEvent_t ev[3];
  uint64_t last_use;
  int in_use;
};
constexpr size_t kWebAuxMax = 16;
static std::mutex g_web_aux_mu;
static std::list<WebAux> g_web_aux;   // stable addresses: leases point into it
static uint64_t g_web_aux_tick = 0;

// releases the set at the end of the call that leased it
struct WebAuxLease {
  WebAux *a = nullptr;
  ~WebAuxLease() {
    if (a) {
      std::lock_guard<std::mutex> lk(g_web_aux_mu);
      --a->in_use;
    }
  }
};

static int web_aux(hipStream_t caller, WebAuxLease *lease, hipStream_t *gs, hipEvent_t *evF,
                   hipEvent_t *evG) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return SG_ERR_HIP;
  WebAux *a = nullptr;
  bool drain = false;
  {
    std::lock_guard<std::mutex> lk(g_web_aux_mu);
    for (WebAux &x : g_web_aux)
      if (x.dev == dev && x.caller == caller) a = &x;
    if (!a && g_web_aux.size() >= kWebAuxMax) {
      // recycle the least recently used idle set of this device
      for (WebAux &y : g_web_aux)
        if (y.dev == dev && y.in_use == 0 && (!a || y.last_use < a->last_use)) a = &y;
      if (a) {
        a->caller = caller;
        drain = true;
      }
    }
    if (!a) {
      WebAux x;
      x.dev = dev;
      x.caller = caller;
      x.in_use = 0;
      for (int e = 0; e < 3; ++e)
        if (hipEventCreateWithFlags(&x.ev[e], hipEventDisableTiming) != hipSuccess)
          return SG_ERR_HIP;
      if (hipStreamCreateWithFlags(&x.aux, hipStreamNonBlocking) != hipSuccess)
        return SG_ERR_HIP;
      g_web_aux.push_back(x);
      a = &g_web_aux.back();
    }
    a->last_use = ++g_web_aux_tick;
    ++a->in_use;
    lease->a = a;
  }
  // the recycled set's earlier work (another caller's) is done before this call reuses it;
  // the lease keeps any other caller off the set meanwhile
  if (drain && hipStreamSynchronize(a->aux) != hipSuccess) return SG_ERR_HIP;
  *gs = a->aux;
  *evF = a->ev[0];
  evG[0] = a->ev[1];
  evG[1] = a->ev[2];
  return SG_OK;
}

int sg_web_release_aux() {
  std::lock_guard<std::mutex> lk(g_web_aux_mu);
  int rc = SG_OK;
  int cur = 0;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  for (auto it = g_web_aux.begin(); it != g_web_aux.end();) {
    WebAux &x = *it;
    // a set leased by a call still in flight on another thread stays (its lease points at
    // it); a later sg_web_release frees it
    if (x.in_use > 0 || hipSetDevice(x.dev) != hipSuccess) {
      if (x.in_use == 0) rc = SG_ERR_HIP;
      ++it;
      continue;
    }
    // the second stream's work must be done before its objects go
    if (hipStreamSynchronize(x.aux) != hipSuccess) rc = SG_ERR_HIP;
    for (int e = 0; e < 3; ++e) (void)hipEventDestroy(x.ev[e]);
    if (hipStreamDestroy(x.aux) != hipSuccess) rc = SG_ERR_HIP;
    it = g_web_aux.erase(it);
  }
  if (have_cur) (void)hipSetDevice(cur);
  return rc;
}

int sg_web_run(const sg_model_t *m, const sg_csr_store_t *store, const int32_t *pairs,
               const float *labels, int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
               const float *params, uint64_t seed, const float *y_stats, int add_label,
               float *s_out, float *grad_out, float *loss_out, void *workspace, int64_t chunk,
               bool bwd, hipStream_t st) {
  WebPlan W;
  int rc = web_plan(m, &W);
  if (rc != SG_OK) return rc;
  if (!store || !store->node_off || !store->types || !store->row_ptr || !store->col ||
      !store->val || store->n_max > W.D || store->n_max > m->n_max || store->max_nnz < 0)
    return SG_ERR_ARG;
  if (!sg_web_lds_ok(m)) return SG_ERR_UNSUPPORTED;
  if (chunk <= 0) chunk = n_pairs > 0 ? n_pairs : 1;
  (void)hipGetLastError();   // report only this call's launch errors
  const WebWs ws = web_ws(W, chunk);
  float *base = (float *)workspace;
  float *Wg = base + ws.Wg, *Wh = base + ws.Wh, *GWS = base + ws.GWS, *GVS = base + ws.GVS;
  float *GSLAB = base + ws.GSLAB, *HS = base + ws.HSLABo;
  const int Dp = W.Dp, K = W.K, D = W.D;

  if (bwd) {
    if (hipMemsetAsync(GWS, 0, (size_t)WSPLIT * K * Dp * Dp * 4u, st) != hipSuccess ||
        hipMemsetAsync(GVS, 0, (size_t)WSPLIT * WKP * 2 * Dp * 4u, st) != hipSuccess ||
        hipMemsetAsync(GSLAB, 0, (size_t)ws.gcn_blocks * W.n_gcn * 4u, st) != hipSuccess ||
        hipMemsetAsync(HS, 0, (size_t)ws.head_blocks * 4 * HSLAB * 4u, st) != hipSuccess)
      return SG_ERR_HIP;
  }
  if (n_pairs > 0) {
    hipLaunchKernelGGL(web_wprep_g, dim3(Dp, Dp / 64), dim3(256), 0, st, params + W.oW, D, Dp, K,
                       Wg);
    if (bwd)
      hipLaunchKernelGGL(web_wprep_h, dim3(Dp / 32, Dp / 32, K), dim3(256), 0, st, Wg, Dp, Wh);
  }
  GcnArgs G;
  G.node_off = store->node_off;
  G.types = store->types;
  G.row_ptr = store->row_ptr;
  G.col = store->col;
  G.val = store->val;
  G.Cp = ws.Cp;
  G.params = params;
  G.slab = GSLAB;
  G.key = sg_seed_key(seed);
  G.thr0 = W.thr0; G.thr1 = W.thr1; G.thr2 = W.thr2; G.thr4 = W.thr4;
  G.ik0 = W.ik0; G.ik1 = W.ik1; G.ik2 = W.ik2; G.ik4 = W.ik4;
  G.padv = W.padv;
  G.d_in = W.d_in; G.D = D; G.Dp = Dp; G.n_gcn = W.n_gcn; G.n_max = store->n_max;
  G.max_nnz = store->max_nnz;
  G.ob0 = W.ob0; G.oW1 = W.oW1; G.ob1 = W.ob1; G.oWd = W.oWd; G.obd = W.obd;
  HeadArgs H;
  H.params = params; H.y_stats = y_stats; H.s_out = nullptr; H.hslab = HS;
  H.Cp = ws.Cp; H.D = D; H.Dp = Dp; H.K = K; H.oV = W.oV; H.oU = W.oU; H.obn = W.obn;
  H.final_act = W.final_act; H.loss_mode = W.loss_mode; H.ntn_mode = W.ntn_mode;
  H.yeta = W.yeta;
  H.inv_batch = batch_total > 0 ? 1.f / (float)batch_total : 0.f;
  const size_t head_lds = (size_t)K * 2 * Dp * 4u;
  const int full = W.padv != 0.f ? 1 : 0;
  // instance units (GcnArgs::isorted); SG_WEB_UNITS=0 runs one instance per workgroup
  static const bool units = [] {
    const char *e = getenv("SG_WEB_UNITS");
    return !(e && e[0] == '0');
  }();
  // XCD partitions of the units, opt-in (SG_WEB_XCD=1; read per call: a test compares the
  // two).  Measured 2% slower on C5 than the plain size-class order (3.81-3.83 vs 3.88 M
  // pairs/s, profiles/r03_c5v1): the partitions' work differs by XCD
  const char *xcd_e = getenv("SG_WEB_XCD");
  const int xparts = (xcd_e && xcd_e[0] == '1') ? kXcdParts : 1;

  // Two-stream pipeline over the chunks.  The instance kernels are latency-bound (most
  // wave cycles wait on the CSR gathers) and the NTN GEMMs are MFMA work, so the forward
  // instance kernel of chunk c + 1 (stream st) runs while the GEMMs and the head of chunk
  // c run on a second stream (gs); the backward instance kernel of chunk c then waits
  // for them.  Per-chunk buffers alternate between two slots.  Every accumulation keeps
  // its order (GWS/GVS/HS on gs, GSLAB on st, chunks in order), so results are bitwise
  // those of the one-stream sequence (SG_WEB_PIPE=0).
  const char *pipe_e = getenv("SG_WEB_PIPE");   // read per call (a test toggles it)
  const bool pipe_env = !(pipe_e && pipe_e[0] == '0');

  hipStream_t gs = st;
  hipEvent_t evF = nullptr, evG[2] = {nullptr, nullptr};
  const int64_t nch = n_pairs > 0 ? (n_pairs + chunk - 1) / chunk : 0;
  WebAuxLease lease;   // held until this call has enqueued all of its work
  if (pipe_env && nch > 1) {
    if (web_aux(st, &lease, &gs, &evF, evG) != SG_OK) return SG_ERR_HIP;
  }
  const bool pipe = gs != st;
  struct Slot {
    float *X, *GX, *T, *GM;
    uint16_t *MASK;
    float *D2;
    int2 *EXT, *EXT16, *EXT128;
    int4 *INST;
    int32_t *isort, *icnt, *icls;
  };
  auto slot = [&](int64_t c) {
    float *sb = base + ws.S0 + (pipe ? (c & 1) * ws.SLOT : 0);
    Slot S;
    S.X = sb + ws.X; S.GX = sb + ws.GX; S.T = sb + ws.T; S.GM = sb + ws.GM;
    S.EXT = (int2 *)(sb + ws.EXT); S.EXT16 = (int2 *)(sb + ws.EXT16);
    S.EXT128 = (int2 *)(sb + ws.EXT128); S.INST = (int4 *)(sb + ws.INST);
    S.isort = (int32_t *)(sb + ws.ISORT); S.icnt = (int32_t *)(sb + ws.ICNT);
    S.icls = (int32_t *)(sb + ws.ICLS);
    S.MASK = (uint16_t *)(sb + ws.MASK);
    S.D2 = sb + ws.D2;
    return S;
  };
  auto gcn_args = [&](int64_t c, const Slot &S) {
    const int64_t c0 = c * chunk, n = n_pairs - c0 < chunk ? n_pairs - c0 : chunk;
    GcnArgs g = G;
    g.pairs = pairs + 2 * c0;
    g.inst = S.INST;
    g.isorted = units ? S.isort : nullptr;
    g.icls = units ? S.icls : nullptr;
    g.X = S.X;
    // the forward's dropout bits for the backward (training calls)
    g.masks = bwd ? S.MASK : nullptr;
    g.d2 = bwd ? S.D2 : nullptr;
    g.GX = S.GX;
    g.n_pairs = n;
    g.pair_offset = pair_offset + c0;
    return g;
  };
  // chunk c's extents, unit order and forward instance kernel (stream st)
  auto front = [&](int64_t c) -> int {
    const Slot S = slot(c);
    const int64_t c0 = c * chunk, n = n_pairs - c0 < chunk ? n_pairs - c0 : chunk;
    const int64_t nblk = (n + TB - 1) / TB;
    hipLaunchKernelGGL(web_ext_kernel, dim3((unsigned)nblk), dim3(TB), 0, st, pairs + 2 * c0, n,
                       store->node_off, store->row_ptr, full, D, S.EXT, S.EXT16, S.EXT128, S.INST);
    if (units) {   // instance units: small instances share a workgroup (web_gcn_kernel)
      const int n16 = (store->n_max + 15) & ~15;
      const int cap4 = (n16 / 4) & ~15, cap2 = (n16 / 2) & ~15;
      const int nbu = (int)((2 * n + kUnitChunk - 1) / kUnitChunk);
      const int32_t *cp = pairs + 2 * c0;
      hipLaunchKernelGGL(web_icls_count, dim3(nbu), dim3(256), 0, st, S.INST, cp, 2 * n, cap4,
                         cap2, xparts, nbu, S.icnt);
      hipLaunchKernelGGL(web_icls_scan, dim3(1), dim3(kScanT), 0, st, S.icnt, nbu, 2 * n, xparts,
                         S.icls);
      hipLaunchKernelGGL(web_icls_scatter, dim3(nbu), dim3(256), 0, st, S.INST, cp, 2 * n, cap4,
                         cap2, xparts, nbu, (const int32_t *)S.icnt, S.isort);
    }
    return gcn_launch(false, W, gcn_args(c, S), 2 * n, st);
  };
  // chunk c's NTN GEMMs and head (stream gs)
  auto middle = [&](int64_t c) {
    const Slot S = slot(c);
    const int64_t c0 = c * chunk, n = n_pairs - c0 < chunk ? n_pairs - c0 : chunk;
    const int64_t nblk = (n + TB - 1) / TB;
    float *X = S.X, *GX = S.GX, *T = S.T, *GM = S.GM;
    // SG_WEB_TKG=0: web_t_kernel_b3, one k per block (read per call: a test compares the two)
    const char *tkg_e = getenv("SG_WEB_TKG");
    const bool tkg = !(tkg_e && tkg_e[0] == '0');
    if (tkg)
      hipLaunchKernelGGL(web_t_kernel_kg, dim3((unsigned)nblk, Dp / TB, (K + TKG - 1) / TKG),
                         dim3(512), 0, gs, X + ws.Cp * Dp, Wg, S.EXT128, n, Dp, K, T, X);
    else
      hipLaunchKernelGGL(web_t_kernel_b3<true>, web_pb_grid(nblk, Dp / TB, K), dim3(256),
                         web_lds_pad("SG_WEB_TPAD", (const void *)web_t_kernel_b3<true>), gs,
                         X + ws.Cp * Dp, Wg, S.EXT128, n, Dp, K, T, X);
    HeadArgs h = H;
    h.X = X; h.T = T; h.ext = S.EXT; h.ext128 = S.EXT128; h.GX = GX; h.GM = GM;
    h.n = n;
    h.labels = labels ? labels + c0 : nullptr;
    h.s_out = s_out ? s_out + c0 : nullptr;
    const int hb = (int)((n + 3) / 4 < ws.head_blocks ? (n + 3) / 4 : ws.head_blocks);
    if (bwd) {
      hipLaunchKernelGGL((web_head_kernel<true, true>), dim3(hb), dim3(256), head_lds, gs, h);
      hipLaunchKernelGGL(web_gx1_kernel_b3, web_pb_grid(nblk, Dp / TB, 1), dim3(256),
                         web_lds_pad("SG_WEB_GXPAD", (const void *)web_gx1_kernel_b3), gs,
                         X + ws.Cp * Dp, GM, Wg, S.EXT128, n, Dp, K, GX);
      hipLaunchKernelGGL(web_gx2_kernel_b3, web_pb_grid(nblk, Dp / TB, 1), dim3(256),
                         web_lds_pad("SG_WEB_GXPAD", (const void *)web_gx2_kernel_b3), gs, X,
                         GM, Wh, S.EXT128, n, Dp, K, GX + ws.Cp * Dp);
      // gV rides along
      hipLaunchKernelGGL(web_wgrad_kernel_b3, dim3((Dp / TB) * (Dp / TB), K, WSPLIT), dim3(256),
                         web_lds_pad("SG_WEB_WGPAD", (const void *)web_wgrad_kernel_b3), gs, X,
                         X + ws.Cp * Dp, GM, S.EXT16, n, Dp, K, GWS, GVS);
    } else {
      hipLaunchKernelGGL((web_head_kernel<false, true>), dim3(hb), dim3(256), head_lds, gs, h);
    }
  };
  // chunk c's backward instance kernel (stream st)
  auto back = [&](int64_t c) -> int {
    const Slot S = slot(c);
    const int64_t n = n_pairs - c * chunk < chunk ? n_pairs - c * chunk : chunk;
    return gcn_launch(true, W, gcn_args(c, S), 2 * n, st);
  };
  // enqueue order: front(c) after middle(c - 2) (slot reuse) | back(c - 1) after
  // middle(c - 1) | middle(c) after front(c)
  for (int64_t c = 0; c < nch; ++c) {
    if (pipe && c >= 2 && hipStreamWaitEvent(st, evG[c & 1], 0) != hipSuccess) return SG_ERR_HIP;
    if ((rc = front(c)) != SG_OK) return rc;
    if (pipe && hipEventRecord(evF, st) != hipSuccess) return SG_ERR_HIP;
    if (pipe && c > 0 && bwd) {
      if (hipStreamWaitEvent(st, evG[(c - 1) & 1], 0) != hipSuccess) return SG_ERR_HIP;
      if ((rc = back(c - 1)) != SG_OK) return rc;
    }
    if (pipe && hipStreamWaitEvent(gs, evF, 0) != hipSuccess) return SG_ERR_HIP;
    middle(c);
    if (pipe && hipEventRecord(evG[c & 1], gs) != hipSuccess) return SG_ERR_HIP;
    if (!pipe && bwd && (rc = back(c)) != SG_OK) return rc;
  }
  if (pipe) {   // join: st waits for the last chunk's GEMMs (gs runs them in order)
    if (hipStreamWaitEvent(st, evG[(nch - 1) & 1], 0) != hipSuccess) return SG_ERR_HIP;
    if (bwd && (rc = back(nch - 1)) != SG_OK) return rc;
  }
  if (!bwd) return web_status();

  // gradient assembly in the reference's variable order
  hipLaunchKernelGGL(web_colsum, dim3((W.n_gcn + 63) / 64), dim3(1024), 0, st, GSLAB,
                     ws.gcn_blocks, W.n_gcn, W.n_gcn, grad_out, 1, (const float *)nullptr, -1);
  hipLaunchKernelGGL(web_wsum, dim3(D, Dp / 64), dim3(256), 0, st, GWS, D, Dp, K,
                     grad_out + W.oW);
  hipLaunchKernelGGL(web_vsum, dim3((K * 2 * D + 255) / 256), dim3(256), 0, st, GVS, D, Dp, K,
                     grad_out + W.oV);
  const int hrows = ws.head_blocks * 4;
  hipLaunchKernelGGL(web_colsum, dim3(1), dim3(1024), 0, st, HS + 1, hrows, K, HSLAB,
                     grad_out + W.oU, 1, (const float *)nullptr, -1);
  if (W.obn >= 0)
    hipLaunchKernelGGL(web_colsum, dim3(1), dim3(1024), 0, st, HS + 1 + WKP, hrows, K, HSLAB,
                       grad_out + W.obn, 1, (const float *)nullptr, -1);
  if (loss_out) {
    const bool lab = add_label && m->loss_mode == SG_LOSS_BROADCAST && y_stats;
    hipLaunchKernelGGL(web_colsum, dim3(1), dim3(1024), 0, st, HS, hrows, 1, HSLAB, loss_out, 1,
                       lab ? y_stats + 1 : (const float *)nullptr, 0);
  }
  return web_status();
}
