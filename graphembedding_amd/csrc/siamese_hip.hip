// siamese_hip.hip — C-ABI entry points of libsiamese_hip.so (include/siamese_hip.h)
// plus the small kernels around the fused pair kernels: pair packing, label
// statistics, the deterministic gradient-slab reduction and TF-form Adam.
#include <mutex>

#include "sg_plan.h"

// ---------------------------------------------------------------------------
// Device properties
// ---------------------------------------------------------------------------
int sg_num_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    cache[dev] = cus;
  }
  return cache[dev];
}

// generic path (sg_generic.hip)
int sg_generic_lds_ok(const SgGenPlan &P, bool bwd);
int64_t sg_generic_slab_floats(const SgGenPlan &P, int64_t n_pairs);
int sg_generic_run(const SgGenPlan &P, bool bwd, const void *recs, const int32_t *order,
                   int64_t n_pairs, int64_t pair_offset, int64_t batch_total, const float *params, uint64_t seed,
                   const float *y_stats, float *s_out, float *slab, int *blocks_out,
                   hipStream_t stream);
// fused fast path (sg_fast.hip)
int sg_fast_supported(const sg_model_t *m, const SgGenPlan &P);
int64_t sg_fast_slab_floats(const SgGenPlan &P, int64_t n_pairs);
int sg_fast_needs_ntn(const SgGenPlan &P);
int sg_fast_run(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                const int32_t *order, int64_t n_pairs, int64_t pair_offset, int64_t batch_total, const float *params,
                uint64_t seed, const float *y_stats, float *s_out, float *slab, float *ntn,
                int *blocks_out, hipStream_t stream, const uint64_t *seed_dev = nullptr,
                const sg_pair_source_t *src = nullptr, const int32_t *class_start = nullptr,
                const SgAdamPre *adam_pre = nullptr);
// fused capacity-32 path (sg_fast32.hip)
int sg_fast32_supported(const sg_model_t *m, const SgGenPlan &P);
// graph-store path for Web-sized graphs (sg_web.hip)
int sg_web_plan_params(const sg_model_t *m, int64_t *n_params);
int sg_web_lds_ok(const sg_model_t *m);
int64_t sg_web_ws_bytes(const sg_model_t *m, int64_t chunk, int64_t n_pairs);
int sg_web_release_aux();
int sg_web_run(const sg_model_t *m, const sg_csr_store_t *store, const int32_t *pairs,
               const float *labels, int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
               const float *params, uint64_t seed, const float *y_stats, int add_label,
               float *s_out, float *grad_out, float *loss_out, void *workspace, int64_t chunk,
               bool bwd, hipStream_t st);
int64_t sg_fast32_slab_floats(const SgGenPlan &P, int64_t n_pairs);
int64_t sg_fast32_ntn_floats(int64_t n_pairs);
int sg_fast32_run(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                  const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                  int64_t batch_total, const float *params, uint64_t seed, const float *y_stats,
                  float *s_out, float *slab, float *ntn, int *blocks_out, hipStream_t stream,
                  const sg_pair_source_t *src = nullptr);

namespace {

constexpr int kReduceStrands = 16;  // second-level partial rows
constexpr int kOnePassRows = 1024;  // slabs up to this many rows reduce in one launch

// TF ApplyAdam of one element (+ the weight-decay gradient, models.py:67-73): one
// expression for every Adam kernel, so that they contract it alike (bitwise the same θ, m,
// v from sg_adam_tf, sg_adam_tf_ex and sg_train_step)
__device__ __forceinline__ float adam_elem(float tv, float gv, float &mv, float &vv, float wd,
                                           float c1, float c2, float alpha, float eps) {
  const float gi = gv + wd * tv;
  mv = mv + (gi - mv) * c1;
  vv = vv + (gi * gi - vv) * c2;
  return tv - (mv * alpha) / (sqrtf(vv) + eps);
}

// slab [nblk][C] → part [S][C]; strand order fixed ⇒ bitwise reproducible.
__global__ void __launch_bounds__(256) sg_reduce_stage1(const float *__restrict__ slab, int nblk,
                                                        int C, float *__restrict__ part) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int strand = blockIdx.y * 4 + w, nstrand = gridDim.y * 4;
  float acc = 0.f;
  if (col < C)
    for (int b = strand; b < nblk; b += nstrand) acc += slab[(size_t)b * C + col];
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && col < C)
    part[(size_t)blockIdx.y * C + col] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// slab [nblk][C] → grad[C-1], loss in one pass (nblk <= kOnePassRows): block x owns
// columns 64x .. 64x+63; wave w of 16 sums rows w + 16 i into four independent
// partials (i mod 4), combined in fixed order (deterministic)
__global__ void __launch_bounds__(1024) sg_reduce_one(const float *__restrict__ slab, int nblk, int C,
                                                      float *__restrict__ grad,
                                                      float *__restrict__ loss,
                                                      const float *__restrict__ y_stats,
                                                      int add_label) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  // wave w sums rows w + 16 k in a fixed order; 16 rows per batch with every load
  // in flight (one memory latency per 256 slab rows)
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < C) {
    const float *p = slab + col;
    int b = w;
    for (; b + 16 * 15 < nblk; b += 256) {
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = p[(size_t)(b + 16 * k) * C];
#pragma unroll
      for (int k = 0; k < 16; ++k) a[k & 3] += v[k];
    }
    for (; b < nblk; b += 16) a[0] += p[(size_t)b * C];
  }
  red[w][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (w == 0 && col < C) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][lane];
    if (col < C - 1)
      grad[col] = v;
    else if (loss)
      loss[0] = v + ((add_label && y_stats) ? y_stats[1] : 0.f);
  }
}

// sg_reduce_one + the update of sg_adam_kernel in one launch (sg_train_step): block x
// reduces columns 64x .. 64x+63 of the slab exactly as sg_reduce_one (grad, loss), then
// wave 0 applies ApplyAdam to those parameters (adam_elem).  The step scalars pre[4] =
// {α, β1^t·β1, β2^t·β2, wd·½Σθ²} come from the fused kernel's block 0 (FastArgs::ad_out),
// so no block waits on another: block 0 stores the new β powers and reg_loss.
__global__ void __launch_bounds__(1024) sg_reduce_adam(
    const float *__restrict__ slab, int nblk, int C, float *__restrict__ grad,
    float *__restrict__ loss, const float *__restrict__ y_stats, int add_label,
    float *__restrict__ th, float *__restrict__ m, float *__restrict__ v, float b1, float b2,
    float eps, float wd, const float *__restrict__ pre, float *__restrict__ bp,
    float *__restrict__ reg_loss) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int n = C - 1;
  // wave 0's Adam operands: loaded first, their latency under the slab's
  float tv = 0.f, mv = 0.f, vv = 0.f, alpha = 0.f;
  if (w == 0) {
    alpha = pre[0];
    if (col < n) {
      tv = th[col];
      mv = m[col];
      vv = v[col];
    }
  }
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < C) {
    const float *p = slab + col;
    int b = w;
    for (; b + 16 * 15 < nblk; b += 256) {
      float x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = p[(size_t)(b + 16 * k) * C];
#pragma unroll
      for (int k = 0; k < 16; ++k) a[k & 3] += x[k];
    }
    for (; b < nblk; b += 16) a[0] += p[(size_t)b * C];
  }
  red[w][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (w != 0) return;
  float gsum = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) gsum += red[k][lane];
  if (col < n) {
    grad[col] = gsum;
    const float ti = adam_elem(tv, gsum, mv, vv, wd, 1.f - b1, 1.f - b2, alpha, eps);
    m[col] = mv;
    v[col] = vv;
    th[col] = ti;
  } else if (col == n && loss) {
    loss[0] = gsum + ((add_label && y_stats) ? y_stats[1] : 0.f);
  }
  if (blockIdx.x == 0 && lane == 0) {
    bp[0] = pre[1];
    bp[1] = pre[2];
    if (reg_loss) reg_loss[0] = pre[3];
  }
}

// part [S][C] → grad[C-1], loss = part[:, C-1] (+ label term)
__global__ void __launch_bounds__(256) sg_reduce_stage2(const float *__restrict__ part, int S, int C,
                                                        float *__restrict__ grad,
                                                        float *__restrict__ loss,
                                                        const float *__restrict__ y_stats,
                                                        int add_label) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= C) return;
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += part[(size_t)s * C + col];
  if (col < C - 1)
    grad[col] = acc;
  else if (loss)
    loss[0] = acc + ((add_label && y_stats) ? y_stats[1] : 0.f);
}

// ---- label statistics (double accumulation) ----
__global__ void __launch_bounds__(256) sg_label_partial(const uint8_t *__restrict__ recs, int64_t n,
                                                        int rec_words, int label_off,
                                                        const double *__restrict__ mean,
                                                        double *__restrict__ part) {
  __shared__ double red[256];
  double acc = 0.0;
  const double mu = mean ? mean[0] : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float y = ((const float *)(recs + (size_t)i * rec_words * 4u))[label_off];
    const double d = (double)y - mu;
    acc += mean ? d * d : (double)y;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) sg_label_final(const double *__restrict__ part, int np,
                                                      int64_t n, int which, double *__restrict__ mean,
                                                      float *__restrict__ stats) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (which == 0) {
      const double mu = n > 0 ? red[0] / (double)n : 0.0;
      mean[0] = mu;
      stats[0] = (float)mu;
    } else {
      stats[1] = (float)(0.5 * red[0]);
    }
  }
}

// ---- pair packing: one wave per pair, record words written lane-parallel ----
// Â is stored as f32 or as bf16 pairs (sg_dtype); the rest of the record is the
// same words after the adjacency block, then zero padding to 16 B.
__global__ void __launch_bounds__(256) sg_pack_kernel(const float *__restrict__ sadj,
                                                      const int32_t *__restrict__ stypes,
                                                      const int32_t *__restrict__ sn, int n_graphs,
                                                      int nmax, int bf16, const int32_t *__restrict__ pidx,
                                                      const float *__restrict__ labels, int64_t n,
                                                      uint32_t *__restrict__ recs, int rec_words,
                                                      int32_t *__restrict__ status) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (p >= n) return;
  sg_pack_record(sadj, stypes, sn, n_graphs, nmax, bf16, pidx[2 * p], pidx[2 * p + 1],
                 labels ? labels[p] : 0.f, p, recs + (size_t)p * rec_words, rec_words, lane,
                 status);
}

// ---- processing order: stable counting sort of the records by cost class ----
// Key of a record = the cost class of its pair in the kernel that will run it:
// fused path (N0 > 8) + (N1 > 8) (third Â k-step per side, and the shared-tile
// PACK body when both sides fit 8 nodes); capacity-32 fused path
// ceil(N0/4) + ceil(N1/4) (node k-blocks); generic path N0 + N1.  Blocks own
// contiguous chunks; counts are stored key-major so one exclusive scan gives
// every (key, chunk) its output base; the scatter keeps record order within a
// key (ballot ranks), so the permutation is deterministic.
constexpr int kOrderChunk = 8192;   // records per block
constexpr int kOrderKeys = 129;     // 2·n_max + 1 keys at n_max ≤ 64

// Node counts of pair p: from its packed record, or from the store (pair source)
struct OrderRecs {
  const uint8_t *recs;
  int rec_words, n_off;
  __device__ void n01(int64_t p, int &n0, int &n1) const {
    const int32_t *r = (const int32_t *)(recs + (size_t)p * (size_t)rec_words * 4u) + n_off;
    n0 = r[0];
    n1 = r[1];
  }
};
struct OrderStore {
  const int32_t *sn, *pairs;
  int64_t grid_base;
  int G;
  __device__ void n01(int64_t p, int &n0, int &n1) const {
    int g0, g1;
    if (pairs) {
      g0 = pairs[2 * p];
      g1 = pairs[2 * p + 1];
    } else {
      const int64_t q = grid_base + p;
      g0 = (int)(q / G);
      g1 = (int)(q - (int64_t)g0 * G);
    }
    const bool ok = (unsigned)g0 < (unsigned)G && (unsigned)g1 < (unsigned)G;
    n0 = ok ? sn[g0] : 0;   // invalid ids read as a zero record
    n1 = ok ? sn[g1] : 0;
  }
};

template <class S>
__device__ __forceinline__ int sg_order_key(const S &src, int64_t p, int nmax, int fast) {
  int n0, n1;
  src.n01(p, n0, n1);
  n0 = n0 < 0 ? 0 : (n0 > nmax ? nmax : n0);
  n1 = n1 < 0 ? 0 : (n1 > nmax ? nmax : n1);
  // fast: 1 = sg_fast: class (N0 > 8) + 2 (N1 > 8), the kernel's four (K0, K1) bodies
  // (third Â k-step per side); 2 = sg_fast32: class-major, the tile-count class
  // (N0 > 16) + 2 (N1 > 16) of its four (T0, T1) bodies, then the k-blocks of 4 nodes, so
  // that a wave's consecutive pairs run one body and cost about the same
  if (fast == 2) {
    const int kb0 = (n0 + 3) >> 2, kb1 = (n1 + 3) >> 2;
    return ((n0 > 16) + 2 * (n1 > 16)) * 17 + kb0 + kb1;
  }
  return fast ? (n0 > 8) + 2 * (n1 > 8) : n0 + n1;
}

template <class S>
__global__ void __launch_bounds__(256) sg_order_count(S src, int64_t n, int nmax, int fast, int K,
                                                      int nb, int32_t *__restrict__ cnt) {
  __shared__ int h[kOrderKeys];
  for (int k = threadIdx.x; k < K; k += blockDim.x) h[k] = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * kOrderChunk;
  for (int i = threadIdx.x; i < kOrderChunk && b0 + i < n; i += blockDim.x)
    atomicAdd(&h[sg_order_key(src, b0 + i, nmax, fast)], 1);
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x) cnt[(size_t)k * nb + blockIdx.x] = h[k];
}

// in-place exclusive scan of m ints, one workgroup (m = K · chunks: small)
__global__ void __launch_bounds__(1024) sg_order_scan(int32_t *__restrict__ a, int64_t m) {
  __shared__ int s[1024];
  __shared__ int carry;
  const int t = threadIdx.x;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < m; c0 += 1024) {
    const int v = c0 + t < m ? a[c0 + t] : 0;
    s[t] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const int u = t >= d ? s[t - d] : 0;
      __syncthreads();
      s[t] += u;
      __syncthreads();
    }
    const int base = carry;
    if (c0 + t < m) a[c0 + t] = base + s[t] - v;
    __syncthreads();
    if (t == 1023) carry = base + s[1023];
    __syncthreads();
  }
}

template <class S>
__global__ void __launch_bounds__(256) sg_order_scatter(S src, int64_t n, int nmax, int fast,
                                                        int K, int nb,
                                                        const int32_t *__restrict__ base,
                                                        int32_t *__restrict__ order) {
  __shared__ int run[kOrderKeys];
  __shared__ int wc[4][kOrderKeys];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int k = t; k < K; k += blockDim.x) run[k] = base[(size_t)k * nb + blockIdx.x];
  const int64_t b0 = (int64_t)blockIdx.x * kOrderChunk;
  const int64_t b1 = b0 + kOrderChunk < n ? b0 + kOrderChunk : n;
  for (int64_t t0 = b0; t0 < b1; t0 += 256) {
    for (int i = t; i < 4 * kOrderKeys; i += blockDim.x) (&wc[0][0])[i] = 0;
    __syncthreads();
    const int64_t p = t0 + t;
    const bool valid = p < b1;
    const int key = valid ? sg_order_key(src, p, nmax, fast) : -1;
    // rank among the earlier lanes of this wave with the same key
    int rank = 0;
    uint64_t active = __ballot(valid);
    while (active) {
      const int k = __builtin_amdgcn_readlane(key, __builtin_ctzll(active));
      const uint64_t m = __ballot(valid && key == k);
      if (key == k) rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wc[w][k] = __popcll(m);
      active &= ~m;
    }
    __syncthreads();
    if (valid) {
      int off = run[key] + rank;
      for (int v = 0; v < w; ++v) off += wc[v][key];
      order[off] = (int32_t)p;
    }
    __syncthreads();
    for (int k = t; k < K; k += blockDim.x) run[k] += wc[0][k] + wc[1][k] + wc[2][k] + wc[3][k];
    __syncthreads();
  }
}

// class table of an order: class_start[k] = first slot of key k (the exclusive scan of
// the key-major counts at chunk 0), class_start[K] = n
__global__ void sg_order_starts(const int32_t *__restrict__ base, int K, int nb, int64_t n,
                                int32_t *__restrict__ class_start) {
  const int k = threadIdx.x;
  if (k < K) class_start[k] = base[(size_t)k * nb];
  if (k == K) class_start[K] = (int32_t)n;
}

// ---- TF ApplyAdam (+ weight decay gradient) in one workgroup ----
__global__ void __launch_bounds__(1024) sg_adam_kernel(float *__restrict__ th, float *__restrict__ m,
                                                       float *__restrict__ v,
                                                       const float *__restrict__ g, int64_t n,
                                                       float lr, float b1, float b2, float eps,
                                                       float wd, float *__restrict__ bp,
                                                       float *__restrict__ reg_loss) {
  __shared__ double red[16];
  const float b1p = bp[0], b2p = bp[1];
  const float alpha = lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float c1 = 1.f - b1, c2 = 1.f - b2;
  const int t = threadIdx.x;
  double reg = 0.0;
  // 4 parameters per thread per pass, all loads issued before any update
  for (int64_t base = 0; base < n; base += 4096) {
    float tv[4], gv[4], mv[4], vv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + k * 1024 + t;
      if (i < n) {
        tv[k] = th[i];
        gv[k] = g[i];
        mv[k] = m[i];
        vv[k] = v[i];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + k * 1024 + t;
      if (i < n) {
        reg += (double)tv[k] * (double)tv[k];
        float mi = mv[k], vi = vv[k];
        const float ti = adam_elem(tv[k], gv[k], mi, vi, wd, c1, c2, alpha, eps);
        m[i] = mi;
        v[i] = vi;
        th[i] = ti;
      }
    }
  }
  // Σθ²: butterfly within each wave, then the 16 wave sums in order (deterministic)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) reg += __shfl_xor(reg, o);
  if ((t & 63) == 0) red[t >> 6] = reg;
  __syncthreads();
  if (t == 0)
    for (int w = 1; w < 16; ++w) red[0] += red[w];
  if (threadIdx.x == 0) {
    bp[0] = b1p * b1;
    bp[1] = b2p * b2;
    if (reg_loss) reg_loss[0] = (float)((double)wd * 0.5 * red[0]);
  }
}

// Multi-block ApplyAdam for large parameter vectors (config C5: 2.6 M parameters):
// pass 1 updates θ, m, v and writes one Σθ² partial (double) per block; pass 2 sums
// the partials in order and advances the β powers.
constexpr int kAdamBlocks = 512;
__global__ void __launch_bounds__(256) sg_adam_multi(float *__restrict__ th, float *__restrict__ m,
                                                    float *__restrict__ v,
                                                    const float *__restrict__ g, int64_t n,
                                                    float lr, float b1, float b2, float eps,
                                                    float wd, const float *__restrict__ bp,
                                                    double *__restrict__ part) {
  __shared__ double red[4];
  const float alpha = lr * sqrtf(1.f - bp[1]) / (1.f - bp[0]);
  const float c1 = 1.f - b1, c2 = 1.f - b2;
  double reg = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float tv = th[i];
    reg += (double)tv * (double)tv;
    float mi = m[i], vi = v[i];
    const float ti = adam_elem(tv, g[i], mi, vi, wd, c1, c2, alpha, eps);
    m[i] = mi;
    v[i] = vi;
    th[i] = ti;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) reg += __shfl_xor(reg, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = reg;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(64) sg_adam_final(const double *__restrict__ part, int nb,
                                                   float b1, float b2, float wd,
                                                   float *__restrict__ bp,
                                                   float *__restrict__ reg_loss) {
  double v = 0.0;
  for (int b = threadIdx.x; b < nb; b += 64) v += part[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (threadIdx.x == 0) {
    bp[0] *= b1;
    bp[1] *= b2;
    if (reg_loss) reg_loss[0] = (float)((double)wd * 0.5 * v);
  }
}

int launch_reduce(const float *slab, int nblk, int C, float *part, float *grad, float *loss,
                  const float *y_stats, int add_label, hipStream_t st) {
  if (nblk <= kOnePassRows) {   // the fused kernel's one-block-per-CU slabs
    hipLaunchKernelGGL(sg_reduce_one, dim3((C + 63) / 64), dim3(1024), 0, st, slab, nblk, C, grad,
                       loss, y_stats, add_label);
    return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
  }
  const int S = nblk < kReduceStrands ? (nblk > 0 ? nblk : 1) : kReduceStrands;
  hipLaunchKernelGGL(sg_reduce_stage1, dim3((C + 63) / 64, S), dim3(256), 0, st, slab, nblk, C, part);
  hipLaunchKernelGGL(sg_reduce_stage2, dim3((C + 255) / 256), dim3(256), 0, st, part, S, C, grad,
                     loss, y_stats, add_label);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

struct PathChoice {
  int status;
  int path;   // 0 generic, 1 fused (sg_fast), 2 fused capacity 32 (sg_fast32)
  bool fast;  // path != 0
  SgGenPlan plan;
};

PathChoice choose_path(const sg_model_t *m, bool bwd) {
  PathChoice c;
  c.status = sg_build_plan(m, &c.plan);
  c.fast = false;
  c.path = 0;
  if (c.status != SG_OK) return c;
  if (sg_fast_supported(m, c.plan)) {
    c.fast = true;
    c.path = 1;
    return c;
  }
  if (sg_fast32_supported(m, c.plan)) {
    c.fast = true;
    c.path = 2;
    return c;
  }
  if (!sg_generic_lds_ok(c.plan, bwd)) c.status = SG_ERR_UNSUPPORTED;
  return c;
}

// workspace layout: [slab rows | reduce partials | (sg_fast32) per-pair NTN buffer];
// the slab is sized for any path (SG_DISABLE_FAST may route a fused-path model to
// the generic kernel after the workspace was sized)
int64_t ntn_offset_floats(const PathChoice &c, int64_t n_pairs) {
  const int64_t C = c.plan.n_params + 1;
  int64_t slab = sg_generic_slab_floats(c.plan, n_pairs);
  if (c.path == 1) {
    const int64_t f = sg_fast_slab_floats(c.plan, n_pairs);
    if (f > slab) slab = f;
  } else if (c.path == 2) {
    const int64_t f = sg_fast32_slab_floats(c.plan, n_pairs);
    if (f > slab) slab = f;
  }
  return (slab + (int64_t)kReduceStrands * C + 63) & ~(int64_t)63;
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int32_t sg_version(void) { return 10900; }   /* 1.9.0: sg_train_step (gradient reduction + Adam in one launch) */

int64_t sg_record_bytes(int32_t n_max) { return sg_record_bytes_ex(n_max, SG_DTYPE_F32); }

int64_t sg_record_bytes_ex(int32_t n_max, int32_t adj_dtype) {
  if (n_max <= 0 || !sg_dtype_ok(adj_dtype)) return 0;
  return (int64_t)sg_rec_layout(n_max, adj_dtype).words * 4;
}

int32_t sg_model_validate(const sg_model_t *model, int64_t *n_params_out, int32_t *path_out) {
  int64_t wn = 0;
  if (sg_web_plan_params(model, &wn) == SG_OK && sg_web_lds_ok(model)) {
    if (n_params_out) *n_params_out = wn;
    if (path_out) *path_out = 3;
    return SG_OK;
  }
  PathChoice c = choose_path(model, true);
  if (c.status != SG_OK) return c.status;
  if (n_params_out) *n_params_out = c.plan.n_params;
  if (path_out) *path_out = c.path;
  return SG_OK;
}

int64_t sg_workspace_bytes(const sg_model_t *model, int64_t n_pairs) {
  PathChoice c = choose_path(model, true);
  if (c.status != SG_OK) return -1;
  const int64_t C = c.plan.n_params + 1;
  // room for either path (SG_DISABLE_FAST may route a fast-path model to the
  // generic kernel after the workspace was sized)
  int64_t bytes = ntn_offset_floats(c, n_pairs) * 4;
  if (c.path == 2 || (c.path == 1 && sg_fast_needs_ntn(c.plan)))
    bytes += sg_fast32_ntn_floats(n_pairs) * 4;   // per-pair NTN-gradient buffer
  bytes = (bytes + 255) & ~(int64_t)255;
  const int64_t label_bytes = (256 + 2) * 8;
  return (bytes > label_bytes ? bytes : label_bytes) + 256;
}

int32_t sg_pack_pairs(const float *store_adj, const int32_t *store_types, const int32_t *store_n,
                      int32_t n_graphs, int32_t n_max, const int32_t *pair_idx,
                      const float *labels, int64_t n_pairs, void *records,
                      int32_t *status_out, sg_stream_t stream) {
  return sg_pack_pairs_ex(store_adj, store_types, store_n, n_graphs, n_max, SG_DTYPE_F32, pair_idx,
                          labels, n_pairs, records, status_out, stream);
}

int32_t sg_pack_pairs_ex(const float *store_adj, const int32_t *store_types,
                         const int32_t *store_n, int32_t n_graphs, int32_t n_max,
                         int32_t adj_dtype, const int32_t *pair_idx, const float *labels,
                         int64_t n_pairs, void *records, int32_t *status_out,
                         sg_stream_t stream) {
  if (n_pairs < 0 || n_max <= 0 || n_max > 64 || n_graphs <= 0) return SG_ERR_ARG;
  if (!sg_dtype_ok(adj_dtype)) return SG_ERR_ARG;
  if (n_pairs == 0) return SG_OK;
  if (!store_adj || !store_types || !store_n || !pair_idx || !records) return SG_ERR_ARG;
  const SgRecLayout rl = sg_rec_layout(n_max, adj_dtype);
  const int wpb = 4;
  const int64_t blocks = (n_pairs + wpb - 1) / wpb;
  if (blocks > 0x7FFFFFFF) return SG_ERR_ARG;
  hipLaunchKernelGGL(sg_pack_kernel, dim3((unsigned)blocks), dim3(64 * wpb), 0, (hipStream_t)stream,
                     store_adj, store_types, store_n, n_graphs, n_max,
                     adj_dtype == SG_DTYPE_BF16 ? 1 : 0, pair_idx, labels, n_pairs,
                     (uint32_t *)records, rl.words, status_out);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int32_t sg_label_stats(const void *records, int64_t n_pairs, int32_t n_max, float *stats_out,
                       void *workspace, sg_stream_t stream) {
  return sg_label_stats_ex(records, n_pairs, n_max, SG_DTYPE_F32, stats_out, workspace, stream);
}

int32_t sg_label_stats_ex(const void *records, int64_t n_pairs, int32_t n_max, int32_t adj_dtype,
                          float *stats_out, void *workspace, sg_stream_t stream) {
  if (!records || !stats_out || !workspace || n_pairs <= 0 || n_max <= 0 || n_max > 64)
    return SG_ERR_ARG;
  if (!sg_dtype_ok(adj_dtype)) return SG_ERR_ARG;
  const SgRecLayout rl = sg_rec_layout(n_max, adj_dtype);
  hipStream_t st = (hipStream_t)stream;
  double *part = (double *)workspace;
  double *mean = part + 256;
  const int nb = 256;
  hipLaunchKernelGGL(sg_label_partial, dim3(nb), dim3(256), 0, st, (const uint8_t *)records,
                     n_pairs, rl.words, rl.label, (const double *)nullptr, part);
  hipLaunchKernelGGL(sg_label_final, dim3(1), dim3(256), 0, st, part, nb, n_pairs, 0, mean,
                     stats_out);
  hipLaunchKernelGGL(sg_label_partial, dim3(nb), dim3(256), 0, st, (const uint8_t *)records,
                     n_pairs, rl.words, rl.label, (const double *)mean, part);
  hipLaunchKernelGGL(sg_label_final, dim3(1), dim3(256), 0, st, part, nb, n_pairs, 1, mean,
                     stats_out);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int64_t sg_pair_order_workspace_bytes(const sg_model_t *model, int64_t n_pairs) {
  if (!model || n_pairs < 0) return -1;
  const int64_t nb = (n_pairs + kOrderChunk - 1) / kOrderChunk;
  return nb * kOrderKeys * 4 + 256;
}

extern "C++" template <class S>
static int32_t launch_order(S src, int nmax, int fast, int64_t n_pairs, int32_t *order_out,
                            void *workspace, hipStream_t st, int32_t *class_start = nullptr) {
  const int K = fast == 1 ? 4 : (fast == 2 ? 4 * 17 : 2 * nmax + 1);
  const int nb = (int)((n_pairs + kOrderChunk - 1) / kOrderChunk);
  int32_t *cnt = (int32_t *)workspace;
  hipLaunchKernelGGL(sg_order_count<S>, dim3(nb), dim3(256), 0, st, src, n_pairs, nmax, fast, K,
                     nb, cnt);
  hipLaunchKernelGGL(sg_order_scan, dim3(1), dim3(1024), 0, st, cnt, (int64_t)K * nb);
  hipLaunchKernelGGL(sg_order_scatter<S>, dim3(nb), dim3(256), 0, st, src, n_pairs, nmax, fast, K,
                     nb, (const int32_t *)cnt, order_out);
  if (class_start)
    hipLaunchKernelGGL(sg_order_starts, dim3(1), dim3(256), 0, st, (const int32_t *)cnt, K, nb,
                       n_pairs, class_start);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int32_t sg_pair_order(const sg_model_t *model, const void *records, int64_t n_pairs,
                      int32_t *order_out, void *workspace, sg_stream_t stream) {
  if (n_pairs < 0 || n_pairs > 0x7FFFFFFF) return SG_ERR_ARG;
  if (n_pairs == 0) return SG_OK;
  if (!records || !order_out || !workspace) return SG_ERR_ARG;
  PathChoice c = choose_path(model, true);
  if (c.status != SG_OK) return c.status;
  const int nmax = c.plan.n_max;
  const SgRecLayout rl = sg_rec_layout(nmax, c.plan.adj_dtype);
  OrderRecs src{(const uint8_t *)records, rl.words, rl.adj_words + 2 * nmax};
  return launch_order(src, nmax, c.path, n_pairs, order_out, workspace, (hipStream_t)stream);
}

int32_t sg_pair_order_cls(const sg_model_t *model, const void *records, int64_t n_pairs,
                          int32_t *order_out, int32_t *class_start, void *workspace,
                          sg_stream_t stream) {
  if (n_pairs < 0 || n_pairs > 0x7FFFFFFF) return SG_ERR_ARG;
  if (!class_start) return SG_ERR_ARG;
  PathChoice c = choose_path(model, true);
  if (c.status != SG_OK) return c.status;
  if (c.path != 1) return SG_ERR_UNSUPPORTED;   // the class-exclusive schedule is sg_fast's
  hipStream_t st = (hipStream_t)stream;
  if (n_pairs == 0)
    return hipMemsetAsync(class_start, 0, SG_FAST_CLASSES_P1 * 4u, st) == hipSuccess ? SG_OK
                                                                                     : SG_ERR_HIP;
  if (!records || !order_out || !workspace) return SG_ERR_ARG;
  const int nmax = c.plan.n_max;
  const SgRecLayout rl = sg_rec_layout(nmax, c.plan.adj_dtype);
  OrderRecs src{(const uint8_t *)records, rl.words, rl.adj_words + 2 * nmax};
  return launch_order(src, nmax, 1, n_pairs, order_out, workspace, st, class_start);
}

// a store-sourced call's checks: fused capacity-32 path, f32 Â, store shape = n_max
static int32_t src_check(const PathChoice &c, const sg_pair_source_t *src) {
  if (!src || !src->adj || !src->types || !src->n || src->n_graphs <= 0) return SG_ERR_ARG;
  if ((c.path != 1 && c.path != 2) || c.plan.adj_dtype != SG_DTYPE_F32) return SG_ERR_UNSUPPORTED;
  if (src->n_max != c.plan.n_max || src->grid_base < 0) return SG_ERR_ARG;
  return SG_OK;
}

int32_t sg_pair_order_src(const sg_model_t *model, const sg_pair_source_t *src,
                          int64_t n_pairs, int32_t *order_out, void *workspace,
                          sg_stream_t stream) {
  if (n_pairs < 0 || n_pairs > 0x7FFFFFFF) return SG_ERR_ARG;
  PathChoice c = choose_path(model, true);
  if (c.status != SG_OK) return c.status;
  const int32_t rc = src_check(c, src);
  if (rc != SG_OK) return rc;
  if (n_pairs == 0) return SG_OK;
  if (!order_out || !workspace) return SG_ERR_ARG;
  OrderStore os{src->n, src->pair_idx, src->grid_base, src->n_graphs};
  return launch_order(os, c.plan.n_max, c.path, n_pairs, order_out, workspace,
                      (hipStream_t)stream);
}

int32_t sg_forward(const sg_model_t *model, const void *records, int64_t n_pairs,
                   int64_t pair_offset, const float *params, uint64_t seed, float *s_out,
                   void *workspace, sg_stream_t stream) {
  return sg_forward_ex(model, records, nullptr, n_pairs, pair_offset, params, seed, s_out,
                       workspace, stream);
}

static int32_t forward_impl(const sg_model_t *model, const void *records, const int32_t *order,
                            const int32_t *class_start, int64_t n_pairs, int64_t pair_offset,
                            const float *params, uint64_t seed, float *s_out,
                            sg_stream_t stream) {
  if (n_pairs < 0 || pair_offset < 0) return SG_ERR_ARG;
  if (order && n_pairs > 0x7FFFFFFF) return SG_ERR_ARG;
  if (class_start && !order) return SG_ERR_ARG;
  if (n_pairs == 0) return SG_OK;
  if (!records || !params || !s_out) return SG_ERR_ARG;
  PathChoice c = choose_path(model, false);
  if (c.status != SG_OK) return c.status;
  if (class_start && c.path != 1) return SG_ERR_UNSUPPORTED;
  if (c.path == 1)
    return sg_fast_run(model, c.plan, false, records, order, n_pairs, pair_offset, n_pairs, params,
                       seed, nullptr, s_out, nullptr, nullptr, nullptr, (hipStream_t)stream,
                       nullptr, nullptr, class_start);
  if (c.path == 2)
    return sg_fast32_run(model, c.plan, false, records, order, n_pairs, pair_offset, n_pairs,
                         params, seed, nullptr, s_out, nullptr, nullptr, nullptr,
                         (hipStream_t)stream);
  return sg_generic_run(c.plan, false, records, order, n_pairs, pair_offset, n_pairs, params, seed,
                        nullptr, s_out, nullptr, nullptr, (hipStream_t)stream);
}

int32_t sg_forward_ex(const sg_model_t *model, const void *records, const int32_t *order,
                      int64_t n_pairs, int64_t pair_offset, const float *params, uint64_t seed,
                      float *s_out, void *workspace, sg_stream_t stream) {
  (void)workspace;
  return forward_impl(model, records, order, nullptr, n_pairs, pair_offset, params, seed, s_out,
                      stream);
}

int32_t sg_forward_cls(const sg_model_t *model, const void *records, const int32_t *order,
                       const int32_t *class_start, int64_t n_pairs, int64_t pair_offset,
                       const float *params, uint64_t seed, float *s_out, void *workspace,
                       sg_stream_t stream) {
  (void)workspace;
  if (!order || !class_start) return SG_ERR_ARG;
  return forward_impl(model, records, order, class_start, n_pairs, pair_offset, params, seed,
                      s_out, stream);
}

int32_t sg_fwd_bwd(const sg_model_t *model, const void *records, int64_t n_pairs,
                   int64_t pair_offset, int64_t batch_total, const float *params, uint64_t seed,
                   const float *y_stats, int32_t add_label_term, float *s_out, float *grad_out,
                   float *loss_out, void *workspace, sg_stream_t stream) {
  return sg_fwd_bwd_ex(model, records, nullptr, n_pairs, pair_offset, batch_total, params, seed,
                       y_stats, add_label_term, s_out, grad_out, loss_out, workspace, stream);
}

static int32_t fwd_bwd_impl(const sg_model_t *model, const void *records, const int32_t *order,
                            int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                            const float *params, uint64_t seed, const uint64_t *seed_dev,
                            const float *y_stats, int32_t add_label_term, float *s_out,
                            float *grad_out, float *loss_out, void *workspace,
                            sg_stream_t stream, const sg_pair_source_t *src = nullptr,
                            const int32_t *class_start = nullptr,
                            const sg_adam_args_t *adam = nullptr) {
  if (n_pairs < 0 || pair_offset < 0) return SG_ERR_ARG;
  if (order && n_pairs > 0x7FFFFFFF) return SG_ERR_ARG;
  if (class_start && !order) return SG_ERR_ARG;
  if (!params || !grad_out || !workspace) return SG_ERR_ARG;
  PathChoice c = choose_path(model, true);
  if (c.status != SG_OK) return c.status;
  if (src) {
    const int32_t rc = src_check(c, src);
    if (rc != SG_OK) return rc;
  }
  if (seed_dev && c.path != 1) return SG_ERR_UNSUPPORTED;   // device seed: fused path only
  if (class_start && c.path != 1) return SG_ERR_UNSUPPORTED;   // class table: sg_fast only
  if (model->loss_mode == SG_LOSS_BROADCAST && !y_stats) return SG_ERR_ARG;
  if (model->loss_mode == SG_LOSS_ALIGNED && batch_total <= 0) return SG_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int C = c.plan.n_params + 1;
  float *slab = (float *)workspace;
  if (adam && n_pairs == 0) return SG_ERR_ARG;   // (no update from an empty batch)
  // one-call Adam covers up to 65,536 parameters (the fused reduction's columns, or
  // sg_adam_tf's single workgroup); larger models call sg_fwd_bwd_* + sg_adam_tf_ex
  if (adam && C - 1 > 65536) return SG_ERR_UNSUPPORTED;
  if (n_pairs == 0) {
    if (hipMemsetAsync(grad_out, 0, (size_t)c.plan.n_params * 4u, st) != hipSuccess)
      return SG_ERR_HIP;
    if (loss_out && hipMemsetAsync(loss_out, 0, 4u, st) != hipSuccess) return SG_ERR_HIP;
    return SG_OK;
  }
  if (!records && !src) return SG_ERR_ARG;
  // sg_train_step: the fused path's gradient reduction applies Adam in the same launch
  // (sg_reduce_adam) with the step scalars the fused kernel's block 0 leaves in the
  // reduction's partial rows (unused by the one-pass reduction)
  const bool fuse_adam = adam && c.path == 1;
  float *adam_pre = slab + ntn_offset_floats(c, n_pairs) - (int64_t)kReduceStrands * C;
  SgAdamPre pre_args;
  if (fuse_adam) {
    pre_args.bp = adam->beta_powers;
    pre_args.out = adam_pre;
    pre_args.lr = adam->lr;
    pre_args.b1 = adam->beta1;
    pre_args.b2 = adam->beta2;
    pre_args.wd = adam->weight_decay;
  }
  int nblk = 0;
  int rc;
  if (c.path == 1)
    rc = sg_fast_run(model, c.plan, true, records, order, n_pairs, pair_offset, batch_total,
                     params, seed, y_stats, s_out, slab, slab + ntn_offset_floats(c, n_pairs),
                     &nblk, st, seed_dev, src, class_start, fuse_adam ? &pre_args : nullptr);
  else if (c.path == 2)
    rc = sg_fast32_run(model, c.plan, true, records, order, n_pairs, pair_offset, batch_total,
                       params, seed, y_stats, s_out, slab, slab + ntn_offset_floats(c, n_pairs),
                       &nblk, st, src);
  else
    rc = sg_generic_run(c.plan, true, records, order, n_pairs, pair_offset, batch_total, params,
                        seed, y_stats, s_out, slab, &nblk, st);
  if (rc != SG_OK) return rc;
  const int add_label = model->loss_mode == SG_LOSS_BROADCAST ? add_label_term : 0;
  if (fuse_adam && nblk <= kOnePassRows) {
    hipLaunchKernelGGL(sg_reduce_adam, dim3((C + 63) / 64), dim3(1024), 0, st, slab, nblk, C,
                       grad_out, loss_out, y_stats, add_label, (float *)params, adam->m, adam->v,
                       adam->beta1, adam->beta2, adam->eps, adam->weight_decay,
                       (const float *)adam_pre, adam->beta_powers, adam->reg_loss_out);
    return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
  }
  float *part = slab + (size_t)nblk * C;
  rc = launch_reduce(slab, nblk, C, part, grad_out, loss_out, y_stats, add_label, st);
  if (rc != SG_OK || !adam) return rc;
  return sg_adam_tf((float *)params, adam->m, adam->v, grad_out, C - 1, adam->lr, adam->beta1,
                    adam->beta2, adam->eps, adam->weight_decay, adam->beta_powers,
                    adam->reg_loss_out, stream);
}

int32_t sg_fwd_bwd_ex(const sg_model_t *model, const void *records, const int32_t *order,
                      int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                      const float *params, uint64_t seed, const float *y_stats,
                      int32_t add_label_term, float *s_out, float *grad_out, float *loss_out,
                      void *workspace, sg_stream_t stream) {
  return fwd_bwd_impl(model, records, order, n_pairs, pair_offset, batch_total, params, seed,
                      nullptr, y_stats, add_label_term, s_out, grad_out, loss_out, workspace,
                      stream);
}

int32_t sg_fwd_bwd_cls(const sg_model_t *model, const void *records, const int32_t *order,
                       const int32_t *class_start, int64_t n_pairs, int64_t pair_offset,
                       int64_t batch_total, const float *params, uint64_t seed,
                       const float *y_stats, int32_t add_label_term, float *s_out,
                       float *grad_out, float *loss_out, void *workspace, sg_stream_t stream) {
  if (!order || !class_start) return SG_ERR_ARG;
  return fwd_bwd_impl(model, records, order, n_pairs, pair_offset, batch_total, params, seed,
                      nullptr, y_stats, add_label_term, s_out, grad_out, loss_out, workspace,
                      stream, nullptr, class_start);
}

int32_t sg_train_step(const sg_model_t *model, const void *records, const int32_t *order,
                      const int32_t *class_start, int64_t n_pairs, int64_t pair_offset,
                      int64_t batch_total, float *params, uint64_t seed, const float *y_stats,
                      int32_t add_label_term, float *s_out, float *grad_out, float *loss_out,
                      void *workspace, const sg_adam_args_t *adam, sg_stream_t stream) {
  if (!adam || !adam->m || !adam->v || !adam->beta_powers) return SG_ERR_ARG;
  if (class_start && !order) return SG_ERR_ARG;
  return fwd_bwd_impl(model, records, order, n_pairs, pair_offset, batch_total, params, seed,
                      nullptr, y_stats, add_label_term, s_out, grad_out, loss_out, workspace,
                      stream, nullptr, class_start, adam);
}

int32_t sg_train_step_dseed(const sg_model_t *model, const void *records, const int32_t *order,
                            int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                            float *params, const uint64_t *seed_dev, const float *y_stats,
                            int32_t add_label_term, float *s_out, float *grad_out,
                            float *loss_out, void *workspace, const sg_adam_args_t *adam,
                            sg_stream_t stream) {
  if (!seed_dev || !adam || !adam->m || !adam->v || !adam->beta_powers) return SG_ERR_ARG;
  return fwd_bwd_impl(model, records, order, n_pairs, pair_offset, batch_total, params, 0,
                      seed_dev, y_stats, add_label_term, s_out, grad_out, loss_out, workspace,
                      stream, nullptr, nullptr, adam);
}

int32_t sg_fwd_bwd_src(const sg_model_t *model, const sg_pair_source_t *src,
                       const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                       int64_t batch_total, const float *params, uint64_t seed,
                       const float *y_stats, int32_t add_label_term, float *s_out,
                       float *grad_out, float *loss_out, void *workspace, sg_stream_t stream) {
  if (!src) return SG_ERR_ARG;
  return fwd_bwd_impl(model, nullptr, order, n_pairs, pair_offset, batch_total, params, seed,
                      nullptr, y_stats, add_label_term, s_out, grad_out, loss_out, workspace,
                      stream, src);
}

int32_t sg_forward_src(const sg_model_t *model, const sg_pair_source_t *src,
                       const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                       const float *params, uint64_t seed, float *s_out, void *workspace,
                       sg_stream_t stream) {
  (void)workspace;
  if (n_pairs < 0 || pair_offset < 0) return SG_ERR_ARG;
  if (order && n_pairs > 0x7FFFFFFF) return SG_ERR_ARG;
  PathChoice c = choose_path(model, false);
  if (c.status != SG_OK) return c.status;
  const int32_t rc = src_check(c, src);
  if (rc != SG_OK) return rc;
  if (n_pairs == 0) return SG_OK;
  if (!params || !s_out) return SG_ERR_ARG;
  if (c.path == 1)
    return sg_fast_run(model, c.plan, false, nullptr, order, n_pairs, pair_offset, n_pairs, params,
                       seed, nullptr, s_out, nullptr, nullptr, nullptr, (hipStream_t)stream,
                       nullptr, src);
  return sg_fast32_run(model, c.plan, false, nullptr, order, n_pairs, pair_offset, n_pairs, params,
                       seed, nullptr, s_out, nullptr, nullptr, nullptr, (hipStream_t)stream, src);
}

int32_t sg_fwd_bwd_dseed(const sg_model_t *model, const void *records, const int32_t *order,
                         int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                         const float *params, const uint64_t *seed_dev, const float *y_stats,
                         int32_t add_label_term, float *s_out, float *grad_out, float *loss_out,
                         void *workspace, sg_stream_t stream) {
  if (!seed_dev) return SG_ERR_ARG;
  return fwd_bwd_impl(model, records, order, n_pairs, pair_offset, batch_total, params, 0,
                      seed_dev, y_stats, add_label_term, s_out, grad_out, loss_out, workspace,
                      stream);
}

__global__ void sg_seed_add_kernel(uint64_t *seed, uint64_t delta) {
  if (threadIdx.x == 0) seed[0] += delta;
}

int32_t sg_seed_advance(uint64_t *seed_dev, uint64_t delta, sg_stream_t stream) {
  if (!seed_dev) return SG_ERR_ARG;
  hipLaunchKernelGGL(sg_seed_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, seed_dev,
                     delta);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int32_t sg_adam_tf(float *params, float *m, float *v, const float *grad, int64_t n, float lr,
                   float beta1, float beta2, float eps, float weight_decay, float *beta_powers,
                   float *reg_loss_out, sg_stream_t stream) {
  if (!params || !m || !v || !grad || !beta_powers || n <= 0) return SG_ERR_ARG;
  hipLaunchKernelGGL(sg_adam_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, params, m, v,
                     grad, n, lr, beta1, beta2, eps, weight_decay, beta_powers, reg_loss_out);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int64_t sg_adam_workspace_bytes(int64_t n) {
  if (n < 0) return -1;
  return (int64_t)kAdamBlocks * 8 + 256;
}

int32_t sg_adam_tf_ex(float *params, float *m, float *v, const float *grad, int64_t n, float lr,
                      float beta1, float beta2, float eps, float weight_decay, float *beta_powers,
                      float *reg_loss_out, void *workspace, sg_stream_t stream) {
  if (!params || !m || !v || !grad || !beta_powers || n <= 0) return SG_ERR_ARG;
  if (n <= 65536 || !workspace)
    return sg_adam_tf(params, m, v, grad, n, lr, beta1, beta2, eps, weight_decay, beta_powers,
                      reg_loss_out, stream);
  hipStream_t st = (hipStream_t)stream;
  int64_t nb = (n + 255) / 256;
  if (nb > kAdamBlocks) nb = kAdamBlocks;
  double *part = (double *)workspace;
  hipLaunchKernelGGL(sg_adam_multi, dim3((unsigned)nb), dim3(256), 0, st, params, m, v, grad, n,
                     lr, beta1, beta2, eps, weight_decay, (const float *)beta_powers, part);
  hipLaunchKernelGGL(sg_adam_final, dim3(1), dim3(64), 0, st, (const double *)part, (int)nb, beta1,
                     beta2, weight_decay, beta_powers, reg_loss_out);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int64_t sg_web_workspace_bytes(const sg_model_t *model, int64_t chunk) {
  if (!model || chunk <= 0) return -1;   // chunk 0 = n_pairs: use sg_web_workspace_bytes_ex
  return sg_web_ws_bytes(model, chunk, -1);   // any n_pairs: both pipeline slots
}

int32_t sg_web_release(void) { return sg_web_release_aux(); }

int64_t sg_web_workspace_bytes_ex(const sg_model_t *model, int64_t chunk, int64_t n_pairs) {
  if (!model || chunk < 0 || n_pairs < 0) return -1;
  return sg_web_ws_bytes(model, chunk, n_pairs);
}

int32_t sg_web_forward(const sg_model_t *model, const sg_csr_store_t *store,
                       const int32_t *pair_idx, int64_t n_pairs, int64_t pair_offset,
                       const float *params, uint64_t seed, float *s_out, void *workspace,
                       int64_t chunk, sg_stream_t stream) {
  if (n_pairs < 0 || pair_offset < 0 || chunk < 0) return SG_ERR_ARG;
  if (n_pairs == 0) return SG_OK;
  if (!pair_idx || !params || !s_out || !workspace) return SG_ERR_ARG;
  return sg_web_run(model, store, pair_idx, nullptr, n_pairs, pair_offset, n_pairs, params, seed,
                    nullptr, 0, s_out, nullptr, nullptr, workspace, chunk, false,
                    (hipStream_t)stream);
}

int32_t sg_web_fwd_bwd(const sg_model_t *model, const sg_csr_store_t *store,
                       const int32_t *pair_idx, const float *labels, int64_t n_pairs,
                       int64_t pair_offset, int64_t batch_total, const float *params,
                       uint64_t seed, const float *y_stats, int32_t add_label_term, float *s_out,
                       float *grad_out, float *loss_out, void *workspace, int64_t chunk,
                       sg_stream_t stream) {
  if (n_pairs < 0 || pair_offset < 0 || chunk < 0) return SG_ERR_ARG;
  if (!params || !grad_out || !workspace) return SG_ERR_ARG;
  if (n_pairs > 0 && !pair_idx) return SG_ERR_ARG;
  if (model && model->loss_mode == SG_LOSS_BROADCAST && !y_stats) return SG_ERR_ARG;
  if (model && model->loss_mode == SG_LOSS_ALIGNED && (batch_total <= 0 || (n_pairs > 0 && !labels)))
    return SG_ERR_ARG;
  return sg_web_run(model, store, pair_idx, labels, n_pairs, pair_offset, batch_total, params,
                    seed, y_stats, add_label_term, s_out, grad_out, loss_out, workspace, chunk,
                    true, (hipStream_t)stream);
}

}  // extern "C"
