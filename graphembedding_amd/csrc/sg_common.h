// sg_common.h — shared device helpers of libsiamese_hip (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/siamese_hip.h"

#define SG_WAVE 64

// Timing ablations (scripts/gpu_abl_*.sh) remove work and give WRONG results.  They
// compile only together with SG_TIMING_ABLATION_BUILD, which build.py never passes to
// the product library (graphembedding_amd/lib/libsiamese_hip.so), so a hand build
// with one ablation macro alone fails here instead of producing a silently wrong .so.
#if (defined(SG32_ABL_NOREC) || defined(SG32_ABL_NONTN) || defined(SG_WEB_ABL_NOH2)) && \
    !defined(SG_TIMING_ABLATION_BUILD)
#error "timing ablation macro without SG_TIMING_ABLATION_BUILD: results would be invalid"
#endif

// sg_train_step: what the fused kernel's block 0 needs to compute ApplyAdam's step
// scalars out[4] = {α, β1^t·β1, β2^t·β2, wd·½Σθ²} before the reduction launch applies the
// update (host struct, copied into the kernel arguments)
struct SgAdamPre {
  const float *bp;   // device [2] β powers {β1^t, β2^t}
  float *out;        // device [4]
  float lr, b1, b2, wd;
};

// ---------------------------------------------------------------------------
// Counter-based dropout RNG.  Bit-exact twin of oracle/siamese_oracle.py
// (sg_mix, seed_key, dropout_mask).  Replaces TF's unseeded
// floor(keep + U[0,1)) masks of layers.py:332-338 / tf.nn.dropout.
// ---------------------------------------------------------------------------
// 24-bit-multiply lowbias32 variant: (x & 0xFFFFFF) * C is one full-rate
// v_mul_u32_u24 on gfx950.
__host__ __device__ __forceinline__ uint32_t sg_mix(uint32_t x) {
  x ^= x >> 16;
  x = (x & 0xFFFFFFu) * 0x7FEB35u;
  x ^= x >> 15;
  x = (x & 0xFFFFFFu) * 0x846CA7u;
  x ^= x >> 16;
  return x;
}

static inline uint32_t sg_seed_key(uint64_t seed) {
  const uint32_t lo = (uint32_t)(seed & 0xFFFFFFFFull);
  const uint32_t hi = (uint32_t)(seed >> 32);
  return (lo * 0x85EBCA6Bu) ^ hi;
}

static inline uint32_t sg_keep_threshold(float keep) {
  if (keep >= 1.0f) return 65536u;
  double t = (double)keep * 65536.0;
  long r = (long)(t + 0.5);  // round half up == numpy round for these values
  if (r < 0) r = 0;
  if (r > 65536) r = 65536;
  return (uint32_t)r;
}

__device__ __forceinline__ uint32_t sg_pair_key(uint32_t key, uint32_t pair) {
  return sg_mix(pair ^ key);
}

// One 32-bit hash per (pair, layer, element e of one side's tensor) serves that
// element of both sides: low 16 bits side 0, high 16 bits side 1 (e < 2^26).
__device__ __forceinline__ uint32_t sg_hash(uint32_t pk, uint32_t layer, uint32_t e) {
  return sg_mix(((layer << 26) | e) ^ pk);
}

__device__ __forceinline__ bool sg_keep(uint32_t pk, uint32_t layer, uint32_t side, uint32_t e,
                                        uint32_t thr) {
  if (thr >= 65536u) return true;
  const uint32_t h = sg_hash(pk, layer, e);
  const uint32_t d = side ? (h >> 16) : (h & 0xFFFFu);
  return d < thr;
}

// ---------------------------------------------------------------------------
// Activations (layers_factory.py:101-114); gradients as TF's (ReluGrad: x>0).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sg_act(int act, float x) {
  switch (act) {
    case SG_ACT_RELU: return x > 0.f ? x : 0.f;
    case SG_ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    case SG_ACT_TANH: return tanhf(x);
    default: return x;
  }
}

__device__ __forceinline__ float sg_act_grad(int act, float pre, float out, float g) {
  switch (act) {
    case SG_ACT_RELU: return pre > 0.f ? g : 0.f;
    case SG_ACT_SIGMOID: return g * out * (1.f - out);
    case SG_ACT_TANH: return g * (1.f - out * out);
    default: return g;
  }
}

// Final activation and its derivative (similarity.py:55-60, layers_factory.py:101-114).
__device__ __forceinline__ float sg_final(int fa, float yeta, float s) {
  switch (fa) {
    case SG_FINAL_GAUSSIAN: return expf(-yeta * s * s);
    case SG_FINAL_RELU: return s > 0.f ? s : 0.f;
    case SG_FINAL_SIGMOID: return 1.f / (1.f + expf(-s));
    case SG_FINAL_TANH: return tanhf(s);
    default: return s;
  }
}

__device__ __forceinline__ float sg_final_grad(int fa, float yeta, float s, float yhat) {
  switch (fa) {
    case SG_FINAL_GAUSSIAN: return -2.f * yeta * s * yhat;
    case SG_FINAL_RELU: return s > 0.f ? 1.f : 0.f;
    case SG_FINAL_SIGMOID: return yhat * (1.f - yhat);
    case SG_FINAL_TANH: return 1.f - yhat * yhat;
    default: return 1.f;
  }
}

// Wave-local LDS hand-off: every prior LDS access of this wave has landed and
// the compiler may not move memory operations across.
__device__ __forceinline__ void sg_wsync() {
  // a wavefront-scope fence: orders this wave's LDS accesses in the compiler and emits no
  // wait (a wave's DS operations are performed in program order; the compiler still waits
  // for the values it reads)
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float sg_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Pair record field offsets in 4-byte words (see siamese_hip.h).  The HBM
// record stores Â as f32 or bf16 (adj_dtype); kernels stage every record into
// LDS in the f32 layout (sg_rec_layout(n_max)).
struct SgRecLayout {
  int n_max;
  int dtype;      // sg_dtype of Â
  int words;      // record size in 4-byte words (multiple of 4: 16-B records)
  int adj;        // [2][n_max][n_max] f32, or bf16 packed two per word
  int adj_words;  // 2 n_max² (f32) or n_max² (bf16)
  int types;      // [2][n_max] i32
  int nnodes;     // [2] i32
  int label;      // f32
  int tag;        // i32
};

static inline SgRecLayout sg_rec_layout(int n_max, int dtype = SG_DTYPE_F32) {
  SgRecLayout r;
  r.n_max = n_max;
  r.dtype = dtype;
  r.adj = 0;
  r.adj_words = dtype == SG_DTYPE_BF16 ? n_max * n_max : 2 * n_max * n_max;
  r.types = r.adj_words;
  r.nnodes = r.types + 2 * n_max;
  r.label = r.nnodes + 2;
  r.tag = r.label + 1;
  r.words = (r.tag + 1 + 3) & ~3;
  return r;
}

static inline bool sg_dtype_ok(int dtype) { return dtype == SG_DTYPE_F32 || dtype == SG_DTYPE_BF16; }

// bf16 (RNE) of an f32, the record encoding of SG_DTYPE_BF16 (NaN-free inputs)
__host__ __device__ __forceinline__ uint32_t sg_f32_to_bf16(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// One pair record (layout in siamese_hip.h) gathered from a dense-slot graph store by
// one wavefront (lane = 0..63): store Â [G][nmax][nmax] f32, types [G][nmax], n [G].
// Invalid graph ids write a zero record and SG_ERR_ARG into *status.
__device__ __forceinline__ void sg_pack_record(const float *__restrict__ sadj,
                                               const int32_t *__restrict__ stypes,
                                               const int32_t *__restrict__ sn, int n_graphs,
                                               int nmax, int bf16, int g0, int g1, float label,
                                               int64_t tag, uint32_t *__restrict__ dst,
                                               int rec_words, int lane,
                                               int32_t *__restrict__ status) {
  const bool bad = g0 < 0 || g0 >= n_graphs || g1 < 0 || g1 >= n_graphs;
  if (bad && lane == 0 && status) atomicExch(status, (int32_t)SG_ERR_ARG);
  const int nn = nmax * nmax;
  const int aw = bf16 ? nn : 2 * nn;               // adjacency words
  const int tail = 2 * nmax + 4;                    // types, n_nodes, label, tag
  auto adj_at = [&](int e) -> float {               // e in [0, 2 nn): side e / nn
    const int s = e / nn, o = e - s * nn;
    return sadj[(size_t)(s ? g1 : g0) * nn + o];
  };
  for (int w = lane; w < rec_words; w += SG_WAVE) {
    uint32_t v = 0u;
    if (!bad) {
      if (w < aw) {
        v = bf16 ? (sg_f32_to_bf16(adj_at(2 * w)) | (sg_f32_to_bf16(adj_at(2 * w + 1)) << 16))
                 : __float_as_uint(adj_at(w));
      } else if (w < aw + tail) {
        const int o = w - aw;
        if (o < 2 * nmax) {
          const int s = o / nmax, i = o - s * nmax;
          v = (uint32_t)stypes[(size_t)(s ? g1 : g0) * nmax + i];
        } else if (o < 2 * nmax + 2) {
          v = (uint32_t)sn[(o == 2 * nmax) ? g0 : g1];
        } else if (o == 2 * nmax + 2) {
          v = __float_as_uint(label);
        } else {
          v = (uint32_t)(tag & 0x7FFFFFFF);
        }
      }
    }
    dst[w] = v;
  }
}
