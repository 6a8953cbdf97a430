// sg_fast.hip — fused fwd(+bwd) kernel for the reference's default Siamese
// stack (config.py:44-66): GCN(d_in→32, relu, sparse one-hot) → GCN(32→16,
// identity) → Dense(16→1, relu) → Padding(D) → NTN(D, K=10, relu), every layer
// with bias and dropout, Gaussian final act, broadcast or aligned MSE.
//
// AVG = true instantiates the tuning.py stack (tuning.py:66-93): GCN → GCN →
// Average (layers.py:136-140) → NTN(16, K=10): the NTN input is the node mean of H2
// (16 features) instead of the Dense/Padding node vector; the GCN part is shared.
//
// One wavefront owns one graph pair at a time.  The pair record is staged in
// LDS; each graph instance is one 16-row MFMA tile whose rows are the nodes.
// All seven GCN products (Â·Z0, D1·W1, Â·Z1 forward; Âᵀ·gH2, D1ᵀ·gZ1, gZ1·W1ᵀ,
// Âᵀ·gP1 backward) run on v_mfma_f32_16x16x4_f32 — exact f32, bit-for-bit a
// k-ordered fmaf chain.  Node n lives in tile row ρ(n) = 4·(n%4) + n/4, so the
// accumulator of one product (lane (g,j) holds rows 4g..4g+3) IS the B operand
// of the next Â product with the K index permuted (k-step κ ↔ rows 4g+κ), and
// rows 4g+3 are empty for n ≤ 12: Â products need 3 k-steps, not 4 (2 for
// sides of ≤ 8 nodes: the pair body is instantiated per (K0, K1) class, and
// pairs of two ≤ 8-node sides share one tile in the feature products).  The
// feature-contracting products need one 16×32 / 16×16 transpose through LDS.
// The one-hot gW0 = Xᵀ·gZ0 product runs on bf16 MFMA with gZ0 split in three
// bf16 parts (one-hot is exact in bf16).  The NTN head runs on VALU (D = K = 10
// is too small for MFMA to pay): lanes (g, k = j) own NTN weight rows
// a ∈ {g, g+4, g+8}, the tiles' node map; cross-row sums use DPP and permlanes.
// Parameter gradients accumulate in registers (gW1, gW0 in MFMA accumulators),
// are flushed once per launch through LDS, waves summed in a fixed order, into
// one slab row per workgroup (deterministic).
#include <type_traits>

#include "sg_plan.h"
#include "sg_mfma.h"

int sg_num_cus();

namespace {

using namespace sgk;

constexpr int FH1 = 32, FH2 = 16, FK = 10;
constexpr int TS1 = 36;  // D1 tile row stride (floats)
constexpr int TS2 = 20;  // gZ1 tile row stride
constexpr int W1S = 20;  // W1 table row stride (16 + pad)
constexpr int W1TS = 36; // W1ᵀ table row stride (32 + pad)
// gD1 = gZ1·W1ᵀ runs on bf16 MFMA with both operands split in three parts (x = h + m + l,
// the six leading products: ≈ f32 accuracy); W1's parts are built once per launch.  It
// takes gZ1 with nodes on the lanes' rows (its A operand): the gZ1 tile (nodes on the
// accumulator rows, as Âᵀ·gH2 leaves it) goes through the wave's LDS and is read back
// transposed.  (The variants these replaced, and their measurements, are in
// profiles/HISTORY.md: f32 gD1, gZ1ᵀ recomputed on the f32 MFMA.)
//
// Scheduling fence around each f32 MFMA product: its MFMAs then issue back to back instead
// of one at a time between VALU instructions.  On gfx950 every switch between
// v_mfma_f32_16x16x4_f32 and VALU in a wave's stream costs issue cycles
// (scripts/mfma_valu_mix.hip: 4 MFMAs + 48 FMAs take 7.6% longer interleaved than grouped);
// the scheduler's default is to interleave.  Measured 470.3 -> 480.7 M pairs/s.
__device__ __forceinline__ void mfma_fence() { __builtin_amdgcn_sched_barrier(0); }
// waves per block: 8 = 2 waves per SIMD at up to 256 VGPRs per lane
constexpr int MAXW = 8;

struct FastArgs {
  const uint8_t *recs;
  const int32_t *order;   // processing order (sg_pair_order) or null
  // class table of the order (sg_pair_order_cls) or null: the order's slots
  // [cls[c], cls[c + 1]) hold the records of cost class c = (N0 > 8) + 2 (N1 > 8); each
  // wave then runs ONE class (its own loop: no register copies at a class join), the
  // waves split over the classes by work (count x cost weight cw[c])
  const int32_t *cls;
  float cw[4];
  // relative pair throughput of the 8 XCDs (block b is assumed to run on XCD b % 8, which
  // only decides speed: any placement gives the same results), scaled integers; a class's
  // slots are split over its waves in proportion to their XCD's weight when the waves hold
  // many pairs (SG_XCD_W)
  int xw[8];
  int xw_even;   // all eight weights equal (the default): the split is plain integer shares
  int64_t n_pairs;
  int64_t pair_offset;
  int rw4h;      // 16-B words per HBM record (f32 or bf16 Â)
  int rec_bf16;  // Â stored as bf16: widened to the f32 LDS layout while staging
  const float *params;
  const float *y_stats;
  float *s_out;
  float *slab;
  float *ntn;     // AVG backward: [n_pairs][80] = x1|1 (32) | x2|1 (32) | gm (16), for the
                  // NTN W/V/b gradients of sg_ntn_wgrad (sg_fast32.hip)
  uint32_t key;
  const uint64_t *seed_dev;   // non-null: the dropout seed is read from device memory
                              // (graph-captured steps, sg_fwd_bwd_dseed)
  // sg_train_step (backward, ad_out non-null): block 0 computes ApplyAdam's step scalars
  // from the parameters it stages, ad_out[4] = {α, β1^t·β1, β2^t·β2, wd·½Σθ²} with
  // β^t = ad_bp[0..1], so that the reduction launch's blocks (sg_reduce_adam) only read them
  const float *ad_bp;
  float *ad_out;
  float ad_lr, ad_b1, ad_b2, ad_wd;
  uint32_t thr0, thr1, thr2, thr4;
  float ik0, ik1, ik2, ik4;
  float yeta;
  float inv_batch;
  int d_in, n_params;
  int shared_floats, wave_floats;
  int oW0, ob0, oW1, ob1, oWd, obd, oW, oV, oU, obn;
  int oWa;   // Attention weights (ATT), -1 otherwise
  // pair source (sg_pair_source_t): src_store = 1 gathers each record from the dense
  // graph store instead of reading a packed one
  int src_store, G;
  const float *sadj;
  const int32_t *stypes, *sn, *spairs;
  int64_t grid_base;
  const float *slabels;
  int32_t *status;
};

// 16-B word w4 of pair p's f32 record (sg_rec_layout(D): Â of both sides, types of
// both sides, n0, n1, label, tag) gathered from the dense store, one dword at a time
// (the store rows are D·D and D words: no 16-B alignment to rely on).  Invalid graph
// ids read as a zero record and raise *status, as sg_pack_pairs does.
template <int D>
__device__ __forceinline__ uint4 fast_store_word(const FastArgs &A, int p, int w4, int lane) {
  int g0, g1;
  if (A.spairs) {
    g0 = A.spairs[2 * (int64_t)p];
    g1 = A.spairs[2 * (int64_t)p + 1];
  } else {
    const int64_t q = A.grid_base + p;
    g0 = (int)(q / A.G);
    g1 = (int)(q - (int64_t)g0 * A.G);
  }
  const bool ok = (unsigned)g0 < (unsigned)A.G && (unsigned)g1 < (unsigned)A.G;
  if (!ok && lane == 0 && A.status) atomicExch(A.status, (int32_t)SG_ERR_ARG);
  constexpr int NN = D * D;
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int w = 4 * w4 + k;
    uint32_t x = 0u;
    if (ok) {
      if (w < 2 * NN) {
        const int s = w >= NN;
        x = __float_as_uint(A.sadj[(size_t)(s ? g1 : g0) * NN + (w - s * NN)]);
      } else if (w < 2 * NN + 2 * D) {
        const int t = w - 2 * NN, s = t >= D;
        x = (uint32_t)A.stypes[(size_t)(s ? g1 : g0) * D + (t - s * D)];
      } else if (w == 2 * NN + 2 * D) {
        x = (uint32_t)A.sn[g0];
      } else if (w == 2 * NN + 2 * D + 1) {
        x = (uint32_t)A.sn[g1];
      } else if (w == 2 * NN + 2 * D + 2) {
        x = __float_as_uint(A.slabels ? A.slabels[p] : 0.f);
      } else if (w == 2 * NN + 2 * D + 3) {
        x = (uint32_t)p;
      }
    }
    v[k] = x;
  }
  return uint4{v[0], v[1], v[2], v[3]};
}

// Attention pooling (ATT, with AVG = true: the 16-feature pooled head): the 16x16
// weight table at row stride 17 (conflict-free row and column reads)
constexpr int WAS = 17;

template <int D, bool AVG = false, bool ATT = false>
struct FastLds {
  // NTN width DN (the Padding width D, or H2's 16 features after Average), the row
  // stride WR of the NTN W tables and VS of the V table
  // VS = 34 (≡ 2 mod 32): the V reads sV[kc·VS + a] of lanes (g, kc) hit distinct banks
  // (2 kc + g); a stride of 24 or 32 put three or ten rows kc on one bank
  static constexpr int DN = AVG ? FH2 : D, WR = AVG ? 16 : 12, VS = 34;
  static_assert(2 * DN <= VS, "V row");
  static constexpr int RW = 2 * D * D + 2 * D + 4;  // record words (multiple of 4)
  static constexpr int REC = 0;
  static constexpr int TILE = REC + RW;               // 2 x 16 x TS1 (D1 tiles)
  static constexpr int X = TILE + 2 * 16 * TS1;       // x1 | x2 (at 12, or 16 for AVG); [47] = 0
  static constexpr int GE = X + 48;                   // AVG: ∂L/∂x1 | ∂L/∂x2 (16 each)
  static constexpr int TMP = GE + 32;                 // ATT: node means of H2 (16 per side)
  static constexpr int GU = TMP + 32;                 // ATT: ∂L/∂(tanh input) (16 per side)
  static constexpr int GT = GU + 32;                  // gZ1 tiles, 2 x 16 x TS2
  // (the gZ1 tiles only in the backward: the forward-only kernel keeps its smaller
  // regions and with them two blocks per CU)
  static int wave_floats(int, bool bwd) {
    return bwd ? GT + 2 * 16 * TS2 : X + 48 + (AVG ? 32 : 0) + (ATT ? 64 : 0);
  }
  static int shared_floats(int d_in) {
    return (d_in + 1) * FH1 + 2 * DN * FK * WR + FK * VS + FH1 * W1S + FH2 * W1TS +
           2 * 3 * 64 * 4 + (ATT ? FH2 * WAS : 0);
  }
};


// Flush slots of one lane: gW1 (8) | gW0/ik0 (16) | NTN dW (RN·DN) | dV (RN + RN) |
// dbn, dU, loss | db0 (2), db1, dWd, dbd (pre-summed over row groups) | ATT: gWa (4)
template <int D, bool AVG = false, bool ATT = false>
struct FlushSlots {
  static constexpr int DN = FastLds<D, AVG>::DN, RN = (DN + 3) / 4;
  // AVG: the NTN W, V and bias gradients go through the per-pair buffer instead
  static constexpr int NWS = AVG ? 0 : RN * DN, NVS = AVG ? 0 : 2 * RN;
  static constexpr int NS = 8 + 16 + NWS + NVS + 3 + 5 + (ATT ? 4 : 0);
};

// parameter index of slot s on lane l = 16 g + j, or -1 if the slot is padding
template <int D, bool AVG, bool ATT>
__device__ __forceinline__ int fast_param(const FastArgs &A, int s, int l) {
  constexpr int DN = FastLds<D, AVG>::DN, RN = (DN + 3) / 4;
  constexpr int NWS = FlushSlots<D, AVG>::NWS, NVS = FlushSlots<D, AVG>::NVS;
  const int g = l >> 4, j = l & 15;
  if (s < 8) return A.oW1 + (16 * (s >> 2) + 4 * g + (s & 3)) * FH2 + j;
  s -= 8;
  if (s < 16) {
    const int ty = 16 * (s >> 3) + 4 * g + (s & 3);
    return ty < A.d_in ? A.oW0 + ty * FH1 + 16 * ((s >> 2) & 1) + j : -1;
  }
  s -= 16;
  if (s < NWS) {
    const int a = 4 * (s / DN) + g, b = s % DN;
    return (a < DN && j < FK) ? A.oW + (a * DN + b) * FK + j : -1;
  }
  s -= NWS;
  if (s < NVS) {
    const int a = 4 * (s % RN) + g;
    return (a < DN && j < FK) ? A.oV + j * 2 * DN + (s >= RN ? DN : 0) + a : -1;
  }
  s -= NVS;
  switch (s) {
    case 0: return (!AVG && g == 0 && j < FK) ? A.obn + j : -1;
    case 1: return (g == 0 && j < FK) ? A.oU + j : -1;
    case 2: return l == 0 ? A.n_params : -1;
    case 3: return g == 0 ? A.ob0 + j : -1;
    case 4: return g == 0 ? A.ob0 + 16 + j : -1;
    case 5: return g == 0 ? A.ob1 + j : -1;
    case 6: return (!AVG && g == 0) ? A.oWd + j : -1;
    case 7: return (!AVG && l == 0) ? A.obd : -1;
    default: break;
  }
  s -= 8;
  // ATT: lane (g, j) slot i holds gWa[4i + g][j] (Attention weights [input_dim][input_dim])
  return (ATT && s < 4) ? A.oWa + (4 * s + g) * FH2 + j : -1;
}

// The NTN head's FMAs over element pairs (b, b + 1): one v_pk_fma_f32, the same two fmaf
// chains as two v_fma_f32.  Unlike split3's packed subtractions (SG_SPLIT_PK), these keep
// their register pairs: the plain form measured 1.1% slower on C2 (profiles/r05_n).
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// tanh and the logistic function from v_exp_f32 and v_rcp_f32 (the Attention layer's h
// and att, layers.py:156-157).  Both are ≈1e-7 ABSOLUTE error: sg_tanh's 1 - 2/(e^2z + 1)
// cancels for small |z| (relative error ≈1e-7/|z|, e.g. 1e-3 at |z| = 1e-4), which the
// oracle tolerances (1e-4 on the score) absorb
__device__ __forceinline__ float sg_tanh(float z) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * z) + 1.f);
}
__device__ __forceinline__ float sg_sigmoid(float z) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-z));
}

// xsum32(xsum16(a)) and xsum32(xsum16(b)) at once, bitwise the same sums ((x0 + x1) +
// (x2 + x3) over the four rows of 16 lanes): v_permlane16_swap(a, b) leaves [a0, b0, a2, b2]
// and [a1, b1, a3, b3], one add gives [a01, b01, a23, b23]; a permlane32 swap and an add
// give [a, b, a, b], and a last permlane16 swap spreads a and b to every lane.  7 VALU
// (two of them register copies) for what two separate reductions do in 12.
__device__ __forceinline__ void xsum_pair(float &a, float &b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false,
                                                  false);
  const float s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false,
                                                  false);
  const float t = __uint_as_float(q[0]) + __uint_as_float(q[1]);
  const auto z = __builtin_amdgcn_permlane16_swap(__float_as_uint(t), __float_as_uint(t), false,
                                                  false);
  a = __uint_as_float(z[0]);
  b = __uint_as_float(z[1]);
}

#ifdef SG_FAST_TIMING
// Diagnostic build only (scripts/fast_timing.py): per-wave s_memrealtime stamps
// (100 MHz) at start / after the prologue / after the pair loop / at the end,
// plus the wave's pair count.
constexpr int kTimeWaves = 4096;
__device__ unsigned long long sg_fast_times[kTimeWaves * 5];
#define SG_STAMP(slot, val)                                                        \
  do {                                                                             \
    const int tw_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);            \
    if ((threadIdx.x & 63) == 0 && tw_ < kTimeWaves) sg_fast_times[tw_ * 5 + (slot)] = (val); \
  } while (0)
#else
#define SG_STAMP(slot, val) do {} while (0)
#endif

template <int D, bool BWD, bool ALIGNED, bool INTENDED, bool AVG, bool SRC, bool ATT>
__global__ void __launch_bounds__(64 * MAXW) sg_fast_kernel(FastArgs A) {
  static_assert(!ATT || AVG, "Attention pooling uses the 16-feature pooled head");
  SG_STAMP(0, __builtin_amdgcn_s_memrealtime());
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using L = FastLds<D, AVG, ATT>;
  constexpr int DN = L::DN, RN = (DN + 3) / 4, WR = L::WR, VS = L::VS;
  constexpr int XO2 = AVG ? 16 : 12;       // x2 offset in the wave's x region
  constexpr uint32_t NL = AVG ? 3u : 4u;   // layer index of the NTN (its dropout key)
  constexpr int RW4 = L::RW / 4;
  constexpr int NREC = (RW4 + 63) / 64;
  const int tid = threadIdx.x;
  const int l = tid & 63, nw = blockDim.x >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: pair index in SGPRs
  const int g = l >> 4, j = l & 15;
  // dropout hash inputs pk ^ (layer << 26 | e): e = this lane's element index splits
  // into a uniform part (r, t) and these per-lane parts (disjoint bit fields)
  const uint32_t lb1 = (uint32_t)(FH1 * g + j);   // layer 1: e = 32 n + f, n = 4r+g, f = 16t+j
  const uint32_t lb2 = (uint32_t)(FH2 * g + j);   // layer 2: e = 16 n + j
  const int d_in = A.d_in;
  const float *__restrict__ prm = A.params;
  uint32_t key = A.key;   // sg_seed_key of the dropout seed
  const uint32_t thr0s = __builtin_amdgcn_readfirstlane(A.thr0);
  const uint32_t thr4s = __builtin_amdgcn_readfirstlane(A.thr4);
  if (A.seed_dev) {
    const uint64_t sd = *A.seed_dev;
    key = ((uint32_t)sd * 0x85EBCA6Bu) ^ (uint32_t)(sd >> 32);
  }

  // the parameter staging's loads go out first: their latency overlaps the class table's
  // and the order's (the first record waits for those: class table -> slot -> order entry)
  float *stg = smem + A.shared_floats;   // fast_cfg sizes LDS for n_params floats here
  const int nprm = A.n_params, bdx = (int)blockDim.x;
  float stv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = k * bdx + tid;
    stv[k] = i < nprm ? prm[i] : 0.f;
  }
  const bool ad_blk = BWD && A.ad_out != nullptr && blockIdx.x == 0 && wv == 0;
  float ad_b1p = 0.f, ad_b2p = 0.f;
  if (ad_blk) {
    ad_b1p = A.ad_bp[0];
    ad_b2p = A.ad_bp[1];
  }

  // ---- pair schedule; the first record is loaded during the prologue ----
  // Slots are handed out round by round (round r: slots [r·S, r·S + S), S = all
  // waves of the grid).  With an order (sg_pair_order: records sorted by cost
  // class) the waves walk the rounds as a snake (odd rounds reversed), so every
  // wave gets the same class mix and the launch has no slow tail; slot q then
  // holds record order[q].  p is the record (= batch pair index) either way.
  // (32-bit indices: sg_fast_run admits n_pairs < 2^31 - grid)
  const int npairs = (int)A.n_pairs;
  const int stride = (int)gridDim.x * nw;
  const int gw = (int)blockIdx.x * nw + wv;
  const int32_t *__restrict__ ord = A.order;
  // Class-exclusive schedule (A.cls): wave gw takes class cwave and the slot range
  // [cs0, cs1) of that class; every wave computes the same split (scalar code).  The
  // waves are divided over the classes in proportion to count x cost weight (largest
  // remainder), then each class's slots evenly over its waves.  Needs one wave per
  // non-empty class; otherwise (tiny batches) the mixed schedule runs.
  int cwave = -1, cs0 = 0, cs1 = 0;
  if (ord != nullptr && A.cls != nullptr) {
    int cb[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) cb[c] = __builtin_amdgcn_readfirstlane(A.cls[c]);
    float wt[4], tot = 0.f;
    int nonempty = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int nc = cb[c + 1] - cb[c];
      wt[c] = nc > 0 ? (float)nc * A.cw[c] : 0.f;
      tot += wt[c];
      nonempty += nc > 0;
    }
    // the two waves of a SIMD (w and w ^ 4 of a block) always take the same class: the
    // waves are allocated in SIMD pairs and enumerated block by block in the order
    // (0, 4, 1, 5, 2, 6, 3, 7), so no SIMD runs pairs of two classes side by side (two
    // classes' pair costs were fitted with partners of their own class)
    const bool align = nw == 8;
    const int units = align ? stride >> 1 : stride;
    const int pos = align ? (gw & ~7) + 2 * (gw & 3) + ((gw >> 2) & 1) : gw;
    if (nonempty > 0 && units >= nonempty) {
      int wc[4], used = 0;
      float fr[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float x = wt[c] > 0.f ? (float)(units - nonempty) * (wt[c] / tot) : 0.f;
        const int fl = (int)x;
        wc[c] = wt[c] > 0.f ? 1 + fl : 0;   // at least one unit per non-empty class
        fr[c] = x - (float)fl;
        used += wc[c];
      }
      for (int left = units - used; left > 0; --left) {   // largest remainders, ties to low c
        int bc = 0;
        float bf = -1.f;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (wt[c] > 0.f && fr[c] > bf) {
            bf = fr[c];
            bc = c;
          }
        wc[bc] += 1;
        fr[bc] = -2.f;
      }
      if (align) {
#pragma unroll
        for (int c = 0; c < 4; ++c) wc[c] *= 2;   // waves
      }
      int cum = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (cwave < 0 && pos < cum + wc[c]) {
          const int nc = cb[c + 1] - cb[c];
          cwave = c;
          // A class's nc slots over its wc waves.  Waves holding many pairs (N = 1 sizes)
          // split them in proportion to their XCD's weight: the XCDs run the pair loop at
          // measurably different speeds, the same on every box measured (profiles/r05_f,
          // timing.log: XCD 3 and 7 the slowest, 0 and 4 the fastest), and the launch
          // ends with the slowest XCD.  F(x) is the weight of the positions below x
          // (8 positions per block, block b on XCD b % 8); the boundaries are integer
          // quotients of cumulative weights, so the shares tile the class exactly.
          const int q = nc / wc[c], r = nc - q * wc[c];
          if (q >= 64 && A.xw_even) {
            // equal weights: F(x) = w·x below, so the shares are floor(nc·k / wc) exactly;
            // in 32 bits when nc·wc fits (a 64-bit division expands to a long scalar+VALU
            // sequence on the prologue's critical path)
            const int k = pos - cum;
            // (the 32-bit division expands on VALU: readfirstlane keeps the wave-uniform
            // bounds in SGPRs, else the pair loop's slot tests become divergent branches)
            if ((uint64_t)(uint32_t)nc * (uint32_t)wc[c] < (1ull << 32)) {
              cs0 = cb[c] + __builtin_amdgcn_readfirstlane(
                                (int)(((uint32_t)nc * (uint32_t)k) / (uint32_t)wc[c]));
              cs1 = cb[c] + __builtin_amdgcn_readfirstlane(
                                (int)(((uint32_t)nc * (uint32_t)(k + 1)) / (uint32_t)wc[c]));
            } else {
              cs0 = cb[c] + (int)((int64_t)nc * k / wc[c]);
              cs1 = cb[c] + (int)((int64_t)nc * (k + 1) / wc[c]);
            }
          } else if (q >= 64) {
            auto F = [&](int x) -> int64_t {
              const int xb = (x >> 3) & 7;
              int64_t pre = 0, tot = 0;
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                tot += A.xw[i];
                pre += i < xb ? A.xw[i] : 0;
              }
              return (int64_t)(x >> 6) * 8 * tot + 8 * pre + (int64_t)(x & 7) * A.xw[xb];
            };
            const int64_t f0 = F(cum), span = F(cum + wc[c]) - f0;
            cs0 = cb[c] + (int)((int64_t)nc * (F(pos) - f0) / span);
            cs1 = cb[c] + (int)((int64_t)nc * (F(pos + 1) - f0) / span);
          } else {
            // Few pairs per wave (an 8-GPU rank's share): q or q + 1 each, and the r = nc %
            // wc waves that take q + 1 are the OLDER waves of their SIMD pair (bit 2 of the
            // grid wave index clear) first: the last pair of a long wave then tends to run
            // beside a partner that has finished, at the single-wave rate, instead of beside
            // another long wave (the launch tail is about one pair).  old(x) counts the older
            // waves in [0, x) of the enumeration (every other position when aligned).
            int k;
            if (align) {
              k = ((gw & 4) == 0 ? 0 : wc[c] >> 1) + ((pos - cum) >> 1);
            } else {
              auto old_below = [](int x) -> int { return (x >> 3) * 4 + min(x & 7, 4); };
              const int end = cum + wc[c];
              const int n_old = old_below(end) - old_below(cum);
              k = (gw & 4) == 0 ? old_below(gw) - old_below(cum)
                                : n_old + (gw - old_below(gw)) - (cum - old_below(cum));
            }
            cs0 = cb[c] + k * q + min(k, r);
            cs1 = cs0 + q + (k < r ? 1 : 0);
          }
        }
        cum += wc[c];
      }
    }
  }
  const bool cls_mode = cwave >= 0;
  const int qend = cls_mode ? cs1 : npairs;   // slots of this wave run below qend
  auto slot_of = [&](int r) -> int {
    if (cls_mode) return cs0 + r;
    return r * stride + ((ord != nullptr && (r & 1)) ? stride - 1 - gw : gw);
  };
  // record indices of 64 rounds, lane i ↔ round r0 + i (read back with readlane)
  auto load_ord = [&](int r0) -> int {
    const int s = slot_of(r0 + l);
    return s < qend ? ord[s] : 0;
  };
  // an entry read back from ordA, clamped (scalar) so a bad order never reads out of bounds
  auto ord_at = [&](int v, int lane) -> int {
    const int x = __builtin_amdgcn_readlane(v, lane);
    return x < 0 ? 0 : (x >= npairs ? npairs - 1 : x);
  };
  int ordA = 0, ordB = 0;
  if (ord) {
    ordA = load_ord(0);
    ordB = load_ord(64);
  }

  float *sW0 = smem;                            // W0 · ik0 · ik1, row d_in zero
  float *sWa = sW0 + (d_in + 1) * FH1;          // [a][k][12]: W[a][b][k] at b
  float *sWb = sWa + DN * FK * WR;              // [b][k][WR]: W[a][b][k] at a
  float *sV = sWb + DN * FK * WR;               // [k][VS]
  float *sW1 = sV + FK * VS;                    // W1 · ik1 [32][16], row stride W1S (gD1)
  float *sW1T = sW1 + FH1 * W1S;                // W1ᵀ [16][32], row stride W1TS (Z1)
  // [t][term][lane] bf16 B operands of gD1: lane (g, j) ↔ column 16t + j,
  // k-slots 8g..8g+3 / 8g+4..8g+7 ↔ parts of W1[16t + j][4g..4g+3]·ik1
  uint4 *sW1B = (uint4 *)(sW1T + FH2 * W1TS);
  // ATT: Attention weights Wa[j'][k] at row stride WAS
  float *sWat = (float *)(sW1B + 2 * 3 * 64);
  float *W = smem + A.shared_floats + wv * A.wave_floats;
  float *sRec = W + L::REC;
  float *sT = W + L::TILE;
  float *sX = W + L::X;

  // Prologue.  The raw parameter vector is staged into LDS (in the wave regions,
  // unused until the pair loop) in one pass with all loads in flight, and the
  // tables are built from there: one global-load latency instead of one per table.
  // Dropout scales are folded into the tables that feed the dropped tensors:
  // Z0 = (W0 · ik0 · ik1)[type] (with b0 · ik1: P1 comes out scaled by the layer-1
  // dropout scale, relu(ik1 x) = ik1 relu(x)) and gP1 = keep·relu' · (gZ1 (W1 · ik1)ᵀ).
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = k * bdx + tid;
    if (i < nprm) stg[i] = stv[k];
  }
  for (int i = 8 * bdx + tid; i < nprm; i += bdx) stg[i] = prm[i];   // small blocks only
  // first record: its HBM latency overlaps the table build below
  int q = slot_of(0);
  int p = (ord && q < qend) ? ord_at(ordA, 0) : q;
  // HBM record: rw4h 16-B words (RW4 for f32 Â, fewer for bf16 Â)
  const int rw4h = A.rw4h;
  constexpr int ADJ4 = D * D / 4;   // 16-B words of a bf16 adjacency block (D even)
  uint4 pre[NREC];
#pragma unroll
  for (int c = 0; c < NREC; ++c) {
    const int w4 = l + 64 * c;
    pre[c] = (q < qend && w4 < rw4h)
                 ? (SRC ? fast_store_word<D>(A, p, w4, l)
                                : ((const uint4 *)(A.recs + (size_t)p * (size_t)rw4h * 16u))[w4])
                 : uint4{0u, 0u, 0u, 0u};
  }
  __syncthreads();
  if (ad_blk) {   // sg_train_step's step scalars (see FastArgs::ad_out), from the staged θ
    double ss = 0.0;
    for (int i = l; i < nprm; i += 64) {
      const double t = (double)stg[i];
      ss += t * t;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if (l == 0) {
      A.ad_out[0] = A.ad_lr * sqrtf(1.f - ad_b2p) / (1.f - ad_b1p);
      A.ad_out[1] = ad_b1p * A.ad_b1;
      A.ad_out[2] = ad_b2p * A.ad_b2;
      A.ad_out[3] = (float)((double)A.ad_wd * 0.5 * ss);
    }
  }
  // the tables' elements of this thread: (a) the sources of every table read from the staged
  // copy, then (b) all stores (512-thread blocks, the launch's shape).  Strided loops that
  // read and store in turn took one LDS round trip per element (the compiler may not move
  // a read above a store to the same array): ≈20 round trips of the 1.8 µs table build.
  auto wa_src = [&](int i, bool tr) -> float {   // sWa (tr: sWb) element i
    const int x = i / (FK * WR), rem = i - x * FK * WR, k = rem / WR, y = rem - k * WR;
    return y < DN ? stg[A.oW + (tr ? (y * DN + x) : (x * DN + y)) * FK + k] : 0.f;
  };
  auto v_src = [&](int i) -> float {
    const int k = i / VS, c = i - k * VS;
    return c < 2 * DN ? stg[A.oV + k * 2 * DN + c] : 0.f;
  };
  constexpr int NWA = DN * FK * WR, KWA = (NWA + 511) / 512, NVT = FK * VS, KV = (NVT + 511) / 512;
  static_assert(FH1 * FH2 == 512, "one W1 element per thread of a 512-thread block");
  const int nw0 = (d_in + 1) * FH1;
  if (bdx == 512 && nw0 <= 3 * 512) {
    float r0[3], ra[KWA], rb[KWA], rv[KV];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = min(tid + 512 * k, nw0 - 1);
      r0[k] = i < d_in * FH1 ? stg[A.oW0 + i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KWA; ++k) {
      const int i = min(tid + 512 * k, NWA - 1);
      ra[k] = wa_src(i, false);
      rb[k] = wa_src(i, true);
    }
#pragma unroll
    for (int k = 0; k < KV; ++k) rv[k] = v_src(min(tid + 512 * k, NVT - 1));
    const float w1 = stg[A.oW1 + tid];
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (tid + 512 * k < nw0) sW0[tid + 512 * k] = r0[k] * (A.ik0 * A.ik1);
#pragma unroll
    for (int k = 0; k < KWA; ++k)
      if (tid + 512 * k < NWA) {
        sWa[tid + 512 * k] = ra[k];
        sWb[tid + 512 * k] = rb[k];
      }
#pragma unroll
    for (int k = 0; k < KV; ++k)
      if (tid + 512 * k < NVT) sV[tid + 512 * k] = rv[k];
    sW1[(tid / FH2) * W1S + tid % FH2] = w1 * A.ik1;
    sW1T[(tid % FH2) * W1TS + tid / FH2] = w1;
  } else {   // smaller blocks (batches of a few pairs)
    for (int i = tid; i < nw0; i += bdx)
      sW0[i] = i < d_in * FH1 ? stg[A.oW0 + i] * (A.ik0 * A.ik1) : 0.f;
    for (int i = tid; i < NWA; i += bdx) {
      sWa[i] = wa_src(i, false);
      sWb[i] = wa_src(i, true);
    }
    for (int i = tid; i < NVT; i += bdx) sV[i] = v_src(i);
    for (int i = tid; i < FH1 * FH2; i += bdx) {
      const float w = stg[A.oW1 + i];
      sW1[(i / FH2) * W1S + i % FH2] = w * A.ik1;
      sW1T[(i % FH2) * W1TS + i / FH2] = w;
    }
  }
  for (int i = tid; i < 2 * 3 * 64; i += blockDim.x) {
    const int t = i / 192, term = (i / 64) % 3, ln = i & 63;
    const int f = 16 * t + (ln & 15), k0 = 4 * (ln >> 4);
    const float *wr = stg + A.oW1 + f * FH2 + k0;
    uint32_t h01, m01, l01, h23, m23, l23;
    split3(wr[0] * A.ik1, wr[1] * A.ik1, h01, m01, l01);
    split3(wr[2] * A.ik1, wr[3] * A.ik1, h23, m23, l23);
    sW1B[i] = term == 0 ? uint4{h01, h23, h01, h23}
                        : (term == 1 ? uint4{m01, m23, h01, h23} : uint4{l01, l23, m01, m23});
  }
  if constexpr (ATT)
    for (int i = tid; i < FH2 * FH2; i += blockDim.x) sWat[(i >> 4) * WAS + (i & 15)] = stg[A.oWa + i];
  // per-lane parameters, also from the staged copy
  const int j_ = tid & 15;
  const float b0v0 = stg[A.ob0 + j_] * A.ik1, b0v1 = stg[A.ob0 + 16 + j_] * A.ik1;
  const float b1v = stg[A.ob1 + j_];
  // Dense weight with the layer-2 dropout scale folded in (D2 is kept unscaled; the
  // Dense weight gradient takes ik2 at the flush)
  const float wdv = AVG ? 0.f : stg[A.oWd + j_] * A.ik2;
  const float bd = AVG ? 0.f : stg[A.obd];
  const bool kv = j_ < FK;
  const int kc = kv ? j_ : FK - 1;
  const float Uk = kv ? stg[A.oU + kc] : 0.f;
  const float bnk = kv ? stg[A.obn + kc] : 0.f;
  float usum = 0.f;
#pragma unroll
  for (int k = 0; k < FK; ++k) usum += stg[A.oU + k];
  __syncthreads();   // the staging area is dead: the waves take their regions
  static_assert((2 * 16 * TS1) % 4 == 0, "D1 tiles in float4s");
  for (int i = l; i < 2 * 16 * TS1 / 4; i += 64) ((f4 *)sT)[i] = f4{0.f, 0.f, 0.f, 0.f};
  if (l < 48) sX[l] = 0.f;   // wave-private: the pair loop's first sg_wsync orders it
  SG_STAMP(1, __builtin_amdgcn_s_memrealtime());

  // ---- per-lane constants ----
  // MFMA B fragment of W1 read from LDS at use: W1[8g+q][j] (Z1 = D1 W1)
  const float *w1bp = sW1T + j * W1TS + 8 * g;
  // NTN lane role: k = j (valid < FK); rows a = 4r + g, r < 3 (valid < D)
  // A-operand row of this lane: tile row i = j ↔ node ni.  Â is read at static
  // per-lane offsets; entries outside the n_max × n_max block (tile rows and
  // columns past n_max) read the always-zero sX[47].  Entries of absent nodes
  // inside the block are zero by the record contract (siamese_hip.h).
  const int ri = j & 3, ni = 4 * ri + (j >> 2);
  int afo[2][3];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int c = 4 * q + g;
      afo[s][q] = (ri < 3 && ni < D && c < D) ? L::REC + s * D * D + ni * D + c : L::X + 47;
    }
  // Pairs with both sides <= 8 nodes share one 16-row tile in the feature products
  // (D1·W1 and gZ1·W1ᵀ): tile rows with r = i % 4 < 2 are side 0's, rows with r >= 2
  // side 1's row i - 2.  This lane's A row i = j comes from side jp, row jr.
  const int jp = (j >> 1) & 1, jr = j - 2 * jp;
  const float *sTp = sT + jp * 16 * TS1 + jr * TS1 + 8 * g;   // shared-tile D1 row j
  int tyo[3];   // record word of the type of node 4r + g (side 0; side 1 at + D)
#pragma unroll
  for (int r = 0; r < 3; ++r) tyo[r] = 2 * D * D + (4 * r + g < D ? 4 * r + g : 0);

  // ---- accumulators ----
  f4 gw1[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  // gW0 / ik0 = Σ Xᵀ·gZ0 on MFMA: [type tile τ][feature tile t], rows = types 16τ + 4g + r
  f4 gw0[2][2] = {{f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}},
                  {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}}};
  float gb0a0 = 0.f, gb0a1 = 0.f, gb1a = 0.f, gwda = 0.f, gbda = 0.f;
  constexpr int RW_ = AVG ? 1 : RN, DW_ = AVG ? 1 : DN;   // AVG: per-pair buffer instead
  // the NTN head's FMAs run as v_pk_fma_f32 over element pairs (b, b + 1): one issue
  // for two FMAs (scripts/pk_fma_rate.hip); the x / W rows are 8-byte aligned in LDS
  f2 gWn[RW_][(DW_ + 1) / 2];
  float gVa[RW_], gVb[RW_];
#pragma unroll
  for (int r = 0; r < RW_; ++r) {
    gVa[r] = gVb[r] = 0.f;
#pragma unroll
    for (int b = 0; b < (DW_ + 1) / 2; ++b) gWn[r][b] = f2{0.f, 0.f};
  }
  float gbn = 0.f, gUa = 0.f, lossa = 0.f;
  float gwa[4] = {0.f, 0.f, 0.f, 0.f};   // ATT: gWa[4i + g][j]
  const float ybar = (BWD && !ALIGNED) ? A.y_stats[0] : 0.f;

  // Waves w and w ^ 4 share a SIMD (round-robin placement).  Issue arbitration
  // favours the older wave, which would finish its pairs far ahead and leave the
  // younger one alone on the SIMD for the last ~third of the launch.  The higher
  // priority alternates between the two by pair count (PRIO_PERIOD pairs, the
  // younger wave holding it in PRIO_YOUNG of them); ties still favour the
  // older wave.  The pair → wave assignment is unchanged.
  constexpr int PRIO_PERIOD = 3, PRIO_YOUNG = 2;
  int it = 0;
  const int young = wv >> 2;   // 0 / 1, wave-uniform (scalar)
  // The pair loop: CLS < 0 = mixed schedule (each pair dispatches to its (K0, K1) body);
  // CLS = c: every pair of this wave has class c, one body, so the loop-carried
  // accumulators need no copies at a join of four bodies (≈55 v_mov_b32 per pair)
  auto pair_loop = [&](auto CLSc) __attribute__((always_inline)) {
  constexpr int CLS = decltype(CLSc)::value;
  for (; q < qend; ++it) {
    // (scalar integers: as bools the comparison went through VALU selects; one
    // conditional instead of an if / else)
    const int yturn = (int)((unsigned)((it % PRIO_PERIOD) - PRIO_YOUNG) >> 31);   // < YOUNG
    __builtin_amdgcn_s_setprio(0);
    if ((yturn ^ young) == 0) __builtin_amdgcn_s_setprio(1);
    sg_wsync();
    if (A.rec_bf16) {
#pragma unroll
      for (int c = 0; c < NREC; ++c) {
        const int w4 = l + 64 * c;
        const uint4 v = pre[c];
        if (w4 < ADJ4) {   // 8 bf16 entries of Â → 8 f32
          f4 lo = {__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xFFFF0000u),
                   __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xFFFF0000u)};
          f4 hi = {__uint_as_float(v.z << 16), __uint_as_float(v.z & 0xFFFF0000u),
                   __uint_as_float(v.w << 16), __uint_as_float(v.w & 0xFFFF0000u)};
          ((f4 *)sRec)[2 * w4] = lo;
          ((f4 *)sRec)[2 * w4 + 1] = hi;
        } else if (w4 < rw4h) {
          ((uint4 *)sRec)[w4 + ADJ4] = v;
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < NREC; ++c) {
        const int w4 = l + 64 * c;
        if (w4 < RW4) ((uint4 *)sRec)[w4] = pre[c];
      }
    }
    sg_wsync();
    const int pcur = p;
    {
      const int qn = slot_of(it + 1);
      int pn = qn;
      if (ord) {
        const int rl = (it + 1) & 63;
        if (rl == 0) {
          ordA = ordB;
          ordB = load_ord(it + 65);
        }
        pn = qn < qend ? ord_at(ordA, rl) : 0;
      }
#pragma unroll
      for (int c = 0; c < NREC; ++c) {
        const int w4 = l + 64 * c;
        if (qn < qend && w4 < rw4h)
          pre[c] = SRC
                       ? fast_store_word<D>(A, pn, w4, l)
                       : ((const uint4 *)(A.recs + (size_t)pn * (size_t)rw4h * 16u))[w4];
      }
      q = qn;
      p = pn;
    }
    const int *ty = (const int *)sRec;
    // wave-uniform node counts (clamped to n_max)
    int N0 = __builtin_amdgcn_readfirstlane(((const int *)sRec)[2 * D * D + 2 * D]);
    int N1 = __builtin_amdgcn_readfirstlane(((const int *)sRec)[2 * D * D + 2 * D + 1]);
    N0 = N0 < 0 ? 0 : (N0 > D ? D : N0);
    N1 = N1 < 0 ? 0 : (N1 > D ? D : N1);
    const uint32_t pk = sg_pair_key(key, (uint32_t)(A.pair_offset + pcur));
    // the hash inputs of layers 1 and 2 as (pk ^ lb) ^ element constant (sg_fast32 hides
    // pk ^ lb from re-association against spills; here that measured 1.2% slower)
    const uint32_t pk1 = pk ^ lb1, pk2 = pk ^ lb2;

    // ---- layer-0 (node) and NTN-input dropout masks: one hash per lane, two ballots ----
    // lanes 0..15: layer 0, node e = l; lanes 16..31: layer 4, element e = l - 16.
    // Node presence (e < N_side) is folded in (padded NTN inputs are 0).
    uint32_t km, km4;   // this lane's view: bit 16s + 4r ↔ node / element 4r + g of side s
    uint32_t m4;        // bit 16s + e ↔ NTN-input element e of side s kept
    {
      const int e = l & 15;
      const bool hi = l >= 16;
      const uint32_t h = sg_hash(pk, hi ? NL : 0u, (uint32_t)e);
      // both thresholds as scalar values first: a select between two kernel-argument
      // fields compiled to a per-lane load from the argument block inside the pair loop
      // (global_load + s_waitcnt vmcnt(0), which also waited for the next record's prefetch)
      const uint32_t thr = hi ? thr4s : thr0s;
      // node presence folds into the node mask, and into the NTN mask when the NTN
      // input is indexed by node (Padding); after Average it is indexed by feature
      const bool p0 = (hi && AVG) || e < N0, p1 = (hi && AVG) || e < N1;
      const uint64_t b0 = __ballot((l < 32) & p0 & ((h & 0xFFFFu) < thr));
      const uint64_t b1 = __ballot((l < 32) & p1 & ((h >> 16) < thr));
      const uint32_t m0 = (uint32_t)(b0 & 0xFFFFu) | ((uint32_t)(b1 & 0xFFFFu) << 16);
      m4 = (uint32_t)((b0 >> 16) & 0xFFFFu) | ((uint32_t)b1 & 0xFFFF0000u);
      km = m0 >> g;
      km4 = m4 >> g;
    }
    const float invn0 = N0 > 0 ? 1.f / (float)N0 : 0.f, invn1 = N1 > 0 ? 1.f / (float)N1 : 0.f;

    // Pair body for K0 / K1 node k-steps per side: a side with at most 8 nodes
    // has an all-zero third k-step (nodes 8..11), dropped from every
    // node-contracting product.  Four straight-line instantiations.
    auto body = [&](auto K0c, auto K1c) __attribute__((always_inline)) {
      constexpr int K0 = decltype(K0c)::value, K1 = decltype(K1c)::value;
      // ================= forward =================
      float af[2][3];
      f4 p1[2][2];
      uint32_t tys[2];   // types of rows 4g+r, 6 bits each; 63 = node dropped or absent
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int KS = s ? K1 : K0;
#pragma unroll
        for (int q = 0; q < 3; ++q) af[s][q] = q < KS ? W[afo[s][q]] : 0.f;
        f4 z0[2];
        uint32_t tp = 0u;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          if (r < KS) {
            uint32_t t_ = (uint32_t)ty[tyo[r] + s * D];
            t_ = min(t_, (uint32_t)(d_in - 1));
            const uint32_t k0 = (km >> (16 * s + 4 * r)) & 1u;   // 0 for absent nodes
            const uint32_t tk = k0 ? t_ : 63u;
            tp |= tk << (6 * r);
            const float *w0 = sW0 + (k0 ? t_ : (uint32_t)d_in) * FH1 + j;
            z0[0][r] = w0[0];
            z0[1][r] = w0[16];
          } else {
            tp |= 63u << (6 * r);
            z0[0][r] = z0[1][r] = 0.f;
          }
        }
        tys[s] = tp;
        mfma_fence();
#pragma unroll
        for (int t = 0; t < 2; ++t) {   // ik1 · P1 = Â Z0 + ik1 b0  (absent rows: ik1 b0, never read)
          const float bb = t ? b0v1 : b0v0;
          f4 acc = {bb, bb, bb, bb};
#pragma unroll
          for (int q = 0; q < KS; ++q) acc = mfma4(af[s][q], z0[t][q], acc);
          p1[s][t] = acc;
        }
        mfma_fence();
      }
      // D1 = dropout(ik1 relu(P1)): one hash per element (node 4r+g, feature
      // 16t+j) gives both sides' draws.  The backward reads keep·relu' back as D1 > 0.
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (r < K0 || r < K1) {
            const uint32_t h = sg_mix(pk1 ^ ((1u << 26) | (uint32_t)(128 * r + 16 * t)));
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              float *T = sT + s * 16 * TS1 + (4 * g + r) * TS1 + 16 * t + j;
              if (r < (s ? K1 : K0)) {
                const uint32_t d = s ? (h >> 16) : (h & 0xFFFFu);
                const float v = relu_bits(p1[s][t][r]);
                *T = d < A.thr1 ? v : 0.f;
              } else {
                *T = 0.f;
              }
            }
          } else {
            sT[(4 * g + r) * TS1 + 16 * t + j] = 0.f;
            sT[16 * TS1 + (4 * g + r) * TS1 + 16 * t + j] = 0.f;
          }
        }
      }
      sg_wsync();   // rows 4g+3 of the tiles stay zero from the prologue
      constexpr bool PACK = K0 == 2 && K1 == 2;   // both sides share the feature-product tile
      f4 h2[2];
      if constexpr (PACK) {   // Z1 of both sides in one 16-row tile; H2 = Â Z1 + b1 per side
        const f4 lo = *(const f4 *)sTp, hi = *(const f4 *)(sTp + 4);
        const f4 wlo = *(const f4 *)w1bp, whi = *(const f4 *)(w1bp + 4);
        f4 z1 = {0.f, 0.f, 0.f, 0.f};
        mfma_fence();
#pragma unroll
        for (int q = 0; q < 4; ++q) z1 = mfma4(lo[q], wlo[q], z1);
#pragma unroll
        for (int q = 0; q < 4; ++q) z1 = mfma4(hi[q], whi[q], z1);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          f4 acc = {b1v, b1v, b1v, b1v};
          acc = mfma4(af[s][0], z1[2 * s], acc);
          acc = mfma4(af[s][1], z1[2 * s + 1], acc);
          h2[s] = acc;
        }
        mfma_fence();
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) {   // Z1 = D1 W1 ; H2 = Â Z1 + b1
          const int KS = s ? K1 : K0;
          const float *T = sT + s * 16 * TS1 + j * TS1 + 8 * g;
          const f4 lo = *(const f4 *)T, hi = *(const f4 *)(T + 4);
          const f4 wlo = *(const f4 *)w1bp, whi = *(const f4 *)(w1bp + 4);
          f4 z1 = {0.f, 0.f, 0.f, 0.f};
          mfma_fence();
#pragma unroll
          for (int q = 0; q < 4; ++q) z1 = mfma4(lo[q], wlo[q], z1);
#pragma unroll
          for (int q = 0; q < 4; ++q) z1 = mfma4(hi[q], whi[q], z1);
          f4 acc = {b1v, b1v, b1v, b1v};
#pragma unroll
          for (int q = 0; q < KS; ++q) acc = mfma4(af[s][q], z1[q], acc);
          h2[s] = acc;
          mfma_fence();
        }
      }
      // D2 = dropout(H2) (one hash per element, both sides); zpre = D2·Wd + bd;
      // x = dropout(pad(relu(zpre))): row group g holds x_s[4r+g].  x > 0 exactly when
      // the node is present, zpre > 0 and the NTN-input element is kept: the backward
      // uses it as the whole mask of the Dense/Padding/dropout chain.
      float xo[2][RN], d2[2][3];
      uint32_t kb = 0u;   // layer-2 keep bits, bit 3s + r
      float hA[2] = {0.f, 0.f};                             // ATT: h_s[j]
      float att[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};  // ATT: att of node 4r + g
      if constexpr (ATT) {
        // Attention (layers.py:154-160): temp = mean of the node rows of H2, h = tanh(temp
        // Wa), att_n = sigmoid(H2[n] · h), e = Σ_n att_n H2[n]; x_s[j] = keep · e_j · ik4.
        // Lane (g, j) holds H2 rows 4r + g at feature j; absent rows (b1) are masked.
        float *sTmp = W + L::TMP;
        float part[2] = {0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int KS = s2 ? K1 : K0, Ns = s2 ? N1 : N0;
#pragma unroll
          for (int r = 0; r < KS; ++r) part[s2] += (4 * r + g < Ns) ? h2[s2][r] : 0.f;
        }
        xsum_pair(part[0], part[1]);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          if (g == 0) sTmp[16 * s2 + j] = part[s2] * (s2 ? invn1 : invn0);
        sg_wsync();
        float hp[2];   // row group g: the terms j' = 4g..4g+3 of (temp · Wa)[j]
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            a = fmaf(sTmp[16 * s2 + 4 * g + i], sWat[(4 * g + i) * WAS + j], a);
          hp[s2] = a;
        }
        xsum_pair(hp[0], hp[1]);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) hA[s2] = sg_tanh(hp[s2]);
        float dd[K0 + K1];   // H2[n] · h: the node rows' sums, both sides interleaved
#pragma unroll
        for (int r = 0; r < K0; ++r) dd[r] = h2[0][r] * hA[0];
#pragma unroll
        for (int r = 0; r < K1; ++r) dd[K0 + r] = h2[1][r] * hA[1];
        row_sum16_n(dd);
        float po[2] = {0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int KS = s2 ? K1 : K0, Ns = s2 ? N1 : N0;
#pragma unroll
          for (int r = 0; r < KS; ++r) {
            const float a = sg_sigmoid(dd[s2 * K0 + r]);
            att[s2][r] = a;
            po[s2] += (4 * r + g < Ns) ? a * h2[s2][r] : 0.f;
          }
        }
        xsum_pair(po[0], po[1]);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bool k4 = (m4 >> (16 * s2 + j)) & 1u;
          if (g == 0) sX[XO2 * s2 + j] = k4 ? po[s2] * A.ik4 : 0.f;
        }
        sg_wsync();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int r = 0; r < RN; ++r) xo[s2][r] = sX[XO2 * s2 + 4 * r + g];
#pragma unroll
        for (int r = 0; r < 3; ++r) d2[0][r] = d2[1][r] = 0.f;
      } else if constexpr (AVG) {
        // x_s[j] = keep · mean over the side's nodes of H2[·][j] · ik4 (layers.py:136-140,
        // 287-288): lane (g, j) holds the rows of nodes 4r + g; absent rows hold b1
        float part[2] = {0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int KS = s2 ? K1 : K0, Ns = s2 ? N1 : N0;
#pragma unroll
          for (int r = 0; r < KS; ++r) part[s2] += (4 * r + g < Ns) ? h2[s2][r] : 0.f;
        }
        xsum_pair(part[0], part[1]);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const float e = part[s2] * (s2 ? invn1 : invn0);
          const bool k4 = (m4 >> (16 * s2 + j)) & 1u;
          if (g == 0) sX[XO2 * s2 + j] = k4 ? e * A.ik4 : 0.f;
        }
        sg_wsync();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int r = 0; r < RN; ++r) xo[s2][r] = sX[XO2 * s2 + 4 * r + g];
#pragma unroll
        for (int r = 0; r < 3; ++r) d2[0][r] = d2[1][r] = 0.f;
      } else {
      // the K0 + K1 Dense row sums run step-interleaved (row_sum16_n): slot r of side 0,
      // K0 + r of side 1
      float zs[K0 + K1];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        if (r < K0 || r < K1) {
          const uint32_t h = sg_mix(pk2 ^ ((2u << 26) | (uint32_t)(64 * r)));
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            if (r < (s ? K1 : K0)) {
              const bool k2 = (s ? (h >> 16) : (h & 0xFFFFu)) < A.thr2;
              d2[s][r] = k2 ? h2[s][r] : 0.f;   // D2 / ik2
              kb |= (k2 ? 1u : 0u) << (3 * s + r);
              zs[s * K0 + r] = d2[s][r] * wdv;
            } else {
              d2[s][r] = 0.f;
            }
          }
        } else {
          d2[0][r] = d2[1][r] = 0.f;
        }
      }
      row_sum16_n(zs);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (r < (s ? K1 : K0)) {
            const float z = zs[s * K0 + r] + bd;
            const bool k4 = (km4 >> (16 * s + 4 * r)) & 1u;   // includes n < Ns
            xo[s][r] = ((z > 0.f) & k4) ? z * A.ik4 : 0.f;
          } else {
            xo[s][r] = 0.f;
          }
        }
      // publish x1 | x2 for the lanes that need every element
      if (j < 3) {
        const float v0 = j == 0 ? xo[0][0] : (j == 1 ? xo[0][1] : xo[0][2]);
        const float v1 = j == 0 ? xo[1][0] : (j == 1 ? xo[1][1] : xo[1][2]);
        const int n = 4 * j + g;
        if (n < D) {
          sX[n] = v0;
          sX[12 + n] = v1;
        }
      }
      sg_wsync();
      }   // !AVG

      // ================= NTN head (layers.py:282-310) =================
      // x_s is zero past 4 K_s elements: terms with a zero factor are dropped
      // (each is an exact fmaf(0, ·, acc) = acc)
      // (after Average every element can be nonzero: full width)
      constexpr int BL0 = AVG ? DN : (4 * K0 < D ? 4 * K0 : D);
      constexpr int BL1 = AVG ? DN : (4 * K1 < D ? 4 * K1 : D);
      constexpr int RA = AVG ? RN : K0, RB = AVG ? RN : K1;   // row groups holding x_s
      constexpr int BP0 = (BL0 + 1) / 2, BP1 = (BL1 + 1) / 2;   // element pairs
      f2 x2[(DN + 1) / 2];
#pragma unroll
      for (int b = 0; b < BP1; ++b) x2[b] = *(const f2 *)(sX + XO2 + 2 * b);
      float u[RN];
      float mpart = 0.f;
#pragma unroll
      for (int r = 0; r < RN; ++r) {
        const int a = 4 * r + g;
        const int ac = a < DN ? a : 0;
        if (r < RA) {
          const float *wa = sWa + (ac * FK + kc) * WR;
          f2 acc2 = {0.f, 0.f};
#pragma unroll
          for (int b = 0; b < BP1; ++b)
            acc2 = pfma(*(const f2 *)(wa + 2 * b), x2[b], acc2);
          const float acc = acc2.x + acc2.y;
          u[r] = acc;
          // x1[a] u[a][k] + V[k][a] x1[a] + V[k][D+a] x2[a]   (x of invalid a is 0)
          mpart = fmaf(xo[0][r], acc + sV[kc * VS + ac], mpart);
        }
        if (r < RB) mpart = fmaf(xo[1][r], sV[kc * VS + DN + ac], mpart);
      }
      const float m = xsum32(xsum16(mpart)) + bnk;
      const float rk = (kv & (m > 0.f)) ? m : 0.f;
      const float rsum = row_sum16(rk);
      const float sv = INTENDED ? row_sum16(Uk * rk) : usum * rsum;
      if (!BWD) {
        // every lane stores the (wave-uniform) score: a store behind a lane test is not
        // counted on every path, and the loop's wait for the next record would become a
        // vmcnt(0) that also waits for this store
        A.s_out[pcur] = sv;
        return;
      }
      if (A.s_out && l == 0) A.s_out[pcur] = sv;
      const float yhat = __expf(-A.yeta * sv * sv);   // v_exp_f32: ~1e-7 relative
      float gy;
      if (!ALIGNED) {
        gy = yhat - ybar;
        lossa += 0.5f * gy * gy;
      } else {
        const float dl = yhat - sRec[2 * D * D + 2 * D + 2];
        gy = dl * A.inv_batch;
        lossa += 0.5f * dl * dl * A.inv_batch;
      }
      const float gs = gy * (-2.f * A.yeta * sv * yhat);

      // ================= NTN backward =================
      const float gmk = (kv & (m > 0.f)) ? (INTENDED ? gs * Uk : gs * usum) : 0.f;
      if (g == 0) {
        if (!AVG) gbn += gmk;
        gUa += INTENDED ? gs * rk : gs * rsum;
      }
      if constexpr (AVG) {
        // this pair's row of the NTN-gradient buffer, sg_ntn_wgrad's compact D = 16 layout
        // (NBUF16, 48 floats): x1 | x2 | gm, zeros, the constant 1 in slot 47.  One store by
        // every lane, no branch: lanes 0-31 write x1 | x2 (sX[0..31]), lanes 32-47 gm_k or
        // the pad, and lanes 48-63 repeat lanes 32-47's stores (the four row groups hold the
        // same gm_k).  A store behind a branch made the loop's wait for the next record's
        // prefetch a vmcnt(0), which also waited for this pair's stores (their HBM latency,
        // every pair).
        static_assert(DN == 16 && XO2 == 16, "the compact row holds 16-element x1 and x2");
        float *nb_ = A.ntn + (size_t)(uint32_t)pcur * 48u;
        {
          const float xv = sX[l & 31];
          const float gv = j < FK ? gmk : (j == 15 ? 1.f : 0.f);
          nb_[l < 48 ? l : l - 16] = l < 32 ? xv : gv;
        }
      }
      const float gmk4 = gmk * A.ik4;
      float ge[2][RN];   // dL/dx · ik4 (before the x > 0 mask)
      {
        f2 x1[(DN + 1) / 2];
#pragma unroll
        for (int a = 0; a < BP0; ++a) x1[a] = *(const f2 *)(sX + 2 * a);
        // the RA + RB row sums run step-interleaved: slot r of side 0, RA + r of side 1
        float tt[RA + RB];
#pragma unroll
        for (int r = 0; r < RN; ++r) {
          const int a = 4 * r + g;
          const int ac = a < DN ? a : 0;
          if (r < RA) {
            if constexpr (!AVG) {
              const float c = gmk * xo[0][r];
              const f2 c2 = {c, c};
#pragma unroll
              for (int b = 0; b < BP1; ++b) gWn[r][b] = pfma(c2, x2[b], gWn[r][b]);
              gVa[r] = fmaf(gmk, xo[0][r], gVa[r]);
            }
            tt[r] = gmk4 * (sV[kc * VS + ac] + u[r]);
          }
          if (r < RB) {
            if constexpr (!AVG) gVb[r] = fmaf(gmk, xo[1][r], gVb[r]);
            const float *wb = sWb + (ac * FK + kc) * WR;
            f2 w2 = {0.f, 0.f};
#pragma unroll
            for (int aa = 0; aa < BP0; ++aa)
              w2 = pfma(x1[aa], *(const f2 *)(wb + 2 * aa), w2);
            const float w = w2.x + w2.y;
            tt[RA + r] = gmk4 * (sV[kc * VS + DN + ac] + w);
          }
        }
        row_sum16_n(tt);
#pragma unroll
        for (int r = 0; r < RN; ++r) {
          ge[0][r] = r < RA ? tt[r] : 0.f;
          ge[1][r] = r < RB ? tt[RA + r] : 0.f;
        }
      }

      // ================= GCN backward =================
      f4 gh2[2], gz1t[2];
      float dq[2][2][3];   // [side][t][q]: this lane's D1 entries
      float gej[2] = {0.f, 0.f};   // AVG: ∂L/∂e_s[j] / N_s;  ATT: ∂L/∂e_s[j]
      float gxa[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};   // ATT: ∂L/∂H2 of node 4r + g
      if constexpr (AVG) {
        // ∂L/∂x of element a = 4r + g (equal on a row's 16 lanes) → by feature j
        float *sGE = W + L::GE;
        if (j == 0) {
#pragma unroll
          for (int r = 0; r < RN; ++r) {
            sGE[4 * r + g] = ge[0][r];
            sGE[16 + 4 * r + g] = ge[1][r];
          }
        }
        sg_wsync();
        gej[0] = ((m4 >> j) & 1u) ? sGE[j] * (ATT ? 1.f : invn0) : 0.f;
        gej[1] = ((m4 >> (16 + j)) & 1u) ? sGE[16 + j] * (ATT ? 1.f : invn1) : 0.f;
      }
      if constexpr (ATT) {
        // Attention backward (adjoint of layers.py:154-160, oracle _node_backward):
        //   gatt_n = gout · H2[n],  gz_n = gatt_n att_n (1 - att_n),  gh = Σ_n gz_n H2[n],
        //   gu = gh (1 - h²),  gWa += temp ⊗ gu,  gtemp = Wa gu,
        //   ∂L/∂H2[n] = att_n gout + gz_n h + gtemp / N
        float *sTmp = W + L::TMP, *sGU = W + L::GU;
        float ga[K0 + K1];
#pragma unroll
        for (int r = 0; r < K0; ++r) ga[r] = gej[0] * h2[0][r];
#pragma unroll
        for (int r = 0; r < K1; ++r) ga[K0 + r] = gej[1] * h2[1][r];
        row_sum16_n(ga);
        float ghp[2] = {0.f, 0.f}, gz[2][3];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int KS = s2 ? K1 : K0, Ns = s2 ? N1 : N0;
#pragma unroll
          for (int r = 0; r < KS; ++r) {
            const float a = att[s2][r];
            const float z = (4 * r + g < Ns) ? ga[s2 * K0 + r] * (a * (1.f - a)) : 0.f;
            gz[s2][r] = z;
            ghp[s2] = fmaf(z, h2[s2][r], ghp[s2]);
          }
        }
        float gu[2];
        xsum_pair(ghp[0], ghp[1]);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const float gh = ghp[s2];
          gu[s2] = gh * (1.f - hA[s2] * hA[s2]);
          if (g == 0) sGU[16 * s2 + j] = gu[s2];
        }
        sg_wsync();
        float gtp[2];   // row group g: the terms k = 4g..4g+3 of (Wa gu)[j]
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
          for (int i = 0; i < 4; ++i) gwa[i] = fmaf(sTmp[16 * s2 + 4 * i + g], gu[s2], gwa[i]);
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) a = fmaf(sGU[16 * s2 + 4 * g + i], sWat[j * WAS + 4 * g + i], a);
          gtp[s2] = a;
        }
        xsum_pair(gtp[0], gtp[1]);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int KS = s2 ? K1 : K0;
          const float gt = gtp[s2] * (s2 ? invn1 : invn0);
#pragma unroll
          for (int r = 0; r < KS; ++r)
            gxa[s2][r] = fmaf(att[s2][r], gej[s2], fmaf(gz[s2][r], hA[s2], gt));
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int KS = s ? K1 : K0;
        gh2[s] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          if constexpr (AVG) {   // mean: every present node gets ∂L/∂e / N (ATT: gxa)
            const float v = (4 * r + g < (s ? N1 : N0)) ? (ATT ? gxa[s][r] : gej[s]) : 0.f;
            gb1a += v;
            gh2[s][r] = v;
          } else {
            const float gp = xo[s][r] > 0.f ? ge[s][r] : 0.f;   // dropout4 · relu' · present
            gwda = fmaf(d2[s][r], gp, gwda);
            gbda += gp;   // equal on the 16 lanes of a row: lane j == 0 is flushed
            const float v = ((kb >> (3 * s + r)) & 1u) ? gp * wdv : 0.f;
            gb1a += v;
            gh2[s][r] = v;
          }
        }
        // gZ1 = Âᵀ gH2 in both orientations (Â symmetric, checked at pack time):
        //   gz1  rows = nodes (B of gW1 = D1ᵀ gZ1),  gz1t rows = j (A of gD1 = gZ1 W1ᵀ)
        f4 gz1 = {0.f, 0.f, 0.f, 0.f};
        gz1t[s] = f4{0.f, 0.f, 0.f, 0.f};
        // this lane's D1 entries: A operand of gW1 += D1ᵀ gZ1 and, as D1 > 0, the
        // keep·relu' mask of gP1
        const float *T1 = sT + s * 16 * TS1 + 4 * g * TS1 + j;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int q = 0; q < KS; ++q) dq[s][t][q] = T1[q * TS1 + 16 * t];
        mfma_fence();
#pragma unroll
        for (int q = 0; q < KS; ++q) {
          gz1 = mfma4(af[s][q], gh2[s][q], gz1);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int q = 0; q < KS; ++q) gw1[t] = mfma4(dq[s][t][q], gz1[q], gw1[t]);
        mfma_fence();
        {   // gZ1 rows 4g + r, feature j (a shared tile: side 1's rows 2 below side 0's)
          float *gt = W + L::GT + (PACK ? 0 : s * 16 * TS2) + j;
#pragma unroll
          for (int r = 0; r < KS; ++r) gt[(4 * g + r + ((PACK && s) ? 2 : 0)) * TS2] = gz1[r];
        }
      }
      sg_wsync();
#pragma unroll
      for (int s = 0; s < (PACK ? 1 : 2); ++s)
        gz1t[s] = *(const f4 *)(W + L::GT + s * 16 * TS2 + j * TS2 + 4 * g);
      // gD1 · ik1 = gZ1 (W1 ik1)ᵀ per feature tile t (one chain per tile when packed)
      f4 gd[2][2];   // [side, or 0 = shared][t]
      // A k-slots 8g..8g+7 = (h | m) or (h | l) of gZ1[i][4g..4g+3]; with the B parts
      // (Wh | Wh), (Wm | Wh), (Wl | Wm): hh + mh + hm + lh + hl + mm in three MFMAs
      uint4 ahm[2], ahl[2];
#pragma unroll
      for (int s = 0; s < (PACK ? 1 : 2); ++s) {
        uint32_t h01, m01, l01, h23, m23, l23;
        split3(gz1t[s][0], gz1t[s][1], h01, m01, l01);
        split3(gz1t[s][2], gz1t[s][3], h23, m23, l23);
        ahm[s] = uint4{h01, h23, m01, m23};
        ahl[s] = uint4{h01, h23, l01, l23};
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint4 *wb = sW1B + t * 192 + l;
        const uint4 b1 = wb[0], b2 = wb[64], b3 = wb[128];
#pragma unroll
        for (int s = 0; s < (PACK ? 1 : 2); ++s) {
          f4 acc = {0.f, 0.f, 0.f, 0.f};
          acc = mfbf(ahm[s], b1, acc);
          acc = mfbf(ahl[s], b2, acc);
          acc = mfbf(ahm[s], b3, acc);
          gd[s][t] = acc;
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int KS = s ? K1 : K0;
        // one-hot Xᵀ for gW0 as a bf16 A operand: row i = j ↔ type 16τ + j.
        // Three node rows per group (4g + q): three 16x16x16 MFMAs, k-slot 4g + e ↔ node
        // row 4g + e, A = (o01 | o23) against the h, m and l parts of gZ0 in turn.
        // A side of at most 8 nodes has only rows 4g, 4g+1: the h, l and m parts of both
        // fit one 16x16x32 MFMA's 8 k-slots (A = (o | o | o | 0), B = (h | l | m | h)).
        uint4 ohA[2];
        uint2 oh2[2];
#pragma unroll
        for (int tau = 0; tau < 2; ++tau) {
          uint32_t o[3];
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const uint32_t tq = (tys[s] >> (6 * q)) & 63u;
            o[q] = (q < KS && tq == (uint32_t)(16 * tau + j)) ? 0x3F80u : 0u;   // bf16 1.0
          }
          const uint32_t o01 = o[0] | (o[1] << 16), o23 = o[2];
          if (KS > 2) {
            oh2[tau] = uint2{o01, o23};
          } else {
            ohA[tau] = uint4{o01, o01, o01, 0u};
          }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          f4 gp1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int r = 0; r < KS; ++r) {
            const float gdv = PACK ? gd[0][t][2 * s + r] : gd[s][t][r];
            gp1[r] = dq[s][t][r] > 0.f ? gdv : 0.f;
          }
          if (t) gb0a1 += (gp1[0] + gp1[1]) + gp1[2];
          else gb0a0 += (gp1[0] + gp1[1]) + gp1[2];
          f4 gz0 = {0.f, 0.f, 0.f, 0.f};  // gZ0 = Âᵀ gP1
          mfma_fence();
#pragma unroll
          for (int q = 0; q < KS; ++q) gz0 = mfma4(af[s][q], gp1[q], gz0);
          mfma_fence();
          // gW0 / ik0 += Xᵀ gZ0 (rows 4g+3 of gZ0 are always zero)
          uint32_t h01, m01, l01, h23 = 0u, m23 = 0u, l23 = 0u;
          split3(gz0[0], gz0[1], h01, m01, l01);
          if (KS > 2) {
            split3(gz0[2], 0.f, h23, m23, l23);
            const uint2 bh = {h01, h23}, bm = {m01, m23}, bl = {l01, l23};
#pragma unroll
            for (int tau = 0; tau < 2; ++tau) {
              gw0[tau][t] = mfbf16(oh2[tau], bl, gw0[tau][t]);
              gw0[tau][t] = mfbf16(oh2[tau], bm, gw0[tau][t]);
              gw0[tau][t] = mfbf16(oh2[tau], bh, gw0[tau][t]);
            }
          } else {   // the fourth B dword meets a zero A dword: any finite value
            const uint4 b = {h01, l01, m01, h01};
#pragma unroll
            for (int tau = 0; tau < 2; ++tau) gw0[tau][t] = mfbf(ohA[tau], b, gw0[tau][t]);
          }
        }
      }
    };
    if constexpr (CLS < 0) {
      const bool big0 = N0 > 8, big1 = N1 > 8;
      if (big0) {
        if (big1) body(std::integral_constant<int, 3>{}, std::integral_constant<int, 3>{});
        else body(std::integral_constant<int, 3>{}, std::integral_constant<int, 2>{});
      } else {
        if (big1) body(std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{});
        else body(std::integral_constant<int, 2>{}, std::integral_constant<int, 2>{});
      }
    } else {   // the class table guarantees (N0 > 8, N1 > 8) == (CLS & 1, CLS & 2)
      body(std::integral_constant<int, (CLS & 1) ? 3 : 2>{},
           std::integral_constant<int, (CLS & 2) ? 3 : 2>{});
    }
  }
  };
  if (cls_mode) {
    if (cwave == 0) pair_loop(std::integral_constant<int, 0>{});
    else if (cwave == 1) pair_loop(std::integral_constant<int, 1>{});
    else if (cwave == 2) pair_loop(std::integral_constant<int, 2>{});
    else pair_loop(std::integral_constant<int, 3>{});
  } else {
    pair_loop(std::integral_constant<int, -1>{});
  }

  SG_STAMP(2, __builtin_amdgcn_s_memrealtime());
  SG_STAMP(4, (unsigned long long)it | ((unsigned long long)(cwave + 1) << 32));
  if (!BWD) return;
  // ---- flush: every wave dumps its accumulator slots to LDS, all threads sum ----
  // Slot s of lane (g, j) maps to at most one parameter (fast_param below) and
  // every parameter is hit exactly once, so the slab row is written directly.
  // Waves are summed in fixed order (deterministic).  The block owns the CU's
  // LDS (one block per CU), so all its waves' slots fit (fast_cfg).
  constexpr int NS = FlushSlots<D, AVG, ATT>::NS;
  {
    // per-feature bias / Dense gradients: sum the four row groups in registers
    gb0a0 = xsum32(xsum16(gb0a0));
    gb0a1 = xsum32(xsum16(gb0a1));
    gb1a = xsum32(xsum16(gb1a));
    gwda = xsum32(xsum16(gwda)) * A.ik2;
    gbda = xsum32(xsum16(gbda));
  }
  float *F = smem;
  __syncthreads();   // every wave has left the pair loop: the tables are dead
  {
    float *Fw = F + (size_t)wv * NS * 64 + l;
    int s = 0;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) Fw[64 * s++] = gw1[t][r];
#pragma unroll
    for (int tau = 0; tau < 2; ++tau)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) Fw[64 * s++] = gw0[tau][t][r] * A.ik0;
    if constexpr (!AVG) {
#pragma unroll
      for (int r = 0; r < RN; ++r)
#pragma unroll
        for (int b = 0; b < DN; ++b) Fw[64 * s++] = gWn[r][b >> 1][b & 1];
#pragma unroll
      for (int r = 0; r < RN; ++r) Fw[64 * s++] = gVa[r];
#pragma unroll
      for (int r = 0; r < RN; ++r) Fw[64 * s++] = gVb[r];
    }
    Fw[64 * s++] = gbn;
    Fw[64 * s++] = gUa;
    Fw[64 * s++] = lossa;
    Fw[64 * s++] = gb0a0;
    Fw[64 * s++] = gb0a1;
    Fw[64 * s++] = gb1a;
    Fw[64 * s++] = gwda;
    Fw[64 * s++] = gbda;
    if constexpr (ATT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) Fw[64 * s++] = gwa[i];
    }
  }
  __syncthreads();
  float *dst = A.slab + (size_t)blockIdx.x * (size_t)(A.n_params + 1);
  // wave wv sums slots wv, wv + nw, ...: the slot index is wave-uniform, so fast_param's
  // region decode runs on scalar registers and only its lane part on VALU (the waves are
  // summed in the same order as before: bitwise the same row)
  for (int s = wv; s < NS; s += nw) {
    const int prm_i = fast_param<D, AVG, ATT>(A, s, l);
    float acc = 0.f;
    for (int w = 0; w < nw; ++w) acc += F[((size_t)w * NS + s) * 64 + l];
    if (prm_i >= 0) dst[prm_i] = acc;
  }
  SG_STAMP(3, __builtin_amdgcn_s_memrealtime());
}

struct FastCfg {
  int D;
  int waves;
  int blocks;
  size_t lds;
  int shared_floats, wave_floats;
};

template <int D, bool AVG, bool ATT>
FastCfg fast_cfg_t(int d_in, int n_params, int64_t n_pairs, bool bwd) {
  FastCfg c;
  c.D = D;
  using LL = FastLds<D, AVG, ATT>;
  using FS = FlushSlots<D, AVG, ATT>;
  c.shared_floats = LL::shared_floats(d_in);
  c.wave_floats = LL::wave_floats(d_in, bwd);
  // resident waves per CU allowed by registers: the backward kernel uses up to
  // 256 VGPRs (2 waves / SIMD), the forward-only one ~120 (4 waves / SIMD)
  const int wcap = bwd ? MAXW : 2 * MAXW;
  // pick waves/block maximising resident waves per CU under 160 KiB of LDS
  int best = 1, best_res = 0;
  const char *ev = getenv("SG_FAST_WAVES");
  const int force = ev ? atoi(ev) : 0;
  for (int nw = 1; nw <= MAXW; ++nw) {
    if (force > 0 && nw != force) continue;
    const size_t lds = (size_t)(c.shared_floats + nw * c.wave_floats) * 4u;
    if (lds > 163840u) break;
    if (bwd && (size_t)nw * FS::NS * 256u > 163840u) break;   // flush slots fit
    int per_cu = (int)(163840u / lds);
    int res = per_cu * nw;
    if (res > wcap) res = wcap;  // register-limited occupancy
    if (res > best_res || (res == best_res && nw > best)) {
      best = nw;
      best_res = res;
    }
  }
  c.waves = best;
  c.lds = (size_t)(c.shared_floats + best * c.wave_floats) * 4u;
  // resident blocks per CU: LDS- and register-limited (MAXW waves per CU); a
  // grid of exactly that many blocks per CU pays the prologue/flush once per block
  int per_cu = (int)(163840u / c.lds);
  if (per_cu > wcap / best) per_cu = wcap / best;
  if (per_cu < 1) per_cu = 1;
  // the flush dumps every wave's accumulator slots into the block's LDS
  const size_t fl = bwd ? (size_t)best * FS::NS * 64u * 4u : 0u;
  // the prologue stages the parameter vector behind the shared tables
  const size_t stage = (size_t)(c.shared_floats + n_params) * 4u;
  const size_t need = fl > stage ? fl : stage;
  if (need > c.lds) {
    c.lds = need;
    per_cu = (int)(163840u / c.lds);
  }
  const int64_t want = (n_pairs + best - 1) / best;
  const int64_t cap = (int64_t)sg_num_cus() * per_cu;
  c.blocks = (int)(want < cap ? (want > 0 ? want : 1) : cap);
  return c;
}

template <int D, bool BWD, bool ALIGNED, bool INTENDED, bool AVG, bool SRC, bool ATT>
void launch_one(const FastCfg &c, const FastArgs &A, hipStream_t st) {
  const void *fn = (const void *)sg_fast_kernel<D, BWD, ALIGNED, INTENDED, AVG, SRC, ATT>;
  if (c.lds > 65536u)
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds);
  hipLaunchKernelGGL((sg_fast_kernel<D, BWD, ALIGNED, INTENDED, AVG, SRC, ATT>), dim3(c.blocks),
                     dim3(64 * c.waves), c.lds, st, A);
}

template <int D, bool AVG, bool SRC, bool ATT>
void launch_fast_src(const FastCfg &c, bool bwd, bool aligned, bool intended,
                     const FastArgs &A, hipStream_t st) {
  if (!bwd) {
    if (intended) launch_one<D, false, false, true, AVG, SRC, ATT>(c, A, st);
    else launch_one<D, false, false, false, AVG, SRC, ATT>(c, A, st);
  } else if (aligned) {
    if (intended) launch_one<D, true, true, true, AVG, SRC, ATT>(c, A, st);
    else launch_one<D, true, true, false, AVG, SRC, ATT>(c, A, st);
  } else {
    if (intended) launch_one<D, true, false, true, AVG, SRC, ATT>(c, A, st);
    else launch_one<D, true, false, false, AVG, SRC, ATT>(c, A, st);
  }
}

// SRC: store-sourced pairs (a separate instantiation: the gather's registers would
// otherwise cost the record path spills)
template <int D, bool AVG, bool ATT = false>
void launch_fast(const FastCfg &c, bool bwd, bool aligned, bool intended,
                 const FastArgs &A, hipStream_t st) {
  if (A.src_store) launch_fast_src<D, AVG, true, ATT>(c, bwd, aligned, intended, A, st);
  else launch_fast_src<D, AVG, false, ATT>(c, bwd, aligned, intended, A, st);
}

}  // namespace

// --------------------------------------------------------------------------
// Pooled-head stacks (tuning.py:66-93): GCN(d_in→32, relu) → GCN(32→16) → Average or
// Attention(16) (layers.py:121-160) → NTN(16, K=10)
static bool fast_pool_shape(const sg_model_t *m, const SgGenPlan &P) {
  if (m->num_layers != 4) return false;
  const sg_layer_t *Ly = m->layers;
  if (Ly[0].kind != SG_GCN || !Ly[0].sparse_inputs || Ly[0].output_dim != FH1 ||
      Ly[0].act != SG_ACT_RELU || !Ly[0].bias)
    return false;
  if (Ly[1].kind != SG_GCN || Ly[1].input_dim != FH1 || Ly[1].output_dim != FH2 ||
      Ly[1].act != SG_ACT_IDENTITY || !Ly[1].bias)
    return false;
  if (Ly[2].kind != SG_AVERAGE && !(Ly[2].kind == SG_ATTENTION && Ly[2].input_dim == FH2))
    return false;
  if (Ly[3].kind != SG_NTN || Ly[3].input_dim != FH2 || Ly[3].output_dim != FK ||
      Ly[3].act != SG_ACT_RELU || !Ly[3].bias)
    return false;
  if (m->n_max != 10 && m->n_max != 12) return false;
  if (m->final_act != SG_FINAL_GAUSSIAN) return false;
  if (m->d_in > 32) return false;
  return P.n_params > 0;
}

static bool fast_shape(const sg_model_t *m, const SgGenPlan &P) {
  if (fast_pool_shape(m, P)) return true;
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
  if (m->n_max != D || (D != 10 && D != 12)) return false;
  if (m->final_act != SG_FINAL_GAUSSIAN) return false;
  if (m->d_in > 32) return false;   // two 16-row type tiles for the one-hot gW0 MFMA
  return P.n_params > 0;
}

// the pooled 16-feature head (Average or Attention: no Dense / Padding, NTN at layer 3)
static bool plan_avg(const SgGenPlan &P) {
  return P.nl == 3 && (P.L[2].kind == SG_AVERAGE || P.L[2].kind == SG_ATTENTION);
}
static bool plan_att(const SgGenPlan &P) { return P.nl == 3 && P.L[2].kind == SG_ATTENTION; }

static FastCfg fast_cfg(const SgGenPlan &P, int64_t n_pairs, bool bwd) {
  if (plan_att(P))
    return P.n_max == 12 ? fast_cfg_t<12, true, true>(P.d_in, P.n_params, n_pairs, bwd)
                         : fast_cfg_t<10, true, true>(P.d_in, P.n_params, n_pairs, bwd);
  if (plan_avg(P))
    return P.n_max == 12 ? fast_cfg_t<12, true, false>(P.d_in, P.n_params, n_pairs, bwd)
                         : fast_cfg_t<10, true, false>(P.d_in, P.n_params, n_pairs, bwd);
  return P.n_max == 12 ? fast_cfg_t<12, false, false>(P.d_in, P.n_params, n_pairs, bwd)
                       : fast_cfg_t<10, false, false>(P.d_in, P.n_params, n_pairs, bwd);
}

struct ClassWeights {
  float w[4];
  bool set;   // SG_CLS_W given: it applies to every stack
};

static ClassWeights class_weights_from_env() {
  ClassWeights c = {{1.f, 1.f, 1.f, 1.f}, false};
  if (const char *ev = getenv("SG_CLS_W")) {
    float w[4];
    if (sscanf(ev, "%f,%f,%f,%f", &w[0], &w[1], &w[2], &w[3]) == 4) {
      for (int k = 0; k < 4; ++k) c.w[k] = w[k] > 0.f ? w[k] : 1.f;
      c.set = true;
    }
  }
  return c;
}

// Relative cost of a pair of class (N0 > 8) + 2 (N1 > 8) per stack: the median per-class
// µs/pair of the per-wave timing build (scripts/fast_timing.py), N = 1 (W = 8 within 0.5%).
// Round 6 (profiles/r06_p … r06_u): the default stack on f32 records 1 : 1.355 : 1.351 :
// 1.546 (its pair body changed since round 4's 1 : 1.315 : 1.316 : 1.493, which left the
// (2, 2) class's waves ending 23 µs early; C2 +0.7%, an emulated W = 8 rank −1.5%); on
// bf16 records (C3) 1 : 1.307 : 1.316 : 1.497, where round 4's weights stay (larger or
// smaller weights measured slower); Average 1 : 1.212 : 1.211 : 1.330 (+5.2%); Attention
// (its kernel is in another translation unit, which the timing build does not read back) by
// an A/B sweep, 1 : 1.18 : 1.18 : 1.28 (+6.6%).  The default stack's forward-only launches
// (eval) by sweep, 1 : 1.28 : 1.28 : 1.44 (profiles/r06_cc, r06_dd).
static void class_weights_for(bool avg, bool att, bool bf16, bool bwd, float *w) {
  static const float kDefault[4] = {1.f, 1.355f, 1.351f, 1.546f};
  static const float kDefaultFwd[4] = {1.f, 1.28f, 1.28f, 1.44f};
  static const float kBf16[4] = {1.f, 1.315f, 1.316f, 1.493f};
  static const float kAverage[4] = {1.f, 1.212f, 1.211f, 1.330f};
  static const float kAttention[4] = {1.f, 1.18f, 1.18f, 1.28f};
  static const ClassWeights env = class_weights_from_env();   // parsed once per process
  const float *src =
      env.set ? env.w
              : (att ? kAttention
                     : (avg ? kAverage : (bf16 ? kBf16 : (bwd ? kDefault : kDefaultFwd))));
  for (int k = 0; k < 4; ++k) w[k] = src[k];
}

// Relative pair-loop speed of XCD x (block b on XCD b % 8), ×10^4.  The default is equal
// weights (the even split).  Measured and not adopted (profiles/r05_g): weights from the
// median pair-loop end per XCD on four boxes (XCD 0 .991, 1 1.005, 2 1.000, 3 1.013,
// 4 .986, 5 .999, 6 .998, 7 1.009 of the mean time) ran 546.4 / 546.9 against 546.0 / 548.5
// M pairs/s: on a fifth box only XCD 3 (slow) and 4 (fast) kept their place, and XCD 0,
// given more pairs, ended last.  SG_XCD_W="w0,...,w7" sets them.
struct XcdWeights {
  int w[8];
};

static XcdWeights xcd_weights_from_env() {
  XcdWeights x = {{10000, 10000, 10000, 10000, 10000, 10000, 10000, 10000}};
  if (const char *ev = getenv("SG_XCD_W")) {
    int w[8];
    if (sscanf(ev, "%d,%d,%d,%d,%d,%d,%d,%d", &w[0], &w[1], &w[2], &w[3], &w[4], &w[5], &w[6],
               &w[7]) == 8)
      for (int k = 0; k < 8; ++k) x.w[k] = w[k] > 0 ? w[k] : 10000;
  }
  return x;
}

int sg_ntn_wgrad_run(const float *ntn, int64_t n_pairs, int D, int oW, int oV, int obn, int C,
                     float *slab, int blocks, hipStream_t st, bool compact);

// The host side of sg_fast_run.  The translation unit sg_fast_att.hip compiles this file
// again with SG_FAST_ATT_TU defined and instantiates only the Attention kernels (the
// default TU instantiates the rest): the two compile in parallel.
static int fast_run_impl(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                         const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                         int64_t batch_total, const float *params, uint64_t seed,
                         const float *y_stats, float *s_out, float *slab, float *ntn,
                         int *blocks_out, hipStream_t stream, const uint64_t *seed_dev,
                         const sg_pair_source_t *src, const int32_t *class_start,
                         const SgAdamPre *adam_pre) {
  const int D = P.n_max;
  FastCfg c = fast_cfg(P, n_pairs, bwd);
  // the kernel indexes pairs in 32 bits (2^31 records would be ≥ 1 TB)
  if (n_pairs > 0x7FFFFFFF - (int64_t)c.blocks * c.waves * 2) return SG_ERR_ARG;
  FastArgs A;
  A.recs = (const uint8_t *)recs;
  A.src_store = src ? 1 : 0;
  A.G = src ? src->n_graphs : 0;
  A.sadj = src ? src->adj : nullptr;
  A.stypes = src ? src->types : nullptr;
  A.sn = src ? src->n : nullptr;
  A.spairs = src ? src->pair_idx : nullptr;
  A.grid_base = src ? src->grid_base : 0;
  A.slabels = src ? src->labels : nullptr;
  A.status = src ? src->status : nullptr;
  if (src && (P.adj_dtype != SG_DTYPE_F32 || src->n_max != D || src->n_graphs <= 0))
    return SG_ERR_ARG;
  A.order = order;
  A.cls = order ? class_start : nullptr;
  // the class-exclusive schedule gives each class waves in proportion to count x cost
  // (class_weights_for; SG_CLS_W="w0,w1,w2,w3" to tune); the environment is parsed once
  // per process, and only for class-scheduled launches
  if (A.cls) {
    class_weights_for(plan_avg(P), plan_att(P), P.adj_dtype == SG_DTYPE_BF16, bwd, A.cw);
    static const XcdWeights xwt = xcd_weights_from_env();
    for (int k = 0; k < 8; ++k) A.xw[k] = xwt.w[k];
  } else {
    for (int k = 0; k < 4; ++k) A.cw[k] = 1.f;
    for (int k = 0; k < 8; ++k) A.xw[k] = 10000;
  }
  A.xw_even = 1;
  for (int k = 1; k < 8; ++k) A.xw_even &= A.xw[k] == A.xw[0] ? 1 : 0;
  A.n_pairs = n_pairs;
  A.rw4h = P.hbm_words / 4;
  A.rec_bf16 = P.adj_dtype == SG_DTYPE_BF16 ? 1 : 0;
  A.pair_offset = pair_offset;
  A.params = params;
  A.y_stats = y_stats;
  A.s_out = s_out;
  A.slab = slab;
  A.ntn = ntn;
  A.key = sg_seed_key(seed);
  A.seed_dev = seed_dev;
  A.ad_bp = nullptr;
  A.ad_out = nullptr;
  A.ad_lr = A.ad_b1 = A.ad_b2 = A.ad_wd = 0.f;
  if (bwd && adam_pre != nullptr) {
    A.ad_bp = adam_pre->bp;
    A.ad_out = adam_pre->out;
    A.ad_lr = adam_pre->lr;
    A.ad_b1 = adam_pre->b1;
    A.ad_b2 = adam_pre->b2;
    A.ad_wd = adam_pre->wd;
  }
  const float keep = m->keep_prob;
  const bool avg = plan_avg(P);   // NTN is layer 3 after Average / Attention
  const bool att = plan_att(P);
  const float k0 = m->layers[0].dropout ? keep : 1.f, k1 = m->layers[1].dropout ? keep : 1.f;
  const float k2 = (!avg && m->layers[2].dropout) ? keep : 1.f;
  const float k4 = m->layers[avg ? 3 : 4].dropout ? keep : 1.f;
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
  A.d_in = P.d_in;
  A.n_params = P.n_params;
  A.shared_floats = c.shared_floats;
  A.wave_floats = c.wave_floats;
  A.oW0 = P.L[0].offW;
  A.ob0 = P.L[0].offB;
  A.oW1 = P.L[1].offW;
  A.ob1 = P.L[1].offB;
  A.oWd = avg ? -1 : P.L[2].offW;
  A.obd = avg ? -1 : P.L[2].offB;
  A.oWa = att ? P.L[2].offW : -1;
  A.oW = P.offW;
  A.oV = P.offV;
  A.oU = P.offU;
  A.obn = P.offB;
  const bool aligned = m->loss_mode == SG_LOSS_ALIGNED;
  const bool intended = m->ntn_mode == SG_NTN_INTENDED;
  if (avg && bwd && !ntn) return SG_ERR_ARG;
#ifdef SG_FAST_ATT_TU
  if (!att) return SG_ERR_UNSUPPORTED;
  if (D == 12) launch_fast<12, true, true>(c, bwd, aligned, intended, A, stream);
  else launch_fast<10, true, true>(c, bwd, aligned, intended, A, stream);
#else
  if (att) return SG_ERR_UNSUPPORTED;   // sg_fast_att.hip
  if (avg) {
    if (D == 12) launch_fast<12, true>(c, bwd, aligned, intended, A, stream);
    else launch_fast<10, true>(c, bwd, aligned, intended, A, stream);
  } else {
    if (D == 12) launch_fast<12, false>(c, bwd, aligned, intended, A, stream);
    else launch_fast<10, false>(c, bwd, aligned, intended, A, stream);
  }
#endif
  if (avg && bwd) {   // the NTN W / V / bias gradients from the per-pair buffer
    const int rc = sg_ntn_wgrad_run(ntn, n_pairs, FH2, P.offW, P.offV, P.offB, P.n_params + 1,
                                    slab, c.blocks, stream, true);   // compact rows
    if (rc != SG_OK) return rc;
  }
  if (blocks_out) *blocks_out = c.blocks;
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

#ifdef SG_FAST_ATT_TU
int sg_fast_att_run(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                    const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                    int64_t batch_total, const float *params, uint64_t seed,
                    const float *y_stats, float *s_out, float *slab, float *ntn, int *blocks_out,
                    hipStream_t stream, const uint64_t *seed_dev, const sg_pair_source_t *src,
                    const int32_t *class_start, const SgAdamPre *adam_pre) {
  return fast_run_impl(m, P, bwd, recs, order, n_pairs, pair_offset, batch_total, params, seed,
                       y_stats, s_out, slab, ntn, blocks_out, stream, seed_dev, src, class_start,
                       adam_pre);
}
#else
int sg_fast_att_run(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                    const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                    int64_t batch_total, const float *params, uint64_t seed,
                    const float *y_stats, float *s_out, float *slab, float *ntn, int *blocks_out,
                    hipStream_t stream, const uint64_t *seed_dev, const sg_pair_source_t *src,
                    const int32_t *class_start, const SgAdamPre *adam_pre);

int sg_fast_supported(const sg_model_t *m, const SgGenPlan &P) {
  if (getenv("SG_DISABLE_FAST")) return 0;
  return fast_shape(m, P) ? 1 : 0;
}

int64_t sg_fast_slab_floats(const SgGenPlan &P, int64_t n_pairs) {
  FastCfg c = fast_cfg(P, n_pairs, true);
  return (int64_t)c.blocks * (P.n_params + 1);
}

int sg_fast_needs_ntn(const SgGenPlan &P) { return plan_avg(P) ? 1 : 0; }

int sg_fast_run(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                const int32_t *order, int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                const float *params, uint64_t seed, const float *y_stats, float *s_out,
                float *slab, float *ntn, int *blocks_out, hipStream_t stream,
                const uint64_t *seed_dev, const sg_pair_source_t *src,
                const int32_t *class_start, const SgAdamPre *adam_pre) {
  if (plan_att(P))
    return sg_fast_att_run(m, P, bwd, recs, order, n_pairs, pair_offset, batch_total, params,
                           seed, y_stats, s_out, slab, ntn, blocks_out, stream, seed_dev, src,
                           class_start, adam_pre);
  return fast_run_impl(m, P, bwd, recs, order, n_pairs, pair_offset, batch_total, params, seed,
                       y_stats, s_out, slab, ntn, blocks_out, stream, seed_dev, src, class_start,
                       adam_pre);
}
#endif

#if defined(SG_FAST_TIMING) && !defined(SG_FAST_ATT_TU)
extern "C" int sg_fast_timing_fetch(unsigned long long *host, int n) {
  if (n > kTimeWaves * 5) n = kTimeWaves * 5;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(sg_fast_times), (size_t)n * 8u, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif
