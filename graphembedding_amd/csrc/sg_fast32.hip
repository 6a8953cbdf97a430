// sg_fast32.hip — fused fwd(+bwd) kernel for the reference's default Siamese
// stack at node capacity 32: config C4 (AIDS10knef, N <= 30, Padding/NTN
// input_dim D in (12, 32]; config.py:44-66 with max_in_dims = input_dim = D).
//
// Same scheme as sg_fast.hip (one wavefront per pair, f32 MFMA for every GCN
// product, masks folded into data), for graphs of up to 32 nodes:
//  * each graph is two 16-row tiles; node n sits in tile n/16, row
//    ρ(n % 16) = 4·(n%4) + (n%16)/4, so an accumulator is the B operand of the next
//    Â product and node-contracting products run over the ceil(N/4) k-blocks of
//    4 nodes that hold nodes (runtime trip counts: N is 5..30 in C4);
//  * records are stored at capacity 32 (Â row stride 32), so the whole 32×32
//    block can be read without bounds checks (zero beyond N: record contract);
//  * the NTN head (D up to 32) runs on VALU from one LDS table Wa[a][k][b]:
//    ge2 = Σ_a x1[a] W[a][b][k] gm[k] is formed as per-lane partials over the
//    lane's rows a and reduce-scattered across the four row groups with
//    v_permlane32/16_swap (no transposed copy of W in LDS);
//  * the NTN weight gradient Σ_pairs gm[k] x1[a] x2[b] (D·D·K = 9,000 entries)
//    does not fit per-lane registers, so each pair writes (x1 | 1, x2 | 1, gm) to
//    a buffer and sg_ntn_wgrad_kernel computes Σ gm ⊗ (x1|1) ⊗ (x2|1) with MFMA:
//    gW, and through the constant entries gV and the NTN bias gradient too
//    (split over the same workgroups, written into the same slab rows: the
//    reduction is unchanged).  Hence D <= 31 (slot D holds the 1).
#include <type_traits>

#include "sg_mfma.h"
#include "sg_plan.h"

int sg_num_cus();

namespace {
using namespace sgk;

constexpr int FH1 = 32, FH2 = 16, FK = 10;
constexpr int NC = 32;     // record node capacity
constexpr int TS1 = 36;    // D1 transpose tile row stride
constexpr int W1S = 20;    // W1·ik1 [32][16] row stride
constexpr int W1TS = 36;   // W1ᵀ [16][32] row stride
constexpr int WAS = 32;    // Wa[a][k][b] row stride (b)
constexpr int RS = 34;     // LDS row stride of the record's Â image: 2·ni + g distinct mod 32,
                           // so an Â fragment read (ds_read_b32) is bank-conflict free
// Wa rows (row = a·K + k, 128 B; 32 rows of a, zero past D) are read 16 B at a time; a ds_read_b128 lane group
// holds lanes (a, k) of two row groups, and the identity layout puts ~6 of them on
// one 16-B bank slot.  The chunk index is XOR-swizzled by f(k, a & 1) (a 3-bit
// table found by search, scripts/lds_swizzle_search.py) so that every lane group
// hits distinct slots: conflict-free.  a & 1 = g & 1 for the reading lane.
constexpr uint32_t WA_SWZ0 = 0x2ccb8ff2u, WA_SWZ1 = 0x17a0853u;
__device__ __forceinline__ int wa_swz(int k, int a) {
  return (int)(((a & 1) ? WA_SWZ1 : WA_SWZ0) >> (3 * k)) & 7;
}
// V[k][c] row stride (c < 2D): 66 ≡ 2 mod 32, so the reads sV[kc·VS + a] of lanes (g, kc)
// hit distinct banks (2 kc + g); at 64 the ten rows kc shared one bank (10-way conflicts)
constexpr int VS = 66;
constexpr int NBUF = 80;   // NTN buffer floats per pair: x1[32] | x2[32] | gm[16]
constexpr int MAXW = 8;    // waves per block (2 per SIMD)
// The NTN V rows are read ahead of the W products (C4 165.45 / 165.35 against 163.83 /
// 163.85 M pairs/s read at use, profiles/r05_z2).  gD1 = gZ1·W1ᵀ takes gZ1 with nodes on
// the lanes' rows (its A operand): the gZ1 tiles (nodes on the accumulator rows) go through
// the wave's D1 tile, free in the backward, and are read back transposed (164.15 / 164.05
// against 159.59 / 159.51 recomputing that orientation on the f32 MFMA, profiles/r05_z).
// The losing variants of these and the other round-4/5 A/Bs are in profiles/HISTORY.md.


struct F32Args {
  const uint8_t *recs;
  const int32_t *order;
  int64_t n_pairs;
  int64_t pair_offset;
  int rw4h;       // 16-B words per HBM record
  int rec_bf16;
  const float *params;
  const float *y_stats;
  float *s_out;
  float *slab;
  float *ntn;     // [n_pairs][NBUF] (backward)
  uint32_t key;
  uint32_t thr0, thr1, thr2, thr4;
  float ik0, ik1, ik2, ik4;
  float yeta, inv_batch;
  int d_in, n_params, D;
  int shared_floats, wave_floats;
  int oW0, ob0, oW1, ob1, oWd, obd, oW, oV, oU, obn;
  // pair source (sg_pair_source_t): src_store = 1 gathers each pair from the dense
  // graph store instead of reading a packed record
  int src_store, G;
  const uint4 *sadj, *stypes;   // [G][NC·NC/4], [G][NC/4] 16-B words
  const int32_t *sn, *spairs;   // [G], [n_pairs][2] or NULL (all-pairs grid)
  int64_t grid_base;
  // all-pairs grid with G² < 2^32: q = grid_base + p splits as (q / G, q % G) by one
  // 32-bit multiply-high with gm = ceil(2^32 / G) and one correction (scalar code) instead
  // of the 64-bit division routine (≈130 SALU and two branches per pair)
  uint32_t gm;
  int g32;
  const float *slabels;
  int32_t *status;
};

// Graph ids of local pair p of a store-sourced launch (all lanes, wave-uniform);
// false for ids outside [0, G) (the pair then reads as a zero record)
__device__ __forceinline__ bool f32_pair_ids(const F32Args &A, int p, int &g0, int &g1) {
  if (A.spairs) {
    g0 = A.spairs[2 * (int64_t)p];
    g1 = A.spairs[2 * (int64_t)p + 1];
  } else if (A.g32) {
    // q < 2^32: gm = ceil(2^32 / G) overestimates q / G by less than q / 2^32 < 1, so the
    // high product is q / G rounded down or one above it
    const uint32_t q = (uint32_t)(A.grid_base + p), G = (uint32_t)A.G;
    uint32_t d = __umulhi(q, A.gm);
    d -= (d * G > q) ? 1u : 0u;
    g0 = (int)d;
    g1 = (int)(q - d * G);
  } else {
    const int64_t q = A.grid_base + p;
    g0 = (int)(q / A.G);
    g1 = (int)(q - (int64_t)g0 * A.G);
  }
  const bool ok = (unsigned)g0 < (unsigned)A.G && (unsigned)g1 < (unsigned)A.G;
  if (!ok) g0 = g1 = 0;
  return ok;
}

// per-wave LDS (floats): record image (Â rows at stride RS, then types, n, label,
// tag) | D1 transpose tile (one side) | x1 | x2 | pad
struct Lds32 {
  static constexpr int RW = 2 * NC * NC + 2 * NC + 4;   // 2116 HBM record words
  static constexpr int ADJ = 2 * NC * RS;               // LDS Â image (2176)
  static constexpr int TAIL = ADJ;                      // types | n | label | tag
  static constexpr int REC = 0;
  static constexpr int TILE = 2248;
  static constexpr int X = TILE + 2 * 16 * TS1;          // x1[32] | x2[32]
  static constexpr int WAVE = X + 72;
  static int shared_floats(int d_in, int D) {
    return (d_in + 1) * FH1 + NC * FK * WAS + FK * VS + FH1 * W1S + FH2 * W1TS;
  }
};

// flush slots of one lane: gW1 (8) | gW0/ik0 (16) | dU, loss | db0 (2), db1, dWd, dbd
// (the NTN W, V and bias gradients come from sg_ntn_wgrad_kernel)
constexpr int NS32 = 8 + 16 + 2 + 5;

__device__ __forceinline__ int f32_param(const F32Args &A, int s, int l) {
  const int g = l >> 4, j = l & 15;
  if (s < 8) return A.oW1 + (16 * (s >> 2) + 4 * g + (s & 3)) * FH2 + j;
  s -= 8;
  if (s < 16) {
    const int ty = 16 * (s >> 3) + 4 * g + (s & 3);
    return ty < A.d_in ? A.oW0 + ty * FH1 + 16 * ((s >> 2) & 1) + j : -1;
  }
  s -= 16;
  switch (s) {
    case 0: return (g == 0 && j < FK) ? A.oU + j : -1;
    case 1: return l == 0 ? A.n_params : -1;
    case 2: return g == 0 ? A.ob0 + j : -1;
    case 3: return g == 0 ? A.ob0 + 16 + j : -1;
    case 4: return g == 0 ? A.ob1 + j : -1;
    case 5: return g == 0 ? A.oWd + j : -1;
    case 6: return l == 0 ? A.obd : -1;
    default: return -1;
  }
}

template <bool BWD, bool ALIGNED, bool INTENDED>
__global__ void __launch_bounds__(64 * MAXW) sg_fast32_kernel(F32Args A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using L = Lds32;
  constexpr int RW4 = L::RW / 4;   // 529
  const int tid = threadIdx.x;
  const int l = tid & 63, nw = blockDim.x >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = l >> 4, j = l & 15;
  const uint32_t lb1 = (uint32_t)(FH1 * g + j);   // layer 1: e = 32 n + f
  const uint32_t lb2 = (uint32_t)(FH2 * g + j);   // layer 2: e = 16 n + j
  const int d_in = A.d_in, D = A.D;
  const float *__restrict__ prm = A.params;
  const uint32_t thr0s = __builtin_amdgcn_readfirstlane(A.thr0);
  const uint32_t thr4s = __builtin_amdgcn_readfirstlane(A.thr4);

  // ---- parameter staging (behind the shared tables) and tables ----
  float *sW0 = smem;                            // W0 · ik0 · ik1, row d_in zero
  float *sWa = sW0 + (d_in + 1) * FH1;          // [a][k][WAS]: W[a][b][k] at b
  float *sV = sWa + NC * FK * WAS;              // [k][VS]
  float *sW1 = sV + FK * VS;                    // W1 · ik1 [32][W1S]
  float *sW1T = sW1 + FH1 * W1S;                // W1ᵀ [16][W1TS]
  float *stg = smem + A.shared_floats;
  {
    const int n = A.n_params, bdx = (int)blockDim.x;
    for (int b = 0; b < n; b += 8 * bdx) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = b + k * bdx + tid;
        v[k] = i < n ? prm[i] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = b + k * bdx + tid;
        if (i < n) stg[i] = v[k];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < (d_in + 1) * FH1; i += blockDim.x)
    sW0[i] = i < d_in * FH1 ? stg[A.oW0 + i] * (A.ik0 * A.ik1) : 0.f;
  for (int i = tid; i < NC * FK * WAS; i += blockDim.x) {
    const int row = i / WAS, b = i - row * WAS, a = row / FK, k = row - a * FK;
    sWa[row * WAS + 4 * ((b >> 2) ^ wa_swz(k, a)) + (b & 3)] =
        (a < D && b < D) ? stg[A.oW + (a * D + b) * FK + k] : 0.f;
  }
  for (int i = tid; i < FK * VS; i += blockDim.x) {
    const int k = i / VS, c = i - k * VS;
    sV[i] = c < 2 * D ? stg[A.oV + k * 2 * D + c] : 0.f;
  }
  for (int i = tid; i < FH1 * FH2; i += blockDim.x) {
    const float w = stg[A.oW1 + i];
    sW1[(i / FH2) * W1S + i % FH2] = w * A.ik1;
    sW1T[(i % FH2) * W1TS + i / FH2] = w;
  }
  // P1 comes out scaled by ik1 (relu(ik1 x) = ik1 relu(x)): W0 and b0 carry it
  const float b0v0 = stg[A.ob0 + j] * A.ik1, b0v1 = stg[A.ob0 + 16 + j] * A.ik1;
  const float b1v = stg[A.ob1 + j];
  // Dense weight with the layer-2 dropout scale folded in (D2 kept unscaled; the Dense
  // weight gradient takes ik2 at the flush)
  const float wdv = stg[A.oWd + j] * A.ik2;
  const float bd = stg[A.obd];
  const bool kv = j < FK;
  const int kc = kv ? j : FK - 1;
  const float Uk = kv ? stg[A.oU + kc] : 0.f;
  const float bnk = kv ? stg[A.obn + kc] : 0.f;
  float usum = 0.f;
#pragma unroll
  for (int k = 0; k < FK; ++k) usum += stg[A.oU + k];
  __syncthreads();   // staging area dead: the waves take their regions
  float *W = smem + A.shared_floats + wv * A.wave_floats;
  float *sRec = W + L::REC;
  float *sT = W + L::TILE;
  float *sX = W + L::X;
  for (int i = l; i < 72; i += 64) sX[i] = 0.f;

  // per-lane constants: A row of this lane in an Â product = node(to, j) =
  // 16 to + 4 (j % 4) + j / 4, k column 4 b + g (record row stride NC)
  const int ni = 4 * (j & 3) + (j >> 2);
  const int abase0 = L::REC + ni * RS + g;   // + s·NC·RS + 16·RS·to + 4 b
  const float *w1bp = sW1T + j * W1TS + 8 * g;   // W1[8g+q][j] (Z1 = D1 W1)
  const float *w1tp = sW1 + j * W1S + 4 * g;     // ik1·W1[16t+j][4g+q] (gD1)
  const int wswz = 4 * wa_swz(kc, g);             // Wa chunk swizzle of this lane's rows (floats)
  const int walane = (g * FK + kc) * WAS;         // + rr·4·FK·WAS (an immediate offset)

  // ---- accumulators ----
  f4 gw1[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  f4 gw0[2][2] = {{f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}},
                  {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}}};
  float gb0a0 = 0.f, gb0a1 = 0.f, gb1a = 0.f, gwda = 0.f, gbda = 0.f;
  float gUa = 0.f, lossa = 0.f;
  const float ybar = (BWD && !ALIGNED) ? A.y_stats[0] : 0.f;

  // ---- schedule (as sg_fast: snake over the waves when an order is given) ----
  const int npairs = (int)A.n_pairs;
  const int stride = (int)gridDim.x * nw;
  const int gw = (int)blockIdx.x * nw + wv;
  const int32_t *__restrict__ ord = A.order;
  auto slot_of = [&](int r) -> int {
    return r * stride + ((ord != nullptr && (r & 1)) ? stride - 1 - gw : gw);
  };
  const int rw4h = A.rw4h;
  constexpr int ADJ4 = NC * NC / 4;   // 16-B words of a bf16 adjacency block

  // The order entries of this wave's next 64 iterations (ordA) and the 64 after
  // (ordB), one per lane, as vector loads: the next pair's id is known a whole pair
  // ahead, with no scalar load that every LDS hand-off (lgkmcnt) would wait on.
  auto load_ord = [&](int r0) -> int {
    const int s_ = slot_of(r0 + l);
    return s_ < npairs ? ord[s_] : 0;
  };
  auto ord_at = [&](int v, int lane) -> int {   // clamped: a bad order never reads out of bounds
    const int x = __builtin_amdgcn_readlane(v, lane);
    return x < 0 ? 0 : (x >= npairs ? npairs - 1 : x);
  };
  int ordA = 0, ordB = 0;
  if (ord) {
    ordA = load_ord(0);
    ordB = load_ord(64);
  }
  int pnext = (ord && slot_of(0) < npairs) ? ord_at(ordA, 0) : slot_of(0);

  // wave priority as sg_fast: waves w and w ^ 4 share a SIMD; the higher priority
  // alternates between them by pair count so that neither finishes far ahead
  const int young = wv >> 2;   // 0 / 1, wave-uniform (scalar)
  for (int it = 0;; ++it) {
    const int q = slot_of(it);
    if (q >= npairs) break;
    {   // period 3 pairs, the younger wave first in 2 of them
      const int yturn = (int)((unsigned)((it % 3) - 2) >> 31);
      __builtin_amdgcn_s_setprio(0);   // (scalar, one conditional, as sg_fast)
      if ((yturn ^ young) == 0) __builtin_amdgcn_s_setprio(1);
    }
    const int p = pnext;
    // ---- stage the record (f32 LDS image; bf16 Â widened) ----
#ifdef SG32_ABL_NOREC   // timing ablation only (results invalid): every pair reuses the first
                        // record's Â and types with its own node counts (store source only)
    if (it > 0 && A.src_store && A.sn != nullptr) {
      int g0, g1;
      f32_pair_ids(A, p, g0, g1);
      const int n0 = A.sn[g0], n1 = A.sn[g1];
      sg_wsync();
      if (l == 0) {
        ((int *)sRec)[L::TAIL + 2 * NC] = n0;
        ((int *)sRec)[L::TAIL + 2 * NC + 1] = n1;
      }
      sg_wsync();
    } else
#endif
    {
      constexpr int NREC = (RW4 + 63) / 64;
      uint4 v[NREC];
      if (A.src_store) {
        // the record's 16-B words from the store: Â of g0 | Â of g1 | types of g0 |
        // types of g1 | (n0, n1, label, tag) — the layout sg_pack_pairs writes
        int g0, g1;
        const bool ok = f32_pair_ids(A, p, g0, g1);
        if (!ok && l == 0 && A.status) atomicExch(A.status, (int32_t)SG_ERR_ARG);
        const uint4 *a0 = A.sadj + (size_t)g0 * ADJ4, *a1 = A.sadj + (size_t)g1 * ADJ4;
        const uint4 *t0 = A.stypes + (size_t)g0 * (NC / 4), *t1 = A.stypes + (size_t)g1 * (NC / 4);
        // the loads go out unconditionally (f32_pair_ids clamps invalid ids to graph 0);
        // an invalid pair's words are zeroed afterwards, in one uniform branch
#pragma unroll
        for (int c = 0; c < NREC; ++c) {
          const int w4 = l + 64 * c;
          uint4 x = uint4{0u, 0u, 0u, 0u};
          if (w4 < ADJ4) x = a0[w4];
          else if (w4 < 2 * ADJ4) x = a1[w4 - ADJ4];
          else if (w4 < 2 * ADJ4 + NC / 4) x = t0[w4 - 2 * ADJ4];
          else if (w4 < 2 * ADJ4 + NC / 2) x = t1[w4 - 2 * ADJ4 - NC / 4];
          else if (w4 == 2 * ADJ4 + NC / 2)
            x = uint4{(uint32_t)A.sn[g0], (uint32_t)A.sn[g1],
                      __float_as_uint(A.slabels ? A.slabels[p] : 0.f), (uint32_t)p};
          v[c] = x;
        }
        if (__builtin_expect(!ok, 0)) {
#pragma unroll
          for (int c = 0; c < NREC; ++c) v[c] = uint4{0u, 0u, 0u, 0u};
        }
      } else {
        const uint4 *src = (const uint4 *)(A.recs + (size_t)(uint32_t)p * (size_t)rw4h * 16u);
#pragma unroll
        for (int c = 0; c < NREC; ++c) {
          const int w4 = l + 64 * c;
          v[c] = w4 < rw4h ? src[w4] : uint4{0u, 0u, 0u, 0u};
        }
      }
      sg_wsync();   // the previous pair's LDS reads are done
      // HBM word w of the Â block (row r = w / NC, column w % NC) -> LDS r·RS + w % NC
      auto put4 = [&](int w, f4 v) __attribute__((always_inline)) {
        float *d = sRec + (w / NC) * RS + (w % NC);
        *(float2 *)d = float2{v[0], v[1]};
        *(float2 *)(d + 2) = float2{v[2], v[3]};
      };
      if (A.rec_bf16) {
#pragma unroll
        for (int c = 0; c < NREC; ++c) {
          const int w4 = l + 64 * c;
          if (w4 < ADJ4) {   // 8 bf16 entries of Â -> 8 f32
            const uint4 x = v[c];
            put4(8 * w4, f4{__uint_as_float(x.x << 16), __uint_as_float(x.x & 0xFFFF0000u),
                            __uint_as_float(x.y << 16), __uint_as_float(x.y & 0xFFFF0000u)});
            put4(8 * w4 + 4, f4{__uint_as_float(x.z << 16), __uint_as_float(x.z & 0xFFFF0000u),
                                __uint_as_float(x.w << 16), __uint_as_float(x.w & 0xFFFF0000u)});
          } else if (w4 < rw4h) {
            ((uint4 *)(sRec + L::TAIL))[w4 - ADJ4] = v[c];
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < NREC; ++c) {
          const int w4 = l + 64 * c;
          if (w4 < 2 * ADJ4) {
            const uint4 x = v[c];
            put4(4 * w4, f4{__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z),
                            __uint_as_float(x.w)});
          } else if (w4 < RW4) {
            ((uint4 *)(sRec + L::TAIL))[w4 - 2 * ADJ4] = v[c];
          }
        }
      }
      sg_wsync();
    }
    // the next pair's id (an early L2 touch of its record measured 2% slower: the other
    // wave of the SIMD already hides the record loads)
    {
      const int qn = slot_of(it + 1);
      int pn = qn;
      if (ord) {
        const int rl = (it + 1) & 63;
        if (rl == 0) {
          ordA = ordB;
          ordB = load_ord(it + 65);
        }
        pn = qn < npairs ? ord_at(ordA, rl) : 0;
      }
      pnext = pn;
    }
    const int *ty = (const int *)sRec + L::TAIL;
    int N0 = __builtin_amdgcn_readfirstlane(ty[2 * NC]);
    int N1 = __builtin_amdgcn_readfirstlane(ty[2 * NC + 1]);
    N0 = N0 < 0 ? 0 : (N0 > D ? D : N0);
    N1 = N1 < 0 ? 0 : (N1 > D ? D : N1);
    // The pair body per tile-count class (T0, T1) = (N0 > 16, N1 > 16) + 1: every tile loop and
    // the first tile's k-blocks are straight-line code of the exact length, only the last
    // tile's k-blocks keep a runtime test (KB <= 4 for one tile, KB >= 5 for two)
    auto body = [&](auto T0c, auto T1c) __attribute__((always_inline)) {
      const int KB0 = (N0 + 3) >> 2, KB1 = (N1 + 3) >> 2;   // k-blocks of 4 nodes
      constexpr int T0 = decltype(T0c)::value, T1 = decltype(T1c)::value;   // tiles per side
      constexpr int TM = T0 > T1 ? T0 : T1;
      const int KBm = KB0 > KB1 ? KB0 : KB1;
      // k-block b of a side with T tiles and KB k-blocks holds nodes: T = 1 has KB <= 4, T = 2
      // has KB >= 5, so only the blocks of the last tile need the runtime test
      auto kb_live = [&](int b, int T, int KB) __attribute__((always_inline)) -> bool {
        return b < 4 * T && (b < 4 * (T - 1) || b < KB);
      };
      const uint32_t pk = sg_pair_key(A.key, (uint32_t)(A.pair_offset + p));
      const float label = sRec[L::TAIL + 2 * NC + 2];
      // the hash inputs of layers 1 and 2 as (pk ^ lb) ^ element constant, with pk ^ lb
      // opaque: re-associated as pk ^ (constant ^ lb), the 24 per-lane invariants were kept
      // across the pair loop, spilled, and reloaded from scratch in every pair's hash loop
      uint32_t pk1 = pk ^ lb1, pk2 = pk ^ lb2;
      asm("" : "+v"(pk1), "+v"(pk2));

      // ---- layer-0 (node) and NTN-input dropout masks: one hash per lane ----
      // lanes 0..31: layer 0, node e = l; lanes 32..63: layer 4, element e = l - 32
      uint32_t km0[2], km4[2];   // bit n ↔ node / element n of side s (0 when n >= N_s)
      {
        const int e = l & 31;
        const bool hi = l >= 32;
        const uint32_t h = sg_hash(pk, hi ? 4u : 0u, (uint32_t)e);
        // both thresholds as scalar values first: a select between two kernel-argument
        // fields compiled to a per-lane load from the argument block inside the pair loop
        // (global_load + s_waitcnt vmcnt(0), which also waited for the next record's prefetch)
        const uint32_t thr = hi ? thr4s : thr0s;
        const uint64_t b0 = __ballot((e < N0) & ((h & 0xFFFFu) < thr));
        const uint64_t b1 = __ballot((e < N1) & ((h >> 16) < thr));
        km0[0] = (uint32_t)b0;
        km4[0] = (uint32_t)(b0 >> 32);
        km0[1] = (uint32_t)b1;
        km4[1] = (uint32_t)(b1 >> 32);
      }

      // Â A-fragments of side s: Â[node(to, j)][4b + g] for the side's tiles / k-blocks,
      // re-read from the record image (intact for the whole pair) in each phase
      auto load_af = [&](int s, int T, int KB, float (&af)[2][8]) __attribute__((always_inline)) {
  #pragma unroll
        for (int b = 0; b < 8; ++b) {
          const int ab = abase0 + s * NC * RS + 4 * b;
          // unconditional: entries past N are zero (record contract), and reads without a
          // per-k-block branch issue together (one LDS round trip instead of one per block)
          af[0][b] = b < 4 * T ? W[ab] : 0.f;
          af[1][b] = T > 1 ? W[ab + 16 * RS] : 0.f;
        }
      };

      // ================= forward: ik1 · P1 = Â Z0 + ik1 b0 =================
      uint32_t tyA[2][2];     // [s][tile]: types of node rows 4g+r, 6 bits; 63 = dropped/absent
      f4 d1[2][2][2];         // [s][to][f]: P1, then D1 in place
  #pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int KB = s ? KB1 : KB0, T = s ? T1 : T0;
        const uint32_t kms = km0[s];
        uint32_t tp[2] = {0u, 0u};
  #pragma unroll
        for (int to = 0; to < 2; ++to) {
          d1[s][to][0] = f4{b0v0, b0v0, b0v0, b0v0};
          d1[s][to][1] = f4{b0v1, b0v1, b0v1, b0v1};
        }
        // types, W0 rows and Â fragments of all eight k-blocks first (unconditional reads,
        // two dependent LDS round trips per side instead of two per k-block): nodes past N
        // are masked (k0 = 0 -> the zero row d_in), Â is zero there
        uint32_t t8[8];
  #pragma unroll
        for (int b = 0; b < 8; ++b) t8[b] = (uint32_t)ty[s * NC + 4 * b + g];
  #pragma unroll
        for (int b = 0; b < 8; ++b) {
          const uint32_t t_ = min(t8[b], (uint32_t)(d_in - 1));
          const uint32_t k0 = (kms >> (4 * b + g)) & 1u;
          t8[b] = k0 ? t_ : 63u;   // 63: dropped / absent (the W0 row read is d_in's zero row)
          tp[b >> 2] |= t8[b] << (6 * (b & 3));
        }
        // two halves of four k-blocks (the second only for sides of more than 16 nodes):
        // the reads of a half issue together
  #pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          if (hb < T) {   // the second half only for sides of two tiles (KB > 4)
            float z0a[4], z0b[4], a0v[4], a1v[4];
  #pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int b = 4 * hb + i;
              const float *w0 = sW0 + (t8[b] == 63u ? (uint32_t)d_in : t8[b]) * FH1 + j;
              z0a[i] = w0[0];
              z0b[i] = w0[16];
              const int ab = abase0 + s * NC * RS + 4 * b;
              a0v[i] = W[ab];
              a1v[i] = W[ab + 16 * RS];
            }
  #pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int b = 4 * hb + i;
              if (kb_live(b, T, KB)) {
                d1[s][0][0] = mfma4(a0v[i], z0a[i], d1[s][0][0]);
                d1[s][0][1] = mfma4(a0v[i], z0b[i], d1[s][0][1]);
                if (T > 1) {
                  d1[s][1][0] = mfma4(a1v[i], z0a[i], d1[s][1][0]);
                  d1[s][1][1] = mfma4(a1v[i], z0b[i], d1[s][1][1]);
                }
              }
            }
          }
        }
        tyA[s][0] = tp[0];
        tyA[s][1] = tp[1];
      }
      // D1 = dropout(ik1 relu(P1)): one hash per element (node 16to+4r+g, feature 16f+j)
      // gives both sides' draws; k-blocks past a side's nodes are zeroed
  #pragma unroll
      for (int to = 0; to < 2; ++to)
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nb = 4 * to + r;
  #pragma unroll
          for (int f = 0; f < 2; ++f) {
            if (to < TM && nb < KBm) {
              const uint32_t h =
                  sg_mix(pk1 ^ ((1u << 26) | (uint32_t)(512 * to + 128 * r + 16 * f)));
  #pragma unroll
              for (int s = 0; s < 2; ++s) {
                const uint32_t dr = s ? (h >> 16) : (h & 0xFFFFu);
                const float v = relu_bits(d1[s][to][f][r]);
                d1[s][to][f][r] = (nb < (s ? KB1 : KB0) && dr < A.thr1) ? v : 0.f;
              }
            } else {
              d1[0][to][f][r] = d1[1][to][f][r] = 0.f;
            }
          }
        }

      // Z1 = D1 W1 (D1 transposed through the tile), H2 = Â Z1 + b1, per side
      f4 h2[2][2];
  #pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int KB = s ? KB1 : KB0, T = s ? T1 : T0;
  #pragma unroll
        for (int to = 0; to < 2; ++to) {
          if (to < T) {
  #pragma unroll
            for (int f = 0; f < 2; ++f)
  #pragma unroll
              for (int r = 0; r < 4; ++r) sT[(16 * to + 4 * g + r) * TS1 + 16 * f + j] = d1[s][to][f][r];
          }
        }
        sg_wsync();
        f4 z1[2];
        const f4 wlo = *(const f4 *)w1bp, whi = *(const f4 *)(w1bp + 4);
  #pragma unroll
        for (int to = 0; to < 2; ++to) {
          z1[to] = f4{0.f, 0.f, 0.f, 0.f};
          if (to < T) {
            const float *Tr = sT + (16 * to + j) * TS1 + 8 * g;
            const f4 lo = *(const f4 *)Tr, hi = *(const f4 *)(Tr + 4);
  #pragma unroll
            for (int qq = 0; qq < 4; ++qq) z1[to] = mfma4(lo[qq], wlo[qq], z1[to]);
  #pragma unroll
            for (int qq = 0; qq < 4; ++qq) z1[to] = mfma4(hi[qq], whi[qq], z1[to]);
          }
        }
        float af[2][8];
        load_af(s, T, KB, af);
  #pragma unroll
        for (int to = 0; to < 2; ++to) {
          h2[s][to] = f4{b1v, b1v, b1v, b1v};
          if (to < T) {
  #pragma unroll
            for (int b = 0; b < 8; ++b)
              if (kb_live(b, T, KB)) h2[s][to] = mfma4(af[to][b], z1[b >> 2][b & 3], h2[s][to]);
          }
        }
        sg_wsync();   // the tile is rewritten by the next side
      }

      // D2 = dropout(H2); zpre = D2·Wd + bd; x = dropout(pad(relu(zpre)))
      float xo[2][8], d2[2][8];   // [s][4 to + r] ↔ node 16 to + 4 r + g
      uint32_t kb2[2] = {0u, 0u};
  #pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        const int to = nb >> 2, r = nb & 3;
        if (to < TM && nb < KBm) {
          const uint32_t h = sg_mix(pk2 ^ ((2u << 26) | (uint32_t)(256 * to + 64 * r)));
  #pragma unroll
          for (int s = 0; s < 2; ++s) {
            if (nb < (s ? KB1 : KB0)) {
              const bool k2 = (s ? (h >> 16) : (h & 0xFFFFu)) < A.thr2;
              d2[s][nb] = k2 ? h2[s][to][r] : 0.f;   // D2 / ik2
              kb2[s] |= (k2 ? 1u : 0u) << nb;
              const float z = row_sum16(d2[s][nb] * wdv) + bd;
              const bool k4 = (km4[s] >> (16 * to + 4 * r + g)) & 1u;   // includes n < N
              xo[s][nb] = ((z > 0.f) & k4) ? z * A.ik4 : 0.f;
            } else {
              d2[s][nb] = xo[s][nb] = 0.f;
            }
          }
        } else {
          d2[0][nb] = d2[1][nb] = xo[0][nb] = xo[1][nb] = 0.f;
        }
      }
      if (j == 0) {   // x1 | x2 for every lane (node 16to+4r+g of row group g)
  #pragma unroll
        for (int nb = 0; nb < 8; ++nb) {
          sX[4 * nb + g] = xo[0][nb];
          sX[NC + 4 * nb + g] = xo[1][nb];
        }
      }
      sg_wsync();

      // ================= NTN head (layers.py:282-310) =================
      // lane (g, k = j) owns rows a = 4r' + g.  Per 4-column block bq of b (outer loop):
      // u[r'] += Σ_b W[a][b][k] x2[b] (forward), and the partials Σ_{own a} x1[a] W[a][b][k]
      // of ge2 = Σ_a x1[a] W[a][b][k] gm[k] share the Wa reads; the partials of the
      // block are reduce-scattered over the four row groups at once (half 0 = g < 2
      // keeps b % 4 < 2, then row g keeps b % 4 == g): cs[bq] ↔ b = 4 bq + g.
      float u[8], cs[8];
  #pragma unroll
      for (int rr = 0; rr < 8; ++rr) u[rr] = cs[rr] = 0.f;
  #ifdef SG32_ABL_NONTN   // timing ablation only (results invalid): no NTN W products
      constexpr int NTN_BQ = 0;
  #else
      constexpr int NTN_BQ = 8;
  #endif
      // The Wa rows of one column block are read together (one LDS round trip per block):
      // KR rows, KB0 rounded up to even, as straight-line code per KR.  Rows KB0..KR-1 of
      // x1 are zero, so their u rows go unused and their cb terms are exact fmaf(0, w, cb).
      auto ntn_fwd = [&](auto KRc) __attribute__((always_inline)) {
        constexpr int KR = decltype(KRc)::value;
  #pragma unroll
        for (int bq = 0; bq < NTN_BQ; ++bq) {
          if (kb_live(bq, T1, KB1)) {
            const f4 x2 = *(const f4 *)(sX + NC + 4 * bq);
            const float *wb = sWa + walane + ((4 * bq) ^ wswz);
            f4 w[KR];
  #pragma unroll
            for (int rr = 0; rr < KR; ++rr) w[rr] = *(const f4 *)(wb + rr * 4 * FK * WAS);   // rows a >= D are zero
            float cb[4] = {0.f, 0.f, 0.f, 0.f};
  #pragma unroll
            for (int rr = 0; rr < KR; ++rr) {
              const float x1a = xo[0][rr];
  #pragma unroll
              for (int e = 0; e < 4; ++e) {
                u[rr] = fmaf(w[rr][e], x2[e], u[rr]);
                cb[e] = fmaf(x1a, w[rr][e], cb[e]);
              }
            }
            float hs[2];
  #pragma unroll
            for (int e = 0; e < 2; ++e) {
              const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(cb[e]),
                                                                __float_as_uint(cb[e + 2]), false, false);
              hs[e] = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
            }
            const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(hs[0]),
                                                              __float_as_uint(hs[1]), false, false);
            cs[bq] = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
          }
        }
      };
      if constexpr (T0 == 2) {
        if (KB0 > 6) ntn_fwd(std::integral_constant<int, 8>{});
        else ntn_fwd(std::integral_constant<int, 6>{});
      } else {
        if (KB0 > 2) ntn_fwd(std::integral_constant<int, 4>{});
        else ntn_fwd(std::integral_constant<int, 2>{});
      }
      // V entries of the lane's rows, read unconditionally (one LDS round trip; rows past
      // the sides' k-blocks are never used): vu = u + V[k][a] (forward and ∂L/∂x1)
      float vu[8], vb[8];
  #pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int a = 4 * rr + g;
        const int ac = a < D ? a : 0;
        vu[rr] = u[rr] + sV[kc * VS + ac];
        vb[rr] = sV[kc * VS + D + ac];
      }
      float mpart = 0.f;
  #pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        if (kb_live(rr, T0, KB0)) mpart = fmaf(xo[0][rr], vu[rr], mpart);
        if (kb_live(rr, T1, KB1)) mpart = fmaf(xo[1][rr], vb[rr], mpart);
      }
      const float m = xsum32(xsum16(mpart)) + bnk;
      const float rk = (kv & (m > 0.f)) ? m : 0.f;
      const float rsum = row_sum16(rk);
      const float sv = INTENDED ? row_sum16(Uk * rk) : usum * rsum;
      if (!BWD) {
        if (l == 0) A.s_out[p] = sv;
        return;
      }
      if (A.s_out && l == 0) A.s_out[p] = sv;
      const float yhat = __expf(-A.yeta * sv * sv);
      float gy;
      if (!ALIGNED) {
        gy = yhat - ybar;
        lossa += 0.5f * gy * gy;
      } else {
        const float dl = yhat - label;
        gy = dl * A.inv_batch;
        lossa += 0.5f * dl * dl * A.inv_batch;
      }
      const float gs = gy * (-2.f * A.yeta * sv * yhat);

      // ================= NTN backward =================
      const float gmk = (kv & (m > 0.f)) ? (INTENDED ? gs * Uk : gs * usum) : 0.f;
      if (g == 0) gUa += INTENDED ? gs * rk : gs * rsum;
      // deferred NTN gradients: this pair's (x1 | 1, x2 | 1, gm)
      {
        float *nb_ = A.ntn + (size_t)(uint32_t)p * NBUF;
        nb_[l] = ((l & (NC - 1)) == D) ? 1.f : sX[l];
        if (g == 0) nb_[2 * NC + j] = gmk;
      }
      const float gmk4 = gmk * A.ik4;
      float ge[2][8];   // dL/dx · ik4 (before the x > 0 mask) of the lane's rows
  #pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        ge[0][rr] = ge[1][rr] = 0.f;
        if (kb_live(rr, T0, KB0)) {
          ge[0][rr] = row_sum16(gmk4 * vu[rr]);
        }
      }
  #pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        if (kb_live(rr, T1, KB1)) {
          const int b = 4 * rr + g;
          const int bc = b < D ? b : 0;
          ge[1][rr] = row_sum16(gmk4 * (sV[kc * VS + D + bc] + cs[rr]));
        }
      }

      // ================= GCN backward, per side =================
  #pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int KB = s ? KB1 : KB0, T = s ? T1 : T0;
        float af[2][8];
        load_af(s, T, KB, af);
        f4 gh2[2];
  #pragma unroll
        for (int to = 0; to < 2; ++to) {
          gh2[to] = f4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nb = 4 * to + r;
            if (kb_live(nb, T, KB)) {
              const float gp = xo[s][nb] > 0.f ? ge[s][nb] : 0.f;
              gwda = fmaf(d2[s][nb], gp, gwda);
              gbda += gp;
              const float v = ((kb2[s] >> nb) & 1u) ? gp * wdv : 0.f;
              gb1a += v;
              gh2[to][r] = v;
            }
          }
        }
        // gZ1 = Âᵀ gH2 (Â symmetric) in both orientations
        f4 gz1[2], gz1t[2];
  #pragma unroll
        for (int to = 0; to < 2; ++to) {
          gz1[to] = gz1t[to] = f4{0.f, 0.f, 0.f, 0.f};
          if (to < T) {
  #pragma unroll
            for (int b = 0; b < 8; ++b) {
              if (kb_live(b, T, KB)) {
                gz1[to] = mfma4(af[to][b], gh2[b >> 2][b & 3], gz1[to]);
              }
            }
          }
        }
        // gW1 += D1ᵀ gZ1 (D1's C-layout entries are the A operand)
  #pragma unroll
        for (int b = 0; b < 8; ++b) {
          if (kb_live(b, T, KB)) {
  #pragma unroll
            for (int f = 0; f < 2; ++f) gw1[f] = mfma4(d1[s][b >> 2][f][b & 3], gz1[b >> 2][b & 3], gw1[f]);
          }
        }
        // gZ1 rows 16 to + 4g + r, feature j into the tile; read back as row 16 to + j,
        // features 4g..4g+3 (the previous side's reads are done: program order)
  #pragma unroll
        for (int to = 0; to < 2; ++to)
          if (to < T)
  #pragma unroll
            for (int r = 0; r < 4; ++r) sT[(16 * to + 4 * g + r) * TS1 + j] = gz1[to][r];
        sg_wsync();
  #pragma unroll
        for (int to = 0; to < 2; ++to)
          if (to < T) gz1t[to] = *(const f4 *)(sT + (16 * to + j) * TS1 + 4 * g);
        // gD1 · ik1 = gZ1 (W1 ik1)ᵀ; gP1 = keep·relu' (D1 > 0); gZ0 = Âᵀ gP1
        f4 gp1[2][2];   // [to][f]
  #pragma unroll
        for (int f = 0; f < 2; ++f) {
          const f4 wt = *(const f4 *)(w1tp + 16 * f * W1S);
  #pragma unroll
          for (int to = 0; to < 2; ++to) {
            gp1[to][f] = f4{0.f, 0.f, 0.f, 0.f};
            if (to < T) {
              f4 acc = {0.f, 0.f, 0.f, 0.f};
  #pragma unroll
              for (int qq = 0; qq < 4; ++qq) acc = mfma4(gz1t[to][qq], wt[qq], acc);
  #pragma unroll
              for (int r = 0; r < 4; ++r) gp1[to][f][r] = d1[s][to][f][r] > 0.f ? acc[r] : 0.f;
              const float gsum = (gp1[to][f][0] + gp1[to][f][1]) + (gp1[to][f][2] + gp1[to][f][3]);
              if (f) gb0a1 += gsum;
              else gb0a0 += gsum;
            }
          }
        }
  #pragma unroll
        for (int to = 0; to < 2; ++to) {
          if (to < T) {
            // one-hot Xᵀ rows: type 16τ + j, k-slots 8g + e ↔ node rows 4g + (e & 3)
            uint4 ohA[2], ohL[2];
  #pragma unroll
            for (int tau = 0; tau < 2; ++tau) {
              uint32_t o[4];
  #pragma unroll
              for (int r = 0; r < 4; ++r)
                o[r] = (((tyA[s][to] >> (6 * r)) & 63u) == (uint32_t)(16 * tau + j)) ? 0x3F80u : 0u;
              const uint32_t o01 = o[0] | (o[1] << 16), o23 = o[2] | (o[3] << 16);
              ohA[tau] = uint4{o01, o23, o01, o23};
              ohL[tau] = uint4{o01, o23, 0u, 0u};
            }
  #pragma unroll
            for (int f = 0; f < 2; ++f) {
              f4 gz0 = {0.f, 0.f, 0.f, 0.f};
  #pragma unroll
              for (int b = 0; b < 8; ++b)
                if (kb_live(b, T, KB)) gz0 = mfma4(af[to][b], gp1[b >> 2][f][b & 3], gz0);
              uint32_t h01, m01, l01, h23, m23, l23;
              split3(gz0[0], gz0[1], h01, m01, l01);
              split3(gz0[2], gz0[3], h23, m23, l23);
              const uint4 bhm = {h01, h23, m01, m23}, bl = {l01, l23, 0u, 0u};
  #pragma unroll
              for (int tau = 0; tau < 2; ++tau) {
                gw0[tau][f] = mfbf(ohL[tau], bl, gw0[tau][f]);
                gw0[tau][f] = mfbf(ohA[tau], bhm, gw0[tau][f]);
              }
            }
          }
        }
      }
    };
    const bool two0 = N0 > 16, two1 = N1 > 16;
    if (two0) {
      if (two1) body(std::integral_constant<int, 2>{}, std::integral_constant<int, 2>{});
      else body(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
    } else {
      if (two1) body(std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});
      else body(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    }
  }

  if (!BWD) return;
  // ---- flush: every wave dumps its slots to LDS, all threads sum the waves ----
  gb0a0 = xsum32(xsum16(gb0a0));
  gb0a1 = xsum32(xsum16(gb0a1));
  gb1a = xsum32(xsum16(gb1a));
  gwda = xsum32(xsum16(gwda)) * A.ik2;
  gbda = xsum32(xsum16(gbda));
  float *F = smem;
  __syncthreads();
  {
    float *Fw = F + (size_t)wv * NS32 * 64 + l;
    int s = 0;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) Fw[64 * s++] = gw1[f][r];
#pragma unroll
    for (int tau = 0; tau < 2; ++tau)
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) Fw[64 * s++] = gw0[tau][f][r] * A.ik0;
    Fw[64 * s++] = gUa;
    Fw[64 * s++] = lossa;
    Fw[64 * s++] = gb0a0;
    Fw[64 * s++] = gb0a1;
    Fw[64 * s++] = gb1a;
    Fw[64 * s++] = gwda;
    Fw[64 * s++] = gbda;
  }
  __syncthreads();
  float *dst = A.slab + (size_t)blockIdx.x * (size_t)(A.n_params + 1);
  for (int idx = tid; idx < NS32 * 64; idx += blockDim.x) {
    const int prm_i = f32_param(A, idx >> 6, idx & 63);
    if (prm_i < 0) continue;
    float acc = 0.f;
    for (int w = 0; w < nw; ++w) acc += F[(size_t)w * NS32 * 64 + idx];
    dst[prm_i] = acc;
  }
}

// ---- NTN gradients: O[a][b'][k] = Σ_p gm_p[k] x1_p[a] x2_p[b'], a, b' <= D ----
// with x1_p[D] = x2_p[D] = 1: gW = O[a < D][b' < D], gV[k][a] = O[a][D],
// gV[k][D + b'] = O[D][b'], gb = O[D][D].  Workgroup b sums its contiguous share
// of the pairs with MFMA: output rows a (16-row tiles), columns c = b'·K + k (the
// ceil((D + 1) K / 16) column tiles, NTW per wave, dealt round-robin over the NWV waves),
// the pairs are the K dimension (4 per k-step), operands from an LDS-staged chunk whose
// successor is loaded into registers meanwhile.  The result goes to the NTN columns of slab
// row b (the fused kernel writes the other columns of the same row).  ROW1: a second row
// tile (D > 16, rows 16..D); at D = 16 (the Average / Attention stacks) its one live row
// a = 16 is x1's constant 1, so O[16][c] = Σ_p gm_p[k] x2_p[b'] is a column sum, kept on
// VALU per lane and summed over the four row groups at the end.  Round 6 (Average stack,
// 490,000 pairs): 188 µs per launch with 20 column tiles x 2 row tiles at any D and one
// global round trip per 64-pair chunk, 131 µs with D's tiles only, 70 µs double-buffered,
// 62 µs at 8 waves (profiles/r06_e, r06_f).
constexpr int WG_CHUNK = 64;   // pairs staged per LDS round
// The pooled stacks' (D = 16) compact row: x1[16] | x2[16] | gm[10], zeros, and a 1 in the
// last slot (x2's constant entry; x1's is the kernel's VALU column sum, !ROW1)
constexpr int NBUF16 = 48;
constexpr int NB16_ZERO = 46, NB16_ONE = 47;

template <int NTW, bool ROW1, int NWV, int NB>
__global__ void __launch_bounds__(64 * NWV) sg_ntn_wgrad_kernel(const float *__restrict__ ntn,
                                                          int64_t n_pairs, int D, int oW,
                                                          int oV, int obn, int C,
                                                          float *__restrict__ slab) {
  static_assert(NB == NBUF || (NB == NBUF16 && !ROW1), "row layouts");
  constexpr int NBUF = NB;   // floats per pair row (the capacity-32 layout or the compact one)
  constexpr int CH = WG_CHUNK * NWV / 4, NT = 64 * NWV;   // pairs per chunk, threads
  __shared__ __attribute__((aligned(16))) float st[CH * NBUF];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int g = l >> 4, j = l & 15;
  const int nb = gridDim.x;
  const int64_t p0 = n_pairs * blockIdx.x / nb, p1 = n_pairs * (blockIdx.x + 1) / nb;
  const int DK = (D + 1) * FK;   // columns b' <= D
  // this lane's columns in its wave's NTW column tiles (tiles past DK read gm slot 15,
  // which is 0: their products are zero and they are not written)
  int cb_[NTW], ck_[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int c = 16 * (w + NWV * t) + j;
    const int cc = c < DK ? c : 0;
    if constexpr (NB == NBUF16) {   // (D = 16)
      cb_[t] = cc / FK < 16 ? 16 + cc / FK : NB16_ONE;
      ck_[t] = c < DK ? 32 + cc % FK : NB16_ZERO;
    } else {
      cb_[t] = NC + cc / FK;          // x2[b'] offset in the pair's buffer row
      ck_[t] = c < DK ? 2 * NC + cc % FK : 2 * NC + 15;   // gm[k] (slot 15 is 0: k < FK only)
    }
  }
  f4 acc[2][NTW];
  float csum[NTW];   // !ROW1: Σ of this lane's pairs' products, column 16 (w + 4t) + j
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    acc[0][t] = acc[1][t] = f4{0.f, 0.f, 0.f, 0.f};
    csum[t] = 0.f;
  }
  // the chunks are double-buffered through registers: chunk i + 1's loads are in flight
  // while chunk i is multiplied out of LDS (one global round trip per chunk otherwise,
  // ≈30 of them per block, each exposed)
  constexpr int PER = CH * NBUF / 4 / NT;   // f4 per thread per chunk
  static_assert(PER * NT * 4 == CH * NBUF, "chunk split");
  f4 nx[PER];
  auto fetch = [&](int64_t c0) __attribute__((always_inline)) {
    const int np = (int)((p1 - c0) < CH ? (p1 - c0) : CH);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = tid + NT * u, pp = i / (NBUF / 4);
      nx[u] = pp < np ? ((const f4 *)(ntn + (size_t)c0 * NBUF))[i] : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (p0 < p1) fetch(p0);
  for (int64_t c0 = p0; c0 < p1; c0 += CH) {
    const int np = (int)((p1 - c0) < CH ? (p1 - c0) : CH);
    __syncthreads();   // the previous chunk's reads are done
#pragma unroll
    for (int u = 0; u < PER; ++u) ((f4 *)st)[tid + NT * u] = nx[u];
    __syncthreads();
    if (c0 + CH < p1) fetch(c0 + CH);
#pragma unroll 2
    for (int k0 = 0; k0 < np; k0 += 4) {
      const float *row = st + (k0 + g) * NBUF;   // pair k0 + g (zero rows past np)
      const float a0 = row[j];
      const float a1 = ROW1 ? row[16 + j] : 0.f;
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const float bv = row[ck_[t]] * row[cb_[t]];
        acc[0][t] = mfma4(a0, bv, acc[0][t]);
        if (ROW1) acc[1][t] = mfma4(a1, bv, acc[1][t]);
        else csum[t] += bv;
      }
    }
  }
  if (!ROW1) {   // row a = D = 16: the column sums over the four row groups
#pragma unroll
    for (int t = 0; t < NTW; ++t) csum[t] = xsum32(xsum16(csum[t]));
  }
  float *dst = slab + (size_t)blockIdx.x * C;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      const int c = 16 * (w + NWV * t) + j;
      const int bb = c / FK, k = c - bb * FK;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int a = 16 * rt + 4 * g + r;
        if (a > D || c >= DK) continue;
        if (!ROW1 && rt == 1 && (g != 0 || r != 0)) continue;   // a = 16 only, from csum
        int prm_i;
        if (a < D) prm_i = bb < D ? oW + (a * D + bb) * FK + k : oV + k * 2 * D + a;
        else prm_i = bb < D ? oV + k * 2 * D + D + bb : obn + k;
        dst[prm_i] = (!ROW1 && rt == 1) ? csum[t] : acc[rt][t][r];
      }
    }
}

struct F32Cfg {
  int waves, blocks, shared_floats, wave_floats;
  size_t lds;
};

F32Cfg f32_cfg(const SgGenPlan &P, int64_t n_pairs, bool bwd) {
  F32Cfg c;
  c.shared_floats = Lds32::shared_floats(P.d_in, P.D);
  c.wave_floats = Lds32::WAVE;
  c.waves = MAXW;
  size_t lds = (size_t)(c.shared_floats + MAXW * c.wave_floats) * 4u;
  const size_t stage = (size_t)(c.shared_floats + P.n_params) * 4u;
  const size_t fl = bwd ? (size_t)MAXW * NS32 * 64u * 4u : 0u;
  if (stage > lds) lds = stage;
  if (fl > lds) lds = fl;
  c.lds = lds;
  const int64_t want = (n_pairs + MAXW - 1) / MAXW;
  const int64_t cap = (int64_t)sg_num_cus();
  c.blocks = (int)(want < cap ? (want > 0 ? want : 1) : cap);
  return c;
}

}  // namespace

// --------------------------------------------------------------------------
int sg_fast32_supported(const sg_model_t *m, const SgGenPlan &P) {
  if (getenv("SG_DISABLE_FAST")) return 0;
  if (m->num_layers != 5) return 0;
  const sg_layer_t *Ly = m->layers;
  if (Ly[0].kind != SG_GCN || !Ly[0].sparse_inputs || Ly[0].output_dim != FH1 ||
      Ly[0].act != SG_ACT_RELU || !Ly[0].bias)
    return 0;
  if (Ly[1].kind != SG_GCN || Ly[1].input_dim != FH1 || Ly[1].output_dim != FH2 ||
      Ly[1].act != SG_ACT_IDENTITY || !Ly[1].bias)
    return 0;
  if (Ly[2].kind != SG_DENSE || Ly[2].input_dim != FH2 || Ly[2].output_dim != 1 ||
      Ly[2].act != SG_ACT_RELU || !Ly[2].bias)
    return 0;
  if (Ly[3].kind != SG_PADDING || Ly[3].padding_value != 0.f) return 0;
  const int D = Ly[3].output_dim;
  if (Ly[4].kind != SG_NTN || Ly[4].input_dim != D || Ly[4].output_dim != FK ||
      Ly[4].act != SG_ACT_RELU || !Ly[4].bias)
    return 0;
  if (m->n_max != NC || D <= 12 || D >= NC) return 0;   // slot D of x holds the 1
  if (m->final_act != SG_FINAL_GAUSSIAN) return 0;
  if (m->d_in > 32 || m->d_in < 1) return 0;
  // LDS: the shared tables, 8 wave regions and the flush must fit one CU
  const size_t lds = (size_t)(Lds32::shared_floats(m->d_in, D) + MAXW * Lds32::WAVE) * 4u;
  if (lds > 163840u) return 0;
  return P.n_params > 0 ? 1 : 0;
}

int64_t sg_fast32_slab_floats(const SgGenPlan &P, int64_t n_pairs) {
  const F32Cfg c = f32_cfg(P, n_pairs, true);
  return (int64_t)c.blocks * (P.n_params + 1);
}

int64_t sg_fast32_ntn_floats(int64_t n_pairs) { return n_pairs * NBUF; }

// NTN W / V / bias gradients from a per-pair buffer into the NTN columns of slab rows
// 0..blocks-1: rows [n_pairs][80] (x1|1, x2|1 at capacity 32, gm at 64) for sg_fast32,
// or with `compact` (sg_fast's Average / Attention stacks, D = 16) the compact rows
// [n_pairs][48] (x1 | x2 | gm, 0, 1: NBUF16): 192 instead of 320 bytes written and read per
// pair
int sg_ntn_wgrad_run(const float *ntn, int64_t n_pairs, int D, int oW, int oV, int obn, int C,
                     float *slab, int blocks, hipStream_t st, bool compact) {
  if (D < 1 || D > 31 || obn < 0 || (compact && D != 16)) return SG_ERR_ARG;
  // column tiles: ceil((D + 1) K / 16)
  const int nct = ((D + 1) * FK + 15) / 16;
  // D <= 15: rows a <= D fit the first tile; D = 16: row a = 16 on VALU
  if (compact)   // 8 waves of 2 tiles, compact rows
    hipLaunchKernelGGL((sg_ntn_wgrad_kernel<2, false, 8, NBUF16>), dim3(blocks), dim3(512), 0,
                       st, ntn, n_pairs, D, oW, oV, obn, C, slab);
  else if (D <= 16 && nct <= 16)
    hipLaunchKernelGGL((sg_ntn_wgrad_kernel<2, false, 8, NBUF>), dim3(blocks), dim3(512), 0, st,
                       ntn, n_pairs, D, oW, oV, obn, C, slab);
  else
    hipLaunchKernelGGL((sg_ntn_wgrad_kernel<5, true, 4, NBUF>), dim3(blocks), dim3(256), 0, st,
                       ntn, n_pairs, D, oW, oV, obn, C, slab);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int sg_fast32_run(const sg_model_t *m, const SgGenPlan &P, bool bwd, const void *recs,
                  const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                  int64_t batch_total, const float *params, uint64_t seed, const float *y_stats,
                  float *s_out, float *slab, float *ntn, int *blocks_out, hipStream_t stream,
                  const sg_pair_source_t *src) {
  const F32Cfg c = f32_cfg(P, n_pairs, bwd);
  if (n_pairs > 0x7FFFFFFF - (int64_t)c.blocks * c.waves * 2) return SG_ERR_ARG;
  F32Args A;
  A.recs = (const uint8_t *)recs;
  A.src_store = src ? 1 : 0;
  A.G = src ? src->n_graphs : 0;
  A.sadj = src ? (const uint4 *)src->adj : nullptr;
  A.stypes = src ? (const uint4 *)src->types : nullptr;
  A.sn = src ? src->n : nullptr;
  A.spairs = src ? src->pair_idx : nullptr;
  A.grid_base = src ? src->grid_base : 0;
  {
    const uint64_t G = src ? (uint64_t)(src->n_graphs > 0 ? src->n_graphs : 1) : 1u;
    A.g32 = (src && src->pair_idx == nullptr && G * G <= 0xFFFFFFFFull &&
             src->grid_base >= 0 && (uint64_t)src->grid_base + (uint64_t)n_pairs <= G * G) ? 1 : 0;
    A.gm = (uint32_t)(((1ull << 32) + G - 1) / G);   // ceil(2^32 / G) (G >= 2: fits 32 bits)
  }
  A.slabels = src ? src->labels : nullptr;
  A.status = src ? src->status : nullptr;
  if (src && (P.adj_dtype != SG_DTYPE_F32 || src->n_max != NC || src->n_graphs <= 0 ||
              !src->adj || !src->types || !src->n))
    return SG_ERR_ARG;
  A.order = order;
  A.n_pairs = n_pairs;
  A.pair_offset = pair_offset;
  A.rw4h = P.hbm_words / 4;
  A.rec_bf16 = P.adj_dtype == SG_DTYPE_BF16 ? 1 : 0;
  A.params = params;
  A.y_stats = y_stats;
  A.s_out = s_out;
  A.slab = slab;
  A.ntn = ntn;
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
  A.d_in = P.d_in;
  A.n_params = P.n_params;
  A.D = P.D;
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
  const bool aligned = m->loss_mode == SG_LOSS_ALIGNED;
  const bool intended = m->ntn_mode == SG_NTN_INTENDED;
  auto launch = [&](const void *fn, auto kern) {
    if (c.lds > 65536u)
      (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds);
    hipLaunchKernelGGL(kern, dim3(c.blocks), dim3(64 * c.waves), c.lds, stream, A);
  };
#define SG32_LAUNCH(B, AL, IN) \
  launch((const void *)sg_fast32_kernel<B, AL, IN>, sg_fast32_kernel<B, AL, IN>)
  if (!bwd) {
    if (intended) SG32_LAUNCH(false, false, true);
    else SG32_LAUNCH(false, false, false);
  } else if (aligned) {
    if (intended) SG32_LAUNCH(true, true, true);
    else SG32_LAUNCH(true, true, false);
  } else {
    if (intended) SG32_LAUNCH(true, false, true);
    else SG32_LAUNCH(true, false, false);
  }
#undef SG32_LAUNCH
  if (bwd) {
    const int rc = sg_ntn_wgrad_run((const float *)ntn, n_pairs, P.D, P.offW, P.offV, P.offB,
                                    P.n_params + 1, slab, c.blocks, stream, false);
    if (rc != SG_OK) return rc;
  }
  if (blocks_out) *blocks_out = c.blocks;
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}
