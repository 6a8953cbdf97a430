/*
 * TEST INFRASTRUCTURE ONLY — C restatement of the reference's default Siamese
 * stack for the timed CPU baseline of bench.py ("kind": "port").
 *
 * Restates (paths relative to /root/reference):
 *   GCN  layers.py:91-118 (sparse dropout 332-338), Dense 192-205, Padding
 *   223-227, NTN 282-310 incl. the (ΣU)·Σrelu(m) broadcast (305-308),
 *   Gaussian final act similarity.py:58-60, broadcast MSE model_mse.py:145-151,
 *   TF autodiff of the same graph.
 * Stack: config.py:44-66 (GCN d_in→32 relu, GCN 32→16 identity, Dense 16→1
 * relu, Padding n_max, NTN(n_max, K=10, relu)), every layer with dropout/bias.
 * Input: the packed pair records of include/siamese_hip.h; dropout masks from
 * the shared counter RNG (oracle/siamese_oracle.py:dropout_mask).
 * float32 arithmetic like TF-CPU; OpenMP over pairs, per-thread gradients.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define H1 32
#define H2 16
#define KNT 10

static inline uint32_t sg_mix(uint32_t x) {
  x ^= x >> 16; x = (x & 0xFFFFFFu) * 0x7FEB35u; x ^= x >> 15; x = (x & 0xFFFFFFu) * 0x846CA7u;
  x ^= x >> 16;
  return x;
}
static inline int keep_draw(uint32_t pk, uint32_t layer, uint32_t side, uint32_t e, uint32_t thr) {
  if (thr >= 65536u) return 1;
  uint32_t h = sg_mix(((layer << 26) | e) ^ pk);   /* one hash: side 0 low, side 1 high */
  uint32_t d = side ? (h >> 16) : (h & 0xFFFFu);
  return d < thr;
}

int64_t sgc_n_params(int d_in, int n_max) {
  return (int64_t)d_in * H1 + H1 + H1 * H2 + H2 + H2 + 1 + (int64_t)n_max * n_max * KNT +
         KNT * 2 * n_max + KNT + KNT;
}

typedef struct {
  float *W0, *b0, *W1, *b1, *Wd, *bd, *W, *V, *U, *bn;
} Params;

static void split(float *p, int d_in, int D, Params *P) {
  P->W0 = p; p += d_in * H1;
  P->b0 = p; p += H1;
  P->W1 = p; p += H1 * H2;
  P->b1 = p; p += H2;
  P->Wd = p; p += H2;
  P->bd = p; p += 1;
  P->W = p; p += D * D * KNT;
  P->V = p; p += KNT * 2 * D;
  P->U = p; p += KNT;
  P->bn = p;
}

typedef struct {
  double *W0, *b0, *W1, *b1, *Wd, *bd, *W, *V, *U, *bn;
} ParamsD;

static void split_d(double *p, int d_in, int D, ParamsD *P) {
  P->W0 = p; p += d_in * H1;
  P->b0 = p; p += H1;
  P->W1 = p; p += H1 * H2;
  P->b1 = p; p += H2;
  P->Wd = p; p += H2;
  P->bd = p; p += 1;
  P->W = p; p += D * D * KNT;
  P->V = p; p += KNT * 2 * D;
  P->U = p; p += KNT;
  P->bn = p;
}

/* float32 arithmetic like TF-CPU with per-thread float gradients: the timed baseline */
#define SGC_FN sgc_fwd_bwd
#define SGC_ACC float
#define SGC_GP Params
#define SGC_SPLIT split
#include "siamese_cpu_body.inc"
#undef SGC_FN
#undef SGC_ACC
#undef SGC_GP
#undef SGC_SPLIT

/* the same per-pair float32 arithmetic, gradients summed in double: the checker for
   full-batch parity (490,000 pairs, where float sums would add their own error) */
#define SGC_FN sgc_fwd_bwd_f64acc
#define SGC_ACC double
#define SGC_GP ParamsD
#define SGC_SPLIT split_d
#include "siamese_cpu_body.inc"
#undef SGC_FN
#undef SGC_ACC
#undef SGC_GP
#undef SGC_SPLIT
