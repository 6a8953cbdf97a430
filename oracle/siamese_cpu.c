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

/* returns 0 ok; grad_out gets Σ ∂loss_mse/∂θ; loss_out = ½Σ(ŷ-ȳ)² */
int sgc_fwd_bwd(const uint32_t *recs, int64_t n_pairs, int64_t pair_offset, int n_max, int d_in,
                const float *params, uint64_t seed, float keep, float yeta, float ybar,
                float *s_out, float *grad_out, double *loss_out, int n_threads) {
  const int D = n_max, NN = n_max * n_max;
  const int words = 2 * NN + 2 * n_max + 4;
  const int64_t np_ = sgc_n_params(d_in, n_max);
  uint32_t thr = 65536u;
  if (keep < 1.f) {
    long r = (long)((double)keep * 65536.0 + 0.5);
    thr = (uint32_t)(r < 0 ? 0 : (r > 65536 ? 65536 : r));
  }
  const float ik = 1.f / keep;
  const uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
  const uint32_t key = (lo * 0x85EBCA6Bu) ^ hi;
  Params P;
  split((float *)params, d_in, D, &P);  /* read-only use */
  int nt = n_threads > 0 ? n_threads : 1;
#ifdef _OPENMP
  omp_set_num_threads(nt);
#else
  nt = 1;
#endif
  float *gbuf = (float *)calloc((size_t)nt * np_, sizeof(float));
  double *lbuf = (double *)calloc((size_t)nt, sizeof(double));
  if (!gbuf || !lbuf) return 1;
#pragma omp parallel
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    float *g = gbuf + (size_t)tid * np_;
    Params G;
    split(g, d_in, D, &G);
    float *m0 = malloc(sizeof(float) * 2 * n_max), *P1 = malloc(sizeof(float) * 2 * n_max * H1);
    float *D1 = malloc(sizeof(float) * 2 * n_max * H1), *T = malloc(sizeof(float) * n_max * H1);
    float *D2 = malloc(sizeof(float) * 2 * n_max * H2), *zp = malloc(sizeof(float) * 2 * n_max);
    float *x = malloc(sizeof(float) * 2 * D), *u = malloc(sizeof(float) * D * KNT);
    float *gx = malloc(sizeof(float) * 2 * D), *gH2 = malloc(sizeof(float) * n_max * H2);
    float *gZ = malloc(sizeof(float) * n_max * H1), *gP = malloc(sizeof(float) * n_max * H1);
    double lacc = 0.0;
#pragma omp for schedule(static)
    for (int64_t p = 0; p < n_pairs; ++p) {
      const uint32_t *rec = recs + (size_t)p * words;
      const float *adj = (const float *)rec;
      const int32_t *types = (const int32_t *)(rec + 2 * NN);
      const int32_t *nn = (const int32_t *)(rec + 2 * NN + 2 * n_max);
      const uint32_t pk = sg_mix((uint32_t)(pair_offset + p) ^ key);
      for (int s = 0; s < 2; ++s) {
        const int n = nn[s];
        const float *A = adj + s * NN;
        const int32_t *t = types + s * n_max;
        float *p1 = P1 + s * n_max * H1, *d1 = D1 + s * n_max * H1, *d2 = D2 + s * n_max * H2;
        for (int i = 0; i < n; ++i) m0[s * n_max + i] = keep_draw(pk, 0, s, i, thr) ? ik : 0.f;
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < H1; ++j) T[i * H1 + j] = m0[s * n_max + i] * P.W0[t[i] * H1 + j];
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < H1; ++j) {
            float a = 0.f;
            for (int k = 0; k < n; ++k) a += A[i * n_max + k] * T[k * H1 + j];
            a += P.b0[j];
            p1[i * H1 + j] = a;
            const float h = a > 0.f ? a : 0.f;
            d1[i * H1 + j] = keep_draw(pk, 1, s, i * H1 + j, thr) ? h * ik : 0.f;
          }
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < H2; ++j) {
            float a = 0.f;
            for (int k = 0; k < H1; ++k) a += d1[i * H1 + k] * P.W1[k * H2 + j];
            T[i * H2 + j] = a;
          }
        for (int i = 0; i < n; ++i) {
          float z = 0.f;
          for (int j = 0; j < H2; ++j) {
            float a = 0.f;
            for (int k = 0; k < n; ++k) a += A[i * n_max + k] * T[k * H2 + j];
            a += P.b1[j];
            const float v = keep_draw(pk, 2, s, i * H2 + j, thr) ? a * ik : 0.f;
            d2[i * H2 + j] = v;
            z += v * P.Wd[j];
          }
          zp[s * n_max + i] = z + P.bd[0];
        }
        for (int q = 0; q < D; ++q) {
          const float e = q < n ? (zp[s * n_max + q] > 0.f ? zp[s * n_max + q] : 0.f) : 0.f;
          x[s * D + q] = keep_draw(pk, 4, s, q, thr) ? e * ik : 0.f;
        }
      }
      /* NTN */
      float mk[KNT], rsum = 0.f, usum = 0.f;
      for (int a = 0; a < D; ++a)
        for (int k = 0; k < KNT; ++k) {
          float acc = 0.f;
          for (int b = 0; b < D; ++b) acc += P.W[(a * D + b) * KNT + k] * x[D + b];
          u[a * KNT + k] = acc;
        }
      for (int k = 0; k < KNT; ++k) {
        float acc = 0.f;
        for (int i = 0; i < 2 * D; ++i) acc += P.V[k * 2 * D + i] * x[i];
        for (int a = 0; a < D; ++a) acc += x[a] * u[a * KNT + k];
        mk[k] = acc + P.bn[k];
        rsum += mk[k] > 0.f ? mk[k] : 0.f;
        usum += P.U[k];
      }
      const float s = usum * rsum;
      if (s_out) s_out[p] = s;
      const float yh = expf(-yeta * s * s);
      const float gy = yh - ybar;
      lacc += 0.5 * (double)gy * gy;
      const float gs = gy * (-2.f * yeta * s * yh);
      float gm[KNT];
      for (int k = 0; k < KNT; ++k) {
        G.U[k] += gs * rsum;
        gm[k] = mk[k] > 0.f ? gs * usum : 0.f;
        G.bn[k] += gm[k];
        for (int i = 0; i < 2 * D; ++i) G.V[k * 2 * D + i] += gm[k] * x[i];
      }
      for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) {
          const float xy = x[a] * x[D + b];
          for (int k = 0; k < KNT; ++k) G.W[(a * D + b) * KNT + k] += gm[k] * xy;
        }
      for (int a = 0; a < D; ++a) {
        float acc = 0.f;
        for (int k = 0; k < KNT; ++k) acc += (P.V[k * 2 * D + a] + u[a * KNT + k]) * gm[k];
        gx[a] = acc;
      }
      for (int b = 0; b < D; ++b) {
        float acc = 0.f;
        for (int k = 0; k < KNT; ++k) {
          float w = 0.f;
          for (int a = 0; a < D; ++a) w += x[a] * P.W[(a * D + b) * KNT + k];
          acc += (P.V[k * 2 * D + D + b] + w) * gm[k];
        }
        gx[D + b] = acc;
      }
      for (int s = 0; s < 2; ++s) {
        const int n = nn[s];
        const float *A = adj + s * NN;
        const int32_t *t = types + s * n_max;
        const float *p1 = P1 + s * n_max * H1, *d1 = D1 + s * n_max * H1, *d2 = D2 + s * n_max * H2;
        for (int i = 0; i < n; ++i) {
          float ge = keep_draw(pk, 4, s, i, thr) ? gx[s * D + i] * ik : 0.f;
          const float gp = zp[s * n_max + i] > 0.f ? ge : 0.f;
          G.bd[0] += gp;
          for (int j = 0; j < H2; ++j) {
            G.Wd[j] += d2[i * H2 + j] * gp;
            gH2[i * H2 + j] = keep_draw(pk, 2, s, i * H2 + j, thr) ? gp * P.Wd[j] * ik : 0.f;
            G.b1[j] += gH2[i * H2 + j];
          }
        }
        for (int i = 0; i < n; ++i)       /* gZ1 = Âᵀ gH2 */
          for (int j = 0; j < H2; ++j) {
            float a = 0.f;
            for (int k = 0; k < n; ++k) a += A[k * n_max + i] * gH2[k * H2 + j];
            gZ[i * H2 + j] = a;
          }
        for (int i = 0; i < n; ++i)
          for (int k = 0; k < H1; ++k) {
            float gd = 0.f;
            for (int j = 0; j < H2; ++j) {
              G.W1[k * H2 + j] += d1[i * H1 + k] * gZ[i * H2 + j];
              gd += gZ[i * H2 + j] * P.W1[k * H2 + j];
            }
            const float gh = keep_draw(pk, 1, s, i * H1 + k, thr) ? gd * ik : 0.f;
            gP[i * H1 + k] = p1[i * H1 + k] > 0.f ? gh : 0.f;
            G.b0[k] += gP[i * H1 + k];
          }
        for (int i = 0; i < n; ++i) {     /* gZ0 = Âᵀ gP1 → rows of W0 */
          const float sc = m0[s * n_max + i];
          if (sc == 0.f) continue;
          for (int j = 0; j < H1; ++j) {
            float a = 0.f;
            for (int k = 0; k < n; ++k) a += A[k * n_max + i] * gP[k * H1 + j];
            G.W0[t[i] * H1 + j] += sc * a;
          }
        }
      }
    }
    lbuf[tid] = lacc;
    free(m0); free(P1); free(D1); free(T); free(D2); free(zp); free(x); free(u); free(gx);
    free(gH2); free(gZ); free(gP);
  }
  for (int64_t i = 0; i < np_; ++i) {
    double a = 0.0;
    for (int t = 0; t < nt; ++t) a += gbuf[(size_t)t * np_ + i];
    grad_out[i] = (float)a;
  }
  double l = 0.0;
  for (int t = 0; t < nt; ++t) l += lbuf[t];
  if (loss_out) *loss_out = l;
  free(gbuf);
  free(lbuf);
  return 0;
}
