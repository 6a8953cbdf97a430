// sg_plan.h — host-side validation of a reference layer stack and the
// per-wave LDS plan of the generic kernel.  Validation mirrors the shape
// rules TF enforced implicitly (layers.py / layers_factory.py) and the
// restrictions of the Siamese model (model_mse.py:104-129: the first layer is
// the sparse-feature GCN; Dot/NTN pair ins[i] with ins[i+B]).
#pragma once
#include <string.h>

#include "sg_common.h"

struct SgGenLayer {
  int kind, act, bias, li;     // li = index in model.layers (dropout RNG layer id)
  int sparse;
  int din, dout;
  int rin_fixed;               // rows entering: -1 = graph nodes n, else fixed (P or 1)
  int rout_fixed;              // rows leaving
  int Rin, Rout;               // row capacities of the LDS tensors
  uint32_t thr;                // dropout keep threshold (65536 = no dropout)
  float inv_keep;
  float padv;
  int offW, offB;              // flat param offsets (-1 = none)
  int l_in;                    // LDS offset of the input tensor (-1: sparse one-hot X)
  int l_xd, l_pre, l_out;      // dropped input / pre-activation / output
  int l_temp, l_hv, l_att, l_gz, l_gu, l_gt;  // Attention scratch
};

struct SgGenPlan {
  int nl;                      // node-level layers before the head
  SgGenLayer L[SG_MAX_LAYERS];
  int head_kind, head_li, head_act, head_bias;
  int D, K;                    // NTN input_dim / feature_map_dim (Dot: D = flattened size)
  uint32_t head_thr;
  float head_inv_keep;
  int offW, offV, offU, offB;  // NTN params
  int head_in_rows;            // rows of the pooled tensor (Rout of the last node layer)
  int head_in_d;
  int l_rec, l_x12, l_u, l_m, l_gm, l_tmp, l_tmp2, l_g0, l_g1;
  int wave_floats;             // per-wave LDS floats
  int n_params;
  int n_max, rec_words, rec_types, rec_nnodes, rec_label;   // LDS (f32) record layout
  int adj_dtype, hbm_words, hbm_adj_words;                  // HBM record (sg_dtype of Â)
  int d_in;
  int final_act, loss_mode, ntn_mode;
  float yeta;
};

// Returns SG_OK and fills *plan, or an SG_ERR_* code.
static int sg_build_plan(const sg_model_t *m, SgGenPlan *P) {
  if (!m || !P) return SG_ERR_ARG;
  memset(P, 0, sizeof(*P));
  const int nlay = m->num_layers;
  if (nlay < 2 || nlay > SG_MAX_LAYERS) return SG_ERR_ARG;  // check_flags: num_layers >= 2
  if (m->d_in <= 0 || m->n_max <= 0 || m->n_max > 64) return SG_ERR_ARG;
  if (!(m->keep_prob > 0.f && m->keep_prob <= 1.f)) return SG_ERR_ARG;
  if (m->final_act < SG_FINAL_GAUSSIAN || m->final_act > SG_FINAL_TANH) return SG_ERR_ARG;
  if (m->loss_mode != SG_LOSS_BROADCAST && m->loss_mode != SG_LOSS_ALIGNED) return SG_ERR_ARG;
  if (m->ntn_mode != SG_NTN_REFERENCE && m->ntn_mode != SG_NTN_INTENDED) return SG_ERR_ARG;
  if (!sg_dtype_ok(m->adj_dtype)) return SG_ERR_ARG;
  const int nmax = m->n_max;
  const SgRecLayout rl = sg_rec_layout(nmax);
  const SgRecLayout rh = sg_rec_layout(nmax, m->adj_dtype);
  P->n_max = nmax;
  P->adj_dtype = m->adj_dtype;
  P->hbm_words = rh.words;
  P->hbm_adj_words = rh.adj_words;
  P->rec_words = rl.words;
  P->rec_types = rl.types;
  P->rec_nnodes = rl.nnodes;
  P->rec_label = rl.label;
  P->d_in = m->d_in;
  P->final_act = m->final_act;
  P->loss_mode = m->loss_mode;
  P->ntn_mode = m->ntn_mode;
  P->yeta = m->yeta;

  int off = 0;                 // param offset
  int lds = 0;                 // per-wave LDS floats
  auto alloc = [&](int n) { int o = lds; lds += (n + 3) & ~3; return o; };
  P->l_rec = alloc(rl.words);

  int width = -1;              // current feature width (-1: one-hot X)
  int rows_fixed = -1;         // -1 = n graph rows
  int R = nmax;                // row capacity
  bool pooled = false;
  int cur_out = -1;            // LDS offset of the current tensor
  int max_tensor = 2 * nmax * 1;
  int head = -1;
  for (int li = 0; li < nlay; ++li) {
    const sg_layer_t &L = m->layers[li];
    const float keep = L.dropout ? m->keep_prob : 1.f;
    if (L.kind == SG_NTN || L.kind == SG_DOT) {
      if (li != nlay - 1) return SG_ERR_UNSUPPORTED;  // head must be last
      head = li;
      break;
    }
    if (P->nl >= SG_MAX_LAYERS) return SG_ERR_ARG;
    SgGenLayer &G = P->L[P->nl];
    G.kind = L.kind;
    G.act = L.act;
    G.bias = L.bias ? 1 : 0;
    G.li = li;
    G.sparse = L.sparse_inputs ? 1 : 0;
    G.thr = sg_keep_threshold(keep);
    G.inv_keep = 1.f / keep;
    G.padv = L.padding_value;
    G.offW = G.offB = -1;
    G.l_in = cur_out;
    G.l_xd = G.l_pre = G.l_out = G.l_temp = G.l_hv = G.l_att = G.l_gz = G.l_gu = G.l_gt = -1;
    G.rin_fixed = rows_fixed;
    G.Rin = R;
    if (L.act < SG_ACT_IDENTITY || L.act > SG_ACT_TANH) return SG_ERR_ARG;
    switch (L.kind) {
      case SG_GCN: {
        if (pooled) return SG_ERR_UNSUPPORTED;  // Â·x needs the graph's own rows
        if (li == 0) {
          if (!L.sparse_inputs) return SG_ERR_ARG;  // features are sparse placeholders
          const int din = L.input_dim > 0 ? L.input_dim : m->d_in;
          if (din != m->d_in) return SG_ERR_ARG;
          G.din = din;
        } else {
          if (L.sparse_inputs) return SG_ERR_ARG;
          if (L.input_dim != width) return SG_ERR_ARG;
          G.din = width;
        }
        if (L.output_dim <= 0 || L.output_dim > 256) return SG_ERR_ARG;
        G.dout = L.output_dim;
        G.offW = off; off += G.din * G.dout;
        if (G.bias) { G.offB = off; off += G.dout; }
        G.l_xd = G.sparse ? alloc(2 * nmax) : alloc(2 * R * G.din);
        G.l_pre = alloc(2 * R * G.dout);
        G.l_out = alloc(2 * R * G.dout);
        G.rout_fixed = rows_fixed;
        G.Rout = R;
        width = G.dout;
        break;
      }
      case SG_DENSE: {
        if (li == 0) return SG_ERR_ARG;
        if (L.input_dim != width || L.output_dim <= 0 || L.output_dim > 256) return SG_ERR_ARG;
        G.din = width;
        G.dout = L.output_dim;
        G.offW = off; off += G.din * G.dout;
        if (G.bias) { G.offB = off; off += G.dout; }
        G.l_xd = alloc(2 * R * G.din);
        G.l_pre = alloc(2 * R * G.dout);
        G.l_out = alloc(2 * R * G.dout);
        G.rout_fixed = rows_fixed;
        G.Rout = R;
        width = G.dout;
        break;
      }
      case SG_PADDING: {
        if (li == 0) return SG_ERR_ARG;
        const int Pr = L.output_dim;  // max_in_dims
        if (Pr <= 0 || Pr > 64) return SG_ERR_ARG;
        if (rows_fixed > Pr) return SG_ERR_SHAPE;
        G.din = G.dout = width;
        G.l_out = alloc(2 * Pr * width);
        rows_fixed = Pr;
        R = Pr;
        G.rout_fixed = Pr;
        G.Rout = Pr;
        pooled = true;
        break;
      }
      case SG_AVERAGE:
      case SG_ATTENTION: {
        if (li == 0) return SG_ERR_ARG;
        G.din = G.dout = width;
        if (L.kind == SG_ATTENTION) {
          if (L.input_dim != width) return SG_ERR_ARG;
          G.offW = off; off += width * width;
          G.l_temp = alloc(2 * width);
          G.l_hv = alloc(2 * width);
          G.l_att = alloc(2 * R);
          G.l_gz = alloc(2 * R);
          G.l_gu = alloc(2 * width);
          G.l_gt = alloc(2 * width);
        }
        G.l_out = alloc(2 * width);
        rows_fixed = 1;
        R = 1;
        G.rout_fixed = 1;
        G.Rout = 1;
        pooled = true;
        break;
      }
      default:
        return SG_ERR_ARG;
    }
    cur_out = G.l_out;
    int t = 2 * G.Rin * (G.din > 0 ? G.din : 1);
    if (t > max_tensor) max_tensor = t;
    t = 2 * G.Rout * G.dout;
    if (t > max_tensor) max_tensor = t;
    P->nl++;
  }
  if (head < 0 || P->nl == 0) return SG_ERR_ARG;
  if (!pooled) return SG_ERR_UNSUPPORTED;  // per-graph row count must be fixed before the head
  const sg_layer_t &H = m->layers[head];
  const SgGenLayer &last = P->L[P->nl - 1];
  P->head_kind = H.kind;
  P->head_li = head;
  P->head_in_rows = last.Rout;
  P->head_in_d = last.dout;
  const int flat = last.Rout * last.dout;
  if (H.kind == SG_NTN) {
    if (H.input_dim != flat) return SG_ERR_ARG;
    if (H.output_dim <= 0 || H.output_dim > 64) return SG_ERR_ARG;
    if (H.act < SG_ACT_IDENTITY || H.act > SG_ACT_TANH) return SG_ERR_ARG;
    P->D = flat;
    P->K = H.output_dim;
    P->head_act = H.act;
    P->head_bias = H.bias ? 1 : 0;
    const float keep = H.dropout ? m->keep_prob : 1.f;
    P->head_thr = sg_keep_threshold(keep);
    P->head_inv_keep = 1.f / keep;
    P->offW = off; off += P->D * P->D * P->K;
    P->offV = off; off += P->K * 2 * P->D;
    P->offU = off; off += P->K;
    P->offB = -1;
    if (P->head_bias) { P->offB = off; off += P->K; }
    P->l_x12 = alloc(2 * P->D);
    P->l_u = alloc(P->D * P->K);
    P->l_m = alloc(P->K);
    P->l_gm = alloc(P->K);
  } else {
    P->D = flat;
    P->K = 0;
    P->head_thr = 65536u;
    P->head_inv_keep = 1.f;
    P->offW = P->offV = P->offU = P->offB = -1;
  }
  if (2 * P->D > max_tensor) max_tensor = 2 * P->D;
  P->l_tmp = alloc(max_tensor);
  P->l_tmp2 = alloc(max_tensor);
  P->l_g0 = alloc(max_tensor);
  P->l_g1 = alloc(max_tensor);
  P->wave_floats = lds;
  P->n_params = off;
  return SG_OK;
}
