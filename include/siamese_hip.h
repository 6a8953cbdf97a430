/*
 * siamese_hip.h — C-ABI of libsiamese_hip.so, the MI355X (gfx950) hot path of
 * the Siamese GCN → pooling → NTN → Gaussian-similarity → MSE model of
 * kangzf/GraphEmbedding (model/Siamese).
 *
 * The reference has no FFI: its hot path is the TensorFlow 1.x graph executed by
 * `sess.run` at model/Siamese/train.py:92, fed by
 * SiameseGCNTNMSE.get_feed_dict (model/Siamese/model_mse.py:52-94).  Each entry
 * point below replaces one piece of that `sess.run`, called from the host mirror
 * graphembedding_amd/model_mse.py via ctypes:
 *
 *   sg_pack_pairs    get_feed_dict's per-pair sparse-tuple feeds
 *                    (model_mse.py:65-81) → one packed pair record per pair.
 *   sg_forward       sess.run([model.pred_sim_without_act()])  (train.py:87,92;
 *                    models.py:90-91) — pre-activation score s per pair.
 *   sg_fwd_bwd       the forward + MSE loss + autodiff of
 *                    sess.run([opt_op, loss])  (train.py:85,92; models.py:34-36;
 *                    model_mse.py:145-151), gradient summed over the batch.
 *   sg_adam_tf       AdamOptimizer(lr).minimize's ApplyAdam update incl. the
 *                    weight-decay term of models.py:67-73.
 *   sg_label_stats   the label side of the B×B broadcast loss
 *                    (model_mse.py:148-151): mean label and ½Σ(y-ȳ)².
 *
 * Conventions: every pointer is a caller-owned DEVICE buffer unless noted;
 * every call is stream-ordered on `stream` (a hipStream_t, 0 = null stream),
 * performs no allocation and no host synchronisation, and returns SG_OK (0) or
 * an SG_ERR_* code.  Calls are thread-compatible (one stream per caller).
 */
#ifndef SIAMESE_HIP_H
#define SIAMESE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *sg_stream_t; /* hipStream_t */

enum sg_status {
  SG_OK = 0,
  SG_ERR_ARG = 1,          /* invalid argument / inconsistent model (reference: RuntimeError) */
  SG_ERR_UNSUPPORTED = 2,  /* valid reference model this build has no kernel for */
  SG_ERR_HIP = 3,          /* a HIP runtime call failed */
  SG_ERR_SHAPE = 4         /* e.g. Padding with N > max_in_dims (tf.pad error, layers.py:226) */
};

/* Layer kinds of the layer-string grammar (layers_factory.py:8-34). */
enum sg_layer_kind {
  SG_GCN = 1,       /* GraphConvolution   layers.py:52-118  */
  SG_DENSE = 2,     /* Dense              layers.py:163-205 */
  SG_PADDING = 3,   /* Padding            layers.py:208-227 */
  SG_AVERAGE = 4,   /* Average            layers.py:121-140 */
  SG_ATTENTION = 5, /* Attention          layers.py:143-160 (dead code in the reference; build option) */
  SG_NTN = 6,       /* NTN                layers.py:255-310 */
  SG_DOT = 7        /* Dot                layers.py:230-252 */
};

/* Activations (layers_factory.py:101-114). */
enum sg_act { SG_ACT_IDENTITY = 0, SG_ACT_RELU = 1, SG_ACT_SIGMOID = 2, SG_ACT_TANH = 3 };

/* Final activation (config.py:81-83 FLAGS.final_act with FLAGS.sim_kernel). */
enum sg_final {
  SG_FINAL_GAUSSIAN = 0, /* 'sim_kernel' with 'gaussian': exp(-yeta s^2) (similarity.py:58-60) */
  SG_FINAL_IDENTITY = 1, /* 'identity', or 'sim_kernel' with 'identity' */
  SG_FINAL_RELU = 2,
  SG_FINAL_SIGMOID = 3,
  SG_FINAL_TANH = 4
};

enum sg_loss_mode {
  SG_LOSS_BROADCAST = 0, /* reference quirk A2: l2_loss((B,1)-(B,))/B */
  SG_LOSS_ALIGNED = 1    /* per-pair MSE: ½Σ(y_i-ŷ_i)²/B */
};

enum sg_ntn_mode {
  SG_NTN_REFERENCE = 0, /* quirk A1: s = (ΣU)·Σ_k act(m_k)  (layers.py:305-308) */
  SG_NTN_INTENDED = 1   /* s = Σ_k U_k act(m_k) */
};

#define SG_MAX_LAYERS 8

/* Storage type of Â in the packed pair records (compute is fp32 either way). */
typedef enum sg_dtype {
  SG_DTYPE_F32 = 0,   /* 4 B per entry: the reference's float32 placeholders (A11) */
  SG_DTYPE_BF16 = 1   /* 2 B per entry, RNE from f32: config C3, 496 B/pair at n_max 10 */
} sg_dtype;

typedef struct sg_layer {
  int32_t kind;          /* sg_layer_kind */
  int32_t input_dim;     /* GCN/Dense/Attention/NTN input width (GCN layer 0: d_in) */
  int32_t output_dim;    /* GCN/Dense output; NTN feature_map_dim; Padding max_in_dims */
  int32_t act;           /* sg_act (GCN/Dense act, NTN inneract) */
  int32_t bias;          /* 0/1 */
  int32_t dropout;       /* 0/1: layer reads FLAGS.dropout (layers.py:45-49) */
  int32_t sparse_inputs; /* GCN: 1 for the one-hot feature layer */
  float padding_value;   /* Padding */
} sg_layer_t;

typedef struct sg_model {
  int32_t num_layers;
  int32_t d_in;       /* one-hot width = NodeFeatureOneHotEncoder.input_dim() */
  int32_t n_max;      /* node capacity of one graph slot of a pair record */
  int32_t final_act;  /* sg_final */
  int32_t loss_mode;  /* sg_loss_mode */
  int32_t ntn_mode;   /* sg_ntn_mode */
  float keep_prob;    /* 1 - FLAGS.dropout */
  float yeta;         /* FLAGS.yeta */
  sg_layer_t layers[SG_MAX_LAYERS];
  int32_t adj_dtype;  /* sg_dtype of Â in the records passed to sg_forward / sg_fwd_bwd */
} sg_model_t;

/*
 * Packed pair record (fp32), little-endian, 16-byte aligned, one per pair:
 *   float   adj[2][n_max][n_max];   Â of graph 1 / graph 2, rows/cols >= n zero
 *   int32_t types[2][n_max];        one-hot column of each node (graphs.py:108-111)
 *   int32_t n_nodes[2];
 *   float   label;                  y = sim_kernel(norm_dist) of the pair (aligned loss)
 *   int32_t tag;                    free (host bookkeeping: source pair index)
 * sg_record_bytes(10) == 896.
 */
int64_t sg_record_bytes(int32_t n_max);

/*
 * Record with Â stored as adj_dtype.  SG_DTYPE_BF16 layout:
 *   uint16_t adj[2][n_max][n_max] (bf16, RNE of the f32 Â; 2·n_max² entries in
 *            n_max² words), then types, n_nodes, label, tag as above, the record
 *            padded to a multiple of 16 B.  sg_record_bytes_ex(10, BF16) == 496.
 * The kernels widen Â to f32 while staging a record into LDS.
 */
int64_t sg_record_bytes_ex(int32_t n_max, int32_t adj_dtype);

/* Library version (major*10000 + minor*100 + patch). */
int32_t sg_version(void);

/*
 * Validate a model against the reference grammar and this build's kernels.
 * n_params_out: length of the flat fp32 parameter vector (variables in layer
 * order: GCN weights_0,bias; Dense weights,bias; Attention weights;
 * NTN weights_W[D][D][K], weights_V[K][2D], weights_U[K][1], bias[K]).
 * path_out: 1 = fused MFMA path (default stack, n_max = Padding dim <= 12),
 * 2 = fused capacity-32 MFMA path (default stack, n_max = 32, Padding dim in
 * (12, 31]: config C4), 3 = graph-store path (default stack, Padding dim in
 * [32, 512]: config C5, sg_web_* entry points), 0 = generic path.  Host-only, no GPU.
 * The capacity-32 path needs sg_workspace_bytes(model, n_pairs) of workspace,
 * which includes 320 B per pair for the NTN weight-gradient operands.
 */
int32_t sg_model_validate(const sg_model_t *model, int64_t *n_params_out, int32_t *path_out);

/* Workspace bytes needed by sg_forward / sg_fwd_bwd / sg_label_stats for n_pairs. */
int64_t sg_workspace_bytes(const sg_model_t *model, int64_t n_pairs);

/*
 * Gather pair records from a device graph store.
 *   store_adj   [n_graphs][n_max][n_max] f32, store_types [n_graphs][n_max] i32,
 *   store_n     [n_graphs] i32, pair_idx [n_pairs][2] i32 (graph ids),
 *   labels      [n_pairs] f32 or NULL (label := 0), records out.
 * Invalid graph ids give SG_ERR_ARG in *status_out (device int, may be NULL).
 */
int32_t sg_pack_pairs(const float *store_adj, const int32_t *store_types, const int32_t *store_n,
                      int32_t n_graphs, int32_t n_max, const int32_t *pair_idx,
                      const float *labels, int64_t n_pairs, void *records,
                      int32_t *status_out, sg_stream_t stream);

/* sg_pack_pairs writing records with Â stored as adj_dtype (sg_dtype). */
int32_t sg_pack_pairs_ex(const float *store_adj, const int32_t *store_types,
                         const int32_t *store_n, int32_t n_graphs, int32_t n_max,
                         int32_t adj_dtype, const int32_t *pair_idx, const float *labels,
                         int64_t n_pairs, void *records, int32_t *status_out,
                         sg_stream_t stream);

/* stats_out[0] = mean label ȳ, stats_out[1] = ½Σ(y-ȳ)² over the n_pairs records. */
int32_t sg_label_stats(const void *records, int64_t n_pairs, int32_t n_max, float *stats_out,
                       void *workspace, sg_stream_t stream);

/* sg_label_stats over records with Â stored as adj_dtype. */
int32_t sg_label_stats_ex(const void *records, int64_t n_pairs, int32_t n_max, int32_t adj_dtype,
                          float *stats_out, void *workspace, sg_stream_t stream);

/*
 * Forward only: s_out[i] = pre-activation score of record i (the test path:
 * pred_sim_without_act, train.py:87).  Dropout masks are keyed by
 * (seed, pair_offset + i) so a sharded batch reproduces the unsharded one.
 */
int32_t sg_forward(const sg_model_t *model, const void *records, int64_t n_pairs,
                   int64_t pair_offset, const float *params, uint64_t seed, float *s_out,
                   void *workspace, sg_stream_t stream);

/*
 * Forward + loss + backward over n_pairs records.
 *   y_stats     device [2] = {ȳ, ½Σ(y-ȳ)²} of the WHOLE batch (broadcast loss);
 *               ignored in aligned mode.
 *   batch_total global batch size B (aligned loss divides by it).
 *   grad_out    [n_params] Σ_pairs ∂loss_mse/∂θ (no weight decay; that is added
 *               by sg_adam_tf so that a multi-GPU all-reduce sums it once).
 *   loss_out    [1] this shard's loss_mse contribution: ½Σ_j(ŷ_j-ȳ)² (+ ½Σ(y-ȳ)²
 *               when add_label_term != 0) in broadcast mode, ½Σ(y-ŷ)²/B aligned.
 *   s_out       [n_pairs] or NULL.
 */
int32_t sg_fwd_bwd(const sg_model_t *model, const void *records, int64_t n_pairs,
                   int64_t pair_offset, int64_t batch_total, const float *params, uint64_t seed,
                   const float *y_stats, int32_t add_label_term, float *s_out, float *grad_out,
                   float *loss_out, void *workspace, sg_stream_t stream);

/*
 * Processing order (library 1.2).  The per-pair cost of the kernels depends on
 * the pair's node counts; records in batch order hand every wavefront a random
 * mix, so the launch waits for the unluckiest one.  sg_pair_order writes a
 * permutation of [0, n_pairs) that sorts the records by cost class (stable, so
 * deterministic); sg_forward_ex / sg_fwd_bwd_ex walk it so that every wavefront
 * gets the same mix.  Results are those of the unordered call up to the
 * summation order of the gradient: record i still keys its dropout masks by
 * pair_offset + i and writes s_out[i].  Compute the order once per packed
 * batch and reuse it for every step.  order == NULL is batch order.
 * Entries outside [0, n_pairs) are clamped (never read out of bounds), but
 * only a permutation gives the batch's result.
 */
int64_t sg_pair_order_workspace_bytes(const sg_model_t *model, int64_t n_pairs);
int32_t sg_pair_order(const sg_model_t *model, const void *records, int64_t n_pairs,
                      int32_t *order_out, void *workspace, sg_stream_t stream);
int32_t sg_forward_ex(const sg_model_t *model, const void *records, const int32_t *order,
                      int64_t n_pairs, int64_t pair_offset, const float *params, uint64_t seed,
                      float *s_out, void *workspace, sg_stream_t stream);
int32_t sg_fwd_bwd_ex(const sg_model_t *model, const void *records, const int32_t *order,
                      int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                      const float *params, uint64_t seed, const float *y_stats,
                      int32_t add_label_term, float *s_out, float *grad_out, float *loss_out,
                      void *workspace, sg_stream_t stream);

/*
 * Class-exclusive schedule (library 1.7; fused path, sg_model_validate path 1 only,
 * else SG_ERR_UNSUPPORTED).  sg_pair_order_cls writes the order of sg_pair_order and
 * class_start[0 .. SG_FAST_CLASSES_P1): the order's slots [class_start[c],
 * class_start[c + 1]) hold the records of cost class c = (N0 > 8) + 2 (N1 > 8),
 * class_start[4] = n_pairs.  sg_forward_cls / sg_fwd_bwd_cls then give every
 * wavefront the slots of ONE class, so it runs one specialised pair body for the whole
 * launch (no register copies where the four class bodies would join); the classes
 * get wavefronts in proportion to their work.  Results equal sg_*_ex on the same
 * order: scores bitwise, the gradient up to summation order.  class_start must come
 * from sg_pair_order_cls on the same records and order (a wrong table drops nodes).
 */
#define SG_FAST_CLASSES_P1 5
int32_t sg_pair_order_cls(const sg_model_t *model, const void *records, int64_t n_pairs,
                          int32_t *order_out, int32_t *class_start, void *workspace,
                          sg_stream_t stream);
int32_t sg_forward_cls(const sg_model_t *model, const void *records, const int32_t *order,
                       const int32_t *class_start, int64_t n_pairs, int64_t pair_offset,
                       const float *params, uint64_t seed, float *s_out, void *workspace,
                       sg_stream_t stream);
int32_t sg_fwd_bwd_cls(const sg_model_t *model, const void *records, const int32_t *order,
                       const int32_t *class_start, int64_t n_pairs, int64_t pair_offset,
                       int64_t batch_total, const float *params, uint64_t seed,
                       const float *y_stats, int32_t add_label_term, float *s_out,
                       float *grad_out, float *loss_out, void *workspace, sg_stream_t stream);

/*
 * Graph-captured training steps (library 1.5).  sg_fwd_bwd_ex with the dropout seed
 * read from device memory at kernel time, so one hipGraph capture of a step
 * (feed → fwd_bwd → Adam → sg_seed_advance) replays with a new seed each time: the
 * reference's train loop (train.py:8-44, B = 5 pairs per sess.run) is launch-bound.
 * Fused path (sg_model_validate path 1) only; other models give SG_ERR_UNSUPPORTED.
 * sg_seed_advance adds delta to *seed_dev on the stream.
 */
int32_t sg_fwd_bwd_dseed(const sg_model_t *model, const void *records, const int32_t *order,
                         int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                         const float *params, const uint64_t *seed_dev, const float *y_stats,
                         int32_t add_label_term, float *s_out, float *grad_out, float *loss_out,
                         void *workspace, sg_stream_t stream);
int32_t sg_seed_advance(uint64_t *seed_dev, uint64_t delta, sg_stream_t stream);

/*
 * Device-side pair samplers (library 1.4; samplers.py:19-68).  The reference's
 * samplers draw only from fresh random.Random(seed) generators with known seeds,
 * so the host builds their tables once with CPython's `random`; these calls then
 * advance the sampler state in device memory and write `count` pairs of store
 * ids to pairs_out [count][2], exactly the reference's get_pair() stream.
 *   sg_sampler_random (RandomSampler): state [1 + 2n] = idx | current list | scratch,
 *     sigma [n] = random.Random(123).shuffle(list(range(n))) (applied on each wrap).
 *   sg_sampler_density (DistributionSampler): state [2] = cur | item_idx,
 *     dens_order [n] (store ids sorted by (density, idx)), bins [n_bins] (shuffled
 *     bin ids, truncated to 2 * sample_num), item_table [ceil(n_bins / 2)]:
 *     entry c / 2 = random.Random(123 + c).randint(0, bin_size - 1).
 */
int32_t sg_sampler_random(int32_t *state, const int32_t *sigma, int32_t n, int64_t count,
                          int32_t *pairs_out, sg_stream_t stream);
int32_t sg_sampler_density(int32_t *state, const int32_t *dens_order, const int32_t *bins,
                           int32_t n_bins, int32_t bin_size, const int32_t *item_table,
                           int64_t count, int32_t *pairs_out, sg_stream_t stream);

/*
 * One step's get_feed_dict (model_mse.py:52-94) in one launch (library 1.5): the
 * sampler calls (B + B² in compat mode, quirk A3; else B), the labels
 * label_matrix[g1][g2] of the input pairs (compat: of the last B calls), the label
 * statistics {ȳ, ½Σ(y-ȳ)²} (double accumulation, in order) and the B input records
 * packed from the dense-slot store.  sg_feed_t is a host struct of device pointers.
 * pairs_out holds count × 2 ids; status_out (may be NULL) gets SG_ERR_ARG for ids
 * outside the store.
 */
typedef struct sg_feed {
  int32_t kind;                 /* 0 RandomSampler (sigma, n), 1 DistributionSampler */
  int32_t *state;               /* as sg_sampler_random / sg_sampler_density */
  const int32_t *sigma;
  int32_t n;
  const int32_t *dens_order, *bins, *item_table;
  int32_t n_bins, bin_size;
  int32_t batch;                /* B */
  int32_t compat;               /* 1: label stream of quirk A3 */
  const float *label_matrix;    /* [label_n][label_n], indexed by store id */
  int32_t label_n;
  const float *store_adj;       /* dense-slot graph store (sg_pack_pairs) */
  const int32_t *store_types, *store_n;
  int32_t n_graphs, n_max, adj_dtype;
} sg_feed_t;
int32_t sg_feed_step(const sg_feed_t *feed, int32_t *pairs_out, void *records, float *labels_out,
                     float *y_stats_out, int32_t *status_out, sg_stream_t stream);

/*
 * Graph-store path for Web-sized graphs (library 1.5; BASELINE config C5).
 *
 * Pair records hold Â densely (n_max² per side), which stops scaling at a few
 * dozen nodes.  For models that sg_model_validate reports as path 3 (the
 * default stack GCN(d_in→32, relu) → GCN(32→16) → Dense(16→1, relu) →
 * Padding(D) → NTN(D, K) with D in [32, 512]) the kernels instead read the
 * graphs from a device CSR store and a list of pair ids, and the NTN bilinear
 * term e1ᵀ W[:,:,k] e2 (layers.py:295-298) and its gradients run as batched
 * MFMA GEMMs over the pairs.  Same math, dropout keys and loss conventions as
 * sg_forward / sg_fwd_bwd: pair i of the list keys its masks by pair_offset + i.
 *
 * sg_csr_store_t is a HOST struct holding DEVICE pointers:
 *   node_off [n_graphs + 1]  first node of graph g in the node arrays
 *   types    [n_nodes]       one-hot column of each node (graphs.py:108-111)
 *   row_ptr  [n_nodes + 1]   CSR row offsets of Â (graphs.py:64-76) into col/val
 *   col      [nnz]           neighbour as a node index LOCAL to its graph
 *   val      [nnz]           Â entry (f32 cast of the reference's float64, A11)
 *   max_nnz                  largest Â entry count of one graph (LDS staging size)
 * Â must be symmetric (undirected graphs, as the reference's).  Every graph
 * must have 1 <= n <= n_max <= D nodes (tf.pad, quirk A9), checked by the host.
 */
typedef struct sg_csr_store {
  int32_t n_graphs;
  int32_t n_max;
  const int32_t *node_off;
  const int32_t *types;
  const int32_t *row_ptr;
  const int32_t *col;
  const float *val;
  int32_t max_nnz;
} sg_csr_store_t;

/* Workspace bytes for sg_web_forward / sg_web_fwd_bwd processing chunks of up
 * to `chunk` pairs (any n_pairs is processed chunk by chunk).  chunk must be >= 1: a call
 * with chunk <= 0 runs one chunk of n_pairs, sized by sg_web_workspace_bytes_ex; -1 here. */
int64_t sg_web_workspace_bytes(const sg_model_t *model, int64_t chunk);

/* Workspace bytes for sg_web_forward / sg_web_fwd_bwd calls of at most n_pairs pairs in
 * chunks of `chunk` (library 1.8; chunk 0 = one chunk of n_pairs, as the calls read it).  A call of several chunks pipelines them over two
 * workspace slots (the NTN inputs, dropout keep bits and D2 rows of one chunk each, which
 * grow with chunk x node capacity); when n_pairs <= chunk there is one chunk and one slot,
 * about half of sg_web_workspace_bytes.  A workspace sized for n_pairs serves calls of up
 * to n_pairs pairs. */
int64_t sg_web_workspace_bytes_ex(const sg_model_t *model, int64_t chunk, int64_t n_pairs);

/* Destroys the auxiliary streams and events of the sg_web_* chunk pipeline (one set per
 * device and caller stream, created on first use), after waiting for their work: call at
 * teardown, when no sg_web_* call is in flight (library 1.8).  Returns SG_OK or SG_ERR_HIP. */
int32_t sg_web_release(void);

/* Pre-activation scores of the pairs pair_idx [n_pairs][2] (store graph ids);
 * replaces sess.run([pred_sim_without_act()]) like sg_forward. */
int32_t sg_web_forward(const sg_model_t *model, const sg_csr_store_t *store,
                       const int32_t *pair_idx, int64_t n_pairs, int64_t pair_offset,
                       const float *params, uint64_t seed, float *s_out, void *workspace,
                       int64_t chunk, sg_stream_t stream);

/* Forward + loss + backward over the pairs, as sg_fwd_bwd (same y_stats,
 * batch_total, add_label_term, grad_out and loss_out conventions).  labels
 * [n_pairs] are read in aligned loss mode only (may be NULL in broadcast mode). */
int32_t sg_web_fwd_bwd(const sg_model_t *model, const sg_csr_store_t *store,
                       const int32_t *pair_idx, const float *labels, int64_t n_pairs,
                       int64_t pair_offset, int64_t batch_total, const float *params,
                       uint64_t seed, const float *y_stats, int32_t add_label_term, float *s_out,
                       float *grad_out, float *loss_out, void *workspace, int64_t chunk,
                       sg_stream_t stream);

/*
 * TF ApplyAdam (training_ops ApplyAdam, non-Nesterov) with the weight-decay
 * gradient wd·θ added first (models.py:69-73):
 *   g = grad + wd·θ; α = lr·√(1-β2^t)/(1-β1^t); m += (g-m)(1-β1);
 *   v += (g²-v)(1-β2); θ -= α·m/(√v+ε); then β1^t *= β1, β2^t *= β2.
 * beta_powers: device [2] {β1^t, β2^t}, initialised by the caller to {β1, β2}.
 * reg_loss_out: device [1] or NULL: wd·½Σθ² of the parameters BEFORE the update.
 */
int32_t sg_adam_tf(float *params, float *m, float *v, const float *grad, int64_t n, float lr,
                   float beta1, float beta2, float eps, float weight_decay, float *beta_powers,
                   float *reg_loss_out, sg_stream_t stream);

/*
 * sg_adam_tf over many blocks (library 1.5), for large parameter vectors (config
 * C5's NTN has D²K weights): same update and outputs; workspace holds
 * sg_adam_workspace_bytes(n) bytes of per-block Σθ² partials.  n <= 65536 or a NULL
 * workspace runs sg_adam_tf.
 */
int64_t sg_adam_workspace_bytes(int64_t n);
int32_t sg_adam_tf_ex(float *params, float *m, float *v, const float *grad, int64_t n, float lr,
                      float beta1, float beta2, float eps, float weight_decay, float *beta_powers,
                      float *reg_loss_out, void *workspace, sg_stream_t stream);

/*
 * One training step (library 1.9): sg_fwd_bwd_cls (or sg_fwd_bwd_ex when class_start is
 * NULL; order may then be NULL too) followed by sg_adam_tf on its gradient, i.e.
 * sess.run([opt_op, loss]) (train.py:85,92) for one process.  On the fused path
 * (sg_model_validate path 1) the gradient reduction applies the update in the same
 * launch; other paths run the two calls.  params, grad_out, loss_out, m, v and
 * beta_powers end as after sg_fwd_bwd_cls + sg_adam_tf, bitwise; reg_loss_out holds the
 * same wd·½Σθ² summed in another order (double partials).  A multi-GPU step, whose
 * gradient is all-reduced between the two, keeps the separate calls.  Models of more than
 * 65,536 parameters return SG_ERR_UNSUPPORTED (call sg_fwd_bwd_* + sg_adam_tf_ex).
 * Replaces the train op of models.py:28-36 (AdamOptimizer(lr).minimize(loss)).
 */
typedef struct sg_adam_args {
  float *m, *v;            /* device [n_params] moments */
  float lr, beta1, beta2, eps, weight_decay;
  float *beta_powers;      /* device [2] {β1^t, β2^t} (sg_adam_tf) */
  float *reg_loss_out;     /* device [1] or NULL */
} sg_adam_args_t;
int32_t sg_train_step(const sg_model_t *model, const void *records, const int32_t *order,
                      const int32_t *class_start, int64_t n_pairs, int64_t pair_offset,
                      int64_t batch_total, float *params, uint64_t seed, const float *y_stats,
                      int32_t add_label_term, float *s_out, float *grad_out, float *loss_out,
                      void *workspace, const sg_adam_args_t *adam, sg_stream_t stream);
/* The same with the dropout seed read from device memory (sg_fwd_bwd_dseed): one
 * hipGraph-captured reference step is feed → sg_train_step_dseed → sg_seed_advance. */
int32_t sg_train_step_dseed(const sg_model_t *model, const void *records, const int32_t *order,
                            int64_t n_pairs, int64_t pair_offset, int64_t batch_total,
                            float *params, const uint64_t *seed_dev, const float *y_stats,
                            int32_t add_label_term, float *s_out, float *grad_out,
                            float *loss_out, void *workspace, const sg_adam_args_t *adam,
                            sg_stream_t stream);

/*
 * Pairs straight from the dense graph store (library 1.6).  sg_pack_pairs writes a
 * record per pair that the fused kernel then reads back: for a stream that does not
 * fit HBM at once (config C4, AIDS10knef all-pairs: 100.4 M pairs, 850 GB of
 * records) that round trip is a quarter of the step.  These calls take the
 * sg_pack_pairs inputs instead and the kernel gathers each pair's two graphs from
 * the store itself (41 MB at C4: cache-resident).  Same pair ids, labels, dropout
 * keys, order and results as packing + sg_fwd_bwd_ex bit for bit.
 *
 * sg_pair_source_t is a HOST struct holding DEVICE pointers:
 *   adj [n_graphs][n_max][n_max] f32, types [n_graphs][n_max] i32, n [n_graphs] i32
 *       (the sg_pack_pairs store);
 *   pair_idx  [n_pairs][2] i32 graph ids, or NULL: the all-pairs grid, pair i =
 *             (q / n_graphs, q % n_graphs) with q = grid_base + i (row-major);
 *   labels    [n_pairs] f32 or NULL (label := 0);
 *   status    device int or NULL: invalid graph ids set SG_ERR_ARG and read as a
 *             zero record, as in sg_pack_pairs.
 * Fused paths (sg_model_validate paths 1 and 2) with f32 Â only; other models give
 * SG_ERR_UNSUPPORTED.  Workspace sizes are sg_workspace_bytes /
 * sg_pair_order_workspace_bytes.
 */
typedef struct sg_pair_source {
  const float *adj;
  const int32_t *types;
  const int32_t *n;
  int32_t n_graphs;
  int32_t n_max;
  const int32_t *pair_idx;
  int64_t grid_base;
  const float *labels;
  int32_t *status;
} sg_pair_source_t;

int32_t sg_pair_order_src(const sg_model_t *model, const sg_pair_source_t *src,
                          int64_t n_pairs, int32_t *order_out, void *workspace,
                          sg_stream_t stream);
int32_t sg_forward_src(const sg_model_t *model, const sg_pair_source_t *src,
                       const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                       const float *params, uint64_t seed, float *s_out, void *workspace,
                       sg_stream_t stream);
int32_t sg_fwd_bwd_src(const sg_model_t *model, const sg_pair_source_t *src,
                       const int32_t *order, int64_t n_pairs, int64_t pair_offset,
                       int64_t batch_total, const float *params, uint64_t seed,
                       const float *y_stats, int32_t add_label_term, float *s_out,
                       float *grad_out, float *loss_out, void *workspace, sg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SIAMESE_HIP_H */
