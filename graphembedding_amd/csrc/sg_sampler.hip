// sg_sampler.hip — device-side pair samplers (model/Siamese/samplers.py:19-68).
//
// Every random draw of the reference's samplers comes from a FRESH generator with a
// known seed: RandomSampler re-shuffles its list with random.Random(123) on every
// wrap (samplers.py:28), i.e. applies the same permutation σ each time;
// DistributionSampler walks bins shuffled by random.Random(123) and takes its item
// index from random.Random(123 + cur).randint(0, bin_size - 1) (samplers.py:51-68).
// So the host builds σ, the density order, the bin order and the per-cur item table
// once with CPython's own `random` (graphembedding_amd/device_sampler.py), and these
// kernels advance the sampler state and emit the pair-id stream on the device, so a
// training step needs no host work.  Streams equal the reference's bit for bit
// (tests/test_gpu_sampler.py replays the golden F2 streams).
#include "sg_plan.h"

namespace {

// state: [0] = idx, [1, 1 + n) = the list (store ids), [1 + n, 1 + 2n) = scratch
__global__ void __launch_bounds__(1024) sg_sampler_random_kernel(int32_t *__restrict__ st,
                                                                const int32_t *__restrict__ sigma,
                                                                int n, int64_t count,
                                                                int32_t *__restrict__ out) {
  int32_t *L = st + 1, *tmp = st + 1 + n;
  const int t = threadIdx.x;
  int idx = st[0];
  if (idx < 0 || idx >= n) idx = 0;
  for (int64_t c = 0; c < count; ++c) {
    const int g1 = L[idx];
    ++idx;
    if (idx >= n) {   // random.Random(123).shuffle(self.gs): L <- L ∘ σ
      __syncthreads();
      for (int i = t; i < n; i += blockDim.x) tmp[i] = L[sigma[i]];
      __syncthreads();
      for (int i = t; i < n; i += blockDim.x) L[i] = tmp[i];
      __syncthreads();
      idx = 0;
    }
    if (t == 0) {
      out[2 * c] = g1;
      out[2 * c + 1] = L[idx];
    }
  }
  __syncthreads();
  if (t == 0) st[0] = idx;
}

// state: [0] = cur, [1] = item_idx
__global__ void sg_sampler_density_kernel(int32_t *__restrict__ st,
                                          const int32_t *__restrict__ dens_order,
                                          const int32_t *__restrict__ bins, int n_bins,
                                          int bin_size, const int32_t *__restrict__ item_table,
                                          int64_t count, int32_t *__restrict__ out) {
  if (threadIdx.x != 0) return;
  int cur = st[0], item = st[1];
  for (int64_t c = 0; c < count; ++c) {
    out[2 * c] = dens_order[bins[cur] * bin_size + item];
    out[2 * c + 1] = dens_order[bins[cur + 1] * bin_size + item];
    cur += 2;
    if (cur >= n_bins - 1) cur = 0;
    item = item_table[cur >> 1];   // random.Random(123 + cur).randint(0, bin_size - 1)
  }
  st[0] = cur;
  st[1] = item;
}

// One training step's feed (get_feed_dict, model_mse.py:52-94) in one launch: the
// sampler calls of the step, the label gather from the device label matrix, the label
// statistics of the broadcast loss, and the packing of the B input pairs.
__global__ void __launch_bounds__(1024) sg_feed_kernel(sg_feed_t F, int32_t *__restrict__ pairs,
                                                      uint32_t *__restrict__ recs, int rec_words,
                                                      float *__restrict__ labels,
                                                      float *__restrict__ y_stats,
                                                      int32_t *__restrict__ status) {
  const int t = threadIdx.x;
  const int B = F.batch;
  // B + B² sampler calls in 'compat' mode: int64 (B >= 46,341 would overflow int)
  const int64_t count = F.compat ? (int64_t)B + (int64_t)B * B : (int64_t)B;
  if (F.kind == 0) {   // RandomSampler (samplers.py:24-31)
    int32_t *st = F.state, *L = st + 1, *tmp = st + 1 + F.n;
    int idx = st[0];
    if (idx < 0 || idx >= F.n) idx = 0;
    for (int64_t c = 0; c < count; ++c) {
      const int g1 = L[idx];
      ++idx;
      if (idx >= F.n) {
        __syncthreads();
        for (int i = t; i < F.n; i += blockDim.x) tmp[i] = L[F.sigma[i]];
        __syncthreads();
        for (int i = t; i < F.n; i += blockDim.x) L[i] = tmp[i];
        __syncthreads();
        idx = 0;
      }
      if (t == 0) {
        pairs[2 * c] = g1;
        pairs[2 * c + 1] = L[idx];
      }
    }
    __syncthreads();
    if (t == 0) st[0] = idx;
  } else if (t == 0) {   // DistributionSampler (samplers.py:51-68)
    int cur = F.state[0], item = F.state[1];
    for (int64_t c = 0; c < count; ++c) {
      pairs[2 * c] = F.dens_order[F.bins[cur] * F.bin_size + item];
      pairs[2 * c + 1] = F.dens_order[F.bins[cur + 1] * F.bin_size + item];
      cur += 2;
      if (cur >= F.n_bins - 1) cur = 0;
      item = F.item_table[cur >> 1];
    }
    F.state[0] = cur;
    F.state[1] = item;
  }
  __syncthreads();
  // labels: of the input pairs, or (quirk A3) of the last B calls
  for (int i = t; i < B; i += blockDim.x) {   // any B, not just one per thread
    const int64_t c = F.compat ? count - B + i : i;
    const int a = pairs[2 * c], b = pairs[2 * c + 1];
    const bool ok = a >= 0 && a < F.label_n && b >= 0 && b < F.label_n;
    labels[i] = ok ? F.label_matrix[(size_t)a * F.label_n + b] : 0.f;
  }
  __syncthreads();
  if (t == 0) {   // ȳ and ½Σ(y - ȳ)² in double, in order
    double sum = 0.0;
    for (int i = 0; i < B; ++i) sum += (double)labels[i];
    const double ybar = B > 0 ? sum / (double)B : 0.0;
    double half = 0.0;
    for (int i = 0; i < B; ++i) half += ((double)labels[i] - ybar) * ((double)labels[i] - ybar);
    y_stats[0] = (float)ybar;
    y_stats[1] = (float)(0.5 * half);
  }
  // pack the B input pairs: one wavefront per record
  const int w = t >> 6, nw = blockDim.x >> 6;
  for (int p = w; p < B; p += nw)
    sg_pack_record(F.store_adj, F.store_types, F.store_n, F.n_graphs, F.n_max, F.adj_dtype,
                   pairs[2 * p], pairs[2 * p + 1], labels[p], p,
                   recs + (size_t)p * rec_words, rec_words, t & 63, status);
}

}  // namespace

extern "C" {

int32_t sg_feed_step(const sg_feed_t *feed, int32_t *pairs_out, void *records, float *labels_out,
                     float *y_stats_out, int32_t *status_out, sg_stream_t stream) {
  if (!feed || !pairs_out || !records || !labels_out || !y_stats_out) return SG_ERR_ARG;
  const sg_feed_t &F = *feed;
  if (F.batch < 1 || !F.state || !F.label_matrix || F.label_n < 1 || !F.store_adj ||
      !F.store_types || !F.store_n || F.n_graphs < 1 || F.n_max < 1 || F.n_max > 64 ||
      !sg_dtype_ok(F.adj_dtype))
    return SG_ERR_ARG;
  if (F.kind == 0 && (F.n < 2 || !F.sigma)) return SG_ERR_ARG;
  if (F.kind == 1 && (F.n_bins < 2 || F.bin_size < 1 || !F.dens_order || !F.bins || !F.item_table))
    return SG_ERR_ARG;
  if (F.kind != 0 && F.kind != 1) return SG_ERR_ARG;
  const SgRecLayout rl = sg_rec_layout(F.n_max, F.adj_dtype);
  hipLaunchKernelGGL(sg_feed_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, F, pairs_out,
                     (uint32_t *)records, rl.words, labels_out, y_stats_out, status_out);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int32_t sg_sampler_random(int32_t *state, const int32_t *sigma, int32_t n, int64_t count,
                          int32_t *pairs_out, sg_stream_t stream) {
  if (n < 2 || count < 0 || !state || !sigma || (count > 0 && !pairs_out)) return SG_ERR_ARG;
  if (count == 0) return SG_OK;
  hipLaunchKernelGGL(sg_sampler_random_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, state,
                     sigma, n, count, pairs_out);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

int32_t sg_sampler_density(int32_t *state, const int32_t *dens_order, const int32_t *bins,
                           int32_t n_bins, int32_t bin_size, const int32_t *item_table,
                           int64_t count, int32_t *pairs_out, sg_stream_t stream) {
  if (n_bins < 2 || bin_size < 1 || count < 0 || !state || !dens_order || !bins || !item_table ||
      (count > 0 && !pairs_out))
    return SG_ERR_ARG;
  if (count == 0) return SG_OK;
  hipLaunchKernelGGL(sg_sampler_density_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state,
                     dens_order, bins, n_bins, bin_size, item_table, count, pairs_out);
  return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_HIP;
}

}  // extern "C"
