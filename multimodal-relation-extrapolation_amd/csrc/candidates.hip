// candidates.hip -- candidate-list rankings of the repo's evaluation surfaces.
//
// k_candidate_rank_transe: main.evaluate (main.py:232-250). Per (head, relation) query the
//   candidate tails (true tail first) are scored with NegativeSampling.evaluate
//   (module/NegativeSampling.py:294-302: TransE, p = 1, no normalisation):
//   s = |(h + r) - t|_1 (canonical: hr = h + r element-wise, then a sequential k sum), and
//   rank = #(s_j < s_0) + #(s_j == s_0) // 2 + 1 over j >= 1.
// k_cosine_rank: ZSLmodule.eval (zsl_module.py:699-706): score_c = mean_s cos(cand_c, rel_s)
//   (sklearn cosine_similarity: rows L2-normalised, then dot products); rank of the true
//   candidate (row 0) in descending order = 1 + #(score_j > score_0) (tie-free inputs).
// One workgroup per query; the query-side vectors are staged in LDS.
#include "mmre_common.h"

namespace mmre {

constexpr int CR_MAXD = 1024;

__device__ __forceinline__ int block_reduce_int(int v, int* red) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

__global__ __launch_bounds__(256) void k_candidate_rank_transe(const float* __restrict__ ent,
                                                               const float* __restrict__ rel, int dim,
                                                               const int64_t* __restrict__ qh,
                                                               const int64_t* __restrict__ qr, int64_t n_query,
                                                               const int64_t* __restrict__ off,
                                                               const int64_t* __restrict__ ids,
                                                               float* __restrict__ scores, int32_t* __restrict__ rank) {
  __shared__ float hr[CR_MAXD];
  __shared__ float s_p;
  __shared__ int red[8];
  for (int64_t q = blockIdx.x; q < n_query; q += gridDim.x) {
    const int64_t a = off[q], b = off[q + 1];
    __syncthreads();
    const float* hv = ent + qh[q] * dim;
    const float* rv = rel + qr[q] * dim;
    for (int k = threadIdx.x; k < dim; k += blockDim.x) hr[k] = hv[k] + rv[k];
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.0f;
      const float* t = ent + ids[a] * dim;
      for (int k = 0; k < dim; ++k) s = s + fabsf(hr[k] - t[k]);
      s_p = s;
      if (scores) scores[a] = s;
    }
    __syncthreads();
    const float p = s_p;
    int less = 0, eq = 0;
    for (int64_t c = a + 1 + threadIdx.x; c < b; c += blockDim.x) {
      const float* t = ent + ids[c] * dim;
      float s = 0.0f;
      for (int k = 0; k < dim; ++k) s = s + fabsf(hr[k] - t[k]);
      if (scores) scores[c] = s;
      less += s < p;
      eq += s == p;
    }
    less = block_reduce_int(less, red);
    eq = block_reduce_int(eq, red);
    if (threadIdx.x == 0 && b > a) rank[q] = less + eq / 2 + 1;
  }
}

constexpr int CS_MAXS = 64;

__global__ __launch_bounds__(256) void k_cosine_rank(const float* __restrict__ cand, int dim,
                                                     const int64_t* __restrict__ off, int64_t n_query,
                                                     const float* __restrict__ rel_vecs, int n_samples,
                                                     const int64_t* __restrict__ rel_of_query,
                                                     float* __restrict__ scores, int32_t* __restrict__ rank) {
  extern __shared__ __attribute__((aligned(16))) float ys[];  // [n_samples][dim] normalised
  __shared__ float s0;
  __shared__ int red[8];
  __shared__ float ynorm[CS_MAXS];
  for (int64_t q = blockIdx.x; q < n_query; q += gridDim.x) {
    const int64_t a = off[q], b = off[q + 1];
    const float* Y = rel_vecs + rel_of_query[q] * (int64_t)n_samples * dim;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int s = w; s < n_samples; s += (int)(blockDim.x >> 6)) {
      float ss = 0.0f;
      for (int k = lane; k < dim; k += 64) ss += Y[s * dim + k] * Y[s * dim + k];
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) ss += __shfl_xor(ss, sh);
      if (lane == 0) ynorm[s] = sqrtf(ss);
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < n_samples * dim; idx += blockDim.x) {
      const float n = ynorm[idx / dim];
      ys[idx] = n > 0.0f ? Y[idx] / n : 0.0f;
    }
    __syncthreads();
    auto score_of = [&](int64_t c) {
      const float* x = cand + c * dim;
      float ss = 0.0f;
      for (int k = 0; k < dim; ++k) ss += x[k] * x[k];
      const float nx = sqrtf(ss);
      float tot = 0.0f;
      for (int s = 0; s < n_samples; ++s) {
        float dot = 0.0f;
        for (int k = 0; k < dim; ++k) dot += x[k] * ys[s * dim + k];
        tot += nx > 0.0f ? dot / nx : 0.0f;
      }
      return tot / (float)n_samples;
    };
    if (threadIdx.x == 0) {
      s0 = score_of(a);
      if (scores) scores[a] = s0;
    }
    __syncthreads();
    int better = 0;
    for (int64_t c = a + 1 + threadIdx.x; c < b; c += blockDim.x) {
      const float v = score_of(c);
      if (scores) scores[c] = v;
      better += v > s0;
    }
    better = block_reduce_int(better, red);
    if (threadIdx.x == 0 && b > a) rank[q] = better + 1;
  }
}

}  // namespace mmre

using namespace mmre;

extern "C" int mmre_candidate_rank_transe(const float* d_ent, const float* d_rel, int dim, const int64_t* d_qh,
                                          const int64_t* d_qr, int64_t n_query, const int64_t* d_cand_off,
                                          const int64_t* d_cand_ids, float* d_scores, int32_t* d_rank, void* stream) {
  if (!d_ent || !d_rel || !d_qh || !d_qr || !d_cand_off || !d_cand_ids || !d_rank || n_query <= 0 || dim <= 0)
    return MMRE_ERR_ARG;
  if (dim > CR_MAXD) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const unsigned blocks = (unsigned)(n_query < 8192 ? n_query : 8192);
  hipLaunchKernelGGL(k_candidate_rank_transe, dim3(blocks), dim3(256), 0, st, d_ent, d_rel, dim, d_qh, d_qr, n_query,
                     d_cand_off, d_cand_ids, d_scores, d_rank);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_cosine_rank(const float* d_cand, int dim, const int64_t* d_cand_off, int64_t n_query,
                                const float* d_rel_vecs, int n_samples, const int64_t* d_rel_of_query,
                                float* d_scores, int32_t* d_rank, void* stream) {
  if (!d_cand || !d_cand_off || !d_rel_vecs || !d_rel_of_query || !d_rank || n_query <= 0 || dim <= 0 ||
      n_samples <= 0)
    return MMRE_ERR_ARG;
  if (n_samples > CS_MAXS || (size_t)n_samples * dim * sizeof(float) > 96 * 1024) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const unsigned blocks = (unsigned)(n_query < 8192 ? n_query : 8192);
  hipLaunchKernelGGL(k_cosine_rank, dim3(blocks), dim3(256), sizeof(float) * n_samples * dim, st, d_cand, dim,
                     d_cand_off, n_query, d_rel_vecs, n_samples, d_rel_of_query, d_scores, d_rank);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
