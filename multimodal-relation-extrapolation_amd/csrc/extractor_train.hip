// extractor_train.hip -- the ZSL Extractor in TRAINING mode (dropout active): the inputs of
// its differentiable part, for pretrain_Extractor (module/zsl_module.py:289-348) and for the
// GAN loop while the Extractor is still in training mode (zsl_module.py:371-383, 430-440).
//
// Reference, one (e1, e2) row with its neighbour lists (zsl_module.py:47-67, submodule.py:254-258):
//   nb(x)  = tanh( sum_s gcn_w(dropout(emb[conn[x][s][1]])) / deg[x] )         dropout p = 0.2
//   ent    = tanh( cat(fc1(dropout_e(emb[e1])), fc2(dropout_e(emb[e2]))) )      dropout p = 0.2
//   g      = LayerNorm( dropout(proj2(relu(proj1(x)))) + x ),  x = reshape(cat(nb(e1), ent, nb(e2)))
//
// symbol_emb is frozen (requires_grad = False, :38), so everything up to the linears is a
// constant of the step: k_extractor_train_inputs gathers it once per row -- the dropped
// neighbour SUM of each side (gcn_w is linear: sum_s (W x_s + b) = W sum_s x_s + max_nb b, the
// linear and its bias then run as a GEMM on the host side) and the two dropped entity rows.
// The linears, tanh, relu, LayerNorm and their gradients are the autograd chain of
// mmre/extractor_train.py on the split-K GEMM (gemm.hip). k_dropout is the SupportEncoder's
// dropout (and any other elementwise one), keeping its mask for the backward.
//
// Dropout masks come from a counter-based hash of (seed, offset, stream, element): a draw is
// a pure function of its coordinates, so a step captured in a hipGraph draws fresh masks at
// every replay when the offset -- a device word the step advances (an in-graph add) -- changes, and two runs
// with the same seed draw the same masks. keep <=> u24 >= p * 2^24 (u24 = top 24 bits);
// kept values are x * (1 / (1 - p)), the multiplier torch's dropout applies (1.25 at p 0.2).
// Tests inject explicit 0/1 masks instead (same kernels, mask pointers non-null).
#include "mmre_common.h"

namespace mmre {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// 24-bit uniform draw of element `idx` of dropout stream `stream`
__device__ __forceinline__ uint32_t drop_u24(uint64_t key, uint32_t stream, uint64_t idx) {
  return (uint32_t)(mix64(key ^ mix64(idx * 0x9e3779b97f4a7c15ull + ((uint64_t)stream << 48) + stream)) >> 40);
}

__device__ __forceinline__ uint64_t drop_key(const uint64_t* st) {
  return mix64(st[0] + 0x632be59bd9b4e019ull * (st[1] + 1));
}

// One workgroup per row, threads over the embedding width. Per side: sum over the max_nb
// neighbour slots (ascending s) of the dropped symbol row; entity rows dropped once.
__global__ __launch_bounds__(256) void k_extractor_train_inputs(
    int dim, const float* __restrict__ emb, const int64_t* __restrict__ pairs, const int64_t* __restrict__ conn_l,
    const int64_t* __restrict__ conn_r, int max_nb, int64_t n_rows, uint32_t thr, float scale,
    const uint64_t* __restrict__ rng, const uint8_t* __restrict__ m_nb_l, const uint8_t* __restrict__ m_nb_r,
    const uint8_t* __restrict__ m_ent, float* __restrict__ nsum_l, float* __restrict__ nsum_r,
    float* __restrict__ e1d, float* __restrict__ e2d) {
  const int64_t row = blockIdx.x;
  if (row >= n_rows) return;
  const uint64_t key = rng ? drop_key(rng) : 0;
  const bool use_rng = m_nb_l == nullptr;
  __shared__ int64_t sym[2][64];
  // neighbour symbol ids of both sides, staged once (conn is (row, s, 2): [rel, ent])
  for (int i = threadIdx.x; i < 2 * max_nb && i < 128; i += blockDim.x) {
    const int side = i / max_nb, s = i % max_nb;
    const int64_t* c = side ? conn_r : conn_l;
    sym[side][s] = c[(row * max_nb + s) * 2 + 1];
  }
  __syncthreads();
  const int64_t e1 = pairs[row * 2], e2 = pairs[row * 2 + 1];
  for (int k = threadIdx.x; k < dim; k += blockDim.x) {
    float acc[2] = {0.f, 0.f};
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const uint8_t* mm = side ? m_nb_r : m_nb_l;
      for (int s = 0; s < max_nb; ++s) {
        const uint64_t idx = ((uint64_t)row * max_nb + s) * dim + k;
        const float x = emb[sym[side][s] * dim + k];
        const bool keep = use_rng ? drop_u24(key, side, idx) >= thr : mm[idx] != 0;
        acc[side] += keep ? x * scale : 0.f;
      }
    }
    nsum_l[row * dim + k] = acc[0];
    nsum_r[row * dim + k] = acc[1];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint64_t idx = ((uint64_t)row * 2 + j) * dim + k;
      const float x = emb[(j ? e2 : e1) * dim + k];
      const bool keep = use_rng ? drop_u24(key, 2, idx) >= thr : m_ent[idx] != 0;
      (j ? e2d : e1d)[row * dim + k] = keep ? x * scale : 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void k_dropout(const float* __restrict__ x, float* __restrict__ y,
                                                 uint8_t* __restrict__ mask, int64_t n, uint32_t thr, float scale,
                                                 const uint64_t* __restrict__ rng, uint32_t stream) {
  const uint64_t key = drop_key(rng);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool keep = drop_u24(key, stream, (uint64_t)i) >= thr;
    y[i] = keep ? x[i] * scale : 0.f;
    if (mask) mask[i] = keep;
  }
}

static uint32_t keep_threshold(float p) {
  double t = (double)p * 16777216.0;
  if (t < 0) t = 0;
  if (t > 16777216.0) t = 16777216.0;
  return (uint32_t)(t + 0.5);
}

}  // namespace mmre

using namespace mmre;

extern "C" int mmre_extractor_train_inputs(int dim, const float* d_sym_emb, const int64_t* d_pairs,
                                           const int64_t* d_conn_left, const int64_t* d_conn_right, int max_nb,
                                           int64_t n_rows, float p, const uint64_t* d_rng_state,
                                           const uint8_t* d_mask_nb_left, const uint8_t* d_mask_nb_right,
                                           const uint8_t* d_mask_ent, float* d_nsum_left, float* d_nsum_right,
                                           float* d_e1, float* d_e2, void* stream) {
  if (!d_sym_emb || !d_pairs || !d_conn_left || !d_conn_right || !d_nsum_left || !d_nsum_right || !d_e1 || !d_e2)
    return MMRE_ERR_ARG;
  if (dim <= 0 || n_rows < 0 || max_nb < 0 || max_nb > 64 || !(p >= 0.f && p < 1.f)) return MMRE_ERR_ARG;
  const bool masks = d_mask_nb_left || d_mask_nb_right || d_mask_ent;
  if (masks && !(d_mask_nb_left && d_mask_nb_right && d_mask_ent)) return MMRE_ERR_ARG;
  if (!masks && !d_rng_state) return MMRE_ERR_ARG;
  if (n_rows == 0) return MMRE_OK;
  hipStream_t st = (hipStream_t)stream;
  const float scale = 1.0f / (1.0f - p);
  hipLaunchKernelGGL(k_extractor_train_inputs, dim3((unsigned)n_rows), dim3(256), 0, st, dim, d_sym_emb, d_pairs,
                     d_conn_left, d_conn_right, max_nb, n_rows, keep_threshold(p), scale,
                     masks ? nullptr : d_rng_state, d_mask_nb_left, d_mask_nb_right, d_mask_ent, d_nsum_left,
                     d_nsum_right, d_e1, d_e2);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_dropout(const float* d_x, float* d_y, uint8_t* d_mask, int64_t n, float p,
                            const uint64_t* d_rng_state, int stream_id, void* stream) {
  if (!d_x || !d_y || !d_rng_state || n < 0 || !(p >= 0.f && p < 1.f) || stream_id < 0) return MMRE_ERR_ARG;
  if (n == 0) return MMRE_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_dropout, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, d_x, d_y, d_mask, n,
                     keep_threshold(p), 1.0f / (1.0f - p), d_rng_state, (uint32_t)stream_id);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
