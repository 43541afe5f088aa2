// generator.hip -- the zero-shot relation-embedding generator (module/model.py:674-686):
//   x  = cat([noise, cls], 1)                                   (model.py:680)
//   h1 = x  (W0/s0)^T + b0     generate_fc_layer   399 -> 384   (model.py:681, SN Linear)
//   h2 = h1 (W1/s1)^T + b1     des_rel_map_layer1  384 -> D     (model.py:682)
//   h3 = h2 (W2/s2)^T + b2     des_rel_map_layer2  D   -> D     (model.py:684)
//   out = LayerNormalization(h3): (z - mean) / (std_unbiased + eps) * a + b   (submodule.py:58-77)
// Spectral norm (spectral_norm.py:39-89): s = u . (W v); in training mode one power
// iteration first sets v = normalize(W^T u), u = normalize(W v) in place (eps 1e-12).
//
// k_sn_sigma: one workgroup per layer (the three mat-vecs), writes sigma[3] (+ u, v).
// k_generator_mlp: one workgroup per 32 rows; the three layers run back to back on
// v_mfma_f32_32x32x2_f32 with the activations kept in LDS (A operand) and the weights
// read from global as W[c][k] / sigma -- the reference's normalised weight values --
// as the B operand; bias add in the epilogue; LayerNormalization by one wave per row.
#include "mmre_common.h"

namespace mmre {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.0f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

struct SNLayer {
  const float* w;  // (out, in) row-major
  float* u;        // (out)
  float* v;        // (in)
  int out, in;
};

// One workgroup per layer. scratch: >= in + out floats per layer (workspace).
__global__ __launch_bounds__(256) void k_sn_sigma(SNLayer l0, SNLayer l1, SNLayer l2, int power_iteration, float eps,
                                                  float* __restrict__ sigma, float* __restrict__ scratch) {
  __shared__ float red[4];
  const SNLayer L = blockIdx.x == 0 ? l0 : (blockIdx.x == 1 ? l1 : l2);
  float* wv = scratch + blockIdx.x * 2048;  // W v   (out <= 1024)
  float* tv = wv + 1024;                    // W^T u (in <= 1024)
  if (power_iteration) {
    for (int k = threadIdx.x; k < L.in; k += blockDim.x) {
      float s = 0.0f;
      for (int o = 0; o < L.out; ++o) s += L.w[(int64_t)o * L.in + k] * L.u[o];
      tv[k] = s;
    }
    __syncthreads();
    float ss = 0.0f;
    for (int k = threadIdx.x; k < L.in; k += blockDim.x) ss += tv[k] * tv[k];
    const float nv = fmaxf(sqrtf(block_sum(ss, red)), eps);
    __syncthreads();
    for (int k = threadIdx.x; k < L.in; k += blockDim.x) L.v[k] = tv[k] / nv;
    __syncthreads();
  }
  for (int o = threadIdx.x; o < L.out; o += blockDim.x) {
    float s = 0.0f;
    for (int k = 0; k < L.in; ++k) s += L.w[(int64_t)o * L.in + k] * L.v[k];
    wv[o] = s;
  }
  __syncthreads();
  if (power_iteration) {
    float ss = 0.0f;
    for (int o = threadIdx.x; o < L.out; o += blockDim.x) ss += wv[o] * wv[o];
    const float nu = fmaxf(sqrtf(block_sum(ss, red)), eps);
    __syncthreads();
    for (int o = threadIdx.x; o < L.out; o += blockDim.x) L.u[o] = wv[o] / nu;
    __syncthreads();
  }
  float dot = 0.0f;
  for (int o = threadIdx.x; o < L.out; o += blockDim.x) dot += L.u[o] * wv[o];
  dot = block_sum(dot, red);
  if (threadIdx.x == 0) sigma[blockIdx.x] = dot;
}

constexpr int GM = 32;  // rows per workgroup

// out_lds[i][c] = sum_k a_lds[i][k] * (W[c][k] / s) + b[c] for c < out (K padded to even).
__device__ void mfma_layer(const float* a_lds, int lda, int in, const float* __restrict__ w,
                           const float* __restrict__ bias, float s, int out, float* out_lds, int ldo) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int i = lane & 31, kh = lane >> 5;
  const int n_tiles = (out + 31) / 32;
  for (int tile = wave; tile < n_tiles; tile += nw) {
    const int c = tile * 32 + i;  // B operand column for this lane
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    const float* wrow = w + (int64_t)c * in;
    for (int k0 = 0; k0 < in; k0 += 2) {
      const int k = k0 + kh;
      const float a = k < in ? a_lds[i * lda + k] : 0.0f;
      const float b = (c < out && k < in) ? wrow[k] / s : 0.0f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    const int col = tile * 32 + i;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * kh;
      if (col < out) out_lds[row * ldo + col] = acc[r] + bias[col];
    }
  }
}

__global__ __launch_bounds__(256) void k_generator_mlp(const float* __restrict__ noise, int nd,
                                                       const float* __restrict__ cls, int cd, int64_t n_rows,
                                                       const float* __restrict__ w0, const float* __restrict__ b0,
                                                       int o0, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, int o1,
                                                       const float* __restrict__ w2, const float* __restrict__ b2,
                                                       int o2, const float* __restrict__ sigma,
                                                       const float* __restrict__ ln_a, const float* __restrict__ ln_b,
                                                       float ln_eps, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int in0 = nd + cd;
  const int lda = in0 | 1, ld1 = o0 | 1, ld2 = o1 | 1, ld3 = o2 | 1;  // odd strides: conflict-free column reads
  float* x0 = smem;                 // [GM][lda]
  float* x1 = x0 + GM * lda;        // [GM][ld1]
  float* x2 = x0;                   // reuse
  float* x3 = x1;                   // reuse (o2 <= o0 checked on the host)
  const int64_t r0 = (int64_t)blockIdx.x * GM;
  for (int idx = threadIdx.x; idx < GM * in0; idx += blockDim.x) {
    const int i = idx / in0, k = idx % in0;
    const int64_t row = r0 + i;
    float v = 0.0f;
    if (row < n_rows) v = k < nd ? noise[row * nd + k] : cls[row * cd + (k - nd)];
    x0[i * lda + k] = v;
  }
  __syncthreads();
  mfma_layer(x0, lda, in0, w0, b0, sigma[0], o0, x1, ld1);
  __syncthreads();
  mfma_layer(x1, ld1, o0, w1, b1, sigma[1], o1, x2, ld2);
  __syncthreads();
  mfma_layer(x2, ld2, o1, w2, b2, sigma[2], o2, x3, ld3);
  __syncthreads();
  // LayerNormalization: one wave per row
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int i = wave; i < GM; i += nw) {
    const int64_t row = r0 + i;
    if (row >= n_rows) continue;
    const float* z = x3 + i * ld3;
    if (o2 == 1) {
      if (lane == 0) out[row] = z[0];
      continue;
    }
    float s = 0.0f;
    for (int k = lane; k < o2; k += 64) s += z[k];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) s += __shfl_xor(s, sh);
    const float mu = s / (float)o2;
    float v = 0.0f;
    for (int k = lane; k < o2; k += 64) v += (z[k] - mu) * (z[k] - mu);
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) v += __shfl_xor(v, sh);
    const float sd = sqrtf(v / (float)(o2 - 1));
    for (int k = lane; k < o2; k += 64) out[row * o2 + k] = (z[k] - mu) / (sd + ln_eps) * ln_a[k] + ln_b[k];
  }
}

}  // namespace mmre

using namespace mmre;

extern "C" int64_t mmre_generator_workspace(int64_t n_rows, int in0, int out0, int out1, int out2) {
  (void)n_rows; (void)in0; (void)out0; (void)out1; (void)out2;
  return 3 * 2048 + 16;  // mat-vec scratch + sigma[3]
}

extern "C" int mmre_generator_forward(const float* d_noise, int noise_dim, const float* d_cls, int cls_dim,
                                      int64_t n_rows, const float* d_w0, const float* d_b0, float* d_u0, float* d_v0,
                                      int out0, const float* d_w1, const float* d_b1, float* d_u1, float* d_v1,
                                      int out1, const float* d_w2, const float* d_b2, float* d_u2, float* d_v2,
                                      int out2, const float* d_ln_a, const float* d_ln_b, float ln_eps,
                                      int power_iteration, float sn_eps, float* d_out, float* d_work, void* stream) {
  if (!d_noise || !d_cls || !d_w0 || !d_b0 || !d_u0 || !d_v0 || !d_w1 || !d_b1 || !d_u1 || !d_v1 || !d_w2 || !d_b2 ||
      !d_u2 || !d_v2 || !d_ln_a || !d_ln_b || !d_out || !d_work)
    return MMRE_ERR_ARG;
  const int in0 = noise_dim + cls_dim;
  if (n_rows <= 0 || noise_dim < 0 || cls_dim <= 0 || out0 <= 0 || out1 <= 0 || out2 <= 0) return MMRE_ERR_ARG;
  if (in0 > 1024 || out0 > 1024 || out1 > 1024 || out2 > out0 || (out1 | 1) > (in0 | 1)) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  float* sigma = d_work + 3 * 2048;
  SNLayer l0{d_w0, d_u0, d_v0, out0, in0}, l1{d_w1, d_u1, d_v1, out1, out0}, l2{d_w2, d_u2, d_v2, out2, out1};
  hipLaunchKernelGGL(k_sn_sigma, dim3(3), dim3(256), 0, st, l0, l1, l2, power_iteration, sn_eps, sigma, d_work);
  MMRE_CHECK_LAUNCH();
  const size_t lds = sizeof(float) * (size_t)GM * ((in0 | 1) + (out0 | 1));
  if (lds > 160 * 1024) return MMRE_ERR_SHAPE;
  const unsigned blocks = (unsigned)((n_rows + GM - 1) / GM);
  hipLaunchKernelGGL(k_generator_mlp, dim3(blocks), dim3(256), lds, st, d_noise, noise_dim, d_cls, cls_dim, n_rows,
                     d_w0, d_b0, out0, d_w1, d_b1, out1, d_w2, d_b2, out2, sigma, d_ln_a, d_ln_b, ln_eps, d_out);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
