// generator.hip -- the zero-shot relation-embedding generator (module/model.py:674-686):
//   x  = cat([noise, cls], 1)                                   (model.py:680)
//   h1 = x  (W0/s0)^T + b0     generate_fc_layer   399 -> 384   (model.py:681, SN Linear)
//   h2 = h1 (W1/s1)^T + b1     des_rel_map_layer1  384 -> D     (model.py:682)
//   h3 = h2 (W2/s2)^T + b2     des_rel_map_layer2  D   -> D     (model.py:684)
//   out = LayerNormalization(h3): (z - mean) / (std_unbiased + eps) * a + b   (submodule.py:58-77)
// Spectral norm (spectral_norm.py:39-89): s = u . (W v); in training mode one power
// iteration first sets v = normalize(W^T u), u = normalize(W v) in place (eps 1e-12).
//
// Forward launches (all small: N <= ~1k rows, so the design is about parallelism, not reuse):
//   k_sn_sigma   one 1024-thread workgroup per layer: the power-iteration mat-vecs split over
//                16 waves (column sums lane-parallel over 4 row quarters, row dots wave-parallel)
//   k_sn_scale   W_hat = W_orig / sigma element-wise (the reference's normalised weight values),
//                kept in the activation buffer for the backward
//   k_gen_concat x0 = [noise | cls]
//   linears      x W_hat^T + b on the split-K GEMM of gemm.hip (32 x 32 MFMA tiles, bias in its
//                epilogue)
//   k_gen_ln     LayerNormalization, one wave per row
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

constexpr int SN_T = 1024;

// sigma of one layer by one SN_T-thread workgroup (returned to every thread); in training
// mode the power iteration first updates L.u, L.v in place. wv / tv: 1024 floats each of scratch.
__device__ float sn_sigma_layer(const SNLayer& L, int power_iteration, float eps, float* __restrict__ wv,
                                float* __restrict__ tv, float* red, float (*part)[1024]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = SN_T / 64;
  if (power_iteration) {
    // tv[k] = sum_o W[o][k] u[o]: 256 columns per pass x 4 quarters of the rows
    const int q = threadIdx.x >> 8, tk = threadIdx.x & 255;
    const int o0 = (int)((int64_t)q * L.out / 4), o1 = (int)((int64_t)(q + 1) * L.out / 4);
    for (int k0 = 0; k0 < L.in; k0 += 256) {
      const int k = k0 + tk;
      float s = 0.0f;
      if (k < L.in) {
#pragma unroll 8
        for (int o = o0; o < o1; ++o) s += L.w[(int64_t)o * L.in + k] * L.u[o];
      }
      part[q][tk] = s;
      __syncthreads();
      if (q == 0 && k < L.in) tv[k] = part[0][tk] + part[1][tk] + part[2][tk] + part[3][tk];
      __syncthreads();
    }
    float ss = 0.0f;
    for (int k = threadIdx.x; k < L.in; k += SN_T) ss += tv[k] * tv[k];
    const float nv = fmaxf(sqrtf(block_sum(ss, red)), eps);
    __syncthreads();
    for (int k = threadIdx.x; k < L.in; k += SN_T) L.v[k] = tv[k] / nv;
    __syncthreads();
  }
  // wv[o] = W[o] . v: one wave per row, lanes over k (coalesced)
  for (int o = wave; o < L.out; o += nw) {
    float s = 0.0f;
    for (int k = lane; k < L.in; k += 64) s += L.w[(int64_t)o * L.in + k] * L.v[k];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) s += __shfl_xor(s, sh);
    if (lane == 0) wv[o] = s;
  }
  __syncthreads();
  if (power_iteration) {
    float ss = 0.0f;
    for (int o = threadIdx.x; o < L.out; o += SN_T) ss += wv[o] * wv[o];
    const float nu = fmaxf(sqrtf(block_sum(ss, red)), eps);
    __syncthreads();
    for (int o = threadIdx.x; o < L.out; o += SN_T) L.u[o] = wv[o] / nu;
    __syncthreads();
  }
  float dot = 0.0f;
  for (int o = threadIdx.x; o < L.out; o += SN_T) dot += L.u[o] * wv[o];
  return block_sum(dot, red);
}

// One workgroup per layer. scratch: 2048 floats per layer (W v, then W^T u).
__global__ __launch_bounds__(SN_T) void k_sn_sigma(SNLayer l0, SNLayer l1, SNLayer l2, int power_iteration,
                                                   float eps, float* __restrict__ sigma, float* __restrict__ scratch) {
  __shared__ float red[SN_T / 64];
  __shared__ float part[4][1024];
  const SNLayer L = blockIdx.x == 0 ? l0 : (blockIdx.x == 1 ? l1 : l2);
  float* wv = scratch + blockIdx.x * 2048;
  const float s = sn_sigma_layer(L, power_iteration, eps, wv, wv + 1024, red, part);
  if (threadIdx.x == 0) sigma[blockIdx.x] = s;
}

// spectral_norm.compute_weight (spectral_norm.py:39-89, torch.nn.utils.spectral_norm) of one
// layer in one launch: power iteration (training mode), sigma, W_hat = W / sigma, and copies
// of the u, v the weight was normalised with (the autograd snapshot: later calls update the
// buffers in place).
__global__ __launch_bounds__(SN_T) void k_sn_weight(SNLayer L, int power_iteration, float eps,
                                                    float* __restrict__ sigma, float* __restrict__ scratch,
                                                    float* __restrict__ u_snap, float* __restrict__ v_snap,
                                                    float* __restrict__ w_hat) {
  __shared__ float red[SN_T / 64];
  __shared__ float part[4][1024];
  const float s = sn_sigma_layer(L, power_iteration, eps, scratch, scratch + 1024, red, part);
  if (threadIdx.x == 0) sigma[0] = s;
  const int64_t n = (int64_t)L.out * L.in;
  for (int64_t i = threadIdx.x; i < n; i += SN_T) w_hat[i] = L.w[i] / s;
  for (int o = threadIdx.x; o < L.out; o += SN_T) u_snap[o] = L.u[o];
  for (int k = threadIdx.x; k < L.in; k += SN_T) v_snap[k] = L.v[k];
}

// W_hat = W_orig / sigma for the three layers (one grid over their concatenation).
__global__ __launch_bounds__(256) void k_sn_scale(const float* __restrict__ w0, int64_t n0,
                                                  const float* __restrict__ w1, int64_t n1,
                                                  const float* __restrict__ w2, int64_t n2,
                                                  const float* __restrict__ sigma, float* __restrict__ out) {
  const int64_t total = n0 + n1 + n2, stride = (int64_t)gridDim.x * blockDim.x;
  const float s0 = sigma[0], s1 = sigma[1], s2 = sigma[2];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride)
    out[i] = i < n0 ? w0[i] / s0 : (i < n0 + n1 ? w1[i - n0] / s1 : w2[i - n0 - n1] / s2);
}

__global__ __launch_bounds__(256) void k_gen_concat(const float* __restrict__ noise, int nd,
                                                    const float* __restrict__ cls, int cd, int64_t n_rows,
                                                    float* __restrict__ x0) {
  const int in0 = nd + cd;
  const int64_t total = n_rows * in0, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t r = i / in0;
    const int k = (int)(i % in0);
    x0[i] = k < nd ? noise[r * nd + k] : cls[r * cd + (k - nd)];
  }
}

// LayerNormalization forward (submodule.py:68-77), one wave per row.
__global__ __launch_bounds__(256) void k_gen_ln(const float* __restrict__ z, const float* __restrict__ ln_a,
                                                const float* __restrict__ ln_b, float eps, int64_t n_rows, int D,
                                                float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const float* zr = z + row * D;
  if (D == 1) {
    if (lane == 0) out[row] = zr[0];
    return;
  }
  float s = 0.0f;
  for (int k = lane; k < D; k += 64) s += zr[k];
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) s += __shfl_xor(s, sh);
  const float mu = s / (float)D;
  float v = 0.0f;
  for (int k = lane; k < D; k += 64) v += (zr[k] - mu) * (zr[k] - mu);
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) v += __shfl_xor(v, sh);
  const float sd = sqrtf(v / (float)(D - 1));
  for (int k = lane; k < D; k += 64) out[row * D + k] = (zr[k] - mu) / (sd + eps) * ln_a[k] + ln_b[k];
}

// ----------------------------------------------------------------------------------------
// Backward (training step of the generator, zsl_module.py:526-597: loss_G.backward()).
// ----------------------------------------------------------------------------------------
// LayerNormalization backward, one wave per row: out = (z - mu) / (sd + eps) * a + b with the
// unbiased sd. With c = z - mu, d = sd + eps, g = dL/dout * a:
//   dL/dz_k = (g_k - mean(g)) / d - c_k * sum_i(g_i c_i) / (d^2 * sd * (D - 1)).
// Writes gz (N, D) and zhat (N, D) (for the a_2 gradient). D == 1: identity (submodule.py:69-70).
__global__ __launch_bounds__(256) void k_gen_ln_bwd(const float* __restrict__ gout, const float* __restrict__ z,
                                                    const float* __restrict__ ln_a, float eps, int64_t n_rows, int D,
                                                    float* __restrict__ gz, float* __restrict__ zhat) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const float* zr = z + row * D;
  const float* gr = gout + row * D;
  if (D == 1) {
    if (lane == 0) { gz[row] = gr[0]; zhat[row] = 0.0f; }
    return;
  }
  float s = 0.0f;
  for (int k = lane; k < D; k += 64) s += zr[k];
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) s += __shfl_xor(s, sh);
  const float mu = s / (float)D;
  float v = 0.0f, sg = 0.0f, sgc = 0.0f;
  for (int k = lane; k < D; k += 64) {
    const float c = zr[k] - mu, g = gr[k] * ln_a[k];
    v += c * c;
    sg += g;
    sgc += g * c;
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) {
    v += __shfl_xor(v, sh);
    sg += __shfl_xor(sg, sh);
    sgc += __shfl_xor(sgc, sh);
  }
  const float sd = sqrtf(v / (float)(D - 1)), d = sd + eps;
  const float mg = sg / (float)D;
  const float coef = sgc / (d * d * sd * (float)(D - 1));
  for (int k = lane; k < D; k += 64) {
    const float c = zr[k] - mu;
    gz[row * D + k] = (gr[k] * ln_a[k] - mg) / d - c * coef;
    zhat[row * D + k] = c / d;
  }
}

// out[j] = sum_n A[n][j] (* B[n][j]): 64 columns x 16 row slices per workgroup, fixed
// summation order (deterministic).
__global__ __launch_bounds__(1024) void k_colsum(const float* __restrict__ A, const float* __restrict__ B,
                                                 int64_t n_rows, int width, float* __restrict__ out) {
  __shared__ float part[16][64];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  const int64_t r0 = sl * n_rows / 16, r1 = (sl + 1) * n_rows / 16;
  float t = 0.0f;
  if (j < width)
    for (int64_t n = r0; n < r1; ++n) t += B ? A[n * width + j] * B[n * width + j] : A[n * width + j];
  part[sl][c] = t;
  __syncthreads();
  if (sl == 0 && j < width) {
    float s = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += part[q][c];
    out[j] = s;
  }
}

// Spectral-norm chain rule (one workgroup per matrix; GW may alias G): G = dL/d(W/s) ->
// dL/dW = G / s - <G, W> / s^2 * u v^T   (u, v, s: the forward's values, spectral_norm.py:85-89).
__global__ __launch_bounds__(1024) void k_sn_grad(const float* G, const float* __restrict__ W,
                                                  const float* __restrict__ u, const float* __restrict__ v,
                                                  const float* __restrict__ sigma, int out, int in, float* GW) {
  __shared__ float red[16];
  const int64_t n = (int64_t)out * in;
  float t = 0.0f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) t += G[i] * W[i];
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) t += __shfl_xor(t, sh);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  float dot = 0.0f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) dot += red[w];
  const float s = *sigma, c = dot / (s * s);
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) GW[i] = G[i] / s - c * u[i / in] * v[i % in];
}

// C (M x N) = A B / (*div if div), strided operands (the split-K GEMM of gemm.hip)
static int gemm(hipStream_t st, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                int M, int N, int64_t K, const float* div, float* C) {
  return gemm_launch(st, A, sam, sak, B, sbk, sbn, M, N, K, div, nullptr, C, nullptr, nullptr);
}

}  // namespace mmre

using namespace mmre;

// Forward workspace: mat-vec scratch (3 x 2048) + sigma[3] (at 3 * 2048) + the activations
// and W_hat when the caller keeps none.
static int64_t acts_floats(int64_t n, int in0, int o0, int o1, int o2) {
  return n * ((int64_t)in0 + o0 + o1 + o2) + (int64_t)o0 * in0 + (int64_t)o1 * o0 + (int64_t)o2 * o1;
}

extern "C" int64_t mmre_generator_workspace(int64_t n_rows, int in0, int out0, int out1, int out2) {
  return 3 * 2048 + 16 + acts_floats(n_rows, in0, out0, out1, out2);
}

extern "C" int64_t mmre_generator_acts_size(int64_t n_rows, int in0, int out0, int out1, int out2) {
  return acts_floats(n_rows, in0, out0, out1, out2);
}

extern "C" int mmre_generator_forward_save(const float* d_noise, int noise_dim, const float* d_cls, int cls_dim,
                                           int64_t n_rows, const float* d_w0, const float* d_b0, float* d_u0,
                                           float* d_v0, int out0, const float* d_w1, const float* d_b1, float* d_u1,
                                           float* d_v1, int out1, const float* d_w2, const float* d_b2, float* d_u2,
                                           float* d_v2, int out2, const float* d_ln_a, const float* d_ln_b,
                                           float ln_eps, int power_iteration, float sn_eps, float* d_out,
                                           float* d_work, float* d_acts, void* stream) {
  if (!d_noise || !d_cls || !d_w0 || !d_b0 || !d_u0 || !d_v0 || !d_w1 || !d_b1 || !d_u1 || !d_v1 || !d_w2 || !d_b2 ||
      !d_u2 || !d_v2 || !d_ln_a || !d_ln_b || !d_out || !d_work)
    return MMRE_ERR_ARG;
  const int in0 = noise_dim + cls_dim;
  if (n_rows <= 0 || noise_dim < 0 || cls_dim <= 0 || out0 <= 0 || out1 <= 0 || out2 <= 0) return MMRE_ERR_ARG;
  if (in0 > 1024 || out0 > 1024 || out1 > 1024 || out2 > 1024) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  float* sigma = d_work + 3 * 2048;
  float* acts = d_acts ? d_acts : d_work + 3 * 2048 + 16;
  float* x0 = acts;
  float* h1 = x0 + n_rows * in0;
  float* h2 = h1 + n_rows * out0;
  float* h3 = h2 + n_rows * out1;
  float* wh0 = h3 + n_rows * out2;
  float* wh1 = wh0 + (int64_t)out0 * in0;
  float* wh2 = wh1 + (int64_t)out1 * out0;
  SNLayer l0{d_w0, d_u0, d_v0, out0, in0}, l1{d_w1, d_u1, d_v1, out1, out0}, l2{d_w2, d_u2, d_v2, out2, out1};
  hipLaunchKernelGGL(k_sn_sigma, dim3(3), dim3(SN_T), 0, st, l0, l1, l2, power_iteration, sn_eps, sigma, d_work);
  MMRE_CHECK_LAUNCH();
  const int64_t nw = (int64_t)out0 * in0 + (int64_t)out1 * out0 + (int64_t)out2 * out1;
  hipLaunchKernelGGL(k_sn_scale, dim3((unsigned)((nw + 255) / 256 < 2048 ? (nw + 255) / 256 : 2048)), dim3(256), 0, st,
                     d_w0, (int64_t)out0 * in0, d_w1, (int64_t)out1 * out0, d_w2, (int64_t)out2 * out1, sigma, wh0);
  MMRE_CHECK_LAUNCH();
  const int64_t nx = n_rows * in0;
  hipLaunchKernelGGL(k_gen_concat, dim3((unsigned)((nx + 255) / 256 < 4096 ? (nx + 255) / 256 : 4096)), dim3(256), 0,
                     st, d_noise, noise_dim, d_cls, cls_dim, n_rows, x0);
  MMRE_CHECK_LAUNCH();
  // x W_hat^T + b: B(k, n) = W_hat[n][k]
  int rc;
  if ((rc = gemm_launch(st, x0, in0, 1, wh0, 1, in0, n_rows, out0, in0, nullptr, d_b0, h1, nullptr, nullptr))) return rc;
  if ((rc = gemm_launch(st, h1, out0, 1, wh1, 1, out0, n_rows, out1, out0, nullptr, d_b1, h2, nullptr, nullptr)))
    return rc;
  if ((rc = gemm_launch(st, h2, out1, 1, wh2, 1, out1, n_rows, out2, out1, nullptr, d_b2, h3, nullptr, nullptr)))
    return rc;
  hipLaunchKernelGGL(k_gen_ln, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, st, h3, d_ln_a, d_ln_b, ln_eps,
                     n_rows, out2, d_out);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_generator_forward(const float* d_noise, int noise_dim, const float* d_cls, int cls_dim,
                                      int64_t n_rows, const float* d_w0, const float* d_b0, float* d_u0, float* d_v0,
                                      int out0, const float* d_w1, const float* d_b1, float* d_u1, float* d_v1,
                                      int out1, const float* d_w2, const float* d_b2, float* d_u2, float* d_v2,
                                      int out2, const float* d_ln_a, const float* d_ln_b, float ln_eps,
                                      int power_iteration, float sn_eps, float* d_out, float* d_work, void* stream) {
  return mmre_generator_forward_save(d_noise, noise_dim, d_cls, cls_dim, n_rows, d_w0, d_b0, d_u0, d_v0, out0, d_w1,
                                     d_b1, d_u1, d_v1, out1, d_w2, d_b2, d_u2, d_v2, out2, d_ln_a, d_ln_b, ln_eps,
                                     power_iteration, sn_eps, d_out, d_work, nullptr, stream);
}

extern "C" int64_t mmre_generator_backward_workspace(int64_t n_rows, int in0, int out0, int out1, int out2) {
  (void)in0;
  return n_rows * (2 * (int64_t)out2 + out1 + out0);
}

extern "C" int mmre_generator_backward(const float* d_gout, int64_t n_rows, int in0, int out0, int out1, int out2,
                                       const float* d_acts, const float* d_sigma, const float* d_w0,
                                       const float* d_u0, const float* d_v0, const float* d_w1, const float* d_u1,
                                       const float* d_v1, const float* d_w2, const float* d_u2, const float* d_v2,
                                       const float* d_ln_a, float ln_eps, float* d_gw0, float* d_gb0, float* d_gw1,
                                       float* d_gb1, float* d_gw2, float* d_gb2, float* d_gln_a, float* d_gln_b,
                                       float* d_work, void* stream) {
  const void* need[] = {d_gout, d_acts, d_sigma, d_w0, d_u0, d_v0, d_w1, d_u1, d_v1, d_w2, d_u2, d_v2, d_ln_a,
                        d_gw0, d_gb0, d_gw1, d_gb1, d_gw2, d_gb2, d_gln_a, d_gln_b, d_work};
  for (const void* p : need)
    if (!p) return MMRE_ERR_ARG;
  if (n_rows <= 0 || in0 <= 0 || out0 <= 0 || out1 <= 0 || out2 <= 0) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const float* x0 = d_acts;
  const float* h1 = x0 + n_rows * in0;
  const float* h2 = h1 + n_rows * out0;
  const float* h3 = h2 + n_rows * out1;
  const float* wh0 = h3 + n_rows * out2;  // W_hat = W_orig / sigma of the forward
  const float* wh1 = wh0 + (int64_t)out0 * in0;
  const float* wh2 = wh1 + (int64_t)out1 * out0;
  (void)wh0;
  float* gz = d_work;                 // (N, out2)  dL/dh3
  float* zhat = gz + n_rows * out2;   // (N, out2)
  float* g2 = zhat + n_rows * out2;   // (N, out1)  dL/dh2
  float* g1 = g2 + n_rows * out1;     // (N, out0)  dL/dh1
  hipLaunchKernelGGL(k_gen_ln_bwd, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, st, d_gout, h3, d_ln_a, ln_eps,
                     n_rows, out2, gz, zhat);
  MMRE_CHECK_LAUNCH();
  auto colsum = [&](const float* A, const float* B, int width, float* out) -> int {
    hipLaunchKernelGGL(k_colsum, dim3((unsigned)((width + 63) / 64)), dim3(1024), 0, st, A, B, n_rows, width, out);
    MMRE_CHECK_LAUNCH();
    return MMRE_OK;
  };
  int rc;
  if (out2 == 1) {  // LayerNormalization is the identity: no a_2 / b_2 gradient
    MMRE_CHECK(hipMemsetAsync(d_gln_a, 0, sizeof(float), st));
    MMRE_CHECK(hipMemsetAsync(d_gln_b, 0, sizeof(float), st));
  } else {
    if ((rc = colsum(d_gout, zhat, out2, d_gln_a))) return rc;
    if ((rc = colsum(d_gout, nullptr, out2, d_gln_b))) return rc;
  }
  auto sn = [&](float* G, const float* W, const float* u, const float* v, int layer, int o, int i) -> int {
    hipLaunchKernelGGL(k_sn_grad, dim3(1), dim3(1024), 0, st, G, W, u, v, d_sigma + layer, o, i, G);
    MMRE_CHECK_LAUNCH();
    return MMRE_OK;
  };
  const int N = (int)n_rows;
  // layer 2: h3 = h2 (W2/s2)^T + b2
  if ((rc = colsum(gz, nullptr, out2, d_gb2))) return rc;
  if ((rc = gemm(st, gz, 1, out2, h2, out1, 1, out2, out1, n_rows, nullptr, d_gw2))) return rc;   // gz^T h2
  if ((rc = gemm(st, gz, out2, 1, wh2, out1, 1, N, out1, out2, nullptr, g2))) return rc;         // gz W_hat2
  if ((rc = sn(d_gw2, d_w2, d_u2, d_v2, 2, out2, out1))) return rc;
  // layer 1: h2 = h1 (W1/s1)^T + b1
  if ((rc = colsum(g2, nullptr, out1, d_gb1))) return rc;
  if ((rc = gemm(st, g2, 1, out1, h1, out0, 1, out1, out0, n_rows, nullptr, d_gw1))) return rc;
  if ((rc = gemm(st, g2, out1, 1, wh1, out0, 1, N, out0, out1, nullptr, g1))) return rc;
  if ((rc = sn(d_gw1, d_w1, d_u1, d_v1, 1, out1, out0))) return rc;
  // layer 0: h1 = x0 (W0/s0)^T + b0 (no input gradient: noise and the frozen encoder's CLS)
  if ((rc = colsum(g1, nullptr, out0, d_gb0))) return rc;
  if ((rc = gemm(st, g1, 1, out0, x0, in0, 1, out0, in0, n_rows, nullptr, d_gw0))) return rc;
  if ((rc = sn(d_gw0, d_w0, d_u0, d_v0, 0, out0, in0))) return rc;
  return MMRE_OK;
}

extern "C" int mmre_sn_weight(const float* d_w, int out, int in, float* d_u, float* d_v, int power_iteration,
                              float eps, float* d_sigma, float* d_u_snap, float* d_v_snap, float* d_w_hat,
                              float* d_work, void* stream) {
  if (!d_w || !d_u || !d_v || !d_sigma || !d_u_snap || !d_v_snap || !d_w_hat || !d_work || out <= 0 || in <= 0)
    return MMRE_ERR_ARG;
  if (out > 1024 || in > 1024) return MMRE_ERR_SHAPE;
  SNLayer L{d_w, d_u, d_v, out, in};
  hipLaunchKernelGGL(k_sn_weight, dim3(1), dim3(SN_T), 0, (hipStream_t)stream, L, power_iteration, eps, d_sigma,
                     d_work, d_u_snap, d_v_snap, d_w_hat);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_sn_weight_backward(const float* d_g, const float* d_w, int out, int in, const float* d_u,
                                       const float* d_v, const float* d_sigma, float* d_gw, void* stream) {
  if (!d_g || !d_w || !d_u || !d_v || !d_sigma || !d_gw || out <= 0 || in <= 0) return MMRE_ERR_ARG;
  hipLaunchKernelGGL(k_sn_grad, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_g, d_w, d_u, d_v, d_sigma, out, in,
                     d_gw);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_layernorm_unbiased(const float* d_z, int64_t n_rows, int d, const float* d_a, const float* d_b,
                                       float eps, float* d_out, void* stream) {
  if (!d_z || !d_a || !d_b || !d_out || n_rows < 0 || d <= 0) return MMRE_ERR_ARG;
  if (n_rows == 0) return MMRE_OK;
  hipLaunchKernelGGL(k_gen_ln, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, d_z, d_a, d_b,
                     eps, n_rows, d, d_out);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_layernorm_unbiased_backward(const float* d_g, const float* d_z, int64_t n_rows, int d,
                                                const float* d_a, float eps, float* d_gz, float* d_ga, float* d_gb,
                                                float* d_work, void* stream) {
  if (!d_g || !d_z || !d_a || !d_gz || !d_ga || !d_gb || !d_work || n_rows <= 0 || d <= 0) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_gen_ln_bwd, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, st, d_g, d_z, d_a, eps, n_rows,
                     d, d_gz, d_work);
  MMRE_CHECK_LAUNCH();
  const dim3 g((unsigned)((d + 63) / 64));
  hipLaunchKernelGGL(k_colsum, g, dim3(1024), 0, st, d_g, d_work, n_rows, d, d_ga);
  MMRE_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_colsum, g, dim3(1024), 0, st, d_g, nullptr, n_rows, d, d_gb);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
