// gemm.hip -- small fp32 GEMM of the ZSL GAN step: the Discriminator's products
// (module/zsl_module.py:112-138) and their autograd (mmre/gemm.py) -- the gradient penalty's
// double backward included (module/utils.py:692-707) -- and the generator's SN linears and
// their weight gradients (generator.hip). Every side is 200-512: a library GEMM picks one
// 256 x 224 tile and runs the whole product on ONE workgroup (120 us for a 200 x 200 x 512
// weight gradient, measured in the GAN step's trace). Here each 32 x 32 output tile is one
// workgroup of S waves (S <= 8), wave w computing K slice w on v_mfma_f32_32x32x2_f32; the S
// partial tiles meet in LDS and the same workgroup sums them in slice order (deterministic),
// so one launch does the product and the split-K reduction.
//   C (M x N) = alpha A (M x K) B (K x N) + bias, A(m, k) = A[m sam + k sak],
//   B(k, n) = B[k sbk + n sbn]  (any strides: transposed operands are views);
// alpha = 1 / *div when div is given; bias (N) optional. Optional epilogue for the
// spectral-norm chain rule: tile_dot[tile] = sum over the tile of C * Wd (Wd row-major M x N),
// in a fixed order.
#include "mmre_common.h"

namespace mmre {

typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int GK = 8;  // K pairs per operand load round
constexpr int GEMM_MAXS = 8;

__global__ __launch_bounds__(64 * GEMM_MAXS) void k_gemm(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                         const float* __restrict__ B, int64_t sbk, int64_t sbn,
                                                         int M, int N, int64_t K, int64_t kslice,
                                                         const float* __restrict__ div,
                                                         const float* __restrict__ bias, float* __restrict__ C,
                                                         const float* __restrict__ Wd, float* __restrict__ tile_dot) {
  __shared__ float part[GEMM_MAXS][32 * 32];
  __shared__ float red[GEMM_MAXS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, S = blockDim.x >> 6;
  const int i = lane & 31, kh = lane >> 5;
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32;
  const int64_t k_lo = (int64_t)w * kslice, k_hi = min(K, k_lo + kslice);
  const int m = m0 + i, n = n0 + i;
  const bool mv = m < M, nv = n < N;
  const float* ap = A + (mv ? (int64_t)m * sam : 0);
  const float* bp = B + (nv ? (int64_t)n * sbn : 0);
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  for (int64_t k0 = k_lo; k0 < k_hi; k0 += 2 * GK) {
    float a[GK], b[GK];
#pragma unroll
    for (int j = 0; j < GK; ++j) {
      const int64_t k = k0 + 2 * j + kh;
      const bool kv = k < k_hi;
      a[j] = (mv && kv) ? ap[k * sak] : 0.0f;
      b[j] = (nv && kv) ? bp[k * sbk] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < GK; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) part[w][((r & 3) + 8 * (r >> 2) + 4 * kh) * 32 + i] = acc[r];
  __syncthreads();
  const float alpha = div ? 1.0f / *div : 1.0f;
  float dot = 0.0f;
  for (int e = threadIdx.x; e < 32 * 32; e += blockDim.x) {
    float v = part[0][e];
    for (int s = 1; s < S; ++s) v += part[s][e];
    const int row = m0 + (e >> 5), col = n0 + (e & 31);
    if (row < M && col < N) {
      if (div) v *= alpha;
      if (bias) v += bias[col];
      C[(int64_t)row * N + col] = v;
      if (Wd) dot += v * Wd[(int64_t)row * N + col];
    }
  }
  if (tile_dot) {
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) dot += __shfl_xor(dot, sh);
    if (lane == 0) red[w] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.0f;
      for (int s = 0; s < S; ++s) t += red[s];
      tile_dot[blockIdx.y * gridDim.x + blockIdx.x] = t;
    }
  }
}

int64_t gemm_tiles(int64_t M, int64_t N) { return ((M + 31) / 32) * ((N + 31) / 32); }

int gemm_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = gemm_tiles(M, N);
  int64_t s = (1024 + tiles - 1) / (tiles > 0 ? tiles : 1);  // about one wave per SIMD (256 CUs x 4)
  const int64_t by_k = K / 32;                               // slices of at least 32 k
  if (s > by_k) s = by_k;
  if (s > GEMM_MAXS) s = GEMM_MAXS;
  return s < 1 ? 1 : (int)s;
}

int gemm_launch(hipStream_t st, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                int64_t M, int64_t N, int64_t K, const float* div, const float* bias, float* C, const float* Wd,
                float* tile_dot) {
  if (M == 0 || N == 0) return MMRE_OK;
  const int S = gemm_splits(M, N, K);
  const int64_t kslice = (K + S - 1) / S;
  const dim3 g((unsigned)((N + 31) / 32), (unsigned)((M + 31) / 32));
  hipLaunchKernelGGL(k_gemm, g, dim3(64 * S), 0, st, A, sam, sak, B, sbk, sbn, (int)M, (int)N, K, kslice, div, bias,
                     C, Wd, tile_dot);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

}  // namespace mmre

using namespace mmre;

extern "C" int mmre_gemm_splits(int64_t m, int64_t n, int64_t k) {
  if (m < 0 || n < 0 || k < 0) return -1;
  return gemm_splits(m, n, k);
}

extern "C" int mmre_gemm_f32(const float* d_a, int64_t sam, int64_t sak, const float* d_b, int64_t sbk, int64_t sbn,
                             int64_t m, int64_t n, int64_t k, const float* d_bias, float* d_c, void* stream) {
  if (m < 0 || n < 0 || k < 0 || m > 0x7fffffe0LL || n > 0x7fffffe0LL || !d_c || (k > 0 && (!d_a || !d_b)))
    return MMRE_ERR_ARG;
  return gemm_launch((hipStream_t)stream, d_a, sam, sak, d_b, sbk, sbn, m, n, k, nullptr, d_bias, d_c, nullptr,
                     nullptr);
}
