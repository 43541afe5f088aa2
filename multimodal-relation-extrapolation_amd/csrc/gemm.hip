// gemm.hip -- small fp32 GEMM for the ZSL GAN step's Discriminator (module/zsl_module.py:112-138)
// and its autograd (mmre/gemm.py): x W^T of the spectral-normalised layers, the class scores
// against the centroids, and their gradients -- including the gradient penalty's double
// backward (module/utils.py:692-707). The shapes are 200-512 on every side: a library GEMM
// picks one 256 x 224 tile and runs the whole product on ONE workgroup (120 us for a
// 200 x 200 x 512 weight gradient, measured in the GAN step's trace). Here the output is cut in
// 32 x 32 tiles, one wave each, and K is split until the chip holds about one wave per SIMD;
// the K slices' partial tiles are summed in slice order by a second launch (deterministic).
//   C (M x N) = A (M x K) B (K x N), A(m, k) = A[m sam + k sak], B(k, n) = B[k sbk + n sbn]
// (any strides: transposed operands are views).
#include "mmre_common.h"

namespace mmre {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int GK = 8;  // K pairs per operand load round

// One wave per (32 x 32 tile, K slice). Lane (i, kh) feeds row / column i and the kh-th k of
// each MFMA pair; out = C when S == 1, else the slice's partial tile in work[s].
__global__ __launch_bounds__(64) void k_gemm_slice(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                   const float* __restrict__ B, int64_t sbk, int64_t sbn, int M,
                                                   int N, int64_t K, int64_t kslice, float* __restrict__ out) {
  const int lane = threadIdx.x, i = lane & 31, kh = lane >> 5;
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32, s = blockIdx.z;
  const int64_t k_lo = (int64_t)s * kslice, k_hi = min(K, k_lo + kslice);
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
  float* o = out + (int64_t)s * M * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
    if (row < M && nv) o[(int64_t)row * N + n] = acc[r];
  }
}

// C = sum over the S slices, in slice order.
__global__ __launch_bounds__(256) void k_gemm_reduce(const float* __restrict__ work, int64_t mn, int S,
                                                     float* __restrict__ C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= mn) return;
  float v = work[i];
  for (int s = 1; s < S; ++s) v += work[(int64_t)s * mn + i];
  C[i] = v;
}

int splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + 31) / 32) * ((N + 31) / 32);
  int64_t s = 1024 / (tiles > 0 ? tiles : 1);  // about one wave per SIMD (256 CUs x 4)
  const int64_t by_k = K / 64;                  // slices of at least 64 k
  if (s > by_k) s = by_k;
  if (s > 16) s = 16;
  return s < 1 ? 1 : (int)s;
}

}  // namespace
}  // namespace mmre

using namespace mmre;

extern "C" int mmre_gemm_splits(int64_t m, int64_t n, int64_t k) {
  if (m < 0 || n < 0 || k < 0) return -1;
  return splits(m, n, k);
}

extern "C" int mmre_gemm_f32(const float* d_a, int64_t sam, int64_t sak, const float* d_b, int64_t sbk, int64_t sbn,
                             int64_t m, int64_t n, int64_t k, float* d_work, int64_t work_floats, float* d_c,
                             void* stream) {
  if (m < 0 || n < 0 || k < 0 || m > 0x7fffffe0LL || n > 0x7fffffe0LL || !d_c || (k > 0 && (!d_a || !d_b)))
    return MMRE_ERR_ARG;
  if (m == 0 || n == 0) return MMRE_OK;
  hipStream_t st = (hipStream_t)stream;
  const int S = splits(m, n, k);
  if (S > 1 && (!d_work || work_floats < (int64_t)S * m * n)) return MMRE_ERR_WORKSPACE;
  const int64_t kslice = (k + S - 1) / S;
  const dim3 g((unsigned)((n + 31) / 32), (unsigned)((m + 31) / 32), (unsigned)S);
  hipLaunchKernelGGL(k_gemm_slice, g, dim3(64), 0, st, d_a, sam, sak, d_b, sbk, sbn, (int)m, (int)n, k, kslice,
                     S > 1 ? d_work : d_c);
  if (S > 1)
    hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((m * n + 255) / 256)), dim3(256), 0, st, d_work, m * n, S, d_c);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
