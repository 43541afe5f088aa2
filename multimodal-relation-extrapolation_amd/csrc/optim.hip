// optim.hip -- plain SGD step over a list of parameter tensors in one launch.
//
// Replaces, for the reference's default optimizer (OpenKE Trainer.py:82-86, optim.SGD with
// no momentum / weight decay), torch's multi-tensor SGD kernel after the fused gradient:
// p <- p - lr g elementwise as one fma with lr in float32 -- bit-identical to torch's default
// (foreach) SGD step on this ROCm build, which is the same fma (scripts/probes/sgd_rounding.py),
// float4 streams over every tensor, one workgroup per
// 4,096 elements so the whole table is in flight at once (torch's multi_tensor_apply gives a
// 2.9 M-float table ~45 workgroups).
#include "mmre_common.h"

namespace mmre {

constexpr int SGD_MAX_T = 8;

struct SgdList {
  float* p[SGD_MAX_T];
  const float* g[SGD_MAX_T];
  int64_t begin[SGD_MAX_T + 1];  // tensor t owns float4 chunks [begin[t], begin[t + 1])
  int64_t n[SGD_MAX_T];          // elements
  int count;
};

__global__ __launch_bounds__(256) void k_sgd_step(SgdList L, float lr) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // float4 chunk
  if (c >= L.begin[L.count]) return;
  int t = 0;
#pragma unroll
  for (int i = 1; i < SGD_MAX_T; ++i) t += (i < L.count && c >= L.begin[i]) ? 1 : 0;
  const int64_t e = 4 * (c - L.begin[t]);
  float* p = L.p[t];
  const float* g = L.g[t];
  if (e + 4 <= L.n[t]) {
    float4 pv = *reinterpret_cast<const float4*>(p + e);
    const float4 gv = *reinterpret_cast<const float4*>(g + e);
    pv.x = __builtin_fmaf(-lr, gv.x, pv.x);
    pv.y = __builtin_fmaf(-lr, gv.y, pv.y);
    pv.z = __builtin_fmaf(-lr, gv.z, pv.z);
    pv.w = __builtin_fmaf(-lr, gv.w, pv.w);
    *reinterpret_cast<float4*>(p + e) = pv;
  } else {
    for (int64_t k = e; k < L.n[t]; ++k) p[k] = __builtin_fmaf(-lr, g[k], p[k]);
  }
}

}  // namespace mmre

using namespace mmre;

extern "C" int mmre_sgd_step(float* const* params, const float* const* grads, const int64_t* numel, int count,
                             float lr, void* stream) {
  if (!params || !grads || !numel || count <= 0 || count > SGD_MAX_T) return MMRE_ERR_ARG;
  SgdList L{};
  L.count = count;
  L.begin[0] = 0;
  for (int t = 0; t < count; ++t) {
    if (!params[t] || !grads[t] || numel[t] < 0) return MMRE_ERR_ARG;
    if ((reinterpret_cast<uintptr_t>(params[t]) | reinterpret_cast<uintptr_t>(grads[t])) & 15) return MMRE_ERR_ARG;
    L.p[t] = params[t];
    L.g[t] = grads[t];
    L.n[t] = numel[t];
    L.begin[t + 1] = L.begin[t] + (numel[t] + 3) / 4;
  }
  for (int t = count; t < SGD_MAX_T; ++t) L.begin[t + 1] = L.begin[count];
  const int64_t chunks = L.begin[count];
  if (chunks == 0) return MMRE_OK;
  hipLaunchKernelGGL(k_sgd_step, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, (hipStream_t)stream, L, lr);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
