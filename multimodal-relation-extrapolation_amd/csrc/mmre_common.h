// mmre_common.h -- shared device helpers for the MI355X (gfx950) kernels.
//
// Every kernel in this library is compiled with -ffp-contract=off: floating-point
// results follow the "canonical arithmetic" (CA) written out in DESIGN.md §3, so a
// score computed by the all-entity sweep, by the truth kernel and by the filter
// correction kernel is the same bit pattern, and ranks are exact integers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmre.h"

#define MMRE_CHECK(expr)                                                  \
  do {                                                                    \
    hipError_t _e = (expr);                                               \
    if (_e != hipSuccess) return MMRE_ERR_HIP_BASE + (int)_e;             \
  } while (0)

#define MMRE_CHECK_LAUNCH() MMRE_CHECK(hipGetLastError())

namespace mmre {

constexpr int kWave = 64;

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Small split-K fp32 GEMM (gemm.hip): C = A B / (*div if div) + bias, strided operands;
// tile_dot[t] = sum over output tile t of C * Wd when both are given. One launch.
int gemm_launch(hipStream_t st, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                int64_t M, int64_t N, int64_t K, const float* div, const float* bias, float* C, const float* Wd,
                float* tile_dot);
int64_t gemm_tiles(int64_t M, int64_t N);

// Row width of the k-major entity / query planes for a model.
__host__ __device__ inline int model_k(int model, int dim) {
  return (model == MMRE_COMPLEX || model == MMRE_ROTATE) ? 2 * dim : dim;
}

// Prediction transform applied to a raw score: what OpenKE's model.predict returns.
//   0: s (TransE)   1: m - (m - s) (TransE with margin)   2: -s (DistMult/ComplEx)
//   3: -(m - s) (RotatE)   4: m - s (forward() of TransE with margin / RotatE)
//                                      (TransE.py:88-110, DistMult.py:70-72, RotatE.py:86-91)
__device__ __forceinline__ float apply_pred(int kind, float m, float s) {
  switch (kind) {
    case 0: return s;
    case 1: return m - (m - s);
    case 2: return -s;
    case 3: return -(m - s);
    default: return m - s;
  }
}

// apply_pred with the kind fixed at compile time (sweep epilogues: no per-element branch)
template <int K>
struct PredK {
  float m;
  __device__ __forceinline__ float operator()(float s) const {
    if constexpr (K == 0) return s;
    else if constexpr (K == 1) return m - (m - s);
    else if constexpr (K == 2) return -s;
    else if constexpr (K == 3) return -(m - s);
    else return m - s;
  }
};
// ... and decoded once into uniform selects, for the other kinds. Same operations, bit-identical.
struct PredFn {
  float m;
  bool use_m, twice;  // x = use_m ? m - s : s; x = twice ? m - x : x
  uint32_t neg;       // sign-bit flip: exactly IEEE negation
  __device__ __forceinline__ explicit PredFn(int kind, float margin)
      : m(margin), use_m(kind == 1 || kind == 3 || kind >= 4), twice(kind == 1),
        neg((kind == 2 || kind == 3) ? 0x80000000u : 0u) {}
  __device__ __forceinline__ float operator()(float s) const {
    float x = use_m ? m - s : s;
    x = twice ? m - x : x;
    return __uint_as_float(__float_as_uint(x) ^ neg);
  }
};
// PredSel<K>: the compile-time kind K, or (K = -1) the run-time kind decoded into selects
template <int K>
struct PredSel : PredK<K> {
  __device__ __forceinline__ PredSel(int, float margin) : PredK<K>{margin} {}
};
template <>
struct PredSel<-1> : PredFn {
  __device__ __forceinline__ PredSel(int kind, float margin) : PredFn(kind, margin) {}
};

// Canonical single-precision sincos: Cody-Waite reduction by pi/2 in fma form and
// cephes minimax polynomials on [-pi/4, pi/4]. Same operation sequence as the CA
// specification, so the RotatE rotation is reproducible bit-for-bit.
__device__ __forceinline__ void canon_sincos(float x, float* s_out, float* c_out) {
  const float TWO_OVER_PI = 0.636619772367581343f;
  const float P1 = 1.57079637050628662109375f;
  const float P2 = -4.37113900018624283e-8f;
  const float P3 = -1.71512986e-15f;
  float j = rintf(x * TWO_OVER_PI);
  float r = __builtin_fmaf(-j, P1, x);
  r = __builtin_fmaf(-j, P2, r);
  r = __builtin_fmaf(-j, P3, r);
  float z = r * r;
  float sp = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  float sv = __builtin_fmaf(sp * z, r, r);
  float cp = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                            4.166664568298827e-2f);
  float cv = __builtin_fmaf(cp * z, z, __builtin_fmaf(-0.5f, z, 1.0f));
  int q = ((int)j) & 3;
  float s, c;
  if (q == 0) { s = sv; c = cv; }
  else if (q == 1) { s = cv; c = -sv; }
  else if (q == 2) { s = -sv; c = -cv; }
  else { s = -cv; c = sv; }
  *s_out = s;
  *c_out = c;
}

}  // namespace mmre
