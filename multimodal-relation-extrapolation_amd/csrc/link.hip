// link.hip -- link prediction on MI355X: the all-entity score sweep with a fused
// rank epilogue (replaces Tester.run_link_prediction's per-query loop,
// OpenKE/openke/config/Tester.py:70-91, with getHeadBatch/getTailBatch Test.h:36-53,
// model.predict and testHead/testTail Test.h:65-192).
//
// Data layout in HBM: the entity table and the query vectors are
// stored "k-major" -- plane[k][n] with n padded to 128 -- so that one K step of a
// 128-wide tile is a single contiguous 512-byte row: coalesced 16-B loads into LDS,
// conflict-free LDS reads, no transposes inside the hot loop.
//
// Kernels (per evaluation, one stream):
//   k_prep_rows       table -> k-major plane + row-major copy (F.normalize for TransE norm_flag)
//   k_prep_queries    (h, r, t, mode) -> k-major query vectors (+ truth ids)
//   k_truth_filter    pred(truth) per query (the sweep's arithmetic) and the filtered-rank
//                     correction, one workgroup per filter group (queries sharing a list)
//   k_sweep_valu      TransE L1/L2, RotatE: VALU 8x8 register micro-tiles
//   k_sweep_mfma      DistMult/ComplEx: v_mfma_f32_32x32x2_f32, register-counter epilogue
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "mmre_common.h"

namespace mmre {

typedef float f32x2 __attribute__((ext_vector_type(2)));  // a v_pk_*_f32 operand pair

constexpr int TQ = 128;   // queries per workgroup tile
constexpr int TE = 128;   // entities per workgroup tile
constexpr int KC = 8;     // K rows per LDS stage
constexpr int NT = 256;   // threads per workgroup

// rows per plane: TransE/DistMult use one plane of plane_rows(model, d) rows;
// ComplEx/RotatE use two planes (re, im) of plane_rows(model, d) rows each.
// DistMult/ComplEx planes are padded to whole 16-row LDS stages of the MFMA sweep (zero rows
// add exact zeros to the fma chain; a 32-row stage measured slower: C3 1.27 vs 1.18 ms, C5
// 37.9 vs 36.6 ms at 248 VGPRs); TransE/RotatE to the VALU sweep's 8.
constexpr int KS_MFMA = 16;
__host__ __device__ inline int n_planes(int model) { return (model == MMRE_COMPLEX || model == MMRE_ROTATE) ? 2 : 1; }
__host__ __device__ inline bool mfma_model(int model) { return model == MMRE_DISTMULT || model == MMRE_COMPLEX; }
// MFMA planes: K = n_planes x plane_rows a multiple of 16 (ComplEx d = 200: 2 x 200, no padding)
inline int plane_rows(int model, int dim) {
  return (int)round_up(dim, !mfma_model(model) ? KC : KS_MFMA / n_planes(model));
}

// ------------------------------------------------------------------ prep ----
// Both prep kernels stage a block of rows through LDS (row stride kt+1: odd, so the
// per-row sequential reads and the column-wise k-major writes are bank-conflict free):
// global reads are contiguous row segments, global writes are contiguous in both the
// row-major and the k-major layout.

// Rows per LDS block for a row width kt: a power of two <= 16 (so it divides the 256
// threads; 64-B k-major write runs, ~900 workgroups at |E| = 14k) with <= 64 KB of LDS.
__host__ inline int stage_rows(int kt) {
  int rb = 16;
  while (rb > 1 && (int64_t)rb * (kt + 1) * 4 > 64 * 1024) rb >>= 1;
  return rb;
}

// Value k (< np*kp) of source row e in the plane layout [re 0..kp) [im kp..2kp).
__device__ __forceinline__ float plane_src(int model, const float* __restrict__ src, const float* __restrict__ src_im,
                                           int64_t e, int dim, int kp, int k) {
  const int pl = k >= kp;
  const int kk = k - pl * kp;
  if (kk >= dim) return 0.0f;
  if (model == MMRE_COMPLEX) return (pl ? src_im : src)[e * dim + kk];
  if (model == MMRE_ROTATE) return src[e * 2 * dim + pl * dim + kk];  // RotatE rows [re | im] (RotatE.py:48-49)
  return src[e * dim + kk];
}

// Thread layouts of the staging kernels (256 threads): row phases use 8 row slots x 32
// lanes along k (coalesced row segments, independent loads per thread); the k-major write
// uses rb lanes along the rows x 256/rb k slots (contiguous rb-float runs per k).
__device__ __forceinline__ void write_k_major(const float* lds, int ls, int rb, int kt, float* __restrict__ out,
                                              int64_t pad, int64_t r0) {
  const int i = threadIdx.x % rb, ks = threadIdx.x / rb, kstep = 256 / rb;
  const int64_t e = r0 + i;
  if (e >= pad) return;
#pragma unroll 4
  for (int k = ks; k < kt; k += kstep) out[(int64_t)k * pad + e] = lds[i * ls + k];
}

// Table rows -> (optional) k-major planes out_km[kt][pad] and row-major rows[n][rw]
// (rw <= kt). TransE with norm_flag: F.normalize(x, 2, -1) = x / max(||x||_2, 1e-12)
// (TransE.py:63-66), ||x|| from the canonical sequential sum of squares.
__device__ __forceinline__ void prep_rows_body(int model, int norm_flag, const float* __restrict__ src,
                                               const float* __restrict__ src_im, int64_t n, int dim, int kp, int rb,
                                               float* __restrict__ out_km, int64_t pad, float* __restrict__ rows,
                                               int rw, float* lds, float* s_norm) {
  const int kt = n_planes(model) * kp, ls = kt + 1;
  const int lane = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const int64_t e0 = (int64_t)blockIdx.x * rb;
  for (int i = slot; i < rb; i += 8) {
    const int64_t e = e0 + i;
    float* x = lds + i * ls;
#pragma unroll 4
    for (int k = lane; k < kt; k += 32) x[k] = e < n ? plane_src(model, src, src_im, e, dim, kp, k) : 0.0f;
  }
  __syncthreads();
  const bool transe = model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2;
  if (transe && norm_flag) {
    if (threadIdx.x < rb) {
      const float* x = lds + threadIdx.x * ls;
      float ss = 0.0f;  // canonical sequential order; LDS reads batched 16 per round
      int k = 0;
      for (; k + 16 <= dim; k += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = x[k + u];
#pragma unroll
        for (int u = 0; u < 16; ++u) ss = ss + v[u] * v[u];
      }
      for (; k < dim; ++k) ss = ss + x[k] * x[k];
      const float nr = sqrtf(ss);
      s_norm[threadIdx.x] = nr < 1e-12f ? 1e-12f : nr;
    }
    __syncthreads();
    for (int i = slot; i < rb; i += 8) {
      float* x = lds + i * ls;
      const float nr = s_norm[i];
      for (int k = lane; k < kt; k += 32) x[k] = x[k] / nr;
    }
    __syncthreads();
  }
  for (int i = slot; i < rb; i += 8) {
    const int64_t e = e0 + i;
    if (e >= n) break;
    const float* x = lds + i * ls;
#pragma unroll 4
    for (int k = lane; k < rw; k += 32) rows[e * rw + k] = x[k];
  }
  if (out_km) write_k_major(lds, ls, rb, kt, out_km, pad, e0);
}
__global__ __launch_bounds__(256) void k_prep_rows(int model, int norm_flag, const float* __restrict__ src,
                                                   const float* __restrict__ src_im, int64_t n, int dim, int kp,
                                                   int rb, float* __restrict__ out_km, int64_t pad,
                                                   float* __restrict__ rows, int rw) {
  extern __shared__ float lds[];
  __shared__ float s_norm[32];
  prep_rows_body(model, norm_flag, src, src_im, n, dim, kp, rb, out_km, pad, rows, rw, lds, s_norm);
}
// The k-major planes of a table whose row-major copy is the raw table itself (DistMult, d a
// multiple of 16: mmre_link_sweep_bf3_rows), gated: only when *gate != 0 -- the split-bf16
// filter's list overflowed and the exact f32 sweep that reads these planes is about to count.
__global__ __launch_bounds__(256) void k_prep_km_gated(const uint32_t* __restrict__ gate, int model,
                                                       const float* __restrict__ src, int64_t n, int dim, int kp,
                                                       int rb, float* __restrict__ out_km, int64_t pad) {
  extern __shared__ float lds[];
  __shared__ float s_norm[32];
  if (__builtin_amdgcn_readfirstlane(*gate) == 0u) return;
  prep_rows_body(model, 0, src, nullptr, n, dim, kp, rb, out_km, pad, nullptr, 0, lds, s_norm);
}

// Query vectors, one LDS block of rb queries: the anchor rows (t for head_batch, h for
// tail_batch) are copied from the prepared entity rows, combined element-wise with the
// relation row (rel = normalised relation rows for TransE norm_flag), written k-major.
__global__ __launch_bounds__(256) void k_prep_queries(int model, const float* __restrict__ ent_rows,
                                                      const float* __restrict__ rel, const float* __restrict__ rel_im,
                                                      int dim, int kp, int rb, float phase_denom,
                                                      const int64_t* __restrict__ qh, const int64_t* __restrict__ qr,
                                                      const int64_t* __restrict__ qt, const int8_t* __restrict__ qmode,
                                                      int64_t n_query, float* __restrict__ out, int64_t q_pad,
                                                      int32_t* __restrict__ qtrue, float* __restrict__ q_rows,
                                                      int rel_norm) {
  extern __shared__ float lds[];
  __shared__ int64_t s_anchor[32], s_rel[32];
  __shared__ int s_head[32];
  __shared__ float s_rnorm[32];
  const int np = n_planes(model);
  const int kt = np * kp, ls = kt + 1;
  const int lane = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const int64_t q0 = (int64_t)blockIdx.x * rb;
  if (threadIdx.x < rb) {
    const int64_t q = q0 + threadIdx.x;
    int64_t a = -1, r = 0;
    int head = 0;
    if (q < n_query) {
      head = qmode[q] == MMRE_HEAD_BATCH;
      a = head ? qt[q] : qh[q];
      r = qr[q];
      qtrue[q] = (int32_t)(head ? qh[q] : qt[q]);
    }
    s_anchor[threadIdx.x] = a;
    s_rel[threadIdx.x] = r;
    s_head[threadIdx.x] = head;
    if (rel_norm) {  // TransE norm_flag: F.normalize of the relation row (TransE.py:63-66), in
                     // k_prep_rows' canonical order, so r / |r| is bit-identical to its output
      const float* rp = rel + r * dim;
      float ss = 0.0f;
      int k = 0;
      if ((dim & 3) == 0) {  // 16-B aligned rows: 64 values per round trip (a short latency chain)
        for (; k + 64 <= dim; k += 64) {
          float4 v[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) v[u] = reinterpret_cast<const float4*>(rp + k)[u];
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            ss = ss + v[u].x * v[u].x;
            ss = ss + v[u].y * v[u].y;
            ss = ss + v[u].z * v[u].z;
            ss = ss + v[u].w * v[u].w;
          }
        }
      }
      for (; k + 16 <= dim; k += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = rp[k + u];
#pragma unroll
        for (int u = 0; u < 16; ++u) ss = ss + v[u] * v[u];
      }
      for (; k < dim; ++k) ss = ss + rp[k] * rp[k];
      const float nr = sqrtf(ss);
      s_rnorm[threadIdx.x] = nr < 1e-12f ? 1e-12f : nr;
    }
  }
  __syncthreads();
  for (int i = slot; i < rb; i += 8) {
    const int64_t a = s_anchor[i];
    float* x = lds + i * ls;
    const float* src = ent_rows + (a < 0 ? 0 : a) * kt;
#pragma unroll 4
    for (int k = lane; k < kt; k += 32) x[k] = a < 0 ? 0.0f : src[k];
  }
  __syncthreads();
  for (int i = slot; i < rb; i += 8) {
    float* x = lds + i * ls;
    const bool valid = s_anchor[i] >= 0;
    const int64_t r = s_rel[i];
    const bool head = s_head[i];
#pragma unroll 2
    for (int k = lane; k < kp; k += 32) {
      if (!valid || k >= dim) {
        x[k] = 0.0f;
        if (np == 2) x[kp + k] = 0.0f;
        continue;
      }
      if (model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2) {
        // head_batch: score = h + (r - t) -> q = -(r - t); tail_batch: (h + r) - t -> q = h + r
        // (TransE.py:71-74). |q - e| reproduces both element-wise bit-for-bit.
        const float b = rel_norm ? rel[r * dim + k] / s_rnorm[i] : rel[r * dim + k];
        x[k] = head ? -(b - x[k]) : (x[k] + b);
      } else if (model == MMRE_DISTMULT) {  // head: h*(r*t) ; tail: (h*r)*t  (DistMult.py:37-42)
        const float b = rel[r * dim + k];
        x[k] = head ? b * x[k] : x[k] * b;
      } else if (model == MMRE_COMPLEX) {  // ComplEx.py:20-27 regrouped by the candidate entity
        const float rr = rel[r * dim + k], ri = rel_im[r * dim + k];
        const float ar = x[k], ai = x[kp + k];  // anchor (t for head_batch, h for tail_batch)
        if (head) { x[k] = ar * rr + ai * ri; x[kp + k] = ai * rr - ar * ri; }
        else      { x[k] = ar * rr - ai * ri; x[kp + k] = ai * rr + ar * ri; }
      } else {  // RotatE (RotatE.py:51-72): rotate by the relation phase, regrouped per candidate
        float sn, cs;
        canon_sincos(rel[r * dim + k] / phase_denom, &sn, &cs);
        const float ar = x[k], ai = x[kp + k];
        if (head) { x[k] = cs * ar + sn * ai; x[kp + k] = cs * ai - sn * ar; }
        else      { x[k] = ar * cs - ai * sn; x[kp + k] = ar * sn + ai * cs; }
      }
    }
  }
  __syncthreads();
  write_k_major(lds, ls, rb, kt, out, q_pad, q0);
  if (q_rows) {  // row-major copy for the per-group loads of k_truth_filter
    for (int i = slot; i < rb; i += 8) {
      const int64_t q = q0 + i;
      if (q >= n_query) break;
      const float* x = lds + i * ls;
#pragma unroll 4
      for (int k = lane; k < kt; k += 32) q_rows[q * kt + k] = x[k];
    }
  }
}

// A value the compiler cannot see through: what is computed from it is computed where it is
// used, not hoisted out of a loop into a register (or scratch) kept live across the loop.
__device__ __forceinline__ int vgpr_opaque(int x) {
  __asm__ volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ float vgpr_opaque_f(float x) {
  __asm__ volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ uint64_t sgpr_opaque64(uint64_t x) {
  __asm__ volatile("" : "+s"(x));
  return x;
}
__device__ __forceinline__ uint32_t sgpr_opaque(uint32_t x) {
  __asm__ volatile("" : "+s"(x));
  return x;
}
__device__ __forceinline__ int sgpr_opaque(int x) {
  __asm__ volatile("" : "+s"(x));
  return x;
}

// v_writelane_b32 with an immediate lane select (the lane must be a compile-time constant after
// unrolling: the switch folds away). Writes the wave-uniform s into lane `lane` of v.
template <int L>
__device__ __forceinline__ int writelane_c(int v, int s) {
  __asm__ volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s), "n"(L));
  return v;
}
__device__ __forceinline__ int writelane_imm(int v, int s, int lane) {
  switch (lane) {
    case 0: return writelane_c<0>(v, s);
    case 1: return writelane_c<1>(v, s);
    case 2: return writelane_c<2>(v, s);
    case 3: return writelane_c<3>(v, s);
    case 4: return writelane_c<4>(v, s);
    case 5: return writelane_c<5>(v, s);
    case 6: return writelane_c<6>(v, s);
    case 7: return writelane_c<7>(v, s);
    case 8: return writelane_c<8>(v, s);
    case 9: return writelane_c<9>(v, s);
    case 10: return writelane_c<10>(v, s);
    case 11: return writelane_c<11>(v, s);
    case 12: return writelane_c<12>(v, s);
    case 13: return writelane_c<13>(v, s);
    case 14: return writelane_c<14>(v, s);
    case 15: return writelane_c<15>(v, s);
    case 16: return writelane_c<16>(v, s);
    case 17: return writelane_c<17>(v, s);
    case 18: return writelane_c<18>(v, s);
    case 19: return writelane_c<19>(v, s);
    case 20: return writelane_c<20>(v, s);
    case 21: return writelane_c<21>(v, s);
    case 22: return writelane_c<22>(v, s);
    case 23: return writelane_c<23>(v, s);
    case 24: return writelane_c<24>(v, s);
    case 25: return writelane_c<25>(v, s);
    case 26: return writelane_c<26>(v, s);
    case 27: return writelane_c<27>(v, s);
    case 28: return writelane_c<28>(v, s);
    case 29: return writelane_c<29>(v, s);
    case 30: return writelane_c<30>(v, s);
    case 31: return writelane_c<31>(v, s);
    case 32: return writelane_c<32>(v, s);
    case 33: return writelane_c<33>(v, s);
    case 34: return writelane_c<34>(v, s);
    case 35: return writelane_c<35>(v, s);
    case 36: return writelane_c<36>(v, s);
    case 37: return writelane_c<37>(v, s);
    case 38: return writelane_c<38>(v, s);
    case 39: return writelane_c<39>(v, s);
    case 40: return writelane_c<40>(v, s);
    case 41: return writelane_c<41>(v, s);
    case 42: return writelane_c<42>(v, s);
    case 43: return writelane_c<43>(v, s);
    case 44: return writelane_c<44>(v, s);
    case 45: return writelane_c<45>(v, s);
    case 46: return writelane_c<46>(v, s);
    case 47: return writelane_c<47>(v, s);
    case 48: return writelane_c<48>(v, s);
    case 49: return writelane_c<49>(v, s);
    case 50: return writelane_c<50>(v, s);
    case 51: return writelane_c<51>(v, s);
    case 52: return writelane_c<52>(v, s);
    case 53: return writelane_c<53>(v, s);
    case 54: return writelane_c<54>(v, s);
    case 55: return writelane_c<55>(v, s);
    case 56: return writelane_c<56>(v, s);
    case 57: return writelane_c<57>(v, s);
    case 58: return writelane_c<58>(v, s);
    case 59: return writelane_c<59>(v, s);
    case 60: return writelane_c<60>(v, s);
    case 61: return writelane_c<61>(v, s);
    case 62: return writelane_c<62>(v, s);
    case 63: return writelane_c<63>(v, s);
    default: return v;
  }
}

// ------------------------------------------------------------ score ops ----
// OP: 0 TransE L1, 1 TransE L2, 2 RotatE, 3 DistMult, 4 ComplEx, 5 / 6 TransE L1 on 16-bit /
// 8-bit codes (the integer filter; acc carries a uint32 in float bits). One k step.
template <int OP>
__device__ __forceinline__ float op_step(float acc, float qa, float qb, float x, float y) {
  if constexpr (OP == 0) {
    return acc + fabsf(qa - x);
  } else if constexpr (OP == 1) {
    float d = qa - x;
    return acc + d * d;
  } else if constexpr (OP == 2) {
    float dr = qa - x, di = qb - y;
    return acc + sqrtf(__builtin_fmaf(di, di, dr * dr));
  } else if constexpr (OP == 5) {  // TransE L1 integer filter: two 16-bit codes per dword
    return __uint_as_float(__builtin_amdgcn_sad_u16(__float_as_uint(qa), __float_as_uint(x), __float_as_uint(acc)));
  } else if constexpr (OP == 6) {  // TransE L1 integer filter: four 8-bit codes per dword
    return __uint_as_float(__builtin_amdgcn_sad_u8(__float_as_uint(qa), __float_as_uint(x), __float_as_uint(acc)));
  } else {
    return __builtin_fmaf(x, qa, acc);
  }
}
template <int OP>
__device__ __forceinline__ float op_final(float acc) {
  if constexpr (OP == 1) return sqrtf(acc);
  else return acc;
}
// RotatE's |(dr, di)| = sqrt(v), v = fma(di, di, dr*dr), correctly rounded, for the sweep's inner
// loop, in full-rate f32 arithmetic only: y = v_rsq_f32(v), s = v*y, h = y/2, then one
// Newton step s + (v - s*s)*h in fma form. Checked exhaustively on MI355X against IEEE
// sqrtf over every float input (scripts/probes/sqrt_candidates.hip): exact for all
// v in [2^-96, FLT_MAX]; it is not for v = 0, v < 2^-96 or v = inf, so the caller tracks
// min(v) and the accumulators' NaN-ness and recomputes such a (rare) tile with sqrtf.
__device__ __forceinline__ float rot_mag(float v, float y) {  // y = v_rsq_f32(v)
  const float s = v * y, h = 0.5f * y;
  const float e = __builtin_fmaf(-s, s, v);
  return __builtin_fmaf(e, h, s);
}
constexpr float kRotMin = 0x1p-96f;

// RotatE's fast filter (the plain and type-constrained sweeps; the score-storing sweep keeps
// the exact chain): the inner loop takes the raw v_sqrt_f32, which is within 1 ulp of the
// correctly rounded sqrtf on every normal input and within 2^-63 on denormal ones
// (scripts/probes/sqrt_ulp.hip, exhaustive on MI355X). Both chains add non-negative terms in
// the same order, so with S' the fast sum and S the canonical one
//   |S' - S| <= sum_k |m'_k - m_k| + the two chains' rounding errors
//            <= (kp + 1) 2^-23 S' (1 + small) + kp 2^-63,
// and rot_bound() returns a bound above that. A pair whose prediction is on the same side of
// the threshold at both ends of [S' - B, S' + B] (every apply_pred kind is monotone in S) is
// decided; the few others (~2e-4 of the pairs on the C4 tables) and any non-finite S' are
// rescored exactly by rot_exact (IEEE sqrtf, the canonical chain), so the counts are the
// canonical ones bit for bit.
__device__ __forceinline__ float rot_bound(float s, int kp) {
  const float f = (float)(kp + 4) * 0x1p-23f * (1.0f + 0x1p-8f);
  return __builtin_fmaf(s, f, (float)kp * 0x1p-62f);
}
__device__ __forceinline__ float rot_exact(const float* __restrict__ q_km, int64_t q_pad, int64_t q,
                                        const float* __restrict__ ent_km, int64_t e_pad, int64_t e, int kp) {
  float acc = 0.0f;
#pragma unroll 8
  for (int k = 0; k < kp; ++k)
    acc = op_step<2>(acc, q_km[(int64_t)k * q_pad + q], q_km[(int64_t)(kp + k) * q_pad + q],
                     ent_km[(int64_t)k * e_pad + e], ent_km[(int64_t)(kp + k) * e_pad + e]);
  return acc;
}

// TransE L1's integer filter (count-only sweeps, mmre_link_sweep_l1q). The k-major planes are
// quantized once per evaluation to 16-bit codes Q(x) = rint((x + M) * 65535 / 2M), M the
// largest |x| over both planes, two consecutive k per dword, and the sweep's inner loop is
// one v_sad_u16 per two elements (|a.lo - b.lo| + |a.hi - b.hi| + acc: half rate, i.e. one
// issue slot per element against two for sub + add-with-abs; scripts/probes/sad_rate.hip).
// delta * sum|Qq - Qe| is within K delta (1 + small) of the real sum |q - e| (each code is off
// by at most 1/2 + the float rounding of the map), and the canonical f32 chain is within
// (K + 1) 2^-24 S of it, so B = 1.03 K delta + (K + 4) 2^-23 S' bounds |S' - S|; decided /
// undecided pairs as for RotatE (rot_bound), the undecided rescored exactly from the
// row-major copies (l1_exact_rows: the canonical chain, acc + |q_k - e_k| in k order).
// M non-finite (an inf / NaN anywhere in the planes): delta = inf, every pair is undecided.
// Round 4: the default code width is 8 bits -- four k per dword, ONE v_sad_u8 per four elements
// at the issue cost of one v_sad_u16 (scripts/probes/sad8_rate.hip: 4.4 vs 4.7 SIMD-cycles per
// wave-instruction), i.e. half the inner loop -- with the same bound at delta = 2M / 255 (a band
// 257x wider: 0.38 % of the trained C2 pairs undecided, scripts/probes/transe_quant_frac.py).
// Whether that band pays depends on the data (how many scores sit that close to the
// thresholds: xavier-init tables, whose truths rank mid-table, put tens of percent there), so
// k_l1q_probe counts the undecided pairs of a fixed sample with the 8-bit codes and, over
// L1Q_PROBE_FRAC of it, the 16-bit codes are made and swept instead. The choice is one device
// word (hdr[1]); the three sweeps (8-bit, 16-bit, f32) are launched gated on it, and the one it
// names counts -- no host round trip.
// Workspace header (L1Q_HDR bytes before the code planes): word 0 = bits of M, word 1 = the
// code-width word (L1Q_CODES8 / L1Q_F32 / L1Q_CODES16), word 2 = the probe's undecided pairs,
// L1Q_SLOTS undecided-pair counters (uint64, L1Q_SLOT_STRIDE apart: separate cache lines) from
// byte 256, the absmax blocks' partial sums of |x| from byte L1Q_PART. Zeroed up to L1Q_PART by
// the launch sequence. The 16-bit planes follow the header, then the 8-bit planes.
constexpr uint32_t L1Q_CODES8 = 0u, L1Q_F32 = 1u, L1Q_CODES16 = 2u;
constexpr int L1Q_HDR = 8192;
constexpr int L1Q_SLOTS = 16;
constexpr int L1Q_SLOT_STRIDE = 32;  // uint64 units = 256 B
constexpr int L1Q_PART = 256 + L1Q_SLOTS * L1Q_SLOT_STRIDE * 8;
constexpr int L1Q_MAX_BLOCKS = 512;
struct L1Q {
  const float* q_rows;     // (queries, kt) row-major query vectors
  const float* ent_rows;   // (whole table, kt) row-major entity rows
  const uint32_t* hdr;     // workspace header: hdr[0] bits of M, hdr[1] code-width word, hdr[2] probe count
  unsigned long long* undecided;  // counter slots
  const float* q_f;        // fallback: the f32 k-major planes (query, entity slice) and their rows
  const float* ent_f;
  int kp_f;
  int kt;                  // floats per row (the canonical chain's length, padding rows are 0)
  const uint32_t* gate;    // gated launches: run only if *gate is the sweep's code-width word (L1Q_F32 for the f32 sweep)
  const float* q_l1c;      // 8-bit codes, tight bound: per query row sum |eps_q| (upper bound); nullptr: uniform bound
  uint32_t* guard;         // hdr[4]: pairs the rescoring refused (query or entity id out of range; must stay 0)
  uint32_t* und_q;         // optional per-query count of rescored pairs (cost calibration of the sharding)
  int32_t* fin_counts;     // gated f32 launch of the fused evaluation: the finalize (filtered += raw) rides
  int64_t fin_n;           // on it -- every workgroup's slice when the gate is shut, the last workgroup's
  uint32_t* fin_ticket;    // pass after the sweep when it is open (fin_counts nullptr: a separate launch)
  uint32_t* wq;            // dynamic unit scheduling: one zeroed work counter per XCD group (nullptr: static ranges)
};
// The sweeps' dynamic-scheduling work counters (L1Q::wq): one per XCD group, each on a 128-B
// line of its own -- the second half of an undecided-pair counter slot (L1Q_SLOT_STRIDE bytes
// apart from byte 256; the slot's counter uses its first 8 bytes) -- zeroed with the header
// before every evaluation (k_zero_words / k_eval_prep). (Eight counters on one line serialised
// every claim of the grid on that line: C2 sweep 1.03 -> 2.33 ms.) MMRE_SWEEP_DYN=0: the
// static contiguous unit ranges (A/B).
constexpr int L1Q_WQ_STRIDE = L1Q_SLOT_STRIDE * 2;  // uint32 words between two groups' counters
inline uint32_t* l1q_work_counters(const uint32_t* hdr) {
  static_assert(L1Q_SLOTS >= 8 && L1Q_SLOT_STRIDE * 8 >= 256, "a 128-B half slot per XCD group");
  static const char* env = getenv("MMRE_SWEEP_DYN");
  return (env && env[0] == '0') ? nullptr : const_cast<uint32_t*>(hdr) + (256 + 128) / 4;
}
__device__ __forceinline__ float l1q_delta(const uint32_t* absmax, float levels) {
  const float m = __uint_as_float(*absmax);
  return m == 0.0f ? 0.0f : (m < INFINITY ? (2.0f * m) / levels : INFINITY);
}
// Integer thresholds of the L1 filter for one query row (prediction = the score): with a = delta
// S_int, |S - a| <= l1f a + l1c, so S_int < x = (th - l1c) / (delta (1 + l1f)) gives S < th and
// S_int >= y = (th + l1c) / (delta (1 - l1f)) gives S >= th; x, y shrunk / grown by 2^-18 against
// the float rounding of their own computation. With the tight 8-bit bound the accumulator also
// holds the entity's error offset o_e (its code row `words`: S_int + o_e), l1c is the query's own
// error sum, and o_e >= sum |eps_e| / (delta (1 - l1f)): S_int + o_e < t_sure proves S < th and
// S_int + o_e >= t_out + 2 o_max proves S >= th (o_max: the largest offset of the slice).
__device__ __forceinline__ void l1_int_thresholds(float th, float l1c, float l1d, float l1f, uint32_t omax2,
                                                  uint32_t& t_sure, uint32_t& t_span) {
  uint32_t ts = 0u, to = 0xFFFFFFFFu;
  if (l1d < INFINITY) {
    const float x = (th - l1c) / (l1d * (1.0f + l1f)) * (1.0f - 0x1p-18f);
    const float y = (th + l1c) / (l1d * (1.0f - l1f)) * (1.0f + 0x1p-18f);
    ts = x > 0.0f ? (uint32_t)floorf(fminf(x, 0x1p31f)) : 0u;
    to = y > 0.0f ? (uint32_t)ceilf(fminf(y, 0x1p31f)) : 0u;
    // y <= 0 or NaN (a padding query row's -inf threshold, a NaN truth): no pair beats it, no
    // band -- the offsets must not open one (a band there sent padding rows to the rescoring)
    if (to != 0u) to = to + omax2 < to ? 0xFFFFFFFFu : to + omax2;
  }
  t_sure = ts;
  t_span = to > ts ? to - ts : 0u;
}

__device__ __forceinline__ float l1_exact_rows(const float* __restrict__ q, const float* __restrict__ e, int kt) {
  const float4* q4 = reinterpret_cast<const float4*>(q);
  const float4* e4 = reinterpret_cast<const float4*>(e);
  float acc = 0.0f;
#pragma unroll 5
  for (int k = 0; k < kt / 4; ++k) {
    const float4 a = q4[k], b = e4[k];
    acc = acc + fabsf(a.x - b.x);
    acc = acc + fabsf(a.y - b.y);
    acc = acc + fabsf(a.z - b.z);
    acc = acc + fabsf(a.w - b.w);
  }
  return acc;
}

__host__ __device__ inline int op_of_model(int model) {
  return model == MMRE_TRANSE_L1 ? 0 : model == MMRE_TRANSE_L2 ? 1 : model == MMRE_ROTATE ? 2
         : model == MMRE_DISTMULT ? 3 : 4;
}

__device__ __forceinline__ bool type_bit(const uint32_t* __restrict__ mask, int64_t words, int64_t r, int64_t e) {
  return (mask[r * words + (e >> 5)] >> (e & 31)) & 1u;
}
// The type bits of a VALU-sweep thread's 8 entity columns for relation r: columns 0-3 are ids
// e0 .. e0 + 3, columns 4-7 e0 + 64 .. e0 + 67 (e0 a multiple of 4: each group of four lies in
// one 32-bit word); bit j = column j. Two loads per query row instead of one per pair, and no
// per-pair branch (the per-pair `better && type_bit(...)` kept ~100 VGPRs of masks and
// addresses live in the type-constrained sweeps: they spilled). Columns at or past e_end: 0.
__device__ __forceinline__ uint32_t type_bits8(const uint32_t* __restrict__ mask, int64_t words, int64_t r, int e0,
                                               int e_end) {
  const uint32_t* row = mask + r * words;
  const uint32_t lo = e0 < e_end ? (row[e0 >> 5] >> (e0 & 31)) & 15u : 0u;
  const uint32_t hi = e0 + 64 < e_end ? (row[(e0 + 64) >> 5] >> (e0 & 31)) & 15u : 0u;
  return lo | (hi << 4);
}

// Two scores of the query vector sq against entity rows e1 and e2 at once (two independent
// canonical chains; their loads share the round trips): 32 floats of each row per round
// (RotatE: 16 re + 16 im of each). kp % 8 == 0.
template <int OP>
__device__ void pair_score2_lds(const float* __restrict__ ent_rows, const float* sq, int kp, int64_t e1, int64_t e2,
                                float* s1, float* s2) {
  constexpr int NP = (OP == 2 || OP == 4) ? 2 : 1;
  constexpr int W = (OP == 2) ? 16 : 32;  // floats of one plane per row per round
  const int kt = NP * kp;
  const float* r1 = ent_rows + e1 * (int64_t)kt;
  const float* r2 = ent_rows + e2 * (int64_t)kt;
  float a1 = 0.0f, a2 = 0.0f;
  const int kend = (OP == 2) ? kp : kt;  // RotatE walks k over one plane, pairing re/im
  int k0 = 0;
  for (; k0 + W <= kend; k0 += W) {
    float4 x1[W / 4], x2[W / 4], y1[OP == 2 ? W / 4 : 1], y2[OP == 2 ? W / 4 : 1];
#pragma unroll
    for (int i = 0; i < W / 4; ++i) {
      x1[i] = *reinterpret_cast<const float4*>(r1 + k0 + 4 * i);
      x2[i] = *reinterpret_cast<const float4*>(r2 + k0 + 4 * i);
      if constexpr (OP == 2) {
        y1[i] = *reinterpret_cast<const float4*>(r1 + kp + k0 + 4 * i);
        y2[i] = *reinterpret_cast<const float4*>(r2 + kp + k0 + 4 * i);
      }
    }
#pragma unroll
    for (int i = 0; i < W / 4; ++i) {
      const int k = k0 + 4 * i;
      if constexpr (OP == 2) {
        a1 = op_step<OP>(a1, sq[k + 0], sq[kp + k + 0], x1[i].x, y1[i].x);
        a2 = op_step<OP>(a2, sq[k + 0], sq[kp + k + 0], x2[i].x, y2[i].x);
        a1 = op_step<OP>(a1, sq[k + 1], sq[kp + k + 1], x1[i].y, y1[i].y);
        a2 = op_step<OP>(a2, sq[k + 1], sq[kp + k + 1], x2[i].y, y2[i].y);
        a1 = op_step<OP>(a1, sq[k + 2], sq[kp + k + 2], x1[i].z, y1[i].z);
        a2 = op_step<OP>(a2, sq[k + 2], sq[kp + k + 2], x2[i].z, y2[i].z);
        a1 = op_step<OP>(a1, sq[k + 3], sq[kp + k + 3], x1[i].w, y1[i].w);
        a2 = op_step<OP>(a2, sq[k + 3], sq[kp + k + 3], x2[i].w, y2[i].w);
      } else {
        a1 = op_step<OP>(a1, sq[k + 0], 0.0f, x1[i].x, 0.0f);
        a2 = op_step<OP>(a2, sq[k + 0], 0.0f, x2[i].x, 0.0f);
        a1 = op_step<OP>(a1, sq[k + 1], 0.0f, x1[i].y, 0.0f);
        a2 = op_step<OP>(a2, sq[k + 1], 0.0f, x2[i].y, 0.0f);
        a1 = op_step<OP>(a1, sq[k + 2], 0.0f, x1[i].z, 0.0f);
        a2 = op_step<OP>(a2, sq[k + 2], 0.0f, x2[i].z, 0.0f);
        a1 = op_step<OP>(a1, sq[k + 3], 0.0f, x1[i].w, 0.0f);
        a2 = op_step<OP>(a2, sq[k + 3], 0.0f, x2[i].w, 0.0f);
      }
    }
  }
  for (; k0 < kend; k0 += 8) {
    float x1[8], x2[8], y1[8], y2[8];
    *reinterpret_cast<float4*>(&x1[0]) = *reinterpret_cast<const float4*>(r1 + k0);
    *reinterpret_cast<float4*>(&x1[4]) = *reinterpret_cast<const float4*>(r1 + k0 + 4);
    *reinterpret_cast<float4*>(&x2[0]) = *reinterpret_cast<const float4*>(r2 + k0);
    *reinterpret_cast<float4*>(&x2[4]) = *reinterpret_cast<const float4*>(r2 + k0 + 4);
    if constexpr (OP == 2) {
      *reinterpret_cast<float4*>(&y1[0]) = *reinterpret_cast<const float4*>(r1 + kp + k0);
      *reinterpret_cast<float4*>(&y1[4]) = *reinterpret_cast<const float4*>(r1 + kp + k0 + 4);
      *reinterpret_cast<float4*>(&y2[0]) = *reinterpret_cast<const float4*>(r2 + kp + k0);
      *reinterpret_cast<float4*>(&y2[4]) = *reinterpret_cast<const float4*>(r2 + kp + k0 + 4);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float qb = (OP == 2) ? sq[kp + k0 + i] : 0.0f;
      a1 = op_step<OP>(a1, sq[k0 + i], qb, x1[i], (OP == 2) ? y1[i] : 0.0f);
      a2 = op_step<OP>(a2, sq[k0 + i], qb, x2[i], (OP == 2) ? y2[i] : 0.0f);
    }
  }
  *s1 = op_final<OP>(a1);
  *s2 = op_final<OP>(a2);
}

// Truth scores + filtered-rank correction, one 64-thread workgroup (one wave) per filter
// group. A filter group is a set of queries with the same (mode, r, anchor) -- the lookup
// key of Test.h:85's `_find` ((r, t) for head_batch, (h, r) for tail_batch) -- so its
// members share the query vector and the known-entity list. Per pass, lane i scores listed
// entity i of the pass and (first pass) the truth of member query i in one fused pair of
// chains, then every member counts the listed entities that beat its own truth:
//   thr[q]        = pred(true(q))                 (same arithmetic as the sweep)
//   counts[.][q]  = {0, -c, 0, -cc}, c = #{listed j != true(q) : pred(j) < thr[q]}
//                   (cc: those allowed by the type constraint); the sweep adds the raw counts.
// Groups of more than 64 queries are walked 64 at a time (FilterIndex.groups splits them).
// grp_qoff/grp_q == NULL: every query is its own group (off indexed by query).
constexpr int FT = 64;  // threads per filter workgroup = listed entities per pass
template <int OP>
__global__ __launch_bounds__(FT) void k_truth_filter(
    const float* __restrict__ ent_rows, int64_t n_ent, const float* __restrict__ q_km, int64_t q_pad, int kp,
    const float* __restrict__ q_rows, const int32_t* __restrict__ qtrue, const int64_t* __restrict__ qr,
    const int8_t* __restrict__ qmode, int64_t n_query, int pred_kind, float margin, const int64_t* __restrict__ grp_qoff,
    const int32_t* __restrict__ grp_q, int64_t n_groups, const int64_t* __restrict__ off,
    const int32_t* __restrict__ ids, const uint32_t* __restrict__ type_head, const uint32_t* __restrict__ type_tail,
    int64_t type_words, float* __restrict__ thr, int32_t* __restrict__ counts) {
  extern __shared__ float sq[];  // [NP * kp] query vector of the group
  __shared__ float s_v[FT];
  __shared__ int32_t s_id[FT];
  __shared__ uint8_t s_tb[FT];
  constexpr int NP = (OP == 2 || OP == 4) ? 2 : 1;
  const int tid = threadIdx.x;
  for (int64_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
    const int64_t qa = grp_qoff ? grp_qoff[g] : g, qb = grp_qoff ? grp_qoff[g + 1] : g + 1;
    const int64_t la = off ? off[g] : 0, lb = off ? off[g + 1] : 0;
    const int64_t q0 = grp_q ? grp_q[qa] : qa;
    __syncthreads();  // previous group done with sq / s_*
    if (q_rows) {  // one contiguous row (the k-major column would touch one cache line per k)
      for (int k = tid; k < NP * kp; k += FT) sq[k] = q_rows[q0 * NP * kp + k];
    } else {
      for (int k = tid; k < NP * kp; k += FT) sq[k] = q_km[(int64_t)k * q_pad + q0];
    }
    const uint32_t* tm = type_head ? (qmode[q0] == MMRE_HEAD_BATCH ? type_head : type_tail) : nullptr;
    const int64_t r = qr[q0];
    __syncthreads();
    for (int64_t qc = qa; qc < qb; qc += FT) {
      const int64_t qi = qc + tid;
      const bool active = qi < qb;
      const int64_t q = active ? (grp_q ? grp_q[qi] : qi) : 0;
      const int32_t tr = active ? qtrue[q] : 0;
      float th = 0.0f;
      int c = 0, cc = 0;
      int64_t lc = la;
      bool first = true;
      do {  // at least one pass: the truth scores ride on the first
        const int nl = (int)((lb - lc) < FT ? (lb - lc) : FT);
        const int64_t j = tid < nl ? (int64_t)ids[lc + tid] : -1;
        const bool ok = j >= 0 && j < n_ent;
        float vt, vj;
        pair_score2_lds<OP>(ent_rows, sq, kp, tr, ok ? j : 0, &vt, &vj);
        if (first) {
          th = apply_pred(pred_kind, margin, vt);
          if (active) thr[q] = th;
        }
        s_id[tid] = ok ? (int32_t)j : -1;
        s_v[tid] = apply_pred(pred_kind, margin, vj);
        s_tb[tid] = (ok && tm) ? (uint8_t)type_bit(tm, type_words, r, j) : (uint8_t)0;
        __syncthreads();
        if (active) {
          for (int i = 0; i < nl; ++i) {
            const int32_t e = s_id[i];
            if (e >= 0 && e != tr && s_v[i] < th) {
              c += 1;
              cc += s_tb[i];
            }
          }
        }
        __syncthreads();  // s_* reuse
        lc += nl;
        first = false;
      } while (lc < lb);
      if (active) {
        counts[0 * n_query + q] = 0;
        counts[1 * n_query + q] = -c;
        counts[2 * n_query + q] = 0;
        counts[3 * n_query + q] = -cc;
      }
    }
  }
}

// --------------------------------------------- grouped truth + filter (2 phases) ---
// Phase 1, k_filter_scores: one lane per score task, all tasks of the evaluation in one
// flat launch (~1.3k waves at FB15K-237-ZS, resident at once): task t < n_query is the
// truth of query t -> thr[t]; task n_query + p is listed entity p of the filter CSR, scored
// with the query vector of its group's representative query entry_q[p] -> list_v[p].
// Both rows stream from global 32 floats per round (RotatE 16 re + 16 im).
template <int OP>
__device__ float row_score(const float* __restrict__ qv, const float* __restrict__ ev, int kp) {
  constexpr int W = (OP == 2) ? 16 : 32;  // 64 VGPRs of loads in flight per round
  const int kend = (OP == 2) ? kp : ((OP == 4) ? 2 * kp : kp);
  float acc = 0.0f;
  int k0 = 0;
  for (; k0 + W <= kend; k0 += W) {
    float4 a[W / 4], x[W / 4], b[OP == 2 ? W / 4 : 1], y[OP == 2 ? W / 4 : 1];
#pragma unroll
    for (int i = 0; i < W / 4; ++i) {
      a[i] = *reinterpret_cast<const float4*>(qv + k0 + 4 * i);
      x[i] = *reinterpret_cast<const float4*>(ev + k0 + 4 * i);
      if constexpr (OP == 2) {
        b[i] = *reinterpret_cast<const float4*>(qv + kp + k0 + 4 * i);
        y[i] = *reinterpret_cast<const float4*>(ev + kp + k0 + 4 * i);
      }
    }
#pragma unroll
    for (int i = 0; i < W / 4; ++i) {
      if constexpr (OP == 2) {
        acc = op_step<OP>(acc, a[i].x, b[i].x, x[i].x, y[i].x);
        acc = op_step<OP>(acc, a[i].y, b[i].y, x[i].y, y[i].y);
        acc = op_step<OP>(acc, a[i].z, b[i].z, x[i].z, y[i].z);
        acc = op_step<OP>(acc, a[i].w, b[i].w, x[i].w, y[i].w);
      } else {
        acc = op_step<OP>(acc, a[i].x, 0.0f, x[i].x, 0.0f);
        acc = op_step<OP>(acc, a[i].y, 0.0f, x[i].y, 0.0f);
        acc = op_step<OP>(acc, a[i].z, 0.0f, x[i].z, 0.0f);
        acc = op_step<OP>(acc, a[i].w, 0.0f, x[i].w, 0.0f);
      }
    }
  }
  for (; k0 < kend; k0 += 4) {  // kp % 8 == 0, so whole float4s remain
    const float4 a = *reinterpret_cast<const float4*>(qv + k0);
    const float4 x = *reinterpret_cast<const float4*>(ev + k0);
    if constexpr (OP == 2) {
      const float4 b = *reinterpret_cast<const float4*>(qv + kp + k0);
      const float4 y = *reinterpret_cast<const float4*>(ev + kp + k0);
      acc = op_step<OP>(acc, a.x, b.x, x.x, y.x);
      acc = op_step<OP>(acc, a.y, b.y, x.y, y.y);
      acc = op_step<OP>(acc, a.z, b.z, x.z, y.z);
      acc = op_step<OP>(acc, a.w, b.w, x.w, y.w);
    } else {
      acc = op_step<OP>(acc, a.x, 0.0f, x.x, 0.0f);
      acc = op_step<OP>(acc, a.y, 0.0f, x.y, 0.0f);
      acc = op_step<OP>(acc, a.z, 0.0f, x.z, 0.0f);
      acc = op_step<OP>(acc, a.w, 0.0f, x.w, 0.0f);
    }
  }
  return op_final<OP>(acc);
}

template <int OP>
__global__ __launch_bounds__(256) void k_filter_scores(const float* __restrict__ ent_rows, int64_t n_ent,
                                                       const float* __restrict__ q_rows, int kp,
                                                       const int32_t* __restrict__ qtrue, int64_t n_query,
                                                       int pred_kind, float margin, const int32_t* __restrict__ entry_q,
                                                       const int32_t* __restrict__ ids, int64_t n_entries,
                                                       float* __restrict__ thr, float* __restrict__ list_v) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_query + n_entries) return;
  const int64_t kt = (int64_t)((OP == 2 || OP == 4) ? 2 : 1) * kp;
  if (t < n_query) {
    thr[t] = apply_pred(pred_kind, margin, row_score<OP>(q_rows + t * kt, ent_rows + (int64_t)qtrue[t] * kt, kp));
    return;
  }
  const int64_t p = t - n_query;
  const int64_t j = ids[p];
  const int64_t vq = entry_q[p];
  if (j < 0 || j >= n_ent || vq < 0 || vq >= n_query) {
    list_v[p] = __builtin_nanf("");  // never < a threshold: an invalid id is not counted
    return;
  }
  list_v[p] = apply_pred(pred_kind, margin, row_score<OP>(q_rows + vq * kt, ent_rows + j * kt, kp));
}

// Phase 2, k_filter_count: one wave per filter group (queries sharing (mode, r, anchor),
// see mmre_link_truth_grouped); the group's listed scores are staged in LDS 64 at a time and
// every member query (one per lane) counts those that beat its own truth:
//   counts[.][q] = {0, -c, 0, -cc}, c = #{listed j != true(q) : pred(j) < thr[q]} (Test.h:85)
__global__ __launch_bounds__(64) void k_filter_count(const int64_t* __restrict__ grp_qoff,
                                                     const int32_t* __restrict__ grp_q, int64_t n_groups,
                                                     const int64_t* __restrict__ off, const int32_t* __restrict__ ids,
                                                     const float* __restrict__ list_v,
                                                     const int32_t* __restrict__ qtrue, const float* __restrict__ thr,
                                                     const int64_t* __restrict__ qr, const int8_t* __restrict__ qmode,
                                                     int64_t n_query, int64_t n_ent,
                                                     const uint32_t* __restrict__ type_head,
                                                     const uint32_t* __restrict__ type_tail, int64_t type_words,
                                                     int32_t* __restrict__ counts) {
  // staged list: id (-1 = invalid), score, type bit; read back 4 entries per LDS access
  __shared__ __attribute__((aligned(16))) int32_t s_id[64];
  __shared__ __attribute__((aligned(16))) float s_v[64];
  __shared__ __attribute__((aligned(16))) int32_t s_tb[64];
  const int tid = threadIdx.x;
  for (int64_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
    const int64_t qa = grp_qoff[g], qb = grp_qoff[g + 1];
    const int64_t la = off[g], lb = off[g + 1];
    const int64_t q0 = grp_q[qa];
    const uint32_t* tm = type_head ? (qmode[q0] == MMRE_HEAD_BATCH ? type_head : type_tail) : nullptr;
    const int64_t r = qr[q0];
    for (int64_t qc = qa; qc < qb; qc += 64) {
      const int64_t qi = qc + tid;
      const bool active = qi < qb;
      const int64_t q = active ? grp_q[qi] : 0;
      const int32_t tr = active ? qtrue[q] : -1;
      const float th = active ? thr[q] : 0.0f;
      int c = 0, cc = 0;
      for (int64_t lc = la; lc < lb; lc += 64) {
        const int nl = (int)((lb - lc) < 64 ? (lb - lc) : 64);
        __syncthreads();  // s_* reuse
        {
          int32_t id = -1, tb = 0;
          float v = 0.0f;
          if (tid < nl) {
            const int64_t j = ids[lc + tid];
            if (j >= 0 && j < n_ent) {
              id = (int32_t)j;
              v = list_v[lc + tid];
              tb = tm ? (int32_t)type_bit(tm, type_words, r, j) : 0;
            }
          }
          s_id[tid] = id;  // entries nl..63 stay invalid: the loop below reads whole quads
          s_v[tid] = v;
          s_tb[tid] = tb;
        }
        __syncthreads();
        if (active) {
          for (int i = 0; i < nl; i += 4) {  // branch-free, 4 entries per LDS read
            const int4 e = *reinterpret_cast<const int4*>(&s_id[i]);
            const float4 v = *reinterpret_cast<const float4*>(&s_v[i]);
            const int4 t = *reinterpret_cast<const int4*>(&s_tb[i]);
            const int b0 = (e.x >= 0) & (e.x != tr) & (v.x < th);
            const int b1 = (e.y >= 0) & (e.y != tr) & (v.y < th);
            const int b2 = (e.z >= 0) & (e.z != tr) & (v.z < th);
            const int b3 = (e.w >= 0) & (e.w != tr) & (v.w < th);
            c += b0 + b1 + b2 + b3;
            cc += (b0 & t.x) + (b1 & t.y) + (b2 & t.z) + (b3 & t.w);
          }
        }
      }
      if (active) {
        counts[0 * n_query + q] = 0;
        counts[1 * n_query + q] = -c;
        counts[2 * n_query + q] = 0;
        counts[3 * n_query + q] = -cc;
      }
    }
  }
}

// ------------------------------------------------------- work-unit map ---
// Work unit = (query tile of TQ) x (entity tile of TE). XCD group g (workgroups g, g + G,
// g + 2G, ...: the ones round-robin dispatch places on one XCD when the grid is a multiple of
// G = 8) owns m = n_et / G whole entity tiles for every query tile (query-tile major, so its
// L2 keeps streaming the same 1/G of the table and a workgroup leaves a query tile rarely),
// then a 1/G share of the n_et % G leftover tiles' units. Every group gets the same number of
// units +-1, so no XCD runs a whole extra round of units (C3: 100 entity tiles = 8 x 12 + 4;
// whole-tile groups of 12 and 13 left the 13-tile XCDs 10 units per workgroup against 8.7).
struct UnitMap {
  int m, r, ex0, el0, n_main, lo0, count, nq;
  bool emajor;  // entity-tile-major order inside the group (consecutive units share an entity tile)
  __device__ __forceinline__ UnitMap(int grp, int n_groups, int n_qt, int n_et, bool emajor_ = false) {
    nq = n_qt;
    emajor = emajor_;
    m = n_et / n_groups;
    r = n_et - m * n_groups;
    ex0 = grp * m;
    el0 = m * n_groups;  // first leftover entity tile
    n_main = n_qt * m;
    const int64_t left = (int64_t)n_qt * r;
    lo0 = (int)(left * grp / n_groups);
    count = n_main + (int)(left * (grp + 1) / n_groups) - lo0;
  }
  // unit i (< count) of the group -> (query tile, entity tile)
  __device__ __forceinline__ void at(int i, int& qt, int& et) const {
    if (i < n_main) {
      if (emajor) {
        qt = i % nq;
        et = ex0 + i / nq;
      } else {
        qt = i / m;
        et = ex0 + i % m;
      }
    } else {
      const int j = lo0 + (i - n_main);
      qt = j / r;
      et = el0 + j % r;
    }
  }
};

// Work units for a persistent grid whose P workgroups per XCD group run in lock-step windows
// (k_sweep_bf3, round 5): the group owns the contiguous entity tiles [e_lo, e_hi); a window is
// QB query tiles x EB entity tiles (QB x EB <= P), member m of the group always takes window
// position (m / EB, m % EB); windows advance along the entity tiles first, then to the next QB
// query tiles. The P concurrent units of a group therefore share QB query tiles (resident in the
// XCD's L2 for the whole entity pass) and EB entity tiles (each fetched once per window from
// HBM / MALL), instead of ~P different tiles of each operand (the contiguous ranges of UnitMap:
// at C5 every unit re-streamed both 128-KB operand tiles, 120 GB per launch). A member's unit i:
// query-block i / n_e, entity-block i % n_e (n_e = its entity windows): consecutive units of a
// workgroup keep their query tile, so counts flush once per query block.
struct BlockMap {
  int count, qin, ein, QB, EB, e_lo, n_e;
  __device__ __forceinline__ BlockMap(int grp, int n_groups, int member, int P, int n_qt, int n_et, int qb, int eb) {
    e_lo = (int)((int64_t)n_et * grp / n_groups);
    const int e_hi = (int)((int64_t)n_et * (grp + 1) / n_groups);
    const int m_e = e_hi - e_lo;
    QB = qb;
    EB = eb;
    qin = member / EB;
    ein = member - qin * EB;
    count = 0;
    n_e = 0;
    if (qin >= QB || m_e <= 0) return;
    n_e = ein < m_e ? (m_e - ein + EB - 1) / EB : 0;                  // entity windows holding its column
    const int n_q = qin < n_qt ? (n_qt - qin + QB - 1) / QB : 0;     // query windows holding its row
    count = n_q * n_e;
  }
  __device__ __forceinline__ void at(int i, int& qt, int& et) const {
    const int a = i / n_e, b = i - a * n_e;
    qt = a * QB + qin;
    et = e_lo + b * EB + ein;
  }
};

// ------------------------------------------------------------ VALU sweep ---
// Work unit = (query tile of 128) x (entity tile of 128); units are ordered query-tile
// major and split into equal contiguous ranges over a persistent grid sized to the
// resident capacity (4 workgroups per CU), so no tail round is left half empty.
// Within a unit: 256 threads as 16 (q) x 16 (e); each thread owns queries
// {4tq..4tq+3, 64+4tq..} and entities {4te..4te+3, 64+4te..}: 64 fp32 accumulators, one
// sequential k chain each (the canonical order). K is staged through LDS in
// double-buffered steps of 8 rows (16 B per thread per plane per operand). Per-query
// counts stay in registers until the workgroup moves to the next query tile.
// LDS of one VALU-sweep workgroup. A struct declared once in the kernel, so that the L1
// filter's kernel and its f32 fallback path (the same kernel, one uniform branch) share it.
template <int NPL, bool TC, bool LIST>
struct ValuSmem {
  float4 sq[2][NPL][KC][TQ / 4];
  float4 se[2][NPL][KC][TE / 4];
  float s_thr[2][TQ];
  int32_t s_true[2][TQ];
  int32_t s_rel[2][TC ? TQ : 1];
  int8_t s_mode[2][TC ? TQ : 1];
  // per-thread counters (off the VGPR budget); 16-bit with type constraints, so that the wave
  // lists fit beside them at four workgroups per CU (a thread adds <= 8 per unit and row; the
  // sweep flushes every unit where a query tile could hold more than 8,190 of a workgroup's units)
  std::conditional_t<TC, uint16_t, int32_t> s_cnt[TC ? 2 : 1][8][NT];
  uint32_t s_unc[NT / 64];           // undecided pairs per wave (the L1 filter's counter)
  uint32_t s_ts[2][TQ];              // L1 filter, prediction = score: per query row, the integer
  uint32_t s_tw[2][TQ];              // thresholds t_sure and t_out - t_sure (load_meta)
  int s_unit;                        // dynamic scheduling: the unit after the one being swept
  // type constraints: per unit (two in flight, by unit parity), the type words of its 128 query
  // rows over its 128 entity columns -- words 0, 2, 1, 3 of the tile, so a thread's two words
  // (columns 4te.., 64 + 4te..) are one 8-B read -- staged with the unit's first stage
  uint32_t s_tb[TC ? 2 : 1][TC ? TQ : 1][4];
  int2 s_pairs[LIST ? NT / 64 : 1][LIST ? 128 : 1];  // L1 filter: each wave's undecided (query, entity) pairs
};

// The sweep body. Counts go to the raw columns only (counts[0][q], counts[2][q]); the filtered
// columns (initialised to minus the listed entities that beat the truth by the truth pass)
// receive them in k_counts_finalize, one coalesced pass after the sweep (half the atomics).
template <int OP, bool TC, bool STORE, int PK, int NPL, int DYNC>
__device__ __forceinline__ void sweep_valu_body(
    ValuSmem<NPL, TC, (OP == 5 || OP == 6)>& sm, const float* __restrict__ ent_km, int64_t e_pad, int64_t n_ent,
    const float* __restrict__ q_km, int64_t q_pad, int64_t n_query, int kp, int n_et, int e_base, int n_groups,
    int pred_kind, float margin, const float* __restrict__ thr, const int32_t* __restrict__ qtrue,
    const int64_t* __restrict__ qr, const int8_t* __restrict__ qmode, const uint32_t* __restrict__ type_head,
    const uint32_t* __restrict__ type_tail, int64_t type_words, int32_t* __restrict__ counts,
    float* __restrict__ scores, const L1Q& l1) {
  static_assert(NPL == ((OP == 2) ? 2 : 1), "planes");
  // filters: RotatE's raw-sqrt sum (rot_bound / rot_exact), TransE L1's 16-bit codes (L1Q)
  constexpr bool L1F = OP == 5 || OP == 6;  // TransE L1's integer filter (16- / 8-bit codes)
  constexpr bool w8 = OP == 6;
  constexpr bool FAST = (OP == 2 || L1F) && !STORE;
  auto& sq = sm.sq;
  auto& se = sm.se;
  auto& s_thr = sm.s_thr;
  auto& s_true = sm.s_true;
  auto& s_rel = sm.s_rel;
  auto& s_mode = sm.s_mode;
  auto& s_cnt = sm.s_cnt;

  const int tid = threadIdx.x;
  const int tq = tid >> 4, te = tid & 15;
  const PredSel<PK> pred(pred_kind, margin);
  // XCD-aware split (UnitMap): the group's units split evenly over its workgroups, each a
  // contiguous range -- or, with l1.wq (dynamic scheduling, a persistent grid), member m takes
  // unit m of its group first and every further unit from the group's work counter. The loader
  // runs one stage ahead of the compute and enters unit U at the top of compute stage nkc - 2 of
  // the unit before; one stage later thread 0 claims U's successor and publishes it in LDS (its
  // wave waits for the reply there; the other waves of the CU run on), and the loader reads it
  // when it leaves U, >= 1 barrier later. (Holding the reply in a register across the stage
  // instead made it loop-carried: 160 B of scratch per lane.) Units of uneven cost (the
  // rescoring of undecided pairs) balance themselves instead of leaving a tail of workgroups.
  const int grp = blockIdx.x % n_groups, gmem = blockIdx.x / n_groups;
  const int per_grp = gridDim.x / n_groups;
  const UnitMap um(grp, n_groups, (int)(q_pad / TQ), n_et);
  const int nkc = kp / KC;
  // (compiled per mode and chunk: a runtime choice between the modes, or a runtime chunk size,
  // kept values of both live across the loop -- 160-168 B of scratch per lane; the host passes
  // l1.wq only with nkc >= 2)
  constexpr bool dyn = DYNC > 0;
  // dynamic scheduling claims chunks of consecutive units (the units of a group are query-tile
  // major: a chunk mostly keeps its query tile, so its counts flush and its query metadata loads
  // once, not at every unit): 4 when a workgroup sweeps many units, 1 for a rank's small share
  // (launch_valu_one; C2 N = 1, per evaluation: chunks of 1 / 2 / 4 / 8 / 16 units 1.053 / 1.007 /
  // 0.975 / 0.997 / 1.017 ms; 8-way shares: 1 or 2 best)
  constexpr int ch_log2 = DYNC >= 4 ? 2 : DYNC >= 2 ? 1 : 0;
  constexpr int ch_mask = (1 << ch_log2) - 1;
  const int u0 = dyn ? gmem << ch_log2 : (int)((int64_t)gmem * um.count / per_grp);
  const int u1 = dyn ? um.count : (int)((int64_t)(gmem + 1) * um.count / per_grp);
  if (u0 >= u1) return;  // uniform over the workgroup

  // L1 filter constants (uniform): code step, bound slope and offset
  float l1d = 0.0f, l1f = 0.0f, l1c = 0.0f;
  if constexpr (L1F) {
    l1d = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(l1q_delta(l1.hdr, w8 ? 255.0f : 65535.0f))));
    l1f = (float)(l1.kt + 4) * 0x1p-23f * (1.0f + 0x1p-8f);
    l1c = __builtin_fmaf((float)l1.kt * 1.03f, l1d, 0x1p-120f);
  }

  // load_meta and the count flush run once per query tile; what they compute from tid and the
  // filter constants is recomputed there from opaque copies (vgpr_opaque / sgpr_opaque), not
  // hoisted by the compiler into per-lane values kept live across the sweep (that kept ~21 of
  // them in scratch: a scratch store of ~90 B per lane at every wave's start)
  auto load_meta = [&](int qtile, int slot) {
    const int tid = vgpr_opaque(threadIdx.x);
    if (tid < TQ) {
      const int64_t q = (int64_t)qtile * TQ + tid;
      const bool v = q < n_query;
      const float th = v ? thr[q] : -INFINITY;
      s_thr[slot][tid] = th;
      s_true[slot][tid] = v ? qtrue[q] : -1;
      if constexpr (L1F && PK == 0) {
        // prediction = the score: the filter decides in the integer domain. With a = delta *
        // S_int, |S - a| <= l1f a + l1c, so S_int < x = (th - l1c) / (delta (1 + l1f)) gives
        // S < th and S_int >= y = (th + l1c) / (delta (1 - l1f)) gives S >= th; x, y are shrunk /
        // grown by 2^-18 against the float rounding of their own computation. Once per query
        // row and query tile, not per unit.
        uint32_t t_sure, t_span;
        const bool tight = w8 && l1.q_l1c != nullptr;
        const int ktm = sgpr_opaque(l1.kt);
        const float md = __uint_as_float(sgpr_opaque(__float_as_uint(l1d)));
        const float mf = (float)(ktm + 4) * 0x1p-23f * (1.0f + 0x1p-8f);  // = l1f
        const float mc = __builtin_fmaf((float)ktm * 1.03f, md, 0x1p-120f);  // = l1c
        l1_int_thresholds(th, tight ? (v ? l1.q_l1c[q] : 0.0f) + 0x1p-120f : mc, md, mf, tight ? 2u * l1.hdr[3] : 0u,
                          t_sure, t_span);
        sm.s_ts[slot][tid] = t_sure;
        sm.s_tw[slot][tid] = t_span;
      }
      if constexpr (TC) {
        s_rel[slot][tid] = v ? (int32_t)qr[q] : 0;
        s_mode[slot][tid] = v ? qmode[q] : 0;
      }
    }
  };

  const int srow = tid >> 5, sc4 = tid & 31;
  float4 rq0, re0, rq1, re1;  // plane 0 / plane 1 (RotatE) staging: scalars, kept in VGPRs
  // staging position (unit, kc) of the next load, advanced incrementally (no divisions)
  int ld_unit = u0, ld_kc = 0, ld_qt, ld_et;
  um.at(u0, ld_qt, ld_et);
  // type constraints: the staged unit's type words (row tid / 2, words (tid & 1) and 2 + (tid & 1)),
  // whether the pending stage carries them, and the unit parity they go to (the epilogue's
  // ep_par reads them back); the loader's parity starts at 1 so that unit u0 gets 0
  uint32_t rt0 = 0u, rt1 = 0u;
  bool st_new = false;
  int ld_tpar = 1, st_par = 0, ep_par = 0;
  auto gload = [&]() {
    if constexpr (TC) {
      st_new = ld_kc == 0;
      if (st_new) {  // the unit's first stage: its rows' type words ride along
        ld_tpar ^= 1;
        st_par = ld_tpar;
        const int tt = vgpr_opaque(threadIdx.x);
        const int rr = tt >> 1, jw = tt & 1;
        const int64_t q = (int64_t)ld_qt * TQ + rr;
        uint32_t w0 = 0u, w1 = 0u;
        if (q < n_query) {
          const uint32_t* tm = (qmode[q] == MMRE_HEAD_BATCH ? type_head : type_tail) + qr[q] * type_words;
          const int64_t wb = (e_base + (int64_t)ld_et * TE) >> 5;  // e_base and tiles: whole words
          if (wb + jw < type_words) w0 = tm[wb + jw];
          if (wb + 2 + jw < type_words) w1 = tm[wb + 2 + jw];
        }
        rt0 = w0;
        rt1 = w1;
      }
    }
    const int k = ld_kc * KC + srow;
    const int64_t q0 = (int64_t)ld_qt * TQ, e0 = (int64_t)ld_et * TE;
    const float* qp = q_km + (int64_t)k * q_pad + q0 + sc4 * 4;
    const float* ep = ent_km + (int64_t)k * e_pad + e0 + sc4 * 4;
    rq0 = *reinterpret_cast<const float4*>(qp);
    re0 = *reinterpret_cast<const float4*>(ep);
    if constexpr (NPL == 2) {
      rq1 = *reinterpret_cast<const float4*>(qp + (int64_t)kp * q_pad);
      re1 = *reinterpret_cast<const float4*>(ep + (int64_t)kp * e_pad);
    }
    if (++ld_kc == nkc) {
      ld_kc = 0;
      if (dyn) {
        // the next unit of the chunk, or the first of the claimed chunk (published >= 1 barrier ago)
        ld_unit = ((ld_unit + 1) & ch_mask) != 0 ? ld_unit + 1 : sm.s_unit;
        if (ld_unit < u1) um.at(ld_unit, ld_qt, ld_et);
      } else if (++ld_unit < u1) {
        um.at(ld_unit, ld_qt, ld_et);
      }
    }
  };
  auto swrite = [&](int buf) {
    if constexpr (TC) {
      if (st_new) {
        const int tt = vgpr_opaque(threadIdx.x);
        *reinterpret_cast<uint2*>(&sm.s_tb[st_par][tt >> 1][(tt & 1) * 2]) = make_uint2(rt0, rt1);
      }
    }
    sq[buf][0][srow][sc4] = rq0;
    se[buf][0][srow][sc4] = re0;
    if constexpr (NPL == 2) {
      sq[buf][NPL - 1][srow][sc4] = rq1;
      se[buf][NPL - 1][srow][sc4] = re1;
    }
  };

  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
  f32x2 accp[4][8];  // RotatE filter: the packed accumulators (pair layout at the inner loop)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) accp[i][j] = f32x2{0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s_cnt[0][i][tid] = 0;
    if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] = 0;
  }
  if (L1F && tid < NT / 64) sm.s_unc[tid] = 0u;
  // L1 filter: the wave's undecided pairs are appended to its LDS list (ballot order, no
  // atomics) and rescored 64 at a time, one pair per lane, whenever the list holds a full
  // batch -- the dependent row loads of the canonical chain are paid once per 64 pairs, not once
  // per lane-pair with the wave waiting on its busiest lane (which made the 8-bit codes' 0.4 %
  // of undecided pairs cost 0.8 ms at C2). Rescored pairs that beat their threshold go straight
  // to the raw count columns (the query tile's counts may have been flushed already).
  // (Type-constrained sweeps too, since round 6: 16-bit LDS counters make room for the list at
  // four workgroups per CU; their per-lane loop kept 232-240 B of scratch per lane.)
  constexpr bool LIST = L1F;
  int list_n = 0;         // wave-uniform
  uint32_t n_listed = 0;  // the wave's undecided pairs (the filter's counter; per lane without the list)
  // A batch of listed pairs, one per lane (active lanes): each rescored with the canonical chain;
  // the beating pairs' raw counts go out as ONE atomic per distinct query of the batch (a wave's
  // 64 pairs come from its 32 query rows, and the undecided pairs concentrate on few queries --
  // C2: half of the 1.09 M in 103 queries of ~7,000 beating pairs each -- whose count words were
  // a same-address chain of per-pair atomics, serialised at ~13 ns each).
  auto rescore = [&](int2 p, bool active) {
    const int64_t q = p.x;
    const int e = p.y;
    // a guard on the list's invariant: every entry is a (query row, slice column) pair of the
    // unit just swept, with q < n_query (padding query rows open no band) and 0 <= e < n_ent.
    // A pair outside is counted in hdr[4] (mmre_link_l1q_stats, asserted 0 by the filter tests)
    // and never reaches a row gather.
    bool ok = active;
    if (active && ((uint64_t)q >= (uint64_t)n_query || (uint32_t)e >= (uint32_t)n_ent)) {
      if (l1.guard) atomicAdd(l1.guard, 1u);
      ok = false;
    }
    bool beat = false;
    if (ok) {
      if (l1.und_q) atomicAdd(&l1.und_q[q], 1u);
      const float th = thr[q];
      const float sx = l1_exact_rows(l1.q_rows + q * (int64_t)l1.kt, l1.ent_rows + (int64_t)(e + e_base) * l1.kt, l1.kt);
      beat = pred(sx) < th;
      if constexpr (TC) {
        const uint32_t* tm = qmode[q] == MMRE_HEAD_BATCH ? type_head : type_tail;
        if (beat && type_bit(tm, type_words, qr[q], e + e_base)) atomicAdd(&counts[2 * n_query + q], 1);
      }
    }
    const int qi = (int)q;  // (int32 ids: check_link_args)
    uint64_t pend = __ballot(beat);
    while (pend) {  // uniform: one query of the batch per round
      const int leader = __builtin_ctzll(pend);
      const int ql = __builtin_amdgcn_readlane(qi, leader);
      const bool mine = beat && qi == ql;
      const uint64_t same = __ballot(mine);
      if ((int)(threadIdx.x & 63) == leader) atomicAdd(&counts[ql], (int)__builtin_popcountll(same));
      if (mine) beat = false;
      pend &= ~same;
    }
  };

  int cur_qt, cur_et;
  um.at(u0, cur_qt, cur_et);
  int slot = 0;
  uint32_t lo = 0xFFFFFFFFu;  // RotatE: min of the sqrt inputs' bits over this unit (see rot_mag)
  // L1 filter: the code rows actually used in the last stage (the plane is padded to whole
  // stages; 100 of 104 rows at d = 200: the pad rows' zeros are not swept)
  // (OP 6: the words of the k values + the entity error-offset row, l1q_quant8)
  const int kk_last = L1F ? ((((l1.kt + (w8 ? 3 : 1)) >> (w8 ? 2 : 1)) + (w8 ? 2 : 1)) & ~1) - (nkc - 1) * KC
                          : KC;
  // the L1 filter's code-width word (L1Q_CODES8 / _CODES16 / _F32: which of the gated sweeps
  // counts), in flight with the stage
  const uint32_t fb_flag = L1F ? l1.hdr[1] : 0u;
  load_meta(cur_qt, 0);
  gload();
  swrite(0);
  __syncthreads();
  if (L1F && __builtin_amdgcn_readfirstlane(fb_flag) != (w8 ? L1Q_CODES8 : L1Q_CODES16)) return;  // uniform
  if (dyn && ch_mask == 0) {  // u0's successor (after the gate: a shut launch claims none); the
                              // loader reads it at compute stage nkc - 2 of u0, which may be stage 0
    if (tid == 0) sm.s_unit = per_grp + (int)atomicAdd(&l1.wq[grp * L1Q_WQ_STRIDE], 1u);
    __syncthreads();
  }

  constexpr int KKU = 2;  // LDS rows of operands per inner-loop iteration
  int buf = 0;
  for (int unit = u0; unit < u1;) {
    int unit_next = unit + 1;
    for (int kc = 0; kc < nkc; ++kc) {
      const bool more = ld_unit < u1;
      if (more) gload();
      const int kk_n = (L1F && kc == nkc - 1) ? kk_last : KC;
#pragma unroll KKU
      for (int kk = 0; kk < kk_n; ++kk) {
        float4 a0 = sq[buf][0][kk][tq], a1 = sq[buf][0][kk][16 + tq];
        float4 x0 = se[buf][0][kk][te], x1 = se[buf][0][kk][16 + te];
        const float qa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        if constexpr (OP == 2 && FAST) {
          // packed f32: every v_pk_* computes two pairs' IEEE-identical results (the scalar
          // chain's sub, sub, mul, fma, add per half), so one full-rate issue covers two
          // elements and only the two v_sqrt_f32 stay per-element. Pair (ip, jp) of query rows
          // (2ip, 2ip+1) and entity columns (2jp, 2jp+1): the straight product takes
          // (2ip, 2jp) | (2ip+1, 2jp+1), the swapped one (op_sel) (2ip, 2jp+1) | (2ip+1, 2jp).
          float4 b0 = sq[buf][NPL - 1][kk][tq], b1 = sq[buf][NPL - 1][kk][16 + tq];
          float4 y0 = se[buf][NPL - 1][kk][te], y1 = se[buf][NPL - 1][kk][16 + te];
          const f32x2 qa2[4] = {{a0.x, a0.y}, {a0.z, a0.w}, {a1.x, a1.y}, {a1.z, a1.w}};
          const f32x2 qb2[4] = {{b0.x, b0.y}, {b0.z, b0.w}, {b1.x, b1.y}, {b1.z, b1.w}};
          const f32x2 xv2[4] = {{x0.x, x0.y}, {x0.z, x0.w}, {x1.x, x1.y}, {x1.z, x1.w}};
          const f32x2 yv2[4] = {{y0.x, y0.y}, {y0.z, y0.w}, {y1.x, y1.y}, {y1.z, y1.w}};
#pragma unroll
          for (int ip = 0; ip < 4; ++ip)
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) {  // the straight and swapped chains issued side by side
              const f32x2 dr0 = qa2[ip] - xv2[jp], dr1 = qa2[ip] - xv2[jp].yx;
              const f32x2 di0 = qb2[ip] - yv2[jp], di1 = qb2[ip] - yv2[jp].yx;
              const f32x2 p0 = dr0 * dr0, p1 = dr1 * dr1;
              const f32x2 v0 = __builtin_elementwise_fma(di0, di0, p0), v1 = __builtin_elementwise_fma(di1, di1, p1);
              const f32x2 m0 = {__builtin_amdgcn_sqrtf(v0.x), __builtin_amdgcn_sqrtf(v0.y)};
              const f32x2 m1 = {__builtin_amdgcn_sqrtf(v1.x), __builtin_amdgcn_sqrtf(v1.y)};
              accp[ip][2 * jp] = accp[ip][2 * jp] + m0;
              accp[ip][2 * jp + 1] = accp[ip][2 * jp + 1] + m1;
            }
        } else if constexpr (OP == 2) {
          float4 b0 = sq[buf][NPL - 1][kk][tq], b1 = sq[buf][NPL - 1][kk][16 + tq];
          float4 y0 = se[buf][NPL - 1][kk][te], y1 = se[buf][NPL - 1][kk][16 + te];
          const float qb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
          const float yv[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
          // software pipeline across rows: row i + 1's v and v_rsq_f32 are issued before row i's
          // uses, so every rsq result is consumed a whole row later (C4 83.6 -> 81.2 ms; the 16
          // extra VGPRs cost a few dwords of scratch at 168)
          float v[8], y[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float dr = qa[0] - xv[j], di = qb[0] - yv[j];
            v[j] = __builtin_fmaf(di, di, dr * dr);
            y[j] = __builtin_amdgcn_rsqf(v[j]);
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            float vn[8], yn[8];
            if (i + 1 < 8) {
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const float dr = qa[i + 1] - xv[j], di = qb[i + 1] - yv[j];
                vn[j] = __builtin_fmaf(di, di, dr * dr);
                yn[j] = __builtin_amdgcn_rsqf(vn[j]);
              }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
              lo = min(min(lo, __float_as_uint(v[j])), __float_as_uint(v[j + 1]));  // v >= 0: bit order; one v_min3
              acc[i][j] = acc[i][j] + rot_mag(v[j], y[j]);
              acc[i][j + 1] = acc[i][j + 1] + rot_mag(v[j + 1], y[j + 1]);
            }
            if (i + 1 < 8) {
#pragma unroll
              for (int j = 0; j < 8; ++j) { v[j] = vn[j]; y[j] = yn[j]; }
            }
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = op_step<OP>(acc[i][j], qa[i], 0.0f, xv[j], 0.0f);
        }
      }
      if (kc == nkc - 1) {  // unit finished: rank epilogue
        const int64_t q0 = (int64_t)cur_qt * TQ;
        const int64_t ebase = (int64_t)cur_et * TE;
        // type constraints: this thread's 8 type bits of query row ql (bit j = column j), from the
        // unit's staged words
        auto tbits = [&](int ql) -> uint32_t {
          const uint2 w = *reinterpret_cast<const uint2*>(&sm.s_tb[TC ? ep_par : 0][TC ? ql : 0][(te >> 3) * 2]);
          const int sh = (te & 7) * 4;
          return ((w.x >> sh) & 15u) | (((w.y >> sh) & 15u) << 4);
        };
        if constexpr (FAST) {
          if constexpr (OP == 2) {  // unpack the pair layout (register renames) and restart it
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const f32x2 p = accp[i >> 1][(j & ~1) + ((i ^ j) & 1)];
                acc[i][j] = (i & 1) ? p.y : p.x;
              }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int j = 0; j < 8; ++j) accp[i][j] = f32x2{0.0f, 0.0f};
          }
          // undecided pairs: pair (i, j) is bit 31 - ((i & 3) * 8 + j) of unc[i >> 2] (rows 0-3 /
          // 4-7; the whole-tile epilogue shifts the bits in, pair by pair)
          uint32_t unc[2] = {0u, 0u};
          bool whole = false;
          if constexpr (L1F && PK == 0 && !TC) {
            // L1 filter, a whole entity tile (every tile but the last, uniform), ONE pass: per
            // pair d = S_int - t_sure (its borrow, S_int < t_sure, carry-added to the count) and
            // the undecided band d < t_out - t_sure carry-shifted into the pair's bit: four VALU
            // per pair (v_sub_co, v_addc, v_cmp, v_addc). The count needs no truth test: the
            // truth's S is th itself, which no pair below t_sure reaches (S_int < t_sure proves
            // S < th). The truth's own pair is in the band; the rescoring list skips it. (A first
            // pass with a wave-wide "any" ballot and the per-pair bits rebuilt when it was set
            // paid ~420 more VALU per wave and unit: at C2 nearly every wave holds an undecided
            // pair in every unit -- a quarter of them hold a truth.)
            if (ebase + TE <= n_ent) {
              whole = true;
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
                const uint32_t t_sure = sm.s_ts[slot][ql], t_span = sm.s_tw[slot][ql];
                // type constraints: the row's 8 type bits (a pair below t_sure is never the truth)
                const uint32_t tb = TC ? tbits(ql) : 0u;
                int c = 0, cc = 0;
                uint32_t u = unc[i >> 2];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const uint32_t si = __float_as_uint(acc[i][j]);
                  const uint32_t d = si - t_sure;
                  const bool sure = si < t_sure;
                  c += sure;
                  if constexpr (TC) cc += sure & ((tb >> j) & 1u);
                  u = u + u + (uint32_t)(d < t_span);
                }
                unc[i >> 2] = u;
                s_cnt[0][i][tid] += c;
                if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] += cc;
              }
            }
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            if (whole) break;
            const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
            const float th = s_thr[slot][ql];
            const int32_t tr = s_true[slot][ql];
            int c = 0, cc = 0;
            const uint32_t tb = TC ? tbits(ql) : 0u;
            if constexpr (L1F && PK == 0) {
              // prediction = the score: the integer thresholds of load_meta
              const uint32_t t_sure = sm.s_ts[slot][ql], t_span = sm.s_tw[slot][ql];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const int e = (int)ebase + ((j < 4) ? te * 4 + j : 64 + te * 4 + (j - 4));
                const bool valid = (e + e_base != tr) & (e < n_ent);
                const uint32_t si = __float_as_uint(acc[i][j]);
                const bool sure = si < t_sure;
                const bool better = sure & valid;
                c += better;
                if constexpr (TC) cc += better & ((tb >> j) & 1u);
                unc[i >> 2] |= (uint32_t)((si - t_sure < t_span) & valid) << (31 - ((i & 3) * 8 + j));
              }
              s_cnt[0][i][tid] += c;
              if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] += cc;
              continue;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int e = (int)ebase + ((j < 4) ? te * 4 + j : 64 + te * 4 + (j - 4));
              const bool valid = (e + e_base != tr) & (e < n_ent);
              float a, bnd;
              if constexpr (L1F) {
                a = (float)__float_as_uint(acc[i][j]) * l1d;
                bnd = __builtin_fmaf(a, l1f, l1c);
              } else {
                a = acc[i][j];
                bnd = rot_bound(a, kp);
              }
              const float p1 = pred(a - bnd), p2 = pred(a + bnd);
              const bool fin = a < INFINITY;  // false for inf and NaN: rescored
              const bool sure = fin & (fmaxf(p1, p2) < th);
              const bool out = (fin & (fminf(p1, p2) >= th)) | (th != th);
              const bool better = sure & valid;
              c += better;
              if constexpr (TC) cc += better & ((tb >> j) & 1u);
              unc[i >> 2] |= (uint32_t)(!sure & !out & valid) << (31 - ((i & 3) * 8 + j));
            }
            s_cnt[0][i][tid] += c;
            if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] += cc;
          }
          if constexpr (LIST) {
            int2* wl = sm.s_pairs[tid >> 6];
            const int lane = tid & 63;
            for (;;) {  // uniform: one undecided pair per lane and round into the list
              const bool has = (unc[0] | unc[1]) != 0u;
              if (__ballot(has) == 0) break;
              bool keep = false;
              int2 pr = make_int2(0, 0);
              if (has) {
                const int h = unc[0] ? 0 : 1;
                const int p = __builtin_clz(unc[h]);  // pair p = (i & 3) * 8 + j sits at bit 31 - p
                unc[h] &= ~(0x80000000u >> p);
                const int i = h * 4 + (p >> 3), j = p & 7;
                const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
                const int e = (int)ebase + ((j < 4) ? te * 4 + j : 64 + te * 4 + (j - 4));
                keep = (int)(e + e_base) != s_true[slot][ql];  // the truth's own pair is not rescored
                pr = make_int2((int)(q0 + ql), e);
              }
              const uint64_t bal = __ballot(keep);
              if (keep) {
                // list_n < 64 at the top of every round and a round appends <= 64: pos < 128
                const int pos = list_n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                wl[pos] = pr;
              }
              const int nb = __builtin_popcountll(bal);
              list_n += nb;
              n_listed += (uint32_t)nb;
              if (list_n >= 64) {  // a full batch (the list holds < 128: < 64 before this round)
                list_n -= 64;
                rescore(wl[list_n + lane], true);
              }
            }
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            uint32_t m = LIST ? 0u : unc[h];  // (the L1 filter's pairs went to the wave's list)
            while (m) {  // rare: exact rescoring, one pair at a time
              const int p = __builtin_clz(m);
              m &= ~(0x80000000u >> p);
              const int i = h * 4 + (p >> 3), j = p & 7;
              const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
              const int e = (int)ebase + ((j < 4) ? te * 4 + j : 64 + te * 4 + (j - 4));
              float sx;
              if constexpr (L1F) {
                ++n_listed;
                sx = l1_exact_rows(l1.q_rows + (q0 + ql) * (int64_t)l1.kt, l1.ent_rows + (int64_t)(e + e_base) * l1.kt,
                                   l1.kt);
              } else {
                sx = rot_exact(q_km, q_pad, q0 + ql, ent_km, e_pad, e, kp);
              }
              const float v = pred(sx);
              if (v < s_thr[slot][ql]) {
                s_cnt[0][i][tid] += 1;
                if constexpr (TC) {
                  const uint32_t* tm = s_mode[slot][ql] == MMRE_HEAD_BATCH ? type_head : type_tail;
                  s_cnt[TC ? 1 : 0][i][tid] += type_bit(tm, type_words, s_rel[slot][ql], e + e_base) ? 1 : 0;
                }
              }
            }
          }
          // the accumulators restart here, after the rescoring: dead while it runs, so its row
          // loads have the registers
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
        } else {
        if constexpr (OP == 2) {
          bool bad = lo < __float_as_uint(kRotMin);  // v = 0 or v < 2^-96
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) bad |= acc[i][j] != acc[i][j];  // v = inf (or a NaN input)
          if (__ballot(bad)) {  // rare: redo this wave's tiles with the IEEE sqrtf
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
            for (int k = 0; k < kp; ++k) {
              float qa[8], qb[8], xv[8], yv[8];
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                const int64_t ql = q0 + ((i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4));
                const int64_t ec = ebase + ((i < 4) ? te * 4 + i : 64 + te * 4 + (i - 4));
                qa[i] = q_km[(int64_t)k * q_pad + ql];
                qb[i] = q_km[(int64_t)(kp + k) * q_pad + ql];
                xv[i] = ent_km[(int64_t)k * e_pad + ec];
                yv[i] = ent_km[(int64_t)(kp + k) * e_pad + ec];
              }
#pragma unroll
              for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[i][j] = op_step<2>(acc[i][j], qa[i], qb[i], xv[j], yv[j]);
            }
          }
          lo = 0xFFFFFFFFu;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
          const float th = s_thr[slot][ql];
          const int32_t tr = s_true[slot][ql];
          int c = 0, cc = 0;
          const uint32_t tb = TC ? tbits(ql) : 0u;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            // 32-bit ids (int32 by check_link_args); bitwise &: no per-pair branch
            const int e = (int)ebase + ((j < 4) ? te * 4 + j : 64 + te * 4 + (j - 4));
            const float v = pred(op_final<OP>(acc[i][j]));
            const bool better = (v < th) & (e + e_base != tr) & (e < n_ent);
            c += better;
            if constexpr (TC) cc += better & ((tb >> j) & 1u);
            if constexpr (STORE) {
              if (q0 + ql < n_query && e < n_ent) scores[(q0 + ql) * n_ent + e] = v;
            }
            acc[i][j] = 0.0f;
          }
          s_cnt[0][i][tid] += c;
          if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] += cc;
        }
        }  // !FAST
        if (dyn) unit_next = ld_unit;  // the loader entered it at the top of the stage before
        const bool last = unit_next >= u1;
        int next_qt = cur_qt, next_et = cur_et;
        if (!last) um.at(unit_next, next_qt, next_et);
        // (TC: 16-bit counters -- flush every unit where a group's query tile could exceed them)
        if (last || next_qt != cur_qt || (TC && n_et > 8 * 8190)) {  // uniform: flush this query tile's counts
          const int tid = vgpr_opaque(threadIdx.x);  // (see load_meta)
          const int tq = tid >> 4, te = tid & 15;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            int c = s_cnt[0][i][tid], cc = TC ? s_cnt[TC ? 1 : 0][i][tid] : 0;
#pragma unroll
            for (int sh = 1; sh < 16; sh <<= 1) {
              c += __shfl_xor(c, sh);
              if constexpr (TC) cc += __shfl_xor(cc, sh);
            }
            const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
            const int64_t q = q0 + ql;
            if (te == 0 && q < n_query) {  // raw columns only: k_counts_finalize adds them to the filtered ones
              if (c) atomicAdd(&counts[q], c);
              if constexpr (TC) {
                if (cc) atomicAdd(&counts[2 * n_query + q], cc);
              }
            }
            s_cnt[0][i][tid] = 0;
            if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] = 0;
          }
          if (!last) {
            slot ^= 1;
            load_meta(next_qt, slot);
          }
        }
        // the loader entered the last unit of its chunk one stage ago: the next chunk, claimed for
        // the loader's exit from it >= 1 barrier later (the previous claim was read long before);
        // here, after the accumulators were reset, where the claim costs no registers
        if (dyn && !last && ((unit_next + 1) & ch_mask) == 0 && threadIdx.x == 0)
          sm.s_unit = (per_grp + (int)atomicAdd(&l1.wq[grp * L1Q_WQ_STRIDE], 1u)) << ch_log2;
        if constexpr (TC) ep_par ^= 1;  // the next unit's staged type words
        cur_qt = next_qt;
        cur_et = next_et;
      }
      if (more) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
    unit = unit_next;
  }
  if constexpr (L1F) {  // the filter's undecided pairs: one atomic per workgroup, 16 slots
    if constexpr (LIST) {
      if (list_n > 0) rescore(sm.s_pairs[tid >> 6][tid & 63], (tid & 63) < list_n);  // the last partial batch
      if ((tid & 63) == 0) sm.s_unc[tid >> 6] = n_listed;
    } else {
      if (n_listed) atomicAdd(&sm.s_unc[tid >> 6], n_listed);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t t = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) t += sm.s_unc[w];
      // 32-bit counter in the slot's low word (the stats kernel reads only that word)
      if (t) atomicAdd(reinterpret_cast<uint32_t*>(l1.undecided + (blockIdx.x & (L1Q_SLOTS - 1)) * L1Q_SLOT_STRIDE), t);
    }
  }
}

template <int OP, bool TC, bool STORE, int PK, int DYNC = 0>
__global__ __launch_bounds__(NT, (OP == 2) ? 3 : 4) void k_sweep_valu(
    const float* __restrict__ ent_km, int64_t e_pad, int64_t n_ent, const float* __restrict__ q_km,
    int64_t q_pad, int64_t n_query, int kp, int n_et, int e_base, int n_groups, int pred_kind, float margin,
    const float* __restrict__ thr, const int32_t* __restrict__ qtrue, const int64_t* __restrict__ qr,
    const int8_t* __restrict__ qmode, const uint32_t* __restrict__ type_head,
    const uint32_t* __restrict__ type_tail, int64_t type_words, int32_t* __restrict__ counts,
    float* __restrict__ scores, L1Q l1) {
  constexpr int NPL = (OP == 2) ? 2 : 1;
  __shared__ ValuSmem<NPL, TC, (OP == 5 || OP == 6)> sm;
  // the L1 filter's fallback (k_l1q_quant decided that the codes are too coarse for these
  // planes -- one outlier value sets the code step for everything): the filter launch does
  // nothing (sweep_valu_body tests the flag once its first stage is loaded, so the flag's load
  // latency hides under the stage's) and the exact f32 sweep launched after it, gated on the
  // same flag, counts. A separate launch, not a branch here: inlining the f32 body beside the
  // filter's grew the kernel by half and its register spills (18 -> 23)
  if (l1.gate != nullptr) {
    const uint32_t want = OP == 6 ? L1Q_CODES8 : OP == 5 ? L1Q_CODES16 : L1Q_F32;
    if (__builtin_amdgcn_readfirstlane(*l1.gate) != want) {
      if (l1.fin_counts != nullptr) {  // shut (the codes counted): this workgroup's slice of the finalize
        for (int64_t q = (int64_t)blockIdx.x * NT + threadIdx.x; q < l1.fin_n; q += (int64_t)gridDim.x * NT) {
          l1.fin_counts[l1.fin_n + q] += l1.fin_counts[q];
          if constexpr (TC) l1.fin_counts[3 * l1.fin_n + q] += l1.fin_counts[2 * l1.fin_n + q];
        }
      }
      return;
    }
  }
  sweep_valu_body<OP, TC, STORE, PK, NPL, DYNC>(sm, ent_km, e_pad, n_ent, q_km, q_pad, n_query, kp, n_et, e_base,
                                          n_groups, pred_kind, margin, thr, qtrue, qr, qmode, type_head, type_tail,
                                          type_words, counts, scores, l1);
  if (l1.gate != nullptr && l1.fin_counts != nullptr) {
    // open (the rare f32 fallback): the finalize after every workgroup's counts, by the last
    // workgroup (each wave's count atomics drained, then ONE ticket add per workgroup)
    __shared__ uint32_t s_last;
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(l1.fin_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (s_last) {
      for (int64_t q = threadIdx.x; q < l1.fin_n; q += NT) {
        atomicAdd(&l1.fin_counts[l1.fin_n + q],
                  __hip_atomic_load(&l1.fin_counts[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if constexpr (TC)
          atomicAdd(&l1.fin_counts[3 * l1.fin_n + q],
                    __hip_atomic_load(&l1.fin_counts[2 * l1.fin_n + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
      if (threadIdx.x == 0) *l1.fin_ticket = 0u;
    }
  }
}

// filtered columns += raw columns (after the sweep): counts[1] = counts[0] + (minus the listed
// entities that beat the truth, written by the truth pass), likewise counts[3] from counts[2]
__global__ __launch_bounds__(256) void k_counts_finalize(int32_t* __restrict__ counts, int64_t n_query, int tc) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_query) return;
  counts[n_query + q] += counts[q];
  if (tc) counts[3 * n_query + q] += counts[2 * n_query + q];
}

// ------------------------------------------------------------ MFMA sweep ---
// DistMult / ComplEx: S = Q (queries x K) . E^T (K x entities) with the f32-input MFMA
// v_mfma_f32_32x32x2_f32 (exact f32, a k-ordered fma chain: the canonical order).
// Work units and the XCD-grouped split are the VALU sweep's (UnitMap): (query tile of 128) x
// (entity tile of 128). 4 waves as 2 (q) x 2 (e); each wave 64 x 64 = 2 x 2 blocks of 32 x 32
// accumulators. K goes through double-buffered LDS stages of KS rows, register-staged, the
// next stage's global loads issued at the top of the current one (scripts/probes/
// mfma_stage.hip: this beats LDS-DMA rings and a single 256 x 128 workgroup). The plain
// sweep runs KS = 16 at four 256-thread workgroups per CU (33 KB LDS, 112 VGPRs); the type-
// constrained / score-storing variants KS = 32 at two. Epilogue: each lane holds 32 query rows
// x 1 entity column of the 64 x 64 block and reads the rows' thresholds from LDS (b128 reads,
// once per unit). KS = 16: each row's 64 compares are counted by two ballots into a counter
// held by the lane of that row (one register for the wave's 64 rows); KS = 32: per-lane
// register counters for its 32 rows, reduced across the 32 column lanes. Either way the
// counts reach HBM only when the workgroup leaves the query tile. The truth needs no exclusion
// test: its score is bit-identical to the threshold (same canonical chain), so `< thr`
// rejects it.
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <bool TC, bool STORE, int PK, int KS>
__global__ __launch_bounds__(NT, KS == 16 && !TC && !STORE ? 4 : 2) void k_sweep_mfma(
    const float* __restrict__ ent_km, int64_t e_pad, int64_t n_ent, const float* __restrict__ q_km,
    int64_t q_pad, int64_t n_query, int ktot, int n_et, int e_base, int n_groups, int pred_kind, float margin,
    const float* __restrict__ thr, const int64_t* __restrict__ qr, const int8_t* __restrict__ qmode,
    const uint32_t* __restrict__ type_head, const uint32_t* __restrict__ type_tail, int64_t type_words,
    int32_t* __restrict__ counts, float* __restrict__ scores, int emajor, const uint32_t* __restrict__ gate) {
  static_assert(KS == 16 || KS == 32, "stage of 16 or 32 K rows");
  if (gate != nullptr && *gate == 0u) return;  // the split-bf16 filter's fallback: runs only on its overflow
  // 16-row stages (33 KB of LDS) run 4 workgroups per CU: the row counters then live one row
  // per lane (ballot counts), which frees the 32 registers of per-lane row counters
  constexpr bool BAL = KS == 16;
  __shared__ float sq[2][KS][TQ];
  __shared__ float se[2][KS][TE];
  __shared__ int32_t s_rel[TC ? TQ : 1];
  __shared__ int8_t s_mode[TC ? TQ : 1];
  __shared__ __attribute__((aligned(16))) float s_th[2][TQ];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const PredSel<PK> pred(pred_kind, margin);
  const int wq = wave >> 1, we = wave & 1;
  const int lrow = lane >> 5, lcol = lane & 31;
  const int grp = blockIdx.x % n_groups, gmem = blockIdx.x / n_groups;
  const int per_grp = gridDim.x / n_groups;
  const UnitMap um(grp, n_groups, (int)(q_pad / TQ), n_et, emajor != 0);
  const int u0 = (int)((int64_t)gmem * um.count / per_grp);
  const int u1 = (int)((int64_t)(gmem + 1) * um.count / per_grp);
  if (u0 >= u1) return;  // uniform over the workgroup
  // stages of KS rows; with KS = 32 and K = 32 n + 16 (plane_rows: K is a multiple of 16) the
  // unit's last stage holds 16 rows (a uniform branch skips its upper half)
  const int nkc = (ktot + KS - 1) / KS;
  const bool half_tail = KS == 32 && (ktot % 32) != 0;

  // rows of this lane: ql(bi, r) = wq*64 + bi*32 + (r&3) + 8*(r>>2) + 4*lrow
  int tpar = 0;  // s_th slot of the current query tile
  // per-row counters of the current query tile. BAL: one row per lane, lane L holds wave row L
  // (tile row wq * 64 + L), each row's 64 compares counted by two ballots; else each lane
  // counts its own column of its 32 rows, reduced over the 32 column lanes at the flush
  int cntv = 0, cntv_tc = 0;
  int cnt[BAL ? 1 : 2][BAL ? 1 : 16], cnt_tc[TC && !BAL ? 2 : 1][TC && !BAL ? 16 : 1];
  auto row_of = [&](int bi, int r) { return wq * 64 + bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lrow; };
  auto load_rows = [&](int qtile) {
    const int64_t q0 = (int64_t)qtile * TQ;
    // thresholds into the other s_th slot: visible after the stage's closing barrier, and the
    // slot's previous tile was left at least one stage ago
    tpar ^= 1;
    if (tid < TQ) {
      const int64_t q = q0 + tid;
      s_th[tpar][tid] = q < n_query ? thr[q] : -INFINITY;  // -inf: nothing beats a padded row
    }
    cntv = 0;
    cntv_tc = 0;
    if constexpr (!BAL) {
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          cnt[bi][r] = 0;
          if constexpr (TC) cnt_tc[bi][r] = 0;
        }
    }
    if constexpr (TC) {
      __syncthreads();  // previous tile's s_rel/s_mode readers are done
      if (tid < TQ) {
        const int64_t q = q0 + tid;
        s_rel[tid] = q < n_query ? (int32_t)qr[q] : 0;
        s_mode[tid] = q < n_query ? qmode[q] : 0;
      }
    }
  };
  auto flush_rows = [&](int qtile) {
    if constexpr (BAL) {  // each lane its row's count (both column waves add)
      const int64_t q = (int64_t)qtile * TQ + wq * 64 + lane;
      if (q < n_query) {
        if (cntv) atomicAdd(&counts[q], cntv);  // raw only (k_counts_finalize)
        if constexpr (TC) {
          if (cntv_tc) atomicAdd(&counts[2 * n_query + q], cntv_tc);
        }
      }
    } else {
      const int64_t q0 = (int64_t)qtile * TQ;
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int c = cnt[bi][r];
#pragma unroll
          for (int sh = 1; sh < 32; sh <<= 1) c += __shfl_xor(c, sh);  // the 32 column lanes
          int cc = 0;
          if constexpr (TC) {
            cc = cnt_tc[bi][r];
#pragma unroll
            for (int sh = 1; sh < 32; sh <<= 1) cc += __shfl_xor(cc, sh);
          }
          const int64_t q = q0 + row_of(bi, r);
          if (lcol == 0 && q < n_query) {
            if (c) atomicAdd(&counts[q], c);  // raw only (k_counts_finalize)
            if constexpr (TC) {
              if (cc) atomicAdd(&counts[2 * n_query + q], cc);
            }
          }
        }
    }
  };

  const int srow = tid >> 5, sc4 = tid & 31;  // rows srow + 8 i of the stage
  float4 rq0, rq1, re0, re1, rq2, rq3, re2, re3;  // named scalars, not an array: kept in VGPRs
  int ld_unit = u0, ld_kc = 0, ld_qt, ld_et;
  um.at(u0, ld_qt, ld_et);
  auto gload = [&]() {
    const int k = ld_kc * KS + srow;
    const float* qp = q_km + (int64_t)k * q_pad + (int64_t)ld_qt * TQ + sc4 * 4;
    const float* ep = ent_km + (int64_t)k * e_pad + (int64_t)ld_et * TE + sc4 * 4;
    rq0 = *reinterpret_cast<const float4*>(qp);
    rq1 = *reinterpret_cast<const float4*>(qp + 8 * q_pad);
    re0 = *reinterpret_cast<const float4*>(ep);
    re1 = *reinterpret_cast<const float4*>(ep + 8 * e_pad);
    if (KS == 32 && !(half_tail && ld_kc == nkc - 1)) {  // rows past K are never read
      rq2 = *reinterpret_cast<const float4*>(qp + 16 * q_pad);
      rq3 = *reinterpret_cast<const float4*>(qp + 24 * q_pad);
      re2 = *reinterpret_cast<const float4*>(ep + 16 * e_pad);
      re3 = *reinterpret_cast<const float4*>(ep + 24 * e_pad);
    }
    if (++ld_kc == nkc) {
      ld_kc = 0;
      if (++ld_unit < u1) um.at(ld_unit, ld_qt, ld_et);
    }
  };
  auto swrite = [&](int buf) {
    *reinterpret_cast<float4*>(&sq[buf][srow][sc4 * 4]) = rq0;
    *reinterpret_cast<float4*>(&sq[buf][srow + 8][sc4 * 4]) = rq1;
    *reinterpret_cast<float4*>(&se[buf][srow][sc4 * 4]) = re0;
    *reinterpret_cast<float4*>(&se[buf][srow + 8][sc4 * 4]) = re1;
    if constexpr (KS == 32) {
      *reinterpret_cast<float4*>(&sq[buf][srow + 16][sc4 * 4]) = rq2;
      *reinterpret_cast<float4*>(&sq[buf][srow + 24][sc4 * 4]) = rq3;
      *reinterpret_cast<float4*>(&se[buf][srow + 16][sc4 * 4]) = re2;
      *reinterpret_cast<float4*>(&se[buf][srow + 24][sc4 * 4]) = re3;
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  int cur_qt, cur_et;
  um.at(u0, cur_qt, cur_et);
  load_rows(cur_qt);
  gload();
  swrite(0);
  __syncthreads();

  int buf = 0;
  for (int unit = u0; unit < u1; ++unit) {
    for (int kc = 0; kc < nkc; ++kc) {
      const bool more = ld_unit < u1;
      if (more) gload();
      // the next stage's loads stay at the top of this one: hipcc otherwise sinks them to
      // their use at the stage's end and every stage waits a full L2 / MALL latency
      __builtin_amdgcn_sched_barrier(0);
      auto mfma_rows = [&](int k0) {  // 16 K rows = 8 k pairs from stage row k0
#pragma unroll
        for (int kp2 = 0; kp2 < 16; kp2 += 2) {
          const float a0 = sq[buf][k0 + kp2 + lrow][wq * 64 + lcol];
          const float a1 = sq[buf][k0 + kp2 + lrow][wq * 64 + 32 + lcol];
          const float b0 = se[buf][k0 + kp2 + lrow][we * 64 + lcol];
          const float b1 = se[buf][k0 + kp2 + lrow][we * 64 + 32 + lcol];
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
      };
      mfma_rows(0);
      if (KS == 32 && !(half_tail && kc == nkc - 1)) mfma_rows(16);
      if (kc == nkc - 1) {  // unit finished: rank epilogue
        const int64_t q0 = (int64_t)cur_qt * TQ;
        const int64_t ebase = (int64_t)cur_et * TE + we * 64;
        const int64_t e0 = ebase + lcol, e1 = ebase + 32 + lcol;
        const bool ev0 = e0 < n_ent, ev1 = e1 < n_ent;
        if constexpr (BAL) {
#pragma unroll
          for (int bi = 0; bi < 2; ++bi) {
            float tv[16];  // the lane's 16 row thresholds of block bi: 4 LDS reads issued together
#pragma unroll
            for (int r4 = 0; r4 < 16; r4 += 4) {
              const float4 t4 = *reinterpret_cast<const float4*>(&s_th[tpar][row_of(bi, r4)]);
              tv[r4] = t4.x;
              tv[r4 + 1] = t4.y;
              tv[r4 + 2] = t4.z;
              tv[r4 + 3] = t4.w;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              // row (bi, r) of lane half lrow is wave row L0 + 4 lrow; its 64 compares (2 column
              // blocks x 32 lanes) are counted by two ballots
              const float v0 = pred(acc[bi][0][r]), v1 = pred(acc[bi][1][r]);
              const bool b0 = ev0 && v0 < tv[r], b1 = ev1 && v1 < tv[r];
              const uint64_t m0 = __ballot(b0), m1 = __ballot(b1);
              const int L0 = bi * 32 + (r & 3) + 8 * (r >> 2);
              const int c_lo = __popcll(m0 & 0xffffffffull) + __popcll(m1 & 0xffffffffull);
              const int c_hi = __popcll(m0 >> 32) + __popcll(m1 >> 32);
              cntv += lane == L0 ? c_lo : (lane == L0 + 4 ? c_hi : 0);
              if constexpr (TC) {
                const int ql = row_of(bi, r);
                const uint32_t* tm = s_mode[ql] == MMRE_HEAD_BATCH ? type_head : type_tail;
                const uint64_t t0 = __ballot(b0 && type_bit(tm, type_words, s_rel[ql], e0 + e_base));
                const uint64_t t1 = __ballot(b1 && type_bit(tm, type_words, s_rel[ql], e1 + e_base));
                cntv_tc += lane == L0 ? __popcll(t0 & 0xffffffffull) + __popcll(t1 & 0xffffffffull)
                                      : (lane == L0 + 4 ? __popcll(t0 >> 32) + __popcll(t1 >> 32) : 0);
              }
              if constexpr (STORE) {
                const int64_t q = q0 + row_of(bi, r);
                if (q < n_query) {
                  if (ev0) scores[q * n_ent + e0] = v0;
                  if (ev1) scores[q * n_ent + e1] = v1;
                }
              }
            }
          }
        } else {
          // the lane's 32 row thresholds, 8 LDS reads issued together (a read per compare
          // serialised 64 LDS latencies per unit); rows row_of(bi, 4i) .. + 3 are contiguous
          float tv[2][16];
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int r4 = 0; r4 < 16; r4 += 4) {
              const float4 t4 = *reinterpret_cast<const float4*>(&s_th[tpar][row_of(bi, r4)]);
              tv[bi][r4] = t4.x;
              tv[bi][r4 + 1] = t4.y;
              tv[bi][r4 + 2] = t4.z;
              tv[bi][r4 + 3] = t4.w;
            }
#pragma unroll
          for (int bj = 0; bj < 2; ++bj) {
            const int64_t e = bj ? e1 : e0;
            if (bj ? ev1 : ev0) {  // one exec mask per column block (lanes diverge in the last tile only)
#pragma unroll
              for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                  const float v = pred(acc[bi][bj][r]);
                  const bool better = v < tv[bi][r];
                  cnt[bi][r] += better;
                  if constexpr (TC) {
                    const int ql = row_of(bi, r);
                    const uint32_t* tm = s_mode[ql] == MMRE_HEAD_BATCH ? type_head : type_tail;
                    cnt_tc[bi][r] += better && type_bit(tm, type_words, s_rel[ql], e + e_base);
                  }
                  if constexpr (STORE) {
                    const int64_t q = q0 + row_of(bi, r);
                    if (q < n_query) scores[q * n_ent + e] = v;
                  }
                }
            }
          }
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[bi][bj][r] = 0.0f;
        const bool last = unit + 1 >= u1;
        int next_qt = cur_qt, next_et = cur_et;
        if (!last) um.at(unit + 1, next_qt, next_et);
        if (last || next_qt != cur_qt) {  // uniform: leave this query tile
          flush_rows(cur_qt);
          if (!last) load_rows(next_qt);
        }
        cur_qt = next_qt;
        cur_et = next_et;
      }
      if (more) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
}

// ------------------------------------------------------ L1 integer filter ---
// M = max |x| over the query plane and the entity slice (non-finite values make M = inf),
// as float bits in hdr[0] (zeroed by the launch sequence just before), and per block the sum
// of |x| (finite x) into the partials at byte L1Q_PART -- the fallback test's mean |x|.
__global__ __launch_bounds__(256) void k_l1q_absmax(const float* __restrict__ q_km, int64_t q_pad,
                                                    const float* __restrict__ e_km, int64_t e_pad, int64_t e_cols,
                                                    int kp, uint32_t* __restrict__ work) {
  // work items (plane row r, column chunk y of 8) of both planes, strided over the blocks (no
  // index division per element); one atomic per block at most (same-address atomics serialize)
  float m = 0.0f, sa = 0.0f;
  for (int it = blockIdx.x; it < kp * 8; it += gridDim.x) {
    const int r = it >> 3;
    const int64_t st = 8 * (int64_t)blockDim.x, c0 = (int64_t)(it & 7) * blockDim.x + threadIdx.x;
    const float4* q4 = reinterpret_cast<const float4*>(q_km + (int64_t)r * q_pad);
#pragma unroll 4
    for (int64_t c = c0; c < q_pad / 4; c += st) {
      const float4 v = q4[c];
      const float a = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
      m = fmaxf(m, a);
      if (!(v.x - v.x == 0.0f && v.y - v.y == 0.0f && v.z - v.z == 0.0f && v.w - v.w == 0.0f)) m = INFINITY;
      else sa += (fabsf(v.x) + fabsf(v.y)) + (fabsf(v.z) + fabsf(v.w));
    }
    const float4* e4 = reinterpret_cast<const float4*>(e_km + (int64_t)r * e_pad);
#pragma unroll 4
    for (int64_t c = c0; c < e_cols / 4; c += st) {
      const float4 v = e4[c];
      const float a = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
      m = fmaxf(m, a);
      if (!(v.x - v.x == 0.0f && v.y - v.y == 0.0f && v.z - v.z == 0.0f && v.w - v.w == 0.0f)) m = INFINITY;
      else sa += (fabsf(v.x) + fabsf(v.y)) + (fabsf(v.z) + fabsf(v.w));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m = fmaxf(m, __shfl_xor(m, o));
    sa += __shfl_xor(sa, o);
  }
  __shared__ float s_m[4], s_s[4];
  if ((threadIdx.x & 63) == 0) {
    s_m[threadIdx.x >> 6] = m;
    s_s[threadIdx.x >> 6] = sa;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
    reinterpret_cast<float*>(reinterpret_cast<char*>(work) + L1Q_PART)[blockIdx.x] = (s_s[0] + s_s[1]) + (s_s[2] + s_s[3]);
    // non-negative floats order as their bits; inf = no filter. Skip the atomic when the word
    // already holds at least m (a stale read only costs a redundant atomic).
    if (__float_as_uint(m) > __hip_atomic_load(work, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(work, __float_as_uint(m));
  }
}

// The fallback test (every block of k_l1q_quant evaluates it identically; block 0 writes it):
// the code step is 2M / 65535 and a pair stays undecided when its score lies within ~1.03 K
// steps of its threshold, so the filter pays off while M is a modest multiple of the typical
// magnitude. M > ratio x mean|x| (one outlier value stretching the code range: every other value
// then lands in a few codes and most pairs would be rescored one at a time) or M non-finite
// -> the sweep runs the f32 path instead (same counts either way).
__device__ __forceinline__ bool l1q_fallback(const uint32_t* __restrict__ work, int n_part, double n_elem,
                                             float ratio) {
  __shared__ float s_p[4];
  const float* part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(work) + L1Q_PART);
  float v = 0.0f;
  for (int i = threadIdx.x; i < n_part; i += blockDim.x) v += part[i];  // fixed order per thread
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) s_p[threadIdx.x >> 6] = v;
  __syncthreads();
  const float sum = (s_p[0] + s_p[1]) + (s_p[2] + s_p[3]);
  const float mx = __uint_as_float(work[0]);
  if (!(mx < INFINITY)) return true;
  return (double)mx > (double)ratio * ((double)sum / n_elem);
}

// Codes of columns [c0, c0 + n) of a k-major float plane (kp rows, stride pad) into dword rows
// r < kw, Q(x) = rint((x + M) (2^BITS - 1) / 2M): BITS 16 packs Q(x[2r]) | Q(x[2r + 1]) << 16,
// BITS 8 the four codes Q(x[4r + h]) << 8h (k >= kp: code 0 in both planes).
// mode 0 (the first codes made): the fallback test decides between these codes and the f32
// sweep and writes the code-width word. mode 1 (the 16-bit codes after k_l1q_probe): made only
// while the f32 fallback is off and the probe counted more than probe_max undecided pairs; the
// first block writes L1Q_CODES16 (the other blocks read the word before or after that store
// and reach the same decision either way).
// Both planes in one launch: blockIdx.y 0 = the query plane, 1 = the entity slice.
struct L1QPlane {
  const float* km;  // k-major float plane, row stride pad
  int64_t pad, c0, n;  // columns [c0, c0 + n)
  uint32_t* out;    // code rows, row stride pad
};
template <int BITS>
__global__ __launch_bounds__(256) void k_l1q_quant(L1QPlane pq, L1QPlane pe, int kp, int kw,
                                                   uint32_t* __restrict__ work, int n_part, double n_elem,
                                                   float ratio, int mode, uint32_t probe_max) {
  const float* __restrict__ km = blockIdx.y ? pe.km : pq.km;
  const int64_t pad = blockIdx.y ? pe.pad : pq.pad, c0 = blockIdx.y ? pe.c0 : pq.c0, n = blockIdx.y ? pe.n : pq.n;
  uint32_t* __restrict__ out = blockIdx.y ? pe.out : pq.out;
  if (mode == 1) {
    const uint32_t w = __builtin_amdgcn_readfirstlane(work[1]);
    if (w == L1Q_F32) return;
    if (w != L1Q_CODES16 && __builtin_amdgcn_readfirstlane(work[2]) <= probe_max) return;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) work[1] = L1Q_CODES16;
  } else {
    const bool fb = l1q_fallback(work, n_part, n_elem, ratio);
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) work[1] = fb ? L1Q_F32 : (BITS == 8 ? L1Q_CODES8 : L1Q_CODES16);
    if (fb) return;
  }
  constexpr int PER = 32 / BITS;
  constexpr float LEVELS = BITS == 8 ? 255.0f : 65535.0f;
  const float mx = __uint_as_float(*work);
  const float inv = (mx > 0.0f && mx < INFINITY) ? LEVELS / (2.0f * mx) : 0.0f;
  const float off = (mx < INFINITY) ? mx : 0.0f;
  const int64_t total = (int64_t)kw * n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int r = (int)(i / n);
    const int64_t c = c0 + i % n;
    uint32_t word = 0u;
#pragma unroll
    for (int h = 0; h < PER; ++h) {
      const int k = PER * r + h;
      float t = k < kp ? (km[(int64_t)k * pad + c] + off) * inv : 0.0f;
      t = t == t ? fminf(fmaxf(t, 0.0f), LEVELS) : 0.0f;
      word |= (uint32_t)rintf(t) << (BITS * h);
    }
    out[(int64_t)r * pad + c] = word;
  }
}

// The 8-bit codes (mode 0: the fallback test first, then the code-width word = 8-bit), written
// word row by word row like k_l1q_quant, plus one more row after the k values' words: with
// TIGHT (prediction = the score, no type masks, kt <= 1984) each column's quantization error
// sum E = sum_k |x_k - (delta code_k - M)| is reduced in the workgroup (32 columns x 8 row
// groups); a query row stores its bound 1.01 E + kt 2^-20 M (float rounding of the map and the
// sum) for the thresholds (q_l1c), an entity column stores o = ceil(bound / (delta (1 - l1f)))
// as four bytes summing to o in that row, so the sweep's own v_sad_u8 adds o to every pair's sum
// (the query's row is 0), and hdr[3] gets the slice's largest o. The pair's bound is then the
// two rows' error sums -- about K delta / 2 -- instead of 1.03 K delta.
template <bool TIGHT>
__global__ __launch_bounds__(256) void k_l1q_quant8(L1QPlane pq, L1QPlane pe, int kp, int kw, int kt,
                                                    uint32_t* __restrict__ work, int n_part, double n_elem,
                                                    float ratio, float* __restrict__ q_l1c) {
  const bool fb = l1q_fallback(work, n_part, n_elem, ratio);
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) work[1] = fb ? L1Q_F32 : L1Q_CODES8;
  if (fb) return;
  const bool ent = blockIdx.y != 0;
  const float* __restrict__ km = ent ? pe.km : pq.km;
  const int64_t pad = ent ? pe.pad : pq.pad, c0 = ent ? pe.c0 : pq.c0, n = ent ? pe.n : pq.n;
  uint32_t* __restrict__ out = ent ? pe.out : pq.out;
  const float mx = __uint_as_float(*work);
  const float inv = (mx > 0.0f && mx < INFINITY) ? 255.0f / (2.0f * mx) : 0.0f;
  const float off = (mx < INFINITY) ? mx : 0.0f;
  const float delta = (mx > 0.0f && mx < INFINITY) ? (2.0f * mx) / 255.0f : 0.0f;  // l1q_delta's
  const float l1f = (float)(kt + 4) * 0x1p-23f * (1.0f + 0x1p-8f);
  const int words = (kt + 3) >> 2;  // row `words`: the error offsets
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  __shared__ float s_err[8][32];
  for (int64_t cb = (int64_t)blockIdx.x * 32; cb < n; cb += (int64_t)gridDim.x * 32) {  // uniform
    const bool live = cb + cl < n;
    const int64_t c = c0 + cb + cl;
    float err = 0.0f;
#pragma unroll 4
    for (int r = g; r < kw; r += 8) {  // 4 word rows' loads in flight per thread
      uint32_t word = 0u;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int k = 4 * r + h;
        if (live && k < kp) {
          const float x = km[(int64_t)k * pad + c];
          float t = (x + off) * inv;
          t = t == t ? fminf(fmaxf(t, 0.0f), 255.0f) : 0.0f;
          const float code = rintf(t);
          word |= (uint32_t)code << (8 * h);
          if constexpr (TIGHT) err += fabsf(x - (code * delta - off));
        }
      }
      if (live && !(TIGHT && r == words)) out[(int64_t)r * pad + c] = word;
    }
    if constexpr (TIGHT) {
      s_err[g][cl] = err;
      __syncthreads();
      if (g == 0 && live) {
        float e = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) e += s_err[i][cl];
        const float eb = __builtin_fmaf(e, 1.01f, (float)kt * 0x1p-20f * mx);
        uint32_t wv = 0u;
        if (!ent) {
          q_l1c[c] = eb;
        } else {
          // o <= 1020 (four bytes of 255) without the clamp ever acting: each element's code error
          // is at most delta / 2 (rounding to nearest; |x| <= M, so no value is clipped) plus the
          // float rounding of the map, so E <= kt delta / 2 (1 + 2^-20) and o <= 1.01 kt / 2 (1 +
          // 2^-16) + kt 2^-20 M / delta + 1 <= 0.506 kt + 1 = 1,005 at the host guard kt <= 1,984
          // (tests/test_sweep_filters_gpu.py::test_l1_tight_offsets_at_kt_1984 reads the largest o)
          uint32_t o = delta > 0.0f ? (uint32_t)ceilf(fminf(eb / (delta * (1.0f - l1f)) * (1.0f + 0x1p-17f), 1020.0f))
                                    : 0u;
          if (o) atomicMax(work + 3, o);
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const uint32_t b = o < 255u ? o : 255u;
            wv |= b << (8 * h);
            o -= b;
          }
        }
        out[(int64_t)words * pad + c] = wv;
      }
      __syncthreads();
    }
  }
}

// The code-width probe (runs when the 8-bit codes were made): L1Q_PROBE_Q workgroups, each one
// query column (evenly spaced over the queries) against L1Q_PROBE_E consecutive entity columns
// of the slice (the start spread over the slice), scored with the 8-bit codes; the pairs inside
// their query's undecided band (the epilogue's test in its float form) are counted into hdr[2].
// 512 queries x 256 entities: the undecided pairs concentrate on a few queries (C2: a sample of
// 64 queries read 0.19 % where the whole evaluation has 0.38 %), so many queries, short windows.
// The threshold: where the 8-bit sweep's rescoring stops paying. Spread over every query tile
// (C2 at N = 1, 0.38 %) the rescoring overlaps the other waves' sums and 8-bit wins (1.32 vs
// 1.62 ms); concentrated in a rank's share of a few relations it does not: 8-way C2 shares at
// 0.77 % / 1.18 % took 0.32 / 0.51 ms against 0.26 ms with 16-bit codes (profiles/r4).
constexpr int L1Q_PROBE_Q = 512, L1Q_PROBE_E = 256;
constexpr double L1Q_PROBE_FRAC = 0.006;  // undecided fraction of the sample above which 16-bit codes
// The probe's switch point in undecided pairs for a sample of n_slice entity columns -- ONE helper
// for both entry points (mmre_link_sweep_l1q and the fused mmre_link_evaluate_l1q), so that
// MMRE_L1_PROBE_FRAC (experiments) moves both alike and their code widths / stats agree.
static uint32_t l1q_probe_max(int64_t n_slice) {
  static const char* pf_env = getenv("MMRE_L1_PROBE_FRAC");
  const double pfrac = pf_env ? atof(pf_env) : L1Q_PROBE_FRAC;
  const int64_t sample = (int64_t)L1Q_PROBE_Q * std::min<int64_t>(L1Q_PROBE_E, n_slice);
  return (uint32_t)std::min(pfrac * (double)sample, 4.0e9);
}

__global__ __launch_bounds__(256) void k_l1q_probe(const uint32_t* __restrict__ uq, int64_t q_pad, int64_t n_query,
                                                   const uint32_t* __restrict__ ue, int64_t e_pad, int64_t n_slice,
                                                   int kw, int kt, const float* __restrict__ thr, int pred_kind,
                                                   float margin, uint32_t* __restrict__ work,
                                                   const float* __restrict__ q_l1c) {
  if (__builtin_amdgcn_readfirstlane(work[1]) != L1Q_CODES8) return;
  const PredSel<-1> pred(pred_kind, margin);
  const int64_t q = (int64_t)blockIdx.x * n_query / gridDim.x;
  const int64_t span = n_slice > L1Q_PROBE_E ? n_slice - L1Q_PROBE_E : 0;
  const int64_t c = (((int64_t)blockIdx.x * span / gridDim.x) & ~(int64_t)3) + 4 * threadIdx.x;  // 64 threads
  const float l1d = l1q_delta(work, 255.0f);
  const float l1f = (float)(kt + 4) * 0x1p-23f * (1.0f + 0x1p-8f);
  const float l1c = __builtin_fmaf((float)kt * 1.03f, l1d, 0x1p-120f);
  uint32_t acc[4] = {0u, 0u, 0u, 0u};
  if (c < n_slice) {  // columns c .. c + 3 lie inside the slice's whole tiles
#pragma unroll 8
    for (int r = 0; r < kw; ++r) {
      const uint32_t a = uq[(int64_t)r * q_pad + q];
      const uint4 e = *reinterpret_cast<const uint4*>(ue + (int64_t)r * e_pad + c);
      acc[0] = __builtin_amdgcn_sad_u8(a, e.x, acc[0]);
      acc[1] = __builtin_amdgcn_sad_u8(a, e.y, acc[1]);
      acc[2] = __builtin_amdgcn_sad_u8(a, e.z, acc[2]);
      acc[3] = __builtin_amdgcn_sad_u8(a, e.w, acc[3]);
    }
  }
  const float th = thr[q];
  uint32_t und = 0u;
  if (q_l1c != nullptr) {  // the tight bound (prediction = the score): the sweep's integer test
    uint32_t t_sure, t_span;
    l1_int_thresholds(th, q_l1c[q] + 0x1p-120f, l1d, l1f, 2u * work[3], t_sure, t_span);
#pragma unroll
    for (int j = 0; j < 4; ++j) und += (uint32_t)((acc[j] - t_sure < t_span) & (c + j < n_slice));
  } else
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = (float)acc[j] * l1d;
    const float bnd = __builtin_fmaf(a, l1f, l1c);
    const float p1 = pred(a - bnd), p2 = pred(a + bnd);
    const bool fin = a < INFINITY;
    const bool sure = fin & (fmaxf(p1, p2) < th);
    const bool out = (fin & (fminf(p1, p2) >= th)) | (th != th);
    und += (uint32_t)(!sure & !out & (c + j < n_slice));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) und += __shfl_xor(und, o);
  if ((threadIdx.x & 63) == 0 && und) atomicAdd(work + 2, und);
}

// Zeroes n words: the filters' workspace headers at the start of each sweep. A kernel, not
// hipMemsetAsync: replayed from a captured hipGraph, the memset node of the 4,352-byte L1
// header left words 2-3 holding stale bytes (the probe's count read garbage and the graph's
// evaluations switched to the 16-bit codes), while eager runs were right.
__global__ __launch_bounds__(256) void k_zero_words(uint32_t* __restrict__ p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0u;
}

// Sum of the undecided-pair slots, the code-width word, the rescoring guard's count and the largest
// error offset of the tight bound -> out[0..3] (mmre_link_l1q_stats).
__global__ void k_l1q_stats(const uint32_t* __restrict__ work, unsigned long long* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const unsigned long long* sl =
      reinterpret_cast<const unsigned long long*>(reinterpret_cast<const char*>(work) + 256);
  unsigned long long t = 0;
  for (int i = 0; i < L1Q_SLOTS; ++i) t += *reinterpret_cast<const uint32_t*>(sl + i * L1Q_SLOT_STRIDE);
  out[0] = t;
  out[1] = work[1];
  out[2] = work[4];
  out[3] = work[3];
}

static int l1q_rows(int dim) { return (int)round_up((plane_rows(MMRE_TRANSE_L1, dim) + 1) / 2, KC); }
// (+ 1: the entity error-offset row of the tight bound, k_l1q_quant8)
static int l1q_rows8(int dim) { return (int)round_up((plane_rows(MMRE_TRANSE_L1, dim) + 3) / 4 + 1, KC); }

// ------------------------------------------------- split-bf16 MFMA filter ---
// DistMult / ComplEx count-only sweeps through a filter with exact rescoring, as the VALU
// sweeps' (rot_bound, L1Q): every f32 plane value x is split into two bf16 values hi = bf16(x)
// and lo = bf16(x - hi) (round to nearest even), and the sweep computes
//     S' = Qhi . Ehi + Qhi . Elo + Qlo . Ehi
// on v_mfma_f32_32x32x16_bf16: three MFMAs of 16 k each per 32 x 32 block where the exact
// sweep issues eight v_mfma_f32_32x32x2_f32 of 2 k (16x the f32 rate per MFMA cycle,
// 5.3x per scored element). Bound on |S' - S|, S the canonical f32 fma chain (what the exact
// sweep and the truth kernels compute), P the exact dot product, with Sigma = sum |q_k||e_k|
// <= |q|_2 |e|_2 (Cauchy-Schwarz):
//   |P - T|  <= 3.02 x 2^-16 Sigma      T = the three products' exact sum; the dropped terms
//                                       are lo.lo + (hi+lo).r_e + r_q.e with |lo| <= 2^-8 (1+2^-8) |x|
//                                       and |r| = |x - hi - lo| <= 2^-16 |x| (bf16: 8-bit significand)
//   |T - S'| <= 3K x 2u (1 + 2^-7) Sigma   any order / grouping of the 3K exact bf16 products
//                                       summed with at most one rounding (RN or toward zero,
//                                       2u) per addition -- MFMA's internal summation order is
//                                       not documented, so no more is assumed
//   |S - P|  <= K u (1 + small) Sigma      the canonical chain (u = 2^-24)
// plus 2^-29 sqrt(K) |q||e| for the values |x| < 2^-60 the split sets to zero (norms are
// clamped to >= 2^-30). So B = cb |q|_2 |e|_2, cb = 1.02 (7K 2^-24 (1 + 2^-7) + 3.02 2^-16 +
// 2^-29 sqrt K) (computed on the host, the norms' own rounding inside the 2 %). A pair whose
// prediction is on the same side of its query's threshold at both ends of [S' - B, S' + B]
// is decided (apply_pred is monotone); every other valid pair -- the truth itself, near ties,
// any non-finite S' (an inf / NaN operand is split into a NaN hi) -- is appended to a pair
// list and rescored with the canonical chain from the row-major copies (k_bf3_rescore), so
// the counts are the exact sweep's bit for bit. ~2e-4 of the C3 pairs and 2e-5 of C5's land
// in the list. A list that overflows its capacity sets a flag on the device: the raw counts
// are reset and the exact f32 sweep runs instead (gated launches, no host round trip).
// Workspace: header (BF3_HDR bytes: word 1 overflow flag, words 2-3 the appended pairs (uint64)) | pair list
// (bf3_cap int2) | |q| (q_pad floats) | |e| (e_pad floats) | split query planes (K/16 blocks
// x q_pad rows x 64 B: hi[16] | lo[16]) | split entity planes (K/16 x e_pad x 64 B).
// The list: half of it cut into BF3_SEGS segments of cap / (2 BF3_SEGS) pairs, each with its own
// counter on a 128-B line of the header (32-bit words BF3_SEG_W0 + 32 s), the other half shared
// (its counter: segment index BF3_SEGS). A sweep workgroup b appends to segment b % BF3_SEGS and,
// once that is full, to the shared half (bf3_list). One counter for the whole list serialised
// every append chip-wide (~13 ns per same-address atomic): C3's 46 k listed pairs ~0.35 of a
// 0.74-ms sweep (a build with the decision pass compiled out ran 0.39 ms); the shared half keeps
// a burst of one workgroup (a non-finite row's pairs) from overflowing its segment. A full shared
// half sets the overflow flag (word 1): the exact sweep then counts, as for a full list before.
// A counter that wraps (> 4 G appends) cannot clear the flag its first overflow set.
constexpr int BF3_SEGS = 64;
constexpr int BF3_SEG_W0 = 64;
constexpr int BF3_HDR = 4 * (BF3_SEG_W0 + 32 * (BF3_SEGS + 1));
#ifndef BF3_WG_PER_CU
#define BF3_WG_PER_CU 3  // workgroups per CU the sweep is compiled for (168 VGPRs)
#endif
inline int64_t bf3_cap(int64_t q_pad, int64_t e_pad) {
  const char* cap_env = getenv("MMRE_BF3_CAP");  // tests: a tiny list forces the overflow fallback
  if (cap_env && atoll(cap_env) > 0) return atoll(cap_env);
  int64_t c = q_pad * e_pad / 512;
  c = c < (1 << 16) ? (1 << 16) : c;
  return c > (1 << 26) ? (1 << 26) : c;
}
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// append one undecided pair to the calling workgroup's segment of the list, or to the shared
// half when the segment is full (see BF3_SEGS)
__device__ __forceinline__ void bf3_list(uint32_t* __restrict__ hdr, int2* __restrict__ pairs, int64_t cap, int2 p) {
  const int sgm = (int)(blockIdx.x & (BF3_SEGS - 1));
  const int64_t seg_cap = cap / (2 * BF3_SEGS);
  const uint32_t i = atomicAdd(hdr + BF3_SEG_W0 + 32 * sgm, 1u);
  if ((int64_t)i < seg_cap) {
    pairs[sgm * seg_cap + i] = p;
    return;
  }
  const uint32_t j = atomicAdd(hdr + BF3_SEG_W0 + 32 * BF3_SEGS, 1u);
  if ((int64_t)j < cap - BF3_SEGS * seg_cap) pairs[BF3_SEGS * seg_cap + j] = p;
  else hdr[1] = 1u;
}

__device__ __forceinline__ uint32_t bf16_rn_bits(float x) {  // finite x: round to nearest even
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// The split of 16 consecutive k values of one column into the 64-B block {hi[16], lo[16]}.
__device__ __forceinline__ void bf3_split_store(const float (&x)[16], uint4* __restrict__ o) {
  uint32_t hw[8], lw[8];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t hb = 0u, lb = 0u;
    if (!(fabsf(x[j]) < INFINITY)) {
      hb = 0x7FC0u;  // inf / NaN: a NaN operand, every product NaN: the pair is undecided
    } else if (fabsf(x[j]) >= 0x1p-60f) {
      hb = bf16_rn_bits(x[j]);
      lb = bf16_rn_bits(x[j] - __uint_as_float(hb << 16));  // x - hi is exact (Sterbenz)
    }
    if (j & 1) { hw[j >> 1] |= hb << 16; lw[j >> 1] |= lb << 16; }
    else { hw[j >> 1] = hb; lw[j >> 1] = lb; }
  }
  o[0] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
  o[1] = make_uint4(hw[4], hw[5], hw[6], hw[7]);
  o[2] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
  o[3] = make_uint4(lw[4], lw[5], lw[6], lw[7]);
}

// One thread per (column c, 16-k block kb) of a k-major plane (K rows x pad, columns col0 + c):
// the split block out[kb][c] = {hi[16], lo[16]} (4 x 16 B). Consecutive threads take
// consecutive columns of one block: coalesced 64-B-per-thread reads and writes.
__global__ __launch_bounds__(256) void k_bf3_split(const float* __restrict__ km, int64_t pad, int64_t col0,
                                                   int64_t n_cols, int nkb, uint4* __restrict__ out,
                                                   int64_t out_pad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_cols * nkb) return;
  const int kb = (int)(i / n_cols);
  const int64_t c = i - (int64_t)kb * n_cols;
  const float* src = km + col0 + c + (int64_t)kb * 16 * pad;
  float x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = src[(int64_t)j * pad];  // all in flight together
  bf3_split_store(x, out + ((int64_t)kb * out_pad + c) * 4);
}

// The split planes, norms and (wide sweep) 32-column norm maxima straight from a ROW-MAJOR
// table (mmre_link_sweep_bf3_rows: DistMult, whose row-major copy is the raw table itself, so
// no re-laid-out copy is written per evaluation): one read of the rows, one write of the split
// blocks. 256 threads = 32 rows x 8 lanes; lane j of a row takes its 16-k blocks j, j + 8, ...
// (8 lanes read 512 contiguous bytes of the row; for one block the 32 rows' 64-B outputs are
// contiguous). Same split as k_bf3_split, norms as k_bf3_norms / k_bf3_enorms (any summation
// order serves: the bound's 2 % slack covers the norm's rounding); rows past n_rows (the
// slice's last tile) are zero with norm 0.
__global__ __launch_bounds__(256) void k_bf3_split_rows(const float* __restrict__ rows, int64_t n_rows, int64_t r0,
                                                        int ktot, uint4* __restrict__ out, int64_t out_pad,
                                                        float* __restrict__ norms, float* __restrict__ bmax) {
  __shared__ float wm[4];
  const int i = threadIdx.x >> 3, j = threadIdx.x & 7;
  const int64_t c = (int64_t)blockIdx.x * 32 + i;  // slice column
  const int64_t r = r0 + c;
  const bool valid = r < n_rows;
  const float* src = rows + (valid ? r : 0) * (int64_t)ktot;
  const int nkb = ktot / 16;
  float ss = 0.0f;
  for (int kb = j; kb < nkb; kb += 8) {
    float x[16];
    const float4* s4 = reinterpret_cast<const float4*>(src + kb * 16);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 v = valid ? s4[u] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      x[4 * u] = v.x; x[4 * u + 1] = v.y; x[4 * u + 2] = v.z; x[4 * u + 3] = v.w;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) ss = __builtin_fmaf(x[u], x[u], ss);
    bf3_split_store(x, out + ((int64_t)kb * out_pad + c) * 4);
  }
  ss += __shfl_xor(ss, 1);
  ss += __shfl_xor(ss, 2);
  ss += __shfl_xor(ss, 4);
  const float nv = valid ? fmaxf(sqrtf(ss), 0x1p-30f) : 0.0f;
  if (j == 0) norms[c] = nv;
  if (bmax) {
    float m = nv;  // the 8 rows of this wave (lanes 0, 8, .., 56 hold distinct rows)
    m = fmaxf(m, __shfl_xor(m, 8));
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) bmax[blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
  }
}

// The bound's 2-norms, one wave per row of a row-major copy (rows r0 .. r0 + n_out - 1, K
// floats each; rows >= n_rows get 0 -- padding the sweep never counts): |x|_2 clamped to
// >= 2^-30, inf / NaN kept (the bound is then inf / NaN: undecided). Any summation order
// serves -- the bound's 2 % slack covers the norm's rounding.
// With thr_out (the query rows of the wide sweep, k_sweep_bf3w): also the padded per-row side
// data its DMA copies whole -- thr_out[i] = the threshold (-inf past the queries: nothing beats
// a padded row) and qb_out[i] = cb |q|.
__global__ __launch_bounds__(256) void k_bf3_norms(const float* __restrict__ rows, int64_t n_rows, int64_t r0,
                                                   int64_t n_out, int ktot, float* __restrict__ norms,
                                                   const float* __restrict__ thr_in, float* __restrict__ thr_out,
                                                   float* __restrict__ qb_out, float cb) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n_out) return;
  const int64_t r = r0 + i;
  float ss = 0.0f;
  if (r < n_rows) {
    const float* x = rows + r * (int64_t)ktot;
    for (int k = lane; k < ktot; k += 64) ss = __builtin_fmaf(x[k], x[k], ss);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  if (lane == 0) {
    const float nv = r < n_rows ? fmaxf(sqrtf(ss), 0x1p-30f) : 0.0f;
    norms[i] = nv;
    if (thr_out) {
      thr_out[i] = r < n_rows ? thr_in[r] : -INFINITY;
      qb_out[i] = cb * nv;
    }
  }
}

// The entity norms of the wide sweep: k_bf3_norms' rows (one wave per row, 8 rows per wave) and,
// per block of 32 consecutive columns, their largest norm (bmax[blockIdx.x]; NaN norms skipped by
// fmaxf -- such a row's S' is NaN, undecided whatever the bound), the bound factor of
// k_sweep_bf3w's thresholds.
__global__ __launch_bounds__(256) void k_bf3_enorms(const float* __restrict__ rows, int64_t n_rows, int64_t r0,
                                                    int64_t n_out, int ktot, float* __restrict__ norms,
                                                    float* __restrict__ bmax) {
  __shared__ float wm[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ss[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) ss[t] = 0.0f;
  const int64_t rb = r0 + (int64_t)blockIdx.x * 32 + wave * 8;
  for (int k = lane; k < ktot; k += 64) {
    float x[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {  // the wave's 8 rows' loads in flight together (past the table: its last row, unused)
      const int64_t r = rb + t < n_rows ? rb + t : n_rows - 1;
      x[t] = rows[r * (int64_t)ktot + k];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) ss[t] = __builtin_fmaf(x[t], x[t], ss[t]);
  }
  float m = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int64_t i = (int64_t)blockIdx.x * 32 + wave * 8 + t;
    const int64_t r = r0 + i;
    float v = ss[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const float nv = r < n_rows ? fmaxf(sqrtf(v), 0x1p-30f) : 0.0f;
    if (lane == 0 && i < n_out) norms[i] = nv;
    if (i < n_out) m = fmaxf(m, nv);
  }
  if (lane == 0) wm[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) bmax[blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// The sweep: units, grid and staging as k_sweep_mfma's 16-row plain variant (4 workgroups per
// CU, ballot row counters), one split block (16 k) per stage: 8 KB per operand tile, read into
// LDS as 16-B chunks at position chunk ^ ((row >> 2) & 3) of the row's 64 B (the 32 lanes of
// an MFMA operand read hit 32 different 16-B bank groups: conflict-free).
template <int PK>
__global__ __launch_bounds__(NT, BF3_WG_PER_CU) void k_sweep_bf3(
    const uint4* __restrict__ ent_b, int64_t e_pad, int64_t n_ent, const uint4* __restrict__ q_b, int64_t q_pad,
    int64_t n_query, int nkb, int n_et, int e_base, int n_groups, int pred_kind, float margin,
    const float* __restrict__ thr, const float* __restrict__ qn, const float* __restrict__ en, float cb,
    int32_t* __restrict__ counts, uint32_t* __restrict__ hdr, int2* __restrict__ pairs, int64_t cap, int emajor,
    int blk_qb, int blk_eb) {
  __shared__ uint4 sq[2][TQ * 4];
  __shared__ uint4 se[2][TE * 4];
  __shared__ __attribute__((aligned(16))) float s_th[2][TQ];
  __shared__ __attribute__((aligned(16))) float s_qb[2][TQ];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const PredSel<PK> pred(pred_kind, margin);
  const int wq = wave >> 1, we = wave & 1;
  const int lrow = lane >> 5, lcol = lane & 31;
  const int grp = blockIdx.x % n_groups, gmem = blockIdx.x / n_groups;
  const int per_grp = gridDim.x / n_groups;
  // blk_qb > 0: the lock-step window order (BlockMap, one unit range per member); else the
  // contiguous ranges of UnitMap
  const bool blocked = blk_qb > 0;
  const UnitMap um(grp, n_groups, (int)(q_pad / TQ), n_et, emajor != 0);
  const BlockMap bm(grp, n_groups, gmem, per_grp, (int)(q_pad / TQ), n_et, blocked ? blk_qb : 1, blocked ? blk_eb : 1);
  const int u0 = blocked ? 0 : (int)((int64_t)gmem * um.count / per_grp);
  const int u1 = blocked ? bm.count : (int)((int64_t)(gmem + 1) * um.count / per_grp);
  if (u0 >= u1) return;  // uniform over the workgroup
  auto unit_at = [&](int i, int& qt, int& et) {
    if (blocked) bm.at(i, qt, et);
    else um.at(i, qt, et);
  };

  int tpar = 0;
  int cntv = 0;  // lane L: the count of wave row L (tile row wq * 64 + L) in the current query tile
  auto row_of = [&](int bi, int r) { return wq * 64 + bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lrow; };
  auto load_rows = [&](int qtile) {
    const int64_t q0 = (int64_t)qtile * TQ;
    tpar ^= 1;
    if (tid < TQ) {
      const int64_t q = q0 + tid;
      s_th[tpar][tid] = q < n_query ? thr[q] : -INFINITY;  // -inf: nothing beats a padded row
      s_qb[tpar][tid] = q < n_query ? cb * qn[q] : 0.0f;
    }
    cntv = 0;
  };
  auto flush_rows = [&](int qtile) {
    const int64_t q = (int64_t)qtile * TQ + wq * 64 + lane;
    if (q < n_query && cntv) atomicAdd(&counts[q], cntv);  // raw only (k_counts_finalize)
  };
  auto sidx = [](int row, int c) { return row * 4 + (c ^ ((row >> 2) & 3)); };

  uint4 rq0, rq1, re0, re1;
  int ld_unit = u0, ld_kb = 0, ld_qt, ld_et;
  unit_at(u0, ld_qt, ld_et);
  auto gload = [&]() {
    const uint4* qp = q_b + ((int64_t)ld_kb * q_pad + (int64_t)ld_qt * TQ) * 4;
    const uint4* ep = ent_b + ((int64_t)ld_kb * e_pad + (int64_t)ld_et * TE) * 4;
    rq0 = qp[tid];
    rq1 = qp[tid + NT];
    re0 = ep[tid];
    re1 = ep[tid + NT];
    if (++ld_kb == nkb) {
      ld_kb = 0;
      if (++ld_unit < u1) unit_at(ld_unit, ld_qt, ld_et);
    }
  };
  auto swrite = [&](int buf) {
    const int r0 = tid >> 2, c = tid & 3;
    sq[buf][sidx(r0, c)] = rq0;
    sq[buf][sidx(r0 + 64, c)] = rq1;
    se[buf][sidx(r0, c)] = re0;
    se[buf][sidx(r0 + 64, c)] = re1;
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  int cur_qt, cur_et;
  unit_at(u0, cur_qt, cur_et);
  load_rows(cur_qt);
  gload();
  swrite(0);
  __syncthreads();

  int buf = 0;
  for (int unit = u0; unit < u1; ++unit) {
    for (int kb = 0; kb < nkb; ++kb) {
      const bool more = ld_unit < u1;
      if (more) gload();
      __builtin_amdgcn_sched_barrier(0);  // the next stage's loads stay at the top (k_sweep_mfma)
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int qrow = wq * 64 + i * 32 + lcol, ecol = we * 64 + i * 32 + lcol;
        ah[i] = __builtin_bit_cast(bf16x8, sq[buf][sidx(qrow, lrow)]);
        al[i] = __builtin_bit_cast(bf16x8, sq[buf][sidx(qrow, 2 + lrow)]);
        bh[i] = __builtin_bit_cast(bf16x8, se[buf][sidx(ecol, lrow)]);
        bl[i] = __builtin_bit_cast(bf16x8, se[buf][sidx(ecol, 2 + lrow)]);
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
          acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[bi], bh[bj], acc[bi][bj], 0, 0, 0);
          acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[bi], bl[bj], acc[bi][bj], 0, 0, 0);
          acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[bi], bh[bj], acc[bi][bj], 0, 0, 0);
        }
      if (kb == nkb - 1) {  // unit finished: decide, count, list the undecided
        const int64_t q0 = (int64_t)cur_qt * TQ;
        const int64_t ebase = (int64_t)cur_et * TE + we * 64;
        const int64_t e0 = ebase + lcol, e1 = ebase + 32 + lcol;
        const bool ev0 = e0 < n_ent, ev1 = e1 < n_ent;
        const float ne0 = ev0 ? en[e0] : 0.0f, ne1 = ev1 ? en[e1] : 0.0f;
        const uint64_t evm[2] = {__ballot(ev0), __ballot(ev1)};
        // this unit's per-row counts, assembled lane by lane: row L0's count into lane L0 by
        // v_writelane (the popcounts are wave-uniform), one add into cntv at the end -- a
        // `lane == L0 ? c : ...` select per row made the compiler keep 32 lane-compare masks
        // live across the sweep (SGPR spills into VGPR lanes)
        // Per pair: the bound (one multiply), S' - B and S' + B, and three compares whose results
        // are the wave's masks (v_cmp into an SGPR pair: "beats at both ends", "beats at neither",
        // non-finite S'); what is counted and what is listed is 64-bit mask logic on the scalar
        // unit, per row and column block (round 4's per-lane booleans: ~21 VALU instructions per
        // pair at C5 -- as many issue cycles as the three MFMAs)
        int ctmp = 0;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int r4 = 0; r4 < 16; r4 += 4) {  // four rows' thresholds and bound factors per LDS read pair
            const float4 t4 = *reinterpret_cast<const float4*>(&s_th[tpar][row_of(bi, r4)]);
            const float4 b4 = *reinterpret_cast<const float4*>(&s_qb[tpar][row_of(bi, r4)]);
            const float tv[4] = {t4.x, t4.y, t4.z, t4.w}, qb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int r = r4; r < r4 + 4; ++r) {
            const uint64_t mnan = __ballot(tv[r - r4] != tv[r - r4]);  // a NaN threshold: nothing beats it
            uint64_t msure[2], mund[2];
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) {
              const float s = acc[bi][bj][r];
              const float bnd = qb[r - r4] * (bj ? ne1 : ne0);
              uint64_t hi, lo;
              if constexpr (PK == 2) {
                // predict = -s: better iff S > -th. Rounding is monotone, so fl(s - B) > -th
                // implies s - B > -th (every S of the bracket beats the truth) and
                // fl(s + B) < -th implies s + B < -th (none does); a NaN S' or bound decides nothing
                const float nt = -tv[r - r4];
                hi = __ballot(s - bnd > nt);
                lo = __ballot(s + bnd < nt);
              } else {
                const float p1 = pred(s - bnd), p2 = pred(s + bnd);
                hi = __ballot(fmaxf(p1, p2) < tv[r - r4]);
                lo = __ballot(fminf(p1, p2) >= tv[r - r4]);
              }
              const uint64_t nf = __ballot(!__builtin_isfinite(s));  // inf and NaN: undecided
              msure[bj] = hi & ~nf & evm[bj];
              mund[bj] = evm[bj] & ~(msure[bj] | (lo & ~nf) | mnan);
            }
            const int L0 = bi * 32 + (r & 3) + 8 * (r >> 2);
            const int c_lo = __popcll(msure[0] & 0xffffffffull) + __popcll(msure[1] & 0xffffffffull);
            const int c_hi = __popcll(msure[0] >> 32) + __popcll(msure[1] >> 32);
            ctmp = writelane_imm(ctmp, c_lo, L0);
            ctmp = writelane_imm(ctmp, c_hi, L0 + 4);
            if (__builtin_expect((mund[0] | mund[1]) != 0ull, 0)) {  // rare (uniform): list the pair(s) for exact rescoring
              // (the row from an opaque lane id: recomputed here, not 32 row indices kept live)
              const int ol = vgpr_opaque(lane);
              const int64_t q = q0 + wq * 64 + bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ol >> 5);
              if (q < n_query) {
#pragma unroll
                for (int bj = 0; bj < 2; ++bj) {
                  if (!((mund[bj] >> ol) & 1ull)) continue;
                  bf3_list(hdr, pairs, cap, make_int2((int)q, (int)((bj ? e1 : e0) + e_base)));
                }
              }
            }
          }
        }
        cntv += ctmp;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[bi][bj][r] = 0.0f;
        const bool last = unit + 1 >= u1;
        int next_qt = cur_qt, next_et = cur_et;
        if (!last) unit_at(unit + 1, next_qt, next_et);
        if (last || next_qt != cur_qt) {  // uniform: leave this query tile
          flush_rows(cur_qt);
          if (!last) load_rows(next_qt);
        }
        cur_qt = next_qt;
        cur_et = next_et;
      }
      if (more) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
}

// The wide variant (round 5). k_sweep_bf3 stages one 16-k split block per barrier through
// registers at 128 x 128 per workgroup and decides each pair with a per-pair bound and mask
// logic on the scalar unit (~40 scalar + ~20 vector instructions per 64 pairs): at C5 it held
// ~0.33 of the bf16 MFMA peak, with the decision pass alone ~18 % of the time and the operand
// traffic from L2 (134 GB per launch) the rest of the ceiling. Here:
//  * a workgroup covers QT queries x 256 entities, waves of 64 queries x 128 entities
//    (QT = 128: 4 waves, two workgroups per CU; QT = 256: 8 waves, one per CU, 1.5x the MFMAs
//    per operand byte): 24 MFMAs per stage per wave for 12 ds_read_b128;
//  * stages are copied global -> LDS by the DMA path (global_load_lds_dwordx4: no staging
//    registers, no ds_write) into three buffers, two stages in flight across each barrier (a
//    counted s_waitcnt vmcnt, a raw s_barrier); the per-unit side data -- the entity tile's |e|,
//    the query tile's thresholds and bound factors cb |q| -- rides with the unit's first stage;
//  * the MFMA's A operand is the entity rows and B the queries, so a lane's accumulator values
//    all belong to two queries (its columns): per-lane thresholds in registers, per-lane counts
//    (one compare + one add-with-carry per 64 pairs), and the bound is taken per 32-entity
//    block -- B = cb |q| max|e| over the block -- folded into two thresholds per query,
//    T_hi >= -thr + B and T_lo <= -thr - B (one ulp outward of the rounded sums): S' > T_hi
//    beats the truth for every S within the bound, S' < T_lo for none, anything else (NaN S'
//    included: both compares fail) is undecided and listed. No S' is +-inf unless |q| max|e|
//    overflows, and then B and the thresholds are inf: the block's pairs are undecided
//    (conservative; an inf-norm row costs its block's 32 x n_query pairs on the list).
//    Per 64 pairs: two compares, one add, two scalar ORs for the per-block "any undecided"
//    flag; blocks with a flag are re-scanned for the list (rare: truths and near ties).
// LDS image of a stage: the query rows then the entity rows, 64 B each (hi[16] | lo[16]),
// 16-B chunk c of row r at slot 4 r + (c ^ ((r >> 2) & 3)) as k_sweep_bf3's (conflict-free
// operand reads); the DMA writes a wave-instruction's 1 KB lane-linearly, so the swizzle is
// applied to the source addresses.
constexpr int W3E = 256;
#ifndef W3_DEEP
#define W3_DEEP 0  // 1: four stage buffers at QT = 256 (three stages in flight; A/B)
#endif
#ifndef W3_PAIR
#define W3_PAIR 0  // 1: four stage buffers, one barrier per two stages (A/B)
#endif
template <int QT>
struct W3Geom {
  static constexpr int WAVES = QT / 32;                 // (QT / 64) x 2 waves
  static constexpr int NT = WAVES * 64;
  static constexpr int QB = QT * 64, STAGE = QB + W3E * 64;
  static constexpr int EPW = W3E * 64 / 1024 / WAVES;   // entity DMA instructions per wave and stage
  static constexpr int NDMA = 2 + EPW;                  // + two for the query rows
  static constexpr int SIDE = 1024 + 8 * QT;            // block max |e| [8] (1 KB piece) | threshold [QT] | cb |q| [QT]
  static constexpr int PIECES = SIDE / 1024;            // side DMA instructions (waves 0 .. PIECES - 1)
  static constexpr int NBUF = ((W3_DEEP && QT == 256) || W3_PAIR) ? 4 : 3;  // stage (and side) buffers
  static constexpr int LDS = NBUF * (STAGE + SIDE);
  static constexpr int WG_PER_CU = QT == 128 ? 2 : 1;
};

__device__ __forceinline__ void w3_glds(const void* src, char* lds_dst) {  // lds_dst wave-uniform
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}
// wait until at most n of this wave's vector-memory operations are outstanding (n wave-uniform:
// the DMA instructions issued for the next stage, 0 / NDMA / NDMA + 1)
template <int NDMA>
__device__ __forceinline__ void w3_wait(int n) {
  if (n == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == NDMA) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA + 1) : "memory");
}
template <int N>
__device__ __forceinline__ void w3_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void w3_wait_n(int n) {  // n wave-uniform, 0 .. 15 (a larger n: wait for all)
  switch (n) {
    case 1: w3_vmwait<1>(); break;
    case 2: w3_vmwait<2>(); break;
    case 3: w3_vmwait<3>(); break;
    case 4: w3_vmwait<4>(); break;
    case 5: w3_vmwait<5>(); break;
    case 6: w3_vmwait<6>(); break;
    case 7: w3_vmwait<7>(); break;
    case 8: w3_vmwait<8>(); break;
    case 9: w3_vmwait<9>(); break;
    case 10: w3_vmwait<10>(); break;
    case 11: w3_vmwait<11>(); break;
    case 12: w3_vmwait<12>(); break;
    case 13: w3_vmwait<13>(); break;
    case 14: w3_vmwait<14>(); break;
    case 15: w3_vmwait<15>(); break;
    default: w3_vmwait<0>(); break;
  }
}
__device__ __forceinline__ float w3_next_up(float x) {  // the next float above x (x not NaN, inf kept; selects)
  const uint32_t u = __float_as_uint(x);
  const uint32_t r = x == 0.0f ? 1u : (x > 0.0f ? u + 1u : u - 1u);  // +-0 -> the smallest subnormal
  return x == INFINITY ? x : __uint_as_float(r);
}

// BLK: the lock-step XCD windows (BlockMap) or contiguous ranges (UnitMap), a template parameter
// so that only one map's state lives in registers
template <int PK, int QT, bool BLK>
__global__ __launch_bounds__(W3Geom<QT>::NT, W3Geom<QT>::WG_PER_CU) void k_sweep_bf3w(
    const uint4* __restrict__ ent_b, int64_t e_pad, int64_t e_cols, int64_t n_ent, const uint4* __restrict__ q_b,
    int64_t q_pad, int64_t n_query, int nkb, int n_et, int e_base, int n_groups, const float* __restrict__ thr_pad,
    const float* __restrict__ qbf, const float* __restrict__ en /* block maxima */, int32_t* __restrict__ counts,
    uint32_t* __restrict__ hdr, int2* __restrict__ pairs, int64_t cap, int emajor, int blk_qb, int blk_eb) {
  static_assert(PK == 2, "the wide sweep folds the bound into thresholds on S (prediction = -S)");
  using G = W3Geom<QT>;
  __shared__ __attribute__((aligned(16))) char lds[G::LDS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = wave >> 1, we = wave & 1;
  const int lrow = lane >> 5, lcol = lane & 31;
  const int grp = blockIdx.x % n_groups, gmem = blockIdx.x / n_groups;
  const int per_grp = gridDim.x / n_groups;
  const int n_qt = (int)(q_pad / QT);
  auto make_map = [&]() {
    if constexpr (BLK) return BlockMap(grp, n_groups, gmem, per_grp, n_qt, n_et, blk_qb, blk_eb);
    else return UnitMap(grp, n_groups, n_qt, n_et, emajor != 0);
  };
  const auto map = make_map();
  const int u0 = BLK ? 0 : (int)((int64_t)gmem * map.count / per_grp);
  const int u1 = BLK ? map.count : (int)((int64_t)(gmem + 1) * map.count / per_grp);
  if (u0 >= u1) return;  // uniform over the workgroup
  auto unit_at = [&](int i, int& qt, int& et) { map.at(i, qt, et); };
  auto sidx = [](int row, int c) { return row * 4 + (c ^ ((row >> 2) & 3)); };

  // the DMA cursor: the stage (unit, k block) whose copies are issued next, and its buffers.
  // Per lane, the source offsets (uint4 units) of its DMA rows are fixed: the query rows'
  // relative to the query tile, the entity rows' (clamped to the slice's last column) set once
  // per unit; a stage adds only the uniform k-block plane base (round 6: the per-stage 64-bit
  // address arithmetic had been ~30 VALU per wave and stage, plus SGPR spill traffic).
  const int sl = lane & 3;
  uint32_t qoff[2], erow[G::EPW], eoff[G::EPW];
#pragma unroll
  for (int j = 0; j < 2; ++j) {  // query rows 32 wave .. + 31: two 1-KB instructions of 16 rows
    const int row = 16 * (wave * 2 + j) + (lane >> 2);
    qoff[j] = (uint32_t)(row * 4 + (sl ^ ((row >> 2) & 3)));
  }
#pragma unroll
  for (int j = 0; j < G::EPW; ++j) erow[j] = (uint32_t)(16 * (wave * G::EPW + j) + (lane >> 2));
  int ld_unit = u0, ld_kb = 0, ld_qt, ld_et, ld_buf = 0, ld_sbuf = 0;
  auto enter_unit = [&]() {  // the cursor's unit: its tiles and the entity rows' offsets
    unit_at(ld_unit, ld_qt, ld_et);
    const uint32_t c0 = (uint32_t)ld_et * W3E, last = (uint32_t)e_cols - 1u;
#pragma unroll
    for (int j = 0; j < G::EPW; ++j) {  // past the slice's columns: its last one
      const uint32_t er = c0 + erow[j] <= last ? c0 + erow[j] : last;
      eoff[j] = er * 4u + (uint32_t)(sl ^ ((erow[j] >> 2) & 3));
    }
  };
  enter_unit();
  auto issue = [&]() -> int {  // this wave's share of the cursor's stage; returns its instruction count
    if (ld_unit >= u1) return 0;
    char* sb = lds + ld_buf * G::STAGE;
    const int64_t q0 = (int64_t)ld_qt * QT;
    const uint4* qp = q_b + ((int64_t)ld_kb * q_pad + q0) * 4;
    const uint4* ep = ent_b + (int64_t)ld_kb * e_pad * 4;
#pragma unroll
    for (int j = 0; j < 2; ++j) w3_glds(qp + qoff[j], sb + (wave * 2 + j) * 1024);
#pragma unroll
    for (int j = 0; j < G::EPW; ++j) w3_glds(ep + eoff[j], sb + G::QB + (wave * G::EPW + j) * 1024);
    int n = G::NDMA;
    if (ld_kb == 0 && wave < G::PIECES) {  // the unit's side data, one 1-KB piece per wave
      char* sd = lds + G::NBUF * G::STAGE + ld_sbuf * G::SIDE + wave * 1024;
      const int64_t c0 = (int64_t)ld_et * W3E;
      const float* src;
      if (wave == 0) {  // the tile's 8 block maxima (lanes 0-1; the others re-read them)
        src = en + (c0 / 32 + 4 * (lane & 1) + 4 <= e_cols / 32 ? c0 / 32 + 4 * (lane & 1) : e_cols / 32 - 4);
      } else {  // [threshold | cb |q|] of the tile's QT queries
        const int f = (wave - 1) * 256 + 4 * lane;
        src = f < QT ? thr_pad + q0 + f : qbf + q0 + (f - QT);
      }
      w3_glds(src, sd);
      n = G::NDMA + 1;
    }
    ld_buf = ld_buf == G::NBUF - 1 ? 0 : ld_buf + 1;
    if (++ld_kb == nkb) {
      ld_kb = 0;
      ld_sbuf = ld_sbuf == G::NBUF - 1 ? 0 : ld_sbuf + 1;
      if (++ld_unit < u1) enter_unit();
    }
    return n;
  };

  // lane L: the count of query wq * 64 + j * 32 + (L & 31) of the current query tile over the
  // entity rows it holds (lanes L and L ^ 32 hold the same query)
  int cnt[2] = {0, 0};
  auto flush_rows = [&](int qtile) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = cnt[j] + __shfl_xor(cnt[j], 32);
      const int64_t q = (int64_t)qtile * QT + wq * 64 + j * 32 + lcol;
      if (lrow == 0 && q < n_query && c) atomicAdd(&counts[q], c);  // raw only (k_counts_finalize)
      cnt[j] = 0;
    }
  };

  floatx16 acc[4][2];  // [entity block][query block]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  // the decision pass of a finished unit; FULL: every entity of the wave's 128 is in the slice
  // (else the first nval are). Entity of (bi, r, lane): ebase + bi * 32 + (r & 3) + 8 (r >> 2) +
  // 4 lrow -- the lanes 0-31 / 32-63 halves of a register hold two entity rows, so a row's
  // validity is a wave-uniform half mask.
  // Thresholds of the lane's two queries against entity block bi (32 rows of the wave's 128):
  // B = cb |q| max |e| over the block (k_bf3_enorms: a NaN norm is skipped, and that row's S' is
  // NaN: undecided; blocks past the slice hold no counted row), T_hi >= nt + B,
  // T_lo <= nt - B one ulp outward of the rounded sums.
  // (branch-free: per-lane branches here cost exec-mask juggling on every unit)
  auto thresholds = [&](float nm, const float nt[2], const float qbv[2], float th[2], float tl[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float b = qbv[j] * nm, a = nt[j] + b, c = nt[j] - b;
      const bool nt_nan = nt[j] != nt[j];       // a NaN threshold: nothing beats it (decided)
      const bool bad = a != a || c != c;        // a NaN / inf bound (inf - inf): every pair undecided
      th[j] = nt_nan || bad ? INFINITY : w3_next_up(a);
      tl[j] = nt_nan ? INFINITY : (bad ? -INFINITY : -w3_next_up(-c));
    }
  };
  // the decision pass of a finished unit; FULL: every entity of the wave's 128 is in the slice
  // (else the first nval are). Entity of (bi, r, lane): ebase + bi * 32 + (r & 3) + 8 (r >> 2) +
  // 4 lrow -- the lanes 0-31 / 32-63 halves of a register hold two entity rows, so a row's
  // validity is a wave-uniform half mask. nt: -threshold of the lane's queries; qbv: cb |q|.
  auto decide = [&](auto full_tag, const float* s_bm, int64_t q0, int64_t ebase, int nval, float nt0, float nt1,
                    float qb0, float qb1) {
    constexpr bool FULL = decltype(full_tag)::value;
    // (opaque copies: the two instances' compares are not merged and hoisted above the branch
    // between them -- with all 256 masks live)
    const float nt[2] = {vgpr_opaque_f(nt0), vgpr_opaque_f(nt1)};
    const float qbv[2] = {vgpr_opaque_f(qb0), vgpr_opaque_f(qb1)};
    // the wave's four block maxima: one LDS read, held in SGPRs (wave-uniform)
    const float4 bm4 = *reinterpret_cast<const float4*>(&s_bm[we * 4]);
    auto rfl = [](float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); };
    const float nmb[4] = {rfl(bm4.x), rfl(bm4.y), rfl(bm4.z), rfl(bm4.w)};
    uint64_t und[4][2];
#pragma unroll
    for (int bi = 0; bi < 4; ++bi) {
      float thi[2], tlo[2];
      thresholds(nmb[bi], nt, qbv, thi, tlo);
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        uint64_t u = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float s = acc[bi][bj][r];
          bool h = s > thi[bj];
          uint64_t vm = ~0ull;
          if constexpr (!FULL) {
            const int row0 = bi * 32 + (r & 3) + 8 * (r >> 2);
            vm = (row0 < nval ? 0xffffffffull : 0ull) | (row0 + 4 < nval ? 0xffffffff00000000ull : 0ull);
            h = h && row0 + 4 * lrow < nval;
          }
          cnt[bj] += h ? 1 : 0;
          u |= vm & ~(__ballot(h) | __ballot(s < tlo[bj]));
          // consumed here, group by group: left alone the compiler hoists all 128 groups'
          // compares and re-associates the sums, keeping 256 masks live (SGPR spills)
          cnt[bj] = vgpr_opaque(cnt[bj]);
          u = sgpr_opaque64(u);
        }
        und[bi][bj] = u;
      }
    }
#pragma unroll
    for (int bi = 0; bi < 4; ++bi) {
      if (__builtin_expect((und[bi][0] | und[bi][1]) != 0ull, 0)) {  // rare (uniform): list the undecided pairs
        // the thresholds recomputed from opaque copies: the compares are redone here, not the
        // pass's masks kept live (the compiler would merge the two)
        const float ntc[2] = {vgpr_opaque_f(nt[0]), vgpr_opaque_f(nt[1])};
        float th[2], tl[2];
        thresholds(nmb[bi], ntc, qbv, th, tl);
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
          if (und[bi][bj] == 0ull) continue;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float s = acc[bi][bj][r];
            const int row0 = bi * 32 + (r & 3) + 8 * (r >> 2);
            uint64_t um = ~(__ballot(s > th[bj]) | __ballot(s < tl[bj]));
            if constexpr (!FULL)
              um &= (row0 < nval ? 0xffffffffull : 0ull) | (row0 + 4 < nval ? 0xffffffff00000000ull : 0ull);
            if (um == 0ull) continue;  // uniform
            // (the lane's query and entity from an opaque lane id: recomputed here, not 64 indices
            // kept live across the sweep)
            const int ol = vgpr_opaque(lane);
            const int64_t q = q0 + wq * 64 + bj * 32 + (ol & 31);
            if (((um >> ol) & 1ull) && q < n_query)
              bf3_list(hdr, pairs, cap, make_int2((int)q, (int)(ebase + row0 + 4 * (ol >> 5) + e_base)));
          }
        }
      }
    }
  };

  issue();               // stage 0
  int nxt = issue();     // stage 1: the instructions still allowed in flight when stage 0 is read
  int nxt2 = (G::NBUF == 4 && !W3_PAIR) ? issue() : 0;  // (four buffers) stage 2 as well
  int g = 0;  // stages swept by this workgroup
  int cur_qt, cur_et;
  unit_at(u0, cur_qt, cur_et);
  int buf = 0, sbuf = 0;
  for (int unit = u0; unit < u1; ++unit) {
    for (int kb = 0; kb < nkb; ++kb) {
      if constexpr (W3_PAIR) {
        // one barrier per two stages: at an even stage every copy of this pair has landed
        // (nothing else is in flight), then the next pair's two stages are issued into the
        // buffers the previous pair was read from
        if ((g & 1) == 0) {
          w3_vmwait<0>();
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          issue();
          issue();
        }
      } else {
        if constexpr (G::NBUF == 4) w3_wait_n(nxt + nxt2);
        else w3_wait<G::NDMA>(nxt);  // this wave's copies of the stage have landed ...
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // ... and every wave's; every wave is done with the buffer refilled next
        asm volatile("" ::: "memory");
        if constexpr (G::NBUF == 4) {
          nxt = nxt2;
          nxt2 = issue();  // three stages ahead
        } else {
          nxt = issue();  // the stage after next, into the buffer read in the previous stage
        }
      }
      ++g;
      const uint4* sq = reinterpret_cast<const uint4*>(lds + buf * G::STAGE);
      const uint4* se = reinterpret_cast<const uint4*>(lds + buf * G::STAGE + G::QB);
      bf16x8 eh[4], el[4], qh[2], ql[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int erow = we * 128 + i * 32 + lcol;
        eh[i] = __builtin_bit_cast(bf16x8, se[sidx(erow, lrow)]);
        el[i] = __builtin_bit_cast(bf16x8, se[sidx(erow, 2 + lrow)]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int qrow = wq * 64 + j * 32 + lcol;
        qh[j] = __builtin_bit_cast(bf16x8, sq[sidx(qrow, lrow)]);
        ql[j] = __builtin_bit_cast(bf16x8, sq[sidx(qrow, 2 + lrow)]);
      }
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
          acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(eh[bi], qh[bj], acc[bi][bj], 0, 0, 0);
          acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(el[bi], qh[bj], acc[bi][bj], 0, 0, 0);
          acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(eh[bi], ql[bj], acc[bi][bj], 0, 0, 0);
        }
      buf = buf == G::NBUF - 1 ? 0 : buf + 1;
      if (kb == nkb - 1) {  // unit finished: decide, count, list the undecided
        const float* s_bm = reinterpret_cast<const float*>(lds + G::NBUF * G::STAGE + sbuf * G::SIDE);
        const float* s_th = s_bm + 256;
        const float* s_qb = s_th + QT;
        const int64_t q0 = (int64_t)cur_qt * QT;
        const int64_t ebase = (int64_t)cur_et * W3E + we * 128;
        float ntv[2], qbv[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ql_ = wq * 64 + j * 32 + lcol;
          ntv[j] = -s_th[ql_];  // prediction -S beats the truth iff S > nt
          qbv[j] = s_qb[ql_];
        }
        if (ebase + 128 <= n_ent) decide(std::true_type{}, s_bm, q0, ebase, 128, ntv[0], ntv[1], qbv[0], qbv[1]);
        else decide(std::false_type{}, s_bm, q0, ebase, (int)(n_ent > ebase ? n_ent - ebase : 0), ntv[0], ntv[1],
                    qbv[0], qbv[1]);
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[bi][bj][r] = 0.0f;
        sbuf = sbuf == G::NBUF - 1 ? 0 : sbuf + 1;
        const bool last = unit + 1 >= u1;
        int next_qt = cur_qt, next_et = cur_et;
        if (!last) unit_at(unit + 1, next_qt, next_et);
        if (last || next_qt != cur_qt) flush_rows(cur_qt);  // uniform: leave this query tile
        cur_qt = next_qt;
        cur_et = next_et;
      }
    }
  }
}

// Overflowed list: reset the raw counts the filter sweep added (the truth pass left them 0);
// the gated f32 sweep that follows recounts them.
__global__ __launch_bounds__(256) void k_bf3_fallback_zero(const uint32_t* __restrict__ hdr,
                                                           int32_t* __restrict__ counts, int64_t n_query) {
  if (hdr[1] == 0u) return;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n_query) counts[q] = 0;
}

// The listed pairs, one thread each: the canonical chain (acc = fma(e_k, q_k, acc), k in
// order -- the truth kernels' and the f32 MFMA's arithmetic) from the row-major copies, and
// the strict Test.h compare against the query's threshold.
template <int PK>
__global__ __launch_bounds__(256) void k_bf3_rescore(const uint32_t* __restrict__ hdr, const int2* __restrict__ pairs,
                                                     int64_t cap, const float* __restrict__ q_rows,
                                                     const float* __restrict__ ent_rows, int ktot, int pred_kind,
                                                     float margin, const float* __restrict__ thr,
                                                     int32_t* __restrict__ counts) {
  if (hdr[1] != 0u) return;  // overflow: the exact sweep counted everything
  const PredSel<PK> pred(pred_kind, margin);
  // gridDim.x / (BF3_SEGS + 1) workgroups per segment; segment BF3_SEGS: the shared half
  const int sgm = (int)(blockIdx.x % (BF3_SEGS + 1)), part = (int)(blockIdx.x / (BF3_SEGS + 1));
  const int parts = (int)(gridDim.x / (BF3_SEGS + 1));
  const int64_t seg_cap = cap / (2 * BF3_SEGS);
  const int64_t scap = sgm < BF3_SEGS ? seg_cap : cap - BF3_SEGS * seg_cap;
  const int64_t listed = hdr[BF3_SEG_W0 + 32 * sgm];
  const int64_t n = listed < scap ? listed : scap;
  const int2* seg = pairs + sgm * seg_cap;
  for (int64_t i = (int64_t)part * blockDim.x + threadIdx.x; i < n; i += (int64_t)parts * blockDim.x) {
    const int2 p = seg[i];
    const float4* a = reinterpret_cast<const float4*>(q_rows + (int64_t)p.x * ktot);
    const float4* b = reinterpret_cast<const float4*>(ent_rows + (int64_t)p.y * ktot);
    float acc = 0.0f;
#pragma unroll 4
    for (int k = 0; k < ktot / 4; ++k) {
      const float4 x = b[k], y = a[k];
      acc = __builtin_fmaf(x.x, y.x, acc);
      acc = __builtin_fmaf(x.y, y.y, acc);
      acc = __builtin_fmaf(x.z, y.z, acc);
      acc = __builtin_fmaf(x.w, y.w, acc);
    }
    if (pred(acc) < thr[p.x]) atomicAdd(&counts[p.x], 1);
  }
}

// the list header zeroed, with word 4 = the segment capacity (read by k_bf3_stats)
__global__ __launch_bounds__(256) void k_bf3_hdr_init(uint32_t* __restrict__ hdr, int64_t cap) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < BF3_HDR / 4; i += gridDim.x * blockDim.x)
    hdr[i] = i == 4 ? (uint32_t)(cap / (2 * BF3_SEGS)) : 0u;
}

__global__ void k_bf3_stats(const uint32_t* __restrict__ hdr, unsigned long long* __restrict__ out) {
  // one wave: the pairs listed = the segments' kept appends + the shared half's appends (a full
  // segment's further appends are counted there; past the shared half's end: the fallback ran)
  const int64_t seg_cap = hdr[4];
  unsigned long long t = 0;
  if (threadIdx.x < BF3_SEGS) {
    const unsigned long long c = hdr[BF3_SEG_W0 + 32 * threadIdx.x];
    t = c < (unsigned long long)seg_cap ? c : (unsigned long long)seg_cap;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
  if (threadIdx.x == 0) {
    out[0] = t + hdr[BF3_SEG_W0 + 32 * BF3_SEGS];
    out[1] = hdr[1];
  }
}

// ---------------------------------------------------------------- launch ---
// Resident workgroups of a persistent sweep: the occupancy API's blocks per CU (capped at 4,
// the VGPR-limited residency of a 256-thread group at <= 128 VGPRs) x the device's CUs.
static int resident_groups(const void* kernel, int threads) {
  int dev = 0, cus = 256, per = 0;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
  }
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess || per <= 0) per = 1;
  if (per > 4) per = 4;
  return cus * per;
}

static int launch_finalize(hipStream_t st, int32_t* counts, int64_t n_query, bool tc) {
  hipLaunchKernelGGL(k_counts_finalize, dim3((unsigned)((n_query + 255) / 256)), dim3(256), 0, st, counts, n_query,
                     tc ? 1 : 0);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

template <int OP, bool TCV, bool STV, int PK>
static void launch_valu_one(hipStream_t st, const float* ent_km, int64_t e_pad, int64_t n_ent, int n_et, int e_base,
                            const float* q_km, int64_t q_pad, int64_t n_query, int kp, int pk, float m,
                            const float* thr, const int32_t* qtrue, const int64_t* qr, const int8_t* qmode,
                            const uint32_t* th, const uint32_t* tt, int64_t tw, int32_t* counts, float* scores,
                            L1Q l1) {
  // 16 workgroups per resident slot: short per-workgroup ranges let the dispatcher balance
  // CUs that run at different speeds (C2 on MI355X: 1,024 groups 4.0 ms, 8,192 3.43 ms,
  // 16,384 3.30 ms, 30,528 (one unit each) 3.36 ms).
  int g = 16 * resident_groups((const void*)k_sweep_valu<OP, TCV, STV, PK>, NT);
  // a gated launch (the L1 filter's f32 fallback, l1.gate) runs 4 workgroups per resident
  // slot: when the gate is shut -- every time but the rare fallback -- its workgroups only
  // read the flag and leave, and a 16x grid of such workgroups cost 77 us per evaluation at
  // C2; one per slot (1x) made the open-gate sweep 15% slower than the plain f32 sweep
  static const char* fbdiv = getenv("MMRE_L1_FB_DIV");
  if (l1.gate != nullptr) {
    const int div = fbdiv ? atoi(fbdiv) : 4;
    g /= div > 1 ? div : 1;
  }
  // Dynamic scheduling (l1.wq, the TransE L1 filter sweeps): one persistent workgroup per
  // resident slot, units from the XCD groups' work counters -- the shut gated launch too (its
  // workgroups only read the gate).
  constexpr bool DYN_OK = OP == 5 || OP == 6;
  const bool dyn = DYN_OK && l1.wq != nullptr && kp / KC >= 2;
  int chunk = 0;  // dynamic scheduling: units per claim (0: static ranges)
  if (dyn) {
    g = resident_groups((const void*)k_sweep_valu<OP, TCV, STV, PK, DYN_OK ? 4 : 0>, NT);
    const int64_t per_wg = (q_pad / TQ) * n_et / (g > 0 ? g : 1);
    static const char* ch_env = getenv("MMRE_SWEEP_CHUNK");  /* A/B: 1 or 4 units per claim */
    chunk = ch_env ? (atoi(ch_env) >= 4 ? 4 : 1) : (per_wg >= 16 ? 4 : 1);
  }
  // Small sweeps (a rank's share under relation sharding): no more workgroups than the
  // busiest XCD group has units, so every workgroup gets at most one unit and no empty
  // workgroups are dispatched (C2 at 8-way: 4,380 sweeps 0.52 -> 0.47 ms; 4-way 0.89 -> 0.85).
  {
    const int64_t q_tiles = q_pad / TQ;
    const int64_t units = (n_et >= 8) ? 8 * q_tiles * ((n_et + 7) / 8) : q_tiles * n_et;
    if (units < g) g = (int)(units > 0 ? units : 1);
    // Dynamic scheduling of a small share: as many workgroups per XCD group as make its units an
    // (almost) whole number of rounds -- the same rounds as the full grid, no nearly empty last
    // round (an 8-way C2 share: 527 units per group over 128 workgroups = 4.1 rounds, the fifth
    // run by 15 of them; over 106 workgroups, 5 rounds). Measured no faster on 8-way C2 shares
    // (ranks 1 / 3 / 7: 0.190 / 0.203 / 0.199 against 0.185 / 0.193 / 0.196 ms, profiles/r6): off
    // unless MMRE_SWEEP_BALANCE=1 (A/B).
    static const char* bal_env = getenv("MMRE_SWEEP_BALANCE");
    if (dyn && g % 8 == 0 && n_et >= 8 && bal_env && bal_env[0] == '1') {
      const int64_t per_group = (q_tiles * n_et + 7) / 8;  // UnitMap: every group within +-1 of this
      const int64_t slots = g / 8;
      const int64_t rounds = (per_group + slots - 1) / slots;
      if (rounds <= 16) g = 8 * (int)((per_group + rounds - 1) / rounds);
    }
  }
  // MMRE_SWEEP_GRID (experiments): "tiles" = one workgroup per (query tile, 1/8 of the
  // entity tiles); a number = that many persistent workgroups.
  static const char* gmode = getenv("MMRE_SWEEP_GRID");
  if (gmode && gmode[0] == 't') g = 8 * (int)(q_pad / TQ);
  else if (gmode && gmode[0] >= '1' && gmode[0] <= '9') g = atoi(gmode);
  const int ng = (g % 8 == 0 && n_et >= 8) ? 8 : 1;
  if (chunk == 4)
    hipLaunchKernelGGL((k_sweep_valu<OP, TCV, STV, PK, DYN_OK ? 4 : 0>), dim3((unsigned)g), dim3(NT), 0, st, ent_km,
                       e_pad, n_ent, q_km, q_pad, n_query, kp, n_et, e_base, ng, pk, m, thr, qtrue, qr, qmode, th, tt, tw,
                       counts, scores, l1);
  else if (chunk == 1)
    hipLaunchKernelGGL((k_sweep_valu<OP, TCV, STV, PK, DYN_OK ? 1 : 0>), dim3((unsigned)g), dim3(NT), 0, st, ent_km,
                       e_pad, n_ent, q_km, q_pad, n_query, kp, n_et, e_base, ng, pk, m, thr, qtrue, qr, qmode, th, tt, tw,
                       counts, scores, l1);
  else
    hipLaunchKernelGGL((k_sweep_valu<OP, TCV, STV, PK>), dim3((unsigned)g), dim3(NT), 0, st, ent_km, e_pad, n_ent, q_km,
                       q_pad, n_query, kp, n_et, e_base, ng, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores, l1);
}

template <int OP>
static int launch_valu(bool tc, bool store, hipStream_t st, const float* ent_km, int64_t e_pad, int64_t n_ent,
                       int n_et, int e_base, const float* q_km, int64_t q_pad, int64_t n_query, int kp, int pk, float m, const float* thr,
                       const int32_t* qtrue, const int64_t* qr, const int8_t* qmode, const uint32_t* th,
                       const uint32_t* tt, int64_t tw, int32_t* counts, float* scores, L1Q l1 = {},
                       bool finalize = true) {
#define MMRE_LV1(TCV, STV, PKV) \
  launch_valu_one<OP, TCV, STV, PKV>(st, ent_km, e_pad, n_ent, n_et, e_base, q_km, q_pad, n_query, kp, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores, l1)
  // the model's usual prediction kind is compiled into the epilogue of the plain sweep
  constexpr int fast = (OP == 2) ? 3 : 0;  // RotatE -(m - s), TransE s
  if constexpr (OP == 5 || OP == 6) {  // the integer filter: count-only sweeps
    if (store) return MMRE_ERR_ARG;
    if (tc && pk == fast) MMRE_LV1(true, false, fast);  // integer thresholds (prediction = the score)
    else if (tc) MMRE_LV1(true, false, -1);
    else if (pk == fast) MMRE_LV1(false, false, fast);
    else MMRE_LV1(false, false, -1);
  } else {
    if (tc && store) MMRE_LV1(true, true, -1);
    else if (tc) MMRE_LV1(true, false, -1);
    else if (store) MMRE_LV1(false, true, -1);
    else if (pk == fast) MMRE_LV1(false, false, fast);  // C2 3.27 -> 3.23 ms
    else MMRE_LV1(false, false, -1);
  }
#undef MMRE_LV1
  MMRE_CHECK_LAUNCH();
  return finalize ? launch_finalize(st, counts, n_query, tc) : MMRE_OK;
}

// ------------------------------------------ fused TransE L1 evaluation (round 5) ---
// mmre_link_evaluate_l1q: the whole count-only TransE L1 evaluation of a query set -- entity
// prep, query prep, truth scores, filter-list scores and counts, the L1 filter's quantization
// and code-width probe, the sweep -- in seven launches instead of thirteen, with what is
// independent fused into the same launch (block ranges of one grid doing different work):
//   K1 k_eval_prep        entity rows (normalised, k-major + row-major) | query rows, each
//                         query block normalising its own anchor and truth rows from the raw
//                         table (no dependency on the entity blocks), the truth scores; per
//                         block max |x| / sum |x| of the planes (plain stores); block 0 zeroes
//                         the filter header
//   K2 k_eval_quant_list  filter-list scores | 8-bit codes + the tight bound's error sums +
//                         16-bit codes, one read of the planes; every quantization block reduces
//                         K1's per-block statistics itself (same order: the same M everywhere),
//                         the first writes M and the codes / f32 word
//   K3 k_eval_count_probe filter counts, a wave per group | the code-width probe, a wave per
//                         sampled query (the last of its 128 blocks decides 8 vs 16 bits)
//   K4-K6                 the three gated sweeps (8-bit, 16-bit, f32; the code-width word
//                         names the one that counts); the f32 launch also carries the
//                         finalize (filtered += raw): each workgroup's slice when its gate is
//                         shut, the last workgroup's pass (ticket) when it is open
// No cross-workgroup hand-off inside K1 / K2: grid-wide results pass at kernel boundaries.
// Measured on the way (MI355X, C2, per evaluation): a __threadfence() per K1 block (L2
// write-back of each block's freshly written rows) 163 us for K1; per-block partials read back by
// a ticket's last block ~30 us of serial sc1 loads; three same-address atomics per block
// (max, sum, ticket: ~3,100 blocks) 128 us -- same-address atomics serialise at ~13 ns each.
// Values are bit-identical to the separate path (same canonical chains in the same order):
// tests/test_eval_fused_gpu.py holds counts, truths and planes equal.
struct EvalL1 {
  const float* ent;      // raw entity table (n_ent, dim)
  const float* rel;      // raw relation table (n_rel, dim)
  int64_t n_ent;
  int dim, kp, norm, rb, rbq;  // rows per entity block, queries per query block (two row sets)
  const int64_t* qh;
  const int64_t* qr;
  const int64_t* qt;
  const int8_t* qmode;
  int64_t n_query;
  float* ent_km;
  int64_t e_pad;
  float* ent_rows;
  float* q_km;
  int64_t q_pad;
  float* q_rows;
  int32_t* q_true;
  float* truth;
  int64_t e_begin, e_cols;  // the swept slice (its columns feed M)
  int n_eblk, n_qblk;
  uint32_t* und_q;          // optional per-query rescored-pair counters (zeroed here)
  float* pstat;             // per K1 block: max |x|, sum |x|
  uint32_t* ticket;         // [1]: the probe's ticket
  uint32_t* hdr;            // the L1 filter header
  double n_elem;
  float ratio;
};

// canonical sum of squares over x[0..dim) (k ascending, LDS reads batched 16 per round) and
// F.normalize's clamp: the divisor k_prep_rows uses
__device__ __forceinline__ float canon_norm(const float* x, int dim) {
  float ss = 0.0f;
  int k = 0;
  for (; k + 16 <= dim; k += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = x[k + u];
#pragma unroll
    for (int u = 0; u < 16; ++u) ss = ss + v[u] * v[u];
  }
  for (; k < dim; ++k) ss = ss + x[k] * x[k];
  const float nr = sqrtf(ss);
  return nr < 1e-12f ? 1e-12f : nr;
}

__device__ __forceinline__ void abs_stat(float v, float& mx, float& sa) {
  if (!(v - v == 0.0f)) mx = INFINITY;  // inf / NaN: no codes (the f32 sweep counts)
  else {
    mx = fmaxf(mx, fabsf(v));
    sa += fabsf(v);
  }
}

__global__ __launch_bounds__(256, 7) void k_eval_prep(EvalL1 P) {
  extern __shared__ float lds[];
  __shared__ float s_nrm[64];
  __shared__ int64_t s_a[32], s_t[32], s_r[32];
  __shared__ int s_head[32];
  __shared__ float s_m[4], s_s[4];
  const int kp = P.kp, kt = kp, ls = kt + 1, rb = P.rb, rbq = P.rbq, dim = P.dim;
  const int tid = threadIdx.x, lane = tid & 31, slot = tid >> 5;
  float mx = 0.0f, sa = 0.0f;
  if ((int)blockIdx.x < P.n_eblk) {  // ---- entity rows (k_prep_rows for TransE)
    const int64_t e0 = (int64_t)blockIdx.x * rb;
    for (int i = slot; i < rb; i += 8) {
      const int64_t e = e0 + i;
      float* x = lds + i * ls;
#pragma unroll 4
      for (int k = lane; k < kt; k += 32) x[k] = (e < P.n_ent && k < dim) ? P.ent[e * dim + k] : 0.0f;
    }
    __syncthreads();
    if (P.norm) {
      if (tid < rb) s_nrm[tid] = canon_norm(lds + tid * ls, dim);
      __syncthreads();
      for (int i = slot; i < rb; i += 8) {
        float* x = lds + i * ls;
        const float nr = s_nrm[i];
        for (int k = lane; k < kt; k += 32) x[k] = x[k] / nr;
      }
      __syncthreads();
    }
    const bool in_slice = e0 >= P.e_begin && e0 < P.e_begin + P.e_cols;
    for (int i = slot; i < rb; i += 8) {
      const int64_t e = e0 + i;
      const float* x = lds + i * ls;
      if (e < P.n_ent) {
#pragma unroll 4
        for (int k = lane; k < kt; k += 32) P.ent_rows[e * kt + k] = x[k];
      }
      if (in_slice && e < P.e_pad)
        for (int k = lane; k < kt; k += 32) abs_stat(x[k], mx, sa);
    }
    write_k_major(lds, ls, rb, kt, P.ent_km, P.e_pad, e0);
  } else {  // ---- query rows: q = h + r (tail) / -(r - t) (head), and the truth scores
    // Two dependent global rounds: the ids, then the anchor, truth and relation rows of every
    // query at once (into LDS); the norms and the combine work from LDS. (Reading the relation
    // row for its norm and again for the combine, each in its own dependent rounds, made a
    // block's latency ~27 us: K1 31.7 us for an 8-way share of C2.)
    const int64_t q0 = (int64_t)(blockIdx.x - P.n_eblk) * rbq;
    float* y0 = lds + rbq * ls;      // the truth rows
    float* z0 = lds + 2 * rbq * ls;  // the relation rows
    if (tid < rbq) {
      const int64_t q = q0 + tid;
      int64_t a = -1, tr = -1, r = 0;
      int head = 0;
      if (q < P.n_query) {
        head = P.qmode[q] == MMRE_HEAD_BATCH;
        a = head ? P.qt[q] : P.qh[q];
        tr = head ? P.qh[q] : P.qt[q];
        r = P.qr[q];
        P.q_true[q] = (int32_t)tr;
        if (P.und_q) P.und_q[q] = 0u;
      }
      s_a[tid] = a;
      s_t[tid] = tr;
      s_r[tid] = r;
      s_head[tid] = head;
    }
    __syncthreads();
    for (int i = slot; i < rbq; i += 8) {
      const int64_t a = s_a[i], tr = s_t[i], r = s_r[i];
      float* x = lds + i * ls;
      float* y = y0 + i * ls;
      float* z = z0 + i * ls;
#pragma unroll 8
      for (int k = lane; k < kt; k += 32) {
        x[k] = (a >= 0 && k < dim) ? P.ent[a * dim + k] : 0.0f;
        y[k] = (tr >= 0 && k < dim) ? P.ent[tr * dim + k] : 0.0f;
        z[k] = (a >= 0 && k < dim) ? P.rel[r * dim + k] : 0.0f;
      }
    }
    __syncthreads();
    if (P.norm) {  // anchor, truth (k_prep_rows' canonical order) and relation rows
      // (k_prep_queries' order: the same k-ascending sum of squares and clamp)
      if (tid < 3 * rbq) s_nrm[tid] = canon_norm(lds + tid * ls, dim);  // x | y | z rows
      __syncthreads();
      for (int i = slot; i < 2 * rbq; i += 8) {
        float* x = lds + i * ls;
        const float nr = s_nrm[i];
        for (int k = lane; k < kt; k += 32) x[k] = x[k] / nr;
      }
      __syncthreads();
    }
    for (int i = slot; i < rbq; i += 8) {
      float* x = lds + i * ls;
      const float* z = z0 + i * ls;
      const bool valid = s_a[i] >= 0;
      const bool head = s_head[i];
      const float rn = P.norm ? s_nrm[2 * rbq + i] : 1.0f;
      for (int k = lane; k < kp; k += 32) {
        if (!valid || k >= dim) {
          x[k] = 0.0f;
          continue;
        }
        // head_batch: score = h + (r - t) -> q = -(r - t); tail_batch: (h + r) - t -> q = h + r
        const float b = P.norm ? z[k] / rn : z[k];
        x[k] = head ? -(b - x[k]) : (x[k] + b);
      }
    }
    __syncthreads();
    if (tid < rbq && q0 + tid < P.n_query) {  // the truth's score: the canonical chain, k ascending
      const float* x = lds + tid * ls;
      const float* y = y0 + tid * ls;
      float acc = 0.0f;
      int k = 0;
      for (; k + 8 <= kp; k += 8) {
        float a[8], b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          a[u] = x[k + u];
          b[u] = y[k + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + fabsf(a[u] - b[u]);
      }
      for (; k < kp; ++k) acc = acc + fabsf(x[k] - y[k]);
      P.truth[q0 + tid] = acc;  // prediction = the score (TransE.py:104-110)
    }
    write_k_major(lds, ls, rbq, kt, P.q_km, P.q_pad, q0);
    for (int i = slot; i < rbq; i += 8) {
      const int64_t q = q0 + i;
      const float* x = lds + i * ls;
      if (q < P.n_query) {
#pragma unroll 4
        for (int k = lane; k < kt; k += 32) P.q_rows[q * kt + k] = x[k];
      }
      if (q < P.q_pad)
        for (int k = lane; k < kt; k += 32) abs_stat(x[k], mx, sa);
    }
  }
  // ---- the block's |x| statistics (K2 reduces them); block 0 zeroes the filter header's
  // counters (probe count, largest offset, guard, undecided slots) for K2 / K3 / the sweeps
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o));
    sa += __shfl_xor(sa, o);
  }
  if ((tid & 63) == 0) {
    s_m[tid >> 6] = mx;
    s_s[tid >> 6] = sa;
  }
  __syncthreads();
  if (tid == 0) {
    P.pstat[2 * blockIdx.x] = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
    P.pstat[2 * blockIdx.x + 1] = (s_s[0] + s_s[1]) + (s_s[2] + s_s[3]);
  }
  if (blockIdx.x == 0)
    for (int i = 2 + tid; i < L1Q_PART / 4; i += 256) P.hdr[i] = 0u;
}

// The filter-list score of one entry (k_filter_scores' list task, TransE L1, prediction = the
// score): the canonical chain over kp floats, 64 floats of each row in flight per round.
__device__ __forceinline__ float l1_row_score64(const float* __restrict__ qv, const float* __restrict__ ev, int kp) {
  float acc = 0.0f;
  int k0 = 0;
  for (; k0 + 64 <= kp; k0 += 64) {
    float4 a[16], x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      a[i] = *reinterpret_cast<const float4*>(qv + k0 + 4 * i);
      x[i] = *reinterpret_cast<const float4*>(ev + k0 + 4 * i);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc = acc + fabsf(a[i].x - x[i].x);
      acc = acc + fabsf(a[i].y - x[i].y);
      acc = acc + fabsf(a[i].z - x[i].z);
      acc = acc + fabsf(a[i].w - x[i].w);
    }
  }
  for (; k0 < kp; k0 += 8) {  // kp % 8 == 0
    float4 a[2], x[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = *reinterpret_cast<const float4*>(qv + k0 + 4 * i);
      x[i] = *reinterpret_cast<const float4*>(ev + k0 + 4 * i);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      acc = acc + fabsf(a[i].x - x[i].x);
      acc = acc + fabsf(a[i].y - x[i].y);
      acc = acc + fabsf(a[i].z - x[i].z);
      acc = acc + fabsf(a[i].w - x[i].w);
    }
  }
  return acc;
}

struct EvalQuant {  // K2's quantization operands (k_l1q_quant8<TIGHT> + the 16-bit words)
  L1QPlane pq, pe;  // 8-bit planes
  uint32_t* out16q;
  uint32_t* out16e;
  int kw, k2, kt, n_blk;  // 8-bit word rows, 16-bit word rows, floats per row, blocks per plane
  int tight;
  float* q_l1c;
};

__global__ __launch_bounds__(256, 4) void k_eval_quant_list(EvalL1 P, EvalQuant Q, const int32_t* __restrict__ ids,
                                                         const int32_t* __restrict__ entry_q, int64_t n_entries,
                                                         float* __restrict__ list_v, int n_lblk) {
  if ((int)blockIdx.x < n_lblk) {  // ---- filter-list scores (k_filter_scores' list tasks)
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n_entries) return;
    const int64_t j = ids[p], vq = entry_q[p];
    if (j < 0 || j >= P.n_ent || vq < 0 || vq >= P.n_query) {
      list_v[p] = __builtin_nanf("");  // never < a threshold: an invalid id is not counted
      return;
    }
    list_v[p] = l1_row_score64(P.q_rows + vq * P.kp, P.ent_rows + j * P.kp, P.kp);
    return;
  }
  // ---- M and the codes / f32 decision from K1's per-block statistics: every quantization block
  // reduces them in the same order (the same M and decision everywhere, deterministic); the
  // first one publishes them in the header for K3 and the sweeps (the l1q_fallback test:
  // M non-finite, or M > ratio x mean |x|)
  __shared__ float s_rm[4], s_rs[4];
  {
    const int nst = P.n_eblk + P.n_qblk;
    float m = 0.0f, sm = 0.0f;
#pragma unroll 8
    for (int i = threadIdx.x; i < nst; i += 256) {
      const float2 v = reinterpret_cast<const float2*>(P.pstat)[i];
      m = fmaxf(m, v.x);
      sm += v.y;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      m = fmaxf(m, __shfl_xor(m, o));
      sm += __shfl_xor(sm, o);
    }
    if ((threadIdx.x & 63) == 0) {
      s_rm[threadIdx.x >> 6] = m;
      s_rs[threadIdx.x >> 6] = sm;
    }
    __syncthreads();
  }
  const float mx = fmaxf(fmaxf(s_rm[0], s_rm[1]), fmaxf(s_rm[2], s_rm[3]));
  const float msum = (s_rs[0] + s_rs[1]) + (s_rs[2] + s_rs[3]);
  const bool fb = !(mx < INFINITY) || (double)mx > (double)P.ratio * ((double)msum / P.n_elem);
  if ((int)blockIdx.x == n_lblk && threadIdx.x == 0) {
    P.hdr[0] = __float_as_uint(mx < INFINITY ? mx : INFINITY);
    P.hdr[1] = fb ? L1Q_F32 : L1Q_CODES8;
  }
  if (fb) return;  // the f32 sweep counts: no codes
  // ---- the codes: 8-bit words (+ the tight bound's error row) and 16-bit words in one pass
  const int b = (int)blockIdx.x - n_lblk;
  const bool ent = b >= Q.n_blk;
  const int bx = ent ? b - Q.n_blk : b;
  const L1QPlane& pl = ent ? Q.pe : Q.pq;
  const float* __restrict__ km = pl.km;
  const int64_t pad = pl.pad, c0 = pl.c0, n = pl.n;
  uint32_t* __restrict__ out = pl.out;
  uint32_t* __restrict__ out16 = ent ? Q.out16e : Q.out16q;
  const int kp = P.kp, kw = Q.kw, k2 = Q.k2, kt = Q.kt;
  const float inv = (mx > 0.0f && mx < INFINITY) ? 255.0f / (2.0f * mx) : 0.0f;
  const float inv16 = (mx > 0.0f && mx < INFINITY) ? 65535.0f / (2.0f * mx) : 0.0f;
  const float off = (mx < INFINITY) ? mx : 0.0f;
  const float delta = (mx > 0.0f && mx < INFINITY) ? (2.0f * mx) / 255.0f : 0.0f;
  const float l1f = (float)(kt + 4) * 0x1p-23f * (1.0f + 0x1p-8f);
  const int words = (kt + 3) >> 2;
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  __shared__ float s_err[8][32];
  for (int64_t cb = (int64_t)bx * 32; cb < n; cb += (int64_t)Q.n_blk * 32) {  // uniform
    const bool live = cb + cl < n;
    const int64_t c = c0 + cb + cl;
    float err = 0.0f;
    // four word rows of a thread in flight together (kw <= 64 word rows -- d <= 256 -- is two
    // load rounds instead of four; eight took 167 VGPRs), then coded in the same order as before
    for (int r0 = g; r0 < kw; r0 += 32) {
      float xv[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int k = 4 * (r0 + 8 * j) + h;
          xv[j][h] = (live && r0 + 8 * j < kw && k < kp) ? km[(int64_t)k * pad + c] : 0.0f;
        }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = r0 + 8 * j;
        if (r >= kw) break;
        uint32_t word = 0u, w16a = 0u, w16b = 0u;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int k = 4 * r + h;
          if (live && k < kp) {
            const float x = xv[j][h];
            float t = (x + off) * inv;
            t = t == t ? fminf(fmaxf(t, 0.0f), 255.0f) : 0.0f;
            const float code = rintf(t);
            word |= (uint32_t)code << (8 * h);
            if (Q.tight) err += fabsf(x - (code * delta - off));
            float t16 = (x + off) * inv16;
            t16 = t16 == t16 ? fminf(fmaxf(t16, 0.0f), 65535.0f) : 0.0f;
            const uint32_t c16 = (uint32_t)rintf(t16);
            if (h < 2) w16a |= c16 << (16 * h);
            else w16b |= c16 << (16 * (h - 2));
          }
        }
        if (live) {
          if (!(Q.tight && r == words)) out[(int64_t)r * pad + c] = word;
          if (2 * r < k2) out16[(int64_t)(2 * r) * pad + c] = w16a;
          if (2 * r + 1 < k2) out16[(int64_t)(2 * r + 1) * pad + c] = w16b;
        }
      }
    }
    if (Q.tight) {
      s_err[g][cl] = err;
      __syncthreads();
      uint32_t o_max = 0u;  // this chunk's largest entity offset (wave 0), one atomic per chunk
      if (g == 0 && live) {
        float e = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) e += s_err[i][cl];
        const float eb = __builtin_fmaf(e, 1.01f, (float)kt * 0x1p-20f * mx);
        uint32_t wv = 0u;
        if (!ent) {
          Q.q_l1c[c] = eb;
        } else {
          // (<= 1,005 at kt <= 1,984 without the clamp acting: see k_l1q_quant8)
          uint32_t o = delta > 0.0f ? (uint32_t)ceilf(fminf(eb / (delta * (1.0f - l1f)) * (1.0f + 0x1p-17f), 1020.0f))
                                    : 0u;
          o_max = o;
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const uint32_t bb = o < 255u ? o : 255u;
            wv |= bb << (8 * h);
            o -= bb;
          }
        }
        out[(int64_t)words * pad + c] = wv;
      }
      if (ent && threadIdx.x < 64) {  // uniform per wave: 32 lanes' offsets -> one atomicMax
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) o_max = max(o_max, (uint32_t)__shfl_xor((int)o_max, sh));
        if (threadIdx.x == 0 && o_max) atomicMax(P.hdr + 3, o_max);
      }
      __syncthreads();
    }
  }
}

// K3: filter counts (k_filter_count without type masks, one WAVE per filter group, four per
// block) | the code-width probe (k_l1q_probe's sample, one wave per sampled query: 128 blocks, so
// the probe's count and ticket take 128 same-address atomics each, not 512), whose last block
// turns the code-width word to the 16-bit codes when the sample's undecided fraction is over
// the threshold. force_bits 8 / 16 (MMRE_L1_BITS): no probe; 16 sets the word (unless f32).
__global__ __launch_bounds__(256) void k_eval_count_probe(
    const int64_t* __restrict__ grp_qoff, const int32_t* __restrict__ grp_q, int64_t n_groups, int n_cblk,
    const int64_t* __restrict__ off, const int32_t* __restrict__ ids, const float* __restrict__ list_v,
    const int32_t* __restrict__ qtrue, const float* __restrict__ thr, int64_t n_query, int64_t n_ent,
    int32_t* __restrict__ counts, const uint32_t* __restrict__ uq, int64_t q_pad, const uint32_t* __restrict__ ue,
    int64_t e_pad, int64_t n_slice, int kw, int kt, const float* __restrict__ q_l1c, uint32_t* __restrict__ hdr,
    uint32_t* __restrict__ ticket, uint32_t probe_max, int force_bits) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if ((int)blockIdx.x < n_cblk) {
    // the wave's own LDS slices: written and read by the same wave (wave barriers, no block sync)
    __shared__ __attribute__((aligned(16))) int32_t s_id[4][64];
    __shared__ __attribute__((aligned(16))) float s_v[4][64];
    for (int64_t g = (int64_t)blockIdx.x * 4 + wv; g < n_groups; g += (int64_t)n_cblk * 4) {
      const int64_t qa = grp_qoff[g], qb = grp_qoff[g + 1];
      const int64_t la = off[g], lb = off[g + 1];
      for (int64_t qc = qa; qc < qb; qc += 64) {
        const int64_t qi = qc + lane;
        const bool active = qi < qb;
        const int64_t q = active ? grp_q[qi] : 0;
        const int32_t tr = active ? qtrue[q] : -1;
        const float th = active ? thr[q] : 0.0f;
        int c = 0;
        for (int64_t lc = la; lc < lb; lc += 64) {
          const int nl = (int)((lb - lc) < 64 ? (lb - lc) : 64);
          int32_t id = -1;
          float v = 0.0f;
          if (lane < nl) {
            const int64_t j = ids[lc + lane];
            if (j >= 0 && j < n_ent) {
              id = (int32_t)j;
              v = list_v[lc + lane];
            }
          }
          __builtin_amdgcn_wave_barrier();  // the previous round's reads are done
          s_id[wv][lane] = id;  // entries nl..63 stay invalid: the loop below reads whole quads
          s_v[wv][lane] = v;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (active) {
            for (int i = 0; i < nl; i += 4) {  // branch-free, 4 entries per LDS read
              const int4 e = *reinterpret_cast<const int4*>(&s_id[wv][i]);
              const float4 vv = *reinterpret_cast<const float4*>(&s_v[wv][i]);
              c += ((e.x >= 0) & (e.x != tr) & (vv.x < th)) + ((e.y >= 0) & (e.y != tr) & (vv.y < th)) +
                   ((e.z >= 0) & (e.z != tr) & (vv.z < th)) + ((e.w >= 0) & (e.w != tr) & (vv.w < th));
            }
          }
        }
        if (active) {
          counts[0 * n_query + q] = 0;
          counts[1 * n_query + q] = -c;
          counts[2 * n_query + q] = 0;
          counts[3 * n_query + q] = 0;
        }
      }
    }
    return;
  }
  // ---- the probe
  const uint32_t w = __builtin_amdgcn_readfirstlane(hdr[1]);
  if (force_bits != 0) {
    if (force_bits == 16 && w != L1Q_F32 && blockIdx.x == (unsigned)n_cblk && tid == 0) hdr[1] = L1Q_CODES16;
    return;
  }
  if (w != L1Q_CODES8) return;  // the f32 fallback: no codes to probe
  const int pb = ((int)blockIdx.x - n_cblk) * 4 + wv, n_pb = ((int)gridDim.x - n_cblk) * 4;
  const int64_t q = (int64_t)pb * n_query / n_pb;
  const int64_t span = n_slice > L1Q_PROBE_E ? n_slice - L1Q_PROBE_E : 0;
  const int64_t c = (((int64_t)pb * span / n_pb) & ~(int64_t)3) + 4 * lane;
  const float l1d = l1q_delta(hdr, 255.0f);
  const float l1f = (float)(kt + 4) * 0x1p-23f * (1.0f + 0x1p-8f);
  const float l1c = __builtin_fmaf((float)kt * 1.03f, l1d, 0x1p-120f);
  uint32_t acc[4] = {0u, 0u, 0u, 0u};
  if (c < n_slice) {
#pragma unroll 8
    for (int r = 0; r < kw; ++r) {
      const uint32_t a = uq[(int64_t)r * q_pad + q];
      const uint4 e = *reinterpret_cast<const uint4*>(ue + (int64_t)r * e_pad + c);
      acc[0] = __builtin_amdgcn_sad_u8(a, e.x, acc[0]);
      acc[1] = __builtin_amdgcn_sad_u8(a, e.y, acc[1]);
      acc[2] = __builtin_amdgcn_sad_u8(a, e.z, acc[2]);
      acc[3] = __builtin_amdgcn_sad_u8(a, e.w, acc[3]);
    }
  }
  uint32_t t_sure, t_span;
  l1_int_thresholds(thr[q], (q_l1c ? q_l1c[q] : l1c) + (q_l1c ? 0x1p-120f : 0.0f), l1d, l1f, q_l1c ? 2u * hdr[3] : 0u,
                    t_sure, t_span);
  uint32_t und = 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) und += (uint32_t)((acc[j] - t_sure < t_span) & (c + j < n_slice));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) und += __shfl_xor(und, o);
  __shared__ uint32_t s_und[4];
  __shared__ uint32_t s_last;
  if (lane == 0) s_und[wv] = und;
  __syncthreads();
  if (tid == 0) {  // the block's count, then the ticket (the hand-off of K1's table row 1: atomics, vmcnt(0))
    const uint32_t bu = (s_und[0] + s_und[1]) + (s_und[2] + s_und[3]);
    if (bu) __hip_atomic_fetch_add(hdr + 2, bu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = __hip_atomic_fetch_add(&ticket[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (uint32_t)(gridDim.x - n_cblk) - 1;
  }
  __syncthreads();
  if (s_last && tid == 0) {
    const uint32_t total = __hip_atomic_load(hdr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (total > probe_max) hdr[1] = L1Q_CODES16;
    ticket[1] = 0u;
  }
}

}  // namespace mmre

using namespace mmre;

extern "C" int64_t mmre_link_k(int model, int dim) { return (int64_t)n_planes(model) * plane_rows(model, dim); }
extern "C" int64_t mmre_link_pad(int64_t n) { return round_up(n > 0 ? n : 1, 128); }

static bool valid_model(int m) { return m >= MMRE_TRANSE_L1 && m <= MMRE_ROTATE; }

extern "C" int mmre_link_prepare_entities(int model, int norm_flag, const float* d_ent, const float* d_ent_im,
                                          int64_t n_ent, int dim, float* d_ent_km, int64_t e_pad, float* d_ent_rows,
                                          void* stream) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (!d_ent || !d_ent_km || !d_ent_rows || n_ent <= 0 || dim <= 0 || e_pad < n_ent || e_pad % TE) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && !d_ent_im) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(model, dim), kt = n_planes(model) * kp;
  const int rb = stage_rows(kt);
  const size_t lds = sizeof(float) * (size_t)rb * (kt + 1);
  if (lds > 64 * 1024) return MMRE_ERR_SHAPE;
  hipLaunchKernelGGL(k_prep_rows, dim3((unsigned)((e_pad + rb - 1) / rb)), dim3(256), lds, st, model, norm_flag, d_ent,
                     d_ent_im, n_ent, dim, kp, rb, d_ent_km, e_pad, d_ent_rows, kt);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_link_prepare_queries(int model, int norm_flag, const float* d_ent_rows, const float* d_rel,
                                         const float* d_rel_im, int64_t n_ent, int64_t n_rel, int dim,
                                         float phase_denom, const int64_t* d_qh, const int64_t* d_qr,
                                         const int64_t* d_qt, const int8_t* d_qmode, int64_t n_query,
                                         float* d_q_km, int64_t q_pad, int32_t* d_q_true, float* d_rel_work,
                                         float* d_q_rows, void* stream) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (!d_ent_rows || !d_rel || !d_qh || !d_qr || !d_qt || !d_qmode || !d_q_km || !d_q_true) return MMRE_ERR_ARG;
  if (n_query <= 0 || q_pad < n_query || q_pad % TQ || dim <= 0 || n_ent <= 0 || n_rel <= 0) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && !d_rel_im) return MMRE_ERR_ARG;
  if (model == MMRE_ROTATE && !(phase_denom != 0.0f)) return MMRE_ERR_ARG;
  const bool transe = model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2;
  if (transe && norm_flag && !d_rel_work) return MMRE_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(model, dim), kt = n_planes(model) * kp;
  // TransE norm_flag: each query block normalises its relation rows itself (no separate
  // relation-prep launch; d_rel_work stays part of the ABI as caller-provided scratch)
  const int rel_norm = (transe && norm_flag) ? 1 : 0;
  const int rb = stage_rows(kt);
  const size_t lds = sizeof(float) * (size_t)rb * (kt + 1);
  if (lds > 64 * 1024) return MMRE_ERR_SHAPE;
  hipLaunchKernelGGL(k_prep_queries, dim3((unsigned)((q_pad + rb - 1) / rb)), dim3(256), lds, st, model, d_ent_rows,
                     d_rel, d_rel_im, dim, kp, rb, phase_denom, d_qh, d_qr, d_qt, d_qmode, n_query, d_q_km, q_pad,
                     d_q_true, d_q_rows, rel_norm);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

template <int OP>
static int launch_truth_filter(hipStream_t st, const float* ent_rows, int64_t n_ent, const float* q_km, int64_t q_pad,
                               int kp, const float* q_rows, const int32_t* qtrue, const int64_t* qr, const int8_t* qmode, int64_t n_query,
                               int pk, float m, const int64_t* grp_qoff, const int32_t* grp_q, int64_t n_groups,
                               const int64_t* off, const int32_t* ids, const uint32_t* th, const uint32_t* tt,
                               int64_t tw, float* thr, int32_t* counts) {
  constexpr int NP = (OP == 2 || OP == 4) ? 2 : 1;
  const size_t lds = sizeof(float) * (size_t)NP * kp;
  if (lds > 64 * 1024) return MMRE_ERR_SHAPE;
  const unsigned blocks = (unsigned)(n_groups < (1 << 20) ? n_groups : (1 << 20));
  hipLaunchKernelGGL((k_truth_filter<OP>), dim3(blocks), dim3(FT), lds, st, ent_rows, n_ent, q_km, q_pad, kp, q_rows,
                     qtrue, qr, qmode, n_query, pk, m, grp_qoff, grp_q, n_groups, off, ids, th, tt, tw, thr, counts);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

static int check_link_args(int model, int pred_kind, const float* d_ent_km, int64_t n_ent, int64_t e_pad,
                           const float* d_q_km, const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode,
                           int64_t n_query, int64_t q_pad, const uint32_t* d_type_head, const uint32_t* d_type_tail,
                           const int32_t* d_counts, const float* d_truth) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (pred_kind < 0 || pred_kind > 4) return MMRE_ERR_ARG;
  if (!d_ent_km || !d_q_km || !d_q_true || !d_counts || !d_truth || !d_qmode || !d_qr) return MMRE_ERR_ARG;
  if (n_query <= 0 || n_ent <= 0 || e_pad < n_ent || e_pad % TE || q_pad < n_query || q_pad % TQ) return MMRE_ERR_ARG;
  if ((d_type_head == nullptr) != (d_type_tail == nullptr)) return MMRE_ERR_ARG;
  if (n_ent > (int64_t)INT32_MAX - 256) return MMRE_ERR_SHAPE;  // padded ids stay int32
  return MMRE_OK;
}

template <int OP>
static int launch_filter_scores(hipStream_t st, const float* ent_rows, int64_t n_ent, const float* q_rows, int kp,
                                const int32_t* qtrue, int64_t n_query, int pk, float m, const int32_t* entry_q,
                                const int32_t* ids, int64_t n_entries, float* thr, float* list_v) {
  const int64_t tasks = n_query + n_entries;
  hipLaunchKernelGGL((k_filter_scores<OP>), dim3((unsigned)((tasks + 255) / 256)), dim3(256), 0, st, ent_rows, n_ent,
                     q_rows, kp, qtrue, n_query, pk, m, entry_q, ids, n_entries, thr, list_v);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_link_truth_grouped(int model, int pred_kind, float margin, const float* d_ent_rows, int64_t n_ent,
                                       const float* d_q_rows, const int32_t* d_q_true, const int64_t* d_qr,
                                       const int8_t* d_qmode, int64_t n_query, int dim, const int64_t* d_grp_qoff,
                                       const int32_t* d_grp_q, int64_t n_groups, const int64_t* d_filt_off,
                                       const int32_t* d_filt_ids, const int32_t* d_entry_q, int64_t n_entries,
                                       const uint32_t* d_type_head, const uint32_t* d_type_tail,
                                       float* d_list_scores, int32_t* d_counts, float* d_truth, void* stream) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (pred_kind < 0 || pred_kind > 4) return MMRE_ERR_ARG;
  if (!d_ent_rows || !d_q_rows || !d_q_true || !d_qr || !d_qmode || !d_counts || !d_truth) return MMRE_ERR_ARG;
  if (!d_grp_qoff || !d_grp_q || !d_filt_off) return MMRE_ERR_ARG;
  if (n_query <= 0 || n_ent <= 0 || dim <= 0 || n_groups <= 0 || n_groups > n_query || n_entries < 0)
    return MMRE_ERR_ARG;
  if (n_entries > 0 && (!d_filt_ids || !d_entry_q || !d_list_scores)) return MMRE_ERR_WORKSPACE;
  if ((d_type_head == nullptr) != (d_type_tail == nullptr)) return MMRE_ERR_ARG;
  if (n_ent >= (int64_t)INT32_MAX || n_query >= (int64_t)INT32_MAX) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(model, dim);
  int rc;
#define MMRE_FS(OPV)                                                                                              \
  launch_filter_scores<OPV>(st, d_ent_rows, n_ent, d_q_rows, kp, d_q_true, n_query, pred_kind, margin, d_entry_q, \
                            d_filt_ids, n_entries, d_truth, d_list_scores)
  switch (op_of_model(model)) {
    case 0: rc = MMRE_FS(0); break;
    case 1: rc = MMRE_FS(1); break;
    case 2: rc = MMRE_FS(2); break;
    case 3: rc = MMRE_FS(3); break;
    default: rc = MMRE_FS(4); break;
  }
#undef MMRE_FS
  if (rc) return rc;
  const unsigned blocks = (unsigned)(n_groups < (1 << 20) ? n_groups : (1 << 20));
  hipLaunchKernelGGL(k_filter_count, dim3(blocks), dim3(64), 0, st, d_grp_qoff, d_grp_q, n_groups, d_filt_off,
                     d_filt_ids, d_list_scores, d_q_true, d_truth, d_qr, d_qmode, n_query, n_ent, d_type_head,
                     d_type_tail, (n_ent + 31) / 32, d_counts);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_link_truth(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                               int64_t e_pad, const float* d_ent_rows, const float* d_q_km, const int32_t* d_q_true,
                               const int64_t* d_qr, const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                               const int64_t* d_filt_off, const int32_t* d_filt_ids, const uint32_t* d_type_head,
                               const uint32_t* d_type_tail, int32_t* d_counts, float* d_truth, void* stream) {
  int rc = check_link_args(model, pred_kind, d_ent_km, n_ent, e_pad, d_q_km, d_q_true, d_qr, d_qmode, n_query, q_pad,
                           d_type_head, d_type_tail, d_counts, d_truth);
  if (rc) return rc;
  if (!d_ent_rows) return MMRE_ERR_ARG;
  if ((d_filt_off == nullptr) != (d_filt_ids == nullptr)) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(model, dim);
  const int64_t tw = (n_ent + 31) / 32;
#define MMRE_TF(OPV)                                                                                              \
  launch_truth_filter<OPV>(st, d_ent_rows, n_ent, d_q_km, q_pad, kp, nullptr, d_q_true, d_qr, d_qmode, n_query,   \
                           pred_kind, margin, nullptr, nullptr, n_query, d_filt_off, d_filt_ids, d_type_head,      \
                           d_type_tail, tw, d_truth, d_counts)
  switch (op_of_model(model)) {
    case 0: return MMRE_TF(0);
    case 1: return MMRE_TF(1);
    case 2: return MMRE_TF(2);
    case 3: return MMRE_TF(3);
    default: return MMRE_TF(4);
  }
#undef MMRE_TF
}

// The f32 MFMA sweep's launch (DistMult / ComplEx; d_ent_km already at the slice's first
// column). gate != NULL: every workgroup returns at once unless *gate != 0 (the split-bf16
// filter's overflow fallback, mmre_link_sweep_bf3).
static void launch_mfma(bool tc, bool store, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                        int64_t e_pad, int n_et, int e_base, const float* d_q_km, int64_t q_pad, int64_t n_query,
                        int ktot, const float* d_truth, const int64_t* d_qr, const int8_t* d_qmode,
                        const uint32_t* d_type_head, const uint32_t* d_type_tail, int64_t tw, int32_t* d_counts,
                        float* d_scores, hipStream_t st, const uint32_t* gate) {
  // persistent XCD-grouped grid as for the VALU sweep, 2 workgroups per resident slot (MI355X,
  // KCM = 16: C3 1.20 / 1.24 / 1.22 / 1.24 ms and C5 36.5 / 36.5 / 36.5 / 36.6 ms at 1/2/3/4x)
  // K stages of 32 rows (a unit's last one 16 when K = 32 n + 16: C3 ComplEx 2 x 200): half the
  // per-stage staging and barriers per MFMA of 16-row stages (scripts/probes/mfma_stage.hip:
  // 0.79 -> 0.86 of the f32 MFMA peak, L2-resident or HBM-streamed alike)
  // The plain sweep (no type constraint, no score store) runs 16-row stages at 4 workgroups
  // per CU (33 KB of LDS, 112 VGPRs with the ballot row counters): C3 1.03 -> 0.97 ms, C5
  // 33.7 -> 33.0 ms against 32-row stages at 2 per CU; the TC / STORE variants keep 32-row
  // stages (their extra registers would spill at 4 per CU).
  static const char* ks_env = getenv("MMRE_MFMA_STAGE"); /* experiments: 16 / 32 force the stage */
  const int ks_force = ks_env ? atoi(ks_env) : 0;
  const bool ks32 = ks_force == 32 || (ks_force != 16 && (tc || store));
  static const char* grid_env = getenv("MMRE_SWEEP_GRID"); /* experiments: workgroup count */
  // Units entity-tile-major inside each XCD group when the entity planes outgrow the caches
  // (> 64 MB; the 256 MB MALL also holds the query planes): a workgroup's consecutive units then
  // share its entity tile (L2-resident) and sweep the query tiles, which stay MALL-resident, so
  // the table streams from HBM about once instead of once per query tile (C5, a 1 GB table:
  // 35.8 -> 34.5 ms on one box, 60 -> ~1 GB of entity reads per launch); C3's 20 MB planes keep
  // the query-major order (0.979 vs 0.982 ms).
  static const char* order_env = getenv("MMRE_MFMA_EMAJOR"); /* experiments: 0 / 1 force the order */
  const int emajor = order_env ? atoi(order_env) : ((double)e_pad * ktot * 4.0 > 64.0 * (1 << 20) ? 1 : 0);
#define MMRE_MFMA_K(KERNEL)                                                                                       \
  do {                                                                                                            \
    /* 16 units per workgroup, between 1 (2 with 32-row stages) and 8 x the resident slots:    */                \
    /* short ranges let the dispatcher balance CUs of different speed (C5 1,024 / 4,096 groups:  */                \
    /* 35.1 / 34.3 ms) while the few-unit C3 keeps ranges long enough to amortise each group's   */                \
    /* first stage (16-row stages at 4 / CU, C3: 1,024 groups 0.97 ms, 2,048 1.04, 4,096 1.02)   */                \
    const int res = resident_groups((const void*)KERNEL, NT);                                                     \
    const int64_t units = (q_pad / TQ) * (int64_t)n_et;                                                           \
    const int64_t lo = ks32 ? 2LL * res : (int64_t)res;                                                           \
    int g = (int)std::min<int64_t>(8LL * res, std::max<int64_t>(lo, units / 16)) & ~7;                            \
    if (gate != nullptr) g = (int)lo & ~7; /* gated (the bf3 fallback): one residency round when shut */          \
    if (grid_env && grid_env[0] >= '1' && grid_env[0] <= '9') g = atoi(grid_env);                              \
    const int ng = (g % 8 == 0 && n_et >= 8) ? 8 : 1;                                                             \
    hipLaunchKernelGGL(KERNEL, dim3((unsigned)g), dim3(NT), 0, st, d_ent_km, e_pad, n_ent, d_q_km, q_pad,       \
                       n_query, ktot, n_et, e_base, ng, pred_kind, margin, d_truth, d_qr, d_qmode, d_type_head,  \
                       d_type_tail, tw, d_counts, d_scores, emajor, gate);                                              \
  } while (0)
#define MMRE_MFMA(TCV, STV, PKV)                                                                           \
  do {                                                                                                 \
    if (ks32) MMRE_MFMA_K((k_sweep_mfma<TCV, STV, PKV, 32>));                                          \
    else MMRE_MFMA_K((k_sweep_mfma<TCV, STV, PKV, 16>));                                               \
  } while (0)
  // DistMult / ComplEx predict -s: compiled into the plain sweep's epilogue (one compare with a
  // negated operand per pair); other kinds and the TC / STORE variants decode it at run time
  if (tc) { if (store) MMRE_MFMA(true, true, -1); else MMRE_MFMA(true, false, -1); }
  else if (store) MMRE_MFMA(false, true, -1);
  else if (pred_kind == 2) MMRE_MFMA(false, false, 2);
  else MMRE_MFMA(false, false, -1);
#undef MMRE_MFMA
#undef MMRE_MFMA_K
}

// The sweep over entities [e_begin, e_end) of the table (e_begin a multiple of TE): the kernels
// see the slice (pointer offset by e_begin columns, row stride e_pad, n_ent_local ids) and add
// e_begin back wherever an absolute id matters (truth exclusion, type-constraint bits).
static int sweep_impl(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent, int64_t e_pad,
                      int64_t e_begin, int64_t e_end, const float* d_q_km, const int32_t* d_q_true,
                      const int64_t* d_qr, const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                      const uint32_t* d_type_head, const uint32_t* d_type_tail, int32_t* d_counts,
                      const float* d_truth, float* d_scores, hipStream_t st) {
  int rc = check_link_args(model, pred_kind, d_ent_km, n_ent, e_pad, d_q_km, d_q_true, d_qr, d_qmode, n_query, q_pad,
                           d_type_head, d_type_tail, d_counts, d_truth);
  if (rc) return rc;
  if (e_begin < 0 || e_begin % TE || e_end <= e_begin || e_end > n_ent) return MMRE_ERR_ARG;
  if (d_scores && (e_begin != 0 || e_end != n_ent)) return MMRE_ERR_ARG;  // score rows are whole-table
  const int64_t tw = (n_ent + 31) / 32;  // type bitsets span the whole table
  const int e_base = (int)e_begin;
  d_ent_km += e_begin;
  n_ent = e_end - e_begin;
  const int n_et = (int)((n_ent + TE - 1) / TE);
  const int kp = plane_rows(model, dim);
  const bool tc = d_type_head != nullptr;
  const bool store = d_scores != nullptr;
  const int op = op_of_model(model);
  if (op <= 2) {
#define MMRE_LV(OPV) launch_valu<OPV>(tc, store, st, d_ent_km, e_pad, n_ent, n_et, e_base, d_q_km, q_pad, n_query, kp, pred_kind, \
                                      margin, d_truth, d_q_true, d_qr, d_qmode, d_type_head, d_type_tail, tw, d_counts, d_scores)
    if (op == 0) return MMRE_LV(0);
    if (op == 1) return MMRE_LV(1);
    return MMRE_LV(2);
#undef MMRE_LV
  }
  const int ktot = n_planes(model) * kp;
  launch_mfma(tc, store, pred_kind, margin, d_ent_km, n_ent, e_pad, n_et, e_base, d_q_km, q_pad, n_query, ktot,
              d_truth, d_qr, d_qmode, d_type_head, d_type_tail, tw, d_counts, d_scores, st, nullptr);
  MMRE_CHECK_LAUNCH();
  return launch_finalize(st, d_counts, n_query, tc);
}

extern "C" int mmre_link_sweep(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                               int64_t e_pad, const float* d_q_km, const int32_t* d_q_true, const int64_t* d_qr,
                               const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                               const uint32_t* d_type_head, const uint32_t* d_type_tail, int32_t* d_counts,
                               const float* d_truth, float* d_scores, void* stream) {
  if (n_ent <= 0) return MMRE_ERR_ARG;
  return sweep_impl(model, pred_kind, margin, d_ent_km, n_ent, e_pad, 0, n_ent, d_q_km, d_q_true, d_qr, d_qmode,
                    n_query, q_pad, dim, d_type_head, d_type_tail, d_counts, d_truth, d_scores, (hipStream_t)stream);
}

extern "C" int64_t mmre_link_l1q_workspace(int dim, int64_t e_pad, int64_t q_pad) {
  if (dim <= 0 || e_pad <= 0 || q_pad <= 0) return 0;
  return L1Q_HDR + 4 * (int64_t)(l1q_rows(dim) + l1q_rows8(dim)) * (e_pad + q_pad) + 4 * q_pad;
}

extern "C" int mmre_link_l1q_stats(const void* d_work, int64_t work_bytes, uint64_t* d_out, void* stream) {
  if (!d_work || !d_out || work_bytes < L1Q_HDR) return MMRE_ERR_ARG;
  hipLaunchKernelGGL(k_l1q_stats, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint32_t*)d_work,
                     (unsigned long long*)d_out);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_link_sweep_l1q(int pred_kind, float margin, const float* d_ent_km, const float* d_ent_rows,
                                   int64_t n_ent, int64_t e_pad, int64_t e_begin, int64_t e_end, const float* d_q_km,
                                   const float* d_q_rows, const int32_t* d_q_true, const int64_t* d_qr,
                                   const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                                   const uint32_t* d_type_head, const uint32_t* d_type_tail, int32_t* d_counts,
                                   const float* d_truth, void* d_work, int64_t work_bytes, void* stream) {
  int rc = check_link_args(MMRE_TRANSE_L1, pred_kind, d_ent_km, n_ent, e_pad, d_q_km, d_q_true, d_qr, d_qmode, n_query,
                           q_pad, d_type_head, d_type_tail, d_counts, d_truth);
  if (rc) return rc;
  if (!d_ent_rows || !d_q_rows || !d_work || work_bytes < mmre_link_l1q_workspace(dim, e_pad, q_pad)) return MMRE_ERR_WORKSPACE;
  if (e_begin < 0 || e_begin % TE || e_end <= e_begin || e_end > n_ent) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(MMRE_TRANSE_L1, dim), k2 = l1q_rows(dim), k4 = l1q_rows8(dim);
  uint32_t* hdr = (uint32_t*)d_work;
  uint32_t* uq = (uint32_t*)((char*)d_work + L1Q_HDR);  // 16-bit planes
  uint32_t* ue = uq + (int64_t)k2 * q_pad;
  uint32_t* vq = ue + (int64_t)k2 * e_pad;              // 8-bit planes
  uint32_t* ve = vq + (int64_t)k4 * q_pad;
  float* q_l1c = (float*)(ve + (int64_t)k4 * e_pad);     // tight bound: per query row error sums
  const int64_t e_cols = round_up(e_end, TE) - e_begin;  // the slice's whole tiles
  // fallback ratio M / mean|x| (MMRE_L1Q_RATIO: experiments; <= 0 forces the fallback)
  static const char* ratio_env = getenv("MMRE_L1Q_RATIO");
  const float ratio = ratio_env ? (float)atof(ratio_env) : 128.0f;
  const int n_abs = std::min(kp * 8, L1Q_MAX_BLOCKS);
  const double n_elem = (double)kp * (double)(q_pad + e_cols);
  // code width (MMRE_L1_BITS: experiments and tests): 8 / 16 forces it, otherwise the 8-bit
  // codes unless k_l1q_probe finds their band too wide for this data
  const char* bits_env = getenv("MMRE_L1_BITS");
  const int bits = bits_env ? atoi(bits_env) : 0;
  const int64_t tw = (n_ent + 31) / 32;
  const int64_t n_slice = e_end - e_begin;
  const int n_et = (int)((n_slice + TE - 1) / TE);
  hipLaunchKernelGGL(k_zero_words, dim3(1), dim3(256), 0, st, hdr, L1Q_PART / 4);
  hipLaunchKernelGGL(k_l1q_absmax, dim3((unsigned)n_abs), dim3(256), 0, st, d_q_km, q_pad, d_ent_km + e_begin, e_pad, e_cols,
                     kp, hdr);
  const L1QPlane p8q{d_q_km, q_pad, 0, q_pad, vq}, p8e{d_ent_km, e_pad, e_begin, e_cols, ve};
  const L1QPlane p16q{d_q_km, q_pad, 0, q_pad, uq}, p16e{d_ent_km, e_pad, e_begin, e_cols, ue};
  // the tight per-pair bound (k_l1q_quant8): prediction = the score, no type masks (their sweep
  // keeps the uniform bound), and error offsets that fit one code row (kt <= 1984);
  // MMRE_L1_TIGHT=0 keeps the uniform bound (A/B)
  const char* tight_env = getenv("MMRE_L1_TIGHT");
  const int kt = n_planes(MMRE_TRANSE_L1) * kp;
  const bool tight = pred_kind == 0 && d_type_head == nullptr && kt <= 1984 && !(tight_env && tight_env[0] == '0');
  if (bits != 16) {
    if (tight)
      hipLaunchKernelGGL(k_l1q_quant8<true>, dim3(2048, 2), dim3(256), 0, st, p8q, p8e, kp, k4, kt, hdr, n_abs, n_elem,
                         ratio, q_l1c);
    else
      hipLaunchKernelGGL(k_l1q_quant8<false>, dim3(2048, 2), dim3(256), 0, st, p8q, p8e, kp, k4, kt, hdr, n_abs, n_elem,
                         ratio, q_l1c);
  }
  if (bits == 0) {
    hipLaunchKernelGGL(k_l1q_probe, dim3(L1Q_PROBE_Q), dim3(L1Q_PROBE_E / 4), 0, st, vq, q_pad, n_query, ve + e_begin, e_pad,
                       n_slice, k4, kt, d_truth, pred_kind, margin, hdr, tight ? q_l1c : nullptr);
    const uint32_t probe_max = l1q_probe_max(n_slice);
    hipLaunchKernelGGL(k_l1q_quant<16>, dim3(1024, 2), dim3(256), 0, st, p16q, p16e, kp, k2, hdr, n_abs, n_elem, ratio,
                       1, probe_max);
  } else if (bits == 16) {
    hipLaunchKernelGGL(k_l1q_quant<16>, dim3(1024, 2), dim3(256), 0, st, p16q, p16e, kp, k2, hdr, n_abs, n_elem, ratio,
                       0, 0u);
  }
  MMRE_CHECK_LAUNCH();
  L1Q l1{d_q_rows, d_ent_rows, hdr, (unsigned long long*)((char*)d_work + 256), d_q_km, d_ent_km + e_begin, kp,
         kt, nullptr, tight ? q_l1c : nullptr, hdr + 4};
  l1.wq = l1q_work_counters(hdr);
  const bool tc = d_type_head != nullptr;
  // the gated sweeps: the one the code-width word names counts, the others' workgroups leave
  if (bits != 16) {
    rc = launch_valu<6>(tc, false, st, (const float*)(ve + e_begin), e_pad, n_slice, n_et, (int)e_begin,
                        (const float*)vq, q_pad, n_query, k4, pred_kind, margin, d_truth, d_q_true, d_qr, d_qmode,
                        d_type_head, d_type_tail, tw, d_counts, nullptr, l1, false);
    if (rc) return rc;
  }
  if (bits != 8) {
    // after the 8-bit sweep the 16-bit one rarely counts: gated at its top (one flag load per
    // workgroup, 4 workgroups per resident slot) like the f32 fallback below
    L1Q l16 = l1;
    if (bits == 0) l16.gate = hdr + 1;
    rc = launch_valu<5>(tc, false, st, (const float*)(ue + e_begin), e_pad, n_slice, n_et, (int)e_begin,
                        (const float*)uq, q_pad, n_query, k2, pred_kind, margin, d_truth, d_q_true, d_qr, d_qmode,
                        d_type_head, d_type_tail, tw, d_counts, nullptr, l16, false);
    if (rc) return rc;
  }
  // the fallback: the exact f32 sweep of the float planes, gated on the flag k_l1q_quant wrote
  // (its workgroups return at once when the codes were used)
  L1Q gate{};
  gate.gate = hdr + 1;
  return launch_valu<0>(tc, false, st, d_ent_km + e_begin, e_pad, n_slice, n_et, (int)e_begin, d_q_km, q_pad, n_query,
                        kp, pred_kind, margin, d_truth, d_q_true, d_qr, d_qmode, d_type_head, d_type_tail, tw,
                        d_counts, nullptr, gate, true);
}

// The lock-step window QB x EB for P workgroups per XCD group (BlockMap): about 8 query tiles
// (MMRE_BF3_QB) by P / QB entity tiles, evened out so the last window along each axis is not
// mostly empty (C5: P 96, 64 query tiles, 976 entity tiles per group -> 8 x 12; C3: 89 x 12-13
// -> 7 x 13).
static void bf3_window(int P, int n_qt, int m_e, int& qb, int& eb) {
  static const char* qb_env = getenv("MMRE_BF3_QB");
  int q = qb_env ? atoi(qb_env) : 8;
  q = std::max(1, std::min(q, std::min(P, n_qt)));
  int e = std::max(1, std::min(P / q, m_e));
  const int ne = (m_e + e - 1) / e;      // windows along the entity tiles, then even them out
  e = (m_e + ne - 1) / ne;
  q = std::max(1, std::min(P / e, n_qt));
  const int nq = (n_qt + q - 1) / q;
  q = (n_qt + nq - 1) / nq;
  qb = q;
  eb = e;
}

extern "C" int64_t mmre_link_bf3_workspace(int model, int dim, int64_t e_pad, int64_t q_pad) {
  if (!mfma_model(model) || dim <= 0 || e_pad <= 0 || q_pad <= 0) return 0;
  const int64_t ktot = (int64_t)n_planes(model) * plane_rows(model, dim);
  // ... | the wide sweep's padded thresholds and bound factors (2 x q_pad floats) | its 32-column
  // block maxima of |e| (e_pad / 32 floats)
  return BF3_HDR + 8 * bf3_cap(q_pad, e_pad) + 4 * (q_pad + e_pad) + 4 * ktot * (q_pad + e_pad) + 8 * q_pad +
         4 * (e_pad / 32);
}

extern "C" int mmre_link_bf3_stats(const void* d_work, int64_t work_bytes, uint64_t* d_out, void* stream) {
  if (!d_work || !d_out || work_bytes < BF3_HDR) return MMRE_ERR_ARG;
  hipLaunchKernelGGL(k_bf3_stats, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint32_t*)d_work,
                     (unsigned long long*)d_out);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

// The wide sweep's launch (prediction -S only): a persistent grid of resident workgroups, the
// lock-step windows where the planes overflow the caches (as k_sweep_bf3's), else contiguous
// unit ranges.
template <int QT>
static void launch_bf3w(hipStream_t st, const uint4* eb, int64_t e_pad, int64_t e_cols, int64_t n_slice,
                        const uint4* qb, int64_t q_pad, int64_t n_query, int nkb, int e_begin, const float* thr_pad,
                        const float* qbf, const float* en, int32_t* d_counts, uint32_t* hdr, int2* pairs, int64_t cap,
                        int emajor, bool blocked, const char* grid_env) {
  using G = W3Geom<QT>;
  const int n_etw = (int)((n_slice + W3E - 1) / W3E);
  const int res = resident_groups((const void*)k_sweep_bf3w<2, QT, true>, G::NT);
  const int64_t units = (q_pad / QT) * (int64_t)n_etw;
  int g = (int)std::min<int64_t>(8LL * res, std::max<int64_t>((int64_t)res, units / 16)) & ~7;
  int bq = 0, be = 0;
  const bool blk = blocked && n_etw >= 8 && res % 8 == 0;
  if (blk) g = res;
  if (grid_env && grid_env[0] >= '1' && grid_env[0] <= '9') g = atoi(grid_env);
  if (blk) {  // the windows of the grid actually launched (an env grid: a multiple of 8)
    g = std::max(8, g & ~7);
    bf3_window(g / 8, (int)(q_pad / QT), n_etw / 8, bq, be);
  }
  if (g < 1) g = 1;
  const int ng = (g % 8 == 0 && n_etw >= 8) ? 8 : 1;
  if (blk)
    hipLaunchKernelGGL((k_sweep_bf3w<2, QT, true>), dim3((unsigned)g), dim3(G::NT), 0, st, eb, e_pad, e_cols, n_slice,
                       qb, q_pad, n_query, nkb, n_etw, e_begin, ng, thr_pad, qbf, en, d_counts, hdr, pairs, cap,
                       emajor, bq, be);
  else
    hipLaunchKernelGGL((k_sweep_bf3w<2, QT, false>), dim3((unsigned)g), dim3(G::NT), 0, st, eb, e_pad, e_cols, n_slice,
                       qb, q_pad, n_query, nkb, n_etw, e_begin, ng, thr_pad, qbf, en, d_counts, hdr, pairs, cap,
                       emajor, bq, be);
}

// rows_src (mmre_link_sweep_bf3_rows): the entity split planes, norms and block maxima come from
// the row-major table d_ent_rows in one pass (k_bf3_split_rows), and d_ent_km is written only by
// the gated overflow fallback, right before the exact f32 sweep that reads it.
static int sweep_bf3_impl(int model, int pred_kind, float margin, float* d_ent_km, const float* d_ent_rows,
                          int64_t n_ent, int64_t e_pad, int64_t e_begin, int64_t e_end, const float* d_q_km,
                          const float* d_q_rows, const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode,
                          int64_t n_query, int64_t q_pad, int dim, int32_t* d_counts, const float* d_truth,
                          void* d_work, int64_t work_bytes, void* stream, bool rows_src) {
  if (!mfma_model(model)) return MMRE_ERR_MODEL;
  int rc = check_link_args(model, pred_kind, d_ent_km, n_ent, e_pad, d_q_km, d_q_true, d_qr, d_qmode, n_query,
                           q_pad, nullptr, nullptr, d_counts, d_truth);
  if (rc) return rc;
  if (!d_ent_rows || !d_q_rows || !d_work || work_bytes < mmre_link_bf3_workspace(model, dim, e_pad, q_pad))
    return MMRE_ERR_WORKSPACE;
  if (e_begin < 0 || e_begin % TE || e_end <= e_begin || e_end > n_ent) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(model, dim);
  const int ktot = n_planes(model) * kp;  // a multiple of 16 (plane_rows)
  const int64_t cap = bf3_cap(q_pad, e_pad);
  char* w = (char*)d_work;
  uint32_t* hdr = (uint32_t*)w;
  int2* pairs = (int2*)(w + BF3_HDR);
  float* qn = (float*)(w + BF3_HDR + 8 * cap);
  float* en = qn + q_pad;
  uint4* qb = (uint4*)(en + e_pad);
  uint4* eb = qb + (int64_t)ktot * q_pad / 4;
  float* thr_pad = reinterpret_cast<float*>(eb + (int64_t)ktot * e_pad / 4);
  float* qbf = thr_pad + q_pad;
  float* ebm = qbf + q_pad;  // e_pad / 32 block maxima
  const int64_t e_cols = round_up(e_end, TE) - e_begin;  // the slice's whole tiles
  const int64_t n_slice = e_end - e_begin;
  const int n_et = (int)((n_slice + TE - 1) / TE);
  // bound coefficient (see k_sweep_bf3's header): 1.02 (7K 2^-24 (1 + 2^-7) + 3.02 2^-16 + 2^-29 sqrt K)
  const double K = (double)ktot;
  const float cb = (float)(1.02 * (7.0 * K * std::ldexp(1.0, -24) * (1.0 + std::ldexp(1.0, -7)) +
                                   3.02 * std::ldexp(1.0, -16) + std::ldexp(1.0, -29) * std::sqrt(K)));
  static_assert(BF3_SEGS == 64, "k_bf3_stats sums one segment per lane of a wave");
  hipLaunchKernelGGL(k_bf3_hdr_init, dim3((BF3_HDR / 4 + 255) / 256), dim3(256), 0, st, hdr, cap);
  const int nkb = ktot / 16;
  hipLaunchKernelGGL(k_bf3_split, dim3((unsigned)((q_pad * nkb + 255) / 256)), dim3(256), 0, st, d_q_km, q_pad,
                     (int64_t)0, q_pad, nkb, qb, q_pad);
  if (!rows_src)
    hipLaunchKernelGGL(k_bf3_split, dim3((unsigned)((e_cols * nkb + 255) / 256)), dim3(256), 0, st, d_ent_km, e_pad,
                       e_begin, e_cols, nkb, eb, e_pad);
  static const char* order_env = getenv("MMRE_MFMA_EMAJOR");
  const int emajor = order_env ? atoi(order_env) : ((double)e_pad * ktot * 4.0 > 64.0 * (1 << 20) ? 1 : 0);
  // the wide sweep (k_sweep_bf3w, prediction -S) where the planes overflow the caches (C5: 15.9
  // -> 14.5 ms per evaluation); on cache-resident planes the 128 x 128 one is faster (C3: 0.74 vs
  // 0.86-0.88 ms -- its per-pair bound lists fewer pairs than the wide sweep's per-tile one on
  // trained tables, whose norms vary); MMRE_BF3_WIDE=1 / 0 forces either (tests, A/B)
  const char* wide_env = getenv("MMRE_BF3_WIDE");  // read per call: tests switch it
  const bool wide = pred_kind == 2 && (wide_env ? wide_env[0] != '0' : emajor != 0);
  const char* qt_env = getenv("MMRE_BF3_QT");  // the wide sweep's query tile, 256 or 128
  const int wide_qt = qt_env ? atoi(qt_env) : 256;
  hipLaunchKernelGGL(k_bf3_norms, dim3((unsigned)((q_pad + 3) / 4)), dim3(256), 0, st, d_q_rows, n_query, (int64_t)0,
                     q_pad, ktot, qn, d_truth, wide ? thr_pad : nullptr, qbf, cb);
  if (rows_src)  // split planes, norms and block maxima in one read of the rows (e_cols: whole tiles)
    hipLaunchKernelGGL(k_bf3_split_rows, dim3((unsigned)(e_cols / 32)), dim3(256), 0, st, d_ent_rows, n_ent, e_begin,
                       ktot, eb, e_pad, en, wide ? ebm : nullptr);
  else if (wide)
    hipLaunchKernelGGL(k_bf3_enorms, dim3((unsigned)((e_cols + 31) / 32)), dim3(256), 0, st, d_ent_rows, n_ent,
                       e_begin, e_cols, ktot, en, ebm);
  else
    hipLaunchKernelGGL(k_bf3_norms, dim3((unsigned)((e_cols + 3) / 4)), dim3(256), 0, st, d_ent_rows, n_ent, e_begin,
                       e_cols, ktot, en, nullptr, nullptr, nullptr, 0.0f);
  MMRE_CHECK_LAUNCH();
  static const char* grid_env = getenv("MMRE_SWEEP_GRID"); /* experiments: workgroup count */
  // the lock-step windows pay where the planes overflow the caches (C5, 1 GB: 16.45 -> 16.24 ms);
  // on planes that stay L2 / MALL resident the contiguous ranges are faster (C3, 20 MB: 0.75 vs
  // 0.85 ms, profiles/r5) -- the emajor threshold; MMRE_BF3_BLOCKED=0 / 1 forces either (A/B)
  static const char* blk_env = getenv("MMRE_BF3_BLOCKED");
  const bool blocked = blk_env ? blk_env[0] != '0' : emajor != 0;
#define MMRE_BF3(PKV)                                                                                           \
  do {                                                                                                          \
    if (wide && PKV == 2) {                                                                                     \
      if (q_pad % 256 == 0 && wide_qt == 256)                                                                  \
        launch_bf3w<256>(st, eb, e_pad, e_cols, n_slice, qb, q_pad, n_query, ktot / 16, (int)e_begin, thr_pad,   \
                         qbf, ebm, d_counts, hdr, pairs, cap, emajor, blocked, grid_env);                       \
      else                                                                                                     \
        launch_bf3w<128>(st, eb, e_pad, e_cols, n_slice, qb, q_pad, n_query, ktot / 16, (int)e_begin, thr_pad,   \
                         qbf, ebm, d_counts, hdr, pairs, cap, emajor, blocked, grid_env);                       \
      MMRE_CHECK_LAUNCH();                                                                                     \
    } else {                                                                                                   \
    const int res = resident_groups((const void*)k_sweep_bf3<PKV>, NT);                                        \
    const int64_t units = (q_pad / TQ) * (int64_t)n_et;                                                        \
    /* whole rounds of the resident capacity, ~3 units per workgroup: static ranges of ~12 units left    \
       the list-heavy units' workgroups last (C3, 8,900 units at 768 resident: 4 rounds 0.454 ms against    \
       0.479 for one, profiles/r6) */                                                                        \
    const int64_t rounds = std::max<int64_t>(1, std::min<int64_t>(8, units / (3LL * res)));                   \
    int g = (int)(rounds * res) & ~7;                                                                          \
    int bq = 0, be = 0;                                                                                        \
    const bool blk = blocked && n_et >= 8 && res % 8 == 0;                                                    \
    if (blk) g = res; /* the lock-step windows: one resident wave of workgroups */                            \
    if (grid_env && grid_env[0] >= '1' && grid_env[0] <= '9') g = atoi(grid_env);                           \
    if (blk) { /* the windows of the grid actually launched (an env grid: a multiple of 8) */                  \
      g &= ~7;                                                                                                 \
      if (g < 8) g = 8;                                                                                        \
      bf3_window(g / 8, (int)(q_pad / TQ), n_et / 8, bq, be);                                                  \
    }                                                                                                           \
    const int ng = (g % 8 == 0 && n_et >= 8) ? 8 : 1;                                                          \
    hipLaunchKernelGGL((k_sweep_bf3<PKV>), dim3((unsigned)g), dim3(NT), 0, st, eb, e_pad, n_slice, qb, q_pad,   \
                       n_query, ktot / 16, n_et, (int)e_begin, ng, pred_kind, margin, d_truth, qn, en, cb,     \
                       d_counts, hdr, pairs, cap, emajor, bq, be);                                             \
    MMRE_CHECK_LAUNCH();                                                                                       \
    }                                                                                                          \
    hipLaunchKernelGGL((k_bf3_fallback_zero), dim3((unsigned)((n_query + 255) / 256)), dim3(256), 0, st, hdr,  \
                       d_counts, n_query);                                                                     \
    if (rows_src) { /* the fallback's k-major planes, only when it runs */                                      \
      const int rb = stage_rows(ktot);                                                                         \
      hipLaunchKernelGGL(k_prep_km_gated, dim3((unsigned)((e_cols + rb - 1) / rb)), dim3(256),                  \
                         sizeof(float) * (size_t)rb * (ktot + 1), st, hdr + 1, model,                          \
                         d_ent_rows + e_begin * (int64_t)ktot, n_slice, dim, kp, rb, d_ent_km + e_begin, e_pad); \
    }                                                                                                          \
    launch_mfma(false, false, pred_kind, margin, d_ent_km + e_begin, n_slice, e_pad, n_et, (int)e_begin,       \
                d_q_km, q_pad, n_query, ktot, d_truth, nullptr, nullptr, nullptr, nullptr, 0, d_counts,        \
                nullptr, st, hdr + 1);                                                                         \
    MMRE_CHECK_LAUNCH();                                                                                       \
    hipLaunchKernelGGL((k_bf3_rescore<PKV>), dim3(16 * (BF3_SEGS + 1)), dim3(256), 0, st, hdr, pairs, cap,     \
                       d_q_rows,                                                                               \
                       d_ent_rows, ktot, pred_kind, margin, d_truth, d_counts);                               \
    MMRE_CHECK_LAUNCH();                                                                                       \
  } while (0)
  if (pred_kind == 2) MMRE_BF3(2);
  else MMRE_BF3(-1);
#undef MMRE_BF3
  return launch_finalize(st, d_counts, n_query, false);
}

extern "C" int mmre_link_sweep_bf3(int model, int pred_kind, float margin, const float* d_ent_km,
                                   const float* d_ent_rows, int64_t n_ent, int64_t e_pad, int64_t e_begin,
                                   int64_t e_end, const float* d_q_km, const float* d_q_rows,
                                   const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode,
                                   int64_t n_query, int64_t q_pad, int dim, int32_t* d_counts, const float* d_truth,
                                   void* d_work, int64_t work_bytes, void* stream) {
  return sweep_bf3_impl(model, pred_kind, margin, const_cast<float*>(d_ent_km), d_ent_rows, n_ent, e_pad, e_begin,
                        e_end, d_q_km, d_q_rows, d_q_true, d_qr, d_qmode, n_query, q_pad, dim, d_counts, d_truth,
                        d_work, work_bytes, stream, false);
}

extern "C" int mmre_link_sweep_bf3_rows(int model, int pred_kind, float margin, const float* d_ent_rows,
                                        int64_t n_ent, int64_t e_pad, int64_t e_begin, int64_t e_end,
                                        float* d_ent_km, const float* d_q_km, const float* d_q_rows,
                                        const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode,
                                        int64_t n_query, int64_t q_pad, int dim, int32_t* d_counts,
                                        const float* d_truth, void* d_work, int64_t work_bytes, void* stream) {
  // the row-major table must be the plane layout itself: DistMult with d a multiple of 16 (K = d)
  if (model != MMRE_DISTMULT || plane_rows(model, dim) != dim) return MMRE_ERR_SHAPE;
  if (!d_ent_rows || !d_ent_km || (reinterpret_cast<uintptr_t>(d_ent_rows) & 15)) return MMRE_ERR_ARG;
  return sweep_bf3_impl(model, pred_kind, margin, d_ent_km, d_ent_rows, n_ent, e_pad, e_begin, e_end, d_q_km,
                        d_q_rows, d_q_true, d_qr, d_qmode, n_query, q_pad, dim, d_counts, d_truth, d_work,
                        work_bytes, stream, true);
}

extern "C" int mmre_link_sweep_range(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                                     int64_t e_pad, int64_t e_begin, int64_t e_end, const float* d_q_km,
                                     const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode,
                                     int64_t n_query, int64_t q_pad, int dim, const uint32_t* d_type_head,
                                     const uint32_t* d_type_tail, int32_t* d_counts, const float* d_truth,
                                     void* stream) {
  return sweep_impl(model, pred_kind, margin, d_ent_km, n_ent, e_pad, e_begin, e_end, d_q_km, d_q_true, d_qr, d_qmode,
                    n_query, q_pad, dim, d_type_head, d_type_tail, d_counts, d_truth, nullptr, (hipStream_t)stream);
}

// ---------------------------------------- fused TransE L1 evaluation (round 5) ---
// K1's blocks: rb entity rows, or rb / 2 queries with their truth rows (two row sets): the
// same LDS, 16 rows of kt + 1 floats at C2 (12.9 KB)
static int eval_rb(int kp) { return stage_rows(kp); }
static int eval_rbq(int kp) { return std::max(1, eval_rb(kp) / 2); }
static int64_t eval_blocks(int dim, int64_t e_pad, int64_t q_pad) {
  const int kp = plane_rows(MMRE_TRANSE_L1, dim);
  return (e_pad + eval_rb(kp) - 1) / eval_rb(kp) + (q_pad + eval_rbq(kp) - 1) / eval_rbq(kp);
}
static int64_t eval_extra_bytes(int dim, int64_t e_pad, int64_t q_pad) {
  return 256 + round_up(8 * eval_blocks(dim, e_pad, q_pad), 256);  // tickets, K1's per-block statistics
}

extern "C" int64_t mmre_link_evaluate_l1q_workspace(int dim, int64_t e_pad, int64_t q_pad) {
  const int64_t base = mmre_link_l1q_workspace(dim, e_pad, q_pad);
  return base > 0 ? base + eval_extra_bytes(dim, e_pad, q_pad) : 0;
}

extern "C" int mmre_link_evaluate_l1q(int norm_flag, const float* d_ent, int64_t n_ent, const float* d_rel,
                                      int64_t n_rel, int dim, const int64_t* d_qh, const int64_t* d_qr,
                                      const int64_t* d_qt, const int8_t* d_qmode, int64_t n_query,
                                      const int64_t* d_grp_qoff, const int32_t* d_grp_q, int64_t n_groups,
                                      const int64_t* d_filt_off, const int32_t* d_filt_ids, const int32_t* d_entry_q,
                                      int64_t n_entries, int64_t e_begin, int64_t e_end, float* d_ent_km,
                                      int64_t e_pad, float* d_ent_rows, float* d_q_km, int64_t q_pad, float* d_q_rows,
                                      int32_t* d_q_true, float* d_list_scores, int32_t* d_counts, float* d_truth,
                                      uint32_t* d_undecided_q, void* d_work, int64_t work_bytes, void* stream) {
  if (!d_ent || !d_rel || !d_qh || !d_qr || !d_qt || !d_qmode || !d_ent_km || !d_ent_rows || !d_q_km || !d_q_rows ||
      !d_q_true || !d_counts || !d_truth || !d_grp_qoff || !d_grp_q || !d_filt_off)
    return MMRE_ERR_ARG;
  if (n_ent <= 0 || n_rel <= 0 || dim <= 0 || n_query <= 0 || n_groups <= 0 || n_groups > n_query || n_entries < 0)
    return MMRE_ERR_ARG;
  if (e_pad < n_ent || e_pad % TE || q_pad < n_query || q_pad % TQ) return MMRE_ERR_ARG;
  if (e_begin < 0 || e_begin % TE || e_end <= e_begin || e_end > n_ent) return MMRE_ERR_ARG;
  if (n_entries > 0 && (!d_filt_ids || !d_entry_q || !d_list_scores)) return MMRE_ERR_WORKSPACE;
  if (n_ent > (int64_t)INT32_MAX - 256 || n_query >= (int64_t)INT32_MAX) return MMRE_ERR_SHAPE;
  if (!d_work || work_bytes < mmre_link_evaluate_l1q_workspace(dim, e_pad, q_pad)) return MMRE_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(MMRE_TRANSE_L1, dim), kt = kp, k2 = l1q_rows(dim), k4 = l1q_rows8(dim);
  const int rb = eval_rb(kp), rbq = eval_rbq(kp);
  const size_t lds1 = sizeof(float) * (size_t)std::max(rb, 3 * rbq) * (kt + 1);
  if (lds1 > 64 * 1024) return MMRE_ERR_SHAPE;
  char* w = (char*)d_work;
  uint32_t* hdr = (uint32_t*)w;
  uint32_t* uq = (uint32_t*)(w + L1Q_HDR);
  uint32_t* ue = uq + (int64_t)k2 * q_pad;
  uint32_t* vq = ue + (int64_t)k2 * e_pad;
  uint32_t* ve = vq + (int64_t)k4 * q_pad;
  float* q_l1c = (float*)(ve + (int64_t)k4 * e_pad);
  char* extra = w + mmre_link_l1q_workspace(dim, e_pad, q_pad);
  uint32_t* ticket = (uint32_t*)extra;  // zero before the first call (the caller zeroes the workspace once)
  float* pstat = (float*)(extra + 256);
  const int64_t e_cols = round_up(e_end, TE) - e_begin;
  const int64_t n_slice = e_end - e_begin;
  const int n_et = (int)((n_slice + TE - 1) / TE);
  static const char* ratio_env = getenv("MMRE_L1Q_RATIO");
  static const char* tight_env = getenv("MMRE_L1_TIGHT");
  const char* bits_env = getenv("MMRE_L1_BITS");
  const int bits = bits_env ? atoi(bits_env) : 0;
  const bool tight = kt <= 1984 && !(tight_env && tight_env[0] == '0');
  EvalL1 P{};
  P.ent = d_ent;
  P.rel = d_rel;
  P.n_ent = n_ent;
  P.dim = dim;
  P.kp = kp;
  P.norm = norm_flag ? 1 : 0;
  P.rb = rb;
  P.rbq = rbq;
  P.qh = d_qh;
  P.qr = d_qr;
  P.qt = d_qt;
  P.qmode = d_qmode;
  P.n_query = n_query;
  P.ent_km = d_ent_km;
  P.e_pad = e_pad;
  P.ent_rows = d_ent_rows;
  P.q_km = d_q_km;
  P.q_pad = q_pad;
  P.q_rows = d_q_rows;
  P.q_true = d_q_true;
  P.truth = d_truth;
  P.e_begin = e_begin;
  P.e_cols = e_cols;
  P.n_eblk = (int)((e_pad + rb - 1) / rb);
  P.n_qblk = (int)((q_pad + rbq - 1) / rbq);
  P.pstat = pstat;
  P.und_q = d_undecided_q;
  P.ticket = ticket;
  P.hdr = hdr;
  P.n_elem = (double)kp * (double)(q_pad + e_cols);
  P.ratio = ratio_env ? (float)atof(ratio_env) : 128.0f;
  // K1: prep + truths + |x| statistics (the last block decides codes vs f32 and resets the header)
  hipLaunchKernelGGL(k_eval_prep, dim3((unsigned)(P.n_eblk + P.n_qblk)), dim3(256), lds1, st, P);
  MMRE_CHECK_LAUNCH();
  // K2: list scores | codes (8-bit words + error row, 16-bit words)
  EvalQuant Q{};
  Q.pq = L1QPlane{d_q_km, q_pad, 0, q_pad, vq};
  Q.pe = L1QPlane{d_ent_km, e_pad, e_begin, e_cols, ve};
  Q.out16q = uq;
  Q.out16e = ue;
  Q.kw = k4;
  Q.k2 = k2;
  Q.kt = kt;
  const int n_lblk = (int)((n_entries + 255) / 256);
  // quantization blocks per plane: the list blocks and both planes' blocks resident at once (one
  // round: 2 x 512 + the list blocks took two at an 8-way share of C2, 23 us)
  Q.n_blk = (int)std::min<int64_t>(512, std::max<int64_t>(64, (resident_groups((const void*)k_eval_quant_list, 256) -
                                                              n_lblk) / 2));
  Q.tight = tight ? 1 : 0;
  Q.q_l1c = q_l1c;
  hipLaunchKernelGGL(k_eval_quant_list, dim3((unsigned)(n_lblk + 2 * Q.n_blk)), dim3(256), 0, st, P, Q, d_filt_ids,
                     d_entry_q, n_entries, d_list_scores, n_lblk);
  MMRE_CHECK_LAUNCH();
  // K3: filter counts | the code-width probe
  const int n_cblk = (int)std::min<int64_t>((n_groups + 3) / 4, 65536);  // four groups (waves) per block
  const uint32_t probe_max = l1q_probe_max(n_slice);
  hipLaunchKernelGGL(k_eval_count_probe, dim3((unsigned)(n_cblk + L1Q_PROBE_Q / 4)), dim3(256), 0, st, d_grp_qoff, d_grp_q,
                     n_groups, n_cblk, d_filt_off, d_filt_ids, d_list_scores, d_q_true, d_truth, n_query, n_ent,
                     d_counts, vq, q_pad, ve + e_begin, e_pad, n_slice, k4, kt, tight ? q_l1c : nullptr, hdr,
                     ticket, probe_max, bits == 8 || bits == 16 ? bits : 0);
  MMRE_CHECK_LAUNCH();
  // the sweeps: the one the code-width word names counts, the others' workgroups leave
  const int64_t tw = (n_ent + 31) / 32;
  L1Q l1{d_q_rows, d_ent_rows, hdr, (unsigned long long*)((char*)d_work + 256), d_q_km, d_ent_km + e_begin, kp,
         kt, nullptr, tight ? q_l1c : nullptr, hdr + 4, d_undecided_q};
  l1.wq = l1q_work_counters(hdr);
  // the 8-bit sweep (it leaves unless the word names the 8-bit codes) and the gated 16-bit one
  // (one launch for both widths was tried: with both SAD loops in one kernel the allocator
  // spilled 58-81 VGPRs)
  int rc = launch_valu<6>(false, false, st, (const float*)(ve + e_begin), e_pad, n_slice, n_et, (int)e_begin,
                          (const float*)vq, q_pad, n_query, k4, 0, 0.0f, d_truth, d_q_true, d_qr, d_qmode, nullptr,
                          nullptr, tw, d_counts, nullptr, l1, false);
  if (rc) return rc;
  L1Q l16 = l1;
  l16.gate = hdr + 1;
  rc = launch_valu<5>(false, false, st, (const float*)(ue + e_begin), e_pad, n_slice, n_et, (int)e_begin,
                      (const float*)uq, q_pad, n_query, k2, 0, 0.0f, d_truth, d_q_true, d_qr, d_qmode, nullptr, nullptr,
                      tw, d_counts, nullptr, l16, false);
  if (rc) return rc;
  // the f32 fallback, gated on the word; it also carries the finalize (filtered += raw)
  L1Q gate{};
  gate.gate = hdr + 1;
  gate.fin_counts = d_counts;
  gate.fin_n = n_query;
  gate.fin_ticket = hdr + 6;
  return launch_valu<0>(false, false, st, d_ent_km + e_begin, e_pad, n_slice, n_et, (int)e_begin, d_q_km, q_pad,
                        n_query, kp, 0, 0.0f, d_truth, d_q_true, d_qr, d_qmode, nullptr, nullptr, tw, d_counts,
                        nullptr, gate, false);
}
