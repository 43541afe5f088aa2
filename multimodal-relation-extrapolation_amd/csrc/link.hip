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
//   k_prep_entities   table -> k-major plane (F.normalize for TransE norm_flag)
//   k_prep_queries    (h, r, t, mode) -> k-major query vectors (+ truth ids)
//   k_truth           pred(truth) per query, same arithmetic as the sweep
//   k_filter_correct  subtracts known (filtered) entities that beat the truth
//   k_sweep_valu      TransE L1/L2, RotatE: VALU 8x8 register micro-tiles
//   k_sweep_mfma      DistMult/ComplEx: v_mfma_f32_32x32x2_f32, ballot/popcount epilogue
#include "mmre_common.h"

namespace mmre {

constexpr int TQ = 128;   // queries per workgroup tile
constexpr int TE = 128;   // entities per workgroup tile
constexpr int KC = 8;     // K rows per LDS stage
constexpr int NT = 256;   // threads per workgroup

// rows per plane: TransE/DistMult use one plane of round_up(d, KC) rows;
// ComplEx/RotatE use two planes (re, im) of round_up(d, KC) rows each.
__host__ __device__ inline int plane_rows(int dim) { return (int)round_up(dim, KC); }
__host__ __device__ inline int n_planes(int model) { return (model == MMRE_COMPLEX || model == MMRE_ROTATE) ? 2 : 1; }

// ------------------------------------------------------------------ prep ----
__global__ void k_prep_entities(int model, int norm_flag, const float* __restrict__ ent,
                                const float* __restrict__ ent_im, int64_t n_ent, int dim, int kp,
                                float* __restrict__ out, int64_t e_pad) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= e_pad) return;
  const int np = n_planes(model);
  if (e >= n_ent) {
    for (int k = 0; k < np * kp; ++k) out[(int64_t)k * e_pad + e] = 0.0f;
    return;
  }
  if (model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2) {
    const float* x = ent + e * dim;
    float n = 1.0f;
    if (norm_flag) {  // F.normalize(x, 2, -1): x / max(||x||_2, 1e-12)   (TransE.py:63-66)
      float ss = 0.0f;
      for (int k = 0; k < dim; ++k) ss = ss + x[k] * x[k];
      n = sqrtf(ss);
      if (n < 1e-12f) n = 1e-12f;
    }
    for (int k = 0; k < kp; ++k) out[(int64_t)k * e_pad + e] = k < dim ? (norm_flag ? x[k] / n : x[k]) : 0.0f;
  } else if (model == MMRE_DISTMULT) {
    const float* x = ent + e * dim;
    for (int k = 0; k < kp; ++k) out[(int64_t)k * e_pad + e] = k < dim ? x[k] : 0.0f;
  } else if (model == MMRE_COMPLEX) {
    const float* re = ent + e * dim;
    const float* im = ent_im + e * dim;
    for (int k = 0; k < kp; ++k) {
      out[(int64_t)k * e_pad + e] = k < dim ? re[k] : 0.0f;
      out[(int64_t)(kp + k) * e_pad + e] = k < dim ? im[k] : 0.0f;
    }
  } else {  // RotatE rows are [re | im] of width 2d (RotatE.py:48-49)
    const float* x = ent + e * 2 * dim;
    for (int k = 0; k < kp; ++k) {
      out[(int64_t)k * e_pad + e] = k < dim ? x[k] : 0.0f;
      out[(int64_t)(kp + k) * e_pad + e] = k < dim ? x[dim + k] : 0.0f;
    }
  }
}

__device__ __forceinline__ float row_norm(const float* x, int dim) {
  float ss = 0.0f;
  for (int k = 0; k < dim; ++k) ss = ss + x[k] * x[k];
  float n = sqrtf(ss);
  return n < 1e-12f ? 1e-12f : n;
}

__global__ void k_prep_queries(int model, int norm_flag, const float* __restrict__ ent,
                               const float* __restrict__ ent_im, const float* __restrict__ rel,
                               const float* __restrict__ rel_im, int dim, int kp, float phase_denom,
                               const int64_t* __restrict__ qh, const int64_t* __restrict__ qr,
                               const int64_t* __restrict__ qt, const int8_t* __restrict__ qmode,
                               int64_t n_query, float* __restrict__ out, int64_t q_pad,
                               int32_t* __restrict__ qtrue) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= q_pad) return;
  const int np = n_planes(model);
  if (q >= n_query) {
    for (int k = 0; k < np * kp; ++k) out[(int64_t)k * q_pad + q] = 0.0f;
    return;
  }
  const int64_t h = qh[q], r = qr[q], t = qt[q];
  const bool head = qmode[q] == MMRE_HEAD_BATCH;
  qtrue[q] = (int32_t)(head ? h : t);
  if (model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2) {
    // head_batch: score = h + (r - t) -> q = -(r - t); tail_batch: (h + r) - t -> q = h + r
    // (TransE.py:71-74). |q - e| reproduces both element-wise bit-for-bit.
    const float* hv = ent + h * dim;
    const float* rv = rel + r * dim;
    const float* tv = ent + t * dim;
    float nh = 1.0f, nr = 1.0f, nt = 1.0f;
    if (norm_flag) { nh = row_norm(hv, dim); nr = row_norm(rv, dim); nt = row_norm(tv, dim); }
    for (int k = 0; k < kp; ++k) {
      float v = 0.0f;
      if (k < dim) {
        float a = norm_flag ? hv[k] / nh : hv[k];
        float b = norm_flag ? rv[k] / nr : rv[k];
        float c = norm_flag ? tv[k] / nt : tv[k];
        v = head ? -(b - c) : (a + b);
      }
      out[(int64_t)k * q_pad + q] = v;
    }
  } else if (model == MMRE_DISTMULT) {  // head: h*(r*t) ; tail: (h*r)*t  (DistMult.py:37-42)
    const float* hv = ent + h * dim;
    const float* rv = rel + r * dim;
    const float* tv = ent + t * dim;
    for (int k = 0; k < kp; ++k)
      out[(int64_t)k * q_pad + q] = k < dim ? (head ? rv[k] * tv[k] : hv[k] * rv[k]) : 0.0f;
  } else if (model == MMRE_COMPLEX) {  // ComplEx.py:20-27 regrouped by the candidate entity
    const float *hr = ent + h * dim, *hi = ent_im + h * dim, *tr = ent + t * dim, *ti = ent_im + t * dim;
    const float *rr = rel + r * dim, *ri = rel_im + r * dim;
    for (int k = 0; k < kp; ++k) {
      float a = 0.0f, b = 0.0f;
      if (k < dim) {
        if (head) { a = tr[k] * rr[k] + ti[k] * ri[k]; b = ti[k] * rr[k] - tr[k] * ri[k]; }
        else      { a = hr[k] * rr[k] - hi[k] * ri[k]; b = hi[k] * rr[k] + hr[k] * ri[k]; }
      }
      out[(int64_t)k * q_pad + q] = a;
      out[(int64_t)(kp + k) * q_pad + q] = b;
    }
  } else {  // RotatE (RotatE.py:51-72): rotate by the relation phase, regrouped per candidate
    const float* hrow = ent + h * 2 * dim;
    const float* trow = ent + t * 2 * dim;
    const float* rv = rel + r * dim;
    for (int k = 0; k < kp; ++k) {
      float a = 0.0f, b = 0.0f;
      if (k < dim) {
        float s, c;
        canon_sincos(rv[k] / phase_denom, &s, &c);
        if (head) { float tre = trow[k], tim = trow[dim + k]; a = c * tre + s * tim; b = c * tim - s * tre; }
        else      { float hre = hrow[k], him = hrow[dim + k]; a = hre * c - him * s; b = hre * s + him * c; }
      }
      out[(int64_t)k * q_pad + q] = a;
      out[(int64_t)(kp + k) * q_pad + q] = b;
    }
  }
}

// ------------------------------------------------------------ score ops ----
// OP: 0 TransE L1, 1 TransE L2, 2 RotatE, 3 DistMult, 4 ComplEx. One k step.
template <int OP>
__device__ __forceinline__ float op_step(float acc, float qa, float qb, float x, float y) {
  if constexpr (OP == 0) {
    return acc + fabsf(qa - x);
  } else if constexpr (OP == 1) {
    float d = qa - x;
    return acc + d * d;
  } else if constexpr (OP == 2) {
    float dr = qa - x, di = qb - y;
    return acc + sqrtf(dr * dr + di * di);
  } else {
    return __builtin_fmaf(x, qa, acc);
  }
}
template <int OP>
__device__ __forceinline__ float op_final(float acc) {
  if constexpr (OP == 1) return sqrtf(acc);
  else return acc;
}
__host__ __device__ inline int op_of_model(int model) {
  return model == MMRE_TRANSE_L1 ? 0 : model == MMRE_TRANSE_L2 ? 1 : model == MMRE_ROTATE ? 2
         : model == MMRE_DISTMULT ? 3 : 4;
}

// Score of one (query, entity) pair in the canonical k order.
template <int OP>
__device__ float pair_score(const float* __restrict__ ent_km, int64_t e_pad, const float* __restrict__ q_km,
                            int64_t q_pad, int kp, int64_t q, int64_t e) {
  float acc = 0.0f;
  if constexpr (OP == 2) {
    for (int k = 0; k < kp; ++k)
      acc = op_step<OP>(acc, q_km[(int64_t)k * q_pad + q], q_km[(int64_t)(kp + k) * q_pad + q],
                        ent_km[(int64_t)k * e_pad + e], ent_km[(int64_t)(kp + k) * e_pad + e]);
  } else if constexpr (OP == 4) {  // ComplEx: re plane then im plane, one fma chain
    for (int k = 0; k < 2 * kp; ++k)
      acc = op_step<OP>(acc, q_km[(int64_t)k * q_pad + q], 0.0f, ent_km[(int64_t)k * e_pad + e], 0.0f);
  } else {
    for (int k = 0; k < kp; ++k)
      acc = op_step<OP>(acc, q_km[(int64_t)k * q_pad + q], 0.0f, ent_km[(int64_t)k * e_pad + e], 0.0f);
  }
  return op_final<OP>(acc);
}

template <int OP>
__global__ void k_truth(const float* __restrict__ ent_km, int64_t e_pad, const float* __restrict__ q_km,
                        int64_t q_pad, int kp, const int32_t* __restrict__ qtrue, int64_t n_query,
                        int pred_kind, float margin, float* __restrict__ thr) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_query) return;
  thr[q] = apply_pred(pred_kind, margin, pair_score<OP>(ent_km, e_pad, q_km, q_pad, kp, q, qtrue[q]));
}

__device__ __forceinline__ bool type_bit(const uint32_t* __restrict__ mask, int64_t words, int64_t r, int64_t e) {
  return (mask[r * words + (e >> 5)] >> (e & 31)) & 1u;
}

// Filtered rank correction: for each known entity j of query q (filter CSR), j != truth,
// that beats the truth, subtract one from the filtered counts (Test.h:85 `not _find`).
template <int OP>
__global__ void k_filter_correct(const float* __restrict__ ent_km, int64_t e_pad, int64_t n_ent,
                                 const float* __restrict__ q_km, int64_t q_pad, int kp,
                                 const int32_t* __restrict__ qtrue, const int64_t* __restrict__ qr,
                                 const int8_t* __restrict__ qmode, int64_t n_query, int pred_kind, float margin,
                                 const float* __restrict__ thr, const int64_t* __restrict__ off,
                                 const int32_t* __restrict__ ids, const uint32_t* __restrict__ type_head,
                                 const uint32_t* __restrict__ type_tail, int64_t type_words,
                                 int32_t* __restrict__ counts) {
  const int64_t total = off[n_query];
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = n_query;  // q with off[q] <= p < off[q+1]
    while (hi - lo > 1) {
      int64_t mid = (lo + hi) >> 1;
      if (off[mid] <= p) lo = mid; else hi = mid;
    }
    const int64_t q = lo;
    const int64_t j = ids[p];
    if (j == qtrue[q] || j < 0 || j >= n_ent) continue;
    float v = apply_pred(pred_kind, margin, pair_score<OP>(ent_km, e_pad, q_km, q_pad, kp, q, j));
    if (v < thr[q]) {
      atomicSub(&counts[1 * n_query + q], 1);
      if (type_head) {
        const uint32_t* m = qmode[q] == MMRE_HEAD_BATCH ? type_head : type_tail;
        if (type_bit(m, type_words, qr[q], j)) atomicSub(&counts[3 * n_query + q], 1);
      }
    }
  }
}

// ------------------------------------------------------------ VALU sweep ---
// Workgroup tile 128 queries x 128 entities, 256 threads as 16 (q) x 16 (e); each thread
// owns queries {4tq..4tq+3, 64+4tq..} and entities {4te..4te+3, 64+4te..}: 64 fp32
// accumulators, one sequential k chain each (the canonical order). K is staged through
// LDS in double-buffered steps of 8 rows (16 B per thread per plane per operand).
// blockIdx -> (query tile, entity chunk) with chunk = blockIdx % n_chunk: with n_chunk a
// multiple of 8 every XCD keeps streaming the same 1/8 of the entity table from its L2.
template <int OP, bool TC, bool STORE>
__global__ __launch_bounds__(NT) void k_sweep_valu(
    const float* __restrict__ ent_km, int64_t e_pad, int64_t n_ent, const float* __restrict__ q_km,
    int64_t q_pad, int64_t n_query, int kp, int n_chunk, int et_per_chunk, int pred_kind, float margin,
    const float* __restrict__ thr, const int32_t* __restrict__ qtrue, const int64_t* __restrict__ qr,
    const int8_t* __restrict__ qmode, const uint32_t* __restrict__ type_head,
    const uint32_t* __restrict__ type_tail, int64_t type_words, int32_t* __restrict__ counts,
    float* __restrict__ scores) {
  constexpr int NPL = (OP == 2) ? 2 : 1;
  __shared__ float4 sq[2][NPL][KC][TQ / 4];
  __shared__ float4 se[2][NPL][KC][TE / 4];
  __shared__ float s_thr[TQ];
  __shared__ int32_t s_true[TQ];
  __shared__ int32_t s_rel[TC ? TQ : 1];
  __shared__ int8_t s_mode[TC ? TQ : 1];

  const int tid = threadIdx.x;
  const int tq = tid >> 4, te = tid & 15;
  const int chunk = blockIdx.x % n_chunk;
  const int qtile = blockIdx.x / n_chunk;
  const int64_t q0 = (int64_t)qtile * TQ;
  const int n_et = (int)(e_pad / TE);
  const int et_begin = chunk * et_per_chunk;
  const int et_end = min(et_begin + et_per_chunk, n_et);
  if (et_begin >= et_end) return;  // uniform over the workgroup
  const int nkc = kp / KC;
  const int nsteps = (et_end - et_begin) * nkc;

  if (tid < TQ) {
    int64_t q = q0 + tid;
    bool v = q < n_query;
    s_thr[tid] = v ? thr[q] : -INFINITY;
    s_true[tid] = v ? qtrue[q] : -1;
    if constexpr (TC) {
      s_rel[tid] = v ? (int32_t)qr[q] : 0;
      s_mode[tid] = v ? qmode[q] : 0;
    }
  }

  const int srow = tid >> 5, sc4 = tid & 31;
  float4 rq[NPL], re[NPL];
  auto gload = [&](int step) {
    const int et = et_begin + step / nkc;
    const int k = (step % nkc) * KC + srow;
#pragma unroll
    for (int p = 0; p < NPL; ++p) {
      rq[p] = *reinterpret_cast<const float4*>(q_km + (int64_t)(p * kp + k) * q_pad + q0 + sc4 * 4);
      re[p] = *reinterpret_cast<const float4*>(ent_km + (int64_t)(p * kp + k) * e_pad + (int64_t)et * TE + sc4 * 4);
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int p = 0; p < NPL; ++p) {
      sq[buf][p][srow][sc4] = rq[p];
      se[buf][p][srow][sc4] = re[p];
    }
  };

  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
  int cnt[8], cntc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { cnt[i] = 0; cntc[i] = 0; }

  gload(0);
  swrite(0);
  __syncthreads();

  for (int step = 0; step < nsteps; ++step) {
    const int buf = step & 1;
    if (step + 1 < nsteps) gload(step + 1);
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      float4 a0 = sq[buf][0][kk][tq], a1 = sq[buf][0][kk][16 + tq];
      float4 x0 = se[buf][0][kk][te], x1 = se[buf][0][kk][16 + te];
      const float qa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      if constexpr (OP == 2) {
        float4 b0 = sq[buf][NPL - 1][kk][tq], b1 = sq[buf][NPL - 1][kk][16 + tq];
        float4 y0 = se[buf][NPL - 1][kk][te], y1 = se[buf][NPL - 1][kk][16 + te];
        const float qb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        const float yv[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = op_step<OP>(acc[i][j], qa[i], qb[i], xv[j], yv[j]);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = op_step<OP>(acc[i][j], qa[i], 0.0f, xv[j], 0.0f);
      }
    }
    if ((step + 1) % nkc == 0) {  // entity tile finished: rank epilogue
      const int64_t ebase = (int64_t)(et_begin + step / nkc) * TE;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
        const float th = s_thr[ql];
        const int32_t tr = s_true[ql];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int64_t e = ebase + ((j < 4) ? te * 4 + j : 64 + te * 4 + (j - 4));
          const float v = apply_pred(pred_kind, margin, op_final<OP>(acc[i][j]));
          const bool better = (v < th) && (e != tr) && (e < n_ent);
          cnt[i] += better;
          if constexpr (TC) {
            const uint32_t* m = s_mode[ql] == MMRE_HEAD_BATCH ? type_head : type_tail;
            cntc[i] += better && type_bit(m, type_words, s_rel[ql], e);
          }
          if constexpr (STORE) {
            if (q0 + ql < n_query && e < n_ent) scores[(q0 + ql) * n_ent + e] = v;
          }
          acc[i][j] = 0.0f;
        }
      }
    }
    if (step + 1 < nsteps) swrite(buf ^ 1);
    __syncthreads();
  }

  // reduce over the 16 entity-lanes that share a query (lane bits 0..3), one atomic per query
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    int c = cnt[i], cc = cntc[i];
#pragma unroll
    for (int s = 1; s < 16; s <<= 1) {
      c += __shfl_xor(c, s);
      if constexpr (TC) cc += __shfl_xor(cc, s);
    }
    const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
    const int64_t q = q0 + ql;
    if (te == 0 && q < n_query) {
      if (c) { atomicAdd(&counts[q], c); atomicAdd(&counts[n_query + q], c); }
      if constexpr (TC) {
        if (cc) { atomicAdd(&counts[2 * n_query + q], cc); atomicAdd(&counts[3 * n_query + q], cc); }
      }
    }
  }
}

// ------------------------------------------------------------ MFMA sweep ---
// DistMult / ComplEx: S = Q (queries x K) . E^T (K x entities) with the f32-input MFMA
// v_mfma_f32_32x32x2_f32 (exact f32, a k-ordered fma chain: the canonical order).
// 4 waves as 2 (q) x 2 (e); each wave 64 x 64 = 2 x 2 blocks of 32 x 32 accumulators.
// Epilogue: per accumulator register one ballot over "beats the truth"; the two 32-lane
// halves are two query rows, so two popcounts give exact per-row counts.
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <bool TC, bool STORE>
__global__ __launch_bounds__(NT) void k_sweep_mfma(
    const float* __restrict__ ent_km, int64_t e_pad, int64_t n_ent, const float* __restrict__ q_km,
    int64_t q_pad, int64_t n_query, int ktot, int n_chunk, int et_per_chunk, int pred_kind, float margin,
    const float* __restrict__ thr, const int32_t* __restrict__ qtrue, const int64_t* __restrict__ qr,
    const int8_t* __restrict__ qmode, const uint32_t* __restrict__ type_head,
    const uint32_t* __restrict__ type_tail, int64_t type_words, int32_t* __restrict__ counts,
    float* __restrict__ scores) {
  __shared__ float sq[2][KC][TQ];
  __shared__ float se[2][KC][TE];
  __shared__ float s_thr[TQ];
  __shared__ int32_t s_true[TQ];
  __shared__ int32_t s_rel[TC ? TQ : 1];
  __shared__ int8_t s_mode[TC ? TQ : 1];
  __shared__ int32_t s_cnt[2][2][TQ];  // [we][raw|tc][q]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wq = wave >> 1, we = wave & 1;
  const int chunk = blockIdx.x % n_chunk;
  const int qtile = blockIdx.x / n_chunk;
  const int64_t q0 = (int64_t)qtile * TQ;
  const int n_et = (int)(e_pad / TE);
  const int et_begin = chunk * et_per_chunk;
  const int et_end = min(et_begin + et_per_chunk, n_et);
  if (et_begin >= et_end) return;
  const int nkc = ktot / KC;
  const int nsteps = (et_end - et_begin) * nkc;

  if (tid < TQ) {
    int64_t q = q0 + tid;
    bool v = q < n_query;
    s_thr[tid] = v ? thr[q] : -INFINITY;
    s_true[tid] = v ? qtrue[q] : -1;
    if constexpr (TC) {
      s_rel[tid] = v ? (int32_t)qr[q] : 0;
      s_mode[tid] = v ? qmode[q] : 0;
    }
  }
  for (int i = tid; i < 2 * 2 * TQ; i += NT) (&s_cnt[0][0][0])[i] = 0;

  const int srow = tid >> 5, sc4 = tid & 31;
  float4 rq, re;
  auto gload = [&](int step) {
    const int et = et_begin + step / nkc;
    const int k = (step % nkc) * KC + srow;
    rq = *reinterpret_cast<const float4*>(q_km + (int64_t)k * q_pad + q0 + sc4 * 4);
    re = *reinterpret_cast<const float4*>(ent_km + (int64_t)k * e_pad + (int64_t)et * TE + sc4 * 4);
  };
  auto swrite = [&](int buf) {
    *reinterpret_cast<float4*>(&sq[buf][srow][sc4 * 4]) = rq;
    *reinterpret_cast<float4*>(&se[buf][srow][sc4 * 4]) = re;
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  gload(0);
  swrite(0);
  __syncthreads();

  const int lrow = lane >> 5, lcol = lane & 31;
  for (int step = 0; step < nsteps; ++step) {
    const int buf = step & 1;
    if (step + 1 < nsteps) gload(step + 1);
#pragma unroll
    for (int kp2 = 0; kp2 < KC; kp2 += 2) {
      const float a0 = sq[buf][kp2 + lrow][wq * 64 + lcol];
      const float a1 = sq[buf][kp2 + lrow][wq * 64 + 32 + lcol];
      const float b0 = se[buf][kp2 + lrow][we * 64 + lcol];
      const float b1 = se[buf][kp2 + lrow][we * 64 + 32 + lcol];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if ((step + 1) % nkc == 0) {
      const int64_t ebase = (int64_t)(et_begin + step / nkc) * TE + we * 64;
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
          const int64_t e = ebase + bj * 32 + lcol;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ql = wq * 64 + bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lrow;
            const float v = apply_pred(pred_kind, margin, acc[bi][bj][r]);
            const bool better = (v < s_thr[ql]) && (e != s_true[ql]) && (e < n_ent);
            const uint64_t m = __ballot(better);
            if (lane == 0) {
              const int qlo = wq * 64 + bi * 32 + (r & 3) + 8 * (r >> 2);
              s_cnt[we][0][qlo] += __popcll(m & 0xffffffffull);
              s_cnt[we][0][qlo + 4] += __popcll(m >> 32);
            }
            if constexpr (TC) {
              const uint32_t* tm = s_mode[ql] == MMRE_HEAD_BATCH ? type_head : type_tail;
              const uint64_t mc = __ballot(better && type_bit(tm, type_words, s_rel[ql], e));
              if (lane == 0) {
                const int qlo = wq * 64 + bi * 32 + (r & 3) + 8 * (r >> 2);
                s_cnt[we][1][qlo] += __popcll(mc & 0xffffffffull);
                s_cnt[we][1][qlo + 4] += __popcll(mc >> 32);
              }
            }
            if constexpr (STORE) {
              if (q0 + ql < n_query && e < n_ent) scores[(q0 + ql) * n_ent + e] = v;
            }
            acc[bi][bj][r] = 0.0f;
          }
        }
      }
    }
    if (step + 1 < nsteps) swrite(buf ^ 1);
    __syncthreads();
  }
  if (tid < TQ) {
    const int64_t q = q0 + tid;
    if (q < n_query) {
      int c = s_cnt[0][0][tid] + s_cnt[1][0][tid];
      if (c) { atomicAdd(&counts[q], c); atomicAdd(&counts[n_query + q], c); }
      if constexpr (TC) {
        int cc = s_cnt[0][1][tid] + s_cnt[1][1][tid];
        if (cc) { atomicAdd(&counts[2 * n_query + q], cc); atomicAdd(&counts[3 * n_query + q], cc); }
      }
    }
  }
}

// ---------------------------------------------------------------- launch ---
template <int OP>
static int launch_valu(bool tc, bool store, dim3 grid, hipStream_t st, const float* ent_km, int64_t e_pad,
                       int64_t n_ent, const float* q_km, int64_t q_pad, int64_t n_query, int kp, int n_chunk,
                       int etpc, int pk, float m, const float* thr, const int32_t* qtrue, const int64_t* qr,
                       const int8_t* qmode, const uint32_t* th, const uint32_t* tt, int64_t tw, int32_t* counts,
                       float* scores) {
#define MMRE_VALU(TCV, STV)                                                                                \
  hipLaunchKernelGGL((k_sweep_valu<OP, TCV, STV>), grid, dim3(NT), 0, st, ent_km, e_pad, n_ent, q_km, q_pad, \
                     n_query, kp, n_chunk, etpc, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores)
  if (tc) { if (store) MMRE_VALU(true, true); else MMRE_VALU(true, false); }
  else    { if (store) MMRE_VALU(false, true); else MMRE_VALU(false, false); }
#undef MMRE_VALU
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

}  // namespace mmre

using namespace mmre;

extern "C" int64_t mmre_link_k(int model, int dim) { return (int64_t)n_planes(model) * plane_rows(dim); }
extern "C" int64_t mmre_link_pad(int64_t n) { return round_up(n > 0 ? n : 1, 128); }

static bool valid_model(int m) { return m >= MMRE_TRANSE_L1 && m <= MMRE_ROTATE; }

extern "C" int mmre_link_prepare_entities(int model, int norm_flag, const float* d_ent, const float* d_ent_im,
                                          int64_t n_ent, int dim, float* d_ent_km, int64_t e_pad, void* stream) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (!d_ent || !d_ent_km || n_ent <= 0 || dim <= 0 || e_pad < n_ent || e_pad % TE) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && !d_ent_im) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int threads = 256;
  hipLaunchKernelGGL(k_prep_entities, dim3((unsigned)((e_pad + threads - 1) / threads)), dim3(threads), 0, st,
                     model, norm_flag, d_ent, d_ent_im, n_ent, dim, plane_rows(dim), d_ent_km, e_pad);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_link_prepare_queries(int model, int norm_flag, const float* d_ent, const float* d_ent_im,
                                         const float* d_rel, const float* d_rel_im, int64_t n_ent, int64_t n_rel,
                                         int dim, float phase_denom, const int64_t* d_qh, const int64_t* d_qr,
                                         const int64_t* d_qt, const int8_t* d_qmode, int64_t n_query,
                                         float* d_q_km, int64_t q_pad, int32_t* d_q_true, void* stream) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (!d_ent || !d_rel || !d_qh || !d_qr || !d_qt || !d_qmode || !d_q_km || !d_q_true) return MMRE_ERR_ARG;
  if (n_query <= 0 || q_pad < n_query || q_pad % TQ || dim <= 0 || n_ent <= 0 || n_rel <= 0) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!d_ent_im || !d_rel_im)) return MMRE_ERR_ARG;
  if (model == MMRE_ROTATE && !(phase_denom != 0.0f)) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int threads = 256;
  hipLaunchKernelGGL(k_prep_queries, dim3((unsigned)((q_pad + threads - 1) / threads)), dim3(threads), 0, st,
                     model, norm_flag, d_ent, d_ent_im, d_rel, d_rel_im, dim, plane_rows(dim), phase_denom, d_qh,
                     d_qr, d_qt, d_qmode, n_query, d_q_km, q_pad, d_q_true);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

template <int OP>
static int launch_aux(hipStream_t st, const float* ent_km, int64_t e_pad, int64_t n_ent, const float* q_km,
                      int64_t q_pad, int kp, const int32_t* qtrue, const int64_t* qr, const int8_t* qmode,
                      int64_t n_query, int pk, float m, float* thr, const int64_t* off, const int32_t* ids,
                      const uint32_t* th, const uint32_t* tt, int64_t tw, int32_t* counts) {
  const int threads = 256;
  hipLaunchKernelGGL((k_truth<OP>), dim3((unsigned)((n_query + threads - 1) / threads)), dim3(threads), 0, st,
                     ent_km, e_pad, q_km, q_pad, kp, qtrue, n_query, pk, m, thr);
  MMRE_CHECK_LAUNCH();
  if (off) {
    hipLaunchKernelGGL((k_filter_correct<OP>), dim3(1024), dim3(threads), 0, st, ent_km, e_pad, n_ent, q_km,
                       q_pad, kp, qtrue, qr, qmode, n_query, pk, m, thr, off, ids, th, tt, tw, counts);
    MMRE_CHECK_LAUNCH();
  }
  return MMRE_OK;
}

static int check_link_args(int model, int pred_kind, const float* d_ent_km, int64_t n_ent, int64_t e_pad,
                           const float* d_q_km, const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode,
                           int64_t n_query, int64_t q_pad, const uint32_t* d_type_head, const uint32_t* d_type_tail,
                           const int32_t* d_counts, const float* d_truth) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (pred_kind < 0 || pred_kind > 3) return MMRE_ERR_ARG;
  if (!d_ent_km || !d_q_km || !d_q_true || !d_counts || !d_truth || !d_qmode || !d_qr) return MMRE_ERR_ARG;
  if (n_query <= 0 || n_ent <= 0 || e_pad < n_ent || e_pad % TE || q_pad < n_query || q_pad % TQ) return MMRE_ERR_ARG;
  if ((d_type_head == nullptr) != (d_type_tail == nullptr)) return MMRE_ERR_ARG;
  if (n_ent >= (int64_t)INT32_MAX) return MMRE_ERR_SHAPE;
  return MMRE_OK;
}

extern "C" int mmre_link_truth(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                               int64_t e_pad, const float* d_q_km, const int32_t* d_q_true, const int64_t* d_qr,
                               const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                               const int64_t* d_filt_off, const int32_t* d_filt_ids, const uint32_t* d_type_head,
                               const uint32_t* d_type_tail, int32_t* d_counts, float* d_truth, void* stream) {
  int rc = check_link_args(model, pred_kind, d_ent_km, n_ent, e_pad, d_q_km, d_q_true, d_qr, d_qmode, n_query, q_pad,
                           d_type_head, d_type_tail, d_counts, d_truth);
  if (rc) return rc;
  if ((d_filt_off == nullptr) != (d_filt_ids == nullptr)) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(dim);
  const int64_t tw = (n_ent + 31) / 32;
  MMRE_CHECK(hipMemsetAsync(d_counts, 0, sizeof(int32_t) * 4 * n_query, st));
  switch (op_of_model(model)) {
    case 0: return launch_aux<0>(st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, kp, d_q_true, d_qr, d_qmode, n_query,
                                 pred_kind, margin, d_truth, d_filt_off, d_filt_ids, d_type_head, d_type_tail, tw, d_counts);
    case 1: return launch_aux<1>(st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, kp, d_q_true, d_qr, d_qmode, n_query,
                                 pred_kind, margin, d_truth, d_filt_off, d_filt_ids, d_type_head, d_type_tail, tw, d_counts);
    case 2: return launch_aux<2>(st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, kp, d_q_true, d_qr, d_qmode, n_query,
                                 pred_kind, margin, d_truth, d_filt_off, d_filt_ids, d_type_head, d_type_tail, tw, d_counts);
    case 3: return launch_aux<3>(st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, kp, d_q_true, d_qr, d_qmode, n_query,
                                 pred_kind, margin, d_truth, d_filt_off, d_filt_ids, d_type_head, d_type_tail, tw, d_counts);
    default: return launch_aux<4>(st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, kp, d_q_true, d_qr, d_qmode, n_query,
                                  pred_kind, margin, d_truth, d_filt_off, d_filt_ids, d_type_head, d_type_tail, tw, d_counts);
  }
}

extern "C" int mmre_link_sweep(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                               int64_t e_pad, const float* d_q_km, const int32_t* d_q_true, const int64_t* d_qr,
                               const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                               const uint32_t* d_type_head, const uint32_t* d_type_tail, int32_t* d_counts,
                               const float* d_truth, float* d_scores, void* stream) {
  int rc = check_link_args(model, pred_kind, d_ent_km, n_ent, e_pad, d_q_km, d_q_true, d_qr, d_qmode, n_query, q_pad,
                           d_type_head, d_type_tail, d_counts, d_truth);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const int kp = plane_rows(dim);
  const int64_t tw = (n_ent + 31) / 32;
  const bool tc = d_type_head != nullptr;
  const bool store = d_scores != nullptr;
  const int op = op_of_model(model);
  // grid: (query tiles) x (entity chunks); chunk count a multiple of 8 for XCD affinity
  const int n_qt = (int)(q_pad / TQ);
  const int n_et = (int)(e_pad / TE);
  int n_chunk = (2048 + n_qt - 1) / n_qt;
  n_chunk = (int)round_up(n_chunk, 8);
  if (n_chunk > n_et) n_chunk = n_et;
  const int etpc = (n_et + n_chunk - 1) / n_chunk;
  const dim3 grid((unsigned)(n_qt * n_chunk));
  if (op <= 2) {
    if (op == 0) return launch_valu<0>(tc, store, grid, st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, n_query, kp, n_chunk, etpc,
                                       pred_kind, margin, d_truth, d_q_true, d_qr, d_qmode, d_type_head, d_type_tail, tw, d_counts, d_scores);
    if (op == 1) return launch_valu<1>(tc, store, grid, st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, n_query, kp, n_chunk, etpc,
                                       pred_kind, margin, d_truth, d_q_true, d_qr, d_qmode, d_type_head, d_type_tail, tw, d_counts, d_scores);
    return launch_valu<2>(tc, store, grid, st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, n_query, kp, n_chunk, etpc,
                          pred_kind, margin, d_truth, d_q_true, d_qr, d_qmode, d_type_head, d_type_tail, tw, d_counts, d_scores);
  }
  const int ktot = n_planes(model) * kp;
#define MMRE_MFMA(TCV, STV)                                                                                     \
  hipLaunchKernelGGL((k_sweep_mfma<TCV, STV>), grid, dim3(NT), 0, st, d_ent_km, e_pad, n_ent, d_q_km, q_pad,    \
                     n_query, ktot, n_chunk, etpc, pred_kind, margin, d_truth, d_q_true, d_qr, d_qmode,         \
                     d_type_head, d_type_tail, tw, d_counts, d_scores)
  if (tc) { if (store) MMRE_MFMA(true, true); else MMRE_MFMA(true, false); }
  else    { if (store) MMRE_MFMA(false, true); else MMRE_MFMA(false, false); }
#undef MMRE_MFMA
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
