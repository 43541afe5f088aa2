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
#include <stdlib.h>

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
// Canonical sum of squares of a row: sequential in k (loads issued 8 at a time).
__device__ __forceinline__ float seq_sumsq(const float* __restrict__ r, int dim) {
  float ss = 0.0f;
  int k = 0;
  for (; k + 8 <= dim; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = r[k + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) ss = ss + v[u] * v[u];
  }
  for (; k < dim; ++k) ss = ss + r[k] * r[k];
  return ss;
}

__global__ void k_prep_entities(int model, int norm_flag, const float* __restrict__ ent,
                                const float* __restrict__ ent_im, int64_t n_ent, int dim, int kp,
                                float* __restrict__ out, int64_t e_pad, float* __restrict__ rows) {
  // out: k-major planes [np*kp][e_pad] for the sweep; rows: the same values row-major
  // [n_ent][np*kp] for the per-entity gathers of the truth / filter kernels.
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= e_pad) return;
  const int np = n_planes(model);
  const int kt = np * kp;
  if (e >= n_ent) {
    for (int k = 0; k < kt; ++k) out[(int64_t)k * e_pad + e] = 0.0f;
    return;
  }
  float* row = rows + e * kt;
  if (model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2) {
    const float* x = ent + e * dim;
    float n = 1.0f;
    if (norm_flag) {  // F.normalize(x, 2, -1): x / max(||x||_2, 1e-12)   (TransE.py:63-66)
      n = sqrtf(seq_sumsq(x, dim));
      if (n < 1e-12f) n = 1e-12f;
    }
    for (int k = 0; k < kp; ++k) {
      const float v = k < dim ? (norm_flag ? x[k] / n : x[k]) : 0.0f;
      out[(int64_t)k * e_pad + e] = v;
      row[k] = v;
    }
  } else if (model == MMRE_DISTMULT) {
    const float* x = ent + e * dim;
    for (int k = 0; k < kp; ++k) {
      const float v = k < dim ? x[k] : 0.0f;
      out[(int64_t)k * e_pad + e] = v;
      row[k] = v;
    }
  } else {
    // ComplEx: planes re | im from two tables; RotatE rows are [re | im] of width 2d (RotatE.py:48-49)
    const float* re = model == MMRE_COMPLEX ? ent + e * dim : ent + e * 2 * dim;
    const float* im = model == MMRE_COMPLEX ? ent_im + e * dim : ent + e * 2 * dim + dim;
    for (int k = 0; k < kp; ++k) {
      const float a = k < dim ? re[k] : 0.0f, b = k < dim ? im[k] : 0.0f;
      out[(int64_t)k * e_pad + e] = a;
      out[(int64_t)(kp + k) * e_pad + e] = b;
      row[k] = a;
      row[kp + k] = b;
    }
  }
}

// F.normalize of the relation rows (TransE norm_flag), one sequential row per thread.
__global__ void k_norm_rows(const float* __restrict__ x, int64_t n, int dim, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = x + i * dim;
  const float ss = seq_sumsq(r, dim);
  float nrm = sqrtf(ss);
  if (nrm < 1e-12f) nrm = 1e-12f;
  for (int k = 0; k < dim; ++k) out[i * dim + k] = r[k] / nrm;
}

// Query vectors, one thread per (query, k): element-wise ops on prepared rows
// (ent_rows = the sweep's entity values; rel = normalised relation rows for TransE).
__global__ void k_prep_queries(int model, const float* __restrict__ ent_rows, const float* __restrict__ rel,
                               const float* __restrict__ rel_im, int dim, int kp, float phase_denom,
                               const int64_t* __restrict__ qh, const int64_t* __restrict__ qr,
                               const int64_t* __restrict__ qt, const int8_t* __restrict__ qmode,
                               int64_t n_query, float* __restrict__ out, int64_t q_pad,
                               int32_t* __restrict__ qtrue) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;  // 0 .. kp-1
  if (q >= q_pad) return;
  const int np = n_planes(model);
  const int kt = np * kp;
  if (q >= n_query || k >= dim) {
    out[(int64_t)k * q_pad + q] = 0.0f;
    if (np == 2) out[(int64_t)(kp + k) * q_pad + q] = 0.0f;
    return;
  }
  const int64_t h = qh[q], r = qr[q], t = qt[q];
  const bool head = qmode[q] == MMRE_HEAD_BATCH;
  if (k == 0) qtrue[q] = (int32_t)(head ? h : t);
  const float* hrow = ent_rows + h * kt;
  const float* trow = ent_rows + t * kt;
  if (model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2) {
    // head_batch: score = h + (r - t) -> q = -(r - t); tail_batch: (h + r) - t -> q = h + r
    // (TransE.py:71-74). |q - e| reproduces both element-wise bit-for-bit.
    const float b = rel[r * dim + k];
    out[(int64_t)k * q_pad + q] = head ? -(b - trow[k]) : (hrow[k] + b);
  } else if (model == MMRE_DISTMULT) {  // head: h*(r*t) ; tail: (h*r)*t  (DistMult.py:37-42)
    const float b = rel[r * dim + k];
    out[(int64_t)k * q_pad + q] = head ? b * trow[k] : hrow[k] * b;
  } else if (model == MMRE_COMPLEX) {  // ComplEx.py:20-27 regrouped by the candidate entity
    const float rr = rel[r * dim + k], ri = rel_im[r * dim + k];
    const float tr = trow[k], ti = trow[kp + k], hr = hrow[k], hi = hrow[kp + k];
    float a, b;
    if (head) { a = tr * rr + ti * ri; b = ti * rr - tr * ri; }
    else      { a = hr * rr - hi * ri; b = hi * rr + hr * ri; }
    out[(int64_t)k * q_pad + q] = a;
    out[(int64_t)(kp + k) * q_pad + q] = b;
  } else {  // RotatE (RotatE.py:51-72): rotate by the relation phase, regrouped per candidate
    float s, c;
    canon_sincos(rel[r * dim + k] / phase_denom, &s, &c);
    float a, b;
    if (head) { const float tre = trow[k], tim = trow[kp + k]; a = c * tre + s * tim; b = c * tim - s * tre; }
    else      { const float hre = hrow[k], him = hrow[kp + k]; a = hre * c - him * s; b = hre * s + him * c; }
    out[(int64_t)k * q_pad + q] = a;
    out[(int64_t)(kp + k) * q_pad + q] = b;
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

// Score of one (query, entity) pair in the canonical k order; entity values from the
// row-major copy (one contiguous row per entity, loaded 8 at a time), query values from
// the k-major plane. kp is a multiple of 8 (KC).
template <int OP>
__device__ float pair_score(const float* __restrict__ ent_rows, const float* __restrict__ q_km, int64_t q_pad,
                            int kp, int64_t q, int64_t e) {
  float acc = 0.0f;
  const int np = (OP == 2 || OP == 4) ? 2 : 1;
  const float* row = ent_rows + e * (int64_t)np * kp;
  const float* qc = q_km + q;
  if constexpr (OP == 2) {
    for (int k0 = 0; k0 < kp; k0 += 8) {
      float x[8], y[8], a[8], b[8];
      *reinterpret_cast<float4*>(&x[0]) = *reinterpret_cast<const float4*>(row + k0);
      *reinterpret_cast<float4*>(&x[4]) = *reinterpret_cast<const float4*>(row + k0 + 4);
      *reinterpret_cast<float4*>(&y[0]) = *reinterpret_cast<const float4*>(row + kp + k0);
      *reinterpret_cast<float4*>(&y[4]) = *reinterpret_cast<const float4*>(row + kp + k0 + 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        a[i] = qc[(int64_t)(k0 + i) * q_pad];
        b[i] = qc[(int64_t)(kp + k0 + i) * q_pad];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc = op_step<OP>(acc, a[i], b[i], x[i], y[i]);
    }
  } else {
    const int kt = np * kp;  // ComplEx: re plane then im plane, one fma chain
    for (int k0 = 0; k0 < kt; k0 += 8) {
      float x[8], a[8];
      *reinterpret_cast<float4*>(&x[0]) = *reinterpret_cast<const float4*>(row + k0);
      *reinterpret_cast<float4*>(&x[4]) = *reinterpret_cast<const float4*>(row + k0 + 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = qc[(int64_t)(k0 + i) * q_pad];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc = op_step<OP>(acc, a[i], 0.0f, x[i], 0.0f);
    }
  }
  return op_final<OP>(acc);
}

template <int OP>
__global__ void k_truth(const float* __restrict__ ent_rows, const float* __restrict__ q_km,
                        int64_t q_pad, int kp, const int32_t* __restrict__ qtrue, int64_t n_query,
                        int pred_kind, float margin, float* __restrict__ thr) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_query) return;
  thr[q] = apply_pred(pred_kind, margin, pair_score<OP>(ent_rows, q_km, q_pad, kp, q, qtrue[q]));
}

__device__ __forceinline__ bool type_bit(const uint32_t* __restrict__ mask, int64_t words, int64_t r, int64_t e) {
  return (mask[r * words + (e >> 5)] >> (e & 31)) & 1u;
}

// Filtered rank correction: for each known entity j of query q (filter CSR), j != truth,
// that beats the truth, subtract one from the filtered counts (Test.h:85 `not _find`).
// One 64-thread workgroup per query (grid-stride), lanes over its list.
template <int OP>
__global__ __launch_bounds__(64) void k_filter_correct(
    const float* __restrict__ ent_rows, int64_t n_ent, const float* __restrict__ q_km, int64_t q_pad, int kp,
    const int32_t* __restrict__ qtrue, const int64_t* __restrict__ qr, const int8_t* __restrict__ qmode,
    int64_t n_query, int pred_kind, float margin, const float* __restrict__ thr, const int64_t* __restrict__ off,
    const int32_t* __restrict__ ids, const uint32_t* __restrict__ type_head, const uint32_t* __restrict__ type_tail,
    int64_t type_words, int32_t* __restrict__ counts) {
  for (int64_t q = blockIdx.x; q < n_query; q += gridDim.x) {
    const int64_t a = off[q], b = off[q + 1];
    const float th = thr[q];
    const int32_t tr = qtrue[q];
    int c = 0, cc = 0;
    for (int64_t p = a + threadIdx.x; p < b; p += blockDim.x) {
      const int64_t j = ids[p];
      if (j == tr || j < 0 || j >= n_ent) continue;
      const float v = apply_pred(pred_kind, margin, pair_score<OP>(ent_rows, q_km, q_pad, kp, q, j));
      if (v < th) {
        c += 1;
        if (type_head) {
          const uint32_t* m = qmode[q] == MMRE_HEAD_BATCH ? type_head : type_tail;
          cc += type_bit(m, type_words, qr[q], j);
        }
      }
    }
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      c += __shfl_xor(c, s);
      cc += __shfl_xor(cc, s);
    }
    if (threadIdx.x == 0) {
      if (c) atomicSub(&counts[1 * n_query + q], c);
      if (cc) atomicSub(&counts[3 * n_query + q], cc);
    }
  }
}

// ------------------------------------------------------------ VALU sweep ---
// Work unit = (query tile of 128) x (entity tile of 128); units are ordered query-tile
// major and split into equal contiguous ranges over a persistent grid sized to the
// resident capacity (4 workgroups per CU), so no tail round is left half empty.
// Within a unit: 256 threads as 16 (q) x 16 (e); each thread owns queries
// {4tq..4tq+3, 64+4tq..} and entities {4te..4te+3, 64+4te..}: 64 fp32 accumulators, one
// sequential k chain each (the canonical order). K is staged through LDS in
// double-buffered steps of 8 rows (16 B per thread per plane per operand). Per-query
// counts stay in registers until the workgroup moves to the next query tile.
template <int OP, bool TC, bool STORE>
__global__ __launch_bounds__(NT, (OP == 2) ? 3 : 4) void k_sweep_valu(
    const float* __restrict__ ent_km, int64_t e_pad, int64_t n_ent, const float* __restrict__ q_km,
    int64_t q_pad, int64_t n_query, int kp, int n_et, int n_groups, int pred_kind, float margin,
    const float* __restrict__ thr, const int32_t* __restrict__ qtrue, const int64_t* __restrict__ qr,
    const int8_t* __restrict__ qmode, const uint32_t* __restrict__ type_head,
    const uint32_t* __restrict__ type_tail, int64_t type_words, int32_t* __restrict__ counts,
    float* __restrict__ scores) {
  constexpr int NPL = (OP == 2) ? 2 : 1;
  __shared__ float4 sq[2][NPL][KC][TQ / 4];
  __shared__ float4 se[2][NPL][KC][TE / 4];
  __shared__ float s_thr[2][TQ];
  __shared__ int32_t s_true[2][TQ];
  __shared__ int32_t s_rel[2][TC ? TQ : 1];
  __shared__ int8_t s_mode[2][TC ? TQ : 1];
  __shared__ int32_t s_cnt[TC ? 2 : 1][8][NT];  // per-thread counters (off the VGPR budget)

  const int tid = threadIdx.x;
  const int tq = tid >> 4, te = tid & 15;
  // XCD-aware split: workgroup group x = blockIdx % n_groups (8 when the grid is a multiple of
  // 8: the groups that round-robin dispatch places on one XCD) owns entity tiles
  // [ex0, ex1) for all query tiles, so each XCD's L2 keeps streaming the same ~1/8 of the
  // table; its units (query-tile major) are split evenly over the group's workgroups.
  const int grp = blockIdx.x % n_groups, gmem = blockIdx.x / n_groups;
  const int per_grp = gridDim.x / n_groups;
  const int ex0 = (int)((int64_t)grp * n_et / n_groups), ex1 = (int)((int64_t)(grp + 1) * n_et / n_groups);
  const int n_ex = ex1 - ex0;
  const int units_g = (int)(q_pad / TQ) * n_ex;
  const int u0 = (int)((int64_t)gmem * units_g / per_grp);
  const int u1 = (int)((int64_t)(gmem + 1) * units_g / per_grp);
  if (u0 >= u1) return;  // uniform over the workgroup
  const int nkc = kp / KC;

  auto load_meta = [&](int qtile, int slot) {
    if (tid < TQ) {
      const int64_t q = (int64_t)qtile * TQ + tid;
      const bool v = q < n_query;
      s_thr[slot][tid] = v ? thr[q] : -INFINITY;
      s_true[slot][tid] = v ? qtrue[q] : -1;
      if constexpr (TC) {
        s_rel[slot][tid] = v ? (int32_t)qr[q] : 0;
        s_mode[slot][tid] = v ? qmode[q] : 0;
      }
    }
  };

  const int srow = tid >> 5, sc4 = tid & 31;
  float4 rq[NPL], re[NPL];
  // staging position (unit, kc) of the next load, advanced incrementally (no divisions)
  int ld_unit = u0, ld_kc = 0, ld_qt = u0 / n_ex, ld_et = ex0 + u0 % n_ex;
  auto gload = [&]() {
    const int k = ld_kc * KC + srow;
    const int64_t q0 = (int64_t)ld_qt * TQ, e0 = (int64_t)ld_et * TE;
#pragma unroll
    for (int p = 0; p < NPL; ++p) {
      rq[p] = *reinterpret_cast<const float4*>(q_km + (int64_t)(p * kp + k) * q_pad + q0 + sc4 * 4);
      re[p] = *reinterpret_cast<const float4*>(ent_km + (int64_t)(p * kp + k) * e_pad + e0 + sc4 * 4);
    }
    if (++ld_kc == nkc) {
      ld_kc = 0;
      ++ld_unit;
      if (++ld_et == ex1) { ld_et = ex0; ++ld_qt; }
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
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s_cnt[0][i][tid] = 0;
    if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] = 0;
  }

  int cur_qt = u0 / n_ex, cur_et = ex0 + u0 % n_ex;
  int slot = 0;
  load_meta(cur_qt, 0);
  gload();
  swrite(0);
  __syncthreads();

  int buf = 0;
  for (int unit = u0; unit < u1; ++unit) {
    for (int kc = 0; kc < nkc; ++kc) {
      const bool more = ld_unit < u1;
      if (more) gload();
#pragma unroll 2
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
      if (kc == nkc - 1) {  // unit finished: rank epilogue
        const int64_t q0 = (int64_t)cur_qt * TQ;
        const int64_t ebase = (int64_t)cur_et * TE;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int ql = (i < 4) ? tq * 4 + i : 64 + tq * 4 + (i - 4);
          const float th = s_thr[slot][ql];
          const int32_t tr = s_true[slot][ql];
          int c = 0, cc = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int64_t e = ebase + ((j < 4) ? te * 4 + j : 64 + te * 4 + (j - 4));
            const float v = apply_pred(pred_kind, margin, op_final<OP>(acc[i][j]));
            const bool better = (v < th) && (e != tr) && (e < n_ent);
            c += better;
            if constexpr (TC) {
              const uint32_t* m = s_mode[slot][ql] == MMRE_HEAD_BATCH ? type_head : type_tail;
              cc += better && type_bit(m, type_words, s_rel[slot][ql], e);
            }
            if constexpr (STORE) {
              if (q0 + ql < n_query && e < n_ent) scores[(q0 + ql) * n_ent + e] = v;
            }
            acc[i][j] = 0.0f;
          }
          s_cnt[0][i][tid] += c;
          if constexpr (TC) s_cnt[TC ? 1 : 0][i][tid] += cc;
        }
        const bool last = unit + 1 >= u1;
        int next_qt = cur_qt, next_et = cur_et + 1;
        if (next_et == ex1) { next_et = ex0; ++next_qt; }
        if (last || next_qt != cur_qt) {  // uniform: flush this query tile's counts
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
            if (te == 0 && q < n_query) {
              if (c) { atomicAdd(&counts[q], c); atomicAdd(&counts[n_query + q], c); }
              if constexpr (TC) {
                if (cc) { atomicAdd(&counts[2 * n_query + q], cc); atomicAdd(&counts[3 * n_query + q], cc); }
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
        cur_qt = next_qt;
        cur_et = next_et;
      }
      if (more) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
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

template <int OP, bool TCV, bool STV>
static void launch_valu_one(hipStream_t st, const float* ent_km, int64_t e_pad, int64_t n_ent, const float* q_km,
                            int64_t q_pad, int64_t n_query, int kp, int pk, float m, const float* thr,
                            const int32_t* qtrue, const int64_t* qr, const int8_t* qmode, const uint32_t* th,
                            const uint32_t* tt, int64_t tw, int32_t* counts, float* scores) {
  const int n_et = (int)(e_pad / TE);
  // 16 workgroups per resident slot: short per-workgroup ranges let the dispatcher balance
  // CUs that run at different speeds (C2 on MI355X: 1,024 groups 4.0 ms, 8,192 3.43 ms,
  // 16,384 3.30 ms, 30,528 (one unit each) 3.36 ms).
  int g = 16 * resident_groups((const void*)k_sweep_valu<OP, TCV, STV>, NT);
  // MMRE_SWEEP_GRID (experiments): "tiles" = one workgroup per (query tile, 1/8 of the
  // entity tiles); a number = that many persistent workgroups.
  static const char* gmode = getenv("MMRE_SWEEP_GRID");
  if (gmode && gmode[0] == 't') g = 8 * (int)(q_pad / TQ);
  else if (gmode && gmode[0] >= '1' && gmode[0] <= '9') g = atoi(gmode);
  const int ng = (g % 8 == 0 && n_et >= 8) ? 8 : 1;
  hipLaunchKernelGGL((k_sweep_valu<OP, TCV, STV>), dim3((unsigned)g), dim3(NT), 0, st, ent_km, e_pad, n_ent, q_km,
                     q_pad, n_query, kp, n_et, ng, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores);
}

template <int OP>
static int launch_valu(bool tc, bool store, hipStream_t st, const float* ent_km, int64_t e_pad, int64_t n_ent,
                       const float* q_km, int64_t q_pad, int64_t n_query, int kp, int pk, float m, const float* thr,
                       const int32_t* qtrue, const int64_t* qr, const int8_t* qmode, const uint32_t* th,
                       const uint32_t* tt, int64_t tw, int32_t* counts, float* scores) {
  if (tc && store) launch_valu_one<OP, true, true>(st, ent_km, e_pad, n_ent, q_km, q_pad, n_query, kp, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores);
  else if (tc) launch_valu_one<OP, true, false>(st, ent_km, e_pad, n_ent, q_km, q_pad, n_query, kp, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores);
  else if (store) launch_valu_one<OP, false, true>(st, ent_km, e_pad, n_ent, q_km, q_pad, n_query, kp, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores);
  else launch_valu_one<OP, false, false>(st, ent_km, e_pad, n_ent, q_km, q_pad, n_query, kp, pk, m, thr, qtrue, qr, qmode, th, tt, tw, counts, scores);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

}  // namespace mmre

using namespace mmre;

extern "C" int64_t mmre_link_k(int model, int dim) { return (int64_t)n_planes(model) * plane_rows(dim); }
extern "C" int64_t mmre_link_pad(int64_t n) { return round_up(n > 0 ? n : 1, 128); }

static bool valid_model(int m) { return m >= MMRE_TRANSE_L1 && m <= MMRE_ROTATE; }

extern "C" int mmre_link_prepare_entities(int model, int norm_flag, const float* d_ent, const float* d_ent_im,
                                          int64_t n_ent, int dim, float* d_ent_km, int64_t e_pad, float* d_ent_rows,
                                          void* stream) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (!d_ent || !d_ent_km || !d_ent_rows || n_ent <= 0 || dim <= 0 || e_pad < n_ent || e_pad % TE) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && !d_ent_im) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int threads = 256;
  hipLaunchKernelGGL(k_prep_entities, dim3((unsigned)((e_pad + threads - 1) / threads)), dim3(threads), 0, st,
                     model, norm_flag, d_ent, d_ent_im, n_ent, dim, plane_rows(dim), d_ent_km, e_pad, d_ent_rows);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_link_prepare_queries(int model, int norm_flag, const float* d_ent_rows, const float* d_rel,
                                         const float* d_rel_im, int64_t n_ent, int64_t n_rel, int dim,
                                         float phase_denom, const int64_t* d_qh, const int64_t* d_qr,
                                         const int64_t* d_qt, const int8_t* d_qmode, int64_t n_query,
                                         float* d_q_km, int64_t q_pad, int32_t* d_q_true, float* d_rel_work,
                                         void* stream) {
  if (!valid_model(model)) return MMRE_ERR_MODEL;
  if (!d_ent_rows || !d_rel || !d_qh || !d_qr || !d_qt || !d_qmode || !d_q_km || !d_q_true) return MMRE_ERR_ARG;
  if (n_query <= 0 || q_pad < n_query || q_pad % TQ || dim <= 0 || n_ent <= 0 || n_rel <= 0) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && !d_rel_im) return MMRE_ERR_ARG;
  if (model == MMRE_ROTATE && !(phase_denom != 0.0f)) return MMRE_ERR_ARG;
  const bool transe = model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2;
  if (transe && norm_flag && !d_rel_work) return MMRE_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int threads = 256;
  const float* rel = d_rel;
  if (transe && norm_flag) {
    hipLaunchKernelGGL(k_norm_rows, dim3((unsigned)((n_rel + threads - 1) / threads)), dim3(threads), 0, st, d_rel,
                       n_rel, dim, d_rel_work);
    MMRE_CHECK_LAUNCH();
    rel = d_rel_work;
  }
  const int kp = plane_rows(dim);
  hipLaunchKernelGGL(k_prep_queries, dim3((unsigned)((q_pad + threads - 1) / threads), (unsigned)kp), dim3(threads),
                     0, st, model, d_ent_rows, rel, d_rel_im, dim, kp, phase_denom, d_qh, d_qr, d_qt, d_qmode,
                     n_query, d_q_km, q_pad, d_q_true);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

template <int OP>
static int launch_aux(hipStream_t st, const float* ent_rows, int64_t n_ent, const float* q_km, int64_t q_pad, int kp,
                      const int32_t* qtrue, const int64_t* qr, const int8_t* qmode, int64_t n_query, int pk, float m,
                      float* thr, const int64_t* off, const int32_t* ids, const uint32_t* th, const uint32_t* tt,
                      int64_t tw, int32_t* counts) {
  const int threads = 256;
  hipLaunchKernelGGL((k_truth<OP>), dim3((unsigned)((n_query + threads - 1) / threads)), dim3(threads), 0, st,
                     ent_rows, q_km, q_pad, kp, qtrue, n_query, pk, m, thr);
  MMRE_CHECK_LAUNCH();
  if (off) {
    const unsigned blocks = (unsigned)(n_query < 16384 ? n_query : 16384);
    hipLaunchKernelGGL((k_filter_correct<OP>), dim3(blocks), dim3(64), 0, st, ent_rows, n_ent, q_km, q_pad, kp,
                       qtrue, qr, qmode, n_query, pk, m, thr, off, ids, th, tt, tw, counts);
    MMRE_CHECK_LAUNCH();
  }
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
  if (n_ent >= (int64_t)INT32_MAX) return MMRE_ERR_SHAPE;
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
  const int kp = plane_rows(dim);
  const int64_t tw = (n_ent + 31) / 32;
  MMRE_CHECK(hipMemsetAsync(d_counts, 0, sizeof(int32_t) * 4 * n_query, st));
#define MMRE_AUX(OPV) launch_aux<OPV>(st, d_ent_rows, n_ent, d_q_km, q_pad, kp, d_q_true, d_qr, d_qmode, n_query, \
                                      pred_kind, margin, d_truth, d_filt_off, d_filt_ids, d_type_head, d_type_tail, tw, d_counts)
  switch (op_of_model(model)) {
    case 0: return MMRE_AUX(0);
    case 1: return MMRE_AUX(1);
    case 2: return MMRE_AUX(2);
    case 3: return MMRE_AUX(3);
    default: return MMRE_AUX(4);
  }
#undef MMRE_AUX
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
#define MMRE_LV(OPV) launch_valu<OPV>(tc, store, st, d_ent_km, e_pad, n_ent, d_q_km, q_pad, n_query, kp, pred_kind, \
                                      margin, d_truth, d_q_true, d_qr, d_qmode, d_type_head, d_type_tail, tw, d_counts, d_scores)
    if (op == 0) return MMRE_LV(0);
    if (op == 1) return MMRE_LV(1);
    return MMRE_LV(2);
#undef MMRE_LV
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
