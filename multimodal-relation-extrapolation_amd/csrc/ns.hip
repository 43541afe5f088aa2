// ns.hip -- fused negative-sampling margin loss, forward and backward.
//
// Replaces, per training batch, the torch graph of OpenKE's
// strategy/NegativeSampling.forward (NegativeSampling.py:23-32) = model(data) in 'normal'
// mode (TransE.py:62-90, DistMult.py:43-64, ComplEx.py:20-40, RotatE.py:45-87) ->
// _get_positive_score / _get_negative_score -> MarginLoss (MarginLoss.py:24-28, with the
// detached self-adversarial weights of :19-22) + regul_rate * regularization
// (TransE.py:92-102), and the same assembly in the repo's module/NegativeSampling.py
// (:204-229, :307-314, module/loss.py:19-23).
//
// Layout: N = B * (1 + k) rows, positive b at row b, its negative j at row b + (j+1) B
// (Base.cpp:109-145). One wavefront per positive scores its 1 + k rows (lanes over the
// embedding dimension, shuffle reductions) and writes one partial loss; a single
// workgroup reduces the partials in a fixed order (bit-reproducible loss). No backward uses
// float atomics: every gradient contribution is a SLOT record filed in its table row's bucket
// (integer count atomics only) and one wave per table row sums its slots in slot order, so the
// gradient tables are bit-identical run to run (the fused paths below; the rows backward of
// mmre_score_rows_backward / mmre_ns_backward).
#include "mmre_common.h"
#include "sampler_openke.h"

namespace mmre {

constexpr int NS_WAVES = 4;  // positives per 256-thread workgroup
constexpr int NS_MAXK = 512;  // negatives per positive kept in LDS

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s);
  return v;
}

struct NSArgs {
  int model, norm_flag, use_model_margin, dim;
  float model_margin, phase_denom;
  const float *ent, *ent_im, *rel, *rel_im;
  const int64_t *h, *t, *r;
  int64_t B, K;  // positives, negatives per positive
  float loss_margin, adv_t, regul_rate;
};

// Raw score s of one row (before the model's margin transform) and, optionally, the
// accumulation of g * d(score)/d(embeddings) into gradient tables.
// TransE: s = |(h + r) - t|_p with optional F.normalize; forward returns m - s when the model
// has a margin. DistMult: sum h r t. ComplEx: sum of the four triple products. RotatE:
// forward = m - sum_k |h o r - t|.
__device__ float row_score(const NSArgs& A, int64_t row, int lane) {
  const int d = A.dim;
  const int64_t h = A.h[row], t = A.t[row], r = A.r[row];
  float acc = 0.0f;
  if (A.model == MMRE_TRANSE_L1 || A.model == MMRE_TRANSE_L2) {
    const float *hv = A.ent + h * d, *tv = A.ent + t * d, *rv = A.rel + r * d;
    float nh = 1.0f, nt = 1.0f, nr = 1.0f;
    if (A.norm_flag) {
      float a = 0.0f, b = 0.0f, c = 0.0f;
      for (int k = lane; k < d; k += kWave) { a += hv[k] * hv[k]; b += tv[k] * tv[k]; c += rv[k] * rv[k]; }
      nh = fmaxf(sqrtf(wave_sum(a)), 1e-12f);
      nt = fmaxf(sqrtf(wave_sum(b)), 1e-12f);
      nr = fmaxf(sqrtf(wave_sum(c)), 1e-12f);
    }
    for (int k = lane; k < d; k += kWave) {
      const float x = (hv[k] / nh + rv[k] / nr) - tv[k] / nt;
      acc += A.model == MMRE_TRANSE_L1 ? fabsf(x) : x * x;
    }
    acc = wave_sum(acc);
    if (A.model == MMRE_TRANSE_L2) acc = sqrtf(acc);
    return A.use_model_margin ? A.model_margin - acc : acc;
  } else if (A.model == MMRE_DISTMULT) {
    const float *hv = A.ent + h * d, *tv = A.ent + t * d, *rv = A.rel + r * d;
    for (int k = lane; k < d; k += kWave) acc += (hv[k] * rv[k]) * tv[k];
    return wave_sum(acc);
  } else if (A.model == MMRE_COMPLEX) {
    const float *hr = A.ent + h * d, *hi = A.ent_im + h * d, *tr = A.ent + t * d, *ti = A.ent_im + t * d;
    const float *rr = A.rel + r * d, *ri = A.rel_im + r * d;
    for (int k = lane; k < d; k += kWave)
      acc += hr[k] * tr[k] * rr[k] + hi[k] * ti[k] * rr[k] + hr[k] * ti[k] * ri[k] - hi[k] * tr[k] * ri[k];
    return wave_sum(acc);
  } else {
    const float *hv = A.ent + h * 2 * d, *tv = A.ent + t * 2 * d, *rv = A.rel + r * d;
    for (int k = lane; k < d; k += kWave) {
      float s, c;
      canon_sincos(rv[k] / A.phase_denom, &s, &c);
      const float re = hv[k] * c - hv[d + k] * s - tv[k];
      const float im = hv[k] * s + hv[d + k] * c - tv[d + k];
      acc += sqrtf(re * re + im * im);
    }
    return A.model_margin - wave_sum(acc);
  }
}

// sum of squares of the gathered raw rows (regularization, TransE.py:92-102)
__device__ void row_sq(const NSArgs& A, int64_t row, int lane, float* sq) {
  const int d = A.dim;
  const int64_t h = A.h[row], t = A.t[row], r = A.r[row];
  const int ew = A.model == MMRE_ROTATE ? 2 * d : d;
  float a = 0.0f, b = 0.0f, c = 0.0f, e = 0.0f, f = 0.0f, g = 0.0f;
  for (int k = lane; k < ew; k += kWave) {
    a += A.ent[h * ew + k] * A.ent[h * ew + k];
    b += A.ent[t * ew + k] * A.ent[t * ew + k];
  }
  for (int k = lane; k < d; k += kWave) c += A.rel[r * d + k] * A.rel[r * d + k];
  if (A.model == MMRE_COMPLEX) {
    for (int k = lane; k < d; k += kWave) {
      e += A.ent_im[h * d + k] * A.ent_im[h * d + k];
      f += A.ent_im[t * d + k] * A.ent_im[t * d + k];
      g += A.rel_im[r * d + k] * A.rel_im[r * d + k];
    }
  }
  sq[0] += a; sq[1] += b; sq[2] += c; sq[3] += e; sq[4] += f; sq[5] += g;
}

// per-positive hinge terms; returns (sum_j w_j x_j) and fills gcoef (dL/dscore scale) on request
__global__ __launch_bounds__(256) void k_ns_forward(NSArgs A, float* __restrict__ score, float* __restrict__ part,
                                                     int32_t* __restrict__ zero, int64_t n_zero) {
  __shared__ float s_n[NS_WAVES][NS_MAXK];
  // the fused path's bucket counts (+ overflow count) for the gradient call that follows
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; zero && i < n_zero;
       i += (int64_t)gridDim.x * blockDim.x)
    zero[i] = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * NS_WAVES + w;
  if (b >= A.B) return;  // whole wave exits together
  const float p = row_score(A, b, lane);
  if (lane == 0) score[b] = p;
  float sq[6] = {0, 0, 0, 0, 0, 0};
  if (A.regul_rate != 0.0f) row_sq(A, b, lane, sq);
  // negatives: hinge max(p - n, -m); self-adversarial weights softmax(-n * T) (detached)
  float mx = -INFINITY;
  for (int64_t j = 0; j < A.K; ++j) {
    const int64_t row = b + (j + 1) * A.B;
    const float n = row_score(A, row, lane);  // wave-uniform
    if (lane == 0) { score[row] = n; s_n[w][j] = n; }
    if (A.regul_rate != 0.0f) row_sq(A, row, lane, sq);
    if (A.adv_t > 0.0f) mx = fmaxf(mx, -n * A.adv_t);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  float loss = 0.0f;
  if (lane == 0) {
    if (A.adv_t > 0.0f) {
      float den = 0.0f;
      for (int64_t j = 0; j < A.K; ++j) den += expf(-s_n[w][j] * A.adv_t - mx);
      for (int64_t j = 0; j < A.K; ++j) {
        const float n = s_n[w][j];
        loss += expf(-n * A.adv_t - mx) / den * fmaxf(p - n, -A.loss_margin);
      }
    } else {
      for (int64_t j = 0; j < A.K; ++j) loss += fmaxf(p - s_n[w][j], -A.loss_margin);
    }
    part[b * 7] = loss;
  }
  for (int i = 0; i < 6; ++i) {
    const float v = A.regul_rate != 0.0f ? wave_sum(sq[i]) : 0.0f;
    if (lane == 0) part[b * 7 + 1 + i] = v;
  }
}

// Fixed-order reduction of the per-positive partials (bit-reproducible loss) by threads
// 0..255 of the workgroup (every thread of it must call: it synchronises): strided double sums
// per thread, xor-butterfly wave sums (a + b and b + a agree, so every lane holds the same
// total), the four wave totals in a fixed order; one barrier.
__device__ void ns_reduce_block(const NSArgs& A, const float* part, float* loss) {
  __shared__ double red[7][4];
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};
  const bool mine = threadIdx.x < 256;
  if (A.regul_rate != 0.0f) {
    for (int64_t b = threadIdx.x; mine && b < A.B; b += 256) {
#pragma unroll
      for (int i = 0; i < 7; ++i) acc[i] += part[b * 7 + i];
    }
  } else {  // only the hinge partials: eight positives' loads in flight per round trip
    for (int64_t b0 = threadIdx.x; mine && b0 < A.B; b0 += 256 * 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = b0 + 256 * u < A.B ? part[(b0 + 256 * u) * 7] : 0.0f;
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[0] += x[u];
    }
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) acc[i] += __shfl_xor(acc[i], s);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0 && w < 4)
    for (int i = 0; i < 7; ++i) red[i][w] = acc[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[7];
    for (int i = 0; i < 7; ++i) t[i] = (red[i][0] + red[i][1]) + (red[i][2] + red[i][3]);
    const double Bd = (double)A.B, Kd = (double)A.K;
    double l = A.adv_t > 0.0f ? t[0] / Bd : t[0] / (Bd * Kd);
    l += A.loss_margin;
    if (A.regul_rate != 0.0f) {
      const double N = Bd * (1.0 + Kd);
      const double d = (double)A.dim;
      const double ew = A.model == MMRE_ROTATE ? 2.0 * d : d;
      double reg;
      if (A.model == MMRE_COMPLEX)
        reg = (t[1] / (N * d) + t[4] / (N * d) + t[2] / (N * d) + t[5] / (N * d) + t[3] / (N * d) + t[6] / (N * d)) / 6.0;
      else
        reg = (t[1] / (N * ew) + t[2] / (N * ew) + t[3] / (N * d)) / 3.0;
      l += (double)A.regul_rate * reg;
    }
    loss[0] = (float)l;
  }
}

__global__ __launch_bounds__(256) void k_ns_reduce(NSArgs A, const float* __restrict__ part, float* __restrict__ loss) {
  ns_reduce_block(A, part, loss);
}

// ---------------------------------------------------------------------------------------
// TransE fast path (L1 / L2, with or without norm_flag; dim <= 512).
// One workgroup of NSW waves per positive: every wave loads the positive's h, r, t rows once
// into registers (element lane + 64 c in slot c: every load and every gradient atomic
// instruction covers 64 consecutive floats) with their norms;
// the negatives j = w, w + NSW, ... of the positive are spread over the waves. A negative
// shares the positive's relation and one of its entities (Base.cpp:111-124: head OR tail
// corruption), so per negative only the corrupted row is read and normalised -- the shared
// rows are the register copies (a row that shares nothing is read in full, so any
// [pos | neg_1 | ... | neg_k] batch is handled). The backward accumulates the gradients of
// the shared rows in registers across the positive's negatives and issues atomics only for
// corrupted rows plus one per shared row at the end: k + 3 row atomics per positive instead
// of 3 (k + 1). Per-row arithmetic is the generic path's: x = (h/|h| + r/|r|) - t/|t|.
// ---------------------------------------------------------------------------------------
constexpr int NSW = 4;  // waves per positive

__device__ __forceinline__ void wave_sum3(float& a, float& b, float& c) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    a += __shfl_xor(a, s);
    b += __shfl_xor(b, s);
    c += __shfl_xor(c, s);
  }
}

template <int NC>
struct Vec {
  float v[NC];  // element lane + 64 c of the row in v[c] (zero past the row's end)
};

template <int NC>
__device__ __forceinline__ void vload(Vec<NC>& o, const float* row, int d, int lane) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + c * kWave;
    o.v[c] = i < d ? row[i] : 0.0f;
  }
}

// Row `row` (wave-uniform) of a [*, d] table through a buffer resource sized to the row: the
// padding lanes (element >= d) read 0 and their stores are dropped by the hardware range check,
// so the fast path has no per-element bounds branches.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const float* table, int64_t row, int d) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(table + row * d), (short)0, d * 4, 0x00020000);
}

template <int NC>
__device__ __forceinline__ void vload_row(Vec<NC>& o, const float* table, int64_t row, int d, int lane) {
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(table, row, d);
#pragma unroll
  for (int c = 0; c < NC; ++c) o.v[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (lane + c * kWave) * 4, 0, 0));
}

template <int NC>
__device__ __forceinline__ void vstore_row(float* table, int64_t row, const Vec<NC>& v, int d, int lane) {
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(table, row, d);
#pragma unroll
  for (int c = 0; c < NC; ++c) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.v[c]), rs, (lane + c * kWave) * 4, 0, 0);
}

template <int NC>
__device__ __forceinline__ float vsq(const Vec<NC>& a) {
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < NC; ++c) s += a.v[c] * a.v[c];
  return s;
}

template <int NC>
__device__ __forceinline__ void vadd(Vec<NC>& a, const Vec<NC>& b, float s) {
#pragma unroll
  for (int c = 0; c < NC; ++c) a.v[c] += s * b.v[c];
}

// x = (h / nh + r / nr) - t / nt per element (the forward's association, TransE.py:55-58)
__device__ __forceinline__ float tx(float h, float r, float t, float nh, float nr, float nt) {
  return (h / nh + r / nr) - t / nt;
}

// |x|_1 or |x|_2^2 partial of this lane (padding elements are 0 - 0 = 0)
template <int NC, bool L2>
__device__ __forceinline__ float row_partial(const Vec<NC>& h, const Vec<NC>& r, const Vec<NC>& t, float nh, float nr,
                                             float nt) {
  float acc = 0.0f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float x = tx(h.v[c], r.v[c], t.v[c], nh, nr, nt);
    acc += L2 ? x * x : fabsf(x);
  }
  return acc;
}

// the per-row inputs of one wave: each of h, r, t is the positive's register copy or a row
// read for this row (with its squared norm)
template <int NC>
struct RowCtx {
  Vec<NC> h, r, t;
  float sh, sr, st;   // squared raw norms
  bool own_h, own_r, own_t;
};

// Split in two so that the loads of two rows are in flight before either is reduced.
template <int NC>
__device__ __forceinline__ void row_ctx_load(RowCtx<NC>& o, const NSArgs& A, int64_t row, int64_t ph, int64_t pr,
                                             int64_t pt, const RowCtx<NC>& P, int lane) {
  const int d = A.dim;
  const int64_t h = A.h[row], r = A.r[row], t = A.t[row];
  o.own_h = h == ph;
  o.own_r = r == pr;
  o.own_t = t == pt;
  o.sh = o.sr = o.st = 0.0f;
  if (o.own_h) o.h = P.h; else vload(o.h, A.ent + h * d, d, lane);
  if (o.own_r) o.r = P.r; else vload(o.r, A.rel + r * d, d, lane);
  if (o.own_t) o.t = P.t; else vload(o.t, A.ent + t * d, d, lane);
}

template <int NC>
__device__ __forceinline__ void row_ctx_norms(RowCtx<NC>& o, const RowCtx<NC>& P) {
  float a = o.own_h ? 0.f : vsq(o.h), b = o.own_r ? 0.f : vsq(o.r), c = o.own_t ? 0.f : vsq(o.t);
  if (!(o.own_h && o.own_r && o.own_t)) wave_sum3(a, b, c);
  o.sh = o.own_h ? P.sh : a;
  o.sr = o.own_r ? P.sr : b;
  o.st = o.own_t ? P.st : c;
}

__device__ __forceinline__ float norm_of(float sq, int norm_flag) { return norm_flag ? fmaxf(sqrtf(sq), 1e-12f) : 1.0f; }

template <int NC, bool L2>
__device__ __forceinline__ float row_fwd(const NSArgs& A, const RowCtx<NC>& R, int lane) {
  const float nh = norm_of(R.sh, A.norm_flag), nr = norm_of(R.sr, A.norm_flag), nt = norm_of(R.st, A.norm_flag);
  float acc = row_partial<NC, L2>(R.h, R.r, R.t, nh, nr, nt);
  acc = wave_sum(acc);
  if (L2) acc = sqrtf(acc);
  return A.use_model_margin ? A.model_margin - acc : acc;
}

template <int NC, bool L2>
__global__ __launch_bounds__(256) void k_ns_transe_forward(NSArgs A, float* __restrict__ score,
                                                           float* __restrict__ part) {
  __shared__ float s_n[NS_MAXK];
  __shared__ float s_sq[NSW][3];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = blockIdx.x;
  const int d = A.dim;
  const int64_t ph = A.h[b], pr = A.r[b], pt = A.t[b];
  RowCtx<NC> P;
  vload(P.h, A.ent + ph * d, d, lane);
  vload(P.r, A.rel + pr * d, d, lane);
  vload(P.t, A.ent + pt * d, d, lane);
  P.sh = vsq(P.h); P.sr = vsq(P.r); P.st = vsq(P.t);
  wave_sum3(P.sh, P.sr, P.st);
  P.own_h = P.own_r = P.own_t = true;
  const float p = row_fwd<NC, L2>(A, P, lane);
  float qh = 0.f, qt = 0.f, qr = 0.f;  // regularization: sums of squared raw rows handled by this wave
  if (w == 0) {
    if (lane == 0) score[b] = p;
    qh = P.sh; qt = P.st; qr = P.sr;
  }
  int64_t j = w;
  for (; j + NSW < A.K; j += 2 * NSW) {  // two negatives per step: both rows in flight together
    const int64_t row0 = b + (j + 1) * A.B, row1 = row0 + NSW * A.B;
    RowCtx<NC> R0, R1;
    row_ctx_load(R0, A, row0, ph, pr, pt, P, lane);
    row_ctx_load(R1, A, row1, ph, pr, pt, P, lane);
    row_ctx_norms(R0, P);
    row_ctx_norms(R1, P);
    const float n0 = row_fwd<NC, L2>(A, R0, lane);
    const float n1 = row_fwd<NC, L2>(A, R1, lane);
    if (lane == 0) { score[row0] = n0; s_n[j] = n0; score[row1] = n1; s_n[j + NSW] = n1; }
    qh += R0.sh + R1.sh; qt += R0.st + R1.st; qr += R0.sr + R1.sr;
  }
  if (j < A.K) {
    const int64_t row = b + (j + 1) * A.B;
    RowCtx<NC> R;
    row_ctx_load(R, A, row, ph, pr, pt, P, lane);
    row_ctx_norms(R, P);
    const float n = row_fwd<NC, L2>(A, R, lane);
    if (lane == 0) { score[row] = n; s_n[j] = n; }
    qh += R.sh; qt += R.st; qr += R.sr;
  }
  if (lane == 0) { s_sq[w][0] = qh; s_sq[w][1] = qt; s_sq[w][2] = qr; }
  __syncthreads();
  if (w != 0) return;
  // hinge max(p - n, -m) over the negatives, self-adversarial weights softmax(-n T) (detached)
  const float m = A.loss_margin;
  float loss = 0.0f;
  if (A.adv_t > 0.0f) {
    float mx = -INFINITY;
    for (int64_t j = lane; j < A.K; j += kWave) mx = fmaxf(mx, -s_n[j] * A.adv_t);
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
    float den = 0.0f, num = 0.0f;
    for (int64_t j = lane; j < A.K; j += kWave) {
      const float e = expf(-s_n[j] * A.adv_t - mx);
      den += e;
      num += e * fmaxf(p - s_n[j], -m);
    }
    wave_sum3(den, num, loss);
    loss = num / den;
  } else {
    for (int64_t j = lane; j < A.K; j += kWave) loss += fmaxf(p - s_n[j], -m);
    loss = wave_sum(loss);
  }
  if (lane == 0) {
    float a = 0.f, c = 0.f, e = 0.f;
    for (int i = 0; i < NSW; ++i) { a += s_sq[i][0]; c += s_sq[i][1]; e += s_sq[i][2]; }
    float* o = part + b * 7;
    o[0] = loss;
    o[1] = A.regul_rate != 0.0f ? a : 0.0f;
    o[2] = A.regul_rate != 0.0f ? c : 0.0f;
    o[3] = A.regul_rate != 0.0f ? e : 0.0f;
    o[4] = o[5] = o[6] = 0.0f;
  }
}

// ---------------------------------------------------------------------------------------
// Fused forward + row-owner gradient (TransE fast path, K <= NSW * NSF_MAXJ).
// The margin loss's d(loss)/d(score) of every row depends only on its own positive's scores
// (hinge indicator, self-adversarial softmax over the positive's negatives), so the
// workgroup that scores a positive also forms its gradient, in the normalised space, per unit
// upstream gradient: the rows are read ONCE (kept in registers between the scoring and the
// gradient pass) and the row norms come from a pre-pass. A negative shares the positive's
// relation and one of its entities (Base.cpp:111-124), so what it adds to the positive's own
// three rows is summed in registers across the negatives; per negative one row is left, the
// corrupted one.
// No float atomics anywhere: k_ns_transe_fused writes every contribution to a SLOT (its
// values + the table row it belongs to) and drops the slot's id into its row's BUCKET: the
// place is the return value of the row's integer count atomic (the bucket's CONTENT is fixed,
// its order is not); a bucket holds NS_BUCKET ids, further ones go to an overflow list of
// (row, slot) pairs. k_ns_row_owner -- one wave per table row -- takes its bucket's slots in
// increasing slot id (batch order, the same every run), sums them, maps the sum through the
// row's normalisation, adds the regularization term, scales by the upstream gradient and
// writes the row, every row (untouched ones as zeros): no fills, no scaling pass, no scan,
// bit-reproducible gradient tables.
// Slots of positive b start at b (3 + 3K): slot q < 3 is the positive's h / r / t (row 3b + q
// of `shared` holds its signed sum), slot 3 + 3j + q is negative j's h / r / t when that row
// is not shared with the positive (record bK + j of `rec` holds the negative's gx; a t slot
// takes -gx). Keys: entity id, n_ent + relation id, or the sentinel n_ent + n_rel (no slot).
// For L1 TransE a negative's gx is g sign(x) elementwise, so its record is |g| and two bit
// planes (x > 0, x < 0) -- 2 + 4 NC words instead of d floats (72 B instead of 800 at d 200);
// the row-owner pass rebuilds the same floats (|g| times +-1 is exact). L2 stores gx.
// ---------------------------------------------------------------------------------------
constexpr int NSF_MAXJ = 8;
constexpr int NS_BUCKET = 64;   // slot ids kept in a table row's own bucket (one wave's width)
constexpr int NS_BUCKET_HEAD = 16;  // bucket entries the owner reads with the count (128 B)
constexpr int NS_HUB = 512;     // a row with more slots than a bucket orders them in LDS up to this many
constexpr int NS_HUB_WG = 4;    // owner workgroups for the rows with more slots (HubOrder)

struct NSSlots {        // the row-owner gradient's workspace
  float* shared;        // 3 B rows of dim floats: the positives' own rows (TransE)
  float* rec;           // K B records of a negative's gx (ns_rec_words); other models: per slot, 2 d_pad floats
  int32_t* counts;      // per table row: its slots (zeroed every call)
  int64_t* bucket;      // per table row: NS_BUCKET entries (slot id << 32 | occurrences as float bits), arrival order
  int64_t* ovf;         // (row, entry) pairs past a full bucket
  int32_t* ovf_n;       // overflow pairs (zeroed every call)
  uint32_t sentinel;    // n_ent + n_rel: no slot
};

// The pipelined TransE training step (mmre_ns_step_openke_pipe): what the row owner of step i
// also does for step i + 1, so that step i + 1 is two launches (fused loss kernel, row owner)
// instead of three:
//  * the next batch's sampler workgroups (sa; blocks [block0, block0 + n_blocks) of the grid)
//    -- the sampler reads only the train index and its seeds, so it runs beside the gradient;
//  * the pre-pass of every row this step changes: a row's wave that wrote fma(-lr, g, v) also
//    writes its norm and (norm_flag) its normalised copy, the values k_ns_prepass computes from
//    the updated table (same arithmetic: sum of squares over c, wave_sum, sqrtf, x / max(n, eps)).
//    A row without slots keeps its parameters, so its norm and normalised copy stay current;
//  * the next step's slot counts (the other parity's array, + its overflow count) zeroed.
// Every step still samples one batch, scores it and updates the rows it touches; only the
// launch that sampled and re-normalised the (unchanged) rest of the table is gone.
struct NSNext {
  OpenKESamplerArgs sa;         // the next batch (n_blocks == 0: none)
  int64_t block0, n_blocks;     // its sampler workgroups in the row owner's grid
  int32_t* counts;              // the next step's slot counts [E + R] + overflow count (nullptr: none)
  float* nrm_e;                 // norms of the updated rows (nullptr: no pre-pass)
  float* nrm_r;
  float* ent_n;                 // norm_flag: the updated rows normalised (else nullptr)
  float* rel_n;
};

// slot id and its row's occurrences in the batch (the regularization weight) as one bucket entry:
// ordering entries orders the slot ids
__device__ __forceinline__ int64_t slot_entry(int64_t slot, float mult) {
  return (int64_t)(((uint64_t)slot << 32) | (uint64_t)__float_as_uint(mult));
}
__device__ __forceinline__ int64_t entry_slot(int64_t e) { return (int64_t)((uint64_t)e >> 32); }
__device__ __forceinline__ float entry_mult(int64_t e) { return __uint_as_float((uint32_t)(uint64_t)e); }

// a slot into its row's bucket (or the overflow list)
__device__ __forceinline__ void put_slot(const NSSlots& S, uint32_t key, int64_t slot, float mult) {
  const int p = atomicAdd(&S.counts[key], 1);
  const int64_t e = slot_entry(slot, mult);
  if (p < NS_BUCKET) {
    S.bucket[(int64_t)key * NS_BUCKET + p] = e;
  } else {
    const int o = atomicAdd(S.ovf_n, 1);
    S.ovf[2 * (int64_t)o] = (int64_t)key;
    S.ovf[2 * (int64_t)o + 1] = e;
  }
}

// words per negative record: gx itself (L2), or |g| + pad + NC (x > 0, x < 0) 64-bit masks (L1)
__host__ __device__ constexpr int ns_rec_words(int nc, bool l2, int d) { return l2 ? d : 2 + 4 * nc; }

template <int NC>
__device__ __forceinline__ void vstore(float* row, const Vec<NC>& v, int d, int lane) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + c * kWave;
    if (i < d) row[i] = v.v[c];
  }
}

// negative record idx <- gx = g sign(x) (L1: |g| and the sign planes of gx) or gx (L2)
template <int NC, bool L2>
__device__ __forceinline__ void store_rec(float* rec, int64_t idx, const Vec<NC>& gx, float g, int d, int lane) {
  if constexpr (L2) {
    vstore(rec + idx * d, gx, d, lane);
  } else {
    float* r = rec + idx * ns_rec_words(NC, false, d);
    uint64_t val = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {  // wave-uniform masks; lane 2c / 2c + 1 stores plane c's pair
      const uint64_t pm = __ballot(gx.v[c] > 0.0f), nm = __ballot(gx.v[c] < 0.0f);
      if (lane == 2 * c) val = pm;
      if (lane == 2 * c + 1) val = nm;
    }
    if (lane < 2 * NC) reinterpret_cast<uint64_t*>(r + 2)[lane] = val;
    if (lane == 0) { r[0] = fabsf(g); r[1] = 0.0f; }
  }
}

// a slot's contribution row: a shared sum row, or a negative's record decoded
template <int NC, bool L2>
__device__ __forceinline__ void load_slot(Vec<NC>& v, const float* __restrict__ shared, const float* __restrict__ rec,
                                          int64_t idx, bool neg, int d, int lane) {
  if (!neg) {
    vload_row(v, shared, idx, d, lane);
  } else if constexpr (L2) {
    vload_row(v, rec, idx, d, lane);
  } else {
    const float* r = rec + idx * ns_rec_words(NC, false, d);
    const float mag = r[0];
    const uint64_t* m = reinterpret_cast<const uint64_t*>(r + 2);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int sg = (int)((m[2 * c] >> lane) & 1ull) - (int)((m[2 * c + 1] >> lane) & 1ull);
      v.v[c] = mag * (float)sg;
    }
  }
}

// Pre-pass of the fused launch, one wave per row over the entity rows then the relation
// rows: the row's L2 norm (one scalar per row instead of a wave reduction per use), with
// norm_flag the normalised row itself, x / max(|x|, eps) (the fused kernel's operands, so it
// divides nothing), and the row's slot count zeroed (and the overflow count).
// (A last-workgroup loss reduction inside the fused kernel was tried instead of k_ns_reduce:
// its per-workgroup device-scope fence writes back the XCD's L2 each time, 0.12 -> 0.19 ms.)
__device__ __forceinline__ void ns_prepass_block(const float* __restrict__ ent, int64_t n_ent,
                                                 const float* __restrict__ rel, int64_t n_rel, int d,
                                                 float* __restrict__ nrm_e, float* __restrict__ nrm_r,
                                                 float* __restrict__ ent_n, float* __restrict__ rel_n,
                                                 int32_t* __restrict__ counts, int32_t* __restrict__ ovf_n,
                                                 int64_t block) {
  if (block == 0 && threadIdx.x == 0) ovf_n[0] = 0;  // no overflow pairs yet
  const int lane = threadIdx.x & 63;
  const int64_t row = block * 4 + (threadIdx.x >> 6);
  if (row >= n_ent + n_rel) return;
  if (lane == 0) counts[row] = 0;  // the row's slot bucket, for this call
  const bool is_ent = row < n_ent;
  const float* p = (is_ent ? ent : rel) + (is_ent ? row : row - n_ent) * d;
  float* o = ent_n ? (is_ent ? ent_n : rel_n) + (is_ent ? row : row - n_ent) * d : nullptr;
  float s = 0.0f;
  if (d <= 8 * kWave) {  // the fused path's rows (d <= 512): read once into registers
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int i = lane + c * kWave;
      v[c] = i < d ? p[i] : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) s += v[c] * v[c];  // same order as the strided loop below
    s = wave_sum(s);
    const float nr = sqrtf(s);
    if (lane == 0) (is_ent ? nrm_e : nrm_r)[is_ent ? row : row - n_ent] = nr;
    if (o) {
      const float cn = fmaxf(nr, 1e-12f);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int i = lane + c * kWave;
        if (i < d) o[i] = v[c] / cn;
      }
    }
    return;
  }
  for (int i = lane; i < d; i += kWave) s += p[i] * p[i];
  s = wave_sum(s);
  const float nr = sqrtf(s);
  if (lane == 0) (is_ent ? nrm_e : nrm_r)[is_ent ? row : row - n_ent] = nr;
  if (o) {
    const float cn = fmaxf(nr, 1e-12f);
    for (int i = lane; i < d; i += kWave) o[i] = p[i] / cn;
  }
}

__global__ __launch_bounds__(256) void k_ns_prepass(const float* __restrict__ ent, int64_t n_ent,
                                                    const float* __restrict__ rel, int64_t n_rel, int d,
                                                    float* __restrict__ nrm_e, float* __restrict__ nrm_r,
                                                    float* __restrict__ ent_n, float* __restrict__ rel_n,
                                                    int32_t* __restrict__ counts, int32_t* __restrict__ ovf_n) {
  ns_prepass_block(ent, n_ent, rel, n_rel, d, nrm_e, nrm_r, ent_n, rel_n, counts, ovf_n, blockIdx.x);
}

// First launch of the training step (mmre_ns_step_openke): the sampler's workgroups
// [0, n_sampler) and the pre-pass's after them, in ONE grid -- the two are independent (the
// pre-pass reads only the tables), so the pre-pass runs on the CUs the latency-bound sampler
// leaves idle instead of after it. The sampler's seed ticket counts its own workgroups only.
__global__ __launch_bounds__(256) void k_ns_step_prep(OpenKESamplerArgs sa, int64_t n_sampler,
                                                      const float* __restrict__ ent, int64_t n_ent,
                                                      const float* __restrict__ rel, int64_t n_rel, int d,
                                                      float* __restrict__ nrm_e, float* __restrict__ nrm_r,
                                                      float* __restrict__ ent_n, float* __restrict__ rel_n,
                                                      int32_t* __restrict__ counts, int32_t* __restrict__ ovf_n) {
  if ((int64_t)blockIdx.x < n_sampler) {
    sampler_openke_block(sa, blockIdx.x, n_sampler);
    return;
  }
  ns_prepass_block(ent, n_ent, rel, n_rel, d, nrm_e, nrm_r, ent_n, rel_n, counts, ovf_n,
                   (int64_t)blockIdx.x - n_sampler);
}

// lane src's 64-bit value as a wave-uniform (scalar) value; src must be wave-uniform
__device__ __forceinline__ int64_t readlane64u(int64_t v, int src) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, src);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)v >> 32), src);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <int NC>
__device__ __forceinline__ void vnorm(Vec<NC>& o, const Vec<NC>& v, float c) {
#pragma unroll
  for (int q = 0; q < NC; ++q) o.v[q] = v.v[q] / c;
}

// x of a row given the normalised positive rows and the normalised corrupted row (code 0: h,
// 1: t, 2: r, 3: none; 4: a row sharing fewer than two rows with its positive, whose x =
// (h + r) - t was built in cn when its rows arrived), |x|_1 or |x|_2^2 partial of this lane; x
// kept for the gradient
template <int NC, bool L2>
__device__ __forceinline__ float fused_x(Vec<NC>& x, const Vec<NC>& hn, const Vec<NC>& rn, const Vec<NC>& tn,
                                         const Vec<NC>& cn, int code) {
  float acc = 0.0f;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const float h = code == 0 ? cn.v[q] : hn.v[q];
    const float r = code == 2 ? cn.v[q] : rn.v[q];
    const float t = code == 1 ? cn.v[q] : tn.v[q];
    const float e = code == 4 ? cn.v[q] : (h + r) - t;
    x.v[q] = e;
    acc += L2 ? e * e : fabsf(e);
  }
  return acc;
}

// fused_x specialised on the (wave-uniform) code: the OpenKE shapes replace one row, so x is one
// or two operations per element instead of three selects and three operations. hr = h + r of
// the positive (the same rounding as (h + r) - t computes first). Same values as fused_x.
template <int NC, bool L2>
__device__ __forceinline__ float code_x(Vec<NC>& x, const Vec<NC>& hr, const Vec<NC>& hn, const Vec<NC>& rn,
                                        const Vec<NC>& tn, const Vec<NC>& cn, int code) {
  float acc = 0.0f;
  if (code == 1) {  // tail replaced
#pragma unroll
    for (int q = 0; q < NC; ++q) { x.v[q] = hr.v[q] - cn.v[q]; acc += L2 ? x.v[q] * x.v[q] : fabsf(x.v[q]); }
  } else if (code == 0) {  // head replaced
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      x.v[q] = (cn.v[q] + rn.v[q]) - tn.v[q];
      acc += L2 ? x.v[q] * x.v[q] : fabsf(x.v[q]);
    }
  } else if (code == 2) {  // relation replaced
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      x.v[q] = (hn.v[q] + cn.v[q]) - tn.v[q];
      acc += L2 ? x.v[q] * x.v[q] : fabsf(x.v[q]);
    }
  } else if (code == 4) {  // x built when the rows arrived
#pragma unroll
    for (int q = 0; q < NC; ++q) { x.v[q] = cn.v[q]; acc += L2 ? x.v[q] * x.v[q] : fabsf(x.v[q]); }
  } else {  // the positive's own rows
#pragma unroll
    for (int q = 0; q < NC; ++q) { x.v[q] = hr.v[q] - tn.v[q]; acc += L2 ? x.v[q] * x.v[q] : fabsf(x.v[q]); }
  }
  return acc;
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the wave as a wave-uniform value, without LDS: DPP butterflies inside each row of 16
// lanes (quad xor 1, quad xor 2, half-row mirror, row mirror: every lane ends with its row's
// sum; IEEE addition is commutative, so mirrored pairs agree bit for bit), then the four row
// sums in a fixed order. All 64 lanes must be active.
__device__ __forceinline__ float wave_sum_u(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// One positive's workgroup (k_ns_transe_fused). A negative of the OpenKE batch shape shares two
// of its positive's rows (Base.cpp:111-124): one corrupted row is read. Any other negative
// (a relation corruption sharing h and t is code 2; a copy of the positive code 3; a row
// sharing fewer than two rows, code 4) is handled in the same pass: code 4 builds its x =
// (h + r) - t in the corrupted-row registers as its rows arrive, and each of its rows that is
// not the positive's gets a slot of its own. Every operand is a normalised row of the pre-pass
// (norm_flag) or the table row itself.
template <int NC, bool L2, bool REG>
__device__ __forceinline__ void ns_fused_body(const NSArgs& A, const float* __restrict__ nrm_e,
                                              const float* __restrict__ nrm_r, float* __restrict__ score,
                                              float* __restrict__ part, const NSSlots& S, int64_t n_ent, int64_t b,
                                              const float* __restrict__ ent_n, const float* __restrict__ rel_n) {
  __shared__ float s_n[NSW * NSF_MAXJ];
  __shared__ float s_c[NSW * NSF_MAXJ];
  __shared__ float s_gp;
  __shared__ float s_sq[NSW][3];
  __shared__ float s_acc[NSW - 1][3][NC * kWave];
  __shared__ float s_occ[NSW][3];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int d = A.dim;
  const int64_t ph = A.h[b], pr = A.r[b], pt = A.t[b];
  // this wave's negatives j = w + NSW u, u < nj; lane u holds negative u's row ids
  const int nj = w < A.K ? (int)((A.K - w + NSW - 1) / NSW) : 0;
  int64_t my_h = 0, my_t = 0, my_r = 0;
  if (lane < nj) {
    const int64_t row = b + (w + NSW * (int64_t)lane + 1) * A.B;
    my_h = A.h[row]; my_t = A.t[row]; my_r = A.r[row];
  }
  // the rows as the model uses them: normalised by the pre-pass (norm_flag), else the tables
  Vec<NC> hn, rn, tn;
  vload_row(hn, ent_n, ph, d, lane);
  vload_row(rn, rel_n, pr, d, lane);
  vload_row(tn, ent_n, pt, d, lane);
  const float nph = nrm_e[ph], npr = nrm_r[pr], npt = nrm_e[pt];
  // issue every corrupted-row load of the wave before any arithmetic
  Vec<NC> C[NSF_MAXJ];
  float cnr[NSF_MAXJ];
  int code[NSF_MAXJ];
#pragma unroll
  for (int u = 0; u < NSF_MAXJ; ++u) {
    code[u] = 3;
    cnr[u] = 0.0f;
    if (u < nj) {
      const int64_t h = readlane64u(my_h, u), t = readlane64u(my_t, u), r = readlane64u(my_r, u);
      const bool oh = h == ph, ot = t == pt, orr = r == pr;
      if (orr && ot && !oh) { code[u] = 0; vload_row(C[u], ent_n, h, d, lane); cnr[u] = REG ? nrm_e[h] : 0.0f; }
      else if (orr && oh && !ot) { code[u] = 1; vload_row(C[u], ent_n, t, d, lane); cnr[u] = REG ? nrm_e[t] : 0.0f; }
      else if (oh && ot && !orr) { code[u] = 2; vload_row(C[u], rel_n, r, d, lane); cnr[u] = REG ? nrm_r[r] : 0.0f; }
      else if (!(oh && ot && orr)) {  // shares fewer than two rows: x = (h + r) - t, built here
        code[u] = 4;
        if (oh) C[u] = hn; else vload_row(C[u], ent_n, h, d, lane);
        Vec<NC> o;
        if (orr) o = rn; else vload_row(o, rel_n, r, d, lane);
#pragma unroll
        for (int q = 0; q < NC; ++q) C[u].v[q] = C[u].v[q] + o.v[q];
        if (ot) o = tn; else vload_row(o, ent_n, t, d, lane);
#pragma unroll
        for (int q = 0; q < NC; ++q) C[u].v[q] = C[u].v[q] - o.v[q];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < NSF_MAXJ; ++u) code[u] = __builtin_amdgcn_readfirstlane(code[u]);  // wave-uniform: scalar branches
  Vec<NC> x, hr;
#pragma unroll
  for (int q = 0; q < NC; ++q) hr.v[q] = hn.v[q] + rn.v[q];
  const float p_sum = wave_sum_u(code_x<NC, L2>(x, hr, hn, rn, tn, hn, 3));
  const float p_raw = L2 ? sqrtf(p_sum) : p_sum;
  const float p = A.use_model_margin ? A.model_margin - p_raw : p_raw;
  // every x is kept from here on (the positive's in px, negative u's in C[u]): the gradient pass
  // needs no row, so hn / rn / tn / hr die with the forward
  const Vec<NC> px = x;
  const float psh = nph * nph, psr = npr * npr, pst = npt * npt;
  float qh = 0.f, qt = 0.f, qr = 0.f;
  if (w == 0) {
    if (lane == 0) score[b] = p;
    qh = psh; qt = pst; qr = psr;
  }
  float sraw[NSF_MAXJ];
  // occurrences of the positive's own rows among this wave's rows (the positive itself in wave
  // 0): the regularization weights of its three slots, known before any gradient
  float oh = w == 0 ? 1.0f : 0.0f, orr = oh, ot = oh;
#pragma unroll
  for (int u = 0; u < NSF_MAXJ; ++u) {
    sraw[u] = 0.0f;
    if (u >= nj) continue;
    const int64_t j = w + NSW * u, row = b + (j + 1) * A.B;
    if (code[u] == 4) {
      oh += readlane64u(my_h, u) == ph ? 1.0f : 0.0f;
      orr += readlane64u(my_r, u) == pr ? 1.0f : 0.0f;
      ot += readlane64u(my_t, u) == pt ? 1.0f : 0.0f;
    } else {
      oh += code[u] != 0 ? 1.0f : 0.0f;
      orr += code[u] != 2 ? 1.0f : 0.0f;
      ot += code[u] != 1 ? 1.0f : 0.0f;
    }
    float sv = wave_sum_u(code_x<NC, L2>(x, hr, hn, rn, tn, C[u], code[u]));
    C[u] = x;
    if (L2) sv = sqrtf(sv);
    sraw[u] = sv;
    const float n = A.use_model_margin ? A.model_margin - sv : sv;
    if (code[u] == 4) {  // rare: its raw norms read here (the regularization's squared norms)
      const int64_t h = readlane64u(my_h, u), r = readlane64u(my_r, u), t = readlane64u(my_t, u);
      const float a = h == ph ? nph : nrm_e[h], c = r == pr ? npr : nrm_r[r], e = t == pt ? npt : nrm_e[t];
      qh += a * a; qr += c * c; qt += e * e;
    } else {
      const float sq = cnr[u] * cnr[u];
      qh += code[u] == 0 ? sq : psh;
      qt += code[u] == 1 ? sq : pst;
      qr += code[u] == 2 ? sq : psr;
    }
    if (lane == 0) { score[row] = n; s_n[j] = n; }
  }
  if (lane == 0) {
    s_sq[w][0] = qh; s_sq[w][1] = qt; s_sq[w][2] = qr;
    s_occ[w][0] = oh; s_occ[w][1] = orr; s_occ[w][2] = ot;
  }
  __syncthreads();
  if (w == 0) {  // loss partial and d(loss)/d(forward score) of every row, per unit upstream gradient
    const float m = A.loss_margin;
    const bool have = lane < A.K;
    const float nj_ = have ? s_n[lane] : 0.0f;
    float loss, gp;
    if (A.adv_t > 0.0f) {
      float mx = have ? -nj_ * A.adv_t : -INFINITY;
#pragma unroll
      for (int s = 32; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
      const float e = have ? expf(-nj_ * A.adv_t - mx) : 0.0f;
      float den = e, num = have ? e * fmaxf(p - nj_, -m) : 0.0f, z = 0.0f;
      wave_sum3(den, num, z);
      loss = num / den;
      const float x_ = p - nj_;
      const float ind = x_ > -m ? 1.0f : (x_ == -m ? 0.5f : 0.0f);
      const float c = have ? (e / den) / (float)A.B * ind : 0.0f;
      if (have) s_c[lane] = c;
      gp = wave_sum(c);
    } else {
      loss = wave_sum(have ? fmaxf(p - nj_, -m) : 0.0f);
      const float x_ = p - nj_;
      const float ind = x_ > -m ? 1.0f : (x_ == -m ? 0.5f : 0.0f);
      const float c = have ? ind / (float)(A.B * A.K) : 0.0f;
      if (have) s_c[lane] = c;
      gp = wave_sum(c);
    }
    if (lane == 0) {
      s_gp = gp;
      float a = 0.f, c2 = 0.f, e2 = 0.f;
      for (int i = 0; i < NSW; ++i) { a += s_sq[i][0]; c2 += s_sq[i][1]; e2 += s_sq[i][2]; }
      float* o = part + b * 7;
      o[0] = loss;
      o[1] = A.regul_rate != 0.0f ? a : 0.0f;
      o[2] = A.regul_rate != 0.0f ? c2 : 0.0f;
      o[3] = A.regul_rate != 0.0f ? e2 : 0.0f;
      o[4] = o[5] = o[6] = 0.0f;
    }
  }
  __syncthreads();
  // gradient pass (upstream gradient 1): contributions into slots
  const double N = (double)A.B * (1.0 + (double)A.K);
  const float reg = A.regul_rate != 0.0f ? (float)(A.regul_rate * 2.0 / (3.0 * N * d)) : 0.0f;
  const float sgn = A.use_model_margin ? -1.0f : 1.0f;
  const int64_t sb = b * (3 + 3 * A.K);     // this positive's first slot
  Vec<NC> Gh, Gr, Gt, gx;
#pragma unroll
  for (int q = 0; q < NC; ++q) Gh.v[q] = Gr.v[q] = Gt.v[q] = 0.0f;
  // the slots this wave files, one per lane: lane 3u + k negative u's row k (h, r, t) when that
  // row is not the positive's own; in wave 0 lanes 3 NSF_MAXJ + k the positive's own rows. The
  // bucket places come back from ONE batched atomic round trip per wave, issued before the
  // records are computed and stored.
  uint32_t my_key = S.sentinel;
  int64_t my_slot = 0;
  float my_mult = 1.0f;
  if (w == 0) {
    const int k = lane - 3 * NSF_MAXJ;
    if (k >= 0 && k < 3) {
      float kh = 0.f, kr = 0.f, kt = 0.f;
      for (int i = 0; i < NSW; ++i) { kh += s_occ[i][0]; kr += s_occ[i][1]; kt += s_occ[i][2]; }
      my_key = k == 0 ? (uint32_t)ph : (k == 1 ? (uint32_t)(n_ent + pr) : (uint32_t)pt);
      my_slot = sb + k;
      my_mult = k == 0 ? kh : (k == 1 ? kr : kt);
    }
  }
  bool active[NSF_MAXJ];
#pragma unroll
  for (int u = 0; u < NSF_MAXJ; ++u) {  // keys first (the hinge decides whether a negative adds anything)
    active[u] = false;
    if (u >= nj) continue;
    const int64_t j = w + NSW * u;
    if (s_c[j] == 0.0f && reg == 0.0f) continue;  // inactive hinge, no regularization: adds nothing
    active[u] = true;
    uint32_t kq0 = S.sentinel, kq1 = S.sentinel, kq2 = S.sentinel;
    if (code[u] == 0) kq0 = (uint32_t)readlane64u(my_h, u);
    else if (code[u] == 1) kq2 = (uint32_t)readlane64u(my_t, u);
    else if (code[u] == 2) kq1 = (uint32_t)(n_ent + readlane64u(my_r, u));
    else if (code[u] == 4) {
      const int64_t h = readlane64u(my_h, u), r = readlane64u(my_r, u), t = readlane64u(my_t, u);
      if (h != ph) kq0 = (uint32_t)h;
      if (r != pr) kq1 = (uint32_t)(n_ent + r);
      if (t != pt) kq2 = (uint32_t)t;
    }
    const int64_t sl = sb + 3 + 3 * j;
    if (lane == 3 * u) { my_key = kq0; my_slot = sl; }
    if (lane == 3 * u + 1) { my_key = kq1; my_slot = sl + 1; }
    if (lane == 3 * u + 2) { my_key = kq2; my_slot = sl + 2; }
  }
  const bool filing = my_key != S.sentinel;
  const int place = filing ? atomicAdd(&S.counts[my_key], 1) : 0;
  if (w == 0) {
    const float g = sgn * s_gp;
    // a lane whose x is all zero gets gv = 0 whichever way gs is taken
    const float gs = L2 ? (p_sum > 0.0f ? g / p_raw : 0.0f) : g;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const float gv = L2 ? gs * px.v[q] : (px.v[q] > 0.0f ? g : (px.v[q] < 0.0f ? -g : 0.0f));
      Gh.v[q] += gv; Gr.v[q] += gv; Gt.v[q] -= gv;
    }
  }
#pragma unroll
  for (int u = 0; u < NSF_MAXJ; ++u) {
    if (!active[u]) continue;
    const int64_t j = w + NSW * u;
    const float g = -sgn * s_c[j];
    bool own_h = code[u] != 0, own_r = code[u] != 2, own_t = code[u] != 1;
    if (code[u] == 4) {
      own_h = readlane64u(my_h, u) == ph;
      own_r = readlane64u(my_r, u) == pr;
      own_t = readlane64u(my_t, u) == pt;
    }
    const Vec<NC>& xu = C[u];  // its x, kept by the forward
    const float gs = L2 ? (sraw[u] > 0.0f ? g / sraw[u] : 0.0f) : g;
#pragma unroll
    for (int q = 0; q < NC; ++q) gx.v[q] = L2 ? gs * xu.v[q] : (xu.v[q] > 0.0f ? g : (xu.v[q] < 0.0f ? -g : 0.0f));
    if (own_h) vadd(Gh, gx, 1.0f);
    if (own_r) vadd(Gr, gx, 1.0f);
    if (own_t) vadd(Gt, gx, -1.0f);
    if (!(own_h && own_r && own_t)) store_rec<NC, L2>(S.rec, b * A.K + j, gx, L2 ? 0.0f : gs, d, lane);
  }
  if (filing) {  // the entries, at the places the atomic returned
    const int64_t e = slot_entry(my_slot, my_mult);
    if (place < NS_BUCKET) {
      S.bucket[(int64_t)my_key * NS_BUCKET + place] = e;
    } else {
      const int o = atomicAdd(S.ovf_n, 1);
      S.ovf[2 * (int64_t)o] = (int64_t)my_key;
      S.ovf[2 * (int64_t)o + 1] = e;
    }
  }
  if (w > 0) {
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      s_acc[w - 1][0][q * kWave + lane] = Gh.v[q];
      s_acc[w - 1][1][q * kWave + lane] = Gr.v[q];
      s_acc[w - 1][2][q * kWave + lane] = Gt.v[q];
    }
  }
  __syncthreads();
  if (w == 0) {  // the positive's own rows: one signed sum each, in the fixed wave order
    for (int i = 0; i < NSW - 1; ++i) {
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        Gh.v[q] += s_acc[i][0][q * kWave + lane];
        Gr.v[q] += s_acc[i][1][q * kWave + lane];
        Gt.v[q] += s_acc[i][2][q * kWave + lane];
      }
    }
    vstore_row(S.shared, 3 * b + 0, Gh, d, lane);
    vstore_row(S.shared, 3 * b + 1, Gr, d, lane);
    vstore_row(S.shared, 3 * b + 2, Gt, d, lane);
  }
}

// REG: the regularization's squared norms of the corrupted rows are gathered (regul_rate != 0);
// without it the instance holds no norms of them (fewer registers: 6 waves / SIMD)
template <int NC, bool L2, bool REG>
__global__ __launch_bounds__(256, NC > 4 ? 1 : (L2 ? 5 : 6)) void k_ns_transe_fused(NSArgs A, const float* __restrict__ nrm_e,
                                                         const float* __restrict__ nrm_r, float* __restrict__ score,
                                                         float* __restrict__ part, NSSlots S, int64_t n_ent,
                                                         const float* __restrict__ ent_n,
                                                         const float* __restrict__ rel_n) {
  ns_fused_body<NC, L2, REG>(A, nrm_e, nrm_r, score, part, S, n_ent, blockIdx.x, ent_n, rel_n);
}

__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const int64_t o = __shfl_xor(v, s);
    v = o < v ? o : v;
  }
  return v;
}

// The bucket entries of table row `row` (n = counts[row] of them) in increasing slot id, up
// to 64 at a time (next(take): lane u's entry = the next u-th smallest, INT64_MAX past take).
// `pre` is the lane's entry of the row's bucket, loaded together with the count.
//   n <= NS_BUCKET (nearly every row): ranked in registers -- lane l's rank = how many of the
//     bucket's entries are smaller -- and a ds_permute sends each entry to the lane of its rank;
//   NS_BUCKET < n <= NS_HUB (a hub row, e.g. a frequent relation): bucket + the row's overflow
//     pairs collected into the wave's LDS list and bitonic-sorted there.
// Rows with n > NS_HUB are not ordered by their wave: the owner kernels hand them to extra
// workgroups that order them cooperatively (HubOrder).
struct SlotOrder {
  const int64_t* ovf;
  int n_ovf, n, lane;
  int64_t row;
  int64_t* hub;      // this wave's LDS list (NS_HUB entries)
  int64_t pre;       // lane's bucket entry
  int64_t regs;      // n <= 64: lane u's ordered entry
  int pos;           // entries handed out so far

  __device__ void init() {
    pos = 0;
    if (n <= NS_BUCKET) {
      const int64_t mine = lane < n ? pre : INT64_MAX;
      int rank = 0;
      for (int m = 0; m < n; ++m) rank += readlane64u(mine, m) < mine;
      const int to = (lane < n ? rank : lane) * 4;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)(uint64_t)mine);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)((uint64_t)mine >> 32));
      regs = (int64_t)(((uint64_t)hi << 32) | lo);
      return;
    }
    hub[lane] = pre;  // a full bucket
    int m = NS_BUCKET;
    // the whole overflow list is scanned (every row's pairs past its bucket): eight 64-pair
    // groups' loads in flight per round, then their ballots in list order (one dependent load
    // per 64 pairs made a mid-size row's wave wait ~n_ovf / 64 round trips)
    const longlong2* o2 = reinterpret_cast<const longlong2*>(ovf);
    for (int base = 0; base < n_ovf; base += 8 * kWave) {
      longlong2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = base + u * kWave + lane;
        v[u] = e < n_ovf ? o2[e] : make_longlong2(-1, 0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool mine = v[u].x == row;
        const uint64_t mask = __ballot(mine);
        const int at = m + __popcll(mask & lanes_below(lane));
        if (mine && at < NS_HUB) hub[at] = v[u].y;
        m += __popcll(mask);
      }
    }
    int M = NS_BUCKET;
    while (M < n) M <<= 1;
    for (int i = n + lane; i < M; i += kWave) hub[i] = INT64_MAX;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int k = 2; k <= M; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = lane; i < M; i += kWave) {
          const int x = i ^ j;
          if (x > i) {
            const int64_t a = hub[i], b = hub[x];
            const bool up = (i & k) == 0;
            if ((a > b) == up) { hub[i] = b; hub[x] = a; }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
  }

  __device__ int64_t next(int& take) {
    take = (n - pos) < kWave ? (n - pos) : kWave;
    const int c0 = pos;
    pos += take;
    if (n <= NS_BUCKET) return regs;
    return lane < take ? hub[c0 + lane] : INT64_MAX;
  }
};

// Hub rows (n > NS_HUB slots: a relation shared by thousands of the batch's rows) are ordered by
// a whole workgroup in windows of slot ids: a histogram pass over the row's entries (bucket +
// its pairs in the overflow list) picks the widest window [lo, hi) holding at most HUB_CAP of
// them, a collect pass gathers those into LDS, a bitonic sort over 256 threads orders them,
// and next() hands them out 64 at a time; then the next window. Linear in the row's entries
// per window (the repeated wave minima it replaces were quadratic). Every member of the
// workgroup calls next() the same number of times (it synchronises); LDS: 4 KB of histogram +
// HUB_CAP entries, inside the owner kernels' 16-KB s_hub.
constexpr int HUB_BINS = 1024;
constexpr int HUB_CAP = 1024;
struct HubOrder {
  const int64_t* bucket;
  const int64_t* ovf;
  int n_ovf, n;
  int64_t row, n_slots;  // slot ids are < n_slots
  int32_t* hist;         // HUB_BINS counters
  int64_t* buf;          // HUB_CAP entries
  int32_t* s_cnt;        // LDS scalars: [0] collected, [1] bins taken
  int64_t lo;            // the next window starts at this slot id
  int wn, wi;            // entries in the window, handed out

  __device__ void init() { lo = 0; wn = wi = 0; }

  template <class F>
  __device__ __forceinline__ void for_entries(F&& f) {  // every entry of the row, any order
    const int tid = threadIdx.x;
    if (tid < NS_BUCKET) f(bucket[row * NS_BUCKET + tid]);
    // the overflow list holds every row's pairs past its bucket (thousands when a batch's
    // relations are skewed): 8 pairs' loads in flight per thread, not one dependent round trip
    // per 256 pairs (train_transe on the C2 test triples: row owner 65 us)
    const longlong2* o2 = reinterpret_cast<const longlong2*>(ovf);
#pragma unroll 8
    for (int e = tid; e < n_ovf; e += blockDim.x) {
      const longlong2 p = o2[e];
      if (p.x == row) f(p.y);
    }
  }

  __device__ void build() {
    const int tid = threadIdx.x;
    int64_t span = n_slots - lo;
    int64_t hi = n_slots;
    for (;;) {
      const int64_t binw = (span + HUB_BINS - 1) / HUB_BINS;
      __syncthreads();
      for (int i = tid; i < HUB_BINS; i += blockDim.x) hist[i] = 0;
      __syncthreads();
      for_entries([&](int64_t e) {
        const int64_t sl = entry_slot(e);
        if (sl >= lo && sl < lo + span) atomicAdd(&hist[(int)((sl - lo) / binw)], 1);
      });
      __syncthreads();
      if (tid < kWave) {  // wave 0: the longest run of leading bins holding <= HUB_CAP entries
        constexpr int PER = HUB_BINS / kWave;
        int loc = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) loc += hist[tid * PER + i];
        int inc = loc;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
          const int v = __shfl_up(inc, o);
          if (tid >= o) inc += v;
        }
        const int before = inc - loc;
        // the first lane whose run passes the cap finds the exact bin; all lanes within: every bin
        const uint64_t over = __ballot(inc > HUB_CAP);
        int taken = HUB_BINS;
        if (over) {
          const int L = __builtin_ctzll(over);
          if (tid == L) {
            int c = before, b = 0;
            while (b < PER && c + hist[tid * PER + b] <= HUB_CAP) c += hist[tid * PER + b++];
            s_cnt[1] = L * PER + b;
          }
        } else if (tid == 0) {
          s_cnt[1] = taken;
        }
      }
      __syncthreads();
      const int nb = s_cnt[1];
      if (nb > 0) {
        hi = nb == HUB_BINS ? lo + span : lo + (int64_t)nb * binw;
        break;
      }
      span = binw;  // the first bin alone holds more than HUB_CAP: narrow to it (binw >= 1 id -> <= 1 entry)
    }
    if (tid == 0) s_cnt[0] = 0;
    __syncthreads();
    for_entries([&](int64_t e) {
      const int64_t sl = entry_slot(e);
      if (sl >= lo && sl < hi) buf[atomicAdd(&s_cnt[0], 1)] = e;
    });
    __syncthreads();
    wn = s_cnt[0];
    int M = 2;
    while (M < wn) M <<= 1;
    for (int i = wn + tid; i < M; i += blockDim.x) buf[i] = INT64_MAX;
    __syncthreads();
    for (int k = 2; k <= M; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < M; i += blockDim.x) {
          const int x = i ^ j;
          if (x > i) {
            const int64_t a = buf[i], b = buf[x];
            const bool up = (i & k) == 0;
            if ((a > b) == up) { buf[i] = b; buf[x] = a; }
          }
        }
        __syncthreads();
      }
    }
    lo = hi;
    wi = 0;
  }

  __device__ int64_t next(int& take) {
    while (wi == wn) build();  // uniform over the workgroup (wn, wi come from LDS after a barrier)
    take = (wn - wi) < kWave ? (wn - wi) : kWave;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t e = lane < take ? buf[wi + lane] : INT64_MAX;
    wi += take;
    return e;
  }
};

// The hub rows of the table (n > NS_HUB), in row order, dealt round-robin to the kernel's
// n_hub_wg extra workgroups: hb-th of them calls f(row, n) for the rows k = hb, hb + n_hub_wg, ...
// (the whole workgroup together). The counts are scanned HUB_SCAN rows per pass, each thread
// loading HUB_SCAN / 256 consecutive counts at once (one round trip per pass, not one per 256
// rows: the per-256 scan serialised ~57 load latencies and two barriers each at C2 and kept the
// owner kernel alive for ~70 us); a pass's hub rows are found through one 16-bit mask per
// thread in LDS and four wave ballots.
constexpr int HUB_SCAN = 4096;
template <class F>
__device__ __forceinline__ void for_hub_rows(const int32_t* __restrict__ counts, int64_t n_rows, int hb, int n_hub_wg,
                                             uint16_t* s_bits, F&& f) {
  constexpr int PER = HUB_SCAN / 256;  // 16 consecutive rows per thread
  const int tid = threadIdx.x, lane = tid & 63;
  int64_t k = 0;
  for (int64_t base = 0; base < n_rows; base += HUB_SCAN) {
    const int64_t r0 = base + (int64_t)tid * PER;
    int c[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) c[i] = r0 + i < n_rows ? counts[r0 + i] : 0;  // all in flight together
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) bits |= (uint32_t)(c[i] > NS_HUB) << i;
    __syncthreads();  // the previous pass's readers of s_bits are done
    s_bits[tid] = (uint16_t)bits;
    __syncthreads();
    for (int q = 0; q < 4; ++q) {  // threads 64q .. 64q + 63, in order
      const uint32_t mine = s_bits[q * 64 + lane];
      uint64_t nz = __ballot(mine != 0u);
      while (nz) {
        const int t = __builtin_ctzll(nz);
        nz &= nz - 1;
        uint32_t m = s_bits[q * 64 + t];
        while (m) {
          const int i = __builtin_ctz(m);
          m &= m - 1u;
          if (k % n_hub_wg == hb) {
            const int64_t r = base + (int64_t)(q * 64 + t) * PER + i;
            f(r, counts[r]);
          }
          ++k;
        }
      }
    }
  }
}

// One wave per table row (entities, then relations): the row's slots summed in batch order,
// d(loss)/d(raw row) = (dy - y (y . dy)) / |v| with y = v / max(|v|, eps) when the model
// normalises (dy / eps below eps), + reg * (occurrences) * v, times the upstream gradient;
// written to every row of the gradient table. sgd_lr > 0 (the optimizer's plain SGD step fused
// in, mmre_ns_fused_grad_sgd): the row's parameters also become fma(-lr, g, v), torch's SGD
// arithmetic; rows without slots keep theirs (p - lr * 0 = p).
// One table row's gradient from its ordered slots (Ord: SlotOrder for a wave, HubOrder for a
// workgroup; with a HubOrder every wave of the workgroup calls this for the same row -- next()
// synchronises -- and only the `active` one loads, sums and writes). v / nv: the row and its norm.
template <int NC, bool L2, class Ord>
__device__ __forceinline__ void transe_owner_row(Ord& ord, bool active, int64_t row, int n, const Vec<NC>& v,
                                                 float nv, int64_t n_ent, int d, int norm_flag, float reg,
                                                 const float* __restrict__ shared, const float* __restrict__ rec,
                                                 int64_t K, const float* __restrict__ grad_loss, float* gent,
                                                 float* grel, float sgd_lr, float* pent, float* prel,
                                                 const NSNext& nx) {
  const int lane = threadIdx.x & 63;
  const bool is_ent = row < n_ent;
  const int64_t id = is_ent ? row : row - n_ent;
  const int64_t spp = 3 + 3 * K;
  Vec<NC> dy;
#pragma unroll
  for (int c = 0; c < NC; ++c) dy.v[c] = 0.0f;
  float cnt = 0.0f;
  for (int c0 = 0; c0 < n;) {
    int take;
    const int64_t ordered = ord.next(take);
    c0 += take;
    if (!active) continue;
    int64_t src = 0;  // shared row index, or -(record index + 1) for a negative's record
    float sg = 0.0f, m = 0.0f;
    if (lane < take) {  // lane u decodes its slot: where its contribution lives, and its sign
      const int64_t sl = entry_slot(ordered);
      const int64_t b = sl / spp, t = sl - b * spp;
      if (t < 3) { src = 3 * b + t; sg = 1.0f; }
      else { const int64_t jq = t - 3; src = -(b * K + jq / 3) - 1; sg = jq % 3 == 2 ? -1.0f : 1.0f; }
      m = entry_mult(ordered);
    }
    cnt += wave_sum(m);  // integer-valued: exact in any order
    int u = 0;
    for (; u + 4 <= take; u += 4) {  // four slots in flight, added in slot order
      Vec<NC> v0, v1, v2, v3;
      const int64_t s0 = readlane64u(src, u), s1 = readlane64u(src, u + 1);
      const int64_t s2 = readlane64u(src, u + 2), s3 = readlane64u(src, u + 3);
      load_slot<NC, L2>(v0, shared, rec, s0 < 0 ? -s0 - 1 : s0, s0 < 0, d, lane);
      load_slot<NC, L2>(v1, shared, rec, s1 < 0 ? -s1 - 1 : s1, s1 < 0, d, lane);
      load_slot<NC, L2>(v2, shared, rec, s2 < 0 ? -s2 - 1 : s2, s2 < 0, d, lane);
      load_slot<NC, L2>(v3, shared, rec, s3 < 0 ? -s3 - 1 : s3, s3 < 0, d, lane);
      const float g0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sg), u));
      const float g1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sg), u + 1));
      const float g2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sg), u + 2));
      const float g3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sg), u + 3));
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        dy.v[c] += g0 * v0.v[c];
        dy.v[c] += g1 * v1.v[c];
        dy.v[c] += g2 * v2.v[c];
        dy.v[c] += g3 * v3.v[c];
      }
    }
    for (; u < take; ++u) {
      Vec<NC> v0;
      const int64_t s0 = readlane64u(src, u);
      load_slot<NC, L2>(v0, shared, rec, s0 < 0 ? -s0 - 1 : s0, s0 < 0, d, lane);
      const float g0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sg), u));
#pragma unroll
      for (int c = 0; c < NC; ++c) dy.v[c] += g0 * v0.v[c];
    }
  }
  if (!active) return;
  const float G = grad_loss ? grad_loss[0] : 1.0f;
  const float rr = reg * cnt;
  if (norm_flag) {
    const float cv = fmaxf(nv, 1e-12f);
    float dot = 0.0f;
#pragma unroll
    for (int c = 0; c < NC; ++c) dot += (v.v[c] / cv) * dy.v[c];
    dot = wave_sum(dot);
    const float scale = nv > 1e-12f ? 1.0f / nv : 1.0f / 1e-12f;
    const float proj = nv > 1e-12f ? dot : 0.0f;
#pragma unroll
    for (int c = 0; c < NC; ++c) dy.v[c] = ((dy.v[c] - (v.v[c] / cv) * proj) * scale + rr * v.v[c]) * G;
  } else {
#pragma unroll
    for (int c = 0; c < NC; ++c) dy.v[c] = (dy.v[c] + rr * v.v[c]) * G;
  }
  float* o = (is_ent ? gent : grel) + id * d;
  vstore_row(o, 0, dy, d, lane);
  if (sgd_lr != 0.0f) {
    Vec<NC> p;
#pragma unroll
    for (int c = 0; c < NC; ++c) p.v[c] = __builtin_fmaf(-sgd_lr, dy.v[c], v.v[c]);
    vstore_row(is_ent ? pent : prel, id, p, d, lane);
    if (nx.nrm_e) {  // the next step's pre-pass of this row (ns_prepass_block's arithmetic)
      const float nr = sqrtf(wave_sum(vsq(p)));
      if (lane == 0) (is_ent ? nx.nrm_e : nx.nrm_r)[id] = nr;
      if (nx.ent_n) {
        const float cn = fmaxf(nr, 1e-12f);
        Vec<NC> o;
#pragma unroll
        for (int c = 0; c < NC; ++c) o.v[c] = p.v[c] / cn;
        vstore_row(is_ent ? nx.ent_n : nx.rel_n, id, o, d, lane);
      }
    }
  }
}

// The hub workgroups' LDS view of an owner kernel's s_hub (16 KB): histogram, then entries.
__device__ __forceinline__ HubOrder hub_order(int64_t (*s_hub)[NS_HUB], int32_t* s_hc, const int64_t* bucket,
                                              const int64_t* ovf, int n_ovf, int n, int64_t row, int64_t n_slots) {
  int64_t* flat = &s_hub[0][0];
  static_assert(4 * NS_HUB >= HUB_BINS / 2 + HUB_CAP, "hub LDS");
  HubOrder o{bucket, ovf, n_ovf, n, row, n_slots, reinterpret_cast<int32_t*>(flat), flat + HUB_BINS / 2, s_hc, 0, 0, 0};
  o.init();
  return o;
}

// One wave per table row (entities, then relations): the row's slots summed in batch order,
// d(loss)/d(raw row) = (dy - y (y . dy)) / |v| with y = v / max(|v|, eps) when the model
// normalises (dy / eps below eps), + reg * (occurrences) * v, times the upstream gradient;
// written to every row of the gradient table. sgd_lr > 0 (the optimizer's plain SGD step fused
// in, mmre_ns_fused_grad_sgd): the row's parameters also become fma(-lr, g, v), torch's SGD
// arithmetic; rows without slots keep theirs (p - lr * 0 = p). Rows with more than NS_HUB slots
// go to the first n_hub_wg workgroups (HubOrder); rows start at workgroup row_block0. With SGD the parameter tables
// ent / rel are also pent / prel (read, then written, by the row's own wave): not __restrict__.
template <int NC, bool L2>
__global__ __launch_bounds__(256, NC > 4 ? 5 : 7) void k_ns_row_owner(const float* ent, const float* rel,
                                                      int64_t n_ent, int64_t n_rel, int d, int norm_flag, float reg,
                                                      const float* nrm_e, const float* nrm_r,
                                                      const float* __restrict__ shared, const float* __restrict__ rec,
                                                      const int32_t* __restrict__ counts,
                                                      const int64_t* __restrict__ bucket, const int64_t* __restrict__ ovf,
                                                      const int32_t* __restrict__ ovf_n, int64_t K,
                                                      const float* __restrict__ grad_loss, float* __restrict__ gent,
                                                      float* __restrict__ grel, float sgd_lr, float* pent,
                                                      float* prel, NSArgs RA, const float* __restrict__ part,
                                                      float* __restrict__ loss, int64_t reduce_block,
                                                      int64_t row_block0, int n_hub_wg, int64_t n_slots, NSNext nx) {
  __shared__ int64_t s_hub[4][NS_HUB];
  __shared__ uint16_t s_bits[256];
  __shared__ int32_t s_hc[2];
  if ((int64_t)blockIdx.x == reduce_block) {  // the training step's loss (mmre_ns_step_openke): one extra workgroup
    ns_reduce_block(RA, part, loss);
    return;
  }
  if ((int64_t)blockIdx.x >= nx.block0 && (int64_t)blockIdx.x < nx.block0 + nx.n_blocks) {  // the next batch
    sampler_openke_block(nx.sa, (int64_t)blockIdx.x - nx.block0, nx.n_blocks);
    return;
  }
  const int lane = threadIdx.x & 63;
  if ((int64_t)blockIdx.x < n_hub_wg) {  // hub rows: the first n_hub_wg workgroups (they start first)
    for_hub_rows(counts, n_ent + n_rel, (int)blockIdx.x, n_hub_wg, s_bits,
                 [&](int64_t row, int n) {
                   const bool is_ent = row < n_ent;
                   const int64_t id = is_ent ? row : row - n_ent;
                   Vec<NC> v;
                   vload_row(v, is_ent ? ent : rel, id, d, lane);
                   const float nv = (is_ent ? nrm_e : nrm_r)[id];
                   HubOrder ord = hub_order(s_hub, s_hc, bucket, ovf, ovf_n[0], n, row, n_slots);
                   transe_owner_row<NC, L2>(ord, threadIdx.x < 64, row, n, v, nv, n_ent, d, norm_flag, reg, shared,
                                            rec, K, grad_loss, gent, grel, sgd_lr, pent, prel, nx);
                 });
    return;
  }
  const int64_t row = ((int64_t)blockIdx.x - row_block0) * 4 + (threadIdx.x >> 6);
  if (row >= n_ent + n_rel) return;  // wave-uniform
  if (nx.counts && (threadIdx.x & 63) == 0) {  // the next step's slot counts (the other array)
    nx.counts[row] = 0;
    if (row == 0) nx.counts[n_ent + n_rel] = 0;  // its overflow count
  }
  const bool is_ent = row < n_ent;
  const int64_t id = is_ent ? row : row - n_ent;
  // the count, the bucket's first entries, the row itself and its norm: one round trip, all in
  // flight together. Entity rows read NS_BUCKET_HEAD entries (one 128-B line: every slot of
  // nearly every entity row) and the rest only when they hold more (only the live ones);
  // relation rows -- few, and the kernel's longest chains -- read the whole bucket at once.
  const int n = counts[row];
  const int head = is_ent ? NS_BUCKET_HEAD : NS_BUCKET;
  int64_t pre = lane < head ? bucket[row * NS_BUCKET + lane] : 0;
  Vec<NC> v;
  vload_row(v, is_ent ? ent : rel, id, d, lane);
  const float nv = (is_ent ? nrm_e : nrm_r)[id];
  if (n > NS_HUB) return;  // a hub workgroup's row
  if (n > head && lane >= head && lane < n) pre = bucket[row * NS_BUCKET + lane];
  if (n == 0) {  // not in the batch: zero gradient (and an unchanged parameter row)
    Vec<NC> z;
#pragma unroll
    for (int c = 0; c < NC; ++c) z.v[c] = 0.0f;
    vstore_row((is_ent ? gent : grel) + id * d, 0, z, d, lane);
    return;
  }
  SlotOrder ord{ovf, n > NS_BUCKET ? ovf_n[0] : 0, n, lane, row, s_hub[threadIdx.x >> 6], pre, 0, 0};
  ord.init();
  transe_owner_row<NC, L2>(ord, true, row, n, v, nv, n_ent, d, norm_flag, reg, shared, rec, K, grad_loss, gent, grel,
                           sgd_lr, pent, prel, nx);
}

// ---------------------------------------------------------------------------------------
// Row-owner gradient for DistMult / ComplEx / RotatE: the same slots and buckets, no float
// atomics, bit-reproducible gradient tables. The forward is k_ns_forward + k_ns_reduce (which
// also zeroes the bucket counts); the gradient is k_ns_gen_slots + k_ns_gen_owner.
// A row is two halves of d floats (element lane + 64 c in slot c of each half): DistMult the
// row alone; ComplEx (re, im) -- entity rows from ent / ent_im, relation rows from rel /
// rel_im; RotatE entity rows (first d, last d) of the 2d row, relation rows the phase row.
// ---------------------------------------------------------------------------------------
template <int NC>
struct Row2 {
  Vec<NC> a, b;
};

template <int NC>
__device__ __forceinline__ void vzero(Vec<NC>& o) {
#pragma unroll
  for (int c = 0; c < NC; ++c) o.v[c] = 0.0f;
}

template <int NC>
__device__ __forceinline__ void gen_load(Row2<NC>& o, const NSArgs& A, bool is_ent, int64_t id, int lane) {
  const int d = A.dim;
  if (is_ent) {  // row id (wave-uniform) through row-sized buffer resources: no per-element bounds
    if (A.model == MMRE_COMPLEX) { vload_row(o.a, A.ent, id, d, lane); vload_row(o.b, A.ent_im, id, d, lane); }
    else if (A.model == MMRE_ROTATE) { vload_row(o.a, A.ent, 2 * id, d, lane); vload_row(o.b, A.ent, 2 * id + 1, d, lane); }
    else { vload_row(o.a, A.ent, id, d, lane); vzero(o.b); }
  } else {
    vload_row(o.a, A.rel, id, d, lane);
    if (A.model == MMRE_COMPLEX) vload_row(o.b, A.rel_im, id, d, lane); else vzero(o.b);
  }
}

// g * d(forward score)/d(h, r, t) of one row (the per-element formulas of row_backward).
// RotatE: psn / pcs, when given, are canon_sincos(R / phase_denom) already computed (the
// positive's relation, shared by its entity-corrupted negatives): the same values.
template <int NC>
__device__ __forceinline__ void gen_row_grad(const NSArgs& A, const Row2<NC>& H, const Row2<NC>& R,
                                             const Row2<NC>& T, float g, Row2<NC>& dH, Row2<NC>& dR, Row2<NC>& dT,
                                             const Vec<NC>* psn = nullptr, const Vec<NC>* pcs = nullptr) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (A.model == MMRE_DISTMULT) {
      dH.a.v[c] = g * R.a.v[c] * T.a.v[c];
      dT.a.v[c] = g * H.a.v[c] * R.a.v[c];
      dR.a.v[c] = g * H.a.v[c] * T.a.v[c];
      dH.b.v[c] = dT.b.v[c] = dR.b.v[c] = 0.0f;
    } else if (A.model == MMRE_COMPLEX) {
      const float hr = H.a.v[c], hi = H.b.v[c], tr = T.a.v[c], ti = T.b.v[c], rr = R.a.v[c], ri = R.b.v[c];
      dH.a.v[c] = g * (tr * rr + ti * ri);
      dH.b.v[c] = g * (ti * rr - tr * ri);
      dT.a.v[c] = g * (hr * rr - hi * ri);
      dT.b.v[c] = g * (hi * rr + hr * ri);
      dR.a.v[c] = g * (hr * tr + hi * ti);
      dR.b.v[c] = g * (hr * ti - hi * tr);
    } else {  // RotatE, forward = m - sum_k rho_k
      float sn, cs;
      if (psn) { sn = psn->v[c]; cs = pcs->v[c]; }
      else canon_sincos(R.a.v[c] / A.phase_denom, &sn, &cs);
      const float hre = H.a.v[c], him = H.b.v[c];
      const float re = hre * cs - him * sn - T.a.v[c];
      const float im = hre * sn + him * cs - T.b.v[c];
      const float rho = sqrtf(re * re + im * im);
      const float ga = rho > 0.0f ? -g * re / rho : 0.0f;
      const float gb = rho > 0.0f ? -g * im / rho : 0.0f;
      dH.a.v[c] = ga * cs + gb * sn;
      dH.b.v[c] = -ga * sn + gb * cs;
      dT.a.v[c] = -ga;
      dT.b.v[c] = -gb;
      dR.a.v[c] = (ga * (-hre * sn - him * cs) + gb * (hre * cs - him * sn)) / A.phase_denom;
      dR.b.v[c] = 0.0f;
    }
  }
}

template <int NC>
__device__ __forceinline__ void row2_add(Row2<NC>& a, const Row2<NC>& b) {
#pragma unroll
  for (int c = 0; c < NC; ++c) { a.a.v[c] += b.a.v[c]; a.b.v[c] += b.b.v[c]; }
}

// record of slot sl: the halves of a row gradient, d floats each, back to back (stride 2 d for
// the two-half models -- ComplEx, RotatE -- d for DistMult; RotatE relation rows keep their
// single half). Rows move through row-sized buffer resources (no padding lanes stored).
template <int NC>
__device__ __forceinline__ void rec_store(float* rec, int64_t sl, int d, bool stride2, bool two, const Row2<NC>& r,
                                          int lane) {
  float* o = rec + sl * (stride2 ? 2 * (int64_t)d : (int64_t)d);
  vstore_row(o, 0, r.a, d, lane);
  if (two) vstore_row(o + d, 0, r.b, d, lane);
}

template <int NC>
__device__ __forceinline__ void rec_load(Row2<NC>& r, const float* rec, int64_t sl, int d, bool stride2, bool two,
                                         int lane) {
  const float* o = rec + sl * (stride2 ? 2 * (int64_t)d : (int64_t)d);
  vload_row(r.a, o, 0, d, lane);
  if (two) vload_row(r.b, o + d, 0, d, lane);
  else vzero(r.b);
}

// The corrupted row of a negative of the OpenKE shapes (Base.cpp:111-145): code 0 head, 1 tail,
// 2 relation replaced (one row differs from its positive's), 3 the positive itself, 4 anything
// else (handled by the per-row generic code).
__device__ __forceinline__ int neg_code(int64_t h, int64_t r, int64_t t, int64_t ph, int64_t pr, int64_t pt) {
  const bool oh = h == ph, orr = r == pr, ot = t == pt;
  if (orr && ot && !oh) return 0;
  if (orr && oh && !ot) return 1;
  if (oh && ot && !orr) return 2;
  if (oh && ot && orr) return 3;
  return 4;
}

// row_score of DistMult / ComplEx / RotatE on rows already in registers (same per-element
// expressions, elements in the same lane + 64 c order, padding elements adding +0: the same
// floats bit for bit). RotatE: sn / cs of the relation row (canon_sincos(r / phase_denom)).
template <int NC>
__device__ __forceinline__ float gen_score(const NSArgs& A, const Row2<NC>& H, const Row2<NC>& R, const Row2<NC>& T,
                                           const Vec<NC>& sn, const Vec<NC>& cs) {
  float acc = 0.0f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (A.model == MMRE_DISTMULT) {
      acc += (H.a.v[c] * R.a.v[c]) * T.a.v[c];
    } else if (A.model == MMRE_COMPLEX) {
      const float hr = H.a.v[c], hi = H.b.v[c], tr = T.a.v[c], ti = T.b.v[c], rr = R.a.v[c], ri = R.b.v[c];
      acc += hr * tr * rr + hi * ti * rr + hr * ti * ri - hi * tr * ri;
    } else {
      const float re = H.a.v[c] * cs.v[c] - H.b.v[c] * sn.v[c] - T.a.v[c];
      const float im = H.a.v[c] * sn.v[c] + H.b.v[c] * cs.v[c] - T.b.v[c];
      acc += sqrtf(re * re + im * im);
    }
  }
  acc = wave_sum(acc);
  return A.model == MMRE_ROTATE ? A.model_margin - acc : acc;
}

template <int NC>
__device__ __forceinline__ void rot_sincos(const NSArgs& A, const Row2<NC>& R, Vec<NC>& sn, Vec<NC>& cs) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (A.model == MMRE_ROTATE) canon_sincos(R.a.v[c] / A.phase_denom, &sn.v[c], &cs.v[c]);
    else sn.v[c] = cs.v[c] = 0.0f;
  }
}

constexpr int NSG = 4;  // negatives whose rows are in flight together (generic models)

// Forward of the fused path for DistMult / ComplEx / RotatE (k_ns_forward's outputs: scores,
// per-positive partials, zeroed bucket counts), one wave per positive: the positive's rows stay
// in registers (RotatE: with its relation's sin / cos), the negatives' ids are read lane-parallel
// and NSG corrupted rows are loaded together -- an OpenKE negative differs from its positive in
// one row -- instead of one negative's three rows per dependent round trip.
template <int NC, int MODEL>
__global__ __launch_bounds__(256) void k_ns_gen_forward(NSArgs A_, float* __restrict__ score, float* __restrict__ part,
                                                        int32_t* __restrict__ zero, int64_t n_zero) {
  NSArgs A = A_;
  A.model = MODEL;  // compile-time model: the other models' registers and branches fold away
  // SPLIT (DistMult): one workgroup per positive, its negatives split over the waves; the
  // two-half models keep one wave per positive (their per-wave positive rows, sin / cos and
  // gradient make the split's redundant work cost more than its parallelism gains)
  constexpr bool SPLIT = MODEL == MMRE_DISTMULT;
  __shared__ float s_n[SPLIT ? NS_MAXK : NS_WAVES * NS_MAXK];  // the negative scores (loss)
  __shared__ float s_sq[NS_WAVES][6], s_mx[NS_WAVES];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; zero && i < n_zero;
       i += (int64_t)gridDim.x * blockDim.x)
    zero[i] = 0;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b = SPLIT ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * NS_WAVES + w;
  if (b >= A.B) return;  // workgroup- (SPLIT) or wave-uniform
  float* sn = s_n + (SPLIT ? 0 : w * NS_MAXK);
  const bool lead = SPLIT ? w == 0 : true;  // the wave that owns the positive's own terms
  const int64_t ph = A.h[b], pr = A.r[b], pt = A.t[b];
  Row2<NC> H, R, T;
  gen_load(H, A, true, ph, lane);
  gen_load(R, A, false, pr, lane);
  gen_load(T, A, true, pt, lane);
  Vec<NC> psn, pcs;
  rot_sincos(A, R, psn, pcs);
  const float p = gen_score(A, H, R, T, psn, pcs);
  if (lead && lane == 0) score[b] = p;
  float sq[6] = {0, 0, 0, 0, 0, 0};
  if (lead && A.regul_rate != 0.0f) row_sq(A, b, lane, sq);
  float mx = -INFINITY;
  const int64_t per = SPLIT ? (A.K + NS_WAVES - 1) / NS_WAVES : A.K;
  const int64_t jlo = SPLIT ? (int64_t)w * per : 0, jhi = jlo + per < A.K ? jlo + per : A.K;
  for (int64_t j0 = jlo; j0 < jhi; j0 += kWave) {
    const int nch = (int)(jhi - j0 < kWave ? jhi - j0 : kWave);
    int64_t mh = 0, mt = 0, mr = 0;
    if (lane < nch) {
      const int64_t row = b + (j0 + lane + 1) * A.B;
      mh = A.h[row]; mt = A.t[row]; mr = A.r[row];
    }
    for (int u0 = 0; u0 < nch; u0 += NSG) {
      Row2<NC> X[NSG];
      int code[NSG];
#pragma unroll
      for (int i = 0; i < NSG; ++i) {
        const int u = u0 + i;
        code[i] = 3;
        if (u >= nch) continue;
        const int64_t h = readlane64u(mh, u), t = readlane64u(mt, u), r = readlane64u(mr, u);
        code[i] = __builtin_amdgcn_readfirstlane(neg_code(h, r, t, ph, pr, pt));
        if (code[i] == 0) gen_load(X[i], A, true, h, lane);
        else if (code[i] == 1) gen_load(X[i], A, true, t, lane);
        else if (code[i] == 2) gen_load(X[i], A, false, r, lane);
      }
#pragma unroll
      for (int i = 0; i < NSG; ++i) {
        const int u = u0 + i;
        if (u >= nch) continue;
        const int64_t j = j0 + u, row = b + (j + 1) * A.B;
        float n;
        if (code[i] == 0) n = gen_score(A, X[i], R, T, psn, pcs);
        else if (code[i] == 1) n = gen_score(A, H, R, X[i], psn, pcs);
        else if (code[i] == 2) {
          Vec<NC> sn, cs;
          rot_sincos(A, X[i], sn, cs);
          n = gen_score(A, H, X[i], T, sn, cs);
        } else if (code[i] == 3) n = p;
        else n = row_score(A, row, lane);
        if (lane == 0) { score[row] = n; sn[j] = n; }
        if (A.regul_rate != 0.0f) row_sq(A, row, lane, sq);
        if (A.adv_t > 0.0f) mx = fmaxf(mx, -n * A.adv_t);
      }
    }
  }
  float sqv[6];
  for (int i = 0; i < 6; ++i) sqv[i] = A.regul_rate != 0.0f ? wave_sum(sq[i]) : 0.0f;
  if constexpr (SPLIT) {  // the waves' regularization partials and maxima, combined by wave 0 in wave order
    if (lane == 0) {
      for (int i = 0; i < 6; ++i) s_sq[w][i] = sqv[i];
      s_mx[w] = mx;
    }
    __syncthreads();
    if (w != 0 || lane != 0) return;
    for (int v = 1; v < NS_WAVES; ++v) mx = fmaxf(mx, s_mx[v]);
    for (int i = 0; i < 6; ++i) {
      float v = s_sq[0][i];
      for (int ww = 1; ww < NS_WAVES; ++ww) v += s_sq[ww][i];
      sqv[i] = v;
    }
  } else {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane != 0) return;
  }
  float loss = 0.0f;
  if (A.adv_t > 0.0f) {
    float den = 0.0f;
    for (int64_t j = 0; j < A.K; ++j) den += expf(-sn[j] * A.adv_t - mx);
    for (int64_t j = 0; j < A.K; ++j) {
      const float n = sn[j];
      loss += expf(-n * A.adv_t - mx) / den * fmaxf(p - n, -A.loss_margin);
    }
  } else {
    for (int64_t j = 0; j < A.K; ++j) loss += fmaxf(p - sn[j], -A.loss_margin);
  }
  part[b * 7] = loss;
  for (int i = 0; i < 6; ++i) part[b * 7 + 1 + i] = sqv[i];
}

// One wave per positive: the loss's d/d(score) coefficients of its rows (k_ns_row_coef's
// formulas, unit upstream gradient), each row's gradient; what a negative adds to a row it
// shares with its positive (same role, same id) is summed in registers, every other row gets
// a slot of its own. Inactive rows (zero coefficient, no regularization) add nothing.
// Negatives go in chunks of 21 (63 slot lanes): their ids and coefficients are read
// lane-parallel, the chunk's bucket places come back from ONE batched atomic round trip, and
// NSG corrupted rows are loaded together; sums and records are those of the per-negative loop
// (same formulas, same order).
template <int NC, int MODEL>
__global__ __launch_bounds__(256) void k_ns_gen_slots(NSArgs A_, const float* __restrict__ score, NSSlots S,
                                                      int64_t n_ent, int dpad, int with_reg) {
  constexpr int CH = 21;
  constexpr int NG = MODEL == MMRE_DISTMULT ? NSG : 2;  // two-half rows: fewer in flight (registers)
  // record layout (rec_store): stride 2 d for the two-half models; entity / relation records' halves
  constexpr bool S2 = MODEL != MMRE_DISTMULT, E2 = MODEL != MMRE_DISTMULT, R2 = MODEL == MMRE_COMPLEX;
  (void)dpad;
  NSArgs A = A_;
  A.model = MODEL;  // compile-time model
  constexpr int NH = MODEL == MMRE_DISTMULT ? 1 : 2;  // row halves carried by the own-row partials
  // SPLIT (DistMult): one workgroup per positive, its negatives split over the waves, own-row
  // partials combined in wave order; the two-half models: one wave per positive (k_ns_gen_forward)
  constexpr bool SPLIT = MODEL == MMRE_DISTMULT;
  __shared__ float s_own[SPLIT ? NS_WAVES - 1 : 1][3][NH][NC][kWave];  // waves 1-3's own-row partial sums
  __shared__ float s_occ[NS_WAVES - 1][3];
  const int d = A.dim;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b = SPLIT ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * NS_WAVES + w;
  if (b >= A.B) return;  // workgroup- (SPLIT) or wave-uniform
  const bool lead = SPLIT ? w == 0 : true;
  const float p = score[b];
  float mx = -INFINITY, den = 0.0f;
  if (A.adv_t > 0.0f) {
    for (int64_t j = lane; j < A.K; j += kWave) mx = fmaxf(mx, -score[b + (j + 1) * A.B] * A.adv_t);
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
    for (int64_t j = lane; j < A.K; j += kWave) den += expf(-score[b + (j + 1) * A.B] * A.adv_t - mx);
    den = wave_sum(den);
  }
  auto coef = [&](int64_t j) {
    const float n = score[b + (j + 1) * A.B];
    const float x = p - n, m = -A.loss_margin;
    const float ind = x > m ? 1.0f : (x == m ? 0.5f : 0.0f);  // maximum(): ties split the gradient
    const float c = A.adv_t > 0.0f ? (expf(-n * A.adv_t - mx) / den) / (float)A.B : 1.0f / (float)(A.B * A.K);
    return c * ind;
  };
  float gp = 0.0f;
  for (int64_t j = lane; j < A.K; j += kWave) gp += coef(j);
  gp = wave_sum(gp);
  const int64_t ph = A.h[b], pr = A.r[b], pt = A.t[b];
  Row2<NC> H, R, T, Gh, Gr, Gt, dH, dR, dT;
  gen_load(H, A, true, ph, lane);
  gen_load(R, A, false, pr, lane);
  gen_load(T, A, true, pt, lane);
  Vec<NC> psn, pcs;
  rot_sincos(A, R, psn, pcs);
  // wave 0 starts the own-row sums with the positive's gradient, waves 1-3 from zero; each wave
  // takes a contiguous range of the negatives; the partials are combined in wave order below
  if (lead) {
    gen_row_grad(A, H, R, T, gp, Gh, Gr, Gt, &psn, &pcs);
  } else {
    vzero(Gh.a); vzero(Gh.b); vzero(Gr.a); vzero(Gr.b); vzero(Gt.a); vzero(Gt.b);
  }
  const float k0 = lead ? 1.0f : 0.0f;
  float kh = k0, kr = k0, kt = k0;  // occurrences of the positive's rows (regularization)
  const int64_t sb = b * (3 + 3 * A.K);
  const int64_t per = SPLIT ? (A.K + NS_WAVES - 1) / NS_WAVES : A.K;
  const int64_t jlo = SPLIT ? (int64_t)w * per : 0, jhi = jlo + per < A.K ? jlo + per : A.K;
  for (int64_t j0 = jlo; j0 < jhi; j0 += CH) {
    const int nch = (int)(jhi - j0 < CH ? jhi - j0 : CH);
    int64_t mh = 0, mt = 0, mr = 0;
    float mg = 0.0f;
    if (lane < nch) {
      const int64_t row = b + (j0 + lane + 1) * A.B;
      mh = A.h[row]; mt = A.t[row]; mr = A.r[row];
      mg = -coef(j0 + lane);
    }
    // keys of the chunk's slots (lane 3u + k: negative u's row k when it is not the positive's)
    uint32_t my_key = S.sentinel;
    int64_t my_slot = 0;
    for (int u = 0; u < nch; ++u) {
      const float g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mg), u));
      if (g == 0.0f && !with_reg) continue;
      const int64_t h = readlane64u(mh, u), t = readlane64u(mt, u), r = readlane64u(mr, u);
      const int64_t sl = sb + 3 + 3 * (j0 + u);
      if (lane == 3 * u && h != ph) { my_key = (uint32_t)h; my_slot = sl; }
      if (lane == 3 * u + 1 && r != pr) { my_key = (uint32_t)(n_ent + r); my_slot = sl + 1; }
      if (lane == 3 * u + 2 && t != pt) { my_key = (uint32_t)t; my_slot = sl + 2; }
    }
    const bool filing = my_key != S.sentinel;
    const int place = filing ? atomicAdd(&S.counts[my_key], 1) : 0;
    for (int u0 = 0; u0 < nch; u0 += NG) {
      Row2<NC> X[NG];
      int code[NG];
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const int u = u0 + i;
        code[i] = 3;
        if (u >= nch) continue;
        const float g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mg), u));
        if (g == 0.0f && !with_reg) { code[i] = -1; continue; }  // inactive
        const int64_t h = readlane64u(mh, u), t = readlane64u(mt, u), r = readlane64u(mr, u);
        code[i] = __builtin_amdgcn_readfirstlane(neg_code(h, r, t, ph, pr, pt));
        if (code[i] == 0) gen_load(X[i], A, true, h, lane);
        else if (code[i] == 1) gen_load(X[i], A, true, t, lane);
        else if (code[i] == 2) gen_load(X[i], A, false, r, lane);
      }
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const int u = u0 + i;
        if (u >= nch) continue;
        const int64_t h = readlane64u(mh, u), t = readlane64u(mt, u), r = readlane64u(mr, u);
        const bool oh = h == ph, orr = r == pr, ot = t == pt;
        if (code[i] < 0) {
          kh += oh ? 1.0f : 0.0f; kr += orr ? 1.0f : 0.0f; kt += ot ? 1.0f : 0.0f;
          continue;
        }
        const float g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mg), u));
        if (code[i] == 0) gen_row_grad(A, X[i], R, T, g, dH, dR, dT, &psn, &pcs);
        else if (code[i] == 1) gen_row_grad(A, H, R, X[i], g, dH, dR, dT, &psn, &pcs);
        else if (code[i] == 2) gen_row_grad(A, H, X[i], T, g, dH, dR, dT);
        else if (code[i] == 3) gen_row_grad(A, H, R, T, g, dH, dR, dT, &psn, &pcs);
        else {
          Row2<NC> Hj, Rj, Tj;
          if (oh) Hj = H; else gen_load(Hj, A, true, h, lane);
          if (orr) Rj = R; else gen_load(Rj, A, false, r, lane);
          if (ot) Tj = T; else gen_load(Tj, A, true, t, lane);
          gen_row_grad(A, Hj, Rj, Tj, g, dH, dR, dT);
        }
        const int64_t sl = sb + 3 + 3 * (j0 + u);
        if (oh) { row2_add(Gh, dH); kh += 1.0f; } else { rec_store(S.rec, sl, d, S2, E2, dH, lane); }
        if (orr) { row2_add(Gr, dR); kr += 1.0f; } else { rec_store(S.rec, sl + 1, d, S2, R2, dR, lane); }
        if (ot) { row2_add(Gt, dT); kt += 1.0f; } else { rec_store(S.rec, sl + 2, d, S2, E2, dT, lane); }
      }
    }
    if (filing) {  // the chunk's entries, at the places the atomic returned
      const int64_t e = slot_entry(my_slot, 1.0f);
      if (place < NS_BUCKET) {
        S.bucket[(int64_t)my_key * NS_BUCKET + place] = e;
      } else {
        const int o = atomicAdd(S.ovf_n, 1);
        S.ovf[2 * (int64_t)o] = (int64_t)my_key;
        S.ovf[2 * (int64_t)o + 1] = e;
      }
    }
  }
  // own rows: wave 0 adds waves 1, 2, 3's partials in that order (a fixed order: bit-reproducible)
  auto park = [&](int k, const Row2<NC>& g) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      s_own[w - 1][k][0][c][lane] = g.a.v[c];
      if constexpr (NH == 2) s_own[w - 1][k][NH - 1][c][lane] = g.b.v[c];
    }
  };
  auto gather = [&](int v, int k, Row2<NC>& g) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      g.a.v[c] += s_own[v][k][0][c][lane];
      if constexpr (NH == 2) g.b.v[c] += s_own[v][k][NH - 1][c][lane];
    }
  };
  if constexpr (SPLIT) {
    if (w > 0) {
      park(0, Gh);
      park(1, Gr);
      park(2, Gt);
      if (lane == 0) { s_occ[w - 1][0] = kh; s_occ[w - 1][1] = kr; s_occ[w - 1][2] = kt; }
    }
    __syncthreads();
    if (w > 0) return;
    for (int v = 0; v < NS_WAVES - 1; ++v) {
      gather(v, 0, Gh);
      gather(v, 1, Gr);
      gather(v, 2, Gt);
      kh += s_occ[v][0]; kr += s_occ[v][1]; kt += s_occ[v][2];  // integer-valued
    }
  }
  rec_store(S.rec, sb, d, S2, E2, Gh, lane);
  rec_store(S.rec, sb + 1, d, S2, R2, Gr, lane);
  rec_store(S.rec, sb + 2, d, S2, E2, Gt, lane);
  if (lane < 3) {
    const uint32_t key = lane == 0 ? (uint32_t)ph : (lane == 1 ? (uint32_t)(n_ent + pr) : (uint32_t)pt);
    put_slot(S, key, sb + lane, lane == 0 ? kh : (lane == 1 ? kr : kt));
  }
}

// One table row of the generic owner from its ordered slots (Ord as for transe_owner_row).
template <int NC, class Ord>
__device__ __forceinline__ void gen_owner_row(Ord& ord, bool active, const NSArgs& A, int64_t row, int n,
                                              const Row2<NC>& v, int64_t n_ent, float reg_ent, float reg_rel,
                                              const float* __restrict__ rec, const float* __restrict__ grad_loss,
                                              float* oa, float* ob, float* pa, float* pb, float sgd_lr) {
  const int lane = threadIdx.x & 63;
  const bool is_ent = row < n_ent;
  const int d = A.dim;
  const bool two = A.model == MMRE_COMPLEX || (A.model == MMRE_ROTATE && is_ent);
  const bool s2 = A.model == MMRE_COMPLEX || A.model == MMRE_ROTATE;  // record stride (rec_store); TransE: d
  Row2<NC> dy;
  vzero(dy.a);
  vzero(dy.b);
  float cnt = 0.0f;
  for (int c0 = 0; c0 < n;) {
    int take;
    const int64_t ordered = ord.next(take);
    c0 += take;
    if (!active) continue;
    const int sl = lane < take ? (int)entry_slot(ordered) : 0;
    cnt += wave_sum(lane < take ? entry_mult(ordered) : 0.0f);  // integer-valued: exact in any order
    int u = 0;
    for (; u + 2 <= take; u += 2) {  // two records in flight, added in slot order
      Row2<NC> r0, r1;
      rec_load(r0, rec, __builtin_amdgcn_readlane(sl, u), d, s2, two, lane);
      rec_load(r1, rec, __builtin_amdgcn_readlane(sl, u + 1), d, s2, two, lane);
      row2_add(dy, r0);
      row2_add(dy, r1);
    }
    if (u < take) {
      Row2<NC> r0;
      rec_load(r0, rec, __builtin_amdgcn_readlane(sl, u), d, s2, two, lane);
      row2_add(dy, r0);
    }
  }
  if (!active) return;
  const float G = grad_loss ? grad_loss[0] : 1.0f;
  const float rr = (is_ent ? reg_ent : reg_rel) * cnt;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    dy.a.v[c] = (dy.a.v[c] + rr * v.a.v[c]) * G;
    dy.b.v[c] = (dy.b.v[c] + rr * v.b.v[c]) * G;
  }
  vstore(oa, dy.a, d, lane);
  if (two) vstore(ob, dy.b, d, lane);
  if (sgd_lr != 0.0f) {
    Row2<NC> p;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      p.a.v[c] = __builtin_fmaf(-sgd_lr, dy.a.v[c], v.a.v[c]);
      p.b.v[c] = __builtin_fmaf(-sgd_lr, dy.b.v[c], v.b.v[c]);
    }
    vstore(pa, p.a, d, lane);
    if (two) vstore(pb, p.b, d, lane);
  }
}

// One wave per table row: its slots' records summed in slot order, + reg (occurrences) v, times
// the upstream gradient, written to every row of the gradient tables (and, with sgd_lr, the
// parameter rows updated by fma(-lr, g, v)). Rows with more than NS_HUB slots go to the
// first n_hub_wg workgroups (HubOrder); rows start at workgroup row_block0.
template <int NC>
__global__ __launch_bounds__(256) void k_ns_gen_owner(NSArgs A, int64_t n_ent, int64_t n_rel, float reg_ent,
                                                      float reg_rel, const float* __restrict__ rec,
                                                      const int32_t* __restrict__ counts,
                                                      const int64_t* __restrict__ bucket,
                                                      const int64_t* __restrict__ ovf, const int32_t* __restrict__ ovf_n,
                                                      int dpad, const float* __restrict__ grad_loss, float* gent,
                                                      float* gent_im, float* grel, float* grel_im, float sgd_lr,
                                                      float* pent, float* pent_im, float* prel, float* prel_im,
                                                      int64_t row_block0, int n_hub_wg, int64_t n_slots,
                                                      const float* __restrict__ part, float* __restrict__ loss,
                                                      int64_t reduce_block, NSNext nx) {
  __shared__ int64_t s_hub[4][NS_HUB];
  __shared__ uint16_t s_bits[256];
  __shared__ int32_t s_hc[2];
  (void)dpad;
  // the one-call training step (mmre_ns_step_openke_gen_pipe): the loss reduction and the next
  // batch's sampler workgroups ride in this grid (the forward zeroes the slot counts itself)
  if ((int64_t)blockIdx.x == reduce_block) {
    ns_reduce_block(A, part, loss);
    return;
  }
  if ((int64_t)blockIdx.x >= nx.block0 && (int64_t)blockIdx.x < nx.block0 + nx.n_blocks) {
    sampler_openke_block(nx.sa, (int64_t)blockIdx.x - nx.block0, nx.n_blocks);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int d = A.dim;
  // output rows of the two halves of table row `row`
  auto outs = [&](int64_t row, float*& oa, float*& ob, float*& pa, float*& pb) {
    const bool is_ent = row < n_ent;
    const int64_t id = is_ent ? row : row - n_ent;
    ob = pa = pb = nullptr;
    if (is_ent) {
      if (A.model == MMRE_COMPLEX) { oa = gent + id * d; ob = gent_im + id * d; pa = pent ? pent + id * d : nullptr; pb = pent_im ? pent_im + id * d : nullptr; }
      else if (A.model == MMRE_ROTATE) { oa = gent + id * 2 * d; ob = oa + d; pa = pent ? pent + id * 2 * d : nullptr; pb = pa ? pa + d : nullptr; }
      else { oa = gent + id * d; pa = pent ? pent + id * d : nullptr; }
    } else {
      oa = grel + id * d;
      pa = prel ? prel + id * d : nullptr;
      if (A.model == MMRE_COMPLEX) { ob = grel_im + id * d; pb = prel_im ? prel_im + id * d : nullptr; }
    }
  };
  if ((int64_t)blockIdx.x < n_hub_wg) {  // hub rows: the first n_hub_wg workgroups (they start first)
    for_hub_rows(counts, n_ent + n_rel, (int)blockIdx.x, n_hub_wg, s_bits,
                 [&](int64_t row, int n) {
                   const bool is_ent = row < n_ent;
                   float *oa, *ob, *pa, *pb;
                   outs(row, oa, ob, pa, pb);
                   Row2<NC> v;
                   gen_load(v, A, is_ent, is_ent ? row : row - n_ent, lane);
                   HubOrder ord = hub_order(s_hub, s_hc, bucket, ovf, ovf_n[0], n, row, n_slots);
                   gen_owner_row<NC>(ord, threadIdx.x < 64, A, row, n, v, n_ent, reg_ent, reg_rel, rec, grad_loss, oa,
                                     ob, pa, pb, sgd_lr);
                 });
    return;
  }
  const int64_t row = ((int64_t)blockIdx.x - row_block0) * 4 + (threadIdx.x >> 6);
  if (row >= n_ent + n_rel) return;  // wave-uniform
  const bool is_ent = row < n_ent;
  const int64_t id = is_ent ? row : row - n_ent;
  const int64_t pre = bucket[row * NS_BUCKET + lane];
  const bool two = A.model == MMRE_COMPLEX || (A.model == MMRE_ROTATE && is_ent);
  float *oa, *ob, *pa, *pb;
  outs(row, oa, ob, pa, pb);
  const int n = counts[row];
  if (n > NS_HUB) return;  // a hub workgroup's row
  if (n == 0) {
    Row2<NC> z;
    vzero(z.a);
    vzero(z.b);
    vstore(oa, z.a, d, lane);
    if (two) vstore(ob, z.b, d, lane);
    return;
  }
  Row2<NC> v;
  gen_load(v, A, is_ent, id, lane);
  SlotOrder ord{ovf, n > NS_BUCKET ? ovf_n[0] : 0, n, lane, row, s_hub[threadIdx.x >> 6], pre, 0, 0};
  ord.init();
  gen_owner_row<NC>(ord, true, A, row, n, v, n_ent, reg_ent, reg_rel, rec, grad_loss, oa, ob, pa, pb, sgd_lr);
}

// ---------------------------------------------------------------------------------------
// Deterministic backward of model(data) over ARBITRARY rows (mmre_score_rows_backward: OpenKE
// Model.forward in 'normal' mode under any loss -- SoftplusLoss, SigmoidLoss, cross modes -- and
// the repo's scoring_fn / _calc) and of the non-fused margin loss (mmre_ns_backward). No float
// atomics: scored row i files three slots 3i + q (its h / r / t gradient row, raw space) into
// the buckets of their table rows, and k_ns_gen_owner sums each table row's slots in slot order
// (= batch order), so the gradient tables are bit-identical run to run.
// ---------------------------------------------------------------------------------------

// TransE (L1 / L2, optional norm_flag) gradient of one row in RAW space: the per-element
// expressions of the TransE forward's derivative (x = (h/|h| + r/|r|) - t/|t|, TransE.py:46-74;
// gx = g sign(x) or g x / |x|; the normalisation's Jacobian (dy - y (y . dy)) / |v|), on rows held
// in registers.
template <int NC>
__device__ __forceinline__ void transe_row_grad(const NSArgs& A, const Row2<NC>& H, const Row2<NC>& R,
                                                const Row2<NC>& T, float g, Row2<NC>& dH, Row2<NC>& dR,
                                                Row2<NC>& dT) {
  const bool l2 = A.model == MMRE_TRANSE_L2;
  if (A.use_model_margin) g = -g;  // forward = m - s
  float nh = 1.0f, nt = 1.0f, nr = 1.0f;
  if (A.norm_flag) {
    float a = vsq(H.a), b = vsq(T.a), c = vsq(R.a);
    wave_sum3(a, b, c);
    nh = sqrtf(a); nt = sqrtf(b); nr = sqrtf(c);
  }
  const float ch = fmaxf(nh, 1e-12f), ct = fmaxf(nt, 1e-12f), cr = fmaxf(nr, 1e-12f);
  float s = 0.0f;
  if (l2) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float x = (H.a.v[c] / ch + R.a.v[c] / cr) - T.a.v[c] / ct;
      s += x * x;
    }
    s = sqrtf(wave_sum(s));
  }
  Vec<NC> gx;
  float dh_dot = 0.0f, dt_dot = 0.0f, dr_dot = 0.0f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float x = (H.a.v[c] / ch + R.a.v[c] / cr) - T.a.v[c] / ct;
    gx.v[c] = !l2 ? g * (float)((x > 0.0f) - (x < 0.0f)) : (s > 0.0f ? g * x / s : 0.0f);
    dh_dot += (H.a.v[c] / ch) * gx.v[c];
    dr_dot += (R.a.v[c] / cr) * gx.v[c];
    dt_dot += (T.a.v[c] / ct) * (-gx.v[c]);
  }
  if (A.norm_flag) wave_sum3(dh_dot, dr_dot, dt_dot);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float dh = gx.v[c], dr = gx.v[c], dt = -gx.v[c];
    if (A.norm_flag) {
      dh = nh > 1e-12f ? (dh - (H.a.v[c] / ch) * dh_dot) / nh : dh / 1e-12f;
      dr = nr > 1e-12f ? (dr - (R.a.v[c] / cr) * dr_dot) / nr : dr / 1e-12f;
      dt = nt > 1e-12f ? (dt - (T.a.v[c] / ct) * dt_dot) / nt : dt / 1e-12f;
    }
    dH.a.v[c] = dh; dR.a.v[c] = dr; dT.a.v[c] = dt;
    dH.b.v[c] = dR.b.v[c] = dT.b.v[c] = 0.0f;
  }
}

// d(loss)/d(score) of every row of the margin loss (MarginLoss.py:24-28 with the detached
// self-adversarial weights of :19-22 through NegativeSampling.py:23-32; unit upstream
// gradient): coef[b] = sum_j c_j ind_j for positive b, coef[b + (j + 1) B] = -c_j ind_j.
__global__ __launch_bounds__(256) void k_ns_row_coef(NSArgs A, const float* __restrict__ score,
                                                      float* __restrict__ coef) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * NS_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (b >= A.B) return;
  const float p = score[b];
  float mx = -INFINITY, den = 0.0f;
  if (A.adv_t > 0.0f) {
    for (int64_t j = lane; j < A.K; j += kWave) mx = fmaxf(mx, -score[b + (j + 1) * A.B] * A.adv_t);
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
    for (int64_t j = lane; j < A.K; j += kWave) den += expf(-score[b + (j + 1) * A.B] * A.adv_t - mx);
    den = wave_sum(den);
  }
  float gp = 0.0f;
  for (int64_t j = lane; j < A.K; j += kWave) {
    const float n = score[b + (j + 1) * A.B];
    const float x = p - n, m = -A.loss_margin;
    const float ind = x > m ? 1.0f : (x == m ? 0.5f : 0.0f);  // maximum(): ties split the gradient
    const float c = A.adv_t > 0.0f ? (expf(-n * A.adv_t - mx) / den) / (float)A.B : 1.0f / (float)(A.B * A.K);
    coef[b + (j + 1) * A.B] = -(c * ind);
    gp += c * ind;
  }
  gp = wave_sum(gp);
  if (lane == 0) coef[b] = gp;
}

// One wave per scored row: its three gradient rows as slot records 3i + q (q = h, r, t) and the
// slots filed in their table rows' buckets (occurrence weight 1: the regularization counts every
// gathered row). Rows adding nothing (zero coefficient, no regularization) file nothing.
template <int NC>
__global__ __launch_bounds__(256) void k_rows_slots(NSArgs A, const float* __restrict__ coef, int64_t n_rows,
                                                    NSSlots S, int64_t n_ent, int with_reg) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * NS_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (i >= n_rows) return;  // wave-uniform
  const float g = coef[i];
  if (g == 0.0f && !with_reg) return;
  const int d = A.dim;
  const int64_t h = A.h[i], t = A.t[i], r = A.r[i];
  Row2<NC> H, R, T, dH, dR, dT;
  gen_load(H, A, true, h, lane);
  gen_load(R, A, false, r, lane);
  gen_load(T, A, true, t, lane);
  if (A.model == MMRE_TRANSE_L1 || A.model == MMRE_TRANSE_L2) transe_row_grad(A, H, R, T, g, dH, dR, dT);
  else gen_row_grad(A, H, R, T, g, dH, dR, dT);
  const bool s2 = A.model == MMRE_COMPLEX || A.model == MMRE_ROTATE;  // k_ns_gen_owner's record layout
  const bool e2 = s2, r2 = A.model == MMRE_COMPLEX;
  rec_store(S.rec, 3 * i, d, s2, e2, dH, lane);
  rec_store(S.rec, 3 * i + 1, d, s2, r2, dR, lane);
  rec_store(S.rec, 3 * i + 2, d, s2, e2, dT, lane);
  if (lane < 3) {
    const uint32_t key = lane == 0 ? (uint32_t)h : (lane == 1 ? (uint32_t)(n_ent + r) : (uint32_t)t);
    put_slot(S, key, 3 * i + lane, 1.0f);
  }
}

// which TransE fast-path instance fits: elements per lane (0: none, generic path)
static int transe_fast_nc(const NSArgs& A) {
  if (A.model != MMRE_TRANSE_L1 && A.model != MMRE_TRANSE_L2) return 0;
  if (A.K > NS_MAXK) return 0;
  if (A.dim <= 64) return 1;
  if (A.dim <= 128) return 2;
  if (A.dim <= 256) return 4;
  if (A.dim <= 512) return 8;
  return 0;
}

static int ns_args(NSArgs& A, int model, int norm_flag, float model_margin, int use_model_margin, const float* ent,
                   const float* ent_im, const float* rel, const float* rel_im, int dim, float phase_denom,
                   const int64_t* h, const int64_t* t, const int64_t* r, int64_t batch, int64_t neg,
                   float loss_margin, float adv_t, float regul_rate) {
  if (model < MMRE_TRANSE_L1 || model > MMRE_ROTATE) return MMRE_ERR_MODEL;
  if (!ent || !rel || !h || !t || !r || batch <= 0 || neg < 0 || dim <= 0) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!ent_im || !rel_im)) return MMRE_ERR_ARG;
  if (model == MMRE_ROTATE && !(phase_denom != 0.0f)) return MMRE_ERR_ARG;
  A.model = model; A.norm_flag = norm_flag; A.use_model_margin = use_model_margin; A.dim = dim;
  A.model_margin = model_margin; A.phase_denom = phase_denom;
  A.ent = ent; A.ent_im = ent_im; A.rel = rel; A.rel_im = rel_im;
  A.h = h; A.t = t; A.r = r; A.B = batch; A.K = neg;
  A.loss_margin = loss_margin; A.adv_t = adv_t; A.regul_rate = regul_rate;
  return MMRE_OK;
}

}  // namespace mmre

using namespace mmre;

extern "C" int64_t mmre_ns_workspace(int64_t batch, int64_t neg) {
  (void)neg;
  return 7 * (batch > 0 ? batch : 1);
}

extern "C" int mmre_ns_forward(int model, int norm_flag, float model_margin, int use_model_margin, const float* d_ent,
                               const float* d_ent_im, const float* d_rel, const float* d_rel_im, int dim,
                               float phase_denom, const int64_t* d_h, const int64_t* d_t, const int64_t* d_r,
                               int64_t batch, int64_t neg, float loss_margin, float adv_temperature, float regul_rate,
                               float* d_score, float* d_loss, float* d_work, void* stream) {
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim,
                   phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature, regul_rate);
  if (rc) return rc;
  if (!d_score || !d_work) return MMRE_ERR_ARG;
  if (neg > NS_MAXK) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int nc = transe_fast_nc(A);
  const dim3 grid((unsigned)batch), blk(256);
  const bool l2 = model == MMRE_TRANSE_L2;
#define MMRE_NS_FWD(NC_)                                                                              \
  do {                                                                                                \
    if (l2) hipLaunchKernelGGL((k_ns_transe_forward<NC_, true>), grid, blk, 0, st, A, d_score, d_work); \
    else hipLaunchKernelGGL((k_ns_transe_forward<NC_, false>), grid, blk, 0, st, A, d_score, d_work);   \
  } while (0)
  if (nc == 1) MMRE_NS_FWD(1);
  else if (nc == 2) MMRE_NS_FWD(2);
  else if (nc == 4) MMRE_NS_FWD(4);
  else if (nc == 8) MMRE_NS_FWD(8);
  else {
    hipLaunchKernelGGL(k_ns_forward, dim3((unsigned)((batch + NS_WAVES - 1) / NS_WAVES)), dim3(256), 0, st, A,
                       d_score, d_work, nullptr, (int64_t)0);
  }
#undef MMRE_NS_FWD
  MMRE_CHECK_LAUNCH();
  if (d_loss) {
    hipLaunchKernelGGL(k_ns_reduce, dim3(1), dim3(256), 0, st, A, d_work, d_loss);
    MMRE_CHECK_LAUNCH();
  }
  return MMRE_OK;
}

// Workspace of the rows backward (floats): per-row coefficients, 3 slot records per row,
// per-table-row slot counts (+ the overflow count), buckets, overflow pairs.
struct RowsWs {
  int64_t coef, rec, counts, bucket, ovf, total;
};
static int64_t al64r(int64_t x) { return (x + 63) & ~(int64_t)63; }
static void rows_ws(int model, int64_t n_rows, int64_t E, int64_t R, int d, RowsWs& w) {
  const int64_t width = (model == MMRE_COMPLEX || model == MMRE_ROTATE) ? 2 * (int64_t)d : d;
  int64_t o = 0;
  w.coef = o;   o = al64r(o + n_rows);
  w.rec = o;    o = al64r(o + 3 * n_rows * width);
  w.counts = o; o = al64r(o + E + R + 1);
  w.bucket = o; o = al64r(o + 2 * (E + R) * NS_BUCKET);
  w.ovf = o;    o = al64r(o + 4 * 3 * n_rows);
  w.total = o;
}

extern "C" int64_t mmre_rows_backward_workspace(int model, int64_t n_rows, int64_t n_ent, int64_t n_rel, int dim) {
  if (n_rows <= 0 || n_ent <= 0 || n_rel <= 0 || dim <= 0) return 0;
  RowsWs w;
  rows_ws(model, n_rows, n_ent, n_rel, dim, w);
  return w.total;
}

// 64-float chunks per lane of the rows backward's slot / owner kernels. Up to 2,048 floats per
// row plane (the reference's examples train TransE at dim 1,024 with SigmoidLoss and cross
// sampling, OpenKE/examples/train_transe_WN18_adv_sigmoidloss.py): the wide instances keep
// their rows in more registers (they may spill at NC 32; these rows are not a hot shape).
static int gen_nc_rows(int dim) {
  return dim <= 64 ? 1 : dim <= 128 ? 2 : dim <= 256 ? 4 : dim <= 512 ? 8 : dim <= 1024 ? 16 : dim <= 2048 ? 32 : 0;
}

// coefficients in w.coef already (or to be read from d_coef): slots, then the owner pass
static int rows_backward_impl(const NSArgs& A, const float* d_coef, int64_t n_rows, int64_t n_ent, int64_t n_rel,
                              float reg_ent, float reg_rel, const float* d_grad_loss, float* d_grad_ent,
                              float* d_grad_ent_im, float* d_grad_rel, float* d_grad_rel_im, float* d_work,
                              const RowsWs& w, hipStream_t st) {
  const int nc = gen_nc_rows(A.dim);
  if (nc == 0) return MMRE_ERR_SHAPE;
  if (n_ent + n_rel >= (int64_t)UINT32_MAX || 3 * n_rows >= (int64_t)INT32_MAX) return MMRE_ERR_SHAPE;
  int32_t* counts = reinterpret_cast<int32_t*>(d_work + w.counts);
  NSSlots S{nullptr, d_work + w.rec, counts, reinterpret_cast<int64_t*>(d_work + w.bucket),
            reinterpret_cast<int64_t*>(d_work + w.ovf), counts + n_ent + n_rel, (uint32_t)(n_ent + n_rel)};
  MMRE_CHECK(hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)(n_ent + n_rel + 1), st));
  const dim3 sgrid((unsigned)((n_rows + NS_WAVES - 1) / NS_WAVES)), ogrid((unsigned)((n_ent + n_rel + 3) / 4)),
      hgrid(ogrid.x + NS_HUB_WG), blk(256);
  const int with_reg = (reg_ent != 0.0f || reg_rel != 0.0f) ? 1 : 0;
#define MMRE_ROWS(NC_)                                                                                              \
  do {                                                                                                              \
    hipLaunchKernelGGL((k_rows_slots<NC_>), sgrid, blk, 0, st, A, d_coef, n_rows, S, n_ent, with_reg);              \
    hipLaunchKernelGGL((k_ns_gen_owner<NC_>), hgrid, blk, 0, st, A, n_ent, n_rel, reg_ent, reg_rel, S.rec, S.counts, \
                       S.bucket, S.ovf, S.ovf_n, 0, d_grad_loss, d_grad_ent, d_grad_ent_im, d_grad_rel,             \
                       d_grad_rel_im, 0.0f, nullptr, nullptr, nullptr, nullptr, (int64_t)NS_HUB_WG, NS_HUB_WG,        \
                       3 * n_rows, nullptr, nullptr, (int64_t)-1, NSNext{});                                        \
  } while (0)
  if (nc == 1) MMRE_ROWS(1);
  else if (nc == 2) MMRE_ROWS(2);
  else if (nc == 4) MMRE_ROWS(4);
  else if (nc == 8) MMRE_ROWS(8);
  else if (nc == 16) MMRE_ROWS(16);
  else MMRE_ROWS(32);
#undef MMRE_ROWS
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_ns_backward(int model, int norm_flag, float model_margin, int use_model_margin,
                                const float* d_ent, const float* d_ent_im, const float* d_rel, const float* d_rel_im,
                                int dim, float phase_denom, const int64_t* d_h, const int64_t* d_t,
                                const int64_t* d_r, int64_t batch, int64_t neg, float loss_margin,
                                float adv_temperature, float regul_rate, const float* d_score,
                                const float* d_grad_loss, float* d_grad_ent, float* d_grad_ent_im, float* d_grad_rel,
                                float* d_grad_rel_im, int64_t n_ent, int64_t n_rel, float* d_work,
                                int64_t work_floats, void* stream) {
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim,
                   phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature, regul_rate);
  if (rc) return rc;
  if (!d_score || !d_grad_ent || !d_grad_rel || !d_work || n_ent <= 0 || n_rel <= 0) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!d_grad_ent_im || !d_grad_rel_im)) return MMRE_ERR_ARG;
  const int64_t n_rows = batch * (1 + neg);
  RowsWs w;
  rows_ws(model, n_rows, n_ent, n_rel, dim, w);
  if (work_floats < w.total) return MMRE_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_ns_row_coef, dim3((unsigned)((batch + NS_WAVES - 1) / NS_WAVES)), dim3(256), 0, st, A, d_score,
                     d_work + w.coef);
  MMRE_CHECK_LAUNCH();
  // regularization scale per gathered row (TransE.py:92-102 and its kin, without the upstream gradient: the
  // owner pass multiplies by it)
  const double N = (double)batch * (1.0 + (double)neg);
  const double nterms = model == MMRE_COMPLEX ? 6.0 : 3.0;
  const double ew = model == MMRE_ROTATE ? 2.0 * dim : (double)dim;
  const float reg_ent = regul_rate != 0.0f ? (float)(regul_rate * 2.0 / (nterms * N * ew)) : 0.0f;
  const float reg_rel = regul_rate != 0.0f ? (float)(regul_rate * 2.0 / (nterms * N * dim)) : 0.0f;
  NSArgs R = A;
  R.B = n_rows;
  R.K = 0;
  return rows_backward_impl(R, d_work + w.coef, n_rows, n_ent, n_rel, reg_ent, reg_rel, d_grad_loss, d_grad_ent,
                            d_grad_ent_im, d_grad_rel, d_grad_rel_im, d_work, w, st);
}

extern "C" int mmre_score_rows_backward(int model, int norm_flag, float model_margin, int use_model_margin,
                                        const float* d_ent, const float* d_ent_im, const float* d_rel,
                                        const float* d_rel_im, int dim, float phase_denom, const int64_t* d_h,
                                        const int64_t* d_t, const int64_t* d_r, int64_t n_rows,
                                        const float* d_grad_score, float* d_grad_ent, float* d_grad_ent_im,
                                        float* d_grad_rel, float* d_grad_rel_im, int64_t n_ent, int64_t n_rel,
                                        float* d_work, int64_t work_floats, void* stream) {
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim,
                   phase_denom, d_h, d_t, d_r, n_rows, 0, 0.0f, 0.0f, 0.0f);
  if (rc) return rc;
  if (!d_grad_score || !d_grad_ent || !d_grad_rel || !d_work || n_ent <= 0 || n_rel <= 0) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!d_grad_ent_im || !d_grad_rel_im)) return MMRE_ERR_ARG;
  RowsWs w;
  rows_ws(model, n_rows, n_ent, n_rel, dim, w);
  if (work_floats < w.total) return MMRE_ERR_WORKSPACE;
  return rows_backward_impl(A, d_grad_score, n_rows, n_ent, n_rel, 0.0f, 0.0f, nullptr, d_grad_ent, d_grad_ent_im,
                            d_grad_rel, d_grad_rel_im, d_work, w, (hipStream_t)stream);
}

// Workspace of the fused path, in 4-byte words, 256-B aligned pieces: loss partials, row
// norms (+ the normalised tables with norm_flag), the slot contributions / occurrences, the
// per-row slot counts (then the overflow count), the buckets, the overflow pairs. TransE keeps the positives' sums (3 rows of d) and the negatives' records
// (ns_rec_words each); the other models one record of 2 d_pad floats per slot.
struct FusedWs {
  int64_t part, nrm_e, nrm_r, ent_n, rel_n, shared, rec, counts, bucket, ovf, total, slots;
  int dpad;
  uint32_t sentinel;
};

static int64_t al64(int64_t x) { return (x + 63) & ~(int64_t)63; }

static bool is_transe(int model) { return model == MMRE_TRANSE_L1 || model == MMRE_TRANSE_L2; }

static void fused_ws(int model, int norm_flag, int64_t B, int64_t K, int64_t E, int64_t R, int d, FusedWs& w) {
  w.slots = (3 + 3 * K) * B;
  w.sentinel = (uint32_t)(E + R);
  w.dpad = (int)round_up(d, kWave);
  const bool te = is_transe(model);
  int64_t o = 0;
  w.part = o;    o = al64(o + 7 * B);
  w.nrm_e = o;   o = al64(o + (te ? E : 0));
  w.nrm_r = o;   o = al64(o + (te ? R : 0));
  w.ent_n = o;   o = al64(o + (te && norm_flag ? E * d : 0));
  w.rel_n = o;   o = al64(o + (te && norm_flag ? R * d : 0));
  w.shared = o;  o = al64(o + (te ? 3 * B * d : 0));
  const int64_t rw = ns_rec_words(8, false, d);
  w.rec = o;     o = al64(o + (te ? K * B * (d > rw ? d : rw) : w.slots * (model == MMRE_DISTMULT ? 1 : 2) * d));
  w.counts = o;  o = al64(o + 2 * (E + R + 1));   // + the overflow count; two arrays (the pipelined
                                                  // step's parities: mmre_ns_step_openke_pipe)
  w.bucket = o;  o = al64(o + 2 * (E + R) * NS_BUCKET);   // int64 entries
  w.ovf = o;     o = al64(o + 4 * w.slots);                // int64 (row, entry) pairs
  w.total = o;
}

static NSSlots ws_slots(float* d_work, const FusedWs& w, int64_t E, int64_t R, int parity = 0) {
  int32_t* counts = reinterpret_cast<int32_t*>(d_work + w.counts) + (parity ? E + R + 1 : 0);
  return NSSlots{d_work + w.shared, d_work + w.rec, counts, reinterpret_cast<int64_t*>(d_work + w.bucket),
                 reinterpret_cast<int64_t*>(d_work + w.ovf), counts + E + R, w.sentinel};
}

extern "C" int64_t mmre_ns_fused_workspace(int model, int norm_flag, int64_t batch, int64_t neg, int64_t n_ent,
                                           int64_t n_rel, int dim) {
  FusedWs w;
  fused_ws(model, norm_flag, batch > 0 ? batch : 1, neg > 0 ? neg : 0, n_ent > 0 ? n_ent : 0, n_rel > 0 ? n_rel : 0,
           dim > 0 ? dim : 1, w);
  return w.total > 7 * batch ? w.total : 7 * batch;
}

static bool fused_fast(const NSArgs& A) { return transe_fast_nc(A) != 0 && A.K <= NSW * NSF_MAXJ; }

// elements per lane of the row-owner path of the other models (d <= 512)
static int gen_nc(int dim) { return dim <= 64 ? 1 : dim <= 128 ? 2 : dim <= 256 ? 4 : dim <= 512 ? 8 : 0; }

extern "C" int mmre_ns_fused_forward(int model, int norm_flag, float model_margin, int use_model_margin,
                                     const float* d_ent, const float* d_ent_im, const float* d_rel,
                                     const float* d_rel_im, int64_t n_ent, int64_t n_rel, int dim, float phase_denom,
                                     const int64_t* d_h, const int64_t* d_t, const int64_t* d_r, int64_t batch,
                                     int64_t neg, float loss_margin, float adv_temperature, float regul_rate,
                                     float* d_score, float* d_loss, float* d_work, void* stream) {
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim,
                   phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature, regul_rate);
  if (rc) return rc;
  if (!d_score || !d_loss || !d_work || n_ent <= 0 || n_rel <= 0) return MMRE_ERR_ARG;
  if (neg > NS_MAXK) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  FusedWs w;
  fused_ws(model, norm_flag, batch, neg, n_ent, n_rel, dim, w);
  float* part = d_work + w.part;
  NSSlots S = ws_slots(d_work, w, n_ent, n_rel);
  if (!fused_fast(A)) {  // other models: scores + partials (zeroing the bucket counts), then the loss
    const int gnc = gen_nc(dim);
    if (!is_transe(model) && gnc == 0) return MMRE_ERR_SHAPE;
    const dim3 fgrid((unsigned)((batch + NS_WAVES - 1) / NS_WAVES));
    if (is_transe(model)) {
      hipLaunchKernelGGL(k_ns_forward, fgrid, dim3(256), 0, st, A, d_score, part, S.counts, n_ent + n_rel + 1);
    } else {
      // k_ns_gen_forward: DistMult a workgroup per positive, the two-half models a wave per positive
      const dim3 fgrid((unsigned)(model == MMRE_DISTMULT ? batch : (batch + NS_WAVES - 1) / NS_WAVES));
#define MMRE_NS_GF(NC_, M_)                                                                                        \
  hipLaunchKernelGGL((k_ns_gen_forward<NC_, M_>), fgrid, dim3(256), 0, st, A, d_score, part, S.counts,             \
                     n_ent + n_rel + 1)
#define MMRE_NS_GF_M(NC_)                                                                                          \
  do {                                                                                                             \
    if (model == MMRE_DISTMULT) MMRE_NS_GF(NC_, MMRE_DISTMULT);                                                    \
    else if (model == MMRE_COMPLEX) MMRE_NS_GF(NC_, MMRE_COMPLEX);                                                 \
    else MMRE_NS_GF(NC_, MMRE_ROTATE);                                                                             \
  } while (0)
      if (gnc == 1) MMRE_NS_GF_M(1);
      else if (gnc == 2) MMRE_NS_GF_M(2);
      else if (gnc == 4) MMRE_NS_GF_M(4);
      else MMRE_NS_GF_M(8);
#undef MMRE_NS_GF_M
#undef MMRE_NS_GF
    }
    MMRE_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_ns_reduce, dim3(1), dim3(256), 0, st, A, part, d_loss);
    MMRE_CHECK_LAUNCH();
    return MMRE_OK;
  }
  float* nrm_e = d_work + w.nrm_e;
  float* nrm_r = d_work + w.nrm_r;
  // norm_flag: the fused kernel reads the rows normalised by the pre-pass; else the tables
  float* ent_n = norm_flag ? d_work + w.ent_n : nullptr;
  float* rel_n = norm_flag ? d_work + w.rel_n : nullptr;
  hipLaunchKernelGGL(k_ns_prepass, dim3((unsigned)((n_ent + n_rel + 3) / 4)), dim3(256), 0, st, d_ent, n_ent, d_rel,
                     n_rel, dim, nrm_e, nrm_r, ent_n, rel_n, S.counts, S.ovf_n);
  MMRE_CHECK_LAUNCH();
  const float* ent_u = norm_flag ? ent_n : d_ent;
  const float* rel_u = norm_flag ? rel_n : d_rel;
  const dim3 grid((unsigned)batch), blk(256);
  const bool l2 = model == MMRE_TRANSE_L2;
  const int nc = transe_fast_nc(A);
#define MMRE_NS_FUSED(NC_, L2_)                                                                                    \
  do {                                                                                                             \
    if (A.regul_rate != 0.0f)                                                                                      \
      hipLaunchKernelGGL((k_ns_transe_fused<NC_, L2_, true>), grid, blk, 0, st, A, nrm_e, nrm_r, d_score, part, S, \
                         n_ent, ent_u, rel_u);                                                                     \
    else                                                                                                           \
      hipLaunchKernelGGL((k_ns_transe_fused<NC_, L2_, false>), grid, blk, 0, st, A, nrm_e, nrm_r, d_score, part,  \
                         S, n_ent, ent_u, rel_u);                                                                  \
  } while (0)
  if (nc == 1) { if (l2) MMRE_NS_FUSED(1, true); else MMRE_NS_FUSED(1, false); }
  else if (nc == 2) { if (l2) MMRE_NS_FUSED(2, true); else MMRE_NS_FUSED(2, false); }
  else if (nc == 4) { if (l2) MMRE_NS_FUSED(4, true); else MMRE_NS_FUSED(4, false); }
  else { if (l2) MMRE_NS_FUSED(8, true); else MMRE_NS_FUSED(8, false); }
#undef MMRE_NS_FUSED
  MMRE_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ns_reduce, dim3(1), dim3(256), 0, st, A, part, d_loss);  // the loss, fixed order
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

static int fused_grad_impl(int model, int norm_flag, float model_margin, int use_model_margin, const float* d_ent,
                           const float* d_ent_im, const float* d_rel, const float* d_rel_im, int64_t n_ent,
                           int64_t n_rel, int dim, float phase_denom, const int64_t* d_h, const int64_t* d_t,
                           const int64_t* d_r, int64_t batch, int64_t neg, float loss_margin, float adv_temperature,
                           float regul_rate, const float* d_score, const float* d_grad_loss, float* d_grad_ent,
                           float* d_grad_ent_im, float* d_grad_rel, float* d_grad_rel_im, float* d_work, float lr,
                           float* pe, float* pei, float* pr, float* pri, void* stream, float* d_loss_out = nullptr,
                           int parity = 0, const NSNext* nxp = nullptr) {
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim,
                   phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature, regul_rate);
  if (rc) return rc;
  if (!d_score || !d_work || !d_grad_ent || !d_grad_rel || n_ent <= 0 || n_rel <= 0) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!d_grad_ent_im || !d_grad_rel_im)) return MMRE_ERR_ARG;
  if (lr != 0.0f && (!pe || !pr || (model == MMRE_COMPLEX && (!pei || !pri)))) return MMRE_ERR_ARG;
  if (neg > NS_MAXK) return MMRE_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  FusedWs w;
  fused_ws(model, norm_flag, batch, neg, n_ent, n_rel, dim, w);
  NSSlots S = ws_slots(d_work, w, n_ent, n_rel, parity);
  const double N = (double)batch * (1.0 + (double)neg);
  const dim3 ogrid((unsigned)((n_ent + n_rel + 3) / 4)), blk(256);
  if (!fused_fast(A)) {
    const int nc = gen_nc(dim);
    if (is_transe(model) || nc == 0) return MMRE_ERR_SHAPE;
    const double nterms = model == MMRE_COMPLEX ? 6.0 : 3.0;
    const double ew = model == MMRE_ROTATE ? 2.0 * dim : (double)dim;
    const float reg_ent = regul_rate != 0.0f ? (float)(regul_rate * 2.0 / (nterms * N * ew)) : 0.0f;
    const float reg_rel = regul_rate != 0.0f ? (float)(regul_rate * 2.0 / (nterms * N * dim)) : 0.0f;
    // DistMult: a workgroup per positive; the two-half models: a wave per positive
    const dim3 sgrid((unsigned)(model == MMRE_DISTMULT ? batch : (batch + NS_WAVES - 1) / NS_WAVES));
    // owner grid: the hub workgroups, then (the one-call step) the loss reduction's workgroup and
    // the next batch's sampler workgroups, then one workgroup per 4 table rows
    NSNext gnx{};
    if (nxp) gnx = *nxp;
    const int64_t gen_reduce = d_loss_out ? (int64_t)NS_HUB_WG : -1;
    gnx.block0 = (int64_t)NS_HUB_WG + (d_loss_out ? 1 : 0);
    const int64_t gen_row0 = gnx.block0 + gnx.n_blocks;
#define MMRE_NS_GEN(NC_)                                                                                            \
  do {                                                                                                              \
    if (model == MMRE_DISTMULT)                                                                                     \
      hipLaunchKernelGGL((k_ns_gen_slots<NC_, MMRE_DISTMULT>), sgrid, blk, 0, st, A, d_score, S, n_ent, w.dpad,     \
                         (int)(regul_rate != 0.0f));                                                                \
    else if (model == MMRE_COMPLEX)                                                                                 \
      hipLaunchKernelGGL((k_ns_gen_slots<NC_, MMRE_COMPLEX>), sgrid, blk, 0, st, A, d_score, S, n_ent, w.dpad,      \
                         (int)(regul_rate != 0.0f));                                                                \
    else                                                                                                            \
      hipLaunchKernelGGL((k_ns_gen_slots<NC_, MMRE_ROTATE>), sgrid, blk, 0, st, A, d_score, S, n_ent, w.dpad,       \
                         (int)(regul_rate != 0.0f));                                                                \
    hipLaunchKernelGGL((k_ns_gen_owner<NC_>), dim3(gen_row0 + ogrid.x), blk, 0, st, A, n_ent, n_rel, reg_ent,        \
                       reg_rel, S.rec, S.counts, S.bucket, S.ovf, S.ovf_n, w.dpad, d_grad_loss, d_grad_ent,          \
                       d_grad_ent_im, d_grad_rel, d_grad_rel_im, lr, pe, pei, pr, pri, gen_row0, NS_HUB_WG, w.slots,  \
                       d_work + w.part, d_loss_out, gen_reduce, gnx);                                               \
  } while (0)
    if (nc == 1) MMRE_NS_GEN(1);
    else if (nc == 2) MMRE_NS_GEN(2);
    else if (nc == 4) MMRE_NS_GEN(4);
    else MMRE_NS_GEN(8);
#undef MMRE_NS_GEN
    MMRE_CHECK_LAUNCH();
    return MMRE_OK;
  }
  const float reg = regul_rate != 0.0f ? (float)(regul_rate * 2.0 / (3.0 * N * dim)) : 0.0f;
  // the training step (d_loss_out): one more workgroup reduces the forward's loss partials
  // the hub workgroups first (their count scan starts with the kernel), then (the training
  // step) the loss reduction's workgroup, then one workgroup per 4 table rows
  // (the pipelined step: then the next batch's sampler workgroups, NSNext)
  NSNext nx{};
  if (nxp) nx = *nxp;
  constexpr bool kSamplerFirst = true;  // the next batch's workgroups before the row workgroups (dispatched early)
  const int64_t reduce_block = d_loss_out ? (int64_t)NS_HUB_WG : -1;
  const int64_t head = (int64_t)NS_HUB_WG + (d_loss_out ? 1 : 0);
  nx.block0 = kSamplerFirst ? head : head + ogrid.x;
  const int64_t row_block0 = kSamplerFirst ? head + nx.n_blocks : head;
  const dim3 ogrid2((unsigned)(head + nx.n_blocks + ogrid.x));
#define MMRE_NS_OWNER(NC_, L2_)                                                                                     \
  hipLaunchKernelGGL((k_ns_row_owner<NC_, L2_>), ogrid2, blk, 0, st, d_ent, d_rel, n_ent, n_rel, dim, norm_flag, reg, \
                     d_work + w.nrm_e, d_work + w.nrm_r, S.shared, S.rec, S.counts, S.bucket, S.ovf, S.ovf_n,         \
                     neg, d_grad_loss, d_grad_ent, d_grad_rel, lr, pe, pr, A, d_work + w.part, d_loss_out,           \
                     reduce_block, row_block0, NS_HUB_WG, w.slots, nx)
  const int nc = transe_fast_nc(A);
  const bool l2 = model == MMRE_TRANSE_L2;
  if (nc == 1) { if (l2) MMRE_NS_OWNER(1, true); else MMRE_NS_OWNER(1, false); }
  else if (nc == 2) { if (l2) MMRE_NS_OWNER(2, true); else MMRE_NS_OWNER(2, false); }
  else if (nc == 4) { if (l2) MMRE_NS_OWNER(4, true); else MMRE_NS_OWNER(4, false); }
  else { if (l2) MMRE_NS_OWNER(8, true); else MMRE_NS_OWNER(8, false); }
#undef MMRE_NS_OWNER
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_ns_fused_grad(int model, int norm_flag, float model_margin, int use_model_margin,
                                  const float* d_ent, const float* d_ent_im, const float* d_rel, const float* d_rel_im,
                                  int64_t n_ent, int64_t n_rel, int dim, float phase_denom, const int64_t* d_h,
                                  const int64_t* d_t, const int64_t* d_r, int64_t batch, int64_t neg,
                                  float loss_margin, float adv_temperature, float regul_rate, const float* d_score,
                                  const float* d_grad_loss, float* d_grad_ent, float* d_grad_ent_im, float* d_grad_rel,
                                  float* d_grad_rel_im, float* d_work, void* stream) {
  return fused_grad_impl(model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, n_ent,
                         n_rel, dim, phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature, regul_rate,
                         d_score, d_grad_loss, d_grad_ent, d_grad_ent_im, d_grad_rel, d_grad_rel_im, d_work, 0.0f,
                         nullptr, nullptr, nullptr, nullptr, stream);
}

extern "C" int mmre_ns_fused_grad_sgd(int model, int norm_flag, float model_margin, int use_model_margin,
                                      float* d_ent, float* d_ent_im, float* d_rel, float* d_rel_im, int64_t n_ent,
                                      int64_t n_rel, int dim, float phase_denom, const int64_t* d_h,
                                      const int64_t* d_t, const int64_t* d_r, int64_t batch, int64_t neg,
                                      float loss_margin, float adv_temperature, float regul_rate,
                                      const float* d_score, const float* d_grad_loss, float* d_grad_ent,
                                      float* d_grad_ent_im, float* d_grad_rel, float* d_grad_rel_im, float* d_work,
                                      float lr, void* stream) {
  if (!(lr != 0.0f)) return MMRE_ERR_ARG;
  return fused_grad_impl(model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, n_ent,
                         n_rel, dim, phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature, regul_rate,
                         d_score, d_grad_loss, d_grad_ent, d_grad_ent_im, d_grad_rel, d_grad_rel_im, d_work, lr, d_ent,
                         d_ent_im, d_rel, d_rel_im, stream);
}

extern "C" int mmre_ns_forward_backward(int model, int norm_flag, float model_margin, int use_model_margin,
                                        const float* d_ent, const float* d_ent_im, const float* d_rel,
                                        const float* d_rel_im, int64_t n_ent, int64_t n_rel, int dim,
                                        float phase_denom, const int64_t* d_h, const int64_t* d_t, const int64_t* d_r,
                                        int64_t batch, int64_t neg, float loss_margin, float adv_temperature,
                                        float regul_rate, float* d_score, float* d_loss, float* d_grad_ent,
                                        float* d_grad_ent_im, float* d_grad_rel, float* d_grad_rel_im, float* d_work,
                                        void* stream) {
  int rc = mmre_ns_fused_forward(model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im,
                                 n_ent, n_rel, dim, phase_denom, d_h, d_t, d_r, batch, neg, loss_margin,
                                 adv_temperature, regul_rate, d_score, d_loss, d_work, stream);
  if (rc) return rc;
  return mmre_ns_fused_grad(model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, n_ent,
                            n_rel, dim, phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature,
                            regul_rate, d_score, nullptr, d_grad_ent, d_grad_ent_im, d_grad_rel, d_grad_rel_im, d_work,
                            stream);
}

// One OpenKE training step (Trainer.train_one_step, Trainer.py:43-54, over Base.cpp's sampling)
// for TransE with the fused path's shapes: sample the batch, margin loss + gradients, plain SGD.
// Three launches: the sampler's workgroups beside the pre-pass (k_ns_step_prep), the fused loss
// kernel, the row owner (gradient + SGD) with the loss reduction as one extra workgroup. Same
// values as mmre_sampler_openke_step + mmre_ns_fused_forward + mmre_ns_fused_grad_sgd (upstream
// gradient 1), bit for bit: the same device functions in the same order, only regrouped into
// fewer launches (tests/test_ns_full_gpu.py holds them equal over several steps).
// The pipelined variant (mmre_ns_step_openke_pipe, `prepared` / `parity` / the next batch):
// launch 1 unless `prepared` is 3 (bit 0: the batch is drawn, bit 1: the pre-pass is current);
// the row owner also samples the next batch into the d_next_* buffers and does its pre-pass
// (NSNext), so the next call with prepared = 3 and the other parity is two launches.
static int step_openke_impl(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                            const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                            const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                            const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                            const float* d_right_mean, uint64_t* d_seeds, int64_t work_threads, int64_t mode,
                            const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h, int64_t* d_batch_t,
                            int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket, int model, int norm_flag,
                            float* d_ent, float* d_rel, int64_t n_ent, int64_t n_rel, int dim, int64_t batch,
                            int64_t neg, float loss_margin, float adv_temperature, float regul_rate, float* d_score,
                            float* d_loss, float* d_grad_ent, float* d_grad_rel, float* d_work, float lr,
                            void* stream, int64_t prepared, int64_t parity, int64_t* d_next_h, int64_t* d_next_t,
                            int64_t* d_next_r, float* d_next_y) {
  if (!d_train_list || !d_head_hrt || !d_tail_hrt || !d_lef_head || !d_rig_head || !d_lef_tail || !d_rig_tail ||
      !d_seeds || !d_batch_h || !d_batch_t || !d_batch_r || !d_batch_y || !d_ticket)
    return MMRE_ERR_ARG;
  if ((d_left_mean == nullptr) != (d_right_mean == nullptr)) return MMRE_ERR_ARG;
  if (train_total <= 0 || n_ent <= 1 || work_threads <= 0 || batch <= 0 || neg <= 0 || mode < -1 || mode > 1)
    return MMRE_ERR_ARG;
  if (n_blocks < 0 || (n_blocks > 0 && !d_blocks)) return MMRE_ERR_ARG;
  if (!d_score || !d_loss || !d_grad_ent || !d_grad_rel || !d_work || n_rel <= 0 || !(lr != 0.0f))
    return MMRE_ERR_ARG;
  const bool pipe = d_next_h != nullptr;
  if (pipe && (!d_next_t || !d_next_r || !d_next_y || d_next_h == d_batch_h)) return MMRE_ERR_ARG;
  if (parity < 0 || parity > 1 || prepared < 0 || prepared > 3) return MMRE_ERR_ARG;
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, 0.0f, 0, d_ent, nullptr, d_rel, nullptr, dim, 0.0f, d_batch_h, d_batch_t,
                   d_batch_r, batch, neg, loss_margin, adv_temperature, regul_rate);
  if (rc) return rc;
  if (!is_transe(model) || !fused_fast(A)) return MMRE_ERR_SHAPE;  // the fused TransE path's shapes only
  hipStream_t st = (hipStream_t)stream;
  FusedWs w;
  fused_ws(model, norm_flag, batch, neg, n_ent, n_rel, dim, w);
  NSSlots S = ws_slots(d_work, w, n_ent, n_rel, (int)parity);
  float* nrm_e = d_work + w.nrm_e;
  float* nrm_r = d_work + w.nrm_r;
  float* ent_n = norm_flag ? d_work + w.ent_n : nullptr;
  float* rel_n = norm_flag ? d_work + w.rel_n : nullptr;
  const int64_t rows = batch * (1 + neg);
  const int64_t n_sampler = (rows + 255) / 256;
  const OpenKESamplerArgs sa{d_train_list, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head, d_rig_head, d_lef_tail,
                             d_rig_tail, d_lef_rel, d_rig_rel, d_left_mean, d_right_mean, train_total, n_ent, n_rel,
                             d_seeds, work_threads, batch, neg, 0, mode, d_blocks, n_blocks, d_batch_h, d_batch_t,
                             d_batch_r, d_batch_y, d_ticket, mmre_sampler_draws_per_positive(neg, 0, mode), nullptr};
  if (prepared != 3) {  // 1. sampler workgroups (unless the batch is drawn) + pre-pass workgroups
    const int64_t ns1 = (prepared & 1) ? 0 : n_sampler;
    hipLaunchKernelGGL(k_ns_step_prep, dim3((unsigned)(ns1 + (n_ent + n_rel + 3) / 4)), dim3(256), 0, st, sa, ns1,
                       d_ent, n_ent, d_rel, n_rel, dim, nrm_e, nrm_r, ent_n, rel_n, S.counts, S.ovf_n);
    MMRE_CHECK_LAUNCH();
  }
  // 2. the fused loss kernel (scores, loss partials, slots)
  const float* ent_u = norm_flag ? ent_n : d_ent;
  const float* rel_u = norm_flag ? rel_n : d_rel;
  const bool l2 = model == MMRE_TRANSE_L2;
  const int nc = transe_fast_nc(A);
  float* part = d_work + w.part;
  const dim3 grid((unsigned)batch), blk(256);
#define MMRE_NS_FUSED(NC_, L2_)                                                                                    \
  do {                                                                                                             \
    if (A.regul_rate != 0.0f)                                                                                      \
      hipLaunchKernelGGL((k_ns_transe_fused<NC_, L2_, true>), grid, blk, 0, st, A, nrm_e, nrm_r, d_score, part, S, \
                         n_ent, ent_u, rel_u);                                                                     \
    else                                                                                                           \
      hipLaunchKernelGGL((k_ns_transe_fused<NC_, L2_, false>), grid, blk, 0, st, A, nrm_e, nrm_r, d_score, part,  \
                         S, n_ent, ent_u, rel_u);                                                                  \
  } while (0)
  if (nc == 1) { if (l2) MMRE_NS_FUSED(1, true); else MMRE_NS_FUSED(1, false); }
  else if (nc == 2) { if (l2) MMRE_NS_FUSED(2, true); else MMRE_NS_FUSED(2, false); }
  else if (nc == 4) { if (l2) MMRE_NS_FUSED(4, true); else MMRE_NS_FUSED(4, false); }
  else { if (l2) MMRE_NS_FUSED(8, true); else MMRE_NS_FUSED(8, false); }
#undef MMRE_NS_FUSED
  MMRE_CHECK_LAUNCH();
  // 3. gradient + SGD, and the loss (+ the pipelined step's next batch and pre-pass)
  NSNext nx{};
  if (pipe) {
    nx.sa = sa;
    nx.sa.bh = d_next_h;
    nx.sa.bt = d_next_t;
    nx.sa.br = d_next_r;
    nx.sa.by = d_next_y;
    nx.n_blocks = n_sampler;
    nx.counts = ws_slots(d_work, w, n_ent, n_rel, (int)(1 - parity)).counts;
    nx.nrm_e = nrm_e;
    nx.nrm_r = nrm_r;
    nx.ent_n = ent_n;
    nx.rel_n = rel_n;
  }
  return fused_grad_impl(model, norm_flag, 0.0f, 0, d_ent, nullptr, d_rel, nullptr, n_ent, n_rel, dim, 0.0f,
                         d_batch_h, d_batch_t, d_batch_r, batch, neg, loss_margin, adv_temperature, regul_rate, d_score,
                         nullptr, d_grad_ent, nullptr, d_grad_rel, nullptr, d_work, lr, d_ent, nullptr, d_rel, nullptr,
                         stream, d_loss, (int)parity, pipe ? &nx : nullptr);
}

// The one-call training step for DistMult / ComplEx / RotatE (the generic fused path), pipelined
// like the TransE one: [the sampler, when the batch was not drawn by the previous call] -> the
// forward (scores, loss partials; it zeroes the slot counts) -> the slot records -> the row owner
// (gradient + SGD, with the loss reduction and the NEXT batch's sampler workgroups in its grid).
// Same kernels and values as OpenKESampler.sample + fused_ns_loss(...).backward() with the SGD
// fused (mmre.optim.SGD), bit for bit; three launches a step instead of five.
static int step_openke_gen_impl(const OpenKESamplerArgs& sa, int64_t n_sampler, int model, float model_margin,
                                int use_model_margin, float* d_ent, float* d_ent_im, float* d_rel, float* d_rel_im,
                                int64_t n_ent, int64_t n_rel, int dim, float phase_denom, int64_t batch, int64_t neg,
                                float loss_margin, float adv_temperature, float regul_rate, float* d_score,
                                float* d_loss, float* d_grad_ent, float* d_grad_ent_im, float* d_grad_rel,
                                float* d_grad_rel_im, float* d_work, float lr, hipStream_t st, int64_t prepared,
                                int64_t* d_next_h, int64_t* d_next_t, int64_t* d_next_r, float* d_next_y) {
  NSArgs A;
  int rc = ns_args(A, model, 0, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim, phase_denom,
                   sa.bh, sa.bt, sa.br, batch, neg, loss_margin, adv_temperature, regul_rate);
  if (rc) return rc;
  const int gnc = gen_nc(dim);
  if (is_transe(model) || gnc == 0 || neg > NS_MAXK) return MMRE_ERR_SHAPE;
  FusedWs w;
  fused_ws(model, 0, batch, neg, n_ent, n_rel, dim, w);
  NSSlots S = ws_slots(d_work, w, n_ent, n_rel);
  float* part = d_work + w.part;
  if (!(prepared & 1)) {  // 1. the batch (the sampler's workgroups alone: no pre-pass for these models)
    hipLaunchKernelGGL(k_ns_step_prep, dim3((unsigned)n_sampler), dim3(256), 0, st, sa, n_sampler, nullptr, n_ent,
                       nullptr, n_rel, dim, nullptr, nullptr, nullptr, nullptr, S.counts, S.ovf_n);
    MMRE_CHECK_LAUNCH();
  }
  // 2. the forward: scores + loss partials (zeroes the slot counts)
  const dim3 fgrid((unsigned)(model == MMRE_DISTMULT ? batch : (batch + NS_WAVES - 1) / NS_WAVES));
#define MMRE_NS_GF(NC_, M_)                                                                                        \
  hipLaunchKernelGGL((k_ns_gen_forward<NC_, M_>), fgrid, dim3(256), 0, st, A, d_score, part, S.counts,             \
                     n_ent + n_rel + 1)
#define MMRE_NS_GF_M(NC_)                                                                                          \
  do {                                                                                                             \
    if (model == MMRE_DISTMULT) MMRE_NS_GF(NC_, MMRE_DISTMULT);                                                    \
    else if (model == MMRE_COMPLEX) MMRE_NS_GF(NC_, MMRE_COMPLEX);                                                 \
    else MMRE_NS_GF(NC_, MMRE_ROTATE);                                                                             \
  } while (0)
  if (gnc == 1) MMRE_NS_GF_M(1);
  else if (gnc == 2) MMRE_NS_GF_M(2);
  else if (gnc == 4) MMRE_NS_GF_M(4);
  else MMRE_NS_GF_M(8);
#undef MMRE_NS_GF_M
#undef MMRE_NS_GF
  MMRE_CHECK_LAUNCH();
  // 3.-4. slots, then the row owner with SGD, the loss reduction and the next batch
  NSNext nx{};
  if (d_next_h) {
    nx.sa = sa;
    nx.sa.bh = d_next_h;
    nx.sa.bt = d_next_t;
    nx.sa.br = d_next_r;
    nx.sa.by = d_next_y;
    nx.n_blocks = n_sampler;
  }
  return fused_grad_impl(model, 0, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, n_ent, n_rel, dim,
                         phase_denom, sa.bh, sa.bt, sa.br, batch, neg, loss_margin, adv_temperature, regul_rate,
                         d_score, nullptr, d_grad_ent, d_grad_ent_im, d_grad_rel, d_grad_rel_im, d_work, lr, d_ent,
                         d_ent_im, d_rel, d_rel_im, st, d_loss, 0, d_next_h ? &nx : nullptr);
}

#define MMRE_STEP_OPENKE_PARAMS                                                                                      \
  const int64_t *d_train_list, int64_t train_total, const int64_t *d_head_hrt, const int64_t *d_tail_hrt,             \
      const int64_t *d_rel_hrt, const int64_t *d_lef_head, const int64_t *d_rig_head, const int64_t *d_lef_tail,      \
      const int64_t *d_rig_tail, const int64_t *d_lef_rel, const int64_t *d_rig_rel, const float *d_left_mean,       \
      const float *d_right_mean, uint64_t *d_seeds, int64_t work_threads, int64_t mode, const int32_t *d_blocks,     \
      int64_t n_blocks, int64_t *d_batch_h, int64_t *d_batch_t, int64_t *d_batch_r, float *d_batch_y,               \
      int32_t *d_ticket, int model, int norm_flag, float *d_ent, float *d_rel, int64_t n_ent, int64_t n_rel, int dim, \
      int64_t batch, int64_t neg, float loss_margin, float adv_temperature, float regul_rate, float *d_score,         \
      float *d_loss, float *d_grad_ent, float *d_grad_rel, float *d_work, float lr, void *stream
#define MMRE_STEP_OPENKE_ARGS                                                                                        \
  d_train_list, train_total, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head, d_rig_head, d_lef_tail, d_rig_tail,     \
      d_lef_rel, d_rig_rel, d_left_mean, d_right_mean, d_seeds, work_threads, mode, d_blocks, n_blocks, d_batch_h,  \
      d_batch_t, d_batch_r, d_batch_y, d_ticket, model, norm_flag, d_ent, d_rel, n_ent, n_rel, dim, batch, neg,      \
      loss_margin, adv_temperature, regul_rate, d_score, d_loss, d_grad_ent, d_grad_rel, d_work, lr, stream

extern "C" int mmre_ns_step_openke(MMRE_STEP_OPENKE_PARAMS) {
  return step_openke_impl(MMRE_STEP_OPENKE_ARGS, 0, 0, nullptr, nullptr, nullptr, nullptr);
}

extern "C" int mmre_ns_step_openke_pipe(MMRE_STEP_OPENKE_PARAMS, int64_t prepared, int64_t parity, int64_t* d_next_h,
                                        int64_t* d_next_t, int64_t* d_next_r, float* d_next_y) {
  return step_openke_impl(MMRE_STEP_OPENKE_ARGS, prepared, parity, d_next_h, d_next_t, d_next_r, d_next_y);
}


// The one-call step for DistMult / ComplEx / RotatE (step_openke_gen_impl): the sampler arguments of
// mmre_ns_step_openke, then the generic model's (ComplEx im tables, RotatE's model margin and phase),
// then prepared (bit 0: d_batch_* already drawn) and the next batch's buffers (nullable).
extern "C" int mmre_ns_step_openke_gen_pipe(
    const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt, const int64_t* d_tail_hrt,
    const int64_t* d_rel_hrt, const int64_t* d_lef_head, const int64_t* d_rig_head, const int64_t* d_lef_tail,
    const int64_t* d_rig_tail, const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
    const float* d_right_mean, uint64_t* d_seeds, int64_t work_threads, int64_t mode, const int32_t* d_blocks,
    int64_t n_blocks, int64_t* d_batch_h, int64_t* d_batch_t, int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket,
    int model, float model_margin, int use_model_margin, float* d_ent, float* d_ent_im, float* d_rel, float* d_rel_im,
    int64_t n_ent, int64_t n_rel, int dim, float phase_denom, int64_t batch, int64_t neg, float loss_margin,
    float adv_temperature, float regul_rate, float* d_score, float* d_loss, float* d_grad_ent, float* d_grad_ent_im,
    float* d_grad_rel, float* d_grad_rel_im, float* d_work, float lr, void* stream, int64_t prepared,
    int64_t* d_next_h, int64_t* d_next_t, int64_t* d_next_r, float* d_next_y) {
  if (!d_train_list || !d_head_hrt || !d_tail_hrt || !d_lef_head || !d_rig_head || !d_lef_tail || !d_rig_tail ||
      !d_seeds || !d_batch_h || !d_batch_t || !d_batch_r || !d_batch_y || !d_ticket)
    return MMRE_ERR_ARG;
  if ((d_left_mean == nullptr) != (d_right_mean == nullptr)) return MMRE_ERR_ARG;
  if (train_total <= 0 || n_ent <= 1 || work_threads <= 0 || batch <= 0 || neg <= 0 || mode < -1 || mode > 1)
    return MMRE_ERR_ARG;
  if (n_blocks < 0 || (n_blocks > 0 && !d_blocks)) return MMRE_ERR_ARG;
  if (!d_score || !d_loss || !d_grad_ent || !d_grad_rel || !d_work || n_rel <= 0 || !(lr != 0.0f)) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!d_ent_im || !d_rel_im || !d_grad_ent_im || !d_grad_rel_im)) return MMRE_ERR_ARG;
  if (prepared < 0 || prepared > 3) return MMRE_ERR_ARG;
  if (d_next_h && (!d_next_t || !d_next_r || !d_next_y || d_next_h == d_batch_h)) return MMRE_ERR_ARG;
  const int64_t n_sampler = (batch * (1 + neg) + 255) / 256;
  const OpenKESamplerArgs sa{d_train_list, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head, d_rig_head, d_lef_tail,
                             d_rig_tail, d_lef_rel, d_rig_rel, d_left_mean, d_right_mean, train_total, n_ent, n_rel,
                             d_seeds, work_threads, batch, neg, 0, mode, d_blocks, n_blocks, d_batch_h, d_batch_t,
                             d_batch_r, d_batch_y, d_ticket, mmre_sampler_draws_per_positive(neg, 0, mode), nullptr};
  return step_openke_gen_impl(sa, n_sampler, model, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im,
                              n_ent, n_rel, dim, phase_denom, batch, neg, loss_margin, adv_temperature, regul_rate,
                              d_score, d_loss, d_grad_ent, d_grad_ent_im, d_grad_rel, d_grad_rel_im, d_work, lr,
                              (hipStream_t)stream, prepared, d_next_h, d_next_t, d_next_r, d_next_y);
}
