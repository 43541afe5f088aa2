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
// workgroup reduces the partials in a fixed order (bit-reproducible loss). The backward
// recomputes each row's intermediates and scatters d(loss)/d(row) into the dense
// gradient tables with float atomics.
#include "mmre_common.h"

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

// g = d(loss)/d(forward score of this row) ; regw = regul_rate * d(loss)/dL scale for the
// regularisation term applied to the raw gathered rows.
__device__ void row_backward(const NSArgs& A, int64_t row, int lane, float g, float reg_ent, float reg_rel,
                             float* gent, float* gent_im, float* grel, float* grel_im) {
  const int d = A.dim;
  const int64_t h = A.h[row], t = A.t[row], r = A.r[row];
  if (A.model == MMRE_TRANSE_L1 || A.model == MMRE_TRANSE_L2) {
    const float *hv = A.ent + h * d, *tv = A.ent + t * d, *rv = A.rel + r * d;
    if (A.use_model_margin) g = -g;  // forward = m - s
    float nh = 1.0f, nt = 1.0f, nr = 1.0f;
    if (A.norm_flag) {
      float a = 0.0f, b = 0.0f, c = 0.0f;
      for (int k = lane; k < d; k += kWave) { a += hv[k] * hv[k]; b += tv[k] * tv[k]; c += rv[k] * rv[k]; }
      nh = sqrtf(wave_sum(a)); nt = sqrtf(wave_sum(b)); nr = sqrtf(wave_sum(c));
    }
    const float ch = fmaxf(nh, 1e-12f), ct = fmaxf(nt, 1e-12f), cr = fmaxf(nr, 1e-12f);
    float s = 0.0f;
    if (A.model == MMRE_TRANSE_L2) {
      for (int k = lane; k < d; k += kWave) {
        const float x = (hv[k] / ch + rv[k] / cr) - tv[k] / ct;
        s += x * x;
      }
      s = sqrtf(wave_sum(s));
    }
    // dL/dx_k = g * sign(x_k) (L1) or g * x_k / s (L2); x = h^ + r^ - t^
    // through y = v / max(|v|, eps): dv = (dy - y (y . dy)) / |v|   (|v| > eps), dy / eps otherwise
    float dh_dot = 0.0f, dt_dot = 0.0f, dr_dot = 0.0f;
    if (A.norm_flag) {
      for (int k = lane; k < d; k += kWave) {
        const float x = (hv[k] / ch + rv[k] / cr) - tv[k] / ct;
        const float gx = A.model == MMRE_TRANSE_L1 ? g * (float)((x > 0.0f) - (x < 0.0f)) : (s > 0.0f ? g * x / s : 0.0f);
        dh_dot += (hv[k] / ch) * gx;
        dr_dot += (rv[k] / cr) * gx;
        dt_dot += (tv[k] / ct) * (-gx);
      }
      dh_dot = wave_sum(dh_dot); dr_dot = wave_sum(dr_dot); dt_dot = wave_sum(dt_dot);
    }
    for (int k = lane; k < d; k += kWave) {
      const float x = (hv[k] / ch + rv[k] / cr) - tv[k] / ct;
      const float gx = A.model == MMRE_TRANSE_L1 ? g * (float)((x > 0.0f) - (x < 0.0f)) : (s > 0.0f ? g * x / s : 0.0f);
      float dh = gx, dr = gx, dt = -gx;
      if (A.norm_flag) {
        dh = nh > 1e-12f ? (dh - (hv[k] / ch) * dh_dot) / nh : dh / 1e-12f;
        dr = nr > 1e-12f ? (dr - (rv[k] / cr) * dr_dot) / nr : dr / 1e-12f;
        dt = nt > 1e-12f ? (dt - (tv[k] / ct) * dt_dot) / nt : dt / 1e-12f;
      }
      atomicAdd(&gent[h * d + k], dh + reg_ent * hv[k]);
      atomicAdd(&gent[t * d + k], dt + reg_ent * tv[k]);
      atomicAdd(&grel[r * d + k], dr + reg_rel * rv[k]);
    }
  } else if (A.model == MMRE_DISTMULT) {
    const float *hv = A.ent + h * d, *tv = A.ent + t * d, *rv = A.rel + r * d;
    for (int k = lane; k < d; k += kWave) {
      atomicAdd(&gent[h * d + k], g * rv[k] * tv[k] + reg_ent * hv[k]);
      atomicAdd(&gent[t * d + k], g * hv[k] * rv[k] + reg_ent * tv[k]);
      atomicAdd(&grel[r * d + k], g * hv[k] * tv[k] + reg_rel * rv[k]);
    }
  } else if (A.model == MMRE_COMPLEX) {
    const float *hr = A.ent + h * d, *hi = A.ent_im + h * d, *tr = A.ent + t * d, *ti = A.ent_im + t * d;
    const float *rr = A.rel + r * d, *ri = A.rel_im + r * d;
    for (int k = lane; k < d; k += kWave) {
      atomicAdd(&gent[h * d + k], g * (tr[k] * rr[k] + ti[k] * ri[k]) + reg_ent * hr[k]);
      atomicAdd(&gent_im[h * d + k], g * (ti[k] * rr[k] - tr[k] * ri[k]) + reg_ent * hi[k]);
      atomicAdd(&gent[t * d + k], g * (hr[k] * rr[k] - hi[k] * ri[k]) + reg_ent * tr[k]);
      atomicAdd(&gent_im[t * d + k], g * (hi[k] * rr[k] + hr[k] * ri[k]) + reg_ent * ti[k]);
      atomicAdd(&grel[r * d + k], g * (hr[k] * tr[k] + hi[k] * ti[k]) + reg_rel * rr[k]);
      atomicAdd(&grel_im[r * d + k], g * (hr[k] * ti[k] - hi[k] * tr[k]) + reg_rel * ri[k]);
    }
  } else {  // RotatE: forward = m - sum_k rho_k
    const float *hv = A.ent + h * 2 * d, *tv = A.ent + t * 2 * d, *rv = A.rel + r * d;
    for (int k = lane; k < d; k += kWave) {
      float s, c;
      const float th = rv[k] / A.phase_denom;
      canon_sincos(th, &s, &c);
      const float hre = hv[k], him = hv[d + k];
      const float re = hre * c - him * s - tv[k];
      const float im = hre * s + him * c - tv[d + k];
      const float rho = sqrtf(re * re + im * im);
      const float ga = rho > 0.0f ? -g * re / rho : 0.0f;  // dL/d re
      const float gb = rho > 0.0f ? -g * im / rho : 0.0f;  // dL/d im
      atomicAdd(&gent[h * 2 * d + k], ga * c + gb * s + reg_ent * hre);
      atomicAdd(&gent[h * 2 * d + d + k], -ga * s + gb * c + reg_ent * him);
      atomicAdd(&gent[t * 2 * d + k], -ga + reg_ent * tv[k]);
      atomicAdd(&gent[t * 2 * d + d + k], -gb + reg_ent * tv[d + k]);
      const float dth = ga * (-hre * s - him * c) + gb * (hre * c - him * s);
      atomicAdd(&grel[r * d + k], dth / A.phase_denom + reg_rel * rv[k]);
    }
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
__global__ __launch_bounds__(256) void k_ns_forward(NSArgs A, float* __restrict__ score, float* __restrict__ part) {
  __shared__ float s_n[NS_WAVES][NS_MAXK];
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

// Fixed-order reduction of the per-positive partials (bit-reproducible loss).
__global__ __launch_bounds__(256) void k_ns_reduce(NSArgs A, const float* __restrict__ part, float* __restrict__ loss) {
  __shared__ double red[7][256];
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int64_t b = threadIdx.x; b < A.B; b += blockDim.x)
    for (int i = 0; i < 7; ++i) acc[i] += part[b * 7 + i];
  for (int i = 0; i < 7; ++i) red[i][threadIdx.x] = acc[i];
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int i = 0; i < 7; ++i) red[i][threadIdx.x] += red[i][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double Bd = (double)A.B, Kd = (double)A.K;
    double l = A.adv_t > 0.0f ? red[0][0] / Bd : red[0][0] / (Bd * Kd);
    l += A.loss_margin;
    if (A.regul_rate != 0.0f) {
      const double N = Bd * (1.0 + Kd);
      const double d = (double)A.dim;
      const double ew = A.model == MMRE_ROTATE ? 2.0 * d : d;
      double reg;
      if (A.model == MMRE_COMPLEX)
        reg = (red[1][0] / (N * d) + red[4][0] / (N * d) + red[2][0] / (N * d) + red[5][0] / (N * d) +
               red[3][0] / (N * d) + red[6][0] / (N * d)) / 6.0;
      else
        reg = (red[1][0] / (N * ew) + red[2][0] / (N * ew) + red[3][0] / (N * d)) / 3.0;
      l += (double)A.regul_rate * reg;
    }
    loss[0] = (float)l;
  }
}

__global__ __launch_bounds__(256) void k_ns_backward(NSArgs A, const float* __restrict__ score,
                                                      const float* __restrict__ grad_loss, float* gent, float* gent_im,
                                                      float* grel, float* grel_im) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * NS_WAVES + (threadIdx.x >> 6);
  if (b >= A.B) return;
  const float G = grad_loss[0];
  const float p = score[b];
  float mx = -INFINITY, den = 0.0f;
  if (A.adv_t > 0.0f) {
    for (int64_t j = 0; j < A.K; ++j) mx = fmaxf(mx, -score[b + (j + 1) * A.B] * A.adv_t);
    for (int64_t j = 0; j < A.K; ++j) den += expf(-score[b + (j + 1) * A.B] * A.adv_t - mx);
  }
  // regularization gradient scale: regul_rate * (1/3 or 1/6) * 2 v / (N * width)
  const double N = (double)A.B * (1.0 + (double)A.K);
  const int ew = A.model == MMRE_ROTATE ? 2 * A.dim : A.dim;
  const float nterms = A.model == MMRE_COMPLEX ? 6.0f : 3.0f;
  const float reg_ent = A.regul_rate != 0.0f ? (float)(G * A.regul_rate * 2.0 / (nterms * N * ew)) : 0.0f;
  const float reg_rel = A.regul_rate != 0.0f ? (float)(G * A.regul_rate * 2.0 / (nterms * N * A.dim)) : 0.0f;
  float gp = 0.0f;
  for (int64_t j = 0; j < A.K; ++j) {
    const float n = score[b + (j + 1) * A.B];
    const float x = p - n, m = -A.loss_margin;
    const float ind = x > m ? 1.0f : (x == m ? 0.5f : 0.0f);  // maximum(): ties split the gradient
    const float c = A.adv_t > 0.0f ? G * (expf(-n * A.adv_t - mx) / den) / (float)A.B : G / (float)(A.B * A.K);
    gp += c * ind;
    row_backward(A, b + (j + 1) * A.B, lane, -c * ind, reg_ent, reg_rel, gent, gent_im, grel, grel_im);
  }
  row_backward(A, b, lane, gp, reg_ent, reg_rel, gent, gent_im, grel, grel_im);
}

// model(data) backward for arbitrary rows: dL/d(score of row i) = grad_score[i] (one wave per row).
__global__ __launch_bounds__(256) void k_rows_backward(NSArgs A, const float* __restrict__ grad_score, float* gent,
                                                       float* gent_im, float* grel, float* grel_im) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * NS_WAVES + (threadIdx.x >> 6);
  if (row >= A.B) return;
  const float g = grad_score[row];
  if (g != 0.0f) row_backward(A, row, lane, g, 0.0f, 0.0f, gent, gent_im, grel, grel_im);
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
  hipLaunchKernelGGL(k_ns_forward, dim3((unsigned)((batch + NS_WAVES - 1) / NS_WAVES)), dim3(256), 0, st, A, d_score,
                     d_work);
  MMRE_CHECK_LAUNCH();
  if (d_loss) {
    hipLaunchKernelGGL(k_ns_reduce, dim3(1), dim3(256), 0, st, A, d_work, d_loss);
    MMRE_CHECK_LAUNCH();
  }
  return MMRE_OK;
}

extern "C" int mmre_ns_backward(int model, int norm_flag, float model_margin, int use_model_margin,
                                const float* d_ent, const float* d_ent_im, const float* d_rel, const float* d_rel_im,
                                int dim, float phase_denom, const int64_t* d_h, const int64_t* d_t,
                                const int64_t* d_r, int64_t batch, int64_t neg, float loss_margin,
                                float adv_temperature, float regul_rate, const float* d_score,
                                const float* d_grad_loss, float* d_grad_ent, float* d_grad_ent_im, float* d_grad_rel,
                                float* d_grad_rel_im, float* d_work, void* stream) {
  (void)d_work;
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim,
                   phase_denom, d_h, d_t, d_r, batch, neg, loss_margin, adv_temperature, regul_rate);
  if (rc) return rc;
  if (!d_score || !d_grad_loss || !d_grad_ent || !d_grad_rel) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!d_grad_ent_im || !d_grad_rel_im)) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_ns_backward, dim3((unsigned)((batch + NS_WAVES - 1) / NS_WAVES)), dim3(256), 0, st, A,
                     d_score, d_grad_loss, d_grad_ent, d_grad_ent_im, d_grad_rel, d_grad_rel_im);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_score_rows_backward(int model, int norm_flag, float model_margin, int use_model_margin,
                                        const float* d_ent, const float* d_ent_im, const float* d_rel,
                                        const float* d_rel_im, int dim, float phase_denom, const int64_t* d_h,
                                        const int64_t* d_t, const int64_t* d_r, int64_t n_rows,
                                        const float* d_grad_score, float* d_grad_ent, float* d_grad_ent_im,
                                        float* d_grad_rel, float* d_grad_rel_im, void* stream) {
  NSArgs A;
  int rc = ns_args(A, model, norm_flag, model_margin, use_model_margin, d_ent, d_ent_im, d_rel, d_rel_im, dim,
                   phase_denom, d_h, d_t, d_r, n_rows, 0, 0.0f, 0.0f, 0.0f);
  if (rc) return rc;
  if (!d_grad_score || !d_grad_ent || !d_grad_rel) return MMRE_ERR_ARG;
  if (model == MMRE_COMPLEX && (!d_grad_ent_im || !d_grad_rel_im)) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_rows_backward, dim3((unsigned)((n_rows + NS_WAVES - 1) / NS_WAVES)), dim3(256), 0, st, A,
                     d_grad_score, d_grad_ent, d_grad_ent_im, d_grad_rel, d_grad_rel_im);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
