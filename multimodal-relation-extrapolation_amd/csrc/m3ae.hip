// m3ae.hip -- the frozen M3AE text encoder that turns relation descriptions into the CLS
// vector the generator consumes (UnifiedModel.generate / forward_relation_emb,
// module/model.py:599-604, 674-679 -> MaskedMultimodalAutoencoder.forward_representation,
// text branch, model.py:323-356 -> Transformer / Block / Attention / TransformerMLP,
// module/submodule.py:128-238). SURVEY 8(f) rank 4.
//
// Reference computation per description row (deterministic=True, dropout / drop-path off):
//   x = cat([cls_token, (text_embedding[tok] + pos_sincos[p]) + type_emb])    (n = 1 + len rows)
//   per block:  x = x + fc(attn(qkv(LN1(x))))                                  (submodule.py:205-209)
//               x = x + fc2(gelu(fc1(LN2(x))))                                 (submodule.py:211-214)
//   attn: s = (q k^T) * hd^-0.5; s[:, pad] = -1e7; softmax; . v                (submodule.py:164-186)
//   cls = LN_final(x)[0]                                                      (submodule.py:237, model.py:354)
//
// MI355X design -- padding-free and CLS-only where the math allows it, both exact:
//  * A padded token (mask > 0) is a key whose logit is -1e7, so its softmax weight
//    exp(-1e7 - max) is exactly 0 in fp32, and every other op is row-wise: padded rows never
//    reach an unpadded row. Only the CLS row and the unpadded tokens are computed, packed
//    back to back over all sequences ("rows", CSR offsets d_off), so a 12-token description
//    costs 13 rows, not the reference's 321.
//  * Only the CLS row leaves the encoder, so the last block runs attention / fc / MLP /
//    final LN on the CLS rows alone (K and V of every row are still formed).
// Kernels:
//   k_m3ae_count / k_m3ae_scan   rows per sequence (1 + unpadded tokens) -> offsets
//   k_m3ae_embed                 one workgroup per sequence: compaction + embedding sum
//   k_m3ae_ln<V>                 nn.LayerNorm (biased var, eps), one wave per row
//   k_m3ae_linear<EPI>           C = A W^T + b (+GELU | +residual), fp32 MFMA
//                                v_mfma_f32_32x32x2_f32, 64 x 128 tiles, K staged 32 deep
//                                through double-buffered LDS (conflict-free k-major writes)
//   k_m3ae_attn<HD>              one workgroup per (sequence, head, 16 query rows): full
//                                logit rows in LDS, exact two-pass softmax, . v
//   k_m3ae_gather_cls            x[off[b]] -> compact CLS rows (last block)
#include <math.h>

#include "mmre_common.h"

namespace mmre {
namespace {

constexpr int M3_MAXLEN = 335;  // tokens per description row (attention keeps 1 + len logits per row in LDS)
constexpr int M3_AQ = 16;       // query rows per attention workgroup
constexpr int M3_AKC = 64;      // keys per staged K / V chunk
constexpr int M3_MAXR = 336;    // 1 + M3_MAXLEN

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) v += __shfl_xor(v, sh);
  return v;
}

// rows[b] = 1 + #{p : !(mask[b][p] > 0)} (torch.where(padding_mask > 0, -1e7, .) masks exactly
// the entries with mask > 0, submodule.py:174-177). One wave per sequence.
__global__ __launch_bounds__(256) void k_m3ae_count(const float* __restrict__ mask, int64_t n_seq, int64_t len,
                                                    int32_t* __restrict__ off) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= n_seq) return;
  int c = 0;
  for (int64_t p = lane; p < len; p += 64) c += !(mask[b * len + p] > 0.0f);
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) c += __shfl_xor(c, sh);
  if (lane == 0) off[b + 1] = 1 + c;
}

// Inclusive scan of off[1..n] in place (off[0] = 0); one 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_m3ae_scan(int32_t* __restrict__ off, int64_t n) {
  __shared__ int32_t s_w[16];
  __shared__ int32_t s_carry;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) {
    s_carry = 0;
    off[0] = 0;
  }
  __syncthreads();
  for (int64_t c0 = 0; c0 < n; c0 += 1024) {
    const int64_t i = c0 + tid;
    int x = i < n ? off[i + 1] : 0;
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const int y = __shfl_up(x, sh);
      if (lane >= sh) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    int pre = s_carry;
    for (int k = 0; k < w; ++k) pre += s_w[k];
    if (i < n) off[i + 1] = pre + x;
    __syncthreads();
    if (tid == 1023) s_carry = pre + x;
    __syncthreads();
  }
}

// One workgroup per sequence: list the unpadded positions in order (ballot prefix), then
// write row off[b] = cls_token and row off[b] + 1 + i = (emb[tok] + pos[p]) + type for the
// i-th unpadded position p (model.py:341-351, same fp32 association). A token id outside
// [0, vocab) yields a NaN row (never an out-of-bounds read); the host checks ids first.
__global__ __launch_bounds__(256) void k_m3ae_embed(const int32_t* __restrict__ tokens, const float* __restrict__ mask,
                                                    int64_t len, const int32_t* __restrict__ off,
                                                    const float* __restrict__ emb, int64_t vocab,
                                                    const float* __restrict__ pos, const float* __restrict__ type_emb,
                                                    const float* __restrict__ cls, int d, float* __restrict__ x) {
  __shared__ int32_t s_pos[M3_MAXLEN + 256];
  __shared__ int32_t s_w[4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int base = 0;
  for (int64_t c0 = 0; c0 < len; c0 += 256) {
    const int64_t p = c0 + tid;
    const bool v = p < len && !(mask[b * len + p] > 0.0f);
    const uint64_t bal = __ballot(v);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) s_w[w] = __popcll(bal);
    __syncthreads();
    int wb = 0;
    for (int k = 0; k < w; ++k) wb += s_w[k];
    const int tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    if (v) s_pos[base + wb + pre] = (int32_t)p;
    base += tot;
    __syncthreads();
  }
  const int64_t r0 = off[b];
  for (int k = tid; k < d; k += 256) x[r0 * d + k] = cls[k];
  for (int i = 0; i < base; ++i) {
    const int p = s_pos[i];
    const int32_t id = tokens[b * len + p];
    const bool ok = id >= 0 && (int64_t)id < vocab;
    const float* er = emb + (ok ? (int64_t)id : 0) * d;
    const float* pr = pos + (int64_t)p * d;
    float* xr = x + (r0 + 1 + i) * d;
    for (int k = tid; k < d; k += 256) xr[k] = ok ? (er[k] + pr[k]) + type_emb[k] : __int_as_float(0x7fc00000);
  }
}

// nn.LayerNorm over D = 64 V: y = (x - mean) / sqrt(var + eps) * w + b, biased variance.
// One wave per row, 4 rows per workgroup.
template <int V>
__global__ __launch_bounds__(256) void k_m3ae_ln(const float* __restrict__ x, int64_t n, const float* __restrict__ w,
                                                 const float* __restrict__ bb, float eps, float* __restrict__ y) {
  constexpr int D = 64 * V;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const float* xr = x + r * D;
  float v[V];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    v[i] = xr[lane + 64 * i];
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float t = v[i] - mean;
    q += t * t;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
  float* yr = y + r * D;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int k = lane + 64 * i;
    yr[k] = (v[i] - mean) * rstd * w[k] + bb[k];
  }
}

// C (M x N) = A (M x K) . W (N x K)^T + bias, then EPI: 0 none, 1 GELU (erf form, F.gelu),
// 2 C = resid + C (resid may alias C: each element is read and written by one lane).
// 256 threads = 4 waves as 2 (m) x 2 (n); a wave owns 32 x 64 = two 32 x 32 MFMA blocks.
// N % 128 == 0, K % 32 == 0 (checked by the host entry).
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int LM = 64, LN = 128, LK = 32;

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_m3ae_linear(const float* __restrict__ A, int64_t M, int K,
                                                        const float* __restrict__ W, int N,
                                                        const float* __restrict__ bias, const float* resid,
                                                        float* out) {
  __shared__ float sA[2][LK][LM];
  __shared__ float sB[2][LK][LN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lrow = lane >> 5, lcol = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * LM;
  const int n0 = blockIdx.y * LN;
  const int ar = tid & 63, ak = tid >> 6;   // A stage: row ar, k quads ak and ak + 4
  const int br = tid & 127, bk = tid >> 7;  // B stage: row br, k quads bk, bk + 2, bk + 4, bk + 6
  const bool a_ok = m0 + ar < M;
  const float* Ap = A + (a_ok ? (m0 + ar) * (int64_t)K : 0);
  const float* Bp = W + (int64_t)(n0 + br) * K;
  float4 ra0, ra1, rb0, rb1, rb2, rb3;
  auto gload = [&](int kt) {
    const int k0 = kt * LK;
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    ra0 = a_ok ? *reinterpret_cast<const float4*>(Ap + k0 + 4 * ak) : z;
    ra1 = a_ok ? *reinterpret_cast<const float4*>(Ap + k0 + 4 * (ak + 4)) : z;
    rb0 = *reinterpret_cast<const float4*>(Bp + k0 + 4 * bk);
    rb1 = *reinterpret_cast<const float4*>(Bp + k0 + 4 * (bk + 2));
    rb2 = *reinterpret_cast<const float4*>(Bp + k0 + 4 * (bk + 4));
    rb3 = *reinterpret_cast<const float4*>(Bp + k0 + 4 * (bk + 6));
  };
  auto swrite = [&](int buf) {
    // k-major LDS: the 64 lanes of a wave write 64 consecutive columns of one k row
    sA[buf][4 * ak][ar] = ra0.x;
    sA[buf][4 * ak + 1][ar] = ra0.y;
    sA[buf][4 * ak + 2][ar] = ra0.z;
    sA[buf][4 * ak + 3][ar] = ra0.w;
    sA[buf][4 * ak + 16][ar] = ra1.x;
    sA[buf][4 * ak + 17][ar] = ra1.y;
    sA[buf][4 * ak + 18][ar] = ra1.z;
    sA[buf][4 * ak + 19][ar] = ra1.w;
    const float4 rb[4] = {rb0, rb1, rb2, rb3};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 4 * (bk + 2 * i);
      sB[buf][k][br] = rb[i].x;
      sB[buf][k + 1][br] = rb[i].y;
      sB[buf][k + 2][br] = rb[i].z;
      sB[buf][k + 3][br] = rb[i].w;
    }
  };

  floatx16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc0[r] = 0.0f;
    acc1[r] = 0.0f;
  }
  const int nkt = K / LK;
  gload(0);
  swrite(0);
  __syncthreads();
  int buf = 0;
  for (int kt = 0; kt < nkt; ++kt) {
    const bool more = kt + 1 < nkt;
    if (more) gload(kt + 1);
#pragma unroll
    for (int kk = 0; kk < LK; kk += 2) {
      const float a = sA[buf][kk + lrow][wm * 32 + lcol];
      const float b0 = sB[buf][kk + lrow][wn * 64 + lcol];
      const float b1 = sB[buf][kk + lrow][wn * 64 + 32 + lcol];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
    }
    if (more) swrite(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
    const int n = n0 + wn * 64 + bj * 32 + lcol;
    const float bn = bias[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lrow;
      if (m < M) {
        float v = (bj ? acc1[r] : acc0[r]) + bn;
        if constexpr (EPI == 1) v = (v * 0.5f) * (1.0f + erff(v * 0.70710678118654752f));
        if constexpr (EPI == 2) v = resid[m * N + n] + v;
        out[m * N + n] = v;
      }
    }
  }
}

// Multi-head attention of one (sequence b, head h, block of M3_AQ query rows) over the
// sequence's rows [off[b], off[b+1]) of qkv (row layout [q | k | v], each heads x HD:
// qkv.view(B, n, 3, heads, HD), submodule.py:166-169). Logits s = (q . k) * scale for all
// keys are kept in LDS, then softmax = exp(s - max) / sum (two passes over the row), then
// out[:, h*HD + c] = sum_j p_j v_j[c] (the permute/reshape of :183). cls_only: only query
// row 0 of each sequence, written to out row b (the last block).
template <int HD>
__global__ __launch_bounds__(256) void k_m3ae_attn(const float* __restrict__ qkv, const int32_t* __restrict__ off,
                                                   int heads, float scale, int cls_only, float* __restrict__ out) {
  constexpr int HP = HD + 1;  // padded row stride: the 16 lanes of a row group hit distinct banks
  __shared__ float sQ[M3_AQ][HP];
  __shared__ float sKV[M3_AKC][HP];
  __shared__ float sS[M3_AQ][M3_MAXR];
  const int b = blockIdx.z, h = blockIdx.y;
  const int r0 = off[b], nrow = off[b + 1] - r0;
  const int q0 = blockIdx.x * M3_AQ;
  const int nq = cls_only ? 1 : min(M3_AQ, nrow - q0);
  if (nq <= 0) return;  // uniform
  const int D = heads * HD, D3 = 3 * D;
  const int tid = threadIdx.x;
  const int qi = tid >> 4, sub = tid & 15;  // query row of this thread, lane within its 16-lane row group

  for (int e = tid; e < M3_AQ * HD; e += 256) {
    const int i = e / HD, c = e % HD;
    sQ[i][c] = i < nq ? qkv[(int64_t)(r0 + q0 + i) * D3 + h * HD + c] : 0.0f;
  }
  // pass 1: logits of every key
  for (int kc = 0; kc < nrow; kc += M3_AKC) {
    const int nk = min(M3_AKC, nrow - kc);
    __syncthreads();  // sQ written / previous chunk's readers done
    for (int e = tid; e < M3_AKC * HD; e += 256) {
      const int j = e / HD, c = e % HD;
      sKV[j][c] = j < nk ? qkv[(int64_t)(r0 + kc + j) * D3 + D + h * HD + c] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < M3_AKC / 16; ++jj) {
      const int j = sub + 16 * jj;
      float s = 0.0f;
#pragma unroll 8
      for (int c = 0; c < HD; ++c) s = __builtin_fmaf(sQ[qi][c], sKV[j][c], s);
      if (j < nk) sS[qi][kc + j] = s * scale;
    }
  }
  __syncthreads();
  // softmax of each row, 16 lanes per row
  float mx = -INFINITY;
  for (int j = sub; j < nrow; j += 16) mx = fmaxf(mx, sS[qi][j]);
#pragma unroll
  for (int sh = 8; sh >= 1; sh >>= 1) mx = fmaxf(mx, __shfl_xor(mx, sh));
  float sum = 0.0f;
  for (int j = sub; j < nrow; j += 16) {
    const float e = expf(sS[qi][j] - mx);
    sS[qi][j] = e;
    sum += e;
  }
#pragma unroll
  for (int sh = 8; sh >= 1; sh >>= 1) sum += __shfl_xor(sum, sh);
  const float inv = 1.0f / sum;
  // pass 2: p . v; this thread owns columns c = sub + 16 cc of row qi
  constexpr int NC = HD / 16;
  float o[NC];
#pragma unroll
  for (int cc = 0; cc < NC; ++cc) o[cc] = 0.0f;
  for (int kc = 0; kc < nrow; kc += M3_AKC) {
    const int nk = min(M3_AKC, nrow - kc);
    __syncthreads();  // softmax writes to sS / previous chunk's readers done
    for (int e = tid; e < M3_AKC * HD; e += 256) {
      const int j = e / HD, c = e % HD;
      sKV[j][c] = j < nk ? qkv[(int64_t)(r0 + kc + j) * D3 + 2 * D + h * HD + c] : 0.0f;
    }
    __syncthreads();
    for (int j = 0; j < nk; ++j) {
      const float p = sS[qi][kc + j] * inv;
#pragma unroll
      for (int cc = 0; cc < NC; ++cc) o[cc] = __builtin_fmaf(p, sKV[j][sub + 16 * cc], o[cc]);
    }
  }
  if (qi < nq) {
    const int64_t row = cls_only ? (int64_t)b : (int64_t)(r0 + q0 + qi);
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) out[row * D + h * HD + sub + 16 * cc] = o[cc];
  }
}

__global__ __launch_bounds__(256) void k_m3ae_gather_cls(const float* __restrict__ x, const int32_t* __restrict__ off,
                                                         int64_t n_seq, int d, float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_seq * d) return;
  const int64_t b = i / d, k = i % d;
  y[i] = x[(int64_t)off[b] * d + k];
}

int launch_ln(const float* x, int64_t n, int d, const float* w, const float* b, float eps, float* y, hipStream_t st) {
  if (n <= 0) return MMRE_OK;
  const dim3 g((unsigned)((n + 3) / 4));
  switch (d) {
    case 384: hipLaunchKernelGGL(k_m3ae_ln<6>, g, dim3(256), 0, st, x, n, w, b, eps, y); break;
    case 768: hipLaunchKernelGGL(k_m3ae_ln<12>, g, dim3(256), 0, st, x, n, w, b, eps, y); break;
    case 1024: hipLaunchKernelGGL(k_m3ae_ln<16>, g, dim3(256), 0, st, x, n, w, b, eps, y); break;
    case 1280: hipLaunchKernelGGL(k_m3ae_ln<20>, g, dim3(256), 0, st, x, n, w, b, eps, y); break;
    default: return MMRE_ERR_SHAPE;
  }
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

int launch_linear(int epi, const float* A, int64_t M, int K, const float* W, int N, const float* bias,
                  const float* resid, float* out, hipStream_t st) {
  if (M < 0 || K <= 0 || N <= 0 || K % LK || N % LN || M > 0x7fffffffLL * LM) return MMRE_ERR_SHAPE;
  if (!A || !W || !bias || !out || (epi == 2 && !resid)) return MMRE_ERR_ARG;
  if (M == 0) return MMRE_OK;
  const dim3 g((unsigned)((M + LM - 1) / LM), (unsigned)(N / LN));
  switch (epi) {
    case 0: hipLaunchKernelGGL(k_m3ae_linear<0>, g, dim3(256), 0, st, A, M, K, W, N, bias, resid, out); break;
    case 1: hipLaunchKernelGGL(k_m3ae_linear<1>, g, dim3(256), 0, st, A, M, K, W, N, bias, resid, out); break;
    case 2: hipLaunchKernelGGL(k_m3ae_linear<2>, g, dim3(256), 0, st, A, M, K, W, N, bias, resid, out); break;
    default: return MMRE_ERR_ARG;
  }
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

int launch_attn(const float* qkv, const int32_t* off, int64_t n_seq, int max_rows, int heads, int hd, float scale,
                int cls_only, float* out, hipStream_t st) {
  if (n_seq <= 0) return MMRE_OK;
  if (max_rows < 1 || max_rows > M3_MAXR || n_seq > 65535 || heads < 1 || heads > 1024) return MMRE_ERR_SHAPE;
  const dim3 g(cls_only ? 1u : (unsigned)((max_rows + M3_AQ - 1) / M3_AQ), (unsigned)heads, (unsigned)n_seq);
  switch (hd) {
    case 64: hipLaunchKernelGGL(k_m3ae_attn<64>, g, dim3(256), 0, st, qkv, off, heads, scale, cls_only, out); break;
    case 80: hipLaunchKernelGGL(k_m3ae_attn<80>, g, dim3(256), 0, st, qkv, off, heads, scale, cls_only, out); break;
    default: return MMRE_ERR_SHAPE;
  }
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

#define M3_TRY(expr)                \
  do {                              \
    int _rc = (expr);               \
    if (_rc != MMRE_OK) return _rc; \
  } while (0)

bool m3ae_dims_ok(int d, int heads) {
  return (d == 384 || d == 768 || d == 1024 || d == 1280) && heads > 0 && d % heads == 0 &&
         (d / heads == 64 || d / heads == 80);
}

}  // namespace
}  // namespace mmre

using namespace mmre;

extern "C" int mmre_m3ae_max_len(void) { return M3_MAXLEN; }

extern "C" int mmre_m3ae_rows(const float* d_mask, int64_t n_seq, int64_t len, int32_t* d_off, void* stream) {
  if (n_seq < 0 || len < 0 || len > M3_MAXLEN || !d_off || (n_seq > 0 && len > 0 && !d_mask)) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n_seq > 0)
    hipLaunchKernelGGL(k_m3ae_count, dim3((unsigned)((n_seq + 3) / 4)), dim3(256), 0, st, d_mask, n_seq, len, d_off);
  hipLaunchKernelGGL(k_m3ae_scan, dim3(1), dim3(1024), 0, st, d_off, n_seq);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int64_t mmre_m3ae_workspace(int64_t n_rows, int64_t n_seq, int d) {
  if (n_rows < 0 || n_seq < 0 || d <= 0) return -1;
  // x | xn | qkv | att | hidden (4d) over the rows, then x_cls | xn_cls | att_cls | hidden_cls
  return n_rows * (int64_t)d * (1 + 1 + 3 + 1 + 4) + n_seq * (int64_t)d * (1 + 1 + 1 + 4);
}

extern "C" int mmre_m3ae_layernorm(const float* d_x, int64_t n_rows, int d, const float* d_w, const float* d_b,
                                   float eps, float* d_y, void* stream) {
  if (n_rows < 0 || !d_x || !d_w || !d_b || !d_y) return MMRE_ERR_ARG;
  return launch_ln(d_x, n_rows, d, d_w, d_b, eps, d_y, (hipStream_t)stream);
}

extern "C" int mmre_m3ae_linear(int epilogue, const float* d_a, int64_t m, int k, const float* d_w, int n,
                                const float* d_bias, const float* d_resid, float* d_out, void* stream) {
  return launch_linear(epilogue, d_a, m, k, d_w, n, d_bias, d_resid, d_out, (hipStream_t)stream);
}

extern "C" int mmre_m3ae_attention(const float* d_qkv, const int32_t* d_off, int64_t n_seq, int max_rows, int heads,
                                   int head_dim, float scale, int cls_only, float* d_out, void* stream) {
  if (!d_qkv || !d_off || !d_out) return MMRE_ERR_ARG;
  return launch_attn(d_qkv, d_off, n_seq, max_rows, heads, head_dim, scale, cls_only, d_out, (hipStream_t)stream);
}

extern "C" int mmre_m3ae_encode(const float* const* h_params, int depth, int d, int heads, float ln_eps,
                                const int32_t* d_tokens, const float* d_mask, int64_t n_seq, int64_t len,
                                int64_t vocab, const int32_t* d_off, int64_t n_rows, int max_rows, float* d_work,
                                int64_t work_floats, float* d_cls, void* stream) {
  if (!h_params || depth < 1 || !m3ae_dims_ok(d, heads)) return MMRE_ERR_SHAPE;
  if (n_seq < 0 || len < 0 || len > M3_MAXLEN || n_rows < n_seq || max_rows < 1 || max_rows > len + 1 || !d_off ||
      !d_work || !d_cls || vocab <= 0 || (n_seq > 0 && (!d_tokens || !d_mask)))
    return MMRE_ERR_ARG;
  if (work_floats < mmre_m3ae_workspace(n_rows, n_seq, d)) return MMRE_ERR_WORKSPACE;
  for (int i = 0; i < 4 + 12 * depth + 2; ++i)
    if (!h_params[i]) return MMRE_ERR_ARG;
  if (n_seq == 0) return MMRE_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t R = n_rows, S = n_seq;
  const int hd = d / heads, d3 = 3 * d, d4 = 4 * d;
  const float scale = 1.0f / sqrtf((float)hd);  // (dim // num_heads) ** -0.5 (submodule.py:156): 0.125 at hd 64
  float* x = d_work;
  float* xn = x + R * d;
  float* qkv = xn + R * d;
  float* att = qkv + R * d3;
  float* hid = att + R * d;
  float* xc = hid + R * d4;
  float* xnc = xc + S * d;
  float* attc = xnc + S * d;
  float* hidc = attc + S * d;

  hipLaunchKernelGGL(k_m3ae_embed, dim3((unsigned)S), dim3(256), 0, st, d_tokens, d_mask, len, d_off, h_params[0],
                     vocab, h_params[1], h_params[2], h_params[3], d, x);
  MMRE_CHECK_LAUNCH();
  for (int l = 0; l < depth; ++l) {
    const float* const* p = h_params + 4 + 12 * l;
    // p: ln1 w, b | qkv w, b | fc w, b | ln2 w, b | fc1 w, b | fc2 w, b
    M3_TRY(launch_ln(x, R, d, p[0], p[1], ln_eps, xn, st));
    M3_TRY(launch_linear(0, xn, R, d, p[2], d3, p[3], nullptr, qkv, st));
    if (l + 1 < depth) {
      M3_TRY(launch_attn(qkv, d_off, S, max_rows, heads, hd, scale, 0, att, st));
      M3_TRY(launch_linear(2, att, R, d, p[4], d, p[5], x, x, st));
      M3_TRY(launch_ln(x, R, d, p[6], p[7], ln_eps, xn, st));
      M3_TRY(launch_linear(1, xn, R, d, p[8], d4, p[9], nullptr, hid, st));
      M3_TRY(launch_linear(2, hid, R, d4, p[10], d, p[11], x, x, st));
    } else {  // last block: only the CLS rows go on
      M3_TRY(launch_attn(qkv, d_off, S, max_rows, heads, hd, scale, 1, attc, st));
      hipLaunchKernelGGL(k_m3ae_gather_cls, dim3((unsigned)((S * d + 255) / 256)), dim3(256), 0, st, x, d_off, S, d,
                         xc);
      MMRE_CHECK_LAUNCH();
      M3_TRY(launch_linear(2, attc, S, d, p[4], d, p[5], xc, xc, st));
      M3_TRY(launch_ln(xc, S, d, p[6], p[7], ln_eps, xnc, st));
      M3_TRY(launch_linear(1, xnc, S, d, p[8], d4, p[9], nullptr, hidc, st));
      M3_TRY(launch_linear(2, hidc, S, d4, p[10], d, p[11], xc, xc, st));
    }
  }
  const float* const* f = h_params + 4 + 12 * depth;
  return launch_ln(xc, S, d, f[0], f[1], ln_eps, d_cls, st);
}
