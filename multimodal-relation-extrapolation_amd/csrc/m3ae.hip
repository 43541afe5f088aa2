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
// MI355X design -- only the work that can reach a CLS output, all of it exact:
//  * A padded token (mask > 0) is a key whose logit is -1e7, so its softmax weight
//    exp(-1e7 - max) is exactly 0 in fp32, and every other op is row-wise: padded rows never
//    reach an unpadded row. Only the CLS row and the unpadded tokens are computed, packed
//    back to back over all sequences ("rows", CSR offsets), so a 9-token description costs
//    10 rows, not the reference's 321.
//  * A description row equal to the previous one on its unpadded (position, token) pairs is
//    not encoded again (the reference repeats each description test_sample / G_batch_size
//    times, zsl_module.py:662-665, utils.py:686): the frozen encoder is a deterministic
//    function of those pairs, so the repeat's CLS is a copy.
//  * Only the CLS row leaves the encoder, so the last block runs attention / fc / MLP /
//    final LN on the CLS rows alone (K and V of every row are still formed).
// Kernels:
//   k_m3ae_plan_rows / _scan     per row: unpadded count, same-as-previous flag, bad token ids;
//                                then the unique sequences, their packed row offsets, sizes
//   k_m3ae_embed                 one workgroup per unique sequence: compaction + embedding sum
//   k_m3ae_ln<V>                 nn.LayerNorm (biased var, eps), one wave per row (optional
//                                row gather: the final LN writes every input row's CLS)
//   k_m3ae_linear<EPI, BN>       C = A W^T + b (+GELU | +residual), fp32 MFMA
//                                v_mfma_f32_32x32x2_f32, 64 x BN tiles (BN 128, or 64 when
//                                the grid would not fill the chip), K staged 32 deep through
//                                double-buffered row-major LDS (b128 reads and writes, padded
//                                pitch: conflict-free) with two register stages in flight;
//                                XCD-aware tile order
//   k_m3ae_attn<HD>              one workgroup per (sequence, head, 16 query rows): logit rows
//                                in LDS sized to the longest sequence, exact two-pass softmax
//   k_m3ae_gather_cls            x[off[u]] -> compact CLS rows (last block)
#include <math.h>

#include "mmre_common.h"

namespace mmre {
namespace {

constexpr int M3_MAXLEN = 335;  // tokens per description row (attention keeps 1 + len logits per row in LDS)
constexpr int M3_AQ = 16;       // query rows per attention workgroup
constexpr int M3_AKC = 64;      // most keys per staged K / V chunk
constexpr int M3_MAXR = 336;    // 1 + M3_MAXLEN

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) v += __shfl_xor(v, sh);
  return v;
}

// Plan buffer (int32), n = n_seq:
//   uniq[n]    unique-sequence index of each input row
//   src[n]     first input row of each unique sequence
//   off[n+1]   packed row offsets of the unique sequences (CLS row first)
//   info[4]    n_unique, n_rows (= off[n_unique]), max_rows, bad token ids
//   scratch    cnt[n], head[n], bad[n]
struct Plan {
  int32_t *uniq, *src, *off, *info, *cnt, *head, *bad;
  __host__ __device__ Plan(int32_t* p, int64_t n)
      : uniq(p), src(p + n), off(p + 2 * n), info(p + 3 * n + 1), cnt(p + 3 * n + 5), head(p + 4 * n + 5),
        bad(p + 5 * n + 5) {}
};

// One wave per input row b: cnt = 1 + #{p : !(mask > 0)} (torch.where(padding_mask > 0, -1e7, .)
// masks exactly the entries with mask > 0, submodule.py:174-177); head = 0 when row b equals row
// b - 1 on the padding pattern and on every unpadded token; bad = unpadded ids outside [0, vocab).
__global__ __launch_bounds__(256) void k_m3ae_plan_rows(const int32_t* __restrict__ tokens,
                                                        const float* __restrict__ mask, int64_t n_seq, int64_t len,
                                                        int dedupe, int64_t vocab, int32_t* __restrict__ plan) {
  Plan P(plan, n_seq);
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= n_seq) return;
  const bool cmp = dedupe && b > 0;
  int c = 0, nb = 0;
  bool diff = false;
  for (int64_t p = lane; p < len; p += 64) {
    const bool v = !(mask[b * len + p] > 0.0f);
    const int32_t id = tokens[b * len + p];
    c += v;
    nb += v && (id < 0 || (int64_t)id >= vocab);
    if (cmp) {
      const bool vp = !(mask[(b - 1) * len + p] > 0.0f);
      diff |= (v != vp) || (v && id != tokens[(b - 1) * len + p]);
    }
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) {
    c += __shfl_xor(c, sh);
    nb += __shfl_xor(nb, sh);
  }
  const bool any_diff = __ballot(diff) != 0;
  if (lane == 0) {
    P.cnt[b] = 1 + c;
    P.head[b] = !cmp || any_diff;
    P.bad[b] = nb;
  }
}

// Inclusive scan of one value per thread over a 1024-thread workgroup; *total = the sum.
__device__ int block_scan(int x, int32_t* s_w, int* total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int sh = 1; sh < 64; sh <<= 1) {
    const int y = __shfl_up(x, sh);
    if (lane >= sh) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  int pre = 0, tot = 0;
  for (int k = 0; k < 16; ++k) {
    pre += k < w ? s_w[k] : 0;
    tot += s_w[k];
  }
  __syncthreads();
  *total = tot;
  return pre + x;
}

// One 1024-thread workgroup: unique sequences (scan of head), their sources and row counts,
// then the packed offsets (scan of the counts), the longest sequence and the bad-id total.
__global__ __launch_bounds__(1024) void k_m3ae_plan_scan(int64_t n_seq, int32_t* __restrict__ plan) {
  Plan P(plan, n_seq);
  __shared__ int32_t s_w[16];
  const int tid = threadIdx.x;
  int carry = 0, mx = 1, nbad = 0;
  for (int64_t c0 = 0; c0 < n_seq; c0 += 1024) {
    const int64_t i = c0 + tid;
    const int h = i < n_seq ? P.head[i] : 0;
    int tot;
    const int incl = block_scan(h, s_w, &tot);
    if (i < n_seq) {
      const int u = carry + incl - 1;
      P.uniq[i] = u;
      if (h) {
        P.src[u] = (int32_t)i;
        P.off[u + 1] = P.cnt[i];
        mx = max(mx, P.cnt[i]);
      }
      nbad += P.bad[i];
    }
    carry += tot;
  }
  __syncthreads();  // off[1..n_unique] written
  const int n_unique = carry;
  int run = 0;
  for (int64_t c0 = 0; c0 < n_unique; c0 += 1024) {
    const int64_t i = c0 + tid;
    const int v = i < n_unique ? P.off[i + 1] : 0;
    int tot;
    const int incl = block_scan(v, s_w, &tot);
    if (i < n_unique) P.off[i + 1] = run + incl;
    run += tot;
  }
  // max / sum of the per-thread partials
  __shared__ int32_t s_mx[1024 / 64], s_bad[1024 / 64];
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) {
    mx = max(mx, __shfl_xor(mx, sh));
    nbad += __shfl_xor(nbad, sh);
  }
  if ((tid & 63) == 0) {
    s_mx[tid >> 6] = mx;
    s_bad[tid >> 6] = nbad;
  }
  __syncthreads();
  if (tid == 0) {
    int m = 1, nb = 0;
    for (int k = 0; k < 16; ++k) {
      m = max(m, s_mx[k]);
      nb += s_bad[k];
    }
    P.off[0] = 0;
    P.info[0] = n_unique;
    P.info[1] = run;
    P.info[2] = m;
    P.info[3] = nb;
  }
}

// One workgroup per unique sequence u (input row src[u]): list the unpadded positions in order
// (ballot prefix), then write row off[u] = cls_token and row off[u] + 1 + i = (emb[tok] +
// pos[p]) + type for the i-th unpadded position p (model.py:341-351, same fp32 association).
// A token id outside [0, vocab) yields a NaN row (never an out-of-bounds read); the host
// refuses such rows first (info[3]).
__global__ __launch_bounds__(256) void k_m3ae_embed(const int32_t* __restrict__ tokens, const float* __restrict__ mask,
                                                    int64_t len, const int32_t* __restrict__ src,
                                                    const int32_t* __restrict__ off, const float* __restrict__ emb,
                                                    int64_t vocab, const float* __restrict__ pos,
                                                    const float* __restrict__ type_emb, const float* __restrict__ cls,
                                                    int d, float* __restrict__ x) {
  __shared__ int32_t s_pos[M3_MAXLEN + 256];
  __shared__ int32_t s_w[4];
  const int64_t u = blockIdx.x;
  const int64_t b = src[u];
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
  const int64_t r0 = off[u];
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

// nn.LayerNorm over D = 64 V: y[r] = (x - mean) / sqrt(var + eps) * w + b, biased variance,
// x = x[gather ? gather[r] : r]. One wave per row, 4 rows per workgroup.
template <int V>
__global__ __launch_bounds__(256) void k_m3ae_ln(const float* __restrict__ x, const int32_t* __restrict__ gather,
                                                 int64_t n, const float* __restrict__ w, const float* __restrict__ bb,
                                                 float eps, float* __restrict__ y) {
  constexpr int D = 64 * V;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const float* xr = x + (gather ? (int64_t)gather[r] : r) * D;
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
// 256 threads = 4 waves as 2 (m) x 2 (n); a wave owns 32 x BN/2 = BN/64 MFMA blocks of 32 x 32.
// N % BN == 0, K % 32 == 0 (checked by the host entry).
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int LM = 64, LK = 32;

template <int EPI, int BN>
__global__ __launch_bounds__(256, 2) void k_m3ae_linear(const float* __restrict__ A, int64_t M, int K,
                                                        const float* __restrict__ W, int N,
                                                        const float* __restrict__ bias, const float* resid,
                                                        float* out) {
  constexpr int NB = BN / 64;             // MFMA column blocks per wave
  constexpr int BQ = BN * LK / 4 / 256;   // W-stage float4 per thread
  constexpr int BSTEP = 256 / BN;         // quad stride between a thread's W loads
  constexpr int PITCH = LK + 4;           // row pitch (floats): b128 accesses of 16 rows hit 64 distinct banks
  // row-major (m / n rows, 32 k each) stages: the MFMA of sub-step i takes k = i from lanes 0-31
  // and k = 16 + i from lanes 32-63, so a lane's 16 operands of a K step are 4 aligned float4s
  __shared__ float sA[2][LM][PITCH];
  __shared__ float sB[2][BN][PITCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lrow = lane >> 5, lcol = lane & 31;
  // XCD-aware tile order: round-robin dispatch puts workgroup b on XCD b % 8, so XCD x takes
  // the contiguous, M-major tile range [x * per, (x + 1) * per): its L2 holds one slice of A
  // rows and the W rows, instead of every XCD streaming all of both.
  const int n_nt = N / BN;
  const int64_t n_tiles = (int64_t)((M + LM - 1) / LM) * n_nt;
  const int64_t per = (n_tiles + 7) / 8;
  const int64_t t = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= n_tiles) return;  // uniform over the workgroup
  const int64_t m0 = (t / n_nt) * LM;
  const int n0 = (int)(t % n_nt) * BN;
  const int ar = tid & 63, aq = tid >> 6;   // A stage: row ar, k quads aq and aq + 4
  const int br = tid % BN, bq = tid / BN;   // W stage: row br, k quads bq + BSTEP i
  // rows past M load row M - 1 (no branches in the load path); their outputs are never stored
  const int nkt = K / LK;
  const float* Ap = A + min(m0 + ar, M - 1) * (int64_t)K;
  const float* Bp = W + (int64_t)(n0 + br) * K;
  // two register stages: the loads of K step s are issued two steps before they are written to
  // LDS, so two steps of MFMA work (not one) cover their latency
  // register stages (named scalars: a runtime-indexed array would live in scratch)
  float4 ra00, ra01, rb00, rb01, rb02, rb03, ra10, ra11, rb10, rb11, rb12, rb13;
  static_assert(BQ == 2 || BQ == 4, "W stage: 2 or 4 float4 per thread");
#define M3_GLOAD(kt, RA0, RA1, RB0, RB1, RB2, RB3)                                                  \
  do {                                                                                              \
    const int k0_ = (kt) * LK;                                                                      \
    RA0 = *reinterpret_cast<const float4*>(Ap + k0_ + 4 * aq);                                      \
    RA1 = *reinterpret_cast<const float4*>(Ap + k0_ + 4 * (aq + 4));                                \
    RB0 = *reinterpret_cast<const float4*>(Bp + k0_ + 4 * bq);                                      \
    RB1 = *reinterpret_cast<const float4*>(Bp + k0_ + 4 * (bq + BSTEP));                            \
    if constexpr (BQ == 4) {                                                                        \
      RB2 = *reinterpret_cast<const float4*>(Bp + k0_ + 4 * (bq + 2 * BSTEP));                      \
      RB3 = *reinterpret_cast<const float4*>(Bp + k0_ + 4 * (bq + 3 * BSTEP));                      \
    }                                                                                               \
  } while (0)
#define M3_SWRITE(buf, RA0, RA1, RB0, RB1, RB2, RB3)                                                \
  do {                                                                                              \
    *reinterpret_cast<float4*>(&sA[buf][ar][4 * aq]) = RA0;                                         \
    *reinterpret_cast<float4*>(&sA[buf][ar][4 * (aq + 4)]) = RA1;                                   \
    *reinterpret_cast<float4*>(&sB[buf][br][4 * bq]) = RB0;                                         \
    *reinterpret_cast<float4*>(&sB[buf][br][4 * (bq + BSTEP)]) = RB1;                               \
    if constexpr (BQ == 4) {                                                                        \
      *reinterpret_cast<float4*>(&sB[buf][br][4 * (bq + 2 * BSTEP)]) = RB2;                         \
      *reinterpret_cast<float4*>(&sB[buf][br][4 * (bq + 3 * BSTEP)]) = RB3;                         \
    }                                                                                               \
  } while (0)

  floatx16 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
#define M3_COMPUTE(buf)                                                                             \
  do {                                                                                              \
    const float* arow_ = &sA[buf][wm * 32 + lcol][16 * lrow];                                       \
    const float* brow_ = &sB[buf][wn * (BN / 2) + lcol][16 * lrow];                                 \
    _Pragma("unroll") for (int q_ = 0; q_ < 4; ++q_) {                                              \
      const float4 av_ = *reinterpret_cast<const float4*>(arow_ + 4 * q_);                          \
      _Pragma("unroll") for (int j_ = 0; j_ < NB; ++j_) {                                           \
        const float4 bv_ = *reinterpret_cast<const float4*>(brow_ + 32 * j_ * PITCH + 4 * q_);      \
        acc[j_] = __builtin_amdgcn_mfma_f32_32x32x2f32(av_.x, bv_.x, acc[j_], 0, 0, 0);             \
        acc[j_] = __builtin_amdgcn_mfma_f32_32x32x2f32(av_.y, bv_.y, acc[j_], 0, 0, 0);             \
        acc[j_] = __builtin_amdgcn_mfma_f32_32x32x2f32(av_.z, bv_.z, acc[j_], 0, 0, 0);             \
        acc[j_] = __builtin_amdgcn_mfma_f32_32x32x2f32(av_.w, bv_.w, acc[j_], 0, 0, 0);             \
      }                                                                                             \
    }                                                                                               \
  } while (0)
  // K step s lives in LDS buffer s & 1 and register stage s & 1
  M3_GLOAD(0, ra00, ra01, rb00, rb01, rb02, rb03);
  if (nkt > 1) M3_GLOAD(1, ra10, ra11, rb10, rb11, rb12, rb13);
  M3_SWRITE(0, ra00, ra01, rb00, rb01, rb02, rb03);
  if (nkt > 2) M3_GLOAD(2, ra00, ra01, rb00, rb01, rb02, rb03);
  __syncthreads();
  for (int kt = 0; kt < nkt; kt += 2) {
    M3_COMPUTE(0);
    if (kt + 1 < nkt) M3_SWRITE(1, ra10, ra11, rb10, rb11, rb12, rb13);
    if (kt + 3 < nkt) M3_GLOAD(kt + 3, ra10, ra11, rb10, rb11, rb12, rb13);
    __syncthreads();
    if (kt + 1 >= nkt) break;
    M3_COMPUTE(1);
    if (kt + 2 < nkt) M3_SWRITE(0, ra00, ra01, rb00, rb01, rb02, rb03);
    if (kt + 4 < nkt) M3_GLOAD(kt + 4, ra00, ra01, rb00, rb01, rb02, rb03);
    __syncthreads();
  }
#undef M3_GLOAD
#undef M3_SWRITE
#undef M3_COMPUTE
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = n0 + wn * (BN / 2) + 32 * j + lcol;
    const float bn = bias[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lrow;
      if (m < M) {
        float v = acc[j][r] + bn;
        if constexpr (EPI == 1) v = (v * 0.5f) * (1.0f + erff(v * 0.70710678118654752f));
        if constexpr (EPI == 2) v = resid[m * N + n] + v;
        out[m * N + n] = v;
      }
    }
  }
}

// Multi-head attention of one (sequence s, head h, block of M3_AQ query rows) over the
// sequence's rows [off[s], off[s+1]) of qkv (row layout [q | k | v], each heads x HD:
// qkv.view(B, n, 3, heads, HD), submodule.py:166-169). Logits s = (q . k) * scale for all
// keys are kept in LDS, then softmax = exp(s - max) / sum (two passes over the row), then
// out[:, h*HD + c] = sum_j p_j v_j[c] (the permute/reshape of :183). cls_only: only query
// row 0 of each sequence, written to out row s (the last block). Dynamic LDS:
// sQ[AQ][HD+1] | sKV[kc][HD+1] | sS[AQ][rp], kc = keys per chunk (<= 64, multiple of 16),
// rp >= the longest sequence's row count.
template <int HD>
__global__ __launch_bounds__(256) void k_m3ae_attn(const float* __restrict__ qkv, const int32_t* __restrict__ off,
                                                   int heads, float scale, int cls_only, int kc_max, int rp,
                                                   float* __restrict__ out) {
  constexpr int HP = HD + 1;  // padded row stride: the 16 lanes of a row group hit distinct banks
  extern __shared__ float smem[];
  float (*sQ)[HP] = reinterpret_cast<float (*)[HP]>(smem);
  float (*sKV)[HP] = reinterpret_cast<float (*)[HP]>(smem + M3_AQ * HP);
  float* sS = smem + (M3_AQ + kc_max) * HP;
  const int s = blockIdx.z, h = blockIdx.y;
  const int r0 = off[s], nrow = off[s + 1] - r0;
  const int q0 = blockIdx.x * M3_AQ;
  const int nq = cls_only ? 1 : min(M3_AQ, nrow - q0);
  if (nq <= 0) return;  // uniform
  const int D = heads * HD, D3 = 3 * D;
  const int tid = threadIdx.x;
  const int qi = tid >> 4, sub = tid & 15;  // query row of this thread, lane within its 16-lane row group
  float* srow = sS + qi * rp;

  for (int e = tid; e < M3_AQ * HD; e += 256) {
    const int i = e / HD, c = e % HD;
    sQ[i][c] = i < nq ? qkv[(int64_t)(r0 + q0 + i) * D3 + h * HD + c] : 0.0f;
  }
  // pass 1: logits of every key
  for (int kc = 0; kc < nrow; kc += kc_max) {
    const int nk = min(kc_max, nrow - kc);
    __syncthreads();  // sQ written / previous chunk's readers done
    for (int e = tid; e < nk * HD; e += 256) {
      const int j = e / HD, c = e % HD;
      sKV[j][c] = qkv[(int64_t)(r0 + kc + j) * D3 + D + h * HD + c];
    }
    __syncthreads();
    for (int j = sub; j < nk; j += 16) {
      float acc = 0.0f;
#pragma unroll 16
      for (int c = 0; c < HD; ++c) acc = __builtin_fmaf(sQ[qi][c], sKV[j][c], acc);
      srow[kc + j] = acc * scale;
    }
  }
  __syncthreads();
  // softmax of each row, 16 lanes per row
  float mx = -INFINITY;
  for (int j = sub; j < nrow; j += 16) mx = fmaxf(mx, srow[j]);
#pragma unroll
  for (int sh = 8; sh >= 1; sh >>= 1) mx = fmaxf(mx, __shfl_xor(mx, sh));
  float sum = 0.0f;
  for (int j = sub; j < nrow; j += 16) {
    const float e = expf(srow[j] - mx);
    srow[j] = e;
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
  for (int kc = 0; kc < nrow; kc += kc_max) {
    const int nk = min(kc_max, nrow - kc);
    __syncthreads();  // softmax writes to sS / previous chunk's readers done
    for (int e = tid; e < nk * HD; e += 256) {
      const int j = e / HD, c = e % HD;
      sKV[j][c] = qkv[(int64_t)(r0 + kc + j) * D3 + 2 * D + h * HD + c];
    }
    __syncthreads();
    for (int j = 0; j < nk; ++j) {
      const float p = srow[kc + j] * inv;
#pragma unroll
      for (int cc = 0; cc < NC; ++cc) o[cc] = __builtin_fmaf(p, sKV[j][sub + 16 * cc], o[cc]);
    }
  }
  if (qi < nq) {
    const int64_t row = cls_only ? (int64_t)s : (int64_t)(r0 + q0 + qi);
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

int launch_ln(const float* x, const int32_t* gather, int64_t n, int d, const float* w, const float* b, float eps,
              float* y, hipStream_t st) {
  if (n <= 0) return MMRE_OK;
  const dim3 g((unsigned)((n + 3) / 4));
  switch (d) {
    case 384: hipLaunchKernelGGL(k_m3ae_ln<6>, g, dim3(256), 0, st, x, gather, n, w, b, eps, y); break;
    case 768: hipLaunchKernelGGL(k_m3ae_ln<12>, g, dim3(256), 0, st, x, gather, n, w, b, eps, y); break;
    case 1024: hipLaunchKernelGGL(k_m3ae_ln<16>, g, dim3(256), 0, st, x, gather, n, w, b, eps, y); break;
    case 1280: hipLaunchKernelGGL(k_m3ae_ln<20>, g, dim3(256), 0, st, x, gather, n, w, b, eps, y); break;
    default: return MMRE_ERR_SHAPE;
  }
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

template <int BN>
void launch_linear_bn(int epi, int64_t mt, hipStream_t st, const float* A, int64_t M, int K, const float* W, int N,
                      const float* bias, const float* resid, float* out) {
  const dim3 g((unsigned)(8 * ((mt * (N / BN) + 7) / 8)));
  if (epi == 0) hipLaunchKernelGGL((k_m3ae_linear<0, BN>), g, dim3(256), 0, st, A, M, K, W, N, bias, resid, out);
  else if (epi == 1) hipLaunchKernelGGL((k_m3ae_linear<1, BN>), g, dim3(256), 0, st, A, M, K, W, N, bias, resid, out);
  else hipLaunchKernelGGL((k_m3ae_linear<2, BN>), g, dim3(256), 0, st, A, M, K, W, N, bias, resid, out);
}

int launch_linear(int epi, const float* A, int64_t M, int K, const float* W, int N, const float* bias,
                  const float* resid, float* out, hipStream_t st) {
  if (M < 0 || K <= 0 || N <= 0 || K % LK || N % 64 || (M + LM - 1) / LM * (N / 64) > 0x7fffff00LL)
    return MMRE_ERR_SHAPE;
  if (epi < 0 || epi > 2 || !A || !W || !bias || !out || (epi == 2 && !resid)) return MMRE_ERR_ARG;
  if (M == 0) return MMRE_OK;
  const int64_t mt = (M + LM - 1) / LM;
  // 64 x 64 tiles: measured faster than 64 x 128 on every encoder shape at 2,261 rows
  // (scripts/m3ae_gemm_ab.py; an in-workgroup split-K was no faster either); 64 x 128 only
  // once the grid holds 8 tiles per CU
  static const char* force = getenv("MMRE_M3AE_TILE");  // experiments: "128" or "64"
  const bool wide = N % 128 == 0 && (force && force[0] ? force[0] == '1' : mt * (N / 128) >= 2048);
  if (wide) launch_linear_bn<128>(epi, mt, st, A, M, K, W, N, bias, resid, out);
  else launch_linear_bn<64>(epi, mt, st, A, M, K, W, N, bias, resid, out);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

int launch_attn(const float* qkv, const int32_t* off, int64_t n_seq, int max_rows, int heads, int hd, float scale,
                int cls_only, float* out, hipStream_t st) {
  if (n_seq <= 0) return MMRE_OK;
  if (max_rows < 1 || max_rows > M3_MAXR || n_seq > 65535 || heads < 1 || heads > 1024) return MMRE_ERR_SHAPE;
  const int kc = max_rows >= M3_AKC ? M3_AKC : (int)round_up(max_rows, 16);
  const int rp = (int)round_up(max_rows, 4) + 1;  // odd-ish row pitch: row groups start on different banks
  const size_t lds = (size_t)((M3_AQ + kc) * (hd + 1) + M3_AQ * rp) * sizeof(float);
  const dim3 g(cls_only ? 1u : (unsigned)((max_rows + M3_AQ - 1) / M3_AQ), (unsigned)heads, (unsigned)n_seq);
  switch (hd) {
    case 64:
      hipLaunchKernelGGL(k_m3ae_attn<64>, g, dim3(256), lds, st, qkv, off, heads, scale, cls_only, kc, rp, out);
      break;
    case 80:
      hipLaunchKernelGGL(k_m3ae_attn<80>, g, dim3(256), lds, st, qkv, off, heads, scale, cls_only, kc, rp, out);
      break;
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

extern "C" int64_t mmre_m3ae_plan_size(int64_t n_seq) { return n_seq < 0 ? -1 : 6 * n_seq + 5; }

extern "C" int mmre_m3ae_plan(const int32_t* d_tokens, const float* d_mask, int64_t n_seq, int64_t len, int dedupe,
                              int64_t vocab, int32_t* d_plan, void* stream) {
  if (n_seq < 0 || len < 0 || len > M3_MAXLEN || !d_plan || vocab <= 0 ||
      (n_seq > 0 && len > 0 && (!d_mask || !d_tokens)))
    return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n_seq > 0)
    hipLaunchKernelGGL(k_m3ae_plan_rows, dim3((unsigned)((n_seq + 3) / 4)), dim3(256), 0, st, d_tokens, d_mask, n_seq,
                       len, dedupe, vocab, d_plan);
  hipLaunchKernelGGL(k_m3ae_plan_scan, dim3(1), dim3(1024), 0, st, n_seq, d_plan);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int64_t mmre_m3ae_workspace(int64_t n_rows, int64_t n_unique, int d) {
  if (n_rows < 0 || n_unique < 0 || d <= 0) return -1;
  // x | xn | qkv | att | hidden (4d) over the rows, then x_cls | xn_cls | att_cls | hidden_cls
  return n_rows * (int64_t)d * (1 + 1 + 3 + 1 + 4) + n_unique * (int64_t)d * (1 + 1 + 1 + 4);
}

extern "C" int mmre_m3ae_layernorm(const float* d_x, int64_t n_rows, int d, const float* d_w, const float* d_b,
                                   float eps, float* d_y, void* stream) {
  if (n_rows < 0 || !d_x || !d_w || !d_b || !d_y) return MMRE_ERR_ARG;
  return launch_ln(d_x, nullptr, n_rows, d, d_w, d_b, eps, d_y, (hipStream_t)stream);
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
                                int64_t vocab, const int32_t* d_plan, int64_t n_unique, int64_t n_rows, int max_rows,
                                float* d_work, int64_t work_floats, float* d_cls, void* stream) {
  if (!h_params || depth < 1 || !m3ae_dims_ok(d, heads)) return MMRE_ERR_SHAPE;
  if (n_seq < 0 || len < 0 || len > M3_MAXLEN || n_unique < (n_seq > 0 ? 1 : 0) || n_unique > n_seq ||
      n_rows < n_unique || max_rows < 1 || max_rows > len + 1 || !d_plan || !d_work || !d_cls || vocab <= 0 ||
      (n_seq > 0 && (!d_tokens || !d_mask)))
    return MMRE_ERR_ARG;
  if (work_floats < mmre_m3ae_workspace(n_rows, n_unique, d)) return MMRE_ERR_WORKSPACE;
  for (int i = 0; i < 4 + 12 * depth + 2; ++i)
    if (!h_params[i]) return MMRE_ERR_ARG;
  if (n_seq == 0) return MMRE_OK;
  hipStream_t st = (hipStream_t)stream;
  const Plan P(const_cast<int32_t*>(d_plan), n_seq);
  const int64_t R = n_rows, S = n_unique;
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

  hipLaunchKernelGGL(k_m3ae_embed, dim3((unsigned)S), dim3(256), 0, st, d_tokens, d_mask, len, P.src, P.off,
                     h_params[0], vocab, h_params[1], h_params[2], h_params[3], d, x);
  MMRE_CHECK_LAUNCH();
  for (int l = 0; l < depth; ++l) {
    const float* const* p = h_params + 4 + 12 * l;
    // p: ln1 w, b | qkv w, b | fc w, b | ln2 w, b | fc1 w, b | fc2 w, b
    M3_TRY(launch_ln(x, nullptr, R, d, p[0], p[1], ln_eps, xn, st));
    M3_TRY(launch_linear(0, xn, R, d, p[2], d3, p[3], nullptr, qkv, st));
    if (l + 1 < depth) {
      M3_TRY(launch_attn(qkv, P.off, S, max_rows, heads, hd, scale, 0, att, st));
      M3_TRY(launch_linear(2, att, R, d, p[4], d, p[5], x, x, st));
      M3_TRY(launch_ln(x, nullptr, R, d, p[6], p[7], ln_eps, xn, st));
      M3_TRY(launch_linear(1, xn, R, d, p[8], d4, p[9], nullptr, hid, st));
      M3_TRY(launch_linear(2, hid, R, d4, p[10], d, p[11], x, x, st));
    } else {  // last block: only the CLS rows go on
      M3_TRY(launch_attn(qkv, P.off, S, max_rows, heads, hd, scale, 1, attc, st));
      hipLaunchKernelGGL(k_m3ae_gather_cls, dim3((unsigned)((S * d + 255) / 256)), dim3(256), 0, st, x, P.off, S, d,
                         xc);
      MMRE_CHECK_LAUNCH();
      M3_TRY(launch_linear(2, attc, S, d, p[4], d, p[5], xc, xc, st));
      M3_TRY(launch_ln(xc, nullptr, S, d, p[6], p[7], ln_eps, xnc, st));
      M3_TRY(launch_linear(1, xnc, S, d, p[8], d4, p[9], nullptr, hidc, st));
      M3_TRY(launch_linear(2, hidc, S, d4, p[10], d, p[11], xc, xc, st));
    }
  }
  // final LayerNorm, written for every input row from its unique sequence's CLS
  const float* const* f = h_params + 4 + 12 * depth;
  return launch_ln(xc, P.uniq, n_seq, d, f[0], f[1], ln_eps, d_cls, st);
}
