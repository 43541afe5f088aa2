// extractor.hip -- the ZSL Extractor of ZSLmodule.eval (module/zsl_module.py:17-110, 666-706),
// eval mode (dropout = identity), fused with the cosine-rank epilogue.
//
// Reference forward for one (e1, e2) pair, d = embed_dim, h = d/2 (zsl_module.py:47-110):
//   nb(x)   = tanh( sum_{s < max_nb} (gcn_w . emb[conn[x][s][1]] + gcn_b) / deg[x] )      :47-59
//   ent     = tanh( cat(fc1 . emb[e1] + b1, fc2 . emb[e2] + b2) )                        :61-67
//   x       = reshape_layer( cat(nb(e1), ent, nb(e2)) )                      2d -> d      :88-96
//   g       = LayerNorm( proj2 . relu(proj1 . x + p1) + p2 + x )   SupportEncoder d->2d->d  submodule.py:254-258
//   ZSL score of a candidate = mean_s cos(g, rel_vec[s])          (sklearn, zsl_module.py:699-701)
//
// MI355X restructuring (same function, reassociated):
//   * reshape_layer is linear, so x = L[e1] + R[e2] with per-NODE tables
//       L[n] = Wr[:, 0:h] nb(n) + Wr[:, h:d] tanh(fc1 . emb[n] + b1) + br
//       R[n] = Wr[:, d:d+h] tanh(fc2 . emb[n] + b2) + Wr[:, d+h:2d] nb(n)
//     and sum_s (gcn_w . e_s + gcn_b) = gcn_w . (sum_s e_s) + max_nb * gcn_b.
//     k_extractor_nodes builds L / R once per entity (a ZSL evaluation's 17.6 M candidate
//     pairs share 14 k entities), instead of once per candidate row.
//   * k_extractor_encode runs the SupportEncoder for 16 rows per wave on
//     v_mfma_f32_16x16x4_f32 in a transposed orientation: H^T = W1 . X^T leaves each lane
//     holding 4 consecutive hidden features of one row, which is exactly the B operand of
//     Y^T = W2 . H^T when the contraction index is permuted to match (the order of a sum
//     is free; the A operand W2 is packed with the same permutation). The 2d hidden
//     activations therefore never leave registers: no LDS, no barriers. Weights are
//     pre-packed (mmre_extractor_pack) in per-lane MFMA order so every operand load is one
//     coalesced 1-KB float4 wave load (L2-resident: 2 x 320 KB at d = 200).
//   * Epilogue: bias, residual, LayerNorm (biased variance, eps inside the sqrt: nn.LayerNorm)
//     over the 4 lanes sharing a row, then cos(g, t) = (g . t) / |g| against the mean of the
//     row's normalised relation vectors (mean_s cos(g, y_s) = g/|g| . mean_s y_s/|y_s|).
// k_rank_desc: rank of the true candidate (first of each list) = 1 + #(score > score[true]).
#include "mmre_common.h"

namespace mmre {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Compile-time geometry for an embedding width D.
template <int D>
struct XG {
  static constexpr int H = D / 2;                  // gcn / fc1 / fc2 width
  static constexpr int NH = (2 * D + 15) / 16;     // hidden (proj1 output) blocks of 16
  static constexpr int NY = (D + 15) / 16;         // output blocks of 16
  static constexpr int KC = (D + 3) / 4;           // input features per lane group (stage 1)
  static constexpr int S1 = (KC + 3) / 4 * 4;      // stage-1 steps, padded to float4 packs
  // Weight stream: 1-KB pieces (64 lanes x float4) in the order the encode kernel consumes
  // them -- stage 1: for s4, for b: W1 block b, steps 4*s4..4*s4+3; stage 2: for hb, for ob:
  // W2 block ob, hidden features hb*16 + 4*(l/16) + q -- grouped in chunks of CH pieces
  // (an even number NC of chunks, zero padded).
  static constexpr int NP1 = (S1 / 4) * NH;
  static constexpr int NP = NP1 + NH * NY;
  static constexpr int CH = 8;    // 8-KB chunks: 2 float4 per thread of a 256-thread group
  static constexpr int NC = ((NP + CH - 1) / CH + 1) / 2 * 2;
  // packed buffer offsets (floats)
  static constexpr int64_t PS = 0;                               // [NC*CH][64][4] weight stream
  static constexpr int64_t PB1 = PS + (int64_t)NC * CH * 256;    // [NH*16] proj1 bias
  static constexpr int64_t PB2 = PB1 + NH * 16;                  // [NY*16] proj2 bias
  static constexpr int64_t PLW = PB2 + NY * 16;                  // [NY*16] LayerNorm weight
  static constexpr int64_t PLB = PLW + NY * 16;                  // [NY*16] LayerNorm bias
  static constexpr int64_t PGT = PLB + NY * 16;                  // [D][H]  gcn_w^T
  static constexpr int64_t PGB = PGT + (int64_t)D * H;           // [H]     gcn_w bias
  static constexpr int64_t PF1 = PGB + H;                        // [D][H]  fc1^T
  static constexpr int64_t PF1B = PF1 + (int64_t)D * H;          // [H]
  static constexpr int64_t PF2 = PF1B + H;                       // [D][H]  fc2^T
  static constexpr int64_t PF2B = PF2 + (int64_t)D * H;          // [H]
  static constexpr int64_t PRS = PF2B + H;                       // [2D][D] reshape_layer^T
  static constexpr int64_t PRSB = PRS + (int64_t)2 * D * D;      // [D]
  static constexpr int64_t SIZE = PRSB + D;
};

// ---------------------------------------------------------------------------------------
// Packing: nn.Linear weights (out, in) row-major -> MFMA lane order / transposed.
// ---------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void k_extractor_pack(const float* __restrict__ gcn_w, const float* __restrict__ gcn_b,
                                                        const float* __restrict__ fc1_w, const float* __restrict__ fc1_b,
                                                        const float* __restrict__ fc2_w, const float* __restrict__ fc2_b,
                                                        const float* __restrict__ rs_w, const float* __restrict__ rs_b,
                                                        const float* __restrict__ p1_w, const float* __restrict__ p1_b,
                                                        const float* __restrict__ p2_w, const float* __restrict__ p2_b,
                                                        const float* __restrict__ ln_w, const float* __restrict__ ln_b,
                                                        float* __restrict__ pack) {
  using G = XG<D>;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < G::SIZE; i += stride) {
    float v = 0.0f;
    if (i < G::PB1) {  // weight stream
      const int64_t j = i - G::PS;
      const int e = (int)(j & 3), lane = (int)((j >> 2) & 63), g = lane >> 4;
      const int piece = (int)(j >> 8);
      if (piece < G::NP1) {  // proj1: lane l, step s -> W1[b*16 + l%16][g*KC + s]
        const int s4 = piece / G::NH, b = piece % G::NH;
        const int st = s4 * 4 + e, row = b * 16 + (lane & 15), col = g * G::KC + st;
        if (row < 2 * D && st < G::KC && col < D) v = p1_w[(int64_t)row * D + col];
      } else if (piece < G::NP) {  // proj2: lane l, (hb, q) -> W2[ob*16 + l%16][hb*16 + 4g + q]
        const int p2 = piece - G::NP1, hb = p2 / G::NY, ob = p2 % G::NY;
        const int row = ob * 16 + (lane & 15), col = hb * 16 + 4 * g + e;
        if (row < D && col < 2 * D) v = p2_w[(int64_t)row * (2 * D) + col];
      }
    } else if (i < G::PB2) {
      const int f = (int)(i - G::PB1);
      v = f < 2 * D ? p1_b[f] : 0.0f;
    } else if (i < G::PLW) {
      const int f = (int)(i - G::PB2);
      v = f < D ? p2_b[f] : 0.0f;
    } else if (i < G::PLB) {
      const int f = (int)(i - G::PLW);
      v = f < D ? ln_w[f] : 0.0f;
    } else if (i < G::PGT) {
      const int f = (int)(i - G::PLB);
      v = f < D ? ln_b[f] : 0.0f;
    } else if (i < G::PGB) {
      const int64_t j = i - G::PGT;
      v = gcn_w[(j % G::H) * D + j / G::H];
    } else if (i < G::PF1) {
      v = gcn_b[i - G::PGB];
    } else if (i < G::PF1B) {
      const int64_t j = i - G::PF1;
      v = fc1_w[(j % G::H) * D + j / G::H];
    } else if (i < G::PF2) {
      v = fc1_b[i - G::PF1B];
    } else if (i < G::PF2B) {
      const int64_t j = i - G::PF2;
      v = fc2_w[(j % G::H) * D + j / G::H];
    } else if (i < G::PRS) {
      v = fc2_b[i - G::PF2B];
    } else if (i < G::PRSB) {
      const int64_t j = i - G::PRS;  // [k][o] = Wr[o][k], k < 2D
      v = rs_w[(j % D) * (2 * D) + j / D];
    } else {
      v = rs_b[i - G::PRSB];
    }
    pack[i] = v;
  }
}

// ---------------------------------------------------------------------------------------
// Node tables L / R: NB nodes per workgroup; node inputs in LDS, weights read transposed
// (coalesced across threads), every weight element reused for the NB nodes.
// ---------------------------------------------------------------------------------------
constexpr int NB = 16;

template <int D>
__global__ __launch_bounds__(256) void k_extractor_nodes(const float* __restrict__ pack, const float* __restrict__ emb,
                                                         const int64_t* __restrict__ node_sym,
                                                         const int64_t* __restrict__ conn, int max_nb,
                                                         const float* __restrict__ deg, int64_t n_nodes,
                                                         float* __restrict__ left, float* __restrict__ right) {
  using G = XG<D>;
  constexpr int H = G::H;
  __shared__ float se[NB][D];   // emb[node]
  __shared__ float sn[NB][D];   // sum of the neighbours' embeddings
  __shared__ float sa[NB][H];   // tanh(fc1 . e + b1)
  __shared__ float sb[NB][H];   // tanh(fc2 . e + b2)
  __shared__ float sg[NB][H];   // nb(node)
  const int64_t n0 = (int64_t)blockIdx.x * NB;
  const int nn = (int)((n_nodes - n0) < NB ? (n_nodes - n0) : NB);
  for (int idx = threadIdx.x; idx < NB * D; idx += blockDim.x) {
    const int i = idx / D, k = idx % D;
    float e = 0.0f, s = 0.0f;
    if (i < nn) {
      const int64_t node = n0 + i;
      e = emb[node_sym[node] * D + k];
      const int64_t* c = conn + node * max_nb * 2;
      for (int j = 0; j < max_nb; ++j) s += emb[c[2 * j + 1] * D + k];
    }
    se[i][k] = e;
    sn[i][k] = s;
  }
  __syncthreads();
  const float* gt = pack + G::PGT;
  const float* f1 = pack + G::PF1;
  const float* f2 = pack + G::PF2;
  for (int o = threadIdx.x; o < 3 * H; o += blockDim.x) {
    const int which = o / H, j = o % H;
    const float* wt = which == 0 ? gt : (which == 1 ? f1 : f2);
    float acc[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) acc[i] = 0.0f;
    for (int k = 0; k < D; ++k) {
      const float w = wt[k * H + j];
      if (which == 0) {
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i] = __builtin_fmaf(w, sn[i][k], acc[i]);
      } else {
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i] = __builtin_fmaf(w, se[i][k], acc[i]);
      }
    }
    if (which == 0) {
      const float b = pack[G::PGB + j] * (float)max_nb;
#pragma unroll
      for (int i = 0; i < NB; ++i) sg[i][j] = tanhf((acc[i] + b) / (i < nn ? deg[n0 + i] : 1.0f));
    } else {
      const float b = pack[(which == 1 ? G::PF1B : G::PF2B) + j];
#pragma unroll
      for (int i = 0; i < NB; ++i) (which == 1 ? sa : sb)[i][j] = tanhf(acc[i] + b);
    }
  }
  __syncthreads();
  const float* rt = pack + G::PRS;  // [k][o], k < 2D
  for (int o = threadIdx.x; o < 2 * D; o += blockDim.x) {
    const bool is_left = o < D;
    const int c = is_left ? o : o - D;
    if (is_left ? !left : !right) continue;
    float acc[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) acc[i] = 0.0f;
    // left: columns [0, h) <- nb, [h, d) <- fc1 part; right: [d, d+h) <- fc2 part, [d+h, 2d) <- nb
    const float(*x0)[H] = is_left ? sg : sb;
    const float(*x1)[H] = is_left ? sa : sg;
    const int kb = is_left ? 0 : D;
    for (int k = 0; k < H; ++k) {
      const float w = rt[(int64_t)(kb + k) * D + c];
#pragma unroll
      for (int i = 0; i < NB; ++i) acc[i] = __builtin_fmaf(w, x0[i][k], acc[i]);
    }
    for (int k = 0; k < H; ++k) {
      const float w = rt[(int64_t)(kb + H + k) * D + c];
#pragma unroll
      for (int i = 0; i < NB; ++i) acc[i] = __builtin_fmaf(w, x1[i][k], acc[i]);
    }
    const float b = is_left ? pack[G::PRSB + c] : 0.0f;
    float* dst = is_left ? left : right;
    for (int i = 0; i < nn; ++i) dst[(n0 + i) * D + c] = acc[i] + b;
  }
}

// ---------------------------------------------------------------------------------------
// Fused SupportEncoder + LayerNorm + cosine epilogue. Persistent workgroups of 4 waves take
// tiles of 64 rows (16 per wave). The weight stream (650 KB at d = 200, identical for every
// tile) flows through a 2 x 16-KB LDS ring shared by the 4 waves: each chunk is loaded into
// registers one chunk ahead (4 x 16-B coalesced loads per thread) and written to LDS after
// the barrier that frees its buffer, so every wave reads its A operands from LDS
// (ds_read_b128, lane-linear, conflict-free) and L2 sees each weight byte once per 64 rows.
// ---------------------------------------------------------------------------------------
// Per-use opaque copy of a kernel-argument pointer: loads through it cannot be hoisted out of
// the persistent tile loop (LICM would otherwise park every loop-invariant weight / bias load
// of the fully unrolled body in registers for the kernel's lifetime).
__device__ __forceinline__ const float* opaque(const float* p) {
  asm volatile("" : "+s"(p));
  return p;
}

template <int D>
__device__ __forceinline__ void load_chunk(const floatx4* stream, int c, floatx4 (&st)[2]) {
  // opaque base: keeps the compiler from hoisting the (loop-invariant) weight loads of every
  // chunk out of the tile loop into registers -- they must stream through the LDS ring
  asm volatile("" : "+s"(stream));
  const floatx4* src = stream + (int64_t)c * (XG<D>::CH * 64) + threadIdx.x;
#pragma unroll
  for (int j = 0; j < 2; ++j) st[j] = src[j * 256];
}

// One chunk of the weight stream (compile-time index CHK, so every accumulator / operand index
// below is a constant: the register arrays never spill to scratch), then the next.
template <int D, int CHK>
__device__ __forceinline__ void run_chunks(floatx4 (&ring)[2][XG<D>::CH * 64], floatx4 (&st)[2],
                                           const floatx4* stream, const floatx4* xs,
                                           floatx4 (&hacc)[XG<D>::NH], floatx4 (&yacc)[XG<D>::NY],
                                           const float* pack, int lane, int g) {
  using G = XG<D>;
  constexpr int NH = G::NH, NY = G::NY, CH = G::CH, NC = G::NC, NP1 = G::NP1, NP = G::NP;
  __syncthreads();  // chunk CHK is in ring[CHK & 1]; everyone is done reading ring[(CHK + 1) & 1]
#pragma unroll
  for (int j = 0; j < 2; ++j) ring[(CHK + 1) & 1][j * 256 + threadIdx.x] = st[j];
  load_chunk<D>(stream, (CHK + 2) % NC, st);  // the stream repeats for the next tile
  const floatx4* buf = ring[CHK & 1] + lane;
  // one MFMA step e of piece p with A fragment a (p is a compile-time constant here)
  auto step = [&](int p, const floatx4& a, const floatx4& xv, int e) {
    if (p < NP1) {  // H^T = W1 . X^T
      const int b = p % NH;
      hacc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], xv[e], hacc[b], 0, 0, 0);
    } else if (p < NP) {  // Y^T = W2 . H^T, B operand straight from the stage-1 accumulators
      const int p2 = p - NP1, hb = p2 / NY, ob = p2 % NY;
      yacc[ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], hacc[hb][e], yacc[ob], 0, 0, 0);
    }
  };
  auto stage_switch = [&]() {  // stage 1 done (accumulators started at the bias): relu; stage 2 starts at p2
#pragma unroll
    for (int b = 0; b < NH; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) hacc[b][q] = fmaxf(hacc[b][q], 0.0f);
    const floatx4* pb2 = reinterpret_cast<const floatx4*>(opaque(pack) + G::PB2);
#pragma unroll
    for (int b = 0; b < NY; ++b) yacc[b] = pb2[b * 4 + g];
  };
  // pieces in pairs: the two 4-step accumulation chains interleave, so no MFMA waits on the
  // 40-cycle dependent latency of the one before it (16x16x4 f32 issues every 32 cycles)
#pragma unroll
  for (int slot = 0; slot < CH; slot += 2) {
    const int p0 = CHK * CH + slot, p1 = p0 + 1;
    if (p0 >= NP) break;
    if (p0 == NP1) stage_switch();
    const floatx4 a0 = buf[slot * 64];
    const floatx4 a1 = buf[(slot + 1) * 64];
    const floatx4 x0 = p0 < NP1 ? xs[(p0 / NH) * 64] : floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    const floatx4 x1 = p1 < NP1 ? xs[(p1 / NH) * 64] : floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    if (p1 == NP1) {  // the pair straddles the stage switch
#pragma unroll
      for (int e = 0; e < 4; ++e) step(p0, a0, x0, e);
      stage_switch();
#pragma unroll
      for (int e = 0; e < 4; ++e) step(p1, a1, x1, e);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        step(p0, a0, x0, e);
        step(p1, a1, x1, e);
      }
    }
  }
  if constexpr (CHK + 1 < NC) run_chunks<D, CHK + 1>(ring, st, stream, xs, hacc, yacc, pack, lane, g);
}

template <int D>
__global__ __launch_bounds__(256, 2) void k_extractor_encode(const float* __restrict__ pack, float ln_eps,
                                                             const float* __restrict__ left,
                                                             const int64_t* __restrict__ li,
                                                             const float* __restrict__ right,
                                                             const int64_t* __restrict__ ri, int64_t n_rows,
                                                             const float* __restrict__ targets,
                                                             const int64_t* __restrict__ row_target, int normalize,
                                                             float* __restrict__ out_g, float* __restrict__ score) {
  using G = XG<D>;
  constexpr int NH = G::NH, NY = G::NY, KC = G::KC, S1 = G::S1, CH = G::CH;
  __shared__ floatx4 ring[2][CH * 64];
  // lane-private stage-1 B operands, parked in LDS (lane-linear float4 per step group s4):
  // keeps the 4*S1/4 x values out of the VGPR budget of the two accumulator sets
  __shared__ floatx4 xlds[4][S1 / 4][64];
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15, wave = threadIdx.x >> 6;
  const floatx4* stream = reinterpret_cast<const floatx4*>(pack + G::PS);
  const int64_t n_tiles = (n_rows + 63) / 64;

  floatx4 st[2];
  load_chunk<D>(stream, 0, st);
#pragma unroll
  for (int j = 0; j < 2; ++j) ring[0][j * 256 + threadIdx.x] = st[j];
  load_chunk<D>(stream, 1, st);
  floatx4* xs = &xlds[wave][0][lane];

  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t row = tile * 64 + wave * 16 + c;
    const bool valid = row < n_rows;
    const int64_t rr = valid ? row : 0;
    const float* lrow = left + li[rr] * D;
    const float* rrow = right + ri[rr] * D;
    // stage-1 B operand: X[row][g*KC + s] for s < KC (zero padded to S1); D % 4 == 0, so
    // g*KC + s < D whenever s < KC
#pragma unroll
    for (int s4 = 0; s4 < S1 / 4; ++s4) {
      floatx4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s = 4 * s4 + e;
        const float t = s < KC ? lrow[g * KC + s] + rrow[g * KC + s] : 0.0f;
        v[e] = valid ? t : 0.0f;
      }
      xs[s4 * 64] = v;  // read back only by this lane (no barrier needed)
    }
    floatx4 hacc[NH];  // proj1 accumulators start at the bias p1 (hidden b*16 + 4g + q)
    const floatx4* pb1 = reinterpret_cast<const floatx4*>(opaque(pack) + G::PB1);
#pragma unroll
    for (int b = 0; b < NH; ++b) hacc[b] = pb1[b * 4 + g];
    floatx4 yacc[NY];

    run_chunks<D, 0>(ring, st, stream, xs, hacc, yacc, pack, lane, g);

    // epilogue: y = acc (started at p2) + x (residual), LayerNorm over the D features of row
    // c, which live in the 4 lanes c, c+16, c+32, c+48 (features ob*16 + 4g + q).
    float sum = 0.0f;
#pragma unroll
    for (int ob = 0; ob < NY; ++ob) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = ob * 16 + 4 * g + q;
        const float res = (f < D) ? lrow[f] + rrow[f] : 0.0f;
        const float y = (f < D) ? yacc[ob][q] + res : 0.0f;
        yacc[ob][q] = y;
        sum += y;
      }
    }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float mean = sum / (float)D;
    float var = 0.0f;
#pragma unroll
    for (int ob = 0; ob < NY; ++ob) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = ob * 16 + 4 * g + q;
        const float dlt = yacc[ob][q] - mean;
        var += (f < D) ? dlt * dlt : 0.0f;
      }
    }
    var += __shfl_xor(var, 16);
    var += __shfl_xor(var, 32);
    const float rstd = 1.0f / sqrtf(var / (float)D + ln_eps);
    const floatx4* plw = reinterpret_cast<const floatx4*>(opaque(pack) + G::PLW);
    const floatx4* plb = reinterpret_cast<const floatx4*>(opaque(pack) + G::PLB);
    const float* tgt = targets ? targets + (row_target ? row_target[rr] : 0) * D : nullptr;
    float dot = 0.0f, nz = 0.0f;
#pragma unroll
    for (int ob = 0; ob < NY; ++ob) {
      const floatx4 w = plw[ob * 4 + g], bb = plb[ob * 4 + g];
      floatx4 z;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = ob * 16 + 4 * g + q;
        z[q] = (f < D) ? (yacc[ob][q] - mean) * rstd * w[q] + bb[q] : 0.0f;
        if (f < D) dot += z[q] * (tgt ? tgt[f] : 0.0f);
        nz += z[q] * z[q];
      }
      if (out_g && valid) {
        const int f0 = ob * 16 + 4 * g;
        if (f0 + 3 < D && (D % 4) == 0) {
          *reinterpret_cast<floatx4*>(out_g + row * D + f0) = z;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (f0 + q < D) out_g[row * D + f0 + q] = z[q];
        }
      }
    }
    if (score) {
      dot += __shfl_xor(dot, 16);
      dot += __shfl_xor(dot, 32);
      nz += __shfl_xor(nz, 16);
      nz += __shfl_xor(nz, 32);
      if (g == 0 && valid) {
        float sc = dot;
        if (normalize) {
          const float n = sqrtf(nz);
          sc = n > 0.0f ? dot / n : 0.0f;
        }
        score[row] = sc;
      }
    }
  }
}

// Mean over samples of the (optionally L2-normalised) rows: targets[t][k] = mean_s v[t][s][k] / |v[t][s]|.
__global__ __launch_bounds__(256) void k_extractor_targets(const float* __restrict__ vecs, int n_samples, int dim,
                                                           int normalize, float* __restrict__ targets) {
  __shared__ float inv[64];
  const float* V = vecs + (int64_t)blockIdx.x * n_samples * dim;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int s = w; s < n_samples; s += (int)(blockDim.x >> 6)) {
    float ss = 0.0f;
    for (int k = lane; k < dim; k += 64) ss += V[s * dim + k] * V[s * dim + k];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) ss += __shfl_xor(ss, sh);
    if (lane == 0) inv[s] = normalize ? (ss > 0.0f ? 1.0f / sqrtf(ss) : 0.0f) : 1.0f;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < dim; k += blockDim.x) {
    float t = 0.0f;
    for (int s = 0; s < n_samples; ++s) t += V[s * dim + k] * inv[s];
    targets[(int64_t)blockIdx.x * dim + k] = t / (float)n_samples;
  }
}

// rank of the first entry of each list among its list, descending: 1 + #(s_j > s_0).
__global__ __launch_bounds__(256) void k_rank_desc(const float* __restrict__ scores, const int64_t* __restrict__ off,
                                                   int64_t n_query, int32_t* __restrict__ rank) {
  __shared__ int red[4];
  for (int64_t q = blockIdx.x; q < n_query; q += gridDim.x) {
    const int64_t a = off[q], b = off[q + 1];
    int better = 0;
    if (b > a) {
      const float s0 = scores[a];
      for (int64_t j = a + 1 + threadIdx.x; j < b; j += blockDim.x) better += scores[j] > s0;
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) better += __shfl_xor(better, s);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = better;
    __syncthreads();
    if (threadIdx.x == 0) rank[q] = b > a ? red[0] + red[1] + red[2] + red[3] + 1 : 0;
  }
}

template <int D>
struct XDispatch {
  static int pack(const float* const* w, float* d_pack, hipStream_t st) {
    hipLaunchKernelGGL(k_extractor_pack<D>, dim3(512), dim3(256), 0, st, w[0], w[1], w[2], w[3], w[4], w[5], w[6],
                       w[7], w[8], w[9], w[10], w[11], w[12], w[13], d_pack);
    MMRE_CHECK_LAUNCH();
    return MMRE_OK;
  }
  static int nodes(const float* pack, const float* emb, const int64_t* node_sym, const int64_t* conn, int max_nb,
                   const float* deg, int64_t n_nodes, float* left, float* right, hipStream_t st) {
    const unsigned blocks = (unsigned)((n_nodes + NB - 1) / NB);
    hipLaunchKernelGGL(k_extractor_nodes<D>, dim3(blocks), dim3(256), 0, st, pack, emb, node_sym, conn, max_nb, deg,
                       n_nodes, left, right);
    MMRE_CHECK_LAUNCH();
    return MMRE_OK;
  }
  static int encode(const float* pack, float ln_eps, const float* left, const int64_t* li, const float* right,
                    const int64_t* ri, int64_t n_rows, const float* targets, const int64_t* row_target, int normalize,
                    float* out_g, float* score, hipStream_t st) {
    const int64_t tiles = (n_rows + 63) / 64;
    static int resident = 0;
    if (!resident) {
      int dev = 0, cus = 256, per = 0;
      if (hipGetDevice(&dev) == hipSuccess) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
      }
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(k_extractor_encode<D>),
                                                       256, 0) != hipSuccess || per <= 0)
        per = 1;
      resident = cus * per;
    }
    const unsigned blocks = (unsigned)(tiles < resident ? tiles : resident);
    hipLaunchKernelGGL(k_extractor_encode<D>, dim3(blocks), dim3(256), 0, st, pack, ln_eps, left, li, right, ri,
                       n_rows, targets, row_target, normalize, out_g, score);
    MMRE_CHECK_LAUNCH();
    return MMRE_OK;
  }
};

#define MMRE_X_DISPATCH(dim, CALL)   \
  switch (dim) {                     \
    case 64: return XDispatch<64>::CALL;   \
    case 100: return XDispatch<100>::CALL; \
    case 128: return XDispatch<128>::CALL; \
    case 200: return XDispatch<200>::CALL; \
    case 256: return XDispatch<256>::CALL; \
    default: return MMRE_ERR_SHAPE;  \
  }

static int64_t pack_size(int dim) {
  switch (dim) {
    case 64: return XG<64>::SIZE;
    case 100: return XG<100>::SIZE;
    case 128: return XG<128>::SIZE;
    case 200: return XG<200>::SIZE;
    case 256: return XG<256>::SIZE;
    default: return -1;
  }
}

}  // namespace mmre

using namespace mmre;

extern "C" int64_t mmre_extractor_pack_size(int dim) { return pack_size(dim); }

extern "C" int mmre_extractor_pack(int dim, const float* d_gcn_w, const float* d_gcn_b, const float* d_fc1_w,
                                   const float* d_fc1_b, const float* d_fc2_w, const float* d_fc2_b,
                                   const float* d_rs_w, const float* d_rs_b, const float* d_p1_w, const float* d_p1_b,
                                   const float* d_p2_w, const float* d_p2_b, const float* d_ln_w, const float* d_ln_b,
                                   float* d_pack, void* stream) {
  const float* w[14] = {d_gcn_w, d_gcn_b, d_fc1_w, d_fc1_b, d_fc2_w, d_fc2_b, d_rs_w,
                        d_rs_b,  d_p1_w,  d_p1_b,  d_p2_w,  d_p2_b,  d_ln_w, d_ln_b};
  for (const float* p : w)
    if (!p) return MMRE_ERR_ARG;
  if (!d_pack) return MMRE_ERR_ARG;
  MMRE_X_DISPATCH(dim, pack(w, d_pack, (hipStream_t)stream));
}

extern "C" int mmre_extractor_nodes(int dim, const float* d_pack, const float* d_sym_emb, const int64_t* d_node_sym,
                                    const int64_t* d_conn, int max_nb, const float* d_deg, int64_t n_nodes,
                                    float* d_left, float* d_right, void* stream) {
  if (!d_pack || !d_sym_emb || !d_node_sym || !d_deg || (!d_left && !d_right) || n_nodes <= 0 || max_nb < 0)
    return MMRE_ERR_ARG;
  if (max_nb > 0 && !d_conn) return MMRE_ERR_ARG;
  MMRE_X_DISPATCH(dim, nodes(d_pack, d_sym_emb, d_node_sym, d_conn, max_nb, d_deg, n_nodes, d_left, d_right,
                             (hipStream_t)stream));
}

extern "C" int mmre_extractor_encode(int dim, const float* d_pack, float ln_eps, const float* d_left,
                                     const int64_t* d_li, const float* d_right, const int64_t* d_ri, int64_t n_rows,
                                     const float* d_targets, const int64_t* d_row_target, int normalize,
                                     float* d_out_g, float* d_score, void* stream) {
  if (!d_pack || !d_left || !d_li || !d_right || !d_ri || n_rows <= 0 || (!d_out_g && !d_score)) return MMRE_ERR_ARG;
  if (d_score && !d_targets) return MMRE_ERR_ARG;
  MMRE_X_DISPATCH(dim, encode(d_pack, ln_eps, d_left, d_li, d_right, d_ri, n_rows, d_targets, d_row_target, normalize,
                              d_out_g, d_score, (hipStream_t)stream));
}

extern "C" int mmre_extractor_targets(const float* d_vecs, int64_t n_sets, int n_samples, int dim, int normalize,
                                      float* d_targets, void* stream) {
  if (!d_vecs || !d_targets || n_sets <= 0 || n_samples <= 0 || dim <= 0) return MMRE_ERR_ARG;
  if (n_samples > 64) return MMRE_ERR_SHAPE;
  hipLaunchKernelGGL(k_extractor_targets, dim3((unsigned)n_sets), dim3(256), 0, (hipStream_t)stream, d_vecs,
                     n_samples, dim, normalize, d_targets);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_rank_desc(const float* d_scores, const int64_t* d_off, int64_t n_query, int32_t* d_rank,
                              void* stream) {
  if (!d_scores || !d_off || !d_rank || n_query <= 0) return MMRE_ERR_ARG;
  const unsigned blocks = (unsigned)(n_query < 16384 ? n_query : 16384);
  hipLaunchKernelGGL(k_rank_desc, dim3(blocks), dim3(256), 0, (hipStream_t)stream, d_scores, d_off, n_query, d_rank);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
