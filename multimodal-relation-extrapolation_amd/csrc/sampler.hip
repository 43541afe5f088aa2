// sampler.hip -- negative samplers on the GPU.
//
// 1. OpenKE's filtered sampler (Base.cpp:78-197 getBatch/sampling, Corrupt.h:7-163,
//    Random.h:11-29), bit-exact. The reference runs `workThreads` pthreads, thread `id`
//    filling the slice [lef, rig) of the batch sequentially from its own 64-bit LCG
//    (next = next * 25214903917 + 11). Every positive consumes a FIXED number of draws
//    (1 + 2*neg_rate in mode 0, 1 + neg_rate otherwise, + neg_rel_rate), so the state at
//    the start of positive b is the thread seed advanced by (b - lef) * draws via an
//    affine jump-ahead -- and so is the state before any negative's draws: one GPU thread per
//    output row, same outputs as the pthreads.
// 2. The repo's per-edge sampler (module/NegativeSampling.py:114-140, 321-375): per
//    positive, Bernoulli(0.5) head/tail split of the neg_ent negatives, candidates drawn
//    uniformly from the local node list [0, n_local) (NegativeSampling.py:210) and rejected
//    when their global id is a known head of (t, r) / tail of (h, r) (filter_flag), distinct
//    within a positive. The reference's draws come from the unseeded Python `random` (P13),
//    so parity is distributional; this kernel uses a counter-based generator (SplitMix64) so
//    a given seed is reproducible.
#include "mmre_common.h"
#include "sampler_openke.h"

namespace mmre {

// Per train row i (h, r, t): the (h, r) block of head_hrt with its first / last tail and the
// (t, r) block of tail_hrt with its first / last head -- what corrupt_head / corrupt_tail find
// before their draw -- as int32 [i][8]. Built once per train index, it shortens a sampled
// row's chain of dependent loads to seeds -> train row -> its blocks (-> rarely the skip).
__global__ __launch_bounds__(256) void k_sampler_blocks(const int64_t* __restrict__ train_list, int64_t n,
                                                        const int64_t* __restrict__ head_hrt,
                                                        const int64_t* __restrict__ tail_hrt,
                                                        const int64_t* __restrict__ lef_head,
                                                        const int64_t* __restrict__ rig_head,
                                                        const int64_t* __restrict__ lef_tail,
                                                        const int64_t* __restrict__ rig_tail, int32_t* __restrict__ blk) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t h = train_list[3 * i], r = train_list[3 * i + 1], t = train_list[3 * i + 2];
  int64_t ll, rr, tl, tr;
  key_block(head_hrt, 1, lef_head[h], rig_head[h], r, ll, rr);
  key_block(tail_hrt, 1, lef_tail[t], rig_tail[t], r, tl, tr);
  int4* o = reinterpret_cast<int4*>(blk + 8 * i);
  o[0] = make_int4((int)ll, (int)rr, (int)head_hrt[3 * ll + 2], (int)head_hrt[3 * rr + 2]);
  o[1] = make_int4((int)tl, (int)tr, (int)tail_hrt[3 * tl + 0], (int)tail_hrt[3 * tr + 0]);
}

// One sampling() call: sampler_openke_block over the grid.
__global__ __launch_bounds__(256) void k_sampler_openke(OpenKESamplerArgs a) {
  sampler_openke_block(a, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------- repo sampler --
__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// Is global entity g in the sorted value list of `key` (CSR over sorted keys)?
__device__ bool in_filter(const int64_t* __restrict__ keys, const int64_t* __restrict__ off,
                          const int64_t* __restrict__ vals, int64_t n_keys, int64_t key, int64_t g) {
  int64_t lo = 0, hi = n_keys;
  while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (keys[mid] < key) lo = mid + 1; else hi = mid; }
  if (lo >= n_keys || keys[lo] != key) return false;
  int64_t a = off[lo], b = off[lo + 1];
  while (a < b) { int64_t mid = (a + b) >> 1; if (vals[mid] < g) a = mid + 1; else b = mid; }
  return a < off[lo + 1] && vals[a] == g;
}

__global__ void k_sampler_repo(const int64_t* __restrict__ eh, const int64_t* __restrict__ et,
                               const int64_t* __restrict__ er, int64_t B, int64_t neg, int64_t n_local,
                               const int64_t* __restrict__ local_to_global, int64_t n_rel,
                               const int64_t* __restrict__ hf_keys, const int64_t* __restrict__ hf_off,
                               const int64_t* __restrict__ hf_vals, int64_t hf_n,
                               const int64_t* __restrict__ tf_keys, const int64_t* __restrict__ tf_off,
                               const int64_t* __restrict__ tf_vals, int64_t tf_n, uint64_t seed, int filter_flag,
                               int64_t* __restrict__ out_h, int64_t* __restrict__ out_t, int64_t* __restrict__ out_r) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t h = eh[b], t = et[b], r = er[b];
  out_h[b] = h; out_t[b] = t; out_r[b] = r;
  uint64_t ctr = splitmix(seed ^ (uint64_t)b * 0xD1B54A32D192ED03ULL);
  // Bernoulli(0.5) split (NegativeSampling.py:324-329): heads first, then tails
  int64_t n_head = 0;
  for (int64_t k = 0; k < neg; ++k) {
    ctr = splitmix(ctr);
    n_head += (ctr >> 11) * (1.0 / 9007199254740992.0) < 0.5;
  }
  const int64_t gh = local_to_global ? local_to_global[h] : h;
  const int64_t gt = local_to_global ? local_to_global[t] : t;
  for (int64_t k = 0; k < neg; ++k) {
    const bool corrupt_h = k < n_head;
    int64_t cand = 0;
    for (int tries = 0; tries < 4096; ++tries) {
      ctr = splitmix(ctr);
      cand = (int64_t)(ctr % (uint64_t)n_local);
      const int64_t g = local_to_global ? local_to_global[cand] : cand;
      bool bad = false;
      if (filter_flag) {
        bad = corrupt_h ? in_filter(hf_keys, hf_off, hf_vals, hf_n, gt * n_rel + r, g)
                        : in_filter(tf_keys, tf_off, tf_vals, tf_n, gh * n_rel + r, g);
      }
      for (int64_t j = 0; j < k && !bad; ++j) {  // distinct within a positive (random.sample)
        const bool same_side = (j < n_head) == corrupt_h;
        if (same_side) bad = (corrupt_h ? out_h[b + (j + 1) * B] : out_t[b + (j + 1) * B]) == cand;
      }
      if (!bad) break;
    }
    const int64_t row = b + (k + 1) * B;
    out_h[row] = corrupt_h ? cand : h;
    out_t[row] = corrupt_h ? t : cand;
    out_r[row] = r;
  }
}

// The per-pthread LCG states after one sampling call, on the device (a launch of its own).
__global__ void k_sampler_advance(uint64_t* seeds, int64_t work_threads, int64_t batch_size, int64_t per) {
  const int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (id >= work_threads) return;
  seeds[id] = advanced_seed(seeds[id], id, work_threads, batch_size, per);
}

}  // namespace mmre

using namespace mmre;

extern "C" int mmre_sampler_advance_device(uint64_t* d_seeds, int64_t work_threads, int64_t batch_size,
                                           int64_t neg_rate, int64_t neg_rel_rate, int64_t mode, void* stream) {
  if (!d_seeds || work_threads <= 0 || batch_size <= 0 || neg_rate < 0 || neg_rel_rate < 0) return MMRE_ERR_ARG;
  const int64_t per = mmre_sampler_draws_per_positive(neg_rate, neg_rel_rate, mode);
  hipLaunchKernelGGL(k_sampler_advance, dim3((unsigned)((work_threads + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     d_seeds, work_threads, batch_size, per);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

static int sampler_impl(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                        const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                        const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                        const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                        const float* d_right_mean, int64_t n_ent, int64_t n_rel, const uint64_t* d_seeds,
                        int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate, int64_t mode,
                        const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h, int64_t* d_batch_t,
                        int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket, const float* d_rel_prob,
                        void* stream) {
  if (!d_train_list || !d_head_hrt || !d_tail_hrt || !d_lef_head || !d_rig_head || !d_lef_tail || !d_rig_tail ||
      !d_seeds || !d_batch_h || !d_batch_t || !d_batch_r || !d_batch_y)
    return MMRE_ERR_ARG;
  if (neg_rel_rate > 0 && (!d_rel_hrt || !d_lef_rel || !d_rig_rel)) return MMRE_ERR_ARG;
  if ((d_left_mean == nullptr) != (d_right_mean == nullptr)) return MMRE_ERR_ARG;
  if (train_total <= 0 || n_ent <= 1 || work_threads <= 0 || batch_size <= 0 || neg_rate < 0 || neg_rel_rate < 0)
    return MMRE_ERR_ARG;
  if (mode < -1 || mode > 1) return MMRE_ERR_ARG;
  if (n_blocks < 0 || (n_blocks > 0 && !d_blocks)) return MMRE_ERR_ARG;
  if (d_rel_prob && n_rel < 2) return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int threads = 256;
  const int64_t rows = batch_size * (1 + neg_rate + neg_rel_rate);
  const OpenKESamplerArgs a{d_train_list, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head, d_rig_head, d_lef_tail,
                            d_rig_tail, d_lef_rel, d_rig_rel, d_left_mean, d_right_mean, train_total, n_ent, n_rel,
                            const_cast<uint64_t*>(d_seeds), work_threads, batch_size, neg_rate, neg_rel_rate, mode,
                            d_blocks, n_blocks, d_batch_h, d_batch_t, d_batch_r, d_batch_y, d_ticket,
                            mmre_sampler_draws_per_positive(neg_rate, neg_rel_rate, mode), d_rel_prob};
  hipLaunchKernelGGL(k_sampler_openke, dim3((unsigned)((rows + threads - 1) / threads)), dim3(threads), 0, st, a);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_sampler_openke_blocked(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                                   const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                                   const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                                   const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                                   const float* d_right_mean, int64_t n_ent, int64_t n_rel, const uint64_t* d_seeds,
                                   int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate,
                                   int64_t mode, const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h,
                                   int64_t* d_batch_t, int64_t* d_batch_r, float* d_batch_y, void* stream) {
  return sampler_impl(d_train_list, train_total, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head, d_rig_head,
                      d_lef_tail, d_rig_tail, d_lef_rel, d_rig_rel, d_left_mean, d_right_mean, n_ent, n_rel, d_seeds,
                      work_threads, batch_size, neg_rate, neg_rel_rate, mode, d_blocks, n_blocks, d_batch_h,
                      d_batch_t, d_batch_r, d_batch_y, nullptr, nullptr, stream);
}

extern "C" int mmre_sampler_openke_step(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                                        const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                                        const int64_t* d_rig_head, const int64_t* d_lef_tail,
                                        const int64_t* d_rig_tail, const int64_t* d_lef_rel, const int64_t* d_rig_rel,
                                        const float* d_left_mean, const float* d_right_mean, int64_t n_ent,
                                        int64_t n_rel, uint64_t* d_seeds, int64_t work_threads, int64_t batch_size,
                                        int64_t neg_rate, int64_t neg_rel_rate, int64_t mode, const int32_t* d_blocks,
                                        int64_t n_blocks, int64_t* d_batch_h, int64_t* d_batch_t, int64_t* d_batch_r,
                                        float* d_batch_y, int32_t* d_ticket, void* stream) {
  if (!d_ticket) return MMRE_ERR_ARG;
  return sampler_impl(d_train_list, train_total, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head, d_rig_head,
                      d_lef_tail, d_rig_tail, d_lef_rel, d_rig_rel, d_left_mean, d_right_mean, n_ent, n_rel, d_seeds,
                      work_threads, batch_size, neg_rate, neg_rel_rate, mode, d_blocks, n_blocks, d_batch_h,
                      d_batch_t, d_batch_r, d_batch_y, d_ticket, nullptr, stream);
}

extern "C" int mmre_sampler_openke_p(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                                     const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                                     const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                                     const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                                     const float* d_right_mean, int64_t n_ent, int64_t n_rel, uint64_t* d_seeds,
                                     int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate,
                                     int64_t mode, const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h,
                                     int64_t* d_batch_t, int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket,
                                     const float* d_rel_prob, void* stream) {
  if (!d_rel_prob) return MMRE_ERR_ARG;
  return sampler_impl(d_train_list, train_total, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head, d_rig_head,
                      d_lef_tail, d_rig_tail, d_lef_rel, d_rig_rel, d_left_mean, d_right_mean, n_ent, n_rel, d_seeds,
                      work_threads, batch_size, neg_rate, neg_rel_rate, mode, d_blocks, n_blocks, d_batch_h,
                      d_batch_t, d_batch_r, d_batch_y, d_ticket, d_rel_prob, stream);
}

extern "C" int mmre_sampler_openke(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                                   const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                                   const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                                   const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                                   const float* d_right_mean, int64_t n_ent, int64_t n_rel, const uint64_t* d_seeds,
                                   int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate,
                                   int64_t mode, int64_t* d_batch_h, int64_t* d_batch_t, int64_t* d_batch_r,
                                   float* d_batch_y, void* stream) {
  return mmre_sampler_openke_blocked(d_train_list, train_total, d_head_hrt, d_tail_hrt, d_rel_hrt, d_lef_head,
                                     d_rig_head, d_lef_tail, d_rig_tail, d_lef_rel, d_rig_rel, d_left_mean,
                                     d_right_mean, n_ent, n_rel, d_seeds, work_threads, batch_size, neg_rate,
                                     neg_rel_rate, mode, nullptr, 0, d_batch_h, d_batch_t, d_batch_r, d_batch_y,
                                     stream);
}

extern "C" int mmre_sampler_blocks(const int64_t* d_train_list, int64_t n_train, const int64_t* d_head_hrt,
                                   const int64_t* d_tail_hrt, const int64_t* d_lef_head, const int64_t* d_rig_head,
                                   const int64_t* d_lef_tail, const int64_t* d_rig_tail, int32_t* d_blocks,
                                   void* stream) {
  if (!d_train_list || !d_head_hrt || !d_tail_hrt || !d_lef_head || !d_rig_head || !d_lef_tail || !d_rig_tail ||
      !d_blocks || n_train <= 0)
    return MMRE_ERR_ARG;
  if (n_train > INT32_MAX) return MMRE_ERR_SHAPE;  // int32 block rows
  hipLaunchKernelGGL(k_sampler_blocks, dim3((unsigned)((n_train + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     d_train_list, n_train, d_head_hrt, d_tail_hrt, d_lef_head, d_rig_head, d_lef_tail, d_rig_tail,
                     d_blocks);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}

extern "C" int mmre_sampler_repo(const int64_t* d_eh, const int64_t* d_et, const int64_t* d_er, int64_t batch,
                                 int64_t neg, int64_t n_local, const int64_t* d_local_to_global, int64_t n_rel,
                                 const int64_t* d_hf_keys, const int64_t* d_hf_off, const int64_t* d_hf_vals,
                                 int64_t hf_n, const int64_t* d_tf_keys, const int64_t* d_tf_off,
                                 const int64_t* d_tf_vals, int64_t tf_n, uint64_t seed, int filter_flag,
                                 int64_t* d_out_h, int64_t* d_out_t, int64_t* d_out_r, void* stream) {
  if (!d_eh || !d_et || !d_er || !d_out_h || !d_out_t || !d_out_r || batch <= 0 || neg < 0 || n_local <= 0)
    return MMRE_ERR_ARG;
  if (filter_flag && (!d_hf_keys || !d_hf_off || !d_hf_vals || !d_tf_keys || !d_tf_off || !d_tf_vals))
    return MMRE_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int threads = 64;
  hipLaunchKernelGGL(k_sampler_repo, dim3((unsigned)((batch + threads - 1) / threads)), dim3(threads), 0, st, d_eh,
                     d_et, d_er, batch, neg, n_local, d_local_to_global, n_rel, d_hf_keys, d_hf_off, d_hf_vals, hf_n,
                     d_tf_keys, d_tf_off, d_tf_vals, tf_n, seed, filter_flag, d_out_h, d_out_t, d_out_r);
  MMRE_CHECK_LAUNCH();
  return MMRE_OK;
}
