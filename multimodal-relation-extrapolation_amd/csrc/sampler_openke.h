// sampler_openke.h -- device code of OpenKE's filtered sampler (Base.cpp:78-197 getBatch /
// sampling, Corrupt.h:7-163, Random.h:11-29), bit-exact with Base.so: shared by sampler.hip's
// kernels and the training-step kernel of ns.hip (mmre_ns_step_openke), which runs the sampler's
// workgroups beside the NS pre-pass in one launch. Static device functions only (included by
// more than one translation unit).
#pragma once
#include "mmre_common.h"

namespace mmre {

static __device__ __forceinline__ uint64_t lcg_next(uint64_t* st) {
  *st = *st * 25214903917ULL + 11ULL;
  return *st;
}
static __device__ __forceinline__ int64_t rand_max(uint64_t* st, int64_t x) {
  return (int64_t)(lcg_next(st) % (uint64_t)x);
}
static __device__ uint64_t lcg_jump(uint64_t x, uint64_t n) {
  uint64_t A = 1, C = 0, a = 25214903917ULL, c = 11ULL;
  while (n) {
    if (n & 1) { A = A * a; C = C * a + c; }
    c = c * a + c;
    a = a * a;
    n >>= 1;
  }
  return A * x + C;
}

// The block [ll, rr] of rows whose column `kc` equals `key` inside the sorted range
// [lef0, rig0] (Corrupt.h's two binary searches, same midpoints and results) -- the lower and
// upper searches advance together, so their dependent loads are issued in pairs and the chain
// is as long as one search.
static __device__ __forceinline__ void key_block(const int64_t* __restrict__ T, int kc, int64_t lef0, int64_t rig0,
                                          int64_t key, int64_t& ll, int64_t& rr) {
  int64_t al = lef0 - 1, ar = rig0, bl = lef0, br = rig0 + 1;
  while (al + 1 < ar || bl + 1 < br) {
    const bool ga = al + 1 < ar, gb = bl + 1 < br;
    const int64_t ma = (al + ar) >> 1, mb = (bl + br) >> 1;
    const int64_t va = ga ? T[3 * ma + kc] : 0, vb = gb ? T[3 * mb + kc] : 0;
    if (ga) { if (va >= key) ar = ma; else al = ma; }
    if (gb) { if (vb <= key) bl = mb; else br = mb; }
  }
  ll = ar;
  rr = bl;
}

// The draw and the final skip of Corrupt.h's corruption, given the block [ll, rr] of rows of T
// sharing the kept (entity, relation) and its first / last value `tll` / `trr` in column col:
// a uniform id among the n - (rr - ll + 1) ids not in the block.
static __device__ int64_t corrupt_in_block(const int64_t* __restrict__ T, int col, int64_t n, uint64_t* st, int64_t ll,
                                    int64_t rr, int64_t tll, int64_t trr) {
  const int64_t tmp = rand_max(st, n - (rr - ll + 1));
  if (tmp < tll) return tmp;
  if (tmp > trr - rr + ll - 1) return tmp + rr - ll + 1;
  int64_t lef = ll, rig = rr + 1, mid;
  while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + col] - mid + ll - 1 < tmp) lef = mid; else rig = mid; }
  return tmp + lef - ll + 1;
}

// corrupt_head (Corrupt.h:7-43): uniform entity not among the known TAILS of (h, r),
// found by skipping the sorted tails of the (h, r) block of trainHead.
static __device__ int64_t corrupt_head(const int64_t* __restrict__ T, const int64_t* __restrict__ lef_head,
                                const int64_t* __restrict__ rig_head, int64_t n_ent, uint64_t* st, int64_t h,
                                int64_t r) {
  int64_t ll, rr;
  key_block(T, 1, lef_head[h], rig_head[h], r, ll, rr);
  return corrupt_in_block(T, 2, n_ent, st, ll, rr, T[3 * ll + 2], T[3 * rr + 2]);
}

// corrupt_tail (Corrupt.h:45-81): uniform entity not among the known HEADS of (t, r);
// T rows are (h, r, t) sorted by (t, r, h).
static __device__ int64_t corrupt_tail(const int64_t* __restrict__ T, const int64_t* __restrict__ lef_tail,
                                const int64_t* __restrict__ rig_tail, int64_t n_ent, uint64_t* st, int64_t t,
                                int64_t r) {
  int64_t ll, rr;
  key_block(T, 1, lef_tail[t], rig_tail[t], r, ll, rr);
  return corrupt_in_block(T, 0, n_ent, st, ll, rr, T[3 * ll + 0], T[3 * rr + 0]);
}

// corrupt_rel with p == true (Corrupt.h:111-147): the draw among the relations not in the (h, t)
// block, weighted by r's row of importProb's table P (Reader.h:26-49; n_rel - 1 columns, r's own
// left out: column c is relation c below r, c + 1 from r on). The reference builds, per draw, the
// cumulative list of P[c] / sum over the unmarked columns (sum = 1 - the marked columns' mass,
// subtracted in block order) and binary-searches it for m = rand_max(10000) / 10000. Here the
// list is never stored: each probe of the same binary search recomputes its prefix in the same
// order (the block's columns are ascending, so one merge walk marks them), which yields the
// same float values, hence the same index (the compacted index; corrupt_rel maps it to an id).
static __device__ float rel_prob_prefix(const int64_t* __restrict__ T, const float* __restrict__ P, int64_t n_rel,
                                 int64_t r, int64_t ll, int64_t rr, float sum, int64_t upto) {
  float rec = 0.0f;
  int64_t q = ll, c = 0;
  for (int64_t i = 0; i < n_rel - 1; ++i) {
    int64_t col = -1;  // the next marked column at or after i
    while (q <= rr) {
      const int64_t rel = T[3 * q + 1];
      col = rel > r ? rel - 1 : (rel < r ? rel : -1);
      if (col >= i) break;
      ++q;
      col = -1;
    }
    if (col == i) continue;  // in the (h, t) block
    rec += P[i] / sum;
    if (c == upto) return rec;
    ++c;
  }
  return rec;
}

static __device__ int64_t rel_prob_draw(const int64_t* __restrict__ T, const float* __restrict__ prob, int64_t n_rel,
                                 uint64_t* st, int64_t r, int64_t ll, int64_t rr) {
  const float* P = prob + r * (n_rel - 1);
  float sum = 1.0f;
  int64_t marked = 0;
  for (int64_t i = ll; i <= rr; ++i) {
    const int64_t rel = T[3 * i + 1];
    if (rel > r) { sum -= P[rel - 1]; ++marked; }
    else if (rel < r) { sum -= P[rel]; ++marked; }
  }
  const int64_t cnt = (n_rel - 1) - marked;
  const float m = (float)((double)rand_max(st, 10000) / 10000.0);
  int64_t lef = 0, rig = cnt - 1;
  while (lef < rig) {
    const int64_t mid = (lef + rig) >> 1;
    if (rel_prob_prefix(T, P, n_rel, r, ll, rr, sum, mid) < m) lef = mid + 1;
    else rig = mid;
  }
  return rig;
}

// corrupt_rel (Corrupt.h:85-162); T rows (h, r, t) sorted by (h, t, r). prob NULL: p == false,
// a uniform draw; else importProb's table (p == true).
static __device__ int64_t corrupt_rel(const int64_t* __restrict__ T, const int64_t* __restrict__ lef_rel,
                               const int64_t* __restrict__ rig_rel, int64_t n_rel, uint64_t* st, int64_t h, int64_t t,
                               int64_t r, const float* __restrict__ prob) {
  int64_t lef, rig, mid, ll, rr;
  key_block(T, 2, lef_rel[h], rig_rel[h], t, ll, rr);
  const int64_t tmp = prob ? rel_prob_draw(T, prob, n_rel, st, r, ll, rr) : rand_max(st, n_rel - (rr - ll + 1));
  if (tmp < T[3 * ll + 1]) return tmp;
  if (tmp > T[3 * rr + 1] - rr + ll - 1) return tmp + rr - ll + 1;
  lef = ll; rig = rr + 1;
  while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 1] - mid + ll - 1 < tmp) lef = mid; else rig = mid; }
  return tmp + lef - ll + 1;
}

// One GPU thread per output ROW (positive or negative): the state before any draw is the
// pthread's seed advanced by an affine jump, so the rows of one positive -- a chain of up to
// 1 + 2 neg dependent draws and binary searches in the reference -- are produced in parallel
// (B (1 + neg + neg_rel) threads instead of B).
static __device__ __forceinline__ void sampler_openke_row(int64_t row, 
    const int64_t* __restrict__ train_list, int64_t train_total, const int64_t* __restrict__ head_hrt,
    const int64_t* __restrict__ tail_hrt, const int64_t* __restrict__ rel_hrt, const int64_t* __restrict__ lef_head,
    const int64_t* __restrict__ rig_head, const int64_t* __restrict__ lef_tail, const int64_t* __restrict__ rig_tail,
    const int64_t* __restrict__ lef_rel, const int64_t* __restrict__ rig_rel, const float* __restrict__ left_mean,
    const float* __restrict__ right_mean, int64_t n_ent, int64_t n_rel, const uint64_t* __restrict__ seeds,
    int64_t work_threads, int64_t B, int64_t neg, int64_t neg_rel, int64_t mode, const int32_t* __restrict__ blk,
    int64_t n_blk, int64_t* __restrict__ bh, int64_t* __restrict__ bt, int64_t* __restrict__ br,
    float* __restrict__ by, const float* __restrict__ rel_prob) {
  const int64_t b = row % B, j = row / B;  // j = 0: the positive; 1..neg: entity negatives; then relation ones
  // slice of the reference's pthread `id` that owns position b (Base.cpp:93-100)
  const int64_t per = B % work_threads == 0 ? B / work_threads : B / work_threads + 1;
  const int64_t id = b / per, lef = id * per;
  const int64_t per_neg = mode == 0 ? 2 : 1;  // draws per entity negative: [prob draw,] corrupt draw
  const int64_t draws = 1 + per_neg * neg + neg_rel;
  const uint64_t base = (uint64_t)((b - lef) * draws);
  uint64_t st = lcg_jump(seeds[id], base);
  const int64_t i = rand_max(&st, train_total);  // Base.cpp:104
  const int64_t h = train_list[3 * i], r = train_list[3 * i + 1], t = train_list[3 * i + 2];
  if (j == 0) {
    bh[row] = h; bt[row] = t; br[row] = r; by[row] = 1.0f;
    return;
  }
  if (j <= neg) {
    const int64_t k = j - 1;
    st = lcg_jump(seeds[id], base + 1 + (uint64_t)(per_neg * k));
    bool replace_tail;
    if (mode == 0) {
      float prob = 500.0f;
      if (left_mean) prob = 1000.0f * right_mean[r] / (right_mean[r] + left_mean[r]);
      replace_tail = (float)(lcg_next(&st) % 1000ULL) < prob;
    } else {
      replace_tail = mode != -1;
    }
    // the kept (entity, relation)'s block: from the per-train-row table when there is one
    const bool pre = i < n_blk;
    int4 kb = make_int4(0, 0, 0, 0);
    if (pre) kb = reinterpret_cast<const int4*>(blk + 8 * i)[replace_tail ? 0 : 1];
    if (replace_tail) {  // corrupt_head returns a replacement TAIL (Base.cpp:116)
      bh[row] = h; br[row] = r;
      bt[row] = pre ? corrupt_in_block(head_hrt, 2, n_ent, &st, kb.x, kb.y, kb.z, kb.w)
                    : corrupt_head(head_hrt, lef_head, rig_head, n_ent, &st, h, r);
    } else {
      bt[row] = t; br[row] = r;
      bh[row] = pre ? corrupt_in_block(tail_hrt, 0, n_ent, &st, kb.x, kb.y, kb.z, kb.w)
                    : corrupt_tail(tail_hrt, lef_tail, rig_tail, n_ent, &st, t, r);
    }
  } else {
    const int64_t k = j - 1 - neg;
    st = lcg_jump(seeds[id], base + 1 + (uint64_t)(per_neg * neg + k));
    bh[row] = h; bt[row] = t; br[row] = corrupt_rel(rel_hrt, lef_rel, rig_rel, n_rel, &st, h, t, r, rel_prob);
  }
  by[row] = -1.0f;
}


// The per-pthread LCG states after one sampling call (mmre_sampler_advance's arithmetic):
// thread id's state jumps by (its positives) x (draws per positive), its positives being
// Base.cpp:161-197's [lef, rig) split of the batch.
static __device__ __forceinline__ uint64_t advanced_seed(uint64_t seed, int64_t id, int64_t work_threads,
                                                  int64_t batch_size, int64_t per) {
  int64_t lef, rig;
  if (batch_size % work_threads == 0) {
    lef = id * (batch_size / work_threads);
    rig = (id + 1) * (batch_size / work_threads);
  } else {
    lef = id * (batch_size / work_threads + 1);
    rig = (id + 1) * (batch_size / work_threads + 1);
    if (rig > batch_size) rig = batch_size;
  }
  const int64_t cnt = rig > lef ? rig - lef : 0;
  return lcg_jump(seed, (uint64_t)(cnt * per));
}

// The OpenKE sampler's arguments (mmre_sampler_openke*): the Reader.h train index, bern
// statistics, per-pthread LCG states, batch shape and outputs.
struct OpenKESamplerArgs {
  const int64_t *train_list, *head_hrt, *tail_hrt, *rel_hrt, *lef_head, *rig_head, *lef_tail, *rig_tail, *lef_rel,
      *rig_rel;
  const float *left_mean, *right_mean;
  int64_t train_total, n_ent, n_rel;
  uint64_t* seeds;
  int64_t work_threads, B, neg, neg_rel, mode;
  const int32_t* blk;
  int64_t n_blk;
  int64_t *bh, *bt, *br;
  float* by;
  int32_t* ticket;
  int64_t adv_per;
  const float* rel_prob;
};

// One workgroup `block` of `nblocks` sampler workgroups, one thread per output row. With `ticket`
// (mmre_sampler_openke_step) the call also advances the seeds for the next call: every
// workgroup takes a ticket once all its threads have read the seeds; the last one writes the
// advanced states and resets the ticket -- no separate advance launch behind every batch.
static __device__ void sampler_openke_block(const OpenKESamplerArgs& a, int64_t block, int64_t nblocks) {
  const int64_t row = block * blockDim.x + threadIdx.x;
  if (row < a.B * (1 + a.neg + a.neg_rel))
    sampler_openke_row(row, a.train_list, a.train_total, a.head_hrt, a.tail_hrt, a.rel_hrt, a.lef_head, a.rig_head,
                       a.lef_tail, a.rig_tail, a.lef_rel, a.rig_rel, a.left_mean, a.right_mean, a.n_ent, a.n_rel,
                       a.seeds, a.work_threads, a.B, a.neg, a.neg_rel, a.mode, a.blk, a.n_blk, a.bh, a.bt, a.br, a.by,
                       a.rel_prob);
  if (a.ticket == nullptr) return;  // uniform
  __syncthreads();  // every thread of the workgroup has read (and used) its seed
  __shared__ int s_last;
  if (threadIdx.x == 0) s_last = atomicAdd(a.ticket, 1) == (int)nblocks - 1;
  __syncthreads();
  if (!s_last) return;
  for (int64_t id = threadIdx.x; id < a.work_threads; id += blockDim.x)
    a.seeds[id] = advanced_seed(a.seeds[id], id, a.work_threads, a.B, a.adv_per);
  if (threadIdx.x == 0) *a.ticket = 0;
}

}  // namespace mmre
