// host.cpp -- host-side parts of the C ABI: version, the Test.h metric reduction
// with the reference's float accumulation order, glibc rand() seeds and the
// sampler's per-thread LCG bookkeeping.
#include <stdint.h>
#include <stdlib.h>

#include <vector>

#include "../../include/mmre.h"

extern "C" int mmre_version(void) { return 100; }

// test_link_prediction (Test.h:232-327): per side, accumulate in query order into
// float globals exactly as testHead/testTail do (Test.h:102-112: `+= 1` on float,
// `+= (count+1)` long->float, `+= 1.0/(count+1)` in double then stored as float),
// then divide by testTotal (float) and average the two sides (float).
static void side(const int32_t* c, int64_t n, int64_t stride, int col, float tot, float out[5]) {
  float t10 = 0, t3 = 0, t1 = 0, rank = 0, reci = 0;
  const int32_t* p = c + (int64_t)col * stride;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = p[i];
    if (s < 10) t10 += 1;
    if (s < 3) t3 += 1;
    if (s < 1) t1 += 1;
    rank += (float)(s + 1);
    reci = (float)((double)reci + 1.0 / (double)(s + 1));
  }
  out[0] = reci / tot;
  out[1] = rank / tot;
  out[2] = t10 / tot;
  out[3] = t3 / tot;
  out[4] = t1 / tot;
}

extern "C" int mmre_link_metrics(const int32_t* h_head_counts, const int32_t* h_tail_counts, int64_t n,
                                 int64_t stride, float* h_out) {
  if (!h_head_counts || !h_tail_counts || !h_out || n <= 0 || stride < n) return MMRE_ERR_ARG;
  const float tot = (float)n;
  const int cols[4] = {1, 0, 3, 2};  // filter, raw, filter_tc, raw_tc
  for (int g = 0; g < 4; ++g) {
    float l[5], r[5];
    side(h_head_counts, n, stride, cols[g], tot, l);
    side(h_tail_counts, n, stride, cols[g], tot, r);
    for (int i = 0; i < 5; ++i) h_out[5 * g + i] = (l[i] + r[i]) / 2;
  }
  return MMRE_OK;
}

// glibc random() TYPE_3 after srand(1): r[i] = r[i-31] + r[i-3], output r[i+344] >> 1.
// randReset (Random.h:11-15) seeds thread i with the next rand() of the process.
extern "C" int mmre_glibc_rand(int64_t skip, int64_t n, int64_t* h_out) {
  if (skip < 0 || n < 0 || (n > 0 && !h_out)) return MMRE_ERR_ARG;
  const int64_t total = 344 + skip + n;
  std::vector<int32_t> v((size_t)total + 1);
  v[0] = 1;
  for (int i = 1; i < 31; ++i) {
    int64_t hi = v[i - 1] / 127773, lo = v[i - 1] % 127773;
    int64_t w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    v[i] = (int32_t)w;
  }
  for (int i = 31; i < 34; ++i) v[i] = v[i - 31];
  for (int64_t i = 34; i < total; ++i) v[i] = (int32_t)((uint32_t)v[i - 31] + (uint32_t)v[i - 3]);
  for (int64_t i = 0; i < n; ++i) h_out[i] = (int64_t)(((uint32_t)v[344 + skip + i]) >> 1);
  return MMRE_OK;
}

// Draws per positive in getBatch (Base.cpp:103-146): 1 (the positive) + 2 per
// entity negative in mode 0 (Bernoulli draw + corrupt), 1 per negative otherwise,
// + 1 per relation negative.
extern "C" int64_t mmre_sampler_draws_per_positive(int64_t neg_rate, int64_t neg_rel_rate, int64_t mode) {
  return 1 + (mode == 0 ? 2 : 1) * neg_rate + neg_rel_rate;
}

static uint64_t lcg_pow_apply(uint64_t x, uint64_t n) {
  // x -> a^n x + c (a^{n-1} + ... + 1), a = 25214903917, c = 11 (mod 2^64)
  uint64_t A = 1, C = 0, a = 25214903917ULL, c = 11ULL;
  while (n) {
    if (n & 1) { A = A * a; C = C * a + c; }
    c = c * a + c;
    a = a * a;
    n >>= 1;
  }
  return A * x + C;
}

extern "C" int mmre_sampler_advance(uint64_t* h_seeds, int64_t work_threads, int64_t batch_size, int64_t neg_rate,
                                    int64_t neg_rel_rate, int64_t mode) {
  if (!h_seeds || work_threads <= 0 || batch_size <= 0 || neg_rate < 0 || neg_rel_rate < 0) return MMRE_ERR_ARG;
  const int64_t per = mmre_sampler_draws_per_positive(neg_rate, neg_rel_rate, mode);
  for (int64_t id = 0; id < work_threads; ++id) {
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
    h_seeds[id] = lcg_pow_apply(h_seeds[id], (uint64_t)(cnt * per));
  }
  return MMRE_OK;
}
