// host.cpp -- host-side parts of the C ABI: version, the Test.h metric reduction
// with the reference's float accumulation order, glibc rand() seeds and the
// sampler's per-thread LCG bookkeeping.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <emmintrin.h>

#include <vector>

#include "../../include/mmre.h"

extern "C" int mmre_version(void) { return 100; }

// test_link_prediction (Test.h:232-327): per side, accumulate in query order into
// float globals exactly as testHead/testTail do (Test.h:102-112: `+= 1` on float,
// `+= (count+1)` long->float, `+= 1.0/(count+1)` in double then stored as float),
// then divide by testTotal (float) and average the two sides (float).
// The 8 (side, column) accumulations are independent serial chains: they advance together
// in one pass as the 8 lanes of SSE2 vectors. The hit@k sums are exact small integers in
// float (< 2^24), so they are counted as integers and converted once. Counts must be
// >= 0 and < 2^24 (true for ranks of |E| < 2^24 entities).
extern "C" int mmre_link_metrics(const int32_t* h_head_counts, const int32_t* h_tail_counts, int64_t n,
                                 int64_t stride, float* h_out) {
  if (!h_head_counts || !h_tail_counts || !h_out || n <= 0 || stride < n) return MMRE_ERR_ARG;
  if (n >= (int64_t)1 << 24) return MMRE_ERR_SHAPE;
  const float tot = (float)n;
  const int32_t* p[8];
  for (int j = 0; j < 8; ++j) p[j] = (j < 4 ? h_head_counts : h_tail_counts) + (int64_t)(j & 3) * stride;
  // Lanes j = 0..7 of two SSE float vectors (rank, reci) and four double pairs: every lane
  // performs exactly the scalar sequence of its own chain (IEEE add / convert per lane).
  __m128 rank_lo = _mm_setzero_ps(), rank_hi = _mm_setzero_ps();
  __m128 reci_lo = _mm_setzero_ps(), reci_hi = _mm_setzero_ps();
  __m128i c10_lo = _mm_setzero_si128(), c10_hi = _mm_setzero_si128();
  __m128i c3_lo = _mm_setzero_si128(), c3_hi = _mm_setzero_si128();
  __m128i c1_lo = _mm_setzero_si128(), c1_hi = _mm_setzero_si128();
  const __m128i ten = _mm_set1_epi32(10), three = _mm_set1_epi32(3), one_i = _mm_set1_epi32(1);
  const __m128d one = _mm_set1_pd(1.0);
  auto reci_step = [&](__m128 r, __m128i s1) {
    // r[k] = (float)((double)r[k] + 1.0 / (double)s1[k]) for the 4 lanes
    const __m128d lo = _mm_add_pd(_mm_cvtps_pd(r), _mm_div_pd(one, _mm_cvtepi32_pd(s1)));
    const __m128d hi = _mm_add_pd(_mm_cvtps_pd(_mm_movehl_ps(r, r)),
                                  _mm_div_pd(one, _mm_cvtepi32_pd(_mm_shuffle_epi32(s1, 0x4E))));
    return _mm_movelh_ps(_mm_cvtpd_ps(lo), _mm_cvtpd_ps(hi));
  };
  for (int64_t i = 0; i < n; ++i) {
    const __m128i s_lo = _mm_set_epi32(p[3][i], p[2][i], p[1][i], p[0][i]);
    const __m128i s_hi = _mm_set_epi32(p[7][i], p[6][i], p[5][i], p[4][i]);
    c10_lo = _mm_sub_epi32(c10_lo, _mm_cmplt_epi32(s_lo, ten));
    c10_hi = _mm_sub_epi32(c10_hi, _mm_cmplt_epi32(s_hi, ten));
    c3_lo = _mm_sub_epi32(c3_lo, _mm_cmplt_epi32(s_lo, three));
    c3_hi = _mm_sub_epi32(c3_hi, _mm_cmplt_epi32(s_hi, three));
    c1_lo = _mm_sub_epi32(c1_lo, _mm_cmplt_epi32(s_lo, one_i));
    c1_hi = _mm_sub_epi32(c1_hi, _mm_cmplt_epi32(s_hi, one_i));
    const __m128i s1_lo = _mm_add_epi32(s_lo, one_i), s1_hi = _mm_add_epi32(s_hi, one_i);
    rank_lo = _mm_add_ps(rank_lo, _mm_cvtepi32_ps(s1_lo));  // (float)(s + 1): exact below 2^24
    rank_hi = _mm_add_ps(rank_hi, _mm_cvtepi32_ps(s1_hi));
    reci_lo = reci_step(reci_lo, s1_lo);
    reci_hi = reci_step(reci_hi, s1_hi);
  }
  float rank[8], reci[8];
  int32_t c10[8], c3[8], c1[8];
  _mm_storeu_ps(rank, rank_lo); _mm_storeu_ps(rank + 4, rank_hi);
  _mm_storeu_ps(reci, reci_lo); _mm_storeu_ps(reci + 4, reci_hi);
  _mm_storeu_si128((__m128i*)c10, c10_lo); _mm_storeu_si128((__m128i*)(c10 + 4), c10_hi);
  _mm_storeu_si128((__m128i*)c3, c3_lo); _mm_storeu_si128((__m128i*)(c3 + 4), c3_hi);
  _mm_storeu_si128((__m128i*)c1, c1_lo); _mm_storeu_si128((__m128i*)(c1 + 4), c1_hi);
  const int cols[4] = {1, 0, 3, 2};  // filter, raw, filter_tc, raw_tc
  for (int g = 0; g < 4; ++g) {
    float v[2][5];
    for (int sd = 0; sd < 2; ++sd) {
      const int j = sd * 4 + cols[g];
      v[sd][0] = reci[j] / tot;
      v[sd][1] = rank[j] / tot;
      v[sd][2] = (float)c10[j] / tot;
      v[sd][3] = (float)c3[j] / tot;
      v[sd][4] = (float)c1[j] / tot;
    }
    for (int i = 0; i < 5; ++i) h_out[5 * g + i] = (v[0][i] + v[1][i]) / 2;
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

// importProb (Reader.h:26-49): kl_prob.txt holds n_rel x (n_rel - 1) floats (relation i's KL
// distance to every other relation, i's own column left out), read with fscanf("%f") like the
// reference (a short file leaves the remaining entries 0, as its calloc does); each row becomes
// exp(-kl / temperature) normalised by the row's sum, in float, summed in column order.
extern "C" int mmre_import_prob(const char* path, int64_t n_rel, float temperature, float* h_prob) {
  if (!path || !h_prob || n_rel < 2) return MMRE_ERR_ARG;
  FILE* fin = fopen(path, "r");
  if (!fin) return MMRE_ERR_ARG;
  const int64_t n = n_rel * (n_rel - 1);
  for (int64_t i = 0; i < n; ++i) h_prob[i] = 0.0f;
  for (int64_t i = 0; i < n; ++i)
    if (fscanf(fin, "%f", &h_prob[i]) != 1) break;
  fclose(fin);
  for (int64_t i = 0; i < n_rel; ++i) {
    float* row = h_prob + i * (n_rel - 1);
    float sum = 0.0f;
    for (int64_t j = 0; j < n_rel - 1; ++j) {
      // Reader.h:40 calls unqualified exp on a float with only <cmath> included and no `using
      // namespace std`: libstdc++ resolves it to ::exp(double), so the value is (float)exp((double)x)
      const float e = (float)exp((double)(-row[j] / temperature));
      sum += e;
      row[j] = e;
    }
    for (int64_t j = 0; j < n_rel - 1; ++j) row[j] /= sum;
  }
  return MMRE_OK;
}
