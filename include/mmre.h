/*
 * mmre.h -- C ABI of libmmre_hip.so, the MI355X-native hot path of
 * luisrui/Multimodal-Relation-Extrapolation (KG scoring sweep, negative-sampling
 * margin loss, zero-shot relation-embedding generator).
 *
 * Conventions
 *   - extern "C", plain pointers and sizes, no torch types.
 *   - Pointers named d_* are DEVICE pointers (hipMalloc / torch CUDA tensors);
 *     pointers named h_* are HOST pointers. Every device entry point takes an
 *     explicit hipStream_t (passed as void*; NULL = default stream) and only
 *     enqueues work: no allocation, no synchronisation, graph-capturable.
 *   - Return value: 0 on success, MMRE_ERR_* (> 0) on a bad argument, or
 *     MMRE_ERR_HIP_BASE + hipError_t for a HIP failure. Nothing aborts.
 *   - The library is stateless: all state lives in caller-owned buffers.
 *   - Model ids: MMRE_TRANSE_L1 / _L2 / DISTMULT / COMPLEX / ROTATE.
 *
 * Each entry point names the reference interface it replaces (file:line under
 * the reference tree). INTEGRATION.md shows the ctypes binding a maintainer of
 * the reference would add.
 */
#ifndef MMRE_H
#define MMRE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  MMRE_TRANSE_L1 = 0,
  MMRE_TRANSE_L2 = 1,
  MMRE_DISTMULT = 2,
  MMRE_COMPLEX = 3,
  MMRE_ROTATE = 4
};
enum { MMRE_HEAD_BATCH = 0, MMRE_TAIL_BATCH = 1 };
enum {
  MMRE_OK = 0,
  MMRE_ERR_ARG = 1,
  MMRE_ERR_MODEL = 2,
  MMRE_ERR_SHAPE = 3,
  MMRE_ERR_WORKSPACE = 4,
  MMRE_ERR_HIP_BASE = 1000
};

/* Library / ABI version (major*10000 + minor*100 + patch). */
int mmre_version(void);

/* ====================================================================== *
 *  Link prediction: the all-entity score sweep with fused rank epilogue.  *
 *  Replaces, per evaluation, the Tester loop (OpenKE/openke/config/       *
 *  Tester.py:70-91) = getHeadBatch/getTailBatch (Test.h:36-53) +          *
 *  model.predict (TransE.py:104-110, DistMult.py:70-72, ComplEx.py:60-62, *
 *  RotatE.py:89-91) + testHead/testTail (Test.h:65-192, _find            *
 *  Corrupt.h:166-177).                                                    *
 * ====================================================================== */

/* Width K of the k-major planes for a model (d, or 2d for ComplEx/RotatE),
 * rounded up to the sweep's K step. */
int64_t mmre_link_k(int model, int dim);
/* Padded entity / query counts used by the k-major planes. */
int64_t mmre_link_pad(int64_t n);

/* Entity table -> k-major planes d_ent_km[K][e_pad] for the sweep and the same
 * values row-major in d_ent_rows[n_ent][K] for per-entity gathers (F.normalize
 * first when norm_flag, TransE.py:63-66). Tables: TransE/DistMult (E, d);
 * ComplEx re/im (E, d) each; RotatE (E, 2d) = [re | im] (RotatE.py:48-49). */
int mmre_link_prepare_entities(int model, int norm_flag, const float* d_ent, const float* d_ent_im,
                               int64_t n_ent, int dim, float* d_ent_km, int64_t e_pad, float* d_ent_rows,
                               void* stream);

/* Query vectors for each (h, r, t, mode) -> d_q_km[K][q_pad] (element-wise from the
 * prepared d_ent_rows); d_q_true[i] = the entity the sweep must rank (h for
 * head_batch, t for tail_batch). d_rel_work: (n_rel, d) floats, required for
 * TransE with norm_flag (normalised relation rows). phase_denom: RotatE's
 * rel_range/pi as torch evaluates it (RotatE.py:51). d_q_rows (nullable): the
 * same vectors row-major [n_query][K], for mmre_link_truth_grouped. */
int mmre_link_prepare_queries(int model, int norm_flag, const float* d_ent_rows, const float* d_rel,
                              const float* d_rel_im, int64_t n_ent, int64_t n_rel, int dim, float phase_denom,
                              const int64_t* d_qh, const int64_t* d_qr, const int64_t* d_qt,
                              const int8_t* d_qmode, int64_t n_query, float* d_q_km, int64_t q_pad,
                              int32_t* d_q_true, float* d_rel_work, float* d_q_rows, void* stream);

/* Per-query threshold and filter bookkeeping, enqueued before the sweep:
 * writes d_truth[i] = pred(true(i)) with exactly the sweep's arithmetic and
 * initialises d_counts[.][i] = {0, -c, 0, -c_tc}, c = the known entities j of query i
 * (j != true) with pred(j) < pred(true) -- Test.h:85 `not _find(...)` -- so the
 * sweep's raw additions leave the filtered columns filtered.
 * filter CSR: d_filt_off[n_query+1] (int64), d_filt_ids (int32): the known heads
 *   (head_batch) / tails (tail_batch) of the query in train+valid+test
 *   (Reader.h:201-226); NULL/NULL = no filtering.
 * type masks: uint32 [n_rel][ceil(E/32)] bitsets of the relation's allowed heads
 *   / tails (type_constrain.txt, Reader.h:266-317); NULL/NULL disables.
 * d_counts: int32 [4][n_query] = raw, filt, raw_tc, filt_tc.
 * pred_kind: 0 s, 1 m-(m-s), 2 -s, 3 -(m-s), 4 m-s  (DESIGN.md §3). */
int mmre_link_truth(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                    int64_t e_pad, const float* d_ent_rows, const float* d_q_km, const int32_t* d_q_true, const int64_t* d_qr,
                    const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                    const int64_t* d_filt_off, const int32_t* d_filt_ids, const uint32_t* d_type_head,
                    const uint32_t* d_type_tail, int32_t* d_counts, float* d_truth, void* stream);

/* mmre_link_truth for filter GROUPS: queries with the same (mode, r, anchor) -- the
 * key of Test.h:85's _find: (r, t) for head_batch, (h, r) for tail_batch -- share one
 * known-entity list, so each listed entity is scored once per group. Two launches:
 * every truth and every listed entity scored as one flat set of lanes (listed entity
 * p with the query vector of query d_entry_q[p], any member of its group), then one
 * wave per group counts, for each member, the listed entities that beat its truth.
 * d_q_rows: row-major query vectors [n_query][K] (mmre_link_prepare_queries).
 * d_grp_qoff[n_groups+1] (int64) / d_grp_q (int32): a partition of 0..n_query-1
 *   (every query in exactly one group; groups of <= 64 queries run best).
 * d_filt_off[n_groups+1] (int64) / d_filt_ids[n_entries] (int32): each group's list.
 * d_list_scores: float workspace [n_entries]. Writes d_truth and all of d_counts
 * exactly as mmre_link_truth does. */
int mmre_link_truth_grouped(int model, int pred_kind, float margin, const float* d_ent_rows, int64_t n_ent,
                            const float* d_q_rows, const int32_t* d_q_true, const int64_t* d_qr,
                            const int8_t* d_qmode, int64_t n_query, int dim, const int64_t* d_grp_qoff,
                            const int32_t* d_grp_q, int64_t n_groups, const int64_t* d_filt_off,
                            const int32_t* d_filt_ids, const int32_t* d_entry_q, int64_t n_entries,
                            const uint32_t* d_type_head, const uint32_t* d_type_tail, float* d_list_scores,
                            int32_t* d_counts, float* d_truth, void* stream);

/* The sweep (after mmre_link_truth[_grouped] on the same stream). For every query i and
 * every entity j != true(i):  raw += pred(j) < pred(true)   (Test.h:80-86, strict
 * <, ties favour the truth), added to the raw AND filtered columns (and the _tc
 * columns for allowed j when type masks are given, Test.h:88-98). The kernel adds to the
 * raw columns and a short pass after it adds them to the filtered ones, so every sweep
 * call completes the count table the truth pass initialised (one sweep call per truth pass).
 * d_scores (nullable): (n_query, E) predicted values, for parity tests only. */
int mmre_link_sweep(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                    int64_t e_pad, const float* d_q_km, const int32_t* d_q_true, const int64_t* d_qr,
                    const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim,
                    const uint32_t* d_type_head, const uint32_t* d_type_tail, int32_t* d_counts,
                    const float* d_truth, float* d_scores, void* stream);

/* The same sweep over the entity slice [e_begin, e_end) only (e_begin a multiple of 128), for
 * entity-sharded evaluation (the alternative for huge E): each rank sweeps every
 * query against its slice after a truth pass whose filter lists hold only the slice's entities
 * (mmre_link_truth[_grouped] with restricted lists), so summing d_counts over the ranks
 * (one all-reduce of int32) gives exactly the whole-table counts. Replaces the per-query
 * testHead/testTail scan of Test.h:65-192 for the slice. No score rows. */
int mmre_link_sweep_range(int model, int pred_kind, float margin, const float* d_ent_km, int64_t n_ent,
                          int64_t e_pad, int64_t e_begin, int64_t e_end, const float* d_q_km,
                          const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode, int64_t n_query,
                          int64_t q_pad, int dim, const uint32_t* d_type_head, const uint32_t* d_type_tail,
                          int32_t* d_counts, const float* d_truth, void* stream);

/* TransE L1 (model MMRE_TRANSE_L1) count-only sweep through an integer filter: same counts as
 * mmre_link_sweep / mmre_link_sweep_range (bit for bit; replaces the same Test.h:65-192 scan),
 * faster. The k-major planes are quantized over the largest |x| of both to 8-bit codes (four k
 * per dword, summed with one v_sad_u8 per four elements) or, when a fixed sample of pairs
 * scored with those codes leaves more than 0.6 % undecided, to 16-bit codes (v_sad_u16, two
 * elements per instruction); the choice is made on the device (short launches on the stream,
 * no host round trip). Every pair the quantization error bound leaves on both sides of its
 * query's threshold is rescored with the canonical f32 chain from the row-major copies
 * d_ent_rows (whole table, mmre_link_prepare_entities) and d_q_rows
 * (mmre_link_prepare_queries). e_begin / e_end as for mmre_link_sweep_range (0, n_ent: whole
 * table). d_work: mmre_link_l1q_workspace(dim, e_pad, q_pad) bytes of device scratch.
 * Environment MMRE_L1_BITS=8 / 16 forces a code width (tests, experiments). */
int64_t mmre_link_l1q_workspace(int dim, int64_t e_pad, int64_t q_pad);
/* The filter's own record of the last mmre_link_sweep_l1q on d_work (one tiny launch, no
 * synchronisation): d_out[0] = pairs the code bound left undecided (each rescored with the
 * canonical f32 chain), d_out[1] = the code width the sweep used: 0 = 8-bit codes, 2 = 16-bit
 * codes, 1 = the f32 fallback instead of the codes. The fallback is taken on the device when M
 * (the largest |x|) exceeds 128 x the mean |x| of the two planes -- one outlier value stretching
 * the code range, which would leave most pairs undecided -- or is not finite. Counts are the
 * same either way. d_out[2] = undecided-list entries the rescoring refused because their query
 * or entity id was out of range (a guard on the list's invariant: 0 unless the build is
 * defective), d_out[3] = the largest per-entity error offset of the 8-bit codes' tight bound (in
 * code steps; 0 with the uniform bound). d_out holds 4 uint64. */
int mmre_link_l1q_stats(const void* d_work, int64_t work_bytes, uint64_t* d_out, void* stream);
int mmre_link_sweep_l1q(int pred_kind, float margin, const float* d_ent_km, const float* d_ent_rows, int64_t n_ent,
                        int64_t e_pad, int64_t e_begin, int64_t e_end, const float* d_q_km, const float* d_q_rows,
                        const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode, int64_t n_query,
                        int64_t q_pad, int dim, const uint32_t* d_type_head, const uint32_t* d_type_tail,
                        int32_t* d_counts, const float* d_truth, void* d_work, int64_t work_bytes, void* stream);

/* The whole count-only TransE L1 link-prediction evaluation of a query set in ONE call (prediction
 * = the score, filter groups, no type constraints) -- what mmre_link_prepare_entities +
 * mmre_link_prepare_queries + mmre_link_truth_grouped + mmre_link_sweep_l1q compute, with the same
 * outputs bit for bit (the entity / query planes and rows, q_true, truth scores, counts), in
 * seven launches instead of thirteen: query blocks normalise their own anchor and truth rows
 * from the raw table (no wait on the entity prep), the truth scores ride on the query prep,
 * list scores share a launch with the quantization, filter counts with the code-width probe.
 * Replaces Tester.run_link_prediction's loop (Tester.py:70-91: getHeadBatch/getTailBatch
 * Test.h:36-53, TransE.predict TransE.py:104-110, testHead/testTail Test.h:65-192) for TransE.
 * d_ent / d_rel: the raw tables (n_ent x dim, n_rel x dim); norm_flag as TransE's. Filter
 * groups as for mmre_link_truth_grouped (FilterIndex.groups; restricted to [e_begin, e_end)
 * for an entity slice). d_work: mmre_link_evaluate_l1q_workspace(dim, e_pad, q_pad) bytes,
 * ZEROED before the first call (it holds grid tickets; every call leaves them zero).
 * d_undecided_q (NULL or n_query uint32): per query, the pairs the filter left undecided and
 * rescored with the canonical chain (the relation-sharded partition's cost calibration). */
int64_t mmre_link_evaluate_l1q_workspace(int dim, int64_t e_pad, int64_t q_pad);
int mmre_link_evaluate_l1q(int norm_flag, const float* d_ent, int64_t n_ent, const float* d_rel, int64_t n_rel,
                           int dim, const int64_t* d_qh, const int64_t* d_qr, const int64_t* d_qt,
                           const int8_t* d_qmode, int64_t n_query, const int64_t* d_grp_qoff, const int32_t* d_grp_q,
                           int64_t n_groups, const int64_t* d_filt_off, const int32_t* d_filt_ids,
                           const int32_t* d_entry_q, int64_t n_entries, int64_t e_begin, int64_t e_end,
                           float* d_ent_km, int64_t e_pad, float* d_ent_rows, float* d_q_km, int64_t q_pad,
                           float* d_q_rows, int32_t* d_q_true, float* d_list_scores, int32_t* d_counts,
                           float* d_truth, uint32_t* d_undecided_q, void* d_work, int64_t work_bytes,
                           void* stream);

/* DistMult / ComplEx (MMRE_DISTMULT, MMRE_COMPLEX) count-only sweep through a split-bf16 MFMA
 * filter: same counts as mmre_link_sweep / mmre_link_sweep_range without type constraints (bit
 * for bit; replaces the same Test.h:65-192 scan), faster. Each f32 plane value x is split into
 * hi = bf16(x) and lo = bf16(x - hi); the sweep computes Qhi.Ehi + Qhi.Elo + Qlo.Ehi on the bf16
 * MFMA (16 k per instruction against the f32 MFMA's 2) and decides a pair only when its
 * prediction is on one side of the query's threshold over the whole error bound
 * cb |q|_2 |e|_2; the rest (the truth, near ties, non-finite values) are listed and rescored
 * with the canonical f32 chain from the row-major copies d_ent_rows (whole table) and d_q_rows.
 * If the list overflows, the device resets the raw counts and runs the exact f32 sweep instead
 * (no host round trip). e_begin / e_end as for mmre_link_sweep_range (0, n_ent: whole table).
 * Where the split planes exceed 64 MB (and pred_kind = -score) the sweep runs its wide form
 * (256 x 256 units, per-query thresholds per 32-entity block, a looser bound than the per-pair
 * one, the same counts); env MMRE_BF3_WIDE=1 / 0 forces either, MMRE_BF3_QT=128 its query tile.
 * d_work: mmre_link_bf3_workspace(model, dim, e_pad, q_pad) bytes of device scratch (0 for a
 * model without the filter). */
int64_t mmre_link_bf3_workspace(int model, int dim, int64_t e_pad, int64_t q_pad);
/* The filter's record of the last mmre_link_sweep_bf3 on d_work (one tiny launch, no
 * synchronisation): d_out[0] = pairs listed for exact rescoring, d_out[1] = 1 if the list
 * overflowed and the exact f32 sweep counted instead. */
int mmre_link_bf3_stats(const void* d_work, int64_t work_bytes, uint64_t* d_out, void* stream);
int mmre_link_sweep_bf3(int model, int pred_kind, float margin, const float* d_ent_km, const float* d_ent_rows,
                        int64_t n_ent, int64_t e_pad, int64_t e_begin, int64_t e_end, const float* d_q_km,
                        const float* d_q_rows, const int32_t* d_q_true, const int64_t* d_qr, const int8_t* d_qmode,
                        int64_t n_query, int64_t q_pad, int dim, int32_t* d_counts, const float* d_truth,
                        void* d_work, int64_t work_bytes, void* stream);
/* mmre_link_sweep_bf3 for a table whose row-major layout IS the plane layout -- DistMult with d a
 * multiple of 16, whose evaluation needs no normalisation (DistMult.py:34-44, 70-72): d_ent_rows
 * is then the raw (n_ent, d) embedding table (16-B aligned), and no prepared copy of it is made
 * per evaluation (mmre_link_prepare_entities writes two, k-major and row-major). The split planes,
 * norms and block maxima come from one read of the rows; d_ent_km (k_pad x e_pad floats, any
 * contents) is written only when the list overflows, by the fallback itself, before the exact
 * f32 sweep reads it. Same counts as mmre_link_sweep_bf3, bit for bit. MMRE_ERR_SHAPE for any
 * other model / d. */
int mmre_link_sweep_bf3_rows(int model, int pred_kind, float margin, const float* d_ent_rows, int64_t n_ent,
                             int64_t e_pad, int64_t e_begin, int64_t e_end, float* d_ent_km, const float* d_q_km,
                             const float* d_q_rows, const int32_t* d_q_true, const int64_t* d_qr,
                             const int8_t* d_qmode, int64_t n_query, int64_t q_pad, int dim, int32_t* d_counts,
                             const float* d_truth, void* d_work, int64_t work_bytes, void* stream);

/* Test.h:232-327 test_link_prediction + getTestLink* (Test.h:356-390), host side,
 * with the reference's float accumulation order (P14). Counts: int32, column c of
 * query i at counts[c*stride + i] (c = raw, filt, raw_tc, filt_tc).
 * h_out[20] = {mrr, mr, hit10, hit3, hit1} x {filter, raw, filter_tc, raw_tc}. */
int mmre_link_metrics(const int32_t* h_head_counts, const int32_t* h_tail_counts, int64_t n, int64_t stride,
                      float* h_out);

/* ====================================================================== *
 *  OpenKE negative sampler (Base.cpp:78-197 sampling/getBatch,           *
 *  Corrupt.h:7-163 corrupt_head/tail/rel, Random.h:11-29).               *
 *  Bit-exact: each positive's LCG state is reached by affine jump-ahead  *
 *  from its thread's seed, so the whole batch samples in parallel.       *
 * ====================================================================== */
/* glibc rand() stream after srand(1) (randReset's seeds, Random.h:11-15). */
int mmre_glibc_rand(int64_t skip, int64_t n, int64_t* h_out);
/* LCG draws one positive consumes in getBatch (Base.cpp:103-146). */
int64_t mmre_sampler_draws_per_positive(int64_t neg_rate, int64_t neg_rel_rate, int64_t mode);
/* Advance host-side per-thread LCG states by one sampling() call. */
int mmre_sampler_advance(uint64_t* h_seeds, int64_t work_threads, int64_t batch_size, int64_t neg_rate,
                         int64_t neg_rel_rate, int64_t mode);
/* The same advance applied to device-resident states on a stream, so a training loop keeps
 * the seeds in HBM (no host copy per batch; the sequence can be captured in a hipGraph). */
int mmre_sampler_advance_device(uint64_t* d_seeds, int64_t work_threads, int64_t batch_size, int64_t neg_rate,
                                int64_t neg_rel_rate, int64_t mode, void* stream);
/* One sampling() call on the GPU. Index arrays are the Reader.h:53-160 train
 * index (int64 rows (h, r, t); head_hrt sorted (h,r,t), tail_hrt (t,r,h),
 * rel_hrt (h,t,r); lef/rig per entity). d_left_mean/d_right_mean NULL = bern off.
 * d_seeds: per-thread states BEFORE this call (device copy). Outputs int64/f32,
 * length batch_size * (1 + neg_rate + neg_rel_rate), negative k at [k*B, (k+1)*B). */
int mmre_sampler_openke(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                        const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                        const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                        const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                        const float* d_right_mean, int64_t n_ent, int64_t n_rel, const uint64_t* d_seeds,
                        int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate,
                        int64_t mode, int64_t* d_batch_h, int64_t* d_batch_t, int64_t* d_batch_r,
                        float* d_batch_y, void* stream);

/* The (h, r) block of head_hrt and the (t, r) block of tail_hrt of every train row i, with
 * their first / last tail / head: int32 d_blocks[n_train][8] = (ll, rr, tail[ll], tail[rr],
 * ll', rr', head[ll'], head[rr']). What corrupt_head / corrupt_tail (Corrupt.h:7-81) look up
 * before their draw, built once per train index (n_train = rows of d_train_list). */
int mmre_sampler_blocks(const int64_t* d_train_list, int64_t n_train, const int64_t* d_head_hrt,
                        const int64_t* d_tail_hrt, const int64_t* d_lef_head, const int64_t* d_rig_head,
                        const int64_t* d_lef_tail, const int64_t* d_rig_tail, int32_t* d_blocks, void* stream);
/* mmre_sampler_openke reading the kept (entity, relation)'s block from d_blocks for train
 * rows i < n_blocks (bit-identical batches: the same blocks, found without the two binary
 * searches per negative); d_blocks NULL / n_blocks 0 is mmre_sampler_openke itself. */
int mmre_sampler_openke_blocked(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                                const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                                const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                                const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                                const float* d_right_mean, int64_t n_ent, int64_t n_rel, const uint64_t* d_seeds,
                                int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate,
                                int64_t mode, const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h,
                                int64_t* d_batch_t, int64_t* d_batch_r, float* d_batch_y, void* stream);
/* mmre_sampler_openke_blocked that also leaves d_seeds advanced for the next call (what
 * mmre_sampler_advance_device does, without a launch of its own): the last workgroup to finish
 * -- an integer ticket in d_ticket, zero before the first call and reset by each call --
 * writes the advanced states once every workgroup has read the old ones. One launch per
 * batch, as Base.cpp's sampling is one call (Base.cpp:161-197). */
int mmre_sampler_openke_step(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                             const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                             const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                             const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                             const float* d_right_mean, int64_t n_ent, int64_t n_rel, uint64_t* d_seeds,
                             int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate,
                             int64_t mode, const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h,
                             int64_t* d_batch_t, int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket,
                             void* stream);

/* importProb (Reader.h:26-49): kl_prob.txt at `path` (n_rel x (n_rel - 1) floats, fscanf
 * "%f") -> h_prob[n_rel][n_rel - 1] = exp(-kl / temperature) / row sum, in float. Host only. */
int mmre_import_prob(const char* path, int64_t n_rel, float temperature, float* h_prob);
/* mmre_sampler_openke_step with sampling(..., p = true): relation negatives drawn by
 * corrupt_rel's KL-weighted path (Corrupt.h:111-147) from d_rel_prob = mmre_import_prob's
 * table on the device; d_ticket may be NULL (seeds then left as they were, like
 * mmre_sampler_openke_blocked). Replaces Base.cpp:142's corrupt_rel(..., p). */
int mmre_sampler_openke_p(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                          const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                          const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                          const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                          const float* d_right_mean, int64_t n_ent, int64_t n_rel, uint64_t* d_seeds,
                          int64_t work_threads, int64_t batch_size, int64_t neg_rate, int64_t neg_rel_rate,
                          int64_t mode, const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h,
                          int64_t* d_batch_t, int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket,
                          const float* d_rel_prob, void* stream);

/* The repo's per-edge filtered sampler (module/NegativeSampling.py:114-140,
 * 321-375): per positive edge b (local ids d_eh/d_et, relation d_er), neg
 * negatives split head/tail by Bernoulli(0.5); candidates uniform over the local
 * node list [0, n_local) (NegativeSampling.py:210), rejected when their global id
 * (d_local_to_global, NULL = identity) is a known head of (t, r) (key t*n_rel+r in
 * the d_hf_* CSR over sorted keys) or a known tail of (h, r) (d_tf_*), distinct
 * within the positive. Counter-based (SplitMix64) draws from `seed` replace the
 * reference's unseeded Python `random` (P13). Output [pos | neg_1 | ... | neg_k]. */
int mmre_sampler_repo(const int64_t* d_eh, const int64_t* d_et, const int64_t* d_er, int64_t batch, int64_t neg,
                      int64_t n_local, const int64_t* d_local_to_global, int64_t n_rel, const int64_t* d_hf_keys,
                      const int64_t* d_hf_off, const int64_t* d_hf_vals, int64_t hf_n, const int64_t* d_tf_keys,
                      const int64_t* d_tf_off, const int64_t* d_tf_vals, int64_t tf_n, uint64_t seed,
                      int filter_flag, int64_t* d_out_h, int64_t* d_out_t, int64_t* d_out_r, void* stream);

/* Plain SGD step p <- p - lr * g (one fma per element) over `count` <= 8 float32 tensors in
 * one launch; params[t] / grads[t] 16-B aligned, numel[t] elements each. Replaces the
 * reference optimizer's step (optim.SGD without momentum / weight decay, OpenKE
 * Trainer.py:82-86) after the fused gradient. */
int mmre_sgd_step(float* const* params, const float* const* grads, const int64_t* numel, int count, float lr,
                  void* stream);

/* ====================================================================== *
 *  Negative-sampling margin loss, fused (OpenKE strategy/NegativeSampling *
 *  .py:23-32 + loss/MarginLoss.py:24-28 + model forward/regularization;   *
 *  repo module/NegativeSampling.py:204-229,307-314 + module/loss.py:19-23)*
 *  Rows: N = B*(1+k), positive b at row b, its negative j at row b+(j+1)B.*
 *  Entity rows come from d_ent[idx], relation rows from d_rel[ridx].       *
 * ====================================================================== */
/* Forward. d_score[N]: model(data) (TransE.py:78-90 etc.); d_loss[0]: margin
 * loss (+ regul_rate * regularization when regul_rate != 0). adv_temperature
 * <= 0 disables the self-adversarial weights. d_work: >= mmre_ns_workspace(B, k) floats. */
int64_t mmre_ns_workspace(int64_t batch, int64_t neg);
int mmre_ns_forward(int model, int norm_flag, float model_margin, int use_model_margin, const float* d_ent,
                    const float* d_ent_im, const float* d_rel, const float* d_rel_im, int dim, float phase_denom,
                    const int64_t* d_h, const int64_t* d_t, const int64_t* d_r, int64_t batch, int64_t neg,
                    float loss_margin, float adv_temperature, float regul_rate, float* d_score, float* d_loss,
                    float* d_work, void* stream);
/* Backward of the forward above: WRITES every row of the dense gradient tables with
 * d(loss)/d(table) * d_grad_loss[0] (d_grad_loss NULL means 1). Deterministic, no float
 * atomics: each scored row files its h / r / t gradient rows as slot records in its table
 * rows' buckets and one wave per table row sums them in batch order (bit-identical run to
 * run). d_work: >= mmre_rows_backward_workspace(model, batch * (1 + neg), n_ent, n_rel, dim)
 * floats. dim <= 512. */
int64_t mmre_rows_backward_workspace(int model, int64_t n_rows, int64_t n_ent, int64_t n_rel, int dim);
int mmre_ns_backward(int model, int norm_flag, float model_margin, int use_model_margin, const float* d_ent,
                     const float* d_ent_im, const float* d_rel, const float* d_rel_im, int dim,
                     float phase_denom, const int64_t* d_h, const int64_t* d_t, const int64_t* d_r, int64_t batch,
                     int64_t neg, float loss_margin, float adv_temperature, float regul_rate,
                     const float* d_score, const float* d_grad_loss, float* d_grad_ent, float* d_grad_ent_im,
                     float* d_grad_rel, float* d_grad_rel_im, int64_t n_ent, int64_t n_rel, float* d_work,
                     int64_t work_floats, void* stream);

/* Training: forward, loss and d(loss)/d(tables). mmre_ns_fused_forward computes the scores and
 * the loss and keeps what the gradient needs in d_work; mmre_ns_fused_grad then WRITES every
 * row of the dense gradient tables (no caller fill): d(loss)/d(table) * d_grad_loss[0] (NULL:
 * 1). mmre_ns_forward_backward is the two in sequence with an upstream gradient of 1. No float
 * atomics for any model -- every gradient contribution goes to a SLOT whose id is dropped into
 * its table row's bucket (integer atomics), and one wave per table row sums its bucket in
 * increasing slot id (batch order): bit-reproducible gradients.
 *   TransE (L1 / L2, dim <= 512, neg <= 32): a norm pre-pass, the fused kernel (each row read
 *   once, scores, loss partials and the contributions of a positive's group of rows), one
 *   workgroup for batches that are not OpenKE-shaped and the fixed-order loss reduction; the
 *   gradient is the row-owner pass.
 *   DistMult / ComplEx / RotatE (dim <= 512): the scoring pass + the loss reduction; the
 *   gradient is a slot pass (one wave per positive) + the row-owner pass.
 * Replaces strategy NegativeSampling.forward + loss.backward() (NegativeSampling.py:23-32,
 * Trainer.py:43-54) for one batch. d_work: >= mmre_ns_fused_workspace(model, norm_flag, B, k,
 * n_ent, n_rel, dim) floats, kept between the two calls. */
int64_t mmre_ns_fused_workspace(int model, int norm_flag, int64_t batch, int64_t neg, int64_t n_ent, int64_t n_rel,
                                int dim);
int mmre_ns_fused_forward(int model, int norm_flag, float model_margin, int use_model_margin, const float* d_ent,
                          const float* d_ent_im, const float* d_rel, const float* d_rel_im, int64_t n_ent,
                          int64_t n_rel, int dim, float phase_denom, const int64_t* d_h, const int64_t* d_t,
                          const int64_t* d_r, int64_t batch, int64_t neg, float loss_margin, float adv_temperature,
                          float regul_rate, float* d_score, float* d_loss, float* d_work, void* stream);
int mmre_ns_fused_grad(int model, int norm_flag, float model_margin, int use_model_margin, const float* d_ent,
                       const float* d_ent_im, const float* d_rel, const float* d_rel_im, int64_t n_ent, int64_t n_rel,
                       int dim, float phase_denom, const int64_t* d_h, const int64_t* d_t, const int64_t* d_r,
                       int64_t batch, int64_t neg, float loss_margin, float adv_temperature, float regul_rate,
                       const float* d_score, const float* d_grad_loss, float* d_grad_ent, float* d_grad_ent_im,
                       float* d_grad_rel, float* d_grad_rel_im, float* d_work, void* stream);
/* mmre_ns_fused_grad with the optimizer's plain SGD step fused in (OpenKE Trainer.py:82-86,
 * optim.SGD without momentum / weight decay; mmre.optim.SGD's fused mode): the gradient tables
 * are written as above AND every parameter row with a nonzero gradient becomes
 * fma(-lr, g, p) -- torch's SGD arithmetic, bit for bit -- in the same pass (rows outside the
 * batch keep p = p - lr 0). The tables are updated in place (d_ent ... are the parameters). */
int mmre_ns_fused_grad_sgd(int model, int norm_flag, float model_margin, int use_model_margin, float* d_ent,
                           float* d_ent_im, float* d_rel, float* d_rel_im, int64_t n_ent, int64_t n_rel, int dim,
                           float phase_denom, const int64_t* d_h, const int64_t* d_t, const int64_t* d_r,
                           int64_t batch, int64_t neg, float loss_margin, float adv_temperature, float regul_rate,
                           const float* d_score, const float* d_grad_loss, float* d_grad_ent, float* d_grad_ent_im,
                           float* d_grad_rel, float* d_grad_rel_im, float* d_work, float lr, void* stream);
int mmre_ns_forward_backward(int model, int norm_flag, float model_margin, int use_model_margin, const float* d_ent,
                             const float* d_ent_im, const float* d_rel, const float* d_rel_im, int64_t n_ent,
                             int64_t n_rel, int dim, float phase_denom, const int64_t* d_h, const int64_t* d_t,
                             const int64_t* d_r, int64_t batch, int64_t neg, float loss_margin, float adv_temperature,
                             float regul_rate, float* d_score, float* d_loss, float* d_grad_ent, float* d_grad_ent_im,
                             float* d_grad_rel, float* d_grad_rel_im, float* d_work, void* stream);

/* One OpenKE training step for TransE (Trainer.train_one_step, Trainer.py:43-54: Base.cpp:161-197's
 * sampling + strategy/NegativeSampling + MarginLoss forward/backward + optim.SGD): the sampler
 * arguments of mmre_sampler_openke_step (neg_rel_rate 0; d_ticket required; the batch lands in
 * d_batch_*), then the loss arguments of mmre_ns_fused_forward / mmre_ns_fused_grad_sgd (upstream
 * gradient 1; d_ent / d_rel updated in place by fma(-lr, g, p)). Values bit-identical to those
 * three calls in sequence; three launches instead of five (the sampler and the pre-pass share one
 * grid, the loss reduction rides in the gradient's). d_work: mmre_ns_fused_workspace. Only the
 * fused TransE shapes (dim <= 512, neg <= 32): MMRE_ERR_SHAPE otherwise. */
int mmre_ns_step_openke(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                        const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                        const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                        const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                        const float* d_right_mean, uint64_t* d_seeds, int64_t work_threads, int64_t mode,
                        const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h, int64_t* d_batch_t,
                        int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket, int model, int norm_flag,
                        float* d_ent, float* d_rel, int64_t n_ent, int64_t n_rel, int dim, int64_t batch, int64_t neg,
                        float loss_margin, float adv_temperature, float regul_rate, float* d_score, float* d_loss,
                        float* d_grad_ent, float* d_grad_rel, float* d_work, float lr, void* stream);

/* The same step, pipelined across calls (a prefetching data loader; Trainer.py:43-54 over the
 * loader's batches): the row owner of this step also samples the NEXT batch into d_next_* (the
 * sampler's seeds advance by that batch) and writes the norms / normalised copies of the rows it
 * updates -- the pre-pass the next step needs (a row without gradient keeps its parameters, so
 * its entries stay current) -- and zeroes the other parity's slot counts. prepared: bit 0 =
 * d_batch_* already holds this step's batch (the previous call's d_next_*), bit 1 = the pre-pass
 * and the slot counts of `parity` are current (the previous call was this one's other parity,
 * d_ent / d_rel / d_work unchanged since). prepared = 3 skips the first launch; otherwise it
 * samples d_batch_* (bit 0 clear) and runs the pre-pass, as mmre_ns_step_openke (whose d_work
 * layout this shares). d_next_h == NULL: no next batch (the next call: prepared bit 0 clear).
 * Batches, losses, gradients, parameters and seeds are bit-identical to consecutive
 * mmre_ns_step_openke calls. */
int mmre_ns_step_openke_pipe(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
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
                             int64_t* d_next_r, float* d_next_y);

/* The one-call training step for DistMult / ComplEx / RotatE (OpenKE Trainer.train_one_step over
 * the loader's sampling, NegativeSampling + MarginLoss, plain SGD; the models' own scoring as in
 * mmre_ns_fused_forward: d_ent_im / d_rel_im for ComplEx, model_margin / phase_denom for RotatE):
 * [sampler, unless prepared bit 0 says d_batch_* was drawn by the previous call] -> the forward
 * (scores + loss partials) -> the slot records -> the row owner (gradient + SGD), whose grid also
 * reduces the loss into d_loss and, with d_next_h, draws the next batch into d_next_*. Values
 * bit-identical to mmre_sampler_openke_step + mmre_ns_fused_forward + mmre_ns_fused_grad_sgd;
 * three launches a step instead of five. d_work: mmre_ns_fused_workspace. dim <= 512. */
int mmre_ns_step_openke_gen_pipe(const int64_t* d_train_list, int64_t train_total, const int64_t* d_head_hrt,
                                 const int64_t* d_tail_hrt, const int64_t* d_rel_hrt, const int64_t* d_lef_head,
                                 const int64_t* d_rig_head, const int64_t* d_lef_tail, const int64_t* d_rig_tail,
                                 const int64_t* d_lef_rel, const int64_t* d_rig_rel, const float* d_left_mean,
                                 const float* d_right_mean, uint64_t* d_seeds, int64_t work_threads, int64_t mode,
                                 const int32_t* d_blocks, int64_t n_blocks, int64_t* d_batch_h, int64_t* d_batch_t,
                                 int64_t* d_batch_r, float* d_batch_y, int32_t* d_ticket, int model,
                                 float model_margin, int use_model_margin, float* d_ent, float* d_ent_im,
                                 float* d_rel, float* d_rel_im, int64_t n_ent, int64_t n_rel, int dim,
                                 float phase_denom, int64_t batch, int64_t neg, float loss_margin,
                                 float adv_temperature, float regul_rate, float* d_score, float* d_loss,
                                 float* d_grad_ent, float* d_grad_ent_im, float* d_grad_rel, float* d_grad_rel_im,
                                 float* d_work, float lr, void* stream, int64_t prepared, int64_t* d_next_h,
                                 int64_t* d_next_t, int64_t* d_next_r, float* d_next_y);

/* model(data) in 'normal' mode for n_rows arbitrary rows is mmre_ns_forward with
 * batch = n_rows, neg = 0, d_loss = NULL. Its backward (OpenKE Model.forward under any loss,
 * Model.py / SoftplusLoss.py:7-31 / SigmoidLoss.py:7-30; the repo's scoring_fn / _calc,
 * module/NegativeSampling.py:69-82): WRITES every row of the dense gradient tables (n_ent /
 * n_rel rows) with sum_i d_grad_score[i] * d(score_i)/d(tables), summed per table row in row
 * order i (no float atomics: bit-identical run to run). d_work: >=
 * mmre_rows_backward_workspace(model, n_rows, n_ent, n_rel, dim) floats. dim <= 512. */
int mmre_score_rows_backward(int model, int norm_flag, float model_margin, int use_model_margin,
                             const float* d_ent, const float* d_ent_im, const float* d_rel, const float* d_rel_im,
                             int dim, float phase_denom, const int64_t* d_h, const int64_t* d_t, const int64_t* d_r,
                             int64_t n_rows, const float* d_grad_score, float* d_grad_ent, float* d_grad_ent_im,
                             float* d_grad_rel, float* d_grad_rel_im, int64_t n_ent, int64_t n_rel, float* d_work,
                             int64_t work_floats, void* stream);

/* ====================================================================== *
 *  Zero-shot relation-embedding generator (module/model.py:674-686):     *
 *  cat(noise, cls) -> SN-Linear -> SN-Linear -> SN-Linear ->            *
 *  LayerNormalization (module/submodule.py:58-77). Spectral norm         *
 *  (module/spectral_norm.py:39-89): sigma = u . (W v); in training mode  *
 *  one power iteration first updates u, v in place.                      *
 * ====================================================================== */
int64_t mmre_generator_workspace(int64_t n_rows, int in0, int out0, int out1, int out2);
int mmre_generator_forward(const float* d_noise, int noise_dim, const float* d_cls, int cls_dim,
                           int64_t n_rows, const float* d_w0, const float* d_b0, float* d_u0, float* d_v0,
                           int out0, const float* d_w1, const float* d_b1, float* d_u1, float* d_v1, int out1,
                           const float* d_w2, const float* d_b2, float* d_u2, float* d_v2, int out2,
                           const float* d_ln_a, const float* d_ln_b, float ln_eps, int power_iteration,
                           float sn_eps, float* d_out, float* d_work, void* stream);
/* Floats of the activation buffer of mmre_generator_forward_save. */
int64_t mmre_generator_acts_size(int64_t n_rows, int in0, int out0, int out1, int out2);
/* Training forward: mmre_generator_forward that also keeps the layer outputs for the
 * backward in d_acts = [x0 (N, in0) | h1 (N, out0) | h2 (N, out1) | h3 (N, out2) |
 * W0/s0 (out0, in0) | W1/s1 (out1, out0) | W2/s2 (out2, out1)] (row-major, in0 =
 * noise_dim + cls_dim); sigma[3] is left at d_work + 3 * 2048. */
int mmre_generator_forward_save(const float* d_noise, int noise_dim, const float* d_cls, int cls_dim,
                                int64_t n_rows, const float* d_w0, const float* d_b0, float* d_u0, float* d_v0,
                                int out0, const float* d_w1, const float* d_b1, float* d_u1, float* d_v1, int out1,
                                const float* d_w2, const float* d_b2, float* d_u2, float* d_v2, int out2,
                                const float* d_ln_a, const float* d_ln_b, float ln_eps, int power_iteration,
                                float sn_eps, float* d_out, float* d_work, float* d_acts, void* stream);
/* Floats of the backward's workspace. */
int64_t mmre_generator_backward_workspace(int64_t n_rows, int in0, int out0, int out1, int out2);
/* Parameter gradients of the generator for loss_G.backward() (zsl_module.py:595; the
 * grad_list of :356-357: weight_orig, bias of the three SN layers, layer_norm a_2 / b_2),
 * written (not accumulated) from d_gout = dL/dout (N, out2). Spectral norm chain rule with
 * the forward's u, v, sigma (u, v constant, spectral_norm.py:85-89):
 *   dL/dW_orig = G / s - <G, W_orig> / s^2 * u v^T,  G = dL/d(W_orig / s). */
int mmre_generator_backward(const float* d_gout, int64_t n_rows, int in0, int out0, int out1, int out2,
                            const float* d_acts, const float* d_sigma, const float* d_w0, const float* d_u0,
                            const float* d_v0, const float* d_w1, const float* d_u1, const float* d_v1,
                            const float* d_w2, const float* d_u2, const float* d_v2, const float* d_ln_a,
                            float ln_eps, float* d_gw0, float* d_gb0, float* d_gw1, float* d_gb1, float* d_gw2,
                            float* d_gb2, float* d_gln_a, float* d_gln_b, float* d_work, void* stream);

/* ====================================================================== *
 *  Candidate-list rankings.                                               *
 * ====================================================================== */
/* main.evaluate (main.py:232-250): TransE L1, no normalisation
 * (module/NegativeSampling.py:294-302): score = |(h + r) - t|_1 for each
 * candidate of query i (CSR, true tail first); rank = #(s<p) + #(s==p)//2 + 1. */
int mmre_candidate_rank_transe(const float* d_ent, const float* d_rel, int dim, const int64_t* d_qh,
                               const int64_t* d_qr, int64_t n_query, const int64_t* d_cand_off,
                               const int64_t* d_cand_ids, float* d_scores, int32_t* d_rank, void* stream);
/* ZSLmodule.eval (zsl_module.py:699-706): score = mean_s cos(cand, rel_vec[s]);
 * rank = 1 + #(score > score[true]) with the true candidate first (tie-free). */
int mmre_cosine_rank(const float* d_cand, int dim, const int64_t* d_cand_off, int64_t n_query,
                     const float* d_rel_vecs, int n_samples, const int64_t* d_rel_of_query, float* d_scores,
                     int32_t* d_rank, void* stream);

/* ====================================================================== *
 *  ZSL Extractor (module/zsl_module.py:17-110) in eval mode, fused with   *
 *  ZSLmodule.eval's cosine ranking (zsl_module.py:666-706). Replaces, per *
 *  query, get_meta (:265-287) + Extractor(query, query, meta, meta)       *
 *  (:690-694) + sklearn cosine_similarity(...).mean(1) (:699-701) +       *
 *  argsort rank (:705-706). d = embed_dim in {64, 100, 128, 200, 256}.    *
 * ====================================================================== */

/* Floats of the packed-weight buffer for embed_dim `dim` (-1 if unsupported). */
int64_t mmre_extractor_pack_size(int dim);
/* Pack the Extractor's weights (nn.Linear layout (out, in) row-major, as in its
 * state_dict: gcn_w (d/2, d) + bias, fc1 / fc2 (d/2, d) + bias, reshape_layer
 * (d, 2d) + bias, support_encoder.proj1 (2d, d) + bias, proj2 (d, 2d) + bias,
 * support_encoder.layer_norm weight / bias (d)) into MFMA lane order. */
int mmre_extractor_pack(int dim, const float* d_gcn_w, const float* d_gcn_b, const float* d_fc1_w,
                        const float* d_fc1_b, const float* d_fc2_w, const float* d_fc2_b, const float* d_rs_w,
                        const float* d_rs_b, const float* d_p1_w, const float* d_p1_b, const float* d_p2_w,
                        const float* d_p2_b, const float* d_ln_w, const float* d_ln_b, float* d_pack, void* stream);
/* Per-node halves of reshape_layer's output (neighbor_encoder :47-59 and
 * entity_encoder :61-67 folded through the linear reshape_layer :92-96):
 *   d_left[n]  (as e1: left neighbours, fc1 part, + bias)   (n_nodes, d), or NULL
 *   d_right[n] (as e2: fc2 part, right neighbours)          (n_nodes, d), or NULL
 * for node n = symbol d_node_sym[n] with neighbour list d_conn[n][max_nb][2]
 * (column 1 = neighbour symbol id, PAD = the zero last row of d_sym_emb; the
 * layout of ZSLmodule.connections, :233-263) and degree d_deg[n] (float). */
int mmre_extractor_nodes(int dim, const float* d_pack, const float* d_sym_emb, const int64_t* d_node_sym,
                         const int64_t* d_conn, int max_nb, const float* d_deg, int64_t n_nodes, float* d_left,
                         float* d_right, void* stream);
/* Row r = (e1 = d_li[r], e2 = d_ri[r]): x = left[e1] + right[e2]; g = SupportEncoder(x)
 * (submodule.py:254-258, nn.LayerNorm eps ln_eps). Writes d_out_g (n_rows, d) if
 * non-NULL (the Extractor's query_g) and d_score[r] = g . t / (normalize ? |g| : 1)
 * with t = d_targets[d_row_target[r]] (row 0 if d_row_target is NULL). */
int mmre_extractor_encode(int dim, const float* d_pack, float ln_eps, const float* d_left, const int64_t* d_li,
                          const float* d_right, const int64_t* d_ri, int64_t n_rows, const float* d_targets,
                          const int64_t* d_row_target, int normalize, float* d_out_g, float* d_score, void* stream);
/* d_targets[t] = mean_s v[t][s] / (normalize ? |v[t][s]| : 1) for d_vecs (n_sets, n_samples, dim),
 * n_samples <= 64: the sklearn-normalised mean relation vector of ZSL scoring, or
 * the support mean of Extractor.forward (:101). */
int mmre_extractor_targets(const float* d_vecs, int64_t n_sets, int n_samples, int dim, int normalize,
                           float* d_targets, void* stream);
/* Rank of the first entry of each list (CSR d_off) in descending order:
 * 1 + #(score > score[first]) (zsl_module.py:705-706, tie-free inputs). */
int mmre_rank_desc(const float* d_scores, const int64_t* d_off, int64_t n_query, int32_t* d_rank, void* stream);

/* ====================================================================== *
 *  ZSL Extractor in TRAINING mode (dropout active): pretrain_Extractor    *
 *  (module/zsl_module.py:289-348) and the GAN loop's Extractor calls      *
 *  while it is in training mode (:371-383, :430-440). The frozen          *
 *  symbol_emb side of the forward; the linears run on mmre_gemm_f32.      *
 * ====================================================================== */

/* Per row r of (d_pairs[r] = (e1, e2) symbol ids, neighbour lists d_conn_left/right[r]
 * (max_nb, 2), column 1 = neighbour symbol; the get_meta layout, :265-287):
 *   d_nsum_left[r]  = sum_s dropout(emb[conn_left[r][s][1]])     (neighbor_encoder :47-59
 *   d_nsum_right[r] = sum_s dropout(emb[conn_right[r][s][1]])     before gcn_w, whose linear
 *                                                                 part is applied to the sum)
 *   d_e1[r], d_e2[r] = dropout_e(emb[e1]), dropout_e(emb[e2])    (entity_encoder :61-67)
 * all (n_rows, dim). Dropout p (0 <= p < 1): kept values x * (1 / (1 - p)); the masks are a
 * counter hash of d_rng_state[0] (seed) and d_rng_state[1] (offset) on device, or -- when
 * d_mask_nb_left / d_mask_nb_right (n_rows, max_nb, dim) and d_mask_ent (n_rows, 2, dim) are
 * all given -- those 0/1 bytes. max_nb <= 64. */
int mmre_extractor_train_inputs(int dim, const float* d_sym_emb, const int64_t* d_pairs, const int64_t* d_conn_left,
                                const int64_t* d_conn_right, int max_nb, int64_t n_rows, float p,
                                const uint64_t* d_rng_state, const uint8_t* d_mask_nb_left,
                                const uint8_t* d_mask_nb_right, const uint8_t* d_mask_ent, float* d_nsum_left,
                                float* d_nsum_right, float* d_e1, float* d_e2, void* stream);
/* Elementwise dropout (nn.Dropout in training mode, e.g. SupportEncoder :257): d_y = keep ?
 * d_x * (1 / (1 - p)) : 0, the keep bytes to d_mask if non-NULL; draws from d_rng_state with
 * dropout stream `stream_id` (distinct streams of one step draw independent masks). */
int mmre_dropout(const float* d_x, float* d_y, uint8_t* d_mask, int64_t n, float p, const uint64_t* d_rng_state,
                 int stream_id, void* stream);

/* ====================================================================== *
 *  Frozen M3AE text encoder: the producer of the generator's CLS input.   *
 *  Replaces MaskedMultimodalAutoencoder.forward_representation(image=None,*
 *  text, text_padding_mask, deterministic=True) (module/model.py:323-356) *
 *  over Transformer/Block/Attention/TransformerMLP (module/submodule.py:  *
 *  128-238), as called by UnifiedModel.generate (model.py:674-679) and    *
 *  forward_relation_emb (model.py:599-604). Only the CLS row is returned. *
 *  Padded tokens (mask > 0) and, in the last block, non-CLS rows are not  *
 *  computed: they cannot reach the CLS output (masked logit -1e7 has      *
 *  softmax weight exactly 0); a row equal to the previous row on its      *
 *  unpadded tokens is encoded once. d in {384, 768, 1024, 1280}, head dim *
 *  64 or 80, len <= mmre_m3ae_max_len().                                  *
 * ====================================================================== */

/* Longest description row (tokens) the encoder accepts. */
int mmre_m3ae_max_len(void);
/* Int32 elements of the plan buffer for n_seq rows (6 n_seq + 5). */
int64_t mmre_m3ae_plan_size(int64_t n_seq);
/* Plan of an encode: per input row of d_tokens (n_seq, len) int32 / d_mask (n_seq, len) float32
 * (> 0 = padding, module/data.py:252-270): uniq[b] (the unique sequence it maps to; a row equal
 * to row b-1 on its padding pattern and unpadded tokens shares b-1's when dedupe != 0), the
 * unique sequences' source rows and packed row offsets (1 + unpadded tokens each, CLS row
 * first), and at d_plan[3 n_seq + 1 ..] info = {n_unique, n_rows, max_rows, unpadded token ids
 * outside [0, vocab)}. The host reads info (4 ints) to size the encode. */
int mmre_m3ae_plan(const int32_t* d_tokens, const float* d_mask, int64_t n_seq, int64_t len, int dedupe,
                   int64_t vocab, int32_t* d_plan, void* stream);
/* Floats of the workspace mmre_m3ae_encode needs for info's n_rows / n_unique. */
int64_t mmre_m3ae_workspace(int64_t n_rows, int64_t n_unique, int d);
/* CLS vectors d_cls (n_seq, d) of the description rows planned by mmre_m3ae_plan. h_params: HOST array
 * of 4 + 12 * depth + 2 DEVICE pointers, fp32 row-major as in the reference state dict:
 *   text_embedding.weight (vocab, d), the sin-cos position table (>= len, d)
 *   (get_1d_sincos_pos_embed, model.py:113-133), encoder_text_type_embedding (d), cls_token (d);
 *   per block i: layer_norm1.{weight,bias}, attention.qkv_linear.{weight (3d, d), bias},
 *   attention.fc.{weight, bias}, layer_norm2.{weight,bias}, transformer_mlp.fc1.{weight (4d, d),
 *   bias}, transformer_mlp.fc2.{weight (d, 4d), bias};
 *   encoder.layer_norm.{weight, bias}.
 * n_unique / n_rows / max_rows: the plan's info. */
int mmre_m3ae_encode(const float* const* h_params, int depth, int d, int heads, float ln_eps,
                     const int32_t* d_tokens, const float* d_mask, int64_t n_seq, int64_t len, int64_t vocab,
                     const int32_t* d_plan, int64_t n_unique, int64_t n_rows, int max_rows, float* d_work,
                     int64_t work_floats, float* d_cls, void* stream);
/* The encoder's building blocks (also exported for tests): nn.LayerNorm over rows;
 * out = a w^T + bias (epilogue 0), GELU(.) (1, F.gelu erf form), resid + (.) (2; resid may
 * alias out), n % 64 == 0, k % 32 == 0; packed multi-head attention over d_off sequences
 * (qkv rows [q | k | v]; cls_only: query row 0 of each sequence only, written to out row b). */
int mmre_m3ae_layernorm(const float* d_x, int64_t n_rows, int d, const float* d_w, const float* d_b, float eps,
                        float* d_y, void* stream);
int mmre_m3ae_linear(int epilogue, const float* d_a, int64_t m, int k, const float* d_w, int n, const float* d_bias,
                     const float* d_resid, float* d_out, void* stream);
int mmre_m3ae_attention(const float* d_qkv, const int32_t* d_off, int64_t n_seq, int max_rows, int heads,
                        int head_dim, float scale, int cls_only, float* d_out, void* stream);

/* ====================================================================== *
 *  Small fp32 GEMM of the GAN step's Discriminator (zsl_module.py:112-138: *
 *  its SN linears and class scores) and of their autograd, the gradient   *
 *  penalty's double backward included (module/utils.py:692-707).          *
 *  d_c (m, n) row-major = A B (+ d_bias[n] when given) with               *
 *  A(i, k) = d_a[i sam + k sak], B(k, j) = d_b[k sbk + j sbn] (transposes *
 *  are strides). One launch: 32 x 32 MFMA tiles, K split over             *
 *  mmre_gemm_splits(m, n, k) waves of a workgroup, summed in slice order. *
 * ====================================================================== */
int mmre_gemm_splits(int64_t m, int64_t n, int64_t k);
int mmre_gemm_f32(const float* d_a, int64_t sam, int64_t sak, const float* d_b, int64_t sbk, int64_t sbn, int64_t m,
                  int64_t n, int64_t k, const float* d_bias, float* d_c, void* stream);

/* Spectral normalisation of one weight (torch.nn.utils.spectral_norm's compute_weight, the
 * reference's SN layers: module/spectral_norm.py:39-89; Discriminator zsl_module.py:115-118).
 * power_iteration != 0 (training mode): one power iteration first updates d_u (out), d_v (in)
 * in place (v = normalize(W^T u), u = normalize(W v), eps). Then sigma = u . (W v),
 * d_w_hat = W / sigma, and d_u_snap / d_v_snap = the u, v used (for the backward).
 * d_work: 2048 floats. out, in <= 1024. */
int mmre_sn_weight(const float* d_w, int out, int in, float* d_u, float* d_v, int power_iteration, float eps,
                   float* d_sigma, float* d_u_snap, float* d_v_snap, float* d_w_hat, float* d_work, void* stream);
/* d_gw = G / s - <G, W> / s^2 u v^T for G = d_g = dL/dW_hat (u, v, s from mmre_sn_weight). */
int mmre_sn_weight_backward(const float* d_g, const float* d_w, int out, int in, const float* d_u, const float* d_v,
                            const float* d_sigma, float* d_gw, void* stream);
/* LayerNormalization (module/submodule.py:58-77): (z - mean) / (std_unbiased + eps) * a + b
 * per row of d_z (n_rows, d); d == 1 is the identity. */
int mmre_layernorm_unbiased(const float* d_z, int64_t n_rows, int d, const float* d_a, const float* d_b, float eps,
                            float* d_out, void* stream);
/* Its backward for dL/dout = d_g: d_gz (n_rows, d), d_ga, d_gb (d). d_work: n_rows * d floats. */
int mmre_layernorm_unbiased_backward(const float* d_g, const float* d_z, int64_t n_rows, int d, const float* d_a,
                                     float eps, float* d_gz, float* d_ga, float* d_gb, float* d_work, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMRE_H */
