/* mmre_base.h -- libmmre_base.so: OpenKE's Base.so C ABI on the MI355X path.
 *
 * The reference binds Base.so with ctypes (OpenKE/openke/config/Tester.py:20-36; the
 * absent openke.data loaders call `sampling`). libmmre_base.so exports the same names,
 * argument types (INT = int64 `long`, REAL = float, Setting.h:3-4) and global-state
 * semantics, so a caller switches by loading this library instead of release/Base.so.
 * `sampling` runs the bit-exact GPU sampler (mmre_sampler_openke) and testHead/testTail
 * rank the caller's score vector on the GPU; everything else is host bookkeeping.
 * Errors the reference would crash on (missing files, out-of-range index) print a message
 * to stderr and abort. Not exported (outside the link-prediction path): triple
 * classification (getNegTest/getTestBatch), relation prediction (getRelBatch/testRel).
 */
#ifndef MMRE_BASE_H
#define MMRE_BASE_H
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Setting.h:17-78 -- file locations (inPath default "../data/FB15K/"; the set*Path
 * overrides replace inPath + "<name>2id.txt"). */
void setInPath(char* path);
void setOutPath(char* path);
void setTrainPath(char* path);
void setValidPath(char* path);
void setTestPath(char* path);
void setEntPath(char* path);
void setRelPath(char* path);
/* Setting.h:84-143 */
void setWorkThreads(int64_t threads);
int64_t getWorkThreads(void);
void setBern(int64_t con);
int64_t getEntityTotal(void);
int64_t getRelationTotal(void);
int64_t getTripleTotal(void);
int64_t getTrainTotal(void);
int64_t getTestTotal(void);
int64_t getValidTotal(void);

/* Random.h:11-15 -- one rand() of the process's C library stream per work thread. */
void randReset(void);

/* Reader.h:53-160 -- train2id.txt ("h t r" lines), deduplicated, with the trainHead /
 * trainTail / trainRel orders, lef/rig blocks and the bern statistics. */
void importTrainFiles(void);
/* Reader.h:167-264 -- test/train/valid lists; testList sorted by (r, h, t) (Reader.h:227);
 * the filter set is train + valid + test. */
void importTestFiles(void);
/* Reader.h:267-317 -- type_constrain.txt: allowed heads / tails per relation. */
void importTypeFiles(void);
/* Reader.h:26-49 -- inPath + "kl_prob.txt" (relationTotal x (relationTotal - 1) KL distances)
 * weighted as exp(-kl / temp), normalised per relation: the table sampling(p = true) draws
 * relation negatives from (Corrupt.h:111-147). Call after importTrainFiles. */
void importProb(float temp);

/* Base.cpp:161-197 -- a training batch into caller arrays of length
 * batch_size * (1 + neg_rate + neg_rel_rate); negative k at [k*B, (k+1)*B). Bit-identical
 * to Base.so for the same seeds; filter_flag is ignored as in the reference; p = true (with
 * neg_rel_rate > 0) draws relation negatives from importProb's table. */
void sampling(int64_t* batch_h, int64_t* batch_t, int64_t* batch_r, float* batch_y, int64_t batch_size,
              int64_t neg_rate, int64_t neg_rel_rate, int64_t mode, bool filter_flag, bool p, bool val_loss);

/* Test.h:23-53 */
void initTest(void);
void getHeadBatch(int64_t* ph, int64_t* pt, int64_t* pr);
void getTailBatch(int64_t* ph, int64_t* pt, int64_t* pr);
/* Test.h:65-192 -- con: host float32[E] scores of query `index` (lower = better). */
void testHead(float* con, int64_t index, bool type_constrain);
void testTail(float* con, int64_t index, bool type_constrain);
/* Test.h:232-327, 356-390 -- filtered metrics in the reference's float order (P14). */
void test_link_prediction(bool type_constrain);
float getTestLinkHit10(bool type_constrain);
float getTestLinkHit3(bool type_constrain);
float getTestLinkHit1(bool type_constrain);
float getTestLinkMR(bool type_constrain);
float getTestLinkMRR(bool type_constrain);

/* Not in Base.so, whose void API crashes on bad input (Reader.h:59-90 ignores fopen
 * failures; OpenKE/README.md:129). Here a failure -- a file that cannot be opened, a test
 * index out of range, type_constrain without importTypeFiles, a HIP error -- prints its
 * message and, by default, abort()s: an unmodified OpenKE caller never checks for errors.
 * mmre_base_set_error_mode(1) (or MMRE_BASE_LATCH_ERRORS=1 in the environment) latches it
 * instead: the failing call returns, every entry point above returns at once while the latch
 * is set, and their outputs are poisoned (sampling / getHeadBatch / getTailBatch ids -1,
 * batch_y NaN, getTestLink* NaN). mmre_base_last_error returns the code (0: none; mmre.h
 * MMRE_ERR_*, HIP errors as MMRE_ERR_HIP_BASE + hipError_t) and copies the message into
 * msg[cap]; mmre_base_clear_error resets the latch. */
void mmre_base_set_error_mode(int latch);
int mmre_base_last_error(char* msg, int cap);
void mmre_base_clear_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MMRE_BASE_H */
