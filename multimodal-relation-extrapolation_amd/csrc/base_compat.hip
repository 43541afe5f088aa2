// base_compat.hip -- libmmre_base.so: the C ABI of OpenKE's Base.so (the library the
// reference's Tester binds with ctypes, OpenKE/openke/config/Tester.py:20-36, and its
// absent data loaders call for `sampling`), re-implemented on the MI355X path so those
// callers run unchanged against it:
//
//   Setting.h:17-143   setInPath/.../setBern, get*Total        host state, same defaults
//   Random.h:11-15     randReset                               seeds = the process's rand() stream
//   Reader.h:53-317    importTrainFiles/importTestFiles/importTypeFiles   host parse + index
//   Base.cpp:161-197   sampling                                GPU: mmre_sampler_openke (bit-exact
//                                                              batches), then D2H into the caller's arrays
//   Test.h:23-53       initTest, getHeadBatch, getTailBatch    host index fills
//   Test.h:65-192      testHead/testTail                       GPU: the caller's score vector is staged
//                                                              to HBM and ranked by k_rank_scores
//                                                              (raw / filtered / type-constrained counts);
//                                                              counts stay on the device
//   Test.h:232-390     test_link_prediction, getTestLink*      one D2H of all counts, then the P14
//                                                              float accumulation in call order
//
// The per-query rank of Test.h walks all E scores and binary-searches the known-triple
// list for every better entity (~0.55 ms per query on the host); here it is one small
// kernel per call whose launch overlaps the caller's next predict. State is global, as in
// the reference (the ctypes caller owns nothing but its arrays). Triple classification
// (getNegTest/getTestBatch) and relation prediction are not part of the link-prediction
// path and are not exported.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/mmre_base.h"
#include "mmre_common.h"

namespace {

typedef int64_t INT;   // Setting.h: INT = long
typedef float REAL;    // Setting.h: REAL = float

struct Trip {
  INT h, r, t;
};
constexpr INT kLowest = INT64_MIN;
bool by_hrt(const Trip& a, const Trip& b) {
  return a.h != b.h ? a.h < b.h : (a.r != b.r ? a.r < b.r : a.t < b.t);
}
bool by_trh(const Trip& a, const Trip& b) {
  return a.t != b.t ? a.t < b.t : (a.r != b.r ? a.r < b.r : a.h < b.h);
}
bool by_htr(const Trip& a, const Trip& b) {
  return a.h != b.h ? a.h < b.h : (a.t != b.t ? a.t < b.t : a.r < b.r);
}
bool by_rht(const Trip& a, const Trip& b) {
  return a.r != b.r ? a.r < b.r : (a.h != b.h ? a.h < b.h : a.t < b.t);
}

struct State {
  std::string in_path = "../data/FB15K/", out_path = "../data/FB15K/";
  std::string ent_file, rel_file, train_file, valid_file, test_file;
  INT work_threads = 1, bern = 0;
  INT ent_total = 0, rel_total = 0, triple_total = 0, train_total = 0, test_total = 0, valid_total = 0;
  std::vector<unsigned long long> seeds;
  // importTrainFiles
  std::vector<Trip> train_head, train_tail, train_rel;  // train_head doubles as trainList
  std::vector<INT> lef_head, rig_head, lef_tail, rig_tail, lef_rel, rig_rel;
  std::vector<REAL> left_mean, right_mean;
  // importTestFiles
  std::vector<Trip> test_list, valid_list, known;  // known = train + valid + test, by (h, r, t)
  std::vector<int64_t> hoff, toff;                 // per test query: CSR offsets of its known lists
  // importTypeFiles: per relation sorted allowed heads / tails
  std::vector<std::vector<INT>> head_type, tail_type;
  bool have_types = false;
  // link-prediction accumulation
  INT last_head = 0, last_tail = 0;
  struct Call {
    int side;  // 0 head, 1 tail
    bool tc;
  };
  std::vector<Call> calls;
  REAL hit10 = 0, hit3 = 0, hit1 = 0, mr = 0, mrr = 0;
  REAL hit10_tc = 0, hit3_tc = 0, hit1_tc = 0, mr_tc = 0, mrr_tc = 0;
};
State S;

// ----------------------------------------------------------------- device ----
struct Device {
  bool init = false;
  hipStream_t st = nullptr;
  // sampler
  bool train_ready = false;
  int64_t *d_train = nullptr, *d_head = nullptr, *d_tail = nullptr, *d_rel = nullptr;
  int64_t *d_lh = nullptr, *d_rh = nullptr, *d_lt = nullptr, *d_rt = nullptr, *d_lr = nullptr, *d_rr = nullptr;
  float *d_lm = nullptr, *d_rm = nullptr;
  float* d_prob = nullptr;  // importProb's table (sampling with p = true)
  uint64_t* d_seeds = nullptr;
  int64_t *d_bh = nullptr, *d_bt = nullptr, *d_br = nullptr;
  float* d_by = nullptr;
  int64_t batch_cap = 0;
  // ranking
  bool test_ready = false;
  int32_t *d_hids = nullptr, *d_tids = nullptr;  // per test query: known heads of (r, t) / tails of (h, r)
  uint32_t *d_th = nullptr, *d_tt = nullptr;  // type bitsets [rel][words]
  static constexpr int kRing = 4;
  float* h_stage[kRing] = {};
  float* d_con[kRing] = {};
  hipEvent_t ev[kRing] = {};
  int32_t* d_counts = nullptr;  // [slot][4]
  int64_t slot_cap = 0;
};
Device D;

// Error policy. Base.so's void API has no status return, and an unmodified OpenKE caller never
// asks for one, so by default a failure ENDS THE PROCESS (message on stderr, abort()): a
// silent no-op would leave its batch / score buffers stale and train or evaluate on garbage.
// A caller that checks (mmre.base.load(), or MMRE_BASE_LATCH_ERRORS=1 in the environment)
// opts into the latched mode with mmre_base_set_error_mode(1): a failure throws BaseError up
// to the exported function, which latches it (code + message, printed once to stderr) and
// returns; while an error is latched every other entry point returns at once, and the outputs
// it would have written are poisoned (sampling's ids -1 and labels NaN, getHeadBatch /
// getTailBatch ids -1, getTestLink* NaN). mmre_base_last_error reads the latch,
// mmre_base_clear_error resets it.
struct BaseError : std::runtime_error {
  int code;
  BaseError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
int g_err_code = 0;
std::string g_err_msg;
int g_latch = -1;  // -1: not chosen yet (environment), 0: abort (default), 1: latch

bool latch_mode() {
  if (g_latch < 0) {
    const char* e = getenv("MMRE_BASE_LATCH_ERRORS");
    g_latch = (e && e[0] == '1') ? 1 : 0;
  }
  return g_latch == 1;
}

[[noreturn]] void fail(int code, const std::string& msg) { throw BaseError(code, msg); }

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) fail(MMRE_ERR_HIP_BASE + (int)e, std::string(what) + " failed: " + hipGetErrorString(e));
}
#define HIP_OR_DIE(x) hip_check((x), #x)

void on_error(int code, const char* what) {
  fprintf(stderr, "libmmre_base: %s\n", what);
  if (!latch_mode()) {
    fprintf(stderr, "libmmre_base: aborting (Base.so-compatible default; set MMRE_BASE_LATCH_ERRORS=1 or call "
                    "mmre_base_set_error_mode(1) to latch errors instead)\n");
    fflush(stderr);
    abort();
  }
  g_err_code = code;
  g_err_msg = what;
}

// returns false (f not run) while an error is latched, or when f fails
template <class F>
bool guarded(F&& f) {
  if (g_err_code) return false;
  try {
    f();
    return true;
  } catch (const BaseError& e) {
    on_error(e.code, e.what());
  } catch (const std::exception& e) {
    on_error(MMRE_ERR_ARG, e.what());
  }
  return false;
}

template <class T>
void poison(T* p, int64_t n, T v) {
  if (p)
    for (int64_t i = 0; i < n; ++i) p[i] = v;
}

template <class T>
T* upload(const std::vector<T>& v) {
  T* d = nullptr;
  const size_t n = v.empty() ? 1 : v.size();
  HIP_OR_DIE(hipMalloc(&d, n * sizeof(T)));
  if (!v.empty()) HIP_OR_DIE(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, D.st));
  return d;
}

void device_init() {
  if (D.init) return;
  HIP_OR_DIE(hipStreamCreateWithFlags(&D.st, hipStreamNonBlocking));
  D.init = true;
}

std::vector<int64_t> flat(const std::vector<Trip>& v) {  // rows (h, r, t)
  std::vector<int64_t> o(v.size() * 3);
  for (size_t i = 0; i < v.size(); ++i) {
    o[3 * i] = v[i].h;
    o[3 * i + 1] = v[i].r;
    o[3 * i + 2] = v[i].t;
  }
  return o;
}

void release(void* p) {
  if (p) HIP_OR_DIE(hipFree(p));
}

void train_device() {
  device_init();
  if (D.train_ready) return;
  for (void* p : {(void*)D.d_train, (void*)D.d_tail, (void*)D.d_rel, (void*)D.d_lh, (void*)D.d_rh, (void*)D.d_lt,
                  (void*)D.d_rt, (void*)D.d_lr, (void*)D.d_rr, (void*)D.d_lm, (void*)D.d_rm, (void*)D.d_seeds})
    release(p);
  D.d_train = upload(flat(S.train_head));
  D.d_head = D.d_train;  // trainHead has trainList's order (cmp_head)
  D.d_tail = upload(flat(S.train_tail));
  D.d_rel = upload(flat(S.train_rel));
  D.d_lh = upload(S.lef_head);
  D.d_rh = upload(S.rig_head);
  D.d_lt = upload(S.lef_tail);
  D.d_rt = upload(S.rig_tail);
  D.d_lr = upload(S.lef_rel);
  D.d_rr = upload(S.rig_rel);
  D.d_lm = upload(S.left_mean);
  D.d_rm = upload(S.right_mean);
  HIP_OR_DIE(hipMalloc(&D.d_seeds, sizeof(uint64_t) * std::max<INT>(S.work_threads, 1)));
  HIP_OR_DIE(hipStreamSynchronize(D.st));
  D.train_ready = true;
}

// Known heads of (r, t) for head_batch and known tails of (h, r) for tail_batch, for every
// test query in testList order (Test.h:85 / :149 `_find` over train+valid+test).
void test_device() {
  device_init();
  if (D.test_ready) return;
  HIP_OR_DIE(hipStreamSynchronize(D.st));
  for (void* p : {(void*)D.d_hids, (void*)D.d_tids, (void*)D.d_th, (void*)D.d_tt, (void*)D.d_counts}) release(p);
  D.d_th = D.d_tt = nullptr;
  D.d_counts = nullptr;
  D.slot_cap = 0;
  for (int i = 0; i < Device::kRing; ++i) {
    if (D.h_stage[i]) HIP_OR_DIE(hipHostFree(D.h_stage[i]));
    release(D.d_con[i]);
    if (D.ev[i]) HIP_OR_DIE(hipEventDestroy(D.ev[i]));
    D.h_stage[i] = nullptr;
    D.d_con[i] = nullptr;
    D.ev[i] = nullptr;
  }
  std::vector<Trip> by_t(S.known);
  std::sort(by_t.begin(), by_t.end(), by_trh);
  std::vector<int64_t> hoff(1, 0), toff(1, 0);
  std::vector<int32_t> hids, tids;
  for (const Trip& q : S.test_list) {
    // heads j with (j, r, t) known: rows of by_t with t = q.t, r = q.r (sorted by h)
    auto a = std::lower_bound(by_t.begin(), by_t.end(), Trip{kLowest, q.r, q.t}, by_trh);
    for (auto it = a; it != by_t.end() && it->t == q.t && it->r == q.r; ++it)
      if (hids.empty() || hoff.back() == (int64_t)hids.size() || hids.back() != (int32_t)it->h)
        hids.push_back((int32_t)it->h);
    hoff.push_back((int64_t)hids.size());
    auto b = std::lower_bound(S.known.begin(), S.known.end(), Trip{q.h, q.r, kLowest}, by_hrt);
    for (auto it = b; it != S.known.end() && it->h == q.h && it->r == q.r; ++it)
      if (tids.empty() || toff.back() == (int64_t)tids.size() || tids.back() != (int32_t)it->t)
        tids.push_back((int32_t)it->t);
    toff.push_back((int64_t)tids.size());
  }
  S.hoff = hoff;
  S.toff = toff;
  D.d_hids = upload(hids);
  D.d_tids = upload(tids);
  if (S.have_types) {
    const INT words = (S.ent_total + 31) / 32;
    std::vector<uint32_t> th((size_t)(S.rel_total * words), 0u), tt((size_t)(S.rel_total * words), 0u);
    for (INT r = 0; r < S.rel_total; ++r) {
      for (INT e : S.head_type[r])
        if (e >= 0 && e < S.ent_total) th[r * words + (e >> 5)] |= 1u << (e & 31);
      for (INT e : S.tail_type[r])
        if (e >= 0 && e < S.ent_total) tt[r * words + (e >> 5)] |= 1u << (e & 31);
    }
    D.d_th = upload(th);
    D.d_tt = upload(tt);
  }
  for (int i = 0; i < Device::kRing; ++i) {
    HIP_OR_DIE(hipHostMalloc(&D.h_stage[i], sizeof(float) * std::max<INT>(S.ent_total, 1), hipHostMallocDefault));
    HIP_OR_DIE(hipMalloc(&D.d_con[i], sizeof(float) * std::max<INT>(S.ent_total, 1)));
    HIP_OR_DIE(hipEventCreateWithFlags(&D.ev[i], hipEventDisableTiming));
  }
  HIP_OR_DIE(hipStreamSynchronize(D.st));
  D.test_ready = true;
}

// ------------------------------------------------------------ rank kernel ----
// One query's counts from a score vector: raw = #{j != truth : con[j] < con[truth]},
// filtered = raw minus the known entities among them, and the same two restricted to the
// relation's allowed entities when a type bitset is given (Test.h:65-126). One workgroup.
__global__ __launch_bounds__(1024) void k_rank_scores(const float* __restrict__ con, int64_t n_ent, int64_t truth,
                                                      const int32_t* __restrict__ known, int64_t n_known,
                                                      const uint32_t* __restrict__ type_row,
                                                      int32_t* __restrict__ out) {
  __shared__ int32_t s[4];
  if (threadIdx.x < 4) s[threadIdx.x] = 0;
  __syncthreads();
  const float minimal = con[truth];
  int raw = 0, raw_tc = 0, kn = 0, kn_tc = 0;
  for (int64_t j = threadIdx.x; j < n_ent; j += blockDim.x) {
    const bool better = j != truth && con[j] < minimal;
    raw += better;
    if (type_row) raw_tc += better && ((type_row[j >> 5] >> (j & 31)) & 1u);
  }
  for (int64_t p = threadIdx.x; p < n_known; p += blockDim.x) {
    const int64_t j = known[p];
    if (j < 0 || j >= n_ent || j == truth || !(con[j] < minimal)) continue;
    kn += 1;
    if (type_row) kn_tc += (type_row[j >> 5] >> (j & 31)) & 1u;
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) {
    raw += __shfl_xor(raw, sh);
    raw_tc += __shfl_xor(raw_tc, sh);
    kn += __shfl_xor(kn, sh);
    kn_tc += __shfl_xor(kn_tc, sh);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&s[0], raw);
    atomicAdd(&s[1], raw - kn);
    atomicAdd(&s[2], raw_tc);
    atomicAdd(&s[3], raw_tc - kn_tc);
  }
  __syncthreads();
  if (threadIdx.x < 4) out[threadIdx.x] = s[threadIdx.x];
}

void rank_call(const REAL* con, INT idx, bool tc, int side) {
  if (idx < 0 || idx >= S.test_total)
    fail(MMRE_ERR_ARG, "test index " + std::to_string((long)idx) + " out of range [0, " +
                           std::to_string((long)S.test_total) + ")");
  if (tc && !S.have_types) fail(MMRE_ERR_ARG, "type_constrain requires importTypeFiles()");
  test_device();
  const int64_t slot = (int64_t)S.calls.size();
  if (slot >= D.slot_cap) {  // grow the count array (rare: sized for one evaluation)
    HIP_OR_DIE(hipStreamSynchronize(D.st));
    const int64_t cap = std::max<int64_t>(2 * S.test_total, 2 * D.slot_cap) + 16;
    int32_t* n = nullptr;
    HIP_OR_DIE(hipMalloc(&n, sizeof(int32_t) * 4 * cap));
    if (D.d_counts) {
      HIP_OR_DIE(hipMemcpy(n, D.d_counts, sizeof(int32_t) * 4 * D.slot_cap, hipMemcpyDeviceToDevice));
      HIP_OR_DIE(hipFree(D.d_counts));
    }
    D.d_counts = n;
    D.slot_cap = cap;
  }
  const int ring = (int)(slot % Device::kRing);
  HIP_OR_DIE(hipEventSynchronize(D.ev[ring]));  // staging slot free again
  memcpy(D.h_stage[ring], con, sizeof(float) * S.ent_total);
  HIP_OR_DIE(hipMemcpyAsync(D.d_con[ring], D.h_stage[ring], sizeof(float) * S.ent_total, hipMemcpyHostToDevice,
                            D.st));
  const Trip& q = S.test_list[idx];
  const int32_t* ids = side == 0 ? D.d_hids : D.d_tids;
  const std::vector<int64_t>& oh = side == 0 ? S.hoff : S.toff;
  const INT words = (S.ent_total + 31) / 32;
  const uint32_t* trow = nullptr;
  if (tc) trow = (side == 0 ? D.d_th : D.d_tt) + q.r * words;
  hipLaunchKernelGGL(k_rank_scores, dim3(1), dim3(1024), 0, D.st, D.d_con[ring], S.ent_total,
                     side == 0 ? q.h : q.t, ids + oh[idx], oh[idx + 1] - oh[idx], trow, D.d_counts + 4 * slot);
  HIP_OR_DIE(hipGetLastError());
  HIP_OR_DIE(hipEventRecord(D.ev[ring], D.st));
  S.calls.push_back({side, tc});
}

// --------------------------------------------------------------- readers ----
FILE* open_or_die(const std::string& p) {
  FILE* f = fopen(p.c_str(), "r");
  if (!f) fail(MMRE_ERR_ARG, "cannot open " + p);
  return f;
}

INT read_count(const std::string& p) {
  FILE* f = open_or_die(p);
  long v = 0;
  if (fscanf(f, "%ld", &v) != 1) v = 0;
  fclose(f);
  return v;
}

std::vector<Trip> read_triples(const std::string& p, INT* total) {
  FILE* f = open_or_die(p);
  long n = 0;
  if (fscanf(f, "%ld", &n) != 1) n = 0;
  std::vector<Trip> v((size_t)n);
  for (long i = 0; i < n; ++i) {  // "h t r" per line (Reader.h:86-90)
    long h = 0, t = 0, r = 0;
    if (fscanf(f, "%ld %ld %ld", &h, &t, &r) != 3) break;
    v[(size_t)i] = Trip{h, r, t};
  }
  fclose(f);
  *total = n;
  return v;
}

std::string path_or(const std::string& set, const char* name) { return set.empty() ? S.in_path + name : set; }

void block_bounds(const std::vector<Trip>& v, INT key_of(const Trip&), std::vector<INT>& lef, std::vector<INT>& rig) {
  lef.assign((size_t)S.ent_total, 0);
  rig.assign((size_t)S.ent_total, -1);
  for (size_t i = 0; i < v.size(); ++i) {
    const INT k = key_of(v[i]);
    if (k < 0 || k >= S.ent_total) continue;
    if (i == 0 || key_of(v[i - 1]) != k) lef[(size_t)k] = (INT)i;
    if (i + 1 == v.size() || key_of(v[i + 1]) != k) rig[(size_t)k] = (INT)i;
  }
}
INT key_head(const Trip& a) { return a.h; }
INT key_tail(const Trip& a) { return a.t; }

void set_str(std::string& dst, const char* p, const char* label) {
  dst = p ? p : "";
  printf("%s : %s\n", label, dst.c_str());
}

}  // namespace

// ------------------------------------------------------------- Setting.h ----
extern "C" void setInPath(char* path) { set_str(S.in_path, path, "Input Files Path"); }
extern "C" void setOutPath(char* path) { set_str(S.out_path, path, "Output Files Path"); }
extern "C" void setTrainPath(char* path) { set_str(S.train_file, path, "Training Files Path"); }
extern "C" void setValidPath(char* path) { set_str(S.valid_file, path, "Valid Files Path"); }
extern "C" void setTestPath(char* path) { set_str(S.test_file, path, "Test Files Path"); }
extern "C" void setEntPath(char* path) { set_str(S.ent_file, path, "Entity Files Path"); }
extern "C" void setRelPath(char* path) { set_str(S.rel_file, path, "Relation Files Path"); }
extern "C" void setWorkThreads(INT threads) { S.work_threads = threads > 0 ? threads : 1; }
extern "C" INT getWorkThreads() { return S.work_threads; }
extern "C" void setBern(INT con) { S.bern = con; }
extern "C" INT getEntityTotal() { return S.ent_total; }
extern "C" INT getRelationTotal() { return S.rel_total; }
extern "C" INT getTripleTotal() { return S.triple_total; }
extern "C" INT getTrainTotal() { return S.train_total; }
extern "C" INT getTestTotal() { return S.test_total; }
extern "C" INT getValidTotal() { return S.valid_total; }

// -------------------------------------------------------------- Random.h ----
// One rand() per work thread from the process's C library stream (Random.h:11-15), so a
// caller that seeds with srand (or not) gets the reference's seeds.
extern "C" void randReset() {
  S.seeds.assign((size_t)S.work_threads, 0ull);
  for (INT i = 0; i < S.work_threads; ++i) S.seeds[(size_t)i] = (unsigned long long)rand();
}

// -------------------------------------------------------------- Reader.h ----
static void importTrainFiles_impl() {
  printf("The toolkit is importing datasets.\n");
  S.rel_total = read_count(path_or(S.rel_file, "relation2id.txt"));
  S.ent_total = read_count(path_or(S.ent_file, "entity2id.txt"));
  printf("The total of relations is %ld.\n", (long)S.rel_total);
  printf("The total of entities is %ld.\n", (long)S.ent_total);
  INT n = 0;
  std::vector<Trip> tr = read_triples(path_or(S.train_file, "train2id.txt"), &n);
  std::sort(tr.begin(), tr.end(), by_hrt);
  tr.erase(std::unique(tr.begin(), tr.end(),
                       [](const Trip& a, const Trip& b) { return a.h == b.h && a.r == b.r && a.t == b.t; }),
           tr.end());
  S.train_total = (INT)tr.size();
  printf("The total of train triples is %ld.\n", (long)S.train_total);
  S.train_head = tr;
  S.train_tail = tr;
  std::sort(S.train_tail.begin(), S.train_tail.end(), by_trh);
  S.train_rel = tr;
  std::sort(S.train_rel.begin(), S.train_rel.end(), by_htr);
  block_bounds(S.train_head, key_head, S.lef_head, S.rig_head);
  block_bounds(S.train_tail, key_tail, S.lef_tail, S.rig_tail);
  block_bounds(S.train_rel, key_head, S.lef_rel, S.rig_rel);
  // bern statistics (Reader.h:140-159): tails per (h, r) and heads per (t, r), per relation
  std::vector<REAL> freq((size_t)S.rel_total, 0.0f), lcnt((size_t)S.rel_total, 0.0f),
      rcnt((size_t)S.rel_total, 0.0f);
  for (size_t i = 0; i < tr.size(); ++i) {
    if (tr[i].r >= 0 && tr[i].r < S.rel_total) freq[(size_t)tr[i].r] += 1.0f;
    if (i == 0 || tr[i].h != tr[i - 1].h || tr[i].r != tr[i - 1].r)
      if (tr[i].r >= 0 && tr[i].r < S.rel_total) lcnt[(size_t)tr[i].r] += 1.0f;
  }
  const std::vector<Trip>& tt = S.train_tail;
  for (size_t i = 0; i < tt.size(); ++i)
    if (i == 0 || tt[i].t != tt[i - 1].t || tt[i].r != tt[i - 1].r)
      if (tt[i].r >= 0 && tt[i].r < S.rel_total) rcnt[(size_t)tt[i].r] += 1.0f;
  S.left_mean.resize((size_t)S.rel_total);
  S.right_mean.resize((size_t)S.rel_total);
  for (INT r = 0; r < S.rel_total; ++r) {
    S.left_mean[(size_t)r] = freq[(size_t)r] / lcnt[(size_t)r];
    S.right_mean[(size_t)r] = freq[(size_t)r] / rcnt[(size_t)r];
  }
  D.train_ready = false;  // re-upload on the next sampling call
}

static void importTestFiles_impl() {
  S.rel_total = read_count(path_or(S.rel_file, "relation2id.txt"));
  S.ent_total = read_count(path_or(S.ent_file, "entity2id.txt"));
  INT n_test = 0, n_train = 0, n_valid = 0;
  S.test_list = read_triples(path_or(S.test_file, "test2id.txt"), &n_test);
  std::vector<Trip> train = read_triples(path_or(S.train_file, "train2id.txt"), &n_train);
  S.valid_list = read_triples(path_or(S.valid_file, "valid2id.txt"), &n_valid);
  S.test_total = n_test;
  S.train_total = n_train;  // as Reader.h:198: the file's count (duplicates included)
  S.valid_total = n_valid;
  S.triple_total = n_test + n_train + n_valid;
  S.known.clear();
  S.known.insert(S.known.end(), S.test_list.begin(), S.test_list.end());
  S.known.insert(S.known.end(), train.begin(), train.end());
  S.known.insert(S.known.end(), S.valid_list.begin(), S.valid_list.end());
  std::sort(S.known.begin(), S.known.end(), by_hrt);
  std::sort(S.test_list.begin(), S.test_list.end(), by_rht);   // testList order (Reader.h:227)
  std::sort(S.valid_list.begin(), S.valid_list.end(), by_rht);
  printf("The total of test triples is %ld.\n", (long)S.test_total);
  printf("The total of valid triples is %ld.\n", (long)S.valid_total);
  D.test_ready = false;
}

static void importTypeFiles_impl() {
  FILE* f = open_or_die(S.in_path + "type_constrain.txt");
  long n = 0;
  if (fscanf(f, "%ld", &n) != 1) n = 0;
  S.head_type.assign((size_t)S.rel_total, {});
  S.tail_type.assign((size_t)S.rel_total, {});
  for (INT i = 0; i < S.rel_total; ++i) {
    for (int side = 0; side < 2; ++side) {
      long rel = 0, tot = 0;
      if (fscanf(f, "%ld %ld", &rel, &tot) != 2) break;
      std::vector<INT> ids((size_t)tot);
      for (long j = 0; j < tot; ++j) {
        long e = 0;
        if (fscanf(f, "%ld", &e) != 1) e = -1;
        ids[(size_t)j] = e;
      }
      std::sort(ids.begin(), ids.end());
      if (rel >= 0 && rel < S.rel_total) (side == 0 ? S.head_type : S.tail_type)[(size_t)rel] = ids;
    }
  }
  fclose(f);
  S.have_types = true;
  D.test_ready = false;
}

// -------------------------------------------------------------- Base.cpp ----
static void sampling_impl(INT* batch_h, INT* batch_t, INT* batch_r, REAL* batch_y, INT batch_size, INT neg_rate,
                         INT neg_rel_rate, INT mode, bool filter_flag, bool p, bool val_loss) {
  (void)filter_flag;  // accepted and ignored, as in Base.cpp:116/:119
  if (batch_size <= 0) return;
  if (val_loss) {  // the first batch_size validation triples as positives (Base.cpp:148-156)
    for (INT b = 0; b < batch_size && b < (INT)S.valid_list.size(); ++b) {
      batch_h[b] = S.valid_list[(size_t)b].h;
      batch_t[b] = S.valid_list[(size_t)b].t;
      batch_r[b] = S.valid_list[(size_t)b].r;
      batch_y[b] = 1.0f;
    }
    return;
  }
  const bool use_p = p && neg_rel_rate > 0;
  if (use_p && !D.d_prob) fail(MMRE_ERR_ARG, "sampling(p=true) needs importProb() first (Reader.h:26)");
  if (S.seeds.size() != (size_t)S.work_threads) fail(MMRE_ERR_ARG, "call randReset() after setWorkThreads() before sampling");
  train_device();
  const int64_t n = batch_size * (1 + neg_rate + neg_rel_rate);
  if (n > D.batch_cap) {
    for (void* p : {(void*)D.d_bh, (void*)D.d_bt, (void*)D.d_br, (void*)D.d_by}) release(p);
    HIP_OR_DIE(hipMalloc(&D.d_bh, sizeof(int64_t) * n));
    HIP_OR_DIE(hipMalloc(&D.d_bt, sizeof(int64_t) * n));
    HIP_OR_DIE(hipMalloc(&D.d_br, sizeof(int64_t) * n));
    HIP_OR_DIE(hipMalloc(&D.d_by, sizeof(float) * n));
    D.batch_cap = n;
  }
  HIP_OR_DIE(hipMemcpyAsync(D.d_seeds, S.seeds.data(), sizeof(uint64_t) * S.work_threads, hipMemcpyHostToDevice,
                            D.st));
  const int rc = use_p
      ? mmre_sampler_openke_p(D.d_train, S.train_total, D.d_head, D.d_tail, D.d_rel, D.d_lh, D.d_rh, D.d_lt, D.d_rt,
                              D.d_lr, D.d_rr, S.bern ? D.d_lm : nullptr, S.bern ? D.d_rm : nullptr, S.ent_total,
                              S.rel_total, D.d_seeds, S.work_threads, batch_size, neg_rate, neg_rel_rate, mode,
                              nullptr, 0, D.d_bh, D.d_bt, D.d_br, D.d_by, nullptr, D.d_prob, D.st)
      : mmre_sampler_openke(D.d_train, S.train_total, D.d_head, D.d_tail, D.d_rel, D.d_lh, D.d_rh, D.d_lt, D.d_rt,
                            D.d_lr, D.d_rr, S.bern ? D.d_lm : nullptr, S.bern ? D.d_rm : nullptr, S.ent_total,
                            S.rel_total, D.d_seeds, S.work_threads, batch_size, neg_rate, neg_rel_rate, mode, D.d_bh,
                            D.d_bt, D.d_br, D.d_by, D.st);
  if (rc != MMRE_OK) fail(rc, "mmre_sampler_openke failed (" + std::to_string(rc) + ")");
  HIP_OR_DIE(hipMemcpyAsync(batch_h, D.d_bh, sizeof(int64_t) * n, hipMemcpyDeviceToHost, D.st));
  HIP_OR_DIE(hipMemcpyAsync(batch_t, D.d_bt, sizeof(int64_t) * n, hipMemcpyDeviceToHost, D.st));
  HIP_OR_DIE(hipMemcpyAsync(batch_r, D.d_br, sizeof(int64_t) * n, hipMemcpyDeviceToHost, D.st));
  HIP_OR_DIE(hipMemcpyAsync(batch_y, D.d_by, sizeof(float) * n, hipMemcpyDeviceToHost, D.st));
  HIP_OR_DIE(hipStreamSynchronize(D.st));
  mmre_sampler_advance(reinterpret_cast<uint64_t*>(S.seeds.data()), S.work_threads, batch_size, neg_rate,
                       neg_rel_rate, mode);
}

// ---------------------------------------------------------------- Test.h ----
static void initTest_impl() {
  S.last_head = S.last_tail = 0;
  if (D.test_ready) HIP_OR_DIE(hipStreamSynchronize(D.st));
  S.calls.clear();
}

static void getHeadBatch_impl(INT* ph, INT* pt, INT* pr) {
  const Trip& q = S.test_list[(size_t)S.last_head];
  for (INT i = 0; i < S.ent_total; ++i) {
    ph[i] = i;
    pt[i] = q.t;
    pr[i] = q.r;
  }
  S.last_head++;
}

static void getTailBatch_impl(INT* ph, INT* pt, INT* pr) {
  const Trip& q = S.test_list[(size_t)S.last_tail];
  for (INT i = 0; i < S.ent_total; ++i) {
    ph[i] = q.h;
    pt[i] = i;
    pr[i] = q.r;
  }
  S.last_tail++;
}

extern "C" void testHead(REAL* con, INT last_head, bool type_constrain) {
  guarded([&] { rank_call(con, last_head, type_constrain, 0); });
}
extern "C" void testTail(REAL* con, INT last_tail, bool type_constrain) {
  guarded([&] { rank_call(con, last_tail, type_constrain, 1); });
}

static void test_link_prediction_impl(bool type_constrain) {
  const size_t n = S.calls.size();
  std::vector<int32_t> c(4 * n + 4);
  if (n) {
    HIP_OR_DIE(hipStreamSynchronize(D.st));
    HIP_OR_DIE(hipMemcpy(c.data(), D.d_counts, sizeof(int32_t) * 4 * n, hipMemcpyDeviceToHost));
  }
  // Test.h:102-126 accumulation, in call order, per side; [side][variant] with variants
  // raw, filter, raw_tc, filter_tc; fields tot10, tot3, tot1, rank, reci
  REAL acc[2][4][5] = {};
  for (size_t i = 0; i < n; ++i) {
    const int side = S.calls[i].side;
    const int nv = S.calls[i].tc ? 4 : 2;
    for (int v = 0; v < nv; ++v) {
      const INT s = c[4 * i + v];
      REAL* a = acc[side][v];
      if (s < 10) a[0] += 1;
      if (s < 3) a[1] += 1;
      if (s < 1) a[2] += 1;
      a[3] += (REAL)(s + 1);
      a[4] = (REAL)((double)a[4] + 1.0 / (double)(s + 1));
    }
  }
  const REAL tot = (REAL)S.test_total;
  for (int side = 0; side < 2; ++side)
    for (int v = 0; v < 4; ++v)
      for (int f = 0; f < 5; ++f) acc[side][v][f] /= tot;
  auto avg = [&](int v, int f) { return (acc[0][v][f] + acc[1][v][f]) / 2; };
  const char* hdr = "metric:\t\t\t MRR \t\t MR \t\t hit@10 \t hit@3  \t hit@1 \n";
  for (int tc = 0; tc <= (type_constrain ? 1 : 0); ++tc) {
    printf(tc ? "type constraint results:\n" : "no type constraint results:\n");
    printf("%s", hdr);
    for (int filt = 0; filt < 2; ++filt) {
      const int v = 2 * tc + filt;
      const char* tag = filt ? "filter" : "raw";
      printf("l(%s):\t\t %f \t %f \t %f \t %f \t %f \n", tag, acc[0][v][4], acc[0][v][3], acc[0][v][0], acc[0][v][1],
             acc[0][v][2]);
      printf("r(%s):\t\t %f \t %f \t %f \t %f \t %f \n", tag, acc[1][v][4], acc[1][v][3], acc[1][v][0], acc[1][v][1],
             acc[1][v][2]);
      printf("averaged(%s):\t %f \t %f \t %f \t %f \t %f \n", tag, avg(v, 4), avg(v, 3), avg(v, 0), avg(v, 1),
             avg(v, 2));
      if (!filt) printf("\n");
    }
  }
  S.mrr = avg(1, 4);
  S.mr = avg(1, 3);
  S.hit10 = avg(1, 0);
  S.hit3 = avg(1, 1);
  S.hit1 = avg(1, 2);
  if (type_constrain) {
    S.mrr_tc = avg(3, 4);
    S.mr_tc = avg(3, 3);
    S.hit10_tc = avg(3, 0);
    S.hit3_tc = avg(3, 1);
    S.hit1_tc = avg(3, 2);
  }
}

extern "C" REAL getTestLinkHit10(bool type_constrain) {
  return g_err_code ? NAN : (type_constrain ? S.hit10_tc : S.hit10);
}
extern "C" REAL getTestLinkHit3(bool type_constrain) {
  return g_err_code ? NAN : (type_constrain ? S.hit3_tc : S.hit3);
}
extern "C" REAL getTestLinkHit1(bool type_constrain) {
  return g_err_code ? NAN : (type_constrain ? S.hit1_tc : S.hit1);
}
extern "C" REAL getTestLinkMR(bool type_constrain) {
  return g_err_code ? NAN : (type_constrain ? S.mr_tc : S.mr);
}
extern "C" REAL getTestLinkMRR(bool type_constrain) {
  return g_err_code ? NAN : (type_constrain ? S.mrr_tc : S.mrr);
}

// --------------------------------------------------- exported entry points ----
extern "C" void importTrainFiles() {
  guarded([&] { importTrainFiles_impl(); });
}

extern "C" void importTestFiles() {
  guarded([&] { importTestFiles_impl(); });
}

extern "C" void importTypeFiles() {
  guarded([&] { importTypeFiles_impl(); });
}

extern "C" void sampling(INT* batch_h, INT* batch_t, INT* batch_r, REAL* batch_y, INT batch_size, INT neg_rate, INT neg_rel_rate, INT mode, bool filter_flag, bool p, bool val_loss) {
  if (!guarded([&] { sampling_impl(batch_h, batch_t, batch_r, batch_y, batch_size, neg_rate, neg_rel_rate, mode, filter_flag, p, val_loss); })) {
    const int64_t n = batch_size > 0 ? batch_size * (1 + (neg_rate > 0 ? neg_rate : 0) + (neg_rel_rate > 0 ? neg_rel_rate : 0)) : 0;
    poison<INT>(batch_h, n, -1);
    poison<INT>(batch_t, n, -1);
    poison<INT>(batch_r, n, -1);
    poison<REAL>(batch_y, n, NAN);
  }
}

// Reader.h:26-49: kl_prob.txt from the input path, weighted by the temperature (the table
// sampling(p = true) draws relation negatives from); rereading replaces the table.
static void importProb_impl(REAL temp) {
  if (S.rel_total < 2) fail(MMRE_ERR_ARG, "importProb: call importTrainFiles() first (relationTotal < 2)");
  printf("Current temperature:%f\n", temp);
  std::vector<float> prob((size_t)(S.rel_total * (S.rel_total - 1)));
  const std::string path = S.in_path + "kl_prob.txt";
  const int rc = mmre_import_prob(path.c_str(), S.rel_total, temp, prob.data());
  if (rc != MMRE_OK) fail(rc, "importProb: cannot read " + path);
  device_init();
  release(D.d_prob);
  D.d_prob = upload(prob);
  HIP_OR_DIE(hipStreamSynchronize(D.st));
}

extern "C" void importProb(REAL temp) { guarded([&] { importProb_impl(temp); }); }

extern "C" void initTest() {
  guarded([&] { initTest_impl(); });
}

extern "C" void getHeadBatch(INT* ph, INT* pt, INT* pr) {
  if (!guarded([&] { getHeadBatch_impl(ph, pt, pr); })) {
    poison<INT>(ph, S.ent_total, -1);
    poison<INT>(pt, S.ent_total, -1);
    poison<INT>(pr, S.ent_total, -1);
  }
}

extern "C" void getTailBatch(INT* ph, INT* pt, INT* pr) {
  if (!guarded([&] { getTailBatch_impl(ph, pt, pr); })) {
    poison<INT>(ph, S.ent_total, -1);
    poison<INT>(pt, S.ent_total, -1);
    poison<INT>(pr, S.ent_total, -1);
  }
}

extern "C" void test_link_prediction(bool type_constrain) {
  guarded([&] { test_link_prediction_impl(type_constrain); });
}

// ------------------------------------------------------------ error latch ----
extern "C" int mmre_base_last_error(char* msg, int cap) {
  if (msg && cap > 0) {
    strncpy(msg, g_err_msg.c_str(), (size_t)cap - 1);
    msg[cap - 1] = 0;
  }
  return g_err_code;
}

extern "C" void mmre_base_clear_error() {
  g_err_code = 0;
  g_err_msg.clear();
}

extern "C" void mmre_base_set_error_mode(int latch) { g_latch = latch ? 1 : 0; }
