// engine.hip — host side of libotsdb_agg.so: the C-ABI of include/otsdb_agg.h.
//
// Plans one query (bucket grid, series chunks), carves a reusable HBM
// workspace, launches the kernel pipeline of kernels.hip on the context's
// stream and maps the device error word back onto the reference's
// exceptions.  No CPU fallback exists: every data point is produced on the
// GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "../../include/otsdb_agg.h"
#include "kernels.hip"
#include "compact.hip"
#include "select.hip"
#include "decode.hip"
#include "raw.hip"
#include "rows.hip"
#include "calendar.hip"
#include "launch.h"

using namespace otsdb;

namespace {

thread_local std::string g_last_error;

otsdb_status fail(otsdb_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return st;
}

#define HIP_TRY(x)                                                        \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess)                                                 \
      return fail(OTSDB_E_DEVICE, "%s: %s", #x, hipGetErrorString(e_));   \
  } while (0)

struct AggInfo {
  const char* key;   // Aggregators.get() name
  const char* name;  // toString()
  int interp;
};

const AggInfo kAggs[OTSDB_AGG_COUNT_IDS] = {
    {"sum", "sum", 0},          {"pfsum", "pfsum", 4},
    {"min", "min", 0},          {"max", "max", 0},
    {"avg", "avg", 0},          {"median", "median", 0},
    {"none", "raw", 1},         {"mult", "multiply", 0},
    {"dev", "dev", 0},          {"diff", "diff", 0},
    {"zimsum", "zimsum", 1},    {"mimmin", "mimmin", 2},
    {"mimmax", "mimmax", 3},    {"squareSum", "squareSum", 1},
    {"count", "count", 1},      {"first", "first", 1},
    {"last", "last", 1},        {"p999", "p999", 0},
    {"p99", "p99", 0},          {"p95", "p95", 0},
    {"p90", "p90", 0},          {"p75", "p75", 0},
    {"p50", "p50", 0},          {"ep999r3", "ep999r3", 0},
    {"ep99r3", "ep99r3", 0},    {"ep95r3", "ep95r3", 0},
    {"ep90r3", "ep90r3", 0},    {"ep75r3", "ep75r3", 0},
    {"ep50r3", "ep50r3", 0},    {"ep999r7", "ep999r7", 0},
    {"ep99r7", "ep99r7", 0},    {"ep95r7", "ep95r7", 0},
    {"ep90r7", "ep90r7", 0},    {"ep75r7", "ep75r7", 0},
    {"ep50r7", "ep50r7", 0},
};

bool is_selection(int agg) {
  return agg == OTSDB_AGG_MEDIAN || agg >= OTSDB_AGG_P999;
}

double pct_of(int agg) {  // PercentileAgg(percentile).evaluate(): p / 100d
  static const double P[6] = {99.9, 99.0, 95.0, 90.0, 75.0, 50.0};
  return P[(agg - OTSDB_AGG_P999) % 6] / 100.0;
}

inline int64_t jmod(int64_t a, int64_t b) { return a % b; }
inline int64_t align_down(int64_t t, int64_t iv) { return t - jmod(t, iv); }

constexpr int64_t kChunk = 256;  // series per cross-series chunk

// k_keys_transpose's grid: KT_M members x OTSDB_KT_SLICES bucket slices
dim3 kt_grid(int64_t M, int64_t NB) {
  const int64_t ntb = (NB + 63) / 64;
  const int64_t sl = ntb < OTSDB_KT_SLICES ? (ntb > 0 ? ntb : 1) : OTSDB_KT_SLICES;
  return dim3((unsigned)((M + KT_M - 1) / KT_M), (unsigned)sl);
}

// members per tile of the ordered fold: one tile is one workgroup that
// streams all its members' points, so big groups (C3's 7.8k-series
// datacenters per GPU) are cut finer than kChunk — 256-member tiles of one
// day of points leave the last round of workgroups half empty (C3 fold:
// 256 -> 2.9 ms, 64 -> 2.57 ms, 32 -> 2.53 ms)
#ifndef OTSDB_FOLD_CHUNK  // tuning builds override
#define OTSDB_FOLD_CHUNK 32
#endif
constexpr int64_t kFoldChunk = OTSDB_FOLD_CHUNK;
// groups of more than kFoldChunk members (C3's 7.8k-series datacenters):
// tiles of kFoldChunkLarge, twice as many workgroups again for the grid's
// last round (C3 fold: 32 -> 2.59 ms, 16 -> 2.50, 8 -> 2.46); groups up to
// kFoldChunk members (C1 / C2 hosts) stay one tile
#ifndef OTSDB_FOLD_CHUNK_LARGE  // tuning builds override
#define OTSDB_FOLD_CHUNK_LARGE 8
#endif
constexpr int64_t kFoldChunkLarge = OTSDB_FOLD_CHUNK_LARGE;
#ifndef OTSDB_FOLD_CTX  // tuning builds: 0 = no preloaded member contexts
#define OTSDB_FOLD_CTX 1
#endif
// Order-sensitive aggregators whose merge of partial states is
// ill-conditioned (dev: Chan's merge of Welford runs over offset data lands
// ~1e-11 from the reference's one sequential pass, Aggregators.java:547-568)
// reduce a group's members in ONE sequential chain per (group, bucket) while
// the group fits: fold tiles of up to kOrderedFoldChunk members (the LDS
// progress marks of one workgroup), then the row path's k_group with one
// chain of up to kOrderedChunk members (one thread walks them in SpanCmp
// order; ~100 ns a member: tools/chain_probe.hip, 69 ns with no memory at
// all, so a 500k-member chain — C4 — would cost ~50 ms).  Larger groups
// merge 256-member chunk partials in order (Chan); across ranks the chain is
// handed on (otsdb_agg_partials_chained_device).
constexpr int64_t kOrderedFoldChunk = 256;
constexpr int64_t kOrderedChunk = 65536;
constexpr int64_t kOrderedChunkMerged = 16384;
// the row path's bucket rows an ordered (dev) query may take for groups past
// one fold tile: fixed, so the path (and the reduction order) never depends
// on the device's free memory at call time
constexpr double kOrderedRowBudget = 48.0e9;
// below this many (tile, window) workgroups the fold narrows its windows,
// down to kFoldMinWindow buckets
#ifndef OTSDB_FOLD_MIN_BLOCKS  // tuning builds override
#define OTSDB_FOLD_MIN_BLOCKS 1024
#endif
#ifndef OTSDB_FOLD_MIN_WINDOW
#define OTSDB_FOLD_MIN_WINDOW 128
#endif
constexpr int64_t kFoldMinBlocks = OTSDB_FOLD_MIN_BLOCKS;
// up to this many (series, window boundary) pairs k_prep and k_fold_prep run
// as one launch (each pair's thread finds its series' bounds again: cheap
// next to a launch on small queries, not on the named query's 400,000)
#ifndef OTSDB_PREP_FOLD_MAX
#define OTSDB_PREP_FOLD_MAX 65536
#endif
// (the environment's OTSDB_PREP_FOLD_MAX overrides it: the tests run both
// forms on one process)
int64_t prep_fold_max() {
  const char* e = getenv("OTSDB_PREP_FOLD_MAX");
  return e ? atoll(e) : (int64_t)OTSDB_PREP_FOLD_MAX;
}
constexpr int64_t kFoldMinWindow = OTSDB_FOLD_MIN_WINDOW;

// the storage rows cannot be taken verbatim (run_raw_verbatim): flagged on
// the context, never returned through the C-ABI
otsdb_status spec_miss(otsdb_ctx* c);

struct Carve {
  char* base;
  size_t off = 0;
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T* p = reinterpret_cast<T*>(base + off);
    off += n * sizeof(T);
    return p;
  }
};

// device buffers of one query's pipeline, carved from the context workspace
struct Work {
  SeriesMeta SM;
  Rows R;
  Packed* partial;
  uint8_t* tile_emit;
  double* out_val;
  uint8_t* out_emit;
  int64_t* counts;
  uint64_t* keys = nullptr;
  uint64_t* key_mm = nullptr;  // per (bucket, 64-member tile) min / max key
  uint32_t* key_cnt = nullptr;  // per (bucket, tile) non-NaN keys (fill mode)
  uint32_t* lg_kept = nullptr;  // per large group: holds a kept series
  SelState* sel = nullptr;
  XSel* xsel = nullptr;        // cross-rank selection (mode 2)
  Packed* comb = nullptr;      // two-level combine: first-level slices
  uint8_t* comb_emit = nullptr;
  uint8_t* redo = nullptr;     // fused-rate series handed back (Params.redo)
  bool sel_fused = false;      // fill-mode selection: keys + counts by the transpose
};

}  // namespace

struct otsdb_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  void* ws = nullptr;
  size_t ws_cap = 0;
  void* stage = nullptr;
  size_t stage_cap = 0;
  int* d_err = nullptr;                 // device error word
  unsigned long long* d_mm = nullptr;   // k_bounds min/max
  int64_t* h_small = nullptr;           // pinned readback
  // {error word, total points} of the last compaction, written by the
  // kernel straight into host memory (coherent, mapped): no read-back copy
  int64_t* h_done = nullptr;
  int64_t* d_done = nullptr;            // its device address
  // tile plan cache (keyed by the group offsets)
  std::vector<int64_t> goff_cache;
  int64_t* d_tiles = nullptr;
  size_t d_tiles_cap = 0;
  int64_t n_tiles = 0, n_multi = 0, n_large = 0, n_large_chunks = 0;
  int64_t max_chunks = 0;  // most chunks in one group
  bool tiles_sel_all = false;
  int64_t tiles_chunk = 0;
  int64_t tiles_whole = 0;
  bool verbatim = false;  // run_raw_verbatim: the cells query's rows as stored
  // the cells fold's uniform kernel met a qualifier that is not its series'
  // (ERR_CELLS_NONUNI): this call's next attempt takes the general kernel
  bool cells_no_uni = false;
  // otsdb_ctx_counters: cells folds launched uniform / general, uniform
  // folds that missed (ERR_CELLS_NONUNI, re-run with the general kernel)
  int64_t n_cells_uniform = 0, n_cells_general = 0, n_cells_uni_miss = 0;
  bool spec_miss = false;  // ... and they cannot be: the caller compacts
  bool result_short = false;  // the last E_CAPACITY was the result's (finish)
  std::mutex mu;  // one query at a time per context
  // stage timing (otsdb_prof_*)
  bool prof = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_pending;
  size_t ev_used = 0;
  double prof_ms[8] = {0};
  int64_t prof_n[8] = {0};
  void* cells_ws = nullptr;  // cells query: series row / point offsets
  size_t cells_ws_cap = 0;
  void* cells_col = nullptr;  // cells query fallback: decoded columns
  size_t cells_col_cap = 0;
  void* cal = nullptr;  // calendar bucket edges of the current query
  size_t cal_cap = 0;
  void* acal_fill = nullptr;  // stage A' (calendar fill): compacted batch
  size_t acal_fill_cap = 0;
  void* acal = nullptr;  // per-series calendar: chains, anchors, series'
  size_t acal_cap = 0;   // chain positions and bucket-start timestamps
  void* dec_ws = nullptr;  // decode workspace
  size_t dec_ws_cap = 0;
  int dec_generic = 0;  // the last decode count pass: bit 0 / 1, k_decode_generic counts / writes
  void* ws2 = nullptr;     // raw group-by: candidates, sort, selection slab
  size_t ws2_cap = 0;
  void* rows_ws = nullptr;  // storage-row compaction / span assembly: per-row
  size_t rows_ws_cap = 0;   // and per-series plan arrays
  void* rows_scr = nullptr;  // GENERAL-row cell records + staging / replay arenas
  size_t rows_scr_cap = 0;
  void* rows_large = nullptr;  // LARGE rows: ranked columns, keys, sort temp
  size_t rows_large_cap = 0;
  void* raw_cells[2] = {nullptr, nullptr};  // raw-row query: compacted rows,
  size_t raw_cells_cap[2] = {0, 0};          // then the assembled spans
  void* raw_stage = nullptr;  // otsdb_agg_run_raw: host rows staged in HBM
  size_t raw_stage_cap = 0;
  // single-pass compaction (k_compact1): per-group look-back granules and
  // the call's epoch; {error word, total} read back in one copy
  void* cmp_flags = nullptr;
  size_t cmp_flags_cap = 0;
  uint32_t cmp_epoch = 0;
  // the device error word is known to be zero (the last call ended with the
  // one-pass compaction, which zeroes it): the next pipeline skips its
  // memset.  clean_entry: that mark as the current call found it (CtxLock)
  bool err_clean = false;
  bool clean_entry = false;
  bool small_ready = false;  // k_compact1 wrote {error word, total}
  // cross-rank selection session (otsdb_sel_*): lives in `ws` between calls
  struct {
    bool active = false;
    Params P;
    otsdb_query_spec spec;
    Work W;
    int64_t G = 0, NB = 0, M = 0;
    int median = 0;
    int32_t next_pass = 0;   // the pass otsdb_sel_hist_device expects
    bool more = false;       // the last planned pass has work
    bool pool_built = false;  // pass 1 compacted the candidates
    bool need_pick = false;
    // diagnostics (otsdb_ctx_counters): passes over the local key matrix
    // and histogram passes of the last session
    int64_t key_reads = 0, passes = 0;
    void* pool = nullptr;    // candidates: keys [cap] | segments [cap]
    size_t pool_bytes = 0;
    int64_t pool_cap = 0;
    // per segment: pool bounds [GB+1] | region offsets [GB+1] | fill [GB] |
    // the offsets' scan storage
    void* segmem = nullptr;
    size_t segmem_bytes = 0, scan_tmp = 0;
  } sel;
};

namespace {

otsdb_status ensure(void** p, size_t* cap, size_t need) {
  if (need <= *cap) return OTSDB_OK;
  if (*p) hipFree(*p);
  *p = nullptr;
  *cap = 0;
  size_t n = std::max(need, (size_t)1 << 20);
  hipError_t e = hipMalloc(p, n);
  if (e != hipSuccess)
    return fail(OTSDB_E_DEVICE, "hipMalloc(%zu): %s", n, hipGetErrorString(e));
  *cap = n;
  return OTSDB_OK;
}

// One call at a time per context.  Also takes the "error word known zero"
// mark for this call (clean_entry) and clears it: only the one-pass
// compaction's read-back (finish) sets it again, after k_compact1 zeroed
// the word — any other call may leave bits in it.
struct CtxLock {
  std::lock_guard<std::mutex> lk;
  explicit CtxLock(otsdb_ctx* c) : lk(c->mu) {
    c->clean_entry = c->err_clean;
    c->err_clean = false;
  }
};

// Binds a caller's stream to the context for one call and restores the
// context's own stream on every exit path (early HIP_TRY returns included).
struct StreamBinding {
  otsdb_ctx* c;
  hipStream_t saved;
  StreamBinding(otsdb_ctx* c_, void* hip_stream) : c(c_), saved(c_->stream) {
    if (hip_stream) c->stream = (hipStream_t)hip_stream;
  }
  ~StreamBinding() { c->stream = saved; }
};

// --------------------------------------------------------------- planning
struct Plan {
  Params P;
  int64_t S, G, M, N;
  bool sel;  // percentile/median across series
};

otsdb_status check_spec(const otsdb_query_spec* s) {
  if (s->agg_id < 0 || s->agg_id >= OTSDB_AGG_COUNT_IDS)
    return fail(OTSDB_E_NO_SUCH_ELEMENT, "No such aggregator: %d", s->agg_id);
  if (s->interp < -1 || s->interp > OTSDB_INTERP_PREV)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "bad interpolation %d", s->interp);
  const bool ds = s->ds_interval_ms > 0 || s->run_all;
  if (!ds) {  // raw group-by (raw.hip)
    if (s->start_ms < 0)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative start");
    return OTSDB_OK;
  }
  if (s->ds_agg_id < 0 || s->ds_agg_id >= OTSDB_AGG_COUNT_IDS)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "No such downsampling function");
  if (s->ds_agg_id == OTSDB_AGG_NONE)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                "cannot use the NONE aggregator for downsampling");
  if (s->use_calendar && !s->run_all && s->n_cal_anchors > 0) {
    // per-series anchors: chains ended by INT64_MAX, anchors ascending, each
    // naming its chain edge
    const int64_t n = s->n_cal_edges, na = s->n_cal_anchors;
    if (!s->cal_edges || n < 3 || !s->cal_anchors || !s->cal_anchor_edge)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT, "anchored calendar without tables");
    if (s->cal_edges[n - 1] != INT64_MAX)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                  "anchored cal_edges must end with INT64_MAX");
    for (int64_t k = 1; k < n; ++k)
      if (s->cal_edges[k - 1] != INT64_MAX && s->cal_edges[k] != INT64_MAX &&
          s->cal_edges[k] <= s->cal_edges[k - 1])
        return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                    "cal_edges chains must increase strictly (index %lld)",
                    (long long)k);
    for (int64_t j = 0; j < na; ++j) {
      const int64_t e = s->cal_anchor_edge[j];
      if ((j && s->cal_anchors[j] <= s->cal_anchors[j - 1]) || e < 0 ||
          e >= n || s->cal_edges[e] != s->cal_anchors[j])
        return fail(OTSDB_E_ILLEGAL_ARGUMENT, "bad calendar anchor %lld",
                    (long long)j);
    }
    if (s->cal_anchors[0] > s->start_ms)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                  "no calendar anchor at or before start_ms");
  } else if (s->use_calendar && !s->run_all) {
    if (!s->cal_edges || s->n_cal_edges < 2)
      return fail(OTSDB_E_UNSUPPORTED,
                  "calendar downsampling without a bucket-edge table");
    for (int64_t k = 1; k < s->n_cal_edges; ++k)
      if (s->cal_edges[k] <= s->cal_edges[k - 1])
        return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                    "cal_edges must increase strictly (index %lld)",
                    (long long)k);
    if (s->cal_edges[0] > s->start_ms)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                  "cal_edges[0] must be previousInterval(start_ms)");
  }
  if (s->fill == OTSDB_FILL_SCALAR)
    return fail(OTSDB_E_UNSUPPORTED, "unhandled fill policy");
  if (s->fill < 0 || s->fill > OTSDB_FILL_SCALAR)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "bad fill policy %d", s->fill);
  if (s->interp < -1 || s->interp > OTSDB_INTERP_PREV)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "bad interpolation %d", s->interp);
  if (!s->run_all && s->start_ms < 0)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative start");
  return OTSDB_OK;
}

// Calendar grid (otsdb_query_spec.cal_edges): the fixed-interval rules of
// make_params restated on the edge table — seek to the first edge >= start
// (ValuesInInterval.seekInterval rounds up, Downsampler.java:431-441), NONE:
// every edge <= end_ms; filling: [previousInterval(start),
// previousInterval(end)) advanced once when both coincide
// (FillingDownsampler.java:113-131).  With a context the table is copied to
// the device and P->cal points at the grid's bucket 0.
otsdb_status make_cal_params(const otsdb_query_spec* s, Params* P,
                             otsdb_ctx* c) {
  const int64_t* e = s->cal_edges;
  const int64_t n = s->n_cal_edges;
  auto first_ge = [&](int64_t t) {
    return (int64_t)(std::lower_bound(e, e + n, t) - e);
  };
  auto last_le = [&](int64_t t) {
    return (int64_t)(std::upper_bound(e, e + n, t) - e) - 1;
  };
  const int64_t k_seek = first_ge(s->start_ms);
  int64_t nb;
  if (P->fill) {
    const int64_t kA = last_le(s->start_ms);
    int64_t kE = last_le(s->end_ms);
    if (kE == kA) kE = kA + 1;
    nb = std::max<int64_t>(0, kE - k_seek);
    if (kA >= 0 && kA < k_seek) {
      P->rate_origin_ts = e[kA];
      P->rate_origin_val = P->fill_value;
    }
  } else {
    nb = std::max<int64_t>(0, last_le(s->end_ms) - k_seek + 1);
  }
  if (k_seek + nb >= n)
    return fail(OTSDB_E_UNSUPPORTED,
                "calendar table ends before the window (%lld edges)",
                (long long)n);
  P->nb = nb;
  P->gbase = e[k_seek];
  P->seek_ts = e[k_seek];
  P->stop_ts = e[k_seek + nb];
  P->narrow = 0;
  P->cal_lo = -k_seek;
  P->cal_n = n - k_seek;
  P->cal = nullptr;
  if (c) {
    otsdb_status rc = ensure(&c->cal, &c->cal_cap, sizeof(int64_t) * n);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->cal, e, sizeof(int64_t) * n,
                           hipMemcpyHostToDevice, c->stream));
    P->cal = (const int64_t*)c->cal + k_seek;
  }
  return OTSDB_OK;
}

// Grid of buckets every series row is laid out on.
otsdb_status make_params(const otsdb_query_spec* s, Params* P,
                         otsdb_ctx* c = nullptr) {
  memset(P, 0, sizeof(*P));
  P->start_ms = s->start_ms;
  P->end_ms = s->end_ms;
  P->run_all = s->run_all;
  P->fill = s->run_all ? 0 : s->fill;
  P->rate = s->rate;
  P->counter = s->counter;
  P->drop_resets = s->drop_resets;
  P->counter_max = s->counter_max;
  P->reset_value = s->reset_value;
  P->interp = s->interp >= 0 ? s->interp : kAggs[s->agg_id].interp;
  P->fill_value = (P->fill == OTSDB_FILL_ZERO) ? 0.0 : NAN;
  P->pct = s->agg_id >= OTSDB_AGG_P999 ? pct_of(s->agg_id) : 0.0;
  P->pct_est = s->agg_id < OTSDB_AGG_P999   ? 0
               : s->agg_id < OTSDB_AGG_EP999R3 ? 0
               : s->agg_id < OTSDB_AGG_EP999R7 ? 3
                                               : 7;
  if (!(s->ds_interval_ms > 0 || s->run_all)) return OTSDB_OK;  // raw
  if (is_selection(s->ds_agg_id)) {
    P->ds_sel = s->ds_agg_id == OTSDB_AGG_MEDIAN ? 1 : 2;
    P->ds_pct = s->ds_agg_id >= OTSDB_AGG_P999 ? pct_of(s->ds_agg_id) : 0.0;
  }
  P->rate_origin_ts = 0;
  P->rate_origin_val = 0.0;
  if (s->run_all) {
    // Downsampler "all": one point at query_start holding the points of
    // [query_start, query_end) after seek(start) (Downsampler.java:354-379)
    P->interval = 1;
    P->inv_interval = 1.0;
    P->gbase = s->query_start_ms;
    P->out_ts0 = s->query_start_ms;
    P->seek_ts = std::max(s->start_ms, s->query_start_ms);
    P->stop_ts = s->query_end_ms;
    P->nb = (s->query_start_ms >= s->start_ms &&
             s->query_start_ms <= s->end_ms) ? 1 : 0;
    P->narrow = 1;  // every point is bucket 0
    return OTSDB_OK;
  }
  const int64_t iv = s->ds_interval_ms;
  P->interval = iv;
  P->inv_interval = 1.0 / (double)iv;
  if (s->use_calendar && s->n_cal_anchors > 0)  // callers derive stage B
    return fail(OTSDB_E_UNSUPPORTED,
                "per-series calendar grids on this entry point");
  if (s->use_calendar) return make_cal_params(s, P, c);
  const int64_t grid0 = align_down(s->start_ms + iv - 1, iv);
  P->gbase = grid0;
  P->seek_ts = grid0;
  if (P->fill) {
    // FillingDownsampler: every bucket of [align(start), align(end)); the
    // aggregation iterator skips those before start (FillingDownsampler.java
    // :136-142, AggregationIterator.java:425-447)
    const int64_t aend = align_down(s->end_ms, iv);
    P->nb = aend > grid0 ? (aend - grid0) / iv : 0;
    P->stop_ts = grid0 + P->nb * iv;
    const int64_t astart = align_down(s->start_ms, iv);
    if (astart < grid0) {
      P->rate_origin_ts = astart;
      P->rate_origin_val = P->fill_value;
    }
  } else {
    P->nb = s->end_ms >= grid0 ? (s->end_ms - grid0) / iv + 1 : 0;
    P->stop_ts = grid0 + P->nb * iv;
  }
  // points fed to the bucket fold lie in [gbase, stop_ts): 32-bit offsets
  P->narrow = iv < (int64_t(1) << 31) && P->nb < (int64_t(1) << 32) / iv;
  return OTSDB_OK;
}

// Per-series calendar grids (calendar.hip): the union grid U of stage B,
// each anchor's chain terminator, the window's seek and the stage-B spec.
struct AnchoredPlan {
  std::vector<int64_t> U, chain_end;
  int64_t seek_ts = 0;
  int64_t stop_b = 0;  // stage B's stop bound (NONE: U's first edge > end)
  // fill != none: FillingDownsampler's own grid FD (U then holds FD, then
  // the table's end t_end and t_end + 1: calendar.hip)
  std::vector<int64_t> FD;
  int64_t t_end = 0;
  otsdb_query_spec derived;
};

bool anchored(const otsdb_query_spec* s) {
  return s->use_calendar && !s->run_all && s->n_cal_anchors > 0 &&
         s->ds_interval_ms > 0;
}

otsdb_status plan_anchored(const otsdb_query_spec* s, AnchoredPlan* A) {
  const int64_t n = s->n_cal_edges, na = s->n_cal_anchors;
  const int64_t* e = s->cal_edges;
  A->U.clear();
  A->U.reserve(n);
  for (int64_t k = 0; k < n; ++k)
    if (e[k] != INT64_MAX) A->U.push_back(e[k]);
  std::sort(A->U.begin(), A->U.end());
  A->U.erase(std::unique(A->U.begin(), A->U.end()), A->U.end());
  std::vector<int64_t> term(n + 1, n);
  for (int64_t k = n - 1; k >= 0; --k) term[k] = e[k] == INT64_MAX ? k : term[k + 1];
  A->chain_end.resize(na);
  for (int64_t j = 0; j < na; ++j) A->chain_end[j] = term[s->cal_anchor_edge[j]];
  // ValuesInInterval.seekInterval(start): previousInterval(start), stepped
  // once when start lies past it (Downsampler.java:419-429)
  const int64_t j = (int64_t)(std::upper_bound(s->cal_anchors,
                                               s->cal_anchors + na,
                                               s->start_ms) -
                              s->cal_anchors) - 1;
  int64_t k = s->cal_anchor_edge[j];
  if (s->start_ms > e[k]) ++k;
  if (e[k] == INT64_MAX)
    return fail(OTSDB_E_UNSUPPORTED, "calendar chain ends before the seek");
  A->seek_ts = e[k];
  if (s->fill != OTSDB_FILL_NONE) {
    // FillingDownsampler.java:113-135: previousInterval(start) = e[k0], then
    // the chain's steps while < previousInterval(end), advanced once when
    // the two coincide
    const int64_t k0 = s->cal_anchor_edge[j];
    const int64_t je = (int64_t)(std::upper_bound(s->cal_anchors,
                                                  s->cal_anchors + na,
                                                  s->end_ms) -
                                 s->cal_anchors) - 1;
    int64_t end_ts = s->cal_anchors[je];
    if (end_ts == e[k0]) {
      if (e[k0 + 1] == INT64_MAX)
        return fail(OTSDB_E_UNSUPPORTED, "calendar chain ends at the start");
      end_ts = e[k0 + 1];
    }
    A->FD.clear();
    int64_t kk = k0;
    for (; e[kk] != INT64_MAX && e[kk] < end_ts; ++kk) A->FD.push_back(e[kk]);
    if (e[kk] == INT64_MAX)
      return fail(OTSDB_E_UNSUPPORTED, "calendar chain ends before the window");
    // every point stage A' keeps lies on an FD edge: the last bucket's end
    // only has to lie past it (and at end_ms, so the table's grid ends there)
    A->t_end = std::max(s->end_ms, A->FD.back() + 1);
    A->U = A->FD;
    A->U.push_back(A->t_end);
    A->U.push_back(A->t_end + 1);
  }
  {
    const auto it = std::upper_bound(A->U.begin(), A->U.end(), s->end_ms);
    A->stop_b = it == A->U.end() ? INT64_MAX : *it;
  }
  A->derived = *s;
  A->derived.cal_edges = A->U.data();
  A->derived.n_cal_edges = (int64_t)A->U.size();
  A->derived.cal_anchors = nullptr;
  A->derived.cal_anchor_edge = nullptr;
  A->derived.n_cal_anchors = 0;
  return check_spec(&A->derived);
}

// sel_all: every group (even one without local members) joins the radix
// select lists — the cross-rank selection protocol needs global segments
// whole_upto: groups of at most this many members are one tile (one
// sequential chain), larger ones are cut into chunks of `chunk`
otsdb_status build_tiles(otsdb_ctx* c, const std::vector<int64_t>& goff,
                         bool sel_all = false, int64_t chunk = kChunk,
                         int64_t whole_upto = 0) {
  if (c->d_tiles && goff == c->goff_cache && sel_all == c->tiles_sel_all &&
      chunk == c->tiles_chunk && whole_upto == c->tiles_whole)
    return OTSDB_OK;
  const int64_t G = (int64_t)goff.size() - 1;
  std::vector<int64_t> tg, tm0, tm1, mg, mt0, mt1, ag, at0, at1;
  std::vector<int64_t> lgg, lgo, lgk, lgc{0};  // groups for radix select
  std::vector<uint8_t> single;
  for (int64_t g = 0; g < G; ++g) {
    const int64_t a = goff[g], b = goff[g + 1];
    const int64_t t0 = (int64_t)tg.size();
    const int64_t ch = (b - a <= whole_upto) ? std::max<int64_t>(b - a, 1) : chunk;
    for (int64_t m = a; m < b; m += ch) {
      tg.push_back(g);
      tm0.push_back(m);
      tm1.push_back(std::min(b, m + ch));
    }
    const int64_t t1 = (int64_t)tg.size();
    for (int64_t t = t0; t < t1; ++t) single.push_back(t1 - t0 == 1);
    if (t1 - t0 > 1) {
      mg.push_back(g);
      mt0.push_back(t0);
      mt1.push_back(t1);
    }
    ag.push_back(g);
    at0.push_back(t0);
    at1.push_back(t1);
    if (b - a > SEL_K || sel_all) {
      lgg.push_back(g);
      lgo.push_back(a);
      lgk.push_back(b - a);
      lgc.push_back(lgc.back() + (b - a + SEL_CHUNK - 1) / SEL_CHUNK);
    }
  }
  const int64_t LG = (int64_t)lgg.size();
  const int64_t T = (int64_t)tg.size(), MG = (int64_t)mg.size();
  int64_t max_chunks = 0;
  for (int64_t k = 0; k < G; ++k) max_chunks = std::max(max_chunks, at1[k] - at0[k]);
  // layout: tg tm0 tm1 [T] | mg mt0 mt1 [MG] | ag at0 at1 [G] |
  //         lg_g lg_off lg_k [LG] | lg_ch0 [LG+1] | single [T]
  const size_t n64 = 3 * T + 3 * MG + 3 * G + 4 * LG + 1;
  const size_t bytes = n64 * 8 + T + 64;
  void* p = c->d_tiles;
  size_t cap = c->d_tiles_cap;
  otsdb_status st = ensure(&p, &cap, bytes);
  c->d_tiles = (int64_t*)p;
  c->d_tiles_cap = cap;
  if (st) return st;
  std::vector<int64_t> h;
  h.reserve(n64);
  h.insert(h.end(), tg.begin(), tg.end());
  h.insert(h.end(), tm0.begin(), tm0.end());
  h.insert(h.end(), tm1.begin(), tm1.end());
  h.insert(h.end(), mg.begin(), mg.end());
  h.insert(h.end(), mt0.begin(), mt0.end());
  h.insert(h.end(), mt1.begin(), mt1.end());
  h.insert(h.end(), ag.begin(), ag.end());
  h.insert(h.end(), at0.begin(), at0.end());
  h.insert(h.end(), at1.begin(), at1.end());
  h.insert(h.end(), lgg.begin(), lgg.end());
  h.insert(h.end(), lgo.begin(), lgo.end());
  h.insert(h.end(), lgk.begin(), lgk.end());
  h.insert(h.end(), lgc.begin(), lgc.end());
  if (!h.empty())
    HIP_TRY(hipMemcpyAsync(c->d_tiles, h.data(), n64 * 8,
                           hipMemcpyHostToDevice, c->stream));
  if (T)
    HIP_TRY(hipMemcpyAsync((char*)c->d_tiles + n64 * 8, single.data(), T,
                           hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->goff_cache = goff;
  c->tiles_sel_all = sel_all;
  c->tiles_chunk = chunk;
  c->tiles_whole = whole_upto;
  c->n_tiles = T;
  c->n_multi = MG;
  c->n_large = LG;
  c->n_large_chunks = lgc.back();
  c->max_chunks = max_chunks;
  return OTSDB_OK;
}

struct Tiles {
  const int64_t *tg, *tm0, *tm1, *mg, *mt0, *mt1, *ag, *at0, *at1;
  const int64_t *lg_g, *lg_off, *lg_k, *lg_ch0;
  const uint8_t* single;
  int64_t T, MG, G, LG, LGCH;
  int64_t max_chunks;
};

Tiles tiles_of(otsdb_ctx* c, int64_t G) {
  Tiles t;
  const int64_t T = c->n_tiles, MG = c->n_multi;
  const int64_t* b = c->d_tiles;
  t.tg = b;
  t.tm0 = b + T;
  t.tm1 = b + 2 * T;
  t.mg = b + 3 * T;
  t.mt0 = t.mg + MG;
  t.mt1 = t.mg + 2 * MG;
  t.ag = b + 3 * T + 3 * MG;
  t.at0 = t.ag + G;
  t.at1 = t.ag + 2 * G;
  const int64_t LG = c->n_large;
  t.lg_g = b + 3 * T + 3 * MG + 3 * G;
  t.lg_off = t.lg_g + LG;
  t.lg_k = t.lg_g + 2 * LG;
  t.lg_ch0 = t.lg_g + 3 * LG;
  t.single = (const uint8_t*)(b + 3 * T + 3 * MG + 3 * G + 4 * LG + 1);
  t.LG = LG;
  t.LGCH = c->n_large_chunks;
  t.T = T;
  t.MG = MG;
  t.G = G;
  t.max_chunks = c->max_chunks;
  return t;
}

// two-level ordered combine for groups of more than kCombineL1 chunks: the
// single-level k_combine is one dependent chain of max_chunks loads per
// (group, bucket) thread (C4: 1,953 chunks, 1.9 ms); first-level slices
// cut it to ~max_chunks / kCombineSlices
constexpr int64_t kCombineL1 = 128;
constexpr int64_t kCombineSlices = 64;

// Brackets a pipeline stage with HIP events when profiling is enabled.
struct StageTimer {
  otsdb_ctx* c;
  int stage;
  hipEvent_t a = nullptr, b = nullptr;
  hipEvent_t get() {
    if (c->ev_used == c->ev_pool.size()) {
      hipEvent_t e;
      hipEventCreate(&e);
      c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_used++];
  }
  StageTimer(otsdb_ctx* c_, int s_) : c(c_), stage(s_) {
    if (c->prof) {
      a = get();
      hipEventRecord(a, c->stream);
    }
  }
  ~StageTimer() {
    if (c->prof) {
      b = get();
      hipEventRecord(b, c->stream);
      c->ev_pending.push_back({stage, {a, b}});
    }
  }
};

inline unsigned blocks_for(int64_t n, int per) {
  return (unsigned)((n + per - 1) / per);
}



template <class M>
void launch_combine(otsdb_ctx* c, const Work& W, int64_t NB, int64_t n,
                    const int64_t* g, const int64_t* t0, const int64_t* t1,
                    double* out_val, uint8_t* out_emit, Packed* out_partial,
                    bool two_level, int keep_empty = 0) {
  hipStream_t st = c->stream;
  if (!two_level) {
    hipLaunchKernelGGL(k_combine<M>, dim3(blocks_for(n * NB, 256)), dim3(256),
                       0, st, NB, n, g, t0, t1, (const Packed*)W.partial,
                       (const uint8_t*)W.tile_emit, out_val, out_emit,
                       out_partial, c->d_err, (int64_t)0, keep_empty);
    return;
  }
  hipLaunchKernelGGL(k_combine_l1<M>,
                     dim3(blocks_for(n * kCombineSlices * NB, 256)), dim3(256),
                     0, st, NB, n, kCombineSlices, t0, t1,
                     (const Packed*)W.partial, (const uint8_t*)W.tile_emit,
                     W.comb, W.comb_emit);
  hipLaunchKernelGGL(k_combine<M>, dim3(blocks_for(n * NB, 256)), dim3(256), 0,
                     st, NB, n, g, t0, t1, (const Packed*)W.comb,
                     (const uint8_t*)W.comb_emit, out_val, out_emit,
                     out_partial, c->d_err, kCombineSlices, keep_empty);
}

// The per-downsampler kernels live in one translation unit per downsampling
// monoid (ds_tu.hip, built in parallel); this fills their launch record.
DsLaunch ds_args(otsdb_ctx* c, const Params& P, const BatchDev& B,
                 const Work& W) {
  DsLaunch a{};
  a.st = c->stream;
  a.P = P;
  a.B = B;
  a.SM = W.SM;
  a.R = W.R;
  a.err = c->d_err;
  return a;
}

// Whether the ordered group fold (fold.hip) runs this query: every
// downsampled, non-rate query with a monoid aggregator, fill or not (from
// compacted cells, cellfold.hip: when the grid fits one fold window).
// Rate queries keep RateSpan in k_bucketize_k's ring flush + k_group: a
// RateSpan-in-the-fold build measured slower on C4.
bool fold_path(const otsdb_query_spec* spec, const Params& P, int mode) {
  return !P.ds_sel && !P.rate && !P.run_all && !is_selection(spec->agg_id) &&
         mode != 2;
}

// Everything up to dense (group, bucket) results / partials.
// mode 0: final dense results; mode 1: per-group partials into `gpart/gemit`;
// mode 2: the cross-rank selection protocol's local part.
// cells != null: the series come as compacted columns (k_bucketize_cells
// decodes them inside the downsample; B carries only S)
otsdb_status run_pipeline(otsdb_ctx* c, const otsdb_query_spec* spec,
                          const BatchDev& B, const int64_t* d_members,
                          std::vector<int64_t>& goff, Params& P, Work& W,
                          int mode, Packed* gpart, uint8_t* gemit,
                          const CellsDev* cells = nullptr,
                          const int64_t* series_row = nullptr,
                          const Packed* ginit = nullptr,
                          const uint8_t* ginit_emit = nullptr) {
  hipStream_t st = c->stream;
  const int64_t S = B.S;
  const int64_t G = (int64_t)goff.size() - 1;
  const int64_t nb = P.nb;
  // chained partials continue each group's state in k_group (the row path)
  bool fold = fold_path(spec, P, mode) && !ginit;

  // grid trimming for very wide windows (NONE fill only): the rows span only
  // the buckets that hold data
  if (!cells && !P.run_all && !P.fill && !P.cal &&
      (double)S * (double)nb > 4.0e9) {
    unsigned long long init[2] = {~0ULL, 0ULL};
    HIP_TRY(hipMemcpyAsync(c->d_mm, init, 16, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_bounds, dim3(blocks_for(S, 256)), dim3(256), 0, st, P,
                       B, c->d_mm);
    unsigned long long mm[2];
    HIP_TRY(hipMemcpyAsync(mm, c->d_mm, 16, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (mm[0] > mm[1]) {
      P.nb = 0;
    } else {
      const int64_t b_lo = ((int64_t)mm[0] - P.gbase) / P.interval;
      const int64_t b_hi = ((int64_t)mm[1] - P.gbase) / P.interval;
      P.gbase += b_lo * P.interval;
      P.nb = b_hi - b_lo + 1;
    }
  }
  const int64_t NB = P.nb;
  // bucket indices are 32-bit inside the kernels (SeriesMeta.kf/kl, the
  // wave-scan keys): a wider grid would wrap silently
  if (NB > (int64_t)INT32_MAX - 2)
    return fail(OTSDB_E_UNSUPPORTED, "bucket grid of %lld buckets per series",
                (long long)NB);
  int64_t WB = 0, NW = 0;
  if (fold) {
    if (!with_monoid(spec->agg_id, [&](auto tag) {
          WB = fold_wb<decltype(tag)>();
        }))
      return fail(OTSDB_E_NO_SUCH_ELEMENT, "aggregator %d", spec->agg_id);
    NW = (NB + WB - 1) / WB;
  }
  // the cells fold runs on narrow grids (32-bit times), windows after the
  // first starting from k_cells_fold_prep's cursors; calendar grids from
  // cells take k_bucketize_cells and the row pipeline
  if (cells && !P.narrow) {
    fold = false;
    WB = NW = 0;
  }
  bool ordered = false;
  with_monoid(spec->agg_id, [&](auto tag) {
    ordered = decltype(tag)::kOrdered;
  });
  // OTSDB_SPEC_EXACT_ORDER: every group one chain, whatever its size
  const bool exact = ordered && (spec->flags & OTSDB_SPEC_EXACT_ORDER) != 0;
  if (ordered && fold) {
    // a group past one fold tile takes the row path (one chain per bucket)
    // when its bucket matrix (8-byte value + state byte per series and
    // bucket) fits the fixed row budget — a bound of the query alone, so
    // identical queries always take the same path (and the same order);
    // otherwise the fold's tiles stay, merged in order (Chan) like a group
    // past the exact-chain bound, or E_CAPACITY when the caller asked for
    // the exact order
    int64_t kmax = 0;
    for (size_t g = 0; g + 1 < goff.size(); ++g)
      kmax = std::max(kmax, goff[g + 1] - goff[g]);
    if (kmax > kOrderedFoldChunk) {
      if ((double)S * (double)NB * 9.0 <= kOrderedRowBudget) {
        fold = false;
        WB = NW = 0;
      } else if (exact) {
        return fail(OTSDB_E_CAPACITY,
                    "exact-order dev: %lld x %lld bucket rows past the row "
                    "budget", (long long)S, (long long)NB);
      }
    }
  }
  const bool cfold = cells && fold;
  // verbatim storage rows: the single-window cells fold only (it checks
  // what compaction would change; window boundaries it does not see)
  if (c->verbatim && (!cfold || NW > 1)) return spec_miss(c);
  // one chain per (group, bucket) up to kOrderedChunk members; partials for
  // the merge across ranks (a group too large to hand on, dist.py) keep
  // round 4's shorter chains, merged in order anyway
  // the chained entry always takes the row path (its chains continue from
  // the previous rank's states): past the row budget a clear E_CAPACITY
  if (ginit && (double)S * (double)NB * 9.0 > kOrderedRowBudget)
    return fail(OTSDB_E_CAPACITY,
                "chained partials: %lld x %lld bucket rows past the row budget",
                (long long)S, (long long)NB);
  if (exact && mode == 1 && !ginit)
    return fail(OTSDB_E_UNSUPPORTED,
                "exact-order dev across ranks: hand the chains on "
                "(otsdb_agg_partials_chained_device)");
  otsdb_status rc = build_tiles(
      c, goff, mode == 2,
      fold ? (ordered ? kFoldChunk : kFoldChunkLarge) : kChunk,
      ordered ? (fold ? kOrderedFoldChunk
                      : (exact ? INT64_MAX
                               : (mode == 1 && !ginit ? kOrderedChunkMerged
                                                      : kOrderedChunk)))
              : (fold ? kFoldChunk : 0));
  if (rc) return rc;
  const Tiles T = tiles_of(c, G);
  P.fold_wb = 0;  // (P may come from an earlier pipeline run)
  P.fold_ctx = 0;
  if (fold && OTSDB_FOLD_CTX) {
    // tiles of up to 64 members load every member context at workgroup
    // start (k_fold; ds_tu.hip drops it when the LDS would cost occupancy)
    // (non-ordered: the largest tile, a group kept whole or one chunk of a
    // larger one; ordered: bounded by its whole-group size)
    int64_t tile_max = 0;
    for (size_t g = 0; g + 1 < goff.size(); ++g) {
      const int64_t k = goff[g + 1] - goff[g];
      tile_max = std::max(
          tile_max, ordered ? std::min(k, kOrderedFoldChunk)
                            : (k <= kFoldChunk ? k : std::min(k, kFoldChunkLarge)));
    }
    if (tile_max > 0 && tile_max <= 64) P.fold_ctx = (int32_t)tile_max;
  }
  // few tiles (small queries, e.g. C1's 100 groups of 10 series): narrower
  // fold windows give the grid more workgroups — each window's workgroup
  // streams only that window's points (k_fold_prep hands it the context)
  if (fold && !c->verbatim && T.T > 0 && NB > kFoldMinWindow &&
      T.T * NW < kFoldMinBlocks) {
    const int64_t want = (kFoldMinBlocks + T.T - 1) / T.T;  // windows
    int64_t wb = (NB + want - 1) / want;
    wb = (wb + 63) / 64 * 64;
    if (wb < kFoldMinWindow) wb = kFoldMinWindow;
    if (wb < WB) {
      WB = wb;
      NW = (NB + WB - 1) / WB;
      P.fold_wb = (int32_t)WB;
    }
  }
  // the bucket matrix (series rows) exists only off the fold path
  if (!fold && (double)S * (double)NB > 2.0e10)
    return fail(OTSDB_E_UNSUPPORTED, "bucket grid too large (%lld x %lld)",
                (long long)S, (long long)NB);

  // workspace
  const bool sel_large = is_selection(spec->agg_id) && (T.LG > 0 || mode == 2);
  const int64_t n_comb = (mode == 1) ? G : T.MG;
  const bool two_level = T.max_chunks > kCombineL1 &&
                         (double)n_comb * kCombineSlices * NB * 33.0 < 2.0e9;
  const size_t rows = fold ? 0 : (size_t)S * NB;
  WinCtx* wc = nullptr;
  CellsFold CF{};
  if (cfold) {
    CF.C = *cells;
    CF.series_row = series_row;
    CF.wide = c->d_err + 1;
  }
  auto carve = [&](char* base) {
    Carve cv{base};
    W.SM.lo = cv.take<int64_t>(S);
    W.SM.hi = cv.take<int64_t>(S);
    W.SM.of_ts = cv.take<int64_t>(S);
    W.SM.of_val = cv.take<double>(S);
    W.SM.of_rate = cv.take<double>(S);
    W.SM.kf = cv.take<int32_t>(S);
    W.SM.kl = cv.take<int32_t>(S);
    W.SM.keep = cv.take<uint8_t>(S);
    W.SM.of_has = cv.take<uint8_t>(S);
    W.redo = cv.take<uint8_t>(S);
    W.R.val = cv.take<double>(rows);
    W.R.state = cv.take<uint8_t>(rows);
    W.partial = cv.take<Packed>((size_t)T.T * NB);
    W.tile_emit = cv.take<uint8_t>((size_t)T.T * NB);
    W.out_val = cv.take<double>((size_t)G * NB);
    W.out_emit = cv.take<uint8_t>((size_t)G * NB);
    W.counts = cv.take<int64_t>(G + 1);
    if (NW > 1) wc = cv.take<WinCtx>((size_t)S * (NW - 1));
    if (cfold) {
      CF.rlo = cv.take<int64_t>(S);
      CF.vlo = cv.take<int64_t>(S);
      CF.qw = cv.take<uint8_t>(S);
      CF.vl0 = cv.take<uint8_t>(S);
      CF.uf = cv.take<uint8_t>(S);
      if (NW > 1) {
        CF.wrlo = cv.take<int64_t>((size_t)S * (NW - 1));
        CF.wvlo = cv.take<int64_t>((size_t)S * (NW - 1));
        CF.wvl0 = cv.take<uint8_t>((size_t)S * (NW - 1));
      }
    }
    if (two_level) {
      W.comb = cv.take<Packed>((size_t)n_comb * kCombineSlices * NB);
      W.comb_emit = cv.take<uint8_t>((size_t)n_comb * kCombineSlices * NB);
    }
    if (sel_large) {
      W.keys = cv.take<uint64_t>((size_t)goff.back() * NB);
      W.key_mm = cv.take<uint64_t>((size_t)((goff.back() + KT_M - 1) / KT_M) * NB * 2);
      W.key_cnt = cv.take<uint32_t>((size_t)((goff.back() + KT_M - 1) / KT_M) * NB);
      W.lg_kept = cv.take<uint32_t>((size_t)T.LG + 1);
      W.sel = cv.take<SelState>((size_t)T.LG * NB);
      if (mode == 2) W.xsel = cv.take<XSel>((size_t)T.LG * NB);
    }
    return cv.off + 256;
  };
  const size_t need = carve(nullptr);
  rc = ensure(&c->ws, &c->ws_cap, need);
  if (rc) return rc;
  carve((char*)c->ws);

  // the error word (+ the cells fold's "wide" word): zero already when the
  // previous call ended in the one-pass compaction
  if (cells || mode != 0 || !c->clean_entry)
    HIP_TRY(hipMemsetAsync(c->d_err, 0, 2 * sizeof(int), st));
  c->clean_entry = false;
  // every (group, bucket) emit flag is written by the fold / k_group /
  // k_combine of a group with members; only empty groups need the zeroes
  bool empty_group = false;
  for (int64_t g = 0; g < G && !empty_group; ++g)
    empty_group = goff[g + 1] == goff[g];
  if (G * NB > 0 && mode != 1 && empty_group)
    HIP_TRY(hipMemsetAsync(W.out_emit, 0, (size_t)G * NB, st));
  // the ring-sink k_bucketize leaves sentinel rows whose states k_transform
  // writes; the cells and selection downsamplers store states into a
  // zeroed row
  P.sentinel = !fold && !cells && !P.ds_sel;
  if (!fold && S > 0 && NB > 0 && !P.sentinel)
    HIP_TRY(hipMemsetAsync(W.R.state, 0, (size_t)S * NB, st));
  // RateSpan inside k_bucketize (NONE fill; the FillingDownsampler's rate
  // origin and fill points stay with k_transform)
  const bool rate_fused = P.sentinel && P.rate && !P.fill && !P.run_all;

  bool ok = true;
  DsLaunch a = ds_args(c, P, B, W);
#ifdef OTSDB_DEBUG_SYNC
  fprintf(stderr, "[otsdb] pipeline S=%lld NB=%lld fold=%d NW=%lld T=%lld G=%lld\n",
          (long long)S, (long long)NB, (int)fold, (long long)NW, (long long)T.T,
          (long long)G);
#endif
  OTSDB_DBG(st, "setup");
  if (fold && S > 0 && NB > 0) {
    // downsample + contribution + aggregator in one ordered pass
    ok = with_monoid(spec->ds_agg_id, [&](auto tag) {
      using M = decltype(tag);
      {
        StageTimer tm(c, 3);
        if (cfold) {
          a.cf = CF;
          launch_cells<M>(DS_CELLS_PREP, a);
          if (!c->cells_no_uni) launch_cells<M>(DS_CELLS_UNIFORM, a);
          if (NW > 1) {
            a.wc = wc;
            a.NW = NW;
            a.WB = WB;
            launch_cells<M>(DS_CELLS_FOLD_PREP, a);
          }
        } else if (NW > 1 && S * (NW - 1) <= prep_fold_max()) {
          a.wc = wc;
          a.NW = NW;
          a.WB = WB;
          launch_ds<M>(DS_PREP_FOLD, a);
        } else {
          launch_ds<M>(DS_PREP, a);
          if (NW > 1) {
            a.wc = wc;
            a.NW = NW;
            a.WB = WB;
            launch_ds<M>(DS_FOLD_PREP, a);
          }
        }
      }
      StageTimer tm(c, 0);
      a.n_tiles = T.T;
      a.tg = T.tg;
      a.tm0 = T.tm0;
      a.tm1 = T.tm1;
      a.single = T.single;
      a.members = d_members;
      a.wc = wc;
      a.NW = NW;
      a.WB = WB;
      a.partial = W.partial;
      a.tile_emit = W.tile_emit;
      a.out_val = W.out_val;
      a.out_emit = W.out_emit;
      a.always_partial = mode == 1;
      a.agg_id = spec->agg_id;
      if (T.T > 0) {
        if (cfold) {
          // the fold with the qualifier width fixed at compile time (one
          // copy of the member loop per kernel: 14 % faster on C2's cells
          // than a width read per member).  k_cells_prep's bits 0 / 1: 4- /
          // 2-byte series kept; both -> ERR_CELLS_GENERIC, and the engine
          // rewrites the batch with one width (k_requal) and runs again
          // k_cells_uniform's bit 2: some kept series is not uniform (or
          // the uniform kernel already missed in this call): the general one
          int widths = 3;
          bool uniform = false;
          if (hipMemcpyAsync(&c->h_small[2], c->d_err, 2 * sizeof(int),
                             hipMemcpyDeviceToHost, st) == hipSuccess &&
              hipStreamSynchronize(st) == hipSuccess) {
            widths = (int)((c->h_small[2] >> 32) & 3);
            uniform = !c->cells_no_uni && !((c->h_small[2] >> 32) & 4);
          }
          if (widths == 3) {
            const int e = (int)(c->h_small[2] & 0xFFFFFFFF) | ERR_CELLS_GENERIC;
            c->h_small[3] = e;
            hipMemcpyAsync(c->d_err, &c->h_small[3], sizeof(int),
                           hipMemcpyHostToDevice, st);
          } else if (uniform) {
            launch_cells<M>(widths == 1 ? DS_CELLS_FOLD4U : DS_CELLS_FOLD2U, a);
            ++c->n_cells_uniform;
          } else {
            launch_cells<M>(widths == 1 ? DS_CELLS_FOLD4 : DS_CELLS_FOLD2, a);
            ++c->n_cells_general;
          }
        }
        else launch_ds<M>(DS_FOLD, a);
      }
    });
    if (!ok) return fail(OTSDB_E_UNSUPPORTED, "downsampler %d", spec->ds_agg_id);
  } else if (cells && S > 0 && NB > 0) {
    // decode fused into the downsample (decode.hip)
    ok = with_monoid(spec->ds_agg_id, [&](auto tag) {
      using M = decltype(tag);
      StageTimer tm(c, 0);
      a.cells = *cells;
      a.series_row = series_row;
      launch_ds<M>(DS_CELLS, a);
    });
    if (!ok) return fail(OTSDB_E_UNSUPPORTED, "downsampler %d", spec->ds_agg_id);
  } else if (S > 0 && NB > 0 && P.ds_sel) {
    // median / percentile downsampling: per-bucket selection
    {
      StageTimer tm(c, 3);
      launch_ds<MSum<3>>(DS_PREP, a);
    }
    StageTimer tm(c, 0);
    hipLaunchKernelGGL(k_ds_select, dim3((unsigned)S), dim3(64), 0, st, P, B,
                       W.SM, W.R);
  } else if (S > 0 && NB > 0) {
    ok = with_monoid(spec->ds_agg_id, [&](auto tag) {
      using M = decltype(tag);
      {
        StageTimer tm(c, 3);
        launch_ds<M>(DS_PREP, a);
      }
      StageTimer tm(c, 0);
      if (rate_fused) {
        // RateSpan fused into the ring flush (1,024-bucket ring: a step
        // hands its series back only across a gap of ~1,000 buckets); then
        // the plain ring kernel for the series handed back
        a.P.redo = W.redo;
        launch_ds<M>(DS_RATE, a);
        a.P.only_redo = 1;
        launch_ds<M>(DS_RING, a);
      } else {
        launch_ds<M>(DS_RING, a);
      }
    });
    if (!ok) return fail(OTSDB_E_UNSUPPORTED, "downsampler %d", spec->ds_agg_id);
  }
  // percentiles over a FillingDownsampler grid with every group large: the
  // keys transpose applies the fill and counts, no k_transform / k_group
  // (cross-rank, mode 2: the same transpose; otsdb_sel_prepare_device
  // derives the counts from its per-tile counts)
  const bool sel_fused = is_selection(spec->agg_id) && (mode == 0 || mode == 2) &&
                         P.sentinel && P.fill && !P.rate && !P.run_all &&
                         T.LG > 0 && T.LG == G;
  if (!fold && S > 0 && NB > 0 && !sel_fused) {
    StageTimer tm(c, 1);
    if (rate_fused) {  // only the series the fused kernel handed back
      P.redo = W.redo;
      P.only_redo = 1;
    }
    hipLaunchKernelGGL(k_transform<0>, dim3(blocks_for(S, 4)), dim3(256), 0,
                       st, P, B, W.SM, W.R, c->d_err);
    P.only_redo = 0;
  }
  if (G > 0 && NB > 0) {
    StageTimer tm(c, 2);
    if (is_selection(spec->agg_id)) {
      if (mode == 1)
        return fail(OTSDB_E_UNSUPPORTED,
                    "percentiles across ranks: use the otsdb_sel_* protocol");
      const int median = spec->agg_id == OTSDB_AGG_MEDIAN ? 1 : 0;
      if (sel_fused) {
        const int64_t M = goff.back();
        const int64_t NSEG = T.LG * NB;
        HIP_TRY(hipMemsetAsync(W.lg_kept, 0, (size_t)T.LG * 4, st));
        SelFill F{W.SM.keep, W.SM.kf, W.SM.kl, P.fill_value, W.key_cnt,
                  T.lg_off, T.LG, W.lg_kept};
        if (M > 0)
          hipLaunchKernelGGL(k_keys_transpose<true>, kt_grid(M, NB),
                             dim3(KT_THREADS), 0, st, NB, M, d_members, W.R, W.keys,
                             W.key_mm, F);
        W.sel_fused = true;
        if (mode == 2) {
          HIP_TRY(hipGetLastError());
          return OTSDB_OK;
        }
        hipLaunchKernelGGL(k_seg_select, dim3((unsigned)NSEG), dim3(SS_THREADS),
                           0, st, NB, M, T.LG, T.lg_g, T.lg_off, T.lg_k,
                           (const uint64_t*)W.keys, (const SelState*)nullptr,
                           (const uint8_t*)nullptr, W.out_val, c->d_err,
                           median, P.pct, (const uint64_t*)W.key_mm,
                           (const uint32_t*)W.key_cnt,
                           (const uint32_t*)W.lg_kept, W.out_emit);
        HIP_TRY(hipGetLastError());
        return OTSDB_OK;
      }
      // n (non-NaN contributions) and the emit mask of every group
      using MC = MSum<3>;
      if (T.T > 0)
        hipLaunchKernelGGL(k_group<MC>, dim3(blocks_for(T.T * NB, 256)),
                           dim3(256), 0, st, NB, T.T, T.tg, T.tm0, T.tm1,
                           T.single, d_members, W.R, W.partial, W.tile_emit,
                           W.out_val, W.out_emit, c->d_err, 0,
                           (const Packed*)nullptr, (const uint8_t*)nullptr);
      if (T.MG > 0)
        launch_combine<MC>(c, W, NB, T.MG, T.mg, T.mt0, T.mt1, W.out_val,
                           W.out_emit, nullptr, two_level);
      if (mode == 2) {
        // cross-rank protocol: local counts + keys only (otsdb_sel_*)
        const int64_t M = goff.back();
        if (M > 0)
          hipLaunchKernelGGL(k_keys_transpose<false>,
                             kt_grid(M, NB),
                             dim3(KT_THREADS), 0, st, NB, M, d_members, W.R, W.keys,
                             W.key_mm, SelFill{});
        HIP_TRY(hipGetLastError());
        return OTSDB_OK;
      }
      // groups of <= SEL_K series: sort in LDS
      hipLaunchKernelGGL(k_group_select,
                         dim3(blocks_for(T.T * NB, SEL_THREADS)),
                         dim3(SEL_THREADS), 0, st, NB, T.T, T.tg, T.tm0, T.tm1,
                         T.single, d_members, W.R, W.out_val, W.out_emit,
                         c->d_err, median, P.pct);
      // larger groups: radix select over transposed keys
      if (T.LG > 0) {
        const int64_t M = goff.back();
        const int64_t NSEG = T.LG * NB;
        hipLaunchKernelGGL(k_keys_transpose<false>,
                           kt_grid(M, NB),
                           dim3(KT_THREADS), 0, st, NB, M, d_members, W.R, W.keys,
                           W.key_mm, SelFill{});
        hipLaunchKernelGGL(k_sel_init, dim3(blocks_for(NSEG, 256)), dim3(256),
                           0, st, NB, T.LG, T.lg_g, (const double*)W.out_val,
                           (const uint8_t*)W.out_emit, W.sel, median, P.pct);
        // one workgroup per (group, bucket) segment: min/max, 11-bit digit
        // passes until <= SS_CAP candidates, LDS gather + count select
        hipLaunchKernelGGL(k_seg_select, dim3((unsigned)NSEG), dim3(SS_THREADS),
                           0, st, NB, M, T.LG, T.lg_g, T.lg_off, T.lg_k,
                           (const uint64_t*)W.keys, (const SelState*)W.sel,
                           (const uint8_t*)W.out_emit, W.out_val, c->d_err,
                           median, P.pct, (const uint64_t*)W.key_mm,
                           (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                           (uint8_t*)nullptr);
      }
    } else {
      ok = with_monoid(spec->agg_id, [&](auto tag) {
        using M = decltype(tag);
        if (!fold && T.T > 0)
          hipLaunchKernelGGL(k_group<M>, dim3(blocks_for(T.T * NB, 256)),
                             dim3(256), 0, st, NB, T.T, T.tg, T.tm0, T.tm1,
                             T.single, d_members, W.R, W.partial, W.tile_emit,
                             W.out_val, W.out_emit, c->d_err, mode, ginit,
                             ginit_emit);
        if (mode == 0) {
          if (T.MG > 0)
            launch_combine<M>(c, W, NB, T.MG, T.mg, T.mt0, T.mt1, W.out_val,
                              W.out_emit, nullptr, two_level);
        } else {
          launch_combine<M>(c, W, NB, G, T.ag, T.at0, T.at1, W.out_val, gemit,
                            gpart, two_level, ginit ? 1 : 0);
        }
      });
      if (!ok) return fail(OTSDB_E_NO_SUCH_ELEMENT, "aggregator %d", spec->agg_id);
    }
  }
  HIP_TRY(hipGetLastError());
  return OTSDB_OK;
}

otsdb_status compact(otsdb_ctx* c, const Params& P, int64_t G,
                     const double* out_val, const uint8_t* out_emit,
                     int64_t* counts, otsdb_result* out) {
  hipStream_t st = c->stream;
  if (G == 0) {
    HIP_TRY(hipMemsetAsync(out->offsets, 0, sizeof(int64_t), st));
    return OTSDB_OK;
  }
  if (P.nb == 0) {
    HIP_TRY(hipMemsetAsync(out->offsets, 0, sizeof(int64_t) * (G + 1), st));
    return OTSDB_OK;
  }
  StageTimer tm(c, 4);
  // grids of up to kCmpRegBuckets: one pass (k_compact1: count, look-back
  // scan, scatter); longer: k_compact_count, k_scan, k_compact_scatter.
  // Either way the call's {error word, total} lands in `small` (mapped host
  // memory) for finish.  Scratch: flags [G] (one pass) or counts [G]
  void* p = c->cmp_flags;
  size_t cap = c->cmp_flags_cap;
  const size_t need = (size_t)G * 8 + 256;
  const bool grow = need > cap;
  otsdb_status rc = ensure(&p, &cap, need);
  c->cmp_flags = p;
  c->cmp_flags_cap = cap;
  if (rc) return rc;
  // epochs 1, 2, ..., 2^24 - 1, then 4, 5, ...: never 0 (fresh granules)
  // and always one ticket slot on from the last call's (k_compact1).  A
  // granule is taken as this call's by its epoch alone, so when the epoch
  // wraps every granule is cleared: one a call 2^24 - 4 calls ago left (a
  // group index only smaller or long-grid calls used since) would otherwise
  // read as published now
  const bool wrap = c->cmp_epoch + 1 == (1u << 24);
  c->cmp_epoch = wrap ? 4u : c->cmp_epoch + 1;
  if (grow || wrap) HIP_TRY(hipMemsetAsync(p, 0, cap, st));  // no stale epochs
  unsigned long long* ticket = (unsigned long long*)((char*)c->d_err + 192);
  int64_t* small = c->d_done;
  // few groups (C1's 100): one group (wavefront) per block, spread over more
  // CUs; many (C2's 10k): four per block (one wave per block ran C2's
  // compaction 0.20 -> 0.27 ms)
  const int gpb = G < 4096 ? 1 : 4;
  if (P.nb <= kCmpRegBuckets) {
    hipLaunchKernelGGL(k_compact1, dim3(blocks_for(G, gpb)),
                       dim3(64 * gpb), 0, st, P, G, out_val, out_emit,
                       (unsigned long long*)p, ticket, c->cmp_epoch,
                       out->offsets, out->capacity, out->ts, out->val,
                       out->is_int, c->d_err, small);
  } else {
    int64_t* cnt = (int64_t*)p;
    hipLaunchKernelGGL(k_compact_count, dim3(blocks_for(G, gpb)),
                       dim3(64 * gpb), 0, st, P, G, out_emit, cnt, ticket,
                       c->cmp_epoch);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, G,
                       (const int64_t*)cnt, out->offsets);
    hipLaunchKernelGGL(k_compact_scatter, dim3(blocks_for(G, gpb)),
                       dim3(64 * gpb), 0, st, P, G, out_val, out_emit,
                       (const int64_t*)cnt, (const int64_t*)out->offsets,
                       out->capacity, out->ts, out->val, out->is_int,
                       c->d_err, small);
  }
  HIP_TRY(hipGetLastError());
  c->small_ready = true;
  return OTSDB_OK;
}

// reads the error word and the total point count; maps to a status
otsdb_status finish(otsdb_ctx* c, int64_t G, otsdb_result* out) {
  hipStream_t st = c->stream;
  if (c->small_ready) {
    // the compaction left {error word, total} in host memory and zeroed the
    // word (one synchronisation, no copy launch)
    c->small_ready = false;
    HIP_TRY(hipStreamSynchronize(st));
    c->h_small[0] = __atomic_load_n(&c->h_done[0], __ATOMIC_ACQUIRE);
    c->h_small[1] = __atomic_load_n(&c->h_done[1], __ATOMIC_ACQUIRE);
    // a look-back that gave up (k_compact1's bounded spin: never expected)
    // marks h_done[2] with a plain store, after the last group may already
    // have swapped the error word out: report it here, and leave the device
    // word (which may hold its bit) to the next call's memset
    if (__atomic_load_n(&c->h_done[2], __ATOMIC_ACQUIRE)) {
      c->h_done[2] = 0;
      c->h_small[0] |= ERR_INTERNAL;
    } else {
      c->err_clean = true;
    }
  } else {
    HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&c->h_small[1], out->offsets + G, sizeof(int64_t),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  const int err = (int)(c->h_small[0] & 0xFFFFFFFF);
  const int64_t total = c->h_small[1];
  if (err & ERR_NONE_MULTI)
    return fail(OTSDB_E_ILLEGAL_DATA, "More than one value in aggregator raw");
  if (err & ERR_RATE_TS)
    return fail(OTSDB_E_ILLEGAL_STATE,
                "Next timestamp is supposed to be strictly greater than the "
                "previous one");
  if (err & ERR_INFINITY)
    return fail(OTSDB_E_ILLEGAL_STATE, "Got Infinity");
  if (err & ERR_RAW_DUP)
    return fail(OTSDB_E_UNSUPPORTED,
                "raw group-by: timestamps decrease inside a span, or a "
                "timestamp repeats more than 65,536 times");
  if (err & ERR_X1_MASK)
    return fail(OTSDB_E_ILLEGAL_STATE, "x1 beyond the millisecond mask");
  if (err & ERR_SEL_TOO_BIG)
    return fail(OTSDB_E_UNSUPPORTED,
                "percentile/median over groups of more than %d series is not "
                "offloaded yet", SEL_K);
  if (err & ERR_CAL_RANGE)
    return fail(OTSDB_E_UNSUPPORTED,
                "a point past the window lies outside the calendar table");
  if (err & ERR_INTERNAL)
    return fail(OTSDB_E_DEVICE, "internal: bucket outside the group row");
  if (total > out->capacity) {
    c->result_short = true;  // the offsets are whole: the host entries return them
    return fail(OTSDB_E_CAPACITY, "result capacity %lld < %lld points",
                (long long)out->capacity, (long long)total);
  }
  return OTSDB_OK;
}

// a host entry's result too small: the caller still gets the offsets the
// whole result needs (offsets[G] = its point count), then the status
otsdb_status copy_offsets_back(otsdb_ctx* c, otsdb_result* out,
                               const int64_t* d_offsets, int64_t G,
                               otsdb_status rc) {
  HIP_TRY(hipMemcpyAsync(out->offsets, d_offsets, 8 * (G + 1),
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return rc;
}

otsdb_status read_goff(otsdb_ctx* c, const otsdb_batch* b, bool device,
                       std::vector<int64_t>& goff) {
  goff.resize(b->n_groups + 1);
  if (b->n_groups < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "n_groups < 0");
  if (!b->group_offsets) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "no groups");
  if (device && b->group_offsets_host) {
    // the caller's host copy of the same offsets: no read-back, no sync
    // (the caller keeps it equal to the device array: include/otsdb_agg.h)
    memcpy(goff.data(), b->group_offsets_host, sizeof(int64_t) * goff.size());
#ifdef OTSDB_DEBUG_SYNC
    {  // debug builds: the host copy's total against the device's
      int64_t last = 0;
      HIP_TRY(hipMemcpyAsync(&last, b->group_offsets + b->n_groups,
                             sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      if (last != goff.back())
        return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                    "group_offsets_host[G] %lld != device %lld",
                    (long long)goff.back(), (long long)last);
    }
#endif
  } else if (device) {
    HIP_TRY(hipMemcpyAsync(goff.data(), b->group_offsets,
                           sizeof(int64_t) * goff.size(),
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  } else {
    memcpy(goff.data(), b->group_offsets, sizeof(int64_t) * goff.size());
  }
  for (size_t i = 1; i < goff.size(); ++i)
    if (goff[i] < goff[i - 1])
      return fail(OTSDB_E_ILLEGAL_ARGUMENT, "group_offsets not monotonic");
  return OTSDB_OK;
}

// Raw (non-downsampled) group-by, raw.hip.  Device pointers throughout.
otsdb_status run_raw(otsdb_ctx* c, const otsdb_query_spec* spec,
                     const otsdb_batch* b, const BatchDev& B,
                     const std::vector<int64_t>& goff, const Params& P,
                     otsdb_result* out) {
  hipStream_t st = c->stream;
  const int64_t S = B.S, N = b->n_points;
  const int64_t G = (int64_t)goff.size() - 1, M = goff.back();
  const bool rate = P.rate != 0;
  int64_t kmax = 0;
  for (int64_t g = 0; g < G; ++g) kmax = std::max(kmax, goff[g + 1] - goff[g]);
  // ---- phase 1 workspace: per series / member / group
  int64_t *lo, *hi, *rts = nullptr, *rval = nullptr, *ccount, *coff, *segb,
      *sege, *counts;
  auto carve1 = [&](char* base) {
    Carve cv{base};
    lo = cv.take<int64_t>(S + 1);
    hi = cv.take<int64_t>(S + 1);
    if (rate) {
      rts = cv.take<int64_t>(N + 1);
      rval = cv.take<int64_t>(N + 1);
    }
    ccount = cv.take<int64_t>(M + 1);
    coff = cv.take<int64_t>(M + 1);
    segb = cv.take<int64_t>(G + 1);
    sege = cv.take<int64_t>(G + 1);
    counts = cv.take<int64_t>(G + 1);
    return cv.off + 256;
  };
  otsdb_status rc = ensure(&c->ws, &c->ws_cap, carve1(nullptr));
  if (rc) return rc;
  carve1((char*)c->ws);
  HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int), st));
  if (G == 0) {
    HIP_TRY(hipMemsetAsync(out->offsets, 0, sizeof(int64_t), st));
    return finish(c, G, out);
  }
  if (S > 0) {
    hipLaunchKernelGGL(k_raw_prep, dim3(blocks_for(S, 256)), dim3(256), 0, st,
                       P, B, lo, hi);
    if (rate)
      hipLaunchKernelGGL(k_raw_rate, dim3(blocks_for(S, 4)), dim3(256), 0, st,
                         P, B, lo, hi, rts, rval, c->d_err);
  }
  RawView V;
  V.ts = rate ? rts : B.ts;
  V.val = rate ? rval : B.val;
  V.is_float = rate ? nullptr : B.is_float;
  V.series_float = rate ? nullptr : B.series_float;
  V.all_double = rate || (!B.is_float && !B.series_float);
  V.lo = lo;
  V.hi = hi;
  const int mixed = !V.all_double;
  HIP_TRY(hipMemsetAsync(coff, 0, sizeof(int64_t) * (M + 1), st));
  if (M > 0) {
    hipLaunchKernelGGL(k_raw_cand_count, dim3(blocks_for(M, 256)), dim3(256), 0,
                       st, P, V, M, b->group_members, ccount);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, M,
                       (const int64_t*)ccount, coff);
  }
  HIP_TRY(hipMemcpyAsync(&c->h_small[2], coff + M, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t C = c->h_small[2];
  if (C >= (int64_t(1) << 32))
    return fail(OTSDB_E_UNSUPPORTED, "raw group-by over %lld candidate points",
                (long long)C);
  // ---- phase 2 workspace: candidates, sort temp, emitted-point groups
  // keys (ts << 16) | occurrence (raw.hip); candidates have ts <= end_ms
  if (spec->end_ms >= kRawTsMax)
    return fail(OTSDB_E_UNSUPPORTED, "raw group-by past 2^47 ms");
  const int end_bit = kOccBits + std::max(1, 64 - __builtin_clzll((uint64_t)std::max<int64_t>(spec->end_ms, 1)));
  size_t sort_tmp = 0;
  if (C > 0)
    HIP_TRY(rocprim::segmented_radix_sort_keys(
        nullptr, sort_tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
        (unsigned)C, (unsigned)G, segb, sege, 0, end_bit, st));
  uint64_t *kin, *kout;
  void* tmp;
  int32_t *ugrp, *uocc;
  auto carve2 = [&](char* base) {
    Carve cv{base};
    kin = cv.take<uint64_t>(C + 1);
    kout = cv.take<uint64_t>(C + 1);
    ugrp = cv.take<int32_t>(C + 1);
    uocc = cv.take<int32_t>(C + 1);
    tmp = cv.take<char>(sort_tmp + 1);
    return cv.off + 256;
  };
  rc = ensure(&c->ws2, &c->ws2_cap, carve2(nullptr));
  if (rc) return rc;
  carve2((char*)c->ws2);
  if (M > 0)
    hipLaunchKernelGGL(k_raw_cand_fill, dim3(blocks_for(M, 4)), dim3(256), 0,
                       st, P, V, M, b->group_members, (const int64_t*)coff, kin,
                       c->d_err);
  hipLaunchKernelGGL(k_raw_segments, dim3(blocks_for(G, 256)), dim3(256), 0, st,
                     G, b->group_offsets, (const int64_t*)coff, segb, sege);
  if (C > 0)
    HIP_TRY(rocprim::segmented_radix_sort_keys(
        tmp, sort_tmp, (const uint64_t*)kin, kout, (unsigned)C, (unsigned)G,
        segb, sege, 0, end_bit, st));
  hipLaunchKernelGGL(k_raw_unique, dim3(blocks_for(G, 4)), dim3(256), 0, st, G,
                     (const int64_t*)segb, (const int64_t*)sege,
                     (const uint64_t*)kout, counts, (const int64_t*)nullptr,
                     (int64_t)0, (int64_t*)nullptr, (int32_t*)nullptr,
                     (int32_t*)nullptr, 0);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, G,
                     (const int64_t*)counts, out->offsets);
  hipLaunchKernelGGL(k_raw_unique, dim3(blocks_for(G, 4)), dim3(256), 0, st, G,
                     (const int64_t*)segb, (const int64_t*)sege,
                     (const uint64_t*)kout, counts,
                     (const int64_t*)out->offsets, out->capacity, out->ts, ugrp,
                     uocc, 1);
  HIP_TRY(hipMemcpyAsync(&c->h_small[2], out->offsets + G, 8,
                         hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t n_out = std::min<int64_t>(c->h_small[2], out->capacity);
  if (n_out > 0) {
    if (is_selection(spec->agg_id)) {
      const int median = spec->agg_id == OTSDB_AGG_MEDIAN ? 1 : 0;
      // keys slab: one kmax-key row per block, at most 64 Mi keys per launch
      const int64_t per = std::max<int64_t>(
          1, std::min<int64_t>(n_out, ((int64_t)1 << 26) / std::max<int64_t>(kmax, 1)));
      void* p = c->dec_ws;
      size_t cap = c->dec_ws_cap;
      rc = ensure(&p, &cap, (size_t)(per * std::max<int64_t>(kmax, 1)) * 8);
      c->dec_ws = p;
      c->dec_ws_cap = cap;
      if (rc) return rc;
      for (int64_t u0 = 0; u0 < n_out; u0 += per) {
        const int64_t nb = std::min(per, n_out - u0);
        hipLaunchKernelGGL(k_raw_select, dim3((unsigned)nb), dim3(64), 0, st, P,
                           V, median, u0, n_out, b->group_offsets,
                           b->group_members, (const int32_t*)ugrp,
                           (const int32_t*)uocc, (const int64_t*)out->ts,
                           out->val, out->is_int,
                           (uint64_t*)c->dec_ws, std::max<int64_t>(kmax, 1),
                           c->d_err);
      }
    } else {
      const bool ok = with_monoid(spec->agg_id, [&](auto tag) {
        using Mo = decltype(tag);
        hipLaunchKernelGGL(k_raw_eval<Mo>, dim3(blocks_for(n_out, 256)),
                           dim3(256), 0, st, P, V, (int)spec->agg_id, mixed,
                           n_out, b->group_offsets, b->group_members,
                           (const int32_t*)ugrp, (const int32_t*)uocc,
                           (const int64_t*)out->ts, out->val, out->is_int,
                           c->d_err);
      });
      if (!ok) return fail(OTSDB_E_NO_SUCH_ELEMENT, "aggregator %d", spec->agg_id);
    }
  }
  HIP_TRY(hipGetLastError());
  return finish(c, G, out);
}

otsdb_status run_device_impl(otsdb_ctx* c, const otsdb_query_spec* spec,
                             const otsdb_batch* b, otsdb_result* out,
                             std::vector<int64_t>& goff);

otsdb_status scan_excl(void* tmp, size_t tmp_bytes, const int64_t* in,
                       int64_t* out, int64_t n, hipStream_t st);
size_t scan_tmp_bytes(int64_t n, hipStream_t st);

// FillingDownsampler over per-series grids (calendar.hip, stage A'): the
// points whose own bucket starts on the filling grid, compacted, then the
// filling calendar pipeline over that grid.
otsdb_status run_anchored_fill(otsdb_ctx* c, const AnchoredPlan& A,
                               const otsdb_batch* b, int64_t* vts,
                               const AnchoredCal& AC,
                               const std::vector<void*>& pp, otsdb_result* out,
                               std::vector<int64_t>& goff) {
  hipStream_t st = c->stream;
  const otsdb_query_spec* spec = &A.derived;
  const int64_t S = b->n_series;
  int64_t Np = 0;
  if (S > 0) {
    HIP_TRY(hipMemcpyAsync(&Np, b->offsets + S, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  const int64_t nfd = (int64_t)A.FD.size();
  const size_t tmpb = scan_tmp_bytes(S, st);
  // (upper bound of the compacted copy: every point + 2 per series)
  const int64_t Nc = Np + 2 * S;
  auto carve = [&](char* base) {
    Carve cv{base};
    void* p[7];
    p[0] = cv.take<int64_t>(nfd);
    p[1] = cv.take<uint8_t>(std::max<int64_t>(Np, 1));
    p[2] = cv.take<int64_t>(S + 1);
    p[3] = cv.take<int64_t>(S + 1);
    p[4] = cv.take<int64_t>(std::max<int64_t>(Nc, 2));
    p[5] = cv.take<int64_t>(std::max<int64_t>(Nc, 2));
    p[6] = cv.take<uint8_t>(std::max<int64_t>(Nc, 1));
    void* t = cv.take<char>(tmpb);
    return std::make_pair(cv.off + 256, std::vector<void*>{p[0], p[1], p[2], p[3],
                                                          p[4], p[5], p[6], t});
  };
  otsdb_status rc = ensure(&c->acal_fill, &c->acal_fill_cap, carve(nullptr).first);
  if (rc) return rc;
  auto q = carve((char*)c->acal_fill).second;
  int64_t* fd = (int64_t*)q[0];
  uint8_t* on = (uint8_t*)q[1];
  int64_t* cnt = (int64_t*)q[2];
  int64_t* offs = (int64_t*)q[3];
  int64_t* ts2 = (int64_t*)q[4];
  int64_t* val2 = (int64_t*)q[5];
  uint8_t* isf2 = b->is_float ? (uint8_t*)q[6] : nullptr;
  HIP_TRY(hipMemcpyAsync(fd, A.FD.data(), 8 * nfd, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(cnt + S, 0, 8, st));
  BatchDev B{S, b->offsets, b->ts_ms, b->val, b->is_float, b->series_float};
  if (S > 0) {
    hipLaunchKernelGGL(k_cal_fill_count, dim3(blocks_for(S, 4)), dim3(256), 0,
                       st, spec->start_ms, spec->end_ms, B, AC,
                       (const int64_t*)pp[4], (const int64_t*)pp[5],
                       (const int64_t*)pp[6], fd, nfd, vts, on, cnt, c->d_err);
    rc = scan_excl(q[7], tmpb, cnt, offs, S, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_cal_fill_write, dim3(blocks_for(S, 4)), dim3(256), 0,
                       st, spec->start_ms, A.t_end, B, (const int64_t*)vts, on,
                       (const int64_t*)offs, ts2, val2, isf2);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c->h_small[0] & ERR_CAL_RANGE)
      return fail(OTSDB_E_UNSUPPORTED,
                  "a point lies before its series' calendar chain");
  }
  otsdb_batch vb = *b;
  vb.n_points = 0;
  if (S > 0) {
    HIP_TRY(hipMemcpyAsync(&vb.n_points, offs + S, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  vb.offsets = offs;
  vb.ts_ms = ts2;
  vb.val = val2;
  vb.is_float = isf2;
  return run_device_impl(c, spec, &vb, out, goff);
}

// Per-series calendar grids: stage A rewrites the timestamps to the series'
// own bucket starts (calendar.hip), stage B runs the calendar pipeline over
// the union grid.
otsdb_status run_anchored(otsdb_ctx* c, const otsdb_query_spec* spec,
                          const otsdb_batch* b, otsdb_result* out,
                          std::vector<int64_t>& goff) {
  AnchoredPlan A;
  otsdb_status rc = plan_anchored(spec, &A);
  if (rc) return rc;
  hipStream_t st = c->stream;
  const int64_t S = b->n_series, n = spec->n_cal_edges,
                na = spec->n_cal_anchors;
  int64_t N = 0;
  if (S > 0) {
    HIP_TRY(hipMemcpyAsync(&N, b->offsets + S, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  auto carve = [&](char* base) {
    Carve cv{base};
    void* p[8];
    p[0] = cv.take<int64_t>(n);
    p[1] = cv.take<int64_t>(na);
    p[2] = cv.take<int64_t>(na);
    p[3] = cv.take<int64_t>(na);
    p[4] = cv.take<int64_t>(S + 1);
    p[5] = cv.take<int64_t>(S + 1);
    p[6] = cv.take<int64_t>(S + 1);
    p[7] = cv.take<int64_t>(std::max<int64_t>(N, 2));
    return std::make_pair(cv.off + 256, std::vector<void*>(p, p + 8));
  };
  rc = ensure(&c->acal, &c->acal_cap, carve(nullptr).first);
  if (rc) return rc;
  auto pp = carve((char*)c->acal).second;
  HIP_TRY(hipMemcpyAsync(pp[0], spec->cal_edges, 8 * n, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(pp[1], spec->cal_anchors, 8 * na, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(pp[2], spec->cal_anchor_edge, 8 * na,
                         hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(pp[3], A.chain_end.data(), 8 * na,
                         hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int), st));
  AnchoredCal AC{(const int64_t*)pp[0], (const int64_t*)pp[1],
                 (const int64_t*)pp[2], (const int64_t*)pp[3], na};
  BatchDev B{S, b->offsets, b->ts_ms, b->val, b->is_float, b->series_float};
  int64_t* vts = (int64_t*)pp[7];
  if (S > 0) {
    hipLaunchKernelGGL(k_cal_anchor, dim3(blocks_for(S, 256)), dim3(256), 0,
                       st, spec->start_ms, spec->end_ms, A.seek_ts, B, AC,
                       (int64_t*)pp[4], (int64_t*)pp[5], (int64_t*)pp[6],
                       c->d_err);
    if (A.FD.empty())
      hipLaunchKernelGGL(k_cal_vts, dim3(blocks_for(S, 4)), dim3(256), 0, st,
                         spec->start_ms, A.stop_b, (int)spec->rate, B, AC,
                         (const int64_t*)pp[4], (const int64_t*)pp[5],
                         (const int64_t*)pp[6], vts, c->d_err);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c->h_small[0] & ERR_CAL_RANGE)
      return fail(OTSDB_E_UNSUPPORTED,
                  "a point lies outside its series' calendar chain");
  }
  otsdb_batch vb = *b;
  vb.ts_ms = vts;
  if (!A.FD.empty()) return run_anchored_fill(c, A, b, vts, AC, pp, out, goff);
  return run_device_impl(c, &A.derived, &vb, out, goff);
}

otsdb_status run_device_impl(otsdb_ctx* c, const otsdb_query_spec* spec,
                             const otsdb_batch* b, otsdb_result* out,
                             std::vector<int64_t>& goff) {
  otsdb_status rc = check_spec(spec);
  if (rc) return rc;
  if (anchored(spec)) return run_anchored(c, spec, b, out, goff);
  Params P;
  rc = make_params(spec, &P, c);
  if (rc) return rc;
  if ((((uintptr_t)b->ts_ms) | ((uintptr_t)b->val)) & 15)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                "ts_ms/val must be 16-byte aligned (16-B streaming loads)");
  BatchDev B{b->n_series, b->offsets, b->ts_ms, b->val, b->is_float,
             b->series_float};
  if (!(spec->ds_interval_ms > 0 || spec->run_all))
    return run_raw(c, spec, b, B, goff, P, out);
  Work W;
  rc = run_pipeline(c, spec, B, b->group_members, goff, P, W, 0, nullptr,
                    nullptr);
  if (rc) return rc;
  const int64_t G = (int64_t)goff.size() - 1;
  rc = compact(c, P, G, W.out_val, W.out_emit, W.counts, out);
  if (rc) return rc;
  return finish(c, G, out);
}

// otsdb_decode_cells_device without the lock (also the fallback of the
// fused cells query)
// counted: an earlier call on the same cells (ts_ms null) left the row
// counts, output offsets and uniform flags in the context's decode workspace
// and the series offsets in `offsets`: only the write pass runs.
otsdb_status decode_impl(otsdb_ctx* c, const otsdb_cells* cells,
                         int64_t n_series, int64_t* offsets, int64_t* ts_ms,
                         int64_t* val, uint8_t* is_float, int64_t capacity,
                         hipStream_t st, bool counted = false) {
  const int64_t R = cells->n_rows, S = n_series;
  if (R < 0 || S < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  // workspace: row counts, row output offsets, uniform-column flags and the
  // device scan's temporary storage
  size_t scan_tmp = 0;
  HIP_TRY(rocprim::exclusive_scan(nullptr, scan_tmp, (const int64_t*)nullptr,
                                  (int64_t*)nullptr, (int64_t)0,
                                  (size_t)(R + 1), rocprim::plus<int64_t>(),
                                  st));
  const size_t ws_need = (size_t)(2 * R + 2) * 8 + (size_t)R + 128 + scan_tmp;
  otsdb_status rc = ensure(&c->dec_ws, &c->dec_ws_cap, ws_need);
  if (rc) return rc;
  int64_t* row_count = (int64_t*)c->dec_ws;
  int64_t* row_out = row_count + (R + 1);
  uint8_t* fast = (uint8_t*)(row_out + (R + 1));
  int* flags = (int*)(((uintptr_t)(fast + R) + 15) & ~(uintptr_t)15);
  void* tmp = (void*)(((uintptr_t)(flags + 4) + 63) & ~(uintptr_t)63);
  CellsDev C{R, cells->row_series, cells->row_base_s, cells->qual_off,
             cells->qual, cells->val_off, cells->val};
  // the write pass: k_decode for the uniform rows, k_decode_generic for the
  // rest when the count pass saw any (c->dec_generic)
  auto write_pass = [&]() -> otsdb_status {
    if (R > 0) {
      hipLaunchKernelGGL(k_decode, dim3(blocks_for(R, 4)), dim3(256), 0, st, C,
                         1, row_count, (const int64_t*)row_out, fast, capacity,
                         ts_ms, val, is_float, c->d_err, flags);
      if (c->dec_generic & 2)
        hipLaunchKernelGGL(k_decode_generic, dim3(blocks_for(R, 4)), dim3(256),
                           0, st, C, 1, row_count, (const int64_t*)row_out,
                           (const uint8_t*)fast, capacity, ts_ms, val, is_float,
                           c->d_err);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
    return OTSDB_OK;
  };
  if (counted) return write_pass();
  HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int), st));
  HIP_TRY(hipMemsetAsync(flags, 0, 2 * sizeof(int), st));
  c->dec_generic = 0;
  if (R > 0) {
    hipLaunchKernelGGL(k_decode, dim3(blocks_for(R, 4)), dim3(256), 0, st, C,
                       0, row_count, (const int64_t*)nullptr, fast, (int64_t)0,
                       (int64_t*)nullptr, (int64_t*)nullptr,
                       (uint8_t*)nullptr, c->d_err, flags);
    int hf[2];
    HIP_TRY(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    c->dec_generic = (hf[0] ? 1 : 0) | (hf[1] ? 2 : 0);
    if (c->dec_generic & 1)
      hipLaunchKernelGGL(k_decode_generic, dim3(blocks_for(R, 4)), dim3(256), 0,
                         st, C, 0, row_count, (const int64_t*)nullptr,
                         (const uint8_t*)fast, (int64_t)0, (int64_t*)nullptr,
                         (int64_t*)nullptr, (uint8_t*)nullptr, c->d_err);
    // row_count[R] = 0, so row_out[R] = the total
    HIP_TRY(hipMemsetAsync(row_count + R, 0, 8, st));
    HIP_TRY(rocprim::exclusive_scan(tmp, scan_tmp, (const int64_t*)row_count,
                                    row_out, (int64_t)0, (size_t)(R + 1),
                                    rocprim::plus<int64_t>(), st));
  } else {
    HIP_TRY(hipMemsetAsync(row_out, 0, 8, st));
  }
  hipLaunchKernelGGL(k_series_offsets, dim3(blocks_for(R + 1, 256)), dim3(256),
                     0, st, R, S, cells->row_series, (const int64_t*)row_out,
                     offsets);
  HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                         hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[1], row_out + R, 8, hipMemcpyDeviceToHost,
                         st));
  HIP_TRY(hipStreamSynchronize(st));
  if (c->h_small[0] & ERR_CORRUPT_CELL)
    return fail(OTSDB_E_ILLEGAL_DATA,
                "Corrupted value: couldn't break down into individual values");
  const int64_t total = c->h_small[1];
  if (!ts_ms) return OTSDB_OK;
  if (total > capacity)
    return fail(OTSDB_E_CAPACITY, "decode capacity %lld < %lld points",
                (long long)capacity, (long long)total);
  return write_pass();
}

// Columns of mixed qualifier widths rewritten with one (k_requal, decode.hip)
// into the context's cells_col buffer: *out views the rewritten qualifier
// pool with the original rows and value pool.  A count pass, a scan of the
// row counts, a write pass.
otsdb_status requal_impl(otsdb_ctx* c, const CellsDev& C, CellsDev* out,
                         hipStream_t st) {
  const int64_t R = C.R;
  size_t scan_tmp = 0;
  HIP_TRY(rocprim::exclusive_scan(nullptr, scan_tmp, (const int64_t*)nullptr,
                                  (int64_t*)nullptr, (int64_t)0,
                                  (size_t)(R + 1), rocprim::plus<int64_t>(),
                                  st));
  otsdb_status rc = ensure(&c->dec_ws, &c->dec_ws_cap,
                           (size_t)(2 * R + 2) * 8 + 128 + scan_tmp);
  if (rc) return rc;
  int64_t* row_count = (int64_t*)c->dec_ws;
  int64_t* row_out = row_count + (R + 1);
  void* tmp = (void*)(((uintptr_t)(row_out + R + 1) + 63) & ~(uintptr_t)63);
  HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int), st));
  HIP_TRY(hipMemsetAsync(row_count + R, 0, 8, st));
  if (R > 0)
    hipLaunchKernelGGL(k_requal<0>, dim3(blocks_for(R, 4 * OTSDB_RQ_RPW)), dim3(256), 0, st,
                       C, row_count, (const int64_t*)nullptr, (int64_t*)nullptr,
                       (uint8_t*)nullptr, c->d_err);
  HIP_TRY(hipGetLastError());
  HIP_TRY(rocprim::exclusive_scan(tmp, scan_tmp, (const int64_t*)row_count,
                                  row_out, (int64_t)0, (size_t)(R + 1),
                                  rocprim::plus<int64_t>(), st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                         hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[1], row_out + R, 8, hipMemcpyDeviceToHost,
                         st));
  HIP_TRY(hipStreamSynchronize(st));
  if (c->h_small[0] & ERR_CORRUPT_CELL)
    return fail(OTSDB_E_ILLEGAL_DATA,
                "Corrupted value: couldn't break down into individual values");
  const int64_t N = c->h_small[1];
  const size_t qo = ((size_t)(R + 1) * 8 + 255) & ~(size_t)255;
  rc = ensure(&c->cells_col, &c->cells_col_cap, qo + 4 * (size_t)N + 64);
  if (rc) return rc;
  int64_t* qoff = (int64_t*)c->cells_col;
  uint8_t* qual = (uint8_t*)c->cells_col + qo;
  if (R > 0)
    hipLaunchKernelGGL(k_requal<1>, dim3(blocks_for(R, 4 * OTSDB_RQ_RPW)), dim3(256), 0, st,
                       C, row_count, (const int64_t*)row_out, qoff, qual,
                       c->d_err);
  else
    HIP_TRY(hipMemsetAsync(qoff, 0, 8, st));
  HIP_TRY(hipGetLastError());
  *out = CellsDev{R, C.row_series, C.row_base_s, qoff, qual, C.val_off, C.val};
  return OTSDB_OK;
}

// Query straight from compacted columns: the fused decode + downsample when
// the query and the columns allow it, else decode -> columnar -> pipeline.
otsdb_status run_cells_impl(otsdb_ctx* c, const otsdb_query_spec* spec,
                            const otsdb_cells* cells, const otsdb_batch* b,
                            otsdb_result* out, std::vector<int64_t>& goff) {
  otsdb_status rc = check_spec(spec);
  if (rc) return rc;
  hipStream_t st = c->stream;
  const int64_t S = b->n_series, R = cells->n_rows;
  if (S < 0 || R < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  const bool ds = spec->ds_interval_ms > 0 || spec->run_all;
  Params P;
  // per-series calendar grids rewrite columnar timestamps: decode first
  const bool fused = ds && !anchored(spec);
  if (fused) {
    rc = make_params(spec, &P, c);
    if (rc) return rc;
  }
  CellsDev C{R, cells->row_series, cells->row_base_s, cells->qual_off,
             cells->qual, cells->val_off, cells->val};
  if (fused && !P.ds_sel && !P.run_all) {
    rc = ensure(&c->cells_ws, &c->cells_ws_cap, (size_t)(S + 1) * 8);
    if (rc) return rc;
    int64_t* series_row = (int64_t*)c->cells_ws;
    hipLaunchKernelGGL(k_series_rows, dim3(blocks_for(R + 1, 256)), dim3(256),
                       0, st, R, S, cells->row_series, series_row);
    BatchDev B{S, nullptr, nullptr, nullptr, nullptr, nullptr};
    P.check_order = c->verbatim ? 1 : 0;
    // a column the fused path does not take (ERR_CELLS_GENERIC) — widths
    // mixed inside a row or across a series' rows — is rewritten with
    // 4-byte qualifiers (k_requal) and the fused path runs again; what it
    // still does not take re-runs through the decode below
    // (a uniform fold that meets a qualifier of other flags is run again
    // with the general kernel: ERR_CELLS_NONUNI, one more attempt)
    CellsDev CQ = C;
    c->cells_no_uni = false;
    bool requaled = false;
    for (int attempt = 0; attempt < 4; ++attempt) {
      Work W;
      rc = run_pipeline(c, spec, B, b->group_members, goff, P, W, 0, nullptr,
                        nullptr, &CQ, series_row);
      if (rc) return rc;
      HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                             hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      const int e = (int)(c->h_small[0] & 0xFFFFFFFF);
      if ((e & ERR_CELLS_NONUNI) && !c->cells_no_uni) {
        ++c->n_cells_uni_miss;
        c->cells_no_uni = true;
        continue;
      }
      if (c->verbatim && (e & (ERR_CORRUPT_CELL | ERR_CELLS_GENERIC |
                               ERR_NOT_SORTED | ERR_SPEC_MISS)))
        return spec_miss(c);
      if (e & ERR_CORRUPT_CELL)
        return fail(OTSDB_E_ILLEGAL_DATA,
                    "Corrupted value: couldn't break down into individual values");
      if (!(e & ERR_CELLS_GENERIC)) {
        const int64_t G = (int64_t)goff.size() - 1;
        rc = compact(c, P, G, W.out_val, W.out_emit, W.counts, out);
        if (rc) return rc;
        return finish(c, G, out);
      }
      if (requaled) break;
      requaled = true;
      c->cells_no_uni = false;
      {
        std::unique_ptr<StageTimer> rq_tm(new StageTimer(c, 7));
        rc = requal_impl(c, C, &CQ, st);
        if (rc) return rc;
      }
    }
    c->cells_no_uni = false;
  }
  // (verbatim storage rows take only the cells fold)
  if (c->verbatim) return spec_miss(c);
  // decode to a columnar batch in the context's own buffer, then the
  // columnar pipeline (raw group-by, median/percentile or "all" downsampling,
  // mixed-width columns)
  rc = ensure(&c->cells_ws, &c->cells_ws_cap, (size_t)(S + 1) * 8 + 64);
  if (rc) return rc;
  int64_t* offs = (int64_t*)c->cells_ws;
  // the generic decode (its own stage; released before the pipeline)
  std::unique_ptr<StageTimer> dec_tm(new StageTimer(c, 7));
  rc = decode_impl(c, cells, S, offs, nullptr, nullptr, nullptr, 0, st);
  if (rc) return rc;
  int64_t N = 0;
  HIP_TRY(hipMemcpyAsync(&N, offs + S, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const size_t col = ((size_t)std::max<int64_t>(N, 2) * 8 + 255) & ~(size_t)255;
  rc = ensure(&c->cells_col, &c->cells_col_cap,
              2 * col + (size_t)std::max<int64_t>(N, 2) + 256);
  if (rc) return rc;
  int64_t* ts = (int64_t*)c->cells_col;
  int64_t* vv = (int64_t*)((char*)c->cells_col + col);
  uint8_t* isf = (uint8_t*)((char*)c->cells_col + 2 * col);
  rc = decode_impl(c, cells, S, offs, ts, vv, isf, N, st, true);
  dec_tm.reset();
  if (rc) return rc;
  otsdb_batch cb = *b;
  cb.n_points = N;
  cb.offsets = offs;
  cb.ts_ms = ts;
  cb.val = vv;
  cb.is_float = isf;
  cb.series_float = nullptr;
  return run_device_impl(c, spec, &cb, out, goff);
}

// ----------------------------------------- storage rows -> compacted rows
otsdb_status row_status(otsdb_ctx*, unsigned long long fe, const char* what) {
  if (fe == ~0ULL) return OTSDB_OK;
  const int code = (int)(fe & 0xFF);
  const long long row = (long long)(fe >> 8);
  switch (code) {
    case RS_ILLEGAL_ARGUMENT:
      return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                  "%s row %lld: Can not parse cell, it is not an appended cell",
                  what, row);
    case RS_UNSUPPORTED:
      return fail(OTSDB_E_UNSUPPORTED,
                  "%s row %lld: more than %d points or %d data columns to "
                  "merge, or appended points beside a column out of time order",
                  what, row, kRowCellCap, kRowColCap);
    default:
      return fail(OTSDB_E_ILLEGAL_DATA,
                  "%s row %lld: corrupted value or duplicate timestamp", what,
                  row);
  }
}

// one exclusive scan of n + 1 int64 (in[n] must be 0), on st
otsdb_status scan_excl(void* tmp, size_t tmp_bytes, const int64_t* in,
                       int64_t* out, int64_t n, hipStream_t st) {
  size_t t = tmp_bytes;
  HIP_TRY(rocprim::exclusive_scan(tmp, t, in, out, (int64_t)0, (size_t)(n + 1),
                                  rocprim::plus<int64_t>(), st));
  return OTSDB_OK;
}

size_t scan_tmp_bytes(int64_t n, hipStream_t st) {
  size_t b = 0;
  rocprim::exclusive_scan(nullptr, b, (const int64_t*)nullptr, (int64_t*)nullptr,
                          (int64_t)0, (size_t)(n + 1), rocprim::plus<int64_t>(),
                          st);
  return (b + 255) & ~(size_t)255;
}

// CompactionQueue.compact of every storage row (rows.hip).  Output: the kept
// rows' compacted columns packed in row order, *n_out rows; *qbytes / *vbytes
// the bytes written.
otsdb_status cells_buffer(otsdb_ctx* c, int which, int64_t R, int64_t qb,
                          int64_t vb, otsdb_cells_out* o);

// own >= 0: the output goes to the context's cells buffer `own`, returned in
// *owned (o is ignored)
// LARGE rows (rows.hip): rank the columns, record the cells, sort the keys,
// merge — through global memory, one segment per row
otsdb_status compact_large(otsdb_ctx* c, const RawDev& D, int fix,
                           const LargeSlots& LS, int64_t n_large, int64_t NC,
                           int64_t ncell, const int64_t* gen_base,
                           const int64_t* gen_n, CellRec* rec, uint8_t* stq,
                           uint8_t* stv, int64_t* out_q, int64_t* out_v,
                           unsigned long long* first_err, hipStream_t st) {
  if (NC >= (int64_t(1) << 32) || ncell >= (int64_t(1) << 32))
    return fail(OTSDB_E_UNSUPPORTED, "compaction of %lld cells in large rows",
                (long long)ncell);
  size_t t_pairs = 0, t_keys = 0;
  HIP_TRY(rocprim::segmented_radix_sort_pairs(
      nullptr, t_pairs, (const uint64_t*)nullptr, (uint64_t*)nullptr,
      (const int64_t*)nullptr, (int64_t*)nullptr, (unsigned)NC,
      (unsigned)n_large, (const int64_t*)nullptr, (const int64_t*)nullptr, 0,
      64, st));
  HIP_TRY(rocprim::segmented_radix_sort_keys(
      nullptr, t_keys, (const uint64_t*)nullptr, (uint64_t*)nullptr,
      (unsigned)ncell, (unsigned)n_large, (const int64_t*)nullptr,
      (const int64_t*)nullptr, 0, kLargeKeyBits, st));
  const size_t t_scan = scan_tmp_bytes(NC, st);
  const size_t t_sort = std::max(std::max(t_pairs, t_keys), t_scan);
  uint64_t *ckey, *ckey2, *rkey, *rkey2;
  int64_t *cidx, *cidx2, *cslot, *ccount, *cbase, *segb, *sege;
  int* bad;
  void* tmp;
  auto carve = [&](char* base) {
    Carve cv{base};
    ckey = cv.take<uint64_t>(NC);
    ckey2 = cv.take<uint64_t>(NC);
    cidx = cv.take<int64_t>(NC);
    cidx2 = cv.take<int64_t>(NC);
    cslot = cv.take<int64_t>(NC);
    ccount = cv.take<int64_t>(NC + 1);
    cbase = cv.take<int64_t>(NC + 1);
    segb = cv.take<int64_t>(n_large);
    sege = cv.take<int64_t>(n_large);
    bad = cv.take<int>(n_large);
    rkey = cv.take<uint64_t>(ncell);
    rkey2 = cv.take<uint64_t>(ncell);
    tmp = cv.take<char>(t_sort + 1);
    return cv.off + 256;
  };
  otsdb_status rc = ensure(&c->rows_large, &c->rows_large_cap, carve(nullptr));
  if (rc) return rc;
  carve((char*)c->rows_large);
  hipLaunchKernelGGL(k_large_cols, dim3(blocks_for(n_large, 4)), dim3(256), 0,
                     st, D, LS, n_large, ckey, cidx, cslot, segb, sege);
  size_t t = t_sort;
  HIP_TRY(rocprim::segmented_radix_sort_pairs(
      tmp, t, (const uint64_t*)ckey, ckey2, (const int64_t*)cidx, cidx2,
      (unsigned)NC, (unsigned)n_large, (const int64_t*)segb,
      (const int64_t*)sege, 0, 64, st));
  HIP_TRY(hipMemsetAsync(ccount + NC, 0, 8, st));
  const unsigned wblocks = blocks_for((NC + 63) / 64, 4);
  hipLaunchKernelGGL(k_large_recs, dim3(wblocks), dim3(256), 0, st, D, LS, NC,
                     (const int64_t*)cidx2, (const int64_t*)cslot, gen_base,
                     ccount, (const int64_t*)nullptr, rec, rkey, bad, 0);
  if ((rc = scan_excl(tmp, t_sort, ccount, cbase, NC, st))) return rc;
  HIP_TRY(hipMemsetAsync(bad, 0, sizeof(int) * n_large, st));
  hipLaunchKernelGGL(k_large_recs, dim3(wblocks), dim3(256), 0, st, D, LS, NC,
                     (const int64_t*)cidx2, (const int64_t*)cslot, gen_base,
                     ccount, (const int64_t*)cbase, rec, rkey, bad, 1);
  hipLaunchKernelGGL(k_large_segs, dim3(blocks_for(n_large, 256)), dim3(256),
                     0, st, LS, n_large, gen_base, gen_n, segb, sege);
  t = t_sort;
  HIP_TRY(rocprim::segmented_radix_sort_keys(
      tmp, t, (const uint64_t*)rkey, rkey2, (unsigned)ncell,
      (unsigned)n_large, (const int64_t*)segb, (const int64_t*)sege, 0,
      kLargeKeyBits, st));
  // (rkey, free after the sort, holds the heap order of rows with unsorted
  // columns)
  hipLaunchKernelGGL(k_large_merge, dim3((unsigned)n_large), dim3(64), 0, st,
                     D, fix, LS, gen_base, gen_n, (const CellRec*)rec,
                     (const uint64_t*)rkey2, (const int*)bad, rkey, stq, stv,
                     out_q, out_v, first_err);
  HIP_TRY(hipGetLastError());
  return OTSDB_OK;
}

otsdb_status compact_impl(otsdb_ctx* c, const otsdb_raw_rows* raw, int fix,
                          const otsdb_cells_out* o, int64_t qcap, int64_t vcap,
                          int64_t* n_out, int64_t* qbytes, int64_t* vbytes,
                          hipStream_t st, int own = -1,
                          otsdb_cells_out* owned = nullptr) {
  const int64_t R = raw->n_rows;
  if (R < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative n_rows");
  if (!raw->row_base_s || !raw->row_col_off || !raw->col_qual_off ||
      !raw->col_val_off || (R > 0 && (!raw->qual || !raw->val)))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null raw row array");
  RawDev D{R, raw->row_col_off, raw->col_qual_off, raw->qual, raw->col_val_off,
           raw->val, raw->col_ts};
  const size_t tmpb = scan_tmp_bytes(R, st);
  const size_t A = ((size_t)(R + 1) * 8 + 255) & ~(size_t)255;
  // kind, lone, gen_n, gen_base, out_q, out_v, kept, oq_off, ov_off, k_off,
  // LARGE slots (row, columns, ranked-column base), first_err, counters,
  // scan temp
  const size_t need = 13 * A + 512 + tmpb;
  otsdb_status rc = ensure(&c->rows_ws, &c->rows_ws_cap, need);
  if (rc) return rc;
  char* w = (char*)c->rows_ws;
  uint8_t* kind = (uint8_t*)w;
  int64_t* lone = (int64_t*)(w + A);
  int64_t* gen_n = (int64_t*)(w + 2 * A);
  int64_t* gen_base = (int64_t*)(w + 3 * A);
  int64_t* out_q = (int64_t*)(w + 4 * A);
  int64_t* out_v = (int64_t*)(w + 5 * A);
  int64_t* kept = (int64_t*)(w + 6 * A);
  int64_t* oq_off = (int64_t*)(w + 7 * A);
  int64_t* ov_off = (int64_t*)(w + 8 * A);
  int64_t* k_off = (int64_t*)(w + 9 * A);
  LargeSlots LS{(unsigned long long*)(w + 13 * A + 256), (int64_t*)(w + 10 * A),
                (int64_t*)(w + 11 * A), (int64_t*)(w + 12 * A)};
  unsigned long long* first_err = (unsigned long long*)(w + 13 * A);
  void* tmp = w + 13 * A + 512;
  HIP_TRY(hipMemsetAsync(first_err, 0xFF, 8, st));
  HIP_TRY(hipMemsetAsync(LS.ctr, 0, 16, st));
  for (int64_t* a : {gen_n, out_q, out_v, kept})
    HIP_TRY(hipMemsetAsync(a + R, 0, 8, st));
  if (R > 0) {
    // the verbatim columns first (64 rows a wavefront), the exact plan only
    // when some row is left (a flag read: one sync)
    int* pend = (int*)(LS.ctr + 8);
    HIP_TRY(hipMemsetAsync(pend, 0, sizeof(int), st));
    hipLaunchKernelGGL(k_rows_uniform, dim3(blocks_for(R, 256)), dim3(256), 0,
                       st, D, kind, lone, gen_n, out_q, out_v, kept, pend);
    int hp = 0;
    HIP_TRY(hipMemcpyAsync(&hp, pend, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (hp)
      hipLaunchKernelGGL(k_rows_plan, dim3(blocks_for(R, 4)), dim3(256), 0, st,
                         D, fix, kind, lone, gen_n, out_q, out_v, kept,
                         first_err, LS);
  }
  HIP_TRY(hipGetLastError());
  if ((rc = scan_excl(tmp, tmpb, gen_n, gen_base, R, st))) return rc;
  HIP_TRY(hipMemcpyAsync(&c->h_small[0], gen_base + R, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[5], LS.ctr, 16, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t ncell = c->h_small[0];
  const int64_t n_large = c->h_small[5], NC = c->h_small[6];
  if (ncell > 0) {
    const size_t recb = ((size_t)ncell * sizeof(CellRec) + 255) & ~(size_t)255;
    const size_t qb = ((size_t)ncell * 4 + 255) & ~(size_t)255;
    rc = ensure(&c->rows_scr, &c->rows_scr_cap, recb + qb + (size_t)ncell * 9 + 256);
    if (rc) return rc;
    CellRec* rec = (CellRec*)c->rows_scr;
    uint8_t* stq = (uint8_t*)c->rows_scr + recb;
    uint8_t* stv = stq + qb;
    hipLaunchKernelGGL(k_rows_general, dim3((unsigned)R), dim3(64), 0, st, D, fix,
                       (const uint8_t*)kind, (const int64_t*)gen_base, rec, stq,
                       stv, out_q, out_v, first_err);
    HIP_TRY(hipGetLastError());
    if (n_large > 0 &&
        (rc = compact_large(c, D, fix, LS, n_large, NC, ncell, gen_base, gen_n,
                            rec, stq, stv, out_q, out_v, first_err, st)))
      return rc;
  }
  HIP_TRY(hipMemcpyAsync(&c->h_small[1], first_err, 8, hipMemcpyDeviceToHost, st));
  if ((rc = scan_excl(tmp, tmpb, out_q, oq_off, R, st))) return rc;
  if ((rc = scan_excl(tmp, tmpb, out_v, ov_off, R, st))) return rc;
  if ((rc = scan_excl(tmp, tmpb, kept, k_off, R, st))) return rc;
  HIP_TRY(hipMemcpyAsync(&c->h_small[2], oq_off + R, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[3], ov_off + R, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[4], k_off + R, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  rc = row_status(c, (unsigned long long)c->h_small[1], "storage");
  if (rc) return rc;
  const int64_t tq = c->h_small[2], tv = c->h_small[3], nk = c->h_small[4];
  *n_out = nk;
  if (qbytes) *qbytes = tq;
  if (vbytes) *vbytes = tv;
  int bytes = 1;
  if (own >= 0) {
    if ((rc = cells_buffer(c, own, nk, 0, 0, owned))) return rc;
    // an engine-owned output aliases the input pools when it can
    // (k_rows_alias): the common scan of single compacted columns moves no
    // value bytes
    unsigned long long* acc = LS.ctr + 2;  // 5 words after the counters
    const unsigned long long init[5] = {~0ULL, 0ULL, ~0ULL, 0ULL, 0ULL};
    HIP_TRY(hipMemcpyAsync(acc, init, sizeof(init), hipMemcpyHostToDevice, st));
    if (R > 0)
      hipLaunchKernelGGL(k_rows_alias,
                         dim3((unsigned)std::min<int64_t>(blocks_for(R, 256), 2048)),
                         dim3(256), 0, st, D, (const uint8_t*)kind,
                         (const int64_t*)lone, (const int64_t*)oq_off,
                         (const int64_t*)ov_off, acc);
    HIP_TRY(hipGetLastError());
    unsigned long long h[5];
    HIP_TRY(hipMemcpyAsync(h, acc, sizeof(h), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (nk > 0 && h[4] == 0 && h[0] == h[1] && h[2] == h[3]) {
      bytes = 0;
      owned->qual = const_cast<uint8_t*>(raw->qual) + h[0];
      owned->val = const_cast<uint8_t*>(raw->val) + h[2];
    } else if ((rc = cells_buffer(c, own, nk, tq, tv, owned))) {
      return rc;
    }
    o = owned;
    qcap = tq;
    vcap = tv;
  }
  if (!o) return OTSDB_OK;  // sizes only
  if (tq > qcap || tv > vcap)
    return fail(OTSDB_E_CAPACITY, "compaction output: %lld qualifier / %lld "
                "value bytes, capacity %lld / %lld", (long long)tq,
                (long long)tv, (long long)qcap, (long long)vcap);
  if (!o->row_base_s || !o->qual_off || !o->val_off || !o->qual || !o->val)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null output array");
  CellRec* rec = (CellRec*)c->rows_scr;
  const size_t recb = ((size_t)ncell * sizeof(CellRec) + 255) & ~(size_t)255;
  const size_t qb = ((size_t)ncell * 4 + 255) & ~(size_t)255;
  const uint8_t* stq = ncell ? (uint8_t*)c->rows_scr + recb : nullptr;
  const uint8_t* stv = ncell ? stq + qb : nullptr;
  (void)rec;
  if (R > 0 && nk > 0 && !bytes) {
    hipLaunchKernelGGL(k_rows_meta, dim3(blocks_for(R, 256)), dim3(256), 0, st,
                       R, raw->row_series, raw->row_base_s, (const uint8_t*)kind,
                       (const int64_t*)oq_off, (const int64_t*)ov_off,
                       (const int64_t*)k_off, o->row_series, o->row_base_s,
                       o->qual_off, o->val_off);
    HIP_TRY(hipGetLastError());
  } else if (R > 0 && nk > 0) {
    // row_series is optional on the output
    hipLaunchKernelGGL(k_rows_write, dim3(blocks_for(R, 4)), dim3(256), 0, st,
                       D, fix, raw->row_series, raw->row_base_s,
                       (const uint8_t*)kind, (const int64_t*)lone,
                       (const int64_t*)gen_base, stq, stv,
                       (const int64_t*)out_q, (const int64_t*)out_v,
                       (const int64_t*)oq_off, (const int64_t*)ov_off,
                       (const int64_t*)k_off, o->row_series, o->row_base_s, o->qual_off, o->qual, o->val_off, o->val);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMemcpyAsync(o->qual_off + nk, oq_off + R, 8, hipMemcpyDeviceToDevice, st));
  HIP_TRY(hipMemcpyAsync(o->val_off + nk, ov_off + R, 8, hipMemcpyDeviceToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

// Span.addRow over every series' compacted rows (rows.hip).  *identity: no
// series needed the replay (the output then equals the input and, when
// o == nullptr, nothing is written).
otsdb_status span_impl(otsdb_ctx* c, const otsdb_cells* in, int64_t S,
                       const otsdb_cells_out* o, int64_t qcap, int64_t vcap,
                       int64_t* n_out, int64_t* qbytes, int64_t* vbytes,
                       bool* identity, hipStream_t st, int own = -1,
                       otsdb_cells_out* owned = nullptr) {
  const int64_t R = in->n_rows;
  if (R < 0 || S < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  CellsDev C{R, in->row_series, in->row_base_s, in->qual_off, in->qual,
             in->val_off, in->val};
  const size_t tmpb = scan_tmp_bytes(S, st);
  const size_t A = ((size_t)(S + 1) * 8 + 255) & ~(size_t)255;
  // series_row, slow, arena_sz, arena_off, o_rows, o_q, o_v, row_off, q_off,
  // v_off, err word, scan temp
  const size_t need = 10 * A + 256 + tmpb;
  otsdb_status rc = ensure(&c->rows_ws, &c->rows_ws_cap, need);
  if (rc) return rc;
  char* w = (char*)c->rows_ws;
  int64_t* series_row = (int64_t*)w;
  uint8_t* slow = (uint8_t*)(w + A);
  int64_t* arena_sz = (int64_t*)(w + 2 * A);
  int64_t* arena_off = (int64_t*)(w + 3 * A);
  int64_t* o_rows = (int64_t*)(w + 4 * A);
  int64_t* o_q = (int64_t*)(w + 5 * A);
  int64_t* o_v = (int64_t*)(w + 6 * A);
  int64_t* row_off = (int64_t*)(w + 7 * A);
  int64_t* q_off = (int64_t*)(w + 8 * A);
  int64_t* v_off = (int64_t*)(w + 9 * A);
  int* err = (int*)(w + 10 * A);
  void* tmp = w + 10 * A + 256;
  HIP_TRY(hipMemsetAsync(err, 0, 4, st));
  for (int64_t* a : {arena_sz, o_rows, o_q, o_v})
    HIP_TRY(hipMemsetAsync(a + S, 0, 8, st));
  hipLaunchKernelGGL(k_series_rows, dim3(blocks_for(R + 1, 256)), dim3(256), 0,
                     st, R, S, in->row_series, series_row);
  if (S > 0)
    hipLaunchKernelGGL(k_span_plan, dim3(blocks_for(S, 4)), dim3(256), 0, st, C,
                       S, (const int64_t*)series_row, slow, arena_sz, o_rows,
                       o_q, o_v, err);
  HIP_TRY(hipGetLastError());
  if ((rc = scan_excl(tmp, tmpb, arena_sz, arena_off, S, st))) return rc;
  HIP_TRY(hipMemcpyAsync(&c->h_small[0], arena_off + S, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[1], err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if ((int)(c->h_small[1] & 0xFFFFFFFF))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "a row without a data point");
  const int64_t arena = c->h_small[0];
  *identity = arena == 0;
  if (arena > 0) {
    rc = ensure(&c->rows_scr, &c->rows_scr_cap, (size_t)arena + 256);
    if (rc) return rc;
    hipLaunchKernelGGL(k_span_replay, dim3((unsigned)S), dim3(64), 0, st, C, S,
                       (const int64_t*)series_row, (const uint8_t*)slow,
                       (const int64_t*)arena_off, (uint8_t*)c->rows_scr, o_rows,
                       o_q, o_v);
    HIP_TRY(hipGetLastError());
  }
  if ((rc = scan_excl(tmp, tmpb, o_rows, row_off, S, st))) return rc;
  if ((rc = scan_excl(tmp, tmpb, o_q, q_off, S, st))) return rc;
  if ((rc = scan_excl(tmp, tmpb, o_v, v_off, S, st))) return rc;
  HIP_TRY(hipMemcpyAsync(&c->h_small[2], row_off + S, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[3], q_off + S, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_small[4], v_off + S, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *n_out = c->h_small[2];
  if (qbytes) *qbytes = c->h_small[3];
  if (vbytes) *vbytes = c->h_small[4];
  if (own >= 0) {
    if (*identity) return OTSDB_OK;  // the input is the span order
    if ((rc = cells_buffer(c, own, *n_out, c->h_small[3], c->h_small[4], owned)))
      return rc;
    o = owned;
    qcap = c->h_small[3];
    vcap = c->h_small[4];
  }
  if (!o) return OTSDB_OK;
  if (c->h_small[3] > qcap || c->h_small[4] > vcap)
    return fail(OTSDB_E_CAPACITY, "span output capacity");
  if (S > 0)
    hipLaunchKernelGGL(k_span_write, dim3(blocks_for(S, 4)), dim3(256), 0, st,
                       C, S, (const int64_t*)series_row, (const uint8_t*)slow,
                       (const int64_t*)arena_off, (const uint8_t*)c->rows_scr,
                       (const int64_t*)row_off, (const int64_t*)q_off,
                       (const int64_t*)v_off, o->row_series, o->row_base_s,
                       o->qual_off, o->qual, o->val_off, o->val);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(o->qual_off + *n_out, q_off + S, 8,
                         hipMemcpyDeviceToDevice, st));
  HIP_TRY(hipMemcpyAsync(o->val_off + *n_out, v_off + S, 8,
                         hipMemcpyDeviceToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

// a context-owned cells buffer for R rows, qb / vb bytes
otsdb_status cells_buffer(otsdb_ctx* c, int which, int64_t R, int64_t qb,
                          int64_t vb, otsdb_cells_out* o) {
  const size_t a = ((size_t)(R + 1) * 8 + 255) & ~(size_t)255;
  const size_t q = ((size_t)qb + 256) & ~(size_t)255;
  const size_t v = ((size_t)vb + 256) & ~(size_t)255;
  otsdb_status rc =
      ensure(&c->raw_cells[which], &c->raw_cells_cap[which], 4 * a + q + v);
  if (rc) return rc;
  char* p = (char*)c->raw_cells[which];
  o->row_series = (int64_t*)p;
  o->row_base_s = (int64_t*)(p + a);
  o->qual_off = (int64_t*)(p + 2 * a);
  o->val_off = (int64_t*)(p + 3 * a);
  o->qual = (uint8_t*)(p + 4 * a);
  o->val = (uint8_t*)(p + 4 * a + q);
  return OTSDB_OK;
}

// The storage rows taken verbatim, when they can be: every row one
// compacted column (k_rows_shape), the rows of each series in base-time
// order, every series in one group — the rows ARE the compacted, assembled
// spans, viewed in place (qual_off / val_off point into the column offsets).
// The cells fold checks the rest as it streams (Params.check_order).
// Flags spec_miss when the view does not hold or the query would not
// stream every point through the cells fold; the caller then compacts.
otsdb_status spec_miss(otsdb_ctx* c) {
  c->spec_miss = true;
  return OTSDB_E_UNSUPPORTED;
}

otsdb_status run_raw_verbatim(otsdb_ctx* c, const otsdb_query_spec* spec,
                              const otsdb_raw_rows* raw, const otsdb_batch* b,
                              otsdb_result* out, std::vector<int64_t>& goff) {
  hipStream_t st = c->stream;
  const int64_t R = raw->n_rows;
  if (R <= 0 || goff.empty() || goff.back() != b->n_series ||
      !(spec->ds_interval_ms > 0) || spec->run_all || anchored(spec))
    return spec_miss(c);
  RawDev D{R, raw->row_col_off, raw->col_qual_off, raw->qual, raw->col_val_off,
           raw->val, raw->col_ts};
  int* bad = (int*)c->d_mm;
  HIP_TRY(hipMemsetAsync(bad, 0, sizeof(int), st));
  hipLaunchKernelGGL(k_rows_shape, dim3(blocks_for(R, 256)), dim3(256), 0, st,
                     D, raw->row_series, raw->row_base_s, bad);
  HIP_TRY(hipGetLastError());
  int h[3] = {0, 0, 0};
  int64_t c0 = 0;
  HIP_TRY(hipMemcpyAsync(h, bad, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c0, raw->row_col_off, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (h[0]) return spec_miss(c);
  const otsdb_cells cc{R, raw->row_series, raw->row_base_s,
                       raw->col_qual_off + c0, raw->qual,
                       raw->col_val_off + c0, raw->val};
  c->verbatim = true;
  const otsdb_status rc = run_cells_impl(c, spec, &cc, b, out, goff);
  c->verbatim = false;
  return rc;
}

// The query from storage rows: compaction -> span assembly -> the cells
// query (DEVICE pointers).
otsdb_status run_raw_impl(otsdb_ctx* c, const otsdb_query_spec* spec,
                          const otsdb_raw_rows* raw, int fix,
                          const otsdb_batch* b, otsdb_result* out,
                          std::vector<int64_t>& goff) {
  hipStream_t st = c->stream;
  if (!raw->row_series) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null row_series");
  if (!raw->row_base_s || !raw->row_col_off || !raw->col_qual_off ||
      !raw->col_val_off || (raw->n_rows > 0 && (!raw->qual || !raw->val)))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null raw row array");
  {
    c->spec_miss = false;
    const otsdb_status v = run_raw_verbatim(c, spec, raw, b, out, goff);
    if (!c->spec_miss) return v;
    c->spec_miss = false;
  }
  int64_t nk = 0, tq = 0, tv = 0;
  otsdb_cells_out co;
  otsdb_status rc;
  {
    StageTimer tm(c, 5);  // query-time compaction
    rc = compact_impl(c, raw, fix, nullptr, 0, 0, &nk, &tq, &tv, st, 0, &co);
  }
  if (rc) return rc;
  otsdb_cells cc{nk, co.row_series, co.row_base_s, co.qual_off, co.qual,
                 co.val_off, co.val};
  int64_t ns = 0, sq = 0, sv = 0;
  bool identity = true;
  otsdb_cells_out so;
  {
    StageTimer tm(c, 6);  // span assembly
    rc = span_impl(c, &cc, b->n_series, nullptr, 0, 0, &ns, &sq, &sv,
                   &identity, st, 1, &so);
  }
  if (rc) return rc;
  if (!identity)
    cc = otsdb_cells{ns, so.row_series, so.row_base_s, so.qual_off, so.qual,
                     so.val_off, so.val};
  return run_cells_impl(c, spec, &cc, b, out, goff);
}

}  // namespace

// =========================================================================
// C-ABI
// =========================================================================
extern "C" {

int otsdb_abi_version(void) { return OTSDB_ABI_VERSION; }

const char* otsdb_last_error(void) { return g_last_error.c_str(); }

otsdb_status otsdb_ctx_create(int device, otsdb_ctx** out) {
  if (!out) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null out");
  *out = nullptr;
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n)
    return fail(OTSDB_E_DEVICE, "no HIP device %d (have %d)", device, n);
  HIP_TRY(hipSetDevice(device));
  otsdb_ctx* c = new otsdb_ctx();
  c->device = device;
  // a blocking stream: ordered with the legacy default stream torch uses,
  // so tensors torch writes are complete before this context reads them
  HIP_TRY(hipStreamCreate(&c->stream));
  HIP_TRY(hipMalloc(&c->d_err, 256));
  HIP_TRY(hipMemset(c->d_err, 0, 256));
  c->d_mm = (unsigned long long*)((char*)c->d_err + 64);
  HIP_TRY(hipHostMalloc(&c->h_small, 64));
  HIP_TRY(hipHostMalloc(&c->h_done, 64,
                        hipHostMallocMapped | hipHostMallocCoherent));
  HIP_TRY(hipHostGetDevicePointer((void**)&c->d_done, c->h_done, 0));
  for (int i = 0; i < 8; ++i) c->h_done[i] = 0;
  *out = c;
  return OTSDB_OK;
}

void otsdb_ctx_destroy(otsdb_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->ws) hipFree(c->ws);
  if (c->stage) hipFree(c->stage);
  if (c->dec_ws) hipFree(c->dec_ws);
  if (c->ws2) hipFree(c->ws2);
  if (c->cal) hipFree(c->cal);
  if (c->acal) hipFree(c->acal);
  if (c->acal_fill) hipFree(c->acal_fill);
  if (c->cells_ws) hipFree(c->cells_ws);
  if (c->cells_col) hipFree(c->cells_col);
  if (c->rows_ws) hipFree(c->rows_ws);
  if (c->rows_scr) hipFree(c->rows_scr);
  if (c->rows_large) hipFree(c->rows_large);
  for (void* p : c->raw_cells)
    if (p) hipFree(p);
  if (c->raw_stage) hipFree(c->raw_stage);
  if (c->d_tiles) hipFree(c->d_tiles);
  if (c->sel.pool) hipFree(c->sel.pool);
  if (c->sel.segmem) hipFree(c->sel.segmem);
  if (c->cmp_flags) hipFree(c->cmp_flags);
  if (c->d_err) hipFree(c->d_err);
  for (auto e : c->ev_pool) hipEventDestroy(e);
  if (c->h_small) hipHostFree(c->h_small);
  if (c->h_done) hipHostFree(c->h_done);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

otsdb_status otsdb_agg_lookup(const char* name, int32_t* agg_id) {
  if (!name || !agg_id) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  for (int i = 0; i < OTSDB_AGG_COUNT_IDS; ++i)
    if (strcmp(kAggs[i].key, name) == 0) {
      *agg_id = i;
      return OTSDB_OK;
    }
  return fail(OTSDB_E_NO_SUCH_ELEMENT, "No such aggregator: %s", name);
}

const char* otsdb_agg_name(int32_t agg_id) {
  if (agg_id < 0 || agg_id >= OTSDB_AGG_COUNT_IDS) return nullptr;
  return kAggs[agg_id].name;
}

int32_t otsdb_agg_interpolation(int32_t agg_id) {
  if (agg_id < 0 || agg_id >= OTSDB_AGG_COUNT_IDS) return -1;
  return kAggs[agg_id].interp;
}

otsdb_status otsdb_agg_plan(otsdb_ctx* c, const otsdb_query_spec* spec,
                            const otsdb_batch* b, otsdb_sizes* out) {
  if (!spec || !b || !out) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  otsdb_status rc = check_spec(spec);
  if (rc) return rc;
  AnchoredPlan A;
  if (anchored(spec)) {  // stage B's union grid
    rc = plan_anchored(spec, &A);
    if (rc) return rc;
    spec = &A.derived;
  }
  Params P;
  rc = make_params(spec, &P);
  if (rc) return rc;
  if (!(spec->ds_interval_ms > 0 || spec->run_all)) {
    // raw: every emitted timestamp is a point of some member span, so the
    // batch's point count bounds the output when each span is in one group
    out->n_buckets = 0;
    out->max_out_points = b->n_points;
    out->workspace_bytes = b->n_series * 16 + b->n_points * (spec->rate ? 48 : 32);
    return OTSDB_OK;
  }
  out->n_buckets = P.nb;
  out->max_out_points = b->n_groups * P.nb;
  out->workspace_bytes =
      b->n_series * (P.nb * 9 + 48) + b->n_groups * (P.nb * 9 + 8);
  return OTSDB_OK;
}

otsdb_status otsdb_agg_run_device(otsdb_ctx* c, const otsdb_query_spec* spec,
                                  const otsdb_batch* b, otsdb_result* out,
                                  void* hip_stream) {
  if (!c || !spec || !b || !out) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  StreamBinding bind(c, hip_stream);
  std::vector<int64_t> goff;
  otsdb_status rc = read_goff(c, b, true, goff);
  if (!rc) rc = run_device_impl(c, spec, b, out, goff);
  return rc;
}

otsdb_status otsdb_agg_run_cells_device(otsdb_ctx* c,
                                        const otsdb_query_spec* spec,
                                        const otsdb_cells* cells,
                                        const otsdb_batch* b,
                                        otsdb_result* out, void* hip_stream) {
  if (!c || !spec || !cells || !b || !out)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  StreamBinding bind(c, hip_stream);
  std::vector<int64_t> goff;
  otsdb_status rc = read_goff(c, b, true, goff);
  if (!rc) rc = run_cells_impl(c, spec, cells, b, out, goff);
  return rc;
}

otsdb_status otsdb_agg_run(otsdb_ctx* c, const otsdb_query_spec* spec,
                           const otsdb_batch* b, otsdb_result* out) {
  if (!c || !spec || !b || !out) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  std::vector<int64_t> goff;
  otsdb_status rc = read_goff(c, b, false, goff);
  if (rc) return rc;
  const int64_t S = b->n_series, N = b->n_points, G = b->n_groups;
  const int64_t M = goff.back();
  if (S < 0 || N < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (S > 0 && b->offsets[S] != N)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "offsets[S] != n_points");
  for (int64_t m = 0; m < M; ++m)
    if (b->group_members[m] < 0 || b->group_members[m] >= S)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT, "group member out of range");
  const int64_t cap = out->capacity;
  // staging layout in HBM
  auto carve = [&](char* base) {
    Carve cv{base};
    void* p[11];
    p[0] = cv.take<int64_t>(S + 1);
    p[1] = cv.take<int64_t>(N + 1);
    p[2] = cv.take<int64_t>(N + 1);
    p[3] = b->is_float ? cv.take<uint8_t>(N + 1) : nullptr;
    p[4] = b->series_float ? cv.take<uint8_t>(S + 1) : nullptr;
    p[5] = cv.take<int64_t>(G + 1);
    p[6] = cv.take<int64_t>(M + 1);
    p[7] = cv.take<int64_t>(G + 1);
    p[8] = cv.take<int64_t>(cap + 1);
    p[9] = cv.take<int64_t>(cap + 1);
    p[10] = cv.take<uint8_t>(cap + 1);
    return std::make_pair(cv.off + 256, std::vector<void*>(p, p + 11));
  };
  const size_t need = carve(nullptr).first;
  rc = ensure(&c->stage, &c->stage_cap, need);
  if (rc) return rc;
  auto pp = carve((char*)c->stage).second;
  hipStream_t st = c->stream;
  auto h2d = [&](void* d, const void* h, size_t n) -> otsdb_status {
    if (n && h) HIP_TRY(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st));
    return OTSDB_OK;
  };
  if ((rc = h2d(pp[0], b->offsets, 8 * (S + 1)))) return rc;
  if ((rc = h2d(pp[1], b->ts_ms, 8 * N))) return rc;
  if ((rc = h2d(pp[2], b->val, 8 * N))) return rc;
  if (b->is_float && (rc = h2d(pp[3], b->is_float, N))) return rc;
  if (b->series_float && (rc = h2d(pp[4], b->series_float, S))) return rc;
  if ((rc = h2d(pp[5], b->group_offsets, 8 * (G + 1)))) return rc;
  if ((rc = h2d(pp[6], b->group_members, 8 * M))) return rc;
  otsdb_batch db = *b;
  db.offsets = (const int64_t*)pp[0];
  db.ts_ms = (const int64_t*)pp[1];
  db.val = (const int64_t*)pp[2];
  db.is_float = (const uint8_t*)pp[3];
  db.series_float = (const uint8_t*)pp[4];
  db.group_offsets = (const int64_t*)pp[5];
  db.group_members = (const int64_t*)pp[6];
  otsdb_result dr;
  dr.capacity = cap;
  dr.offsets = (int64_t*)pp[7];
  dr.ts = (int64_t*)pp[8];
  dr.val = (int64_t*)pp[9];
  dr.is_int = (uint8_t*)pp[10];
  c->result_short = false;
  rc = run_device_impl(c, spec, &db, &dr, goff);
  if (rc == OTSDB_E_CAPACITY && c->result_short)
    return copy_offsets_back(c, out, dr.offsets, G, rc);
  if (rc) return rc;
  const int64_t total = c->h_small[1];
  HIP_TRY(hipMemcpyAsync(out->offsets, dr.offsets, 8 * (G + 1),
                         hipMemcpyDeviceToHost, st));
  if (total > 0) {
    HIP_TRY(hipMemcpyAsync(out->ts, dr.ts, 8 * total, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->val, dr.val, 8 * total, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->is_int, dr.is_int, total, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

}  // extern "C"

namespace {
otsdb_status partials_impl(otsdb_ctx* c, const otsdb_query_spec* spec,
                           const otsdb_batch* b, const otsdb_partial* init,
                           const uint8_t* init_emit, otsdb_partial* partials,
                           uint8_t* emit, void* hip_stream) {
  if (!c || !spec || !b || !partials || !emit || (!init != !init_emit))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  StreamBinding bind(c, hip_stream);
  std::vector<int64_t> goff;
  otsdb_status rc = read_goff(c, b, true, goff);
  Params P;
  if (!rc) rc = check_spec(spec);
  if (!rc) rc = make_params(spec, &P, c);
  if (!rc && !(spec->ds_interval_ms > 0 || spec->run_all))
    rc = fail(OTSDB_E_UNSUPPORTED,
              "raw group-by across ranks (union timestamps need an all-gather)");
  if (!rc && !P.run_all && !P.fill && (double)b->n_series * (double)P.nb > 4.0e9)
    rc = fail(OTSDB_E_UNSUPPORTED, "grid trimming is not supported across ranks");
  if (!rc) {
    BatchDev B{b->n_series, b->offsets, b->ts_ms, b->val, b->is_float,
               b->series_float};
    Work W;
    const int64_t G = (int64_t)goff.size() - 1;
    if (G * P.nb > 0 && init) {
      // groups with no member here pass their state on unchanged
      if (init != partials)
        HIP_TRY(hipMemcpyAsync(partials, init,
                               sizeof(otsdb_partial) * (size_t)G * P.nb,
                               hipMemcpyDeviceToDevice, c->stream));
      if (init_emit != emit)
        HIP_TRY(hipMemcpyAsync(emit, init_emit, (size_t)G * P.nb,
                               hipMemcpyDeviceToDevice, c->stream));
    } else if (G * P.nb > 0) {
      hipMemsetAsync(emit, 0, (size_t)G * P.nb, c->stream);
      hipMemsetAsync(partials, 0, sizeof(otsdb_partial) * (size_t)G * P.nb,
                     c->stream);
    }
    rc = run_pipeline(c, spec, B, b->group_members, goff, P, W, 1,
                      (Packed*)partials, emit, nullptr, nullptr,
                      (const Packed*)init, init_emit);
    if (!rc) {
      HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                             hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      const int err = (int)(c->h_small[0] & 0xFFFFFFFF);
      if (err & ERR_RATE_TS)
        rc = fail(OTSDB_E_ILLEGAL_STATE,
                  "Next timestamp is supposed to be strictly greater");
    }
  }
  return rc;
}
}  // namespace

extern "C" {

otsdb_status otsdb_agg_partials_device(otsdb_ctx* c,
                                       const otsdb_query_spec* spec,
                                       const otsdb_batch* b,
                                       otsdb_partial* partials, uint8_t* emit,
                                       void* hip_stream) {
  return partials_impl(c, spec, b, nullptr, nullptr, partials, emit,
                       hip_stream);
}

otsdb_status otsdb_agg_partials_chained_device(
    otsdb_ctx* c, const otsdb_query_spec* spec, const otsdb_batch* b,
    const otsdb_partial* init, const uint8_t* init_emit,
    otsdb_partial* partials, uint8_t* emit, void* hip_stream) {
  if (!init || !init_emit) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null init");
  return partials_impl(c, spec, b, init, init_emit, partials, emit,
                       hip_stream);
}

otsdb_status otsdb_agg_finalize_device(otsdb_ctx* c,
                                       const otsdb_query_spec* spec,
                                       int64_t n_groups, int64_t n_buckets,
                                       int32_t n_ranks,
                                       const otsdb_partial* partials,
                                       const uint8_t* emit, otsdb_result* out,
                                       void* hip_stream) {
  if (!c || !spec || !out) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  StreamBinding bind(c, hip_stream);
  otsdb_status rc = check_spec(spec);
  Params P;
  if (!rc) rc = make_params(spec, &P, c);
  if (!rc && P.nb != n_buckets)
    rc = fail(OTSDB_E_ILLEGAL_ARGUMENT, "n_buckets %lld != plan %lld",
              (long long)n_buckets, (long long)P.nb);
  if (!rc) {
    const int64_t G = n_groups, GB = G * P.nb;
    auto carve = [&](char* base) {
      Carve cv{base};
      double* v = cv.take<double>(GB + 1);
      uint8_t* e = cv.take<uint8_t>(GB + 1);
      int64_t* cnt = cv.take<int64_t>(G + 1);
      return std::make_tuple(cv.off + 256, v, e, cnt);
    };
    rc = ensure(&c->ws, &c->ws_cap, std::get<0>(carve(nullptr)));
    if (!rc) {
      auto t = carve((char*)c->ws);
      double* ov = std::get<1>(t);
      uint8_t* oe = std::get<2>(t);
      int64_t* cnt = std::get<3>(t);
      hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream);
      bool ok = true;
      if (GB > 0)
        ok = with_monoid(spec->agg_id, [&](auto tag) {
          using M = decltype(tag);
          hipLaunchKernelGGL(k_finalize_ranks<M>, dim3(blocks_for(GB, 256)),
                             dim3(256), 0, c->stream, GB, n_ranks,
                             (const Packed*)partials, emit, ov, oe, c->d_err);
        });
      if (!ok) rc = fail(OTSDB_E_UNSUPPORTED, "aggregator %d across ranks",
                         spec->agg_id);
      if (!rc) rc = compact(c, P, G, ov, oe, cnt, out);
      if (!rc) rc = finish(c, G, out);
    }
  }
  return rc;
}

// ---- cross-rank median / percentile -------------------------
otsdb_status otsdb_sel_prepare_device(otsdb_ctx* c, const otsdb_query_spec* spec,
                                      const otsdb_batch* b, int64_t* counts,
                                      uint8_t* emit, int64_t* krange,
                                      void* hip_stream) {
  if (!c || !spec || !b || !counts || !emit || !krange)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  c->sel.active = false;
  StreamBinding bind(c, hip_stream);
  std::vector<int64_t> goff;
  otsdb_status rc = read_goff(c, b, true, goff);
  Params P;
  if (!rc) rc = check_spec(spec);
  if (!rc && !is_selection(spec->agg_id))
    rc = fail(OTSDB_E_ILLEGAL_ARGUMENT, "otsdb_sel_* needs median/percentile");
  if (!rc && !(spec->ds_interval_ms > 0 || spec->run_all))
    rc = fail(OTSDB_E_UNSUPPORTED, "raw group-by across ranks");
  if (!rc) rc = make_params(spec, &P, c);
  if (!rc && !P.run_all && !P.fill && (double)b->n_series * (double)P.nb > 4.0e9)
    rc = fail(OTSDB_E_UNSUPPORTED, "grid trimming is not supported across ranks");
  if (!rc) {
    BatchDev B{b->n_series, b->offsets, b->ts_ms, b->val, b->is_float,
               b->series_float};
    Work W;
    rc = run_pipeline(c, spec, B, b->group_members, goff, P, W, 2, nullptr,
                      nullptr);
    const int64_t G = (int64_t)goff.size() - 1, GB = G * P.nb;
    const Tiles T = tiles_of(c, G);
    if (!rc && T.LG != G)  // build_tiles(sel_all): segment = (group, bucket)
      rc = fail(OTSDB_E_DEVICE, "selection segments: %lld of %lld groups",
                (long long)T.LG, (long long)G);
    if (!rc && GB > 0) {
      if (!W.sel_fused)
        hipLaunchKernelGGL(k_dense_to_counts, dim3(blocks_for(GB, 256)),
                           dim3(256), 0, c->stream, GB, (const double*)W.out_val,
                           (const uint8_t*)W.out_emit, counts, emit);
      hipLaunchKernelGGL(k_xsel_range, dim3((unsigned)GB), dim3(256), 0,
                         c->stream, P.nb, goff.back(), T.LG, T.lg_off, T.lg_k,
                         (const uint64_t*)W.keys, (const uint64_t*)W.key_mm,
                         krange,
                         W.sel_fused ? (const uint32_t*)W.key_cnt : nullptr,
                         (const uint32_t*)W.lg_kept, counts, emit);
      HIP_TRY(hipGetLastError());
    }
    if (!rc) {
      HIP_TRY(hipMemsetAsync((char*)c->d_err + 128, 0, 32, c->stream));
      HIP_TRY(hipMemcpyAsync(&c->h_small[0], c->d_err, sizeof(int),
                             hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      if ((int)(c->h_small[0] & 0xFFFFFFFF) & ERR_RATE_TS)
        rc = fail(OTSDB_E_ILLEGAL_STATE,
                  "Next timestamp is supposed to be strictly greater");
    }
    if (!rc) {
      auto& S = c->sel;
      S.active = true;
      S.P = P;
      S.spec = *spec;
      S.W = W;
      S.G = G;
      S.NB = P.nb;
      S.M = goff.back();
      S.median = spec->agg_id == OTSDB_AGG_MEDIAN ? 1 : 0;
      S.next_pass = 0;
      S.more = false;
      S.pool_built = false;
      S.need_pick = false;
      S.key_reads = 0;
      S.passes = 0;
    }
  }
  return rc;
}

namespace {
// the protocol's device words, after the error word (d_err + 128 .. 160):
// per-pass flags, the scans' "broken" mark
uint32_t* xs_flags(otsdb_ctx* c) { return (uint32_t*)((char*)c->d_err + 128); }
uint32_t* xs_broken(otsdb_ctx* c) { return (uint32_t*)((char*)c->d_err + 152); }

int64_t* xs_bnd(otsdb_ctx* c) { return (int64_t*)c->sel.segmem; }
int64_t* xs_off(otsdb_ctx* c) {
  return (int64_t*)c->sel.segmem + (c->sel.G * c->sel.NB + 1);
}
uint32_t* xs_segfill(otsdb_ctx* c) {
  return (uint32_t*)(xs_off(c) + (c->sel.G * c->sel.NB + 1));
}
void* xs_scan_tmp(otsdb_ctx* c) {
  const int64_t GB = c->sel.G * c->sel.NB;
  return (char*)c->sel.segmem + (((size_t)(GB + 1) * 16 + (size_t)GB * 4 + 255) & ~(size_t)255);
}

XPool xs_pool(otsdb_ctx* c) {
  auto& S = c->sel;
  XPool p;
  p.key = (uint64_t*)S.pool;
  p.seg = S.pool ? (int64_t*)((char*)S.pool + (size_t)S.pool_cap * 8) : nullptr;
  p.off = xs_off(c);
  p.fill = xs_segfill(c);
  p.cap = S.pool_cap;
  p.flags = xs_broken(c);
  return p;
}
}  // namespace

otsdb_status otsdb_sel_hist_device(otsdb_ctx* c, int32_t pass,
                                   const int64_t* counts, const uint8_t* emit,
                                   const int64_t* krange, uint32_t* hist_prev,
                                   uint32_t* hist_out, int32_t* more,
                                   void* hip_stream) {
  if (!c || !hist_out || !more) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  auto& S = c->sel;
  if (!S.active) return fail(OTSDB_E_ILLEGAL_STATE, "no selection session");
  if (pass != S.next_pass)
    return fail(OTSDB_E_ILLEGAL_STATE, "pass %d, expected %d", pass, S.next_pass);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  const int64_t G = S.G, NB = S.NB, GB = G * NB;
  const Tiles T = tiles_of(c, G);
  HIP_TRY(hipMemsetAsync(xs_flags(c), 0, 4, st));
  if (pass == 0) {
    if (!counts || !emit || !krange)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null counts / krange");
    if (GB > 0) {
      // the per-segment pool bookkeeping (bounds: the trailing one stays 0,
      // so the scan's last offset is the pool's size)
      size_t tmp = 0;
      HIP_TRY(rocprim::exclusive_scan(nullptr, tmp, (const int64_t*)nullptr,
                                      (int64_t*)nullptr, (int64_t)0,
                                      (size_t)(GB + 1), rocprim::plus<int64_t>(),
                                      st));
      S.scan_tmp = tmp;
      const size_t need =
          (((size_t)(GB + 1) * 16 + (size_t)GB * 4 + 255) & ~(size_t)255) + tmp;
      otsdb_status rc = ensure(&S.segmem, &S.segmem_bytes, need);
      if (rc) return rc;
      HIP_TRY(hipMemsetAsync(xs_bnd(c), 0, (size_t)(GB + 1) * 8, st));
      hipLaunchKernelGGL(k_counts_to_dense, dim3(blocks_for(GB, 256)), dim3(256),
                         0, st, GB, counts, emit, S.W.out_val, S.W.out_emit);
      hipLaunchKernelGGL(k_xsel_init, dim3(blocks_for(GB, 256)), dim3(256), 0,
                         st, GB, counts, emit, krange, S.W.xsel, S.median,
                         S.P.pct, xs_flags(c));
    }
  } else {
    if (!hist_prev) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null hist_prev");
    if (!S.more) return fail(OTSDB_E_ILLEGAL_STATE, "no pass planned");
    if (GB > 0)
      hipLaunchKernelGGL(k_xsel_apply, dim3(blocks_for(GB, 4)), dim3(256), 0,
                         st, GB, T.lg_k, NB, (const uint32_t*)hist_prev,
                         S.W.xsel, xs_flags(c), xs_bnd(c));
    if (pass == 1 && GB > 0) {  // the pool's regions: offsets, size off[GB]
      size_t tmp = S.scan_tmp;
      HIP_TRY(rocprim::exclusive_scan(xs_scan_tmp(c), tmp, (const int64_t*)xs_bnd(c),
                                      xs_off(c), (int64_t)0, (size_t)(GB + 1),
                                      rocprim::plus<int64_t>(), st));
      HIP_TRY(hipMemcpyAsync(&c->h_small[5], xs_off(c) + GB, 8,
                             hipMemcpyDeviceToHost, st));
    }
  }
  HIP_TRY(hipGetLastError());
  // the plan is taken from all-reduced data: every rank reads the same flags
  HIP_TRY(hipMemcpyAsync(&c->h_small[4], xs_flags(c), 4, hipMemcpyDeviceToHost,
                         st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint32_t flags = (uint32_t)(c->h_small[4] & 0xFFFFFFFF);
  const int64_t bound = pass == 1 ? c->h_small[5] : 0;
  if (flags & XS_BROKEN) {
    S.active = false;
    return fail(OTSDB_E_DEVICE, "selection: the ranks' counts and keys disagree");
  }
  S.more = (flags & XS_MORE) != 0;
  S.need_pick = (flags & XS_PICK) != 0;
  S.next_pass = pass + 1;
  *more = S.more ? 1 : 0;
  if (!S.more || GB == 0) return OTSDB_OK;
  HIP_TRY(hipMemsetAsync(hist_out, 0, (size_t)GB * XS_BINS * 4, st));
  if (pass <= 1) {
    int mode = 1;
    if (pass == 1) {  // the candidates: every later pass and the pick read them
      const int64_t cap = bound > 0 ? bound : 1;
      otsdb_status rc = ensure(&S.pool, &S.pool_bytes, (size_t)cap * 16);
      if (rc) return rc;
      S.pool_cap = cap;
      HIP_TRY(hipMemsetAsync((char*)S.pool + (size_t)cap * 8, 0xFF,
                             (size_t)cap * 8, st));  // every slot unfilled
      HIP_TRY(hipMemsetAsync(xs_segfill(c), 0, (size_t)GB * 4, st));
      S.pool_built = true;
      mode |= 2;
    }
    if (T.LGCH > 0)
      hipLaunchKernelGGL(k_xsel_scan, dim3((unsigned)(T.LGCH * NB)), dim3(XS_THREADS), 0,
                         st, mode, NB, S.M, T.LG, T.lg_off, T.lg_k, T.lg_ch0,
                         (const uint64_t*)S.W.keys, (const XSel*)S.W.xsel,
                         hist_out, xs_pool(c), (int64_t*)nullptr);
    ++S.key_reads;
  } else {
    const int64_t nblk = std::min<int64_t>(blocks_for(S.pool_cap, 256), 8192);
    hipLaunchKernelGGL(k_xsel_pool, dim3((unsigned)nblk), dim3(256), 0, st, 1,
                       xs_pool(c), (const XSel*)S.W.xsel, hist_out,
                       (int64_t*)nullptr);
  }
  ++S.passes;
  // no host sync: the caller's collective on the same stream consumes
  // hist_out (RCCL enqueues behind it; a gloo staging copy waits for it)
  HIP_TRY(hipGetLastError());
  return OTSDB_OK;
}

otsdb_status otsdb_sel_hist_wait(otsdb_ctx* c, void* hip_stream) {
  if (!c) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(hip_stream ? (hipStream_t)hip_stream : c->stream));
  return OTSDB_OK;
}

otsdb_status otsdb_sel_pick_device(otsdb_ctx* c, int64_t* picks,
                                   void* hip_stream) {
  if (!c || !picks) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  auto& S = c->sel;
  if (!S.active) return fail(OTSDB_E_ILLEGAL_STATE, "no selection session");
  if (S.next_pass == 0 || S.more)
    return fail(OTSDB_E_ILLEGAL_STATE, "selection not resolved: run its passes");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  const int64_t G = S.G, NB = S.NB, GB = G * NB;
  const Tiles T = tiles_of(c, G);
  if (GB > 0) HIP_TRY(hipMemsetAsync(picks, 0, (size_t)GB * 16, st));
  if (S.need_pick && GB > 0) {
    if (S.pool_built) {
      const int64_t nblk = std::min<int64_t>(blocks_for(S.pool_cap, 256), 8192);
      hipLaunchKernelGGL(k_xsel_pool, dim3((unsigned)nblk), dim3(256), 0, st, 4,
                         xs_pool(c), (const XSel*)S.W.xsel, (uint32_t*)nullptr,
                         picks);
    } else if (T.LGCH > 0) {
      hipLaunchKernelGGL(k_xsel_scan, dim3((unsigned)(T.LGCH * NB)), dim3(XS_THREADS), 0,
                         st, 4, NB, S.M, T.LG, T.lg_off, T.lg_k, T.lg_ch0,
                         (const uint64_t*)S.W.keys, (const XSel*)S.W.xsel,
                         (uint32_t*)nullptr, xs_pool(c), picks);
      ++S.key_reads;
    }
  }
  S.next_pass = -1;  // picked
  HIP_TRY(hipGetLastError());
  return OTSDB_OK;
}

otsdb_status otsdb_sel_finish_device(otsdb_ctx* c, const int64_t* picks,
                                     otsdb_result* out, void* hip_stream) {
  if (!c || !picks || !out) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  auto& S = c->sel;
  if (!S.active) return fail(OTSDB_E_ILLEGAL_STATE, "no selection session");
  if (S.next_pass != -1)
    return fail(OTSDB_E_ILLEGAL_STATE, "otsdb_sel_pick_device first");
  HIP_TRY(hipSetDevice(c->device));
  StreamBinding bind(c, hip_stream);
  const int64_t G = S.G, NB = S.NB, GB = G * NB;
  HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream));
  if (GB > 0)
    hipLaunchKernelGGL(k_xsel_finish, dim3(blocks_for(GB, 256)), dim3(256), 0,
                       c->stream, GB, (const XSel*)S.W.xsel, picks,
                       (const uint8_t*)S.W.out_emit, S.W.out_val, c->d_err,
                       S.median, S.P.pct, (const uint32_t*)xs_broken(c));
  otsdb_status rc = compact(c, S.P, G, S.W.out_val, S.W.out_emit, S.W.counts, out);
  if (!rc) rc = finish(c, G, out);
  S.active = false;
  return rc;
}

otsdb_status otsdb_decode_cells_device(otsdb_ctx* c, const otsdb_cells* cells,
                                       int64_t n_series, int64_t* offsets,
                                       int64_t* ts_ms, int64_t* val,
                                       uint8_t* is_float, int64_t capacity,
                                       void* hip_stream) {
  if (!c || !cells || !offsets) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  if (ts_ms && (!val || !is_float))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null output column");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  return decode_impl(c, cells, n_series, offsets, ts_ms, val, is_float,
                     capacity, st);
}

otsdb_status otsdb_encode_cells_device(otsdb_ctx* c, const otsdb_batch* b,
                                       int64_t* series_rows,
                                       int64_t* series_qbytes,
                                       int64_t* series_vbytes,
                                       const otsdb_cells_out* o,
                                       void* hip_stream) {
  if (!c || !b || !series_rows || !series_qbytes || !series_vbytes)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  if (b->is_float)
    return fail(OTSDB_E_UNSUPPORTED, "per-point value types: use series_float");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  const int64_t S = b->n_series;
  if (S > 0)
    hipLaunchKernelGGL(k_encode, dim3(blocks_for(S, 4)), dim3(256), 0, st, S,
                       b->offsets, b->ts_ms, b->val, b->series_float,
                       o ? 1 : 0, series_rows, series_qbytes, series_vbytes,
                       o ? o->row_series : nullptr, o ? o->row_base_s : nullptr,
                       o ? o->qual_off : nullptr, o ? o->val_off : nullptr,
                       o ? o->qual : nullptr, o ? o->val : nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

otsdb_status otsdb_compact_rows_device(otsdb_ctx* c, const otsdb_raw_rows* raw,
                                       int32_t fix_duplicates,
                                       const otsdb_cells_out* out,
                                       int64_t qual_capacity,
                                       int64_t val_capacity, int64_t* n_out_rows,
                                       void* hip_stream) {
  if (!c || !raw || !n_out_rows) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  return compact_impl(c, raw, fix_duplicates != 0, out, qual_capacity,
                      val_capacity, n_out_rows, nullptr, nullptr, st);
}

otsdb_status otsdb_span_assemble_device(otsdb_ctx* c, const otsdb_cells* cells,
                                        int64_t n_series,
                                        const otsdb_cells_out* out,
                                        int64_t qual_capacity,
                                        int64_t val_capacity,
                                        int64_t* n_out_rows, void* hip_stream) {
  if (!c || !cells || !n_out_rows) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  if (out && !out->row_series)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null output row_series");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  bool identity = true;
  return span_impl(c, cells, n_series, out, qual_capacity, val_capacity,
                   n_out_rows, nullptr, nullptr, &identity, st);
}

otsdb_status otsdb_agg_run_raw_device(otsdb_ctx* c, const otsdb_query_spec* spec,
                                      const otsdb_raw_rows* raw,
                                      int32_t fix_duplicates,
                                      const otsdb_batch* b, otsdb_result* out,
                                      void* hip_stream) {
  if (!c || !spec || !raw || !b || !out)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  StreamBinding bind(c, hip_stream);
  std::vector<int64_t> goff;
  otsdb_status rc = read_goff(c, b, true, goff);
  if (!rc) rc = check_spec(spec);
  if (!rc) rc = run_raw_impl(c, spec, raw, fix_duplicates != 0, b, out, goff);
  return rc;
}

otsdb_status otsdb_agg_run_raw(otsdb_ctx* c, const otsdb_query_spec* spec,
                               const otsdb_raw_rows* raw, int32_t fix_duplicates,
                               const otsdb_batch* b, otsdb_result* out) {
  if (!c || !spec || !raw || !b || !out)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  otsdb_status rc = check_spec(spec);
  if (rc) return rc;
  std::vector<int64_t> goff;
  if ((rc = read_goff(c, b, false, goff))) return rc;
  const int64_t R = raw->n_rows, S = b->n_series, G = b->n_groups;
  if (R < 0 || S < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (!raw->row_series || !raw->row_base_s || !raw->row_col_off ||
      !raw->col_qual_off || !raw->col_val_off)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null raw row array");
  const int64_t M = goff.back();
  for (int64_t r = 0; r < R; ++r)
    if (raw->row_series[r] < 0 || raw->row_series[r] >= S ||
        (r && raw->row_series[r] < raw->row_series[r - 1]))
      return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                  "row_series must be nondecreasing series indices");
  for (int64_t m = 0; m < M; ++m)
    if (b->group_members[m] < 0 || b->group_members[m] >= S)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT, "group member out of range");
  const int64_t C = raw->row_col_off[R];
  const int64_t QB = raw->col_qual_off[C], VB = raw->col_val_off[C];
  const int64_t cap = out->capacity;
  auto carve = [&](char* base) {
    Carve cv{base};
    void* p[14];
    p[0] = cv.take<int64_t>(R + 1);
    p[1] = cv.take<int64_t>(R + 1);
    p[2] = cv.take<int64_t>(R + 1);
    p[3] = cv.take<int64_t>(C + 1);
    p[4] = cv.take<uint8_t>(QB + 16);
    p[5] = cv.take<int64_t>(C + 1);
    p[6] = cv.take<uint8_t>(VB + 16);
    p[7] = raw->col_ts ? cv.take<int64_t>(C + 1) : nullptr;
    p[8] = cv.take<int64_t>(G + 1);
    p[9] = cv.take<int64_t>(M + 1);
    p[10] = cv.take<int64_t>(G + 1);
    p[11] = cv.take<int64_t>(cap + 1);
    p[12] = cv.take<int64_t>(cap + 1);
    p[13] = cv.take<uint8_t>(cap + 1);
    return std::make_pair(cv.off + 256, std::vector<void*>(p, p + 14));
  };
  rc = ensure(&c->raw_stage, &c->raw_stage_cap, carve(nullptr).first);
  if (rc) return rc;
  auto pp = carve((char*)c->raw_stage).second;
  hipStream_t st = c->stream;
  auto h2d = [&](void* d, const void* h, size_t n) -> otsdb_status {
    if (n && h) HIP_TRY(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st));
    return OTSDB_OK;
  };
  if ((rc = h2d(pp[0], raw->row_series, 8 * R)) ||
      (rc = h2d(pp[1], raw->row_base_s, 8 * R)) ||
      (rc = h2d(pp[2], raw->row_col_off, 8 * (R + 1))) ||
      (rc = h2d(pp[3], raw->col_qual_off, 8 * (C + 1))) ||
      (rc = h2d(pp[4], raw->qual, QB)) ||
      (rc = h2d(pp[5], raw->col_val_off, 8 * (C + 1))) ||
      (rc = h2d(pp[6], raw->val, VB)) ||
      (rc = h2d(pp[7], raw->col_ts, 8 * C)) ||
      (rc = h2d(pp[8], b->group_offsets, 8 * (G + 1))) ||
      (rc = h2d(pp[9], b->group_members, 8 * M)))
    return rc;
  otsdb_raw_rows dr{R,
                    (const int64_t*)pp[0],
                    (const int64_t*)pp[1],
                    (const int64_t*)pp[2],
                    (const int64_t*)pp[3],
                    (const uint8_t*)pp[4],
                    (const int64_t*)pp[5],
                    (const uint8_t*)pp[6],
                    (const int64_t*)pp[7]};
  otsdb_batch db = *b;
  db.n_points = 0;
  db.offsets = nullptr;
  db.ts_ms = nullptr;
  db.val = nullptr;
  db.is_float = nullptr;
  db.series_float = nullptr;
  db.group_offsets = (const int64_t*)pp[8];
  db.group_members = (const int64_t*)pp[9];
  otsdb_result dres;
  dres.capacity = cap;
  dres.offsets = (int64_t*)pp[10];
  dres.ts = (int64_t*)pp[11];
  dres.val = (int64_t*)pp[12];
  dres.is_int = (uint8_t*)pp[13];
  c->result_short = false;
  rc = run_raw_impl(c, spec, &dr, fix_duplicates != 0, &db, &dres, goff);
  if (rc == OTSDB_E_CAPACITY && c->result_short)
    return copy_offsets_back(c, out, dres.offsets, G, rc);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out->offsets, dres.offsets, 8 * (G + 1),
                         hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t total = out->offsets[G];
  if (total > 0) {
    HIP_TRY(hipMemcpyAsync(out->ts, dres.ts, 8 * total, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->val, dres.val, 8 * total, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->is_int, dres.is_int, total, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

otsdb_status otsdb_agg_run_cells(otsdb_ctx* c, const otsdb_query_spec* spec,
                                 const otsdb_cells* cells, const otsdb_batch* b,
                                 otsdb_result* out) {
  if (!c || !spec || !cells || !b || !out)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  otsdb_status rc = check_spec(spec);
  if (rc) return rc;
  std::vector<int64_t> goff;
  if ((rc = read_goff(c, b, false, goff))) return rc;
  const int64_t R = cells->n_rows, S = b->n_series, G = b->n_groups;
  if (R < 0 || S < 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (R > 0 && (!cells->row_series || !cells->row_base_s || !cells->qual_off ||
                !cells->val_off || !cells->qual || !cells->val))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null cells array");
  for (int64_t r = 0; r < R; ++r)
    if (cells->row_series[r] < 0 || cells->row_series[r] >= S ||
        (r && cells->row_series[r] < cells->row_series[r - 1]))
      return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                  "row_series must be nondecreasing series indices");
  const int64_t M = goff.back();
  for (int64_t m = 0; m < M; ++m)
    if (b->group_members[m] < 0 || b->group_members[m] >= S)
      return fail(OTSDB_E_ILLEGAL_ARGUMENT, "group member out of range");
  // the pooled byte offsets set the H2D copy sizes: exclusive prefix sums
  // from 0, never decreasing
  if (R > 0 && (cells->qual_off[0] != 0 || cells->val_off[0] != 0))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "qual_off / val_off must start at 0");
  for (int64_t r = 0; r < R; ++r)
    if (cells->qual_off[r + 1] < cells->qual_off[r] ||
        cells->val_off[r + 1] < cells->val_off[r])
      return fail(OTSDB_E_ILLEGAL_ARGUMENT,
                  "qual_off / val_off must be nondecreasing");
  const int64_t QB = R ? cells->qual_off[R] : 0, VB = R ? cells->val_off[R] : 0;
  const int64_t cap = out->capacity;
  auto carve = [&](char* base) {
    Carve cv{base};
    void* p[11];
    p[0] = cv.take<int64_t>(R + 1);
    p[1] = cv.take<int64_t>(R + 1);
    p[2] = cv.take<int64_t>(R + 1);
    p[3] = cv.take<uint8_t>(QB + 32);
    p[4] = cv.take<int64_t>(R + 1);
    p[5] = cv.take<uint8_t>(VB + 32);
    p[6] = cv.take<int64_t>(G + 1);
    p[7] = cv.take<int64_t>(M + 1);
    p[8] = cv.take<int64_t>(G + 1);
    p[9] = cv.take<int64_t>(2 * (cap + 1));
    p[10] = cv.take<uint8_t>(cap + 1);
    return std::make_pair(cv.off + 256, std::vector<void*>(p, p + 11));
  };
  rc = ensure(&c->raw_stage, &c->raw_stage_cap, carve(nullptr).first);
  if (rc) return rc;
  auto pp = carve((char*)c->raw_stage).second;
  hipStream_t st = c->stream;
  auto h2d = [&](void* d, const void* h, size_t n) -> otsdb_status {
    if (n && h) HIP_TRY(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st));
    return OTSDB_OK;
  };
  if ((rc = h2d(pp[0], cells->row_series, 8 * R)) ||
      (rc = h2d(pp[1], cells->row_base_s, 8 * R)) ||
      (rc = h2d(pp[2], cells->qual_off, 8 * (R + 1))) ||
      (rc = h2d(pp[3], cells->qual, QB)) ||
      (rc = h2d(pp[4], cells->val_off, 8 * (R + 1))) ||
      (rc = h2d(pp[5], cells->val, VB)) ||
      (rc = h2d(pp[6], b->group_offsets, 8 * (G + 1))) ||
      (rc = h2d(pp[7], b->group_members, 8 * M)))
    return rc;
  if (R == 0) HIP_TRY(hipMemsetAsync(pp[2], 0, 8, st));
  if (R == 0) HIP_TRY(hipMemsetAsync(pp[4], 0, 8, st));
  otsdb_cells dc{R,
                 (const int64_t*)pp[0],
                 (const int64_t*)pp[1],
                 (const int64_t*)pp[2],
                 (const uint8_t*)pp[3],
                 (const int64_t*)pp[4],
                 (const uint8_t*)pp[5]};
  otsdb_batch db = *b;
  db.n_points = 0;
  db.offsets = nullptr;
  db.ts_ms = nullptr;
  db.val = nullptr;
  db.is_float = nullptr;
  db.series_float = nullptr;
  db.group_offsets = (const int64_t*)pp[6];
  db.group_members = (const int64_t*)pp[7];
  otsdb_result dres;
  dres.capacity = cap;
  dres.offsets = (int64_t*)pp[8];
  dres.ts = (int64_t*)pp[9];
  dres.val = (int64_t*)pp[9] + (cap + 1);
  dres.is_int = (uint8_t*)pp[10];
  c->result_short = false;
  rc = run_cells_impl(c, spec, &dc, &db, &dres, goff);
  if (rc == OTSDB_E_CAPACITY && c->result_short)
    return copy_offsets_back(c, out, dres.offsets, G, rc);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out->offsets, dres.offsets, 8 * (G + 1),
                         hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t total = out->offsets[G];
  if (total > 0) {
    HIP_TRY(hipMemcpyAsync(out->ts, dres.ts, 8 * total, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->val, dres.val, 8 * total, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->is_int, dres.is_int, total, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

otsdb_status otsdb_prof_enable(otsdb_ctx* c, int enable) {
  if (!c) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  c->prof = enable != 0;
  return OTSDB_OK;
}

otsdb_status otsdb_prof_read(otsdb_ctx* c, double* ms, int64_t* launches,
                             int n, int reset) {
  if (!c) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (auto& p : c->ev_pending) {
    float t = 0.f;
    HIP_TRY(hipEventSynchronize(p.second.second));
    HIP_TRY(hipEventElapsedTime(&t, p.second.first, p.second.second));
    c->prof_ms[p.first] += t;
    c->prof_n[p.first] += 1;
  }
  c->ev_pending.clear();
  c->ev_used = 0;
  for (int i = 0; i < n && i < 8; ++i) {
    if (ms) ms[i] = c->prof_ms[i];
    if (launches) launches[i] = c->prof_n[i];
  }
  if (reset)
    for (int i = 0; i < 8; ++i) {
      c->prof_ms[i] = 0;
      c->prof_n[i] = 0;
    }
  return OTSDB_OK;
}

otsdb_status otsdb_ctx_counters(otsdb_ctx* c, int64_t* out, int n) {
  if (!c || (n > 0 && !out)) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  CtxLock lk(c);
  const int64_t v[5] = {c->n_cells_uniform, c->n_cells_general,
                        c->n_cells_uni_miss, c->sel.key_reads, c->sel.passes};
  for (int i = 0; i < n && i < 5; ++i) out[i] = v[i];
  return OTSDB_OK;
}

otsdb_status otsdb_test_set_compact_epoch(otsdb_ctx* c, uint32_t epoch) {
  if (!c || epoch == 0 || epoch >= (1u << 24))
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "epoch %u", epoch);
  CtxLock lk(c);
  // forward only: every granule then carries an epoch below the new one
  // until the wrap (a step back would reuse epochs of live granules)
  if (epoch < c->cmp_epoch)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "epoch %u < %u", epoch, c->cmp_epoch);
  // and by whole ticket-slot rotations: the next call's slot is the one the
  // last call's final block cleared (k_compact1)
  if ((epoch - c->cmp_epoch) % kCmpSlots)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "epoch %u: not %u + k x %d", epoch,
                c->cmp_epoch, kCmpSlots);
  c->cmp_epoch = epoch;
  return OTSDB_OK;
}

otsdb_status otsdb_gen_counts_device(otsdb_ctx* c, const otsdb_gen_spec* g,
                                     int64_t series0, int64_t n_series,
                                     int64_t* counts, void* hip_stream) {
  if (!c || !g || !counts) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  if (g->cadence_ms <= 0) return fail(OTSDB_E_ILLEGAL_ARGUMENT, "cadence");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  GenP gp{g->seed, g->t0_ms, g->duration_ms, g->cadence_ms, g->kind, g->flags};
  if (n_series > 0)
    hipLaunchKernelGGL(k_gen_counts, dim3(blocks_for(n_series, 4)), dim3(256),
                       0, st, gp, series0, n_series, counts);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

otsdb_status otsdb_gen_fill_device(otsdb_ctx* c, const otsdb_gen_spec* g,
                                   int64_t series0, int64_t n_series,
                                   const int64_t* offsets, int64_t* ts_ms,
                                   int64_t* val, void* hip_stream) {
  if (!c || !g || !offsets || !ts_ms || !val)
    return fail(OTSDB_E_ILLEGAL_ARGUMENT, "null");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  GenP gp{g->seed, g->t0_ms, g->duration_ms, g->cadence_ms, g->kind, g->flags};
  if (n_series > 0)
    hipLaunchKernelGGL(k_gen_fill, dim3(blocks_for(n_series, 4)), dim3(256),
                       0, st, gp, series0, n_series, offsets, ts_ms, val);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));
  return OTSDB_OK;
}

}  // extern "C"
