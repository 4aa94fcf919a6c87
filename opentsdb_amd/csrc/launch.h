// launch.h — the host-side record through which the engine launches the
// kernels templated on the DOWNSAMPLING monoid.  Those kernels (k_prep, the
// ring k_bucketize_k, the rate-fused one, k_bucketize_cells, k_fold_prep and
// the ordered group fold k_fold x every aggregator) are compiled in one
// translation unit per downsampling monoid (ds_tu.hip), in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dispatch.h"
#include "kernels.h"

namespace otsdb {

// compacted columns of a query (otsdb_cells, device pointers)
struct CellsDev {
  int64_t R;
  const int64_t* row_series;
  const int64_t* row_base_s;
  const int64_t* qual_off;
  const uint8_t* qual;
  const int64_t* val_off;
  const uint8_t* val;
};

// per (series, inner window boundary j = 1 .. NW-1) of the ordered fold,
// window start W = j*WB (fold.hip)
struct WinCtx {
  int64_t bnd;      // first point with ts >= bucket_ts(W)
  int64_t prev_ts;  // last real bucket before W: its timestamp (INT64_MIN:
  double prev_val;  //   none) and downsampled value
  int64_t next_ts;  // first real bucket at or after W (INT64_MIN: none)
  double next_val;
};

// A cells fold (k_cells_prep -> k_fold<..., CELLS = 1>, cellfold.hip): the
// compacted columns and what the prep derives per series.  A series' points
// are numbered by qualifier: point p's qualifier sits at byte
// qual_off[first row] + qw * p (rows are contiguous in the pools).
struct CellsFold {
  CellsDev C;
  const int64_t* series_row;  // [S + 1] first row of each series
  int64_t* rlo;               // row holding point lo
  int64_t* vlo;               // byte offset in C.val of point lo's value
  uint8_t* qw;                // qualifier width of the series (2 / 4)
  uint8_t* vl0;               // value length of point lo (first guess)
  // grids of several fold windows: the stream's cursor at each inner window
  // boundary (per (series, boundary), k_cells_fold_prep)
  int64_t* wrlo;
  int64_t* wvlo;
  uint8_t* wvl0;
  int* wide;                  // k_cells_prep: bit 0 / 1 = some kept series
                              // has 4- / 2-byte qualifiers (one width: the
                              // fold with that width fixed runs); bit 2
                              // (k_cells_uniform): some kept series is not
                              // uniform
  // k_cells_uniform: the series' one flags nibble (value length and type)
  // when every row of it is uniform — one qualifier width, value bytes
  // adding up to points x length (+ the meta byte of a multi-point column)
  // — else 0xFF
  uint8_t* uf;
};

// buckets per fold window: the aggregator states of a window live in LDS
// (2,048 x 24-byte dev / diff states + ring + marks: 57 KB, within the
// 64 KB a workgroup may hold; the states are dynamic LDS sized for the
// grid, fold_lds_bytes)
#ifndef OTSDB_FOLD_WB_MAX  // tuning builds: a smaller window cap
#define OTSDB_FOLD_WB_MAX 2048
#endif
template <class A>
constexpr int fold_wb() {
  return sizeof(A) <= 24 ? OTSDB_FOLD_WB_MAX
                         : (OTSDB_FOLD_WB_MAX < 1024 ? OTSDB_FOLD_WB_MAX : 1024);
}

// the fold's window: P.fold_wb buckets when the engine narrowed it (more
// workgroups for queries with few tiles), else fold_wb<A>()
template <class A>
__host__ __device__ constexpr int64_t fold_window(const Params& P) {
  return P.fold_wb > 0 ? (int64_t)P.fold_wb : (int64_t)fold_wb<A>();
}
// dynamic LDS of k_fold: the states of min(window, nb) buckets, then as
// many emit flags (16-byte aligned pieces)
template <class A>
__host__ __device__ constexpr int64_t fold_cap(const Params& P) {
  return P.nb < fold_window<A>(P) ? P.nb : fold_window<A>(P);
}
template <class A>
__host__ __device__ constexpr size_t fold_lds_states(const Params& P) {
  return (((size_t)fold_cap<A>(P) * sizeof(A)) + 15) & ~(size_t)15;
}
template <class A>
constexpr size_t fold_lds_bytes(const Params& P) {
  return fold_lds_states<A>(P) + ((((size_t)fold_cap<A>(P)) + 15) & ~(size_t)15);
}

enum DsKernel {
  DS_PREP,       // k_prep: bounds, seek, point past the window
  DS_RING,       // k_bucketize_k, LDS ring sink -> sentinel series rows
  DS_RATE,       // k_bucketize_k with RateSpan fused into the ring flush
  DS_CELLS,      // k_bucketize_cells: decode fused into the downsample
  DS_FOLD_PREP,  // k_fold_prep: window boundaries of the ordered fold
  DS_FOLD,       // k_fold: downsample + contribution + ordered aggregator
  DS_CELLS_PREP, // k_cells_prep: bounds / cursors of a cells fold
  DS_CELLS_FOLD, // (unused: a batch whose kept series mix qualifier widths
                 // is rewritten with one width, k_requal)
  DS_CELLS_FOLD_PREP, // k_cells_fold_prep: window boundaries of a cells fold
  DS_CELLS_FOLD2, // the cells fold of a batch whose kept series all have
                  // 2-byte qualifiers (the width a compile-time constant)
  DS_CELLS_FOLD4, // ... all 4-byte ones
  DS_PREP_FOLD,   // k_prep_fold: k_prep + k_fold_prep in one launch
  DS_CELLS_UNIFORM, // k_cells_uniform: which kept series are uniform
  DS_CELLS_FOLD2U,  // the uniform cells fold (fold_member_cells_u), 2-byte
  DS_CELLS_FOLD4U   // ... 4-byte qualifiers
};

struct DsLaunch {
  hipStream_t st;
  Params P;
  BatchDev B;
  SeriesMeta SM;
  Rows R;
  int* err;
  // DS_CELLS
  CellsDev cells;
  const int64_t* series_row;
  // DS_FOLD_PREP / DS_FOLD
  WinCtx* wc;
  int64_t NW, WB;
  int64_t n_tiles;
  const int64_t *tg, *tm0, *tm1;
  const uint8_t* single;
  const int64_t* members;
  Packed* partial;
  uint8_t* tile_emit;
  double* out_val;
  uint8_t* out_emit;
  int always_partial;
  int agg_id;
  // DS_CELLS_PREP / DS_CELLS_FOLD
  CellsFold cf;
};

// Debug builds (-DOTSDB_DEBUG_SYNC): every launch reports itself and waits
// for the device, so a kernel that does not finish names itself.
#ifdef OTSDB_DEBUG_SYNC
#include <cstdio>
#define OTSDB_DBG(st, what)                                              \
  do {                                                                   \
    fprintf(stderr, "[otsdb] %s ...\n", what);                          \
    fflush(stderr);                                                      \
    hipError_t e_ = hipStreamSynchronize(st);                            \
    fprintf(stderr, "[otsdb] %s done (%s)\n", what, hipGetErrorString(e_)); \
    fflush(stderr);                                                      \
  } while (0)
#else
#define OTSDB_DBG(st, what) \
  do {                      \
  } while (0)
#endif

// Defined (explicitly instantiated) in ds_tu.hip for every downsampling
// monoid; false when the kernel does not exist for (M, agg).
template <class M>
bool launch_ds(DsKernel k, const DsLaunch& a);
// the cells fold kernels (ds_tu.hip part 1, their own translation units)
template <class M>
bool launch_cells(DsKernel k, const DsLaunch& a);

}  // namespace otsdb
