// ds_tu.hip — the kernels templated on one downsampling monoid, compiled once
// per monoid with -DOTSDB_DS_MONOID=<n> (opentsdb_amd/build.py runs the
// thirteen compilations in parallel; the engine links them).  Non-template
// kernels are compiled only in engine.hip (OTSDB_DS_TU hides them here).
#define OTSDB_DS_TU 1
// fused cells kernel shape (tuning builds override)
#ifndef OTSDB_CELLS_K
#define OTSDB_CELLS_K 6
#endif
#ifndef OTSDB_CELLS_WAVES
#define OTSDB_CELLS_WAVES 1
#endif
#ifndef OTSDB_RING_NT  // tuning builds: 2 = non-temporal row stores
#define OTSDB_RING_NT 0
#endif
#ifndef OTSDB_DS_PART
#define OTSDB_DS_PART 0  // 0: launch_ds kernels, 1: the cells fold
#endif
// k_bucketize_k ring shape (tuning builds override)
#ifndef OTSDB_RING_WAVES
#define OTSDB_RING_WAVES 1
#endif
#ifndef OTSDB_RING_WIN
#define OTSDB_RING_WIN 256
#endif
#ifndef OTSDB_RING_FL
#define OTSDB_RING_FL 64
#endif
// rate-fused k_bucketize_k shape (tuning builds override)
#ifndef OTSDB_RATE_K
#define OTSDB_RATE_K 8
#endif
#ifndef OTSDB_RATE_WAVES
#define OTSDB_RATE_WAVES 4
#endif
#ifndef OTSDB_RATE_WIN
#define OTSDB_RATE_WIN 1024
#endif
#ifndef OTSDB_RATE_FL
#define OTSDB_RATE_FL 512
#endif
#ifndef OTSDB_PREP_TPB  // threads per block of the latency-bound prep kernels
#define OTSDB_PREP_TPB 64  // (k_prep, k_fold_prep): 4x the CUs of 256-thread
#endif                     // blocks on small queries (C1 prep 33 -> 27 us)
#ifndef OTSDB_RATE_PF
#define OTSDB_RATE_PF 0
#endif
#include "kernels.hip"
#include "decode.hip"
#include "fold.hip"
#if OTSDB_DS_PART == 1
#include "cellfold.hip"
#endif

namespace otsdb {

namespace {
inline unsigned ds_blocks(int64_t n, int per) {
  return (unsigned)((n + per - 1) / per);
}
}  // namespace

#if OTSDB_DS_PART == 1
// the cells fold: prep + k_fold<M, A, 8, 1> x every aggregator
template <class M>
bool launch_cells(DsKernel k, const DsLaunch& a) {
  const int64_t S = a.B.S;
  switch (k) {
    case DS_CELLS_PREP:
      if (S > 0)
        hipLaunchKernelGGL(k_cells_prep<M>, dim3(ds_blocks(S, OTSDB_PREP_TPB)),
                           dim3(OTSDB_PREP_TPB), 0, a.st, a.P, a.cf, S, a.SM,
                           a.err);
      OTSDB_DBG(a.st, "k_cells_prep");
      return true;
    case DS_CELLS_FOLD_PREP:
      if (a.NW > 1 && S > 0)
        hipLaunchKernelGGL(k_cells_fold_prep<M>,
                           dim3(ds_blocks(S * (a.NW - 1), OTSDB_PREP_TPB)),
                           dim3(OTSDB_PREP_TPB), 0,
                           a.st, a.P, a.cf, S, a.SM, a.NW, a.WB, a.wc, a.err);
      OTSDB_DBG(a.st, "k_cells_fold_prep");
      return true;
    case DS_CELLS_FOLD4:
      return with_monoid(a.agg_id, [&](auto tag) {
        using A = decltype(tag);
        hipLaunchKernelGGL((k_fold<M, A, 8, 4>),
                           dim3((unsigned)(a.n_tiles * a.NW)), dim3(FOLD_THREADS),
                           (unsigned)fold_lds_bytes<A>(a.P),
                           a.st, a.P, a.B, a.SM, a.n_tiles, a.tg, a.tm0,
                           a.tm1, a.single, a.members, a.wc, a.NW, a.partial,
                           a.tile_emit, a.out_val, a.out_emit, a.err,
                           a.always_partial, a.cf);
        OTSDB_DBG(a.st, "k_fold<cells, qw 4>");
      });
    case DS_CELLS_UNIFORM:
      if (S > 0)
        hipLaunchKernelGGL(k_cells_uniform<M>, dim3(ds_blocks(S, 4)), dim3(256),
                           0, a.st, a.cf, S, a.SM);
      OTSDB_DBG(a.st, "k_cells_uniform");
      return true;
    case DS_CELLS_FOLD4U:
      return with_monoid(a.agg_id, [&](auto tag) {
        using A = decltype(tag);
        hipLaunchKernelGGL((k_fold<M, A, 8, 12>),
                           dim3((unsigned)(a.n_tiles * a.NW)), dim3(FOLD_THREADS),
                           (unsigned)fold_lds_bytes<A>(a.P),
                           a.st, a.P, a.B, a.SM, a.n_tiles, a.tg, a.tm0,
                           a.tm1, a.single, a.members, a.wc, a.NW, a.partial,
                           a.tile_emit, a.out_val, a.out_emit, a.err,
                           a.always_partial, a.cf);
        OTSDB_DBG(a.st, "k_fold<cells, qw 4, uniform>");
      });
    case DS_CELLS_FOLD2U:
      return with_monoid(a.agg_id, [&](auto tag) {
        using A = decltype(tag);
        hipLaunchKernelGGL((k_fold<M, A, 8, 10>),
                           dim3((unsigned)(a.n_tiles * a.NW)), dim3(FOLD_THREADS),
                           (unsigned)fold_lds_bytes<A>(a.P),
                           a.st, a.P, a.B, a.SM, a.n_tiles, a.tg, a.tm0,
                           a.tm1, a.single, a.members, a.wc, a.NW, a.partial,
                           a.tile_emit, a.out_val, a.out_emit, a.err,
                           a.always_partial, a.cf);
        OTSDB_DBG(a.st, "k_fold<cells, qw 2, uniform>");
      });
    case DS_CELLS_FOLD2:
      return with_monoid(a.agg_id, [&](auto tag) {
        using A = decltype(tag);
        hipLaunchKernelGGL((k_fold<M, A, 8, 2>),
                           dim3((unsigned)(a.n_tiles * a.NW)), dim3(FOLD_THREADS),
                           (unsigned)fold_lds_bytes<A>(a.P),
                           a.st, a.P, a.B, a.SM, a.n_tiles, a.tg, a.tm0,
                           a.tm1, a.single, a.members, a.wc, a.NW, a.partial,
                           a.tile_emit, a.out_val, a.out_emit, a.err,
                           a.always_partial, a.cf);
        OTSDB_DBG(a.st, "k_fold<cells, qw 2>");
      });
    default:
      return false;
  }
}
#define OTSDB_LAUNCH launch_cells
#else
#define OTSDB_LAUNCH launch_ds
template <class M>
bool launch_ds(DsKernel k, const DsLaunch& a) {
  const int64_t S = a.B.S;
  switch (k) {
    case DS_PREP:
      hipLaunchKernelGGL(k_prep<M>, dim3(ds_blocks(S, OTSDB_PREP_TPB)),
                         dim3(OTSDB_PREP_TPB), 0, a.st, a.P, a.B, a.SM, a.err);
      OTSDB_DBG(a.st, "k_prep");
      return true;
    case DS_RING:  // production: LDS ring sink, sentinel rows, DPP scan
      hipLaunchKernelGGL((k_bucketize_k<M, 8, 0, OTSDB_RING_NT, OTSDB_RING_WAVES, 0, 1,
                                        OTSDB_RING_WIN, OTSDB_RING_FL>),
                         dim3(ds_blocks(S, 4)), dim3(256), 0, a.st, a.P, a.B,
                         a.SM, a.R);
      return true;
    case DS_RATE:
      // launch-bounded to 128 VGPRs (4 waves / SIMD instead of the 3 its 140
      // VGPRs allow; 8 cold spills): C4 bucketize 14.1 -> 13.3 ms
      hipLaunchKernelGGL((k_bucketize_k<M, OTSDB_RATE_K, OTSDB_RATE_PF, OTSDB_RING_NT,
                                        OTSDB_RATE_WAVES, 0, 1, OTSDB_RATE_WIN,
                                        OTSDB_RATE_FL, 1>),
                         dim3(ds_blocks(S, 4)), dim3(256), 0, a.st, a.P, a.B,
                         a.SM, a.R);
      return true;
    case DS_CELLS:
      hipLaunchKernelGGL((k_bucketize_cells<M, OTSDB_CELLS_K, OTSDB_CELLS_WAVES>),
                         dim3(ds_blocks(S, 4)),
                         dim3(256), 0, a.st, a.P, a.cells, a.series_row, S,
                         a.SM, a.R, a.err);
      return true;
    case DS_FOLD_PREP:
      if (a.NW > 1 && S > 0)
        hipLaunchKernelGGL(k_fold_prep<M>,
                           dim3(ds_blocks(S * (a.NW - 1), OTSDB_PREP_TPB)),
                           dim3(OTSDB_PREP_TPB), 0,
                           a.st, a.P, a.B, a.SM, a.NW, a.WB, a.wc);
      return true;
    case DS_PREP_FOLD:
      if (a.NW > 1 && S > 0)
        hipLaunchKernelGGL(k_prep_fold<M>,
                           dim3(ds_blocks(S * (a.NW - 1), OTSDB_PREP_TPB)),
                           dim3(OTSDB_PREP_TPB), 0, a.st, a.P, a.B, a.SM,
                           a.err, a.NW, a.WB, a.wc);
      return true;
    case DS_FOLD:
      return with_monoid(a.agg_id, [&](auto tag) {
        using A = decltype(tag);
        // member contexts preloaded into LDS only while the workgroup stays
        // within 40 KB (4 a CU: C2's 2,017-bucket windows leave room for 10)
        Params P = a.P;
        size_t lds = fold_lds_bytes<A>(P);
        if (P.fold_ctx > 0 && lds + (size_t)P.fold_ctx * sizeof(FoldMember) <=
                                  kFoldDynBudget)
          lds += (size_t)P.fold_ctx * sizeof(FoldMember);
        else
          P.fold_ctx = 0;
        hipLaunchKernelGGL((k_fold<M, A, 8>),
                           dim3((unsigned)(a.n_tiles * a.NW)), dim3(FOLD_THREADS),
                           (unsigned)lds,
                           a.st, P, a.B, a.SM, a.n_tiles, a.tg, a.tm0,
                           a.tm1, a.single, a.members, a.wc, a.NW, a.partial,
                           a.tile_emit, a.out_val, a.out_emit, a.err,
                           a.always_partial, a.cf);
        OTSDB_DBG(a.st, "k_fold");
      });
  }
  return false;
}
#endif

#ifndef OTSDB_DS_MONOID
#error "compile with -DOTSDB_DS_MONOID=<0..12>"
#endif
#if OTSDB_DS_MONOID == 0
template bool OTSDB_LAUNCH<MSum<0>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 1
template bool OTSDB_LAUNCH<MSum<1>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 2
template bool OTSDB_LAUNCH<MSum<2>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 3
template bool OTSDB_LAUNCH<MSum<3>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 4
template bool OTSDB_LAUNCH<MMinMax<false>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 5
template bool OTSDB_LAUNCH<MMinMax<true>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 6
template bool OTSDB_LAUNCH<MDev>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 7
template bool OTSDB_LAUNCH<MFirstLast<false>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 8
template bool OTSDB_LAUNCH<MFirstLast<true>>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 9
template bool OTSDB_LAUNCH<MMult>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 10
template bool OTSDB_LAUNCH<MDiff>(DsKernel, const DsLaunch&);
#elif OTSDB_DS_MONOID == 11
template bool OTSDB_LAUNCH<MNone>(DsKernel, const DsLaunch&);
#endif

}  // namespace otsdb
