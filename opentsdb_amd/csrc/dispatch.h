// dispatch.h — aggregator id -> reduction state type (monoids.h), shared by
// the engine and the per-downsampler translation units.
#pragma once
#include "../../include/otsdb_agg.h"
#include "monoids.h"

namespace otsdb {

// Calls f(M{}) with the reduction state type of aggregator `agg`
// (Aggregators.java:175-203 registry; the interpolation method is separate).
template <class F>
bool with_monoid(int agg, F&& f) {
  switch (agg) {
    case OTSDB_AGG_SUM:
    case OTSDB_AGG_PFSUM:
    case OTSDB_AGG_ZIMSUM: f(MSum<0>{}); return true;
    case OTSDB_AGG_AVG: f(MSum<1>{}); return true;
    case OTSDB_AGG_SQUARESUM: f(MSum<2>{}); return true;
    case OTSDB_AGG_COUNT: f(MSum<3>{}); return true;
    case OTSDB_AGG_MIN:
    case OTSDB_AGG_MIMMIN: f(MMinMax<false>{}); return true;
    case OTSDB_AGG_MAX:
    case OTSDB_AGG_MIMMAX: f(MMinMax<true>{}); return true;
    case OTSDB_AGG_DEV: f(MDev{}); return true;
    case OTSDB_AGG_FIRST: f(MFirstLast<false>{}); return true;
    case OTSDB_AGG_LAST: f(MFirstLast<true>{}); return true;
    case OTSDB_AGG_MULT: f(MMult{}); return true;
    case OTSDB_AGG_DIFF: f(MDiff{}); return true;
    case OTSDB_AGG_NONE: f(MNone{}); return true;
    default: return false;
  }
}

}  // namespace otsdb
