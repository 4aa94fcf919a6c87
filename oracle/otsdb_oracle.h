/*
 * otsdb_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of OpenTSDB's query-time aggregation path (the checker the
 * GPU engine is compared against).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product (libotsdb_agg.so) never
 * links or calls it.
 *
 * Parity pinning: the Java reference cannot be built or run in this image (no
 * JVM, dependency jars absent — SURVEY.md §8c), so this restatement is pinned
 * by known-answer vectors transcribed from the reference's own JUnit tests
 * (tests/golden/kat_*.json, tests/test_oracle_kat.py).  The double-path
 * percentile arithmetic of commons-math3 3.4.1 is not covered by any
 * reference test ("parity unpinned" for that corner).
 */
#ifndef OTSDB_ORACLE_H
#define OTSDB_ORACLE_H
#include <stdint.h>
#include "../include/otsdb_agg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One emitted data point. */
typedef struct {
  int64_t ts;
  int64_t bits;    /* long value, or IEEE double bits */
  int32_t is_int;
  int32_t _pad;
} or_point;

/* Full group-by over a host batch (Query.run() semantics, no serializer
 * clipping).  Writes up to `cap` points into `out`, group boundaries into
 * out_offsets[G+1].  Returns otsdb_status; *needed = total points produced
 * (also when cap is too small -> OTSDB_E_CAPACITY).  err (may be NULL)
 * receives a message.                                                       */
int or_group_by(const otsdb_query_spec* spec, const otsdb_batch* batch,
                or_point* out, int64_t cap, int64_t* out_offsets,
                int64_t* needed, char* err, int errlen);

/* Iterates one view chain over one series without an AggregationIterator,
 * the way the reference's unit tests drive Downsampler / FillingDownsampler /
 * RateSpan directly.  chain: ds_interval_ms > 0 -> (Filling)Downsampler;
 * rate -> RateSpan on top.  If do_seek, seek(seek_ts) is called first.      */
/* test-only: scales the junk first rate (comparator mutation tests) */
void or_test_set_junk_rate_scale(double s);

int or_view_stream(const otsdb_query_spec* spec, int do_seek, int64_t seek_ts,
                   int64_t n, const int64_t* ts, const int64_t* bits,
                   const uint8_t* is_float, or_point* out, int64_t cap,
                   int64_t* needed, char* err, int errlen);

/* Aggregator.runDouble / runLong over a plain sequence. */
int or_run_double(int32_t agg_id, const double* v, int64_t n, double* out,
                  char* err, int errlen);
int or_run_long(int32_t agg_id, const int64_t* v, int64_t n, int64_t* out,
                char* err, int errlen);

/* RowSeq decode of one compacted column (qualifier bytes + value bytes) for
 * a row with base time `base_time_s`: RowSeq.Iterator semantics
 * (RowSeq.java:552-643).  Writes up to cap points.                          */
int or_decode_row(const uint8_t* qual, int64_t qlen, const uint8_t* vals,
                  int64_t vlen, int64_t base_time_s, or_point* out,
                  int64_t cap, int64_t* needed, char* err, int errlen);

/* Query-time compaction of one storage row (CompactionQueue.Compaction
 * .compact): columns [0, ncol) with qualifier / value byte ranges and HBase
 * timestamps (NULL: column order).  Output: one compacted column (meta byte
 * on multi-value columns); *out_qlen = 0 when the row holds no data point. */
int or_compact_row(int64_t ncol, const int64_t* col_qoff, const uint8_t* qual,
                   const int64_t* col_voff, const uint8_t* val,
                   const int64_t* col_ts, int fix_duplicates,
                   uint8_t* out_q, int64_t qcap, uint8_t* out_v, int64_t vcap,
                   int64_t* out_qlen, int64_t* out_vlen, char* err,
                   int errlen);

/* Span assembly (Span.addRow + RowSeq.addRow + checkRowOrder) of one
 * series' compacted rows in arrival order; output rows in iteration order. */
int or_span_assemble(int64_t R, const int64_t* row_base_s,
                     const int64_t* qoff, const uint8_t* qual,
                     const int64_t* voff, const uint8_t* val,
                     int64_t* out_rows, int64_t* out_base, int64_t* out_qoff,
                     uint8_t* out_q, int64_t* out_voff, uint8_t* out_v,
                     char* err, int errlen);

/* Synthetic generator (SURVEY §8d as restated in DESIGN.md §Workload). */
int64_t or_gen_count(const otsdb_gen_spec* g, int64_t s);
int64_t or_gen_fill(const otsdb_gen_spec* g, int64_t s, int64_t* ts,
                    int64_t* val);

#ifdef __cplusplus
}
#endif
#endif
