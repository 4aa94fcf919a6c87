/*
 * otsdb_agg_jni.c — JNI shim between net.opentsdb.core.GpuAggregation
 * (integration/java) and libotsdb_agg.so (include/otsdb_agg.h).
 *
 * Built only where a JDK is installed (jni.h; see the Makefile next to this
 * file) — this repository's image has none.  The shim holds no state: every
 * native call maps Java arrays (GetPrimitiveArrayCritical: no copies, the
 * call is synchronous and makes no JNI calls while they are held) onto the
 * C-ABI structs, calls the engine and maps the status onto the exception
 * the reference path throws (otsdb_status, include/otsdb_agg.h:39-61).
 */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "otsdb_agg.h"

/* GpuAggregation.SPEC_* (packed otsdb_query_spec) */
enum {
  SPEC_START_MS, SPEC_END_MS, SPEC_QSTART_MS, SPEC_QEND_MS, SPEC_AGG,
  SPEC_INTERP, SPEC_DS_INTERVAL, SPEC_DS_AGG, SPEC_FILL, SPEC_RUN_ALL,
  SPEC_CALENDAR, SPEC_RATE, SPEC_COUNTER, SPEC_DROP_RESETS, SPEC_COUNTER_MAX,
  SPEC_RESET_VALUE, SPEC_LEN
};

static void throw_status(JNIEnv* env, otsdb_status st) {
  const char* cls;
  switch (st) {
    case OTSDB_E_ILLEGAL_DATA: cls = "net/opentsdb/core/IllegalDataException"; break;
    case OTSDB_E_ILLEGAL_STATE: cls = "java/lang/IllegalStateException"; break;
    case OTSDB_E_ILLEGAL_ARGUMENT: cls = "java/lang/IllegalArgumentException"; break;
    case OTSDB_E_NO_SUCH_ELEMENT: cls = "java/util/NoSuchElementException"; break;
    default: cls = "java/lang/RuntimeException"; break;
  }
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, otsdb_last_error());
}

JNIEXPORT jlong JNICALL Java_net_opentsdb_core_GpuAggregation_nativeCtxCreate(
    JNIEnv* env, jclass cls, jint device) {
  (void)cls;
  otsdb_ctx* ctx = NULL;
  otsdb_status st = otsdb_ctx_create(device, &ctx);
  if (st != OTSDB_OK) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_net_opentsdb_core_GpuAggregation_nativeCtxDestroy(
    JNIEnv* env, jclass cls, jlong ctx) {
  (void)env;
  (void)cls;
  otsdb_ctx_destroy((otsdb_ctx*)(intptr_t)ctx);
}

/* Aggregator.toString() -> otsdb_agg_id (otsdb_agg_name is toString) */
JNIEXPORT jint JNICALL Java_net_opentsdb_core_GpuAggregation_nativeAggId(
    JNIEnv* env, jclass cls, jstring name) {
  (void)cls;
  const char* s = (*env)->GetStringUTFChars(env, name, NULL);
  if (!s) return -1;
  jint id = -1;
  for (int32_t i = 0; i < OTSDB_AGG_COUNT_IDS; ++i)
    if (strcmp(otsdb_agg_name(i), s) == 0) {
      id = i;
      break;
    }
  (*env)->ReleaseStringUTFChars(env, name, s);
  return id;
}

typedef struct {
  jarray arr;
  void* p;
} pinned;

static void* pin(JNIEnv* env, jarray a, pinned* slot) {
  slot->arr = a;
  slot->p = a ? (*env)->GetPrimitiveArrayCritical(env, a, NULL) : NULL;
  return slot->p;
}

static void unpin(JNIEnv* env, pinned* slot, int n, int commit_from) {
  /* inputs: JNI_ABORT (nothing to copy back); outputs: 0 */
  for (int i = n - 1; i >= 0; --i)
    if (slot[i].p)
      (*env)->ReleasePrimitiveArrayCritical(env, slot[i].arr, slot[i].p,
                                            i >= commit_from ? 0 : JNI_ABORT);
}

JNIEXPORT jint JNICALL Java_net_opentsdb_core_GpuAggregation_nativeRunCells(
    JNIEnv* env, jclass cls, jlong ctx, jlongArray jspec, jlongArray jcal,
    jint n_series, jlongArray jrow_series, jlongArray jrow_base,
    jlongArray jqual_off, jbyteArray jqual, jlongArray jval_off,
    jbyteArray jval, jlongArray jgoff, jlongArray jgmem, jlongArray jooff,
    jlongArray jots, jlongArray joval, jbyteArray joisint) {
  (void)cls;
  if ((*env)->GetArrayLength(env, jspec) < SPEC_LEN) {
    throw_status(env, OTSDB_E_ILLEGAL_ARGUMENT);
    return OTSDB_E_ILLEGAL_ARGUMENT;
  }
  jlong spec_v[SPEC_LEN];
  (*env)->GetLongArrayRegion(env, jspec, 0, SPEC_LEN, spec_v);
  otsdb_query_spec s;
  memset(&s, 0, sizeof(s));
  s.start_ms = spec_v[SPEC_START_MS];
  s.end_ms = spec_v[SPEC_END_MS];
  s.query_start_ms = spec_v[SPEC_QSTART_MS];
  s.query_end_ms = spec_v[SPEC_QEND_MS];
  s.agg_id = (int32_t)spec_v[SPEC_AGG];
  s.interp = (int32_t)spec_v[SPEC_INTERP];
  s.ds_interval_ms = spec_v[SPEC_DS_INTERVAL];
  s.ds_agg_id = (int32_t)spec_v[SPEC_DS_AGG];
  s.fill = (int32_t)spec_v[SPEC_FILL];
  s.run_all = (int32_t)spec_v[SPEC_RUN_ALL];
  s.use_calendar = (int32_t)spec_v[SPEC_CALENDAR];
  s.rate = (int32_t)spec_v[SPEC_RATE];
  s.counter = (int32_t)spec_v[SPEC_COUNTER];
  s.drop_resets = (int32_t)spec_v[SPEC_DROP_RESETS];
  s.counter_max = spec_v[SPEC_COUNTER_MAX];
  s.reset_value = spec_v[SPEC_RESET_VALUE];
  const jsize n_rows = (*env)->GetArrayLength(env, jrow_series);
  const jsize n_groups = (*env)->GetArrayLength(env, jgoff) - 1;
  const jsize cap = (*env)->GetArrayLength(env, jots);
  const jsize n_cal = jcal ? (*env)->GetArrayLength(env, jcal) : 0;

  /* inputs first (released with JNI_ABORT), outputs from index 9 on */
  pinned pn[13];
  memset(pn, 0, sizeof(pn));
  s.cal_edges = (const int64_t*)pin(env, jcal, &pn[0]);
  s.n_cal_edges = n_cal;
  otsdb_cells c;
  c.n_rows = n_rows;
  c.row_series = (const int64_t*)pin(env, jrow_series, &pn[1]);
  c.row_base_s = (const int64_t*)pin(env, jrow_base, &pn[2]);
  c.qual_off = (const int64_t*)pin(env, jqual_off, &pn[3]);
  c.qual = (const uint8_t*)pin(env, jqual, &pn[4]);
  c.val_off = (const int64_t*)pin(env, jval_off, &pn[5]);
  c.val = (const uint8_t*)pin(env, jval, &pn[6]);
  otsdb_batch b;
  memset(&b, 0, sizeof(b));
  b.n_series = n_series;
  b.n_groups = n_groups;
  b.group_offsets = (const int64_t*)pin(env, jgoff, &pn[7]);
  b.group_members = (const int64_t*)pin(env, jgmem, &pn[8]);
  otsdb_result r;
  r.capacity = cap;
  r.offsets = (int64_t*)pin(env, jooff, &pn[9]);
  r.ts = (int64_t*)pin(env, jots, &pn[10]);
  r.val = (int64_t*)pin(env, joval, &pn[11]);
  r.is_int = (uint8_t*)pin(env, joisint, &pn[12]);
  otsdb_status st = OTSDB_E_DEVICE;
  if (r.offsets && r.ts && r.val && r.is_int && b.group_offsets)
    st = otsdb_agg_run_cells((otsdb_ctx*)(intptr_t)ctx, &s, &c, &b, &r);
  unpin(env, pn, 13, 9);
  /* CAPACITY and UNSUPPORTED go back to Java (retry larger / keep the Java
   * iterators); the rest are the reference's exceptions */
  if (st != OTSDB_OK && st != OTSDB_E_CAPACITY && st != OTSDB_E_UNSUPPORTED)
    throw_status(env, st);
  return st;
}
