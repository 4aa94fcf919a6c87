/*
 * otsdb_agg_jni.c — JNI shim between net.opentsdb.core.GpuAggregation
 * (integration/java) and libotsdb_agg.so (include/otsdb_agg.h).
 *
 * Built only where a JDK is installed (jni.h; see the Makefile next to this
 * file) — this repository's image has none.  The shim holds no state: every
 * native call copies the Java arrays into native buffers (nothing stays
 * pinned while the GPU works) and maps them onto the C-ABI structs, calls the engine and maps the status onto the exception
 * the reference path throws (otsdb_status, include/otsdb_agg.h:39-61).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
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

/* Inputs are copied out of the Java heap (Get<Type>ArrayRegion) and outputs
 * copied back (Set<Type>ArrayRegion): no array stays pinned while the GPU
 * works, so the query never holds the GC locker.  The copies are host
 * memcpys, small next to the H2D transfer the engine does anyway. */
static void* copy_in(JNIEnv* env, jarray a, size_t elem, int is_byte,
                     int* failed) {
  if (!a || *failed) return NULL;
  const jsize n = (*env)->GetArrayLength(env, a);
  void* p = malloc(n > 0 ? (size_t)n * elem : 1);
  if (!p) {
    *failed = 1;
    return NULL;
  }
  if (is_byte)
    (*env)->GetByteArrayRegion(env, (jbyteArray)a, 0, n, (jbyte*)p);
  else
    (*env)->GetLongArrayRegion(env, (jlongArray)a, 0, n, (jlong*)p);
  if ((*env)->ExceptionCheck(env)) *failed = 1;
  return p;
}

static void* alloc_out(JNIEnv* env, jarray a, size_t elem, int* failed) {
  if (!a || *failed) return NULL;
  const jsize n = (*env)->GetArrayLength(env, a);
  void* p = calloc(n > 0 ? (size_t)n : 1, elem);
  if (!p) *failed = 1;
  return p;
}

JNIEXPORT jint JNICALL Java_net_opentsdb_core_GpuAggregation_nativeRunCells(
    JNIEnv* env, jclass cls, jlong ctx, jlongArray jspec, jlongArray jcal,
    jlongArray janch, jlongArray janch_edge, jint n_series, jlongArray jrow_series, jlongArray jrow_base,
    jlongArray jqual_off, jbyteArray jqual, jlongArray jval_off,
    jbyteArray jval, jlongArray jgoff, jlongArray jgmem, jlongArray jooff,
    jlongArray jots, jlongArray joval, jbyteArray joisint) {
  (void)cls;
  if (!jspec || (*env)->GetArrayLength(env, jspec) < SPEC_LEN || !jgoff ||
      !jooff || !jots || !joval || !joisint) {
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
  /* optional trailing word (ABI 5): otsdb_query_spec.flags, e.g.
   * OTSDB_SPEC_EXACT_ORDER for dev over groups past 65,536 members */
  if ((*env)->GetArrayLength(env, jspec) > SPEC_LEN) {
    jlong fl = 0;
    (*env)->GetLongArrayRegion(env, jspec, SPEC_LEN, 1, &fl);
    s.flags = (int32_t)fl;
  }
  const jsize n_rows = jrow_series ? (*env)->GetArrayLength(env, jrow_series) : 0;
  const jsize n_groups = (*env)->GetArrayLength(env, jgoff) - 1;
  const jsize n_out_off = (*env)->GetArrayLength(env, jooff);
  const jsize cap = (*env)->GetArrayLength(env, jots);
  if (n_groups < 0 || n_out_off < n_groups + 1 ||
      (*env)->GetArrayLength(env, joval) < cap ||
      (*env)->GetArrayLength(env, joisint) < cap) {
    throw_status(env, OTSDB_E_ILLEGAL_ARGUMENT);
    return OTSDB_E_ILLEGAL_ARGUMENT;
  }

  if ((janch == NULL) != (janch_edge == NULL) ||
      (janch && (*env)->GetArrayLength(env, janch) !=
                    (*env)->GetArrayLength(env, janch_edge))) {
    throw_status(env, OTSDB_E_ILLEGAL_ARGUMENT);
    return OTSDB_E_ILLEGAL_ARGUMENT;
  }
  int failed = 0;
  void* in[11];
  in[0] = copy_in(env, jcal, 8, 0, &failed);
  in[1] = copy_in(env, jrow_series, 8, 0, &failed);
  in[2] = copy_in(env, jrow_base, 8, 0, &failed);
  in[3] = copy_in(env, jqual_off, 8, 0, &failed);
  in[4] = copy_in(env, jqual, 1, 1, &failed);
  in[5] = copy_in(env, jval_off, 8, 0, &failed);
  in[6] = copy_in(env, jval, 1, 1, &failed);
  in[7] = copy_in(env, jgoff, 8, 0, &failed);
  in[8] = copy_in(env, jgmem, 8, 0, &failed);
  in[9] = copy_in(env, janch, 8, 0, &failed);
  in[10] = copy_in(env, janch_edge, 8, 0, &failed);
  void* out[4];
  out[0] = alloc_out(env, jooff, 8, &failed);
  out[1] = alloc_out(env, jots, 8, &failed);
  out[2] = alloc_out(env, joval, 8, &failed);
  out[3] = alloc_out(env, joisint, 1, &failed);

  otsdb_status st = OTSDB_E_DEVICE;
  if (!failed) {
    s.cal_edges = (const int64_t*)in[0];
    s.n_cal_edges = jcal ? (*env)->GetArrayLength(env, jcal) : 0;
    s.cal_anchors = (const int64_t*)in[9];
    s.cal_anchor_edge = (const int64_t*)in[10];
    s.n_cal_anchors = janch ? (*env)->GetArrayLength(env, janch) : 0;
    otsdb_cells c;
    c.n_rows = n_rows;
    c.row_series = (const int64_t*)in[1];
    c.row_base_s = (const int64_t*)in[2];
    c.qual_off = (const int64_t*)in[3];
    c.qual = (const uint8_t*)in[4];
    c.val_off = (const int64_t*)in[5];
    c.val = (const uint8_t*)in[6];
    otsdb_batch b;
    memset(&b, 0, sizeof(b));
    b.n_series = n_series;
    b.n_groups = n_groups;
    b.group_offsets = (const int64_t*)in[7];
    b.group_members = (const int64_t*)in[8];
    otsdb_result r;
    r.capacity = cap;
    r.offsets = (int64_t*)out[0];
    r.ts = (int64_t*)out[1];
    r.val = (int64_t*)out[2];
    r.is_int = (uint8_t*)out[3];
    st = otsdb_agg_run_cells((otsdb_ctx*)(intptr_t)ctx, &s, &c, &b, &r);
    if (st == OTSDB_OK || st == OTSDB_E_CAPACITY) {
      /* offsets carry the needed size on CAPACITY too */
      (*env)->SetLongArrayRegion(env, jooff, 0, n_groups + 1,
                                 (const jlong*)out[0]);
    }
    if (st == OTSDB_OK) {
      const jsize n = (jsize)((int64_t*)out[0])[n_groups];
      (*env)->SetLongArrayRegion(env, jots, 0, n, (const jlong*)out[1]);
      (*env)->SetLongArrayRegion(env, joval, 0, n, (const jlong*)out[2]);
      (*env)->SetByteArrayRegion(env, joisint, 0, n, (const jbyte*)out[3]);
    }
  }
  for (int i = 0; i < 11; ++i) free(in[i]);
  for (int i = 0; i < 4; ++i) free(out[i]);
  if ((*env)->ExceptionCheck(env)) return OTSDB_E_DEVICE; /* OOM pending */
  if (failed) {
    jclass oom = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (oom) (*env)->ThrowNew(env, oom, "otsdb_agg_jni: native buffers");
    return OTSDB_E_DEVICE;
  }
  /* CAPACITY and UNSUPPORTED go back to Java (retry larger / keep the Java
   * iterators); the rest are the reference's exceptions */
  if (st != OTSDB_OK && st != OTSDB_E_CAPACITY && st != OTSDB_E_UNSUPPORTED)
    throw_status(env, st);
  return st;
}
