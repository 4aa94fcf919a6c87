/*
 * Test harness (tests only): a fake JNIEnv over plain C arrays, so
 * tests/test_jni_shim*.py drive integration/jni/otsdb_agg_jni.c's exported
 * Java_net_opentsdb_core_GpuAggregation_* functions from Python (ctypes)
 * the way GpuAggregation.java would: Java arrays are {length, data} objects,
 * region copies check their bounds (ArrayIndexOutOfBoundsException), and
 * ThrowNew records the pending exception's class and message for the test
 * to read.  See jni.h here: a test double, not the JDK's header.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

struct fake_jobject {
  int kind;      /* 0 array, 1 string, 2 class */
  jsize len;     /* array length */
  size_t elem;   /* array element size */
  void* data;
  char name[160];
};

static struct fake_jobject g_classes[16];
static int g_nclasses;
static char g_exc_class[160];
static char g_exc_msg[512];
static int g_pending;

static jclass fj_find_class(JNIEnv* env, const char* name) {
  (void)env;
  for (int i = 0; i < g_nclasses; ++i)
    if (strcmp(g_classes[i].name, name) == 0) return &g_classes[i];
  if (g_nclasses == 16) return NULL;
  struct fake_jobject* c = &g_classes[g_nclasses++];
  c->kind = 2;
  snprintf(c->name, sizeof(c->name), "%s", name);
  return c;
}

static jint fj_throw_new(JNIEnv* env, jclass clazz, const char* msg) {
  (void)env;
  g_pending = 1;
  snprintf(g_exc_class, sizeof(g_exc_class), "%s", clazz ? clazz->name : "?");
  snprintf(g_exc_msg, sizeof(g_exc_msg), "%s", msg ? msg : "");
  return 0;
}

static jboolean fj_exception_check(JNIEnv* env) {
  (void)env;
  return (jboolean)g_pending;
}

static const char* fj_get_utf(JNIEnv* env, jstring s, jboolean* is_copy) {
  (void)env;
  if (is_copy) *is_copy = 0;
  return s ? (const char*)s->data : NULL;
}

static void fj_release_utf(JNIEnv* env, jstring s, const char* chars) {
  (void)env;
  (void)s;
  (void)chars;
}

static jsize fj_length(JNIEnv* env, jarray a) {
  (void)env;
  return a ? a->len : 0;
}

static int fj_bounds(jarray a, jsize start, jsize len, size_t elem) {
  if (!a || a->kind != 0 || a->elem != elem || start < 0 || len < 0 ||
      start + len > a->len) {
    g_pending = 1;
    snprintf(g_exc_class, sizeof(g_exc_class), "%s",
             "java/lang/ArrayIndexOutOfBoundsException");
    snprintf(g_exc_msg, sizeof(g_exc_msg), "region [%d, %d) of %d", start,
             start + len, a ? a->len : -1);
    return 0;
  }
  return 1;
}

static void fj_get_long(JNIEnv* env, jlongArray a, jsize s, jsize n, jlong* b) {
  (void)env;
  if (fj_bounds(a, s, n, 8)) memcpy(b, (jlong*)a->data + s, (size_t)n * 8);
}
static void fj_set_long(JNIEnv* env, jlongArray a, jsize s, jsize n,
                        const jlong* b) {
  (void)env;
  if (fj_bounds(a, s, n, 8)) memcpy((jlong*)a->data + s, b, (size_t)n * 8);
}
static void fj_get_byte(JNIEnv* env, jbyteArray a, jsize s, jsize n, jbyte* b) {
  (void)env;
  if (fj_bounds(a, s, n, 1)) memcpy(b, (jbyte*)a->data + s, (size_t)n);
}
static void fj_set_byte(JNIEnv* env, jbyteArray a, jsize s, jsize n,
                        const jbyte* b) {
  (void)env;
  if (fj_bounds(a, s, n, 1)) memcpy((jbyte*)a->data + s, b, (size_t)n);
}

static const struct JNINativeInterface_ g_table = {
    fj_find_class, fj_throw_new, fj_exception_check, fj_get_utf,
    fj_release_utf, fj_length, fj_get_long, fj_set_long, fj_get_byte,
    fj_set_byte};
static JNIEnv g_env = &g_table;

/* the shim's natives (integration/jni/otsdb_agg_jni.c) */
JNIEXPORT jlong JNICALL Java_net_opentsdb_core_GpuAggregation_nativeCtxCreate(
    JNIEnv* env, jclass cls, jint device);
JNIEXPORT void JNICALL Java_net_opentsdb_core_GpuAggregation_nativeCtxDestroy(
    JNIEnv* env, jclass cls, jlong ctx);
JNIEXPORT jint JNICALL Java_net_opentsdb_core_GpuAggregation_nativeAggId(
    JNIEnv* env, jclass cls, jstring name);
JNIEXPORT jint JNICALL Java_net_opentsdb_core_GpuAggregation_nativeRunCells(
    JNIEnv* env, jclass cls, jlong ctx, jlongArray jspec, jlongArray jcal,
    jlongArray janch, jlongArray janch_edge, jint n_series,
    jlongArray jrow_series, jlongArray jrow_base, jlongArray jqual_off,
    jbyteArray jqual, jlongArray jval_off, jbyteArray jval, jlongArray jgoff,
    jlongArray jgmem, jlongArray jooff, jlongArray jots, jlongArray joval,
    jbyteArray joisint);

/* ---- what the tests call (ctypes) ---- */
JNIEXPORT const char* fj_exception_class(void) { return g_pending ? g_exc_class : ""; }
JNIEXPORT const char* fj_exception_message(void) { return g_pending ? g_exc_msg : ""; }
JNIEXPORT void fj_clear(void) { g_pending = 0; }

JNIEXPORT jlong fj_ctx_create(jint device) {
  return Java_net_opentsdb_core_GpuAggregation_nativeCtxCreate(&g_env, NULL, device);
}
JNIEXPORT void fj_ctx_destroy(jlong ctx) {
  Java_net_opentsdb_core_GpuAggregation_nativeCtxDestroy(&g_env, NULL, ctx);
}
JNIEXPORT jint fj_agg_id(const char* name) {
  struct fake_jobject s = {1, 0, 1, (void*)name, ""};
  return Java_net_opentsdb_core_GpuAggregation_nativeAggId(&g_env, NULL, &s);
}

/* A Java array over caller memory: len < 0 means null. */
static void wrap(struct fake_jobject* o, void* data, jlong len, size_t elem) {
  o->kind = 0;
  o->len = (jsize)len;
  o->elem = elem;
  o->data = data;
  o->name[0] = 0;
}
#define ARR(i) (lens[i] < 0 ? NULL : &objs[i])

/* arrays in nativeRunCells' order: spec, cal, anch, anch_edge, row_series,
 * row_base, qual_off, qual (bytes), val_off, val (bytes), goff, gmem, ooff,
 * ots, oval, oisint (bytes) */
JNIEXPORT jint fj_run_cells(jlong ctx, jint n_series, void** ptrs,
                            const jlong* lens) {
  static const size_t elem[16] = {8, 8, 8, 8, 8, 8, 8, 1, 8, 1, 8, 8, 8, 8, 8, 1};
  struct fake_jobject objs[16];
  for (int i = 0; i < 16; ++i) wrap(&objs[i], ptrs[i], lens[i], elem[i]);
  return Java_net_opentsdb_core_GpuAggregation_nativeRunCells(
      &g_env, NULL, ctx, ARR(0), ARR(1), ARR(2), ARR(3), n_series, ARR(4),
      ARR(5), ARR(6), ARR(7), ARR(8), ARR(9), ARR(10), ARR(11), ARR(12),
      ARR(13), ARR(14), ARR(15));
}
