/*
 * TEST DOUBLE — not the JDK's header.  The image has no JDK, so
 * tests/jni_fake stands in for the JVM side of the JNI seam: this file
 * declares the JNI types and the subset of the JNINativeInterface function
 * table that integration/jni/otsdb_agg_jni.c calls (same names, same call
 * shape `(*env)->Fn(env, ...)`), and harness.c implements that table over
 * plain C arrays.  Compiling the shim against it and driving its exported
 * Java_net_opentsdb_core_GpuAggregation_* functions exercises the shim's
 * argument checks, copies, status mapping and exceptions on the real
 * engine; a JDK build uses the real jni.h instead (integration/jni/Makefile).
 */
#ifndef OTSDB_FAKE_JNI_H
#define OTSDB_FAKE_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

struct fake_jobject;  /* harness.c: an array, a string or a class */
typedef struct fake_jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jlongArray;
typedef jarray jbyteArray;
typedef jobject jthrowable;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  const char* (*GetStringUTFChars)(JNIEnv* env, jstring s, jboolean* is_copy);
  void (*ReleaseStringUTFChars)(JNIEnv* env, jstring s, const char* chars);
  jsize (*GetArrayLength)(JNIEnv* env, jarray a);
  void (*GetLongArrayRegion)(JNIEnv* env, jlongArray a, jsize start, jsize len,
                             jlong* buf);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray a, jsize start, jsize len,
                             const jlong* buf);
  void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray a, jsize start, jsize len,
                             jbyte* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray a, jsize start, jsize len,
                             const jbyte* buf);
};

#endif
