/*
 * TEST DOUBLE of <jni.h> for tests/native/jni_harness.c — not the JDK header, not ABI compatible.
 *
 * The image has no JDK, so query-engines_amd/jni/qe_jni.c cannot be built against the real
 * header here. This file declares the JNI types and, in `struct JNINativeInterface_`, ONLY the
 * JNIEnv functions the shim calls, by their JNI 1.8 names and signatures; the harness fills the
 * table with its own implementations (Java arrays, strings, direct buffers and pending exceptions
 * as host structs). Because the shim calls every function through `(*env)->Name(env, ...)`, it
 * compiles unchanged against either header: this one tests its logic, the JDK's builds the
 * shipped libqe_jni.so (query-engines_amd/jni/Makefile). Nothing built with this header ships.
 */
#ifndef QE_TEST_JNI_STUB_H
#define QE_TEST_JNI_STUB_H

#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jobject (*GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
  jbyteArray (*NewByteArray)(JNIEnv* env, jsize len);
  jintArray (*NewIntArray)(JNIEnv* env, jsize len);
  jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
  void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
  void (*GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
  void (*GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
  void (*GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, jdouble* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
  void (*SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
  void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
  jstring (*NewStringUTF)(JNIEnv* env, const char* utf);
  const char* (*GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
  void (*ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
  void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
};

#endif
