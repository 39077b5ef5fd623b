/*
 * qe_jni.c — JNI shim between kquerydiy's Kotlin operators and libqe_hip.so.
 *
 * Every `Java_NativeEngine_*` function here is the native half of one `external fun` of
 * `object NativeEngine` (NativeEngine.kt, same directory); NativeOperators.kt holds the Kotlin
 * operator and expression classes built on them, written against the reference's file-private
 * interfaces in kquerydiy/src/Main.kt ("K:" below):
 *   ColumnVector K:24-27 ............. column handles (device qe_column + ownership)
 *   Expression.evaluate K:448-450 .... evalArith / evalCmp / evalBool / castToDouble
 *   ProjectionExec K:582-603 ......... selectProjectAsync / selectProjectWait (fused with a filter)
 *   HashAggregateExec K:605-660 ...... agg* (create, update, fused update, finalize)
 *   MaxAccumulator K:538-561 ......... QE_AGG_MAX inside the aggregate kernels
 *   main() partial -> final K:1309-1325  aggMergeInto (one process) / aggExchange (RCCL, one per GPU)
 *   CsvDataSource K:276-357 .......... csvParse / csvColumn
 *   RecordBatch K:56-61 in / out ..... importBatch / exportColumns (Arrow C Data Interface)
 *
 * Handles are `long`s: pointers to the small host structs below, created and freed only here.
 * Errors: a failing qe_* status throws the Java exception the reference throws in the same
 * situation (throw_status), and the function returns 0 / NULL; the caller sees the exception.
 * Built by Makefile (needs $JAVA_HOME/include/jni.h, absent in this image); the logic is tested
 * without a JVM by tests/native/jni_harness.c (tests/test_jni_shim.py).
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qe_hip.h"

/* ---- handles ------------------------------------------------------------------------------ */

/* A column (ColumnVector, K:24-27): the device view passed to the C ABI, and the device blocks
 * it owns (none for a view of a batch's or CSV table's column). */
typedef struct qj_col {
  qe_column c;
  qe_ctx* ctx;   /* owner of the blocks below; NULL for a view */
  void* blk[3];  /* values, validity, offsets */
  int64_t capacity;
  qe_strdict* dict; /* dictEncode output: the dictionary its codes belong to */
} qj_col;

/* HashAggregateExec state: the native aggregate and what finalize needs to shape its output. */
typedef struct qj_agg {
  qe_hashagg* h;
  qe_ctx* ctx;
  int32_t nkeys, naggs;
  int32_t key_types[QE_MAX_KEYS];
  qe_agg_desc aggs[QE_MAX_AGGS];
  qe_strdict* bound[QE_MAX_KEYS]; /* dictionaries of keys fed dictEncode codes (bound at the first update) */
  int64_t updates;
} qj_agg;

/* CSV table: the parsed table and the device copy of the file it indexes. */
typedef struct qj_csv {
  qe_csv_table* t;
  qe_ctx* ctx;
  void* data;
} qj_csv;

/* Fused specs carry a tag so that a select spec is never passed as an aggregate spec. */
enum { QJ_SPEC_FUSED = 0x51464431, QJ_SPEC_SELECT = 0x51534C31 };
typedef struct qj_spec {
  int32_t tag;
  int32_t ncols_min; /* columns the spec reads: slots must be < the batch's column count */
  union {
    qe_fused_spec fused;
    qe_select_spec select;
  } u;
} qj_spec;

/* ---- exceptions --------------------------------------------------------------------------- */

static void throw_class(JNIEnv* env, const char* cls, const char* msg) {
  jclass k = (*env)->FindClass(env, cls);
  if (k) (*env)->ThrowNew(env, k, msg);
}

/* Status -> the exception the reference throws for the same condition: a CAST of a bad string is
 * Kotlin's toDouble() NumberFormatException (K:791); other invalid arguments are the
 * IllegalArgumentException of Schema.select (K:49); unsupported types / plans the
 * IllegalStateException of K:195 / K:677 / K:792 / K:799; the rest RuntimeException. */
static void throw_status(JNIEnv* env, int st) {
  const char* msg = qe_last_error();
  const char* cls = "java/lang/RuntimeException";
  if (st == QE_ERR_INVALID_ARG)
    cls = strstr(msg, "NumberFormatException") ? "java/lang/NumberFormatException" : "java/lang/IllegalArgumentException";
  else if (st == QE_ERR_UNSUPPORTED)
    cls = "java/lang/IllegalStateException";
  else if (st == QE_ERR_OOM)
    cls = "java/lang/OutOfMemoryError";
  throw_class(env, cls, msg && *msg ? msg : "libqe_hip error");
}

static void throw_arg(JNIEnv* env, const char* msg) { throw_class(env, "java/lang/IllegalArgumentException", msg); }

#define QJ_TRY(env, expr, ret)          \
  do {                                  \
    int st_ = (expr);                   \
    if (st_ != QE_OK) {                 \
      throw_status(env, st_);           \
      return ret;                       \
    }                                   \
  } while (0)

#define QJ_NEED(env, cond, msg, ret) \
  do {                               \
    if (!(cond)) {                   \
      throw_arg(env, msg);           \
      return ret;                    \
    }                                \
  } while (0)

/* ---- Java array helpers (a negative result: an exception is pending) ---------------------- */

static jsize arr_len(JNIEnv* env, jarray a) { return a ? (*env)->GetArrayLength(env, a) : 0; }

static int get_longs(JNIEnv* env, jlongArray a, int64_t* buf, jsize max, const char* what) {
  const jsize n = arr_len(env, a);
  if (n > max) {
    char m[96];
    snprintf(m, sizeof m, "%s: %d entries, at most %d", what, (int)n, (int)max);
    throw_arg(env, m);
    return -1;
  }
  if (n) (*env)->GetLongArrayRegion(env, a, 0, n, (jlong*)buf);
  return (*env)->ExceptionCheck(env) ? -1 : (int)n;
}

static int get_ints(JNIEnv* env, jintArray a, int32_t* buf, jsize max, const char* what) {
  const jsize n = arr_len(env, a);
  if (n > max) {
    char m[96];
    snprintf(m, sizeof m, "%s: %d entries, at most %d", what, (int)n, (int)max);
    throw_arg(env, m);
    return -1;
  }
  if (n) (*env)->GetIntArrayRegion(env, a, 0, n, (jint*)buf);
  return (*env)->ExceptionCheck(env) ? -1 : (int)n;
}

static jlongArray new_longs(JNIEnv* env, const int64_t* v, jsize n) {
  jlongArray a = (*env)->NewLongArray(env, n);
  if (a && n) (*env)->SetLongArrayRegion(env, a, 0, n, (const jlong*)v);
  return a;
}

/* ---- column helpers ----------------------------------------------------------------------- */

static int type_width(int32_t t) {
  switch (t) {
    case QE_TYPE_INT64:
    case QE_TYPE_FLOAT64: return 8;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: return 4;
    case QE_TYPE_UINT8: return 1;
    default: return 0; /* BOOL (bits), UTF8 (offsets + bytes) */
  }
}

static size_t bitmap_bytes(int64_t rows) { /* whole 32-bit words, at least one (qe_hip.h) */
  const size_t w = (size_t)((rows + 31) / 32);
  return (w ? w : 1) * 4;
}

static qj_col* col_of(JNIEnv* env, jlong h) {
  if (!h) throw_arg(env, "null column handle");
  return (qj_col*)(intptr_t)h;
}

static void col_release(qj_col* c) {
  if (!c) return;
  if (c->ctx)
    for (int i = 0; i < 3; ++i)
      if (c->blk[i]) qe_device_free(c->ctx, c->blk[i]);
  free(c);
}

/* A new owned column of `rows` capacity: fixed-width / BOOL values, or UTF8 offsets + `bytes`;
 * a validity bitmap when `nullable`. NULL (exception pending) on failure. */
static qj_col* col_new(JNIEnv* env, qe_ctx* ctx, int32_t type, int64_t rows, int64_t bytes, int nullable) {
  if (rows < 0 || bytes < 0) {
    throw_arg(env, "negative column size");
    return NULL;
  }
  const int w = type_width(type);
  if (!w && type != QE_TYPE_BOOL && type != QE_TYPE_UTF8) {
    char m[64];
    snprintf(m, sizeof m, "unknown column type %d", (int)type);
    throw_class(env, "java/lang/IllegalStateException", m); /* K:469 */
    return NULL;
  }
  qj_col* c = (qj_col*)calloc(1, sizeof(qj_col));
  if (!c) {
    throw_class(env, "java/lang/OutOfMemoryError", "column handle");
    return NULL;
  }
  c->ctx = ctx;
  c->c.type = type;
  c->c.length = rows;
  c->capacity = rows;
  size_t vb = type == QE_TYPE_BOOL ? bitmap_bytes(rows) : type == QE_TYPE_UTF8 ? (size_t)bytes : (size_t)rows * w;
  int st = qe_device_alloc(ctx, vb ? vb : 8, &c->blk[0]);
  if (st == QE_OK && nullable) st = qe_device_alloc(ctx, bitmap_bytes(rows), &c->blk[1]);
  if (st == QE_OK && type == QE_TYPE_UTF8) st = qe_device_alloc(ctx, (size_t)(rows + 1) * 4, &c->blk[2]);
  if (st != QE_OK) {
    col_release(c);
    throw_status(env, st);
    return NULL;
  }
  c->c.values = c->blk[0];
  c->c.validity = (uint8_t*)c->blk[1];
  c->c.offsets = (int32_t*)c->blk[2];
  return c;
}

/* A handle for a view of someone else's column (batch, CSV table): frees only the struct. */
static jlong col_view(JNIEnv* env, const qe_column* v) {
  qj_col* c = (qj_col*)calloc(1, sizeof(qj_col));
  if (!c) {
    throw_class(env, "java/lang/OutOfMemoryError", "column handle");
    return 0;
  }
  c->c = *v;
  c->capacity = v->length;
  return (jlong)(intptr_t)c;
}

/* Handles of a long[] of columns into a qe_column array (max entries). */
static int get_cols(JNIEnv* env, jlongArray a, qe_column* out, int max, int allow_zero, const char* what) {
  int64_t h[QE_MAX_COLS > QE_MAX_AGGS ? QE_MAX_COLS : QE_MAX_AGGS];
  const int n = get_longs(env, a, h, max, what);
  for (int i = 0; i < n; ++i) {
    if (!h[i]) {
      if (!allow_zero) {
        throw_arg(env, "null column handle");
        return -1;
      }
      memset(&out[i], 0, sizeof(qe_column));
      continue;
    }
    out[i] = ((qj_col*)(intptr_t)h[i])->c;
  }
  return n;
}

static int64_t utf8_bytes(JNIEnv* env, qe_ctx* ctx, const qe_column* c) {
  if (c->length == 0) return 0;
  int32_t o0 = 0, on = 0;
  QJ_TRY(env, qe_copy_to_host(ctx, &o0, c->offsets, 4), -1);
  QJ_TRY(env, qe_copy_to_host(ctx, &on, c->offsets + c->length, 4), -1);
  return (int64_t)on - o0;
}

/* ---- context ------------------------------------------------------------------------------ */

JNIEXPORT jint JNICALL Java_NativeEngine_abiVersion(JNIEnv* env, jclass k) {
  (void)env, (void)k;
  return qe_abi_version();
}

JNIEXPORT jlong JNICALL Java_NativeEngine_ctxCreate(JNIEnv* env, jclass k, jint device) {
  (void)k;
  qe_ctx* ctx = NULL;
  QJ_TRY(env, qe_ctx_create_owned(device, &ctx), 0);
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_NativeEngine_ctxDestroy(JNIEnv* env, jclass k, jlong ctx) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", );
  QJ_TRY(env, qe_ctx_destroy((qe_ctx*)(intptr_t)ctx), );
}

JNIEXPORT void JNICALL Java_NativeEngine_ctxSynchronize(JNIEnv* env, jclass k, jlong ctx) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", );
  QJ_TRY(env, qe_ctx_synchronize((qe_ctx*)(intptr_t)ctx), );
}

/* ---- columns (ColumnVector K:24-27) ------------------------------------------------------- */

JNIEXPORT jlong JNICALL Java_NativeEngine_columnAllocate(JNIEnv* env, jclass k, jlong ctx, jint type, jlong rows,
                                                         jlong utf8Bytes, jboolean nullable) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  qj_col* c = col_new(env, (qe_ctx*)(intptr_t)ctx, type, rows, utf8Bytes, nullable);
  return (jlong)(intptr_t)c;
}

JNIEXPORT void JNICALL Java_NativeEngine_columnFree(JNIEnv* env, jclass k, jlong col) {
  (void)env, (void)k;
  col_release((qj_col*)(intptr_t)col);
}

JNIEXPORT jlong JNICALL Java_NativeEngine_columnLength(JNIEnv* env, jclass k, jlong col) {
  (void)k;
  qj_col* c = col_of(env, col);
  return c ? c->c.length : 0;
}

JNIEXPORT jint JNICALL Java_NativeEngine_columnType(JNIEnv* env, jclass k, jlong col) {
  (void)k;
  qj_col* c = col_of(env, col);
  return c ? c->c.type : 0;
}

JNIEXPORT jboolean JNICALL Java_NativeEngine_columnNullable(JNIEnv* env, jclass k, jlong col) {
  (void)k;
  qj_col* c = col_of(env, col);
  return c && c->c.validity ? JNI_TRUE : JNI_FALSE;
}

/* Host -> device: fixed-width values from a long[] (INT64 / INT32 / DATE32 / UINT8, narrowed) or
 * a double[] (FLOAT64); optional Arrow validity bitmap (LSB first, ceil(n/8) bytes). */
static jlong col_from_host(JNIEnv* env, qe_ctx* ctx, int32_t type, const void* vals, int64_t n, jbyteArray validity) {
  const jsize vn = arr_len(env, validity);
  if (validity && vn < (n + 7) / 8) {
    throw_arg(env, "validity bitmap shorter than ceil(rows / 8) bytes");
    return 0;
  }
  qj_col* c = col_new(env, ctx, type, n, 0, validity != NULL);
  if (!c) return 0;
  int st = QE_OK;
  if (n) st = qe_copy_to_device(ctx, c->c.values, vals, (size_t)n * type_width(type));
  if (st == QE_OK && validity) {
    const size_t bb = bitmap_bytes(n);
    uint8_t* bits = (uint8_t*)calloc(bb, 1);
    if (!bits) st = QE_ERR_OOM;
    if (bits) {
      (*env)->GetByteArrayRegion(env, validity, 0, (jsize)((n + 7) / 8), (jbyte*)bits);
      st = qe_copy_to_device(ctx, c->c.validity, bits, bb);
      free(bits);
    }
  }
  if (st != QE_OK) {
    col_release(c);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)c;
}

JNIEXPORT jlong JNICALL Java_NativeEngine_columnFromLongs(JNIEnv* env, jclass k, jlong ctx, jint type,
                                                          jlongArray values, jbyteArray validity) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  QJ_NEED(env, values, "null values", 0);
  const int w = type_width(type);
  QJ_NEED(env, w && type != QE_TYPE_FLOAT64, "columnFromLongs: INT64, INT32, DATE32 or UINT8", 0);
  const jsize n = arr_len(env, values);
  int64_t* v = (int64_t*)malloc((size_t)(n ? n : 1) * 8);
  QJ_NEED(env, v, "out of host memory", 0);
  (*env)->GetLongArrayRegion(env, values, 0, n, (jlong*)v);
  if (w == 4)
    for (jsize i = 0; i < n; ++i) ((int32_t*)v)[i] = (int32_t)v[i];
  else if (w == 1)
    for (jsize i = 0; i < n; ++i) ((uint8_t*)v)[i] = (uint8_t)v[i];
  const jlong h = col_from_host(env, (qe_ctx*)(intptr_t)ctx, type, v, n, validity);
  free(v);
  return h;
}

JNIEXPORT jlong JNICALL Java_NativeEngine_columnFromDoubles(JNIEnv* env, jclass k, jlong ctx, jdoubleArray values,
                                                            jbyteArray validity) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  QJ_NEED(env, values, "null values", 0);
  const jsize n = arr_len(env, values);
  double* v = (double*)malloc((size_t)(n ? n : 1) * 8);
  QJ_NEED(env, v, "out of host memory", 0);
  (*env)->GetDoubleArrayRegion(env, values, 0, n, v);
  const jlong h = col_from_host(env, (qe_ctx*)(intptr_t)ctx, QE_TYPE_FLOAT64, v, n, validity);
  free(v);
  return h;
}

/* UTF8 column from Arrow-style offsets (rows + 1 entries, offsets[0] = 0) and bytes. */
JNIEXPORT jlong JNICALL Java_NativeEngine_columnFromUtf8(JNIEnv* env, jclass k, jlong ctx, jintArray offsets,
                                                         jbyteArray data, jbyteArray validity) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  QJ_NEED(env, offsets && arr_len(env, offsets) >= 1, "offsets need rows + 1 entries", 0);
  qe_ctx* c = (qe_ctx*)(intptr_t)ctx;
  const jsize no = arr_len(env, offsets), nb = arr_len(env, data);
  const int64_t n = no - 1;
  int32_t* off = (int32_t*)malloc((size_t)no * 4);
  QJ_NEED(env, off, "out of host memory", 0);
  (*env)->GetIntArrayRegion(env, offsets, 0, no, (jint*)off);
  int ok = off[0] == 0 && off[n] <= nb;
  for (int64_t i = 0; ok && i < n; ++i) ok = off[i] <= off[i + 1];
  if (!ok || (validity && arr_len(env, validity) < (n + 7) / 8)) {
    free(off);
    throw_arg(env, "offsets must start at 0, not decrease and end within the data; validity ceil(rows / 8) bytes");
    return 0;
  }
  qj_col* col = col_new(env, c, QE_TYPE_UTF8, n, off[n], validity != NULL);
  if (!col) {
    free(off);
    return 0;
  }
  int st = qe_copy_to_device(c, col->c.offsets, off, (size_t)no * 4);
  uint8_t* bytes = (uint8_t*)malloc((size_t)(off[n] ? off[n] : 1));
  if (!bytes) st = QE_ERR_OOM;
  if (st == QE_OK && off[n]) {
    (*env)->GetByteArrayRegion(env, data, 0, off[n], (jbyte*)bytes);
    st = qe_copy_to_device(c, col->c.values, bytes, (size_t)off[n]);
  }
  free(bytes);
  free(off);
  if (st == QE_OK && validity) {
    const size_t bb = bitmap_bytes(n);
    uint8_t* bits = (uint8_t*)calloc(bb, 1);
    if (!bits) st = QE_ERR_OOM;
    if (bits) {
      (*env)->GetByteArrayRegion(env, validity, 0, (jsize)((n + 7) / 8), (jbyte*)bits);
      st = qe_copy_to_device(c, col->c.validity, bits, bb);
      free(bits);
    }
  }
  if (st != QE_OK) {
    col_release(col);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)col;
}

/* Device -> host for ColumnVector.getValue / printQueryResult (K:24-27, K:1344-1353): fixed-width
 * and BOOL values widened to long (BOOL 0 / 1), or FLOAT64 as double. `out` holds >= length. */
JNIEXPORT void JNICALL Java_NativeEngine_columnToLongs(JNIEnv* env, jclass k, jlong ctx, jlong col, jlongArray out) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", );
  qj_col* c = col_of(env, col);
  if (!c) return;
  const int64_t n = c->c.length;
  const int w = type_width(c->c.type);
  QJ_NEED(env, (w && c->c.type != QE_TYPE_FLOAT64) || c->c.type == QE_TYPE_BOOL, "columnToLongs: integer or BOOL column", );
  QJ_NEED(env, arr_len(env, out) >= n, "output array shorter than the column", );
  if (!n) return;
  const size_t nb = c->c.type == QE_TYPE_BOOL ? (size_t)(n + 7) / 8 : (size_t)n * w;
  uint8_t* raw = (uint8_t*)malloc(nb);
  int64_t* v = (int64_t*)malloc((size_t)n * 8);
  if (!raw || !v) {
    free(raw);
    free(v);
    throw_class(env, "java/lang/OutOfMemoryError", "host copy");
    return;
  }
  const int st = qe_copy_to_host((qe_ctx*)(intptr_t)ctx, raw, c->c.values, nb);
  if (st == QE_OK) {
    for (int64_t i = 0; i < n; ++i)
      v[i] = c->c.type == QE_TYPE_BOOL ? (raw[i >> 3] >> (i & 7)) & 1
             : w == 8                  ? ((const int64_t*)raw)[i]
             : w == 4                  ? ((const int32_t*)raw)[i]
                                       : raw[i];
    (*env)->SetLongArrayRegion(env, out, 0, (jsize)n, (const jlong*)v);
  }
  free(raw);
  free(v);
  if (st != QE_OK) throw_status(env, st);
}

JNIEXPORT void JNICALL Java_NativeEngine_columnToDoubles(JNIEnv* env, jclass k, jlong ctx, jlong col,
                                                         jdoubleArray out) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", );
  qj_col* c = col_of(env, col);
  if (!c) return;
  const int64_t n = c->c.length;
  QJ_NEED(env, c->c.type == QE_TYPE_FLOAT64, "columnToDoubles: FLOAT64 column", );
  QJ_NEED(env, arr_len(env, out) >= n, "output array shorter than the column", );
  if (!n) return;
  double* v = (double*)malloc((size_t)n * 8);
  QJ_NEED(env, v, "out of host memory", );
  const int st = qe_copy_to_host((qe_ctx*)(intptr_t)ctx, v, c->c.values, (size_t)n * 8);
  if (st == QE_OK) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)n, v);
  free(v);
  if (st != QE_OK) throw_status(env, st);
}

/* Arrow validity bitmap (ceil(length / 8) bytes), or null when every row is valid. */
JNIEXPORT jbyteArray JNICALL Java_NativeEngine_columnValidity(JNIEnv* env, jclass k, jlong ctx, jlong col) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", NULL);
  qj_col* c = col_of(env, col);
  if (!c || !c->c.validity) return NULL;
  const jsize nb = (jsize)((c->c.length + 7) / 8);
  jbyteArray a = (*env)->NewByteArray(env, nb);
  if (!a || !nb) return a;
  uint8_t* bits = (uint8_t*)malloc((size_t)nb);
  QJ_NEED(env, bits, "out of host memory", NULL);
  const int st = qe_copy_to_host((qe_ctx*)(intptr_t)ctx, bits, c->c.validity, (size_t)nb);
  if (st == QE_OK) (*env)->SetByteArrayRegion(env, a, 0, nb, (const jbyte*)bits);
  free(bits);
  if (st != QE_OK) {
    throw_status(env, st);
    return NULL;
  }
  return a;
}

/* UTF8 column -> host offsets (length + 1, rebased to 0) and bytes. */
JNIEXPORT jintArray JNICALL Java_NativeEngine_columnUtf8Offsets(JNIEnv* env, jclass k, jlong ctx, jlong col) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", NULL);
  qj_col* c = col_of(env, col);
  if (!c) return NULL;
  QJ_NEED(env, c->c.type == QE_TYPE_UTF8, "columnUtf8Offsets: UTF8 column", NULL);
  const jsize no = (jsize)(c->c.length + 1);
  int32_t* off = (int32_t*)malloc((size_t)no * 4);
  QJ_NEED(env, off, "out of host memory", NULL);
  const int st = qe_copy_to_host((qe_ctx*)(intptr_t)ctx, off, c->c.offsets, (size_t)no * 4);
  jintArray a = NULL;
  if (st == QE_OK) {
    for (jsize i = no - 1; i >= 0; --i) off[i] -= off[0];
    a = (*env)->NewIntArray(env, no);
    if (a) (*env)->SetIntArrayRegion(env, a, 0, no, (const jint*)off);
  }
  free(off);
  if (st != QE_OK) throw_status(env, st);
  return a;
}

JNIEXPORT jbyteArray JNICALL Java_NativeEngine_columnUtf8Bytes(JNIEnv* env, jclass k, jlong ctx, jlong col) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", NULL);
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  qj_col* c = col_of(env, col);
  if (!c) return NULL;
  QJ_NEED(env, c->c.type == QE_TYPE_UTF8, "columnUtf8Bytes: UTF8 column", NULL);
  const int64_t nb = utf8_bytes(env, cx, &c->c);
  if (nb < 0) return NULL;
  int32_t o0 = 0;
  if (c->c.length) QJ_TRY(env, qe_copy_to_host(cx, &o0, c->c.offsets, 4), NULL);
  jbyteArray a = (*env)->NewByteArray(env, (jsize)nb);
  if (!a || !nb) return a;
  uint8_t* b = (uint8_t*)malloc((size_t)nb);
  QJ_NEED(env, b, "out of host memory", NULL);
  const int st = qe_copy_to_host(cx, b, (const uint8_t*)c->c.values + o0, (size_t)nb);
  if (st == QE_OK) (*env)->SetByteArrayRegion(env, a, 0, (jsize)nb, (const jbyte*)b);
  free(b);
  if (st != QE_OK) {
    throw_status(env, st);
    return NULL;
  }
  return a;
}

/* Synthetic column (qe_generate: the measurement harness's counter-based generator). */
JNIEXPORT jlong JNICALL Java_NativeEngine_generate(JNIEnv* env, jclass k, jlong ctx, jint type, jlong rows, jint dist,
                                                   jlong param, jlong seed, jlong colId, jlong row0, jint nullPermille) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  qj_col* c = col_new(env, cx, type, rows, 0, nullPermille > 0);
  if (!c) return 0;
  const int st = qe_generate(cx, &c->c, dist, param, (uint64_t)seed, (uint64_t)colId, row0, nullPermille);
  if (st != QE_OK) {
    col_release(c);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)c;
}

/* ---- RecordBatch over the Arrow C Data Interface (K:56-61, K:635-650) ----------------------- */

JNIEXPORT jlong JNICALL Java_NativeEngine_importBatch(JNIEnv* env, jclass k, jlong ctx, jlong schemaAddr,
                                                      jlong arrayAddr) {
  (void)k;
  QJ_NEED(env, ctx && schemaAddr && arrayAddr, "null ctx / ArrowSchema / ArrowArray address", 0);
  qe_batch* b = NULL;
  QJ_TRY(env,
         qe_batch_import((qe_ctx*)(intptr_t)ctx, (const ArrowSchema*)(intptr_t)schemaAddr,
                         (const ArrowArray*)(intptr_t)arrayAddr, &b),
         0);
  return (jlong)(intptr_t)b;
}

JNIEXPORT void JNICALL Java_NativeEngine_batchDestroy(JNIEnv* env, jclass k, jlong batch) {
  (void)k;
  if (batch) QJ_TRY(env, qe_batch_destroy((qe_batch*)(intptr_t)batch), );
}

JNIEXPORT jint JNICALL Java_NativeEngine_batchNumColumns(JNIEnv* env, jclass k, jlong batch) {
  (void)k;
  QJ_NEED(env, batch, "null batch handle", 0);
  int32_t n = 0;
  int64_t len = 0;
  QJ_TRY(env, qe_batch_num_columns((const qe_batch*)(intptr_t)batch, &n, &len), 0);
  return n;
}

/* View handle of column i (free with columnFree; valid while the batch lives). */
JNIEXPORT jlong JNICALL Java_NativeEngine_batchColumn(JNIEnv* env, jclass k, jlong batch, jint i) {
  (void)k;
  QJ_NEED(env, batch, "null batch handle", 0);
  qe_column c;
  QJ_TRY(env, qe_batch_column((const qe_batch*)(intptr_t)batch, i, &c, NULL), 0);
  return col_view(env, &c);
}

JNIEXPORT jstring JNICALL Java_NativeEngine_batchColumnName(JNIEnv* env, jclass k, jlong batch, jint i) {
  (void)k;
  QJ_NEED(env, batch, "null batch handle", NULL);
  qe_column c;
  const char* name = NULL;
  QJ_TRY(env, qe_batch_column((const qe_batch*)(intptr_t)batch, i, &c, &name), NULL);
  return (*env)->NewStringUTF(env, name ? name : "");
}

/* Device columns -> the ArrowSchema / ArrowArray structs Java allocated (then
 * Data.importVectorSchemaRoot). All columns must have the same length. */
JNIEXPORT void JNICALL Java_NativeEngine_exportColumns(JNIEnv* env, jclass k, jlong ctx, jlongArray cols,
                                                       jobjectArray names, jlong schemaAddr, jlong arrayAddr) {
  (void)k;
  QJ_NEED(env, ctx && schemaAddr && arrayAddr, "null ctx / ArrowSchema / ArrowArray address", );
  const jsize n = arr_len(env, cols);
  QJ_NEED(env, arr_len(env, names) == n, "one name per column", );
  qe_column* c = (qe_column*)calloc((size_t)(n ? n : 1), sizeof(qe_column));
  const char** nm = (const char**)calloc((size_t)(n ? n : 1), sizeof(char*));
  jstring* js = (jstring*)calloc((size_t)(n ? n : 1), sizeof(jstring));
  int ok = c && nm && js;
  if (!ok) throw_class(env, "java/lang/OutOfMemoryError", "export arrays");
  for (jsize i = 0; ok && i < n; ++i) {
    jlong h = 0;
    (*env)->GetLongArrayRegion(env, cols, i, 1, &h);
    js[i] = (jstring)(*env)->GetObjectArrayElement(env, names, i);
    ok = h && js[i];
    if (!ok) {
      throw_arg(env, "null column handle or name");
      break;
    }
    c[i] = ((qj_col*)(intptr_t)h)->c;
    nm[i] = (*env)->GetStringUTFChars(env, js[i], NULL);
    ok = nm[i] != NULL;
  }
  if (ok) {
    const int st = qe_batch_export((qe_ctx*)(intptr_t)ctx, c, n, nm, (ArrowSchema*)(intptr_t)schemaAddr,
                                   (ArrowArray*)(intptr_t)arrayAddr);
    if (st != QE_OK) throw_status(env, st);
  }
  for (jsize i = 0; js && i < n; ++i)
    if (js[i]) {
      if (nm && nm[i]) (*env)->ReleaseStringUTFChars(env, js[i], nm[i]);
      (*env)->DeleteLocalRef(env, js[i]);
    }
  free(c);
  free(nm);
  free(js);
}

/* ---- Expression.evaluate (K:448-450) ----------------------------------------------------- */

static int operand_of(JNIEnv* env, jlong col, jint litType, jlong litBits, jboolean litNull, qe_operand* o) {
  memset(o, 0, sizeof *o);
  if (col) {
    o->col = &((qj_col*)(intptr_t)col)->c;
    return 1;
  }
  if (litType != QE_TYPE_INT64 && litType != QE_TYPE_FLOAT64) {
    throw_arg(env, "literal type must be INT64 or FLOAT64");
    return 0;
  }
  o->lit.type = litType;
  o->lit.is_null = litNull ? 1 : 0;
  o->lit.bits = litBits;
  return 1;
}

static int operand_f64(const qe_operand* o) { return o->col ? o->col->type == QE_TYPE_FLOAT64 : o->lit.type == QE_TYPE_FLOAT64; }

static int64_t operand_rows(const qe_operand* a, const qe_operand* b) {
  return a->col ? a->col->length : b->col ? b->col->length : -1;
}

/* BinaryExpression arithmetic: lhs column, rhs column or literal (rhs = 0). Output INT64, or
 * FLOAT64 when an operand is; always with a validity bitmap (int64 x / 0 is null). */
JNIEXPORT jlong JNICALL Java_NativeEngine_evalArith(JNIEnv* env, jclass k, jlong ctx, jint op, jlong lhs, jlong rhs,
                                                    jint litType, jlong litBits, jboolean litNull) {
  (void)k;
  QJ_NEED(env, ctx && lhs, "null ctx or lhs column handle", 0);
  qe_operand a, b;
  if (!operand_of(env, lhs, 0, 0, 0, &a) || !operand_of(env, rhs, litType, litBits, litNull, &b)) return 0;
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  const int32_t t = operand_f64(&a) || operand_f64(&b) ? QE_TYPE_FLOAT64 : QE_TYPE_INT64;
  qj_col* out = col_new(env, cx, t, operand_rows(&a, &b), 0, 1);
  if (!out) return 0;
  const int st = qe_eval_arith(cx, op, &a, &b, &out->c);
  if (st != QE_OK) {
    col_release(out);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)out;
}

/* Comparison -> BOOL column with validity (null operand -> null). */
JNIEXPORT jlong JNICALL Java_NativeEngine_evalCmp(JNIEnv* env, jclass k, jlong ctx, jint op, jlong lhs, jlong rhs,
                                                  jint litType, jlong litBits, jboolean litNull) {
  (void)k;
  QJ_NEED(env, ctx && lhs, "null ctx or lhs column handle", 0);
  qe_operand a, b;
  if (!operand_of(env, lhs, 0, 0, 0, &a) || !operand_of(env, rhs, litType, litBits, litNull, &b)) return 0;
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  qj_col* out = col_new(env, cx, QE_TYPE_BOOL, operand_rows(&a, &b), 0, 1);
  if (!out) return 0;
  const int st = qe_eval_cmp(cx, op, &a, &b, &out->c);
  if (st != QE_OK) {
    col_release(out);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)out;
}

/* AND / OR / NOT / IS_NULL / IS_NOT_NULL over BOOL columns (rhs = 0 for the unary ops). */
JNIEXPORT jlong JNICALL Java_NativeEngine_evalBool(JNIEnv* env, jclass k, jlong ctx, jint op, jlong lhs, jlong rhs) {
  (void)k;
  QJ_NEED(env, ctx && lhs, "null ctx or lhs column handle", 0);
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  const qe_column* a = &((qj_col*)(intptr_t)lhs)->c;
  const qe_column* b = rhs ? &((qj_col*)(intptr_t)rhs)->c : NULL;
  qj_col* out = col_new(env, cx, QE_TYPE_BOOL, a->length, 0, 1);
  if (!out) return 0;
  const int st = qe_eval_bool(cx, op, a, b, &out->c);
  if (st != QE_OK) {
    col_release(out);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)out;
}

/* CastExpression UTF8 -> FLOAT64 (K:772-805): NumberFormatException naming the first bad row. */
JNIEXPORT jlong JNICALL Java_NativeEngine_castToDouble(JNIEnv* env, jclass k, jlong ctx, jlong in) {
  (void)k;
  QJ_NEED(env, ctx && in, "null ctx or column handle", 0);
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  const qe_column* src = &((qj_col*)(intptr_t)in)->c;
  qj_col* out = col_new(env, cx, QE_TYPE_FLOAT64, src->length, 0, src->validity != NULL);
  if (!out) return 0;
  int64_t row = -1;
  const int st = qe_cast_utf8_to_f64(cx, src, &out->c, &row);
  if (st != QE_OK) {
    col_release(out);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)out;
}

/* ---- SelectionExec (order-preserving compaction) ----------------------------------------- */

JNIEXPORT jlong JNICALL Java_NativeEngine_filterCount(JNIEnv* env, jclass k, jlong ctx, jlong mask) {
  (void)k;
  QJ_NEED(env, ctx && mask, "null ctx or mask handle", 0);
  int64_t n = 0;
  QJ_TRY(env, qe_filter_count((qe_ctx*)(intptr_t)ctx, &((qj_col*)(intptr_t)mask)->c, &n), 0);
  return n;
}

/* The rows of `inputs` whose mask is true (null -> dropped), in order: new owned columns. */
JNIEXPORT jlongArray JNICALL Java_NativeEngine_filter(JNIEnv* env, jclass k, jlong ctx, jlong mask,
                                                      jlongArray inputs) {
  (void)k;
  QJ_NEED(env, ctx && mask, "null ctx or mask handle", NULL);
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  qe_column in[QE_MAX_COLS], out[QE_MAX_COLS];
  const int n = get_cols(env, inputs, in, QE_MAX_COLS, 0, "filter inputs");
  if (n < 0) return NULL;
  const qe_column* m = &((qj_col*)(intptr_t)mask)->c;
  int64_t cnt = 0;
  QJ_TRY(env, qe_filter_count(cx, m, &cnt), NULL);
  qj_col* oc[QE_MAX_COLS] = {0};
  int64_t hs[QE_MAX_COLS];
  for (int i = 0; i < n; ++i) {
    const int64_t bytes = in[i].type == QE_TYPE_UTF8 ? utf8_bytes(env, cx, &in[i]) : 0;
    oc[i] = bytes < 0 ? NULL : col_new(env, cx, in[i].type, cnt, bytes, in[i].validity != NULL);
    if (!oc[i]) {
      for (int j = 0; j < i; ++j) col_release(oc[j]);
      return NULL;
    }
    out[i] = oc[i]->c;
  }
  int64_t got = 0;
  const int st = qe_filter_apply(cx, m, in, n, out, &got);
  if (st != QE_OK) {
    for (int i = 0; i < n; ++i) col_release(oc[i]);
    throw_status(env, st);
    return NULL;
  }
  for (int i = 0; i < n; ++i) {
    oc[i]->c.length = got;
    hs[i] = (int64_t)(intptr_t)oc[i];
  }
  return new_longs(env, hs, n);
}

/* ---- global aggregate (no GROUP BY) ------------------------------------------------------- */

/* {rows, count, type, valid, sum, min, max, avg bits}: sum/min/max are int64 values or fp64 bits. */
JNIEXPORT jlongArray JNICALL Java_NativeEngine_aggGlobal(JNIEnv* env, jclass k, jlong ctx, jlong col, jlong mask) {
  (void)k;
  QJ_NEED(env, ctx && col, "null ctx or column handle", NULL);
  qe_global_agg r;
  QJ_TRY(env,
         qe_agg_global((qe_ctx*)(intptr_t)ctx, &((qj_col*)(intptr_t)col)->c,
                       mask ? &((qj_col*)(intptr_t)mask)->c : NULL, &r),
         NULL);
  int64_t avg_bits;
  memcpy(&avg_bits, &r.avg, 8);
  const int64_t v[8] = {r.rows, r.count, r.type, r.valid, r.sum, r.min, r.max, avg_bits};
  return new_longs(env, v, 8);
}

/* ---- fused plans (filter terms + key slots + postfix programs) ---------------------------- */

/* Shared by fusedSpec / selectSpec: predicate terms and the programs, flattened. Term t compares
 * column slot termCol[t] by termOp[t] with column termRhsCol[t] (>= 0) or the literal
 * (termLitType[t], termLitBits[t]). Program p is tokens [sum(progLen[..p]), + progLen[p]) of
 * (tokOp, tokArg, tokLitType, tokLitBits). Returns the largest column slot used, -2 on error. */
static int spec_parts(JNIEnv* env, jint maskCol, jintArray termCol, jintArray termOp, jintArray termRhsCol,
                      jintArray termLitType, jlongArray termLitBits, jintArray progLen, jintArray tokOp,
                      jintArray tokArg, jintArray tokLitType, jlongArray tokLitBits, int32_t* nterms,
                      qe_pred_term* terms, int32_t* nprog, qe_agg_program* progs) {
  int32_t tc[QE_MAX_TERMS], to[QE_MAX_TERMS], tr[QE_MAX_TERMS], tt[QE_MAX_TERMS];
  int64_t tb[QE_MAX_TERMS];
  const int nt = get_ints(env, termCol, tc, QE_MAX_TERMS, "predicate terms");
  if (nt < 0) return -2;
  if (get_ints(env, termOp, to, QE_MAX_TERMS, "termOp") != nt || get_ints(env, termRhsCol, tr, QE_MAX_TERMS, "termRhsCol") != nt ||
      get_ints(env, termLitType, tt, QE_MAX_TERMS, "termLitType") != nt ||
      get_longs(env, termLitBits, tb, QE_MAX_TERMS, "termLitBits") != nt) {
    if (!(*env)->ExceptionCheck(env)) throw_arg(env, "predicate term arrays differ in length");
    return -2;
  }
  int maxc = maskCol;
  for (int t = 0; t < nt; ++t) {
    if (to[t] < QE_OP_EQ || to[t] > QE_OP_GE || tc[t] < 0 || tc[t] >= QE_MAX_COLS || tr[t] >= QE_MAX_COLS) {
      throw_arg(env, "predicate term: comparison op and column slots in range");
      return -2;
    }
    memset(&terms[t], 0, sizeof terms[t]);
    terms[t].col = tc[t];
    terms[t].op = to[t];
    terms[t].rhs_col = tr[t] >= 0 ? tr[t] : -1;
    terms[t].lit.type = tt[t];
    terms[t].lit.bits = tb[t];
    maxc = tc[t] > maxc ? tc[t] : maxc;
    maxc = tr[t] > maxc ? tr[t] : maxc;
  }
  *nterms = nt;
  int32_t pl[QE_MAX_AGGS];
  const int np = get_ints(env, progLen, pl, QE_MAX_AGGS, "programs");
  if (np < 0) return -2;
  int total = 0;
  for (int p = 0; p < np; ++p) {
    if (pl[p] < 0 || pl[p] > QE_MAX_TOKENS) {
      throw_arg(env, "program length out of range");
      return -2;
    }
    total += pl[p];
  }
  enum { MAXT = QE_MAX_AGGS * QE_MAX_TOKENS };
  int32_t ko[MAXT], ka[MAXT], kt[MAXT];
  int64_t kb[MAXT];
  if (get_ints(env, tokOp, ko, MAXT, "tokOp") != total || get_ints(env, tokArg, ka, MAXT, "tokArg") != total ||
      get_ints(env, tokLitType, kt, MAXT, "tokLitType") != total || get_longs(env, tokLitBits, kb, MAXT, "tokLitBits") != total) {
    if (!(*env)->ExceptionCheck(env)) throw_arg(env, "token arrays must hold sum(progLen) entries");
    return -2;
  }
  int at = 0;
  for (int p = 0; p < np; ++p) {
    memset(&progs[p], 0, sizeof progs[p]);
    progs[p].ntokens = pl[p];
    int depth = 0;
    for (int i = 0; i < pl[p]; ++i, ++at) {
      qe_token* t = &progs[p].tokens[i];
      t->op = ko[at];
      t->arg = ka[at];
      t->lit.type = kt[at];
      t->lit.bits = kb[at];
      if (t->op == QE_TOK_COL) {
        if (t->arg < 0 || t->arg >= QE_MAX_COLS) {
          throw_arg(env, "program column slot out of range");
          return -2;
        }
        maxc = t->arg > maxc ? t->arg : maxc;
        ++depth;
      } else if (t->op == QE_TOK_LIT) {
        ++depth;
      } else if (t->op >= QE_TOK_ADD && t->op <= QE_TOK_DIV) {
        if (depth < 2) {
          throw_arg(env, "program is not a valid postfix expression");
          return -2;
        }
        --depth;
      } else {
        throw_arg(env, "unknown program token");
        return -2;
      }
    }
    if (pl[p] && depth != 1) {
      throw_arg(env, "program is not a valid postfix expression");
      return -2;
    }
  }
  *nprog = np;
  return maxc;
}

/* Filter -> project -> aggregate plan for aggUpdateFused: keyCols are column slots; program j is
 * aggregate j's input (progLen 0 for COUNT_STAR). */
JNIEXPORT jlong JNICALL Java_NativeEngine_fusedSpec(JNIEnv* env, jclass k, jint maskCol, jintArray termCol,
                                                    jintArray termOp, jintArray termRhsCol, jintArray termLitType,
                                                    jlongArray termLitBits, jintArray keyCols, jintArray progLen,
                                                    jintArray tokOp, jintArray tokArg, jintArray tokLitType,
                                                    jlongArray tokLitBits) {
  (void)k;
  QJ_NEED(env, maskCol >= -1 && maskCol < QE_MAX_COLS, "mask column slot out of range", 0);
  qj_spec* s = (qj_spec*)calloc(1, sizeof(qj_spec));
  QJ_NEED(env, s, "out of host memory", 0);
  s->tag = QJ_SPEC_FUSED;
  qe_fused_spec* f = &s->u.fused;
  f->mask_col = maskCol;
  int32_t nprog = 0;
  int maxc = spec_parts(env, maskCol, termCol, termOp, termRhsCol, termLitType, termLitBits, progLen, tokOp, tokArg,
                        tokLitType, tokLitBits, &f->nterms, f->terms, &nprog, f->inputs);
  int32_t kc[QE_MAX_KEYS];
  const int nk = maxc < -1 ? -1 : get_ints(env, keyCols, kc, QE_MAX_KEYS, "key columns");
  for (int i = 0; i < QE_MAX_KEYS; ++i) f->key_cols[i] = -1;
  for (int i = 0; i < nk && maxc >= -1; ++i) {
    if (kc[i] < 0 || kc[i] >= QE_MAX_COLS) {
      throw_arg(env, "key column slot out of range");
      maxc = -2;
      break;
    }
    f->key_cols[i] = kc[i];
    maxc = kc[i] > maxc ? kc[i] : maxc;
  }
  if (maxc < -1 || nk < 0) {
    free(s);
    return 0;
  }
  s->ncols_min = maxc + 1;
  return (jlong)(intptr_t)s;
}

/* Filter -> project plan for selectProjectAsync: program k is output column k. */
JNIEXPORT jlong JNICALL Java_NativeEngine_selectSpec(JNIEnv* env, jclass k, jint maskCol, jintArray termCol,
                                                     jintArray termOp, jintArray termRhsCol, jintArray termLitType,
                                                     jlongArray termLitBits, jintArray progLen, jintArray tokOp,
                                                     jintArray tokArg, jintArray tokLitType, jlongArray tokLitBits) {
  (void)k;
  QJ_NEED(env, maskCol >= -1 && maskCol < QE_MAX_COLS, "mask column slot out of range", 0);
  qj_spec* s = (qj_spec*)calloc(1, sizeof(qj_spec));
  QJ_NEED(env, s, "out of host memory", 0);
  s->tag = QJ_SPEC_SELECT;
  qe_select_spec* q = &s->u.select;
  q->mask_col = maskCol;
  const int maxc = spec_parts(env, maskCol, termCol, termOp, termRhsCol, termLitType, termLitBits, progLen, tokOp, tokArg,
                              tokLitType, tokLitBits, &q->nterms, q->terms, &q->nout, q->outputs);
  if (maxc < -1 || q->nout < 1) {
    if (maxc >= -1) throw_arg(env, "a select-project needs at least one output program");
    free(s);
    return 0;
  }
  for (int p = 0; p < q->nout; ++p)
    if (q->outputs[p].ntokens == 0) {
      throw_arg(env, "empty output program");
      free(s);
      return 0;
    }
  s->ncols_min = maxc + 1;
  return (jlong)(intptr_t)s;
}

JNIEXPORT void JNICALL Java_NativeEngine_specFree(JNIEnv* env, jclass k, jlong spec) {
  (void)env, (void)k;
  free((qj_spec*)(intptr_t)spec);
}

static qj_spec* spec_of(JNIEnv* env, jlong h, int32_t tag) {
  qj_spec* s = (qj_spec*)(intptr_t)h;
  if (!s || s->tag != tag) {
    throw_arg(env, tag == QJ_SPEC_FUSED ? "not a fusedSpec handle" : "not a selectSpec handle");
    return NULL;
  }
  return s;
}

/* ---- HashAggregateExec (K:605-660) ------------------------------------------------------- */

static qj_agg* agg_of(JNIEnv* env, jlong h) {
  if (!h) throw_arg(env, "null aggregate handle");
  return (qj_agg*)(intptr_t)h;
}

/* keyTypes: the group keys' column types, UTF8 included (the state owns the dictionaries: aggUpdate
 * takes the Utf8 key columns, aggFinalize returns Utf8 key columns). fns[j] / inputTypes[j]:
 * aggregate j (QE_AGG_*, input type; ignored for COUNT_STAR). expectedGroups 0 = 1024 (the reference
 * has no hint). flags: QE_HASHAGG_DETERMINISTIC / QE_HASHAGG_FAST_FP64. */
JNIEXPORT jlong JNICALL Java_NativeEngine_aggCreate(JNIEnv* env, jclass k, jlong ctx, jintArray keyTypes,
                                                    jintArray fns, jintArray inputTypes, jlong expectedGroups,
                                                    jint flags) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  qj_agg a;
  memset(&a, 0, sizeof a);
  a.ctx = (qe_ctx*)(intptr_t)ctx;
  int32_t f[QE_MAX_AGGS], t[QE_MAX_AGGS];
  a.nkeys = get_ints(env, keyTypes, a.key_types, QE_MAX_KEYS, "key types");
  if (a.nkeys < 0) return 0;
  a.naggs = get_ints(env, fns, f, QE_MAX_AGGS, "aggregates");
  if (a.naggs < 0) return 0;
  QJ_NEED(env, get_ints(env, inputTypes, t, QE_MAX_AGGS, "input types") == a.naggs, "one input type per aggregate", 0);
  for (int j = 0; j < a.naggs; ++j) {
    a.aggs[j].fn = f[j];
    a.aggs[j].input_type = t[j];
    if (t[j] == QE_TYPE_UTF8 && f[j] != QE_AGG_COUNT && f[j] != QE_AGG_COUNT_STAR) {
      /* MaxAccumulator.accumulate (K:545-550): a String value takes `else -> throw
       * UnsupportedOperationException("MAX is not implemented for data type ${value.javaClass.name}")` */
      char msg[96];
      snprintf(msg, sizeof msg, "%s is not implemented for data type java.lang.String",
               f[j] == QE_AGG_MAX ? "MAX" : f[j] == QE_AGG_MIN ? "MIN" : f[j] == QE_AGG_SUM ? "SUM" : "AVG");
      throw_class(env, "java/lang/UnsupportedOperationException", msg);
      return 0;
    }
  }
  QJ_TRY(env,
         qe_hashagg_create_ex(a.ctx, a.nkeys, a.key_types, a.naggs, a.aggs, expectedGroups > 0 ? expectedGroups : 1024,
                              flags, &a.h),
         0);
  qj_agg* h = (qj_agg*)malloc(sizeof(qj_agg));
  if (!h) {
    qe_hashagg_destroy(a.h);
    throw_class(env, "java/lang/OutOfMemoryError", "aggregate handle");
    return 0;
  }
  *h = a;
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL Java_NativeEngine_aggDestroy(JNIEnv* env, jclass k, jlong agg) {
  (void)k;
  qj_agg* a = (qj_agg*)(intptr_t)agg;
  if (!a) return;
  const int st = qe_hashagg_destroy(a->h);
  free(a);
  if (st != QE_OK) throw_status(env, st);
}

JNIEXPORT void JNICALL Java_NativeEngine_aggReset(JNIEnv* env, jclass k, jlong agg) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  if (a) QJ_TRY(env, qe_hashagg_reset(a->h), );
}

JNIEXPORT void JNICALL Java_NativeEngine_aggSetAsync(JNIEnv* env, jclass k, jlong agg, jboolean enable) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  if (a) QJ_TRY(env, qe_hashagg_set_async(a->h, enable ? 1 : 0), );
}

JNIEXPORT void JNICALL Java_NativeEngine_aggSetRowBase(JNIEnv* env, jclass k, jlong agg, jlong rowBase) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  if (a) QJ_TRY(env, qe_hashagg_set_row_base(a->h, rowBase), );
}

/* One input batch (K:617-632): key columns, aggregate input columns (0 for COUNT_STAR), an
 * optional BOOL mask column selecting rows. */
JNIEXPORT void JNICALL Java_NativeEngine_aggUpdate(JNIEnv* env, jclass k, jlong agg, jlongArray keyCols,
                                                   jlongArray inputCols, jlong maskCol) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  if (!a) return;
  qe_column keys[QE_MAX_KEYS], in[QE_MAX_AGGS];
  const int nk = get_cols(env, keyCols, keys, QE_MAX_KEYS, 0, "key columns");
  if (nk < 0) return;
  const int ni = get_cols(env, inputCols, in, QE_MAX_AGGS, 1, "aggregate inputs");
  if (ni < 0) return;
  QJ_NEED(env, nk == a->nkeys && ni == a->naggs, "one column per key and per aggregate", );
  /* keys that are dictEncode codes: the state learns their dictionary at the first update (so
   * finalize stays codes but merges and exchanges go by string content), and a later batch may not
   * bring codes of another dictionary */
  int64_t kh[QE_MAX_KEYS];
  (void)get_longs(env, keyCols, kh, QE_MAX_KEYS, "key columns");
  for (int i = 0; i < nk; ++i) {
    qe_strdict* d = ((qj_col*)(intptr_t)kh[i])->dict;
    if (a->updates == 0 && d) {
      QJ_TRY(env, qe_hashagg_bind_key_dict(a->h, i, d), );
      a->bound[i] = d;
      a->key_types[i] = QE_TYPE_UTF8; /* finalize decodes through the dictionary */
    }
    QJ_NEED(env, d == a->bound[i], "group key codes from another dictionary than the state's first batch", );
  }
  ++a->updates;
  if (a->nkeys == 0) /* COUNT(*) of a key-less state counts the batch's rows */
    for (int j = 0; j < ni; ++j)
      if (!in[j].values && a->aggs[j].fn == QE_AGG_COUNT_STAR)
        for (int i = 0; i < ni; ++i)
          if (in[i].values) {
            in[j] = in[i];
            break;
          }
  QJ_TRY(env,
         qe_hashagg_update(a->h, nk ? keys : NULL, in, maskCol ? &((qj_col*)(intptr_t)maskCol)->c : NULL), );
}

/* Fused filter -> project -> aggregate over one batch's columns (one pass over HBM). */
JNIEXPORT void JNICALL Java_NativeEngine_aggUpdateFused(JNIEnv* env, jclass k, jlong agg, jlongArray cols, jlong spec) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  qj_spec* s = a ? spec_of(env, spec, QJ_SPEC_FUSED) : NULL;
  if (!s) return;
  qe_column c[QE_MAX_COLS];
  const int n = get_cols(env, cols, c, QE_MAX_COLS, 0, "batch columns");
  if (n < 0) return;
  QJ_NEED(env, n >= s->ncols_min, "the plan reads a column slot beyond the batch's columns", );
  QJ_TRY(env, qe_hashagg_update_fused(a->h, c, n, &s->u.fused), );
  ++a->updates;
}

JNIEXPORT jlong JNICALL Java_NativeEngine_aggNumGroups(JNIEnv* env, jclass k, jlong agg) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  int64_t g = 0;
  if (a) QJ_TRY(env, qe_hashagg_num_groups(a->h, &g), 0);
  return g;
}

static int32_t agg_out_type(const qe_agg_desc* d) {
  if (d->fn == QE_AGG_COUNT || d->fn == QE_AGG_COUNT_STAR) return QE_TYPE_INT64;
  return d->fn == QE_AGG_AVG || d->input_type == QE_TYPE_FLOAT64 ? QE_TYPE_FLOAT64 : QE_TYPE_INT64;
}

/* The ONE output batch (K:635-650): handles of the key columns then one column per aggregate
 * (owned; free with columnFree). The contents are complete when this returns. */
JNIEXPORT jlongArray JNICALL Java_NativeEngine_aggFinalize(JNIEnv* env, jclass k, jlong agg) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  if (!a) return NULL;
  int64_t groups = 0, key_bytes[QE_MAX_KEYS] = {0, 0, 0, 0};
  /* the groups, and the bytes of each Utf8 key's strings (the state decodes its own dictionaries) */
  QJ_TRY(env, qe_hashagg_finalize_sizes(a->h, &groups, key_bytes), NULL);
  const int n = a->nkeys + a->naggs;
  qj_col* oc[QE_MAX_KEYS + QE_MAX_AGGS] = {0};
  qe_column keys[QE_MAX_KEYS], out[QE_MAX_AGGS];
  int st = QE_OK;
  for (int i = 0; i < n && st == QE_OK; ++i) {
    const int is_key = i < a->nkeys;
    const int32_t t = is_key ? a->key_types[i] : agg_out_type(&a->aggs[i - a->nkeys]);
    const int fn = is_key ? 0 : a->aggs[i - a->nkeys].fn;
    oc[i] = col_new(env, a->ctx, t, groups, is_key ? key_bytes[i] : 0,
                    is_key || (fn != QE_AGG_COUNT && fn != QE_AGG_COUNT_STAR));
    if (!oc[i]) st = QE_ERR_OOM;
    else if (is_key) keys[i] = oc[i]->c;
    else out[i - a->nkeys] = oc[i]->c;
  }
  int64_t got = 0;
  if (st == QE_OK) {
    st = qe_hashagg_finalize(a->h, keys, out, &got);
    if (st == QE_OK) st = qe_ctx_synchronize(a->ctx);
    if (st != QE_OK) throw_status(env, st);
  }
  if (st != QE_OK) {
    for (int i = 0; i < n; ++i) col_release(oc[i]);
    return NULL;
  }
  int64_t hs[QE_MAX_KEYS + QE_MAX_AGGS];
  for (int i = 0; i < n; ++i) {
    oc[i]->c.length = got;
    hs[i] = (int64_t)(intptr_t)oc[i];
  }
  return new_longs(env, hs, n);
}

/* main()'s partial -> final merge inside one process (K:1314-1325): every group of `partial`
 * is merged into `owner` (combine semantics per aggregate). Utf8 / key-tuple keyed states merge by
 * key CONTENT (qe_hashagg_merge re-encodes the partial's keys into the owner's dictionaries), so two
 * partitions whose dictionaries number the same string differently still meet in one group. */
JNIEXPORT void JNICALL Java_NativeEngine_aggMergeInto(JNIEnv* env, jclass k, jlong owner, jlong partial) {
  (void)k;
  qj_agg* o = agg_of(env, owner);
  qj_agg* p = o ? agg_of(env, partial) : NULL;
  if (!p) return;
  QJ_NEED(env, o->ctx == p->ctx, "owner and partial must share a ctx", );
  QJ_TRY(env, qe_hashagg_merge(o->h, p->h), );
}

/* Device time (ms) of the last update's aggregation kernels. */
JNIEXPORT jdouble JNICALL Java_NativeEngine_aggLastKernelMs(JNIEnv* env, jclass k, jlong agg) {
  (void)k;
  qj_agg* a = agg_of(env, agg);
  double ms = 0;
  int32_t launches = 0;
  if (a) QJ_TRY(env, qe_hashagg_last_kernel_time(a->h, &ms, &launches), 0);
  return ms;
}

/* ---- fused SelectionExec -> ProjectionExec (K:582-603), pipelined ----------------------- */

static int32_t program_type(const qe_agg_program* p, const qe_column* cols) {
  if (p->ntokens == 1 && p->tokens[0].op == QE_TOK_COL) return cols[p->tokens[0].arg].type;
  for (int i = 0; i < p->ntokens; ++i) {
    const qe_token* t = &p->tokens[i];
    if ((t->op == QE_TOK_COL && cols[t->arg].type == QE_TYPE_FLOAT64) || (t->op == QE_TOK_LIT && t->lit.type == QE_TYPE_FLOAT64))
      return QE_TYPE_FLOAT64;
  }
  return QE_TYPE_INT64;
}

/* Output columns for a select spec over `cols` (capacity = the batch's rows, validity always). */
JNIEXPORT jlongArray JNICALL Java_NativeEngine_selectAllocateOutputs(JNIEnv* env, jclass k, jlong ctx, jlong spec,
                                                                     jlongArray cols) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", NULL);
  qj_spec* s = spec_of(env, spec, QJ_SPEC_SELECT);
  if (!s) return NULL;
  qe_column c[QE_MAX_COLS];
  const int n = get_cols(env, cols, c, QE_MAX_COLS, 0, "batch columns");
  if (n < 0) return NULL;
  QJ_NEED(env, n >= s->ncols_min && n >= 1, "the plan reads a column slot beyond the batch's columns", NULL);
  int64_t hs[QE_MAX_AGGS];
  qj_col* oc[QE_MAX_AGGS] = {0};
  for (int p = 0; p < s->u.select.nout; ++p) {
    const int32_t t = program_type(&s->u.select.outputs[p], c);
    QJ_NEED(env, t != QE_TYPE_UTF8, "select-project outputs are fixed-width", NULL);
    oc[p] = col_new(env, (qe_ctx*)(intptr_t)ctx, t, c[0].length, 0, 1);
    if (!oc[p]) {
      for (int i = 0; i < p; ++i) col_release(oc[i]);
      return NULL;
    }
    hs[p] = (int64_t)(intptr_t)oc[p];
  }
  return new_longs(env, hs, s->u.select.nout);
}

/* Queue one batch's select-project; returns the pending handle for selectProjectWait. The
 * inputs must stay alive and the outputs unread until then. */
JNIEXPORT jlong JNICALL Java_NativeEngine_selectProjectAsync(JNIEnv* env, jclass k, jlong ctx, jlongArray cols,
                                                             jlong spec, jlongArray outs) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  qj_spec* s = spec_of(env, spec, QJ_SPEC_SELECT);
  if (!s) return 0;
  qe_column c[QE_MAX_COLS], o[QE_MAX_AGGS];
  const int n = get_cols(env, cols, c, QE_MAX_COLS, 0, "batch columns");
  if (n < 0) return 0;
  QJ_NEED(env, n >= s->ncols_min, "the plan reads a column slot beyond the batch's columns", 0);
  const int no = get_cols(env, outs, o, QE_MAX_AGGS, 0, "output columns");
  if (no < 0) return 0;
  QJ_NEED(env, no == s->u.select.nout, "one output column per program", 0);
  qe_select_pending* p = NULL;
  QJ_TRY(env, qe_select_project_async((qe_ctx*)(intptr_t)ctx, c, n, &s->u.select, o, &p), 0);
  return (jlong)(intptr_t)p; /* selectProjectWait sets the output handles' lengths */
}

/* Rows the select-project wrote, also set as the length of the `outs` handles given to
 * selectProjectAsync (frees the pending handle). */
JNIEXPORT jlong JNICALL Java_NativeEngine_selectProjectWait(JNIEnv* env, jclass k, jlong pending, jlongArray outs) {
  (void)k;
  QJ_NEED(env, pending, "null pending handle", 0);
  int64_t rows = 0;
  QJ_TRY(env, qe_select_pending_wait((qe_select_pending*)(intptr_t)pending, &rows), 0);
  int64_t hs[QE_MAX_AGGS];
  const int no = get_longs(env, outs, hs, QE_MAX_AGGS, "output columns");
  for (int i = 0; i < no; ++i)
    if (hs[i]) ((qj_col*)(intptr_t)hs[i])->c.length = rows;
  return rows;
}

/* ---- Utf8 group keys: string dictionary (K:620-627) -------------------------------------- */

JNIEXPORT jlong JNICALL Java_NativeEngine_dictCreate(JNIEnv* env, jclass k, jlong ctx, jlong expected) {
  (void)k;
  QJ_NEED(env, ctx, "null ctx handle", 0);
  qe_strdict* d = NULL;
  QJ_TRY(env, qe_strdict_create((qe_ctx*)(intptr_t)ctx, expected > 0 ? expected : 1024, &d), 0);
  return (jlong)(intptr_t)d;
}

JNIEXPORT void JNICALL Java_NativeEngine_dictDestroy(JNIEnv* env, jclass k, jlong dict) {
  (void)k;
  if (dict) QJ_TRY(env, qe_strdict_destroy((qe_strdict*)(intptr_t)dict), );
}

/* UTF8 column -> INT32 codes (new owned column; validity iff the input has one). */
JNIEXPORT jlong JNICALL Java_NativeEngine_dictEncode(JNIEnv* env, jclass k, jlong ctx, jlong dict, jlong in) {
  (void)k;
  QJ_NEED(env, ctx && dict && in, "null ctx, dictionary or column handle", 0);
  const qe_column* src = &((qj_col*)(intptr_t)in)->c;
  qj_col* out = col_new(env, (qe_ctx*)(intptr_t)ctx, QE_TYPE_INT32, src->length, 0, src->validity != NULL);
  if (!out) return 0;
  const int st = qe_strdict_encode((qe_strdict*)(intptr_t)dict, src, &out->c);
  if (st != QE_OK) {
    col_release(out);
    throw_status(env, st);
    return 0;
  }
  out->dict = (qe_strdict*)(intptr_t)dict;
  return (jlong)(intptr_t)out;
}

/* INT32 codes -> UTF8 column (new owned column). */
JNIEXPORT jlong JNICALL Java_NativeEngine_dictDecode(JNIEnv* env, jclass k, jlong ctx, jlong dict, jlong codes) {
  (void)k;
  QJ_NEED(env, ctx && dict && codes, "null ctx, dictionary or column handle", 0);
  qe_strdict* d = (qe_strdict*)(intptr_t)dict;
  const qe_column* src = &((qj_col*)(intptr_t)codes)->c;
  int64_t bytes = 0;
  QJ_TRY(env, qe_strdict_decode_bytes(d, src, &bytes), 0);
  qj_col* out = col_new(env, (qe_ctx*)(intptr_t)ctx, QE_TYPE_UTF8, src->length, bytes, src->validity != NULL);
  if (!out) return 0;
  const int st = qe_strdict_decode(d, src, &out->c);
  if (st != QE_OK) {
    col_release(out);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)out;
}

/* ---- CsvDataSource.scan on the device (K:276-357) ---------------------------------------- */

/* data: a direct ByteBuffer holding the file (nbytes from its position 0). fields: projected
 * 0-based field positions (the host resolved the header). */
JNIEXPORT jlong JNICALL Java_NativeEngine_csvParse(JNIEnv* env, jclass k, jlong ctx, jobject data, jlong nbytes,
                                                   jint delimiter, jboolean hasHeader, jintArray fields) {
  (void)k;
  QJ_NEED(env, ctx && data, "null ctx or data", 0);
  qe_ctx* cx = (qe_ctx*)(intptr_t)ctx;
  const void* host = (*env)->GetDirectBufferAddress(env, data);
  const jlong cap = (*env)->GetDirectBufferCapacity(env, data);
  QJ_NEED(env, host && nbytes >= 0 && nbytes <= cap, "csvParse needs a direct ByteBuffer of at least nbytes", 0);
  int32_t f[32];
  const int nf = get_ints(env, fields, f, 32, "projected fields");
  if (nf < 0) return 0;
  QJ_NEED(env, nf >= 1, "at least one projected field", 0);
  qj_csv* t = (qj_csv*)calloc(1, sizeof(qj_csv));
  QJ_NEED(env, t, "out of host memory", 0);
  t->ctx = cx;
  int st = qe_device_alloc(cx, (size_t)(nbytes ? nbytes : 1), &t->data);
  if (st == QE_OK && nbytes) st = qe_copy_to_device(cx, t->data, host, (size_t)nbytes);
  if (st == QE_OK) {
    qe_csv_options o;
    memset(&o, 0, sizeof o);
    o.delimiter = delimiter;
    o.has_header = hasHeader ? 1 : 0;
    o.nfields = nf;
    o.field_index = f;
    st = qe_csv_parse(cx, (const uint8_t*)t->data, nbytes, &o, &t->t);
  }
  if (st != QE_OK) {
    if (t->data) qe_device_free(cx, t->data);
    free(t);
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)t;
}

/* Streaming scan (ReaderIterator's batches, K:239-252): the end of the last complete record in the
 * direct buffer's first nbytes (quote-aware; nbytes when eof; 0 when none is complete yet). */
JNIEXPORT jlong JNICALL Java_NativeEngine_csvRecordEnd(JNIEnv* env, jclass k, jobject data, jlong nbytes, jboolean eof) {
  (void)k;
  QJ_NEED(env, data, "null data", 0);
  const void* host = (*env)->GetDirectBufferAddress(env, data);
  const jlong cap = (*env)->GetDirectBufferCapacity(env, data);
  QJ_NEED(env, host && nbytes >= 0 && nbytes <= cap, "csvRecordEnd needs a direct ByteBuffer of at least nbytes", 0);
  int64_t cut = 0;
  QJ_TRY(env, qe_csv_record_end((const uint8_t*)host, nbytes, eof ? 1 : 0, &cut), 0);
  return cut;
}

JNIEXPORT jlong JNICALL Java_NativeEngine_csvRows(JNIEnv* env, jclass k, jlong table) {
  (void)k;
  QJ_NEED(env, table, "null CSV table handle", 0);
  int64_t r = 0;
  QJ_TRY(env, qe_csv_rows(((qj_csv*)(intptr_t)table)->t, &r), 0);
  return r;
}

/* View handle of projected column i (UTF8; valid while the table lives; free with columnFree). */
JNIEXPORT jlong JNICALL Java_NativeEngine_csvColumn(JNIEnv* env, jclass k, jlong table, jint i) {
  (void)k;
  QJ_NEED(env, table, "null CSV table handle", 0);
  qe_column c;
  QJ_TRY(env, qe_csv_column(((qj_csv*)(intptr_t)table)->t, i, &c), 0);
  return col_view(env, &c);
}

JNIEXPORT void JNICALL Java_NativeEngine_csvDestroy(JNIEnv* env, jclass k, jlong table) {
  (void)k;
  qj_csv* t = (qj_csv*)(intptr_t)table;
  if (!t) return;
  const int st = qe_csv_destroy(t->t);
  qe_device_free(t->ctx, t->data);
  free(t);
  if (st != QE_OK) throw_status(env, st);
}

/* ---- multi-GPU partial -> final merge over RCCL (K:1309-1325 across GPUs) ---------------- */

JNIEXPORT jbyteArray JNICALL Java_NativeEngine_commUniqueId(JNIEnv* env, jclass k) {
  (void)k;
  uint8_t id[QE_COMM_ID_BYTES];
  QJ_TRY(env, qe_comm_unique_id(id), NULL);
  jbyteArray a = (*env)->NewByteArray(env, QE_COMM_ID_BYTES);
  if (a) (*env)->SetByteArrayRegion(env, a, 0, QE_COMM_ID_BYTES, (const jbyte*)id);
  return a;
}

/* Collective: every rank calls it with rank 0's id. */
JNIEXPORT jlong JNICALL Java_NativeEngine_commCreate(JNIEnv* env, jclass k, jlong ctx, jint world, jint rank,
                                                     jbyteArray id) {
  (void)k;
  QJ_NEED(env, ctx && id && arr_len(env, id) == QE_COMM_ID_BYTES, "null ctx or an id that is not commUniqueId's", 0);
  uint8_t b[QE_COMM_ID_BYTES];
  (*env)->GetByteArrayRegion(env, id, 0, QE_COMM_ID_BYTES, (jbyte*)b);
  qe_comm* c = NULL;
  QJ_TRY(env, qe_comm_create((qe_ctx*)(intptr_t)ctx, world, rank, b, &c), 0);
  return (jlong)(intptr_t)c;
}

JNIEXPORT void JNICALL Java_NativeEngine_commDestroy(JNIEnv* env, jclass k, jlong comm) {
  (void)k;
  if (comm) QJ_TRY(env, qe_comm_destroy((qe_comm*)(intptr_t)comm), );
}

/* Every rank: route partial's groups to their owners and merge what arrives into owner.
 * Returns the records this rank merged. */
JNIEXPORT jlong JNICALL Java_NativeEngine_aggExchange(JNIEnv* env, jclass k, jlong comm, jlong partial, jlong owner,
                                                      jlong slotRecords) {
  (void)k;
  QJ_NEED(env, comm, "null communicator handle", 0);
  qj_agg* p = agg_of(env, partial);
  qj_agg* o = p ? agg_of(env, owner) : NULL;
  if (!o) return 0;
  int64_t n = 0;
  QJ_TRY(env, qe_hashagg_exchange((qe_comm*)(intptr_t)comm, p->h, o->h, slotRecords, &n), 0);
  return n;
}
