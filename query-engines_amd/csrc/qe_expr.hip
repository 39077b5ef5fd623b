// Vectorised expression families K1 (arithmetic), K2 (comparison), K3a (boolean):
// the build-defined Expression.evaluate(RecordBatch): ColumnVector implementations
// (interface K:448-450; the reference has no such expressions).
//
// Layout: one thread = 8 consecutive rows = one validity byte, so output validity / boolean
// bytes are produced without atomics. 8-byte operands are read as 4 x 16-B loads per lane.
// Roofline: HBM-bound (16 B read + 8 B write per row for int64 a+b; 8 B + 1/4 B for a>k).
#include "qe_internal.hpp"

namespace qe {

struct Src {
  const void* p;
  const uint8_t* valid;
  int64_t lit;  // int64 value or fp64 bits (already in compute type for K_LIT)
  int32_t kind; // SrcKind
  int32_t lit_null;
};

typedef long long i64x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Loads 8 rows [i0, i0+8) of `s` as raw 64-bit values (int64 widened / fp64 bits / literal).
__device__ __forceinline__ uint8_t load8(const Src& s, int64_t i0, int nrows, int64_t (&v)[8]) {
  uint8_t valid;
  if (s.kind == K_LIT) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = s.lit;
    return s.lit_null ? 0 : 0xFF;
  }
  valid = s.valid ? s.valid[i0 >> 3] : (uint8_t)0xFF;
  if (nrows == 8) {
    switch (s.kind) {
      case K_I64:
      case K_F64: {
        const i64x2* p = (const i64x2*)((const int64_t*)s.p + i0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          i64x2 t = p[q];
          v[2 * q] = t.x;
          v[2 * q + 1] = t.y;
        }
        break;
      }
      case K_I32: {
        const i32x4* p = (const i32x4*)((const int32_t*)s.p + i0);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          i32x4 t = p[q];
          v[4 * q] = t.x;
          v[4 * q + 1] = t.y;
          v[4 * q + 2] = t.z;
          v[4 * q + 3] = t.w;
        }
        break;
      }
      default: {  // K_U8
        const uint64_t w = *(const uint64_t*)((const uint8_t*)s.p + i0);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (int64_t)((w >> (8 * j)) & 0xFF);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = 0;
      if (j < nrows) {
        switch (s.kind) {
          case K_I64:
          case K_F64: v[j] = ((const int64_t*)s.p)[i0 + j]; break;
          case K_I32: v[j] = ((const int32_t*)s.p)[i0 + j]; break;
          default: v[j] = ((const uint8_t*)s.p)[i0 + j];
        }
      }
    }
    valid &= (uint8_t)((1u << nrows) - 1);
  }
  return valid;
}

// Value of a loaded row in the fp64 compute type.
__device__ __forceinline__ double as_f64(const Src& s, int64_t raw) {
  return (s.kind == K_F64 || s.kind == K_LIT) ? bits_f64(raw) : (double)raw;
}

enum ComputeType : int32_t { CT_I64 = 0, CT_F64 = 1 };

__device__ __forceinline__ void store8(int64_t* out, int64_t i0, int nrows, const int64_t (&r)[8]) {
  if (nrows == 8) {
    i64x2* p = (i64x2*)(out + i0);
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q] = i64x2{r[2 * q], r[2 * q + 1]};
  } else {
    for (int j = 0; j < nrows; ++j) out[i0 + j] = r[j];
  }
}

// dn: a device-side row count (a stream-ordered selection's, qe_filter_apply_async): only rows
// below min(n, *dn) are computed.
__global__ void __launch_bounds__(256) k_arith(Src a, Src b, int32_t op, int32_t ct, int64_t* __restrict__ out,
                                               uint8_t* __restrict__ out_valid, int64_t n,
                                               const int64_t* __restrict__ dn) {
  if (dn) n = min(n, *dn);
  const int64_t ngroups = (n + 7) >> 3;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = g << 3;
    const int nrows = (int)min<int64_t>(8, n - i0);
    int64_t x[8], y[8], r[8];
    uint8_t valid = load8(a, i0, nrows, x) & load8(b, i0, nrows, y);
    if (ct == CT_I64) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint64_t ux = (uint64_t)x[j], uy = (uint64_t)y[j];
        switch (op) {
          case QE_OP_ADD: r[j] = (int64_t)(ux + uy); break;  // JVM Long wrap
          case QE_OP_SUB: r[j] = (int64_t)(ux - uy); break;
          case QE_OP_MUL: r[j] = (int64_t)(ux * uy); break;
          default:  // QE_OP_DIV: truncating; x/0 -> null; MIN/-1 wraps to MIN (JVM)
            if (y[j] == 0) {
              r[j] = 0;
              valid &= (uint8_t)~(1u << j);
            } else if (y[j] == -1) {
              r[j] = (int64_t)(0ull - ux);
            } else {
              r[j] = x[j] / y[j];
            }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const double dx = as_f64(a, x[j]), dy = as_f64(b, y[j]);
        double d;
        switch (op) {
          case QE_OP_ADD: d = dx + dy; break;
          case QE_OP_SUB: d = dx - dy; break;
          case QE_OP_MUL: d = dx * dy; break;
          default: d = dx / dy;
        }
        r[j] = f64_bits(d);
      }
    }
    store8(out, i0, nrows, r);
    if (out_valid) out_valid[g] = valid;
  }
}

__global__ void __launch_bounds__(256) k_cmp(Src a, Src b, int32_t op, int32_t ct, uint8_t* __restrict__ out,
                                             uint8_t* __restrict__ out_valid, int64_t n) {
  const int64_t ngroups = (n + 7) >> 3;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = g << 3;
    const int nrows = (int)min<int64_t>(8, n - i0);
    int64_t x[8], y[8];
    const uint8_t valid = load8(a, i0, nrows, x) & load8(b, i0, nrows, y);
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bool t;
      if (ct == CT_I64) {
        const int64_t u = x[j], w = y[j];
        switch (op) {
          case QE_OP_EQ: t = u == w; break;
          case QE_OP_NE: t = u != w; break;
          case QE_OP_LT: t = u < w; break;
          case QE_OP_LE: t = u <= w; break;
          case QE_OP_GT: t = u > w; break;
          default: t = u >= w;
        }
      } else {
        const double u = as_f64(a, x[j]), w = as_f64(b, y[j]);
        switch (op) {
          case QE_OP_EQ: t = u == w; break;
          case QE_OP_NE: t = u != w; break;
          case QE_OP_LT: t = u < w; break;
          case QE_OP_LE: t = u <= w; break;
          case QE_OP_GT: t = u > w; break;
          default: t = u >= w;
        }
      }
      bits |= (uint32_t)t << j;
    }
    out[g] = (uint8_t)bits & (uint8_t)((1u << nrows) - 1);
    if (out_valid) out_valid[g] = valid;
  }
}

// UTF8 column vs a one-row UTF8 literal: byte equality.
__global__ void __launch_bounds__(256) k_cmp_utf8(const int32_t* __restrict__ offs, const uint8_t* __restrict__ bytes,
                                                  const uint8_t* __restrict__ valid_in, const uint8_t* __restrict__ lit,
                                                  int32_t lit_len, int32_t negate, uint8_t* __restrict__ out,
                                                  uint8_t* __restrict__ out_valid, int64_t n) {
  const int64_t ngroups = (n + 7) >> 3;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = g << 3;
    const int nrows = (int)min<int64_t>(8, n - i0);
    uint32_t bits = 0;
    for (int j = 0; j < nrows; ++j) {
      const int32_t s = offs[i0 + j], e = offs[i0 + j + 1];
      bool eq = (e - s) == lit_len;
      for (int32_t k = 0; eq && k < lit_len; ++k) eq = bytes[s + k] == lit[k];
      bits |= (uint32_t)(eq != (negate != 0)) << j;
    }
    out[g] = (uint8_t)bits;
    if (out_valid) out_valid[g] = (valid_in ? valid_in[g] : (uint8_t)0xFF) & (uint8_t)((1u << nrows) - 1);
  }
}

// Three-valued boolean logic on bitmaps, one byte (8 rows) per thread.
__global__ void __launch_bounds__(256) k_bool(const uint8_t* __restrict__ av, const uint8_t* __restrict__ avalid,
                                              const uint8_t* __restrict__ bv, const uint8_t* __restrict__ bvalid,
                                              int32_t op, uint8_t* __restrict__ out, uint8_t* __restrict__ out_valid,
                                              int64_t n) {
  const int64_t nbytes = (n + 7) >> 3;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nbytes;
       g += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t tail = (g == nbytes - 1 && (n & 7)) ? (uint8_t)((1u << (n & 7)) - 1) : (uint8_t)0xFF;
    const uint8_t a = av ? av[g] : 0, la = avalid ? avalid[g] : 0xFF;
    const uint8_t b = bv ? bv[g] : 0, lb = bvalid ? bvalid[g] : 0xFF;
    uint8_t r, l;
    switch (op) {
      case QE_OP_AND:  // false AND null = false
        r = a & b;
        l = (la & lb) | (la & ~a) | (lb & ~b);
        break;
      case QE_OP_OR:  // true OR null = true
        r = a | b;
        l = (la & lb) | (la & a) | (lb & b);
        break;
      case QE_OP_NOT:
        r = ~a;
        l = la;
        break;
      case QE_OP_IS_NULL:
        r = ~la;
        l = 0xFF;
        break;
      default:  // QE_OP_IS_NOT_NULL
        r = la;
        l = 0xFF;
    }
    out[g] = r & l & tail;  // canonical: value bit 0 under null
    if (out_valid) out_valid[g] = l & tail;
  }
}

static int grid_for(qe_ctx* ctx, int64_t work_items) {
  const int64_t blocks = (int64_t)div_up((uint64_t)work_items, 256);
  const int64_t cap = (int64_t)ctx->num_cus * 8;
  return (int)(blocks < cap ? (blocks > 0 ? blocks : 1) : cap);
}

// Builds a device Src from an operand, checking shape. `ct` is the compute type.
static int make_src(const qe_operand* o, int64_t n, int32_t ct, Src* s, bool* nullable) {
  QE_CHECK(o != nullptr, QE_ERR_INVALID_ARG, "null operand");
  *s = Src{};
  if (o->col == nullptr) {
    QE_CHECK(o->lit.type == QE_TYPE_INT64 || o->lit.type == QE_TYPE_FLOAT64, QE_ERR_UNSUPPORTED,
             "literal type %d not supported", o->lit.type);
    s->kind = K_LIT;
    s->lit_null = o->lit.is_null;
    if (ct == CT_F64 && o->lit.type == QE_TYPE_INT64)
      s->lit = f64_bits((double)o->lit.bits);
    else
      s->lit = o->lit.bits;
    *nullable = *nullable || o->lit.is_null;
    return QE_OK;
  }
  const qe_column* c = o->col;
  QE_CHECK(c->length == n, QE_ERR_INVALID_ARG, "operand length %lld != %lld", (long long)c->length, (long long)n);
  const int32_t k = kind_of(c->type);
  QE_CHECK(k >= K_I64 && k <= K_U8, QE_ERR_UNSUPPORTED, "column type %d not supported here", c->type);
  QE_CHECK(c->values != nullptr || n == 0, QE_ERR_INVALID_ARG, "null values buffer");
  s->p = c->values;
  s->valid = c->validity;
  s->kind = k;
  *nullable = *nullable || c->validity != nullptr;
  return QE_OK;
}

static int operand_len(const qe_operand* a, const qe_operand* b, int64_t* n) {
  QE_CHECK(a && b, QE_ERR_INVALID_ARG, "null operand");
  if (a->col) *n = a->col->length;
  else if (b->col) *n = b->col->length;
  else return fail(QE_ERR_INVALID_ARG, "at least one operand must be a column");
  return QE_OK;
}

static bool operand_is_f64(const qe_operand* o) {
  return o->col ? o->col->type == QE_TYPE_FLOAT64 : o->lit.type == QE_TYPE_FLOAT64;
}

}  // namespace qe

using namespace qe;

extern "C" {

static int eval_arith(qe_ctx* ctx, int32_t op, const qe_operand* lhs, const qe_operand* rhs, qe_column* out,
                      const int64_t* dn) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(op >= QE_OP_ADD && op <= QE_OP_DIV, QE_ERR_INVALID_ARG, "not an arithmetic op: %d", op);
  int64_t n;
  QE_TRY(operand_len(lhs, rhs, &n));
  const int32_t ct = (operand_is_f64(lhs) || operand_is_f64(rhs)) ? CT_F64 : CT_I64;
  Src a, b;
  bool nullable = false;
  QE_TRY(make_src(lhs, n, ct, &a, &nullable));
  QE_TRY(make_src(rhs, n, ct, &b, &nullable));
  QE_CHECK(out && (out->values || n == 0), QE_ERR_INVALID_ARG, "null output");
  const int32_t want = ct == CT_F64 ? QE_TYPE_FLOAT64 : QE_TYPE_INT64;
  QE_CHECK(out->type == want, QE_ERR_INVALID_ARG, "output type %d, expected %d", out->type, want);
  QE_CHECK(out->length >= n, QE_ERR_CAPACITY, "output holds %lld rows, need %lld", (long long)out->length,
           (long long)n);
  const bool needs_valid = nullable || (ct == CT_I64 && op == QE_OP_DIV);
  QE_CHECK(!needs_valid || out->validity, QE_ERR_INVALID_ARG, "result can be null: output validity buffer required");
  out->length = n;
  if (n == 0) return QE_OK;
  hipLaunchKernelGGL(k_arith, dim3(grid_for(ctx, (n + 7) / 8)), dim3(256), 0, ctx->stream, a, b, op, ct,
                     (int64_t*)out->values, out->validity, n, dn);
  return launch_check("k_arith");
}

int qe_eval_arith(qe_ctx* ctx, int32_t op, const qe_operand* lhs, const qe_operand* rhs, qe_column* out) {
  return eval_arith(ctx, op, lhs, rhs, out, nullptr);
}

int qe_eval_arith_dlen(qe_ctx* ctx, int32_t op, const qe_operand* lhs, const qe_operand* rhs, qe_column* out,
                       const int64_t* d_len) {
  QE_CHECK(d_len, QE_ERR_INVALID_ARG, "null device row count");
  return eval_arith(ctx, op, lhs, rhs, out, d_len);
}

int qe_eval_cmp(qe_ctx* ctx, int32_t op, const qe_operand* lhs, const qe_operand* rhs, qe_column* out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(op >= QE_OP_EQ && op <= QE_OP_GE, QE_ERR_INVALID_ARG, "not a comparison op: %d", op);
  int64_t n;
  QE_TRY(operand_len(lhs, rhs, &n));
  QE_CHECK(out && (out->values || n == 0) && out->type == QE_TYPE_BOOL, QE_ERR_INVALID_ARG,
           "comparison output must be a BOOL column");
  QE_CHECK(out->length >= n, QE_ERR_CAPACITY, "output holds %lld rows, need %lld", (long long)out->length,
           (long long)n);
  // UTF8 = / != one-row UTF8 literal column.
  if (lhs->col && lhs->col->type == QE_TYPE_UTF8) {
    const qe_column* c = lhs->col;
    QE_CHECK(op == QE_OP_EQ || op == QE_OP_NE, QE_ERR_UNSUPPORTED, "UTF8 supports only = and !=");
    QE_CHECK(rhs->col && rhs->col->type == QE_TYPE_UTF8 && rhs->col->length == 1, QE_ERR_UNSUPPORTED,
             "UTF8 comparison needs a one-row UTF8 literal column on the right");
    QE_CHECK(c->offsets && rhs->col->offsets, QE_ERR_INVALID_ARG, "UTF8 offsets missing");
    QE_CHECK(!c->validity || out->validity, QE_ERR_INVALID_ARG, "output validity buffer required");
    int32_t lo[2];
    QE_HIP(hipMemcpyAsync(lo, rhs->col->offsets, 8, hipMemcpyDeviceToHost, ctx->stream));
    QE_TRY(ctx_sync(ctx));
    out->length = n;
    if (n == 0) return QE_OK;
    hipLaunchKernelGGL(k_cmp_utf8, dim3(grid_for(ctx, (n + 7) / 8)), dim3(256), 0, ctx->stream, c->offsets,
                       (const uint8_t*)c->values, c->validity, (const uint8_t*)rhs->col->values + lo[0],
                       lo[1] - lo[0], op == QE_OP_NE ? 1 : 0, (uint8_t*)out->values, out->validity, n);
    return launch_check("k_cmp_utf8");
  }
  const int32_t ct = (operand_is_f64(lhs) || operand_is_f64(rhs)) ? CT_F64 : CT_I64;
  Src a, b;
  bool nullable = false;
  QE_TRY(make_src(lhs, n, ct, &a, &nullable));
  QE_TRY(make_src(rhs, n, ct, &b, &nullable));
  QE_CHECK(!nullable || out->validity, QE_ERR_INVALID_ARG, "result can be null: output validity buffer required");
  out->length = n;
  if (n == 0) return QE_OK;
  hipLaunchKernelGGL(k_cmp, dim3(grid_for(ctx, (n + 7) / 8)), dim3(256), 0, ctx->stream, a, b, op, ct,
                     (uint8_t*)out->values, out->validity, n);
  return launch_check("k_cmp");
}

int qe_eval_bool(qe_ctx* ctx, int32_t op, const qe_column* lhs, const qe_column* rhs, qe_column* out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(op >= QE_OP_AND && op <= QE_OP_IS_NOT_NULL, QE_ERR_INVALID_ARG, "not a boolean op: %d", op);
  QE_CHECK(lhs != nullptr, QE_ERR_INVALID_ARG, "null lhs");
  const bool binary = op == QE_OP_AND || op == QE_OP_OR;
  const bool null_test = op == QE_OP_IS_NULL || op == QE_OP_IS_NOT_NULL;
  QE_CHECK(null_test || lhs->type == QE_TYPE_BOOL, QE_ERR_UNSUPPORTED, "boolean op on non-BOOL column");
  const int64_t n = lhs->length;
  if (binary) {
    QE_CHECK(rhs && rhs->type == QE_TYPE_BOOL, QE_ERR_UNSUPPORTED, "boolean op on non-BOOL column");
    QE_CHECK(rhs->length == n, QE_ERR_INVALID_ARG, "operand lengths differ");
  }
  QE_CHECK(out && (out->values || n == 0) && out->type == QE_TYPE_BOOL, QE_ERR_INVALID_ARG,
           "boolean output must be a BOOL column");
  QE_CHECK(out->length >= n, QE_ERR_CAPACITY, "output too small");
  const bool nullable = !null_test && (lhs->validity || (binary && rhs->validity));
  QE_CHECK(!nullable || out->validity, QE_ERR_INVALID_ARG, "result can be null: output validity buffer required");
  out->length = n;
  if (n == 0) return QE_OK;
  hipLaunchKernelGGL(k_bool, dim3(grid_for(ctx, (n + 7) / 8)), dim3(256), 0, ctx->stream,
                     null_test ? nullptr : (const uint8_t*)lhs->values, lhs->validity,
                     binary ? (const uint8_t*)rhs->values : nullptr, binary ? rhs->validity : nullptr, op,
                     (uint8_t*)out->values, out->validity, n);
  return launch_check("k_bool");
}

}  // extern "C"
