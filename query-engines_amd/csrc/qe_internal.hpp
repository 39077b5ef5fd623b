// Internal definitions shared by the HIP translation units of libqe_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "qe_hip.h"

struct qe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int num_cus = 256;
  void* scratch = nullptr;       // grow-only device scratch
  size_t scratch_bytes = 0;
  void* pinned = nullptr;        // small pinned host buffer for read-backs
  size_t pinned_bytes = 0;
};

namespace qe {

// ---- errors ------------------------------------------------------------------------------
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();

#define QE_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t qe_e_ = (call);                                                         \
    if (qe_e_ != hipSuccess)                                                           \
      return ::qe::fail(QE_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(qe_e_)); \
  } while (0)

#define QE_CHECK(cond, code, ...)                  \
  do {                                             \
    if (!(cond)) return ::qe::fail(code, __VA_ARGS__); \
  } while (0)

#define QE_TRY(expr)           \
  do {                         \
    int qe_s_ = (expr);        \
    if (qe_s_ != QE_OK) return qe_s_; \
  } while (0)

int ctx_enter(qe_ctx* ctx);                                   // validates + hipSetDevice
int ctx_scratch(qe_ctx* ctx, size_t bytes, void** out);       // grow-only scratch
int ctx_pinned(qe_ctx* ctx, size_t bytes, void** out);        // grow-only pinned host
int launch_check(const char* what);                           // hipGetLastError wrapper
// Exclusive scan of n int64 on the ctx stream (one block); out[n] = total. (qe_filter.hip)
int exclusive_scan_i64(qe_ctx* ctx, const int64_t* in, int64_t* out, int64_t n);

// ---- type helpers ---------------------------------------------------------------------------
inline int type_width(int32_t t) {
  switch (t) {
    case QE_TYPE_INT64:
    case QE_TYPE_FLOAT64: return 8;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: return 4;
    case QE_TYPE_UINT8: return 1;
    default: return 0;  // BOOL (bits) / UTF8 (var)
  }
}
inline bool is_fixed(int32_t t) { return type_width(t) > 0; }
inline bool is_integral(int32_t t) {
  return t == QE_TYPE_INT64 || t == QE_TYPE_INT32 || t == QE_TYPE_DATE32 || t == QE_TYPE_UINT8;
}

// Operand kinds understood by the device loaders (uniform per launch).
enum SrcKind : int32_t { K_LIT = 0, K_I64 = 1, K_F64 = 2, K_I32 = 3, K_U8 = 4, K_BOOL = 5 };

inline int32_t kind_of(int32_t type) {
  switch (type) {
    case QE_TYPE_INT64: return K_I64;
    case QE_TYPE_FLOAT64: return K_F64;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: return K_I32;
    case QE_TYPE_UINT8: return K_U8;
    case QE_TYPE_BOOL: return K_BOOL;
    default: return -1;
  }
}

inline uint64_t div_up(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// ---- hashing / generator (bit-for-bit restated in oracle/gen.py) ----------------------------
constexpr uint64_t PHI64 = 0x9E3779B97F4A7C15ull;

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + PHI64;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint64_t gen_u64(uint64_t seed, uint64_t col, uint64_t row) {
  return splitmix64(seed ^ (col * PHI64) ^ row);
}

// murmur3 finaliser: partition hash for the multi-GPU exchange and the global table.
__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}

// Cheap slot hash for the per-workgroup LDS table: one 32-bit multiply (Fibonacci hashing).
__device__ __forceinline__ uint32_t lds_hash(uint64_t key) {
  uint32_t x = (uint32_t)key ^ (uint32_t)(key >> 32) * 0x85EBCA6Bu;
  return x * 0x9E3779B1u;
}

__host__ __device__ __forceinline__ int64_t f64_bits(double d) {
  int64_t b;
  memcpy(&b, &d, 8);
  return b;
}
__host__ __device__ __forceinline__ double bits_f64(int64_t b) {
  double d;
  memcpy(&d, &b, 8);
  return d;
}

// Order-preserving int64 key of a non-NaN double with +0.0 and -0.0 mapped to the same key
// (they compare equal under IEEE `>`, K:547; the earliest one is tracked separately).
__host__ __device__ __forceinline__ int64_t f64_okey(double d) {
  int64_t b = f64_bits(d == 0.0 ? 0.0 : d);
  return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
}
__host__ __device__ __forceinline__ double okey_f64(int64_t k) {
  int64_t b = k >= 0 ? k : (k ^ 0x7FFFFFFFFFFFFFFFll);
  return bits_f64(b);
}

}  // namespace qe
