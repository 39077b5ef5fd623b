// K6: CastExpression UTF-8 -> fp64 (Main.kt:772-805). The reference converts each string with
// Kotlin String.toDouble() = java.lang.Double.parseDouble, whose grammar (Double.valueOf javadoc)
// and correctly rounded result these kernels restate:
//   * leading / trailing chars <= 0x20 are trimmed; empty -> NumberFormatException;
//   * optional sign; "NaN" / "Infinity" (case-sensitive, signed allowed, no suffix);
//   * decimal: digits with at most one '.', at least one digit, optional [eE][+-]?digits;
//   * hex: 0[xX] hexdigits with optional '.', mandatory [pP][+-]?digits binary exponent;
//   * optional trailing [fFdD] type suffix (the value is still parsed as a double);
//   * anything else (Python-style "inf", "1_0", "0x1") is a NumberFormatException;
//   * null input -> null output (K:787-788).
// Rounding is IEEE round-half-even, exactly:
//   k_cast_utf8_f64   one thread per row, no scratch: syntax, NaN/Infinity, hex floats, and the
//                     Clinger fast path (<= 19 significant digits, w <= 2^53, w*10^e a single exact
//                     IEEE operation). Rows needing more set a bit in a "slow" bitmap.
//   k_cast_slow       walks that bitmap; per row, refines a double-arithmetic guess by exact
//                     big-integer comparisons of D*10^e against the midpoints of adjacent doubles.
// HBM traffic per row: 4 B offset + string bytes + 8 B value (+ validity / slow bits).
#include "qe_internal.hpp"
#include "qe_cast_parse.hpp"

namespace qe {

namespace {

using namespace castp;

constexpr int CAST_THREADS = 256;
constexpr int SLOW_THREADS = 64;

// Bytes [p, p + n) of a value of at most 16 bytes as two little-endian words: independent byte
// loads issued together (parse_fast walks its bytes one dependent load at a time).
__device__ __forceinline__ void load16_words(const uint8_t* p, int n, uint64_t* w0, uint64_t* w1) {
  uint64_t a = 0, b = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (k < n) {
      const uint64_t c = p[k];
      if (k < 8) a |= c << (8 * k);
      else b |= c << (8 * (k - 8));
    }
  *w0 = a;
  *w1 = b;
}

// The same from one 16-byte load (p need not be aligned; p + 16 must not pass the end of the
// column's bytes): the byte-by-byte form spent ~5 VALU instructions and a memory instruction per
// byte on address arithmetic and assembly.
__device__ __forceinline__ void load16_words_wide(const uint8_t* p, int n, uint64_t* w0, uint64_t* w1) {
  typedef uint64_t u64_unaligned __attribute__((aligned(1)));  // declared unaligned: no aligned-pointer UB
  uint64_t a = ((const u64_unaligned*)p)[0], b = ((const u64_unaligned*)p)[1];
  if (n < 8) {
    a &= (1ull << (8 * n)) - 1ull;
    b = 0;
  } else if (n < 16) {
    b &= (1ull << (8 * (n - 8))) - 1ull;
  }
  *w0 = a;
  *w1 = b;
}

// 8 rows per thread: one validity byte in; one validity byte and one slow-bitmap byte out.
// One thread per row (a wave = 64 consecutive rows = 8 bitmap bytes): the rows' parses run side
// by side instead of 8 after one another per thread. The output validity and slow-path bitmaps
// are built with ballots, and each byte is written by the lane of its first row.
// (One thread per 8 rows: 117 us for tripdata's 4M fares.)
__global__ void __launch_bounds__(CAST_THREADS) k_cast_utf8_f64(const int32_t* __restrict__ offs,
                                                                const uint8_t* __restrict__ bytes,
                                                                const uint8_t* __restrict__ valid, int64_t n,
                                                                double* __restrict__ out, uint8_t* __restrict__ out_valid,
                                                                uint8_t* __restrict__ slow,
                                                                unsigned long long* __restrict__ err_row,
                                                                unsigned int* __restrict__ nslow) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int32_t end = offs[n];  // the column's bytes: a 16-byte load from s0 stays inside while s0 + 16 <= end
  // every lane runs the same trip count: the ballots below see whole waves
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x - lane; i0 < n; i0 += stride) {
    const int64_t i = i0 + lane;
    const bool in = i < n;
    const bool live = in && (!valid || ((valid[i >> 3] >> (i & 7)) & 1));
    double v = 0.0;
    bool ok = false, sl = false;
    if (live) {
      const int32_t s0 = offs[i], s1 = offs[i + 1];
      uint64_t w0 = 0, w1 = 0;
      if (s1 - s0 <= 16) {
        if (s0 + 16 <= end) load16_words_wide(bytes + s0, s1 - s0, &w0, &w1);
        else load16_words(bytes + s0, s1 - s0, &w0, &w1);
      }
      if (s1 - s0 <= 16 && fast_decimal(w0, w1, s1 - s0, &v)) {
        ok = true;
      } else {
        DecScan ds;
        const int r = parse_fast(bytes + s0, s1 - s0, &v, &ds);
        if (r == P_ERR) {
          atomicMax(err_row, ~(unsigned long long)i);  // (the first failing row: the largest complement)
          v = 0.0;
        } else {
          ok = true;
          sl = r == P_SLOW;
        }
      }
    }
    if (in) out[i] = v;
    const uint64_t okm = __ballot(ok), slm = __ballot(sl);
    if ((lane & 7) == 0 && in) {
      const int64_t g = i >> 3;
      if (out_valid) out_valid[g] = (uint8_t)(okm >> lane);
      slow[g] = (uint8_t)(slm >> lane);
    }
    if (lane == 0 && slm) atomicAdd(nslow, (unsigned int)__popcll(slm));
  }
}

__global__ void __launch_bounds__(SLOW_THREADS) k_cast_slow(const int32_t* __restrict__ offs,
                                                            const uint8_t* __restrict__ bytes, int64_t n,
                                                            double* __restrict__ out, const uint8_t* __restrict__ slow) {
  Big A, B;
  const int64_t ngroups = (n + 7) >> 3;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < ngroups; g += (int64_t)gridDim.x * blockDim.x) {
    uint32_t sb = slow[g];
    while (sb) {
      const int j = __builtin_ctz(sb);
      sb &= sb - 1;
      const int64_t i = (g << 3) + j;
      const int32_t s0 = offs[i], s1 = offs[i + 1];
      DecScan ds;
      double guess = 0.0;
      if (parse_fast(bytes + s0, s1 - s0, &guess, &ds) != P_SLOW) continue;
      const double v = decimal_exact(bytes + s0, ds, guess, A, B);
      out[i] = ds.neg ? -v : v;
    }
  }
}

}  // namespace

}  // namespace qe

using namespace qe;

extern "C" int qe_cast_utf8_to_f64(qe_ctx* ctx, const qe_column* in, qe_column* out, int64_t* error_row) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(in && out, QE_ERR_INVALID_ARG, "null argument");
  QE_CHECK(in->type == QE_TYPE_UTF8 && in->offsets, QE_ERR_UNSUPPORTED, "Cannot cast value to Double: type %d",
           in->type);
  QE_CHECK(out->type == QE_TYPE_FLOAT64, QE_ERR_UNSUPPORTED, "Cast to type %d is not supported", out->type);
  const int64_t n = in->length;
  QE_CHECK(out->length >= n && (out->values || n == 0), QE_ERR_CAPACITY, "output too small");
  QE_CHECK(!in->validity || out->validity, QE_ERR_INVALID_ARG, "output validity buffer required");
  if (error_row) *error_row = -1;
  out->length = n;
  if (n == 0) return QE_OK;
  const int64_t groups = (n + 7) / 8;
  void* s;
  QE_TRY(ctx_scratch(ctx, 16 + (size_t)groups, &s));
  unsigned long long* err = (unsigned long long*)s;  // ~(first failing row), 0: none
  unsigned int* nslow = (unsigned int*)((char*)s + 8);
  uint8_t* slow = (uint8_t*)s + 16;
  QE_HIP(hipMemsetAsync(s, 0, 16, ctx->stream));
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, CAST_THREADS), (int64_t)ctx->num_cus * 16);
  hipLaunchKernelGGL(k_cast_utf8_f64, dim3(grid), dim3(CAST_THREADS), 0, ctx->stream, in->offsets,
                     (const uint8_t*)in->values, in->validity, n, (double*)out->values, out->validity, slow, err, nslow);
  QE_TRY(launch_check("k_cast_utf8_f64"));
  void* hp;  // pinned: the read-back is one DMA, not a staged pageable copy
  QE_TRY(ctx_pinned(ctx, 16, &hp));
  QE_HIP(hipMemcpyAsync(hp, s, 16, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  const uint64_t hdr[2] = {((const uint64_t*)hp)[0], ((const uint64_t*)hp)[1]};
  if (hdr[0] != 0) {
    const uint64_t row = ~hdr[0];
    if (error_row) *error_row = (int64_t)row;
    int32_t o[2] = {0, 0};
    char buf[96] = {0};
    if (hipMemcpy(o, in->offsets + row, 8, hipMemcpyDeviceToHost) == hipSuccess) {
      const int len = std::min(o[1] - o[0], 80);
      if (len > 0) (void)hipMemcpy(buf, (const uint8_t*)in->values + o[0], (size_t)len, hipMemcpyDeviceToHost);
    }
    return fail(QE_ERR_INVALID_ARG, "NumberFormatException: For input string: \"%s\" (row %llu)", buf,
                (unsigned long long)row);
  }
  if ((uint32_t)hdr[1] != 0) {
    const int sgrid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)groups, SLOW_THREADS), (int64_t)ctx->num_cus * 4);
    hipLaunchKernelGGL(k_cast_slow, dim3(sgrid), dim3(SLOW_THREADS), 0, ctx->stream, in->offsets,
                       (const uint8_t*)in->values, n, (double*)out->values, (const uint8_t*)slow);
    QE_TRY(launch_check("k_cast_slow"));
  }
  return QE_OK;
}
