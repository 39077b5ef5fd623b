// K4a: global (no GROUP BY) aggregate of one column: COUNT(*), COUNT(x), SUM, MIN, MAX, AVG in
// one pass. Restates MaxAccumulator (K:538-561) and its build-defined siblings:
//   * nulls are skipped; all-null (or no rows) -> SUM/MIN/MAX/AVG null;
//   * MAX/MIN keep the first non-null value unless a later one is strictly greater (less):
//     a NaN seed is sticky, a later NaN never wins, and among +0.0/-0.0 ties the earliest row
//     wins. In parallel this is a reduction of (non-NaN ordered key, first-non-null row,
//     first-NaN row, first -0.0 row, first +0.0 row), each a commutative min/max.
//   * int64 SUM wraps (JVM Long); fp64 SUM is the correctly rounded exact sum (math.fsum's value):
//     a Neumaier-compensated tree sum whose error is bounded at the end (sum_certified: the
//     partials also carry sum |x|, the infinite-input count and the summation depth) gives it
//     when the bound shows that every value within the bound rounds to the same double; otherwise
//     a second pass computes the exact sum (k_agg_global_fx, qe_dev.hpp fixed point and
//     full-range words) — in qe_agg_global directly, and for merged pieces through
//     qe_agg_global_exact_partial / qe_agg_global_merge_exact (QE_NEED_EXACT).
// Layout: lane handles rows base + 128q + 2*lane + {0,1} (q = 0..3) so every 16-B load
// instruction of a wave reads one contiguous KiB. Per-block partials are reduced by a second
// single-block kernel in fixed order: bit-reproducible run to run.
// Roofline: HBM read, 8 B/row (+1/8 B validity, +1/8 B mask).
#include <atomic>
#include <chrono>
#include "qe_internal.hpp"

namespace qe {

struct GPart {
  int64_t rows, count;
  int64_t isum, imin, imax;  // integral input
  double s, c;               // Neumaier sum (both input kinds; AVG of int64 uses it)
  double a;                  // sum of |x| or a bound on it (fp64 inputs): the error bound's condition term
  int64_t ninf;              // infinite fp64 inputs
  int64_t kmin, kmax;        // ordered keys of non-NaN fp64
  uint64_t first_nn, first_nan, first_negz, first_posz;
  int64_t depth;  // summation depth of s and c before this partial's last fold (set by the host)
};

__device__ __forceinline__ void gpart_init(GPart& p) {
  p.rows = p.count = 0;
  p.isum = 0;
  p.imin = INT64_MAX;
  p.imax = INT64_MIN;
  p.s = p.c = 0.0;
  p.a = 0.0;
  p.ninf = 0;
  p.kmin = INT64_MAX;
  p.kmax = INT64_MIN;
  p.first_nn = p.first_nan = p.first_negz = p.first_posz = UINT64_MAX;
  p.depth = 0;
}

__device__ __forceinline__ void neumaier_add(double& s, double& c, double x) {
  const double t = s + x;
  c += (fabs(s) >= fabs(x)) ? ((s - t) + x) : ((x - t) + s);
  s = t;
}

// Knuth's two-sum (s + x = t + err exactly, no compare or select): the dense kernel's row step.
__device__ __forceinline__ void two_sum_add(double& s, double& c, double x) {
  const double t = s + x, bp = t - s;
  c += (s - (t - bp)) + (x - bp);
  s = t;
}

__device__ __forceinline__ void gpart_merge(GPart& a, const GPart& b) {
  a.rows += b.rows;
  a.count += b.count;
  a.isum = (int64_t)((uint64_t)a.isum + (uint64_t)b.isum);
  a.imin = min(a.imin, b.imin);
  a.imax = max(a.imax, b.imax);
  a.c += b.c;
  neumaier_add(a.s, a.c, b.s);
  a.a += b.a;
  a.ninf += b.ninf;
  a.kmin = min(a.kmin, b.kmin);
  a.kmax = max(a.kmax, b.kmax);
  a.first_nn = min(a.first_nn, b.first_nn);
  a.first_nan = min(a.first_nan, b.first_nan);
  a.first_negz = min(a.first_negz, b.first_negz);
  a.first_posz = min(a.first_posz, b.first_posz);
  a.depth = max(a.depth, b.depth);
}

template <typename T>
__device__ __forceinline__ T shfl_x(T v, int m) {
  return __shfl_xor(v, m);
}

__device__ __forceinline__ void gpart_wave_reduce(GPart& p) {
  for (int m = 32; m > 0; m >>= 1) {
    GPart o;
    o.rows = shfl_x(p.rows, m);
    o.count = shfl_x(p.count, m);
    o.isum = shfl_x(p.isum, m);
    o.imin = shfl_x(p.imin, m);
    o.imax = shfl_x(p.imax, m);
    o.s = shfl_x(p.s, m);
    o.c = shfl_x(p.c, m);
    o.a = shfl_x(p.a, m);
    o.ninf = shfl_x(p.ninf, m);
    o.kmin = shfl_x(p.kmin, m);
    o.kmax = shfl_x(p.kmax, m);
    o.first_nn = (uint64_t)shfl_x((int64_t)p.first_nn, m);
    o.first_nan = (uint64_t)shfl_x((int64_t)p.first_nan, m);
    o.first_negz = (uint64_t)shfl_x((int64_t)p.first_negz, m);
    o.first_posz = (uint64_t)shfl_x((int64_t)p.first_posz, m);
    o.depth = shfl_x(p.depth, m);
    // fixed pairing order: the lower lane's partial is the left operand (operands selected, one
    // merge: a branch on the lane bit ran both merges in every wave)
    const bool hi = (threadIdx.x & m) != 0;
    GPart l, r;
    l.rows = hi ? o.rows : p.rows;           r.rows = hi ? p.rows : o.rows;
    l.count = hi ? o.count : p.count;        r.count = hi ? p.count : o.count;
    l.isum = hi ? o.isum : p.isum;           r.isum = hi ? p.isum : o.isum;
    l.imin = hi ? o.imin : p.imin;           r.imin = hi ? p.imin : o.imin;
    l.imax = hi ? o.imax : p.imax;           r.imax = hi ? p.imax : o.imax;
    l.s = hi ? o.s : p.s;                    r.s = hi ? p.s : o.s;
    l.c = hi ? o.c : p.c;                    r.c = hi ? p.c : o.c;
    l.a = hi ? o.a : p.a;                    r.a = hi ? p.a : o.a;
    l.ninf = hi ? o.ninf : p.ninf;           r.ninf = hi ? p.ninf : o.ninf;
    l.kmin = hi ? o.kmin : p.kmin;           r.kmin = hi ? p.kmin : o.kmin;
    l.kmax = hi ? o.kmax : p.kmax;           r.kmax = hi ? p.kmax : o.kmax;
    l.first_nn = hi ? o.first_nn : p.first_nn;       r.first_nn = hi ? p.first_nn : o.first_nn;
    l.first_nan = hi ? o.first_nan : p.first_nan;    r.first_nan = hi ? p.first_nan : o.first_nan;
    l.first_negz = hi ? o.first_negz : p.first_negz; r.first_negz = hi ? p.first_negz : o.first_negz;
    l.first_posz = hi ? o.first_posz : p.first_posz; r.first_posz = hi ? p.first_posz : o.first_posz;
    l.depth = hi ? o.depth : p.depth;                r.depth = hi ? p.depth : o.depth;
    gpart_merge(l, r);
    p = l;
  }
}

typedef long long i64x2 __attribute__((ext_vector_type(2)));

template <bool IS_F64>
__global__ void __launch_bounds__(256) k_agg_global(const int64_t* __restrict__ vals, const uint8_t* __restrict__ valid,
                                                    const uint8_t* __restrict__ mv, const uint8_t* __restrict__ ml,
                                                    int64_t n, GPart* __restrict__ partials) {
  GPart p;
  gpart_init(p);
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t base = wave * 512; base < n; base += nwaves * 512) {
    const bool full = base + 512 <= n;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t r0 = base + 128 * q + 2 * lane;
      int64_t v0 = 0, v1 = 0;
      if (full) {
        const i64x2 t = *(const i64x2*)(vals + r0);
        v0 = t.x;
        v1 = t.y;
      } else {
        if (r0 < n) v0 = vals[r0];
        if (r0 + 1 < n) v1 = vals[r0 + 1];
      }
      const int sh = (int)(r0 & 7);
      uint32_t inrange = full ? 3u : (uint32_t)((r0 < n) | ((r0 + 1 < n) << 1));
      uint32_t sel = inrange;
      // bitmaps are read only for rows < n: an input bitmap may be Arrow-minimal (ceil(n/8) B)
      if (mv && sel) {
        uint32_t m = (uint32_t)(mv[r0 >> 3] >> sh);
        if (ml) m &= (uint32_t)(ml[r0 >> 3] >> sh);
        sel &= m;
      }
      const uint32_t nn = valid && sel ? (sel & (uint32_t)(valid[r0 >> 3] >> sh)) : sel;
      p.rows += __popc(sel & 3u);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (!((nn >> j) & 1)) continue;
        const int64_t x = j ? v1 : v0;
        const uint64_t row = (uint64_t)(r0 + j);
        p.count += 1;
        p.first_nn = min(p.first_nn, row);
        if (IS_F64) {
          const double d = bits_f64(x);
          neumaier_add(p.s, p.c, d);
          p.a += fabs(d);
          if (__builtin_isinf(d)) p.ninf += 1;
          if (d != d) {
            p.first_nan = min(p.first_nan, row);
          } else {
            const int64_t k = f64_okey(d);
            p.kmin = min(p.kmin, k);
            p.kmax = max(p.kmax, k);
            if (d == 0.0) {
              if (x < 0) p.first_negz = min(p.first_negz, row);
              else p.first_posz = min(p.first_posz, row);
            }
          }
        } else {
          p.isum = (int64_t)((uint64_t)p.isum + (uint64_t)x);
          p.imin = min(p.imin, x);
          p.imax = max(p.imax, x);
          neumaier_add(p.s, p.c, (double)x);
        }
      }
    }
  }
  gpart_wave_reduce(p);
  __shared__ GPart wp[4];
  if (lane == 0) wp[threadIdx.x >> 6] = p;
  __syncthreads();
  if (threadIdx.x == 0) {
    GPart b = wp[0];
    for (int w = 1; w < 4; ++w) gpart_merge(b, wp[w]);
    partials[blockIdx.x] = b;
  }
}

// Dense fp64 column (no validity, no mask): the C3 shape. Eight independent compensated sums per
// thread (one per row slot) break the fp64 add dependency chain that otherwise bounds the
// kernel; min/max run on the doubles with fmin/fmax (which ignore NaN: NaN rows are recorded in a
// rare branch), first-row indices are set on first sight (each thread visits rows in order).
__global__ void __launch_bounds__(256) k_agg_global_f64_dense(const int64_t* __restrict__ vals, int64_t n,
                                                              GPart* __restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  double s[8], c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = c[k] = 0.0;
  double mn = __builtin_inf(), mx = -__builtin_inf();
  int64_t count = 0;
  uint64_t first_nn = UINT64_MAX, first_nan = UINT64_MAX, first_negz = UINT64_MAX, first_posz = UINT64_MAX;
  int64_t ninf = 0;
  for (int64_t base = wave * 512; base < n; base += nwaves * 512) {
    const bool full = base + 512 <= n;
    double d[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t r0 = base + 128 * q + 2 * lane;
      if (full) {
        const i64x2 t = __builtin_nontemporal_load((const i64x2*)(vals + r0));  // once-read stream
        d[2 * q] = bits_f64(t.x);
        d[2 * q + 1] = bits_f64(t.y);
      } else {
        d[2 * q] = r0 < n ? bits_f64(vals[r0]) : 0.0;
        d[2 * q + 1] = r0 + 1 < n ? bits_f64(vals[r0 + 1]) : 0.0;
      }
    }
    if (first_nn == UINT64_MAX) first_nn = (uint64_t)(base + 2 * lane);  // rows base+2*lane.. exist
    if (full) {
      count += 8;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) count += (base + 128 * (k >> 1) + 2 * lane + (k & 1) < n) ? 1 : 0;
    }
    // NaN, +-Inf, zeros (and subnormals) have an exponent field of all ones or zero: (hi + 2^20) &
    // 0x7FE00000 is 0 for exactly those (integer ops on the high word, not fp64 compares)
    uint32_t ex_min = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      two_sum_add(s[k], c[k], d[k]);  // out-of-range rows read as 0.0: no effect on the sum
      const bool in = full || base + 128 * (k >> 1) + 2 * lane + (k & 1) < n;
      const double dm = in ? d[k] : __builtin_nan("");  // fmin/fmax ignore NaN
      mn = fmin(mn, dm);
      mx = fmax(mx, dm);
      const uint32_t hi = (uint32_t)((uint64_t)f64_bits(d[k]) >> 32);
      ex_min = min(ex_min, (hi + 0x00100000u) & 0x7FE00000u);
    }
    if (ex_min == 0) {  // NaN, an infinity or a zero among these 8 rows (rare): exact first-occurrence bookkeeping
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t row = base + 128 * (k >> 1) + 2 * lane + (k & 1);
        if (row >= n) continue;
        if (__builtin_isinf(d[k])) ++ninf;
        if (d[k] != d[k]) first_nan = min(first_nan, (uint64_t)row);
        else if (d[k] == 0.0) {
          if (f64_bits(d[k]) < 0) first_negz = min(first_negz, (uint64_t)row);
          else first_posz = min(first_posz, (uint64_t)row);
        }
      }
    }
  }
  GPart p;
  gpart_init(p);
  p.rows = p.count = count;
  p.first_nn = count ? first_nn : UINT64_MAX;
  p.first_nan = first_nan;
  p.first_negz = first_negz;
  p.first_posz = first_posz;
  // the error bound's sum |x| bounded by count x max|x| from the MIN / MAX already kept (no per-row
  // add; an upper bound keeps the certificate sound — NaN rows certify the IEEE result anyway)
  p.a = count ? (double)count * fmax(fabs(mn), fabs(mx)) : 0.0;
  p.ninf = ninf;
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // fixed fold order
    p.c += c[k];
    neumaier_add(p.s, p.c, s[k]);
  }
  if (mn == mn && count) {  // fmin/fmax skipped NaN; all-NaN leaves the identities (+-inf)
    p.kmin = f64_okey(mn);
    p.kmax = f64_okey(mx);
  }
  if (first_nan != UINT64_MAX && mn == __builtin_inf() && mx == -__builtin_inf()) {
    p.kmin = INT64_MAX;  // only NaNs seen by this thread
    p.kmax = INT64_MIN;
  }
  gpart_wave_reduce(p);
  __shared__ GPart wp[4];
  if (lane == 0) wp[threadIdx.x >> 6] = p;
  __syncthreads();
  if (threadIdx.x == 0) {
    GPart b = wp[0];
    for (int w = 1; w < 4; ++w) gpart_merge(b, wp[w]);
    partials[blockIdx.x] = b;
  }
}

static_assert(sizeof(GPart) <= QE_GLOBAL_PARTIAL_BYTES, "partial record size");

// Row indices of a partial -> global rows (multi-batch / multi-GPU merges keep row order); the
// partial's summation depth for the merge's error bound.
__global__ void k_agg_global_rebase(GPart* __restrict__ p, int64_t row_base, int64_t depth) {
  if (threadIdx.x == 0) {
    p->depth = depth;
    if (p->first_nn != UINT64_MAX) p->first_nn += (uint64_t)row_base;
    if (p->first_nan != UINT64_MAX) p->first_nan += (uint64_t)row_base;
    if (p->first_negz != UINT64_MAX) p->first_negz += (uint64_t)row_base;
    if (p->first_posz != UINT64_MAX) p->first_posz += (uint64_t)row_base;
  }
}

// Packed partial records (QE_GLOBAL_PARTIAL_BYTES apart) -> a GPart array.
__global__ void k_agg_global_unpack(const uint8_t* __restrict__ recs, int n, GPart* __restrict__ out) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = *(const GPart*)(recs + (size_t)i * QE_GLOBAL_PARTIAL_BYTES);
}

// Exact fp64 SUM of the selected non-null rows (the fallback when the compensated sum cannot be
// certified): every thread adds its rows into its own 256-bit fixed-point accumulator in LDS
// (qe_dev.hpp fx_*, plain read-modify-writes) and inputs outside its range (|x| >= 2^126, bits
// below 2^-128) into the workgroup's full-range words E (LDS atomics); the workgroup folds them in
// a fixed tree and one thread adds the result into out[0..4] (w0..w3, status) and out[5..38] (E)
// with device atomics. Integer adds are associative, so the words are the exact sum whatever the
// order. Rare by construction, so it is simple rather than fast.
__global__ void __launch_bounds__(256) k_agg_global_fx(const int64_t* __restrict__ vals, const uint8_t* __restrict__ valid,
                                                       const uint8_t* __restrict__ mv, const uint8_t* __restrict__ ml,
                                                       int64_t n, qu64* __restrict__ out) {
  __shared__ qu64 t[256 * 5];
  __shared__ qu64 e[FXE_WORDS];
  __shared__ int any_e;
  qu64* my = t + threadIdx.x * 5;
  for (int w = 0; w < 5; ++w) my[w] = 0;
  if (threadIdx.x < FXE_WORDS) e[threadIdx.x] = 0;
  if (threadIdx.x == 0) any_e = 0;
  __syncthreads();
  auto wp = [&](int w) { return &my[w]; };
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int sh = (int)(i & 7);
    if (mv) {
      uint32_t m = (uint32_t)(mv[i >> 3] >> sh);
      if (ml) m &= (uint32_t)(ml[i >> 3] >> sh);
      if (!(m & 1u)) continue;
    }
    if (valid && !((valid[i >> 3] >> sh) & 1)) continue;
    const FxRow r = fx_row(vals[i]);
    if (r.st & (FX_HUGE | FX_INEXACT)) {
      fxe_add_value<true>(e, vals[i]);
      any_e = 1;
    } else {
      fx_add_row<false>(wp, r, &my[4]);
    }
  }
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      const qu64* o = t + (threadIdx.x + h) * 5;
      fx_add_words<false>(wp, o[0], o[1], o[2], o[3], o[4], &my[4]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    fx_add_words<true>([&](int w) { return &out[w]; }, my[0], my[1], my[2], my[3], my[4], &out[4]);
    if (any_e) fxe_add_words<true>(out + 5, 0, e, FXE_WORDS);
  }
}

// host_out (optional): pinned host memory that also receives the result, so the caller reads it
// after a stream sync with no device-to-host copy launch.
// host_flag (optional): set once host_out is written, for a host polling it (release, system scope).
// (Round 6 A/B: 1024 threads with one load round and an LDS tree took 16.5-19 us, padded or not;
// docs/experiments.md.)
__global__ void __launch_bounds__(256) k_agg_global_final(GPart* __restrict__ partials, int nparts,
                                                          GPart* __restrict__ host_out,
                                                          unsigned long long* __restrict__ host_flag) {
  // Fixed-order reduction: thread t folds partials t, t+256, ... (two loads in flight per round);
  // then a fixed wave / block tree. (1024 threads took 15 us: sixteen waves' shuffle trees on one CU.)
  GPart p;
  gpart_init(p);
  for (int i = threadIdx.x; i < nparts; i += 512) {
    const GPart a = partials[i];
    GPart b;
    const bool two = i + 256 < nparts;
    if (two) b = partials[i + 256];
    gpart_merge(p, a);
    if (two) gpart_merge(p, b);
  }
  gpart_wave_reduce(p);
  __shared__ GPart wp[4];
  if ((threadIdx.x & 63) == 0) wp[threadIdx.x >> 6] = p;
  __syncthreads();
  if (threadIdx.x == 0) {
    GPart b = wp[0];
    for (int w = 1; w < 4; ++w) gpart_merge(b, wp[w]);
    partials[nparts] = b;
    if (host_out) *host_out = b;
    if (host_flag) __hip_atomic_store(host_flag, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Whether R = fl(s + c) of a partial is the correctly rounded exact sum. Every s update is an
// exact two-sum, so exact = s + sum of the error terms e_i, and c is the plain-float sum of those
// terms: |e_i| <= u |t_i| (t_i the intermediate sums; each input is inside at most D of them, D the
// summation depth) and summing them in a tree of depth D costs at most gamma_D of their total, so
// |s + c - exact| <= eb = (1 + 2Du)^2 (Du)^2 sum|x| (u = 2^-53; doubled for the rounding of sum|x|
// itself). Additions whose result is subnormal are exact, so the bound holds down there too. When
// the exact residual of R = fl(s + c) plus eb stays below half the gap from R to its nearer
// neighbour, every value within eb of s + c rounds to R, the exact sum among them. NaN inputs or
// infinities make R the IEEE result of the exact sum (certified); an overflowed partial (non-finite
// R or sum|x| from finite inputs) is not.
static bool sum_certified(const GPart& p, double r, double depth) {
  if (p.count == 0 || p.first_nan != UINT64_MAX || p.ninf > 0) return true;
  if (!std::isfinite(r) || !std::isfinite(p.a)) return false;
  if (p.a == 0.0) return true;  // every input a zero: s and c are exact
  const double u = 0x1p-53, du = depth * u, g = 1.0 + 2.0 * du;
  const double eb = 2.0 * g * g * du * du * p.a;
  const double bp = r - p.s, resid = (p.s - (r - bp)) + (p.c - bp);  // two-sum: s + c = r + resid exactly
  const double gap = std::min(r - std::nextafter(r, -HUGE_VAL), std::nextafter(r, HUGE_VAL) - r);
  return (std::fabs(resid) + eb) * (1.0 + 0x1p-40) < 0.5 * gap;
}

// Host-side finalisation of MIN/MAX for fp64 (MaxAccumulator order semantics).
static int64_t finalize_f64_minmax(const GPart& p, bool is_max) {
  if (p.first_nan != UINT64_MAX && p.first_nan == p.first_nn) return f64_bits(__builtin_nan(""));
  const double v = okey_f64(is_max ? p.kmax : p.kmin);
  if (v == 0.0) return f64_bits(p.first_negz < p.first_posz ? -0.0 : 0.0);
  return f64_bits(v);
}

}  // namespace qe

using namespace qe;

namespace qe {

// Summation depth of the fold of n partials by k_agg_global_final: thread t folds partials t,
// t + 256, ... (two merges per round), then the wave tree (6) and the block's four waves (3).
static int64_t final_fold_depth(int64_t n) { return 2 * (int64_t)div_up((uint64_t)n, 512) + 2 + 6 + 3; }

// The column's partial, reduced on the device into *result (a GPart in scratch); *depth its
// summation depth (sum_certified): a lane's chain of rows, the dense kernel's fold of its eight
// chains, the wave and block trees, and the final fold of the workgroups' partials.
static int agg_global_partial(qe_ctx* ctx, const qe_column* col, const qe_column* mask, GPart** result,
                              int64_t* depth, GPart* host_out = nullptr, unsigned long long* host_flag = nullptr) {
  QE_CHECK(col, QE_ERR_INVALID_ARG, "null argument");
  QE_CHECK(col->type == QE_TYPE_INT64 || col->type == QE_TYPE_FLOAT64, QE_ERR_UNSUPPORTED,
           "global aggregate over type %d not supported (int64/fp64)", col->type);
  const int64_t n = col->length;
  QE_CHECK(n >= 0 && (col->values || n == 0), QE_ERR_INVALID_ARG, "bad column");
  if (mask) {
    QE_CHECK(mask->type == QE_TYPE_BOOL && mask->length == n, QE_ERR_INVALID_ARG, "mask must be BOOL of equal length");
  }
  const bool f64 = col->type == QE_TYPE_FLOAT64;
  const int64_t waves_needed = (int64_t)div_up((uint64_t)(n > 0 ? n : 1), 512);
  int64_t blocks = (int64_t)div_up((uint64_t)waves_needed, 4);
  // eight workgroups per CU (dense fp64, C3 at 100M rows: 8 -> 0.1427 ms per call, 4 -> 0.1443,
  // 5 -> 0.1642; a one-launch form whose last workgroup folded the partials behind a device-scope
  // fence took 0.153-0.229 ms: docs/experiments.md)
  const int64_t cap = (int64_t)ctx->num_cus * 8;
  const bool dense = col->type == QE_TYPE_FLOAT64 && !col->validity && !mask;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  const int64_t iters = (int64_t)div_up((uint64_t)(n > 0 ? n : 1), (uint64_t)blocks * 4 * 512);
  *depth = (dense ? iters + 8 : 8 * iters) + 6 + 3 + final_fold_depth(blocks);
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)(blocks + 1) * sizeof(GPart), &s));
  GPart* parts = (GPart*)s;
  const uint8_t* mv = mask ? (const uint8_t*)mask->values : nullptr;
  const uint8_t* ml = mask ? mask->validity : nullptr;
  if (f64 && !col->validity && !mv)
    hipLaunchKernelGGL(k_agg_global_f64_dense, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                       (const int64_t*)col->values, n, parts);
  else if (f64)
    hipLaunchKernelGGL(k_agg_global<true>, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                       (const int64_t*)col->values, col->validity, mv, ml, n, parts);
  else
    hipLaunchKernelGGL(k_agg_global<false>, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                       (const int64_t*)col->values, col->validity, mv, ml, n, parts);
  QE_TRY(launch_check("k_agg_global"));
  hipLaunchKernelGGL(k_agg_global_final, dim3(1), dim3(256), 0, ctx->stream, parts, (int)blocks, host_out, host_flag);
  QE_TRY(launch_check("k_agg_global_final"));
  *result = parts + blocks;
  return QE_OK;
}

// Device GPart -> qe_global_agg (synchronises). `h`: the pinned copy the final kernel wrote (no
// copy needed), or null.
// `flag`: the final kernel sets it once h is written; polled instead of synchronising the stream
// (~6 us sooner per call: tools/exp_sync_latency.hip), with a stream query every 50 us so a failed
// kernel still ends the wait. The result is then complete; later work on the stream is ordered
// after the kernel as usual.
static int agg_global_finish(qe_ctx* ctx, const GPart* dp, int32_t type, int64_t depth, qe_global_agg* out,
                             bool* certified, void* h = nullptr, volatile unsigned long long* flag = nullptr) {
  if (!h) {
    QE_TRY(ctx_pinned(ctx, sizeof(GPart), &h));
    QE_HIP(hipMemcpyAsync(h, dp, sizeof(GPart), hipMemcpyDeviceToHost, ctx->stream));
  }
  if (flag) {
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; *flag == 0; ++i) {
      if ((i & 1023) != 0 || std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50)) continue;
      t0 = std::chrono::steady_clock::now();
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipSuccess) {
        QE_CHECK(*flag != 0, QE_ERR_DEVICE, "global aggregate finished without publishing its result");
        break;
      }
      if (e != hipErrorNotReady) return fail(QE_ERR_DEVICE, "global aggregate kernel failed: %s", hipGetErrorString(e));
      (void)hipGetLastError();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  } else {
    QE_TRY(ctx_sync(ctx));
  }
  const GPart p = *(const GPart*)h;
  const bool f64 = type == QE_TYPE_FLOAT64;
  memset(out, 0, sizeof(*out));
  out->rows = p.rows;
  out->count = p.count;
  out->type = type;
  out->valid = p.count > 0 ? 1 : 0;
  const double fsum = std::isfinite(p.s) ? p.s + p.c : p.s;
  *certified = !f64 || sum_certified(p, fsum, (double)(depth + p.depth));
  if (p.count > 0) {
    if (f64) {
      out->sum = f64_bits(fsum);
      out->min = finalize_f64_minmax(p, false);
      out->max = finalize_f64_minmax(p, true);
    } else {
      out->sum = p.isum;
      out->min = p.imin;
      out->max = p.imax;
    }
    out->avg = fsum / (double)p.count;
  }
  return QE_OK;
}

}  // namespace qe

namespace qe {

// The exact fp64 SUM words of a column's selected non-null rows (k_agg_global_fx) into words
// (device, QE_GLOBAL_EXACT_BYTES): W, its status (FX_EXT set: E is always read), E.
static int agg_global_exact(qe_ctx* ctx, const qe_column* col, const qe_column* mask, qu64* words) {
  QE_HIP(hipMemsetAsync(words, 0, QE_GLOBAL_EXACT_BYTES, ctx->stream));
  const int64_t n = col->length;
  if (n == 0 || col->type != QE_TYPE_FLOAT64) return QE_OK;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)div_up((uint64_t)n, 256),
                                                                             (int64_t)ctx->num_cus * 4));
  hipLaunchKernelGGL(k_agg_global_fx, dim3(blocks), dim3(256), 0, ctx->stream, (const int64_t*)col->values,
                     col->validity, mask ? (const uint8_t*)mask->values : nullptr, mask ? mask->validity : nullptr, n,
                     words);
  return launch_check("k_agg_global_fx");
}

// out->sum / out->avg from n exact partials (host copies, QE_GLOBAL_EXACT_BYTES apart).
static void exact_result(const uint8_t* words, int32_t n, qe_global_agg* out) {
  qu64 w[5] = {0, 0, 0, 0, 0}, e[FXE_WORDS] = {};
  for (int32_t i = 0; i < n; ++i) {
    const qu64* p = (const qu64*)(words + (size_t)i * QE_GLOBAL_EXACT_BYTES);
    fx_add_words<false>([&](int k) { return &w[k]; }, p[0], p[1], p[2], p[3], p[4] & ~(qu64)FX_EXT, &w[4]);
    fxe_add_words<false>(e, 0, p + 5, FXE_WORDS);
  }
  if (out->count == 0) return;
  const double v = fx_result(w[0], w[1], w[2], w[3], w[4] | FX_EXT, e);
  out->sum = f64_bits(v);
  out->avg = v / (double)out->count;
}

}  // namespace qe

extern "C" int qe_agg_global(qe_ctx* ctx, const qe_column* col, const qe_column* mask, qe_global_agg* out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out, QE_ERR_INVALID_ARG, "null argument");
  void* h;
  constexpr size_t kFlagOff = (sizeof(GPart) + 63) & ~(size_t)63;
  QE_TRY(ctx_pinned_coherent(ctx, kFlagOff + 64, &h));
  unsigned long long* flag = (unsigned long long*)((uint8_t*)h + kFlagOff);
  *(volatile unsigned long long*)flag = 0;  // (the previous call on this ctx has returned: its kernels wrote it)
  GPart* p;
  int64_t depth;
  QE_TRY(agg_global_partial(ctx, col, mask, &p, &depth, (GPart*)h, flag));
  bool certified = true;
  QE_TRY(agg_global_finish(ctx, p, col->type, depth, out, &certified, h, flag));
  if (certified) return QE_OK;
  // not provably the correctly rounded sum: the exact sum from a second pass over the column
  void* s;
  QE_TRY(ctx_scratch(ctx, QE_GLOBAL_EXACT_BYTES, &s));
  QE_TRY(agg_global_exact(ctx, col, mask, (qu64*)s));
  void* hw;
  QE_TRY(ctx_pinned(ctx, QE_GLOBAL_EXACT_BYTES, &hw));
  QE_HIP(hipMemcpyAsync(hw, s, QE_GLOBAL_EXACT_BYTES, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  exact_result((const uint8_t*)hw, 1, out);
  return QE_OK;
}

extern "C" int qe_agg_global_partial(qe_ctx* ctx, const qe_column* col, const qe_column* mask, int64_t row_base,
                                     void* partial) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(partial && row_base >= 0, QE_ERR_INVALID_ARG, "bad arguments");
  GPart* p;
  int64_t depth;
  QE_TRY(agg_global_partial(ctx, col, mask, &p, &depth));
  hipLaunchKernelGGL(k_agg_global_rebase, dim3(1), dim3(64), 0, ctx->stream, p, row_base, depth);
  QE_TRY(launch_check("k_agg_global_rebase"));
  QE_HIP(hipMemsetAsync(partial, 0, QE_GLOBAL_PARTIAL_BYTES, ctx->stream));
  QE_HIP(hipMemcpyAsync(partial, p, sizeof(GPart), hipMemcpyDeviceToDevice, ctx->stream));
  return QE_OK;
}

extern "C" int qe_agg_global_merge(qe_ctx* ctx, int32_t type, const void* partials, int32_t n, qe_global_agg* out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out && partials && n >= 1 && (type == QE_TYPE_INT64 || type == QE_TYPE_FLOAT64), QE_ERR_INVALID_ARG,
           "bad arguments");
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)(n + 1) * sizeof(GPart), &s));
  GPart* parts = (GPart*)s;
  hipLaunchKernelGGL(k_agg_global_unpack, dim3(1), dim3(256), 0, ctx->stream, (const uint8_t*)partials, n, parts);
  QE_TRY(launch_check("k_agg_global_unpack"));
  // fixed-order fold: the same partials give the same bits on every rank
  void* h;
  QE_TRY(ctx_pinned(ctx, sizeof(GPart), &h));
  hipLaunchKernelGGL(k_agg_global_final, dim3(1), dim3(256), 0, ctx->stream, parts, (int)n, (GPart*)h,
                     (unsigned long long*)nullptr);
  QE_TRY(launch_check("k_agg_global_final"));
  bool certified = true;
  QE_TRY(agg_global_finish(ctx, parts + n, type, final_fold_depth(n), out, &certified, h));
  return certified ? QE_OK : QE_NEED_EXACT;
}

extern "C" int qe_agg_global_exact_partial(qe_ctx* ctx, const qe_column* col, const qe_column* mask, void* words) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(col && words, QE_ERR_INVALID_ARG, "null argument");
  QE_CHECK(col->length >= 0 && (col->values || col->length == 0), QE_ERR_INVALID_ARG, "bad column");
  QE_CHECK(!mask || (mask->type == QE_TYPE_BOOL && mask->length == col->length), QE_ERR_INVALID_ARG,
           "mask must be BOOL of equal length");
  return agg_global_exact(ctx, col, mask, (qu64*)words);
}

extern "C" int qe_agg_global_merge_exact(qe_ctx* ctx, const void* words, int32_t n, qe_global_agg* out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(words && out && n >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  if (out->type != QE_TYPE_FLOAT64) return QE_OK;
  void* hw;
  QE_TRY(ctx_pinned(ctx, (size_t)n * QE_GLOBAL_EXACT_BYTES, &hw));
  QE_HIP(hipMemcpyAsync(hw, words, (size_t)n * QE_GLOBAL_EXACT_BYTES, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  exact_result((const uint8_t*)hw, n, out);
  return QE_OK;
}
