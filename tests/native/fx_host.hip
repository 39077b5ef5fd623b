// TEST INFRASTRUCTURE: the exact fp64 SUM accumulator of the hash aggregate (qe_dev.hpp fx_*)
// compiled for the host, so CPU tests check its arithmetic (row images, carries, sign changes,
// wraps, partial merges, rounding to double) against exact rational sums without a GPU. Only the
// plain (non-atomic) word adds are instantiated here; the kernels use the same code with atomics.
#include <hip/hip_runtime.h>

#include "qe_dev.hpp"

using namespace qe;

namespace {
struct Slot {
  qu64 w[4] = {0, 0, 0, 0};
  qu64 st = 0;
  qu64* word(int i) { return &w[i]; }
};
}  // namespace

// Sums xs[0..n) into `nslots` slots round-robin by row (slot = i % nslots), merges the slots into
// one with fx_add_words in the order given by `order` (a permutation of the slots), and returns
// the result of fx_result (nn = n): *err as fx_result reports, words[5] = the merged words + status.
extern "C" double qe_fx_host_sum(const double* xs, long n, int nslots, const int* order, int* err, unsigned long long* words) {
  Slot sl[64];
  if (nslots < 1 || nslots > 64) return 0.0;
  for (long i = 0; i < n; ++i) {
    Slot& s = sl[i % nslots];
    const FxRow r = fx_row(f64_bits(xs[i]));
    fx_add_row<false>([&](int w) { return s.word(w); }, r, &s.st);
  }
  Slot tot;
  for (int k = 0; k < nslots; ++k) {
    Slot& s = sl[order[k]];
    fx_add_words<false>([&](int w) { return tot.word(w); }, s.w[0], s.w[1], s.w[2], s.w[3], s.st, &tot.st);
  }
  for (int i = 0; i < 4; ++i) words[i] = tot.w[i];
  words[4] = tot.st;
  bool e = false;
  const double v = fx_result(tot.w[0], tot.w[1], tot.w[2], tot.w[3], tot.st, (qu64)n, &e);
  *err = e;
  return v;
}

// The plan-specialised kernels' split: rows that are not fx_rare into `nslots` LDS windows
// (fxw_add), the rest straight into the global accumulator as one-row partials (fx_row_words),
// then every window merged as a partial (fxw_words). Returns fx_result; words[5] as above,
// *rare = rows that took the global path.
extern "C" double qe_fx_host_window_sum(const double* xs, long n, int nslots, int* err, long* rare,
                                        unsigned long long* words) {
  qu64 win[64][3] = {};
  Slot tot;
  *rare = 0;
  if (nslots < 1 || nslots > 64) return 0.0;
  for (long i = 0; i < n; ++i) {
    const qi64 b = f64_bits(xs[i]);
    if (fx_rare(b)) {
      qu64 w[5];
      fx_row_words(b, w);
      fx_add_words<false>([&](int k) { return tot.word(k); }, w[0], w[1], w[2], w[3], w[4], &tot.st);
      ++*rare;
    } else {
      qu64* u = win[i % nslots];
      fxw_add<false>([&](int k) { return &u[k]; }, b);
    }
  }
  for (int k = 0; k < nslots; ++k) {
    qu64 v[4];
    fxw_words(win[k][0], win[k][1], win[k][2], v);
    fx_add_words<false>([&](int w) { return tot.word(w); }, v[0], v[1], v[2], v[3], 0, &tot.st);
  }
  for (int i = 0; i < 4; ++i) words[i] = tot.w[i];
  words[4] = tot.st;
  bool e = false;
  const double v = fx_result(tot.w[0], tot.w[1], tot.w[2], tot.w[3], tot.st, (qu64)n, &e);
  *err = e;
  return v;
}

// The same split with the limb window (fxl_add / fxl_partial, the kernels' default).
extern "C" double qe_fx_host_limb_sum(const double* xs, long n, int nslots, int* err, long* rare,
                                      unsigned long long* words) {
  qu64 win[64][FXL_WORDS] = {};
  Slot tot;
  *rare = 0;
  if (nslots < 1 || nslots > 64) return 0.0;
  for (long i = 0; i < n; ++i) {
    const qi64 b = f64_bits(xs[i]);
    if (fx_rare(b)) {
      qu64 w[5];
      fx_row_words(b, w);
      fx_add_words<false>([&](int k) { return tot.word(k); }, w[0], w[1], w[2], w[3], w[4], &tot.st);
      ++*rare;
    } else {
      qu64* u = win[i % nslots];
      fxl_add<false>([&](int k) { return &u[k]; }, b);
    }
  }
  for (int k = 0; k < nslots; ++k) {
    qu64 v[4], st;
    fxl_partial(win[k][0], win[k][1], win[k][2], win[k][3], win[k][4], win[k][5], v, &st);
    fx_add_words<false>([&](int w) { return tot.word(w); }, v[0], v[1], v[2], v[3], st, &tot.st);
  }
  for (int i = 0; i < 4; ++i) words[i] = tot.w[i];
  words[4] = tot.st;
  bool e = false;
  const double v = fx_result(tot.w[0], tot.w[1], tot.w[2], tot.w[3], tot.st, (qu64)n, &e);
  *err = e;
  return v;
}

// The RowVal image of one input (fx_row_words): words[5].
extern "C" void qe_fx_host_row_words(double x, unsigned long long* words) { fx_row_words(f64_bits(x), (qu64*)words); }
