// TEST INFRASTRUCTURE: the exact fp64 SUM accumulator of the hash aggregate (qe_dev.hpp fx_*,
// fxe_*) compiled for the host, so CPU tests check its arithmetic (row images, carries, sign
// changes, wraps, the full-range words E, partial merges in every form, rounding to double) against
// exact rational sums without a GPU. Only the plain (non-atomic) word adds are instantiated here;
// the kernels use the same code with atomics.
#include <hip/hip_runtime.h>

#include "qe_dev.hpp"

using namespace qe;

namespace {
struct Slot {
  qu64 w[4] = {0, 0, 0, 0};
  qu64 st = 0;
  qu64 e[FXE_WORDS] = {};
  qu64* word(int i) { return &w[i]; }
};

// One partial into a slot, dispatched as the global table's gcombine_fx does: RAW / CHUNK forms
// into E, anything else into the words.
void combine(Slot& s, qu64 w0, qu64 w1, qu64 w2, qu64 w3, qu64 st) {
  if (st & (FX_RAW | FX_CHUNK)) {
    fxe_partial<false>(s.e, &s.st, w0, w1, w2, w3, st);
    return;
  }
  fx_add_words<false>([&](int w) { return s.word(w); }, w0, w1, w2, w3, st, &s.st);
}

// A slot merged into another as an exported group is: its record (words and status), then, when it
// has E, one CHUNK record per four words of E (qe_hashagg.hip write_chunk_record).
void merge(Slot& dst, const Slot& src) {
  combine(dst, src.w[0], src.w[1], src.w[2], src.w[3], src.st);
  if (!(src.st & FX_EXT)) return;
  for (int c = 0; c < FXE_CHUNKS; ++c) {
    const qu64* e = src.e + 4 * c;
    const int n = c == FXE_CHUNKS - 1 ? FXE_WORDS - 4 * c : 4;
    combine(dst, e[0], n > 1 ? e[1] : 0, n > 2 ? e[2] : 0, n > 3 ? e[3] : 0, FX_CHUNK | ((qu64)c << 8));
  }
}

void out_words(const Slot& s, unsigned long long* words) {
  for (int i = 0; i < 4; ++i) words[i] = s.w[i];
  words[4] = s.st;
  for (int i = 0; i < FXE_WORDS; ++i) words[5 + i] = s.e[i];
}
}  // namespace

// Sums xs[0..n) into `nslots` slots round-robin by row (slot = i % nslots; a row the words cannot
// hold goes to the slot's E, as the LDS table sends it to the global slot), merges the slots into
// one in the order given by `order` (a permutation of the slots) as exported groups merge, and
// returns fx_result. *err is always 0 (kept for the test's signature); words[39] = the merged words,
// status and E.
extern "C" double qe_fx_host_sum(const double* xs, long n, int nslots, const int* order, int* err, unsigned long long* words) {
  static Slot sl[64];
  *err = 0;
  if (nslots < 1 || nslots > 64) return 0.0;
  for (int k = 0; k < nslots; ++k) sl[k] = Slot{};
  for (long i = 0; i < n; ++i) {
    Slot& s = sl[i % nslots];
    const qi64 b = f64_bits(xs[i]);
    const FxRow r = fx_row(b);
    if (r.st & (FX_HUGE | FX_INEXACT)) {
      qu64 w[5];
      fx_row_words(b, w);  // RAW form
      combine(s, w[0], w[1], w[2], w[3], w[4]);
    } else {
      fx_add_row<false>([&](int w) { return s.word(w); }, r, &s.st);
    }
  }
  Slot tot;
  for (int k = 0; k < nslots; ++k) merge(tot, sl[order[k]]);
  out_words(tot, words);
  return fx_result(tot.w[0], tot.w[1], tot.w[2], tot.w[3], tot.st, tot.e);
}

// The plan-specialised kernels' split: rows that are not fx_rare into `nslots` LDS windows
// (fxw_add), the rest straight into the global slot as one-row partials (fx_row_words: words, or
// RAW for E), then every window merged as a partial (fxw_words). Returns fx_result; words[39] as
// above, *rare = rows that took the global path.
extern "C" double qe_fx_host_window_sum(const double* xs, long n, int nslots, int* err, long* rare,
                                        unsigned long long* words) {
  qu64 win[64][3] = {};
  Slot tot;
  *rare = 0;
  *err = 0;
  if (nslots < 1 || nslots > 64) return 0.0;
  for (long i = 0; i < n; ++i) {
    const qi64 b = f64_bits(xs[i]);
    if (fx_rare(b)) {
      qu64 w[5];
      fx_row_words(b, w);
      combine(tot, w[0], w[1], w[2], w[3], w[4]);
      ++*rare;
    } else {
      qu64* u = win[i % nslots];
      fxw_add<false>([&](int k) { return &u[k]; }, b);
    }
  }
  for (int k = 0; k < nslots; ++k) {
    qu64 v[4];
    fxw_words(win[k][0], win[k][1], win[k][2], v);
    combine(tot, v[0], v[1], v[2], v[3], 0);
  }
  out_words(tot, words);
  return fx_result(tot.w[0], tot.w[1], tot.w[2], tot.w[3], tot.st, tot.e);
}

// The RowVal image of one input (fx_row_words): words[5].
extern "C" void qe_fx_host_row_words(double x, unsigned long long* words) { fx_row_words(f64_bits(x), (qu64*)words); }

// fxe_result of E alone (words W zero): the rounding of a full-range integer in units of 2^-1074.
extern "C" double qe_fx_host_ext_result(const unsigned long long* e) {
  return fxe_result((const qu64*)e, 0, 0, 0, 0, 0);
}
