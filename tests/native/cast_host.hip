// TEST INFRASTRUCTURE: the device CAST parser (query-engines_amd/csrc/qe_cast_parse.hpp) compiled
// for the host, so CPU tests check the kernel's algorithm against the oracle without a GPU. Never
// used by the product path (the product has no CPU path).
#include "qe_cast_parse.hpp"

extern "C" int qe_cast_host(const unsigned char* s, int len, double* out, int* slow) {
  using namespace qe::castp;
  DecScan ds;
  double v = 0.0;
  const int r = parse_fast(s, len, &v, &ds);
  *slow = r == P_SLOW;
  if (r == P_ERR) return 1;
  if (r == P_SLOW) {
    static thread_local Big A, B;
    const double x = decimal_exact(s, ds, v, A, B);
    v = ds.neg ? -x : x;
  }
  *out = v;
  return 0;
}

// The register fast path of the CAST kernel (fast_decimal over the value's bytes as two words):
// 1 and *out when it applies, 0 when the kernel falls back to parse_fast.
extern "C" int qe_cast_host_fast(const unsigned char* s, int len, double* out) {
  if (len < 0 || len > 16) return 0;
  uint64_t w0 = 0, w1 = 0;
  for (int k = 0; k < len; ++k) {
    if (k < 8) w0 |= (uint64_t)s[k] << (8 * k);
    else w1 |= (uint64_t)s[k] << (8 * (k - 8));
  }
  return qe::castp::fast_decimal(w0, w1, len, out) ? 1 : 0;
}
