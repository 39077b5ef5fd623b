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
