// TEST INFRASTRUCTURE (SURVEY §5 sanitizers): the device CAST parser (qe_cast_parse.hpp) built for
// the host under AddressSanitizer + UBSan. Reads one string per line on stdin, prints the result
// bits in hex ("NFE" when the string is not a Java double). tests/test_sanitizers.py compares the
// output with the oracle (oracle/cast_ref.py).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "qe_cast_parse.hpp"

int main() {
  using namespace qe::castp;
  static Big A, B;
  std::string line;
  char buf[1 << 16];
  while (fgets(buf, sizeof buf, stdin)) {
    size_t len = strlen(buf);
    if (len && buf[len - 1] == '\n') --len;
    // exact-size heap copy: any read past the string's end is an ASan report
    std::vector<unsigned char> s(buf, buf + len);
    DecScan ds;
    double v = 0.0;
    const int r = parse_fast(s.data(), (int)len, &v, &ds);
    if (r == P_ERR) {
      puts("NFE");
      continue;
    }
    if (r == P_SLOW) {
      const double x = decimal_exact(s.data(), ds, v, A, B);
      v = ds.neg ? -x : x;
    }
    unsigned long long bits;
    memcpy(&bits, &v, 8);
    printf("%016llx\n", bits);
  }
  return 0;
}
