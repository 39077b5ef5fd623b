// Java Double.parseDouble restated for CAST(utf8 AS double) (Main.kt:791 String.toDouble()).
// Host+device: the kernels in qe_cast.hip call it on the GPU; tests/native/cast_host.hip compiles
// the same code for the host so tests can check the algorithm against the oracle without a GPU.
// Grammar and rounding are documented in qe_cast.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "qe_dev.hpp"

#define QE_HD __host__ __device__

namespace qe {
namespace castp {

constexpr int BIG_LIMBS = 160;  // 5120 bits: D (<= 800 digits) * 5^k * 2^s covers every double
constexpr int MAX_SIG_DIGITS = 800;

enum : int { P_ERR = 0, P_DONE = 1, P_SLOW = 2 };

// Syntax scan of one decimal string that needs the exact path.
struct DecScan {
  int first;    // index of the first significant digit
  int end;      // index after the last mantissa character
  int nd;       // significant digits kept (<= MAX_SIG_DIGITS, trailing zeros stripped)
  bool sticky;  // nonzero digits dropped beyond MAX_SIG_DIGITS
  bool neg;
  int64_t e10;  // |value| = D * 10^e10, D = the nd kept digits
};

QE_HD inline bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
QE_HD inline int hexval(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

QE_HD bool match_to_end(const uint8_t* s, int i, int len, const char* lit) {
  int k = 0;
  for (; lit[k]; ++k)
    if (i + k >= len || s[i + k] != (uint8_t)lit[k]) return false;
  return i + k == len;
}

// Round H * 2^e2 (H != 0; `sticky`: nonzero bits dropped below H) to the nearest double.
QE_HD double round_binary(uint64_t H, int e2, bool sticky) {
  const int top = 63 - __builtin_clzll(H);
  if (top + e2 > 1023) return __builtin_inf();
  int drop = top - 52;                       // normal: keep 53 bits
  if (drop < -1074 - e2) drop = -1074 - e2;  // subnormal: lsb weight 2^-1074
  uint64_t q;
  if (drop <= 0) {
    q = H << (-drop);
  } else if (drop > 64) {
    q = 0;
  } else if (drop == 64) {
    const bool half = (H >> 63) & 1, rest = (H << 1) != 0 || sticky;
    q = (half && rest) ? 1 : 0;
  } else {
    q = H >> drop;
    const uint64_t rem = H & ((1ull << drop) - 1), halfv = 1ull << (drop - 1);
    if (rem > halfv || (rem == halfv && (sticky || (q & 1)))) ++q;
  }
  return ldexp((double)q, e2 + drop);
}

// The common decimal form from registers: [+-] digits [. digits] (at least one digit, at most 15
// in all, no other byte) is m / 10^k with m < 2^53 and k <= 15, both exact doubles, so the one
// IEEE division is the correctly rounded value — what Double.parseDouble returns (K:791). Anything
// else (whitespace, exponent, suffix, NaN / Infinity, hex, more digits) -> false: parse_fast.
QE_HD inline bool fast_decimal(uint64_t w0, uint64_t w1, int n, double* out) {
  if (n <= 0 || n > 16) return false;
  int i = 0;
  uint32_t c0 = (uint32_t)(w0 & 0xFF);
  const bool neg = c0 == '-';
  if (c0 == '-' || c0 == '+') i = 1;
  uint64_t m = 0;
  int digits = 0, frac = -1;
  for (; i < n; ++i) {
    const uint32_t c = (uint32_t)((i < 8 ? w0 >> (8 * i) : w1 >> (8 * (i - 8))) & 0xFF);
    if (c >= '0' && c <= '9') {
      m = m * 10 + (c - '0');
      ++digits;
      if (frac >= 0) ++frac;
    } else if (c == '.' && frac < 0) {
      frac = 0;
    } else {
      return false;
    }
  }
  if (digits == 0 || digits > 15) return false;
  double p10 = 1.0;  // 10^frac, exact (<= 10^15) and built without a table (a dynamically indexed
  for (int k = 0; k < frac; ++k) p10 *= 10.0;  // local array would live in scratch memory)
  double v = (double)m;
  if (frac > 0) v = v / p10;
  *out = neg ? -v : v;
  return true;
}

// Syntax + every case except the exact decimal path. Returns P_ERR, P_DONE (*out set) or P_SLOW
// (*ds filled, *out = a guess of |value| within a few ulps).
QE_HD int parse_fast(const uint8_t* s, int len, double* out, DecScan* ds) {
  int i = 0;
  while (len > 0 && s[len - 1] <= 0x20) --len;
  while (i < len && s[i] <= 0x20) ++i;
  if (i >= len) return P_ERR;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') {
    neg = s[i] == '-';
    ++i;
  }
  if (i >= len) return P_ERR;
  if (s[i] == 'N') {
    if (!match_to_end(s, i, len, "NaN")) return P_ERR;
    *out = __builtin_nan("");
    return P_DONE;
  }
  if (s[i] == 'I') {
    if (!match_to_end(s, i, len, "Infinity")) return P_ERR;
    *out = neg ? -__builtin_inf() : __builtin_inf();
    return P_DONE;
  }
  int end = len;  // optional type suffix
  if (s[end - 1] == 'f' || s[end - 1] == 'F' || s[end - 1] == 'd' || s[end - 1] == 'D') --end;
  if (end - i >= 2 && s[i] == '0' && (s[i + 1] == 'x' || s[i + 1] == 'X')) {
    // ---- 0x H* [. H*] p [+-] D+  (at least one hex digit)
    int j = i + 2, nh = 0, sig = 0, frac = 0, int_dropped = 0;
    uint64_t H = 0;
    bool sticky = false, dot = false;
    for (; j < end; ++j) {
      if (s[j] == '.') {
        if (dot) return P_ERR;
        dot = true;
        continue;
      }
      const int v = hexval(s[j]);
      if (v < 0) break;
      ++nh;
      if (sig == 0 && v == 0) {
        if (dot) ++frac;
      } else if (sig < 15) {
        H = (H << 4) | (uint64_t)v;
        ++sig;
        if (dot) ++frac;
      } else {
        if (v) sticky = true;
        if (!dot) ++int_dropped;
      }
    }
    if (nh == 0 || j >= end || (s[j] != 'p' && s[j] != 'P')) return P_ERR;
    ++j;
    bool eneg = false;
    if (j < end && (s[j] == '+' || s[j] == '-')) {
      eneg = s[j] == '-';
      ++j;
    }
    if (j >= end) return P_ERR;
    int64_t pe = 0;
    for (; j < end; ++j) {
      if (!is_digit(s[j])) return P_ERR;
      if (pe < 100000) pe = pe * 10 + (s[j] - '0');
    }
    if (eneg) pe = -pe;
    double v = 0.0;
    if (H != 0) {
      int64_t e2 = pe - 4 * (int64_t)frac + 4 * (int64_t)int_dropped;
      e2 = e2 > 4000 ? 4000 : (e2 < -4000 ? -4000 : e2);
      v = round_binary(H, (int)e2, sticky);
    }
    *out = neg ? -v : v;
    return P_DONE;
  }
  // ---- D* [. D*] [eE [+-] D+]  (at least one digit)
  int j = i, nd_all = 0, point = -1;
  for (; j < end; ++j) {
    if (s[j] == '.') {
      if (point >= 0) return P_ERR;
      point = nd_all;
      continue;
    }
    if (!is_digit(s[j])) break;
    ++nd_all;
  }
  if (nd_all == 0) return P_ERR;
  const int mant_end = j;
  if (point < 0) point = nd_all;
  int64_t ex = 0;
  if (j < end) {
    if (s[j] != 'e' && s[j] != 'E') return P_ERR;
    ++j;
    bool eneg = false;
    if (j < end && (s[j] == '+' || s[j] == '-')) {
      eneg = s[j] == '-';
      ++j;
    }
    if (j >= end) return P_ERR;
    for (; j < end; ++j) {
      if (!is_digit(s[j])) return P_ERR;
      if (ex < 10000000) ex = ex * 10 + (s[j] - '0');
    }
    if (eneg) ex = -ex;
  }
  // significant digits: skip leading zeros; keep <= MAX_SIG_DIGITS; strip trailing zeros
  int lead = 0, nd = 0, nz = 0, first = -1;
  bool sticky = false;
  uint64_t w = 0;  // first 19 significant digits
  for (int k = i; k < mant_end; ++k) {
    if (s[k] == '.') continue;
    const int d = s[k] - '0';
    if (first < 0) {
      if (d == 0) {
        ++lead;
        continue;
      }
      first = k;
    }
    if (nd < MAX_SIG_DIGITS) {
      if (nd < 19) w = w * 10 + (uint64_t)d;
      ++nd;
      if (d) nz = nd;
    } else if (d) {
      sticky = true;
    }
  }
  if (first < 0) {
    *out = neg ? -0.0 : 0.0;
    return P_DONE;
  }
  int64_t e10 = ex + (int64_t)point - lead - nd;
  if (!sticky) {  // trailing zeros move into the exponent
    for (int k = nz; k < nd && k < 19; ++k) w /= 10;
    e10 += nd - nz;
    nd = nz;
  }
  const int64_t mag = e10 + nd;  // |value| in [10^(mag-1), 10^mag)
  if (mag > 310) {
    *out = neg ? -__builtin_inf() : __builtin_inf();
    return P_DONE;
  }
  if (mag < -343) {
    *out = neg ? -0.0 : 0.0;
    return P_DONE;
  }
  if (nd <= 19 && !sticky && w <= (1ull << 53)) {
    constexpr double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    double v = 0.0;
    bool ok = false;
    if (e10 >= 0 && e10 <= 22) {
      v = (double)w * p10[e10];
      ok = true;
    } else if (e10 < 0 && e10 >= -22) {
      v = (double)w / p10[-e10];
      ok = true;
    } else if (e10 > 22 && e10 <= 22 + 16) {
      uint64_t ww = w;  // w * 10^(e10-22) still exact below 2^53 ?
      ok = true;
      for (int k = 0; k < e10 - 22; ++k) {
        if (ww > (1ull << 53) / 10) {
          ok = false;
          break;
        }
        ww *= 10;
      }
      v = (double)ww * 1e22;
    }
    if (ok) {
      *out = neg ? -v : v;
      return P_DONE;
    }
  }
  ds->first = first;
  ds->end = mant_end;
  ds->nd = nd;
  ds->sticky = sticky;
  ds->neg = neg;
  ds->e10 = e10;
  // guess from the first <= 19 digits in double arithmetic (a few ulps off; refined exactly)
  const int nw = nd < 19 ? nd : 19;
  const int64_t ge = e10 + (nd - nw), h = ge / 2;
  *out = (double)w * pow(10.0, (double)h) * pow(10.0, (double)(ge - h));
  return P_SLOW;
}

// ---- exact path ------------------------------------------------------------------------------------
struct Big {
  uint32_t d[BIG_LIMBS];
  int n;
};

QE_HD void big_mul_add(Big& b, uint32_t m, uint32_t a) {
  uint64_t carry = a;
  for (int i = 0; i < b.n; ++i) {
    const uint64_t t = (uint64_t)b.d[i] * m + carry;
    b.d[i] = (uint32_t)t;
    carry = t >> 32;
  }
  if (carry && b.n < BIG_LIMBS) b.d[b.n++] = (uint32_t)carry;
}

QE_HD void big_mul_pow5(Big& b, int k) {
  for (; k >= 13; k -= 13) big_mul_add(b, 1220703125u, 0);  // 5^13
  uint32_t m = 1;
  while (k-- > 0) m *= 5;
  if (m != 1) big_mul_add(b, m, 0);
}

QE_HD void big_shl(Big& b, int bits) {
  if (b.n == 0 || bits <= 0) return;
  const int limbs = bits >> 5, sh = bits & 31;
  if (sh) {
    uint32_t carry = 0;
    for (int i = 0; i < b.n; ++i) {
      const uint32_t v = b.d[i];
      b.d[i] = (v << sh) | carry;
      carry = v >> (32 - sh);
    }
    if (carry && b.n < BIG_LIMBS) b.d[b.n++] = carry;
  }
  if (limbs) {
    const int nn = b.n + limbs < BIG_LIMBS ? b.n + limbs : BIG_LIMBS;
    for (int i = nn - 1; i >= limbs; --i) b.d[i] = b.d[i - limbs];
    for (int i = 0; i < limbs; ++i) b.d[i] = 0;
    b.n = nn;
  }
}

QE_HD int big_cmp(const Big& a, const Big& b) {
  int na = a.n, nb = b.n;
  while (na > 0 && a.d[na - 1] == 0) --na;
  while (nb > 0 && b.d[nb - 1] == 0) --nb;
  if (na != nb) return na < nb ? -1 : 1;
  for (int i = na - 1; i >= 0; --i)
    if (a.d[i] != b.d[i]) return a.d[i] < b.d[i] ? -1 : 1;
  return 0;
}

// sign(D * 10^e10 - M * 2^e2), D = the ds.nd significant digits of s (sticky: slightly larger).
QE_HD int cmp_exact(const uint8_t* s, const DecScan& ds, uint64_t M, int e2, Big& A, Big& B) {
  A.d[0] = 0;
  A.n = 1;
  uint32_t chunk = 0, mul = 1;
  int taken = 0;
  for (int k = ds.first; k < ds.end && taken < ds.nd; ++k) {
    if (s[k] == '.') continue;
    chunk = chunk * 10 + (uint32_t)(s[k] - '0');
    mul *= 10;
    ++taken;
    if (mul == 1000000000u) {
      big_mul_add(A, mul, chunk);
      chunk = 0;
      mul = 1;
    }
  }
  if (mul != 1) big_mul_add(A, mul, chunk);
  B.d[0] = (uint32_t)M;
  B.d[1] = (uint32_t)(M >> 32);
  B.n = 2;
  const int e10 = (int)ds.e10;
  if (e10 >= 0) big_mul_pow5(A, e10);
  else big_mul_pow5(B, -e10);
  const int m = e10 < e2 ? e10 : e2;
  big_shl(A, e10 - m);
  big_shl(B, e2 - m);
  const int c = big_cmp(A, B);
  return (c == 0 && ds.sticky) ? 1 : c;
}

// Nearest double to D * 10^e10 (positive), starting from `guess`.
QE_HD double decimal_exact(const uint8_t* s, const DecScan& ds, double guess, Big& A, Big& B) {
  const int64_t INF_BITS = 0x7FF0000000000000ll;
  int64_t b = f64_bits(guess);
  if (!(guess == guess) || b < 0) b = 0;
  if (b >= INF_BITS) b = INF_BITS - 1;  // DBL_MAX
  for (int iter = 0; iter < 1000000; ++iter) {
    const int ef = (int)((b >> 52) & 0x7FF);
    const uint64_t frac = (uint64_t)b & 0xFFFFFFFFFFFFFull;
    const uint64_t M = ef ? (frac | (1ull << 52)) : frac;
    const int E = ef ? ef - 1075 : -1074;
    const int cu = cmp_exact(s, ds, 2 * M + 1, E - 1, A, B);  // vs midpoint to the successor
    if (cu > 0 || (cu == 0 && (M & 1))) {
      if (b + 1 >= INF_BITS) return __builtin_inf();
      ++b;
      continue;
    }
    if (b == 0) return 0.0;
    const bool boundary = frac == 0 && ef > 1;  // predecessor lies in the binade below
    const int cd = boundary ? cmp_exact(s, ds, 4 * M - 1, E - 2, A, B) : cmp_exact(s, ds, 2 * M - 1, E - 1, A, B);
    if (cd < 0 || (cd == 0 && (M & 1))) {
      --b;
      continue;
    }
    break;
  }
  return bits_f64(b);
}

}  // namespace castp
}  // namespace qe
