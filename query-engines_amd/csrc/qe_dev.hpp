// qe_dev.hpp — device-side definitions of the hash-aggregate engine, shared by
//   * the ahead-of-time kernels of libqe_hip.so (hipcc, gfx950), and
//   * the per-plan kernels generated at run time (qe_jit.hip -> hipRTC -> gfx950 code object),
// so both compile exactly the same table layout, probing and combine code.
// Self-contained on purpose: no standard headers (hipRTC compiles it on its own).
#ifndef QE_DEV_HPP
#define QE_DEV_HPP

#ifndef QE_OP_EQ  // comparison op codes (include/qe_hip.h)
#define QE_OP_EQ 10
#define QE_OP_NE 11
#define QE_OP_LT 12
#define QE_OP_LE 13
#define QE_OP_GT 14
#define QE_OP_GE 15
#endif
#ifndef QE_MAX_KEYS
#define QE_MAX_KEYS 4
#define QE_MAX_AGGS 8
#define QE_MAX_COLS 8
#define QE_MAX_TERMS 8
#define QE_MAX_TOKENS 16
#endif
#ifndef QE_AGG_SUM
#define QE_AGG_SUM 1
#define QE_AGG_MIN 2
#define QE_AGG_MAX 3
#define QE_AGG_COUNT 4
#define QE_AGG_COUNT_STAR 5
#define QE_AGG_AVG 6
#endif

namespace qe {

typedef long long qi64;
typedef unsigned long long qu64;
typedef int qi32;
typedef unsigned int qu32;
typedef unsigned short qu16;
typedef unsigned char qu8;
typedef long long qi64x2 __attribute__((ext_vector_type(2)));
typedef int qi32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int qu32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int qu32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int qu32x3 __attribute__((ext_vector_type(3)));

constexpr qi64 EMPTY_KEY = (qi64)0x8000000000000000ull;  // LDS/global slot sentinel (INT64_MIN)
constexpr qi64 PART_EXCL = 1ll << 62;  // partition-aggregate slice flag: the slice holds its whole bucket
constexpr qi64 PART_CH = 2048;          // records per chunk of the chunked scatter (>= its 2048-row tiles)
constexpr qu64 NULL_SALT = 0x6A09E667F3BCC909ull;
constexpr int HA_LDS_MAXP = 32;      // probe limit in the LDS table
constexpr int HA_GLOBAL_MAXP = 256;  // probe limit in the global table

// Operand kinds understood by the device loaders (uniform per launch).
enum SrcKind : int { K_LIT = 0, K_I64 = 1, K_F64 = 2, K_I32 = 3, K_U8 = 4, K_BOOL = 5 };
// ACC_SUM_X: fp64 SUM / AVG of a deterministic state (qe_hashagg_create_ex, QE_HASHAGG_DETERMINISTIC):
// exact fixed-point accumulation in 32-bit limbs (fx_* below), so the result does not depend on the
// order rows, workgroups, passes or ranks are combined in.
enum AccKind : int { ACC_NONE = 0, ACC_SUM_I = 1, ACC_SUM_F = 2, ACC_MIN_I = 3, ACC_MAX_I = 4, ACC_MIN_F = 5, ACC_MAX_F = 6,
                     ACC_SUM_X = 7 };
enum TokOp : int {
  T_COL = 1, T_LIT, T_I2F0, T_I2F1,
  T_ADD_I, T_SUB_I, T_MUL_I, T_DIV_I,
  T_ADD_F, T_SUB_F, T_MUL_F, T_DIV_F
};

// ---- launch description (host fills it; kernels read it as their only argument) ---------------
struct DTok {  // 16 bytes: the Plan (kernel argument) stays under 4 KiB
  short op;
  char lit_null, lit_f64;
  qi32 arg;
  qi64 lit;
};

struct DAgg {
  qi32 fn, acc;
  qi32 pkind;     // 0: no input (COUNT_STAR), 1: column slot, 2: token program, 3: slot OP slot|literal
  qi32 col;       // slot for pkind 1, lhs slot for pkind 3
  qi32 cvt_i2f;   // pkind 1: convert integral slot to fp64
  qi32 ntok;
  qi32 track_nn;  // the input can be null in this launch (else nn == cstar)
  qi32 bop;       // pkind 3: typed binary op (T_ADD_I ... T_DIV_F)
  qi32 rhs;       // pkind 3: rhs slot, or -1 => literal
  qi32 rhs_null;  // pkind 3: literal is null
  qi64 rhs_lit;   // pkind 3: literal bits
  qi32 share;     // i + 1: same input and accumulator as aggregate i (SUM / AVG of one expression);
                  // the plan-specialised kernels keep one LDS accumulator for both (0: own)
  qi32 pad;
  DTok tok[QE_MAX_TOKENS];
};

struct DCol {
  const void* p;
  const qu8* valid;
  qi32 kind;  // SrcKind
  qi32 pad;
};

struct DTerm {
  qi32 lhs, op, rhs, f64;  // rhs < 0: literal; f64: compare as fp64
  qi32 lhs_f, rhs_f, lit_null, pad;
  qi64 lit;  // in the compare domain
};

struct DTable {
  qi64* keys;
  qu64* cstar;
  qi64* acc[QE_MAX_AGGS];
  qu64* nn[QE_MAX_AGGS];
  qu64* idx[QE_MAX_AGGS];  // 4 arrays of cap+2 each (fp64 MIN/MAX only)
  qu64* ext[QE_MAX_AGGS];  // exact fp64 SUM: FXE_WORDS words per slot (the full-range part, qe_dev fxe_*)
  qu64 cap;                // power of two; slots cap, cap+1 special
  qu64* ctl;               // [0] groups, [1] deferred rows, [2] overflow records, [3] lost
};

struct Plan {
  DCol cols[QE_MAX_COLS];
  DTerm terms[QE_MAX_TERMS];
  DAgg aggs[QE_MAX_AGGS];
  DTable t;
  qi64 n, row_base;
  const qu32* defer_in;  // retry pass: only these rows
  qu32* defer_out;       // rows the global table could not take
  qu8* ovf;              // overflow records (LDS flush)
  qu64 ovf_cap;
  qi32 ncols, nterms, mask_col, naggs;
  qi32 key_mode, nkeys, key_f64, rec_bytes;
  qi32 key_col[QE_MAX_KEYS], key_shift[QE_MAX_KEYS], key_nullbit[QE_MAX_KEYS], pad0;
  qi64 key_fmask[QE_MAX_KEYS];
  qi32 lds_log2, off_cstar;
  qi32 all8;       // every column slot is 8 bytes wide (straight-line loads)
  qi32 nn_skip;    // bit j: the table keeps aggregate j's non-null count implicit (== COUNT(*)): no nn adds
  qi32 off_acc[QE_MAX_AGGS], off_nn[QE_MAX_AGGS], off_idx[QE_MAX_AGGS];
  // radix-partitioned aggregation (high group counts, qe_jit.hip gen_part_source / gen_pagg_source)
  qu8* part_rec;   // records grouped by key-hash bucket (scatter output, partition-aggregate input)
  qi64* part_off;  // count: per (bucket, workgroup) record counts; scatter: their exclusive scan
  qi64 part_tw;    // rows per workgroup (count / scatter)
  qi64* part_slice;  // partition aggregate: [0] slice count, then (lo, hi | PART_EXCL) per slice
  // chunked scatter (no count pass): part_chunk[0] = chunks claimed, part_chunk[1 + c] =
  // (bucket << 32) | records in chunk c (PART_CH record slots each); part_sorted: chunk ids
  // grouped by bucket; slices are then (first, end | PART_EXCL) ranges of part_sorted
  qi64* part_chunk;
  qi32* part_sorted;
  // multi-pass fused aggregate (groups just beyond one LDS table): pass mp_pass of mp_n keeps the
  // rows whose key hash falls in bucket mp_pass (mp_n = 0: every row)
  qi32 mp_n, mp_pass;
  // radix-partitioned records in 32-bit words when the plan's words are integral (part_layout):
  // the scatter sets t.ctl[7] if a value did not fit, and the aggregation pass then does nothing
  qi32 part_narrow;
  // fused aggregate with a compact LDS table (qe_jit.hip compact_*): this many slots of 32-bit keys
  // (and 32-bit MIN / MAX where the input is a bare column), 0 = the regular 2^lds_log2 table
  qi32 lds_compact;
  // spilling first pass (spill_update): rows with spill_hash(key) >= mp_keep are spilled as records
  qu64 mp_keep;
  // select-project: pinned host words the kernel writes its results to ([0] rows written, [1] the
  // persistent look-back's stall flag), so no copy command follows the kernel (null: device only)
  qu64* host_ctl;
};

// ---- scalar helpers ---------------------------------------------------------------------------------
__host__ __device__ inline qi64 f64_bits(double d) { return __builtin_bit_cast(qi64, d); }
__host__ __device__ inline double bits_f64(qi64 b) { return __builtin_bit_cast(double, b); }

// Order-preserving int64 key of a non-NaN double with +0.0 and -0.0 mapped to the same key
// (they compare equal under IEEE `>`, Main.kt:547; the earliest one is tracked separately).
__host__ __device__ inline qi64 f64_okey(double d) {
  const qi64 b = f64_bits(d == 0.0 ? 0.0 : d);
  return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
}
__host__ __device__ inline double okey_f64(qi64 k) { return bits_f64(k >= 0 ? k : (k ^ 0x7FFFFFFFFFFFFFFFll)); }

// murmur3 finaliser: global-table slot and exchange partition hash.
__host__ __device__ inline qu64 fmix64(qu64 k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}

// Kept / spilled split of the spilling pass (Plan.mp_keep): the murmur3 32-bit finaliser over the
// folded key. Half the multiplies of fmix64's 64-bit ones (this runs for every row of the pass), and
// independent of lds_hash's buckets, so the kept share spreads over the whole LDS table.
__device__ inline qu32 spill_hash(qu64 key) {
  qu32 x = (qu32)key ^ (qu32)(key >> 32) * 0x27D4EB2Fu;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  return x ^ (x >> 16);
}

// Cheap slot hash for the per-workgroup LDS table: one 32-bit multiply (Fibonacci hashing).
__device__ inline qu32 lds_hash(qu64 key) {
  const qu32 x = (qu32)key ^ (qu32)(key >> 32) * 0x85EBCA6Bu;
  return x * 0x9E3779B1u;
}

// JVM Long division: truncating; MIN / -1 wraps to MIN; callers null out b == 0.
__device__ inline qi64 idiv(qi64 a, qi64 b) {
  if (b == 0) return 0;
  if (b == -1) return (qi64)(0ull - (qu64)a);
  return a / b;
}

__host__ __device__ inline bool acc_is_f64mm(int acc) { return acc == ACC_MIN_F || acc == ACC_MAX_F; }
// Aggregates with four extra 64-bit words per slot (the idx arrays): fp64 MIN/MAX keep first-row
// indices there, ACC_SUM_X its upper limbs and out-of-range count.
__host__ __device__ inline bool acc_has_idx(int acc) { return acc_is_f64mm(acc) || acc == ACC_SUM_X; }
__host__ __device__ inline qu64 idx_identity(int acc) { return acc_is_f64mm(acc) ? ~0ull : 0ull; }

// ---- exact fixed-point fp64 sums (ACC_SUM_X) ---------------------------------------------------------
// A slot's fp64 SUM is a 256-bit two's complement integer W in units of 2^-128 (sum = W * 2^-128):
// four 64-bit words w0..w3, w3 the signed top, plus a status word. Words live in acc (w0) and idx
// words 0..2 (w1..w3); idx word 3 is the status:
//   bits 0..7   flags, OR-ed (below)
//   bits 8..63  signed count of net wraps of W: W's part of the sum is (W + wraps * 2^256) * 2^-128
// A row adds its value's (at most 117-bit) two's complement image to the two words its mantissa
// spans, with integer atomics that return the old word; only a carry out of the second word or a
// change of the running sum's sign moves on to the next word. Integer adds are associative, so any
// order of rows, workgroups, passes, batches or ranks gives the same words: the result is the
// correctly rounded exact sum, bit-identical run to run. NaN / +-Inf inputs give the IEEE result
// of the sum (NaN, or the infinity). Every other finite input — |x| >= 2^126, or with bits below
// 2^-128 (subnormals among them) — goes whole into the slot's full-range accumulator E (fxe_*,
// below): a 2176-bit integer in units of 2^-1074 that holds any finite double exactly, so no input
// is ever rounded and the result is the correctly rounded sum over the whole fp64 range (gradual
// underflow and IEEE overflow to +-Inf included). The wrap count then only follows sums of inputs
// below 2^126: it stays in range up to 2^55 such inputs at the top of that range.
// Partials (records, combines) carry such an input in RAW form (word 0 = its bits) and E in CHUNK
// form (E's words 4c .. 4c + 3 in w0..w3; an exported group with E sends FXE_CHUNKS of them); both
// are added to E, never to W.
//   flags: FX_NAN / FX_PINF / FX_NINF the IEEE specials seen; FX_EXT the slot's E may be nonzero
//   (E is zero otherwise); FX_RAW / FX_CHUNK a partial's form (c in bits 8..15); FX_HUGE /
//   FX_INEXACT classify an input (fx_row: it needs E) and never reach a slot.
constexpr qu64 FX_NAN = 1, FX_PINF = 2, FX_NINF = 4, FX_HUGE = 8, FX_INEXACT = 16, FX_EXT = 32, FX_RAW = 64,
               FX_CHUNK = 128, FX_FLAGS = 0xFF, FX_SPECIAL = FX_NAN | FX_PINF | FX_NINF;
constexpr int FXE_WORDS = 34, FXE_CHUNKS = 9, FXE_LSB = 1074;  // 2176 bits, units of 2^-1074
constexpr qu64 FX_WRAP = 1ull << 8;  // one net wrap of W (signed count in bits 8..63)
// rare-path helpers of the exact sums: out of line unless a generated kernel asks otherwise
#ifdef QE_FX_INLINE
#define QE_FX_OUTLINE inline
#else
#define QE_FX_OUTLINE __attribute__((noinline))
#endif
constexpr int FX_LSB = 128;

// One input's image: (hi:lo) two's complement at words k, k+1 (k == -1: nothing to add to W),
// sign extended above; st = its status flags (FX_HUGE / FX_INEXACT: an input for E).
struct FxRow {
  qu64 lo, hi, st;
  int k;
  bool neg;
  qi64 bits;
};
__host__ __device__ inline FxRow fx_row(qi64 bits) {
  FxRow r{0ull, 0ull, 0ull, -1, false, bits};
  const qu64 b = (qu64)bits;
  r.neg = b >> 63;
  const int ex = (int)((b >> 52) & 0x7FF);
  qu64 m = b & ((1ull << 52) - 1);
  if (ex == 0x7FF) {
    r.st = m ? FX_NAN : (r.neg ? FX_NINF : FX_PINF);
    return r;
  }
  int p = -1074 + FX_LSB;  // bit position of m's lowest bit in W
  if (ex) {
    m |= 1ull << 52;
    p = ex - 1075 + FX_LSB;
  }
  if (m == 0) return r;
  if (p < 0) {  // bits below 2^-128 (whole multiples of 2^-128 stay in W)
    const int sh = -p;
    if (sh >= 53 || (m & ((1ull << sh) - 1))) {
      r.st = FX_INEXACT;
      return r;
    }
    m >>= sh;
    p = 0;
  }
  if (p + 64 - __builtin_clzll(m) > 254) {  // |x| >= 2^126: beyond the words' headroom
    r.st = FX_HUGE;
    return r;
  }
  r.k = p >> 6;
  const int q = p & 63;
  qu64 lo = m << q, hi = q ? (m >> (64 - q)) : 0ull;
  if (r.neg) {
    lo = 0ull - lo;
    hi = ~hi + (lo == 0 ? 1ull : 0ull);
  }
  r.lo = lo;
  r.hi = hi;
  return r;
}

// Status-word delta when the top word goes from `old` to old + add (signed): +-FX_WRAP on an
// overflow. Net wraps cancel exactly when the true sum is back in range.
__host__ __device__ inline qu64 fx_wrap(qu64 old, qu64 add) {
  const qi64 o = (qi64)old, a = (qi64)add, n = (qi64)(old + add);
  if (((o ^ n) & (a ^ n)) >= 0) return 0;
  return n < 0 ? FX_WRAP : (qu64)0 - FX_WRAP;
}

// Word add that returns the old word: an LDS / device-scope atomic, or a plain read-modify-write
// for a slot the caller owns alone (also the host build of the CPU algorithm test,
// tests/native/fx_host.hip, which instantiates only the plain form).
template <bool ATOMIC>
__host__ __device__ inline qu64 fx_xadd(qu64* p, qu64 v) {
  if constexpr (ATOMIC) {
    return atomicAdd(p, v);
  } else {
    const qu64 o = *p;
    *p = o + v;
    return o;
  }
}
template <bool ATOMIC>
__host__ __device__ inline void fx_status(qu64* st, qu64 v) {
  if (!v) return;
  if constexpr (ATOMIC) {
    if (v & FX_FLAGS) atomicOr(st, v & FX_FLAGS);
    if (v & ~FX_FLAGS) atomicAdd(st, v & ~FX_FLAGS);
  } else {
    *st = ((*st & ~FX_FLAGS) + (v & ~FX_FLAGS)) | ((*st | v) & FX_FLAGS);
  }
}

// One row (not FX_HUGE / FX_INEXACT: the caller sends those to E) into a slot whose word w is at wp(w).
template <bool ATOMIC, class WP>
__host__ __device__ inline void fx_add_row(WP wp, const FxRow& r, qu64* st) {
  qu64 sd = r.st;
  if (r.k >= 0) {
    int w = r.k;
    qu64 old = fx_xadd<ATOMIC>(wp(w), r.lo);
    if (w == 3) {
      sd += fx_wrap(old, r.lo);
    } else {
      const qu64 t = r.hi + (old + r.lo < old ? 1ull : 0ull);
      ++w;
      old = fx_xadd<ATOMIC>(wp(w), t);
      if (w == 3) {
        sd += fx_wrap(old, t);
      } else {
        // carry out of word w and the image's sign extension: -1, 0 or +1 for the next word
        qi64 d = (qi64)((t < r.hi ? 1 : 0) + (old + t < old ? 1 : 0)) - (r.neg ? 1 : 0);
#pragma unroll 1
        while (d != 0 && ++w <= 3) {
          old = fx_xadd<ATOMIC>(wp(w), (qu64)d);
          if (w == 3) {
            sd += fx_wrap(old, (qu64)d);
            break;
          }
          d = d > 0 ? (old == ~0ull ? 1 : 0) : (old != 0 ? 0 : -1);
        }
      }
    }
  }
  fx_status<ATOMIC>(st, sd);
}

// A whole partial (words v0..v3, status vst) into a slot.
template <bool ATOMIC, class WP>
__host__ __device__ inline void fx_add_words(WP wp, qu64 v0, qu64 v1, qu64 v2, qu64 v3, qu64 vst, qu64* st) {
  const qu64 v[3] = {v0, v1, v2};
  qu64 c = 0;
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const qu64 t = v[w] + c;
    qu64 cb = 0;
    if (t) {
      const qu64 old = fx_xadd<ATOMIC>(wp(w), t);
      cb = old + t < old ? 1ull : 0ull;
    }
    c = (t < v[w] ? 1ull : 0ull) + cb;
  }
  qu64 sd = vst;
  if (c && v3 == 0x7FFFFFFFFFFFFFFFull) sd += FX_WRAP;  // v3 + 1 = 2^63: -2^63 and one wrap
  const qu64 t = v3 + c;
  if (t) sd += fx_wrap(fx_xadd<ATOMIC>(wp(3), t), t);
  fx_status<ATOMIC>(st, sd);
}

// ---- the per-workgroup LDS window of an exact fp64 SUM (plan-specialised kernels) -------------------
// 192-bit two's complement in units of 2^-96: words u0 (2^-96), u1 (2^-32) and u2 (2^32, the signed
// top), 24 bytes per LDS slot instead of the global slot's 40. A row whose value is +-0 or has
// |x| in [2^-44, 2^62) (exponent field 979..1084) adds here exactly: its mantissa lies inside the
// window, and a workgroup's partial stays below 2^62 x 2^31 rows = 2^93, so the top word never
// overflows and needs no status. Every other row (NaN, +-Inf, subnormal, tinier or larger values:
// fx_rare) goes to the global table's full accumulator like a row whose group has no LDS slot.
constexpr int FXW_LSB = 96;
constexpr int FXW_EX_LO = 979, FXW_EX_HI = 1085;  // exponent fields [2^-44, 2^62)
__host__ __device__ inline bool fx_rare(qi64 bits) {
  const qu32 ex = (qu32)((qu64)bits >> 52) & 0x7FFu;
  return (ex - (qu32)FXW_EX_LO) >= (qu32)(FXW_EX_HI - FXW_EX_LO) && ((qu64)bits << 1) != 0;
}

// One row (!fx_rare) into a window whose word w is at wp(w): two LDS atomics that return the old
// word (the carry out of the first feeds the second); a third, rare, when the carry out of u1 and
// the row's sign extension do not cancel (the running sum changed sign).
template <bool ATOMIC = true, class WP>
__host__ __device__ inline void fxw_add(WP wp, qi64 bits) {
  const qu64 b = (qu64)bits;
  const int ex = (int)((b >> 52) & 0x7FF);
  if (ex == 0) return;  // +-0 (a subnormal is an fx_rare row)
  const qu64 m = (b & ((1ull << 52) - 1)) | (1ull << 52);
  const int p = ex - FXW_EX_LO, k = p >> 6, q = p & 63;
  qu64 lo = m << q, hi = q ? (m >> (64 - q)) : 0ull;
  const bool neg = b >> 63;
  if (neg) {
    lo = 0ull - lo;
    hi = ~hi + (lo == 0 ? 1ull : 0ull);
  }
  const qu64 o0 = fx_xadd<ATOMIC>(wp(k), lo);
  const qu64 t = hi + (o0 + lo < o0 ? 1ull : 0ull);
  const qu64 o1 = fx_xadd<ATOMIC>(wp(k + 1), t);  // k == 1: the top word, whose carry out is dropped
  if (k == 0) {
    const qi64 d = (qi64)((t < hi ? 1 : 0) + (o1 + t < o1 ? 1 : 0)) - (neg ? 1 : 0);
    if (d) fx_xadd<ATOMIC>(wp(2), (qu64)d);
  }
}

// A window as a partial of the global accumulator (units 2^-128: shifted up 32 bits): v[0..3].
__host__ __device__ inline void fxw_words(qu64 u0, qu64 u1, qu64 u2, qu64 v[4]) {
  v[0] = u0 << 32;
  v[1] = (u0 >> 32) | (u1 << 32);
  v[2] = (u1 >> 32) | (u2 << 32);
  v[3] = (qu64)((qi64)u2 >> 32);
}


// Whether an input needs the full-range accumulator (>= 2^182, or bits below 2^-128).
__host__ __device__ inline bool fx_needs_ext(qi64 bits) { return (fx_row(bits).st & (FX_HUGE | FX_INEXACT)) != 0; }

// The words of one input alone (RowVal form: the global-table and record paths): w[0..3] and the
// status word; an input for E in RAW form.
__host__ __device__ inline void fx_row_words(qi64 bits, qu64 w[5]) {
  const FxRow r = fx_row(bits);
  const bool raw = (r.st & (FX_HUGE | FX_INEXACT)) != 0;  // (selects, not an early return: the
                                                          // words stay in registers)
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = raw ? (i == 0 ? (qu64)bits : 0ull)
               : (r.k < 0 ? 0ull : i == r.k ? r.lo : i == r.k + 1 ? r.hi : (i > r.k + 1 && r.neg) ? ~0ull : 0ull);
  w[4] = raw ? FX_RAW : r.st;
}

// Correctly rounded double of (w0..w3 + wraps * 2^256) * 2^-128 (ties to even).
__host__ __device__ inline double fx_to_double(qu64 w0, qu64 w1, qu64 w2, qu64 w3, qi64 wraps) {
  qu64 w[5] = {w0, w1, w2, w3, (qu64)(wraps + ((qi64)w3 >> 63))};
  const bool neg = (qi64)w[4] < 0;
  if (neg) {  // magnitude: invert and add one
    qu64 carry = 1;
    for (int k = 0; k < 5; ++k) {
      w[k] = ~w[k] + carry;
      carry = (carry && w[k] == 0) ? 1ull : 0ull;
    }
  }
  int top = 4;
  while (top >= 0 && w[top] == 0) --top;
  if (top < 0) return 0.0;
  const int msb = 64 * top + 63 - __builtin_clzll(w[top]);
  // the 64 bits ending at the leading one, plus a sticky bit for the rest
  qu64 win;
  bool sticky = false;
  const int lowpos = msb - 63;
  if (lowpos <= 0) {
    win = w[0] << (-lowpos);
  } else {
    const int a = lowpos >> 6, sh = lowpos & 63;
    win = sh ? ((w[a] >> sh) | (w[a + 1] << (64 - sh))) : w[a];
    sticky = sh && (w[a] & ((1ull << sh) - 1)) != 0;
    for (int i = 0; i < a && !sticky; ++i) sticky = w[i] != 0;
  }
  qu64 mant = win >> 11;  // 53 bits
  const qu64 rem = win & 0x7FFull;
  if (rem > 0x400 || (rem == 0x400 && (sticky || (mant & 1)))) ++mant;
  int ex = msb - 52 - FX_LSB;  // exponent of the mantissa's lowest bit
  if (mant >> 53) {
    mant >>= 1;
    ++ex;
  }
  // exact scaling by 2^ex: msb < 320 (wraps within +-2^62), so -180 <= ex <= 140, a normal power of two
  const double d = (double)mant * bits_f64((qi64)((qu64)(1023 + ex) << 52));
  return neg ? -d : d;
}

// ---- the full-range accumulator of an exact fp64 SUM ----------------------------------------------------
// A 2176-bit two's complement integer E in units of 2^-1074 (34 words, e[33] the signed top): every
// finite double is a whole number of units, and any sum of fewer than 2^63 of them stays below 2^1101
// in magnitude. A slot's exact sum is E * 2^-1074 + (W + wraps * 2^256) * 2^-128.
// One input into E: its mantissa's two's complement image at the words it spans, the carry and sign
// extension moving up word by word only while they do not cancel (fx_add_row's scheme).
template <bool ATOMIC>
__host__ __device__ inline void fxe_add_value(qu64* e, qi64 bits) {
  const qu64 b = (qu64)bits;
  const int ex = (int)((b >> 52) & 0x7FF);
  qu64 m = b & ((1ull << 52) - 1);
  if (ex) m |= 1ull << 52;
  if (m == 0 || ex == 0x7FF) return;  // +-0; NaN / Inf never come here
  const int p = ex ? ex - 1 : 0;       // the mantissa's lowest bit, in units of 2^-1074
  int w = p >> 6;
  const int q = p & 63;
  const bool neg = b >> 63;
  qu64 lo = m << q, hi = q ? (m >> (64 - q)) : 0ull;
  if (neg) {
    lo = 0ull - lo;
    hi = ~hi + (lo == 0 ? 1ull : 0ull);
  }
  qu64 old = fx_xadd<ATOMIC>(&e[w], lo);
  const qu64 t = hi + (old + lo < old ? 1ull : 0ull);
  if (++w >= FXE_WORDS) return;
  old = fx_xadd<ATOMIC>(&e[w], t);
  qi64 d = (qi64)((t < hi ? 1 : 0) + (old + t < old ? 1 : 0)) - (neg ? 1 : 0);
#pragma unroll 1
  while (d != 0 && ++w < FXE_WORDS) {
    old = fx_xadd<ATOMIC>(&e[w], (qu64)d);
    d = d > 0 ? (old == ~0ull ? 1 : 0) : (old != 0 ? 0 : -1);
  }
}

// Words v[0..n) (a chunk of another accumulator: unsigned, except the top word's sign) into E at
// word w0, the carry moving up.
template <bool ATOMIC>
__host__ __device__ inline void fxe_add_words(qu64* e, int w0, const qu64* v, int n) {
  qu64 c = 0;
  int w = w0;
  for (int i = 0; i < n; ++i, ++w) {
    const qu64 t = v[i] + c;
    qu64 cb = 0;
    if (t) {
      const qu64 old = fx_xadd<ATOMIC>(&e[w], t);
      cb = old + t < old ? 1ull : 0ull;
    }
    c = (t < v[i] ? 1ull : 0ull) + cb;
  }
#pragma unroll 1
  for (; c && w < FXE_WORDS; ++w) c = fx_xadd<ATOMIC>(&e[w], 1ull) == ~0ull ? 1ull : 0ull;
}

// Four words in registers (n of them used: 2 or 4) into E at word w0: fxe_add_words with constant
// indices, so a CHUNK partial's words stay in registers (an array indexed by the loop counter went to
// scratch memory in every generated kernel).
template <bool ATOMIC>
__host__ __device__ inline void fxe_add_words4(qu64* e, int w0, qu64 v0, qu64 v1, qu64 v2, qu64 v3, int n) {
  qu64 c = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const qu64 vi = i == 0 ? v0 : i == 1 ? v1 : i == 2 ? v2 : v3;
    if (i < n) {
      const qu64 t = vi + c;
      qu64 cb = 0;
      if (t) {
        const qu64 old = fx_xadd<ATOMIC>(&e[w0 + i], t);
        cb = old + t < old ? 1ull : 0ull;
      }
      c = (t < vi ? 1ull : 0ull) + cb;
    }
  }
#pragma unroll 1
  for (int w = w0 + n; c && w < FXE_WORDS; ++w) c = fx_xadd<ATOMIC>(&e[w], 1ull) == ~0ull ? 1ull : 0ull;
}

// Correctly rounded double (ties to even; IEEE overflow to +-Inf, gradual underflow) of
// E * 2^-1074 + (W + wraps * 2^256) * 2^-128.
__host__ __device__ inline double fxe_result(const qu64* e, qu64 w0, qu64 w1, qu64 w2, qu64 w3, qi64 wraps) {
  qu64 x[FXE_WORDS];
  for (int i = 0; i < FXE_WORDS; ++i) x[i] = e[i];
  // W (five words with the wraps, signed) shifted up by 1074 - 128 = 946 bits = 14 words + 50
  const qu64 m5[5] = {w0, w1, w2, w3, (qu64)(wraps + ((qi64)w3 >> 63))};
  qu64 sh[FXE_WORDS];
  const qu64 ext = ((qi64)m5[4] < 0) ? ~0ull : 0ull;
  for (int i = 0; i < FXE_WORDS; ++i) {
    const int k = i - 14;  // word of the unshifted W feeding bits [64 i, 64 i + 64): k and k - 1
    const qu64 a = k < 0 ? 0ull : (k < 5 ? m5[k] : ext);
    const qu64 bl = k - 1 < 0 ? 0ull : (k - 1 < 5 ? m5[k - 1] : ext);
    sh[i] = (a << 50) | (k - 1 < 0 ? 0ull : (bl >> 14));
  }
  qu64 c = 0;
  for (int i = 0; i < FXE_WORDS; ++i) {
    const qu64 s1 = x[i] + sh[i], c1 = s1 < sh[i] ? 1ull : 0ull;
    const qu64 s2 = s1 + c, c2 = s2 < s1 ? 1ull : 0ull;
    x[i] = s2;
    c = c1 | c2;
  }
  const bool neg = (qi64)x[FXE_WORDS - 1] < 0;
  if (neg) {
    qu64 carry = 1;
    for (int i = 0; i < FXE_WORDS; ++i) {
      x[i] = ~x[i] + carry;
      carry = (carry && x[i] == 0) ? 1ull : 0ull;
    }
  }
  int top = FXE_WORDS - 1;
  while (top >= 0 && x[top] == 0) --top;
  if (top < 0) return neg ? -0.0 : 0.0;
  const int msb = 64 * top + 63 - __builtin_clzll(x[top]);
  double d;
  if (msb < 53) {  // a whole number of 2^-1074 below 2^53 units: exact (subnormal or the smallest normals)
    d = (double)x[0] * 0x1p-1074;
  } else {
    const int lowpos = msb - 63;
    qu64 win;
    bool sticky = false;
    if (lowpos <= 0) {
      win = x[0] << (-lowpos);
    } else {
      const int a = lowpos >> 6, s = lowpos & 63;
      win = s ? ((x[a] >> s) | (x[a + 1] << (64 - s))) : x[a];
      sticky = s && (x[a] & ((1ull << s) - 1)) != 0;
      for (int i = 0; i < a && !sticky; ++i) sticky = x[i] != 0;
    }
    qu64 mant = win >> 11;
    const qu64 rem = win & 0x7FFull;
    if (rem > 0x400 || (rem == 0x400 && (sticky || (mant & 1)))) ++mant;
    int ex = msb - 52 - FXE_LSB;  // the mantissa's lowest bit: 2^ex
    if (mant >> 53) {
      mant >>= 1;
      ++ex;
    }
    if (ex + 52 > 1023) {
      d = __builtin_inf();
    } else {  // 2^ex in two exact steps (ex in [-1073, 971])
      const int e1 = ex / 2, e2 = ex - e1;
      d = (double)mant * bits_f64((qi64)((qu64)(1023 + e1) << 52)) * bits_f64((qi64)((qu64)(1023 + e2) << 52));
    }
  }
  return neg ? -d : d;
}

// A RAW or CHUNK partial into E at e; the slot's status at st gets FX_EXT and the partial's specials.
template <bool ATOMIC>
__host__ __device__ inline void fxe_partial(qu64* e, qu64* st, qu64 w0, qu64 w1, qu64 w2, qu64 w3, qu64 vst) {
  if (vst & FX_RAW) {
    fxe_add_value<ATOMIC>(e, (qi64)w0);
  } else {
    const int c = (int)((vst >> 8) & 0xFF);
    if (c < FXE_CHUNKS) fxe_add_words4<ATOMIC>(e, 4 * c, w0, w1, w2, w3, c == FXE_CHUNKS - 1 ? FXE_WORDS - 4 * c : 4);
  }
  fx_status<ATOMIC>(st, FX_EXT | (vst & FX_SPECIAL));
}

// The SUM of a slot: words w0..w3, status st, E at e (read only when st has FX_EXT).
__host__ __device__ inline double fx_result(qu64 w0, qu64 w1, qu64 w2, qu64 w3, qu64 st, const qu64* e) {
  const qu64 f = st & FX_FLAGS;
  if ((f & FX_NAN) || ((f & FX_PINF) && (f & FX_NINF))) return bits_f64(0x7FF8000000000000ll);
  if (f & FX_PINF) return bits_f64(0x7FF0000000000000ll);
  if (f & FX_NINF) return bits_f64((qi64)0xFFF0000000000000ull);
  if (f & FX_EXT) return fxe_result(e, w0, w1, w2, w3, (qi64)st >> 8);
  return fx_to_double(w0, w1, w2, w3, (qi64)st >> 8);
}
__host__ __device__ inline qi64 acc_identity(int acc) {
  switch (acc) {
    case ACC_MIN_I:
    case ACC_MIN_F: return 0x7FFFFFFFFFFFFFFFll;
    case ACC_MAX_I:
    case ACC_MAX_F: return EMPTY_KEY;
    default: return 0;
  }
}

// Record layout (export/import/overflow):
// [0] key  [8] flags (bit0 null key)  [16] cstar  then per aggregate: acc, nn, (4 x idx if fp64 MIN/MAX)
__host__ __device__ inline int agg_rec_bytes(int acc) { return 16 + (acc_has_idx(acc) ? 32 : 0); }

// ---- global table -------------------------------------------------------------------------------------
__device__ inline bool gtable_find(const DTable& t, qi64 key, bool knull, qu64& slot) {
  if (knull) {
    slot = t.cap;
    return true;
  }
  if (key == EMPTY_KEY) {
    slot = t.cap + 1;
    return true;
  }
  qu64 h = fmix64((qu64)key) & (t.cap - 1);
#pragma unroll 1
  for (int p = 0; p < HA_GLOBAL_MAXP; ++p) {
    const qi64 k = __hip_atomic_load(&t.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) {
      slot = h;
      return true;
    }
    if (k == EMPTY_KEY) {
      const qi64 old = (qi64)atomicCAS((qu64*)&t.keys[h], (qu64)EMPTY_KEY, (qu64)key);
      if (old == EMPTY_KEY) {
        atomicAdd(&t.ctl[0], 1ull);
        slot = h;
        return true;
      }
      if (old == key) {
        slot = h;
        return true;
      }
    }
    h = (h + 1) & (t.cap - 1);
  }
  return false;
}

// gtable_find for a workgroup flush: a new group is counted in the workgroup's LDS counter
// `newg` (added to ctl[0] once per workgroup) instead of one device-scope add per group on the
// same word. `*inserted` reports whether this call created the group.
__device__ inline bool gtable_find_wg(const DTable& t, qi64 key, bool knull, qu64& slot, qu32* newg) {
  if (knull || key == EMPTY_KEY) {
    slot = knull ? t.cap : t.cap + 1;
    return true;
  }
  qu64 h = fmix64((qu64)key) & (t.cap - 1);
#pragma unroll 1
  for (int p = 0; p < HA_GLOBAL_MAXP; ++p) {
    const qi64 k = __hip_atomic_load(&t.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) {
      slot = h;
      return true;
    }
    if (k == EMPTY_KEY) {
      const qi64 old = (qi64)atomicCAS((qu64*)&t.keys[h], (qu64)EMPTY_KEY, (qu64)key);
      if (old == EMPTY_KEY) {
        atomicAdd(newg, 1u);
        slot = h;
        return true;
      }
      if (old == key) {
        slot = h;
        return true;
      }
    }
    h = (h + 1) & (t.cap - 1);
  }
  return false;
}

// (c == 0: a record that carries only exact-SUM parts; its group is counted by the records with rows)
__device__ inline void gadd_cstar(const DTable& t, qu64 slot, qu64 c) {
  if (!c) return;
  const qu64 old = atomicAdd(&t.cstar[slot], c);
  if (slot >= t.cap && old == 0) atomicAdd(&t.ctl[0], 1ull);  // a special group appears
}

// Combine one aggregate's partial state into global slot `s` (device-scope atomics). add_nn =
// false while the table keeps the aggregate's non-null count implicit (every input row so far was
// non-null: nn == COUNT(*), read from cstar; see qe_hashagg.hip nn_implicit).
// An exact fp64 SUM partial into global slot s (device-scope atomics). Out of line: the kernels call
// it from their flush and from rare rows, and inlined copies of its carry chain at every such site
// made the C5 fused kernel 8x larger than the instruction cache.
// WORDS: the partial is known to be words (an LDS window or slot at a flush): no RAW / CHUNK test,
// so the generated kernels carry E's code only on the rare-row paths.
template <bool WORDS = false>
static __device__ QE_FX_OUTLINE void gcombine_fx(const DTable& t, int j, qu64 s, qu64 w0, qu64 w1,
                                                             qu64 w2, qu64 w3, qu64 st) {
  const qu64 stride = t.cap + 2;
  qu64* ix = t.idx[j];
  if (!WORDS && (st & (FX_RAW | FX_CHUNK))) {  // an input or a chunk for E
    fxe_partial<true>(t.ext[j] + s * FXE_WORDS, &ix[3 * stride + s], w0, w1, w2, w3, st);
    return;
  }
  fx_add_words<true>([&](int w) { return w == 0 ? (qu64*)&t.acc[j][s] : &ix[(w - 1) * stride + s]; }, w0, w1, w2, w3,
                     st, &ix[3 * stride + s]);
}

// One row's exact fp64 SUM input into global slot s (rows whose group has no LDS slot), out of line.
static __device__ QE_FX_OUTLINE void gcombine_fx_row(const DTable& t, int j, qu64 s, qi64 x, bool add_nn) {
  qu64 w[5];
  fx_row_words(x, w);
  if (add_nn) atomicAdd(&t.nn[j][s], 1ull);
  gcombine_fx(t, j, s, w[0], w[1], w[2], w[3], w[4]);
}

// An exact fp64 SUM partial may carry words with nn == 0: a rare input whose row was counted in an
// LDS slot (fx_rare_global). WORDS: as gcombine_fx's (a flush).
template <bool WORDS = false>
__device__ inline void gcombine(const DTable& t, int acck, int j, qu64 s, qi64 acc, qu64 nn, qu64 i0, qu64 i1,
                                qu64 i2, qu64 i3, bool add_nn = true) {
  if (nn == 0 && acck != ACC_SUM_X) return;
  if (add_nn && nn) atomicAdd(&t.nn[j][s], nn);
  switch (acck) {
    case ACC_SUM_I:
      if (acc) atomicAdd((qu64*)&t.acc[j][s], (qu64)acc);
      break;
    case ACC_SUM_F: atomicAdd((double*)&t.acc[j][s], bits_f64(acc)); break;
    case ACC_MIN_I:
    case ACC_MIN_F:
      if (acc != 0x7FFFFFFFFFFFFFFFll) atomicMin(&t.acc[j][s], acc);
      break;
    case ACC_MAX_I:
    case ACC_MAX_F:
      if (acc != EMPTY_KEY) atomicMax(&t.acc[j][s], acc);
      break;
    default: break;
  }
  if (acc_is_f64mm(acck)) {
    const qu64 stride = t.cap + 2;
    qu64* ix = t.idx[j];
    if (i0 != ~0ull) atomicMin(&ix[s], i0);
    if (i1 != ~0ull) atomicMin(&ix[stride + s], i1);
    if (i2 != ~0ull) atomicMin(&ix[2 * stride + s], i2);
    if (i3 != ~0ull) atomicMin(&ix[3 * stride + s], i3);
  } else if (acck == ACC_SUM_X) {  // 256-bit add with carries (words: acc, idx 0..2; status idx 3)
    gcombine_fx<WORDS>(t, j, s, (qu64)acc, i0, i1, i2, i3);
  }
}

// Exclusive forms of gadd_cstar / gcombine: the caller is the only writer of slot `s` during this
// launch (a radix-partitioned slice holding its bucket's every record), so plain read-modify-writes
// replace the device-scope atomics. The table was last written by earlier launches (or not at
// all), whose writes the launch boundary makes visible; same results as the atomic forms.
__device__ inline void gadd_cstar_excl(const DTable& t, qu64 slot, qu64 c, qu32* newg) {
  if (!c) return;
  const qu64 old = t.cstar[slot];
  t.cstar[slot] = old + c;
  if (slot >= t.cap && old == 0) atomicAdd(newg, 1u);
}

template <bool WORDS = false>
__device__ inline void gcombine_excl(const DTable& t, int acck, int j, qu64 s, qi64 acc, qu64 nn, qu64 i0,
                                     qu64 i1, qu64 i2, qu64 i3) {
  if (nn == 0 && acck != ACC_SUM_X) return;
  t.nn[j][s] += nn;
  qi64* a = &t.acc[j][s];
  switch (acck) {
    case ACC_SUM_I: *a = (qi64)((qu64)*a + (qu64)acc); break;
    case ACC_SUM_F: *a = f64_bits(bits_f64(*a) + bits_f64(acc)); break;
    case ACC_MIN_I:
    case ACC_MIN_F:
      if (acc < *a) *a = acc;
      break;
    case ACC_MAX_I:
    case ACC_MAX_F:
      if (acc > *a) *a = acc;
      break;
    default: break;
  }
  if (acc_is_f64mm(acck)) {
    const qu64 stride = t.cap + 2;
    qu64* ix = t.idx[j] + s;
    if (i0 < ix[0]) ix[0] = i0;
    if (i1 < ix[stride]) ix[stride] = i1;
    if (i2 < ix[2 * stride]) ix[2 * stride] = i2;
    if (i3 < ix[3 * stride]) ix[3 * stride] = i3;
  } else if (acck == ACC_SUM_X) {
    const qu64 stride = t.cap + 2;
    qu64* ix = t.idx[j] + s;
    if (!WORDS && (i3 & (FX_RAW | FX_CHUNK))) {
      fxe_partial<false>(t.ext[j] + s * FXE_WORDS, &ix[3 * stride], (qu64)acc, i0, i1, i2, i3);
      return;
    }
    fx_add_words<false>([&](int w) { return w == 0 ? (qu64*)a : &ix[(w - 1) * stride]; }, (qu64)acc, i0, i1, i2, i3,
                        &ix[3 * stride]);
  }
}

// Per-row contribution of one aggregate in partial form.
struct RowVal {
  qi64 acc;
  qu64 i0, i1, i2, i3;
};

__device__ inline RowVal row_partial(int acck, qi64 x, qu64 row) {
  RowVal r{acc_identity(acck), ~0ull, ~0ull, ~0ull, ~0ull};
  switch (acck) {
    case ACC_SUM_I:
    case ACC_SUM_F:
    case ACC_MIN_I:
    case ACC_MAX_I: r.acc = x; break;
    case ACC_SUM_X: {
      qu64 w[5];
      fx_row_words(x, w);
      r.acc = (qi64)w[0];
      r.i0 = w[1];
      r.i1 = w[2];
      r.i2 = w[3];
      r.i3 = w[4];
      break;
    }
    case ACC_MIN_F:
    case ACC_MAX_F: {
      const double d = bits_f64(x);
      r.i0 = row;
      if (d != d) {
        r.i1 = row;
      } else {
        r.acc = f64_okey(d);
        if (d == 0.0) {
          if (x < 0) r.i2 = row;
          else r.i3 = row;
        }
      }
      break;
    }
    default: break;
  }
  return r;
}

__device__ inline void write_record_head(qu8* rec, qi64 key, bool knull, qu64 cstar) {
  ((qi64*)rec)[0] = key;
  ((qu64*)rec)[1] = knull ? 1ull : 0ull;
  ((qu64*)rec)[2] = cstar;
}

// A queued exact-SUM input outside the LDS window (fx_rare; the specialised fused kernel's fx queue)
// for the aggregates in `jmask` (one, or several sharing one LDS accumulator: DAgg.share): straight
// into its group's global slot — the row's COUNT(*) and non-null counts stay in the LDS slot, which
// the flush merges later — or, while the global table has no room for the group, as an overflow
// record (COUNT(*) 0, identity partials but those aggregates) merged after the table grows, like
// the flush's own records.
static __device__ QE_FX_OUTLINE void fx_rare_global(const Plan& P, qu32 jmask, qi64 key, bool knull,
                                                                qi64 x) {
  qu64 w[5];
  fx_row_words(x, w);
  qu64 gs;
  if (gtable_find(P.t, key, knull, gs)) {
#pragma unroll 1  // (one copy of the combine: unrolled over QE_MAX_AGGS it was 8 per call site)
    for (int j = 0; j < P.naggs; ++j)
      if ((jmask >> j) & 1) gcombine(P.t, ACC_SUM_X, j, gs, (qi64)w[0], 0, w[1], w[2], w[3], w[4], false);
    return;
  }
  const qu64 ri = atomicAdd(&P.t.ctl[2], 1ull);
  if (ri >= P.ovf_cap) {
    atomicAdd(&P.t.ctl[3], 1ull);
    return;
  }
  qu8* rec = P.ovf + ri * (qu64)P.rec_bytes;
  write_record_head(rec, key, knull, 0);
  int off = 24;
#pragma unroll 1
  for (int a = 0; a < P.naggs; ++a) {
    qu64* f = (qu64*)(rec + off);
    const int acc = P.aggs[a].acc;
    const bool mine = (jmask >> a) & 1;
    f[0] = mine ? w[0] : (qu64)acc_identity(acc);
    f[1] = 0;
    if (acc_has_idx(acc)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) f[2 + i] = mine ? w[1 + i] : idx_identity(acc);
    }
    off += agg_rec_bytes(acc);
  }
}

// ---- LDS table helpers ----------------------------------------------------------------------------------
// Continue probing the LDS table from slot h (already found to hold another key); inserts the
// key into the first empty slot. Returns the slot, or -1 when the probe limit is hit.
__device__ inline int lds_probe(qi64* keys, int log2, qi64 key, qu32 h) {
  const qu32 mask = (1u << log2) - 1;
#pragma unroll 1
  for (int p = 0; p < HA_LDS_MAXP; ++p) {
    const qi64 k = keys[h];
    if (k == key) return (int)h;
    if (k == EMPTY_KEY) {
      const qi64 old = (qi64)atomicCAS((qu64*)&keys[h], (qu64)EMPTY_KEY, (qu64)key);
      if (old == EMPTY_KEY || old == key) return (int)h;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

// lds_probe for the 32-bit key tables of the fast aggregation pass (qe_jit.hip gen_pagg_fast_source):
// empty slots hold EMPTY_KEY32 (INT32_MIN; that key itself lives in special slot S + 1).
constexpr qi32 EMPTY_KEY32 = (qi32)0x80000000u;
__device__ inline int lds_probe32(qi32* keys, int log2, qi32 key, qu32 h) {
  const qu32 mask = (1u << log2) - 1;
#pragma unroll 1
  for (int p = 0; p < HA_LDS_MAXP; ++p) {
    const qi32 k = keys[h];
    if (k == key) return (int)h;
    if (k == EMPTY_KEY32) {
      const qi32 old = atomicCAS(&keys[h], EMPTY_KEY32, key);
      if (old == EMPTY_KEY32 || old == key) return (int)h;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

// Tables of 32-bit keys in 4-slot buckets (16-byte aligned; the fast aggregation pass and the
// compact fused table): a key lives in its home bucket or, if that filled up first, a later one,
// so a lookup is one 16-byte LDS read and four compares (a home bucket of four slots at <= 65 %
// load almost never overflows). Slots fill in order and are never emptied, so a lookup may stop
// at a bucket with an empty slot. Continues from home bucket b; returns the slot, -1 at the limit.
__device__ inline int lds_probe4(qi32* keys, qu32 nb, qi32 key, qu32 b) {
#pragma unroll 1
  for (int p = 0; p < HA_LDS_MAXP; ++p) {
    const qu32x4 q = *(const volatile qu32x4*)(keys + 4 * b);
    const qi32 kk[4] = {(qi32)q.x, (qi32)q.y, (qi32)q.z, (qi32)q.w};
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
      if (kk[i] == key) return (int)(4 * b) + i;
      if (kk[i] == EMPTY_KEY32) {
        const qi32 old = atomicCAS(&keys[4 * b + i], EMPTY_KEY32, key);
        if (old == EMPTY_KEY32 || old == key) return (int)(4 * b) + i;
        // another key took it: the later slots of the snapshot are still candidates
      }
    }
    b = b + 1 == nb ? 0 : b + 1;
  }
  return -1;
}

// Slot of `kk` among the 8 slots of bucket b and the bucket b2 after it (their 16-byte snapshots q,
// q2), or -1: the hit test of the 4-slot-bucket tables without a branch. Keys that lds_probe4
// placed one bucket past their own are found here too (at a half-full table ~4 % of the keys;
// the home bucket alone sent nearly every 256-record step down the serial probe loop).
__device__ inline int bucket2_hit(qu32x4 q, qu32x4 q2, qu32 kk, qu32 b, qu32 b2) {
  const qu32 m = (qu32)(q.x == kk) | ((qu32)(q.y == kk) << 1) | ((qu32)(q.z == kk) << 2) | ((qu32)(q.w == kk) << 3) |
                 ((qu32)(q2.x == kk) << 4) | ((qu32)(q2.y == kk) << 5) | ((qu32)(q2.z == kk) << 6) |
                 ((qu32)(q2.w == kk) << 7);
  const int i = __builtin_ctz(m | 0x100u);
  return i < 4 ? (int)(4 * b) + i : (i < 8 ? (int)(4 * b2) + i - 4 : -1);
}

// bucket2_hit over three consecutive buckets (b, b2, b3): fuller tables (QE_PAGG_WINDOW=3)
__device__ inline int bucket3_hit(qu32x4 q, qu32x4 q2, qu32x4 q3, qu32 kk, qu32 b, qu32 b2, qu32 b3) {
  const int i = bucket2_hit(q, q2, kk, b, b2);
  const qu32 m = (qu32)(q3.x == kk) | ((qu32)(q3.y == kk) << 1) | ((qu32)(q3.z == kk) << 2) | ((qu32)(q3.w == kk) << 3);
  return i >= 0 ? i : (m ? (int)(4 * b3) + __builtin_ctz(m) : -1);
}

// lds_probe4 for up to four rows of a lane at once (bit r of pm: row r pending; key k_r, home bucket
// h_r; its slot, or -1, into s_r). Each iteration advances the lowest pending row of EVERY lane by
// one bucket, so a wave spends about the longest lane's total probe length instead of, row after
// row, the longest probe of that row. Same probe order and insert rule as lds_probe4 (the first
// EMPTY slot from the home bucket on), so keys are never duplicated.
__device__ inline void lds_probe4_rows(qi32* keys, qu32 nb, qu32 pm, qi32 k0, qi32 k1, qi32 k2, qi32 k3, qu32 h0,
                                       qu32 h1, qu32 h2, qu32 h3, int& s0, int& s1, int& s2, int& s3) {
  const qu32 pm0 = pm;
  int r = pm ? __builtin_ctz(pm) : 0;
  qu32 b = r == 0 ? h0 : r == 1 ? h1 : r == 2 ? h2 : h3;
  int probes = 0;
  qu64 res = 0;
#pragma unroll 1
  while (pm) {
    const qi32 kk = r == 0 ? k0 : r == 1 ? k1 : r == 2 ? k2 : k3;
    const qu32x4 q = *(const volatile qu32x4*)(keys + 4 * b);
    const qu32 m = (qu32)(q.x == (qu32)kk) | ((qu32)(q.y == (qu32)kk) << 1) | ((qu32)(q.z == (qu32)kk) << 2) |
                   ((qu32)(q.w == (qu32)kk) << 3);
    const qu32 e = (qu32)(q.x == (qu32)EMPTY_KEY32) | ((qu32)(q.y == (qu32)EMPTY_KEY32) << 1) |
                   ((qu32)(q.z == (qu32)EMPTY_KEY32) << 2) | ((qu32)(q.w == (qu32)EMPTY_KEY32) << 3);
    int found = -2;  // -2: keep probing
    if (m) {
      found = (int)(4 * b) + __builtin_ctz(m);
    } else if (e) {
      const int i = __builtin_ctz(e);
      const qi32 old = atomicCAS(&keys[4 * b + i], EMPTY_KEY32, kk);
      if (old == EMPTY_KEY32 || old == kk) found = (int)(4 * b) + i;
      // else another key took that slot: read the same bucket again
    } else if (++probes >= HA_LDS_MAXP) {
      found = -1;
    } else {
      b = b + 1 == nb ? 0 : b + 1;
    }
    if (found != -2) {
      // (results packed 16 bits per row: a row-indexed write would put s0..s3 in scratch)
      res = (res & ~(0xFFFFull << (16 * r))) | ((qu64)(qu32)(found & 0xFFFF) << (16 * r));
      pm &= pm - 1;
      if (pm) {
        r = __builtin_ctz(pm);
        b = r == 0 ? h0 : r == 1 ? h1 : r == 2 ? h2 : h3;
        probes = 0;
      }
    }
  }
  auto unpack = [&](int q, int& dst) {
    const qu32 v = (qu32)(res >> (16 * q)) & 0xFFFFu;
    if ((pm0 >> q) & 1) dst = v == 0xFFFFu ? -1 : (int)v;
  };
  unpack(0, s0);
  unpack(1, s1);
  unpack(2, s2);
  unpack(3, s3);
}

// lds_probe32 over a table of `nsl` slots (any count: the compact fused table).
__device__ inline int lds_probe32n(qi32* keys, qu32 nsl, qi32 key, qu32 h) {
#pragma unroll 1
  for (int p = 0; p < HA_LDS_MAXP; ++p) {
    const qi32 k = keys[h];
    if (k == key) return (int)h;
    if (k == EMPTY_KEY32) {
      const qi32 old = atomicCAS(&keys[h], EMPTY_KEY32, key);
      if (old == EMPTY_KEY32 || old == key) return (int)h;
    }
    h = h + 1 == nsl ? 0 : h + 1;
  }
  return -1;
}

// ACC_SUM_X row into an LDS window (acc[s] = u0, idx[s] = u1, idx[SS + s] = u2): plan-specialised
// kernels, rows that are not fx_rare.
__device__ inline void lds_fxw_add(qi64* acc, qu64* idx, int SS, int s, qi64 x) {
  fxw_add([&](int w) { return w == 0 ? (qu64*)&acc[s] : &idx[(w - 1) * SS + s]; }, x);
}

// ACC_SUM_X row into a full LDS slot (acc[s] = word 0, idx[k * SS + s] = word k + 1, idx[3 SS + s] =
// status word). false: the row is an input for E (the caller sends it to the global slot).
__device__ inline bool lds_fx_add(qi64* acc, qu64* idx, int SS, int s, qi64 x) {
  const FxRow r = fx_row(x);
  if (r.st & (FX_HUGE | FX_INEXACT)) return false;
  fx_add_row<true>([&](int w) { return w == 0 ? (qu64*)&acc[s] : &idx[(w - 1) * SS + s]; }, r, &idx[3 * SS + s]);
  return true;
}

// LDS MIN / MAX that read first: the atomic only when the value would change the slot. Slots only
// move one way, so a value no better than what the read returns cannot change it; with few groups
// most rows skip their same-address atomics (64 lanes on one slot serialise), and a same-address
// read is a broadcast.
template <typename T>
__device__ __forceinline__ void lds_min_rf(T* p, T x) {
  if (x < __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) atomicMin(p, x);
}
template <typename T>
__device__ __forceinline__ void lds_max_rf(T* p, T x) {
  if (x > __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) atomicMax(p, x);
}

// fp64 MIN/MAX row into LDS accumulators (MaxAccumulator order semantics, Main.kt:538-561).
template <bool IS_MAX>
__device__ inline void lds_f64mm(qi64* acc, qu64* idx, int SS, int s, qi64 x, qu64 row) {
  const double d = bits_f64(x);
  lds_min_rf(&idx[s], row);
  if (d != d) {
    lds_min_rf(&idx[SS + s], row);
  } else {
    if (IS_MAX) lds_max_rf(&acc[s], f64_okey(d));
    else lds_min_rf(&acc[s], f64_okey(d));
    if (d == 0.0) lds_min_rf(&idx[(x < 0 ? 2 : 3) * SS + s], row);
  }
}

}  // namespace qe

#endif  // QE_DEV_HPP
