// K4b: HashAggregateExec (K:605-660) as a one-pass, device-resident partial aggregate, plus the
// fused SelectionExec -> ProjectionExec -> HashAggregateExec pipeline and the partial-record
// export/import used by the two-phase (K:1309-1325) and multi-GPU exchange.
//
// Reference semantics restated:
//  * the group key is the tuple of key values; a null key is a group of its own (List.equals,
//    K:621-627); fp64 keys use Double.equals (all NaNs equal, +0.0 != -0.0);
//  * every aggregate skips null inputs; SUM/MIN/MAX/AVG of a group with no non-null input is null;
//  * MAX/MIN follow MaxAccumulator order semantics (K:538-561) through per-group
//    (ordered key, first-non-null row, first-NaN row, first -0.0 row, first +0.0 row);
//  * output is one batch: key columns then aggregate columns; group order unspecified (K:639).
//
// Data layout in HBM (per state): a global open-addressing table, SoA, capacity G (power of two)
// plus two special slots (G: null key, G+1: key == INT64_MIN, the EMPTY sentinel):
//   keys int64[G+2] | cstar u64[G+2] | per aggregate: acc 64-bit[G+2], nn u64[G+2],
//   and for fp64 MIN/MAX four u64[G+2] first-row indices.
// Kernel: each workgroup owns a private LDS hash table (2^k slots, keys + per-aggregate
// accumulators, LDS 64-bit atomics ds_add_u64 / ds_min_i64 / ds_max_i64 / ds_add_f64 /
// ds_cmpst_b64); a wave reads 256 rows per step (lane: rows 2*lane+{0,1} and 128+2*lane+{0,1},
// so each 16-B load instruction of the wave covers one contiguous KiB of a column); the
// predicate, key packing and aggregate-input expressions are evaluated in registers; at the end
// the workgroup merges its table into the global table with device-scope atomics. Rows whose key
// does not fit the LDS table go straight to the global table; rows/partials the global table
// cannot take are deferred (bitmap / overflow records) and re-applied after the table grows,
// so every row is applied exactly once.
// Roofline: HBM read. Algorithmic bytes per row = sum of the widths of the columns read
// (24 B/row for the headline: k, a, b int64).
#include "qe_internal.hpp"

namespace qe {

constexpr int HA_THREADS = 256;
constexpr int HA_LDS_MAXP = 32;      // probe limit in the LDS table
constexpr int HA_GLOBAL_MAXP = 256;  // probe limit in the global table
constexpr int64_t EMPTY_KEY = INT64_MIN;
constexpr uint64_t NULL_SALT = 0x6A09E667F3BCC909ull;
constexpr size_t HA_LDS_BUDGET = 80 * 1024;  // bytes of LDS per workgroup (2 workgroups / CU)

enum AccKind : int32_t { ACC_NONE = 0, ACC_SUM_I = 1, ACC_SUM_F = 2, ACC_MIN_I = 3, ACC_MAX_I = 4, ACC_MIN_F = 5, ACC_MAX_F = 6 };
enum TokOp : int32_t {
  T_COL = 1, T_LIT, T_I2F0, T_I2F1,
  T_ADD_I, T_SUB_I, T_MUL_I, T_DIV_I,
  T_ADD_F, T_SUB_F, T_MUL_F, T_DIV_F
};

__host__ __device__ inline bool acc_is_f64mm(int32_t acc) { return acc == ACC_MIN_F || acc == ACC_MAX_F; }
__host__ __device__ inline int64_t acc_identity(int32_t acc) {
  switch (acc) {
    case ACC_MIN_I:
    case ACC_MIN_F: return INT64_MAX;
    case ACC_MAX_I:
    case ACC_MAX_F: return INT64_MIN;
    default: return 0;
  }
}

struct DTok {
  int32_t op, arg;
  int64_t lit;
  int32_t lit_null, pad;
};

struct DAgg {
  int32_t fn, acc;
  int32_t pkind;     // 0: no input (COUNT_STAR), 1: column slot, 2: token program
  int32_t col;       // slot for pkind 1
  int32_t cvt_i2f;   // pkind 1: convert integral slot to fp64
  int32_t ntok;
  int32_t track_nn;  // the input can be null in this launch (else nn == cstar)
  int32_t pad;
  DTok tok[QE_MAX_TOKENS];
};

struct DCol {
  const void* p;
  const uint8_t* valid;
  int32_t kind;  // SrcKind
  int32_t pad;
};

struct DTerm {
  int32_t lhs, op, rhs, f64;  // rhs < 0: literal; f64: compare as fp64
  int32_t lhs_f, rhs_f, lit_null, pad;
  int64_t lit;  // in the compare domain
};

struct DTable {
  int64_t* keys;
  uint64_t* cstar;
  int64_t* acc[QE_MAX_AGGS];
  uint64_t* nn[QE_MAX_AGGS];
  uint64_t* idx[QE_MAX_AGGS];  // 4 arrays of cap+2 each (fp64 MIN/MAX only)
  uint64_t cap;                // power of two; slots cap, cap+1 special
  uint64_t* ctl;               // [0] groups, [1] deferred rows, [2] overflow records, [3] lost
};

struct Plan {
  DCol cols[QE_MAX_COLS];
  DTerm terms[QE_MAX_TERMS];
  DAgg aggs[QE_MAX_AGGS];
  DTable t;
  int64_t n, row_base;
  const uint32_t* defer_in;  // retry pass: only these rows
  uint32_t* defer_out;       // rows the global table could not take
  uint8_t* ovf;              // overflow records (LDS flush)
  uint64_t ovf_cap;
  int32_t ncols, nterms, mask_col, naggs;
  int32_t key_mode, nkeys, key_f64, rec_bytes;
  int32_t key_col[QE_MAX_KEYS], key_shift[QE_MAX_KEYS], key_nullbit[QE_MAX_KEYS], pad0;
  int64_t key_fmask[QE_MAX_KEYS];
  int32_t lds_log2, off_cstar;
  int32_t off_acc[QE_MAX_AGGS], off_nn[QE_MAX_AGGS], off_idx[QE_MAX_AGGS];
};

// ---- record layout (export/import/overflow) --------------------------------------------------
// [0] key  [8] flags (bit0 null key)  [16] cstar  then per aggregate: acc, nn, (4 x idx if fp64 MIN/MAX)
__host__ __device__ inline int agg_rec_bytes(int32_t acc) { return 16 + (acc_is_f64mm(acc) ? 32 : 0); }

// ---- global table ------------------------------------------------------------------------------
__device__ __forceinline__ bool gtable_find(const DTable& t, int64_t key, bool knull, uint64_t& slot) {
  if (knull) {
    slot = t.cap;
    return true;
  }
  if (key == EMPTY_KEY) {
    slot = t.cap + 1;
    return true;
  }
  uint64_t h = fmix64((uint64_t)key) & (t.cap - 1);
#pragma unroll 1
  for (int p = 0; p < HA_GLOBAL_MAXP; ++p) {
    int64_t k = __hip_atomic_load(&t.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) {
      slot = h;
      return true;
    }
    if (k == EMPTY_KEY) {
      const int64_t old = (int64_t)atomicCAS((unsigned long long*)&t.keys[h], (unsigned long long)EMPTY_KEY,
                                             (unsigned long long)key);
      if (old == EMPTY_KEY) {
        atomicAdd((unsigned long long*)&t.ctl[0], 1ull);
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

__device__ __forceinline__ void gadd_cstar(const DTable& t, uint64_t slot, uint64_t c) {
  const uint64_t old = atomicAdd((unsigned long long*)&t.cstar[slot], (unsigned long long)c);
  if (slot >= t.cap && old == 0) atomicAdd((unsigned long long*)&t.ctl[0], 1ull);  // special group appears
}

// Combine one aggregate's partial state into global slot `s`.
__device__ __forceinline__ void gcombine(const DTable& t, const DAgg& a, int j, uint64_t s, int64_t acc, uint64_t nn,
                                         uint64_t i0, uint64_t i1, uint64_t i2, uint64_t i3) {
  if (nn == 0) return;
  atomicAdd((unsigned long long*)&t.nn[j][s], (unsigned long long)nn);
  switch (a.acc) {
    case ACC_SUM_I:
      if (acc) atomicAdd((unsigned long long*)&t.acc[j][s], (unsigned long long)acc);
      break;
    case ACC_SUM_F: atomicAdd((double*)&t.acc[j][s], bits_f64(acc)); break;
    case ACC_MIN_I:
    case ACC_MIN_F:
      if (acc != INT64_MAX) atomicMin((long long*)&t.acc[j][s], (long long)acc);
      break;
    case ACC_MAX_I:
    case ACC_MAX_F:
      if (acc != INT64_MIN) atomicMax((long long*)&t.acc[j][s], (long long)acc);
      break;
    default: break;
  }
  if (acc_is_f64mm(a.acc)) {
    const uint64_t stride = t.cap + 2;
    unsigned long long* ix = (unsigned long long*)t.idx[j];
    if (i0 != UINT64_MAX) atomicMin(&ix[s], (unsigned long long)i0);
    if (i1 != UINT64_MAX) atomicMin(&ix[stride + s], (unsigned long long)i1);
    if (i2 != UINT64_MAX) atomicMin(&ix[2 * stride + s], (unsigned long long)i2);
    if (i3 != UINT64_MAX) atomicMin(&ix[3 * stride + s], (unsigned long long)i3);
  }
}

// Per-row contribution of one aggregate in partial form.
struct RowVal {
  int64_t acc;
  uint64_t i0, i1, i2, i3;
};

__device__ __forceinline__ RowVal row_partial(int32_t acck, int64_t x, uint64_t row) {
  RowVal r{acc_identity(acck), UINT64_MAX, UINT64_MAX, UINT64_MAX, UINT64_MAX};
  switch (acck) {
    case ACC_SUM_I:
    case ACC_SUM_F:
    case ACC_MIN_I:
    case ACC_MAX_I: r.acc = x; break;
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

// ---- LDS table -----------------------------------------------------------------------------------
__device__ __forceinline__ int64_t* lds_keys(char* smem) { return (int64_t*)smem; }

__device__ void lds_init(const Plan& P, char* smem) {
  const int SS = (1 << P.lds_log2) + 2;
  int64_t* keys = lds_keys(smem);
  uint32_t* cst = (uint32_t*)(smem + P.off_cstar);
  for (int s = threadIdx.x; s < SS; s += blockDim.x) {
    keys[s] = EMPTY_KEY;
    cst[s] = 0;
  }
#pragma unroll
  for (int j = 0; j < QE_MAX_AGGS; ++j) {
    if (j >= P.naggs) break;
    const DAgg& a = P.aggs[j];
    if (a.acc != ACC_NONE) {
      int64_t* acc = (int64_t*)(smem + P.off_acc[j]);
      const int64_t id = acc_identity(a.acc);
      for (int s = threadIdx.x; s < SS; s += blockDim.x) acc[s] = id;
    }
    if (a.track_nn) {
      uint32_t* nn = (uint32_t*)(smem + P.off_nn[j]);
      for (int s = threadIdx.x; s < SS; s += blockDim.x) nn[s] = 0;
    }
    if (acc_is_f64mm(a.acc)) {
      uint64_t* ix = (uint64_t*)(smem + P.off_idx[j]);
      for (int s = threadIdx.x; s < 4 * SS; s += blockDim.x) ix[s] = UINT64_MAX;
    }
  }
}

// Slot of `key` in the LDS table, inserting it if absent; -1 when the probe limit is hit.
__device__ __forceinline__ int lds_find(const Plan& P, char* smem, int64_t key, bool knull) {
  const int S = 1 << P.lds_log2;
  if (knull) return S;
  if (key == EMPTY_KEY) return S + 1;
  int64_t* keys = lds_keys(smem);
  uint32_t h = lds_hash((uint64_t)key) >> (32 - P.lds_log2);
#pragma unroll 1
  for (int p = 0; p < HA_LDS_MAXP; ++p) {
    const int64_t k = keys[h];
    if (k == key) return (int)h;
    if (k == EMPTY_KEY) {
      const int64_t old = (int64_t)atomicCAS((unsigned long long*)&keys[h], (unsigned long long)EMPTY_KEY,
                                             (unsigned long long)key);
      if (old == EMPTY_KEY || old == key) return (int)h;
    }
    h = (h + 1) & (uint32_t)(S - 1);
  }
  return -1;
}

__device__ __forceinline__ void lds_accum(const Plan& P, char* smem, int j, int s, int64_t x, bool valid,
                                          uint64_t row) {
  const DAgg& a = P.aggs[j];
  if (!valid) return;
  if (a.track_nn) atomicAdd((uint32_t*)(smem + P.off_nn[j]) + s, 1u);
  int64_t* acc = (int64_t*)(smem + P.off_acc[j]);
  switch (a.acc) {
    case ACC_SUM_I: atomicAdd((unsigned long long*)&acc[s], (unsigned long long)x); break;
    case ACC_SUM_F: atomicAdd((double*)&acc[s], bits_f64(x)); break;
    case ACC_MIN_I: atomicMin((long long*)&acc[s], (long long)x); break;
    case ACC_MAX_I: atomicMax((long long*)&acc[s], (long long)x); break;
    case ACC_MIN_F:
    case ACC_MAX_F: {
      const RowVal r = row_partial(a.acc, x, row);
      const int SS = (1 << P.lds_log2) + 2;
      unsigned long long* ix = (unsigned long long*)(smem + P.off_idx[j]);
      atomicMin(&ix[s], (unsigned long long)r.i0);
      if (r.i1 != UINT64_MAX) {
        atomicMin(&ix[SS + s], (unsigned long long)r.i1);
      } else {
        if (a.acc == ACC_MIN_F) atomicMin((long long*)&acc[s], (long long)r.acc);
        else atomicMax((long long*)&acc[s], (long long)r.acc);
        if (r.i2 != UINT64_MAX) atomicMin(&ix[2 * SS + s], (unsigned long long)r.i2);
        if (r.i3 != UINT64_MAX) atomicMin(&ix[3 * SS + s], (unsigned long long)r.i3);
      }
      break;
    }
    default: break;
  }
}

__device__ __forceinline__ void write_record_head(uint8_t* rec, int64_t key, bool knull, uint64_t cstar) {
  ((int64_t*)rec)[0] = key;
  ((uint64_t*)rec)[1] = knull ? 1ull : 0ull;
  ((uint64_t*)rec)[2] = cstar;
}

// Merge the workgroup's LDS table into the global table (or the overflow records).
__device__ void lds_flush(const Plan& P, char* smem) {
  const int S = 1 << P.lds_log2;
  const int SS = S + 2;
  const int64_t* keys = lds_keys(smem);
  const uint32_t* cst = (const uint32_t*)(smem + P.off_cstar);
  for (int s = threadIdx.x; s < SS; s += blockDim.x) {
    const uint32_t c = cst[s];
    if (c == 0) continue;  // an occupied slot always has at least one row
    const bool knull = s == S;
    const int64_t key = s == S ? 0 : (s == S + 1 ? EMPTY_KEY : keys[s]);
    uint64_t gs;
    const bool ok = gtable_find(P.t, key, knull, gs);
    uint8_t* rec = nullptr;
    if (ok) {
      gadd_cstar(P.t, gs, c);
    } else {
      const uint64_t r = atomicAdd((unsigned long long*)&P.t.ctl[2], 1ull);
      if (r >= P.ovf_cap) {
        atomicAdd((unsigned long long*)&P.t.ctl[3], 1ull);
        continue;
      }
      rec = P.ovf + r * (uint64_t)P.rec_bytes;
      write_record_head(rec, key, knull, c);
    }
    int off = 24;
#pragma unroll
    for (int j = 0; j < QE_MAX_AGGS; ++j) {
      if (j >= P.naggs) break;
      const DAgg& a = P.aggs[j];
      const int64_t acc = a.acc != ACC_NONE ? ((const int64_t*)(smem + P.off_acc[j]))[s] : 0;
      const uint64_t nn = a.track_nn ? ((const uint32_t*)(smem + P.off_nn[j]))[s] : c;
      uint64_t i0 = UINT64_MAX, i1 = UINT64_MAX, i2 = UINT64_MAX, i3 = UINT64_MAX;
      if (acc_is_f64mm(a.acc)) {
        const uint64_t* ix = (const uint64_t*)(smem + P.off_idx[j]);
        i0 = ix[s];
        i1 = ix[SS + s];
        i2 = ix[2 * SS + s];
        i3 = ix[3 * SS + s];
      }
      if (ok) {
        if (a.fn != QE_AGG_COUNT_STAR) gcombine(P.t, a, j, gs, acc, nn, i0, i1, i2, i3);
      } else {
        uint64_t* f = (uint64_t*)(rec + off);
        f[0] = (uint64_t)acc;
        f[1] = nn;
        if (acc_is_f64mm(a.acc)) {
          f[2] = i0;
          f[3] = i1;
          f[4] = i2;
          f[5] = i3;
        }
      }
      off += agg_rec_bytes(a.acc);
    }
  }
}

// ---- column registers -----------------------------------------------------------------------------
// A wave step covers 256 rows; lane holds rows base + 128*q + 2*lane + e (q, e in {0,1}) as r = 2q+e.
// All columns of the step live in ONE register vector V (element 4*slot + r) and one u32 of validity
// nibbles (bit 4*slot + r). Consumers index them with a wave-uniform slot (and a uniform r), which
// hipcc lowers to s_set_gpr_idx VGPR indexing: no scratch, no per-slot select chains.
template <int W>
struct VecT {
  typedef long long type __attribute__((ext_vector_type(W)));
};
template <int NC>
struct ColRegs {
  static constexpr int W = NC <= 1 ? 4 : NC <= 2 ? 8 : NC <= 4 ? 16 : 32;
  typename VecT<W>::type v;
  uint32_t valid;  // nibble per slot
  __device__ __forceinline__ int64_t get(int slot, int r) const { return v[4 * slot + r]; }
  __device__ __forceinline__ bool ok(int slot, int r) const { return (valid >> (4 * slot + r)) & 1u; }
};

typedef long long i64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int64_t row_of(int64_t base, int lane, int r) {
  return base + 128 * (r >> 1) + 2 * lane + (r & 1);
}

template <int NC>
__device__ __forceinline__ void load_cols(const Plan& P, int64_t base, int lane, bool full, ColRegs<NC>& R) {
  R.valid = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c >= P.ncols) {
#pragma unroll
      for (int r = 0; r < 4; ++r) R.v[4 * c + r] = 0;
      continue;
    }
    const DCol& col = P.cols[c];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t r0 = base + 128 * q + 2 * lane;
      int64_t a = 0, b = 0;
      if (full) {
        switch (col.kind) {
          case K_I64:
          case K_F64: {
            const i64x2 t = *(const i64x2*)((const int64_t*)col.p + r0);
            a = t.x;
            b = t.y;
            break;
          }
          case K_I32: {
            const int2 t = *(const int2*)((const int32_t*)col.p + r0);
            a = t.x;
            b = t.y;
            break;
          }
          case K_U8: {
            const uint16_t t = *(const uint16_t*)((const uint8_t*)col.p + r0);
            a = t & 0xFF;
            b = t >> 8;
            break;
          }
          default: {  // K_BOOL
            const uint32_t t = ((const uint8_t*)col.p)[r0 >> 3] >> (r0 & 7);
            a = t & 1;
            b = (t >> 1) & 1;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int64_t r = r0 + e;
          int64_t x = 0;
          if (r < P.n) {
            switch (col.kind) {
              case K_I64:
              case K_F64: x = ((const int64_t*)col.p)[r]; break;
              case K_I32: x = ((const int32_t*)col.p)[r]; break;
              case K_U8: x = ((const uint8_t*)col.p)[r]; break;
              default: x = (((const uint8_t*)col.p)[r >> 3] >> (r & 7)) & 1;
            }
          }
          if (e) b = x;
          else a = x;
        }
      }
      R.v[4 * c + 2 * q] = a;
      R.v[4 * c + 2 * q + 1] = b;
      const uint32_t vv = col.valid ? ((uint32_t)(col.valid[r0 >> 3] >> (r0 & 7)) & 3u) : 3u;
      R.valid |= vv << (4 * c + 2 * q);
    }
  }
}

__device__ __forceinline__ bool cmp_i(int32_t op, int64_t a, int64_t b) {
  switch (op) {
    case QE_OP_EQ: return a == b;
    case QE_OP_NE: return a != b;
    case QE_OP_LT: return a < b;
    case QE_OP_LE: return a <= b;
    case QE_OP_GT: return a > b;
    default: return a >= b;
  }
}
__device__ __forceinline__ bool cmp_f(int32_t op, double a, double b) {
  switch (op) {
    case QE_OP_EQ: return a == b;
    case QE_OP_NE: return a != b;
    case QE_OP_LT: return a < b;
    case QE_OP_LE: return a <= b;
    case QE_OP_GT: return a > b;
    default: return a >= b;
  }
}

// Postfix program with a 4-deep register stack (constant-index rotations only).
template <int NC>
__device__ __forceinline__ int64_t eval_program(const DAgg& a, const ColRegs<NC>& R, int r, bool& valid) {
  int64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  bool n0 = true, n1 = true, n2 = true, n3 = true;  // validity
  for (int t = 0; t < a.ntok; ++t) {
    const DTok& k = a.tok[t];
    const int op = k.op;
    if (op == T_COL || op == T_LIT) {
      s3 = s2; n3 = n2;
      s2 = s1; n2 = n1;
      s1 = s0; n1 = n0;
      if (op == T_COL) {
        s0 = R.get(k.arg, r);
        n0 = R.ok(k.arg, r);
      } else {
        s0 = k.lit;
        n0 = !k.lit_null;
      }
    } else if (op == T_I2F0) {
      s0 = f64_bits((double)s0);
    } else if (op == T_I2F1) {
      s1 = f64_bits((double)s1);
    } else {
      int64_t res;
      bool ok = n0 && n1;
      const uint64_t ua = (uint64_t)s1, ub = (uint64_t)s0;
      switch (op) {
        case T_ADD_I: res = (int64_t)(ua + ub); break;
        case T_SUB_I: res = (int64_t)(ua - ub); break;
        case T_MUL_I: res = (int64_t)(ua * ub); break;
        case T_DIV_I:
          if (s0 == 0) { res = 0; ok = false; }
          else if (s0 == -1) res = (int64_t)(0ull - ua);
          else res = s1 / s0;
          break;
        case T_ADD_F: res = f64_bits(bits_f64(s1) + bits_f64(s0)); break;
        case T_SUB_F: res = f64_bits(bits_f64(s1) - bits_f64(s0)); break;
        case T_MUL_F: res = f64_bits(bits_f64(s1) * bits_f64(s0)); break;
        default: res = f64_bits(bits_f64(s1) / bits_f64(s0)); break;
      }
      s0 = res; n0 = ok;
      s1 = s2; n1 = n2;
      s2 = s3; n2 = n3;
    }
  }
  valid = n0;
  return s0;
}

// Aggregate j's input for row r: value bits, validity in `valid`.
template <int NC>
__device__ __forceinline__ int64_t eval_input(const DAgg& a, const ColRegs<NC>& R, int r, bool& valid) {
  if (a.pkind == 1) {
    valid = R.ok(a.col, r);
    const int64_t x = R.get(a.col, r);
    return a.cvt_i2f ? f64_bits((double)x) : x;
  }
  return eval_program<NC>(a, R, r, valid);
}

template <int NC, bool USE_LDS>
__global__ void __launch_bounds__(HA_THREADS) k_hashagg(const Plan P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (USE_LDS) {
    lds_init(P, smem);
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t base = wave * 256; base < P.n; base += nwaves * 256) {
    const bool full = base + 256 <= P.n;
    ColRegs<NC> R;
    load_cols<NC>(P, base, lane, full, R);
    uint32_t act = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) act |= (uint32_t)(row_of(base, lane, r) < P.n) << r;
    if (P.defer_in) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row_of(base, lane, r);
        if (row < P.n && !((P.defer_in[row >> 5] >> (row & 31)) & 1)) act &= ~(1u << r);
      }
    }
    if (P.mask_col >= 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (!(R.get(P.mask_col, r) & 1) || !R.ok(P.mask_col, r)) act &= ~(1u << r);
    }
    for (int t = 0; t < P.nterms; ++t) {
      const DTerm& T = P.terms[t];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t a = R.get(T.lhs, r);
        const int64_t b = T.rhs >= 0 ? R.get(T.rhs, r) : T.lit;
        const bool bv = T.rhs >= 0 ? R.ok(T.rhs, r) : !T.lit_null;
        bool ok;
        if (T.f64) {
          const double da = T.lhs_f ? bits_f64(a) : (double)a;
          const double db = T.rhs_f ? bits_f64(b) : (double)b;
          ok = cmp_f(T.op, da, db);
        } else {
          ok = cmp_i(T.op, a, b);
        }
        if (!(ok && R.ok(T.lhs, r) && bv)) act &= ~(1u << r);
      }
    }
    if (act == 0) continue;
#pragma unroll 1
    for (int r = 0; r < 4; ++r) {
      if (!((act >> r) & 1)) continue;
      const uint64_t row = (uint64_t)(P.row_base + row_of(base, lane, r));
      // ---- group key
      int64_t key = 0;
      bool knull = false;
      if (P.key_mode == 1) {
        key = R.get(P.key_col[0], r);
        knull = !R.ok(P.key_col[0], r);
        if (P.key_f64 && bits_f64(key) != bits_f64(key)) key = 0x7FF8000000000000ll;  // Double.equals: one NaN
        if (knull) key = 0;
      } else if (P.key_mode == 2) {
        for (int k = 0; k < P.nkeys; ++k) {
          const int c = P.key_col[k];
          const bool isn = !R.ok(c, r);
          const int64_t x = isn ? 0 : (R.get(c, r) & P.key_fmask[k]);
          key |= (x << P.key_shift[k]) | ((int64_t)isn << P.key_nullbit[k]);
        }
      }
      // ---- slot: LDS table first, the global table when the LDS probe fails
      int s = -1;
      uint64_t gs = 0;
      if (USE_LDS) s = lds_find(P, smem, key, knull);
      if (s >= 0) {
        atomicAdd((uint32_t*)(smem + P.off_cstar) + s, 1u);
      } else {
        if (!gtable_find(P.t, key, knull, gs)) {
          const int64_t lr = row_of(base, lane, r);
          atomicOr(&P.defer_out[lr >> 5], 1u << (lr & 31));
          atomicAdd((unsigned long long*)&P.t.ctl[1], 1ull);
          continue;
        }
        gadd_cstar(P.t, gs, 1);
      }
      // ---- aggregate inputs (one inlined evaluator per kernel)
      for (int j = 0; j < P.naggs; ++j) {
        const DAgg& a = P.aggs[j];
        if (a.pkind == 0) continue;
        bool valid;
        const int64_t x = eval_input<NC>(a, R, r, valid);
        if (s >= 0) {
          lds_accum(P, smem, j, s, x, valid, row);
        } else if (valid) {
          const RowVal rv = row_partial(a.acc, x, row);
          gcombine(P.t, a, j, gs, rv.acc, 1, rv.i0, rv.i1, rv.i2, rv.i3);
        }
      }
    }
  }
  if (USE_LDS) {
    __syncthreads();
    lds_flush(P, smem);
  }
}

// ---- table maintenance kernels -------------------------------------------------------------------
struct AggMeta {
  int32_t naggs;
  int32_t fn[QE_MAX_AGGS];
  int32_t acc[QE_MAX_AGGS];
};

__global__ void k_table_init(DTable t, AggMeta m) {
  const uint64_t SS = t.cap + 2;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < SS; s += (uint64_t)gridDim.x * blockDim.x) {
    t.keys[s] = EMPTY_KEY;
    t.cstar[s] = 0;
    for (int j = 0; j < m.naggs; ++j) {
      t.acc[j][s] = acc_identity(m.acc[j]);
      t.nn[j][s] = 0;
      if (acc_is_f64mm(m.acc[j]))
        for (int k = 0; k < 4; ++k) t.idx[j][k * SS + s] = UINT64_MAX;
    }
  }
}

__device__ __forceinline__ bool gslot_occupied(const DTable& t, uint64_t s) {
  return s < t.cap ? t.keys[s] != EMPTY_KEY : t.cstar[s] > 0;
}

// Merge every occupied slot of `src` into `dst` (table growth).
__global__ void k_rehash(DTable src, DTable dst, AggMeta m) {
  const uint64_t SS = src.cap + 2;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < SS; s += (uint64_t)gridDim.x * blockDim.x) {
    if (!gslot_occupied(src, s)) continue;
    const bool knull = s == src.cap;
    const int64_t key = knull ? 0 : (s == src.cap + 1 ? EMPTY_KEY : src.keys[s]);
    uint64_t d;
    if (!gtable_find(dst, key, knull, d)) {
      atomicAdd((unsigned long long*)&dst.ctl[3], 1ull);
      continue;
    }
    gadd_cstar(dst, d, src.cstar[s]);
    for (int j = 0; j < m.naggs; ++j) {
      DAgg a{};
      a.fn = m.fn[j];
      a.acc = m.acc[j];
      uint64_t i[4] = {UINT64_MAX, UINT64_MAX, UINT64_MAX, UINT64_MAX};
      if (acc_is_f64mm(a.acc))
        for (int k = 0; k < 4; ++k) i[k] = src.idx[j][k * SS + s];
      gcombine(dst, a, j, d, src.acc[j][s], src.nn[j][s], i[0], i[1], i[2], i[3]);
    }
  }
}

// Merge fixed-size records (export format) into `dst`.
__global__ void k_import(const uint8_t* __restrict__ recs, int64_t nrec, int32_t rec_bytes, DTable dst, AggMeta m) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrec; r += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* rec = recs + r * rec_bytes;
    const int64_t key = ((const int64_t*)rec)[0];
    const bool knull = ((const uint64_t*)rec)[1] & 1;
    const uint64_t c = ((const uint64_t*)rec)[2];
    uint64_t d;
    if (!gtable_find(dst, key, knull, d)) {
      atomicAdd((unsigned long long*)&dst.ctl[3], 1ull);
      continue;
    }
    gadd_cstar(dst, d, c);
    int off = 24;
    for (int j = 0; j < m.naggs; ++j) {
      DAgg a{};
      a.fn = m.fn[j];
      a.acc = m.acc[j];
      const uint64_t* f = (const uint64_t*)(rec + off);
      if (a.fn != QE_AGG_COUNT_STAR) {
        if (acc_is_f64mm(a.acc)) gcombine(dst, a, j, d, (int64_t)f[0], f[1], f[2], f[3], f[4], f[5]);
        else gcombine(dst, a, j, d, (int64_t)f[0], f[1], UINT64_MAX, UINT64_MAX, UINT64_MAX, UINT64_MAX);
      }
      off += agg_rec_bytes(a.acc);
    }
  }
}

__device__ __forceinline__ uint32_t partition_of(int64_t key, bool knull, int32_t nparts) {
  const uint64_t h = fmix64((uint64_t)key ^ (knull ? NULL_SALT : 0ull));
  return (uint32_t)(((h >> 32) * (uint64_t)nparts) >> 32);
}

__global__ void k_export_count(DTable t, int32_t nparts, unsigned long long* counts) {
  const uint64_t SS = t.cap + 2;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < SS; s += (uint64_t)gridDim.x * blockDim.x) {
    if (!gslot_occupied(t, s)) continue;
    const bool knull = s == t.cap;
    const int64_t key = knull ? 0 : (s == t.cap + 1 ? EMPTY_KEY : t.keys[s]);
    atomicAdd(&counts[partition_of(key, knull, nparts)], 1ull);
  }
}

__global__ void k_export(DTable t, AggMeta m, int32_t nparts, int32_t rec_bytes, unsigned long long* cursor,
                         uint8_t* __restrict__ dst) {
  const uint64_t SS = t.cap + 2;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < SS; s += (uint64_t)gridDim.x * blockDim.x) {
    if (!gslot_occupied(t, s)) continue;
    const bool knull = s == t.cap;
    const int64_t key = knull ? 0 : (s == t.cap + 1 ? EMPTY_KEY : t.keys[s]);
    const uint32_t p = partition_of(key, knull, nparts);
    const uint64_t pos = atomicAdd(&cursor[p], 1ull);
    uint8_t* rec = dst + pos * (uint64_t)rec_bytes;
    write_record_head(rec, key, knull, t.cstar[s]);
    int off = 24;
    for (int j = 0; j < m.naggs; ++j) {
      uint64_t* f = (uint64_t*)(rec + off);
      f[0] = (uint64_t)t.acc[j][s];
      f[1] = t.nn[j][s];
      if (acc_is_f64mm(m.acc[j]))
        for (int k = 0; k < 4; ++k) f[2 + k] = t.idx[j][k * SS + s];
      off += agg_rec_bytes(m.acc[j]);
    }
  }
}

// ---- finalize: occupied slots -> one output batch --------------------------------------------------
__global__ void k_occ_count(DTable t, int64_t* __restrict__ tile_counts, int32_t tile_slots) {
  // one block per tile of `tile_slots` slots
  __shared__ int64_t part[4];
  const uint64_t SS = t.cap + 2;
  const uint64_t s0 = (uint64_t)blockIdx.x * tile_slots;
  int64_t c = 0;
  for (int i = threadIdx.x; i < tile_slots; i += blockDim.x) {
    const uint64_t s = s0 + i;
    if (s < SS && gslot_occupied(t, s)) ++c;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

struct OutCols {
  qe_column keys[QE_MAX_KEYS];
  qe_column aggs[QE_MAX_AGGS];
};

struct KeyMeta {
  int32_t mode, nkeys;
  int32_t type[QE_MAX_KEYS], shift[QE_MAX_KEYS], nullbit[QE_MAX_KEYS];
  int64_t fmask[QE_MAX_KEYS];
};

__device__ __forceinline__ void set_bit(uint8_t* bm, int64_t i, bool v) {
  // bytes are written by whole 32-bit atomics: the host zeroes validity buffers first
  if (v) atomicOr((uint32_t*)bm + (i >> 5), 1u << (i & 31));
}

__device__ __forceinline__ void store_typed(void* p, int32_t type, int64_t i, int64_t x) {
  switch (type) {
    case QE_TYPE_INT64:
    case QE_TYPE_FLOAT64: ((int64_t*)p)[i] = x; break;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: ((int32_t*)p)[i] = (int32_t)x; break;
    default: ((uint8_t*)p)[i] = (uint8_t)x;
  }
}

__global__ void k_finalize(DTable t, AggMeta m, KeyMeta km, const int64_t* __restrict__ tile_offsets,
                           int32_t tile_slots, OutCols out) {
  // one block per tile; each wave scans its slots in order (ballot + popc keeps slot order)
  __shared__ int wtot[4];
  const uint64_t SS = t.cap + 2;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  int64_t base = tile_offsets[blockIdx.x];
  for (int it = 0; it < tile_slots; it += blockDim.x) {
    const uint64_t s = (uint64_t)blockIdx.x * tile_slots + it + threadIdx.x;
    const bool occ = (it + (int)threadIdx.x) < tile_slots && s < SS && gslot_occupied(t, s);
    const uint64_t b = __ballot(occ);
    if (lane == 0) wtot[wid] = __popcll(b);
    __syncthreads();
    int woff = 0, btot = 0;
    for (int w = 0; w < 4; ++w) {
      woff += w < wid ? wtot[w] : 0;
      btot += wtot[w];
    }
    if (occ) {
      const int64_t o = base + woff + __popcll(b & lt);
      const bool knull = s == t.cap;
      const int64_t key = knull ? 0 : (s == t.cap + 1 ? EMPTY_KEY : t.keys[s]);
      // keys
      if (km.mode == 1) {
        store_typed(out.keys[0].values, km.type[0], o, key);
        if (out.keys[0].validity) set_bit(out.keys[0].validity, o, !knull);
      } else if (km.mode == 2) {
        for (int k = 0; k < km.nkeys; ++k) {
          const bool isn = (key >> km.nullbit[k]) & 1;
          int64_t x = (key >> km.shift[k]) & km.fmask[k];
          if (km.type[k] == QE_TYPE_INT32 || km.type[k] == QE_TYPE_DATE32) x = (int64_t)(int32_t)x;  // sign
          store_typed(out.keys[k].values, km.type[k], o, x);
          if (out.keys[k].validity) set_bit(out.keys[k].validity, o, !isn);
        }
      }
      // aggregates
      for (int j = 0; j < m.naggs; ++j) {
        const uint64_t nn = t.nn[j][s];
        const int64_t acc = t.acc[j][s];
        int64_t val = 0;
        bool valid = nn > 0;
        switch (m.fn[j]) {
          case QE_AGG_COUNT: val = (int64_t)nn; valid = true; break;
          case QE_AGG_COUNT_STAR: val = (int64_t)t.cstar[s]; valid = true; break;
          case QE_AGG_AVG: val = f64_bits(bits_f64(acc) / (double)nn); break;
          default:
            if (acc_is_f64mm(m.acc[j])) {
              const uint64_t i0 = t.idx[j][s], i1 = t.idx[j][SS + s];
              const uint64_t i2 = t.idx[j][2 * SS + s], i3 = t.idx[j][3 * SS + s];
              if (i1 != UINT64_MAX && i1 == i0) {
                val = 0x7FF8000000000000ll;  // first non-null value was NaN: sticky seed
              } else {
                const double d = okey_f64(acc);
                val = d == 0.0 ? f64_bits(i2 < i3 ? -0.0 : 0.0) : f64_bits(d);
              }
            } else {
              val = acc;
            }
        }
        ((int64_t*)out.aggs[j].values)[o] = valid ? val : 0;
        if (out.aggs[j].validity) set_bit(out.aggs[j].validity, o, valid);
      }
    }
    base += btot;
    __syncthreads();
  }
}

}  // namespace qe

// =====================================================================================================
// Host side
// =====================================================================================================
using namespace qe;

struct qe_hashagg {
  qe_ctx* ctx = nullptr;
  int32_t nkeys = 0;
  int32_t key_types[QE_MAX_KEYS] = {};
  int32_t naggs = 0;
  qe_agg_desc aggs[QE_MAX_AGGS] = {};
  int32_t acc[QE_MAX_AGGS] = {};
  KeyMeta km{};
  int32_t rec_bytes = 0;
  int64_t row_base = 0;
  // global table
  void* table_mem = nullptr;
  DTable t{};
  uint64_t* ctl = nullptr;  // device, 8 words
  // LDS sizing
  int32_t lds_log2 = 0;  // largest LDS table (log2 slots); 0 => global-only mode
  int32_t lds_log2_min = 0;
  int grid = 0;          // workgroups per launch (cap)
  // overflow records
  uint8_t* ovf = nullptr;
  uint64_t ovf_cap = 0;
  // deferred-row bitmaps
  uint32_t* defer[2] = {nullptr, nullptr};
  size_t defer_words = 0;
  bool defer_dirty[2] = {false, false};
  // HIP events around the aggregation kernel launches of the last update (measurement hook)
  hipEvent_t ev[2] = {nullptr, nullptr};
  double last_kernel_ms = 0.0;
  int last_launches = 0;
};

namespace qe {

static AggMeta agg_meta(const qe_hashagg* h) {
  AggMeta m{};
  m.naggs = h->naggs;
  for (int j = 0; j < h->naggs; ++j) {
    m.fn[j] = h->aggs[j].fn;
    m.acc[j] = h->acc[j];
  }
  return m;
}

static size_t table_bytes(const qe_hashagg* h, uint64_t cap) {
  const uint64_t SS = cap + 2;
  size_t b = 16 * SS;
  for (int j = 0; j < h->naggs; ++j) b += (16 + (acc_is_f64mm(h->acc[j]) ? 32 : 0)) * SS;
  return b;
}

static int table_alloc(qe_hashagg* h, uint64_t cap, void** mem, DTable* t) {
  const size_t bytes = table_bytes(h, cap);
  if (hipMalloc(mem, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return fail(QE_ERR_OOM, "hash table allocation of %zu bytes failed", bytes);
  }
  const uint64_t SS = cap + 2;
  char* p = (char*)*mem;
  *t = DTable{};
  t->keys = (int64_t*)p;
  p += 8 * SS;
  t->cstar = (uint64_t*)p;
  p += 8 * SS;
  for (int j = 0; j < h->naggs; ++j) {
    t->acc[j] = (int64_t*)p;
    p += 8 * SS;
    t->nn[j] = (uint64_t*)p;
    p += 8 * SS;
    if (acc_is_f64mm(h->acc[j])) {
      t->idx[j] = (uint64_t*)p;
      p += 32 * SS;
    }
  }
  t->cap = cap;
  t->ctl = h->ctl;
  const int grid = (int)std::min<uint64_t>(div_up(SS, 256), 4096);
  hipLaunchKernelGGL(k_table_init, dim3(grid), dim3(256), 0, h->ctx->stream, *t, agg_meta(h));
  return launch_check("k_table_init");
}

static int read_ctl(qe_hashagg* h, uint64_t out[4]) {
  void* p;
  QE_TRY(ctx_pinned(h->ctx, 32, &p));
  QE_HIP(hipMemcpyAsync(p, h->ctl, 32, hipMemcpyDeviceToHost, h->ctx->stream));
  QE_HIP(hipStreamSynchronize(h->ctx->stream));
  memcpy(out, p, 32);
  return QE_OK;
}

static uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Grow the global table to at least `want_cap` slots and re-insert every group.
static int table_grow(qe_hashagg* h, uint64_t want_cap) {
  const uint64_t cap = next_pow2(want_cap);
  if (cap <= h->t.cap) return QE_OK;
  void* mem;
  DTable nt;
  QE_TRY(table_alloc(h, cap, &mem, &nt));
  // the group counter is recomputed by the re-insert
  QE_HIP(hipMemsetAsync(h->ctl, 0, 8, h->ctx->stream));
  QE_HIP(hipMemsetAsync(h->ctl + 3, 0, 8, h->ctx->stream));
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 8192);
  hipLaunchKernelGGL(k_rehash, dim3(grid), dim3(256), 0, h->ctx->stream, h->t, nt, agg_meta(h));
  QE_TRY(launch_check("k_rehash"));
  uint64_t c[4];
  QE_TRY(read_ctl(h, c));  // synchronises: the old table can go
  QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash table rehash lost %llu groups", (unsigned long long)c[3]);
  QE_HIP(hipFree(h->table_mem));
  h->table_mem = mem;
  h->t = nt;
  return QE_OK;
}

static int import_records(qe_hashagg* h, const void* recs, int64_t nrec) {
  if (nrec <= 0) return QE_OK;
  const int grid = (int)std::min<uint64_t>(div_up((uint64_t)nrec, 256), 8192);
  hipLaunchKernelGGL(k_import, dim3(grid), dim3(256), 0, h->ctx->stream, (const uint8_t*)recs, nrec, h->rec_bytes,
                     h->t, agg_meta(h));
  QE_TRY(launch_check("k_import"));
  uint64_t c[4];
  QE_TRY(read_ctl(h, c));
  QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash table import lost %llu groups", (unsigned long long)c[3]);
  return QE_OK;
}

static int ensure_defer(qe_hashagg* h, int64_t n) {
  const size_t words = (size_t)div_up((uint64_t)n, 32);
  if (words <= h->defer_words) return QE_OK;
  for (int i = 0; i < 2; ++i) {
    if (h->defer[i]) QE_HIP(hipFree(h->defer[i]));
    h->defer[i] = nullptr;
  }
  for (int i = 0; i < 2; ++i) {
    if (hipMalloc(&h->defer[i], words * 4) != hipSuccess) {
      (void)hipGetLastError();
      return fail(QE_ERR_OOM, "defer bitmap allocation failed");
    }
    QE_HIP(hipMemsetAsync(h->defer[i], 0, words * 4, h->ctx->stream));
    h->defer_dirty[i] = false;
  }
  h->defer_words = words;
  return QE_OK;
}

// Compiled launch description (host side mirror of qe_fused_spec after type checking).
static int compile_plan(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec, Plan* P) {
  *P = Plan{};
  QE_CHECK(ncols >= 1 && ncols <= QE_MAX_COLS, QE_ERR_UNSUPPORTED, "fused aggregate takes 1..%d columns (got %d)",
           QE_MAX_COLS, ncols);
  const int64_t n = cols[0].length;
  bool col_f64[QE_MAX_COLS];
  for (int c = 0; c < ncols; ++c) {
    const qe_column& k = cols[c];
    QE_CHECK(k.length == n, QE_ERR_INVALID_ARG, "column %d has %lld rows, column 0 %lld", c, (long long)k.length,
             (long long)n);
    const int32_t kind = kind_of(k.type);
    QE_CHECK(kind >= K_I64 && kind <= K_BOOL, QE_ERR_UNSUPPORTED, "column %d: type %d not supported", c, k.type);
    QE_CHECK(k.values || n == 0, QE_ERR_INVALID_ARG, "column %d: null values", c);
    P->cols[c] = DCol{k.values, k.validity, kind, 0};
    col_f64[c] = k.type == QE_TYPE_FLOAT64;
  }
  P->ncols = ncols;
  P->n = n;
  P->row_base = h->row_base;
  // mask
  P->mask_col = spec->mask_col;
  if (spec->mask_col >= 0) {
    QE_CHECK(spec->mask_col < ncols && cols[spec->mask_col].type == QE_TYPE_BOOL, QE_ERR_INVALID_ARG,
             "mask_col must name a BOOL column");
  }
  // predicate terms
  QE_CHECK(spec->nterms >= 0 && spec->nterms <= QE_MAX_TERMS, QE_ERR_UNSUPPORTED, "too many predicate terms");
  P->nterms = spec->nterms;
  for (int i = 0; i < spec->nterms; ++i) {
    const qe_pred_term& s = spec->terms[i];
    DTerm& d = P->terms[i];
    QE_CHECK(s.col >= 0 && s.col < ncols && is_fixed(cols[s.col].type), QE_ERR_INVALID_ARG, "term %d: bad lhs column", i);
    QE_CHECK(s.op >= QE_OP_EQ && s.op <= QE_OP_GE, QE_ERR_INVALID_ARG, "term %d: bad comparison op", i);
    d.lhs = s.col;
    d.op = s.op;
    d.lhs_f = col_f64[s.col];
    d.rhs = s.rhs_col;
    if (s.rhs_col >= 0) {
      QE_CHECK(s.rhs_col < ncols && is_fixed(cols[s.rhs_col].type), QE_ERR_INVALID_ARG, "term %d: bad rhs column", i);
      d.rhs_f = col_f64[s.rhs_col];
      d.f64 = d.lhs_f || d.rhs_f;
    } else {
      QE_CHECK(s.lit.type == QE_TYPE_INT64 || s.lit.type == QE_TYPE_FLOAT64, QE_ERR_UNSUPPORTED,
               "term %d: literal type", i);
      const bool lf = s.lit.type == QE_TYPE_FLOAT64;
      d.f64 = d.lhs_f || lf;
      d.rhs_f = 1;
      d.lit_null = s.lit.is_null;
      d.lit = (d.f64 && !lf) ? f64_bits((double)s.lit.bits) : s.lit.bits;
    }
  }
  // keys
  P->key_mode = h->km.mode;
  P->nkeys = h->nkeys;
  for (int k = 0; k < h->nkeys; ++k) {
    const int c = spec->key_cols[k];
    QE_CHECK(c >= 0 && c < ncols, QE_ERR_INVALID_ARG, "key %d: bad column slot", k);
    QE_CHECK(cols[c].type == h->key_types[k], QE_ERR_INVALID_ARG, "key %d: column type %d, declared %d", k,
             cols[c].type, h->key_types[k]);
    P->key_col[k] = c;
    P->key_shift[k] = h->km.shift[k];
    P->key_nullbit[k] = h->km.nullbit[k];
    P->key_fmask[k] = h->km.fmask[k];
  }
  P->key_f64 = h->nkeys == 1 && h->key_types[0] == QE_TYPE_FLOAT64;
  // aggregates
  P->naggs = h->naggs;
  for (int j = 0; j < h->naggs; ++j) {
    DAgg& a = P->aggs[j];
    a.fn = h->aggs[j].fn;
    a.acc = h->acc[j];
    if (a.fn == QE_AGG_COUNT_STAR) {
      a.pkind = 0;
      continue;
    }
    const qe_agg_program& pg = spec->inputs[j];
    QE_CHECK(pg.ntokens >= 1 && pg.ntokens <= QE_MAX_TOKENS, QE_ERR_INVALID_ARG, "aggregate %d: empty program", j);
    // type-check the postfix program; emit typed tokens
    bool st_f[QE_MAX_TOKENS + 4];
    int depth = 0, nt = 0;
    bool nullable = false;
    auto emit = [&](int32_t op, int32_t arg, int64_t lit, int32_t lit_null) -> int {
      QE_CHECK(nt < QE_MAX_TOKENS, QE_ERR_UNSUPPORTED, "aggregate %d: program too long after type promotion", j);
      a.tok[nt++] = DTok{op, arg, lit, lit_null, 0};
      return QE_OK;
    };
    for (int t = 0; t < pg.ntokens; ++t) {
      const qe_token& tk = pg.tokens[t];
      if (tk.op == QE_TOK_COL) {
        QE_CHECK(tk.arg >= 0 && tk.arg < ncols && is_fixed(cols[tk.arg].type), QE_ERR_INVALID_ARG,
                 "aggregate %d: bad column slot %d", j, tk.arg);
        QE_CHECK(depth < 4, QE_ERR_UNSUPPORTED, "aggregate %d: expression deeper than 4", j);
        QE_TRY(emit(T_COL, tk.arg, 0, 0));
        st_f[depth++] = col_f64[tk.arg];
        nullable = nullable || cols[tk.arg].validity != nullptr;
      } else if (tk.op == QE_TOK_LIT) {
        QE_CHECK(tk.lit.type == QE_TYPE_INT64 || tk.lit.type == QE_TYPE_FLOAT64, QE_ERR_UNSUPPORTED,
                 "aggregate %d: literal type", j);
        QE_CHECK(depth < 4, QE_ERR_UNSUPPORTED, "aggregate %d: expression deeper than 4", j);
        QE_TRY(emit(T_LIT, 0, tk.lit.bits, tk.lit.is_null));
        st_f[depth++] = tk.lit.type == QE_TYPE_FLOAT64;
        nullable = nullable || tk.lit.is_null;
      } else if (tk.op >= QE_TOK_ADD && tk.op <= QE_TOK_DIV) {
        QE_CHECK(depth >= 2, QE_ERR_INVALID_ARG, "aggregate %d: stack underflow", j);
        const bool f = st_f[depth - 1] || st_f[depth - 2];
        if (f && !st_f[depth - 1]) QE_TRY(emit(T_I2F0, 0, 0, 0));
        if (f && !st_f[depth - 2]) QE_TRY(emit(T_I2F1, 0, 0, 0));
        const int32_t base_op = f ? T_ADD_F : T_ADD_I;
        QE_TRY(emit(base_op + (tk.op - QE_TOK_ADD), 0, 0, 0));
        if (!f && tk.op == QE_TOK_DIV) nullable = true;  // x / 0 -> null
        --depth;
        st_f[depth - 1] = f;
      } else {
        return fail(QE_ERR_INVALID_ARG, "aggregate %d: bad token op %d", j, tk.op);
      }
    }
    QE_CHECK(depth == 1, QE_ERR_INVALID_ARG, "aggregate %d: program leaves %d values", j, depth);
    const bool want_f = h->aggs[j].fn == QE_AGG_AVG || h->aggs[j].input_type == QE_TYPE_FLOAT64;
    const bool is_f = st_f[0];
    if (a.fn != QE_AGG_COUNT) {
      QE_CHECK(!(is_f && !want_f), QE_ERR_INVALID_ARG,
               "aggregate %d: fp64 input for an int64 aggregate (declare input_type FLOAT64)", j);
      if (want_f && !is_f) QE_TRY(emit(T_I2F0, 0, 0, 0));
    }
    a.ntok = nt;
    a.track_nn = nullable ? 1 : 0;
    if (nt == 1 && a.tok[0].op == T_COL) {
      a.pkind = 1;
      a.col = a.tok[0].arg;
    } else if (nt == 2 && a.tok[0].op == T_COL && a.tok[1].op == T_I2F0) {
      a.pkind = 1;
      a.col = a.tok[0].arg;
      a.cvt_i2f = 1;
    } else {
      a.pkind = 2;
    }
  }
  P->rec_bytes = h->rec_bytes;
  return QE_OK;
}

// LDS layout for a table of 2^log2 slots under this launch's aggregates. Returns bytes.
static size_t lds_layout_at(const qe_hashagg* h, Plan* P, int log2) {
  const size_t SS = ((size_t)1 << log2) + 2;
  size_t off = 8 * SS;  // keys
  P->off_cstar = (int32_t)off;
  off += 4 * SS;
  off = (off + 15) & ~size_t(15);
  for (int j = 0; j < h->naggs; ++j) {
    const DAgg& a = P->aggs[j];
    if (a.acc != ACC_NONE) {
      P->off_acc[j] = (int32_t)off;
      off += 8 * SS;
    }
    if (a.track_nn) {
      P->off_nn[j] = (int32_t)off;
      off += 4 * SS;
      off = (off + 15) & ~size_t(15);
    }
    if (acc_is_f64mm(a.acc)) {
      P->off_idx[j] = (int32_t)off;
      off += 32 * SS;
    }
  }
  P->lds_log2 = log2;
  return off;
}

// Largest LDS table in [lds_log2_min, lds_log2] that fits the per-workgroup budget; 0 bytes =>
// global-only launch (the expected groups do not fit on chip).
static size_t lds_layout(const qe_hashagg* h, Plan* P) {
  if (h->lds_log2 == 0) return 0;
  for (int log2 = h->lds_log2; log2 >= h->lds_log2_min; --log2) {
    const size_t b = lds_layout_at(h, P, log2);
    if (b <= HA_LDS_BUDGET) return b;
  }
  P->lds_log2 = 0;
  return 0;
}

// LDS bytes with no nullable inputs (the smallest layout a launch can have).
static size_t lds_bytes_min(const qe_hashagg* h, int log2) {
  const size_t SS = ((size_t)1 << log2) + 2;
  size_t b = 12 * SS + 16;
  for (int j = 0; j < h->naggs; ++j) {
    if (h->acc[j] != ACC_NONE) b += 8 * SS;
    if (acc_is_f64mm(h->acc[j])) b += 32 * SS;
  }
  return b;
}

template <int NC>
static int launch_nc(const Plan& P, int grid, size_t lds, hipStream_t st) {
  if (lds) {
    // > 64 KiB of dynamic LDS must be opted into (gfx950 has 160 KiB per CU)
    QE_HIP(hipFuncSetAttribute((const void*)k_hashagg<NC, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    hipLaunchKernelGGL((k_hashagg<NC, true>), dim3(grid), dim3(HA_THREADS), lds, st, P);
  } else {
    hipLaunchKernelGGL((k_hashagg<NC, false>), dim3(grid), dim3(HA_THREADS), 0, st, P);
  }
  return QE_OK;
}

static int launch_hashagg(const Plan& P, int grid, size_t lds, hipStream_t st) {
  switch (P.ncols) {
    case 1: return launch_nc<1>(P, grid, lds, st);
    case 2: return launch_nc<2>(P, grid, lds, st);
    case 3: return launch_nc<3>(P, grid, lds, st);
    case 4: return launch_nc<4>(P, grid, lds, st);
    case 5:
    case 6: return launch_nc<6>(P, grid, lds, st);
    default: return launch_nc<8>(P, grid, lds, st);
  }
}

static int run_update(qe_hashagg* h, Plan& P) {
  qe_ctx* ctx = h->ctx;
  const int64_t n = P.n;
  if (n == 0) return QE_OK;
  const size_t lds = lds_layout(h, &P);
  P.ovf = h->ovf;
  P.ovf_cap = h->ovf_cap;
  QE_TRY(ensure_defer(h, n));
  h->last_kernel_ms = 0.0;
  h->last_launches = 0;
  int out_i = 0;
  const uint32_t* defer_in = nullptr;
  for (int pass = 0;; ++pass) {
    QE_CHECK(pass < 64, QE_ERR_CAPACITY, "hash aggregate did not converge after %d passes", pass);
    if (h->defer_dirty[out_i]) {
      QE_HIP(hipMemsetAsync(h->defer[out_i], 0, h->defer_words * 4, ctx->stream));
      h->defer_dirty[out_i] = false;
    }
    QE_HIP(hipMemsetAsync(h->ctl + 1, 0, 24, ctx->stream));
    P.t = h->t;
    P.defer_in = defer_in;
    P.defer_out = h->defer[out_i];
    const int64_t waves = (int64_t)div_up((uint64_t)n, 256);
    const int per_cu = lds ? std::max<int>(1, std::min<int>(8, (int)((160 * 1024) / lds))) : 8;
    const int64_t gcap = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, h->grid);
    int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)waves, HA_THREADS / 64), gcap);
    if (grid < 1) grid = 1;
    QE_HIP(hipEventRecord(h->ev[0], ctx->stream));
    QE_TRY(launch_hashagg(P, grid, lds, ctx->stream));
    QE_TRY(launch_check("k_hashagg"));
    QE_HIP(hipEventRecord(h->ev[1], ctx->stream));
    uint64_t c[4];
    QE_TRY(read_ctl(h, c));
    {
      float ms = 0.f;
      QE_HIP(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
      h->last_kernel_ms += ms;
      h->last_launches += 1;
    }
    QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash aggregate lost %llu groups (overflow area)", (unsigned long long)c[3]);
    const uint64_t groups = c[0], deferred = c[1], ovf_recs = c[2];
    if (deferred == 0 && ovf_recs == 0) {
      if (groups * 2 > h->t.cap) QE_TRY(table_grow(h, 4 * h->t.cap));
      break;
    }
    // grow, then re-apply what could not be inserted
    QE_TRY(table_grow(h, std::max<uint64_t>(4 * h->t.cap, 2 * (groups + ovf_recs))));
    if (ovf_recs) {
      QE_HIP(hipMemsetAsync(h->ctl + 3, 0, 8, ctx->stream));
      QE_TRY(import_records(h, h->ovf, (int64_t)ovf_recs));
    }
    if (deferred == 0) break;
    h->defer_dirty[out_i] = true;
    defer_in = h->defer[out_i];
    out_i ^= 1;
  }
  h->row_base += n;
  return QE_OK;
}

}  // namespace qe

extern "C" {

int qe_hashagg_create(qe_ctx* ctx, int32_t nkeys, const int32_t* key_types, int32_t naggs, const qe_agg_desc* aggs,
                      int64_t expected_groups, qe_hashagg** out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out, QE_ERR_INVALID_ARG, "null out");
  QE_CHECK(nkeys >= 0 && nkeys <= QE_MAX_KEYS, QE_ERR_UNSUPPORTED, "0..%d group keys supported", QE_MAX_KEYS);
  QE_CHECK(naggs >= 0 && naggs <= QE_MAX_AGGS, QE_ERR_UNSUPPORTED, "0..%d aggregates supported", QE_MAX_AGGS);
  QE_CHECK(nkeys == 0 || key_types, QE_ERR_INVALID_ARG, "null key_types");
  QE_CHECK(naggs == 0 || aggs, QE_ERR_INVALID_ARG, "null aggs");
  qe_hashagg* h = new qe_hashagg();
  h->ctx = ctx;
  h->nkeys = nkeys;
  h->naggs = naggs;
  auto bail = [&](int code) {
    delete h;
    return code;
  };
  // key packing
  if (nkeys == 0) {
    h->km.mode = 0;
  } else if (nkeys == 1 && (key_types[0] == QE_TYPE_INT64 || key_types[0] == QE_TYPE_FLOAT64)) {
    h->km.mode = 1;
  } else {
    h->km.mode = 2;
    int bit = 0;
    for (int k = 0; k < nkeys; ++k) {
      int w;
      switch (key_types[k]) {
        case QE_TYPE_INT32:
        case QE_TYPE_DATE32: w = 32; break;
        case QE_TYPE_UINT8: w = 8; break;
        default:
          return bail(fail(QE_ERR_UNSUPPORTED,
                           "group key %d: type %d cannot be packed (multi-key groups take uint8/int32/date32)", k,
                           key_types[k]));
      }
      h->km.shift[k] = bit;
      h->km.fmask[k] = (int64_t)((1ull << w) - 1);
      bit += w;
      h->km.nullbit[k] = bit;
      bit += 1;
    }
    if (bit > 63) return bail(fail(QE_ERR_UNSUPPORTED, "group keys need %d bits (max 63)", bit));
  }
  h->km.nkeys = nkeys;
  for (int k = 0; k < nkeys; ++k) {
    h->key_types[k] = key_types[k];
    h->km.type[k] = key_types[k];
  }
  // aggregates
  h->rec_bytes = 24;
  for (int j = 0; j < naggs; ++j) {
    const qe_agg_desc& d = aggs[j];
    h->aggs[j] = d;
    const bool f = d.input_type == QE_TYPE_FLOAT64;
    if (d.fn != QE_AGG_COUNT_STAR && d.fn != QE_AGG_COUNT && d.input_type != QE_TYPE_INT64 && !f)
      return bail(fail(QE_ERR_UNSUPPORTED, "aggregate %d: input type %d (int64/fp64 only)", j, d.input_type));
    switch (d.fn) {
      case QE_AGG_SUM: h->acc[j] = f ? ACC_SUM_F : ACC_SUM_I; break;
      case QE_AGG_MIN: h->acc[j] = f ? ACC_MIN_F : ACC_MIN_I; break;
      case QE_AGG_MAX: h->acc[j] = f ? ACC_MAX_F : ACC_MAX_I; break;
      case QE_AGG_AVG: h->acc[j] = ACC_SUM_F; break;
      case QE_AGG_COUNT:
      case QE_AGG_COUNT_STAR: h->acc[j] = ACC_NONE; break;
      default: return bail(fail(QE_ERR_UNSUPPORTED, "aggregate %d: unknown function %d", j, d.fn));
    }
    h->rec_bytes += agg_rec_bytes(h->acc[j]);
  }
  // control words
  if (hipEventCreate(&h->ev[0]) != hipSuccess || hipEventCreate(&h->ev[1]) != hipSuccess)
    return bail(fail(QE_ERR_DEVICE, "hipEventCreate failed"));
  if (hipMalloc(&h->ctl, 64) != hipSuccess) return bail(fail(QE_ERR_OOM, "control allocation failed"));
  if (hipMemsetAsync(h->ctl, 0, 64, ctx->stream) != hipSuccess) return bail(fail(QE_ERR_DEVICE, "memset failed"));
  // LDS table: 2x the expected groups (load factor <= 0.5); a launch may shrink it down to
  // 1.25x (lds_log2_min) to fit the per-workgroup budget, else the launch is global-only.
  const int64_t eg = expected_groups > 0 ? expected_groups : 1024;
  int log2 = 8, log2_min = 8;
  while (log2 < 16 && ((int64_t)1 << log2) < 2 * eg) ++log2;
  while (log2_min < 16 && ((int64_t)1 << log2_min) < (5 * eg + 3) / 4) ++log2_min;
  while (log2 > log2_min && lds_bytes_min(h, log2) > HA_LDS_BUDGET) --log2;
  h->lds_log2 = lds_bytes_min(h, log2) <= HA_LDS_BUDGET ? log2 : 0;
  h->lds_log2_min = log2_min;
  // workgroups per CU: as many as the smallest layout of the LDS table allows (max 8)
  const int per_cu = h->lds_log2 ? std::max<int>(1, std::min<int>(8, (int)((160 * 1024) / lds_bytes_min(h, h->lds_log2)))) : 8;
  h->grid = ctx->num_cus * per_cu;
  // overflow records: at most one per LDS slot per workgroup
  if (h->lds_log2) {
    h->ovf_cap = (uint64_t)h->grid * (((uint64_t)1 << h->lds_log2) + 2);
    if (hipMalloc(&h->ovf, h->ovf_cap * h->rec_bytes) != hipSuccess) {
      if (h->ctl) (void)hipFree(h->ctl);
      return bail(fail(QE_ERR_OOM, "overflow area allocation failed"));
    }
  }
  // global table: 2x expected groups
  const int st = table_alloc(h, std::max<uint64_t>(1024, next_pow2((uint64_t)(2 * eg))), &h->table_mem, &h->t);
  if (st != QE_OK) {
    if (h->ovf) (void)hipFree(h->ovf);
    (void)hipFree(h->ctl);
    return bail(st);
  }
  *out = h;
  return QE_OK;
}

int qe_hashagg_destroy(qe_hashagg* h) {
  if (!h) return QE_OK;
  (void)hipSetDevice(h->ctx->device);
  (void)hipStreamSynchronize(h->ctx->stream);
  if (h->table_mem) (void)hipFree(h->table_mem);
  if (h->ctl) (void)hipFree(h->ctl);
  if (h->ovf) (void)hipFree(h->ovf);
  for (int i = 0; i < 2; ++i) {
    if (h->defer[i]) (void)hipFree(h->defer[i]);
    if (h->ev[i]) (void)hipEventDestroy(h->ev[i]);
  }
  delete h;
  return QE_OK;
}

int qe_hashagg_last_kernel_time(qe_hashagg* h, double* ms, int32_t* launches) {
  QE_CHECK(h && ms, QE_ERR_INVALID_ARG, "null argument");
  *ms = h->last_kernel_ms;
  if (launches) *launches = h->last_launches;
  return QE_OK;
}

int qe_hashagg_reset(qe_hashagg* h) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  QE_TRY(ctx_enter(h->ctx));
  QE_HIP(hipMemsetAsync(h->ctl, 0, 64, h->ctx->stream));
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 4096);
  hipLaunchKernelGGL(k_table_init, dim3(grid), dim3(256), 0, h->ctx->stream, h->t, agg_meta(h));
  QE_TRY(launch_check("k_table_init"));
  h->row_base = 0;
  return QE_OK;
}

int qe_hashagg_set_row_base(qe_hashagg* h, int64_t row_base) {
  QE_CHECK(h && row_base >= 0, QE_ERR_INVALID_ARG, "bad arguments");
  h->row_base = row_base;
  return QE_OK;
}

int qe_hashagg_update_fused(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec) {
  QE_CHECK(h && cols && spec, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(h->ctx));
  Plan P;
  QE_TRY(compile_plan(h, cols, ncols, spec, &P));
  return run_update(h, P);
}

int qe_hashagg_update(qe_hashagg* h, const qe_column* keys, const qe_column* agg_inputs, const qe_column* mask) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  QE_TRY(ctx_enter(h->ctx));
  QE_CHECK(h->nkeys == 0 || keys, QE_ERR_INVALID_ARG, "null keys");
  QE_CHECK(h->naggs == 0 || agg_inputs, QE_ERR_INVALID_ARG, "null agg_inputs");
  // Column slots: distinct buffers only (shared columns are read once).
  qe_column cols[QE_MAX_COLS];
  int ncols = 0;
  int64_t n = -1;
  auto slot_of = [&](const qe_column& c, int* slot) -> int {
    if (n < 0) n = c.length;
    QE_CHECK(c.length == n, QE_ERR_INVALID_ARG, "input columns differ in length (%lld vs %lld)",
             (long long)c.length, (long long)n);
    for (int i = 0; i < ncols; ++i)
      if (cols[i].values == c.values && cols[i].validity == c.validity && cols[i].type == c.type) {
        *slot = i;
        return QE_OK;
      }
    QE_CHECK(ncols < QE_MAX_COLS, QE_ERR_UNSUPPORTED, "more than %d distinct input columns", QE_MAX_COLS);
    cols[ncols] = c;
    *slot = ncols++;
    return QE_OK;
  };
  qe_fused_spec spec;
  memset(&spec, 0, sizeof(spec));
  spec.mask_col = -1;
  for (int k = 0; k < h->nkeys; ++k) QE_TRY(slot_of(keys[k], &spec.key_cols[k]));
  for (int j = 0; j < h->naggs; ++j) {
    if (h->aggs[j].fn == QE_AGG_COUNT_STAR) continue;
    int s;
    QE_TRY(slot_of(agg_inputs[j], &s));
    spec.inputs[j].ntokens = 1;
    spec.inputs[j].tokens[0].op = QE_TOK_COL;
    spec.inputs[j].tokens[0].arg = s;
  }
  if (mask) QE_TRY(slot_of(*mask, &spec.mask_col));
  if (ncols == 0) {
    // COUNT(*) only, no keys: still need a row count; use the mask or fail.
    return fail(QE_ERR_INVALID_ARG, "update needs at least one input column");
  }
  Plan P;
  QE_TRY(compile_plan(h, cols, ncols, &spec, &P));
  return run_update(h, P);
}

int qe_hashagg_num_groups(qe_hashagg* h, int64_t* out) {
  QE_CHECK(h && out, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(h->ctx));
  uint64_t c[4];
  QE_TRY(read_ctl(h, c));
  *out = (int64_t)c[0];
  return QE_OK;
}

int qe_hashagg_finalize(qe_hashagg* h, qe_column* out_keys, qe_column* out_aggs, int64_t* out_groups) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  QE_TRY(ctx_enter(h->ctx));
  qe_ctx* ctx = h->ctx;
  int64_t groups;
  QE_TRY(qe_hashagg_num_groups(h, &groups));
  OutCols oc{};
  for (int k = 0; k < h->nkeys; ++k) {
    QE_CHECK(out_keys, QE_ERR_INVALID_ARG, "null out_keys");
    const qe_column& c = out_keys[k];
    QE_CHECK(c.type == h->key_types[k], QE_ERR_INVALID_ARG, "key output %d: type %d, expected %d", k, c.type,
             h->key_types[k]);
    QE_CHECK(c.length >= groups && (c.values || groups == 0), QE_ERR_CAPACITY, "key output %d holds %lld rows, need %lld",
             k, (long long)c.length, (long long)groups);
    QE_CHECK(!c.validity || ((uintptr_t)c.validity & 3) == 0, QE_ERR_INVALID_ARG, "validity must be 4-byte aligned");
    oc.keys[k] = c;
    if (c.validity) QE_HIP(hipMemsetAsync(c.validity, 0, div_up((uint64_t)groups, 32) * 4, ctx->stream));
  }
  for (int j = 0; j < h->naggs; ++j) {
    QE_CHECK(out_aggs, QE_ERR_INVALID_ARG, "null out_aggs");
    const qe_column& c = out_aggs[j];
    const int fn = h->aggs[j].fn;
    const int32_t want = (fn == QE_AGG_COUNT || fn == QE_AGG_COUNT_STAR) ? QE_TYPE_INT64
                         : (fn == QE_AGG_AVG || h->aggs[j].input_type == QE_TYPE_FLOAT64) ? QE_TYPE_FLOAT64
                                                                                          : QE_TYPE_INT64;
    QE_CHECK(c.type == want, QE_ERR_INVALID_ARG, "aggregate output %d: type %d, expected %d", j, c.type, want);
    QE_CHECK(c.length >= groups && (c.values || groups == 0), QE_ERR_CAPACITY,
             "aggregate output %d holds %lld rows, need %lld", j, (long long)c.length, (long long)groups);
    QE_CHECK(!c.validity || ((uintptr_t)c.validity & 3) == 0, QE_ERR_INVALID_ARG, "validity must be 4-byte aligned");
    oc.aggs[j] = c;
    if (c.validity) QE_HIP(hipMemsetAsync(c.validity, 0, div_up((uint64_t)groups, 32) * 4, ctx->stream));
  }
  if (out_groups) *out_groups = groups;
  for (int k = 0; k < h->nkeys; ++k) out_keys[k].length = groups;
  for (int j = 0; j < h->naggs; ++j) out_aggs[j].length = groups;
  if (groups == 0) return QE_OK;
  const int32_t tile_slots = 4096;
  const uint64_t SS = h->t.cap + 2;
  const int64_t ntiles = (int64_t)div_up(SS, tile_slots);
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)(2 * ntiles + 1) * 8, &s));
  int64_t* counts = (int64_t*)s;
  int64_t* offs = counts + ntiles;
  hipLaunchKernelGGL(k_occ_count, dim3((unsigned)ntiles), dim3(256), 0, ctx->stream, h->t, counts, tile_slots);
  QE_TRY(launch_check("k_occ_count"));
  QE_TRY(exclusive_scan_i64(ctx, counts, offs, ntiles));
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)ntiles), dim3(256), 0, ctx->stream, h->t, agg_meta(h), h->km, offs,
                     tile_slots, oc);
  QE_TRY(launch_check("k_finalize"));
  QE_HIP(hipStreamSynchronize(ctx->stream));
  return QE_OK;
}

int qe_hashagg_record_bytes(qe_hashagg* h, int64_t* out) {
  QE_CHECK(h && out, QE_ERR_INVALID_ARG, "null argument");
  *out = h->rec_bytes;
  return QE_OK;
}

int qe_hashagg_export_counts(qe_hashagg* h, int32_t nparts, int64_t* counts) {
  QE_CHECK(h && counts && nparts >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(ctx_enter(h->ctx));
  qe_ctx* ctx = h->ctx;
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)nparts * 8, &s));
  QE_HIP(hipMemsetAsync(s, 0, (size_t)nparts * 8, ctx->stream));
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 8192);
  hipLaunchKernelGGL(k_export_count, dim3(grid), dim3(256), 0, ctx->stream, h->t, nparts, (unsigned long long*)s);
  QE_TRY(launch_check("k_export_count"));
  QE_HIP(hipMemcpyAsync(counts, s, (size_t)nparts * 8, hipMemcpyDeviceToHost, ctx->stream));
  QE_HIP(hipStreamSynchronize(ctx->stream));
  return QE_OK;
}

int qe_hashagg_export(qe_hashagg* h, int32_t nparts, void* dst) {
  QE_CHECK(h && nparts >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(ctx_enter(h->ctx));
  qe_ctx* ctx = h->ctx;
  // counts -> exclusive offsets used as cursors
  int64_t* hc = new int64_t[nparts];
  int st = qe_hashagg_export_counts(h, nparts, hc);
  if (st != QE_OK) {
    delete[] hc;
    return st;
  }
  int64_t total = 0;
  for (int p = 0; p < nparts; ++p) {
    const int64_t c = hc[p];
    hc[p] = total;
    total += c;
  }
  if (total == 0) {
    delete[] hc;
    return QE_OK;
  }
  if (!dst) {
    delete[] hc;
    return fail(QE_ERR_INVALID_ARG, "null destination");
  }
  void* s;
  st = ctx_scratch(ctx, (size_t)nparts * 8, &s);
  if (st == QE_OK) {
    hipError_t e = hipMemcpyAsync(s, hc, (size_t)nparts * 8, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) st = fail(QE_ERR_DEVICE, "cursor upload: %s", hipGetErrorString(e));
  }
  delete[] hc;
  if (st != QE_OK) return st;
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 8192);
  hipLaunchKernelGGL(k_export, dim3(grid), dim3(256), 0, ctx->stream, h->t, agg_meta(h), nparts, h->rec_bytes,
                     (unsigned long long*)s, (uint8_t*)dst);
  QE_TRY(launch_check("k_export"));
  QE_HIP(hipStreamSynchronize(ctx->stream));
  return QE_OK;
}

int qe_hashagg_import(qe_hashagg* h, const void* records, int64_t nrecords) {
  QE_CHECK(h && nrecords >= 0 && (records || nrecords == 0), QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(ctx_enter(h->ctx));
  if (nrecords == 0) return QE_OK;
  uint64_t c[4];
  QE_TRY(read_ctl(h, c));
  if (2 * (c[0] + (uint64_t)nrecords) > h->t.cap) QE_TRY(table_grow(h, 2 * (c[0] + (uint64_t)nrecords)));
  QE_HIP(hipMemsetAsync(h->ctl + 3, 0, 8, h->ctx->stream));
  return import_records(h, records, nrecords);
}

}  // extern "C"
