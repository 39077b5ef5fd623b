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
// plus two special slots (G: null key, G+1: key == EMPTY_KEY, the EMPTY sentinel):
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
#include <map>
#include <memory>
#include <mutex>

#include "qe_internal.hpp"

namespace qe {

constexpr int HA_THREADS = 512;
constexpr size_t HA_LDS_BUDGET = 80 * 1024;  // bytes of LDS per workgroup (2 workgroups / CU)

// ---- LDS table -----------------------------------------------------------------------------------
__device__ __forceinline__ qi64* lds_keys(char* smem) { return (qi64*)smem; }

__device__ __forceinline__ void lds_init(const Plan& P, char* smem) {
  const int SS = (1 << P.lds_log2) + 2;
  qi64* keys = lds_keys(smem);
  qu32* cst = (qu32*)(smem + P.off_cstar);
  for (int s = threadIdx.x; s < SS; s += blockDim.x) {
    keys[s] = EMPTY_KEY;
    cst[s] = 0;
  }
#pragma unroll
  for (int j = 0; j < QE_MAX_AGGS; ++j) {
    if (j >= P.naggs) break;
    const DAgg& a = P.aggs[j];
    if (a.acc != ACC_NONE) {
      qi64* acc = (qi64*)(smem + P.off_acc[j]);
      const qi64 id = acc_identity(a.acc);
      for (int s = threadIdx.x; s < SS; s += blockDim.x) acc[s] = id;
    }
    if (a.track_nn) {
      qu32* nn = (qu32*)(smem + P.off_nn[j]);
      for (int s = threadIdx.x; s < SS; s += blockDim.x) nn[s] = 0;
    }
    if (acc_has_idx(a.acc)) {
      qu64* ix = (qu64*)(smem + P.off_idx[j]);
      const qu64 id = idx_identity(a.acc);
      for (int s = threadIdx.x; s < 4 * SS; s += blockDim.x) ix[s] = id;
    }
  }
}

// Slot of `key` in the LDS table, inserting it if absent; -1 when the probe limit is hit.
__device__ __forceinline__ int lds_find(const Plan& P, char* smem, qi64 key, bool knull) {
  const int S = 1 << P.lds_log2;
  if (knull) return S;
  if (key == EMPTY_KEY) return S + 1;
  return lds_probe(lds_keys(smem), P.lds_log2, key, lds_hash((qu64)key) >> (32 - P.lds_log2));
}

// The accumulator part of one row (the non-null count is the caller's: lds_accum / lds_accum4).
__device__ __forceinline__ void lds_accum_value(const Plan& P, char* smem, int j, int s, qi64 x, qu64 row) {
  const DAgg& a = P.aggs[j];
  qi64* acc = (qi64*)(smem + P.off_acc[j]);
  switch (a.acc) {
    case ACC_SUM_I: atomicAdd((unsigned long long*)&acc[s], (unsigned long long)x); break;
    case ACC_SUM_F: atomicAdd((double*)&acc[s], bits_f64(x)); break;
    case ACC_SUM_X:
      if (!lds_fx_add(acc, (qu64*)(smem + P.off_idx[j]), (1 << P.lds_log2) + 2, s, x)) {
        const int S = 1 << P.lds_log2;  // an input for E: into the global slot (fx_rare_global)
        fx_rare_global(P, 1u << j, s < S ? lds_keys(smem)[s] : (s == S ? 0 : EMPTY_KEY), s == S, x);
      }
      break;
    case ACC_MIN_I: atomicMin((long long*)&acc[s], (long long)x); break;
    case ACC_MAX_I: atomicMax((long long*)&acc[s], (long long)x); break;
    case ACC_MIN_F:
    case ACC_MAX_F: {
      const RowVal r = row_partial(a.acc, x, row);
      const int SS = (1 << P.lds_log2) + 2;
      unsigned long long* ix = (unsigned long long*)(smem + P.off_idx[j]);
      atomicMin(&ix[s], (unsigned long long)r.i0);
      if (r.i1 != ~0ull) {
        atomicMin(&ix[SS + s], (unsigned long long)r.i1);
      } else {
        if (a.acc == ACC_MIN_F) atomicMin((long long*)&acc[s], (long long)r.acc);
        else atomicMax((long long*)&acc[s], (long long)r.acc);
        if (r.i2 != ~0ull) atomicMin(&ix[2 * SS + s], (unsigned long long)r.i2);
        if (r.i3 != ~0ull) atomicMin(&ix[3 * SS + s], (unsigned long long)r.i3);
      }
      break;
    }
    default: break;
  }
}

__device__ __forceinline__ void lds_accum(const Plan& P, char* smem, int j, int s, qi64 x, bool valid,
                                          qu64 row) {
  if (!valid) return;
  if (P.aggs[j].track_nn) atomicAdd((qu32*)(smem + P.off_nn[j]) + s, 1u);
  lds_accum_value(P, smem, j, s, x, row);
}

// Merge the workgroup's LDS table into the global table (or the overflow records).
__device__ __forceinline__ void lds_flush(const Plan& P, char* smem) {
  const int S = 1 << P.lds_log2;
  const int SS = S + 2;
  const qi64* keys = lds_keys(smem);
  const qu32* cst = (const qu32*)(smem + P.off_cstar);
  for (int s = threadIdx.x; s < SS; s += blockDim.x) {
    const qu32 c = cst[s];
    if (c == 0) continue;  // an occupied slot always has at least one row
    const bool knull = s == S;
    const qi64 key = s == S ? 0 : (s == S + 1 ? EMPTY_KEY : keys[s]);
    qu64 gs;
    const bool ok = gtable_find(P.t, key, knull, gs);
    qu8* rec = nullptr;
    if (ok) {
      gadd_cstar(P.t, gs, c);
    } else {
      const qu64 r = atomicAdd((unsigned long long*)&P.t.ctl[2], 1ull);
      if (r >= P.ovf_cap) {
        atomicAdd((unsigned long long*)&P.t.ctl[3], 1ull);
        continue;
      }
      rec = P.ovf + r * (qu64)P.rec_bytes;
      write_record_head(rec, key, knull, c);
    }
    int off = 24;
#pragma unroll
    for (int j = 0; j < QE_MAX_AGGS; ++j) {
      if (j >= P.naggs) break;
      const DAgg& a = P.aggs[j];
      qi64 acc = a.acc != ACC_NONE ? ((const qi64*)(smem + P.off_acc[j]))[s] : 0;
      const qu64 nn = a.track_nn ? ((const qu32*)(smem + P.off_nn[j]))[s] : c;
      qu64 i0 = ~0ull, i1 = ~0ull, i2 = ~0ull, i3 = ~0ull;
      if (acc_has_idx(a.acc)) {
        const qu64* ix = (const qu64*)(smem + P.off_idx[j]);
        i0 = ix[s];
        i1 = ix[SS + s];
        i2 = ix[2 * SS + s];
        i3 = ix[3 * SS + s];
      }
      if (ok) {
        if (a.fn != QE_AGG_COUNT_STAR) gcombine(P.t, a.acc, j, gs, acc, nn, i0, i1, i2, i3);
      } else {
        qu64* f = (qu64*)(rec + off);
        f[0] = (qu64)acc;
        f[1] = nn;
        if (acc_has_idx(a.acc)) {
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
  qu32 valid;  // nibble per slot
  __device__ __forceinline__ qi64 get(int slot, int r) const { return v[4 * slot + r]; }
  __device__ __forceinline__ bool ok(int slot, int r) const { return (valid >> (4 * slot + r)) & 1u; }
};

typedef long long i64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ qi64 row_of(qi64 base, int lane, int r) {
  return base + 128 * (r >> 1) + 2 * lane + (r & 1);
}

template <int NC>
__device__ __forceinline__ void load_cols(const Plan& P, qi64 base, int lane, bool full, ColRegs<NC>& R) {
  if (full && P.all8) {
    // common case: every slot an 8-byte column, whole step in range -> 2*NC straight-line
    // 16-B loads (each wave instruction = one contiguous KiB), validity nibbles after
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c < P.ncols) {
        const qi64* p = (const qi64*)P.cols[c].p + base + 2 * lane;
        const i64x2 t0 = *(const i64x2*)p;
        const i64x2 t1 = *(const i64x2*)(p + 128);
        R.v[4 * c + 0] = t0.x;
        R.v[4 * c + 1] = t0.y;
        R.v[4 * c + 2] = t1.x;
        R.v[4 * c + 3] = t1.y;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) R.v[4 * c + r] = 0;
      }
    }
    qu32 valid = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      qu32 vv = 15u;
      if (c < P.ncols && P.cols[c].valid) {
        const qi64 r0 = base + 2 * lane;
        // bytes past ceil(n/8) are never read: an input bitmap may be Arrow-minimal
        const qu32 lo = r0 < P.n ? (qu32)(P.cols[c].valid[r0 >> 3] >> (r0 & 7)) & 3u : 0u;
        const qu32 hi = r0 + 128 < P.n ? (qu32)(P.cols[c].valid[(r0 + 128) >> 3] >> (r0 & 7)) & 3u : 0u;
        vv = lo | (hi << 2);
      }
      valid |= vv << (4 * c);
    }
    R.valid = valid;
    return;
  }
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
      const qi64 r0 = base + 128 * q + 2 * lane;
      qi64 a = 0, b = 0;
      if (full) {
        switch (col.kind) {
          case K_I64:
          case K_F64: {
            const i64x2 t = *(const i64x2*)((const qi64*)col.p + r0);
            a = t.x;
            b = t.y;
            break;
          }
          case K_I32: {
            const int2 t = *(const int2*)((const qi32*)col.p + r0);
            a = t.x;
            b = t.y;
            break;
          }
          case K_U8: {
            const uint16_t t = *(const uint16_t*)((const qu8*)col.p + r0);
            a = t & 0xFF;
            b = t >> 8;
            break;
          }
          default: {  // K_BOOL
            const qu32 t = ((const qu8*)col.p)[r0 >> 3] >> (r0 & 7);
            a = t & 1;
            b = (t >> 1) & 1;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const qi64 r = r0 + e;
          qi64 x = 0;
          if (r < P.n) {
            switch (col.kind) {
              case K_I64:
              case K_F64: x = ((const qi64*)col.p)[r]; break;
              case K_I32: x = ((const qi32*)col.p)[r]; break;
              case K_U8: x = ((const qu8*)col.p)[r]; break;
              default: x = (((const qu8*)col.p)[r >> 3] >> (r & 7)) & 1;
            }
          }
          if (e) b = x;
          else a = x;
        }
      }
      R.v[4 * c + 2 * q] = a;
      R.v[4 * c + 2 * q + 1] = b;
      const qu32 vv = !col.valid ? 3u : r0 < P.n ? ((qu32)(col.valid[r0 >> 3] >> (r0 & 7)) & 3u) : 0u;
      R.valid |= vv << (4 * c + 2 * q);
    }
  }
}

__device__ __forceinline__ bool cmp_i(qi32 op, qi64 a, qi64 b) {
  switch (op) {
    case QE_OP_EQ: return a == b;
    case QE_OP_NE: return a != b;
    case QE_OP_LT: return a < b;
    case QE_OP_LE: return a <= b;
    case QE_OP_GT: return a > b;
    default: return a >= b;
  }
}
__device__ __forceinline__ bool cmp_f(qi32 op, double a, double b) {
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
__device__ __forceinline__ qi64 eval_program(const DAgg& a, const ColRegs<NC>& R, int r, bool& valid) {
  qi64 s0 = 0, s1 = 0, s2 = 0, s3 = 0;
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
      qi64 res;
      bool ok = n0 && n1;
      const qu64 ua = (qu64)s1, ub = (qu64)s0;
      switch (op) {
        case T_ADD_I: res = (qi64)(ua + ub); break;
        case T_SUB_I: res = (qi64)(ua - ub); break;
        case T_MUL_I: res = (qi64)(ua * ub); break;
        case T_DIV_I:
          if (s0 == 0) { res = 0; ok = false; }
          else if (s0 == -1) res = (qi64)(0ull - ua);
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

__device__ __forceinline__ qi64 binop(qi32 op, qi64 l, qi64 r, bool& ok) {
  const qu64 ua = (qu64)l, ub = (qu64)r;
  switch (op) {
    case T_ADD_I: return (qi64)(ua + ub);
    case T_SUB_I: return (qi64)(ua - ub);
    case T_MUL_I: return (qi64)(ua * ub);
    case T_DIV_I:
      if (r == 0) {
        ok = false;
        return 0;
      }
      return r == -1 ? (qi64)(0ull - ua) : l / r;
    case T_ADD_F: return f64_bits(bits_f64(l) + bits_f64(r));
    case T_SUB_F: return f64_bits(bits_f64(l) - bits_f64(r));
    case T_MUL_F: return f64_bits(bits_f64(l) * bits_f64(r));
    default: return f64_bits(bits_f64(l) / bits_f64(r));
  }
}

// Aggregate input for row r without the interpreter (pkind 1 and 3).
template <int NC>
__device__ __forceinline__ qi64 eval_fast(const DAgg& a, const ColRegs<NC>& R, int r, bool& valid) {
  const qi64 x = R.get(a.col, r);
  valid = R.ok(a.col, r);
  if (a.pkind == 1) return a.cvt_i2f ? f64_bits((double)x) : x;
  const qi64 y = a.rhs >= 0 ? R.get(a.rhs, r) : a.rhs_lit;
  valid = valid && (a.rhs >= 0 ? R.ok(a.rhs, r) : !a.rhs_null);
  return binop(a.bop, x, y, valid);
}

typedef long long i64x4 __attribute__((ext_vector_type(4)));

// Row-parallel accumulate of one aggregate input into its group slot (LDS or global).
__device__ __forceinline__ void accum_row(const Plan& P, char* smem, int j, const DAgg& a, int s, qu64 gs,
                                          qi64 x, bool valid, qu64 row) {
  if (s >= 0) {
    lds_accum(P, smem, j, s, x, valid, row);
  } else if (valid) {
    const RowVal rv = row_partial(a.acc, x, row);
    gcombine(P.t, a.acc, j, gs, rv.acc, 1, rv.i0, rv.i1, rv.i2, rv.i3);
  }
}

// ---- unswitched helpers: every uniform decision is taken once per step, rows loop inside ----
// The 4 rows of slot `c` (compile-time register indices inside each case).
template <int NC>
__device__ __forceinline__ void get4(const ColRegs<NC>& R, int c, qi64 (&x)[4], qu32& ok) {
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    if (c == k) {
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = R.v[4 * k + r];
      ok = (R.valid >> (4 * k)) & 15u;
    }
  }
}

template <typename F>
__device__ __forceinline__ qu32 cmp4(const qi64 (&a)[4], const qi64 (&b)[4], F f) {
  qu32 m = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) m |= (qu32)f(a[r], b[r]) << r;
  return m;
}

// Rows of `a` (op) `b` that are true, as a 4-bit mask (op and domain are wave-uniform).
__device__ __forceinline__ qu32 compare4(qi32 op, bool f64, const qi64 (&a)[4], const qi64 (&b)[4]) {
  if (!f64) {
    switch (op) {
      case QE_OP_EQ: return cmp4(a, b, [](qi64 x, qi64 y) { return x == y; });
      case QE_OP_NE: return cmp4(a, b, [](qi64 x, qi64 y) { return x != y; });
      case QE_OP_LT: return cmp4(a, b, [](qi64 x, qi64 y) { return x < y; });
      case QE_OP_LE: return cmp4(a, b, [](qi64 x, qi64 y) { return x <= y; });
      case QE_OP_GT: return cmp4(a, b, [](qi64 x, qi64 y) { return x > y; });
      default: return cmp4(a, b, [](qi64 x, qi64 y) { return x >= y; });
    }
  }
  switch (op) {
    case QE_OP_EQ: return cmp4(a, b, [](qi64 x, qi64 y) { return bits_f64(x) == bits_f64(y); });
    case QE_OP_NE: return cmp4(a, b, [](qi64 x, qi64 y) { return bits_f64(x) != bits_f64(y); });
    case QE_OP_LT: return cmp4(a, b, [](qi64 x, qi64 y) { return bits_f64(x) < bits_f64(y); });
    case QE_OP_LE: return cmp4(a, b, [](qi64 x, qi64 y) { return bits_f64(x) <= bits_f64(y); });
    case QE_OP_GT: return cmp4(a, b, [](qi64 x, qi64 y) { return bits_f64(x) > bits_f64(y); });
    default: return cmp4(a, b, [](qi64 x, qi64 y) { return bits_f64(x) >= bits_f64(y); });
  }
}

template <typename F>
__device__ __forceinline__ void map4(qi64 (&x)[4], const qi64 (&y)[4], F f) {
#pragma unroll
  for (int r = 0; r < 4; ++r) x[r] = f(x[r], y[r]);
}

// x = x (op) y for the 4 rows; int64 division by zero clears the row's bit in `ok`.
__device__ __forceinline__ void binop4(qi32 op, qi64 (&x)[4], const qi64 (&y)[4], qu32& ok) {
  switch (op) {
    case T_ADD_I: map4(x, y, [](qi64 a, qi64 b) { return (qi64)((qu64)a + (qu64)b); }); break;
    case T_SUB_I: map4(x, y, [](qi64 a, qi64 b) { return (qi64)((qu64)a - (qu64)b); }); break;
    case T_MUL_I: map4(x, y, [](qi64 a, qi64 b) { return (qi64)((qu64)a * (qu64)b); }); break;
    case T_ADD_F: map4(x, y, [](qi64 a, qi64 b) { return f64_bits(bits_f64(a) + bits_f64(b)); }); break;
    case T_SUB_F: map4(x, y, [](qi64 a, qi64 b) { return f64_bits(bits_f64(a) - bits_f64(b)); }); break;
    case T_MUL_F: map4(x, y, [](qi64 a, qi64 b) { return f64_bits(bits_f64(a) * bits_f64(b)); }); break;
    case T_DIV_F: map4(x, y, [](qi64 a, qi64 b) { return f64_bits(bits_f64(a) / bits_f64(b)); }); break;
    default:  // T_DIV_I
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bool v = true;
        x[r] = binop(T_DIV_I, x[r], y[r], v);
        if (!v) ok &= ~(1u << r);
      }
  }
}

// LDS accumulate of one aggregate for the active rows (acc kind switched once).
__device__ __forceinline__ void lds_accum4(const Plan& P, char* smem, int j, const DAgg& a, const int (&slot)[4],
                                           const qi64 (&x)[4], qu32 m, qi64 row0, int lane) {
  if (a.track_nn) {
    qu32* nn = (qu32*)(smem + P.off_nn[j]);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if ((m >> r) & 1) atomicAdd(nn + slot[r], 1u);
  }
  qi64* acc = (qi64*)(smem + P.off_acc[j]);
  switch (a.acc) {
    case ACC_SUM_I:
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((m >> r) & 1) atomicAdd((unsigned long long*)&acc[slot[r]], (unsigned long long)x[r]);
      break;
    case ACC_SUM_F:
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((m >> r) & 1) atomicAdd((double*)&acc[slot[r]], bits_f64(x[r]));
      break;
    case ACC_MIN_I:
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((m >> r) & 1) atomicMin((long long*)&acc[slot[r]], (long long)x[r]);
      break;
    case ACC_MAX_I:
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((m >> r) & 1) atomicMax((long long*)&acc[slot[r]], (long long)x[r]);
      break;
    case ACC_MIN_F:
    case ACC_MAX_F:
    case ACC_SUM_X:
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((m >> r) & 1) lds_accum_value(P, smem, j, slot[r], x[r], (qu64)(row0 + row_of(0, lane, r)));
      break;
    default: break;
  }
}

template <int NC, bool USE_LDS>
__device__ __forceinline__ void process_step(const Plan& P, char* smem, const ColRegs<NC>& R, qi64 base,
                                             int lane) {
  qu32 act = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) act |= (qu32)(row_of(base, lane, r) < P.n) << r;
  if (P.defer_in) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const qi64 row = row_of(base, lane, r);
      if (row < P.n && !((P.defer_in[row >> 5] >> (row & 31)) & 1)) act &= ~(1u << r);
    }
  }
  if (P.mask_col >= 0) {
    qi64 mv[4];
    qu32 ok = 0;
    get4(R, P.mask_col, mv, ok);
    qu32 bits = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) bits |= (qu32)(mv[r] & 1) << r;
    act &= bits & ok;
  }
  for (int t = 0; t < P.nterms; ++t) {
    const DTerm& T = P.terms[t];
    qi64 a[4], b[4];
    qu32 aok = 0, bok = 15u;
    get4(R, T.lhs, a, aok);
    if (T.rhs >= 0) {
      get4(R, T.rhs, b, bok);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) b[r] = T.lit;
      bok = T.lit_null ? 0u : 15u;
    }
    if (T.f64) {  // integral sides promote to fp64
      if (!T.lhs_f) {
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = f64_bits((double)a[r]);
      }
      if (!T.rhs_f) {
#pragma unroll
        for (int r = 0; r < 4; ++r) b[r] = f64_bits((double)b[r]);
      }
    }
    act &= compare4(T.op, T.f64, a, b) & aok & bok;
  }
  if (act == 0) return;
  // ---- group keys of the lane's 4 rows
  qi64 key[4] = {0, 0, 0, 0};
  qu32 knull = 0;
  if (P.key_mode == 1) {
    qu32 ok = 0;
    get4(R, P.key_col[0], key, ok);
    knull = ~ok & 15u;
    if (P.key_f64) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (bits_f64(key[r]) != bits_f64(key[r])) key[r] = 0x7FF8000000000000ll;  // Double.equals: one NaN
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if ((knull >> r) & 1) key[r] = 0;
  } else if (P.key_mode == 2) {
    for (int q = 0; q < P.nkeys; ++q) {
      qi64 x[4];
      qu32 ok = 0;
      get4(R, P.key_col[q], x, ok);
      const qi64 fm = P.key_fmask[q];
      const int sh = P.key_shift[q], nb = P.key_nullbit[q];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool isn = !((ok >> r) & 1);
        key[r] |= ((isn ? 0 : (x[r] & fm)) << sh) | ((qi64)isn << nb);
      }
    }
  }
  // multi-pass (groups beyond one LDS table, run_update): this pass keeps the rows whose key hash
  // falls in bucket mp_pass of mp_n (mp_pass < 0: the share at or above mp_keep), as qe_fused does
  if (P.mp_n > 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool other = P.mp_pass < 0 ? spill_hash((qu64)key[r]) < P.mp_keep
                                        : (qu32)__umul64hi(fmix64((qu64)key[r]), (qu64)P.mp_n) != (qu32)P.mp_pass;
      if (other) act &= ~(1u << r);
    }
    if (act == 0) return;
  }
  // ---- slots: first LDS probe of all 4 rows issued together; collisions (rare) probe on
  int slot[4] = {-1, -1, -1, -1};
  if (USE_LDS) {
    const int S = 1 << P.lds_log2;
    const qi64* keys = lds_keys(smem);
    qu32 h[4];
    qi64 k0[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      h[r] = lds_hash((qu64)key[r]) >> (32 - P.lds_log2);
      k0[r] = ((act >> r) & 1) ? keys[h[r]] : 0;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if ((knull >> r) & 1) slot[r] = S;
      else if (key[r] == EMPTY_KEY) slot[r] = S + 1;
      else if (k0[r] == key[r]) slot[r] = (int)h[r];
    }
    qu32 miss = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) miss |= (qu32)(slot[r] < 0) << r;
    miss &= act;
    if (__any(miss != 0)) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((miss >> r) & 1) slot[r] = lds_find(P, smem, key[r], false);
    }
  }
  qu32 glob = 0;  // rows whose group lives only in the global table (rare slow path)
#pragma unroll
  for (int r = 0; r < 4; ++r) glob |= (qu32)(slot[r] < 0) << r;
  glob &= act;
  const qu32 loc = act & ~glob;
  qu32* cst = (qu32*)(smem + P.off_cstar);
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if ((loc >> r) & 1) atomicAdd(cst + slot[r], 1u);
  // ---- aggregate inputs, LDS rows
  if (__any(loc != 0)) {
    for (int j = 0; j < P.naggs; ++j) {
      const DAgg& a = P.aggs[j];
      if (a.pkind == 0) continue;
      qi64 x[4];
      qu32 xok = 0;
      if (a.pkind == 2) {
        i64x4 xv;
        for (int r = 0; r < 4; ++r) {
          bool ok = false;
          xv[r] = ((loc >> r) & 1) ? eval_program<NC>(a, R, r, ok) : 0;
          xok |= (qu32)ok << r;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = xv[r];
      } else {
        get4(R, a.col, x, xok);
        if (a.pkind == 1) {
          if (a.cvt_i2f) {
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = f64_bits((double)x[r]);
          }
        } else {
          qi64 y[4];
          qu32 yok = 15u;
          if (a.rhs >= 0) {
            get4(R, a.rhs, y, yok);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) y[r] = a.rhs_lit;
            yok = a.rhs_null ? 0u : 15u;
          }
          xok &= yok;
          binop4(a.bop, x, y, xok);
        }
      }
      lds_accum4(P, smem, j, a, slot, x, loc & xok, P.row_base + base, lane);
    }
  }
  // ---- rows whose group is only in the global table (LDS table full / global-only mode)
  if (__any(glob != 0)) {
    for (int r = 0; r < 4; ++r) {
      if (!((glob >> r) & 1)) continue;
      qu64 gs;
      const qi64 lr = row_of(base, lane, r);
      if (!gtable_find(P.t, key[r], (knull >> r) & 1, gs)) {  // global table full: defer the row
        atomicOr(&P.defer_out[lr >> 5], 1u << (lr & 31));
        atomicAdd((unsigned long long*)&P.t.ctl[1], 1ull);
        continue;
      }
      gadd_cstar(P.t, gs, 1);
      const qu64 row = (qu64)(P.row_base + lr);
      for (int j = 0; j < P.naggs; ++j) {
        const DAgg& a = P.aggs[j];
        if (a.pkind == 0) continue;
        bool valid;
        const qi64 x = a.pkind == 2 ? eval_program<NC>(a, R, r, valid) : eval_fast<NC>(a, R, r, valid);
        if (!valid) continue;
        const RowVal rv = row_partial(a.acc, x, row);
        gcombine(P.t, a.acc, j, gs, rv.acc, 1, rv.i0, rv.i1, rv.i2, rv.i3);
      }
    }
  }
}

template <int NC, bool USE_LDS>
__global__ void __launch_bounds__(HA_THREADS, 4) k_hashagg(const Plan P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (USE_LDS) {
    lds_init(P, smem);
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const qi64 wave = (blockIdx.x * (qi64)blockDim.x + threadIdx.x) >> 6;
  const qi64 stride = (((qi64)gridDim.x * blockDim.x) >> 6) * 256;
  // Register double buffer: the next step's columns are in flight while this step is processed.
  ColRegs<NC> cur, nxt;
  qi64 base = wave * 256;
  if (base < P.n) load_cols<NC>(P, base, lane, base + 256 <= P.n, cur);
  for (; base < P.n; base += stride) {
    const qi64 nb = base + stride;
    if (nb < P.n) load_cols<NC>(P, nb, lane, nb + 256 <= P.n, nxt);
    process_step<NC, USE_LDS>(P, smem, cur, base, lane);
    cur = nxt;
  }
  if (USE_LDS) {
    __syncthreads();
    lds_flush(P, smem);
  }
}

// ---- table maintenance kernels -------------------------------------------------------------------
struct AggMeta {
  qi32 naggs;
  qi32 fn[QE_MAX_AGGS];
  qi32 acc[QE_MAX_AGGS];
  qi32 nn_implicit;  // bit j: aggregate j's non-null count is COUNT(*) (cstar); its nn array is unused
  qi32 any_x;        // some aggregate is an exact fp64 SUM (ACC_SUM_X)
};

__device__ __forceinline__ qu64 slot_nn(const DTable& t, const AggMeta& m, int j, qu64 s) {
  return ((m.nn_implicit >> j) & 1) ? t.cstar[s] : t.nn[j][s];
}

// Slice descriptors of the partition-aggregate pass (one workgroup). Bucket b's records are
// [off[b * g], off[(b + 1) * g]) (bucket-major exclusive scan of the (bucket, workgroup) counts,
// off[np * g] = total); a bucket of n records gets ceil(n / cw) slices, and a bucket that is one
// slice is flagged PART_EXCL: its workgroup is the only one to touch its groups. out[0] = slices.
__global__ void __launch_bounds__(1024) k_part_slices(const qi64* __restrict__ off, qi32 np, qi64 g, qi64 cw,
                                                      qi64* __restrict__ out) {
  __shared__ qi64 s_sum[1024];
  const int per = (np + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  qi64 cnt = 0;
  for (int i = 0; i < per; ++i) {
    const int b = b0 + i;
    if (b < np) cnt += (off[(qi64)(b + 1) * g] - off[(qi64)b * g] + cw - 1) / cw;
  }
  s_sum[threadIdx.x] = cnt;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const qi64 v = (int)threadIdx.x >= d ? s_sum[threadIdx.x - d] : 0;
    __syncthreads();
    s_sum[threadIdx.x] += v;
    __syncthreads();
  }
  qi64 pos = s_sum[threadIdx.x] - cnt;
  for (int i = 0; i < per; ++i) {
    const int b = b0 + i;
    if (b >= np) break;
    const qi64 s = off[(qi64)b * g], e = off[(qi64)(b + 1) * g];
    const qi64 ns = (e - s + cw - 1) / cw;
    for (qi64 k = 0; k < ns; ++k, ++pos) {
      const qi64 lo = s + k * cw;
      out[2 + 2 * pos] = lo;
      out[3 + 2 * pos] = (lo + cw < e ? lo + cw : e) | (ns == 1 ? PART_EXCL : 0);
    }
  }
  if (threadIdx.x == 1023) out[0] = s_sum[1023];
}

// Chunked scatter -> aggregation slices, in three launches over the chunk table meta (meta[0] =
// chunks C, meta[1 + c] = bucket << 32 | records). One workgroup doing all of it took 250-355 us
// per update at 1B rows (~250K chunks, LDS atomics on a few counters).
//   k_chunk_hist   per-workgroup LDS histograms of chunks and records per bucket, added to cnt / rec
//   k_chunk_slices one workgroup: bucket bases (exclusive scan of cnt) and slices: each bucket's
//                  chunk list is cut into slices of at most cpc chunks, cpc = 5/4 of an even share
//                  of target = max(buckets, min(tmax, records / 32K)) slices; a bucket that is one
//                  slice is flagged exclusive; out[0] = slices (at most tmax + buckets)
//   k_chunk_place  chunk ids grouped by bucket into `sorted` (per-workgroup LDS ranks, one global
//                  atomic per (workgroup, bucket) on cur; order inside a bucket is arbitrary)
// cnt, rec and cur are zeroed by the caller.
constexpr int CHUNK_PLAN_MAXB = 512;  // buckets of the staged scatter
constexpr int CHUNK_PER_WG = 1024;    // chunks per workgroup of k_chunk_hist / k_chunk_place
__global__ void __launch_bounds__(256) k_chunk_hist(const qi64* __restrict__ meta, qi32 np, qu32* __restrict__ cnt,
                                                   unsigned long long* __restrict__ rec) {
  __shared__ qu32 s_cnt[CHUNK_PLAN_MAXB];
  __shared__ unsigned long long s_rec[CHUNK_PLAN_MAXB];
  const qi64 C = meta[0], lo = (qi64)blockIdx.x * CHUNK_PER_WG;
  if (lo >= C) return;
  const qi64 hi = lo + CHUNK_PER_WG < C ? lo + CHUNK_PER_WG : C;
  for (int b = threadIdx.x; b < np; b += blockDim.x) {
    s_cnt[b] = 0;
    s_rec[b] = 0;
  }
  __syncthreads();
  for (qi64 c = lo + threadIdx.x; c < hi; c += blockDim.x) {
    const qi64 w = meta[1 + c];
    if (w < 0) continue;  // an unused id of a workgroup's range (part_static)
    const int b = (int)(w >> 32);
    atomicAdd(&s_cnt[b], 1u);
    atomicAdd(&s_rec[b], (unsigned long long)(w & 0xFFFFFFFFll));
  }
  __syncthreads();
  for (int b = threadIdx.x; b < np; b += blockDim.x)
    if (s_cnt[b]) {
      atomicAdd(&cnt[b], s_cnt[b]);
      atomicAdd(&rec[b], s_rec[b]);
    }
}

__global__ void __launch_bounds__(1024) k_chunk_slices(const qi64* __restrict__ meta, qi32 np, qi64 tmax,
                                                      const qu32* __restrict__ cnt,
                                                      const unsigned long long* __restrict__ rec,
                                                      qi64* __restrict__ out, qu32* __restrict__ base) {
  // one thread per bucket (np <= 1024): a tree reduction of the records, then Hillis-Steele scans of
  // the chunk counts and slice counts (a serial loop over the buckets' global counters took 60 us)
  __shared__ qu32 s_a[1024], s_b[1024];
  __shared__ unsigned long long s_r[1024];
  const int t = threadIdx.x;
  const qu32 c = t < np ? cnt[t] : 0u;
  s_r[t] = t < np ? rec[t] : 0ull;
  s_a[t] = c;
  __syncthreads();
  for (int d = 512; d > 0; d >>= 1) {
    if (t < d) {
      s_r[t] += s_r[t + d];
      s_a[t] += s_a[t + d];
    }
    __syncthreads();
  }
  // chunks in use (meta[0] may also count unused ids of the workgroups' ranges)
  const qi64 C = (qi64)s_a[0], R = (qi64)s_r[0];
  (void)meta;
  __syncthreads();
  const qi64 target = max((qi64)np, min(tmax, R >> 15));
  const qi64 cpc = max((qi64)1, (5 * C + 4 * target - 1) / (4 * target));
  const qu32 ns = (qu32)((c + cpc - 1) / cpc);
  s_a[t] = c;
  s_b[t] = ns;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const qu32 xa = t >= d ? s_a[t - d] : 0u, xb = t >= d ? s_b[t - d] : 0u;
    __syncthreads();
    s_a[t] += xa;
    s_b[t] += xb;
    __syncthreads();
  }
  if (t < np) {
    const qi64 s0 = s_a[t] - c, e0 = s0 + c, sl = s_b[t] - ns;
    base[t] = (qu32)s0;
    for (qi64 k = 0; k < ns; ++k) {
      const qi64 lo = s0 + k * cpc;
      out[2 + 2 * (sl + k)] = lo;
      out[3 + 2 * (sl + k)] = (lo + cpc < e0 ? lo + cpc : e0) | (ns == 1 ? PART_EXCL : 0);
    }
  }
  if (t == 1023) out[0] = s_b[1023];
}

__global__ void __launch_bounds__(256) k_chunk_place(const qi64* __restrict__ meta, qi32 np,
                                                    const qu32* __restrict__ base, qu32* __restrict__ cur,
                                                    qi32* __restrict__ sorted) {
  constexpr int PER = CHUNK_PER_WG / 256;
  __shared__ qu32 s_cnt[CHUNK_PLAN_MAXB];
  const qi64 C = meta[0], lo = (qi64)blockIdx.x * CHUNK_PER_WG;
  if (lo >= C) return;
  for (int b = threadIdx.x; b < np; b += blockDim.x) s_cnt[b] = 0;
  __syncthreads();
  int bk[PER];
  qu32 rk[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const qi64 c = lo + threadIdx.x + 256 * i;
    bk[i] = -1;
    if (c < C && meta[1 + c] >= 0) {
      bk[i] = (int)(meta[1 + c] >> 32);
      rk[i] = atomicAdd(&s_cnt[bk[i]], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < np; b += blockDim.x)
    if (s_cnt[b]) s_cnt[b] = base[b] + atomicAdd(&cur[b], s_cnt[b]);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (bk[i] >= 0) sorted[s_cnt[bk[i]] + rk[i]] = (qi32)(lo + threadIdx.x + 256 * i);
}

// Slices of the spilled bucket (spill_update): one bucket, so the chunk list is the identity
// (sorted[c] = c) and slices are ranges of at most cpc chunks, about min(tmax, records / 32K) of
// them; a single slice is exclusive. Grid: enough threads for every chunk id.
__global__ void k_spill_plan(const qi64* __restrict__ meta, qi64 tmax, qi64* __restrict__ out, qi32* __restrict__ sorted) {
  const qi64 C = meta[0];
  const qi64 c = (qi64)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) sorted[c] = (qi32)c;
  if (blockIdx.x != 0) return;
  qi64 target = (C * PART_CH) >> 15;
  target = target < 1 ? 1 : (target > tmax ? tmax : target);
  const qi64 cpc = (C + target - 1) / target > 0 ? (C + target - 1) / target : 1;
  const qi64 ns = (C + cpc - 1) / cpc;
  for (qi64 k = threadIdx.x; k < ns; k += blockDim.x) {
    const qi64 lo = k * cpc;
    out[2 + 2 * k] = lo;
    out[3 + 2 * k] = (lo + cpc < C ? lo + cpc : C) | (ns == 1 ? PART_EXCL : 0);
  }
  if (threadIdx.x == 0) out[0] = ns;
}

// zero_ctl: the control words too (a reset, or a new state); reset: the slots' E words were in use
__global__ void k_table_init(DTable t, AggMeta m, qu64* zero_ctl, int reset) {
  const qu64 SS = t.cap + 2;
  if (zero_ctl && blockIdx.x == 0 && threadIdx.x < 8) zero_ctl[threadIdx.x] = 0;
  for (qu64 s = blockIdx.x * (qu64)blockDim.x + threadIdx.x; s < SS; s += (qu64)gridDim.x * blockDim.x) {
    t.keys[s] = EMPTY_KEY;
    t.cstar[s] = 0;
    for (int j = 0; j < m.naggs; ++j) {
      // a reset zeroes the E words a slot used (a new table's come zeroed: table_alloc)
      if (reset && m.acc[j] == ACC_SUM_X && (t.idx[j][3 * SS + s] & FX_EXT))
        for (int w = 0; w < FXE_WORDS; ++w) t.ext[j][s * FXE_WORDS + w] = 0;
      t.acc[j][s] = acc_identity(m.acc[j]);
      t.nn[j][s] = 0;
      if (acc_has_idx(m.acc[j]))
        for (int k = 0; k < 4; ++k) t.idx[j][k * SS + s] = idx_identity(m.acc[j]);
    }
  }
}

// nn[j] := cstar for the aggregates in `mask` (an implicit non-null count made explicit, before a
// launch that adds real non-null counts: nullable inputs, imported records, the generic kernel).
__global__ void k_nn_materialize(DTable t, qi32 mask) {
  const qu64 SS = t.cap + 2;
  for (qu64 s = blockIdx.x * (qu64)blockDim.x + threadIdx.x; s < SS; s += (qu64)gridDim.x * blockDim.x)
    for (int j = 0; j < QE_MAX_AGGS; ++j)
      if ((mask >> j) & 1) t.nn[j][s] = t.cstar[s];
}

__device__ __forceinline__ bool gslot_occupied(const DTable& t, qu64 s) {
  return s < t.cap ? t.keys[s] != EMPTY_KEY : t.cstar[s] > 0;
}

// Merge every occupied slot of `src` into `dst` (table growth).
// New groups are counted per workgroup in LDS and added to ctl[0] once (one device-scope add per
// new group on that single word serialised: ~10 us for 1024 groups).
__device__ __forceinline__ void wg_newg_begin(qu32* newg) {
  if (threadIdx.x == 0) *newg = 0;
  __syncthreads();
}
__device__ __forceinline__ void wg_newg_end(qu32* newg, qu64* ctl) {
  __syncthreads();
  if (threadIdx.x == 0 && *newg) atomicAdd((unsigned long long*)&ctl[0], (unsigned long long)*newg);
}

__global__ void k_rehash(DTable src, DTable dst, AggMeta m) {
  __shared__ qu32 newg;
  wg_newg_begin(&newg);
  const qu64 SS = src.cap + 2;
  for (qu64 s = blockIdx.x * (qu64)blockDim.x + threadIdx.x; s < SS; s += (qu64)gridDim.x * blockDim.x) {
    if (!gslot_occupied(src, s)) continue;
    const bool knull = s == src.cap;
    const qi64 key = knull ? 0 : (s == src.cap + 1 ? EMPTY_KEY : src.keys[s]);
    qu64 d;
    if (!gtable_find_wg(dst, key, knull, d, &newg)) {
      atomicAdd((unsigned long long*)&dst.ctl[3], 1ull);
      continue;
    }
    gadd_cstar(dst, d, src.cstar[s]);
    for (int j = 0; j < m.naggs; ++j) {
      DAgg a{};
      a.fn = m.fn[j];
      a.acc = m.acc[j];
      qu64 i[4] = {~0ull, ~0ull, ~0ull, ~0ull};
      if (acc_has_idx(a.acc))
        for (int k = 0; k < 4; ++k) i[k] = src.idx[j][k * SS + s];
      gcombine(dst, a.acc, j, d, src.acc[j][s], slot_nn(src, m, j, s), i[0], i[1], i[2], i[3]);
      if (a.acc == ACC_SUM_X && (i[3] & FX_EXT))  // (the status word carried FX_EXT over)
        fxe_add_words<true>(dst.ext[j] + d * FXE_WORDS, 0, src.ext[j] + s * FXE_WORDS, FXE_WORDS);
    }
  }
  wg_newg_end(&newg, dst.ctl);
}

// Merge fixed-size records (export format) into `dst`.
__device__ void import_record(const qu8* __restrict__ rec, DTable& dst, const AggMeta& m, qu32* newg) {
  const qi64 key = ((const qi64*)rec)[0];
  const bool knull = ((const qu64*)rec)[1] & 1;
  const qu64 c = ((const qu64*)rec)[2];
  qu64 d;
  if (!gtable_find_wg(dst, key, knull, d, newg)) {
    atomicAdd((unsigned long long*)&dst.ctl[3], 1ull);
    return;
  }
  gadd_cstar(dst, d, c);
  int off = 24;
  for (int j = 0; j < m.naggs; ++j) {
    DAgg a{};
    a.fn = m.fn[j];
    a.acc = m.acc[j];
    const qu64* f = (const qu64*)(rec + off);
    if (a.fn != QE_AGG_COUNT_STAR) {
      if (acc_has_idx(a.acc)) gcombine(dst, a.acc, j, d, (qi64)f[0], f[1], f[2], f[3], f[4], f[5]);
      else gcombine(dst, a.acc, j, d, (qi64)f[0], f[1], ~0ull, ~0ull, ~0ull, ~0ull);
    }
    off += agg_rec_bytes(a.acc);
  }
}

__global__ void k_import(const qu8* __restrict__ recs, qi64 nrec, qi32 rec_bytes, DTable dst, AggMeta m) {
  __shared__ qu32 newg;
  wg_newg_begin(&newg);
  for (qi64 r = blockIdx.x * (qi64)blockDim.x + threadIdx.x; r < nrec; r += (qi64)gridDim.x * blockDim.x)
    import_record(recs + r * rec_bytes, dst, m, &newg);
  wg_newg_end(&newg, dst.ctl);
}

// Received slots (qe_hashagg_import_slots): header word 0 = records in the slot (the sender's
// count; may exceed the capacity), word 1 = the sender's largest count over all its slots. Every
// workgroup first reads the headers: if some sender's largest count exceeds the slot capacity
// (the same verdict on every rank), nothing is imported; block 0 reports ctl[4] = that largest
// count, ctl[5] = records held in total. One launch and one read-back for the whole import.
__global__ void k_import_slots(const qu8* __restrict__ slots, qi32 nslots, qi64 slot_records, qi32 rec_bytes,
                               DTable dst, AggMeta m) {
  __shared__ qu32 newg;
  __shared__ qi32 s_ok;
  const qu64 slot_bytes = QE_SLOT_HEADER + (qu64)slot_records * rec_bytes;
  if (threadIdx.x < 64) {
    qu64 mx = 0, tot = 0;
    for (int i = threadIdx.x; i < nslots; i += 64) {
      const qu64* hd = (const qu64*)(slots + (qu64)i * slot_bytes);
      mx = hd[1] > mx ? hd[1] : mx;
      tot += hd[0] < (qu64)slot_records ? hd[0] : (qu64)slot_records;
    }
    for (int off = 32; off > 0; off >>= 1) {
      const qu64 o = __shfl_xor(mx, off);
      mx = o > mx ? o : mx;
      tot += __shfl_xor(tot, off);
    }
    if (threadIdx.x == 0) {
      s_ok = mx <= (qu64)slot_records;
      if (blockIdx.x == 0) {
        dst.ctl[4] = mx;
        dst.ctl[5] = tot;
      }
    }
  }
  wg_newg_begin(&newg);  // (its barrier also publishes s_ok)
  if (s_ok) {
    const qi64 total = (qi64)nslots * slot_records;
    for (qi64 r = blockIdx.x * (qi64)blockDim.x + threadIdx.x; r < total; r += (qi64)gridDim.x * blockDim.x) {
      const qi64 sl = r / slot_records, i = r - sl * slot_records;
      const qu8* base = slots + (qu64)sl * slot_bytes;
      if ((qu64)i >= ((const qu64*)base)[0]) continue;
      import_record(base + QE_SLOT_HEADER + (qu64)i * rec_bytes, dst, m, &newg);
    }
  }
  wg_newg_end(&newg, dst.ctl);
}

__device__ __forceinline__ qu32 partition_of(qi64 key, bool knull, qi32 nparts) {
  const qu64 h = fmix64((qu64)key ^ (knull ? NULL_SALT : 0ull));
  return (qu32)(((h >> 32) * (qu64)nparts) >> 32);
}

// Position of this lane's record in partition p's run: one cursor add per (wave, partition)
// present instead of one per record (every record of a partition hit the same word). The whole
// wave calls it; `has` = this lane has `mult` records.
__device__ __forceinline__ qu64 wave_cursor(unsigned long long* cursor, bool has, qu32 p, qu32 mult = 1) {
  const int lane = threadIdx.x & 63;
  const qu64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  qu64 todo = __ballot(has);
  qu64 pos = 0;
  while (todo) {
    const int leader = __ffsll((long long)todo) - 1;
    const qu32 lp = (qu32)__shfl((int)p, leader);
    const qu64 same = __ballot(has && p == lp);
    qu64 base = 0;
    if (lane == leader) base = atomicAdd(&cursor[lp], (unsigned long long)__popcll(same) * mult);
    base = (qu64)__shfl((long long)base, leader);
    if (has && p == lp) pos = base + (qu64)__popcll(same & lt) * mult;
    todo &= ~same;
  }
  return pos;
}

// A group whose exact fp64 SUMs have E words (FX_EXT) exports FXE_CHUNKS more records, one per
// chunk of E (qe_dev.hpp fxe_partial): every record of a group goes to its key's partition.
__device__ __forceinline__ bool slot_has_ext(const DTable& t, const AggMeta& m, qu64 s) {
  bool e = false;
  for (int j = 0; j < m.naggs; ++j)
    if (m.acc[j] == ACC_SUM_X) e = e || (t.idx[j][3 * (t.cap + 2) + s] & FX_EXT) != 0;
  return e;
}

__global__ void k_export_count(DTable t, AggMeta m, qi32 nparts, unsigned long long* counts) {
  const qu64 SS = t.cap + 2;
  const qu64 stride = (qu64)gridDim.x * blockDim.x;
  for (qu64 s0 = blockIdx.x * (qu64)blockDim.x; s0 < SS; s0 += stride) {
    const qu64 s = s0 + threadIdx.x;
    const bool has = s < SS && gslot_occupied(t, s);
    const bool knull = s == t.cap;
    const qi64 key = !has ? 0 : knull ? 0 : (s == t.cap + 1 ? EMPTY_KEY : t.keys[s]);
    const qu32 p = has ? partition_of(key, knull, nparts) : 0;
    (void)wave_cursor(counts, has, p);
    if (m.any_x) (void)wave_cursor(counts, has && slot_has_ext(t, m, s), p, FXE_CHUNKS);
  }
}

__device__ void write_record(qu8* rec, const DTable& t, const AggMeta& m, qu64 s, qi64 key, bool knull) {
  const qu64 SS = t.cap + 2;
  write_record_head(rec, key, knull, t.cstar[s]);
  int off = 24;
  for (int j = 0; j < m.naggs; ++j) {
    qu64* f = (qu64*)(rec + off);
    f[0] = (qu64)t.acc[j][s];
    f[1] = slot_nn(t, m, j, s);
    if (acc_has_idx(m.acc[j]))
      for (int k = 0; k < 4; ++k) f[2 + k] = t.idx[j][k * SS + s];
    off += agg_rec_bytes(m.acc[j]);
  }
}

// Chunk c of the E words of group slot s (COUNT(*) 0; identity partials but those SUMs).
__device__ void write_chunk_record(qu8* rec, const DTable& t, const AggMeta& m, qu64 s, qi64 key, bool knull,
                                   int c) {
  const qu64 SS = t.cap + 2;
  write_record_head(rec, key, knull, 0);
  int off = 24;
  for (int j = 0; j < m.naggs; ++j) {
    qu64* f = (qu64*)(rec + off);
    const int acc = m.acc[j];
    f[0] = (qu64)acc_identity(acc);
    f[1] = 0;
    if (acc_has_idx(acc))
      for (int k = 0; k < 4; ++k) f[2 + k] = idx_identity(acc);
    if (acc == ACC_SUM_X && (t.idx[j][3 * SS + s] & FX_EXT)) {
      const qu64* e = t.ext[j] + s * FXE_WORDS + 4 * c;
      const int n = c == FXE_CHUNKS - 1 ? FXE_WORDS - 4 * c : 4;
      f[0] = e[0];
      for (int k = 1; k < n; ++k) f[1 + k] = e[k];
      f[5] = FX_CHUNK | ((qu64)c << 8);
    }
    off += agg_rec_bytes(acc);
  }
}

// counts (nparts) -> exclusive offsets in place; one wave, nparts is a rank count
__global__ void k_counts_to_cursors(unsigned long long* c, qi32 nparts) {
  if (threadIdx.x == 0) {
    unsigned long long run = 0;
    for (int p = 0; p < nparts; ++p) {
      const unsigned long long x = c[p];
      c[p] = run;
      run += x;
    }
  }
}

__global__ void k_export(DTable t, AggMeta m, qi32 nparts, qi32 rec_bytes, unsigned long long* cursor,
                         qu8* __restrict__ dst) {
  const qu64 SS = t.cap + 2;
  const qu64 stride = (qu64)gridDim.x * blockDim.x;
  // trip count uniform per wave (wave_cursor is a whole-wave operation)
  for (qu64 s0 = blockIdx.x * (qu64)blockDim.x; s0 < SS; s0 += stride) {
    const qu64 s = s0 + threadIdx.x;
    const bool has = s < SS && gslot_occupied(t, s);
    const bool knull = s == t.cap;
    const qi64 key = !has ? 0 : knull ? 0 : (s == t.cap + 1 ? EMPTY_KEY : t.keys[s]);
    const qu32 p = has ? partition_of(key, knull, nparts) : 0;
    const qu64 pos = wave_cursor(cursor, has, p);
    if (has) write_record(dst + pos * (qu64)rec_bytes, t, m, s, key, knull);
    if (m.any_x) {
      const bool ext = has && slot_has_ext(t, m, s);
      const qu64 pe = wave_cursor(cursor, ext, p, FXE_CHUNKS);
      if (ext)
        for (int c = 0; c < FXE_CHUNKS; ++c) write_chunk_record(dst + (pe + c) * (qu64)rec_bytes, t, m, s, key, knull, c);
    }
  }
}

// Fixed-capacity slots (qe_hashagg_export_slots): the first `slot_records` groups of partition p
// go to slot p; cursor[p] ends as the partition's full count
__global__ void k_export_slots(DTable t, AggMeta m, qi32 nparts, qi32 rec_bytes, qi64 slot_records,
                               unsigned long long* cursor, qu8* __restrict__ dst) {
  const qu64 SS = t.cap + 2;
  const qu64 slot_bytes = QE_SLOT_HEADER + (qu64)slot_records * rec_bytes;
  const qu64 stride = (qu64)gridDim.x * blockDim.x;
  for (qu64 s0 = blockIdx.x * (qu64)blockDim.x; s0 < SS; s0 += stride) {
    const qu64 s = s0 + threadIdx.x;
    const bool has = s < SS && gslot_occupied(t, s);
    const bool knull = s == t.cap;
    const qi64 key = !has ? 0 : knull ? 0 : (s == t.cap + 1 ? EMPTY_KEY : t.keys[s]);
    const qu32 p = has ? partition_of(key, knull, nparts) : 0;
    const qu64 pos = wave_cursor(cursor, has, p);
    qu8* base = dst + p * slot_bytes + QE_SLOT_HEADER;
    if (has && pos < (qu64)slot_records) write_record(base + pos * (qu64)rec_bytes, t, m, s, key, knull);
    if (m.any_x) {
      const bool ext = has && slot_has_ext(t, m, s);
      const qu64 pe = wave_cursor(cursor, ext, p, FXE_CHUNKS);
      if (ext)
        for (int c = 0; c < FXE_CHUNKS; ++c)
          if (pe + c < (qu64)slot_records) write_chunk_record(base + (pe + c) * (qu64)rec_bytes, t, m, s, key, knull, c);
    }
  }
}

// guard (a stream-ordered update not yet read back): its deferred-row / overflow / lost counters;
// any of them nonzero means the table is incomplete, so word 1 reports "too many" and every rank
// takes the variable-size exchange, which settles the update first.
__global__ void k_slot_headers(const unsigned long long* __restrict__ cursor, qi32 nparts, qu64 slot_bytes,
                               qu8* __restrict__ dst, const qu64* __restrict__ guard) {
  // one wave: word 0 = this slot's count, word 1 = the largest count over all slots
  qu64 mx = 0;
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) mx = cursor[p] > mx ? cursor[p] : mx;
  for (int off = 32; off > 0; off >>= 1) {
    const qu64 o = __shfl_xor(mx, off);
    mx = o > mx ? o : mx;
  }
  if (guard && (guard[1] | guard[2] | guard[3])) mx = 1ull << 62;
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) {
    qu64* hd = (qu64*)(dst + (qu64)p * slot_bytes);
    hd[0] = cursor[p];
    hd[1] = mx;
    for (int w = 2; w < QE_SLOT_HEADER / 8; ++w) hd[w] = 0;
  }
}

// ---- finalize: occupied slots -> one output batch --------------------------------------------------
__global__ void k_occ_count(DTable t, qi64* __restrict__ tile_counts, qi32 tile_slots) {
  // one block per tile of `tile_slots` slots
  __shared__ qi64 part[4];
  const qu64 SS = t.cap + 2;
  const qu64 s0 = (qu64)blockIdx.x * tile_slots;
  qi64 c = 0;
  for (int i = threadIdx.x; i < tile_slots; i += blockDim.x) {
    const qu64 s = s0 + i;
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

__device__ __forceinline__ void set_bit(qu8* bm, qi64 i, bool v) {
  // bytes are written by whole 32-bit atomics: the host zeroes validity buffers first
  if (v) atomicOr((qu32*)bm + (i >> 5), 1u << (i & 31));
}

__device__ __forceinline__ void store_typed(void* p, qi32 type, qi64 i, qi64 x) {
  switch (type) {
    case QE_TYPE_INT64:
    case QE_TYPE_FLOAT64: ((qi64*)p)[i] = x; break;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: ((qi32*)p)[i] = (qi32)x; break;
    default: ((qu8*)p)[i] = (qu8)x;
  }
}

// one occupied slot -> output row o of the batch. Validity bits go to the output bitmaps with
// global atomics, or (lbits != nullptr) to per-column LDS bitmaps of FS_WORDS words each.
constexpr int FS_WORDS = 512;
__device__ __forceinline__ void put_bit(qu8* gbm, qu32* lbits, int col, qi64 o, bool v) {
  if (!v) return;
  if (lbits) atomicOr(lbits + col * FS_WORDS + (o >> 5), 1u << (o & 31));
  else set_bit(gbm, o, true);
}

// An ACC_SUM_X slot's value (word 0 = acc, words 1..3 and the status word in idx, E in ext;
// qe_dev.hpp fx_result): the correctly rounded exact sum.
__device__ __forceinline__ double fx_sum(const DTable& t, int j, qu64 s, qi64 acc) {
  const qu64 SS = t.cap + 2;
  const qu64* ix = t.idx[j];
  return fx_result((qu64)acc, ix[s], ix[SS + s], ix[2 * SS + s], ix[3 * SS + s], t.ext[j] + s * FXE_WORDS);
}

__device__ __forceinline__ void finalize_slot(const DTable& t, const AggMeta& m, const KeyMeta& km,
                                              const OutCols& out, qu64 s, qi64 o, qu32* lbits = nullptr) {
  const qu64 SS = t.cap + 2;
  const bool knull = s == t.cap;
  const qi64 key = knull ? 0 : (s == t.cap + 1 ? EMPTY_KEY : t.keys[s]);
  // keys
  if (km.mode == 1) {
    store_typed(out.keys[0].values, km.type[0], o, key);
    if (out.keys[0].validity) put_bit(out.keys[0].validity, lbits, 0, o, !knull);
  } else if (km.mode == 2) {
    for (int k = 0; k < km.nkeys; ++k) {
      const bool isn = (key >> km.nullbit[k]) & 1;
      qi64 x = (key >> km.shift[k]) & km.fmask[k];
      if (km.type[k] == QE_TYPE_INT32 || km.type[k] == QE_TYPE_DATE32) x = (qi64)(qi32)x;  // sign
      store_typed(out.keys[k].values, km.type[k], o, x);
      if (out.keys[k].validity) put_bit(out.keys[k].validity, lbits, k, o, !isn);
    }
  }
  // aggregates (a rolled loop: the kernel is one workgroup whose run time is mostly instruction
  // fetch, so code size is what counts — unrolled over QE_MAX_AGGS it ran 16 us instead of 13)
  const qu64 cst = t.cstar[s];
#pragma unroll 1
  for (int j = 0; j < m.naggs; ++j) {
    if (!out.aggs[j].values) continue;  // keys only (qe_hashagg_finalize_sizes of a keyed state)
    const qu64 nn = slot_nn(t, m, j, s);
    const qi64 acc = t.acc[j][s];
    qi64 val = 0;
    bool valid = nn > 0;
    switch (m.fn[j]) {
      case QE_AGG_COUNT: val = (qi64)nn; valid = true; break;
      case QE_AGG_COUNT_STAR: val = (qi64)cst; valid = true; break;
      case QE_AGG_AVG:
        if (m.acc[j] == ACC_SUM_X)
          val = f64_bits(fx_sum(t, j, s, acc) / (double)nn);
        else
          val = f64_bits(bits_f64(acc) / (double)nn);
        break;
      default:
        if (m.acc[j] == ACC_SUM_X) {
          val = f64_bits(fx_sum(t, j, s, acc));
        } else if (acc_is_f64mm(m.acc[j])) {
          const qu64 i0 = t.idx[j][s], i1 = t.idx[j][SS + s];
          const qu64 i2 = t.idx[j][2 * SS + s], i3 = t.idx[j][3 * SS + s];
          if (i1 != ~0ull && i1 == i0) {
            val = 0x7FF8000000000000ll;  // first non-null value was NaN: sticky seed
          } else {
            const double d = okey_f64(acc);
            val = d == 0.0 ? f64_bits(i2 < i3 ? -0.0 : 0.0) : f64_bits(d);
          }
        } else {
          val = acc;
        }
    }
    ((qi64*)out.aggs[j].values)[o] = valid ? val : 0;
    if (out.aggs[j].validity) put_bit(out.aggs[j].validity, lbits, QE_MAX_KEYS + j, o, valid);
  }
}

__global__ void k_finalize(DTable t, AggMeta m, KeyMeta km, const qi64* __restrict__ tile_offsets,
                           qi32 tile_slots, OutCols out) {
  // one block per tile; each wave scans its slots in order (ballot + popc keeps slot order)
  __shared__ int wtot[4];
  const qu64 SS = t.cap + 2;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const qu64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  qi64 base = tile_offsets[blockIdx.x];
  for (int it = 0; it < tile_slots; it += blockDim.x) {
    const qu64 s = (qu64)blockIdx.x * tile_slots + it + threadIdx.x;
    const bool occ = (it + (int)threadIdx.x) < tile_slots && s < SS && gslot_occupied(t, s);
    const qu64 b = __ballot(occ);
    if (lane == 0) wtot[wid] = __popcll(b);
    __syncthreads();
    int woff = 0, btot = 0;
    for (int w = 0; w < 4; ++w) {
      woff += w < wid ? wtot[w] : 0;
      btot += wtot[w];
    }
    if (occ) finalize_slot(t, m, km, out, s, base + woff + __popcll(b & lt));
    base += btot;
    __syncthreads();
  }
}

// Small tables (<= FS_THREADS * FS_PER slots): the whole finalize in ONE workgroup — validity
// zeroing, occupancy, slot-order prefix and the writes — instead of memsets + count + scan +
// write launches. Slot s = FS_THREADS * i + tid (chunk i): every occupancy load is coalesced and
// independent of the others; the prefix is ballots + one LDS exchange.
constexpr int FS_THREADS = 1024, FS_PER = 16, FS_WAVES = FS_THREADS / 64;
static_assert(FS_THREADS * FS_PER / 2 / 32 <= FS_WORDS, "LDS bitmaps hold every group of a small table");
__global__ void __launch_bounds__(FS_THREADS) k_finalize_small(DTable t, AggMeta m, KeyMeta km, OutCols out,
                                                               qi64 groups) {
  __shared__ qi32 wcnt[FS_PER][FS_WAVES];  // set slots per (chunk, wave), then their exclusive prefix
  __shared__ qu64 wbal[FS_PER][FS_WAVES];  // their ballots
  __shared__ qu32 lbits[(QE_MAX_KEYS + QE_MAX_AGGS) * FS_WORDS];  // validity, copied out at the end
  const qu64 SS = t.cap + 2;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const qu64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int words = (int)((groups + 31) >> 5);  // <= FS_WORDS: groups <= half the slots
  for (int w = tid; w < (QE_MAX_KEYS + QE_MAX_AGGS) * FS_WORDS; w += FS_THREADS) lbits[w] = 0;
  qu32 occ = 0;
#pragma unroll
  for (int i = 0; i < FS_PER; ++i) {
    const qu64 s = (qu64)i * FS_THREADS + tid;
    if (s < SS && gslot_occupied(t, s)) occ |= 1u << i;
  }
#pragma unroll
  for (int i = 0; i < FS_PER; ++i) {
    const qu64 b = __ballot((occ >> i) & 1);
    if (lane == 0) {
      wbal[i][wid] = b;
      wcnt[i][wid] = __popcll(b);
    }
  }
  __syncthreads();  // also orders the LDS zeroing before any bit is set
  // exclusive prefix of the (chunk, wave) counts in slot order, by wave 0: four per lane, then a
  // wave scan (a serial walk by one thread was 256 dependent LDS reads, ~10 us)
  static_assert(FS_PER * FS_WAVES == 4 * 64, "four (chunk, wave) counts per lane");
  if (wid == 0) {
    qi32* flat = &wcnt[0][0];
    const qi32 c0 = flat[4 * lane], c1 = flat[4 * lane + 1], c2 = flat[4 * lane + 2], c3 = flat[4 * lane + 3];
    const qi32 sum = c0 + c1 + c2 + c3;
    qi32 inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const qi32 y = __shfl_up(inc, d);
      if (lane >= d) inc += y;
    }
    const qi32 ex = inc - sum;
    flat[4 * lane] = ex;
    flat[4 * lane + 1] = ex + c0;
    flat[4 * lane + 2] = ex + c0 + c1;
    flat[4 * lane + 3] = ex + c0 + c1 + c2;
  }
  __syncthreads();
  while (occ) {
    const int i = __ffs(occ) - 1;
    occ &= occ - 1;
    const qi64 o = wcnt[i][wid] + __popcll(wbal[i][wid] & lt);  // wcnt now holds the prefix
    finalize_slot(t, m, km, out, (qu64)i * FS_THREADS + tid, o, lbits);
  }
  __syncthreads();
  for (int w = tid; w < words; w += FS_THREADS) {
    for (int k = 0; k < QE_MAX_KEYS; ++k)
      if (k < km.nkeys && out.keys[k].validity) ((qu32*)out.keys[k].validity)[w] = lbits[k * FS_WORDS + w];
    for (int j = 0; j < m.naggs; ++j)
      if (out.aggs[j].validity) ((qu32*)out.aggs[j].validity)[w] = lbits[(QE_MAX_KEYS + j) * FS_WORDS + w];
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
  int32_t nn_implicit = 0;  // bit j: the table's non-null count of aggregate j is COUNT(*) (AggMeta)
  int64_t row_base = 0;
  int64_t known_groups = 0;  // group count as of the last update/reset; -1 = read the device counter
  // global table
  void* table_mem = nullptr;
  DTable t{};
  qu64* ctl = nullptr;  // device, 8 words
  // LDS sizing
  int32_t lds_log2 = 0;  // largest LDS table (log2 slots); 0 => global-only mode
  int32_t lds_log2_min = 0;
  int64_t expected_groups = 0;  // sizing hint; raised by adapt_after_update once the LDS table is outgrown
  int64_t create_groups = 0;    // qe_hashagg_create's expected groups, never changed (exchange slot sizing)
  int grid = 0;          // workgroups per launch (cap)
  // radix-partitioned updates (expected groups beyond the LDS table): counts / offsets, records
  int64_t* part_cnt = nullptr;
  size_t part_cnt_bytes = 0;
  uint8_t* part_rec = nullptr;
  size_t part_rec_bytes = 0;
  int64_t* part_slc = nullptr;  // slice descriptors of the partition-aggregate pass
  size_t part_slc_bytes = 0;
  // 32-bit partition records (Plan.part_narrow): off for good once a value did not fit
  bool part_wide = false;
  bool narrow_failed = false;  // the last settled launch saw ctl[7] set
  bool compact_off = false;    // a value did not fit the compact fused table (ctl[7] bit 1): not again
  // overflow records
  uint8_t* ovf = nullptr;
  uint64_t ovf_cap = 0;
  // deferred-row bitmaps
  uint32_t* defer[2] = {nullptr, nullptr};
  size_t defer_words = 0;
  bool defer_dirty[2] = {false, false};
  bool ctl_rows_clean = false;  // ctl[1] / ctl[2] known zero (written only by update launches)
  // HIP events around the aggregation kernel launches of the last update (measurement hook)
  hipEvent_t ev[2] = {nullptr, nullptr};
  double last_kernel_ms = 0.0;
  int last_launches = 0;
  int last_specialized = 0;  // 1: the last update ran a hipRTC-specialised kernel
  uint64_t last_sig = 0;     // signature of the last aggregation launch (kernel compile key + shape)
  std::string jit_note;      // why the last update could not specialise (empty if it did)
  // stream-ordered updates (qe_hashagg_set_async): the last update's launch, read back later
  bool async = false;
  bool pending = false;
  std::unique_ptr<qe::Plan> pend_plan;
  size_t pend_lds = 0;
  int pend_out_i = 0;
  // pinned snapshot of the control words queued behind each update launch, and its event
  uint64_t* ctl_pin = nullptr;
  hipEvent_t ev_ctl = nullptr;
  // a stream-ordered update whose settling failed leaves an incomplete table: every later call
  // that reads the state fails with this status until qe_hashagg_reset
  int poisoned = 0;
  std::string poison_msg;
  // the declared (original) key columns and their dictionaries (qe_keyed.hip); the fields above
  // describe the DEVICE key columns the table groups by
  qe::Keyed* keyed = nullptr;
  int32_t flags = 0;      // qe_hashagg_create_ex flags
  uint64_t version = 0;   // bumped by every change of the groups
};

namespace qe {

int hashagg_expected_groups(const qe_hashagg* h, int64_t* out) {
  QE_CHECK(h && out, QE_ERR_INVALID_ARG, "null argument");
  // the create-time value: the exchange sizes equal slots from it, so it must be the same on every
  // rank whatever each rank's own data did to the sizing hint (adapt_after_update)
  *out = h->create_groups;
  return QE_OK;
}

qe_ctx* hashagg_ctx(const qe_hashagg* h) { return h ? h->ctx : nullptr; }

HashaggInfo hashagg_info(const qe_hashagg* h) {
  HashaggInfo I{};
  I.ctx = h->ctx;
  I.km = h->km;
  I.rec_bytes = h->rec_bytes;
  I.naggs = h->naggs;
  I.flags = h->flags;
  for (int j = 0; j < h->naggs; ++j) I.aggs[j] = h->aggs[j];
  I.version = h->version;
  I.ctl = (uint64_t*)h->ctl;
  I.keyed = h->keyed;
  return I;
}

static AggMeta agg_meta(const qe_hashagg* h) {
  AggMeta m{};
  m.naggs = h->naggs;
  for (int j = 0; j < h->naggs; ++j) {
    m.fn[j] = h->aggs[j].fn;
    m.acc[j] = h->acc[j];
    m.any_x = m.any_x || h->acc[j] == ACC_SUM_X;
  }
  m.nn_implicit = h->nn_implicit;
  return m;
}

// Every aggregate's non-null count starts implicit (an empty table: nn == cstar == 0). The fused
// kernel keeps it implicit while the aggregate's input is non-nullable — its flush then skips the
// nn atomics (3 of the C4 flush's 7 per group) — and anything that adds real counts makes it
// explicit first.
static int32_t all_nn_bits(const qe_hashagg* h) {
  static const bool off = [] {  // QE_NN_IMPLICIT=0: always store the counts (A/B and debugging)
    const char* e = getenv("QE_NN_IMPLICIT");
    return e && e[0] == '0';
  }();
  if (off) return 0;
  int32_t b = 0;
  for (int j = 0; j < h->naggs; ++j)
    if (h->aggs[j].fn != QE_AGG_COUNT_STAR) b |= 1 << j;
  return b;
}

static int nn_materialize(qe_hashagg* h, int32_t mask) {
  mask &= h->nn_implicit;
  if (!mask) return QE_OK;
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 4096);
  hipLaunchKernelGGL(k_nn_materialize, dim3(grid), dim3(256), 0, h->ctx->stream, h->t, (qi32)mask);
  QE_TRY(launch_check("k_nn_materialize"));
  h->nn_implicit &= ~mask;
  return QE_OK;
}

// Per slot: key and COUNT(*), and per aggregate its accumulator, non-null count, four idx words
// (fp64 MIN/MAX, exact SUM) and for an exact SUM the FXE_WORDS words of E.
static size_t table_bytes(const qe_hashagg* h, uint64_t cap) {
  const uint64_t SS = cap + 2;
  size_t b = 16 * SS;
  for (int j = 0; j < h->naggs; ++j)
    b += (16 + (acc_has_idx(h->acc[j]) ? 32 : 0) + (h->acc[j] == ACC_SUM_X ? 8 * FXE_WORDS : 0)) * SS;
  return b;
}

// zero_ctl: a new state's control words, zeroed by the same init launch (no separate memset)
static int table_alloc(qe_hashagg* h, uint64_t cap, void** mem, DTable* t, qu64* zero_ctl = nullptr) {
  const size_t bytes = table_bytes(h, cap);
  QE_TRY(dev_alloc(h->ctx, bytes, mem));
  const uint64_t SS = cap + 2;
  char* p = (char*)*mem;
  *t = DTable{};
  t->keys = (qi64*)p;
  p += 8 * SS;
  t->cstar = (qu64*)p;
  p += 8 * SS;
  for (int j = 0; j < h->naggs; ++j) {
    t->acc[j] = (qi64*)p;
    p += 8 * SS;
    t->nn[j] = (qu64*)p;
    p += 8 * SS;
    if (acc_has_idx(h->acc[j])) {
      t->idx[j] = (qu64*)p;
      p += 32 * SS;
    }
  }
  // E words last, one run: zeroed here (k_table_init resets only the slots that used theirs)
  char* e0 = p;
  for (int j = 0; j < h->naggs; ++j)
    if (h->acc[j] == ACC_SUM_X) {
      t->ext[j] = (qu64*)p;
      p += 8 * FXE_WORDS * SS;
    }
  if (p > e0) QE_HIP(hipMemsetAsync(e0, 0, (size_t)(p - e0), h->ctx->stream));
  t->cap = cap;
  t->ctl = h->ctl;
  const int grid = (int)std::min<uint64_t>(div_up(SS, 256), 4096);
  hipLaunchKernelGGL(k_table_init, dim3(grid), dim3(256), 0, h->ctx->stream, *t, agg_meta(h), zero_ctl, 0);
  return launch_check("k_table_init");
}

// ctl words: [0] groups, [1] deferred rows, [2] overflow records, [3] lost groups,
// [4] largest slot count reported by the senders of an import_slots, [5] their records in total,
// ctl[3] is sticky: every path that can drop a group (k_rehash, k_import, k_import_slots, the
// fused kernel's overflow area) adds to it and nothing but a reset clears it, so a loss in a
// launch with no read-back of its own (qe_hashagg_import_slots queues k_import_slots and returns)
// fails the next call that reads the counters — at the latest finalize / num_groups.
static int read_ctl(qe_hashagg* h, uint64_t out[8]) {
  void* p;
  QE_TRY(ctx_pinned(h->ctx, 64, &p));
  QE_HIP(hipMemcpyAsync(p, h->ctl, 64, hipMemcpyDeviceToHost, h->ctx->stream));
  QE_TRY(ctx_sync(h->ctx));
  memcpy(out, p, 64);
  QE_CHECK((out[3] & CTL_KEY_TOO_LONG) == 0, QE_ERR_INVALID_ARG,
           "a UTF8 group key is longer than its column's max_len promised (qe_column.max_len)");
  QE_CHECK(out[3] == 0, QE_ERR_CAPACITY, "hash aggregate lost %llu groups (probe limit or overflow area)",
           (unsigned long long)out[3]);
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
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 8192);
  hipLaunchKernelGGL(k_rehash, dim3(grid), dim3(256), 0, h->ctx->stream, h->t, nt, agg_meta(h));
  QE_TRY(launch_check("k_rehash"));
  uint64_t c[8];
  QE_TRY(read_ctl(h, c));  // synchronises: the old table can go
  QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash table rehash lost %llu groups", (unsigned long long)c[3]);
  dev_free(h->ctx, h->table_mem);
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
  uint64_t c[8];
  QE_TRY(read_ctl(h, c));
  QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash table import lost %llu groups", (unsigned long long)c[3]);
  return QE_OK;
}

static int ensure_defer(qe_hashagg* h, int64_t n) {
  const size_t words = (size_t)div_up((uint64_t)n, 32);
  if (words <= h->defer_words) return QE_OK;
  for (int i = 0; i < 2; ++i) {
    dev_free(h->ctx, h->defer[i]);
    h->defer[i] = nullptr;
  }
  for (int i = 0; i < 2; ++i) {  // (zeroed by launch_pass before a launch first writes one)
    QE_TRY(dev_alloc(h->ctx, words * 4, (void**)&h->defer[i]));
    h->defer_dirty[i] = true;
  }
  h->defer_words = words;
  return QE_OK;
}

// Compiled launch description (host side mirror of qe_fused_spec after type checking).
// Columns, mask and predicate terms of a fused plan (shared with qe_selproj.hip).
int compile_inputs(const qe_column* cols, int32_t ncols, int32_t mask_col, int32_t nterms, const qe_pred_term* terms,
                   Plan* P, bool* col_f64) {
  *P = Plan{};
  QE_CHECK(ncols >= 1 && ncols <= QE_MAX_COLS, QE_ERR_UNSUPPORTED, "fused plan takes 1..%d columns (got %d)",
           QE_MAX_COLS, ncols);
  const int64_t n = cols[0].length;
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
  P->all8 = 1;
  for (int c = 0; c < ncols; ++c) P->all8 &= (cols[c].type == QE_TYPE_INT64 || cols[c].type == QE_TYPE_FLOAT64) ? 1 : 0;
  P->n = n;
  // mask
  P->mask_col = mask_col;
  if (mask_col >= 0) {
    QE_CHECK(mask_col < ncols && cols[mask_col].type == QE_TYPE_BOOL, QE_ERR_INVALID_ARG,
             "mask_col must name a BOOL column");
  }
  // predicate terms
  QE_CHECK(nterms >= 0 && nterms <= QE_MAX_TERMS, QE_ERR_UNSUPPORTED, "too many predicate terms");
  P->nterms = nterms;
  for (int i = 0; i < nterms; ++i) {
    const qe_pred_term& s = terms[i];
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
  return QE_OK;
}

// Type-checks postfix program `pg` and emits its typed tokens into a->tok / a->ntok.
// *is_f: the result is fp64; *nullable: the result can be null (nullable column, null literal,
// or int64 division, whose x / 0 is null).
int compile_program(const qe_column* cols, int32_t ncols, const bool* col_f64, const qe_agg_program& pg, int j,
                    DAgg* a, bool* is_f, bool* nullable) {
  QE_CHECK(pg.ntokens >= 1 && pg.ntokens <= QE_MAX_TOKENS, QE_ERR_INVALID_ARG, "expression %d: empty program", j);
  bool st_f[QE_MAX_TOKENS + 4];
  int depth = 0, nt = 0;
  *nullable = false;
  auto emit = [&](int32_t op, int32_t arg, int64_t lit, int32_t lit_null, int32_t lit_f64 = 0) -> int {
    QE_CHECK(nt < QE_MAX_TOKENS, QE_ERR_UNSUPPORTED, "expression %d: program too long after type promotion", j);
    a->tok[nt++] = DTok{(short)op, (char)lit_null, (char)lit_f64, arg, lit};
    return QE_OK;
  };
  for (int t = 0; t < pg.ntokens; ++t) {
    const qe_token& tk = pg.tokens[t];
    if (tk.op == QE_TOK_COL) {
      QE_CHECK(tk.arg >= 0 && tk.arg < ncols && is_fixed(cols[tk.arg].type), QE_ERR_INVALID_ARG,
               "expression %d: bad column slot %d", j, tk.arg);
      QE_CHECK(depth < 4, QE_ERR_UNSUPPORTED, "expression %d: deeper than 4", j);
      QE_TRY(emit(T_COL, tk.arg, 0, 0));
      st_f[depth++] = col_f64[tk.arg];
      *nullable = *nullable || cols[tk.arg].validity != nullptr;
    } else if (tk.op == QE_TOK_LIT) {
      QE_CHECK(tk.lit.type == QE_TYPE_INT64 || tk.lit.type == QE_TYPE_FLOAT64, QE_ERR_UNSUPPORTED,
               "expression %d: literal type", j);
      QE_CHECK(depth < 4, QE_ERR_UNSUPPORTED, "expression %d: deeper than 4", j);
      QE_TRY(emit(T_LIT, 0, tk.lit.bits, tk.lit.is_null, tk.lit.type == QE_TYPE_FLOAT64 ? 1 : 0));
      st_f[depth++] = tk.lit.type == QE_TYPE_FLOAT64;
      *nullable = *nullable || tk.lit.is_null;
    } else if (tk.op >= QE_TOK_ADD && tk.op <= QE_TOK_DIV) {
      QE_CHECK(depth >= 2, QE_ERR_INVALID_ARG, "expression %d: stack underflow", j);
      const bool f = st_f[depth - 1] || st_f[depth - 2];
      if (f && !st_f[depth - 1]) QE_TRY(emit(T_I2F0, 0, 0, 0));
      if (f && !st_f[depth - 2]) QE_TRY(emit(T_I2F1, 0, 0, 0));
      const int32_t base_op = f ? T_ADD_F : T_ADD_I;
      QE_TRY(emit(base_op + (tk.op - QE_TOK_ADD), 0, 0, 0));
      if (!f && tk.op == QE_TOK_DIV) *nullable = true;  // x / 0 -> null
      --depth;
      st_f[depth - 1] = f;
    } else {
      return fail(QE_ERR_INVALID_ARG, "expression %d: bad token op %d", j, tk.op);
    }
  }
  QE_CHECK(depth == 1, QE_ERR_INVALID_ARG, "expression %d: program leaves %d values", j, depth);
  a->ntok = nt;
  *is_f = st_f[0];
  return QE_OK;
}

static int compile_plan(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec, Plan* P) {
  bool col_f64[QE_MAX_COLS];
  QE_TRY(compile_inputs(cols, ncols, spec->mask_col, spec->nterms, spec->terms, P, col_f64));
  P->row_base = h->row_base;
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
    bool is_f = false, nullable = false;
    QE_TRY(compile_program(cols, ncols, col_f64, spec->inputs[j], j, &a, &is_f, &nullable));
    int nt = a.ntok;
    const bool want_f = h->aggs[j].fn == QE_AGG_AVG || h->aggs[j].input_type == QE_TYPE_FLOAT64;
    if (a.fn != QE_AGG_COUNT) {
      QE_CHECK(!(is_f && !want_f), QE_ERR_INVALID_ARG,
               "aggregate %d: fp64 input for an int64 aggregate (declare input_type FLOAT64)", j);
      if (want_f && !is_f) {
        QE_CHECK(nt < QE_MAX_TOKENS, QE_ERR_UNSUPPORTED, "aggregate %d: program too long after type promotion", j);
        a.tok[nt++] = DTok{(short)T_I2F0, 0, 0, 0, 0};
      }
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
    } else if (nt == 3 && a.tok[0].op == T_COL && (a.tok[1].op == T_COL || a.tok[1].op == T_LIT) &&
               a.tok[2].op >= T_ADD_I) {
      a.pkind = 3;
      a.col = a.tok[0].arg;
      a.bop = a.tok[2].op;
      a.rhs = a.tok[1].op == T_COL ? a.tok[1].arg : -1;
      a.rhs_lit = a.tok[1].lit;
      a.rhs_null = a.tok[1].lit_null;
    } else {
      a.pkind = 2;
    }
  }
  // aggregates that sum the same expression into the same kind of accumulator (TPC-H Q1's
  // SUM(l_extendedprice) and AVG(l_extendedprice)) share one LDS accumulator in the specialised
  // kernels; the global table and the output keep one per aggregate
  for (int j = 0; j < h->naggs; ++j) {
    DAgg& b = P->aggs[j];
    if (b.pkind == 0 || (b.acc != ACC_SUM_I && b.acc != ACC_SUM_F && b.acc != ACC_SUM_X)) continue;
    for (int i = 0; i < j; ++i) {
      const DAgg& a = P->aggs[i];
      if (a.share || a.acc != b.acc || a.pkind != b.pkind || a.track_nn != b.track_nn || a.col != b.col ||
          a.cvt_i2f != b.cvt_i2f || a.ntok != b.ntok || a.bop != b.bop || a.rhs != b.rhs || a.rhs_null != b.rhs_null ||
          a.rhs_lit != b.rhs_lit || memcmp(a.tok, b.tok, sizeof(DTok) * (size_t)a.ntok) != 0)
        continue;
      b.share = i + 1;
      break;
    }
  }
  P->rec_bytes = h->rec_bytes;
  return QE_OK;
}

// LDS layout for a table of 2^log2 slots under this launch's aggregates. Returns bytes.
// LDS words per slot beyond acc of an aggregate with idx arrays: fp64 MIN / MAX keep 4 row
// indices; an exact fp64 SUM keeps 4 more words (256-bit + status) in the generic kernel, and in
// the plan-specialised kernels 5 (limb window, qe_dev.hpp fxl_add) or 2 (192-bit window, fxw_add);
// rare rows go global.
static size_t idx_words(int acc, bool generic) {
  return acc == ACC_SUM_X && !generic ? (size_t)fx_window_idx_words() : 4;
}

static size_t lds_layout_at(const qe_hashagg* h, Plan* P, int log2, bool generic = false) {
  generic = generic || !h->ctx->jit;
  const size_t SS = ((size_t)1 << log2) + 2;
  size_t off = 8 * SS;  // keys
  P->off_cstar = (int32_t)off;
  off += 4 * SS;
  off = (off + 15) & ~size_t(15);
  for (int j = 0; j < h->naggs; ++j) {
    const DAgg& a = P->aggs[j];
    if (!generic && a.share) continue;  // the specialised kernels read the shared accumulator
    if (a.acc != ACC_NONE) {
      P->off_acc[j] = (int32_t)off;
      off += 8 * SS;
    }
    if (a.track_nn) {
      P->off_nn[j] = (int32_t)off;
      off += 4 * SS;
      off = (off + 15) & ~size_t(15);
    }
    if (acc_has_idx(a.acc)) {
      P->off_idx[j] = (int32_t)off;
      off += 8 * idx_words(a.acc, generic) * SS;
    }
  }
  P->lds_log2 = log2;
  return off;
}

// LDS bytes a workgroup's table may take. The generic kernel runs two 512-thread workgroups per
// CU (80 KiB each). The specialised kernel's 1024-thread workgroups run one per CU, so its table
// may take nearly all of the CU's 160 KiB: twice the groups in one pass (C4 shape: up to ~2.5K
// groups in a 4096-slot table instead of ~1.3K in 2048 slots). QE_LDS_BUDGET_KB overrides.
static size_t lds_budget(const qe_ctx* ctx) {
  static const size_t env = [] {
    const char* e = getenv("QE_LDS_BUDGET_KB");
    return e && *e ? (size_t)std::max(16, std::min(156, atoi(e))) * 1024 : (size_t)0;
  }();
  if (env) return env;
  return (ctx->jit && fused_block(0) == 1024) ? (size_t)152 * 1024 : HA_LDS_BUDGET;
}

// Largest LDS table in [lds_log2_min, lds_log2] that fits the per-workgroup budget; 0 bytes =>
// global-only launch (the expected groups do not fit on chip).
static size_t lds_layout(const qe_hashagg* h, Plan* P) {
  if (h->lds_log2 == 0) return 0;
  const size_t budget = lds_budget(h->ctx);
  for (int log2 = h->lds_log2; log2 >= h->lds_log2_min; --log2) {
    const size_t b = lds_layout_at(h, P, log2);
    if (b <= budget) return b;
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
    if (acc_has_idx(h->acc[j])) b += 8 * idx_words(h->acc[j], !h->ctx->jit) * SS;
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

template <typename T>
static int grow_buffer(T** p, size_t* have, size_t need, qe_ctx* ctx, const char* what) {
  if (need <= *have) return QE_OK;
  dev_free(ctx, *p);
  *p = nullptr;
  *have = 0;
  if (dev_alloc(ctx, need, (void**)p) != QE_OK) return fail(QE_ERR_OOM, "%s: allocation of %zu bytes failed", what, need);
  *have = need;
  return QE_OK;
}

// Radix-partitioned update, steps 1-3 (qe_jit.hip, "radix-partitioned aggregation"): count the
// selected rows per (key-hash bucket, workgroup), scan, scatter one record per selected row into
// its bucket. On return P describes the aggregation pass over the records (P.n = records,
// P.part_tw = records per workgroup) and *fn / *grid its kernel.
// Narrow records (QE_PART_NARROW, default 1): integral record words are stored as 32 bits while
// every value of the update fits (sign-extended); the scatter flags ctl[7] otherwise, the
// aggregation pass then does nothing and run_update repeats the update with 64-bit words.
static bool part_narrow_env() {
  static const bool v = [] {
    const char* e = getenv("QE_PART_NARROW");
    return !(e && e[0] == '0');
  }();
  return v;
}

static int partition_rows(qe_hashagg* h, Plan& P, hipFunction_t* fn, int* grid) {
  qe_ctx* ctx = h->ctx;
  P.part_narrow = (!h->part_wide && part_narrow_env() && !part_soa()) ? 1 : 0;
  P.t = h->t;  // the scatter's fit flag (t.ctl[7])
  // aggregation-pass LDS table: the largest that fits the per-workgroup budget
  int tlog2 = 16;
  const size_t pbudget = pagg_block() == 1024 ? (size_t)152 * 1024 : HA_LDS_BUDGET;
  while (tlog2 >= 8 && lds_layout_at(h, &P, tlog2) > pbudget) --tlog2;
  QE_CHECK(tlog2 >= 8, QE_ERR_UNSUPPORTED, "aggregate state too wide for a partitioned LDS table");
  // buckets: about a quarter of the table's slots in groups per bucket while that takes <= 64
  // buckets, half the slots beyond (a slice spans <= 2 buckets; QE_PART_FILL_SHIFT = 1 / 2 fixes
  // half / a quarter). 1B rows, C4 shape, half-full against quarter-full tables: 65,536 groups
  // 13.66 vs 13.50 ms, 262,144 14.87 vs 15.78, 1,048,576 (512 staged buckets instead of 1024
  // direct) 19.1 vs 19.3, 4,194,304 20.9 vs 21.2, 16,777,216 27.6 vs 27.7.
  static const int fill_env = [] {
    const char* e = getenv("QE_PART_FILL_SHIFT");
    const int v = e && *e ? atoi(e) : 0;
    return v >= 1 && v <= 3 ? v : 0;
  }();
  auto buckets_log2 = [&](int shift) {
    int l = 1;
    while (l < 13 && (((int64_t)1 << tlog2) >> shift) * ((int64_t)1 << l) < h->expected_groups) ++l;
    return l;
  };
  int log2p = fill_env ? buckets_log2(fill_env) : buckets_log2(2);
  if (!fill_env && log2p > 6) log2p = buckets_log2(1);
  // QE_PART_FAST_FILL (percent): buckets for the fast aggregation pass's own (larger) table, each
  // bucket's expected groups at most that share of its slots (fewer buckets: longer scatter runs)
  static const int fast_fill = [] {
    const char* e = getenv("QE_PART_FAST_FILL");
    const int v = e && *e ? atoi(e) : 0;
    return v >= 10 && v <= 90 ? v : 0;
  }();
  if (!fill_env && fast_fill) {
    const int64_t fs = (int64_t)pagg_fast_slots(P) * fast_fill / 100;
    if (fs > 0) {
      int l = 1;
      while (l < 13 && fs * ((int64_t)1 << l) < h->expected_groups) ++l;
      log2p = l;
    }
  }
  std::string sc, ss, sa;
  size_t jl = 0;
  const bool staged = part_staged_ok(P, log2p);
  const int sblock = staged ? pscatter_block_for(log2p) : 512;
  const int64_t n = P.n;
  // count / scatter workgroups per CU (QE_PART_WG_PER_CU overrides; see pscatter_block)
  static const int wg_per_cu = [] {
    const char* e = getenv("QE_PART_WG_PER_CU");
    const int v = e && *e ? atoi(e) : 2;
    return v >= 1 && v <= 32 ? v : 2;
  }();
  // (one 1024-thread staged workgroup fits a CU)
  int64_t g = std::min<int64_t>((int64_t)ctx->num_cus * (sblock == 1024 ? 1 : wg_per_cu), (int64_t)div_up((uint64_t)n, 256));
  const PartLayout L = part_layout(P);
  const size_t rb = (size_t)L.bytes();
  if (L.narrow) QE_HIP(hipMemsetAsync(h->ctl + 7, 0, 8, ctx->stream));
  // Chunked scatter (staged buckets): no count pass and no read-back of the record count;
  // workgroups claim PART_CH-record chunks per bucket from a device counter. Record space: every
  // selected row in a full chunk plus one open chunk per (workgroup, bucket) — at most
  // n / PART_CH + g x buckets chunks — so it is taken while the open chunks' slots do not exceed
  // the batch's rows (large batches). QE_PART_CHUNKED (read per call): 0 never, 1 whenever the
  // scatter is staged, unset: by that rule.
  // (forced on a small batch, the scatter runs fewer workgroups so that the open chunks stay
  // within 4x the rows: tests exercise the chunked path at their sizes)
  const char* ce = getenv("QE_PART_CHUNKED");
  const int chunk_env = ce && *ce ? (ce[0] == '0' ? 0 : 1) : -1;
  const int64_t np_all = (int64_t)1 << log2p;
  if (chunk_env == 1 && staged && g * np_all * PART_CH > 4 * n)
    g = std::max<int64_t>(1, 4 * n / (np_all * PART_CH));
  const int64_t tw = (int64_t)div_up(div_up((uint64_t)n, (uint64_t)g), 256) * 256;
  g = (int64_t)div_up((uint64_t)n, (uint64_t)tw);
  const int64_t open_slots = g * np_all * PART_CH;
  // chunk ids: every claim of a device-wide counter, or each workgroup's own range (part_static)
  const int64_t cmax = std::max<int64_t>((int64_t)div_up((uint64_t)n, (uint64_t)PART_CH) + g * np_all + 1,
                                         g * ((int64_t)div_up((uint64_t)tw, (uint64_t)PART_CH) + np_all));
  const bool chunked = chunk_env != 0 && staged && np_all <= CHUNK_PLAN_MAXB &&
                       (chunk_env == 1 || open_slots <= n) && (uint64_t)cmax * PART_CH * rb <= (96ull << 30);
  QE_CHECK((chunked || gen_part_source(P, log2p, false, &sc)) &&
               (staged ? gen_pscatter_staged_source(P, log2p, &ss, chunked, chunked && part_soa())
                       : gen_part_source(P, log2p, true, &ss)) &&
               gen_pagg_source(P, tlog2, &sa, &jl, chunked, chunked && part_soa(),
                               (int64_t)(h->expected_groups >> log2p) + 1),
           QE_ERR_UNSUPPORTED, "plan shape not specialisable");
  hipFunction_t fc = nullptr, fs;
  int bpc = 0;
  if (!chunked) QE_TRY(jit_kernel(ctx, sc, &fc, &bpc, "qe_pcount"));
  QE_TRY(jit_kernel(ctx, ss, &fs, &bpc, "qe_pscatter", sblock));
  QE_TRY(jit_kernel(ctx, sa, fn, &bpc, "qe_pagg", pagg_block()));
  if (chunked) {
    const int64_t np = (int64_t)1 << log2p;
    // [0] chunks claimed | per chunk (bucket << 32 | records) | chunk ids by bucket (int32)
    // chunk table | sorted chunk ids | plan scratch: cnt u32[np], cur u32[np], base u32[np], rec u64[np]
    const size_t tbl = ((size_t)(1 + cmax) * 8 + (size_t)cmax * 4 + 7) & ~(size_t)7;
    QE_TRY(grow_buffer(&h->part_cnt, &h->part_cnt_bytes, tbl + (size_t)np * 20, ctx, "chunk table"));
    qi64* meta = (qi64*)h->part_cnt;
    qi32* sorted = (qi32*)(meta + 1 + cmax);
    unsigned long long* prec = (unsigned long long*)((uint8_t*)h->part_cnt + tbl);
    qu32* pcnt = (qu32*)(prec + np);
    qu32* pcur = pcnt + np;
    qu32* pbase = pcur + np;
    QE_TRY(grow_buffer(&h->part_rec, &h->part_rec_bytes, (size_t)cmax * PART_CH * rb, ctx, "partition records"));
    // aggregation slices: at most QE_PAGG_SLICES_PER_CU (default 8) per CU. One 1024-thread
    // workgroup runs per CU either way; more slices balance better, fewer flush less (each slice
    // of a bucket flushes every group it saw with device-scope atomics)
    static const int spc = [] {
      const char* e = getenv("QE_PAGG_SLICES_PER_CU");
      const int v = e && *e ? atoi(e) : 8;
      return v >= 1 && v <= 64 ? v : 8;
    }();
    const int64_t tmax = (int64_t)ctx->num_cus * spc;
    const int64_t max_slices = tmax + np;
    QE_TRY(grow_buffer(&h->part_slc, &h->part_slc_bytes, (size_t)(2 + 2 * max_slices) * 8, ctx, "partition slices"));
    if (!h->ovf || h->ovf_cap < (1ull << 20)) {
      uint8_t* ovf = nullptr;
      size_t have = 0;
      QE_TRY(grow_buffer(&ovf, &have, (size_t)(1ull << 20) * h->rec_bytes, ctx, "overflow area"));
      dev_free(ctx, h->ovf);
      h->ovf = ovf;
      h->ovf_cap = 1ull << 20;
    }
    QE_TRY(ensure_defer(h, cmax * PART_CH));  // the retry bitmaps index record slots
    P.ovf = h->ovf;
    P.ovf_cap = h->ovf_cap;
    QE_HIP(hipMemsetAsync(meta, 0, 8, ctx->stream));
    QE_HIP(hipMemsetAsync(prec, 0, (size_t)np * 16, ctx->stream));  // rec, cnt, cur
    P.part_tw = tw;
    P.part_rec = h->part_rec;
    P.part_chunk = meta;
    QE_TRY(jit_launch(ctx, fs, (int)g, P, sblock));
    QE_TRY(launch_check("qe_pscatter"));
    const unsigned pg = (unsigned)div_up((uint64_t)cmax, CHUNK_PER_WG);
    hipLaunchKernelGGL(k_chunk_hist, dim3(pg), dim3(256), 0, ctx->stream, (const qi64*)meta, (qi32)np, pcnt, prec);
    QE_TRY(launch_check("k_chunk_hist"));
    hipLaunchKernelGGL(k_chunk_slices, dim3(1), dim3(1024), 0, ctx->stream, (const qi64*)meta, (qi32)np, (qi64)tmax,
                       (const qu32*)pcnt, (const unsigned long long*)prec, (qi64*)h->part_slc, pbase);
    QE_TRY(launch_check("k_chunk_slices"));
    hipLaunchKernelGGL(k_chunk_place, dim3(pg), dim3(256), 0, ctx->stream, (const qi64*)meta, (qi32)np,
                       (const qu32*)pbase, pcur, sorted);
    QE_TRY(launch_check("k_chunk_place"));
    P.n = cmax * PART_CH;
    P.part_slice = (qi64*)h->part_slc;
    P.part_sorted = sorted;
    *grid = (int)max_slices;
    h->jit_note = "radix-partitioned: " + std::to_string(np) + " buckets, chunked records of " + std::to_string(rb) +
                  " B (" + (L.colmode ? "column" : "value") + (L.narrow ? " words, 32-bit" : " words") + "), staged scatter";
    return QE_OK;
  }
  const size_t cells = ((size_t)1 << log2p) * (size_t)g;
  QE_TRY(grow_buffer(&h->part_cnt, &h->part_cnt_bytes, (2 * cells + 1) * 8, ctx, "partition counts"));
  int64_t* cnt = h->part_cnt;
  int64_t* off = cnt + cells;
  P.part_tw = tw;
  P.part_off = (qi64*)cnt;
  QE_TRY(jit_launch(ctx, fc, (int)g, P));
  QE_TRY(launch_check("qe_pcount"));
  QE_TRY(exclusive_scan_i64(ctx, cnt, off, (int64_t)cells));
  void* pin;
  QE_TRY(ctx_pinned(ctx, 8, &pin));
  QE_HIP(hipMemcpyAsync(pin, off + cells, 8, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  const int64_t R = *(int64_t*)pin;
  // overflow records of the aggregation pass (bounded; groups beyond it retry their records)
  if (!h->ovf || h->ovf_cap < (1ull << 20)) {
    uint8_t* ovf = nullptr;
    size_t have = 0;
    QE_TRY(grow_buffer(&ovf, &have, (size_t)(1ull << 20) * h->rec_bytes, ctx, "overflow area"));
    dev_free(ctx, h->ovf);
    h->ovf = ovf;
    h->ovf_cap = 1ull << 20;
  }
  P.ovf = h->ovf;
  P.ovf_cap = h->ovf_cap;
  if (R > 0) {
    QE_TRY(grow_buffer(&h->part_rec, &h->part_rec_bytes, (size_t)R * rb, ctx, "partition records"));
    P.part_off = (qi64*)off;
    P.part_rec = h->part_rec;
    QE_TRY(jit_launch(ctx, fs, (int)g, P, sblock));
    QE_TRY(launch_check("qe_pscatter"));
  }
  // aggregation slices inside bucket boundaries: one per bucket, or more (up to 8 per CU, none
  // below ~32K records) when there are few buckets; cw is 5/4 of the even share, so a bucket of
  // about average size is one slice, whose workgroup then owns its groups outright (plain
  // combines, k_part_slices)
  const int64_t target = std::max<int64_t>((int64_t)1 << log2p, std::min<int64_t>((int64_t)ctx->num_cus * 8, R >> 15));
  const int64_t cw = std::max<int64_t>(256, (int64_t)div_up((uint64_t)std::max<int64_t>(R, 1) * 5, (uint64_t)target * 4));
  const int64_t max_slices = ((int64_t)1 << log2p) + (int64_t)div_up((uint64_t)std::max<int64_t>(R, 1), (uint64_t)cw);
  QE_TRY(grow_buffer(&h->part_slc, &h->part_slc_bytes, (size_t)(2 + 2 * max_slices) * 8, ctx, "partition slices"));
  hipLaunchKernelGGL(k_part_slices, dim3(1), dim3(1024), 0, ctx->stream, (const qi64*)off, (qi32)(1 << log2p), (qi64)g,
                     (qi64)cw, (qi64*)h->part_slc);
  QE_TRY(launch_check("k_part_slices"));
  P.n = R;
  P.part_tw = cw;
  P.part_rec = h->part_rec;
  P.part_slice = (qi64*)h->part_slc;
  *grid = (int)max_slices;
  h->jit_note = "radix-partitioned: " + std::to_string(1 << log2p) + " buckets, " + std::to_string(R) + " records of " +
                std::to_string(rb) + " B (" + (L.colmode ? "column" : "value") + (L.narrow ? " words, 32-bit)" : " words)") +
                (staged ? ", staged scatter" : "");
  return QE_OK;
}

// One launch of an update's aggregation kernel: pass 0 over the batch, pass > 0 over the rows
// deferred by the previous pass (defer_in). Control counters cleared as needed, the kernel
// chosen (plan-specialised when possible), events bracketing it (ev[0] of pass 0 / mp 0 is
// recorded by the caller, before any partitioning work).
static int launch_pass(qe_hashagg* h, Plan& P, size_t& lds, hipFunction_t pfn, int pgrid, int pass, int mp,
                       int out_i, const uint32_t* defer_in, int pblock = 0) {
  qe_ctx* ctx = h->ctx;
  const int64_t n = P.n;
  QE_CHECK(pass < 64, QE_ERR_CAPACITY, "hash aggregate did not converge after %d passes", pass);
  if (h->defer_dirty[out_i]) {
    QE_HIP(hipMemsetAsync(h->defer[out_i], 0, h->defer_words * 4, ctx->stream));
    h->defer_dirty[out_i] = false;
  }
  // deferred-row and overflow-record counters (ctl[3], lost groups, stays: only reset clears
  // it); known zero after a reset or after a launch that read back zeros
  if (!h->ctl_rows_clean) QE_HIP(hipMemsetAsync(h->ctl + 1, 0, 16, ctx->stream));
  h->ctl_rows_clean = false;
  // non-null counts: an aggregate whose input is nullable in this launch needs its real count;
  // the others stay implicit (the specialised kernels then skip their nn atomics; the generic and
  // partitioned kernels still add them, into an array nothing reads while the bit is set)
  int32_t tracked = 0;
  for (int j = 0; j < P.naggs; ++j)
    if (P.aggs[j].track_nn) tracked |= 1 << j;
  QE_TRY(nn_materialize(h, tracked));
  P.nn_skip = h->nn_implicit;
  P.t = h->t;
  P.defer_in = defer_in;
  P.defer_out = h->defer[out_i];
  const int64_t waves = (int64_t)div_up((uint64_t)n, 256);
  const int per_cu = lds ? std::max<int>(1, std::min<int>(8, (int)((160 * 1024) / lds))) : 8;
  const int64_t gcap = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, h->grid);
  int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)waves, HA_THREADS / 64), gcap);
  if (grid < 1) grid = 1;
  // specialised kernel for this plan shape when possible, else the generic interpreter
  hipFunction_t jfn = pfn;
  int jgrid = pgrid;
  if (pfn) {
    // records of the partitioned update
  } else if (lds && ctx->jit) {
    // kernel memoised on the plan's structure: source generation and the source-keyed module
    // lookup ran on every update
    static std::mutex memo_mu;
    static std::map<std::string, std::pair<hipFunction_t, int>> memo;
    const std::string key = plan_shape_key(ctx, P);
    int bpc = 0;
    bool have = false;
    {
      std::lock_guard<std::mutex> g(memo_mu);
      auto it = memo.find(key);
      if (it != memo.end()) {
        jfn = it->second.first;
        bpc = it->second.second;
        have = true;
      }
    }
    std::string src;
    size_t jl = 0;
    if (have || gen_fused_source(P, P.lds_log2, &src, &jl)) {
      if (have || jit_kernel(ctx, src, &jfn, &bpc, "qe_fused", fused_block(P.lds_log2)) == QE_OK) {
        if (!have) {
          std::lock_guard<std::mutex> g(memo_mu);
          memo[key] = {jfn, bpc};
        }
        static const int wg_env = [] {  // QE_FUSED_WG_PER_CU: workgroups per CU (default: the state's)
          const char* e = getenv("QE_FUSED_WG_PER_CU");
          return e && *e ? std::max(1, atoi(e)) : 0;
        }();
        const int64_t per_state = wg_env ? (int64_t)ctx->num_cus * wg_env
                                         : std::max<int64_t>(ctx->num_cus, h->grid * 512 / fused_block(P.lds_log2));
        jgrid = (int)std::min<int64_t>(std::min<int64_t>((int64_t)ctx->num_cus * bpc, per_state),
                                       (int64_t)div_up((uint64_t)waves, fused_block(P.lds_log2) / 64));
        if (jgrid < 1) jgrid = 1;
        h->jit_note.clear();
        if (P.lds_compact) h->jit_note = "compact LDS table: " + std::to_string(P.lds_compact) + " slots";
      } else {
        h->jit_note = qe_last_error();
        jfn = nullptr;
      }
    } else {
      h->jit_note = "plan shape not specialisable";
    }
  } else if (h->jit_note.rfind("partitioning unavailable", 0) != 0) {
    h->jit_note = lds ? "jit disabled" : "global-only launch";
  }
  bool own_layout = false;  // the specialised kernels' LDS layout differs from the generic kernel's
  for (int j = 0; j < h->naggs; ++j) own_layout = own_layout || h->acc[j] == ACC_SUM_X || P.aggs[j].share;
  if (!jfn && lds && (lds > HA_LDS_BUDGET || (own_layout && ctx->jit))) {
    // the 152 KiB budget is for the specialised 1024-thread kernel (one per CU); the generic
    // 512-thread kernel runs two per CU, so its table is re-laid out within HA_LDS_BUDGET (and with
    // the generic kernel's full exact-SUM slots)
    size_t b = 0;
    int log2 = P.lds_log2;
    while (log2 >= h->lds_log2_min && (b = lds_layout_at(h, &P, log2, true)) > HA_LDS_BUDGET) --log2;
    if (log2 < h->lds_log2_min || log2 < 8) {
      P.lds_log2 = 0;
      lds = 0;
    } else {
      lds = b;
    }
    const int pc = lds ? std::max<int>(1, std::min<int>(8, (int)((160 * 1024) / lds))) : 8;
    grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)div_up((uint64_t)waves, HA_THREADS / 64),
                                                       std::min<int64_t>((int64_t)ctx->num_cus * pc, h->grid)));
  }
  if (!jfn) {  // what the generic kernel got: its LDS table and how many of its workgroups share a CU
    const int pcu = lds ? std::max<int>(1, std::min<int>(2048 / HA_THREADS, (int)((160 * 1024) / lds))) : 2048 / HA_THREADS;
    h->jit_note += std::string(h->jit_note.empty() ? "" : "; ") + "generic kernel: " + std::to_string(lds / 1024) +
                   " KiB LDS table, " + std::to_string(pcu) + " workgroups per CU";
  }
  if (pass > 0 || mp > 0) QE_HIP(hipEventRecord(h->ev[0], ctx->stream));
  if (jfn) {
    QE_TRY(jit_launch(ctx, jfn, jgrid, P, pfn ? (pblock ? pblock : pagg_block()) : fused_block(P.lds_log2)));
  } else {
    QE_TRY(launch_hashagg(P, grid, lds, ctx->stream));
  }
  h->last_specialized = jfn ? 1 : 0;
  {  // what ran: the kernel's compile key and its launch shape (measurement hook)
    const uint64_t k = jfn ? jit_kernel_signature(jfn) : 0x6E65726963ull;  // "generic"
    const uint64_t shape = jfn ? ((uint64_t)jgrid << 20) ^ (uint64_t)(pfn ? (pblock ? pblock : pagg_block()) : fused_block(P.lds_log2))
                               : ((uint64_t)grid << 20) ^ (uint64_t)lds;
    h->last_sig = fmix64(k ^ fmix64(shape));
  }
  QE_TRY(launch_check("k_hashagg"));
  QE_HIP(hipEventRecord(h->ev[1], ctx->stream));
  // the counters' snapshot is queued right behind the launch: settling waits for this event only,
  // not for whatever the caller queued on the stream since (an exchange, the next query's work)
  QE_HIP(hipMemcpyAsync(h->ctl_pin, h->ctl, 64, hipMemcpyDeviceToHost, ctx->stream));
  QE_HIP(hipEventRecord(h->ev_ctl, ctx->stream));
  return QE_OK;
}

// After a launch: read the control counters back (synchronises), add the launch's time, and when
// rows were deferred or groups went to the overflow area, grow the table, re-apply the overflow
// records and set up the retry pass (*out_i / *defer_in). *done: nothing left to re-apply.
static int settle_pass(qe_hashagg* h, const Plan& P, int* out_i, const uint32_t** defer_in, bool* done) {
  uint64_t c[8];
  QE_HIP(hipEventSynchronize(h->ev_ctl));
  memcpy(c, h->ctl_pin, 64);
  QE_CHECK((c[3] & CTL_KEY_TOO_LONG) == 0, QE_ERR_INVALID_ARG,
           "a UTF8 group key is longer than its column's max_len promised (qe_column.max_len)");
  QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash aggregate lost %llu groups (probe limit or overflow area)",
           (unsigned long long)c[3]);
  {
    float ms = 0.f;
    QE_HIP(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->last_kernel_ms += ms;
    h->last_launches += 1;
  }
  QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash aggregate lost %llu groups (overflow area)", (unsigned long long)c[3]);
  h->narrow_failed = P.part_narrow && (c[7] & 1) != 0;
  if (P.lds_compact && (c[7] & 2)) h->compact_off = true;
  const uint64_t groups = c[0], deferred = c[1], ovf_recs = std::min<uint64_t>(c[2], P.ovf_cap);
  h->ctl_rows_clean = c[1] == 0 && c[2] == 0;
  *done = true;
  if (deferred == 0 && ovf_recs == 0) {
    if (groups * 2 > h->t.cap) QE_TRY(table_grow(h, 4 * h->t.cap));
    h->known_groups = (int64_t)groups;  // saves finalize a device round trip
    return QE_OK;
  }
  // grow, then re-apply what could not be inserted
  QE_TRY(table_grow(h, std::max<uint64_t>(4 * h->t.cap, 2 * (groups + ovf_recs))));
  if (ovf_recs) QE_TRY(import_records(h, h->ovf, (int64_t)ovf_recs));
  if (deferred == 0) return QE_OK;
  h->defer_dirty[*out_i] = true;
  *defer_in = h->defer[*out_i];
  *out_i ^= 1;
  *done = false;
  return QE_OK;
}

// Adaptive: once the groups seen exceed this launch's LDS table, most rows of later batches
// would take the global-table path; they go through the radix-partitioned update instead,
// sized for the groups seen so far.
static void adapt_after_update(qe_hashagg* h, size_t lds, int lds_log2) {
  if (h->known_groups > 0 && h->ctx->jit) {
    if (lds && h->known_groups * 5 / 4 > ((int64_t)1 << lds_log2)) h->lds_log2 = 0;
    if (h->lds_log2 == 0) h->expected_groups = std::max<int64_t>(h->expected_groups, h->known_groups);
  }
}

// Stream-ordered update (qe_hashagg_set_async): the pass-0 launch is queued and the read-back of
// its counters (with any growth / retry passes, which re-read the update's columns) is done by the
// next call on the state. Nothing pending: no-op.
static int settle_body(qe_hashagg* h) {
  Plan& P = *h->pend_plan;
  int out_i = h->pend_out_i;
  const uint32_t* defer_in = nullptr;
  for (int pass = 1;; ++pass) {
    bool done = false;
    QE_TRY(settle_pass(h, P, &out_i, &defer_in, &done));
    if (done) break;
    QE_TRY(launch_pass(h, P, h->pend_lds, nullptr, 0, pass, 0, out_i, defer_in));
  }
  adapt_after_update(h, h->pend_lds, P.lds_log2);
  return QE_OK;
}

static int settle_pending(qe_hashagg* h) {
  if (h->poisoned)
    return fail(h->poisoned, "an earlier stream-ordered update failed (%s); reset the state", h->poison_msg.c_str());
  if (!h->pending) return QE_OK;
  h->pending = false;
  const int st = settle_body(h);
  if (st != QE_OK) {  // the table is incomplete: keep failing, not just this once
    h->poisoned = st;
    h->poison_msg = qe_last_error();
  }
  return st;
}

// Kept share of the spilling pass in eighths of the kept table's slots (QE_SPILL_LOAD, 4..7, read
// per call; default 6).
static int spill_load8() {
  const char* le = getenv("QE_SPILL_LOAD");
  return le && *le ? std::max(4, std::min(7, atoi(le))) : 6;
}

// Two key-hash buckets (groups just beyond one LDS table; QE_MP_SPILL, read per call, 0 = two
// fused passes): pass 0 of the fused kernel keeps bucket 0 in its LDS tables and appends the other
// bucket's selected rows as partition records (part_layout, chunk-columnar) in per-wave chunks;
// k_spill_plan slices them (at most a slice per CU) and one chunked qe_pagg pass aggregates bucket 1. The columns are read once: C4 shape
// 24 B/row + 2 x 24 B per spilled record (~36 GB at 1B rows) instead of 48 B/row for two passes.
// *used = false: not applicable here (the caller runs the fused passes).
static int spill_update(qe_hashagg* h, Plan& P, size_t lds, int64_t rows, bool* used) {
  qe_ctx* ctx = h->ctx;
  *used = false;
  const char* e = getenv("QE_MP_SPILL");
  if ((e && e[0] == '0') || P.mp_n < 2) return QE_OK;
  const int SB = P.mp_n - 1;  // sub-buckets of the spilled share (a power of two, <= 8)
  if (SB > 8 || (SB & (SB - 1))) return QE_OK;
  P.part_narrow = (!h->part_wide && part_narrow_env()) ? 1 : 0;  // 32-bit record words while values fit
  P.t = h->t;
  const PartLayout L = part_layout(P);
  const size_t rb = (size_t)L.bytes();
  if ((uint64_t)rows * rb > (96ull << 30)) return QE_OK;
  Plan Q = P;
  Q.mp_n = 0;
  Q.mp_pass = 0;
  Q.lds_compact = 0;  // (the spilled records' pass keeps the regular table)
  int tlog2 = 16;
  const size_t pbudget = pagg_block() == 1024 ? (size_t)152 * 1024 : HA_LDS_BUDGET;
  while (tlog2 >= 8 && lds_layout_at(h, &Q, tlog2) > pbudget) --tlog2;
  if (tlog2 < 8) return QE_OK;
  std::string ss, sa;
  size_t jl = 0;
  // (the spilling pass writes whole records: the aggregation pass reads them record-major)
  if (!gen_fused_source(P, P.lds_log2, &ss, &jl, true) || !gen_pagg_source(Q, tlog2, &sa, &jl, true, false)) return QE_OK;
  hipFunction_t fs = nullptr, fa = nullptr;
  int bpc = 0, bpc_a = 0;
  const int sblock = fused_block(P.lds_log2);
  QE_TRY(jit_kernel(ctx, ss, &fs, &bpc, "qe_fused", sblock));
  QE_TRY(jit_kernel(ctx, sa, &fa, &bpc_a, "qe_pagg", pagg_block()));
  const int64_t waves = (int64_t)div_up((uint64_t)rows, 256);
  const int sgrid = (int)std::max<int64_t>(
      1, std::min<int64_t>((int64_t)ctx->num_cus * std::max(1, bpc), (int64_t)div_up((uint64_t)waves, sblock / 64)));
  // chunks: the full ones plus one open chunk per wave of the grid and sub-bucket
  const int64_t cmax = (int64_t)div_up((uint64_t)rows, (uint64_t)PART_CH) + (int64_t)sgrid * (sblock / 64) * SB + 1;
  QE_TRY(grow_buffer(&h->part_rec, &h->part_rec_bytes, (size_t)cmax * PART_CH * rb, ctx, "spill records"));
  // chunk table: meta (count, then bucket << 32 | fill per chunk), the chunk ids grouped by
  // sub-bucket, and (SB > 1) the planning counters: records (8 B), chunks, cursor, base per sub-bucket
  const size_t tbl = ((size_t)(1 + cmax) * 8 + (size_t)cmax * 4 + 7) & ~(size_t)7;
  QE_TRY(grow_buffer(&h->part_cnt, &h->part_cnt_bytes, tbl + (size_t)SB * 20, ctx, "chunk table"));
  qi64* meta = (qi64*)h->part_cnt;
  qi32* sorted = (qi32*)(meta + 1 + cmax);
  unsigned long long* prec = (unsigned long long*)((uint8_t*)h->part_cnt + tbl);
  qu32* pcnt = (qu32*)(prec + SB);
  qu32* pcur = pcnt + SB;
  qu32* pbase = pcur + SB;
  const int64_t tmax = ctx->num_cus;  // aggregation slices of the spilled share (+ one per sub-bucket)
  QE_TRY(grow_buffer(&h->part_slc, &h->part_slc_bytes, (size_t)(2 + 2 * (tmax + SB)) * 8, ctx, "spill slices"));
  QE_TRY(ensure_defer(h, cmax * PART_CH));  // the aggregation pass's retry bitmaps index record slots
  *used = true;
  QE_HIP(hipMemsetAsync(meta, 0, 8, ctx->stream));
  if (L.narrow) QE_HIP(hipMemsetAsync(h->ctl + 7, 0, 8, ctx->stream));
  // kept share: as many groups as one LDS table holds at a 6/8 load, the rest spilled (4096
  // expected groups of the C4 shape: 75 % kept, half the records of an even split; 1B rows, 4096 /
  // 5000 groups: 5/8 7.27 / 8.12 ms, 6/8 6.56 / 7.85, 7/8 6.62 / 10.79). The compact kept table
  // too since round 6's record-major spill (7,000 groups, 1B rows, spilling pass + aggregation
  // pass: 4/8 5.30 + 3.08 ms, 5/8 5.09 + 1.05, 6/8 4.94 + 0.61, 7/8 5.95 + 0.40)
  const int load8 = spill_load8();
  const int64_t kept_cap = P.lds_compact ? (int64_t)P.lds_compact : ((int64_t)1 << P.lds_log2);  // kept table's slots
  const double keep = std::min(1.0, (double)(kept_cap * load8 / 8) / (double)std::max<int64_t>(1, h->expected_groups));
  P.mp_keep = (qu64)(keep * 4294967296.0);
  P.part_rec = h->part_rec;
  P.part_chunk = meta;
  int out_i = 0;
  const uint32_t* defer_in = nullptr;
  // retry passes re-run the spill kernel over deferred rows only: those are bucket-0 rows, so
  // nothing is spilled twice
  bool misfit = false;
  for (int pass = 0;; ++pass) {
    QE_TRY(launch_pass(h, P, lds, fs, sgrid, pass, 0, out_i, defer_in, sblock));
    bool done = false;
    QE_TRY(settle_pass(h, P, &out_i, &defer_in, &done));
    misfit = misfit || h->narrow_failed;
    if (done) break;
  }
  if (misfit) {
    // a spilled value did not fit the 32-bit records: the kept rows are aggregated, the records
    // are not usable. The spilled rows (key hash >= mp_keep) go through one more fused pass over
    // the columns instead (mp_pass -1), and this state's records are 64-bit from now on.
    h->narrow_failed = false;
    h->part_wide = true;
    Plan R = P;
    R.part_narrow = 0;
    R.mp_pass = -1;
    h->defer_dirty[0] = h->defer_dirty[1] = true;
    out_i = 0;
    defer_in = nullptr;
    for (int pass = 0;; ++pass) {
      QE_TRY(launch_pass(h, R, lds, nullptr, 0, pass, 1, out_i, defer_in));
      bool done = false;
      QE_TRY(settle_pass(h, R, &out_i, &defer_in, &done));
      if (done) break;
    }
    h->jit_note = "multi-pass: 2 buckets, bucket 1 spilled, then re-read (a value outside the 32-bit records)";
    return QE_OK;
  }
  if (SB == 1) {
    hipLaunchKernelGGL(k_spill_plan, dim3((unsigned)div_up((uint64_t)cmax, 256)), dim3(256), 0, ctx->stream,
                       (const qi64*)meta, (qi64)tmax, (qi64*)h->part_slc, sorted);
    QE_TRY(launch_check("k_spill_plan"));
  } else {  // chunks grouped by sub-bucket and sliced, as after the radix scatter
    QE_HIP(hipMemsetAsync(prec, 0, (size_t)SB * 20, ctx->stream));
    const unsigned pg = (unsigned)div_up((uint64_t)cmax, CHUNK_PER_WG);
    hipLaunchKernelGGL(k_chunk_hist, dim3(pg), dim3(256), 0, ctx->stream, (const qi64*)meta, (qi32)SB, pcnt, prec);
    QE_TRY(launch_check("k_chunk_hist"));
    hipLaunchKernelGGL(k_chunk_slices, dim3(1), dim3(1024), 0, ctx->stream, (const qi64*)meta, (qi32)SB, (qi64)tmax,
                       (const qu32*)pcnt, (const unsigned long long*)prec, (qi64*)h->part_slc, pbase);
    QE_TRY(launch_check("k_chunk_slices"));
    hipLaunchKernelGGL(k_chunk_place, dim3(pg), dim3(256), 0, ctx->stream, (const qi64*)meta, (qi32)SB,
                       (const qu32*)pbase, pcur, sorted);
    QE_TRY(launch_check("k_chunk_place"));
  }
  Q.n = cmax * PART_CH;  // record slots (the retry bitmaps index them)
  Q.part_rec = h->part_rec;
  Q.part_chunk = meta;
  Q.part_sorted = sorted;
  Q.part_slice = (qi64*)h->part_slc;
  Q.ovf = h->ovf;
  Q.ovf_cap = h->ovf_cap;
  defer_in = nullptr;
  for (int pass = 0;; ++pass) {
    QE_TRY(launch_pass(h, Q, lds, fa, (int)(tmax + SB), pass, 1, out_i, defer_in));
    bool done = false;
    QE_TRY(settle_pass(h, Q, &out_i, &defer_in, &done));
    if (done) break;
  }
  h->jit_note = std::string("multi-pass: 2 buckets") + (P.lds_compact ? " (compact kept table)" : "") +
                ", bucket 1 spilled" + (SB > 1 ? " in " + std::to_string(SB) + " sub-buckets" : std::string()) + " as " +
                std::to_string(rb) + " B records (" + (L.colmode ? "column" : "value") + (L.narrow ? " words, 32-bit)" : " words)");
  return QE_OK;
}

static int run_update(qe_hashagg* h, Plan& P) {
  qe_ctx* ctx = h->ctx;
  QE_TRY(settle_pending(h));
  const int64_t rows = P.n;
  if (rows == 0) return QE_OK;
  size_t lds = lds_layout(h, &P);
  P.mp_n = 0;
  P.mp_pass = 0;
  P.ovf = h->ovf;
  P.ovf_cap = h->ovf_cap;
  QE_TRY(ensure_defer(h, rows));
  h->known_groups = -1;
  h->last_kernel_ms = 0.0;
  h->last_launches = 0;
  // groups beyond the LDS table: radix-partition the selected rows by key hash first, then
  // aggregate record slices in LDS (events bracket the whole sequence)
  hipFunction_t pfn = nullptr;
  int pgrid = 0;
  QE_HIP(hipEventRecord(h->ev[0], ctx->stream));
  // Groups just beyond one LDS table: 2 passes of the fused kernel, each keeping one bucket of
  // key hashes, read the columns twice but write and re-read no records. Measured at 200M rows
  // (C4 shape): 2048 groups 1.86 ms in 2 passes against ~3.1 ms radix-partitioned; 3 passes lose
  // their edge (3000 groups 2.88 ms, 3800 groups 3.44 ms against 3.09 ms partitioned).
  size_t lds_mp = 0;
  int mp_n = 0;
  // Groups just past the regular LDS table: one pass with the compact table (qe_jit.hip
  // compact_*, 32-bit keys, <= 92 % load) when the plan shape and the expected groups allow it
  // (QE_LDS_COMPACT=0: never; read per call), before key-hash passes / spilling.
  const char* ce = getenv("QE_LDS_COMPACT");
  if (!lds && ctx->jit && h->expected_groups > 0 && !h->compact_off && !(ce && ce[0] == '0') && compact_ok(P)) {
    Plan T = P;
    T.lds_log2 = 16;  // (unused by the compact kernel; keeps adapt_after_update from resizing)
    const size_t bps = compact_slot_bytes(T);
    const int64_t nsl = ((int64_t)((lds_budget(ctx) - 512) / bps) - 66) & ~(int64_t)63;  // (+2 special, 64 sinks)
    // expected groups at most QE_COMPACT_LOAD percent of the slots (default 98; 1B rows, one box,
    // 6336 slots: 5,900 / 6,000 / 6,150 / 6,250 groups 4.04 / 4.02–4.15 / 4.24 / 4.97 ms in one pass
    // at 93–99 %, against 5.45–5.71 ms for the spilling pass; round 5: 5,400 / 5,700 groups 3.76 /
    // 3.87 ms at 88–92 %)
    static const int cload = [] {
      const char* e = getenv("QE_COMPACT_LOAD");
      const int v = e && *e ? atoi(e) : 98;
      return v >= 50 && v <= 99 ? v : 98;
    }();
    if (nsl >= 512 && nsl * cload >= h->expected_groups * 100) {
      T.lds_compact = (qi32)nsl;
      std::string src;
      size_t jl = 0;
      hipFunction_t f = nullptr;
      int bpc = 0;
      if (gen_fused_source(T, T.lds_log2, &src, &jl) && jit_kernel(ctx, src, &f, &bpc, "qe_fused", fused_block(16)) == QE_OK) {
        const uint64_t need = (uint64_t)ctx->num_cus * 8 * ((uint64_t)nsl + 2);
        if (h->ovf_cap < need) {
          dev_free(ctx, h->ovf);
          h->ovf = nullptr;
          h->ovf_cap = 0;
          QE_TRY(dev_alloc(ctx, need * h->rec_bytes, (void**)&h->ovf));
          h->ovf_cap = need;
        }
        T.ovf = h->ovf;
        T.ovf_cap = h->ovf_cap;
        QE_HIP(hipMemsetAsync(h->ctl + 7, 0, 8, ctx->stream));
        P = T;
        lds = jl;
      }
    }
  }
  // Past the compact table (~5K groups for C4) and up to ~1.5 tables' worth: ONE spilling pass
  // whose kept share (key hashes below mp_keep, 6/8 of the compact table's slots) stays in the
  // compact table and whose other rows are written as records for one aggregation pass
  // (spill_update), instead of the 8-bucket partitioned path (QE_COMPACT_SPILL=0: off).
  if (!lds && ctx->jit && h->expected_groups > 0 && !h->compact_off && !(ce && ce[0] == '0') && compact_ok(P)) {
    static const bool cs_env = [] {
      const char* e = getenv("QE_COMPACT_SPILL");
      return !(e && e[0] == '0');
    }();
    Plan T = P;
    T.lds_log2 = 16;
    const size_t bps = compact_slot_bytes(T);
    const int64_t nsl = ((int64_t)((lds_budget(ctx) - 512 - 256) / bps) - 66) & ~(int64_t)63;  // (+ spill chunk state)
    // the spilled share goes through the regular aggregation table: at most half of it (1B rows:
    // 5,500 / 6,500 groups 5.95 / 6.59 ms against 8.23 / 8.25 partitioned; 8,192 groups, whose
    // ~3.4K spilled groups fill 84 % of a 4096-slot table, 11.0 against 8.1 ms)
    int tl = 16;
    {
      Plan Q = T;
      Q.lds_compact = 0;
      Q.mp_n = 0;
      const size_t pbudget = pagg_block() == 1024 ? (size_t)152 * 1024 : HA_LDS_BUDGET;
      while (tl >= 8 && lds_layout_at(h, &Q, tl) > pbudget) --tl;
    }
    // QE_SPILL_MAXPCT (default 70): the spilled groups (expected groups beyond the kept share)
    // may fill this percentage of each sub-bucket's aggregation table; 0 = round 4's rule (kept
    // share counted at 3/4, half the table). 1B rows, one box, C4 shape, record-major spill at a
    // 6/8 kept share: 7,500 groups 5.97 ms, 8,192 groups in one spilled bucket (84 % of its table)
    // 6.82 ms, against 7.63 ms partitioned at 8,192; two sub-buckets reach ~10.5K groups (11,500
    // groups at 85 %: 8.63 ms, past the partitioned update's ~8.0). Round 5 (chunk-columnar spill
    // at 7/8): 7.04 ms at 7,000 groups, 8.71 at 8,192, so 60 % stopped at ~7.9K groups
    static const int sp_pct = [] {
      const char* e = getenv("QE_SPILL_MAXPCT");
      const int v = e && *e ? atoi(e) : 70;
      return v >= 10 && v <= 90 ? v : 0;
    }();
    // the spilled share in SB sub-buckets (spill_hash's low bits), each aggregated by its own
    // slices: the fewest (1 or 2) whose aggregation tables stay within that percentage
    // (QE_SPILL_SUBBUCKETS: the most, 1, 2 or 4). 1B rows, one box: 8,192 groups 7.19 ms with
    // one spilled bucket, 7.07 with two (at 7,000 groups one: 6.24 against 6.55); 9,000 / 10,000
    // groups in two 7.28 / 7.66 ms, 12,000 / 16,000 in four 8.57 / 9.53, against 8.0–8.2 ms
    // partitioned on that box
    static const int sb_max = [] {
      const char* e = getenv("QE_SPILL_SUBBUCKETS");
      const int v = e && *e ? atoi(e) : 2;
      return v == 1 || v == 2 || v == 4 ? v : 2;
    }();
    const int64_t kept_share = nsl * spill_load8() / 8, per_sb = ((int64_t)1 << tl) * sp_pct / 100;
    int sb = 1;
    while (sp_pct && sb < sb_max && h->expected_groups - kept_share > sb * per_sb) sb *= 2;
    const int64_t spill_max = sp_pct ? kept_share + sb * per_sb : nsl * 3 / 4 + ((int64_t)1 << tl) / 2;
    if (cs_env && nsl >= 512 && tl >= 8 && h->expected_groups <= spill_max) {
      T.lds_compact = (qi32)nsl;
      T.mp_n = 1 + sb;
      T.mp_pass = 0;
      std::string src;
      size_t jl = 0;
      if (gen_fused_source(T, T.lds_log2, &src, &jl, true)) {
        const uint64_t need = (uint64_t)ctx->num_cus * 8 * ((uint64_t)nsl + 2);
        if (h->ovf_cap < need) {
          dev_free(ctx, h->ovf);
          h->ovf = nullptr;
          h->ovf_cap = 0;
          QE_TRY(dev_alloc(ctx, need * h->rec_bytes, (void**)&h->ovf));
          h->ovf_cap = need;
        }
        T.ovf = h->ovf;
        T.ovf_cap = h->ovf_cap;
        QE_HIP(hipMemsetAsync(h->ctl + 7, 0, 8, ctx->stream));
        bool used = false;
        QE_TRY(spill_update(h, T, jl, rows, &used));
        if (used) {
          h->row_base += rows;
          adapt_after_update(h, jl, T.lds_log2);
          return QE_OK;
        }
      }
    }
  }
  // Beyond the compact spill (~6.75K–10K groups for C4): two key-hash passes over the columns,
  // each keeping half the groups in the compact table (QE_COMPACT_TWOPASS=1, opt-in: 1B rows, one
  // box, 7,000 / 8,192 / 9,500 groups 8.02 / 8.17 / 9.09 ms against 7.78 / 7.81 / 7.96 ms for the
  // partitioned update — each pass's fuller compact table costs ~4 ms).
  bool no_spill = false;
  if (!lds && ctx->jit && h->expected_groups > 0 && !h->compact_off && !(ce && ce[0] == '0') && compact_ok(P)) {
    static const bool c2_env = [] {
      const char* e = getenv("QE_COMPACT_TWOPASS");
      return e && e[0] == '1';
    }();
    Plan T = P;
    T.lds_log2 = 16;
    const size_t bps = compact_slot_bytes(T);
    const int64_t nsl = ((int64_t)((lds_budget(ctx) - 512) / bps) - 66) & ~(int64_t)63;
    if (c2_env && nsl >= 512 && h->expected_groups <= nsl * 8 / 5) {
      T.lds_compact = (qi32)nsl;
      T.mp_n = 2;
      T.mp_pass = 0;
      std::string src;
      size_t jl = 0;
      hipFunction_t f = nullptr;
      int bpc = 0;
      if (gen_fused_source(T, T.lds_log2, &src, &jl) && jit_kernel(ctx, src, &f, &bpc, "qe_fused", fused_block(16)) == QE_OK) {
        const uint64_t need = (uint64_t)ctx->num_cus * 8 * ((uint64_t)nsl + 2);
        if (h->ovf_cap < need) {
          dev_free(ctx, h->ovf);
          h->ovf = nullptr;
          h->ovf_cap = 0;
          QE_TRY(dev_alloc(ctx, need * h->rec_bytes, (void**)&h->ovf));
          h->ovf_cap = need;
        }
        T.ovf = h->ovf;
        T.ovf_cap = h->ovf_cap;
        QE_HIP(hipMemsetAsync(h->ctl + 7, 0, 8, ctx->stream));
        P = T;
        lds = jl;
        mp_n = 2;
        no_spill = true;
      }
    }
  }
  // The generic kernel (JIT off, or no specialised kernel) passes too, with its own 80 KiB budget:
  // it has no partitioned path to fall back on, and global-only rows cost a device atomic each.
  if (!lds && h->expected_groups > 0) {
    int tlog2 = 16;
    Plan T = P;
    const size_t mbudget = ctx->jit ? lds_budget(ctx) : HA_LDS_BUDGET;
    while (tlog2 >= 8 && lds_layout_at(h, &T, tlog2) > mbudget) --tlog2;
    const int64_t per_pass = (((int64_t)1 << tlog2) * 5) / 8;
    const int64_t np = tlog2 >= 8 ? (h->expected_groups + per_pass - 1) / per_pass : 0;
    static const int64_t mp_max = [] {  // QE_MP_MAX: most bucket passes before partitioning
      const char* e = getenv("QE_MP_MAX");
      return (int64_t)(e && *e ? std::max(2, std::min(8, atoi(e))) : 2);
    }();
    if (np >= 2 && np <= (ctx->jit ? mp_max : 8)) {
      T.mp_n = (qi32)np;
      T.mp_pass = 0;
      lds_mp = lds_layout_at(h, &T, tlog2);
      std::string src;
      size_t jl = 0;
      // overflow records: a workgroup flushes at most its table's slots
      const uint64_t need = (uint64_t)ctx->num_cus * 8 * (((uint64_t)1 << tlog2) + 2);
      if (lds_mp && (!ctx->jit || gen_fused_source(T, T.lds_log2, &src, &jl))) {
        if (h->ovf_cap < need) {
          dev_free(ctx, h->ovf);
          h->ovf = nullptr;
          h->ovf_cap = 0;
          QE_TRY(dev_alloc(ctx, need * h->rec_bytes, (void**)&h->ovf));
          h->ovf_cap = need;
        }
        mp_n = (int)np;
        T.ovf = h->ovf;
        T.ovf_cap = h->ovf_cap;
        P = T;
        lds = lds_mp;
      }
    }
  }
  if (mp_n == 2 && ctx->jit && !no_spill) {
    bool used = false;
    QE_TRY(spill_update(h, P, lds, rows, &used));
    if (used) {
      h->row_base += rows;
      adapt_after_update(h, lds, P.lds_log2);
      return QE_OK;
    }
  }
  const Plan P_rows = P;  // the batch's plan, for a partitioned update repeated with 64-bit records
  for (;;) {
  if (!lds && mp_n == 0 && ctx->jit && h->expected_groups > 0) {
    Plan Q = P;
    if (partition_rows(h, Q, &pfn, &pgrid) == QE_OK) {
      P = Q;
      if (P.n == 0) {
        QE_HIP(hipEventRecord(h->ev[1], ctx->stream));
        QE_HIP(hipEventSynchronize(h->ev[1]));
        float ms = 0.f;
        QE_HIP(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
        h->last_kernel_ms = ms;
        h->last_launches = 1;
        h->last_specialized = 1;
        h->row_base += rows;
        return QE_OK;
      }
    } else {
      h->jit_note = std::string("partitioning unavailable: ") + qe_last_error();
      pfn = nullptr;
    }
  }
  int out_i = 0;
  for (int mp = 0; mp < std::max(1, mp_n); ++mp) {
    P.mp_pass = mp;
    const uint32_t* defer_in = nullptr;
    for (int pass = 0;; ++pass) {
      QE_TRY(launch_pass(h, P, lds, pfn, pgrid, pass, mp, out_i, defer_in));
      if (h->async && pass == 0 && mp_n == 0 && !pfn) {
        // one plain launch: its counters are read (and anything deferred re-applied) by the
        // next call on this state
        if (!h->pend_plan) h->pend_plan.reset(new Plan());
        *h->pend_plan = P;
        h->pend_lds = lds;
        h->pend_out_i = out_i;
        h->pending = true;
        h->row_base += rows;
        return QE_OK;
      }
      bool done = false;
      QE_TRY(settle_pass(h, P, &out_i, &defer_in, &done));
      if (done) break;
    }
  }
  if (pfn && h->narrow_failed) {
    // a value did not fit the 32-bit records (the aggregation pass left the table untouched):
    // this state's partitioned updates use 64-bit words from now on
    h->narrow_failed = false;
    h->part_wide = true;
    P = P_rows;
    pfn = nullptr;
    // the repeat is timed from here: the attempt just settled is already in last_kernel_ms once
    QE_HIP(hipEventRecord(h->ev[0], ctx->stream));
    continue;
  }
  break;
  }
  if (mp_n)
    h->jit_note = "multi-pass: " + std::to_string(mp_n) + " bucket passes" + (P.lds_compact ? " (compact table)" : "") +
                  (h->last_specialized ? "" : "; " + h->jit_note);
  h->row_base += rows;
  adapt_after_update(h, lds, P.lds_log2);
  return QE_OK;
}

}  // namespace qe

extern "C" {

int qe_hashagg_create(qe_ctx* ctx, int32_t nkeys, const int32_t* key_types, int32_t naggs, const qe_agg_desc* aggs,
                      int64_t expected_groups, qe_hashagg** out) {
  return qe_hashagg_create_ex(ctx, nkeys, key_types, naggs, aggs, expected_groups, 0, out);
}

int qe_hashagg_create_ex(qe_ctx* ctx, int32_t nkeys, const int32_t* key_types, int32_t naggs, const qe_agg_desc* aggs,
                         int64_t expected_groups, int32_t flags, qe_hashagg** out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK((flags & ~(QE_HASHAGG_DETERMINISTIC | QE_HASHAGG_FAST_FP64)) == 0, QE_ERR_INVALID_ARG, "unknown flags 0x%x",
           flags);
  QE_CHECK((flags & QE_HASHAGG_DETERMINISTIC) == 0 || (flags & QE_HASHAGG_FAST_FP64) == 0, QE_ERR_INVALID_ARG,
           "QE_HASHAGG_DETERMINISTIC and QE_HASHAGG_FAST_FP64 exclude each other");
  // fp64 SUM / AVG: exact (ACC_SUM_X) unless the caller opts into plain fp64 atomics
  const bool det = (flags & QE_HASHAGG_FAST_FP64) == 0;
  QE_CHECK(out, QE_ERR_INVALID_ARG, "null out");
  QE_CHECK(nkeys >= 0 && nkeys <= QE_MAX_KEYS, QE_ERR_UNSUPPORTED, "0..%d group keys supported", QE_MAX_KEYS);
  QE_CHECK(naggs >= 0 && naggs <= QE_MAX_AGGS, QE_ERR_UNSUPPORTED, "0..%d aggregates supported", QE_MAX_AGGS);
  QE_CHECK(nkeys == 0 || key_types, QE_ERR_INVALID_ARG, "null key_types");
  QE_CHECK(naggs == 0 || aggs, QE_ERR_INVALID_ARG, "null aggs");
  qe_hashagg* h = new qe_hashagg();
  h->ctx = ctx;
  h->naggs = naggs;
  h->flags = flags;
  auto bail = [&](int code) {
    for (hipEvent_t e : {h->ev[0], h->ev[1], h->ev_ctl})
      if (e) (void)hipEventDestroy(e);
    if (h->ctl_pin) pinned_slot_free(h->ctl_pin, h->ctx->stream);
    if (h->keyed) keyed_destroy(ctx, h->keyed);
    delete h;
    return code;
  };
  // the declared keys -> the device key columns the table groups by (UTF8 keys and key lists that
  // do not pack into one 64-bit word become dictionary codes, qe_keyed.hip)
  int32_t dev_types[QE_MAX_KEYS] = {};
  {
    int32_t dn = 0;
    const int st = keyed_create(ctx, nkeys, key_types, expected_groups > 0 ? expected_groups : 1024, &h->keyed, &dn,
                                dev_types);
    if (st != QE_OK) return bail(st);
    nkeys = dn;
    key_types = dev_types;
  }
  h->nkeys = nkeys;
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
    // integer inputs of any width accumulate as int64 (the column load sign-/zero-extends)
    const bool i = d.input_type == QE_TYPE_INT64 || d.input_type == QE_TYPE_INT32 ||
                   d.input_type == QE_TYPE_DATE32 || d.input_type == QE_TYPE_UINT8;
    if (d.fn != QE_AGG_COUNT_STAR && d.fn != QE_AGG_COUNT && !i && !f)
      return bail(fail(QE_ERR_UNSUPPORTED, "aggregate %d: input type %d (int64/int32/date32/uint8/fp64 only)", j,
                       d.input_type));
    switch (d.fn) {
      case QE_AGG_SUM: h->acc[j] = f ? (det ? ACC_SUM_X : ACC_SUM_F) : ACC_SUM_I; break;
      case QE_AGG_MIN: h->acc[j] = f ? ACC_MIN_F : ACC_MIN_I; break;
      case QE_AGG_MAX: h->acc[j] = f ? ACC_MAX_F : ACC_MAX_I; break;
      case QE_AGG_AVG: h->acc[j] = det ? ACC_SUM_X : ACC_SUM_F; break;
      case QE_AGG_COUNT:
      case QE_AGG_COUNT_STAR: h->acc[j] = ACC_NONE; break;
      default: return bail(fail(QE_ERR_UNSUPPORTED, "aggregate %d: unknown function %d", j, d.fn));
    }
    h->rec_bytes += agg_rec_bytes(h->acc[j]);
  }
  // control words
  if (hipEventCreate(&h->ev[0]) != hipSuccess || hipEventCreate(&h->ev[1]) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_ctl, hipEventDisableTiming) != hipSuccess)
    return bail(fail(QE_ERR_DEVICE, "hipEventCreate failed"));
  if (pinned_slot_alloc(&h->ctl_pin) != QE_OK) return bail(QE_ERR_OOM);
  if (dev_alloc(ctx, 64, (void**)&h->ctl) != QE_OK) return bail(fail(QE_ERR_OOM, "control allocation failed"));
  // (the control words are zeroed by the table's init launch below)
  // LDS table: 2x the expected groups (load factor <= 0.5); a launch may shrink it down to
  // 1.25x (lds_log2_min) to fit the per-workgroup budget, else the launch is global-only.
  const int64_t eg = expected_groups > 0 ? expected_groups : 1024;
  h->expected_groups = eg;
  h->create_groups = eg;
  int log2 = 8, log2_min = 8;
  while (log2 < 16 && ((int64_t)1 << log2) < 2 * eg) ++log2;
  while (log2_min < 16 && ((int64_t)1 << log2_min) < (5 * eg + 3) / 4) ++log2_min;
  const size_t budget = lds_budget(ctx);
  while (log2 > log2_min && lds_bytes_min(h, log2) > budget) --log2;
  h->lds_log2 = lds_bytes_min(h, log2) <= budget ? log2 : 0;
  h->lds_log2_min = log2_min;
  // workgroups per CU: as many as the smallest layout of the LDS table allows (max 8)
  const int per_cu = h->lds_log2 ? std::max<int>(1, std::min<int>(8, (int)((160 * 1024) / lds_bytes_min(h, h->lds_log2)))) : 8;
  h->grid = ctx->num_cus * per_cu;
  // overflow records: at most one per LDS slot per workgroup
  if (h->lds_log2) {
    h->ovf_cap = (uint64_t)h->grid * (((uint64_t)1 << h->lds_log2) + 2);
    if (dev_alloc(ctx, h->ovf_cap * h->rec_bytes, (void**)&h->ovf) != QE_OK) {
      dev_free(ctx, h->ctl);
      return bail(fail(QE_ERR_OOM, "overflow area allocation failed"));
    }
  }
  // global table: 2x expected groups
  const int st = table_alloc(h, std::max<uint64_t>(1024, next_pow2((uint64_t)(2 * eg))), &h->table_mem, &h->t, h->ctl);
  h->nn_implicit = all_nn_bits(h);
  if (st != QE_OK) {
    dev_free(ctx, h->ovf);
    dev_free(ctx, h->ctl);
    return bail(st);
  }
  h->ctl_rows_clean = true;  // (zeroed by the init launch)
  *out = h;
  return QE_OK;
}

int qe_hashagg_destroy(qe_hashagg* h) {
  if (!h) return QE_OK;
  (void)hipSetDevice(h->ctx->device);
  qe_ctx* ctx = h->ctx;  // blocks go back to the caching allocator behind this stream's work
  void* bufs[] = {h->table_mem, h->ctl, h->ovf, h->part_cnt, h->part_rec, h->part_slc, h->defer[0], h->defer[1]};
  for (void* b : bufs) dev_free(ctx, b);
  if (h->keyed) keyed_destroy(ctx, h->keyed);
  for (int i = 0; i < 2; ++i) {
    if (h->ev[i]) (void)hipEventDestroy(h->ev[i]);
  }
  if (h->ev_ctl) (void)hipEventDestroy(h->ev_ctl);
  pinned_slot_free(h->ctl_pin, ctx->stream);  // a queued snapshot copy may still target it
  delete h;
  return QE_OK;
}

int qe_hashagg_last_kernel_kind(qe_hashagg* h, int32_t* specialized, char* note, int32_t note_len) {
  QE_CHECK(h && specialized, QE_ERR_INVALID_ARG, "null argument");
  *specialized = h->last_specialized;
  if (note && note_len > 0) {
    strncpy(note, h->jit_note.c_str(), (size_t)note_len - 1);
    note[note_len - 1] = 0;
  }
  return QE_OK;
}

int qe_hashagg_last_kernel_signature(qe_hashagg* h, uint64_t* sig) {
  QE_CHECK(h && sig, QE_ERR_INVALID_ARG, "null argument");
  *sig = h->last_sig;
  return QE_OK;
}

int qe_hashagg_last_kernel_time(qe_hashagg* h, double* ms, int32_t* launches) {
  QE_CHECK(h && ms, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(h->ctx));
  QE_TRY(settle_pending(h));
  *ms = h->last_kernel_ms;
  if (launches) *launches = h->last_launches;
  return QE_OK;
}

int qe_hashagg_set_async(qe_hashagg* h, int32_t enable) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  QE_TRY(ctx_enter(h->ctx));
  if (!enable) QE_TRY(settle_pending(h));
  h->async = enable != 0;
  return QE_OK;
}

int qe_hashagg_reset(qe_hashagg* h) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  QE_TRY(ctx_enter(h->ctx));
  if (h->pending) {  // the table restarts: the pending launch's counters no longer matter
    h->pending = false;
    h->defer_dirty[h->pend_out_i] = true;
  }
  h->poisoned = 0;
  h->poison_msg.clear();
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 4096);
  hipLaunchKernelGGL(k_table_init, dim3(grid), dim3(256), 0, h->ctx->stream, h->t, agg_meta(h), (qu64*)h->ctl, 1);
  QE_TRY(launch_check("k_table_init"));
  h->nn_implicit = all_nn_bits(h);
  h->ctl_rows_clean = true;
  h->row_base = 0;
  h->known_groups = 0;
  ++h->version;
  return QE_OK;
}

int qe_hashagg_set_row_base(qe_hashagg* h, int64_t row_base) {
  QE_CHECK(h && row_base >= 0, QE_ERR_INVALID_ARG, "bad arguments");
  h->row_base = row_base;
  return QE_OK;
}

static_assert(sizeof(Plan) <= 4096, "kernel argument must stay under 4 KiB");

int qe_hashagg_update_fused(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec) {
  QE_CHECK(h && cols && spec, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(h->ctx));
  if (keyed_dict(h->keyed)) return keyed_update_fused(h, cols, ncols, spec);
  return hashagg_update_fused_raw(h, cols, ncols, spec);
}

int qe_hashagg_update(qe_hashagg* h, const qe_column* keys, const qe_column* agg_inputs, const qe_column* mask) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  QE_TRY(ctx_enter(h->ctx));
  QE_CHECK(h->nkeys == 0 || keys, QE_ERR_INVALID_ARG, "null keys");
  if (keyed_dict(h->keyed)) return keyed_update(h, keys, agg_inputs, mask);
  return hashagg_update_raw(h, keys, agg_inputs, mask);
}

}  // extern "C"

namespace qe {

int hashagg_update_fused_raw(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec) {
  Plan P;
  QE_TRY(compile_plan(h, cols, ncols, spec, &P));
  ++h->version;
  return run_update(h, P);
}

int hashagg_update_raw(qe_hashagg* h, const qe_column* keys, const qe_column* agg_inputs, const qe_column* mask) {
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
    // COUNT(*) only, no keys: the row count comes from a column passed as a COUNT(*) input
    // (its values are never read; a UTF-8 column is described by its int32 offsets).
    for (int j = 0; j < h->naggs && ncols == 0; ++j) {
      const qe_column& c = agg_inputs[j];
      if (h->aggs[j].fn != QE_AGG_COUNT_STAR || c.type == 0) continue;
      qe_column r = c;
      if (c.type == QE_TYPE_UTF8) {
        QE_CHECK(c.offsets || c.length == 0, QE_ERR_INVALID_ARG, "COUNT(*) row source: null offsets");
        r.type = QE_TYPE_INT32;
        r.values = c.offsets;
        r.offsets = nullptr;
      }
      int s;
      QE_TRY(slot_of(r, &s));
    }
    if (ncols == 0) return fail(QE_ERR_INVALID_ARG, "update needs at least one input column");
  }
  Plan P;
  QE_TRY(compile_plan(h, cols, ncols, &spec, &P));
  ++h->version;
  return run_update(h, P);
}

}  // namespace qe

extern "C" {

int qe_hashagg_num_groups(qe_hashagg* h, int64_t* out) {
  QE_CHECK(h && out, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(h->ctx));
  QE_TRY(settle_pending(h));
  if (h->known_groups >= 0) {
    *out = h->known_groups;
    return QE_OK;
  }
  uint64_t c[8];
  QE_TRY(read_ctl(h, c));
  QE_CHECK(c[3] == 0, QE_ERR_CAPACITY, "hash table lost %llu groups", (unsigned long long)c[3]);
  *out = h->known_groups = (int64_t)c[0];
  return QE_OK;
}

int qe_hashagg_finalize(qe_hashagg* h, qe_column* out_keys, qe_column* out_aggs, int64_t* out_groups) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  QE_TRY(ctx_enter(h->ctx));
  if (keyed_dict(h->keyed)) return keyed_finalize(h, out_keys, out_aggs, out_groups);
  return hashagg_finalize_raw(h, out_keys, out_aggs, out_groups, false);
}

}  // extern "C"

int qe::hashagg_finalize_raw(qe_hashagg* h, qe_column* out_keys, qe_column* out_aggs, int64_t* out_groups,
                             bool keys_only) {
  qe_ctx* ctx = h->ctx;
  int64_t groups;
  QE_TRY(qe_hashagg_num_groups(h, &groups));
  if (out_groups) *out_groups = groups;  // also on QE_ERR_CAPACITY: callers size the outputs from it
  // small tables finalise in one workgroup that also zeroes the validity bitmaps
  const bool small = h->t.cap + 2 <= (uint64_t)FS_THREADS * FS_PER && groups <= (int64_t)FS_WORDS * 32;
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
    if (c.validity && !small) QE_HIP(hipMemsetAsync(c.validity, 0, div_up((uint64_t)groups, 32) * 4, ctx->stream));
  }
  for (int j = 0; j < h->naggs && !keys_only; ++j) {
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
    if (c.validity && !small) QE_HIP(hipMemsetAsync(c.validity, 0, div_up((uint64_t)groups, 32) * 4, ctx->stream));
  }
  for (int k = 0; k < h->nkeys; ++k) out_keys[k].length = groups;
  for (int j = 0; j < h->naggs && !keys_only; ++j) out_aggs[j].length = groups;
  if (groups == 0) return QE_OK;
  if (small) {
    hipLaunchKernelGGL(k_finalize_small, dim3(1), dim3(FS_THREADS), 0, ctx->stream, h->t, agg_meta(h), h->km, oc,
                       (qi64)groups);
    QE_TRY(launch_check("k_finalize_small"));
    return QE_OK;  // stream-ordered: the outputs are ready when the ctx stream's work is
  }
  // one 256-slot tile per workgroup: a single pass each, so the chip finalises in one wave of
  // workgroups instead of a serial walk of long tiles
  const int32_t tile_slots = 256;
  const uint64_t SS = h->t.cap + 2;
  const int64_t ntiles = (int64_t)div_up(SS, tile_slots);
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)(2 * ntiles + 1) * 8, &s));
  int64_t* counts = (int64_t*)s;
  int64_t* offs = counts + ntiles;
  hipLaunchKernelGGL(k_occ_count, dim3((unsigned)ntiles), dim3(256), 0, ctx->stream, h->t, (qi64*)counts, tile_slots);
  QE_TRY(launch_check("k_occ_count"));
  QE_TRY(exclusive_scan_i64(ctx, counts, offs, ntiles));
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)ntiles), dim3(256), 0, ctx->stream, h->t, agg_meta(h), h->km, (const qi64*)offs,
                     tile_slots, oc);
  QE_TRY(launch_check("k_finalize"));
  return QE_OK;
}

namespace {
// The raw record calls carry the table's key word: meaningless to another state when it is a
// dictionary code (K:620-627 keys compare by content), so they refuse such states.
int refuse_dict_records(const qe_hashagg* h) {
  QE_CHECK(!keyed_dict(h->keyed), QE_ERR_UNSUPPORTED,
           "dictionary-keyed state (UTF8 / key-tuple codes are local to it): merge by key content with "
           "qe_hashagg_merge or qe_hashagg_export_keyed / qe_hashagg_import_keyed");
  return QE_OK;
}
}  // namespace

extern "C" {

int qe_hashagg_record_bytes(qe_hashagg* h, int64_t* out) {
  QE_CHECK(h && out, QE_ERR_INVALID_ARG, "null argument");
  *out = h->rec_bytes;
  return QE_OK;
}

int qe_hashagg_export_counts(qe_hashagg* h, int32_t nparts, int64_t* counts) {
  QE_CHECK(h && counts && nparts >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(refuse_dict_records(h));
  QE_TRY(ctx_enter(h->ctx));
  return hashagg_export_counts_raw(h, nparts, counts);
}

}  // extern "C"

// Records per partition of an export: one per group, FXE_CHUNKS more per group with E words.
int qe::hashagg_export_counts_raw(qe_hashagg* h, int32_t nparts, int64_t* counts) {
  QE_TRY(settle_pending(h));
  qe_ctx* ctx = h->ctx;
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)nparts * 8, &s));
  QE_HIP(hipMemsetAsync(s, 0, (size_t)nparts * 8, ctx->stream));
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 8192);
  hipLaunchKernelGGL(k_export_count, dim3(grid), dim3(256), 0, ctx->stream, h->t, agg_meta(h), nparts,
                     (unsigned long long*)s);
  QE_TRY(launch_check("k_export_count"));
  QE_HIP(hipMemcpyAsync(counts, s, (size_t)nparts * 8, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  return QE_OK;
}

extern "C" {

int qe_hashagg_export(qe_hashagg* h, int32_t nparts, void* dst) {
  QE_CHECK(h && nparts >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(refuse_dict_records(h));
  QE_TRY(ctx_enter(h->ctx));
  return hashagg_export_raw(h, nparts, dst);
}

}  // extern "C"

int qe::hashagg_export_raw(qe_hashagg* h, int32_t nparts, void* dst) {
  qe_ctx* ctx = h->ctx;
  int64_t groups;
  QE_TRY(qe_hashagg_num_groups(h, &groups));
  if (groups == 0) return QE_OK;
  QE_CHECK(dst, QE_ERR_INVALID_ARG, "null destination");
  // counts -> exclusive offsets (cursors) on the device: no host round trip
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)nparts * 8, &s));
  QE_HIP(hipMemsetAsync(s, 0, (size_t)nparts * 8, ctx->stream));
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 8192);
  hipLaunchKernelGGL(k_export_count, dim3(grid), dim3(256), 0, ctx->stream, h->t, agg_meta(h), nparts,
                     (unsigned long long*)s);
  QE_TRY(launch_check("k_export_count"));
  hipLaunchKernelGGL(k_counts_to_cursors, dim3(1), dim3(64), 0, ctx->stream, (unsigned long long*)s, nparts);
  QE_TRY(launch_check("k_counts_to_cursors"));
  hipLaunchKernelGGL(k_export, dim3(grid), dim3(256), 0, ctx->stream, h->t, agg_meta(h), nparts, h->rec_bytes,
                     (unsigned long long*)s, (uint8_t*)dst);
  QE_TRY(launch_check("k_export"));
  return QE_OK;
}

extern "C" {

int qe_hashagg_export_slots(qe_hashagg* h, int32_t nparts, int64_t slot_records, void* dst) {
  QE_CHECK(h && nparts >= 1 && slot_records >= 1 && dst, QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(refuse_dict_records(h));
  QE_TRY(ctx_enter(h->ctx));
  // a pending update is NOT settled here: the exchange queues behind it with no host round trip,
  // and the slot headers force the variable-size exchange if it left the table incomplete
  const bool speculative = h->pending;
  qe_ctx* ctx = h->ctx;
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)nparts * 8, &s));
  QE_HIP(hipMemsetAsync(s, 0, (size_t)nparts * 8, ctx->stream));
  const int grid = (int)std::min<uint64_t>(div_up(h->t.cap + 2, 256), 8192);
  hipLaunchKernelGGL(k_export_slots, dim3(grid), dim3(256), 0, ctx->stream, h->t, agg_meta(h), nparts, h->rec_bytes,
                     (qi64)slot_records, (unsigned long long*)s, (uint8_t*)dst);
  QE_TRY(launch_check("k_export_slots"));
  const uint64_t slot_bytes = QE_SLOT_HEADER + (uint64_t)slot_records * h->rec_bytes;
  hipLaunchKernelGGL(k_slot_headers, dim3(1), dim3(64), 0, ctx->stream, (const unsigned long long*)s, nparts,
                     (qu64)slot_bytes, (uint8_t*)dst, speculative ? (const qu64*)h->ctl : (const qu64*)nullptr);
  QE_TRY(launch_check("k_slot_headers"));
  return QE_OK;
}

int qe_hashagg_import_slots(qe_hashagg* h, const void* slots, int32_t nslots, int64_t slot_records,
                            int64_t* max_count, int64_t* nrecords) {
  QE_CHECK(h && slots && nslots >= 1 && slot_records >= 1 && max_count, QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(refuse_dict_records(h));
  QE_TRY(ctx_enter(h->ctx));
  QE_TRY(settle_pending(h));
  ++h->version;
  QE_TRY(nn_materialize(h, h->nn_implicit));  // records carry real non-null counts
  qe_ctx* ctx = h->ctx;
  // room for every record the slots can hold (duplicates counted: an upper bound) before the
  // launch, so the import needs no read-back of its own first; the one read-back after it gives
  // the verdict, the records and the group count (finalize then needs none)
  uint64_t groups_before;
  if (h->known_groups >= 0) {
    groups_before = (uint64_t)h->known_groups;
  } else {
    uint64_t c[8];
    QE_TRY(read_ctl(h, c));
    groups_before = c[0];
  }
  const uint64_t bound = groups_before + (uint64_t)nslots * (uint64_t)slot_records;
  if (2 * bound > h->t.cap) QE_TRY(table_grow(h, 2 * bound));
  h->known_groups = -1;
  const int grid = (int)std::min<uint64_t>(div_up((uint64_t)nslots * slot_records, 256), 8192);
  hipLaunchKernelGGL(k_import_slots, dim3(grid), dim3(256), 0, ctx->stream, (const uint8_t*)slots, nslots,
                     (qi64)slot_records, h->rec_bytes, h->t, agg_meta(h));
  QE_TRY(launch_check("k_import_slots"));
  uint64_t c[8];
  QE_TRY(read_ctl(h, c));
  *max_count = (int64_t)c[4];
  if (nrecords) *nrecords = (int64_t)c[5];
  h->known_groups = (int64_t)c[0];
  return QE_OK;
}

int qe_hashagg_import(qe_hashagg* h, const void* records, int64_t nrecords) {
  QE_CHECK(h && nrecords >= 0 && (records || nrecords == 0), QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(refuse_dict_records(h));
  QE_TRY(ctx_enter(h->ctx));
  return hashagg_import_raw(h, records, nrecords);
}

int qe_hashagg_key_layout(qe_hashagg* h, int32_t* dictionary_keyed, int32_t* device_nkeys, int32_t* device_types) {
  QE_CHECK(h, QE_ERR_INVALID_ARG, "null state");
  if (dictionary_keyed) *dictionary_keyed = !keyed_dict(h->keyed) ? 0 : keyed_tuple(h->keyed) ? 2 : 1;
  if (device_nkeys) *device_nkeys = h->nkeys;
  if (device_types)
    for (int k = 0; k < QE_MAX_KEYS; ++k) device_types[k] = k < h->nkeys ? h->key_types[k] : 0;
  return QE_OK;
}

}  // extern "C"

int qe::hashagg_import_raw(qe_hashagg* h, const void* records, int64_t nrecords) {
  QE_TRY(settle_pending(h));
  if (nrecords == 0) return QE_OK;
  ++h->version;
  QE_TRY(nn_materialize(h, h->nn_implicit));  // records carry real non-null counts
  h->known_groups = -1;
  uint64_t c[8];
  QE_TRY(read_ctl(h, c));
  if (2 * (c[0] + (uint64_t)nrecords) > h->t.cap) QE_TRY(table_grow(h, 2 * (c[0] + (uint64_t)nrecords)));
  return import_records(h, records, nrecords);
}
