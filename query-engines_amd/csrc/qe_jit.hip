// Per-plan kernel specialisation for the fused SelectionExec -> ProjectionExec ->
// HashAggregateExec pipeline (the north star's one-pass hot path).
//
// A query engine's expression interpreter costs instructions on every row; on MI355X the fused
// aggregate is otherwise HBM-bound, so the interpreter is what separates the generic kernel
// (k_hashagg, qe_hashagg.hip) from the HBM roofline. For each distinct plan SHAPE (column types
// and nullability, predicate structure, key packing, aggregate functions and expression trees,
// LDS table size) this file emits a straight-line HIP kernel in which every slot, operator and
// accumulator is a compile-time constant, compiles it once with hipRTC for the device's gfx950
// target, and caches the code object (in memory per device, and on disk by source hash). Literal
// VALUES stay runtime kernel arguments (Plan), so `a > 1` and `a > 2` share one kernel.
//
// The emitted code uses exactly the same table layout / probing / combine helpers as the
// ahead-of-time kernels (qe_dev.hpp is compiled into both), so results are identical; the AOT
// generic kernel remains the fallback when a plan cannot be specialised or hipRTC fails.
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <map>
#include <mutex>
#include <sstream>
#include <vector>

#include "qe_internal.hpp"

namespace qe {

static const char* kDevHeader =
#include "qe_dev.inc"
    ;

// ---- source generation -------------------------------------------------------------------------------
namespace {

struct Expr {
  std::string v;   // C expression (qi64 for integral, double for fp64)
  std::string ok;  // C expression of its validity (0/1)
  bool f;          // fp64
};

std::string col_raw(int c) { return "c" + std::to_string(c) + "[r]"; }
std::string col_ok(const Plan& P, int c) {
  return P.cols[c].valid ? "((v" + std::to_string(c) + " >> r) & 1u)" : std::string("1u");
}
bool col_is_f(const Plan& P, int c) { return P.cols[c].kind == K_F64; }
std::string col_val(const Plan& P, int c) {
  return col_is_f(P, c) ? "bits_f64(" + col_raw(c) + ")" : col_raw(c);
}

// Expression of aggregate j's typed token program (qe_hashagg.hip compile_plan) for row r.
bool agg_expr(const Plan& P, int j, Expr* out) {
  const DAgg& a = P.aggs[j];
  std::vector<Expr> st;
  for (int t = 0; t < a.ntok; ++t) {
    const DTok& k = a.tok[t];
    const std::string litref = "P.aggs[" + std::to_string(j) + "].tok[" + std::to_string(t) + "].lit";
    switch (k.op) {
      case T_COL: st.push_back({col_val(P, k.arg), col_ok(P, k.arg), col_is_f(P, k.arg)}); break;
      case T_LIT:
        st.push_back({k.lit_f64 ? "bits_f64(" + litref + ")" : litref, k.lit_null ? "0u" : "1u", k.lit_f64 != 0});
        break;
      case T_I2F0:
        if (st.empty()) return false;
        st.back() = {"((double)(" + st.back().v + "))", st.back().ok, true};
        break;
      case T_I2F1:
        if (st.size() < 2) return false;
        st[st.size() - 2] = {"((double)(" + st[st.size() - 2].v + "))", st[st.size() - 2].ok, true};
        break;
      default: {
        if (st.size() < 2) return false;
        const Expr b = st.back();
        st.pop_back();
        const Expr l = st.back();
        st.pop_back();
        Expr e;
        e.ok = "(" + l.ok + " & " + b.ok + ")";
        switch (k.op) {
          case T_ADD_I: e = {"((qi64)((qu64)(" + l.v + ") + (qu64)(" + b.v + ")))", e.ok, false}; break;
          case T_SUB_I: e = {"((qi64)((qu64)(" + l.v + ") - (qu64)(" + b.v + ")))", e.ok, false}; break;
          case T_MUL_I: e = {"((qi64)((qu64)(" + l.v + ") * (qu64)(" + b.v + ")))", e.ok, false}; break;
          case T_DIV_I:
            e = {"idiv((" + l.v + "), (" + b.v + "))", "(" + e.ok + " & (qu32)((" + b.v + ") != 0))", false};
            break;
          case T_ADD_F: e = {"((" + l.v + ") + (" + b.v + "))", e.ok, true}; break;
          case T_SUB_F: e = {"((" + l.v + ") - (" + b.v + "))", e.ok, true}; break;
          case T_MUL_F: e = {"((" + l.v + ") * (" + b.v + "))", e.ok, true}; break;
          case T_DIV_F: e = {"((" + l.v + ") / (" + b.v + "))", e.ok, true}; break;
          default: return false;
        }
        st.push_back(e);
      }
    }
  }
  if (st.size() != 1) return false;
  *out = st[0];
  if (out->f) out->v = "f64_bits(" + out->v + ")";
  return true;
}

const char* cmp_sym(int op) {
  switch (op) {
    case QE_OP_EQ: return "==";
    case QE_OP_NE: return "!=";
    case QE_OP_LT: return "<";
    case QE_OP_LE: return "<=";
    case QE_OP_GT: return ">";
    default: return ">=";
  }
}

std::string acc_init(int acc) {
  switch (acc) {
    case ACC_MIN_I:
    case ACC_MIN_F: return "0x7FFFFFFFFFFFFFFFll";
    case ACC_MAX_I:
    case ACC_MAX_F: return "EMPTY_KEY";
    default: return "0";
  }
}

// Load expression for once-read column streams: non-temporal by default (measured on the C4
// headline: 3.87 -> 3.62 ms, stream-read ceiling 6.08 -> 6.33 TB/s); QE_NT=0 restores the default
// cache policy.
bool use_nt() {
  const char* e = getenv("QE_NT");
  return !(e && e[0] == '0');
}
}  // namespace

// Fused aggregate kernel shape knobs (read once per process).
// QE_FUSED_PF=1: load step i+1's columns before step i's LDS work (software pipeline).
bool fused_prefetch() {
  static const bool v = [] {
    const char* e = getenv("QE_FUSED_PF");
    return e && e[0] == '1';
  }();
  return v;
}
// Workgroup size of the fused kernel (QE_FUSED_BLOCK = 256 / 512 / 1024 overrides; the LDS table
// size is an argument so that a shape-dependent rule can come back). 1024 threads: the same 16
// waves per CU as two 512-thread workgroups but ONE LDS table per CU, so the end-of-kernel flush
// into the global table does half the device-scope atomics. Interleaved A/B on one box each:
// C4 (2048-slot table) 3.556 (1024) vs 3.566 ms (512); C5 (16-slot table) 7.28-7.29 (1024) vs
// 7.55-7.58 ms (512), 1024 with 4 workgroups per CU 7.31 ms. (An earlier, non-interleaved pair
// had C5 the other way round and briefly made small tables use 512.)
int fused_block(int lds_log2) {
  (void)lds_log2;
  static const int env = [] {
    const char* e = getenv("QE_FUSED_BLOCK");
    const int b = e ? atoi(e) : 0;
    return (b == 256 || b == 512 || b == 1024) ? b : 0;
  }();
  return env ? env : 1024;
}

namespace {

std::string ld(const std::string& type, const std::string& ptr, bool nt = true) {
  if (nt && use_nt()) return "__builtin_nontemporal_load((const " + type + "*)(" + ptr + "))";
  return "(*(const " + type + "*)(" + ptr + "))";
}

// Mask column and predicate terms: clears bit r of `act` for rows r in [0, rows) that fail.
void emit_predicate(const Plan& P, std::ostringstream& o, int rows) {
  const std::string loop = "#pragma unroll\n    for (int r = 0; r < " + std::to_string(rows) + "; ++r) ";
  if (P.mask_col >= 0) {
    o << loop << "if (!((qu32)(" << col_raw(P.mask_col) << " & 1) & " << col_ok(P, P.mask_col)
      << ")) act &= ~(1u << r);\n";
  }
  for (int t = 0; t < P.nterms; ++t) {
    const DTerm& T = P.terms[t];
    const std::string lit = "P.terms[" + std::to_string(t) + "].lit";
    std::string lhs, rhs, ok = col_ok(P, T.lhs);
    if (T.f64) {
      lhs = col_is_f(P, T.lhs) ? col_val(P, T.lhs) : "((double)" + col_raw(T.lhs) + ")";
      if (T.rhs >= 0) rhs = col_is_f(P, T.rhs) ? col_val(P, T.rhs) : "((double)" + col_raw(T.rhs) + ")";
      else rhs = "bits_f64(" + lit + ")";
    } else {
      lhs = col_raw(T.lhs);
      rhs = T.rhs >= 0 ? col_raw(T.rhs) : lit;
    }
    if (T.rhs >= 0) ok += " & " + col_ok(P, T.rhs);
    else if (T.lit_null) ok = "0u";
    o << loop << "if (!((" << lhs << ") " << cmp_sym(T.op) << " (" << rhs << ")) || !(" << ok
      << ")) act &= ~(1u << r);\n";
  }
}

// Columns read by the predicate (mask + terms) and the group keys.
unsigned pred_key_cols(const Plan& P) {
  unsigned m = 0;
  if (P.mask_col >= 0) m |= 1u << P.mask_col;
  for (int t = 0; t < P.nterms; ++t) {
    m |= 1u << P.terms[t].lhs;
    if (P.terms[t].rhs >= 0) m |= 1u << P.terms[t].rhs;
  }
  if (P.key_mode != 0)
    for (int k = 0; k < P.nkeys; ++k) m |= 1u << P.key_col[k];
  return m;
}

// Column loads of one 256-row wave step (lane rows r0 + {0,1} and r0 + 128 + {0,1}) for the
// slots in `need`: c<slot>[4] values (sign-/zero-extended), v<slot> validity bits. `pre` names
// the destination arrays (the prefetching fused kernel loads the next step into p<slot>/pv<slot>);
// `declare` = false stores into arrays declared earlier.
void emit_col_loads(const Plan& P, std::ostringstream& o, unsigned need, const std::string& pre = "c",
                    bool declare = true) {
  const std::string vpre = pre == "c" ? "v" : "p" + std::string("v");
  for (int c = 0; c < P.ncols; ++c) {
    if (!((need >> c) & 1u)) continue;
    const std::string cs = std::to_string(c);
    const std::string dst = pre + cs;
    if (declare) o << "    qi64 " << dst << "[4];\n";
    const int kind = P.cols[c].kind;
    const char* ty = kind == K_I32 ? "qi32" : kind == K_U8 ? "qu8" : kind == K_BOOL ? "qu8" : "qi64";
    o << "    {\n      const " << ty << "* p = (const " << ty << "*)P.cols[" << cs << "].p;\n";
    if (kind == K_BOOL) {
      o << "      for (int r = 0; r < 4; ++r) { const qi64 row = r0 + 128 * (r >> 1) + (r & 1);\n"
        << "        " << dst << "[r] = (full || row < P.n) ? ((p[row >> 3] >> (row & 7)) & 1) : 0; }\n";
    } else {
      o << "      if (full) {\n";
      if (kind == K_I64 || kind == K_F64) {
        o << "        const qi64x2 a = " << ld("qi64x2", "p + r0") << ", b = " << ld("qi64x2", "p + r0 + 128") << ";\n"
          << "        " << dst << "[0] = a.x; " << dst << "[1] = a.y; " << dst << "[2] = b.x; " << dst << "[3] = b.y;\n";
      } else if (kind == K_I32) {
        o << "        const qi32x2 a = " << ld("qi32x2", "p + r0") << ", b = " << ld("qi32x2", "p + r0 + 128") << ";\n"
          << "        " << dst << "[0] = a.x; " << dst << "[1] = a.y; " << dst << "[2] = b.x; " << dst << "[3] = b.y;\n";
      } else {  // K_U8
        o << "        const qu16 a = " << ld("qu16", "p + r0") << ", b = " << ld("qu16", "p + r0 + 128") << ";\n"
          << "        " << dst << "[0] = a & 0xFF; " << dst << "[1] = a >> 8; " << dst << "[2] = b & 0xFF; " << dst
          << "[3] = b >> 8;\n";
      }
      o << "      } else {\n"
        << "        for (int r = 0; r < 4; ++r) { const qi64 row = r0 + 128 * (r >> 1) + (r & 1);\n"
        << "          " << dst << "[r] = row < P.n ? (qi64)p[row] : 0; }\n      }\n";
    }
    o << "    }\n";
    if (P.cols[c].valid) {
      if (declare) o << "    qu32 " << vpre << cs << ";\n";
      o << "    {\n      const qu8* vb = P.cols[" << cs << "].valid;\n"
        << "      const qu32 lo = (full || r0 < P.n) ? ((qu32)(vb[r0 >> 3] >> (r0 & 7)) & 3u) : 0u;\n"
        << "      const qu32 hi = (full || r0 + 128 < P.n) ? ((qu32)(vb[(r0 + 128) >> 3] >> (r0 & 7)) & 3u) : 0u;\n"
        << "      " << vpre << cs << " = lo | (hi << 2);\n    }\n";
    }
  }
}

// act: rows of this step inside [0, P.n), in the retry set (if any), passing mask and terms.
void emit_active_rows(const Plan& P, std::ostringstream& o, bool retry, bool skip_idle = true) {
  o << "    qu32 act = 15u;\n"
    << "    if (!full) { act = 0; for (int r = 0; r < 4; ++r) act |= (qu32)(r0 + 128 * (r >> 1) + (r & 1) < P.n) << r; }\n";
  if (retry)
    o << "    if (P.defer_in) {\n      for (int r = 0; r < 4; ++r) { const qi64 row = r0 + 128 * (r >> 1) + (r & 1);\n"
      << "        if (row < P.n && !((P.defer_in[row >> 5] >> (row & 31)) & 1)) act &= ~(1u << r); }\n    }\n";
  emit_predicate(P, o, 4);
  if (skip_idle) o << "    if (act == 0) continue;\n";
}

// key[4] (packed / canonical int64 group key) and knull (bit r: the key of row r is null).
void emit_keys(const Plan& P, std::ostringstream& o) {
  o << "    qi64 key[4] = {0, 0, 0, 0};\n    qu32 knull = 0;\n";
  if (P.key_mode == 1) {
    const int c = P.key_col[0];
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n      qi64 k = " << col_raw(c) << ";\n";
    if (P.key_f64) o << "      if (bits_f64(k) != bits_f64(k)) k = 0x7FF8000000000000ll;\n";
    if (P.cols[c].valid)
      o << "      if (!" << col_ok(P, c) << ") { k = 0; knull |= 1u << r; }\n";
    o << "      key[r] = k;\n    }\n";
  } else if (P.key_mode == 2) {
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n      qi64 k = 0;\n";
    for (int q = 0; q < P.nkeys; ++q) {
      const int c = P.key_col[q];
      o << "      { const bool isn = !" << col_ok(P, c) << "; k |= ((isn ? 0ll : (" << col_raw(c) << " & "
        << P.key_fmask[q] << "ll)) << " << P.key_shift[q] << ") | ((qi64)isn << " << P.key_nullbit[q] << "); }\n";
    }
    o << "      key[r] = k;\n    }\n";
  }
}

// Per-workgroup LDS table of 2^log2 (+2 special) slots: declarations and initialisation.
void emit_lds_table(const Plan& P, std::ostringstream& o, int log2, size_t* lds_bytes) {
  const int S = 1 << log2, SS = S + 2;
  o << "  constexpr int LOG2 = " << log2 << ", S = " << S << ", SS = " << SS << ";\n"
    << "  __shared__ qi64 s_keys[SS];\n  __shared__ qu32 s_cst[SS];\n";
  size_t lds = (size_t)SS * 12;
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.share) {  // the accumulator of aggregate share - 1 (same input, same kind)
      const int i = a.share - 1;
      if (a.acc != ACC_NONE) o << "  qi64* const s_acc" << j << " = s_acc" << i << ";\n";
      if (a.track_nn) o << "  qu32* const s_nn" << j << " = s_nn" << i << ";\n";
      if (acc_has_idx(a.acc)) o << "  qu64* const s_idx" << j << " = s_idx" << i << ";\n";
      continue;
    }
    if (a.acc != ACC_NONE) {
      o << "  __shared__ qi64 s_acc" << j << "[SS];\n";
      lds += 8 * SS;
    }
    if (a.track_nn) {
      o << "  __shared__ qu32 s_nn" << j << "[SS];\n";
      lds += 4 * SS;
    }
    if (acc_has_idx(a.acc)) {  // fp64 MIN / MAX: 4 row indices; exact SUM: window words 1..
      const int nw = a.acc == ACC_SUM_X ? fx_window_idx_words() : 4;
      o << "  __shared__ qu64 s_idx" << j << "[" << nw << " * SS];\n";
      lds += 8 * nw * SS;
    }
  }
  *lds_bytes = lds;
  o << "  for (int s = threadIdx.x; s < SS; s += blockDim.x) {\n    s_keys[s] = EMPTY_KEY;\n    s_cst[s] = 0;\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.share) continue;
    if (a.acc != ACC_NONE) o << "    s_acc" << j << "[s] = " << acc_init(a.acc) << ";\n";
    if (a.track_nn) o << "    s_nn" << j << "[s] = 0;\n";
    if (acc_has_idx(a.acc))
      o << "    for (int k = 0; k < " << (a.acc == ACC_SUM_X ? fx_window_idx_words() : 4) << "; ++k) s_idx" << j << "[k * SS + s] = "
        << (acc_is_f64mm(a.acc) ? "~0ull" : "0ull") << ";\n";
  }
  o << "  }\n  __syncthreads();\n";
}

// ---- exact fp64 SUM rows through a per-wave queue (fx queue) -----------------------------------------
// An exact fp64 SUM (ACC_SUM_X) costs a row about 30 VALU instructions and two LDS atomics that
// return (qe_dev.hpp fx_row / fx_add_row). Issued per row position of a step, a wave pays that for
// all 64 lanes however few rows passed the predicate (C5: ~12 %). Instead, every row bound for the
// LDS table appends (slot | input validity bits << 24, the SUM inputs) to its wave's ring of 128
// entries in LDS, and whenever 64 are queued the wave adds them with every lane busy. Only the
// SUM_X adds are queued; COUNT(*), non-null counts and the other aggregates stay direct. The
// kernel's step loop must then be convergent at the append points (no per-lane `continue`).
// Wave-private: a wave's LDS operations complete in order, so its lanes read what other lanes of
// the same wave wrote before (the fences keep the compiler from reordering them).
constexpr int FXQ_CAP = 128;

std::vector<int> fx_queue_aggs(const Plan& P) {
  std::vector<int> q;
  for (int j = 0; j < P.naggs; ++j)
    if (P.aggs[j].pkind != 0 && P.aggs[j].acc == ACC_SUM_X && !P.aggs[j].share) q.push_back(j);
  return q;
}

bool fx_queue_enabled() {
  static const bool v = [] {
    const char* e = getenv("QE_FX_QUEUE");
    return !(e && e[0] == '0');
  }();
  return v;
}

size_t fx_queue_bytes(const Plan& P, int block) {
  const size_t nq = fx_queue_aggs(P).size();
  return nq ? (size_t)(block / 64) * FXQ_CAP * (4 + 8 * nq) : 0;
}

void emit_fx_queue_decl(const Plan& P, std::ostringstream& o, int block) {
  const std::vector<int> q = fx_queue_aggs(P);
  o << "  __shared__ qu32 q_slot[" << (block / 64) * FXQ_CAP << "];\n";
  for (size_t k = 0; k < q.size(); ++k) o << "  __shared__ qi64 q_x" << k << "[" << (block / 64) * FXQ_CAP << "];\n";
  o << "  const qu32 q_base = (threadIdx.x >> 6) * " << FXQ_CAP << "u;\n  qu32 q_head = 0, q_n = 0;\n";
}

// Adds the `m` entries at the head of the wave's ring (m <= 64: one per lane). The window adds of all
// queued aggregates go out phase by phase (first words, then second words) so that their LDS round
// trips overlap; an input outside the window (fx_rare) goes to the group's global slot.
void emit_fx_queue_run(const Plan& P, std::ostringstream& o, const std::string& m) {
  const std::vector<int> q = fx_queue_aggs(P);
  const int nq = (int)q.size();
  o << "      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, \"wavefront\");\n"
    << "      if ((qu32)lane < " << m << ") {\n"
    << "        const qu32 qp = q_base + ((q_head + (qu32)lane) & " << FXQ_CAP - 1 << "u);\n"
    << "        const qu32 qe = q_slot[qp];\n        const int s = (int)(qe & 0xFFFFFFu);\n"
    << "        qi64 qx[" << nq << "];\n        qu32 rare = 0;\n";
  for (int k = 0; k < nq; ++k)
    o << "        qx[" << k << "] = ((qe >> " << 24 + k << ") & 1u) ? q_x" << k << "[qp] : 0ll;\n"
      << "        if (fx_rare(qx[" << k << "])) { rare |= 1u << " << k << "; qx[" << k << "] = 0; }\n";
  {
  o << "        qu64* wp0[" << nq << "];\n        qu64* wp1[" << nq << "];\n        qu64 lo[" << nq << "], hi[" << nq
    << "];\n        bool ng[" << nq << "], k0[" << nq << "];\n";
  for (int k = 0; k < nq; ++k) {
    const std::string j = std::to_string(q[k]), ks = std::to_string(k);
    o << "        {\n          const qu64 b = (qu64)qx[" << ks << "];\n          const int ex = (int)((b >> 52) & 0x7FF);\n"
      << "          const qu64 mm = ex ? ((b & ((1ull << 52) - 1)) | (1ull << 52)) : 0ull;\n"
      << "          const int p = ex ? ex - FXW_EX_LO : 0, kk = p >> 6, qq = p & 63;\n"
      << "          qu64 l = mm << qq, h = qq ? (mm >> (64 - qq)) : 0ull;\n"
      << "          ng[" << ks << "] = ex && (b >> 63);  // (-0.0 adds nothing, like +0.0)\n"
      << "          if (ng[" << ks << "]) { l = 0ull - l; h = ~h + (l == 0 ? 1ull : 0ull); }\n"
      << "          lo[" << ks << "] = l; hi[" << ks << "] = h; k0[" << ks << "] = kk == 0;\n"
      << "          wp0[" << ks << "] = kk ? &s_idx" << j << "[s] : (qu64*)&s_acc" << j << "[s];\n"
      << "          wp1[" << ks << "] = &s_idx" << j << "[kk * SS + s];\n        }\n";
  }
  o << "        qu64 o0[" << nq << "], t[" << nq << "], o1[" << nq << "];\n";
  for (int k = 0; k < nq; ++k) o << "        o0[" << k << "] = atomicAdd(wp0[" << k << "], lo[" << k << "]);\n";
  for (int k = 0; k < nq; ++k)
    o << "        t[" << k << "] = hi[" << k << "] + (o0[" << k << "] + lo[" << k << "] < o0[" << k << "] ? 1ull : 0ull);\n";
  for (int k = 0; k < nq; ++k) o << "        o1[" << k << "] = atomicAdd(wp1[" << k << "], t[" << k << "]);\n";
  for (int k = 0; k < nq; ++k) {
    const std::string j = std::to_string(q[k]), ks = std::to_string(k);
    o << "        if (k0[" << ks << "]) {\n          const qi64 d = (qi64)((t[" << ks << "] < hi[" << ks << "] ? 1 : 0) + (o1[" << ks
      << "] + t[" << ks << "] < o1[" << ks << "] ? 1 : 0)) - (ng[" << ks << "] ? 1 : 0);\n"
      << "          if (d) atomicAdd(&s_idx" << j << "[SS + s], (qu64)d);\n        }\n";
  }
  }
  o << "        if (rare) {\n          const bool knl = s == S;\n"
    << "          const qi64 key = knl ? 0 : (s == S + 1 ? EMPTY_KEY : s_keys[s]);\n";
  for (int k = 0; k < nq; ++k) {
    unsigned jm = 1u << q[k];  // and every aggregate sharing its accumulator (their own global sums)
    for (int j = 0; j < P.naggs; ++j)
      if (P.aggs[j].share == q[k] + 1) jm |= 1u << j;
    o << "          if ((rare >> " << k << ") & 1u) fx_rare_global(P, " << jm << "u, key, knl, q_x" << k << "[qp]);\n";
  }
  o << "        }\n      }\n      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, \"wavefront\");\n";
}

void emit_fx_queue_append(const Plan& P, std::ostringstream& o, const std::vector<std::string>& val,
                          const std::vector<std::string>& ok) {
  const std::vector<int> q = fx_queue_aggs(P);
  const int nq = (int)q.size();
  // the 4 rows' entries in registers first (constant row indices), then ONE rolled loop over the
  // rows appends them and drains full queues: an unrolled loop held 4 copies of the drain
  // (QE_FXQ_ROLL=0: unrolled)
  static const bool roll = [] {
    const char* e = getenv("QE_FXQ_ROLL");
    return !(e && e[0] == '0');
  }();
  o << "    {\n      qu32 qe4[4];\n";
  for (int k = 0; k < nq; ++k) o << "      qi64 qx4_" << k << "[4];\n";
  o << "#pragma unroll\n      for (int r = 0; r < 4; ++r) {\n        qu32 e = (qu32)slot[r];\n";
  for (int k = 0; k < nq; ++k)
    o << "        e |= (" << ok[q[k]] << " ? 1u : 0u) << " << 24 + k << ";\n        qx4_" << k << "[r] = " << val[q[k]] << ";\n";
  o << "        qe4[r] = e;\n      }\n"
    << "      const qu64 below = (1ull << lane) - 1;\n"
    << "#pragma unroll " << (roll ? 1 : 4) << "\n      for (int r = 0; r < 4; ++r) {\n"
    << "        const bool qa = (loc >> r) & 1;\n        const qu64 bq = __ballot(qa);\n"
    << "        if (qa) {\n"
    << "          const qu32 qp = q_base + ((q_head + q_n + (qu32)__popcll(bq & below)) & " << FXQ_CAP - 1 << "u);\n"
    << "          q_slot[qp] = r == 0 ? qe4[0] : r == 1 ? qe4[1] : r == 2 ? qe4[2] : qe4[3];\n";
  for (int k = 0; k < nq; ++k)
    o << "          q_x" << k << "[qp] = r == 0 ? qx4_" << k << "[0] : r == 1 ? qx4_" << k << "[1] : r == 2 ? qx4_" << k
      << "[2] : qx4_" << k << "[3];\n";
  o << "        }\n"
    << "        q_n += (qu32)__popcll(bq);\n"
    << "        if (q_n >= 64u) {\n";
  emit_fx_queue_run(P, o, "64u");
  o << "          q_head = (q_head + 64u) & " << FXQ_CAP - 1 << "u;\n          q_n -= 64u;\n        }\n      }\n    }\n";
}

// Aggregation of the 4 active rows of a step (act, key[4], knull) into the LDS table; rows whose
// group does not fit go to the global table, and rows the global table cannot take are deferred
// (bit `didx` of defer_out). val[j] / ok[j]: aggregate j's input value (int64 bits) and validity
// for row r; `row`: the row's global index (fp64 MIN/MAX order); all are C expressions of r.
void emit_agg_rows(const Plan& P, std::ostringstream& o, const std::vector<std::string>& val,
                   const std::vector<std::string>& ok, const std::string& row, const std::string& didx,
                   bool fx_queue = false, bool few_groups = false) {
  o << "    int slot[4];\n    qu32 h[4];\n    qi64 k0[4];\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) { h[r] = lds_hash((qu64)key[r]) >> (32 - LOG2); k0[r] = ((act >> r) & 1) ? s_keys[h[r]] : 0; }\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) slot[r] = ((knull >> r) & 1) ? S : (key[r] == EMPTY_KEY ? S + 1 : (k0[r] == key[r] ? (int)h[r] : -1));\n"
    << "    qu32 miss = 0;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) miss |= (qu32)(slot[r] < 0) << r;\n"
    << "    miss &= act;\n"
    << "    if (miss) {\n      for (int r = 0; r < 4; ++r) if ((miss >> r) & 1) slot[r] = lds_probe(s_keys, LOG2, key[r], h[r]);\n    }\n"
    << "    qu32 glob = 0;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) glob |= (qu32)(slot[r] < 0) << r;\n";
  // rows with an exact fp64 SUM input outside the LDS window: the global table's full accumulator
  // (with the fx queue the check happens when the queue is drained: fx_rare_global)
  bool any_x = false;
  for (int j = 0; j < P.naggs; ++j) any_x = any_x || (P.aggs[j].pkind != 0 && P.aggs[j].acc == ACC_SUM_X);
  if (any_x && !fx_queue) {
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n      bool rare = false;\n";
    for (int j = 0; j < P.naggs; ++j)
      if (P.aggs[j].pkind != 0 && P.aggs[j].acc == ACC_SUM_X)
        o << "      rare = rare || ((" << ok[j] << ") && fx_rare(" << val[j] << "));\n";
    o << "      glob |= (qu32)rare << r;\n    }\n";
  }
  o << "    glob &= act;\n    const qu32 loc = act & ~glob;\n";
  if (few_groups && !any_x)
    // A table of a few groups (the smallest, 256 slots): most lanes of a row position hit the same
    // few slots, and 64 lanes' atomics on one LDS word serialise. The lanes on the first active
    // lane's slot add their COUNT(*) as one atomic (tripdata, 3 groups; MIN / MAX read first).
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n      const bool lr = (loc >> r) & 1;\n"
      << "      const qu64 am = __ballot(lr);\n      if (am) {\n"
      << "        const int s0 = __builtin_amdgcn_readlane(slot[r], (int)__builtin_ctzll(am));\n"
      << "        const bool mine = lr && slot[r] == s0;\n        const qu64 m = __ballot(mine);\n"
      << "        if (mine) { if (lane == (int)__builtin_ctzll(m)) atomicAdd(&s_cst[s0], (qu32)__popcll(m)); }\n"
      << "        else if (lr) atomicAdd(&s_cst[slot[r]], 1u);\n      }\n    }\n";
  else
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) if ((loc >> r) & 1) atomicAdd(&s_cst[slot[r]], 1u);\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.pkind == 0 || a.share) continue;  // (a shared accumulator takes the row once)
    const std::string js = std::to_string(j);
    o << "    {\n#pragma unroll\n      for (int r = 0; r < 4; ++r) {\n"
      << "        if (!((loc >> r) & 1)) continue;\n"
      << "        if (!(" << ok[j] << ")) continue;\n"
      << "        const qi64 x = " << val[j] << ";\n"
      << "        const int s = slot[r];\n";
    if (a.track_nn) o << "        atomicAdd(&s_nn" << js << "[s], 1u);\n";
    switch (a.acc) {
      case ACC_SUM_I: o << "        atomicAdd((qu64*)&s_acc" << js << "[s], (qu64)x);\n"; break;
      case ACC_SUM_F: o << "        atomicAdd((double*)&s_acc" << js << "[s], bits_f64(x));\n"; break;
      case ACC_SUM_X:
        if (fx_queue) o << "        (void)x; (void)s;\n";
        else o << "        lds_fxw_add(s_acc" << js << ", s_idx" << js << ", SS, s, x);\n";
        break;
      case ACC_MIN_I: o << "        lds_min_rf(&s_acc" << js << "[s], x);\n"; break;
      case ACC_MAX_I: o << "        lds_max_rf(&s_acc" << js << "[s], x);\n"; break;
      case ACC_MIN_F:
      case ACC_MAX_F:
        o << "        lds_f64mm<" << (a.acc == ACC_MAX_F ? "true" : "false") << ">(s_acc" << js << ", s_idx" << js
          << ", SS, s, x, (qu64)(" << row << "));\n";
        break;
      default: break;
    }
    o << "      }\n    }\n";
  }
  // rows whose group only fits the global table (rare)
  o << "    if (glob) {\n      for (int r = 0; r < 4; ++r) {\n        if (!((glob >> r) & 1)) continue;\n"
    << "        const qi64 lr = " << didx << ";\n        qu64 gs;\n"
    << "        if (!gtable_find(P.t, key[r], (knull >> r) & 1, gs)) {\n"
    << "          atomicOr((qu32*)&P.defer_out[lr >> 5], 1u << (lr & 31));\n"
    << "          atomicAdd(&P.t.ctl[1], 1ull);\n          continue;\n        }\n"
    << "        gadd_cstar(P.t, gs, 1);\n        const qu64 row = (qu64)(" << row << ");\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.pkind == 0) continue;
    if (a.acc == ACC_SUM_X)  // (out of line: a rare path)
      o << "        if (" << ok[j] << ") gcombine_fx_row(P.t, " << j << ", gs, " << val[j] << ", "
        << (((P.nn_skip >> j) & 1) ? "false" : "true") << ");\n";
    else
      o << "        if (" << ok[j] << ") { const RowVal rv = row_partial(" << a.acc << ", " << val[j]
        << ", row); gcombine(P.t, " << a.acc << ", " << j << ", gs, rv.acc, 1, rv.i0, rv.i1, rv.i2, rv.i3, "
        << (((P.nn_skip >> j) & 1) ? "false" : "true") << "); }\n";
  }
  o << "      }\n    }\n";
  if (fx_queue) emit_fx_queue_append(P, o, val, ok);
}

// Merge the workgroup's LDS table into the global table (or the overflow records). With
// `mark_full`, a group that finds neither a global slot nor overflow space is flagged in s_cst
// (bit 31) and s_fail is set: the caller then defers that group's records for a retry pass.
//
// `part` (partition aggregate): new groups are counted in the LDS word s_newg, and when the runtime
// flag `excl` says this workgroup holds every record of its groups, the combines are plain
// read-modify-writes (gadd_cstar_excl / gcombine_excl).
void emit_flush(const Plan& P, std::ostringstream& o, bool mark_full = false, bool part = false) {
  // new groups: counted in the workgroup's LDS word s_newg (the caller adds it to ctl[0] once)
  o << "  __syncthreads();\n"
    << "  for (int s = threadIdx.x; s < SS; s += blockDim.x) {\n"
    << "    const qu32 c = s_cst[s];\n    if (c == 0) continue;\n"
    << "    const bool knl = s == S;\n    const qi64 key = knl ? 0 : (s == S + 1 ? EMPTY_KEY : s_keys[s]);\n"
    << "    qu64 gs;\n"
    << "    const bool ok = gtable_find_wg(P.t, key, knl, gs, &s_newg);\n"
    << "    qu8* rec = nullptr;\n"
    << (part ? "    if (ok) {\n      if (excl) gadd_cstar_excl(P.t, gs, c, &s_newg); else gadd_cstar(P.t, gs, c);\n    } else {\n"
             : "    if (ok) {\n      gadd_cstar(P.t, gs, c);\n    } else {\n")
    << "      const qu64 ri = atomicAdd(&P.t.ctl[2], 1ull);\n";
  if (mark_full)
    o << "      if (ri >= P.ovf_cap) { s_cst[s] = c | 0x80000000u; s_fail = 1; continue; }\n";
  else
    o << "      if (ri >= P.ovf_cap) { atomicAdd(&P.t.ctl[3], 1ull); continue; }\n";
  o << "      rec = P.ovf + ri * (qu64)P.rec_bytes;\n      write_record_head(rec, key, knl, c);\n    }\n";
  int off = 24;
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    const std::string js = std::to_string(j);
    o << "    {\n      qi64 acc = " << (a.acc != ACC_NONE ? "s_acc" + js + "[s]" : std::string("0")) << ";\n"
      << "      const qu64 nn = " << (a.track_nn ? "s_nn" + js + "[s]" : std::string("c")) << ";\n";
    if (a.acc == ACC_SUM_X)  // the LDS window as a global partial (status 0: rare rows went global)
      o << "      qu64 i0, i1, i2;\n      const qu64 i3 = 0;\n      {\n        qu64 v[4];\n        fxw_words((qu64)acc, s_idx" << js
        << "[s], s_idx" << js << "[SS + s], v);\n        acc = (qi64)v[0]; i0 = v[1]; i1 = v[2]; i2 = v[3];\n      }\n";
    else if (acc_has_idx(a.acc))
      o << "      qu64 i0 = s_idx" << js << "[s], i1 = s_idx" << js << "[SS + s], i2 = s_idx" << js
        << "[2 * SS + s], i3 = s_idx" << js << "[3 * SS + s];\n";
    else
      o << "      const qu64 i0 = ~0ull, i1 = ~0ull, i2 = ~0ull, i3 = ~0ull;\n";
    const bool skip_nn = (P.nn_skip >> j) & 1;
    const char* add_nn = skip_nn ? "false" : "true";
    const char* words = a.acc == ACC_SUM_X ? "<true>" : "";  // (an exact SUM's window: words, never E)
    if (a.fn != QE_AGG_COUNT_STAR && part)
      o << "      if (ok) { if (excl) gcombine_excl" << words << "(P.t, " << a.acc << ", " << j << ", gs, acc, nn, i0, i1, i2, i3);"
        << " else gcombine" << words << "(P.t, " << a.acc << ", " << j << ", gs, acc, nn, i0, i1, i2, i3, " << add_nn << "); }\n";
    else if (a.fn != QE_AGG_COUNT_STAR && !(a.acc == ACC_NONE && skip_nn))  // implicit COUNT(x): nothing to add
      o << "      if (ok) gcombine" << words << "(P.t, " << a.acc << ", " << j << ", gs, acc, nn, i0, i1, i2, i3, " << add_nn << ");\n";
    o << "      if (!ok) { qu64* f = (qu64*)(rec + " << off << "); f[0] = (qu64)acc; f[1] = nn;";
    if (acc_has_idx(a.acc)) o << " f[2] = i0; f[3] = i1; f[4] = i2; f[5] = i3;";
    o << " }\n    }\n";
    off += agg_rec_bytes(a.acc);
  }
  o << "  }\n";
}

// ---- compact LDS table of the fused aggregate (Plan.lds_compact slots) --------------------------------
// Groups just past the regular table (~2.5K for the C4 shape) used to take two key-hash passes or
// a spilling pass. A slot of 32-bit key + COUNT(*) + per aggregate a 64-bit SUM or a 32-bit MIN /
// MAX (bare column inputs) is 24 B for C4 instead of 36, so one 152 KiB table holds ~6.2K slots:
// up to ~5.8K groups in one pass at <= 92 % load. The slot count is any number (multiply-shift
// slot hash). Speculative like the 32-bit records: a row whose key or 32-bit accumulator input
// does not fit 32 bits goes to the global table directly (correct, slow) and sets ctl[7] bit 1,
// after which the state no longer uses the compact table.
namespace {

void emit_lds_table_c(const Plan& P, std::ostringstream& o, size_t* lds_bytes) {
  const int NSL = P.lds_compact;
  o << "  constexpr qu32 NSL = " << NSL << ", NBK = NSL / 4;\n  constexpr int S = " << NSL << ", SS = " << NSL + 2 << ", SINK = SS;\n"
    << "  __shared__ __attribute__((aligned(16))) qi32 s_keys[SS + 64];\n  __shared__ qu32 s_cst[SS + 64];\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.acc != ACC_NONE) o << "  __shared__ " << (compact_acc32(P, j) ? "qi32" : "qi64") << " s_acc" << j << "[SS + 64];\n";
    if (a.track_nn) o << "  __shared__ qu32 s_nn" << j << "[SS + 64];\n";
  }
  *lds_bytes = (size_t)(NSL + 66) * compact_slot_bytes(P);
  o << "  for (int s = threadIdx.x; s < SS + 64; s += blockDim.x) {\n    s_keys[s] = EMPTY_KEY32;\n    s_cst[s] = 0;\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.acc != ACC_NONE)
      o << "    s_acc" << j << "[s] = "
        << (compact_acc32(P, j) ? (a.acc == ACC_MIN_I ? std::string("0x7FFFFFFF") : std::string("(qi32)0x80000000u"))
                                : acc_init(a.acc))
        << ";\n";
    if (a.track_nn) o << "    s_nn" << j << "[s] = 0;\n";
  }
  o << "  }\n  __syncthreads();\n";
}

void emit_agg_rows_c(const Plan& P, std::ostringstream& o, const std::vector<std::string>& val,
                     const std::vector<std::string>& ok, const std::string& row, const std::string& didx) {
  // rows whose key and 32-bit accumulator inputs fit 32 bits
  o << "    qu32 fit = 0;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n      bool f = key[r] == (qi64)(qi32)key[r];\n";
  for (int j = 0; j < P.naggs; ++j)
    if (P.aggs[j].pkind != 0 && compact_acc32(P, j))
      o << "      { const qi64 x = " << val[j] << "; f = f && (!(" << ok[j] << ") || x == (qi64)(qi32)x); }\n";
  o << "      fit |= (qu32)f << r;\n    }\n"
    << "    if (act & ~fit) atomicOr(&P.t.ctl[7], 2ull);\n"
    << "    int slot[4];\n    qu32 h[4];\n    qu32x4 q[4];\n"
    << "    qu32 h2[4];\n    qu32x4 q2[4];\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
    << "      h[r] = (qu32)(((qu64)lds_hash((qu64)key[r]) * NBK) >> 32); h2[r] = h[r] + 1 == NBK ? 0u : h[r] + 1;\n"
    << "      q[r] = ((const qu32x4*)s_keys)[h[r]]; q2[r] = ((const qu32x4*)s_keys)[h2[r]];\n    }\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
    << "      const qu32 kk = (qu32)key[r];\n"
    << "      const int hs = bucket2_hit(q[r], q2[r], kk, h[r], h2[r]);\n"
    << "      slot[r] = ((knull >> r) & 1) ? S : ((qi32)kk == EMPTY_KEY32 ? S + 1 : hs);\n"
    << "    }\n"
    << "    qu32 miss = 0;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) miss |= (qu32)(slot[r] < 0) << r;\n"
    << "    miss &= act & fit;\n"
    << "    if (miss) {\n      int t0 = slot[0], t1 = slot[1], t2 = slot[2], t3 = slot[3];\n"
    << "      lds_probe4_rows(s_keys, NBK, miss, (qi32)key[0], (qi32)key[1], (qi32)key[2], (qi32)key[3], h[0], h[1], h[2], h[3], t0, t1, t2, t3);\n"
    << "      slot[0] = t0; slot[1] = t1; slot[2] = t2; slot[3] = t3;\n    }\n"
    << "    qu32 glob = ~fit;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) glob |= (qu32)(slot[r] < 0) << r;\n"
    << "    glob &= act;\n    const qu32 loc = act & ~glob;\n"
    << "    int sl[4];\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) sl[r] = ((loc >> r) & 1) ? slot[r] : SINK + lane;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) atomicAdd(&s_cst[sl[r]], 1u);\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.pkind == 0) continue;
    const std::string js = std::to_string(j);
    const bool a32 = compact_acc32(P, j);
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
      << "      const int s = (" << ok[j] << ") ? sl[r] : SINK + lane;\n"
      << "      const qi64 x = " << val[j] << ";\n";
    if (a.track_nn) o << "      atomicAdd(&s_nn" << js << "[s], 1u);\n";
    switch (a.acc) {
      case ACC_SUM_I: o << "      atomicAdd((qu64*)&s_acc" << js << "[s], (qu64)x);\n"; break;
      case ACC_MIN_I: o << "      lds_min_rf(&s_acc" << js << "[s], " << (a32 ? "(qi32)x" : "x") << ");\n"; break;
      case ACC_MAX_I: o << "      lds_max_rf(&s_acc" << js << "[s], " << (a32 ? "(qi32)x" : "x") << ");\n"; break;
      default: break;
    }
    o << "    }\n";
  }
  // rows for the global table: no room in LDS, or a value that does not fit the compact slots
  o << "    if (glob) {\n      for (int r = 0; r < 4; ++r) {\n        if (!((glob >> r) & 1)) continue;\n"
    << "        const qi64 lr = " << didx << ";\n        qu64 gs;\n"
    << "        if (!gtable_find(P.t, key[r], (knull >> r) & 1, gs)) {\n"
    << "          atomicOr((qu32*)&P.defer_out[lr >> 5], 1u << (lr & 31));\n"
    << "          atomicAdd(&P.t.ctl[1], 1ull);\n          continue;\n        }\n"
    << "        gadd_cstar(P.t, gs, 1);\n        const qu64 row = (qu64)(" << row << ");\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.pkind == 0) continue;
    o << "        if (" << ok[j] << ") { const RowVal rv = row_partial(" << a.acc << ", " << val[j]
      << ", row); gcombine(P.t, " << a.acc << ", " << j << ", gs, rv.acc, 1, rv.i0, rv.i1, rv.i2, rv.i3, "
      << (((P.nn_skip >> j) & 1) ? "false" : "true") << "); }\n";
  }
  o << "      }\n    }\n";
}

void emit_flush_c(const Plan& P, std::ostringstream& o) {
  o << "  __syncthreads();\n"
    << "  for (int s = threadIdx.x; s < SS; s += blockDim.x) {\n"
    << "    const qu32 c = s_cst[s];\n    if (c == 0) continue;\n"
    << "    const bool knl = s == S;\n    const qi64 key = knl ? 0 : (s == S + 1 ? (qi64)EMPTY_KEY32 : (qi64)s_keys[s]);\n"
    << "    qu64 gs;\n"
    << "    const bool ok = gtable_find_wg(P.t, key, knl, gs, &s_newg);\n"
    << "    qu8* rec = nullptr;\n"
    << "    if (ok) {\n      gadd_cstar(P.t, gs, c);\n    } else {\n"
    << "      const qu64 ri = atomicAdd(&P.t.ctl[2], 1ull);\n"
    << "      if (ri >= P.ovf_cap) { atomicAdd(&P.t.ctl[3], 1ull); continue; }\n"
    << "      rec = P.ovf + ri * (qu64)P.rec_bytes;\n      write_record_head(rec, key, knl, c);\n    }\n";
  int off = 24;
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    const std::string js = std::to_string(j);
    o << "    {\n      const qi64 acc = " << (a.acc != ACC_NONE ? "(qi64)s_acc" + js + "[s]" : std::string("0")) << ";\n"
      << "      const qu64 nn = " << (a.track_nn ? "s_nn" + js + "[s]" : std::string("c")) << ";\n";
    const bool skip_nn = (P.nn_skip >> j) & 1;
    if (a.fn != QE_AGG_COUNT_STAR && !(a.acc == ACC_NONE && skip_nn))
      o << "      if (ok) gcombine(P.t, " << a.acc << ", " << j << ", gs, acc, nn, ~0ull, ~0ull, ~0ull, ~0ull, "
        << (skip_nn ? "false" : "true") << ");\n";
    o << "      if (!ok) { qu64* f = (qu64*)(rec + " << off << "); f[0] = (qu64)acc; f[1] = nn; }\n    }\n";
    off += agg_rec_bytes(a.acc);
  }
  o << "  }\n";
}

}  // namespace

// Aggregate input expressions of the plan, per row r of a step.
bool agg_inputs(const Plan& P, std::vector<Expr>* ex) {
  ex->assign(P.naggs, Expr{"0", "1u", false});
  for (int j = 0; j < P.naggs; ++j)
    if (P.aggs[j].pkind != 0 && !agg_expr(P, j, &(*ex)[j])) return false;
  return true;
}

}  // namespace

void emit_record_words(const Plan& P, const PartLayout& L, const std::vector<Expr>& ex, const std::string& dst,
                       std::ostringstream& o);
static void emit_fit_check(const PartLayout& L, const std::string& w, std::ostringstream& o);

// Returns false when the plan shape is outside what the generator emits (caller uses the
// generic kernel). `log2` is the LDS table size chosen for this launch.
//
// `spill` (with P.mp_n > 1): rows whose spill_hash(key) is at or above P.mp_keep (the kept share
// sized to fill the LDS table) are not dropped but appended as
// partition records (part_layout) for one chunked qe_pagg pass afterwards: the columns are read
// once, and only the spilled rows' records are written and re-read. Each wave fills its own
// PART_CH-record chunks, claimed from P.part_chunk[0] (one device atomic per 2048 records; one per
// wave step on a single cursor serialised the kernel: 49 ms at 1B rows); in a step the spilling
// lanes take consecutive slots (ballot + mbcnt). Chunk c's fill goes to P.part_chunk[1 + c]
// (bucket 0), as the chunked scatter leaves it. Records are stored whole (record-major, read by
// gen_pagg_source with `soa` off): one or two vector stores per record instead of one store
// instruction per word.
bool compact_acc32(const Plan& P, int j) {
  const DAgg& a = P.aggs[j];
  if (a.acc != ACC_MIN_I && a.acc != ACC_MAX_I) return false;
  if (a.ntok != 1 || a.tok[0].op != T_COL) return false;
  const int k = P.cols[a.tok[0].arg].kind;
  return k == K_I64 || k == K_I32 || k == K_U8 || k == K_BOOL;
}

bool compact_ok(const Plan& P) {
  if (P.key_f64 || P.key_mode == 0) return false;
  for (int j = 0; j < P.naggs; ++j) {
    const int acc = P.aggs[j].acc;
    if (acc != ACC_NONE && acc != ACC_SUM_I && acc != ACC_MIN_I && acc != ACC_MAX_I) return false;
  }
  return true;
}

size_t compact_slot_bytes(const Plan& P) {
  size_t b = 8;  // key, COUNT(*)
  for (int j = 0; j < P.naggs; ++j) {
    if (P.aggs[j].acc != ACC_NONE) b += compact_acc32(P, j) ? 4 : 8;
    if (P.aggs[j].track_nn) b += 4;
  }
  return b;
}

bool gen_fused_source(const Plan& P, int log2, std::string* src, size_t* lds_bytes, bool spill) {
  if (log2 < 4 || log2 > 16 || P.ncols < 1 || P.ncols > QE_MAX_COLS) return false;
  if (spill && P.mp_n < 2) return false;
  const bool compact = P.lds_compact > 0;
  if (compact && !compact_ok(P)) return false;
  std::vector<Expr> ex;
  if (!agg_inputs(P, &ex)) return false;
  std::vector<std::string> val(P.naggs), ok(P.naggs);
  for (int j = 0; j < P.naggs; ++j) {
    val[j] = ex[j].v;
    ok[j] = ex[j].ok;
  }
  std::ostringstream o;
  const bool pf = fused_prefetch();
  o << "\nusing namespace qe;\n"
    << "extern \"C\" __global__ void __launch_bounds__(" << fused_block(log2) << ") qe_fused(const Plan P) {\n"
    << "  __shared__ qu32 s_newg;\n  if (threadIdx.x == 0) s_newg = 0;\n";
  // spilled rows go to SB = mp_n - 1 sub-buckets (spill_hash's low bits), each aggregated by its own
  // slices afterwards; per sub-bucket the wave's open record chunk (-1: none) and its fill, in
  // wave-uniform registers
  const int SB = spill ? P.mp_n - 1 : 0;
  if (spill && (SB & (SB - 1))) return false;  // (a power of two)
  if (spill)
    o << "  constexpr int SB = " << SB << ";\n  qi64 sp_cid[SB];\n  qu32 sp_fill[SB];\n"
      << "#pragma unroll\n  for (int b = 0; b < SB; ++b) { sp_cid[b] = -1; sp_fill[b] = 0; }\n  qu32 nfit = 0;\n";
  if (compact) emit_lds_table_c(P, o, lds_bytes);
  else emit_lds_table(P, o, log2, lds_bytes);
  // exact fp64 SUMs through the per-wave queue when the plan's step loop allows it and it fits
  const int block = fused_block(log2);
  const bool fxq = !compact && !spill && P.mp_n <= 1 && fx_queue_enabled() && !fx_queue_aggs(P).empty() &&
                   fx_queue_aggs(P).size() <= 8 && (1 << log2) + 2 < (1 << 24) &&
                   *lds_bytes + fx_queue_bytes(P, block) <= (size_t)152 * 1024;
  if (fxq) {
    emit_fx_queue_decl(P, o, block);
    *lds_bytes += fx_queue_bytes(P, block);
  }
  o << "  const int lane = threadIdx.x & 63;\n"
    << "  const qi64 wave = (blockIdx.x * (qi64)blockDim.x + threadIdx.x) >> 6;\n"
    << "  const qi64 stride = (((qi64)gridDim.x * blockDim.x) >> 6) * 256;\n";
  if (pf) {
    // software pipeline: the next step's columns are loaded before this step's LDS work
    o << "  {\n    const qi64 base = wave * 256;\n    const bool full = base + 256 <= P.n;\n"
      << "    const qi64 r0 = base + 2 * lane;\n";
    emit_col_loads(P, o, ~0u, "p", true);
    o << "  for (qi64 base = wave * 256; base < P.n; base += stride) {\n"
      << "    const bool full = base + 256 <= P.n;\n"
      << "    const qi64 r0 = base + 2 * lane;\n";
    for (int c = 0; c < P.ncols; ++c) {
      o << "    qi64 c" << c << "[4] = {p" << c << "[0], p" << c << "[1], p" << c << "[2], p" << c << "[3]};\n";
      if (P.cols[c].valid) o << "    const qu32 v" << c << " = pv" << c << ";\n";
    }
    o << "    if (base + stride < P.n) {\n      const qi64 nb = base + stride;\n"
      << "      const bool full = nb + 256 <= P.n;\n      const qi64 r0 = nb + 2 * lane;\n";
    emit_col_loads(P, o, ~0u, "p", false);
    o << "    }\n    do {\n";
  } else {
    o << "  for (qi64 base = wave * 256; base < P.n; base += stride) {\n"
      << "    const bool full = base + 256 <= P.n;\n"
      << "    const qi64 r0 = base + 2 * lane;\n";
    emit_col_loads(P, o, ~0u);
  }
  // (the spilling pass keeps every lane in the step until its wave-uniform chunk state is updated)
  emit_active_rows(P, o, true, !fxq && !spill);
  emit_keys(P, o);
  if (spill) {
    const PartLayout L = part_layout(P);
    // per wave: the open record chunk (PART_CH slots claimed from the chunk counter P.part_chunk[0])
    // and its fill, wave-uniform (scalar registers: a step's spill count is a ballot popcount).
    // Records are whole (record-major): a step whose records fit the open chunk stores each with
    // one or two vector stores off the chunk's buffer descriptor (base in scalar registers, a
    // 32-bit lane offset); a step that opens the next chunk (one in ~PART_CH / spilled-per-step)
    // takes the general form. Round 5 kept the state in LDS, did 64-bit slot arithmetic per row
    // and stored records chunk-columnar (one store instruction per record word): 7,000 groups,
    // 1B rows, 7.37 ms against 6.1 ms now (docs/experiments.md).
    const int RB = L.bytes();
    const int wb = L.narrow ? 4 : 8;
    // the record's words as 16 / 12 / 8 / 4-byte stores: (first word, words) pieces
    std::vector<std::pair<int, int>> pieces;
    for (int q = 0; q < L.words;) {
      const int left = (L.words - q) * wb;
      const int n = (left >= 16 ? 16 : left >= 12 && L.narrow ? 12 : left >= 8 ? 8 : 4) / wb;
      pieces.push_back({q, n});
      q += n;
    }
    auto piece_store = [&](int q, int n) {
      const int bytes = n * wb;
      o << "            {\n";
      if (bytes == 4) {
        o << "              __builtin_amdgcn_raw_buffer_store_b32((qu32)w[" << q << "], cb, off, " << q * wb << ", 0);\n";
      } else {
        const int d = bytes / 4;
        o << "              qu32x" << d << " v;\n";
        for (int i = 0; i < n; ++i)
          if (L.narrow)
            o << "              v[" << i << "] = (qu32)w[" << q + i << "];\n";
          else
            o << "              v[" << 2 * i << "] = (qu32)w[" << q + i << "]; v[" << 2 * i + 1 << "] = (qu32)((qu64)w[" << q + i
              << "] >> 32);\n";
        o << "              __builtin_amdgcn_raw_buffer_store_b" << bytes * 8 << "(v, cb, off, " << q * wb << ", 0);\n";
      }
      o << "            }\n";
    };
    o << "    qu32 sp = 0, sbk[4] = {0, 0, 0, 0};\n"
      << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
      << "      const qu32 hs = spill_hash((qu64)key[r]);\n"
      << "      if (((act >> r) & 1) && hs >= P.mp_keep) sp |= 1u << r;\n"
      << "      sbk[r] = hs & (qu32)(SB - 1);\n    }\n"
      << "    act &= ~sp;\n"
      << "#pragma unroll\n    for (int b = 0; b < SB; ++b) {\n      qu64 bal[4];\n      qu32 tot = 0;\n"
      << "#pragma unroll\n      for (int r = 0; r < 4; ++r) { bal[r] = __ballot(((sp >> r) & 1u) && sbk[r] == (qu32)b); tot += (qu32)__popcll(bal[r]); }\n"
      << "      const qu32 room = sp_cid[b] >= 0 ? (qu32)PART_CH - sp_fill[b] : 0u;\n"
      << "      if (tot && tot <= room) {\n"
      << "        const __amdgpu_buffer_rsrc_t cb = __builtin_amdgcn_make_buffer_rsrc((void*)(P.part_rec + sp_cid[b] * (PART_CH * "
      << RB << "ll)), (short)0, (int)(PART_CH * " << RB << "), 0x00020000);\n"
      << "        qu32 kb = 0;\n"
      << "#pragma unroll\n        for (int r = 0; r < 4; ++r) {\n"
      << "          if ((bal[r] >> lane) & 1) {\n"
      << "            const qu32 k = __builtin_amdgcn_mbcnt_hi((qu32)(bal[r] >> 32), __builtin_amdgcn_mbcnt_lo((qu32)bal[r], kb));\n"
      << "            const int off = (int)((sp_fill[b] + k) * " << RB << "u);\n"
      << "            qi64 w[" << L.words << "];\n";
    emit_record_words(P, L, ex, "w", o);
    emit_fit_check(L, "w", o);
    for (const auto& pc : pieces) piece_store(pc.first, pc.second);
    o << "          }\n          kb += (qu32)__popcll(bal[r]);\n        }\n"
      << "        sp_fill[b] += tot;\n"
      << "      } else if (tot) {\n"
      << "        const int leader = __ffsll((long long)__ballot(1)) - 1;\n"
      << "        qi64 id = 0;\n"
      << "        if (lane == leader) {\n"
      << "          if (sp_cid[b] >= 0) P.part_chunk[1 + sp_cid[b]] = ((qi64)b << 32) | PART_CH;\n"
      << "          id = (qi64)atomicAdd((qu64*)P.part_chunk, 1ull);\n"
      << "        }\n"
      << "        id = __shfl(id, leader);\n"
      << "        const qi64 nid = (qi64)(((qu64)__builtin_amdgcn_readfirstlane((qu32)((qu64)id >> 32)) << 32) |\n"
      << "                                (qu64)__builtin_amdgcn_readfirstlane((qu32)id));\n"
      << "        qu32 kb = 0;\n"
      << "#pragma unroll\n        for (int r = 0; r < 4; ++r) {\n"
      << "          if ((bal[r] >> lane) & 1) {\n"
      << "            const qu32 k = kb + (qu32)__popcll(bal[r] & ((1ull << lane) - 1));\n"
      << "            const qu64 pos = k < room ? (qu64)sp_cid[b] * PART_CH + sp_fill[b] + k : (qu64)nid * PART_CH + (k - room);\n"
      << "            qi64 w[" << L.words << "];\n";
    emit_record_words(P, L, ex, "w", o);
    emit_fit_check(L, "w", o);
    const char* wt = L.narrow ? "qi32" : "qi64";
    o << "            " << wt << "* const dst = (" << wt << "*)(P.part_rec + pos * " << RB << "ull);\n";
    for (int q = 0; q < L.words; ++q) o << "            dst[" << q << "] = (" << wt << ")w[" << q << "];\n";
    o << "          }\n          kb += (qu32)__popcll(bal[r]);\n        }\n"
      << "        sp_cid[b] = nid;\n        sp_fill[b] = tot - room;\n"
      << "      }\n    }\n"
      << "    if (act == 0) continue;\n";
  } else if (P.mp_n > 1)
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r)\n"
      << "      if (((act >> r) & 1) && (P.mp_pass < 0 ? spill_hash((qu64)key[r]) < P.mp_keep\n"
      << "                                              : (qu32)__umul64hi(fmix64((qu64)key[r]), (qu64)P.mp_n) != (qu32)P.mp_pass))\n"
      << "        act &= ~(1u << r);\n"
      << "    if (act == 0) continue;\n";
  if (compact)
    emit_agg_rows_c(P, o, val, ok, "P.row_base + r0 + 128 * (r >> 1) + (r & 1)", "r0 + 128 * (r >> 1) + (r & 1)");
  else
    emit_agg_rows(P, o, val, ok, "P.row_base + r0 + 128 * (r >> 1) + (r & 1)", "r0 + 128 * (r >> 1) + (r & 1)", fxq,
                  log2 <= 8);
  o << (pf ? "    } while (0);\n  }\n  }\n" : "  }\n");
  if (fxq) {  // the rest of the wave's queue
    o << "  if (q_n) {\n";
    emit_fx_queue_run(P, o, "q_n");
    o << "  }\n";
  }
  if (spill)  // each wave's open chunks: sub-bucket and fill
    o << "#pragma unroll\n  for (int b = 0; b < SB; ++b)\n"
      << "    if ((threadIdx.x & 63) == 0 && sp_cid[b] >= 0) P.part_chunk[1 + sp_cid[b]] = ((qi64)b << 32) | (qi64)sp_fill[b];\n"
      << "  if (nfit) atomicOr(&P.t.ctl[7], 1ull);\n";
  if (compact) emit_flush_c(P, o);
  else emit_flush(P, o);
  o << "  __syncthreads();\n  if (threadIdx.x == 0 && s_newg) atomicAdd(&P.t.ctl[0], (qu64)s_newg);\n}\n";
  // The exact sums' rare paths inline in the generated kernels (QE_FX_INLINE=0: out of line). C5,
  // one box (tools/exp_fxq.sh): queue + inline 8.79-8.84 ms, queue + out of line 11.5-11.8 ms,
  // no queue 10.9 (inline) / 14.0 ms (out of line); fp64 atomics 7.25 ms. The out-of-line calls sit
  // in the hot loop, and the call boundary costs the whole kernel registers.
  static const bool fx_inline = [] {
    const char* e = getenv("QE_FX_INLINE");
    return !(e && e[0] == '0');
  }();
  *src = std::string(fx_inline ? "#define QE_FX_INLINE 1\n" : "") + kDevHeader + o.str();
  return true;
}

// ---- radix-partitioned aggregation (group counts beyond the LDS table) ---------------------------------
// When the expected groups do not fit a workgroup's LDS table, every row would otherwise update
// the global table with device-scope atomics (~30 G atomics/s chip-wide: 2 % of the HBM roofline
// at 64K+ groups). Instead the rows are partitioned by key hash so that each workgroup of the
// aggregation pass sees a slice of one bucket's records, whose groups fit its LDS table:
//   qe_pcount   per (bucket, workgroup) counts of the selected rows (reads predicate + key columns)
//   (exclusive scan of the counts, bucket-major: records of one bucket are contiguous)
//   qe_pscatter predicate, key, aggregate inputs -> one fixed-width record per selected row at
//               its bucket's next position (LDS cursors, or an LDS counting sort per tile)
//   k_part_slices (qe_hashagg.hip) slices inside bucket boundaries; a one-slice bucket is exclusive
//   qe_pagg     LDS aggregation of a record slice, then the flush (plain read-modify-writes when
//               the slice is exclusive)
// Record layout: key | aggregate input values, or (colmode) the columns the programs read |
// [flags: bit 0 null key, bit 1+j input j valid (colmode: column slot c valid)] | [global row index,
// fp64 MIN/MAX only]. Whichever of the two forms is narrower is used: C4 (SUM(a+b), MIN(a),
// MAX(b)) stores key, a, b in 24 bytes instead of key, a+b, a, b in 32. Odd widths are written and
// read in 8-byte words, even widths in 16-byte pairs.
PartLayout part_layout(const Plan& P) {
  PartLayout L{};
  bool knull = false, vnull = false, cnull = false;
  for (int k = 0; k < P.nkeys; ++k) knull = knull || P.cols[P.key_col[k]].valid != nullptr;
  int nv = 0;
  unsigned cm = 0;
  for (int j = 0; j < P.naggs; ++j) {
    if (P.aggs[j].pkind == 0) continue;
    ++nv;
    vnull = vnull || P.aggs[j].track_nn;
    L.row = L.row || acc_is_f64mm(P.aggs[j].acc);
    for (int t = 0; t < P.aggs[j].ntok; ++t)
      if (P.aggs[j].tok[t].op == T_COL) cm |= 1u << P.aggs[j].tok[t].arg;
  }
  for (int c = 0; c < P.ncols; ++c)
    if ((cm >> c) & 1u) cnull = cnull || P.cols[c].valid != nullptr;
  const int wv = 1 + nv + ((knull || vnull) ? 1 : 0);
  const int wc = 1 + __builtin_popcount(cm) + ((knull || cnull) ? 1 : 0);
  L.colmode = wc < wv;
  int w = 1;
  for (int j = 0; j < P.naggs; ++j) L.val_word[j] = (!L.colmode && P.aggs[j].pkind != 0) ? w++ : -1;
  for (int c = 0; c < QE_MAX_COLS; ++c) L.col_word[c] = (L.colmode && ((cm >> c) & 1u)) ? w++ : -1;
  L.flags_word = (knull || (L.colmode ? cnull : vnull)) ? w++ : -1;
  L.row_word = L.row ? w++ : -1;
  L.words = w;
  // 32-bit words: every word integral (no fp64 key, value or column, no row index); whether the
  // values fit is checked by the scatter (Plan.part_narrow)
  if (P.part_narrow && !L.row && !P.key_f64) {
    bool ok = true;
    for (int c = 0; c < P.ncols; ++c)
      if (L.col_word[c] >= 0 && P.cols[c].kind == K_F64) ok = false;
    for (int j = 0; j < P.naggs; ++j)
      if (L.val_word[j] >= 0 && P.aggs[j].acc != ACC_SUM_I && P.aggs[j].acc != ACC_MIN_I && P.aggs[j].acc != ACC_MAX_I)
        ok = false;
    L.narrow = ok;
  }
  return L;
}

// Narrow records: the statements that fold `w`'s words (qi64 array expression) into `nfit` (set when
// one does not survive the round trip through 32 bits).
static void emit_fit_check(const PartLayout& L, const std::string& w, std::ostringstream& o) {
  if (!L.narrow) return;
  for (int q = 0; q < L.words; ++q)
    // (nonzero when the high word is not the low word's sign: two ops per word instead of a 64-bit
    // compare and select)
    o << "      nfit |= (qu32)((qu64)" << w << "[" << q << "] >> 32) ^ (qu32)((qi32)" << w << "[" << q << "] >> 31);\n";
}

// Narrow records: chunk value q of a record whose words are `w` (G = 1: one word, G = 2: a pair).
static std::string narrow_chunk(const std::string& w, int G, const std::string& q) {
  if (G == 1) return "(qu32)" + w + "[" + q + "]";
  return "((qu64)(qu32)" + w + "[2 * (" + q + ")] | ((qu64)(qu32)" + w + "[2 * (" + q + ") + 1] << 32))";
}

// Record word assignments for row r of a scatter step into `dst` (an array expression).
void emit_record_words(const Plan& P, const PartLayout& L, const std::vector<Expr>& ex, const std::string& dst,
                       std::ostringstream& o) {
  o << "      " << dst << "[0] = key[r];\n";
  for (int j = 0; j < P.naggs; ++j)
    if (L.val_word[j] >= 0) o << "      " << dst << "[" << L.val_word[j] << "] = " << ex[j].v << ";\n";
  for (int c = 0; c < P.ncols; ++c)
    if (L.col_word[c] >= 0) o << "      " << dst << "[" << L.col_word[c] << "] = " << col_raw(c) << ";\n";
  if (L.flags_word >= 0) {
    o << "      " << dst << "[" << L.flags_word << "] = (qi64)((knull >> r) & 1)";
    for (int j = 0; j < P.naggs; ++j)
      if (L.val_word[j] >= 0) o << " | ((qi64)((" << ex[j].ok << ") & 1u) << " << (1 + j) << ")";
    for (int c = 0; c < P.ncols; ++c)
      if (L.col_word[c] >= 0 && P.cols[c].valid) o << " | ((qi64)" << col_ok(P, c) << " << " << (1 + c) << ")";
    o << ";\n";
  }
  if (L.row_word >= 0)
    o << "      " << dst << "[" << L.row_word << "] = P.row_base + r0 + 128 * (r >> 1) + (r & 1);\n";
}

bool gen_part_source(const Plan& P, int log2p, bool scatter, std::string* src) {
  if (P.ncols < 1 || P.ncols > QE_MAX_COLS || log2p < 1 || log2p > 13) return false;
  std::vector<Expr> ex;
  if (!agg_inputs(P, &ex)) return false;
  const PartLayout L = part_layout(P);
  unsigned need = pred_key_cols(P);
  if (scatter) need = ~0u;
  std::ostringstream o;
  o << "\nusing namespace qe;\n"
    << "extern \"C\" __global__ void __launch_bounds__(512) " << (scatter ? "qe_pscatter" : "qe_pcount")
    << "(const Plan P) {\n"
    << "  constexpr int LOG2P = " << log2p << ", NP = 1 << LOG2P;\n";
  if (scatter)
    o << "  __shared__ qu64 s_cur[NP];\n"
      << "  for (int b = threadIdx.x; b < NP; b += blockDim.x) s_cur[b] = (qu64)P.part_off[(qi64)b * gridDim.x + blockIdx.x];\n";
  else
    o << "  __shared__ qu32 s_cnt[NP];\n"
      << "  for (int b = threadIdx.x; b < NP; b += blockDim.x) s_cnt[b] = 0;\n";
  o << "  __syncthreads();\n"
    << "  const int lane = threadIdx.x & 63;\n"
    << "  qu32 nfit = 0;\n"
    << "  const qi64 lo = (qi64)blockIdx.x * P.part_tw;\n"
    << "  const qi64 hi = lo + P.part_tw < P.n ? lo + P.part_tw : P.n;\n"
    << "  for (qi64 base = lo + (qi64)(threadIdx.x >> 6) * 256; base < hi; base += (qi64)(blockDim.x >> 6) * 256) {\n"
    << "    const bool full = base + 256 <= P.n;\n"
    << "    const qi64 r0 = base + 2 * lane;\n";
  emit_col_loads(P, o, need);
  emit_active_rows(P, o, false);
  emit_keys(P, o);
  o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
    << "      if (!((act >> r) & 1)) continue;\n"
    << "      const qu32 b = (qu32)(fmix64((qu64)key[r]) >> (64 - LOG2P));\n";
  if (!scatter) {
    o << "      atomicAdd(&s_cnt[b], 1u);\n    }\n  }\n  __syncthreads();\n"
      << "  for (int b = threadIdx.x; b < NP; b += blockDim.x) P.part_off[(qi64)b * gridDim.x + blockIdx.x] = s_cnt[b];\n}\n";
  } else {
    o << "      const qu64 pos = atomicAdd(&s_cur[b], 1ull);\n"
      << "      qi64 w[" << L.words << "];\n";
    emit_record_words(P, L, ex, "w", o);
    emit_fit_check(L, "w", o);
    if (L.narrow) {
      const int G = L.words % 2 ? 1 : 2;
      const char* ct = G == 2 ? "qu64" : "qu32";
      o << "      " << ct << "* dst = (" << ct << "*)(P.part_rec + pos * " << L.bytes() << "ull);\n";
      for (int q = 0; q < L.words / G; ++q)
        o << "      dst[" << q << "] = " << narrow_chunk("w", G, std::to_string(q)) << ";\n";
    } else if (L.words % 2 == 0) {
      o << "      qi64x2* dst = (qi64x2*)(P.part_rec + pos * " << 8 * L.words << "ull);\n";
      for (int q = 0; q < L.words / 2; ++q)
        o << "      dst[" << q << "] = qi64x2{w[" << 2 * q << "], w[" << 2 * q + 1 << "]};\n";
    } else {
      o << "      qi64* dst = (qi64*)(P.part_rec + pos * " << 8 * L.words << "ull);\n";
      for (int q = 0; q < L.words; ++q) o << "      dst[" << q << "] = w[" << q << "];\n";
    }
    o << "    }\n  }\n";
    if (L.narrow) o << "  if (nfit) atomicOr(&P.t.ctl[7], 1ull);\n";
    o << "}\n";
  }
  *src = std::string(kDevHeader) + o.str();
  return true;
}

// Staged scatter (few buckets): a workgroup of B threads (512) takes 4B-row tiles; the tile's records
// are counting-sorted by bucket in LDS (rank = LDS atomic on the tile histogram, one wave scans
// it), then written out as contiguous per-bucket runs, 16 bytes per lane in record-stream order
// (8 for odd record widths),
// so the HBM writes coalesce instead of landing as one 2-word record per lane. Rows go to the same
// (bucket, workgroup) ranges as the direct scatter: the records of one bucket and workgroup keep
// a contiguous range of its bucket (their order inside it may differ run to run).
bool part_staged_ok(const Plan& P, int log2p) {
  if (P.n < 2) return false;  // (the staged scatter's prefetch loads row pairs clamped to n - 2)
  if (log2p == 10) return pscatter_wide() && part_layout(P).words <= 3;
  return log2p <= 9 && part_layout(P).words * pscatter_block() <= 8 * 256;
}

// QE_PSCATTER_WIDE=1: 1024 buckets staged by 1024-thread workgroups (4096-row tiles, records of
// <= 3 words: 96 KiB of LDS records + 16 KiB of bucket cursors), one per CU. Off: 1B rows, 1M
// groups (1024 buckets) took 22.6 ms staged this way against 19.3 ms with the direct scatter.
bool pscatter_wide() {
  static const bool w = [] {
    const char* e = getenv("QE_PSCATTER_WIDE");
    return e && *e && atoi(e) == 1;
  }();
  return w;
}

int pscatter_block_for(int log2p) { return log2p == 10 ? 1024 : pscatter_block(); }

// Workgroup size of the staged scatter (tile = 4 rows per thread); QE_PSCATTER_BLOCK overrides.
// Measured at 200M rows, 64K / 256K groups (count + scatter + aggregate): 128 threads 4.05 /
// 4.69 ms, 512 threads (2 per CU) 3.55 / 4.14 ms, 1024 threads 3.64 / 4.37 ms.
int pscatter_block() {
  static const int b = [] {
    const char* e = getenv("QE_PSCATTER_BLOCK");
    const int v = e && *e ? atoi(e) : 512;
    return (v == 128 || v == 256 || v == 512 || v == 1024) ? v : 512;
  }();
  return b;
}

// Workgroup size of the partition-aggregate pass (QE_PAGG_BLOCK = 512 / 1024, default 1024). 1024
// threads run one workgroup per CU with up to 152 KiB of LDS table, so the radix pass needs half the
// buckets of 512-thread tables (76 KiB). 1B rows, C4 shape, interleaved A/B (512 -> 1024, ms):
// 65536 groups 14.52 -> 13.93, 262144 18.32 -> 16.50, 1048576 20.4 -> 20.4, 4194304 24.5 -> 22.0.
int pagg_block() {
  static const int b = [] {
    const char* e = getenv("QE_PAGG_BLOCK");
    return e && *e && atoi(e) == 512 ? 512 : 1024;
  }();
  return b;
}

// Tiles of column loads in flight ahead of the one being sorted (QE_PSCATTER_DEPTH, 1..4).
int pscatter_depth() {
  static const int d = [] {
    const char* e = getenv("QE_PSCATTER_DEPTH");
    const int v = e && *e ? atoi(e) : 2;
    return std::max(1, std::min(4, v));
  }();
  return d;
}

// Chunked partition records chunk-columnar (QE_PART_SOA=1): word q of a chunk's records together,
// as the spilling pass writes them, so the aggregation pass loads each word as one contiguous
// 512-byte run per wave instead of 8-byte words 8 x W bytes apart; the scatter's write-out then
// writes each word of a bucket's run separately.
bool part_soa() {
  static const bool v = [] {
    const char* e = getenv("QE_PART_SOA");
    return e && e[0] == '1';
  }();
  return v;
}

// Chunk ids of the chunked staged scatter (QE_PART_STATIC, default 1): each workgroup owns the
// range [blockIdx.x * cpw, (blockIdx.x + 1) * cpw), cpw = its rows / PART_CH rounded up + buckets
// (every closed chunk is full, so a workgroup never needs more), and claims from it with an LDS
// counter; unused ids are marked -1 (skipped by the chunk planning). 0: one device-wide counter
// (a device atomic with a return value per claim, which waits for every load the claiming wave
// has in flight).
bool part_static() {
  static const bool v = [] {
    const char* e = getenv("QE_PART_STATIC");
    return !(e && e[0] == '0');
  }();
  return v;
}

// (QE_PSCATTER_FAST=1, off by default: 1B rows, same box, 64K / 1M groups 6.41 / 9.00 ms against
// 5.93 / 8.90 for the per-lane chunk write-out)
static bool pscatter_fast_env() {
  static const bool v = [] {
    const char* e = getenv("QE_PSCATTER_FAST");
    return e && e[0] == '1';
  }();
  return v;
}

bool part_blk64(const Plan& P, const PartLayout& L);

bool gen_pscatter_staged_source(const Plan& P, int log2p, std::string* src, bool chunked, bool soa) {
  if (soa && !chunked) return false;
  if (P.ncols < 1 || P.ncols > QE_MAX_COLS || log2p < 1 || !part_staged_ok(P, log2p)) return false;
  std::vector<Expr> ex;
  if (!agg_inputs(P, &ex)) return false;
  const PartLayout L = part_layout(P);
  if (soa && L.narrow) return false;
  const int W = L.words, G = W % 2 ? 1 : 2;
  const char* chunk = L.narrow ? (G == 2 ? "qu64" : "qu32") : (G == 2 ? "qi64x2" : "qi64");
  // fast form (chunked 32-bit records, QE_PSCATTER_FAST=1, opt-in): each row writes its record
  // words to LDS right away (word-major, double-buffered by tile, slot wave*256 + 64r + lane) and
  // after the scan only its 2-byte index to the sorted position; the write-out then moves whole
  // records (W dwords per lane). The records' registers are dead before the first barrier.
  const bool fast = chunked && !soa && L.narrow && pscatter_fast_env();
  const bool blk = fast && part_blk64(P, L);
  std::ostringstream o;
  o << "\nusing namespace qe;\n"
    << "extern \"C\" __global__ void __launch_bounds__(" << pscatter_block_for(log2p) << ") qe_pscatter(const Plan P) {\n"
    << "  constexpr int LOG2P = " << log2p << ", NP = 1 << LOG2P, W = " << W << ", T = " << 4 * pscatter_block_for(log2p) << ";\n"
    << "  __shared__ qu32 s_hist[NP];\n  __shared__ qu32 s_off[NP];\n  __shared__ qu64 s_cur[NP];\n  __shared__ qu64 s_dst[NP];\n"
    << "  constexpr int WC = " << W / G << ";  // " << chunk << " chunks per record\n";
  if (fast)
    o << "  __shared__ qu32 s_w[2][" << W << "][T];\n  __shared__ unsigned short s_perm[T];\n";
  else
    o << "  __shared__ " << chunk << " s_rec[T * WC];\n";
  o << "  __shared__ unsigned short s_bkt[T];\n  __shared__ qu32 s_total;\n";
  if (chunked)
    // per bucket: the open chunk (-1: none) and its end, the tile's second destination base (for
    // the records past the open chunk's room) and the tile-local index where that part starts
    o << "  __shared__ qu64 s_end[NP];\n  __shared__ qu64 s_dst2[NP];\n  __shared__ qu32 s_lim[NP];\n"
      << "  __shared__ qi32 s_chunk[NP];\n"
      << "  for (int b = threadIdx.x; b < NP; b += blockDim.x) {\n"
      << "    s_cur[b] = 0;\n    s_end[b] = 0;\n    s_chunk[b] = -1;\n    s_hist[b] = 0;\n  }\n"
      << (part_static() ? "  __shared__ qu32 s_cnext;\n  if (threadIdx.x == 0) s_cnext = 0;\n"
                          "  const qi64 cpw = (P.part_tw + PART_CH - 1) / PART_CH + NP, cbase = (qi64)blockIdx.x * cpw;\n"
                        : "");
  else
    o << "  for (int b = threadIdx.x; b < NP; b += blockDim.x) {\n"
      << "    s_cur[b] = (qu64)P.part_off[(qi64)b * gridDim.x + blockIdx.x];\n    s_hist[b] = 0;\n  }\n";
  o << "  __syncthreads();\n"
    << "  const int lane = threadIdx.x & 63;\n"
    << "  qu32 nfit = 0;\n"
    << "  const qi64 lo = (qi64)blockIdx.x * P.part_tw;\n"
    << "  const qi64 hi = lo + P.part_tw < P.n ? lo + P.part_tw : P.n;\n"
    << "  const qi64 woff = (qi64)(threadIdx.x >> 6) * 256;\n";
  // Register prefetch over D rotating buffers: the tile loop is unrolled D times, and step k
  // reads buffer k, builds its records, then reloads buffer k with the tile D steps ahead before
  // the LDS sort and write-out. The loads then have D - 1 whole tiles plus this tile's LDS phases
  // to land (barriers wait on LDS only; moving buffers between registers would wait on them).
  // LDS holds the workgroup to 2 per CU, so the buffer registers cost no occupancy.
  const int D = pscatter_depth();
  auto buf = [](int d, const std::string& cs) { return "n" + std::to_string(d) + "_" + cs; };
  // 8-byte columns are buffered as two 16-byte vectors, loaded straight into them on both the
  // full-tile and the tail path: with a 4 x int64 buffer filled from a per-load temporary, the
  // compiler merged the two paths with register moves that waited for each load right after it
  // was issued (s_waitcnt vmcnt(0) per column), which serialised the prefetch
  // (QE_PSCATTER_VEC=0 restores that form)
  // (QE_PSCATTER_VEC=1: vector buffers loaded under the full-tile / in-range branches, = 2 default:
  // loaded unconditionally, below)
  static const int vec = [] {
    const char* e = getenv("QE_PSCATTER_VEC");
    return e && *e ? std::max(0, std::min(2, atoi(e))) : 2;
  }();
  auto wide8 = [&](int c) { return vec && (P.cols[c].kind == K_I64 || P.cols[c].kind == K_F64); };
  for (int c = 0; c < P.ncols; ++c)
    for (int d = 0; d < D; ++d) {
      if (wide8(c))
        o << "  qi64x2 " << buf(d, std::to_string(c)) << "[2] = {qi64x2{0, 0}, qi64x2{0, 0}};\n";
      else
        o << "  qi64 " << buf(d, std::to_string(c)) << "[4] = {0, 0, 0, 0};\n";
      if (P.cols[c].valid) o << "  qu32 v" << buf(d, std::to_string(c)) << " = 0;\n";
    }
  auto load_into = [&](const std::string& nb, int d, const std::string& ind) {
    o << ind << "{\n" << ind << "  const qi64 base = " << nb << ";\n"
      << ind << "  const qi64 r0 = base + 2 * lane;\n";
    // Vector buffers load unconditionally, from row indices clamped to [0, n - 2] (the staged
    // scatter runs only when n >= 2; rows at or past n are masked by act when the tile is used,
    // and a tile past the workgroup's range is never used): the same load instructions issue on
    // every path, so the wait before a buffer is consumed can leave the later buffers' loads in
    // flight (a load under a branch left the in-order count unknown, and the compiler waited for
    // every outstanding load)
    unsigned rest = 0;
    for (int c = 0; c < P.ncols; ++c) {
      if (!wide8(c)) {
        rest |= 1u << c;
        continue;
      }
      const std::string cs = std::to_string(c), n = buf(d, cs);
      if (vec == 1)
        o << ind << "  if (base < hi) {\n" << ind << "    const qi64* p = (const qi64*)P.cols[" << cs << "].p;\n"
          << ind << "    if (base + 256 <= P.n) {\n"
          << ind << "      " << n << "[0] = " << ld("qi64x2", "p + r0") << ";\n"
          << ind << "      " << n << "[1] = " << ld("qi64x2", "p + r0 + 128") << ";\n"
          << ind << "    } else {\n"
          << ind << "      " << n << "[0] = qi64x2{r0 < P.n ? p[r0] : 0, r0 + 1 < P.n ? p[r0 + 1] : 0};\n"
          << ind << "      " << n << "[1] = qi64x2{r0 + 128 < P.n ? p[r0 + 128] : 0, r0 + 129 < P.n ? p[r0 + 129] : 0};\n"
          << ind << "    }\n" << ind << "  }\n";
      else
        o << ind << "  {\n" << ind << "    const qi64* p = (const qi64*)P.cols[" << cs << "].p;\n"
          << ind << "    const qi64 lim = P.n - 2, i0 = r0 < lim ? r0 : lim, i1 = r0 + 128 < lim ? r0 + 128 : lim;\n"
          << ind << "    " << n << "[0] = " << ld("qi64x2", "p + i0") << ";\n"
          << ind << "    " << n << "[1] = " << ld("qi64x2", "p + i1") << ";\n"
          << ind << "  }\n";
      if (P.cols[c].valid)
        o << ind << "  {\n" << ind << "    const qu8* vb = P.cols[" << cs << "].valid;\n"
          << ind << "    const qi64 lim = P.n - 1, i0 = r0 < lim ? r0 : lim, i1 = r0 + 128 < lim ? r0 + 128 : lim;\n"
          << ind << "    const qu32 lo = (qu32)(vb[i0 >> 3] >> (r0 & 7)) & 3u;\n"
          << ind << "    const qu32 hi = (qu32)(vb[i1 >> 3] >> (r0 & 7)) & 3u;\n"
          << ind << "    v" << n << " = lo | (hi << 2);\n" << ind << "  }\n";
    }
    o << ind << "  if (base < hi) {\n" << ind << "  const bool full = base + 256 <= P.n;\n";
    if (rest) {
      emit_col_loads(P, o, rest);
      for (int c = 0; c < P.ncols; ++c) {
        if (!((rest >> c) & 1u)) continue;
        const std::string cs = std::to_string(c), n = buf(d, cs);
        o << ind << "  " << n << "[0] = c" << cs << "[0]; " << n << "[1] = c" << cs << "[1]; " << n << "[2] = c" << cs
          << "[2]; " << n << "[3] = c" << cs << "[3];\n";
        if (P.cols[c].valid) o << ind << "  v" << n << " = v" << cs << ";\n";
      }
    }
    o << ind << "  }\n" << ind << "}\n";
  };
  for (int d = 0; d < D; ++d) load_into("lo + " + std::to_string(d) + " * (qi64)T + woff", d, "  ");
  o << "  for (qi64 t0 = lo; t0 < hi; t0 += " << D << " * (qi64)T) {\n";
  for (int k = 0; k < D; ++k) {
    // Three barriers per tile: (A) the tile histogram is complete (and the previous tile's
    // write-out has finished with s_dst / s_rec); (B) wave 0 has scanned it into s_off, the tile's
    // per-bucket destination bases s_dst, and advanced s_cur; (C) the records sit sorted in LDS
    // and s_hist is cleared for the next tile. The write-out then runs without a barrier behind it.
    o << "  {\n    const qi64 tile = t0 + " << k << " * (qi64)T;\n    if (tile >= hi) break;\n"
      << "    qu32 ract = 0, bk[4], rk[4];\n" << (fast ? "    const int sb = (int)((tile - lo) / T) & 1;\n" : "    qi64 rw[4][W];\n")
      << "    const qi64 base = tile + woff;\n";
    for (int c = 0; c < P.ncols; ++c) {
      const std::string cs = std::to_string(c), n = buf(k, cs);
      if (wide8(c) && vec == 2)  // (a pair clamped at the column's end holds the last row in .y)
        o << "    qi64 c" << cs << "[4] = {base + 2 * lane + 1 < P.n ? " << n << "[0].x : " << n << "[0].y, " << n
          << "[0].y, base + 2 * lane + 129 < P.n ? " << n << "[1].x : " << n << "[1].y, " << n << "[1].y};\n";
      else if (wide8(c))
        o << "    qi64 c" << cs << "[4] = {" << n << "[0].x, " << n << "[0].y, " << n << "[1].x, " << n << "[1].y};\n";
      else
        o << "    qi64 (&c" << cs << ")[4] = " << n << ";\n";
      if (P.cols[c].valid) o << "    const qu32 v" << cs << " = v" << n << ";\n";
    }
    o << "    if (base < hi) do {\n"
      << "    const bool full = base + 256 <= P.n;\n"
      << "    const qi64 r0 = base + 2 * lane;\n";
    emit_active_rows(P, o, false);
    emit_keys(P, o);
    o << "    ract = act;\n"
      << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
      << "      if (!((act >> r) & 1)) continue;\n"
      << "      bk[r] = (qu32)(fmix64((qu64)key[r]) >> (64 - LOG2P));\n"
      << "      rk[r] = atomicAdd(&s_hist[bk[r]], 1u);\n";
    if (fast) {
      o << "      {\n      qi64 w[W];\n";
      emit_record_words(P, L, ex, "w", o);
      emit_fit_check(L, "w", o);
      o << "      const int slot = (int)woff + 64 * r + lane;\n"
        << "#pragma unroll\n      for (int q = 0; q < W; ++q) s_w[sb][q][slot] = (qu32)w[q];\n      }\n";
    } else {
      emit_record_words(P, L, ex, "rw[r]", o);
      emit_fit_check(L, "rw[r]", o);
    }
    o << "    }\n    } while (0);\n";
    // QE_PSCATTER_RELOAD=1 (default): the buffer is reloaded after the scan, whose chunk claims
    // (a device atomic with a return value) would otherwise wait for wave 0's just-issued loads
    // (in-order vmcnt); 0: reloaded before the scan
    static const bool late = [] {
      const char* e = getenv("QE_PSCATTER_RELOAD");
      return !(e && e[0] == '0');
    }();
    const std::string reload_at = "tile + " + std::to_string(D) + " * (qi64)T + woff";
    if (!(late && chunked)) load_into(reload_at, k, "    ");
    o << "    __syncthreads();\n"
      // exclusive scan of the tile histogram by wave 0
      << "    if (threadIdx.x < 64) {\n"
      << "      constexpr int PER = (NP + 63) / 64;\n"
      << "      qu32 loc[PER], s = 0;\n"
      << "#pragma unroll\n      for (int i = 0; i < PER; ++i) { const int b = lane * PER + i; loc[i] = b < NP ? s_hist[b] : 0u; s += loc[i]; }\n"
      << "      qu32 x = s;\n"
      << "#pragma unroll\n      for (int d = 1; d < 64; d <<= 1) { const qu32 y = __shfl_up(x, d); if (lane >= d) x += y; }\n"
      << "      qu32 e = x - s;\n"
      << "#pragma unroll\n      for (int i = 0; i < PER; ++i) {\n"
      << "        const int b = lane * PER + i;\n";
    if (chunked)
      // a run longer than the open chunk's room fills it, and the rest starts a new chunk
      o << "        if (b < NP) {\n"
        << "          s_off[b] = e;\n          const qu64 c = s_cur[b], room = s_end[b] - c;\n          s_dst[b] = c - e;\n"
        << "          if (loc[i] > room) {\n"
        << "            if (s_chunk[b] >= 0) P.part_chunk[1 + s_chunk[b]] = ((qi64)b << 32) | PART_CH;\n"
        << (part_static() ? "            const qi64 id = cbase + (qi64)atomicAdd(&s_cnext, 1u);\n"
                          : "            const qi64 id = (qi64)atomicAdd((unsigned long long*)P.part_chunk, 1ull);\n")
        << "            const qu64 nb = (qu64)id * PART_CH;\n"
        << "            s_lim[b] = e + (qu32)room;\n            s_dst2[b] = nb - (e + room);\n"
        << "            s_cur[b] = nb + (loc[i] - room);\n            s_end[b] = nb + PART_CH;\n            s_chunk[b] = (qi32)id;\n"
        << "          } else {\n            s_lim[b] = e + loc[i];\n            s_cur[b] = c + loc[i];\n          }\n"
        << "        }\n";
    else
      o << "        if (b < NP) { s_off[b] = e; const qu64 c = s_cur[b]; s_dst[b] = c - e; s_cur[b] = c + loc[i]; }\n";
    o << "        e += loc[i];\n      }\n"
      << "      if (lane == 63) s_total = x;\n"
      << "    }\n"
      << "    __syncthreads();\n";
    if (late && chunked) load_into(reload_at, k, "    ");
    o << "    for (int b = threadIdx.x; b < NP; b += blockDim.x) s_hist[b] = 0;\n"
      << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
      << "      if (!((ract >> r) & 1)) continue;\n"
      << "      const qu32 pos = s_off[bk[r]] + rk[r];\n"
      << "      s_bkt[pos] = (unsigned short)bk[r];\n";
    if (fast)
      o << "      s_perm[pos] = (unsigned short)((int)woff + 64 * r + lane);\n";
    else
      o << "#pragma unroll\n      for (int q = 0; q < WC; ++q) s_rec[pos * WC + q] = "
        << (L.narrow ? narrow_chunk("rw[r]", G, "q") : W % 2 ? "rw[r][q]" : "qi64x2{rw[r][2 * q], rw[r][2 * q + 1]}") << ";\n";
    o << "    }\n"
      << "    __syncthreads();\n"
      << "    const qu32 tot = s_total;\n";
    if (fast)
      o << "    for (qu32 j = threadIdx.x; j < tot; j += blockDim.x) {\n"
        << "      const qu32 b = s_bkt[j], src = s_perm[j];\n"
        << "      const qu64 dst = (j < s_lim[b] ? s_dst[b] : s_dst2[b]) + j;\n"
        << (blk ? "      qu32* d = (qu32*)P.part_rec + (dst >> 6) * " + std::to_string(64 * W) + "ull + (dst & 63);  // (blocks of 64, part_blk64)\n"
                  "#pragma unroll\n      for (int q = 0; q < W; ++q) d[64 * q] = s_w[sb][q][src];\n"
                : "      qu32* d = (qu32*)(P.part_rec + dst * " + std::to_string(L.bytes()) + "ull);\n"
                  "#pragma unroll\n      for (int q = 0; q < W; ++q) d[q] = s_w[sb][q][src];\n")
        << "    }\n";
    else if (soa)
      // word-major: consecutive threads write consecutive records' word q (one run per word)
      o << "    for (qu32 c = threadIdx.x; c < tot * W; c += blockDim.x) {\n"
        << "      const qu32 q = c / tot, j = c - q * tot;\n"
        << "      const qu32 b = s_bkt[j];\n      const qu64 dst = (j < s_lim[b] ? s_dst[b] : s_dst2[b]) + j;\n"
        << "      ((qi64*)P.part_rec)[(dst / PART_CH) * (W * PART_CH) + q * PART_CH + dst % PART_CH] = ((const qi64*)s_rec)[j * W + q];\n"
        << "    }\n";
    else
      o << "    for (qu32 c = threadIdx.x; c < tot * WC; c += blockDim.x) {\n"
        << "      const qu32 j = c / WC, q = c % WC;\n"
        << (chunked ? "      const qu32 b = s_bkt[j];\n      const qu64 dst = (j < s_lim[b] ? s_dst[b] : s_dst2[b]) + j;\n"
                    : "      const qu64 dst = s_dst[s_bkt[j]] + j;\n")
        << "      ((" << chunk << "*)(P.part_rec + dst * " << L.bytes() << "ull))[q] = s_rec[c];\n"
        << "    }\n";
    o
      << "  }\n";
  }
  o << "  }\n";
  if (chunked)  // close the open chunks (their last tile's scan is behind a barrier every thread passed)
    o << "  __syncthreads();\n"
      << "  for (int b = threadIdx.x; b < NP; b += blockDim.x)\n"
      << "    if (s_chunk[b] >= 0) P.part_chunk[1 + s_chunk[b]] = ((qi64)b << 32) | (qi64)(s_cur[b] - (qu64)s_chunk[b] * PART_CH);\n";
  if (chunked && part_static())  // the range's unused chunk ids are marked empty; block 0 writes the id count
    o << "  for (qi64 c = (qi64)s_cnext + threadIdx.x; c < cpw; c += blockDim.x) P.part_chunk[1 + cbase + c] = -1;\n"
      << "  if (blockIdx.x == 0 && threadIdx.x == 0) P.part_chunk[0] = (qi64)gridDim.x * cpw;\n";
  if (L.narrow) o << "  if (nfit) atomicOr(&P.t.ctl[7], 1ull);\n";
  o << "}\n";
  *src = std::string(kDevHeader) + o.str();
  return true;
}

// Aggregation pass for chunked 32-bit records (QE_PAGG_FAST, default 1; the general form below
// otherwise). Same walk (a wave takes whole chunks, one step of 256 records in flight ahead), but:
//   * each lane takes 4 CONSECUTIVE records of the step and loads them as W 16-byte vectors (4 x W
//     32-bit words, 16-byte aligned: a chunk is PART_CH x 4W bytes), instead of 4W strided 4-byte
//     loads whose per-lane addresses each cost 64-bit arithmetic;
//   * the LDS table keeps 32-bit keys (every key of a 32-bit record fits; EMPTY_KEY32 = INT32_MIN,
//     that key itself in special slot S + 1) and 32-bit MIN / MAX accumulators where the input is a
//     32-bit word (a value word, or a bare column), so those atomics move half the bytes;
//   * the per-row LDS updates are branch-free: a row that is inactive, goes to the global table or
//     has a null input adds into a sink slot (index SS, never flushed) instead of running under a
//     per-row, per-aggregate exec-mask branch (the SALU half of the general pass's instructions);
//     one sink slot per lane (SS + lane), so inactive lanes never pile onto one LDS address.
constexpr int PAGG_CHCAP = 2048;  // chunk-list entries a fast aggregation slice stages in LDS
// record buffers of the fast aggregation pass in rotation (QE_PAGG_FAST_DEPTH, 2 or 4)
static int pagg_fast_depth() {
  static const int d = [] {
    const char* e = getenv("QE_PAGG_FAST_DEPTH");
    const int v = e && *e ? atoi(e) : 2;
    return v == 4 ? 4 : 2;  // (a divisor of the 8 steps per chunk)
  }();
  return d;
}
static bool pagg_fast_env() {
  static const bool v = [] {
    const char* e = getenv("QE_PAGG_FAST");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Fast-pass LDS slot: 32-bit key, COUNT(*), per aggregate a 64-bit SUM or 32-bit MIN / MAX (a bare
// 32-bit word), a 32-bit non-null count where tracked.
static size_t pagg_fast_slot_bytes(const Plan& P, const std::vector<bool>& acc32) {
  size_t bps = 8;
  for (int j = 0; j < P.naggs; ++j) {
    if (P.aggs[j].acc != ACC_NONE) bps += acc32[j] ? 4 : 8;
    if (P.aggs[j].track_nn) bps += 4;
  }
  return bps;
}
// Slots (multiple of 64, + 2 special + 64 sinks) beside `fixed` bytes of other LDS
static int pagg_fast_slots_for(size_t bps, size_t fixed) {
  constexpr size_t kBudget = 160 * 1024 - 256;  // (s_fail, s_newg, alignment)
  const int64_t s = fixed < kBudget ? ((int64_t)((kBudget - fixed) / bps) - 66) & ~(int64_t)63 : 0;
  return (int)std::min<int64_t>(s, 1 << 14);
}

// Plans the fast aggregation pass takes: 32-bit integral records, integer accumulators.
static bool pagg_fast_ok(const Plan& P, const PartLayout& L) {
  if (!L.narrow || L.row_word >= 0 || P.key_f64) return false;
  for (int j = 0; j < P.naggs; ++j) {
    const int acc = P.aggs[j].acc;
    if (acc != ACC_NONE && acc != ACC_SUM_I && acc != ACC_MIN_I && acc != ACC_MAX_I) return false;
  }
  std::vector<Expr> ex;
  return !L.colmode || agg_inputs(P, &ex);
}

// Chunked 32-bit records in blocks of 64 (word q of the block's 64 records contiguous: record slot
// p's word q at dword (p / 64) * 64W + 64q + p % 64), written by the fast staged scatter and read
// by the fast aggregation pass: a load instruction there takes 4 x 256 contiguous bytes (16 lanes
// x 4 records of one word per block) instead of 16 bytes every 48 (record-major). Measured on the
// records' walk alone (a round-5 timing probe, since removed: docs/experiments.md; 1B rows, 64K groups): 1.70 vs 1.26 ms.
// (QE_PART_BLK64=1; off: the scatter's write-out then stores each record's words 256 B apart and
// took 8.5 instead of 6.5 ms at 64K groups, more than the reads gain)
bool part_blk64(const Plan& P, const PartLayout& L) {
  static const bool on = [] {
    const char* e = getenv("QE_PART_BLK64");
    return e && e[0] == '1';
  }();
  return on && pscatter_fast_env() && pagg_fast_env() && pagg_fast_ok(P, L);
}

static bool gen_pagg_fast_source(const Plan& P, const PartLayout& L, int log2, int64_t bucket_groups, std::string* src,
                                 size_t* lds_bytes) {
  if (!pagg_fast_ok(P, L)) return false;
  const bool blk = part_blk64(P, L);
  const int W = L.words;
  std::vector<std::string> val(P.naggs), ok(P.naggs);
  std::vector<bool> acc32(P.naggs, false);
  std::vector<Expr> ex;
  if (L.colmode && !agg_inputs(P, &ex)) return false;
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.acc != ACC_NONE && a.acc != ACC_SUM_I && a.acc != ACC_MIN_I && a.acc != ACC_MAX_I) return false;
    if (L.colmode) {
      val[j] = ex[j].v;
      ok[j] = ex[j].ok;
    } else {
      val[j] = L.val_word[j] >= 0 ? "w" + std::to_string(L.val_word[j]) + "[r]" : "0";
      ok[j] = (L.val_word[j] >= 0 && a.track_nn)
                  ? "((qu32)(w" + std::to_string(L.flags_word) + "[r] >> " + std::to_string(1 + j) + ") & 1u)"
                  : "1u";
    }
    const bool bare = L.colmode ? (a.ntok == 1 && a.tok[0].op == T_COL) : L.val_word[j] >= 0;
    acc32[j] = (a.acc == ACC_MIN_I || a.acc == ACC_MAX_I) && bare;
  }
  // Table size: as many 4-slot buckets as the LDS holds beside the chunk list (and the per-wave
  // regrouping area, when that is used), not the power of two of the general pass's 36-byte slots:
  // with C4's 24-byte slots ~6K slots instead of 4096, so the half-full tables of 128+ buckets
  // run about a third full. Regrouped loads (QE_PAGG_TRANSPOSE, 48 KiB for C4) only while the
  // table they leave is at most a quarter full: at 1B rows and 262K / 1M groups (2048 groups per
  // bucket) a half-full 4096-slot table spent 5.5 / 6.4 ms in the aggregation pass (general pass:
  // 4.1 / 4.8), the keys displaced past the two-bucket window taking the serial probe loop.
  static const bool tr_env = [] {
    const char* e = getenv("QE_PAGG_TRANSPOSE");
    return !(e && e[0] == '0');
  }();
  const size_t bps = pagg_fast_slot_bytes(P, acc32);
  const size_t tr_bytes = (size_t)(pagg_block() / 64) * W * 1024;
  const int s_tr = pagg_fast_slots_for(bps, (size_t)1024 * 8 + tr_bytes);
  const int s_plain = pagg_fast_slots_for(bps, (size_t)PAGG_CHCAP * 8);
  const bool tr = !blk && tr_env && s_tr >= 256 && (bucket_groups <= 0 || 4 * bucket_groups <= s_tr);
  const int S = tr ? s_tr : s_plain, SS = S + 2;
  if (S < 256) return false;
  // hit window: 2 buckets (default) or 3 (QE_PAGG_WINDOW=3, for fuller tables)
  static const bool win3 = [] {
    const char* e = getenv("QE_PAGG_WINDOW");
    return e && e[0] == '3';
  }();
  (void)log2;
  std::ostringstream o;
  o << "\nusing namespace qe;\n"
    << "extern \"C\" __global__ void __launch_bounds__(" << pagg_block() << ") qe_pagg(const Plan P) {\n"
    << "  if ((qi64)blockIdx.x >= P.part_slice[0]) return;\n"
    << "  const qi64 clo = P.part_slice[2 + 2 * (qi64)blockIdx.x];\n"
    << "  const qi64 hx = P.part_slice[3 + 2 * (qi64)blockIdx.x];\n"
    << "  const bool excl = (hx & PART_EXCL) != 0;\n"
    << "  const qi64 hi = ((hx & ~PART_EXCL) - clo) * PART_CH;\n"
    << "  if (hi <= 0) return;\n"
    << "  if (P.t.ctl[7] & 1) return;  // a value did not fit the 32-bit records: the update reruns wide (bit 1: a compact-table misfit, not ours)\n"
    << "  __shared__ int s_fail;\n  __shared__ qu32 s_newg;\n  if (threadIdx.x == 0) { s_fail = 0; s_newg = 0; }\n"
    << "  constexpr int S = " << S << ", SS = " << SS << ", SINK = SS;\n"
    << "  constexpr qu32 NBK = S / 4;\n"
    << "  __shared__ __attribute__((aligned(16))) qi32 s_keys[SS + 64];\n  __shared__ qu32 s_cst[SS + 64];\n";
  size_t lds = (size_t)(SS + 64) * 8;
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.acc != ACC_NONE) {
      o << "  __shared__ " << (acc32[j] ? "qi32" : "qi64") << " s_acc" << j << "[SS + 64];\n";
      lds += (size_t)(SS + 64) * (acc32[j] ? 4 : 8);
    }
    if (a.track_nn) {
      o << "  __shared__ qu32 s_nn" << j << "[SS + 64];\n";
      lds += (size_t)(SS + 64) * 4;
    }
  }
  // record-major records loaded as contiguous KiB per load instruction and regrouped per lane
  // through a per-wave LDS staging area (W KiB per wave; `tr` above): each lane then holds 4
  // consecutive records as before. Measured on the walk alone (a round-5 timing probe, since removed: docs/experiments.md; 1B rows, 64K
  // groups): 1.70 vs 1.26 ms. (QE_PAGG_TRANSPOSE=0: direct 48-byte lane loads)
  const int chcap = 1024;
  if (tr) lds += tr_bytes;
  *lds_bytes = lds;
  auto init32 = [](int acc) {
    return acc == ACC_MIN_I ? std::string("0x7FFFFFFF") : acc == ACC_MAX_I ? std::string("(qi32)0x80000000u") : "0";
  };
  o << "  for (int s = threadIdx.x; s < SS + 64; s += blockDim.x) {\n    s_keys[s] = EMPTY_KEY32;\n    s_cst[s] = 0;\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.acc != ACC_NONE) o << "    s_acc" << j << "[s] = " << (acc32[j] ? init32(a.acc) : acc_init(a.acc)) << ";\n";
    if (a.track_nn) o << "    s_nn" << j << "[s] = 0;\n";
  }
  // the slice's chunk list (id, fill) staged in LDS, CHCAP chunks per round: the walk's per-step
  // lookups are then LDS reads, off the in-order vector-memory counter the record loads wait on
  // (a global lookup under a branch made the compiler wait for every outstanding load there)
  o << "  }\n"
    << "  constexpr int CHCAP = " << (tr ? chcap : PAGG_CHCAP) << ";\n  __shared__ qu64 s_ch[CHCAP];\n"
    << (tr ? "  __shared__ qu32x4 s_tr[" + std::to_string(pagg_block() / 64) + "][" + std::to_string(64 * W) + "];\n" : std::string())
    << "  const qi64 nch = hi / PART_CH;\n"
    << "  const int lane = threadIdx.x & 63;\n"
    << "  const int ro = " << (blk ? "64 * (lane >> 4) + 4 * (lane & 15)" : "4 * lane") << ";  // the lane's first record of a step\n"
    << "  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nwv = blockDim.x >> 6;\n"
    ;
  lds += (size_t)(tr ? chcap : PAGG_CHCAP) * 8;
  // D rotating record buffers: step t consumes buffer t % D in place and reloads it with step t + D,
  // so each step's loads have the next D - 1 steps' work to land (one buffer copied forward made
  // the loop's back edge wait for the loads it had just issued)
  const int D = pagg_fast_depth();
  for (int k = 0; k < D; ++k) {
    o << "  qu32 b" << k << "_act;\n  qi64 b" << k << "_pb;\n";
    for (int v = 0; v < W; ++v) o << "  qu32x4 b" << k << "_v" << v << ";\n";
  }
  // Step order (QE_PAGG_INTERLEAVE=1): wave w takes steps w, w + nwv, ... of the slice's chunk list
  // (8 per chunk) instead of whole chunks, so a slice of ~150 chunks splits over 16 waves to within
  // one step rather than one chunk (the chunk list is in LDS, so a step's lookup is cheap either way)
  static const bool ilv = [] {
    const char* e = getenv("QE_PAGG_INTERLEAVE");
    return e && e[0] == '1';
  }();
  auto NB = [](const std::string& t) {
    if (ilv) return "((qi64)((wv + (" + t + ") * nwv) >> 3) * PART_CH + (qi64)((wv + (" + t + ") * nwv) & 7) * 256)";
    return "((qi64)(wv + ((" + t + ") >> 3) * nwv) * PART_CH + (qi64)((" + t + ") & 7) * 256)";
  };
  auto load_step = [&](int k, const std::string& nb) {
    const std::string B = "b" + std::to_string(k) + "_";
    // branch-free (a step past the wave's last one loads a real chunk's slots, all inactive)
    o << "    {\n      const qi64 nb = " << nb << ";\n      const bool in = nb < rhi;\n"
      << "      const qu64 m = s_ch[in ? (int)(nb >> 11) : 0];\n"
      << "      const qi32 ko = (qi32)(nb & (PART_CH - 1));\n"
      << "      const qi64 npb = (qi64)(qi32)(qu32)m * PART_CH + ko;\n"
      << "      const qi32 cfill = in ? (qi32)(m >> 32) - ko : 0;\n"
      // (lanes whose records lie past the chunk's fill read the step's first block instead: the
      // unfilled tail of a chunk is never fetched)
      << (blk ? "      const qu32x4* p = (const qu32x4*)((const qu32*)P.part_rec + ((npb >> 6) + (ro < cfill ? (lane >> 4) : 0)) * " +
                    std::to_string(64 * W) + "ull + 4 * (lane & 15));\n"
              : "      const qu32x4* p = (const qu32x4*)(P.part_rec + (qu64)(npb + 4 * lane) * " + std::to_string(L.bytes()) + "ull);\n");
    if (blk) {
      for (int v = 0; v < W; ++v) o << "      " << B << "v" << v << " = " << ld("qu32x4", "p + 16 * " + std::to_string(v)) << ";\n";
    } else if (tr) {  // contiguous KiB per load; a piece past the chunk's fill re-reads the step's first
      o << "      const qu32x4* pc = (const qu32x4*)(P.part_rec + (qu64)npb * " << L.bytes() << "ull);\n";
      for (int v = 0; v < W; ++v)
        o << "      " << B << "v" << v << " = " << ld("qu32x4", "pc + ((" + std::to_string(64 * v) + " + lane) * 16 < cfill * " +
                                                        std::to_string(L.bytes()) + " ? " + std::to_string(64 * v) + " + lane : lane)")
          << ";\n";
    } else
    for (int v = 0; v < W; ++v) o << "      " << B << "v" << v << " = " << ld("qu32x4", "p + " + std::to_string(v)) << ";\n";
    o << "      " << B << "pb = npb;\n      qu32 nact = 0;\n"
      << "#pragma unroll\n      for (int r = 0; r < 4; ++r) nact |= (qu32)(ro + r < cfill) << r;\n"
      << "      if (P.defer_in) {  // (uniform: retry passes only)\n"
      << "        for (int r = 0; r < 4; ++r) { const qi64 i = npb + ro + r; if (!((P.defer_in[i >> 5] >> (i & 31)) & 1)) nact &= ~(1u << r); }\n"
      << "      }\n      " << B << "act = nact;\n    }\n";
  };
  o << "  for (qi64 c0 = 0; c0 < nch; c0 += CHCAP) {\n"
    << "  const qi64 rch = nch - c0 < CHCAP ? nch - c0 : CHCAP, rhi = rch * PART_CH;\n"
    << "  if (c0) __syncthreads();  // every wave is done with the previous round's list\n"
    << "  for (qi64 c = threadIdx.x; c < rch; c += blockDim.x) {\n"
    << "    const qi32 id = P.part_sorted[clo + c0 + c];\n"
    << "    s_ch[c] = (qu64)(qu32)id | ((qu64)P.part_chunk[1 + id] << 32);\n  }\n"
    << "  __syncthreads();\n";
  for (int k = 0; k < D; ++k) load_step(k, NB(std::to_string(k)));
  // the wave's steps: 8 per chunk it takes (wv, wv + nwv, ...), a multiple of D, so the unrolled
  // loop has no exit between a buffer's reload and its use
  if (ilv)
    o << "  const int nsteps = wv < rch * 8 ? (((int)((rch * 8 - 1 - wv) / nwv) + 1 + " << D - 1 << ") / " << D << ") * " << D << " : 0;\n";
  else
    o << "  const int nsteps = wv < rch ? (int)((rch - 1 - wv) / nwv + 1) * 8 : 0;\n";
  o << "  for (int t = 0; t < nsteps; t += " << D << ") {\n";
  for (int k = 0; k < D; ++k) {
  const std::string B = "b" + std::to_string(k) + "_";
  o << "  {\n"
    << "    const qi64 sbase = " << B << "pb;\n    const qu32 act = " << B << "act;\n"
    << "    qu32 d[" << 4 * W << "] = {";
  if (blk) {  // vector v holds word v of the lane's 4 records: d[r * W + q] = word q of record r
    const char* el[4] = {".x", ".y", ".z", ".w"};
    for (int r = 0; r < 4; ++r)
      for (int q = 0; q < W; ++q) o << (r || q ? ", " : "") << B << "v" << q << el[r];
  } else if (tr) {  // through the wave's staging area: piece v of lane l in, the lane's own 4 records out
    // (lanes exchange data through LDS: wave-scope fences keep the compiler from moving a read of
    // another lane's piece above the write that stores it, or the next step's writes above it)
    o << "0};\n    {\n      qu32x4* st = s_tr[threadIdx.x >> 6];\n"
      << "      __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n      __builtin_amdgcn_wave_barrier();\n";
    for (int v = 0; v < W; ++v) o << "      st[" << 64 * v << " + lane] = " << B << "v" << v << ";\n";
    o << "      __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n      __builtin_amdgcn_wave_barrier();\n"
      << "      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");\n";
    for (int v = 0; v < W; ++v)
      o << "      { const qu32x4 t = st[lane * " << W << " + " << v << "]; d[" << 4 * v << "] = t.x; d[" << 4 * v + 1
        << "] = t.y; d[" << 4 * v + 2 << "] = t.z; d[" << 4 * v + 3 << "] = t.w; }\n";
    o << "    }\n";
  } else {
    for (int v = 0; v < W; ++v)
      o << (v ? ", " : "") << B << "v" << v << ".x, " << B << "v" << v << ".y, " << B << "v" << v << ".z, " << B << "v" << v << ".w";
  }
  if (!tr) o << "};\n";
  o << ""
    << "    qi64 key[4];\n";
  for (int q = 1; q < W; ++q) o << "    qi64 w" << q << "[4];\n";
  o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n      key[r] = (qi64)(qi32)d[r * " << W << "];\n";
  for (int q = 1; q < W; ++q) o << "      w" << q << "[r] = (qi64)(qi32)d[r * " << W << " + " << q << "];\n";
  o << "    }\n    qu32 knull = 0;\n";
  if (L.flags_word >= 0)
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) knull |= (qu32)(w" << L.flags_word << "[r] & 1) << r;\n";
  for (int c = 0; c < P.ncols; ++c) {
    if (L.col_word[c] < 0) continue;
    const std::string cs = std::to_string(c);
    o << "    qi64 (&c" << cs << ")[4] = w" << L.col_word[c] << ";\n";
    if (P.cols[c].valid)
      o << "    qu32 v" << cs << " = 0;\n"
        << "#pragma unroll\n    for (int r = 0; r < 4; ++r) v" << cs << " |= ((qu32)(w" << L.flags_word << "[r] >> "
        << (1 + c) << ") & 1u) << r;\n";
  }
  // slots: the first probe of all 4 rows together; collisions (rare) probe on
  o << "    int slot[4];\n    qu32 h[4];\n    qu32x4 q[4];\n"
    << "    qu32 h2[4];\n    qu32x4 q2[4];\n" << (win3 ? "    qu32 h3[4];\n    qu32x4 q3[4];\n" : "")
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
    << "      h[r] = (qu32)(((qu64)lds_hash((qu64)key[r]) * NBK) >> 32); h2[r] = h[r] + 1 == NBK ? 0u : h[r] + 1;\n"
    << "      q[r] = ((const qu32x4*)s_keys)[h[r]]; q2[r] = ((const qu32x4*)s_keys)[h2[r]];\n"
    << (win3 ? "      h3[r] = h2[r] + 1 == NBK ? 0u : h2[r] + 1; q3[r] = ((const qu32x4*)s_keys)[h3[r]];\n" : "")
    << "    }\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
    << "      const qu32 kk = (qu32)key[r];\n"
    << (win3 ? "      const int hs = bucket3_hit(q[r], q2[r], q3[r], kk, h[r], h2[r], h3[r]);\n"
             : "      const int hs = bucket2_hit(q[r], q2[r], kk, h[r], h2[r]);\n")
    << "      slot[r] = ((knull >> r) & 1) ? S : ((qi32)kk == EMPTY_KEY32 ? S + 1 : hs);\n"
    << "    }\n"
    << "    qu32 miss = 0;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) miss |= (qu32)(slot[r] < 0) << r;\n"
    << "    miss &= act;\n"
    << "    if (miss) {\n      int t0 = slot[0], t1 = slot[1], t2 = slot[2], t3 = slot[3];\n"
    << "      lds_probe4_rows(s_keys, NBK, miss, (qi32)key[0], (qi32)key[1], (qi32)key[2], (qi32)key[3], h[0], h[1], h[2], h[3], t0, t1, t2, t3);\n"
    << "      slot[0] = t0; slot[1] = t1; slot[2] = t2; slot[3] = t3;\n    }\n"
    << "    qu32 glob = 0;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) glob |= (qu32)(slot[r] < 0) << r;\n"
    << "    glob &= act;\n    const qu32 loc = act & ~glob;\n"
    << "    int sl[4];\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) sl[r] = ((loc >> r) & 1) ? slot[r] : SINK + lane;\n"
    << "#pragma unroll\n    for (int r = 0; r < 4; ++r) atomicAdd(&s_cst[sl[r]], 1u);\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.pkind == 0) continue;
    const std::string js = std::to_string(j);
    o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) {\n"
      << "      const int s = (" << ok[j] << ") ? sl[r] : SINK + lane;\n"
      << "      const qi64 x = " << val[j] << ";\n";
    if (a.track_nn) o << "      atomicAdd(&s_nn" << js << "[s], 1u);\n";
    switch (a.acc) {
      case ACC_SUM_I: o << "      atomicAdd((qu64*)&s_acc" << js << "[s], (qu64)x);\n"; break;
      case ACC_MIN_I:
        o << "      atomicMin(&s_acc" << js << "[s], " << (acc32[j] ? "(qi32)x" : "x") << ");\n";
        break;
      case ACC_MAX_I:
        o << "      atomicMax(&s_acc" << js << "[s], " << (acc32[j] ? "(qi32)x" : "x") << ");\n";
        break;
      default: break;
    }
    o << "    }\n";
  }
  // rows whose group only fits the global table (rare)
  o << "    if (glob) {\n      for (int r = 0; r < 4; ++r) {\n        if (!((glob >> r) & 1)) continue;\n"
    << "        const qi64 lr = sbase + ro + r;\n        qu64 gs;\n"
    << "        if (!gtable_find(P.t, key[r], (knull >> r) & 1, gs)) {\n"
    << "          atomicOr((qu32*)&P.defer_out[lr >> 5], 1u << (lr & 31));\n"
    << "          atomicAdd(&P.t.ctl[1], 1ull);\n          continue;\n        }\n"
    << "        gadd_cstar(P.t, gs, 1);\n";
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    if (a.pkind == 0) continue;
    o << "        if (" << ok[j] << ") { const RowVal rv = row_partial(" << a.acc << ", " << val[j]
      << ", 0); gcombine(P.t, " << a.acc << ", " << j << ", gs, rv.acc, 1, rv.i0, rv.i1, rv.i2, rv.i3, "
      << (((P.nn_skip >> j) & 1) ? "false" : "true") << "); }\n";
  }
  o << "      }\n    }\n  }\n";
  load_step(k, NB("t + " + std::to_string(k + D)));
  }  // buffers
  o << "  }\n  }\n";
  // flush (exclusive slices: plain read-modify-writes), as emit_flush with 32-bit keys / accumulators
  o << "  __syncthreads();\n"
    << "  for (int s = threadIdx.x; s < SS; s += blockDim.x) {\n"
    << "    const qu32 c = s_cst[s];\n    if (c == 0) continue;\n"
    << "    const bool knl = s == S;\n    const qi64 key = knl ? 0 : (s == S + 1 ? (qi64)EMPTY_KEY32 : (qi64)s_keys[s]);\n"
    << "    qu64 gs;\n"
    << "    const bool ok = gtable_find_wg(P.t, key, knl, gs, &s_newg);\n"
    << "    qu8* rec = nullptr;\n"
    << "    if (ok) {\n      if (excl) gadd_cstar_excl(P.t, gs, c, &s_newg); else gadd_cstar(P.t, gs, c);\n    } else {\n"
    << "      const qu64 ri = atomicAdd(&P.t.ctl[2], 1ull);\n"
    << "      if (ri >= P.ovf_cap) { s_cst[s] = c | 0x80000000u; s_fail = 1; continue; }\n"
    << "      rec = P.ovf + ri * (qu64)P.rec_bytes;\n      write_record_head(rec, key, knl, c);\n    }\n";
  int off = 24;
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    const std::string js = std::to_string(j);
    o << "    {\n      const qi64 acc = " << (a.acc != ACC_NONE ? "(qi64)s_acc" + js + "[s]" : std::string("0")) << ";\n"
      << "      const qu64 nn = " << (a.track_nn ? "s_nn" + js + "[s]" : std::string("c")) << ";\n";
    const bool skip_nn = (P.nn_skip >> j) & 1;
    if (a.fn != QE_AGG_COUNT_STAR)
      o << "      if (ok) { if (excl) gcombine_excl(P.t, " << a.acc << ", " << j << ", gs, acc, nn, ~0ull, ~0ull, ~0ull, ~0ull);"
        << " else gcombine(P.t, " << a.acc << ", " << j << ", gs, acc, nn, ~0ull, ~0ull, ~0ull, ~0ull, "
        << (skip_nn ? "false" : "true") << "); }\n";
    o << "      if (!ok) { qu64* f = (qu64*)(rec + " << off << "); f[0] = (qu64)acc; f[1] = nn; }\n    }\n";
    off += agg_rec_bytes(a.acc);
  }
  o << "  }\n";
  // groups that found no room anywhere: defer their records (the table is final)
  o << "  __syncthreads();\n"
    << "  if (s_fail) {\n"
    << "    for (qi64 v = threadIdx.x; v < hi; v += blockDim.x) {\n"
    << "      const qi64 id = P.part_sorted[clo + v / PART_CH], ko = v % PART_CH;\n"
    << "      if (ko >= (P.part_chunk[1 + id] & 0xFFFFFFFFll)) continue;\n"
    << "      const qi64 i = id * PART_CH + ko;\n"
    << "      if (P.defer_in && !((P.defer_in[i >> 5] >> (i & 31)) & 1)) continue;\n"
    << (blk ? "      const qi32* rp = (const qi32*)P.part_rec + (i >> 6) * " + std::to_string(64 * W) + "ll + (i & 63);\n"
            : "      const qi32* rp = (const qi32*)(P.part_rec + i * " + std::to_string(L.bytes()) + "ull);\n")
    << "      const qi32 k = rp[0];\n"
    << "      const bool kn = " << (L.flags_word >= 0 ? "rp[" + std::to_string(L.flags_word * (blk ? 64 : 1)) + "] & 1" : std::string("false")) << ";\n"
    << "      int s = kn ? S : (k == EMPTY_KEY32 ? S + 1 : -1);\n"
    << "      if (s < 0) s = lds_probe4(s_keys, NBK, k, (qu32)(((qu64)lds_hash((qu64)(qi64)k) * NBK) >> 32));\n"
    << "      if (s >= 0 && (s_cst[s] & 0x80000000u)) {\n"
    << "        atomicOr((qu32*)&P.defer_out[i >> 5], 1u << (i & 31));\n"
    << "        atomicAdd(&P.t.ctl[1], 1ull);\n      }\n    }\n  }\n"
    << "  if (threadIdx.x == 0 && s_newg) atomicAdd(&P.t.ctl[0], (qu64)s_newg);\n}\n";
  *src = std::string(kDevHeader) + o.str();
  return true;
}

// Largest table of the fast aggregation pass without the regrouping area (0: the plan does not take
// the fast pass), for the bucket count of the partitioned update.
int pagg_fast_slots(const Plan& P) {
  const PartLayout L = part_layout(P);
  if (!pagg_fast_env() || !pagg_fast_ok(P, L)) return 0;
  std::vector<bool> acc32(P.naggs, false);
  for (int j = 0; j < P.naggs; ++j) {
    const DAgg& a = P.aggs[j];
    const bool bare = L.colmode ? (a.ntok == 1 && a.tok[0].op == T_COL) : L.val_word[j] >= 0;
    acc32[j] = (a.acc == ACC_MIN_I || a.acc == ACC_MAX_I) && bare;
  }
  return pagg_fast_slots_for(pagg_fast_slot_bytes(P, acc32), (size_t)PAGG_CHCAP * 8);
}

// `soa` (chunked only): records stored chunk-columnar, word q of slot i at
// ((i / PART_CH) * W + q) * PART_CH + i % PART_CH (the spilling fused pass writes them so).
bool gen_pagg_source(const Plan& P, int log2, std::string* src, size_t* lds_bytes, bool chunked, bool soa,
                     int64_t bucket_groups) {
  if (log2 < 4 || log2 > 16 || (soa && !chunked)) return false;
  const PartLayout L = part_layout(P);
  if (chunked && !soa && pagg_fast_env() && gen_pagg_fast_source(P, L, log2, bucket_groups, src, lds_bytes)) return true;
  std::vector<std::string> val(P.naggs), ok(P.naggs);
  if (L.colmode) {
    // the programs run here, over column values read back from the record (c<slot>[r], v<slot>)
    std::vector<Expr> ex;
    if (!agg_inputs(P, &ex)) return false;
    for (int j = 0; j < P.naggs; ++j) {
      val[j] = ex[j].v;
      ok[j] = ex[j].ok;
    }
  } else {
    for (int j = 0; j < P.naggs; ++j) {
      val[j] = L.val_word[j] >= 0 ? "w" + std::to_string(L.val_word[j]) + "[r]" : "0";
      ok[j] = (L.val_word[j] >= 0 && P.aggs[j].track_nn)
                  ? "((qu32)(w" + std::to_string(L.flags_word) + "[r] >> " + std::to_string(1 + j) + ") & 1u)"
                  : "1u";
    }
  }
  std::ostringstream o;
  o << "\nusing namespace qe;\n"
    << "extern \"C\" __global__ void __launch_bounds__(" << pagg_block() << ") qe_pagg(const Plan P) {\n"
    << "  if ((qi64)blockIdx.x >= P.part_slice[0]) return;\n";
  if (chunked)
    // the slice is a range [clo, chi) of the bucket-grouped chunk list; rows lo..hi index its
    // chunks' record slots (PART_CH per chunk, the tail of a partly filled chunk inactive)
    o << "  const qi64 clo = P.part_slice[2 + 2 * (qi64)blockIdx.x];\n"
      << "  const qi64 hx = P.part_slice[3 + 2 * (qi64)blockIdx.x];\n"
      << "  const bool excl = (hx & PART_EXCL) != 0;\n"
      << "  const qi64 lo = 0, hi = ((hx & ~PART_EXCL) - clo) * PART_CH;\n";
  else
    o << "  const qi64 lo = P.part_slice[2 + 2 * (qi64)blockIdx.x];\n"
      << "  const qi64 hx = P.part_slice[3 + 2 * (qi64)blockIdx.x];\n"
      << "  const bool excl = (hx & PART_EXCL) != 0;\n"
      << "  const qi64 hi = hx & ~PART_EXCL;\n";
  o << "  if (hi <= lo) return;  // (the step prefetch below reads the slice's first record)\n";
  if (L.narrow) o << "  if (P.t.ctl[7] & 1) return;  // a value did not fit the 32-bit records: the update reruns wide (bit 1: a compact-table misfit)\n";
  o << "  __shared__ int s_fail;\n  __shared__ qu32 s_newg;\n  if (threadIdx.x == 0) { s_fail = 0; s_newg = 0; }\n";
  emit_lds_table(P, o, log2, lds_bytes);
  // the records of the wave's next step are loaded into n* registers before this step's LDS work
  auto word = [](const std::string& pre, int q) {
    return (q == 0 ? pre + "key" : pre + "w" + std::to_string(q)) + "[r]";
  };
  auto load_step = [&](const std::string& pre, const std::string& nb) {
    o << "    {\n      const qi64 nb = " << nb << ";\n      " << pre << "act = 0;\n";
    if (chunked)
      // the wave's current chunk (slice index, id, fill) is fetched when a step enters a new one
      o << "      qi64 cfill = 0;\n      " << pre << "pb = 0;\n"
        << "      if (nb < hi) {\n"
        << "        const qi64 cix = nb / PART_CH, ko = nb % PART_CH;\n"
        << "        if (cix != mcix) {\n          mcix = cix;\n          mid = P.part_sorted[clo + cix];\n"
        << "          mfill = P.part_chunk[1 + mid] & 0xFFFFFFFFll;\n        }\n"
        << "        " << pre << "pb = mid * PART_CH + ko;\n"
        << "        cfill = mfill - ko;\n      }\n";
    else
      o << "      " << pre << "pb = nb;\n";
    o << "#pragma unroll\n      for (int r = 0; r < 4; ++r) {\n"
      << "        const qi64 i = " << pre << "pb + lane + 64 * r;\n"
      << (chunked ? "        bool on = lane + 64 * r < cfill;\n" : "        bool on = i < hi;\n")
      << "        if (on && P.defer_in) on = (P.defer_in[i >> 5] >> (i & 31)) & 1;\n"
      << "        " << pre << "act |= (qu32)on << r;\n";
    if (L.narrow && soa) {
      o << "        const qi32* p = (const qi32*)P.part_rec + (on ? (i / PART_CH) * (" << L.words
        << " * PART_CH) + i % PART_CH : 0);\n";
      for (int q = 0; q < L.words; ++q)
        o << "        " << word(pre, q) << " = (qi64)" << ld("qi32", "p + " + std::to_string(q) + " * PART_CH") << ";\n";
    } else if (L.narrow) {
      // 32-bit words, sign-extended (pairs loaded as one 8-byte word when the width is even)
      const int G = L.words % 2 ? 1 : 2;
      const char* ct = G == 2 ? "qu64" : "qu32";
      o << "        const " << ct << "* p = (const " << ct << "*)(P.part_rec + (on ? i : 0) * " << L.bytes() << "ull);\n";
      for (int q = 0; q < L.words / G; ++q) {
        o << "        { const " << ct << " v = " << ld(ct, "p + " + std::to_string(q)) << "; ";
        if (G == 1)
          o << word(pre, q) << " = (qi64)(qi32)v; }\n";
        else
          o << word(pre, 2 * q) << " = (qi64)(qi32)(qu32)v; " << word(pre, 2 * q + 1) << " = (qi64)(qi32)(qu32)(v >> 32); }\n";
      }
    } else if (soa) {
      o << "        const qi64* p = (const qi64*)P.part_rec + (on ? (i / PART_CH) * (" << L.words
        << " * PART_CH) + i % PART_CH : 0);\n";
      for (int q = 0; q < L.words; ++q)
        o << "        " << word(pre, q) << " = " << ld("qi64", "p + " + std::to_string(q) + " * PART_CH") << ";\n";
    } else if (L.words % 2 == 0) {
      o << "        const qi64x2* p = (const qi64x2*)(P.part_rec + (on ? i : 0) * " << 8 * L.words << "ull);\n";
      for (int q = 0; q < L.words / 2; ++q)
        o << "        { const qi64x2 v = " << ld("qi64x2", "p + " + std::to_string(q)) << "; " << word(pre, 2 * q)
          << " = v.x; " << word(pre, 2 * q + 1) << " = v.y; }\n";
    } else {
      o << "        const qi64* p = (const qi64*)(P.part_rec + (on ? i : 0) * " << 8 * L.words << "ull);\n";
      for (int q = 0; q < L.words; ++q)
        o << "        " << word(pre, q) << " = " << ld("qi64", "p + " + std::to_string(q)) << ";\n";
    }
    o << "      }\n    }\n";
  };
  o << "  const int lane = threadIdx.x & 63;\n"
    << "  const qi64 step = (qi64)(blockDim.x >> 6) * 256;\n"
    << "  qu32 nact;\n  qi64 nkey[4], npb;\n";
  if (chunked)
    o << "  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nwv = blockDim.x >> 6;\n"
      << "  qi64 mcix = -1, mid = 0, mfill = 0;\n";
  for (int q = 1; q < L.words; ++q) o << "  qi64 nw" << q << "[4];\n";
  const char* pfe = getenv("QE_PAGG_PREFETCH");
  const bool pf = !(pfe && pfe[0] == '0');
  // QE_PAGG_DEPTH = 2: two record buffers (n*, m*) in rotation, the loop unrolled twice, so each
  // buffer is reloaded two steps ahead (copying one buffer into the other would wait on its loads)
  const char* pde = getenv("QE_PAGG_DEPTH");
  const int depth = pf && pde && pde[0] == '2' ? 2 : 1;
  if (depth == 2) {
    o << "  qu32 mact;\n  qi64 mkey[4], mpb;\n";
    for (int q = 1; q < L.words; ++q) o << "  qi64 mw" << q << "[4];\n";
  }
  // one step over the records of buffer `pre` at row `b`, reloading that buffer with row `nb`
  auto body = [&](const std::string& pre, const std::string& b, const std::string& nb) {
    (void)b;  // the step's first record slot is the buffer's pb (= its row for unchunked slices)
    o << "    {\n    const qi64 sbase = " << pre << "pb;\n"
      << "    const qu32 act = " << pre << "act;\n    qu32 knull = 0;\n"
      << "    qi64 key[4] = {" << pre << "key[0], " << pre << "key[1], " << pre << "key[2], " << pre << "key[3]};\n";
    for (int q = 1; q < L.words; ++q)
      o << "    qi64 w" << q << "[4] = {" << pre << "w" << q << "[0], " << pre << "w" << q << "[1], " << pre << "w" << q
        << "[2], " << pre << "w" << q << "[3]};\n";
    if (!nb.empty()) load_step(pre, nb);
    if (L.flags_word >= 0)
      o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) knull |= (qu32)(w" << L.flags_word << "[r] & 1) << r;\n";
    for (int c = 0; c < P.ncols; ++c) {
      if (L.col_word[c] < 0) continue;
      const std::string cs = std::to_string(c);
      o << "    qi64 (&c" << cs << ")[4] = w" << L.col_word[c] << ";\n";
      if (P.cols[c].valid)
        o << "    qu32 v" << cs << " = 0;\n"
          << "#pragma unroll\n    for (int r = 0; r < 4; ++r) v" << cs << " |= ((qu32)(w" << L.flags_word << "[r] >> "
          << (1 + c) << ") & 1u) << r;\n";
    }
    o << "    if (act != 0) {\n";
    emit_agg_rows(P, o, val, ok, L.row_word >= 0 ? "w" + std::to_string(L.row_word) + "[r]" : "0",
                  "sbase + lane + 64 * r");
    o << "    }\n    }\n";
  };
  const std::string first = "lo + (qi64)(threadIdx.x >> 6) * 256";
  // chunk-major walk (chunked slices, one-step prefetch; QE_PAGG_WALK=0: step-major): wave w takes
  // the slice's chunks w, w + waves, ..., each as PART_CH / 256 consecutive steps, so the chunk
  // list and fill are read once per 8 steps instead of every step (each such read waited for all
  // of the wave's outstanding record loads)
  const char* wke = getenv("QE_PAGG_WALK");
  const int walk_lvl = wke && *wke ? atoi(wke) : 1;
  const bool walk = chunked && pf && depth == 1 && walk_lvl >= 1;
  auto NB = [](const std::string& t) {
    return "((qi64)(wv + ((" + t + ") >> 3) * nwv) * PART_CH + (qi64)((" + t + ") & 7) * 256)";
  };
  // QE_PAGG_WALK=2: two record buffers, each consumed in place and reloaded only after its step's
  // LDS work. With one buffer (default) the step first copies the buffer out so that the next
  // step's loads can target it, and the ISA shows each copy waiting for all of the wave's
  // outstanding loads (in-order vmcnt). Measured anyway (1B rows, 8K / 64K / 1M groups, one box):
  // two buffers 8.07 / 8.68 / 14.23 ms, one 7.98 / 8.57 / 14.04: sixteen waves per CU hide it.
  auto body2 = [&](const std::string& pre, const std::string& nb) {
    o << "    {\n    const qi64 sbase = " << pre << "pb;\n"
      << "    const qu32 act = " << pre << "act;\n    qu32 knull = 0;\n"
      << "    qi64 (&key)[4] = " << pre << "key;\n";
    for (int q = 1; q < L.words; ++q) o << "    qi64 (&w" << q << ")[4] = " << pre << "w" << q << ";\n";
    if (L.flags_word >= 0)
      o << "#pragma unroll\n    for (int r = 0; r < 4; ++r) knull |= (qu32)(w" << L.flags_word << "[r] & 1) << r;\n";
    for (int c = 0; c < P.ncols; ++c) {
      if (L.col_word[c] < 0) continue;
      const std::string cs = std::to_string(c);
      o << "    qi64 (&c" << cs << ")[4] = w" << L.col_word[c] << ";\n";
      if (P.cols[c].valid)
        o << "    qu32 v" << cs << " = 0;\n"
          << "#pragma unroll\n    for (int r = 0; r < 4; ++r) v" << cs << " |= ((qu32)(w" << L.flags_word << "[r] >> "
          << (1 + c) << ") & 1u) << r;\n";
    }
    o << "    if (act != 0) {\n";
    emit_agg_rows(P, o, val, ok, L.row_word >= 0 ? "w" + std::to_string(L.row_word) + "[r]" : "0",
                  "sbase + lane + 64 * r");
    o << "    }\n    }\n";
    load_step(pre, nb);
  };
  if (walk && walk_lvl >= 2) {
    static_assert(PART_CH == 8 * 256, "chunk-major walk: 8 steps of 256 records per chunk");
    o << "  qu32 mact;\n  qi64 mkey[4], mpb;\n";
    for (int q = 1; q < L.words; ++q) o << "  qi64 mw" << q << "[4];\n";
    load_step("n", NB("0"));
    load_step("m", NB("1"));
    o << "  for (int t = 0;; t += 2) {\n    if (" << NB("t") << " >= hi) break;\n";
    body2("n", NB("t + 2"));
    o << "    if (" << NB("t + 1") << " >= hi) break;\n";
    body2("m", NB("t + 3"));
    o << "  }\n";
  } else if (walk) {
    load_step("n", NB("0"));
    o << "  for (int t = 0;; ++t) {\n    const qi64 base = " << NB("t") << ";\n    if (base >= hi) break;\n";
    body("n", "base", NB("t + 1"));
    o << "  }\n";
  } else if (depth == 2) {
    load_step("n", first);
    load_step("m", first + " + step");
    o << "  for (qi64 base = " << first << "; base < hi; base += 2 * step) {\n";
    body("n", "base", "base + 2 * step");
    o << "    if (base + step >= hi) break;\n";
    body("m", "base + step", "base + 3 * step");
    o << "  }\n";
  } else {
    if (pf) load_step("n", first);
    o << "  for (qi64 base = " << first << "; base < hi; base += step) {\n";
    if (!pf) load_step("n", "base");
    body("n", "base", pf ? "base + step" : "");
    o << "  }\n";
  }
  emit_flush(P, o, true, true);
  // groups that found no room anywhere: defer their records (the LDS table is final, so a key is
  // in it exactly when its records were aggregated there rather than on the global path)
  o << "  __syncthreads();\n"
    << "  if (s_fail) {\n"
    << (chunked ? "    for (qi64 v = threadIdx.x; v < hi; v += blockDim.x) {\n"
                  "      const qi64 id = P.part_sorted[clo + v / PART_CH], ko = v % PART_CH;\n"
                  "      if (ko >= (P.part_chunk[1 + id] & 0xFFFFFFFFll)) continue;\n"
                  "      const qi64 i = id * PART_CH + ko;\n"
                : "    for (qi64 i = lo + threadIdx.x; i < hi; i += blockDim.x) {\n")
    << "      if (P.defer_in && !((P.defer_in[i >> 5] >> (i & 31)) & 1)) continue;\n"
    << (L.narrow && soa ? "      const qi32* rp = (const qi32*)P.part_rec + (i / PART_CH) * (" + std::to_string(L.words) +
                              " * PART_CH) + i % PART_CH;\n"
        : L.narrow ? "      const qi32* rp = (const qi32*)(P.part_rec + i * " + std::to_string(L.bytes()) + "ull);\n"
        : soa ? "      const qi64* rp = (const qi64*)P.part_rec + (i / PART_CH) * (" + std::to_string(L.words) +
                  " * PART_CH) + i % PART_CH;\n"
            : "      const qi64* rp = (const qi64*)(P.part_rec + i * " + std::to_string(8 * L.words) + "ull);\n")
    << "      const qi64 k = rp[0];\n";
  if (L.flags_word >= 0)
    o << "      const bool kn = rp[" << L.flags_word << (soa ? " * PART_CH" : "") << "] & 1;\n";
  else
    o << "      const bool kn = false;\n";
  o << "      int s = kn ? S : (k == EMPTY_KEY ? S + 1 : -1);\n"
    << "      if (s < 0) { const qu32 hh = lds_hash((qu64)k) >> (32 - LOG2); s = s_keys[hh] == k ? (int)hh : lds_probe(s_keys, LOG2, k, hh); }\n"
    << "      if (s >= 0 && (s_cst[s] & 0x80000000u)) {\n"
    << "        atomicOr((qu32*)&P.defer_out[i >> 5], 1u << (i & 31));\n"
    << "        atomicAdd(&P.t.ctl[1], 1ull);\n      }\n    }\n  }\n"
    << "  if (threadIdx.x == 0 && s_newg) atomicAdd(&P.t.ctl[0], (qu64)s_newg);\n";
  o << "}\n";
  *src = std::string(kDevHeader) + o.str();
  return true;
}

// Fused SelectionExec -> ProjectionExec (qe_selproj.hip): one pass, order-preserving.
// Tile = 256 threads x R stripes of 256 consecutive rows (row = base + r*256 + thread, so loads
// are coalesced and (stripe, wave) chunks are in row order). Per tile: predicate -> ballots ->
// per-(stripe, wave) counts -> wave-0 exclusive scan -> decoupled look-back over the previous
// tiles' status words (flag in bits 62-63: 1 aggregate, 2 inclusive prefix) -> each selected row
// evaluates the projection programs and stores at its global position. Tile order: a persistent
// grid of resident workgroups walking the tiles statically (bounded look-back spins; a stall sets
// t.ctl[2] and the host reruns), or ids from an atomic counter, so that every predecessor of a
// waiting tile is already running (qe_selproj.hip).
// Pointers ride in the Plan's table fields: t.acc[k] output k values, t.nn[k] output k validity
// words (nullable outputs only), t.keys tile status, t.ctl[0] tile counter, t.ctl[1] total,
// t.ctl[2] stall flag, t.cap number of tiles. out_kind[k] = byte width (8, 4, 1) | 0x100 if the
// output is nullable.
// (Measured alternatives, C2 10M rows: a persistent grid pulling tiles, 73 us; a look-back
// reading 4 windows per round trip, 87 us; this one-tile-per-workgroup, one-window form, 64 us.)
// Non-temporal input loads once the inputs exceed the 256 MB MALL (QE_SELPROJ_NT=0/1 forces).
bool selproj_nt(const Plan& P) {
  const char* e = getenv("QE_SELPROJ_NT");
  if (e && *e) return e[0] == '1';
  return P.n > (64ll << 20);
}

std::string plan_shape_key(const qe_ctx* ctx, const Plan& P) {
  Plan k;
  memset(&k, 0, sizeof k);
  memcpy(&k, &P, sizeof P);
  for (int c = 0; c < QE_MAX_COLS; ++c) {
    k.cols[c].p = (const void*)(uintptr_t)(P.cols[c].p != nullptr);
    k.cols[c].valid = (const qu8*)(uintptr_t)(P.cols[c].valid != nullptr);
  }
  for (int t = 0; t < QE_MAX_TERMS; ++t) k.terms[t].lit = 0;
  for (int j = 0; j < QE_MAX_AGGS; ++j) {
    k.aggs[j].rhs_lit = 0;
    for (int t = 0; t < QE_MAX_TOKENS; ++t) k.aggs[j].tok[t].lit = 0;
  }
  memset(&k.t, 0, sizeof k.t);
  k.n = k.row_base = 0;
  k.defer_in = nullptr;
  k.defer_out = nullptr;
  k.ovf = nullptr;
  k.ovf_cap = 0;
  k.part_rec = nullptr;
  k.part_off = nullptr;
  k.part_tw = 0;
  k.part_slice = nullptr;
  k.part_chunk = nullptr;
  k.part_sorted = nullptr;
  k.mp_keep = 0;
  k.host_ctl = nullptr;
  const int32_t extra[2] = {ctx->device, use_nt() ? 1 : 0};
  return std::string((const char*)&k, sizeof k) + std::string((const char*)extra, sizeof extra);
}

// Select-project workgroup size per mode. QE_SELPROJ_BLOCK (256 / 512 / 1024) sets every mode;
// QE_SELPROJ_LB_BLOCK the look-back modes alone (persistent grid and its counter-ordered rerun),
// default 1024: one tile of 16K rows per workgroup step, one workgroup per CU (its staged output
// takes 128 KiB of LDS), so the whole 1B-row input is a quarter of the look-backs of 256-thread
// tiles. 1B rows, C2 shape: 256 threads 4.66-4.71 ms, 512 4.51-4.66, 1024 4.07-4.35 (two boxes);
// a look-back window of 128 or 256 predecessors per round trip was slower (1024 threads: 4.22 /
// 4.39 ms against 4.07; every entry of the window must have published before the sum is taken).
int selproj_block(int mode) {
  static const int all = [] {
    const char* e = getenv("QE_SELPROJ_BLOCK");
    const int b = e && *e ? atoi(e) : 0;
    return (b == 256 || b == 512 || b == 1024) ? b : 0;
  }();
  static const int lb = [] {
    const char* e = getenv("QE_SELPROJ_LB_BLOCK");
    const int b = e && *e ? atoi(e) : 1024;
    return (b == 256 || b == 512) ? b : 1024;
  }();
  if (all) return all;
  return (mode == SP_PERSIST || mode == SP_COUNTER) ? lb : 256;
}

// Look-back window per status round trip, in units of 64 predecessors (QE_SELPROJ_LBW = 1 / 2 / 4;
// default 1, the widest measured slowest).
int selproj_lbw() {
  static const int v = [] {
    const char* e = getenv("QE_SELPROJ_LBW");
    const int k = e && *e ? atoi(e) : 1;
    return (k == 2 || k == 4) ? k : 1;
  }();
  return v;
}

// LDS the staged select-project output may take (a 1024-thread tile of 16 rows per thread, one
// 8-byte output: 128 KiB, one workgroup per CU)
constexpr size_t kSelprojStageBytes = 128 * 1024;

int selproj_rows_per_thread(const Plan& P, int mode) {
  static const int env = [] {
    const char* e = getenv("QE_SELPROJ_ROWS");
    const int v = e && *e ? atoi(e) : 0;
    return (v == 2 || v == 4 || v == 8 || v == 16) ? v : 0;
  }();
  const int by_cols = env ? env : (P.ncols <= 3 ? 16 : (P.ncols <= 6 ? 8 : 4));
  // (R x waves) per-(stripe, wave) counts: at most 4 per lane of the one-wave scan
  int r = std::min(by_cols, 256 / (selproj_block(mode) / 64));
  // fewer rows per thread rather than losing the LDS-staged output (unstaged, every selected row
  // stores 8 bytes from its lane and sets its validity bit with a device-scope atomic)
  while (!env && r > 4 && (size_t)std::max(1, (int)P.naggs) * r * selproj_block(mode) * 8 > kSelprojStageBytes) r /= 2;
  return r;
}

// Software-pipelined look-back tiles (QE_SELPROJ_PIPE=1; off by default): right after a tile's
// predicate and projections are evaluated into registers, the workgroup issues the loads of its
// next tile, which are in flight during this tile's count scan, look-back and stores (8 rows per
// thread, so the two register sets fit 4-5 workgroups per CU). Measured slower at 1B rows: 5.49-
// 5.71 ms against 4.67-4.89 ms unpipelined (same box). The loads sit in front of the look-back's
// status reads in the wave's in-order load counter, so each tile publishes its prefix one memory
// latency later — and the tiles' prefix chain, not the loads, sets the pace: the inclusive
// prefix advances one look-back window (64 tiles) per status round trip.
bool selproj_pipelined() {
  static const bool v = [] {
    const char* e = getenv("QE_SELPROJ_PIPE");
    return e && e[0] == '1';
  }();
  return v;
}

int selproj_rows(const Plan& P, int mode) {
  const int r = selproj_rows_per_thread(P, mode);
  static const bool forced = getenv("QE_SELPROJ_ROWS") && *getenv("QE_SELPROJ_ROWS");
  return (!forced && selproj_pipelined() && (mode == SP_PERSIST || mode == SP_COUNTER)) ? std::min(r, 8) : r;
}

// Persistent look-back tiles that load the next tile while this one's look-back and stores run
// (QE_SELPROJ_PREFETCH, default on; 0 = off): only with staged outputs (all 8 bytes wide, so the
// column registers are dead once the rows — and nullable outputs' validity bits — sit in LDS).
bool selproj_prefetch_ok(const Plan& P, const int32_t* out_kind, int nout, int mode) {
  static const bool on = [] {
    const char* e = getenv("QE_SELPROJ_PREFETCH");
    return !(e && e[0] == '0');
  }();
  if (!on || mode != SP_PERSIST || selproj_pipelined()) return false;
  if ((size_t)nout * selproj_rows(P, mode) * selproj_block(mode) * 8 > kSelprojStageBytes) return false;
  for (int k = 0; k < nout; ++k)
    if ((out_kind[k] & 0xFF) != 8) return false;
  return true;
}

// Row of (thread, r) inside a select-project tile. Stripe map (default): stripe r is BT consecutive
// rows, thread t row t of it. Wave map (QE_SELPROJ_MAP=wave): each wave owns R x 64 consecutive
// rows, lane l row 64 r + l of them, so a thread's R loads of a column share one base address
// (immediate offsets 512 B apart): 127 instead of 141 VGPRs for C2, but 1B rows took 5.20 ms
// against 4.86 ms for the stripe map (one box, same build). The (stripe, wave) count slot follows
// the row order of the map.
bool selproj_wave_map() {
  static const bool v = [] {
    const char* e = getenv("QE_SELPROJ_MAP");
    return e && strcmp(e, "wave") == 0;
  }();
  return v;
}
// Full tiles of 8-byte columns load through a per-tile buffer descriptor (QE_SELPROJ_BUFLD, default
// 1; stripe map only): one shared 32-bit lane offset register instead of a 64-bit address per load.
bool selproj_buffer_loads() {
  static const bool v = [] {
    const char* e = getenv("QE_SELPROJ_BUFLD");
    return !(e && e[0] == '0');
  }();
  return v && !selproj_wave_map();
}
static std::string sp_row(const std::string& b) {
  return selproj_wave_map() ? b + " + w * (R * 64) + r * 64 + lane" : b + " + r * BT + t";
}
static const char* sp_cnt_idx() { return selproj_wave_map() ? "w * R + r" : "r * W + w"; }

// act (bit r: row base + r * BT + t is inside [0, n) and passes the predicate) of a
// select-project tile whose columns are loaded.
void emit_selproj_act(const Plan& P, std::ostringstream& o) {
  o << "  qu32 act = 0;\n"
    << "#pragma unroll\n  for (int r = 0; r < R; ++r) act |= (qu32)(full || " << sp_row("base") << " < P.n) << r;\n";
  std::ostringstream q;
  emit_predicate(P, q, 16);  // emits with a fixed trip count; R <= 16 and bits >= R are clear
  std::string body = q.str();
  const std::string from = "r < 16;", to = "r < R;";
  for (size_t k = body.find(from); k != std::string::npos; k = body.find(from, k)) body.replace(k, from.size(), to);
  o << body;
}

// Column loads of the select-project tile at row `b` (C expression) into <cp><slot>[R] and the
// validity bits into <vp><slot>, for the slots in `need`; `nt`: non-temporal loads.
void emit_selproj_loads(const Plan& P, std::ostringstream& o, unsigned need, bool nt, const std::string& cp,
                        const std::string& vp, const std::string& b, const std::string& ind) {
  for (int c = 0; c < P.ncols; ++c) {
    if (!((need >> c) & 1u)) continue;
    const std::string cs = std::to_string(c);
    const int kind = P.cols[c].kind;
    const char* ty = kind == K_I32 ? "qi32" : (kind == K_U8 || kind == K_BOOL) ? "qu8" : "qi64";
    o << ind << "{\n" << ind << "  const qi64 lb = " << b << ";\n" << ind << "  const bool lfull = lb + R * BT <= P.n;\n"
      << ind << "  const " << ty << "* p = (const " << ty << "*)P.cols[" << cs << "].p;\n"
      << ind << "  if (lfull) {\n";  // whole tile: R loads back to back, no per-row exec branches
    if (std::string(ty) == "qi64" && kind != K_BOOL && selproj_buffer_loads())
      o << ind << "    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p + lb), (short)0, "
        << "(int)(R * BT * 8), 0x00020000);\n";
    o
      << "#pragma unroll\n" << ind << "    for (int r = 0; r < R; ++r) {\n" << ind << "      const qi64 row = " << sp_row("lb") << ";\n";
    if (kind == K_BOOL)
      o << ind << "      " << cp << cs << "[r] = (p[row >> 3] >> (row & 7)) & 1;\n";
    else if (std::string(ty) == "qi64" && selproj_buffer_loads())
      // 8-byte column, stripe map: buffer loads off a per-tile descriptor (tile base in SGPRs), so
      // all R loads share one 32-bit lane offset instead of a 64-bit address register each
      o << ind << "      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)t * 8, r * BT * 8, " << (nt ? 2 : 0)
        << ");\n" << ind << "      " << cp << cs << "[r] = (qi64)(((qu64)v[1] << 32) | (qu64)v[0]);\n";
    else
      // default policy below 64M rows: C2-sized inputs stay in the MALL (nt 68.4 us, default 65.0 us)
      o << ind << "      " << cp << cs << "[r] = (qi64)" << ld(ty, "p + row", nt) << ";\n";
    o << ind << "    }\n" << ind << "  } else {\n"
      << "#pragma unroll\n" << ind << "    for (int r = 0; r < R; ++r) {\n" << ind << "      const qi64 row = " << sp_row("lb") << ";\n";
    if (kind == K_BOOL)
      o << ind << "      " << cp << cs << "[r] = row < P.n ? ((p[row >> 3] >> (row & 7)) & 1) : 0;\n";
    else
      o << ind << "      " << cp << cs << "[r] = row < P.n ? (qi64)" << ld(ty, "p + row", nt) << " : 0;\n";
    o << ind << "    }\n" << ind << "  }\n";
    if (P.cols[c].valid) {
      o << ind << "  const qu8* vb = P.cols[" << cs << "].valid;\n" << ind << "  " << vp << cs << " = 0;\n"
        << "#pragma unroll\n" << ind << "  for (int r = 0; r < R; ++r) {\n" << ind << "    const qi64 row = " << sp_row("lb") << ";\n"
        << ind << "    if (lfull || row < P.n) " << vp << cs << " |= (qu32)((vb[row >> 3] >> (row & 7)) & 1) << r;\n"
        << ind << "  }\n";
    }
    o << ind << "}\n";
  }
}

// Write phase of one select-project tile, after the caller's code has loaded the tile's columns
// (c<slot>[R], v<slot>) and computed `act` (bit r: row base + r * BT + t is selected): ballots,
// per-(stripe, wave) counts, one wave's scan, the tile's output base (decoupled look-back or the
// two-pass prefix), then the compacted stores.
bool emit_selproj_write(const Plan& P, const int32_t* out_kind, int nout, int mode, std::ostringstream& o,
                        bool regs = false, const std::string& prefetch = std::string()) {
  const int R = selproj_rows(P, mode);
  // Staged output (all outputs 8 bytes wide, R x BT x 8 B each within 64 KiB of LDS): selected
  // rows land compacted in LDS, then the tile's output range is written with 16-byte stores, all
  // lanes active. Direct 8-byte stores from the row registers were store-issue bound (half the
  // lanes idle at 50 % selectivity, 16 store instructions per thread).
  bool staged = (size_t)nout * R * selproj_block(mode) * 8 <= kSelprojStageBytes;
  for (int k = 0; k < nout; ++k) staged = staged && (out_kind[k] & 0xFF) == 8;
  std::vector<Expr> ex(nout);
  for (int k = 0; k < nout; ++k) {
    if (!agg_expr(P, k, &ex[k])) return false;
    if (regs) {  // pipelined: values and validity were evaluated into o<k>[R] / ok<k> before the prefetch
      ex[k].v = "o" + std::to_string(k) + "[r]";
      ex[k].ok = "((ok" + std::to_string(k) + " >> r) & 1u)";
    }
  }
  const bool any_null = [&] { for (int k = 0; k < nout; ++k) if (out_kind[k] & 0x100) return true; return false; }();
  if (staged && any_null)
    // the tile's output validity bits, in tile-local order (bit = compacted position), zeroed
    // behind the previous tile's last barrier
    for (int k = 0; k < nout; ++k)
      if (out_kind[k] & 0x100)
        o << "  __shared__ qu32 s_vb" << k << "[R * BT / 32 + 2];\n"
          << "  for (int i = t; i < R * BT / 32 + 2; i += BT) s_vb" << k << "[i] = 0u;\n";
  o << "  qu64 bal[R];\n"
    << "#pragma unroll\n  for (int r = 0; r < R; ++r) bal[r] = __ballot((act >> r) & 1u);\n"
    << "  if (lane == 0) {\n#pragma unroll\n    for (int r = 0; r < R; ++r) s_cnt[" << sp_cnt_idx() << "] = (qu32)__popcll(bal[r]);\n  }\n"
    << "  __syncthreads();\n"
    << "  qu64* st = (qu64*)P.t.keys;\n"
    << "  if (w == 0) {\n"
    // R x W (stripe, wave) counts, E = ceil(R W / 64) consecutive ones per lane
    << "    constexpr int E = (R * W + 63) / 64;\n"
    << "    qu32 xs[E];\n    qu32 x = 0;\n"
    << "#pragma unroll\n    for (int e = 0; e < E; ++e) { xs[e] = lane * E + e < R * W ? s_cnt[lane * E + e] : 0u; x += xs[e]; }\n"
    << "    qu32 inc = x;\n"
    << "#pragma unroll\n    for (int d = 1; d < 64; d <<= 1) { const qu32 y = __shfl_up(inc, d); if (lane >= d) inc += y; }\n"
    << "    const qu64 total = (qu64)__shfl(inc, 63);\n"
    << "    qu32 ex = inc - x;\n"
    << "#pragma unroll\n    for (int e = 0; e < E; ++e) { if (lane * E + e < R * W) s_cnt[lane * E + e] = ex; ex += xs[e]; }\n"
    << (mode == SP_WRITE || mode == SP_WRITE_SCAN ? "    if (lane == 0) s_total = (qu32)total;\n"
                         : "    if (lane == 0) { s_total = (qu32)total; __hip_atomic_store(&st[tile], (tile == 0 ? F_INC : F_AGG) | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }\n")
    << "  }\n";
  const std::string lookback = mode == SP_WRITE || mode == SP_WRITE_SCAN ?
      "    const qu64 total = s_total;\n"
      "    if (lane == 0) {\n      qu64 excl = 0;\n      for (int q = 0; q < W; ++q) excl += s_pre[q];\n      s_base = excl;\n"
      // (host_ctl[2]: the count has landed — the host polls it instead of waiting for the
      // kernel's completion signal, ~6 us sooner)
      "      if ((qu64)tile == P.t.cap - 1) { P.t.ctl[1] = excl + total; if (P.host_ctl) { __hip_atomic_store(&P.host_ctl[0], excl + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); __hip_atomic_store(&P.host_ctl[2], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM); } }\n    }\n" :
      "    const qu64 total = s_total;\n"
      "    qu64 excl = 0;\n"
      "    if (tile > 0) {\n"
      "      qi64 pos = (qi64)tile - 1;\n"
      // window of 64 x LBW predecessors per round trip: lane l reads tiles pos - (l LBW + k)
      "      for (;;) {\n"
      "        qu64 v[LBW];\n"
      "        qu32 spins = 0;\n"
      "        bool pend;\n"
      "        do {\n"
      "          pend = false;\n"
      "#pragma unroll\n"
      "          for (int k = 0; k < LBW; ++k) {\n"
      "            const qi64 idx = pos - (qi64)(lane * LBW + k);\n"
      "            v[k] = idx >= 0 ? __hip_atomic_load(&st[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : F_INC;\n"
      "            pend = pend || (v[k] >> 62) == 0;\n"
      "          }\n"
      "        } while (__any(pend) && (!PERSIST || ++spins < (1u << 20)));\n"
      // persistent grid only: a predecessor that never publishes means a workgroup was not
      // resident after all; flag it (the host reruns with counter-ordered tiles) and let every
      // wave finish instead of hanging the device
      "        if (PERSIST && spins >= (1u << 20)) { if (lane == 0) { __hip_atomic_store(&P.t.ctl[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); if (P.host_ctl) __hip_atomic_store(&P.host_ctl[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }\n"
      "#pragma unroll\n          for (int k = 0; k < LBW; ++k) v[k] = F_INC; }\n"
      "        int kp = LBW;\n"
      "#pragma unroll\n        for (int k = LBW - 1; k >= 0; --k) if ((v[k] >> 62) == 2) kp = k;\n"
      "        const qu64 incm = __ballot(kp < LBW);\n"
      "        const int first = incm ? __ffsll((long long)incm) - 1 : 64;\n"
      "        qu64 c = 0;\n"
      "#pragma unroll\n        for (int k = 0; k < LBW; ++k) if (lane < first || (lane == first && k <= kp)) c += v[k] & VMASK;\n"
      "#pragma unroll\n        for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);\n"
      "        excl += c;\n"
      "        if (incm) break;\n"
      "        pos -= 64 * LBW;\n"
      "      }\n"
      "      if (lane == 0) __hip_atomic_store(&st[tile], F_INC | (excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
      "    }\n"
      "    if (lane == 0) {\n      s_base = excl;\n"
      "      if ((qu64)tile == P.t.cap - 1) { __hip_atomic_store(&P.t.ctl[1], excl + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); if (P.host_ctl) __hip_atomic_store(&P.host_ctl[0], excl + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }\n    }\n";
  o << "  __syncthreads();\n"
    << "  const qu64 below = (1ull << lane) - 1;\n";
  if (staged) {
    // rows -> LDS at their tile-local positions (validity bits straight to the output bitmap
    // once the tile base is known), while wave 0 then runs the look-back
    o << "#pragma unroll\n  for (int r = 0; r < R; ++r) {\n"
      << "    if (!((act >> r) & 1u)) continue;\n"
      << "    const qu32 lp = s_cnt[" << sp_cnt_idx() << "] + (qu32)__popcll(bal[r] & below);\n";
    for (int k = 0; k < nout; ++k) o << "    s_out[" << k << " * (R * BT) + lp] = " << ex[k].v << ";\n";
    for (int k = 0; k < nout; ++k)
      if (out_kind[k] & 0x100) o << "    if (" << ex[k].ok << ") atomicOr(&s_vb" << k << "[lp >> 5], 1u << (lp & 31));\n";
    o << "  }\n";
    if (!prefetch.empty())
      // the tile's rows are in LDS, so its column registers are free: the next tile's loads go
      // out now and are in flight during the look-back and the stores (wave 0 issues its share
      // after the look-back, so its in-order load counter never holds the status reads back)
      o << "  asm volatile(\"\" ::: \"memory\");\n"
        << "  if (w != 0) {\n" << prefetch << "  } else {\n" << lookback << prefetch << "  }\n";
    else
      o << "  if (w == 0) {\n" << lookback << "  }\n";
    o << "  __syncthreads();\n"
      << "  {\n    const qu64 tb = s_base;\n    const qu32 tot = s_total;\n";
    for (int k = 0; k < nout; ++k) {
      const std::string ks = std::to_string(k);
      o << "    {\n      qi64* out = (qi64*)P.t.acc[" << ks << "] + tb;\n"
        << "      const qi64* so = s_out + " << ks << " * (R * BT);\n"
        << "      const qu32 mis = (qu32)(((qu64)out >> 3) & 1), head = mis < tot ? mis : tot;  // 16-byte alignment\n"
        << "      if (head && t == 0) out[0] = so[0];\n"
        << "      for (qu32 i = head + 2 * t; i + 1 < tot; i += 2 * BT) *(qi64x2*)(out + i) = qi64x2{so[i], so[i + 1]};\n"
        << "      if (t == 0 && tot > head && ((tot - head) & 1)) out[tot - 1] = so[tot - 1];\n    }\n";
    }
    if (any_null) {
      // validity words of the output range [tb, tb + tot): the words inside it belong to this tile
      // alone (plain stores); the first and last may share bits with the neighbouring tiles
      // (atomicOr into the zero-initialised bitmap)
      o << "    const qu64 w0 = tb >> 5;\n"
        << "    const qu32 nw = tot ? (qu32)(((tb + tot - 1) >> 5) - w0 + 1) : 0u;\n"
        << "    for (qu32 i = t; i < nw; i += BT) {\n"
        << "      const qi64 l0 = (qi64)((w0 + i) << 5) - (qi64)tb;  // tile-local bit of the word's bit 0\n"
        << "      const bool whole = l0 >= 0 && l0 + 32 <= (qi64)tot;\n";
      for (int k = 0; k < nout; ++k) {
        if (!(out_kind[k] & 0x100)) continue;
        const std::string ks = std::to_string(k);
        o << "      {\n        qu32 v;\n"
          << "        if (l0 < 0) v = s_vb" << ks << "[0] << (qu32)(-l0);\n"
          << "        else { const qu32 q = (qu32)l0 >> 5, sh = (qu32)l0 & 31u;\n"
          << "               v = sh ? (s_vb" << ks << "[q] >> sh) | (s_vb" << ks << "[q + 1] << (32u - sh)) : s_vb" << ks << "[q]; }\n"
          << "        qu32* vw = (qu32*)P.t.nn[" << ks << "] + (w0 + i);\n"
          << "        if (whole) *vw = v; else if (v) atomicOr(vw, v);\n      }\n";
      }
      o << "    }\n";
    }
    o << "  }\n";
  } else {
    o << "  if (w == 0) {\n" << lookback << "  }\n"
      << "  __syncthreads();\n"
      << "  const qu64 tb = s_base;\n"
      << "#pragma unroll\n  for (int r = 0; r < R; ++r) {\n"
      << "    if (!((act >> r) & 1u)) continue;\n"
      << "    const qu64 pos = tb + s_cnt[" << sp_cnt_idx() << "] + (qu64)__popcll(bal[r] & below);\n";
    for (int k = 0; k < nout; ++k) {
      const std::string ks = std::to_string(k);
      const int width = out_kind[k] & 0xFF;
      const bool nullable = (out_kind[k] & 0x100) != 0;
      o << "    {\n      const qi64 x = " << ex[k].v << ";\n";
      if (width == 8) o << "      ((qi64*)P.t.acc[" << ks << "])[pos] = x;\n";
      else if (width == 4) o << "      ((qi32*)P.t.acc[" << ks << "])[pos] = (qi32)x;\n";
      else if (width == 1) o << "      ((qu8*)P.t.acc[" << ks << "])[pos] = (qu8)x;\n";
      else return false;
      if (nullable)
        o << "      if (" << ex[k].ok << ") atomicOr(&((qu32*)P.t.nn[" << ks << "])[pos >> 5], 1u << (pos & 31));\n";
      o << "    }\n";
    }
    o << "  }\n";
  }
  return true;
}

bool gen_selproj_source(const Plan& P, const int32_t* out_kind, int nout, std::string* src, int mode) {
  if (P.ncols < 1 || P.ncols > QE_MAX_COLS || nout < 1 || nout > QE_MAX_AGGS) return false;
  const int R = selproj_rows(P, mode);
  const bool persistent = mode == SP_PERSIST;
  const bool pipe = persistent && selproj_pipelined();
  // the count pass loads only the predicate's columns
  const unsigned need = mode == SP_COUNT ? pred_key_cols(P) : ~0u;
  std::ostringstream o;
  o << "\nusing namespace qe;\n"
    << "extern \"C\" __global__ void __launch_bounds__(" << selproj_block(mode) << ") qe_selproj(const Plan P) {\n"
    << "  constexpr int R = " << R << ", BT = " << selproj_block(mode) << ", W = BT / 64, LBW = " << selproj_lbw() << ";\n"
    << "  constexpr qu64 F_AGG = 1ull << 62, F_INC = 2ull << 62, VMASK = (1ull << 62) - 1;\n"
    << "  constexpr bool PERSIST = " << (persistent ? "true" : "false") << ";\n"
    << "  __shared__ qu32 s_cnt[R * W];\n  __shared__ qu64 s_base;\n  __shared__ qu32 s_tile, s_total;\n"
    << "  __shared__ qi64 s_out[" << ((size_t)nout * R * selproj_block(mode) * 8 <= kSelprojStageBytes ? nout * R * selproj_block(mode) : 1) << "];\n"
    << "  const int t = threadIdx.x, lane = t & 63, w = t >> 6;\n";
  auto emit_loads = [&](const std::string& cp, const std::string& vp, const std::string& b, const std::string& ind) {
    emit_selproj_loads(P, o, need, selproj_nt(P), cp, vp, b, ind);
  };
  if (pipe) {
    // Persistent grid, software-pipelined: tile i+1's loads are issued once tile i's predicate
    // and projections sit in registers (o<k>[R], ok<k>), and are in flight during tile i's count
    // scan, look-back and stores. The asm fence keeps the compiler from sinking the projections
    // below the loads (which would hold both tiles' columns live).
    for (int c = 0; c < P.ncols; ++c) {
      o << "  qi64 c" << c << "[R];\n";
      if (P.cols[c].valid) o << "  qu32 v" << c << " = 0;\n";
    }
    o << "  qu32 tile = blockIdx.x;\n  if ((qu64)tile < P.t.cap) {\n    const qi64 base0 = (qi64)tile * (R * BT);\n";
    emit_loads("c", "v", "base0", "    ");
    o << "  }\n  while ((qu64)tile < P.t.cap) {\n"
      << "  const qu32 next = tile + gridDim.x;\n"
      << "  const qi64 base = (qi64)tile * (R * BT);\n"
      << "  const bool full = base + R * BT <= P.n;\n";
    emit_selproj_act(P, o);
    std::vector<Expr> ex(nout);
    for (int k = 0; k < nout; ++k)
      if (!agg_expr(P, k, &ex[k])) return false;
    for (int k = 0; k < nout; ++k) {
      const std::string ks = std::to_string(k);
      o << "  qi64 o" << ks << "[R];\n  qu32 ok" << ks << " = 0;\n"
        << "#pragma unroll\n  for (int r = 0; r < R; ++r) { o" << ks << "[r] = " << ex[k].v << "; ok" << ks
        << " |= (qu32)(" << ex[k].ok << ") << r; }\n"
        << "#pragma unroll\n  for (int r = 0; r < R; ++r) asm volatile(\"\" :: \"v\"(o" << ks << "[r]) : \"memory\");\n";
    }
    o << "  if ((qu64)next < P.t.cap) {\n    const qi64 nbase = (qi64)next * (R * BT);\n";
    emit_loads("c", "v", "nbase", "    ");
    o << "  }\n";
    if (!emit_selproj_write(P, out_kind, nout, mode, o, true)) return false;
    o << "  __syncthreads();\n  tile = next;\n  }\n}\n";
    *src = std::string(kDevHeader) + o.str();
    return true;
  }
  if (persistent && selproj_prefetch_ok(P, out_kind, nout, mode)) {
    // Persistent grid, next tile's columns loaded into the (then free) column registers once this
    // tile's rows are staged in LDS (emit_selproj_write): with one 1024-thread workgroup per CU
    // nothing else on the CU would keep HBM busy during the look-back and the stores.
    for (int c = 0; c < P.ncols; ++c) {
      o << "  qi64 c" << c << "[R];\n";
      if (P.cols[c].valid) o << "  qu32 v" << c << " = 0;\n";
    }
    o << "  qu32 tile = blockIdx.x;\n  if ((qu64)tile < P.t.cap) {\n    const qi64 base0 = (qi64)tile * (R * BT);\n";
    emit_loads("c", "v", "base0", "    ");
    o << "  }\n  while ((qu64)tile < P.t.cap) {\n"
      << "  const qu32 next = tile + gridDim.x;\n"
      << "  const qi64 base = (qi64)tile * (R * BT);\n"
      << "  const bool full = base + R * BT <= P.n;\n";
    emit_selproj_act(P, o);
    std::ostringstream pf;
    pf << "    if ((qu64)next < P.t.cap) {\n      const qi64 nbase = (qi64)next * (R * BT);\n";
    emit_selproj_loads(P, pf, need, selproj_nt(P), "c", "v", "nbase", "      ");
    pf << "    }\n";
    if (!emit_selproj_write(P, out_kind, nout, mode, o, false, pf.str())) return false;
    o << "  __syncthreads();\n  tile = next;\n  }\n}\n";
    *src = std::string(kDevHeader) + o.str();
    return true;
  }
  if (persistent) {
    // Every workgroup is resident (grid <= CUs x occupancy), so a static tile order cannot
    // deadlock the look-back and no tile counter is needed. (Prefetching the next tile's columns
    // into registers during this tile's look-back measured slower with 256-thread workgroups,
    // 4 per CU: 5.00 vs 4.67 ms at 1B rows; see selproj_prefetch_ok for 1024-thread ones.)
    o << "  for (qu32 tile = blockIdx.x; (qu64)tile < P.t.cap; tile += gridDim.x) {\n"
      << "  const qi64 base = (qi64)tile * (R * BT);\n"
      << "  const bool full = base + R * BT <= P.n;\n";
    for (int c = 0; c < P.ncols; ++c) {
      o << "  qi64 c" << c << "[R];\n";
      if (P.cols[c].valid) o << "  qu32 v" << c << " = 0;\n";
    }
    emit_loads("c", "v", "base", "  ");
  } else {
    if (mode == SP_COUNTER)
      o << "  {\n  if (t == 0) s_tile = (qu32)atomicAdd((unsigned long long*)&P.t.ctl[0], 1ull);\n"
        << "  __syncthreads();\n"
        << "  const qu32 tile = s_tile;\n";
    else  // two-pass: one tile per workgroup in grid order
      o << "  {\n  const qu32 tile = blockIdx.x;\n";
    o << "  const qi64 base = (qi64)tile * (R * BT);\n"
      << "  const bool full = base + R * BT <= P.n;\n";
    for (int c = 0; c < P.ncols; ++c) {
      if (!((need >> c) & 1u)) continue;
      o << "  qi64 c" << c << "[R];\n";
      if (P.cols[c].valid) o << "  qu32 v" << c << " = 0;\n";
    }
    emit_loads("c", "v", "base", "  ");
    if (mode == SP_WRITE)
      // this tile's base: the earlier tiles' counts, summed by the whole workgroup while its
      // column loads are in flight
      o << "  qu64 pre = 0;\n"
        << "  for (qi64 i = t; i < (qi64)tile; i += BT) pre += ((const qu64*)P.t.keys)[i];\n"
        << "#pragma unroll\n  for (int d = 32; d >= 1; d >>= 1) pre += __shfl_xor(pre, d);\n"
        << "  __shared__ qu64 s_pre[W];\n  if (lane == 0) s_pre[w] = pre;\n";
    else if (mode == SP_WRITE_SCAN)  // base from the scanned counts
      o << "  __shared__ qu64 s_pre[W];\n"
        << "  if (lane == 0) s_pre[w] = w == 0 ? ((const qu64*)P.t.keys)[tile] : 0ull;\n";
  }
  emit_selproj_act(P, o);
  if (mode == SP_COUNT) {
    o << "  qu32 n = __popc(act);\n"
      << "#pragma unroll\n  for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d);\n"
      << "  if (lane == 0) s_cnt[w] = n;\n  __syncthreads();\n"
      << "  if (t == 0) { qu64 c = 0; for (int q = 0; q < W; ++q) c += s_cnt[q]; ((qu64*)P.t.keys)[tile] = c; }\n"
      << "  }\n}\n";
    *src = std::string(kDevHeader) + o.str();
    return true;
  }
  if (!emit_selproj_write(P, out_kind, nout, mode, o)) return false;
  if (persistent) o << "  __syncthreads();\n";  // s_cnt / s_base are reused by the next tile
  o << "  }\n}\n";
  *src = std::string(kDevHeader) + o.str();
  return true;
}

// ---- register-resident select-project (SP_RESIDENT) ---------------------------------------------------
// One pass for batches up to ~10M rows per predicate column (C2: filter(a > 2^19) + project(a + b),
// 10M int64, K:589-594). Workgroup w of at most one per CU owns rows [w R BT, (w + 1) R BT): it loads
// its predicate columns (R values per thread, stripe map: row = base + r BT + t) and keeps them in
// registers, counts its selected rows per (stripe, wave), publishes its total, and sums the totals
// of the workgroups before it (epoch-tagged status words, so the buffer needs no memset per call).
// Only then does it load the columns the outputs alone read, stage each group of GS stripes'
// compacted outputs in LDS and write them with 16-byte stores. Against the two passes it replaces
// (count pass over the predicate's columns, then the write pass re-reading them from the MALL) the
// predicate columns cross HBM once and there is one launch. A workgroup waits only for lower ids,
// which the in-order dispatcher placed first, so nothing depends on every workgroup being resident.
namespace {
constexpr int kResBlock = 1024, kResMaxRegs = 96;  // predicate values held: <= 96 VGPRs per thread
bool sp_resident_env() {
  static const bool v = [] {
    const char* e = getenv("QE_SELPROJ_RESIDENT");
    return !(e && e[0] == '0');
  }();
  return v;
}
// QE_SELPROJ_RESIDENT_TEST_STALL=1 (tests only): the last tile reports a stall, so the host's
// rerun path runs (tests/test_selproj.py::test_resident_stall_reruns)
bool sp_resident_test_stall() {
  static const bool v = [] {
    const char* e = getenv("QE_SELPROJ_RESIDENT_TEST_STALL");
    return e && e[0] == '1';
  }();
  return v;
}
// slots read by the outputs' programs
unsigned out_cols(const Plan& P, int nout) {
  unsigned m = 0;
  for (int k = 0; k < nout; ++k)
    for (int t = 0; t < P.aggs[k].ntok; ++t)
      if (P.aggs[k].tok[t].op == T_COL) m |= 1u << P.aggs[k].tok[t].arg;
  return m;
}
}  // namespace

int selproj_resident_rows(const Plan& P, const int32_t* out_kind, int nout, int64_t n, int cus) {
  if (!sp_resident_env() || selproj_wave_map() || n <= 0 || cus <= 0 || nout < 1 || nout > 2) return 0;
  const unsigned pred = pred_key_cols(P), used = pred | out_cols(P, nout);
  int npred = 0;
  for (int c = 0; c < P.ncols; ++c) {
    if (!((used >> c) & 1u)) continue;
    if (P.cols[c].valid) return 0;  // (nullable inputs: the look-back and two-pass kernels)
    const int k = P.cols[c].kind;
    if (k != K_I64 && k != K_F64 && k != K_I32) return 0;
    if ((pred >> c) & 1u) ++npred;
  }
  for (int k = 0; k < nout; ++k)
    if ((out_kind[k] & 0x100) || (out_kind[k] & 0xFF) != 8) return 0;
  const int64_t per = (int64_t)cus * kResBlock;
  int R = (int)((n + per - 1) / per);
  R = (R + 3) & ~3;  // (a few kernel shapes cover every size)
  // larger batches: several rounds of tiles (QE_SELPROJ_RESIDENT_ROUNDS=1; opt-in)
  static const bool rounds = [] {
    const char* e = getenv("QE_SELPROJ_RESIDENT_ROUNDS");
    return e && e[0] == '1';
  }();
  if (R > 48 && rounds) R = 32;
  if (R > 48 || (int64_t)std::max(1, npred) * R * 2 > kResMaxRegs) return 0;
  return R;
}

// Polls status words (4 per lane, in v0..v3: word i = lane + 64 k is `addr(i)`, taking part when
// `part(i)`; "@" stands for i) until all carry this call's tag; `flag` = true if it gave up (bounded
// spins). Scalars, not an array: an array passed to a helper went to scratch.
static std::string poll_code(const std::string& addr, const std::string& part, const std::string& flag) {
  auto sub = [](std::string e, int k) {
    const std::string i = "(lane + " + std::to_string(64 * k) + ")";
    for (size_t p = e.find('@'); p != std::string::npos; p = e.find('@', p + i.size())) e.replace(p, 1, i);
    return e;
  };
  std::string o;
  o += "    {\n";
  for (int k = 0; k < 4; ++k) o += "      v" + std::to_string(k) + " = (" + sub(part, k) + ") ? 0ull : tag;\n";
  o += "      " + flag + " = false;\n";
  o += "      for (qu32 spins = 0;; ++spins) {\n        bool pend = false;\n";
  for (int k = 0; k < 4; ++k) {
    const std::string v = "v" + std::to_string(k);
    o += "        if ((" + v + " & ~VMASK) != tag) { " + v + " = __hip_atomic_load(&" + sub(addr, k) +
         ", __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); pend = pend || (" + v + " & ~VMASK) != tag; }\n";
  }
  o += "        if (!__any(pend)) break;\n";
  o += "        if (spins >= (1u << 22)) { " + flag + " = true; break; }  // (bounded: see the host's stall check)\n";
  o += "        __builtin_amdgcn_s_sleep(1);\n      }\n    }\n";
  return o;
}

bool gen_selproj_resident_source(const Plan& P, const int32_t* out_kind, int nout, int rows, std::string* src) {
  // rows: R (rows per thread) | 0x100 when the workgroups walk several rounds of tiles
  const int R = rows & 0xFF;
  const bool multi = (rows & 0x100) != 0;
  if (R < 4 || R > 48 || (R & 3)) return false;
  const unsigned pred = pred_key_cols(P), rest = out_cols(P, nout) & ~pred;
  std::vector<Expr> ex(nout);
  for (int k = 0; k < nout; ++k)
    if (!agg_expr(P, k, &ex[k])) return false;
  const int GS = std::min(R, 8);  // stripes per staged output group (<= 128 KiB of LDS; their loads in flight)
  std::ostringstream o;
  o << "\nusing namespace qe;\n"
    << "extern \"C\" __global__ void __launch_bounds__(" << kResBlock << ") qe_selproj(const Plan P) {\n"
    << "  constexpr int R = " << R << ", BT = " << kResBlock << ", W = BT / 64, GS = " << GS << ";\n"
    << "  constexpr qu64 VMASK = (1ull << 40) - 1;\n"
    << "  __shared__ qu32 s_cnt[R * W + 1];\n  __shared__ qu64 s_base;\n  __shared__ qu32 s_total;\n"
    << "  __shared__ __attribute__((aligned(16))) qi64 s_out[" << nout << " * GS * BT];\n"
    << "  const int t = threadIdx.x, lane = t & 63, w = t >> 6;\n"
    << "  const qu64 tag = P.mp_keep << 40;  // this call's epoch\n"
    << "  qu64* st = (qu64*)P.t.keys;  // [0, 256): per workgroup, its tiles' prefixes taken (bit 0: a stall); [256, ...): tile totals\n"
    << "  const qu32 bid = blockIdx.x, G = gridDim.x;\n"
    << "  const qu64 ntiles = P.t.cap;\n"
    << "  qu64 pre_prev = 0;  // (wave 0) this workgroup's previous tile's prefix\n"
    << "  bool stalled_any = false;\n"
    // tile T = round * G + workgroup; its prefix = the same workgroup's previous tile's prefix + the
    // totals of the G tiles just before T (one far round trip when they are all there)
    << (multi ? "  for (qu32 T = bid; T < ntiles; T += G) {\n" : "  {\n  const qu32 T = bid;\n")
    << "  const qi64 base = (qi64)T * (R * BT);\n"
    << "  const bool full = base + R * BT <= P.n;\n";
  auto loads = [&](unsigned need, const std::string& r0, const std::string& r1, const std::string& ind) {
    for (int c = 0; c < P.ncols; ++c) {
      if (!((need >> c) & 1u)) continue;
      const std::string cs = std::to_string(c);
      const bool i32 = P.cols[c].kind == K_I32;
      const char* ty = i32 ? "qi32" : "qi64";
      const int wd = i32 ? 4 : 8;
      // buffer loads off a per-workgroup descriptor whose size is the workgroup's rows: the stripe
      // offset sits in the instruction's scalar offset (a global load's 13-bit immediate cannot
      // reach r * 8 KiB, so each of the R loads in flight would hold a 64-bit address: spilled),
      // and rows past the batch's end read as 0 (the hardware range check; `act` masks them)
      o << ind << "{\n"
        << ind << "  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)((const " << ty
        << "*)P.cols[" << cs << "].p + base), (short)0, nrec * " << wd << ", 0x00020000);\n"
        << "#pragma unroll\n" << ind << "  for (int r = " << r0 << "; r < " << r1 << "; ++r) {\n";
      if (i32)
        o << ind << "    c" << cs << "[r] = (qi64)(qi32)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)t * 4, r * BT * 4, 0);\n";
      else
        o << ind << "    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)t * 8, r * BT * 8, 0);\n"
          << ind << "    c" << cs << "[r] = (qi64)(((qu64)v[1] << 32) | (qu64)v[0]);\n";
      o << ind << "  }\n" << ind << "}\n";
    }
  };
  o << "  const int nrec = (int)(P.n - base < (qi64)(R * BT) ? P.n - base : (qi64)(R * BT));  // rows of this workgroup\n";
  for (int c = 0; c < P.ncols; ++c)
    if (((pred | rest) >> c) & 1u) o << "  qi64 c" << c << "[R];\n";
  loads(pred, "0", "R", "  ");
  // act: bit r = row base + r BT + t is in range and selected (64-bit: R may exceed 32)
  {
    std::ostringstream q;
    emit_predicate(P, q, 16);
    std::string body = q.str();
    auto repl = [&](const std::string& from, const std::string& to) {
      for (size_t k = body.find(from); k != std::string::npos; k = body.find(from, k + to.size())) body.replace(k, from.size(), to);
    };
    repl("r < 16;", "r < R;");
    repl("~(1u << r)", "~(1ull << r)");
    o << "  qu64 act = 0;\n"
      << "#pragma unroll\n  for (int r = 0; r < R; ++r) act |= (qu64)(full || base + r * BT + t < P.n) << r;\n"
      << body;
  }
  o << "#pragma unroll\n  for (int r = 0; r < R; ++r) {\n"
    << "    const qu64 b = __ballot((act >> r) & 1u);\n    if (lane == 0) s_cnt[r * W + w] = (qu32)__popcll(b);\n  }\n"
    << "  __syncthreads();\n"
    // wave 0: exclusive scan of the R x W counts (stripe-major: row order), the workgroup's total,
    // its status word, and the sum of the lower workgroups' totals
    << "  if (w == 0) {\n"
    << "    constexpr int E = (R * W + 63) / 64;\n"
    // (the lane's E counts are read twice from LDS rather than held: this kernel has no registers to spare)
    << "    qu32 x = 0;\n"
    << "#pragma unroll\n    for (int e = 0; e < E; ++e) x += lane * E + e < R * W ? s_cnt[lane * E + e] : 0u;\n"
    << "    qu32 inc = x;\n"
    << "#pragma unroll\n    for (int d = 1; d < 64; d <<= 1) { const qu32 y = __shfl_up(inc, d); if (lane >= d) inc += y; }\n"
    << "    const qu64 total = (qu64)__shfl(inc, 63);\n"
    << "    qu32 ex = inc - x;\n"
    << "#pragma unroll\n    for (int e = 0; e < E; ++e) { if (lane * E + e < R * W) { const qu32 c = s_cnt[lane * E + e]; s_cnt[lane * E + e] = ex; ex += c; } }\n"
    << "    if (lane == 0) s_cnt[R * W] = (qu32)total;\n"
    << "    if (lane == 0) __hip_atomic_store(&st[256 + T], tag | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
    // the G tiles before T (window word i: tile T - G + i), 4 per lane, polled together
    << "    const qi64 w0 = (qi64)T - (qi64)G;\n"
    << "    qu64 v0, v1, v2, v3;\n"
    << "    bool stalled;\n"
    << poll_code("st[256 + w0 + @]", "@ < G && w0 + @ >= 0", "stalled")
    << "    qu64 pre = 0;\n"
    << "    pre += (lane < G && w0 + lane >= 0 ? (v0 & VMASK) : 0ull) + (lane + 64 < G && w0 + lane + 64 >= 0 ? (v1 & VMASK) : 0ull) +\n"
    << "           (lane + 128 < G && w0 + lane + 128 >= 0 ? (v2 & VMASK) : 0ull) + (lane + 192 < G && w0 + lane + 192 >= 0 ? (v3 & VMASK) : 0ull);\n"
    << "#pragma unroll\n    for (int d = 32; d >= 1; d >>= 1) pre += __shfl_xor(pre, d);\n"
    << "    pre += pre_prev;\n    pre_prev = pre;\n"
    << "    stalled_any = stalled_any || __any(stalled);\n"
    << "    if (lane == 0) { s_base = pre; s_total = (qu32)total; }\n"
    // this workgroup's last tile has its prefix: say so now, not after its stores, so the last tile
    // can publish the count as soon as every workgroup is past its prefix
    << "    if (lane == 0 && (qu64)T + G >= ntiles) __hip_atomic_store(&st[bid], tag | (stalled_any ? 1ull : 0ull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
    // the last tile publishes the row count once every other workgroup has taken all its tiles'
    // prefixes, with the stall flag first if any gave up waiting (rows misplaced: the host reruns)
    << "    if (T == ntiles - 1) {\n"
    << "      bool bad;\n" << poll_code("st[@]", "@ < G && @ != bid", "bad")
    << "      bad = bad || (lane < G && lane != bid && (v0 & 1)) || (lane + 64 < G && lane + 64 != bid && (v1 & 1)) ||\n"
    << "            (lane + 128 < G && lane + 128 != bid && (v2 & 1)) || (lane + 192 < G && lane + 192 != bid && (v3 & 1));\n"
    << "      bad = __any(bad) || stalled_any" << (sp_resident_test_stall() ? " || true" : "") << ";\n"
    << "      if (lane == 0) {\n"
    << "        if (bad) { __hip_atomic_store(&P.t.ctl[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); if (P.host_ctl) __hip_atomic_store(&P.host_ctl[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }\n"
    << "        P.t.ctl[1] = pre + total;\n"
    << "        if (P.host_ctl) { __hip_atomic_store(&P.host_ctl[0], pre + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); "
    << "__hip_atomic_store(&P.host_ctl[2], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM); }\n"
    << "      }\n    }\n  }\n"
    << "  __syncthreads();\n"
    << "  const qu64 tb = s_base;\n  const qu64 below = (1ull << lane) - 1;\n";
  // output groups of GS stripes: load the outputs' other columns, stage compacted, store
  for (int g0 = 0; g0 < R; g0 += GS) {
    const int g1 = std::min(R, g0 + GS);
    const std::string G0 = std::to_string(g0), G1 = std::to_string(g1);
    o << "  {\n";
    loads(rest, G0, G1, "    ");
    o << "    const qu32 gb = s_cnt[" << g0 << " * W];\n"
      << "    const qu32 ge = " << (g1 < R ? "s_cnt[" + G1 + " * W]" : std::string("s_total")) << ";\n"
      << "#pragma unroll\n    for (int r = " << g0 << "; r < " << g1 << "; ++r) {\n"
      << "      const qu64 b = __ballot((act >> r) & 1u);\n"
      << "      if (!((act >> r) & 1u)) continue;\n"
      << "      const qu32 lp = s_cnt[r * W + w] - gb + (qu32)__popcll(b & below);\n";
    for (int k = 0; k < nout; ++k) o << "      s_out[" << k << " * GS * BT + lp] = " << ex[k].v << ";\n";
    o << "    }\n    __syncthreads();\n"
      << "    const qu32 tot = ge - gb;\n";
    for (int k = 0; k < nout; ++k) {
      const std::string ks = std::to_string(k);
      o << "    {\n      qi64* out = (qi64*)P.t.acc[" << ks << "] + tb + gb;\n"
        << "      const qi64* so = s_out + " << ks << " * GS * BT;\n"
        << "      const qu32 mis = (qu32)(((qu64)out >> 3) & 1), head = mis < tot ? mis : tot;  // 16-byte alignment\n"
        << "      if (head && t == 0) out[0] = so[0];\n"
        << "      for (qu32 i = head + 2 * t; i + 1 < tot; i += 2 * BT) *(qi64x2*)(out + i) = qi64x2{so[i], so[i + 1]};\n"
        << "      if (t == 0 && tot > head && ((tot - head) & 1)) out[tot - 1] = so[tot - 1];\n    }\n";
    }
    o << "    __syncthreads();\n  }\n";
  }
  o << "  }  // tiles\n"
    << "}\n";
  *src = std::string(kDevHeader) + o.str();
  return true;
}

// ---- hipRTC compile + cache ------------------------------------------------------------------------------
namespace {

struct Entry {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  int blocks_per_cu = 0;
};

std::mutex g_mu;
std::map<std::pair<int, std::string>, Entry> g_cache;
std::map<hipFunction_t, uint64_t> g_sig;  // kernel -> fnv1a of its compile key (toolchain, options, source)

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

// On-disk cache of compiled code objects. The directory is private to the effective user:
// $QE_JIT_CACHE, else $XDG_CACHE_HOME/qe_jit, else /tmp/qe_jit_cache-<uid>; created 0700 and used
// only while it is a real directory (not a symlink) owned by this user with no group/other
// access. Returns "" (memory-only caching) otherwise, so no other local user can plant device
// code that this process would load.
std::string cache_dir() {
  static std::string dir = [] {
    std::string d;
    const char* e = getenv("QE_JIT_CACHE");
    const char* x = getenv("XDG_CACHE_HOME");
    if (e && *e) d = e;
    else if (x && *x) d = std::string(x) + "/qe_jit";
    else d = "/tmp/qe_jit_cache-" + std::to_string((long)geteuid());
    mkdir(d.c_str(), 0700);
    struct stat st;
    if (lstat(d.c_str(), &st) != 0 || !S_ISDIR(st.st_mode) || st.st_uid != geteuid() || (st.st_mode & 077) != 0)
      return std::string();
    return d;
  }();
  return dir;
}

// Entry file: magic | u64 key length | u64 code length | u64 fnv1a(code) | key text | code.
// The full key text (hipRTC version, options, kernel source) is compared on load, so a name
// collision or a stale toolchain never loads the wrong code; the code hash catches truncation.
constexpr char kMagic[8] = {'Q', 'E', 'J', 'I', 'T', 'C', 'O', '2'};

bool read_entry(const std::string& path, const std::string& key, std::vector<char>* code) {
  const int fd = open(path.c_str(), O_RDONLY | O_NOFOLLOW | O_CLOEXEC);
  if (fd < 0) return false;
  FILE* f = fdopen(fd, "rb");
  if (!f) {
    close(fd);
    return false;
  }
  struct stat st;
  bool ok = fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_uid == geteuid() && (st.st_mode & 022) == 0;
  char magic[8];
  uint64_t hdr[3] = {0, 0, 0};
  ok = ok && fread(magic, 1, 8, f) == 8 && memcmp(magic, kMagic, 8) == 0 && fread(hdr, 8, 3, f) == 3 &&
       hdr[0] == key.size() && hdr[1] > 0 && (uint64_t)st.st_size == 32 + hdr[0] + hdr[1];
  if (ok) {
    std::string k(hdr[0], '\0');
    ok = fread(&k[0], 1, hdr[0], f) == hdr[0] && k == key;
  }
  if (ok) {
    code->resize(hdr[1]);
    ok = fread(code->data(), 1, hdr[1], f) == hdr[1] &&
         fnv1a(std::string(code->data(), code->size())) == hdr[2];
  }
  fclose(f);
  return ok;
}

void write_entry(const std::string& path, const std::string& key, const std::vector<char>& code) {
  const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
  const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_NOFOLLOW | O_CLOEXEC, 0600);
  if (fd < 0) return;
  FILE* f = fdopen(fd, "wb");
  if (!f) {
    close(fd);
    remove(tmp.c_str());
    return;
  }
  const uint64_t hdr[3] = {key.size(), code.size(), fnv1a(std::string(code.data(), code.size()))};
  const bool ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(hdr, 8, 3, f) == 3 &&
                  fwrite(key.data(), 1, key.size(), f) == key.size() &&
                  fwrite(code.data(), 1, code.size(), f) == code.size();
  if (fclose(f) == 0 && ok) rename(tmp.c_str(), path.c_str());
  else remove(tmp.c_str());
}

}  // namespace

// Compiled kernel for `src` on the ctx's device (compiling / loading it on first use).
int jit_kernel(qe_ctx* ctx, const std::string& src, hipFunction_t* fn, int* blocks_per_cu, const char* kname, int block) {
  std::lock_guard<std::mutex> lk(g_mu);
  const auto key = std::make_pair(ctx->device, src);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) {
    *fn = it->second.fn;
    *blocks_per_cu = it->second.blocks_per_cu;
    return QE_OK;
  }
  hipDeviceProp_t prop;
  QE_HIP(hipGetDeviceProperties(&prop, ctx->device));
  std::string arch = prop.gcnArchName;
  const std::string opt_arch = "--offload-arch=" + arch;
  // no FMA contraction: a*b+c rounds twice, as the reference (JVM) arithmetic does
  const char* opts[] = {opt_arch.c_str(), "-O3", "-ffp-contract=off", "-munsafe-fp-atomics", "-std=c++17"};
  int rtc_major = 0, rtc_minor = 0;
  hiprtcVersion(&rtc_major, &rtc_minor);
  std::string disk_key = "hiprtc " + std::to_string(rtc_major) + "." + std::to_string(rtc_minor) + " HIP " +
                         std::to_string(HIP_VERSION) + " " + arch;
  for (const char* o : opts) disk_key += std::string(" ") + o;
  disk_key += "\n" + src;
  char name[64];
  snprintf(name, sizeof(name), "%016llx", (unsigned long long)fnv1a(disk_key));
  const std::string dir = cache_dir();
  const std::string path = dir.empty() ? std::string() : dir + "/" + name + ".co";
  if (const char* dump = getenv("QE_JIT_DUMP")) {  // kernel sources for offline ISA inspection
    if (FILE* f = fopen((std::string(dump) + "/" + kname + "_" + name + ".hip").c_str(), "w")) {
      fwrite(src.data(), 1, src.size(), f);
      fclose(f);
    }
  }
  std::vector<char> code;
  if (path.empty() || !read_entry(path, disk_key, &code)) {
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "qe_fused.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
      return fail(QE_ERR_DEVICE, "hiprtcCreateProgram failed");
    const hiprtcResult r = hiprtcCompileProgram(prog, (int)(sizeof(opts) / sizeof(opts[0])), opts);
    if (r != HIPRTC_SUCCESS) {
      size_t ls = 0;
      hiprtcGetProgramLogSize(prog, &ls);
      std::string log(ls, '\0');
      if (ls) hiprtcGetProgramLog(prog, &log[0]);
      hiprtcDestroyProgram(&prog);
      return fail(QE_ERR_DEVICE, "hipRTC compile of the fused kernel failed: %s", log.substr(0, 900).c_str());
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.resize(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    if (!path.empty()) write_entry(path, disk_key, code);
  }
  Entry e;
  QE_HIP(hipModuleLoadData(&e.mod, code.data()));
  QE_HIP(hipModuleGetFunction(&e.fn, e.mod, kname));
  int nb = 0;
  QE_HIP(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, e.fn, block, 0));
  e.blocks_per_cu = nb > 0 ? nb : 1;
  g_cache[key] = e;
  g_sig[e.fn] = fnv1a(disk_key);
  *fn = e.fn;
  *blocks_per_cu = e.blocks_per_cu;
  return QE_OK;
}

uint64_t jit_kernel_signature(hipFunction_t fn) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_sig.find(fn);
  return it == g_sig.end() ? 0 : it->second;
}

int jit_launch(qe_ctx* ctx, hipFunction_t fn, int grid, const Plan& P, int block) {
  Plan arg = P;
  size_t sz = sizeof(Plan);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &arg, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  QE_HIP(hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, 0, ctx->stream, nullptr, cfg));
  return QE_OK;
}

}  // namespace qe
