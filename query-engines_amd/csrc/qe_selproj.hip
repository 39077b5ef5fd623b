// Fused SelectionExec -> ProjectionExec: ProjectionExec.execute (Main.kt:589-594) over the
// build-defined SelectionExec, in ONE pass over the scanned columns. The
// per-family chain (qe_eval_cmp -> qe_filter_count -> qe_filter_apply -> qe_eval_arith) writes
// and re-reads a mask, the compacted inputs and synchronises the host between kernels; this
// kernel reads each input once and writes only the projected rows (HBM roofline: read
// ncols*width + write selected*out_width bytes per row).
//
// The kernel is generated per plan shape and compiled with hipRTC (qe_jit.hip gen_selproj_source);
// without hipRTC the call returns QE_ERR_UNSUPPORTED and callers run the per-family operators.
#include <stdio.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>

#include "qe_internal.hpp"

using namespace qe;

namespace {

// Kernel of one plan shape and pass, memoised on the plan's structure (plan_shape_key) plus what
// else the generator reads: output kinds, pass, rows per thread, load policy. Generating the
// source (~6 us) and looking it up in the source-keyed module cache ran on every call, two passes
// per call.
int selproj_kernel(qe_ctx* ctx, const Plan& P, const int32_t* out_kind, int nout, int mode, hipFunction_t* fn,
                   int* bpc) {
  struct Key {
    int32_t out_kind[QE_MAX_AGGS];
    int32_t nout, mode, rows, nt;
  };
  Key k;
  memset(&k, 0, sizeof k);
  for (int j = 0; j < nout; ++j) k.out_kind[j] = out_kind[j];
  k.nout = nout;
  k.mode = mode;
  k.rows = selproj_rows_per_thread(P);
  k.nt = selproj_nt(P);
  const std::string key = plan_shape_key(ctx, P) + std::string((const char*)&k, sizeof k);
  static std::mutex mu;
  static std::map<std::string, std::pair<hipFunction_t, int>> memo;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = memo.find(key);
    if (it != memo.end()) {
      *fn = it->second.first;
      *bpc = it->second.second;
      return QE_OK;
    }
  }
  std::string src;
  if (!gen_selproj_source(P, out_kind, nout, &src, mode))
    return fail(QE_ERR_UNSUPPORTED, "plan shape is outside the select-project generator");
  QE_TRY(jit_kernel(ctx, src, fn, bpc, "qe_selproj", selproj_block()));
  std::lock_guard<std::mutex> g(mu);
  memo[key] = {*fn, *bpc};
  return QE_OK;
}

// Output column type a program produces: a lone column reference keeps the column's type;
// anything else is INT64 or FLOAT64 by promotion.
int32_t program_type(const qe_column* cols, const DAgg& a, bool is_f) {
  if (a.ntok == 1 && a.tok[0].op == T_COL) return cols[a.tok[0].arg].type;
  return is_f ? QE_TYPE_FLOAT64 : QE_TYPE_INT64;
}

}  // namespace

extern "C" int qe_select_project(qe_ctx* ctx, const qe_column* cols, int32_t ncols, const qe_select_spec* spec,
                                 qe_column* outs, int64_t* out_count) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(cols && spec && outs && out_count, QE_ERR_INVALID_ARG, "null argument");
  QE_CHECK(spec->nout >= 1 && spec->nout <= QE_MAX_AGGS, QE_ERR_UNSUPPORTED, "select-project takes 1..%d outputs",
           QE_MAX_AGGS);
  Plan P;
  bool col_f64[QE_MAX_COLS];
  QE_TRY(compile_inputs(cols, ncols, spec->mask_col, spec->nterms, spec->terms, &P, col_f64));
  const int64_t n = P.n;
  int32_t out_kind[QE_MAX_AGGS];
  bool nullable[QE_MAX_AGGS];
  P.naggs = spec->nout;
  for (int k = 0; k < spec->nout; ++k) {
    bool is_f = false;
    DAgg& a = P.aggs[k];
    QE_TRY(compile_program(cols, ncols, col_f64, spec->outputs[k], k, &a, &is_f, &nullable[k]));
    const int32_t t = program_type(cols, a, is_f);
    QE_CHECK(t != QE_TYPE_BOOL, QE_ERR_UNSUPPORTED, "output %d: BOOL pass-through is not fused", k);
    QE_CHECK(outs[k].type == t, QE_ERR_INVALID_ARG, "output %d: column type %d, expression yields %d", k, outs[k].type,
             t);
    QE_CHECK(outs[k].length >= n && (outs[k].values || n == 0), QE_ERR_CAPACITY,
             "output %d: capacity %lld rows, input has %lld", k, (long long)outs[k].length, (long long)n);
    out_kind[k] = type_width(t) | ((nullable[k] && outs[k].validity) ? 0x100 : 0);
    P.t.acc[k] = (qi64*)outs[k].values;
    P.t.nn[k] = (qu64*)outs[k].validity;
  }
  if (!ctx->jit) return fail(QE_ERR_UNSUPPORTED, "fused select-project needs kernel specialisation (jit is off)");
  // Tile order: a persistent grid (every workgroup resident, tiles assigned statically) or one
  // tile per workgroup with ids from a device counter in start order (QE_SELPROJ_PERSIST=0). The
  // counter is one word every workgroup hits: ~88 returning atomics/us, a floor of 2.8 ms for
  // 1B rows in 4096-row tiles. Residency comes from the grid size alone, and the occupancy query
  // is advisory (it can over-report by a block per CU), so the persistent grid keeps at most
  // min(4, occupancy - 1) blocks per CU, and its look-back spins are bounded: a tile whose
  // predecessor never publishes flags ctl[2], and the call reruns with counter-ordered tiles.
  static const bool persist_env = [] {
    const char* e = getenv("QE_SELPROJ_PERSIST");
    return !(e && e[0] == '0');
  }();
  static const int wg_cap = [] {
    const char* e = getenv("QE_SELPROJ_WG_PER_CU");
    return e && *e ? std::max(1, atoi(e)) : 4;
  }();
  // validity: nullable outputs start all-null (the kernel sets bits); others all-valid
  auto init_validity = [&]() -> int {
    for (int k = 0; k < spec->nout; ++k) {
      if (!outs[k].validity) continue;
      const size_t vb = (size_t)div_up((uint64_t)(n > 0 ? n : 1), 32) * 4;
      QE_HIP(hipMemsetAsync(outs[k].validity, (out_kind[k] & 0x100) ? 0 : 0xFF, vb, ctx->stream));
    }
    return QE_OK;
  };
  QE_TRY(init_validity());
  *out_count = 0;
  // Two passes (count per tile, then write at the sum of the earlier tiles' counts) while the
  // predicate's columns fit the MALL, so the second pass reads them from there: no look-back
  // round trips. QE_SELPROJ_TWOPASS=0/1 forces either way.
  const char* tpe = getenv("QE_SELPROJ_TWOPASS");  // read per call: tests switch it
  const int twopass_env = tpe && *tpe ? (tpe[0] == '1' ? 1 : tpe[0] == '2' ? 2 : 0) : -1;
  unsigned pred_cols = P.mask_col >= 0 ? 1u << P.mask_col : 0u;
  for (int t = 0; t < P.nterms; ++t)
    pred_cols |= (1u << P.terms[t].lhs) | (P.terms[t].rhs >= 0 ? 1u << P.terms[t].rhs : 0u);
  size_t pred_bytes = 0;
  for (int c = 0; c < P.ncols; ++c)
    if ((pred_cols >> c) & 1u) pred_bytes += (size_t)n * std::max(1, type_width(cols[c].type));
  // (each write-pass tile sums all earlier tiles' counts, so the tile count is bounded too: a
  // plan with no predicate reads nothing in the count pass but still pays the prefix sums)
  const int64_t tiles_est = (int64_t)div_up((uint64_t)n, (uint64_t)selproj_rows_per_thread(P) * selproj_block());
  const bool twopass = twopass_env >= 0 ? twopass_env == 1 : (pred_bytes <= (96ull << 20) && tiles_est <= 4096);
  // Scanned two passes (QE_SELPROJ_TWOPASS=2): count pass, a device scan of the tile counts, then
  // the write pass reads its tile's base — no look-back chain and no per-tile prefix sums, at the
  // price of reading the predicate's columns twice.
  const bool scanned = twopass_env == 2;
  if (n > 0 && scanned) {
    const int R = selproj_rows_per_thread(P);
    const int64_t tiles = (int64_t)div_up((uint64_t)n, (uint64_t)R * selproj_block());
    QE_CHECK(tiles < (1ll << 31), QE_ERR_CAPACITY, "too many rows for one select-project call");
    void* s;
    QE_TRY(ctx_scratch(ctx, (size_t)(2 * tiles + 4) * 8, &s));
    qu64* ctl = (qu64*)s;
    qu64* cnt = ctl + 3;
    qu64* offs = cnt + tiles;  // tiles + 1 words
    P.t.ctl = ctl;
    P.t.cap = (qu64)tiles;
    void* pin;
    QE_TRY(ctx_pinned(ctx, 16, &pin));
    hipFunction_t fn;
    int bpc = 0;
    P.t.keys = (qi64*)cnt;
    QE_TRY(selproj_kernel(ctx, P, out_kind, spec->nout, SP_COUNT, &fn, &bpc));
    QE_TRY(jit_launch(ctx, fn, (int)tiles, P, selproj_block()));
    QE_TRY(launch_check("qe_selproj (count)"));
    QE_TRY(exclusive_scan_i64(ctx, (const int64_t*)cnt, (int64_t*)offs, tiles));
    P.t.keys = (qi64*)offs;
    QE_TRY(selproj_kernel(ctx, P, out_kind, spec->nout, SP_WRITE_SCAN, &fn, &bpc));
    QE_TRY(jit_launch(ctx, fn, (int)tiles, P, selproj_block()));
    QE_TRY(launch_check("qe_selproj (write)"));
    QE_HIP(hipMemcpyAsync(pin, offs + tiles, 8, hipMemcpyDeviceToHost, ctx->stream));
    QE_TRY(ctx_sync(ctx));
    *out_count = ((int64_t*)pin)[0];
  } else if (n > 0 && twopass) {
    const int R = selproj_rows_per_thread(P);
    const int64_t tiles = (int64_t)div_up((uint64_t)n, (uint64_t)R * selproj_block());
    QE_CHECK(tiles < (1ll << 31), QE_ERR_CAPACITY, "too many rows for one select-project call");
    void* s;
    QE_TRY(ctx_scratch(ctx, (size_t)(tiles + 3) * 8, &s));
    qu64* ctl = (qu64*)s;
    P.t.ctl = ctl;
    P.t.keys = (qi64*)(ctl + 3);
    P.t.cap = (qu64)tiles;
    void* pin;
    QE_TRY(ctx_pinned(ctx, 16, &pin));
    for (int mode : {SP_COUNT, SP_WRITE}) {
      hipFunction_t fn;
      int bpc = 0;
      QE_TRY(selproj_kernel(ctx, P, out_kind, spec->nout, mode, &fn, &bpc));
      QE_TRY(jit_launch(ctx, fn, (int)tiles, P, selproj_block()));
      QE_TRY(launch_check(mode == SP_COUNT ? "qe_selproj (count)" : "qe_selproj (write)"));
    }
    QE_HIP(hipMemcpyAsync(pin, ctl + 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    QE_TRY(ctx_sync(ctx));
    *out_count = ((int64_t*)pin)[0];
  } else if (n > 0) {
    const int R = selproj_rows_per_thread(P);
    const int64_t tiles = (int64_t)div_up((uint64_t)n, (uint64_t)R * selproj_block());
    QE_CHECK(tiles < (1ll << 31), QE_ERR_CAPACITY, "too many rows for one select-project call");
    const size_t sbytes = (size_t)(3 + tiles) * 8;  // ctl[3] | per tile a look-back status word
    void* s;
    QE_TRY(ctx_scratch(ctx, sbytes, &s));
    qu64* ctl = (qu64*)s;
    P.t.ctl = ctl;
    P.t.keys = (qi64*)(ctl + 3);
    P.t.cap = (qu64)tiles;
    void* pin;
    QE_TRY(ctx_pinned(ctx, 16, &pin));
    for (int attempt = 0; attempt < 2; ++attempt) {
      const bool persist = persist_env && attempt == 0;
      const int mode = persist ? SP_PERSIST : SP_COUNTER;
      hipFunction_t fn;
      int bpc = 0;
      QE_TRY(selproj_kernel(ctx, P, out_kind, spec->nout, mode, &fn, &bpc));
      // QE_SELPROJ_OVERSUB (tests only) multiplies the persistent grid past residency, to exercise
      // the bounded look-back and the rerun
      const char* ov = getenv("QE_SELPROJ_OVERSUB");
      const int oversub = ov && *ov ? std::max(1, std::min(64, atoi(ov))) : 1;
      static const int margin = [] {  // QE_SELPROJ_OCC_MARGIN: blocks per CU held back from the occupancy
        const char* e = getenv("QE_SELPROJ_OCC_MARGIN");
        return e && *e ? std::max(0, atoi(e)) : 1;
      }();
      const int per_cu = std::max(1, std::min(wg_cap, bpc - margin));
      const int64_t grid = persist ? std::min<int64_t>(tiles, (int64_t)ctx->num_cus * per_cu * oversub) : tiles;
      QE_HIP(hipMemsetAsync(s, 0, sbytes, ctx->stream));
      QE_TRY(jit_launch(ctx, fn, (int)grid, P, selproj_block()));
      QE_TRY(launch_check("qe_selproj"));
      QE_HIP(hipMemcpyAsync(pin, ctl + 1, 16, hipMemcpyDeviceToHost, ctx->stream));
      QE_TRY(ctx_sync(ctx));
      *out_count = ((int64_t*)pin)[0];
      if (((int64_t*)pin)[1] == 0) break;  // else: a persistent workgroup was not resident
      QE_CHECK(persist, QE_ERR_DEVICE, "select-project look-back did not complete");
      fprintf(stderr, "qe: select-project persistent look-back stalled (grid %lld); rerunning with counter-ordered tiles\n",
              (long long)grid);
      QE_TRY(init_validity());  // the aborted launch may have set bits anywhere
    }
  }
  for (int k = 0; k < spec->nout; ++k) outs[k].length = *out_count;
  return QE_OK;
}
