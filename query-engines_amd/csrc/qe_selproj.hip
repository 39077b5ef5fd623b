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

#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "qe_internal.hpp"

using namespace qe;

namespace {

// QE_HOST_PROFILE=1: per-stage host time of qe_select_project_async, printed at exit (tools only;
// one calling thread: the stage clock is a plain global)
struct HostProf {
  double sum[8] = {};
  long n = 0;
  bool on = [] {
    const char* e = getenv("QE_HOST_PROFILE");
    return e && e[0] == '1';
  }();
  ~HostProf() {
    if (!on || !n) return;
    fprintf(stderr, "{\"select_project_host_us\": {\"compile\": %.2f, \"alloc\": %.2f, \"kernel_lookup\": %.2f, "
            "\"launch\": %.2f, \"event\": %.2f, \"calls\": %ld}}\n", sum[1] / n, sum[2] / n, sum[3] / n, sum[4] / n, sum[5] / n, n);
  }
};
HostProf g_hprof;
inline double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double g_hp_t = 0;
inline void hprof(int stage) {
  if (!g_hprof.on) return;
  const double t = now_us();
  if (stage > 0) g_hprof.sum[stage] += t - g_hp_t;
  g_hp_t = t;
}

// Kernel of one plan shape and pass, memoised on the plan's structure (plan_shape_key) plus what
// else the generator reads: output kinds, pass, rows per thread, load policy. Generating the
// source (~6 us) and looking it up in the source-keyed module cache ran on every call, two passes
// per call.
int selproj_kernel(qe_ctx* ctx, const Plan& P, const int32_t* out_kind, int nout, int mode, hipFunction_t* fn,
                   int* bpc, int rows = 0) {
  struct Key {
    int32_t out_kind[QE_MAX_AGGS];
    int32_t nout, mode, rows, nt;
  };
  Key k;
  memset(&k, 0, sizeof k);
  for (int j = 0; j < nout; ++j) k.out_kind[j] = out_kind[j];
  k.nout = nout;
  k.mode = mode;
  k.rows = rows ? rows : selproj_rows(P, mode);
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
  if (mode == SP_RESIDENT ? !gen_selproj_resident_source(P, out_kind, nout, rows, &src)
                          : !gen_selproj_source(P, out_kind, nout, &src, mode))
    return fail(QE_ERR_UNSUPPORTED, "plan shape is outside the select-project generator");
  QE_TRY(jit_kernel(ctx, src, fn, bpc, "qe_selproj", mode == SP_RESIDENT ? 1024 : selproj_block(mode)));
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

// A queued select-project call (qe_select_project_async): the plan and outputs, and where its
// count (and the persistent look-back's stall flag) land in pinned memory behind an event.
struct qe_select_pending {
  qe_ctx* ctx = nullptr;
  Plan P;
  int32_t out_kind[QE_MAX_AGGS] = {};
  int32_t nout = 0;
  qe_column outs[QE_MAX_AGGS] = {};
  uint64_t* pin = nullptr;  // [0] count, [1] stall flag (persistent look-back)
  hipEvent_t ev = nullptr;
  bool persist = false;     // the launch was the persistent look-back grid (a stall reruns it)
  bool poll = false;        // two passes: the write pass sets pin[2] once the count is in pin[0]
  int32_t col_width[QE_MAX_COLS] = {};
};

namespace {

// validity: nullable outputs start all-null (the kernel sets bits); others all-valid
int init_validity(qe_ctx* ctx, const qe_column* outs, const int32_t* out_kind, int nout, int64_t n) {
  for (int k = 0; k < nout; ++k) {
    if (!outs[k].validity) continue;
    const size_t vb = (size_t)div_up((uint64_t)(n > 0 ? n : 1), 32) * 4;
    QE_HIP(hipMemsetAsync(outs[k].validity, (out_kind[k] & 0x100) ? 0 : 0xFF, vb, ctx->stream));
  }
  return QE_OK;
}

// Queues the kernels of one select-project over P (validity already initialised) and the copy of
// its count into pin[0] (pin[1]: 1 if a persistent look-back tile never saw its predecessor).
// `persist_ok` = false forces counter-ordered tiles (the rerun after a stall).
int launch_select(qe_ctx* ctx, Plan& P, const int32_t* col_width, const int32_t* out_kind, int nout, bool persist_ok,
                  uint64_t* pin, bool* persist_used, bool* poll, bool resident_ok = true) {
  *persist_used = false;
  *poll = false;
  const int64_t n = P.n;
  if (n == 0) return QE_OK;  // pin[] was zeroed by the caller
  // One register-resident pass (SP_RESIDENT, qe_jit.hip gen_selproj_resident_source) while every
  // workgroup's predicate columns fit its registers: ~10M rows of one 8-byte predicate column.
  // QE_SELPROJ_TWOPASS (any value) picks the other modes, QE_SELPROJ_RESIDENT=0 turns it off.
  const char* tpe0 = getenv("QE_SELPROJ_TWOPASS");
  const int rres = (resident_ok && !(tpe0 && *tpe0)) ? selproj_resident_rows(P, out_kind, nout, n, ctx->num_cus) : 0;
  // tiles of R x 1024 rows, one workgroup per CU walking them in rounds (one round up to ~12M rows)
  const int64_t rtiles = rres ? (int64_t)div_up((uint64_t)n, (uint64_t)rres * 1024) : 0;
  const int64_t rgrid = std::min<int64_t>(rtiles, ctx->num_cus);
  if (rres && rgrid <= 256) {
    // status words: 256 per-workgroup "prefixes taken" + one total per tile, epoch-tagged
    const size_t need = (size_t)(256 + rtiles) * 8;
    if (need > ctx->sp_status_bytes) {
      if (ctx->sp_status) {
        QE_HIP(hipStreamSynchronize(ctx->stream));  // (an earlier call may still read the old words)
        (void)hipFree(ctx->sp_status);
        ctx->sp_status = nullptr;
        ctx->sp_status_bytes = 0;
      }
      const size_t bytes = std::max<size_t>(need, 512 * 8);
      QE_HIP(hipMalloc(&ctx->sp_status, bytes));
      QE_HIP(hipMemsetAsync(ctx->sp_status, 0, bytes, ctx->stream));
      ctx->sp_status_bytes = bytes;
    }
    if (++ctx->sp_epoch >= (1u << 24)) {  // epoch tags are 24 bits: clear the words once per 16M calls
      QE_HIP(hipMemsetAsync(ctx->sp_status, 0, ctx->sp_status_bytes, ctx->stream));
      ctx->sp_epoch = 1;
    }
    void* s;
    QE_TRY(ctx_scratch(ctx, 3 * 8, &s));
    P.t.ctl = (qu64*)s;
    P.t.keys = (qi64*)ctx->sp_status;
    P.t.cap = (qu64)rtiles;
    P.mp_keep = ctx->sp_epoch;
    P.host_ctl = (qu64*)pin;
    hipFunction_t fn;
    int bpc = 0;
    hprof(0);
    QE_TRY(selproj_kernel(ctx, P, out_kind, nout, SP_RESIDENT, &fn, &bpc, rres | (rtiles > rgrid ? 0x100 : 0)));
    hprof(3);
    QE_TRY(jit_launch(ctx, fn, (int)rgrid, P, 1024));
    hprof(4);
    QE_TRY(launch_check("qe_selproj (resident)"));
    *poll = true;
    return QE_OK;
  }
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
    if ((pred_cols >> c) & 1u) pred_bytes += (size_t)n * std::max(1, col_width[c]);
  // (each write-pass tile sums all earlier tiles' counts, so the tile count is bounded too: a
  // plan with no predicate reads nothing in the count pass but still pays the prefix sums)
  const int R2 = selproj_rows(P, SP_COUNT);  // two-pass tiles
  const int64_t tiles2 = (int64_t)div_up((uint64_t)n, (uint64_t)R2 * selproj_block(SP_COUNT));
  const bool twopass = twopass_env >= 0 ? twopass_env == 1 : (pred_bytes <= (96ull << 20) && tiles2 <= 4096);
  // the look-back modes (persistent and its counter-ordered rerun) share one tile size
  const bool two = twopass || twopass_env == 2;
  const int R = two ? R2 : selproj_rows(P, SP_PERSIST);
  const int BT = selproj_block(two ? SP_COUNT : SP_PERSIST);  // (SP_COUNTER shares SP_PERSIST's)
  const int64_t tiles = (int64_t)div_up((uint64_t)n, (uint64_t)R * BT);
  QE_CHECK(tiles < (1ll << 31), QE_ERR_CAPACITY, "too many rows for one select-project call");
  // Scanned two passes (QE_SELPROJ_TWOPASS=2): count pass, a device scan of the tile counts, then
  // the write pass reads its tile's base — no look-back chain and no per-tile prefix sums, at the
  // price of reading the predicate's columns twice.
  const bool scanned = twopass_env == 2;
  hipFunction_t fn;
  int bpc = 0;
  if (scanned) {
    void* s;
    QE_TRY(ctx_scratch(ctx, (size_t)(2 * tiles + 4) * 8, &s));
    qu64* ctl = (qu64*)s;
    qu64* cnt = ctl + 3;
    qu64* offs = cnt + tiles;  // tiles + 1 words
    P.t.ctl = ctl;
    P.t.cap = (qu64)tiles;
    P.t.keys = (qi64*)cnt;
    QE_TRY(selproj_kernel(ctx, P, out_kind, nout, SP_COUNT, &fn, &bpc));
    QE_TRY(jit_launch(ctx, fn, (int)tiles, P, BT));
    QE_TRY(launch_check("qe_selproj (count)"));
    QE_TRY(exclusive_scan_i64(ctx, (const int64_t*)cnt, (int64_t*)offs, tiles));
    P.t.keys = (qi64*)offs;
    QE_TRY(selproj_kernel(ctx, P, out_kind, nout, SP_WRITE_SCAN, &fn, &bpc));
    QE_TRY(jit_launch(ctx, fn, (int)tiles, P, BT));
    QE_TRY(launch_check("qe_selproj (write)"));
    QE_HIP(hipMemcpyAsync(pin, offs + tiles, 8, hipMemcpyDeviceToHost, ctx->stream));
    return QE_OK;
  }
  // the kernels write the count (and the stall flag) straight into the pinned words: no copy
  // command behind them on the stream
  P.host_ctl = (qu64*)pin;
  if (twopass) {
    void* s;
    QE_TRY(ctx_scratch(ctx, (size_t)(tiles + 3) * 8, &s));
    qu64* ctl = (qu64*)s;
    P.t.ctl = ctl;
    P.t.keys = (qi64*)(ctl + 3);
    P.t.cap = (qu64)tiles;
    for (int mode : {SP_COUNT, SP_WRITE}) {
      QE_TRY(selproj_kernel(ctx, P, out_kind, nout, mode, &fn, &bpc));
      QE_TRY(jit_launch(ctx, fn, (int)tiles, P, BT));
      QE_TRY(launch_check(mode == SP_COUNT ? "qe_selproj (count)" : "qe_selproj (write)"));
    }
    *poll = true;
    return QE_OK;
  }
  const size_t sbytes = (size_t)(3 + tiles) * 8;  // ctl[3] | per tile a look-back status word
  void* s;
  QE_TRY(ctx_scratch(ctx, sbytes, &s));
  qu64* ctl = (qu64*)s;
  P.t.ctl = ctl;
  P.t.keys = (qi64*)(ctl + 3);
  P.t.cap = (qu64)tiles;
  const bool persist = persist_env && persist_ok;
  const int mode = persist ? SP_PERSIST : SP_COUNTER;
  QE_TRY(selproj_kernel(ctx, P, out_kind, nout, mode, &fn, &bpc));
  // QE_SELPROJ_OVERSUB (tests only) multiplies the persistent grid past residency, to exercise
  // the bounded look-back and the rerun
  const char* ov = getenv("QE_SELPROJ_OVERSUB");
  const int oversub = ov && *ov ? std::max(1, std::min(64, atoi(ov))) : 1;
  // QE_SELPROJ_OCC_MARGIN: blocks per CU held back from the occupancy (1B rows: margin 1 -> 2
  // workgroups per CU 4.89 ms, margin 0 -> 3 per CU 4.67 ms; a non-resident workgroup would only
  // cost the bounded-spin rerun below)
  static const int margin = [] {
    const char* e = getenv("QE_SELPROJ_OCC_MARGIN");
    return e && *e ? std::max(0, atoi(e)) : 0;
  }();
  const int per_cu = std::max(1, std::min(wg_cap, bpc - margin));
  const int64_t grid = persist ? std::min<int64_t>(tiles, (int64_t)ctx->num_cus * per_cu * oversub) : tiles;
  QE_HIP(hipMemsetAsync(s, 0, sbytes, ctx->stream));
  QE_TRY(jit_launch(ctx, fn, (int)grid, P, BT));
  QE_TRY(launch_check("qe_selproj"));
  *persist_used = persist;
  return QE_OK;
}

// Completion events of select-project calls, reused (hipEventCreate per call cost a few us of
// host time on every batch). A returned event has been synchronised on, so it is idle.
// Events of calls that returned on the polled count (their kernels may still be finishing) retire
// to g_ev_busy and are reused once hipEventQuery reports them complete.
std::mutex g_ev_mu;
std::vector<hipEvent_t> g_ev_free;
std::vector<hipEvent_t> g_ev_busy;

int event_alloc(hipEvent_t* ev) {
  {
    std::lock_guard<std::mutex> g(g_ev_mu);
    if (!g_ev_free.empty()) {
      *ev = g_ev_free.back();
      g_ev_free.pop_back();
      return QE_OK;
    }
    for (size_t i = 0; i < g_ev_busy.size(); ++i) {
      if (hipEventQuery(g_ev_busy[i]) != hipSuccess) {
        (void)hipGetLastError();  // hipErrorNotReady must not surface later
        continue;
      }
      *ev = g_ev_busy[i];
      g_ev_busy[i] = g_ev_busy.back();
      g_ev_busy.pop_back();
      return QE_OK;
    }
  }
  QE_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
  return QE_OK;
}

// idle: waited on (complete). busy: recorded, possibly still pending (polled calls). Neither: a
// failed launch, whose event the runtime retires.
void event_release(hipEvent_t ev, bool idle, bool busy = false) {
  if (!ev) return;
  std::lock_guard<std::mutex> g(g_ev_mu);
  if (idle && g_ev_free.size() < 64) g_ev_free.push_back(ev);
  else if (busy && g_ev_busy.size() < 64) g_ev_busy.push_back(ev);
  else (void)hipEventDestroy(ev);
}

void pending_free(qe_select_pending* r, bool waited = false, bool polled = false) {
  if (!r) return;
  event_release(r->ev, waited && !polled, polled);
  if (r->pin) {  // waited: the kernels that write it have completed
    if (waited) pinned_slot_free_idle(r->pin);
    else pinned_slot_free(r->pin, r->ctx->stream);
  }
  delete r;
}

}  // namespace

extern "C" {

int qe_select_project_async(qe_ctx* ctx, const qe_column* cols, int32_t ncols, const qe_select_spec* spec,
                            qe_column* outs, qe_select_pending** pending) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(cols && spec && outs && pending, QE_ERR_INVALID_ARG, "null argument");
  *pending = nullptr;
  hprof(0);
  QE_CHECK(spec->nout >= 1 && spec->nout <= QE_MAX_AGGS, QE_ERR_UNSUPPORTED, "select-project takes 1..%d outputs",
           QE_MAX_AGGS);
  std::unique_ptr<qe_select_pending> r(new qe_select_pending());
  r->ctx = ctx;
  Plan& P = r->P;
  bool col_f64[QE_MAX_COLS];
  QE_TRY(compile_inputs(cols, ncols, spec->mask_col, spec->nterms, spec->terms, &P, col_f64));
  const int64_t n = P.n;
  for (int c = 0; c < ncols && c < QE_MAX_COLS; ++c) r->col_width[c] = type_width(cols[c].type);
  bool nullable[QE_MAX_AGGS];
  P.naggs = spec->nout;
  r->nout = spec->nout;
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
    r->out_kind[k] = type_width(t) | ((nullable[k] && outs[k].validity) ? 0x100 : 0);
    P.t.acc[k] = (qi64*)outs[k].values;
    P.t.nn[k] = (qu64*)outs[k].validity;
    r->outs[k] = outs[k];
  }
  if (!ctx->jit) return fail(QE_ERR_UNSUPPORTED, "fused select-project needs kernel specialisation (jit is off)");
  hprof(1);
  QE_TRY(pinned_slot_alloc(&r->pin));
  r->pin[0] = r->pin[1] = r->pin[2] = 0;  // the slot's previous user is done with it (pinned_slot_alloc)
  QE_TRY(init_validity(ctx, outs, r->out_kind, r->nout, n));
  hprof(2);
  const int st = launch_select(ctx, P, r->col_width, r->out_kind, r->nout, true, r->pin, &r->persist, &r->poll);
  if (st != QE_OK) {
    pending_free(r.release());
    return st;
  }
  hprof(0);
  // polled calls need no completion event (the wait spins on pin[2] and, as a fallback, queries the
  // stream): one runtime call less per batch
  if (!r->poll) {
    QE_TRY(event_alloc(&r->ev));
    QE_HIP(hipEventRecord(r->ev, ctx->stream));
  }
  hprof(5);
  if (g_hprof.on) ++g_hprof.n;
  *pending = r.release();
  return QE_OK;
}

int qe_select_pending_wait(qe_select_pending* r, int64_t* out_count) {
  QE_CHECK(r && out_count, QE_ERR_INVALID_ARG, "null argument");
  qe_ctx* ctx = r->ctx;
  int st = ctx_enter(ctx);
  if (st == QE_OK && r->poll) {
    // Two passes: the write pass's last tile stores the count, then pin[2]. Polling that word
    // returns ~6 us before the kernel's completion signal would (one launch + event wait: 12.6 us,
    // + a polled pinned word instead: 6.7 us; tools/exp_sync_latency.hip). The outputs are then
    // complete in the ctx stream's order (what every later call on the ctx, and a synchronisation
    // of its stream, sees); the event is checked every ~50 us, so a failed kernel still ends the
    // wait.
    volatile uint64_t* pv = r->pin;
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; pv[2] == 0; ++i) {
      if ((i & 1023) != 0) continue;
      if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50)) continue;
      t0 = std::chrono::steady_clock::now();
      const hipError_t e = r->ev ? hipEventQuery(r->ev) : hipStreamQuery(ctx->stream);
      if (e == hipSuccess) {
        if (pv[2] == 0) st = fail(QE_ERR_DEVICE, "select-project finished without publishing its row count");
        break;
      }
      if (e != hipErrorNotReady) {
        st = fail(QE_ERR_DEVICE, "select-project kernel failed: %s", hipGetErrorString(e));
        break;
      }
      (void)hipGetLastError();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (st == QE_OK && pv[1] != 0) {
      // a resident-pass workgroup gave up waiting for a lower one's count (only if its dispatch
      // was held back for seconds): its rows may be misplaced; rerun without the resident pass
      fprintf(stderr, "qe: select-project resident pass stalled; rerunning with two passes\n");
      bool used = false, poll = false;
      st = ctx_sync(ctx);
      if (st == QE_OK) {
        r->pin[0] = r->pin[1] = r->pin[2] = 0;
        st = launch_select(ctx, r->P, r->col_width, r->out_kind, r->nout, true, r->pin, &used, &poll, false);
      }
      if (st == QE_OK) st = ctx_sync(ctx);
      if (st == QE_OK && r->pin[1] != 0) st = fail(QE_ERR_DEVICE, "select-project look-back did not complete");
    }
    if (st == QE_OK) *out_count = (int64_t)pv[0];
    // the slot's last device write (pin[2]) has landed: reusable at once; the event may be pending
    pending_free(r, st == QE_OK, true);
    return st;
  }
  if (st == QE_OK && (r->ev ? hipEventSynchronize(r->ev) : hipStreamSynchronize(ctx->stream)) != hipSuccess)
    st = fail(QE_ERR_DEVICE, "select-project event wait failed");
  if (st == QE_OK && r->pin[1] != 0) {
    // a persistent workgroup was not resident: every wave drained; rerun with counter-ordered tiles
    if (!r->persist) {
      st = fail(QE_ERR_DEVICE, "select-project look-back did not complete");
    } else {
      fprintf(stderr, "qe: select-project persistent look-back stalled; rerunning with counter-ordered tiles\n");
      bool used = false;
      r->pin[0] = r->pin[1] = 0;  // (the aborted launch has drained: the event completed)
      st = init_validity(ctx, r->outs, r->out_kind, r->nout, r->P.n);  // the aborted launch may have set bits anywhere
      bool poll = false;
      if (st == QE_OK) st = launch_select(ctx, r->P, r->col_width, r->out_kind, r->nout, false, r->pin, &used, &poll);
      if (st == QE_OK) st = ctx_sync(ctx);
      if (st == QE_OK && r->pin[1] != 0) st = fail(QE_ERR_DEVICE, "select-project look-back did not complete");
    }
  }
  if (st == QE_OK) *out_count = (int64_t)r->pin[0];
  pending_free(r, st == QE_OK);
  return st;
}

int qe_select_project(qe_ctx* ctx, const qe_column* cols, int32_t ncols, const qe_select_spec* spec,
                      qe_column* outs, int64_t* out_count) {
  QE_CHECK(out_count, QE_ERR_INVALID_ARG, "null argument");
  *out_count = 0;
  qe_select_pending* r = nullptr;
  QE_TRY(qe_select_project_async(ctx, cols, ncols, spec, outs, &r));
  QE_TRY(qe_select_pending_wait(r, out_count));
  // the count can be published before the kernel's last loads and stores retire (the resident
  // pass publishes after its final prefix; the two-pass write kernel's last tile before the
  // others finish): a synchronous call returns only once the kernels have completed, so its inputs
  // may be released and its outputs read from any stream
  QE_TRY(ctx_sync(ctx));
  for (int k = 0; k < spec->nout; ++k) outs[k].length = *out_count;
  return QE_OK;
}

}  // extern "C"
