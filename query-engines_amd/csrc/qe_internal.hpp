// Internal definitions shared by the HIP translation units of libqe_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "qe_hip.h"
#include "qe_dev.hpp"

struct qe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int num_cus = 256;
  void* scratch = nullptr;       // grow-only device scratch
  size_t scratch_bytes = 0;
  uint64_t scratch_epoch = 0;    // bumped by every ctx_scratch call (a user's contents may be gone)
  void* pinned = nullptr;        // small pinned host buffer for read-backs
  size_t pinned_bytes = 0;
  void* pinned_fg = nullptr;     // fine-grained pinned words a host polls (ctx_pinned_coherent)
  size_t pinned_fg_bytes = 0;
  int jit = 1;                   // specialise fused plans with hipRTC (qe_jit.hip)
  void* scan_tmp = nullptr;      // block sums of exclusive_scan_i64 (never aliases `scratch`)
  size_t scan_tmp_bytes = 0;
  void* ws[8] = {};              // grow-only workspace slots (CSV scan intermediates)
  size_t ws_bytes[8] = {};
  void* sp_status = nullptr;     // per-tile counts of the register-resident select-project
  size_t sp_status_bytes = 0;
  uint32_t sp_epoch = 0;         // (epoch-tagged, so no memset per call; qe_selproj.hip)
};

namespace qe {

// ---- errors ------------------------------------------------------------------------------
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();

#define QE_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t qe_e_ = (call);                                                         \
    if (qe_e_ != hipSuccess)                                                           \
      return ::qe::fail(QE_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(qe_e_)); \
  } while (0)

#define QE_CHECK(cond, code, ...)                  \
  do {                                             \
    if (!(cond)) return ::qe::fail(code, __VA_ARGS__); \
  } while (0)

#define QE_TRY(expr)           \
  do {                         \
    int qe_s_ = (expr);        \
    if (qe_s_ != QE_OK) return qe_s_; \
  } while (0)

int ctx_enter(qe_ctx* ctx);                                   // validates + hipSetDevice
// Caching device allocator (qe_runtime.hip): stream-ordered reuse of freed blocks.
int dev_alloc(qe_ctx* ctx, size_t bytes, void** out);
void dev_free(qe_ctx* ctx, void* p);
void dev_forget_stream(qe_ctx* ctx);
int dev_release(int device);
int ctx_scratch(qe_ctx* ctx, size_t bytes, void** out);       // grow-only scratch
int ctx_pinned(qe_ctx* ctx, size_t bytes, void** out);        // grow-only pinned host
int ctx_pinned_coherent(qe_ctx* ctx, size_t bytes, void** out);  // grow-only fine-grained pinned host (polled words)
int pinned_slot_alloc(uint64_t** out);                        // 64 pinned bytes (pooled)
void pinned_slot_free(uint64_t* p, hipStream_t stream);       // reusable once `stream`'s work is done
void pinned_slot_free_idle(uint64_t* p);                        // no device access pending: reusable now
// Wait for everything queued on the ctx stream (blocking; polling an event from this thread
// measured 15 us slower per finalize).
int ctx_sync(qe_ctx* ctx);
int launch_check(const char* what);                           // hipGetLastError wrapper
int ctx_workspace(qe_ctx* ctx, int slot, size_t bytes, void** out);  // grow-only, contents not kept
// Host (pageable) -> device through pinned staging with 8 host threads; synchronous (qe_arrow.hip).
int parallel_h2d_copy(qe_ctx* ctx, void* dst, const void* src, size_t n);
int parallel_h2d_file(qe_ctx* ctx, void* dst, int fd, int64_t off, size_t n);
// Per-plan kernel specialisation (qe_jit.hip).
bool gen_fused_source(const qe::Plan& P, int log2, std::string* src, size_t* lds_bytes, bool spill = false);
// Exact fp64 SUM in the specialised kernels' LDS tables: the 192-bit carry window through the per-wave
// queue. LDS words per slot beyond acc.
inline int fx_window_idx_words() { return 2; }
// compact fused LDS table (Plan.lds_compact): plan shapes it supports, bytes per slot, 32-bit MIN/MAX
bool compact_ok(const qe::Plan& P);
size_t compact_slot_bytes(const qe::Plan& P);
bool compact_acc32(const qe::Plan& P, int j);
// Radix-partitioned aggregation for group counts beyond the LDS table (qe_jit.hip).
struct PartLayout {
  int words = 0;  // record width in 8-byte words
  // colmode: the record holds the columns the aggregate programs read (col_word) and the
  // aggregation pass evaluates the programs; otherwise it holds each program's value (val_word)
  bool colmode = false;
  int val_word[QE_MAX_AGGS] = {};  // word of aggregate j's input value, -1 if it has none
  int col_word[QE_MAX_COLS] = {};  // colmode: word of column slot c, -1 if no program reads it
  int flags_word = -1;  // bit 0 null key, bit 1 + j input j valid (colmode: column c valid); -1 if nothing is nullable
  int row_word = -1;               // global row index (fp64 MIN/MAX); -1 if not needed
  bool row = false;
  // every word stored as 32 bits (sign-extended on load): Plan.part_narrow and integral words only
  bool narrow = false;
  int bytes() const { return (narrow ? 4 : 8) * words; }
};
PartLayout part_layout(const qe::Plan& P);
bool gen_part_source(const qe::Plan& P, int log2p, bool scatter, std::string* src);
// fast aggregation pass's largest table in slots (0: the plan does not take that pass)
int pagg_fast_slots(const qe::Plan& P);
// bucket_groups: expected groups per bucket (0: unknown), which sizes the fast pass's table
bool gen_pagg_source(const qe::Plan& P, int log2, std::string* src, size_t* lds_bytes, bool chunked = false,
                     bool soa = false, int64_t bucket_groups = 0);
bool part_staged_ok(const qe::Plan& P, int log2p);
int pscatter_block();
bool pscatter_wide();
int pscatter_block_for(int log2p);
int pagg_block();
bool fused_prefetch();
int fused_block(int lds_log2);
// hash-aggregate state accessors for other translation units (qe_comm.hip, qe_keyed.hip)
int hashagg_expected_groups(const qe_hashagg* h, int64_t* out);
qe_ctx* hashagg_ctx(const qe_hashagg* h);
// How the table packs its device key columns into the 64-bit group word: mode 0 no keys, 1 one
// INT64/FLOAT64 key (record word 1 = null flag), 2 narrow keys at shift with a null bit each.
struct KeyMeta {
  int32_t mode, nkeys;
  int32_t type[QE_MAX_KEYS], shift[QE_MAX_KEYS], nullbit[QE_MAX_KEYS];
  int64_t fmask[QE_MAX_KEYS];
};
struct Keyed;  // original key columns <-> device key columns (qe_keyed.hip)
struct HashaggInfo {
  qe_ctx* ctx;
  KeyMeta km;
  int32_t rec_bytes, naggs, flags;
  qe_agg_desc aggs[QE_MAX_AGGS];
  uint64_t version;  // bumped by every change of the groups (update, import, reset)
  uint64_t* ctl;     // device control words (ctl[3]: sticky error word)
  Keyed* keyed;
};
HashaggInfo hashagg_info(const qe_hashagg* h);
// The raw record / update / finalize paths (no dictionary handling), for qe_keyed.hip.
int hashagg_export_raw(qe_hashagg* h, int32_t nparts, void* dst);
int hashagg_export_counts_raw(qe_hashagg* h, int32_t nparts, int64_t* counts);
int hashagg_import_raw(qe_hashagg* h, const void* recs, int64_t nrec);
int hashagg_update_raw(qe_hashagg* h, const qe_column* dev_keys, const qe_column* agg_inputs, const qe_column* mask);
int hashagg_update_fused_raw(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec);
// keys_only: write the device key columns and skip the aggregates (out_aggs may be NULL)
int hashagg_finalize_raw(qe_hashagg* h, qe_column* dev_keys, qe_column* out_aggs, int64_t* out_groups, bool keys_only);
// qe_keyed.hip: create from the declared key types (device key list out), destroy, and the
// dictionary-keyed forms of update / fused update / finalize.
int keyed_create(qe_ctx* ctx, int32_t nkeys, const int32_t* types, int64_t expected, Keyed** out, int32_t* dev_nkeys,
                 int32_t* dev_types);
void keyed_destroy(qe_ctx* ctx, Keyed* K);
bool keyed_dict(const Keyed* K);
bool keyed_tuple(const Keyed* K);
int keyed_update(qe_hashagg* h, const qe_column* keys, const qe_column* agg_inputs, const qe_column* mask);
int keyed_update_fused(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec);
int keyed_finalize(qe_hashagg* h, qe_column* out_keys, qe_column* out_aggs, int64_t* out_groups);
// Wide codes of UTF8 values promised to be at most 7 bytes (qe_strdict.hip): a longer value sets
// bit 62 of *err (the hash aggregate's sticky ctl[3]), so the state fails its next read-back.
int strdict_encode_packed_checked(qe_ctx* ctx, const qe_column* in, qe_column* codes, unsigned long long* err);
constexpr uint64_t CTL_KEY_TOO_LONG = 1ull << 62;
bool gen_pscatter_staged_source(const qe::Plan& P, int log2p, std::string* src, bool chunked = false, bool soa = false);
bool part_static();  // chunked staged scatter: per-workgroup chunk id ranges (QE_PART_STATIC)
bool part_soa();  // chunked partition records stored chunk-columnar (QE_PART_SOA)
int jit_kernel(qe_ctx* ctx, const std::string& src, hipFunction_t* fn, int* blocks_per_cu,
               const char* name = "qe_fused", int block = 512);
int jit_launch(qe_ctx* ctx, hipFunction_t fn, int grid, const qe::Plan& P, int block = 512);
// Memo key of a plan's structure: the Plan bytes with run-time values cleared (buffer pointers
// reduced to present / absent; literals, row count and base, table, defer, overflow and partition
// fields zeroed), plus the device and the QE_NT load policy. Two plans with equal keys generate
// the same kernel source.
std::string plan_shape_key(const qe_ctx* ctx, const qe::Plan& P);
// Fused-plan compilation shared by the aggregate and select-project paths (qe_hashagg.hip).
int compile_inputs(const qe_column* cols, int32_t ncols, int32_t mask_col, int32_t nterms, const qe_pred_term* terms,
                   qe::Plan* P, bool* col_f64);
int compile_program(const qe_column* cols, int32_t ncols, const bool* col_f64, const qe_agg_program& pg, int j,
                    qe::DAgg* a, bool* is_f, bool* nullable);
// Select-project kernel source (qe_jit.hip): R rows per thread, selproj_block() threads.
// Select-project tile order / pass: SP_COUNTER (tile ids from a device counter, look-back),
// SP_PERSIST (persistent grid, look-back), SP_COUNT (two-pass, first pass: selected rows per tile
// into t.keys), SP_WRITE (two-pass, second pass: each tile's base = sum of the earlier tiles' counts),
// SP_WRITE_SCAN (second pass after a device scan of the counts: each tile's base = t.keys[tile]).
// SP_RESIDENT: one pass whose workgroups each hold their whole row range's predicate columns in
// registers (gen_selproj_resident_source).
enum { SP_COUNTER = 0, SP_PERSIST = 1, SP_COUNT = 2, SP_WRITE = 3, SP_WRITE_SCAN = 4, SP_RESIDENT = 5 };
// rows per thread of the resident pass for n rows on `cus` CUs, or 0 when the plan or size does
// not take it
int selproj_resident_rows(const qe::Plan& P, const int32_t* out_kind, int nout, int64_t n, int cus);
bool gen_selproj_resident_source(const qe::Plan& P, const int32_t* out_kind, int nout, int R, std::string* src);
bool gen_selproj_source(const qe::Plan& P, const int32_t* out_kind, int nout, std::string* src, int mode);
int selproj_block(int mode);  // select-project workgroup size of a mode (SP_*)
int selproj_rows_per_thread(const qe::Plan& P, int mode);
uint64_t jit_kernel_signature(hipFunction_t fn);  // hash of a specialised kernel's compile key (0: unknown)
bool selproj_pipelined();  // look-back modes load the next tile while this one is compacted
int selproj_rows(const qe::Plan& P, int mode);  // rows per thread of `mode`'s tiles
bool selproj_nt(const qe::Plan& P);  // non-temporal input loads (large inputs)
// Exclusive scan of n int64 on the ctx stream (one block); out[n] = total. (qe_filter.hip)
int exclusive_scan_i64(qe_ctx* ctx, const int64_t* in, int64_t* out, int64_t n);

// ---- type helpers ---------------------------------------------------------------------------
inline int type_width(int32_t t) {
  switch (t) {
    case QE_TYPE_INT64:
    case QE_TYPE_FLOAT64: return 8;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: return 4;
    case QE_TYPE_UINT8: return 1;
    default: return 0;  // BOOL (bits) / UTF8 (var)
  }
}
inline bool is_fixed(int32_t t) { return type_width(t) > 0; }
inline bool is_integral(int32_t t) {
  return t == QE_TYPE_INT64 || t == QE_TYPE_INT32 || t == QE_TYPE_DATE32 || t == QE_TYPE_UINT8;
}

inline int32_t kind_of(int32_t type) {
  switch (type) {
    case QE_TYPE_INT64: return K_I64;
    case QE_TYPE_FLOAT64: return K_F64;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: return K_I32;
    case QE_TYPE_UINT8: return K_U8;
    case QE_TYPE_BOOL: return K_BOOL;
    default: return -1;
  }
}

inline uint64_t div_up(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// ---- hashing / generator (bit-for-bit restated in oracle/gen.py) ----------------------------
constexpr uint64_t PHI64 = 0x9E3779B97F4A7C15ull;

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + PHI64;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint64_t gen_u64(uint64_t seed, uint64_t col, uint64_t row) {
  return splitmix64(seed ^ (col * PHI64) ^ row);
}

// Exclusive prefixes of a block's tile of 8 values per thread, 8 consecutive ones per thread
// (thread t holds elements 8t .. 8t + 7): a serial scan in registers, one wave scan of the thread
// totals, one across the block's NW waves. Returns the tile's total. `ws`: NW words of LDS. (A
// layout with a wave scan per row of 64 needed 8 of them and spilled its int64 form.)
template <typename T, int NW = 16>
__device__ __forceinline__ T tile_excl(const T (&v)[8], T (&ex)[8], T* ws) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ex[k] = s;
    s += v[k];
  }
  T x = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) ws[wid] = x;
  __syncthreads();
  T wp = 0, all = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wid) wp += ws[w];
    all += ws[w];
  }
  __syncthreads();  // ws is rewritten by the next tile
  const T base = wp + x - s;
#pragma unroll
  for (int k = 0; k < 8; ++k) ex[k] += base;
  return all;
}

// Element k of this thread in the tile starting at g0.
__device__ __forceinline__ int64_t tile_elem(int64_t g0, int k) { return g0 + (int64_t)threadIdx.x * 8 + k; }

// This thread's 8 uint32 of a tile: two 16-byte loads when the tile is full (p 32-byte aligned),
// else element by element with `fill` past n.
__device__ __forceinline__ void tile_load_u32(const uint32_t* __restrict__ p, int64_t g0, int64_t n, uint32_t (&v)[8],
                                              uint32_t fill = 0) {
  const int64_t e0 = g0 + (int64_t)threadIdx.x * 8;
  if (e0 + 8 <= n) {
    const uint4 a = *(const uint4*)(p + e0), b = *(const uint4*)(p + e0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = e0 + k < n ? p[e0 + k] : fill;
  }
}

}  // namespace qe
