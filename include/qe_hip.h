/*
 * qe_hip.h — C ABI of the MI355X (gfx950) columnar execution kernel for kquerydiy.
 *
 * This is the drop-in boundary for the reference's hot path: the evaluation inside the
 * physical operators of folkol/query-engines `kquerydiy/src/Main.kt` ("K:" below).
 * The Kotlin DataFrame / LogicalPlan / PhysicalPlan layers stay as they are; a JNI shim
 *  or Python ctypes (kquery/native.py) calls these entry points with plain
 * device pointers and sizes. No torch, no C++ types cross this boundary.
 *
 * Reference interfaces each entry point replaces:
 *   Expression.evaluate(RecordBatch): ColumnVector ............ K:448-450
 *     ColumnExpression (zero-copy column reference) ........... K:452-455  -> no call needed
 *     binary arithmetic / comparison / boolean / literal ...... absent in reference,
 *                                                                build-defined: qe_eval_*
 *   SelectionExec (filter) .................................... absent in reference, build-defined:
 *                                                                qe_filter_count / qe_filter_apply
 *   AggregateExpression/Accumulator, MaxAccumulator ........... K:514-562  -> qe_agg_global,
 *                                                                qe_hashagg_*
 *   HashAggregateExec.execute ................................. K:615-651  -> qe_hashagg_*
 *   main() partial -> final merge (two-phase aggregate) ....... K:1309-1325 -> qe_hashagg_export /
 *                                                                qe_hashagg_import
 *
 * Error behaviour: every entry point returns an int status (QE_OK = 0, negative = error
 * class) and sets a thread-local message readable with qe_last_error(). A JNI shim maps
 * QE_ERR_UNSUPPORTED -> IllegalStateException (K:195, K:469, K:677, K:792, K:799),
 * QE_ERR_INVALID_ARG -> IllegalArgumentException (K:49), the rest -> RuntimeException.
 *
 * Threading: re-entrant. Each qe_ctx owns one HIP stream and its scratch memory (the
 * reference calls the engine concurrently from coroutine workers, one ExecutionContext each,
 * K:1309-1313, K:1333); one ctx must not be used by two threads at once. Process-wide state,
 * each guarded by its own mutex and safe to share between ctxs and threads:
 *   - the thread-local error string (qe_last_error);
 *   - the device caching allocator (qe_runtime.hip dev_alloc/dev_free): freed blocks are kept
 *     per device and size class and reused once the freeing stream's event has completed;
 *     QE_CACHE_LIMIT_GB bounds what it keeps;
 *   - the hipRTC module cache (qe_jit.hip): one code object per (device, plan shape), loaded
 *     on first use and never unloaded for the life of the process, mirrored on disk in a
 *     per-user 0700 directory;
 *   - memo maps from plan structure to kernel (qe_selproj.hip, qe_hashagg.hip), which only
 *     grow (one entry per distinct plan shape).
 *
 * Memory: all column buffers are DEVICE pointers on the ctx's device (hipMalloc'ed or
 * torch-allocated). Layout is the Arrow columnar format: fixed-width values buffer,
 * optional LSB-first validity bitmap (NULL = no nulls), bit-packed booleans, offset 0.
 * Results are written into caller-provided device buffers; sizes are queried first.
 * Every OUTPUT validity or BOOL bitmap must be 4-byte aligned and padded to whole 32-bit
 * words (ceil(rows/32)*4 bytes): kernels write bitmaps a 32-bit word at a time, and some
 * clear the whole last word first. Arrow's recommended 64-byte buffer padding satisfies
 * this; a minimal ceil(rows/8)-byte bitmap does not. Input bitmaps need no padding.
 */
#ifndef QE_HIP_H
#define QE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QE_ABI_VERSION 1

/* ---- status codes ---------------------------------------------------------------------- */
#define QE_OK 0
#define QE_ERR_INVALID_ARG (-1)  /* IllegalArgumentException (K:49) */
#define QE_ERR_UNSUPPORTED (-2)  /* IllegalStateException / UnsupportedOperationException */
#define QE_ERR_OOM (-3)
#define QE_ERR_DEVICE (-4)       /* HIP runtime error */
#define QE_ERR_CAPACITY (-5)     /* output buffer too small */
#define QE_ERR_COMM (-6)         /* RCCL communicator / collective failure */
#define QE_NEED_EXACT 1          /* not an error: qe_agg_global_merge needs the exact round (below) */

/* ---- types ------------------------------------------------------------------------------ */
/* Arrow type ids used by this kernel. The reference knows only Float8 (fp64) and Utf8
 * (K:19-22, K:184-196); int64/int32/uint8/date32/bool are build-added. */
#define QE_TYPE_INT64 1
#define QE_TYPE_FLOAT64 2
#define QE_TYPE_BOOL 3   /* bit-packed values, LSB first */
#define QE_TYPE_UTF8 4   /* int32 offsets (length+1) + bytes */
#define QE_TYPE_INT32 5
#define QE_TYPE_UINT8 6
#define QE_TYPE_DATE32 7 /* int32 days since epoch */

/* One Arrow array (offset 0). Used for inputs and outputs.
 * max_len: UTF8 inputs only — when > 0, the producer's bound on every value's byte length
 * (qe_csv_column fills it from the parse); 0 = unknown. A hash aggregate keyed by a lone UTF8
 * column uses a bound <= 7 to encode the keys with no dictionary and no host round trip; the bound
 * is checked on the device, and a longer value fails the aggregate's next read-back (finalize,
 * num_groups) instead of grouping wrongly. Ignored for other types and for outputs. */
typedef struct qe_column {
  int32_t type;
  int32_t max_len;
  int64_t length;
  uint8_t* validity; /* device; NULL = all valid (inputs) / do not write (outputs) */
  void* values;      /* device; fixed-width values, bit-packed bools, or UTF-8 bytes */
  int32_t* offsets;  /* device; UTF-8 offsets (length+1), NULL otherwise */
} qe_column;

/* A literal (build-defined; the reference SQL has no literals).
 * `bits` holds an int64 value or the IEEE-754 bits of a double. */
typedef struct qe_scalar {
  int32_t type; /* QE_TYPE_INT64 or QE_TYPE_FLOAT64 */
  int32_t is_null;
  int64_t bits;
} qe_scalar;

/* Operand of a binary expression: a column, or a literal when `col` is NULL. */
typedef struct qe_operand {
  const qe_column* col;
  qe_scalar lit;
} qe_operand;

/* ---- context ---------------------------------------------------------------------------- */
typedef struct qe_ctx qe_ctx;

/* Create a context on HIP device `device` that launches on hipStream_t `stream`
 * (NULL = the legacy default stream, e.g. torch's default stream). */
int qe_ctx_create(int device, void* stream, qe_ctx** out);
/* Same, with a non-blocking stream the ctx creates and owns (hosts without streams: JNI). */
int qe_ctx_create_owned(int device, qe_ctx** out);
/* Per-plan kernel specialisation of the fused aggregate (hipRTC, default on; env QE_JIT=0
 * turns it off at ctx creation). 0 = always run the generic (interpreting) kernel. */
int qe_ctx_set_jit(qe_ctx* ctx, int32_t enable);
int qe_ctx_destroy(qe_ctx* ctx);
/* The hipStream_t every kernel of this ctx is launched on. */
void* qe_ctx_stream(qe_ctx* ctx);
/* Wait for all work queued on the ctx's stream. */
int qe_ctx_synchronize(qe_ctx* ctx);
/* Thread-local message of the last failing call on this thread ("" if none). */
const char* qe_last_error(void);
int qe_abi_version(void);

/* Device memory helpers for hosts without their own allocator (JNI). Blocks come from the
 * library's caching allocator: a freed block is reused by the same ctx stream at once, by other
 * streams once the work queued before the free has completed. (The reference never frees its
 * allocators, K:256 / K:465 / K:635; this is the bounded equivalent.) */
int qe_device_alloc(qe_ctx* ctx, size_t bytes, void** out);
int qe_device_free(qe_ctx* ctx, void* ptr);
/* Return the cached free blocks of `device` to the driver (waits for their last users). */
int qe_release_cached_memory(int device);
int qe_copy_to_device(qe_ctx* ctx, void* dst, const void* src, size_t bytes);   /* sync */
int qe_copy_to_host(qe_ctx* ctx, void* dst, const void* src, size_t bytes);     /* sync */
/* `bytes` of the file `path` from `offset` straight into device memory `dst` (sync): the staging
 * threads pread() into pinned buffers and DMA them, so the file is never mapped (CsvDataSource's
 * file -> HBM leg, K:306-316). QE_ERR_INVALID_ARG if the file cannot be read that far. */
int qe_file_to_device(qe_ctx* ctx, const char* path, int64_t offset, int64_t bytes, void* dst);

/* ---- synthetic RecordBatch generator (measurement harness) ------------------------------ */
/* Counter-based: u = splitmix64(seed ^ col*0x9E3779B97F4A7C15 ^ row), row = row0 + i.
 * Distributions (oracle/gen.py restates them bit-for-bit):
 *   QE_GEN_MOD     int64: u mod param              (param > 0)
 *   QE_GEN_RAW     int64: (int64)u                 (full range, exercises wrap)
 *   QE_GEN_UNIT53  fp64 : (u >> 11) * 2^-42 - 1024 (exact in fp64)
 *   QE_GEN_MOD_F64 fp64 : (double)(u mod param) * 0.01
 * If `null_permille` > 0 the validity bitmap is filled: row valid unless
 * splitmix64(seed ^ (col+0x1000)*phi ^ row) mod 1000 < null_permille. */
#define QE_GEN_MOD 1
#define QE_GEN_RAW 2
#define QE_GEN_UNIT53 3
#define QE_GEN_MOD_F64 4
int qe_generate(qe_ctx* ctx, qe_column* out, int32_t dist, int64_t param, uint64_t seed,
                uint64_t col, int64_t row0, int32_t null_permille);

/* Measurement harness: device time (ms) of one pass that reads every byte of `ncols`
 * fixed-width columns with 16-B loads — the achievable stream-read ceiling for the bytes a
 * query scans (reported next to the roofline). */
int qe_stream_read(qe_ctx* ctx, const qe_column* cols, int32_t ncols, double* ms);
/* The same ceiling taken over several launch shapes (row-interleaved or column-serial, 1-4 slabs
 * per step, 256-1024 threads, 1-8 workgroups per CU, non-temporal or cached loads): `reps` launches
 * per shape, the best shape's median in *ms and its description in `shape`. This is the bound
 * bench.py reports beside the fused kernel. */
int qe_stream_read_best(qe_ctx* ctx, const qe_column* cols, int32_t ncols, int32_t reps, double* ms,
                        char* shape, int32_t shape_len);

/* ---- vectorised expressions: Expression.evaluate (K:448-450) ---------------------------- */
#define QE_OP_ADD 1
#define QE_OP_SUB 2
#define QE_OP_MUL 3
#define QE_OP_DIV 4
#define QE_OP_EQ 10
#define QE_OP_NE 11
#define QE_OP_LT 12
#define QE_OP_LE 13
#define QE_OP_GT 14
#define QE_OP_GE 15
#define QE_OP_AND 20
#define QE_OP_OR 21
#define QE_OP_NOT 22
#define QE_OP_IS_NULL 23
#define QE_OP_IS_NOT_NULL 24

/* Arithmetic (K1). int64 +,-,* wrap (two's complement, JVM Long); int64 / truncates,
 * x/0 -> null; any fp64 operand promotes to fp64 (IEEE). Null in -> null out.
 * out->values: length*8 bytes; out->validity required iff an operand can be null. */
int qe_eval_arith(qe_ctx* ctx, int32_t op, const qe_operand* lhs, const qe_operand* rhs,
                  qe_column* out);

/* Comparison (K2) -> QE_TYPE_BOOL bitmap. Signed int64 / IEEE fp64 (NaN: only NE true),
 * mixed int64/fp64 compares as fp64; UTF8 supports EQ/NE against a UTF8 literal column of
 * length 1 (byte equality). out->values: ceil(length/8) bytes. */
int qe_eval_cmp(qe_ctx* ctx, int32_t op, const qe_operand* lhs, const qe_operand* rhs,
                qe_column* out);

/* Boolean (K3a): AND / OR (SQL three-valued), NOT, IS_NULL, IS_NOT_NULL.
 * `rhs` is ignored (may be NULL) for the unary ops. */
int qe_eval_bool(qe_ctx* ctx, int32_t op, const qe_column* lhs, const qe_column* rhs,
                 qe_column* out);

/* CastExpression (K6, K:772-805): UTF8 -> FLOAT64 with java.lang.Double.parseDouble semantics
 * (the reference's `vv.toDouble()`, K:791): trimmed, signed, NaN/Infinity, decimal with optional
 * exponent, hex with binary exponent, optional [fFdD] suffix; correctly rounded (half-even).
 * Null rows stay null (K:787-788). A string outside the grammar fails the whole call with
 * QE_ERR_INVALID_ARG (NumberFormatException, a subclass of IllegalArgumentException) and, if
 * `error_row` is non-NULL, stores the first offending row there (-1 when none).
 * `out` is FLOAT64 with capacity >= in->length rows and a validity buffer when `in` has one. */
int qe_cast_utf8_to_f64(qe_ctx* ctx, const qe_column* in, qe_column* out, int64_t* error_row);

/* ---- SelectionExec (K3b): order-preserving compaction ----------------------------------- */
/* Rows whose mask is true (null -> dropped) are kept, in input order. */
int qe_filter_count(qe_ctx* ctx, const qe_column* mask, int64_t* out_count);
/* Gathers the selected rows of every input column into outs[i] (capacity >= count rows).
 * Fixed-width and UTF8 columns; a UTF8 output needs offsets for count+1 entries and a values
 * buffer as large as the input's (offsets[n] - offsets[0]) bytes. outs[i].validity is written
 * when inputs[i] has one (buffer padded to whole 32-bit words).
 * *out_count receives the number of rows written (also set as outs[i].length). */
int qe_filter_apply(qe_ctx* ctx, const qe_column* mask, const qe_column* inputs,
                    int32_t ncols, qe_column* outs, int64_t* out_count);
/* The same without a host round trip (the per-family chain cmp -> filter -> arith stream-ordered,
 * SelectionExec -> ProjectionExec): fixed-width columns only, every output holds the mask's
 * length rows (an upper bound), and the number of rows written goes to the device word *d_count
 * (queued on the ctx stream like the gather). outs[i].length is set to the mask's length; rows at
 * and beyond *d_count are unspecified. qe_eval_arith_dlen computes only the rows below such a
 * device count; the caller reads the count back once, at the end of the chain. */
int qe_filter_apply_async(qe_ctx* ctx, const qe_column* mask, const qe_column* inputs,
                          int32_t ncols, qe_column* outs, int64_t* d_count);
int qe_eval_arith_dlen(qe_ctx* ctx, int32_t op, const qe_operand* lhs, const qe_operand* rhs,
                       qe_column* out, const int64_t* d_len);

/* ---- aggregates ------------------------------------------------------------------------- */
#define QE_AGG_SUM 1
#define QE_AGG_MIN 2
#define QE_AGG_MAX 3        /* MaxAccumulator semantics, K:538-561 */
#define QE_AGG_COUNT 4      /* COUNT(x): non-null rows */
#define QE_AGG_COUNT_STAR 5 /* COUNT(*): rows */
#define QE_AGG_AVG 6        /* fp64 SUM / COUNT */

/* Global (no GROUP BY) aggregate of one column (K4a), all functions in one pass.
 * min/max follow MaxAccumulator (K:538-561): nulls skipped; the first non-null value
 * seeds; replaced only on strictly greater (less) => a NaN seed is sticky, a later NaN
 * never wins, +0.0/-0.0 ties keep the earliest. `valid` = 1 iff count > 0.
 * fp64 sum: the correctly rounded exact sum over the whole fp64 range (math.fsum's value; the
 * IEEE result with NaN / Inf inputs; +-Inf when the exact sum overflows); avg = that sum / count.
 * A compensated sum gives it when its error bound proves that every value within the bound rounds
 * to the same double; otherwise a second, exact fixed-point pass over the column does.
 * int64 sum wraps; int64 avg is the compensated fp64 mean. */
typedef struct qe_global_agg {
  int64_t rows;   /* COUNT(*) over rows passing the mask */
  int64_t count;  /* COUNT(x) */
  int32_t type;   /* input type: INT64 or FLOAT64 */
  int32_t valid;  /* SUM/MIN/MAX/AVG non-null */
  int64_t sum;    /* int64 value, or fp64 bits */
  int64_t min;    /* int64 value, or fp64 bits */
  int64_t max;    /* int64 value, or fp64 bits */
  double avg;
} qe_global_agg;
int qe_agg_global(qe_ctx* ctx, const qe_column* col, const qe_column* mask /*nullable*/,
                  qe_global_agg* out);
/* The same aggregate over a column split across batches or GPUs (one exchange of a
 * fixed-size partial). qe_agg_global_partial writes this column's mergeable partial (sums, min /
 * max keys and first-row indices, QE_GLOBAL_PARTIAL_BYTES of device memory); `row_base` is the
 * global index of the column's first row, so MIN/MAX keep MaxAccumulator's row-order rules
 * (NaN seed, earliest of +0.0 / -0.0) across the pieces. qe_agg_global_merge folds n partials
 * (device, packed QE_GLOBAL_PARTIAL_BYTES apart, any order) in a fixed order into the final
 * result: every rank merging the same all-gathered partials gets the same bits.
 * When the merged fp64 sum cannot be proven correctly rounded (the pieces' sums cancel),
 * qe_agg_global_merge returns QE_NEED_EXACT with every other field of `out` final: each piece
 * then writes its exact sum words (qe_agg_global_exact_partial, QE_GLOBAL_EXACT_BYTES of device
 * memory), the words are gathered like the partials, and qe_agg_global_merge_exact sets
 * out->sum and out->avg (synchronises). The second round happens on every rank or on none. */
#define QE_GLOBAL_PARTIAL_BYTES 128
#define QE_GLOBAL_EXACT_BYTES 320
int qe_agg_global_partial(qe_ctx* ctx, const qe_column* col, const qe_column* mask /*nullable*/,
                          int64_t row_base, void* partial);
int qe_agg_global_merge(qe_ctx* ctx, int32_t type, const void* partials, int32_t n, qe_global_agg* out);
int qe_agg_global_exact_partial(qe_ctx* ctx, const qe_column* col, const qe_column* mask /*nullable*/,
                                void* words);
int qe_agg_global_merge_exact(qe_ctx* ctx, const void* words, int32_t n, qe_global_agg* out);

/* ---- HashAggregateExec (K4b) ------------------------------------------------------------ */
/* Group keys: 0..4 columns of any type — INT64, FLOAT64 (Double.equals: one NaN group, +0.0 and
 * -0.0 apart), INT32, DATE32, UINT8, BOOL, UTF8 (byte equality of String(bytes), K:620-627). A null
 * key is a group of its own (List.equals semantics, K:621-627). Group order is unspecified
 * (HashMap iteration, K:639).
 * The table groups by one 64-bit word per row. One INT64/FLOAT64 key is that word; narrow keys
 * (INT32/DATE32/UINT8) whose widths + one null bit each fit in 63 bits are packed into it. Every
 * other key list is DICTIONARY-KEYED, and the state owns its dictionaries:
 *   - a lone UTF8 key gets wide INT64 codes (a value of at most 7 bytes is its own code, longer ones
 *     go through a string dictionary: qe_strdict_encode);
 *   - a UTF8 key in a list gets INT32 dictionary codes, packed with the narrow keys;
 *   - a list that still does not pack (INT64 + UTF8, BOOL, three INT32 ...) groups by one INT32
 *     code per distinct key tuple (qe_strdict_encode_tuple).
 * Updates and fused updates take the ORIGINAL key columns (UTF8 included) and encode them; finalize
 * writes the original key types back (qe_hashagg_finalize_sizes sizes UTF8 outputs). The codes are
 * local to the state, so its partials move between states only by key content:
 * qe_hashagg_merge / qe_hashagg_export_keyed / qe_hashagg_import_keyed / qe_hashagg_exchange. The
 * raw record calls (export*, import*) refuse a dictionary-keyed state with QE_ERR_UNSUPPORTED. */
#define QE_MAX_KEYS 4
#define QE_MAX_AGGS 8
#define QE_MAX_COLS 8
#define QE_MAX_TERMS 8
#define QE_MAX_TOKENS 16

typedef struct qe_agg_desc {
  int32_t fn;         /* QE_AGG_* */
  int32_t input_type; /* FLOAT64, or INT64 / INT32 / DATE32 / UINT8 (accumulated as int64, so
                         integer SUM/MIN/MAX outputs are INT64); ignored for COUNT_STAR; AVG
                         accumulates fp64 */
} qe_agg_desc;

typedef struct qe_hashagg qe_hashagg;
typedef struct qe_strdict qe_strdict; /* string / key-tuple dictionary (UTF-8 group keys, below) */

int qe_hashagg_create(qe_ctx* ctx, int32_t nkeys, const int32_t* key_types, int32_t naggs,
                      const qe_agg_desc* aggs, int64_t expected_groups, qe_hashagg** out);
/* qe_hashagg_create with options.
 * fp64 SUM / AVG guarantee (within 1e-9 relative of the exact sum). By default they
 * accumulate exactly, in 256-bit fixed point (least significant bit 2^-128, integer adds: a 192-bit
 * window per LDS slot for |x| in [2^-44, 2^62), the global table's full words for other inputs
 * below 2^126) plus, for inputs of 2^126 or more or with bits below 2^-128 (subnormals included),
 * a per-group 2176-bit accumulator in units of 2^-1074 that holds any finite double exactly.
 * finalize rounds the exact sum once to double: the result is the correctly rounded exact sum over
 * the whole fp64 range (math.fsum's value; +-Inf when it overflows), bit-identical whatever order
 * rows, workgroups, batches or ranks combine in — what the reference's sequential row loop and
 * ordered partition merge give with exact arithmetic (K:617-631, K:1314-1325). NaN / +-Inf inputs
 * give NaN / the infinity, as IEEE addition does. finalize never fails for a sum and does not
 * synchronise (stream-ordered like every other state). A group with such inputs exports
 * FXE_CHUNKS = 9 extra records (qe_hashagg_export_counts counts them; every record of a group goes
 * to its key's partition).
 * QE_HASHAGG_DETERMINISTIC: the default (kept for callers that name it).
 * QE_HASHAGG_FAST_FP64: plain fp64 atomics instead (one LDS atomic per row and aggregate); their
 * rounding depends on arrival order, and a group whose terms cancel can miss the 1e-9 contract. */
#define QE_HASHAGG_DETERMINISTIC 1
#define QE_HASHAGG_FAST_FP64 2
int qe_hashagg_create_ex(qe_ctx* ctx, int32_t nkeys, const int32_t* key_types, int32_t naggs,
                         const qe_agg_desc* aggs, int64_t expected_groups, int32_t flags, qe_hashagg** out);
int qe_hashagg_destroy(qe_hashagg* agg);
/* Forget all groups (keeps allocations). */
int qe_hashagg_reset(qe_hashagg* agg);

/* One input batch: per-row keys and pre-evaluated aggregate inputs (agg_inputs[j] is the
 * column of aggregate j; its values are never read for COUNT_STAR, which may pass a zeroed
 * struct — or, when the state has no keys and no other inputs, any column of the batch, whose
 * length is then the row count). `mask` (BOOL,
 * nullable pointer) selects rows. Row indices continue across calls in call order: they
 * define "first"/"earliest" for MIN/MAX ties exactly like the reference's batch loop. */
int qe_hashagg_update(qe_hashagg* agg, const qe_column* keys, const qe_column* agg_inputs,
                      const qe_column* mask);

/* Fused filter -> project -> partial aggregate over the columns of one batch, one pass
 * over HBM. Predicate = AND of terms (col CMP literal | col CMP col) and optional BOOL mask
 * column; keys are column slots; each aggregate input is a postfix program over column
 * slots and literals (tokens below). Semantics are those of composing
 * SelectionExec -> ProjectionExec -> HashAggregateExec with the per-family functions. */
#define QE_TOK_COL 1 /* push column slot `arg` */
#define QE_TOK_LIT 2 /* push literal */
#define QE_TOK_ADD 3
#define QE_TOK_SUB 4
#define QE_TOK_MUL 5
#define QE_TOK_DIV 6

typedef struct qe_pred_term {
  int32_t col;     /* column slot (lhs) */
  int32_t op;      /* QE_OP_EQ..QE_OP_GE */
  int32_t rhs_col; /* column slot, or -1 => compare against `lit` */
  int32_t reserved;
  qe_scalar lit;
} qe_pred_term;

typedef struct qe_token {
  int32_t op;  /* QE_TOK_* */
  int32_t arg; /* column slot for QE_TOK_COL */
  qe_scalar lit;
} qe_token;

typedef struct qe_agg_program {
  int32_t ntokens; /* 0 for COUNT_STAR */
  int32_t reserved;
  qe_token tokens[QE_MAX_TOKENS];
} qe_agg_program;

typedef struct qe_fused_spec {
  int32_t mask_col; /* BOOL column slot used as selection (null -> dropped), or -1 */
  int32_t nterms;
  qe_pred_term terms[QE_MAX_TERMS];
  int32_t key_cols[QE_MAX_KEYS];
  qe_agg_program inputs[QE_MAX_AGGS];
} qe_fused_spec;

int qe_hashagg_update_fused(qe_hashagg* agg, const qe_column* cols, int32_t ncols,
                            const qe_fused_spec* spec);

/* ---- fused SelectionExec -> ProjectionExec (ProjectionExec.execute K:589-594 over A5) ------
 * One pass over `cols`: rows passing the mask/terms (null -> dropped) are written, in input
 * order, as the value of each output program (same token language and null rules as the
 * aggregate inputs; a lone column reference keeps its type, other programs give INT64 or
 * FLOAT64). outs[k]: capacity >= cols[0].length rows, type = the program's type; validity
 * written when non-NULL. *out_count = rows written (also each outs[k].length).
 * Needs per-plan kernel specialisation: QE_ERR_UNSUPPORTED when it is off or the shape is
 * outside the generator (callers then run qe_eval_cmp + qe_filter_apply + qe_eval_arith). */
typedef struct qe_select_spec {
  int32_t mask_col; /* BOOL column slot used as selection, or -1 */
  int32_t nterms;
  qe_pred_term terms[QE_MAX_TERMS];
  int32_t nout;
  int32_t reserved;
  qe_agg_program outputs[QE_MAX_AGGS];
} qe_select_spec;
int qe_select_project(qe_ctx* ctx, const qe_column* cols, int32_t ncols, const qe_select_spec* spec,
                      qe_column* outs, int64_t* out_count);
/* Stream-ordered form (a pipelined SelectionExec -> ProjectionExec over a Sequence<RecordBatch>,
 * K:589-594): queues the kernels and the copy of the row count into pinned memory, and returns
 * without waiting. *pending must be passed to qe_select_pending_wait exactly once (it frees it);
 * that call waits for this select-project's row count only — not for work queued behind it, such
 * as the next batch's select-project — and returns it. Where the kernel publishes the count itself
 * (the register-resident pass and the two-pass write kernel) the wait polls that word in pinned
 * memory and may return while the kernel still reads its inputs and writes its outputs. So, as for
 * any stream-ordered call: the outputs are complete for every later operation on ctx's stream, and
 * for other streams or the host only after ctx's stream work has completed (qe_ctx_synchronize);
 * the inputs must stay valid until then too — not merely until the wait returns.
 * qe_select_project = async + wait + a synchronisation of ctx's stream: when it returns, the
 * kernels have completed (inputs may be released, outputs read anywhere). */
typedef struct qe_select_pending qe_select_pending;
int qe_select_project_async(qe_ctx* ctx, const qe_column* cols, int32_t ncols, const qe_select_spec* spec,
                            qe_column* outs, qe_select_pending** pending);
int qe_select_pending_wait(qe_select_pending* pending, int64_t* out_count);

/* Number of groups so far (synchronises). */
int qe_hashagg_num_groups(qe_hashagg* agg, int64_t* out);
/* Materialise the single output batch (K:635-650): key columns then one column per
 * aggregate. out_keys[i]/out_aggs[j] must hold num_groups rows; validity buffers are
 * written when non-NULL (required for nullable results: any key, SUM/MIN/MAX/AVG).
 * *out_groups is exact on return; the column contents are stream-ordered: they are written by
 * work queued on the ctx stream (read them on that stream, or after qe_ctx_synchronize).
 * Output types: keys as declared; SUM/MIN/MAX as input type; COUNT/COUNT_STAR int64;
 * AVG fp64. A UTF8 key output needs offsets for groups+1 entries, a validity buffer, and a values
 * buffer of at least the bytes qe_hashagg_finalize_sizes reports for it. */
int qe_hashagg_finalize(qe_hashagg* agg, qe_column* out_keys, qe_column* out_aggs,
                        int64_t* out_groups);
/* Output sizes of the next finalize (synchronises): *groups, and key_bytes[k] (one entry per
 * declared key, may be NULL) = a bound on the value bytes finalize writes for UTF8 key k (0 for
 * other keys). Exact when the key has dictionary codes; 7 bytes per group while a lone UTF8 key's
 * values have all been at most 7 bytes (no device work then). */
int qe_hashagg_finalize_sizes(qe_hashagg* agg, int64_t* groups, int64_t* key_bytes);
/* Without synchronising: *per_group = a bound on the value bytes per group that finalize writes for
 * UTF8 key `key` (7 while every value of a lone UTF8 key has been at most 7 bytes and is its own
 * code), or 0 when only qe_hashagg_finalize_sizes can tell. A caller with a bound sizes the key's
 * output at per_group x its row capacity and calls qe_hashagg_finalize directly (QE_ERR_CAPACITY,
 * with the group count, if the rows do not suffice). */
int qe_hashagg_key_bytes_bound(qe_hashagg* agg, int32_t key, int64_t* per_group);

/* Two-phase / multi-GPU aggregate (K:1309-1325 pattern):
 * export the partial groups bucketed by destination partition = hash(key) mod nparts
 * as fixed-size records, then import records (from any rank) into another state.
 * Records carry the table's key word as is, so these calls (and the slot calls below) refuse a
 * dictionary-keyed state (QE_ERR_UNSUPPORTED): its partials move by content (qe_hashagg_merge,
 * qe_hashagg_export_keyed / qe_hashagg_import_keyed). */
int qe_hashagg_record_bytes(qe_hashagg* agg, int64_t* out);
/* counts[p] = records for partition p (host array of nparts, synchronises). */
int qe_hashagg_export_counts(qe_hashagg* agg, int32_t nparts, int64_t* counts);
/* Writes all records into `dst` (device, sum(counts)*record_bytes), partition-major in
 * partition order (counts as qe_hashagg_export_counts reports them). Stream-ordered, no host
 * synchronisation. */
int qe_hashagg_export(qe_hashagg* agg, int32_t nparts, void* dst);
/* Merge `nrecords` records (device) into this state (combine semantics per aggregate). */
int qe_hashagg_import(qe_hashagg* agg, const void* records, int64_t nrecords);

/* Partials by key CONTENT (K:1309-1325 with the reference's String(bytes) keys, K:620-627): the
 * form every state supports, and the only one for dictionary-keyed states, whose codes mean nothing
 * to another state. A block is self-describing: a 128-byte header (magic, records, key types, UTF8
 * byte counts), the records with their key words cleared, then per key its validity (one byte per
 * record) and its values (8 bytes per record, or UTF8 lengths + bytes). Records are routed by a
 * content hash of the keys (qe_hash_partition), so equal keys reach the same partition on every
 * rank whatever each rank's dictionaries hold; the importer re-encodes the keys into its own
 * dictionaries, so equal strings merge and different strings never share a group.
 * export_keyed_sizes (synchronises) computes block_bytes[p] for each of `nparts` partitions and
 * keeps the state's groups ready for export_keyed, which writes the blocks partition-major into
 * `dst` (device, sum(block_bytes); stream-ordered). Any update, import or reset in between
 * invalidates it (QE_ERR_INVALID_ARG). import_keyed merges `nblocks` received blocks, packed
 * back to back in `blocks` (device) with sizes block_bytes[b] (0 = no block); the blocks' layout
 * must be this state's (same key types, aggregates and options, else QE_ERR_INVALID_ARG). */
#define QE_KEYED_HEADER 128
int qe_hashagg_export_keyed_sizes(qe_hashagg* agg, int32_t nparts, int64_t* block_bytes);
int qe_hashagg_export_keyed(qe_hashagg* agg, int32_t nparts, void* dst);
int qe_hashagg_import_keyed(qe_hashagg* agg, const void* blocks, int32_t nblocks, const int64_t* block_bytes);
/* main()'s partial -> final merge inside one process (K:1314-1325): every group of `src` is merged
 * into `dst` (same ctx, same key types and aggregates). By key content when either state is
 * dictionary-keyed, else by raw records. `src` is unchanged. */
int qe_hashagg_merge(qe_hashagg* dst, qe_hashagg* src);
/* A state created with INT32 (or, for a lone key, wide INT64) key `key` whose codes the CALLER
 * takes from `dict` (qe_strdict_encode): binding the dictionary makes the state dictionary-keyed —
 * finalize, merge and the keyed exchange decode and re-encode through `dict`, and the raw record
 * calls refuse it. Updates then take either the codes or the UTF8 column itself. `dict` must
 * outlive the state. Bind before the first update. */
int qe_hashagg_bind_key_dict(qe_hashagg* agg, int32_t key, qe_strdict* dict);
/* How the state groups: *dictionary_keyed (0: raw key words; 1: string codes; 2: key-tuple codes),
 * and the types of the columns the table groups by (device_types: QE_MAX_KEYS entries). */
int qe_hashagg_key_layout(qe_hashagg* agg, int32_t* dictionary_keyed, int32_t* device_nkeys, int32_t* device_types);

/* Fixed-capacity exchange: ONE equal-split all-to-all and no host synchronisation before it.
 * export_slots writes `nparts` slots of QE_SLOT_HEADER + slot_records * record_bytes bytes into
 * `dst` (device): slot p holds the first `slot_records` groups of partition p (same partition
 * function as qe_hashagg_export); its header's int64 word 0 is the partition's full count, word 1
 * the largest count over all of this state's partitions. import_slots merges `nslots` received
 * slots (one per sender); *max_count = the largest count any sender reported (every receiver sees
 * every sender's word 1, so all ranks get the same value). If *max_count > slot_records some
 * sender's groups did not fit: NOTHING is imported, and every rank should exchange again with
 * qe_hashagg_export / qe_hashagg_import. *nrecords (optional) = records the slots hold.
 * export_slots does not synchronise, not even to settle a pending stream-ordered update: if that
 * update left the table incomplete (deferred rows, overflow), word 1 reports 2^62 so that every
 * rank takes the variable-size exchange, which settles it. import_slots is one launch (each
 * workgroup checks the headers itself) and one read-back; it grows the table beforehand from an
 * upper bound (groups so far + nslots * slot_records). */
#define QE_SLOT_HEADER 64
int qe_hashagg_export_slots(qe_hashagg* agg, int32_t nparts, int64_t slot_records, void* dst);
int qe_hashagg_import_slots(qe_hashagg* agg, const void* slots, int32_t nslots, int64_t slot_records,
                            int64_t* max_count, int64_t* nrecords);
/* Default slot capacity for a `world`-rank exchange: the expected groups given to
 * qe_hashagg_create (never the sizing hint a rank's own data raised) spread over the ranks with
 * headroom — min(eg, ceil(3 eg / 2 world) + 32) — so every rank computes the same slot size. */
int qe_hashagg_slot_capacity(qe_hashagg* agg, int32_t world, int64_t* slot_records);

/* Stream-ordered updates (default 0 = off). With `enable`, an update that needs one kernel launch
 * returns once it is queued; the read-back of its counters — and, when the global table had to
 * grow, the retry pass that re-reads the update's input columns — happens in the next call on
 * this state (update, num_groups, finalize, export*, import*, last_kernel_time), which then also
 * reports the update's errors. The input columns must stay valid until that call returns.
 * qe_hashagg_reset discards a pending update; qe_hashagg_set_async(agg, 0) settles it. */
int qe_hashagg_set_async(qe_hashagg* agg, int32_t enable);

/* ---- multi-GPU exchange over RCCL without a host framework (JNI) ---------------------------
 * One qe_comm per GPU (rank), all on the ctx whose stream runs the aggregation. Rank 0 calls
 * qe_comm_unique_id and the host hands the 128 bytes to every rank (its own transport), then
 * every rank calls qe_comm_create (collective). RCCL is loaded at run time (librccl.so.1);
 * QE_ERR_COMM when it is missing or a call fails. */
#define QE_COMM_ID_BYTES 128
typedef struct qe_comm qe_comm;
int qe_comm_unique_id(void* id /* QE_COMM_ID_BYTES */);
int qe_comm_create(qe_ctx* ctx, int32_t world, int32_t rank, const void* id, qe_comm** out);
int qe_comm_destroy(qe_comm* comm);
/* In-process transport: `world` ranks that are threads of one process, each with its own qe_ctx
 * (one GPU, or several), share a hub; qe_hashagg_exchange then runs its usual export -> grouped
 * send/recv -> import with device copies in place of RCCL (every rank must call it concurrently,
 * as with RCCL). For hosts that run several partitions in one process and for the multi-rank tests
 * on a one-GPU box (RCCL refuses two ranks on one device). The hub outlives its communicators. */
int qe_comm_loopback_hub_create(int32_t world, void** hub);
int qe_comm_loopback_hub_destroy(void* hub);
int qe_comm_create_loopback(qe_ctx* ctx, int32_t world, int32_t rank, void* hub, qe_comm** out);
/* Every rank: move each group of `partial` to the rank that owns its key (hash(key) mod world,
 * as qe_hashagg_export) and merge what this rank receives into `owner` (K:1309-1325 across GPUs).
 * Fixed slots of `slot_records` groups per destination (<= 0: the expected groups spread over the
 * ranks with headroom), one grouped send/recv on the ctx stream, one read-back; if a partition
 * overflowed its slot on any rank, every rank falls back to counts + records. A stream-ordered
 * (qe_hashagg_set_async) partial is exported without a host wait. *nrecords (optional) = records
 * this rank merged. partial, owner and comm must share the ctx.
 * Dictionary-keyed states (UTF8 / key-tuple codes) exchange by key content instead: block sizes in
 * one all-to-all, then the blocks (qe_hashagg_export_keyed / qe_hashagg_import_keyed), routed by a
 * content hash and re-encoded on the owner — the reference's VendorID-keyed merge (K:1336) across
 * GPUs. */
int qe_hashagg_exchange(qe_comm* comm, qe_hashagg* partial, qe_hashagg* owner, int64_t slot_records,
                        int64_t* nrecords);

/* Offset added to row indices of the next update (for shards of one logical stream). */
int qe_hashagg_set_row_base(qe_hashagg* agg, int64_t row_base);

/* Measurement hook: device time (HIP events on the ctx stream) of the aggregation kernel
 * launches made by the last update call, and how many launches it took (1 unless the table
 * had to grow and deferred rows were re-applied). */
int qe_hashagg_last_kernel_time(qe_hashagg* agg, double* ms, int32_t* launches);
/* Measurement hook: a signature of what the last update launched — a hash of the specialised
 * kernel's compile key (hipRTC / HIP versions, options, generated source) and its launch shape —
 * so that counters recorded for one build (bench.py's profiles/traffic.json) are only reused for
 * the identical kernel and launch. */
int qe_hashagg_last_kernel_signature(qe_hashagg* agg, uint64_t* sig);
/* Whether the last update ran a plan-specialised kernel (1) or the generic one (0), and why
 * not (NUL-terminated note, may be NULL). */
int qe_hashagg_last_kernel_kind(qe_hashagg* agg, int32_t* specialized, char* note, int32_t note_len);

/* ---- UTF-8 group keys (K:620-627: row key = String(bytes), HashMap content equality) ------
 * A device string dictionary maps each distinct byte string to a dense int32 code, stable for
 * the dictionary's lifetime (codes are assigned in first-insertion order within a call, which
 * is unordered across rows). A hash aggregate groups by the codes (key type INT32); finalize
 * decodes them back to strings. Equality is byte equality of the whole string. (A hash aggregate
 * with UTF8 keys owns such dictionaries itself; these calls are for callers that encode keys on
 * their own, qe_hashagg_bind_key_dict.) */
int qe_strdict_create(qe_ctx* ctx, int64_t expected_distinct, qe_strdict** out);
int qe_strdict_destroy(qe_strdict* dict);
/* Number of distinct strings inserted so far. */
int qe_strdict_size(qe_strdict* dict, int64_t* out);
/* codes (INT32, capacity >= in->length; validity required iff `in` has one, copied from it):
 * the code of every non-null row of the UTF8 column `in`, inserting new strings.
 * An INT64 codes column asks for WIDE codes: a string of at most 7 bytes is its own code (its
 * bytes little-endian in bits 0..55, its length in bits 56..58) and is not inserted; a longer one
 * is 2^62 | its dictionary code. Equal strings get equal codes, bit 63 is never set, and
 * qe_strdict_decode / _decode_bytes take either code width (qe_strdict_size counts the long
 * strings only). A hash aggregate over wide codes groups by an INT64 key with no dictionary
 * traffic for short keys (the reference's VendorID, K:1336). */
int qe_strdict_encode(qe_strdict* dict, const qe_column* in, qe_column* codes);
/* Total bytes of the strings the non-null rows of `codes` (INT32) decode to. */
int qe_strdict_decode_bytes(qe_strdict* dict, const qe_column* codes, int64_t* out_bytes);
/* out (UTF8): offsets for codes->length+1 entries, values >= decode_bytes bytes, validity
 * iff codes has one. QE_ERR_INVALID_ARG if a code was not issued by this dictionary. */
int qe_strdict_decode(qe_strdict* dict, const qe_column* codes, qe_column* out);
/* The same for codes this dictionary produced (no range check is promised): wide INT64 codes of a
 * dictionary that holds no long key are all packed, and decode then needs no host round trip —
 * `out->values` must hold 7 bytes per row. Otherwise as qe_strdict_decode. */
int qe_strdict_decode_trusted(qe_strdict* dict, const qe_column* codes, qe_column* out);
/* Wide codes without a dictionary, for a UTF8 column whose every value is known to be at most 7
 * bytes (a CSV column with qe_csv_column_max_len <= 7): the packed code qe_strdict_encode gives
 * each value (validity copied), in one streaming kernel with no host round trip, so the
 * aggregation that consumes the codes queues right behind it. The bound is the caller's promise
 * (not checked: a longer value gets a code of its first 7 bytes). */
int qe_strdict_encode_packed(qe_ctx* ctx, const qe_column* in, qe_column* codes);
/* Packed wide codes (encode_packed's, or a trusted dictionary's while it holds no long key) ->
 * UTF8: offsets for codes->length+1 entries, `out->values` 7 bytes per row, validity iff codes has
 * one; stream-ordered, no synchronisation (one kernel up to 65536 rows). */
int qe_strdict_decode_packed(qe_ctx* ctx, const qe_column* codes, qe_column* out);
/* Composite group keys (K:621-626 `List` of key values) whose packing exceeds 63 bits: each row's
 * tuple of up to QE_MAX_KEYS fixed-width / BOOL key columns (nulls and fp64 NaNs as
 * List/Double.equals see them) gets a dense int32 code; codes->validity (optional) is set all-valid.
 * A dictionary holds either strings or tuples of one layout. decode_tuple writes the key columns
 * (types as encoded; validity where outs[k].validity is non-NULL) for `codes`. */
int qe_strdict_encode_tuple(qe_strdict* dict, const qe_column* keys, int32_t nkeys, qe_column* codes);
int qe_strdict_decode_tuple(qe_strdict* dict, const qe_column* codes, int32_t nkeys, qe_column* outs);
/* Destination partition of every row by the CONTENT of its key columns (UTF8 bytes, fixed-width
 * values with fp64 NaNs as one key, nulls): part[i] in [0, nparts), identical on every rank for
 * equal keys. Used to route dictionary-keyed partials, whose codes are local to one state. */
int qe_hash_partition(qe_ctx* ctx, const qe_column* cols, int32_t ncols, int32_t nparts, int32_t* part);

/* ---- Arrow C Data Interface boundary -----------------------------------------
 * Arrow Java exports a VectorSchemaRoot (the reference's batches, K:635-650) as a struct
 * ArrowArray + ArrowSchema (org.apache.arrow.c.Data.exportVectorSchemaRoot); these entry points
 * take and return exactly that, so the JNI shim passes two struct addresses per batch.
 * Standard ABI structs (Arrow C data / C device data interface specification). */
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
  const char* format;
  const char* name;
  const char* metadata;
  int64_t flags;
  int64_t n_children;
  struct ArrowSchema** children;
  struct ArrowSchema* dictionary;
  void (*release)(struct ArrowSchema*);
  void* private_data;
};
struct ArrowArray {
  int64_t length;
  int64_t null_count;
  int64_t offset;
  int64_t n_buffers;
  int64_t n_children;
  const void** buffers;
  struct ArrowArray** children;
  struct ArrowArray* dictionary;
  void (*release)(struct ArrowArray*);
  void* private_data;
};
#endif
#ifndef ARROW_C_DEVICE_DATA_INTERFACE
#define ARROW_C_DEVICE_DATA_INTERFACE
typedef int32_t ArrowDeviceType;
struct ArrowDeviceArray {
  struct ArrowArray array;
  int64_t device_id;
  ArrowDeviceType device_type;
  void* sync_event;
  int64_t reserved[3];
};
#endif
#define QE_ARROW_DEVICE_CPU 1
#define QE_ARROW_DEVICE_ROCM 10
typedef struct ArrowSchema ArrowSchema;
typedef struct ArrowArray ArrowArray;
typedef struct ArrowDeviceArray ArrowDeviceArray;

/* A device-resident batch: the columns of one RecordBatch (K:56-61) in HBM. */
typedef struct qe_batch qe_batch;
/* Host record batch (struct array "+s"; children l/g/u/U/i/C/tdD/b, any offset, nullable) ->
 * device copy owned by the batch. H2D goes through double-buffered pinned staging. The caller
 * keeps ownership of (and later releases) `array`/`schema`. Unsupported formats ->
 * QE_ERR_UNSUPPORTED (cf. K:195). */
int qe_batch_import(qe_ctx* ctx, const ArrowSchema* schema, const ArrowArray* array, qe_batch** out);
/* Zero-copy view of a record batch already in HBM (device_type QE_ARROW_DEVICE_ROCM on the ctx
 * device); waits on `sync_event` (a hipEvent_t*) when given. The buffers must outlive the view. */
int qe_batch_import_device(qe_ctx* ctx, const ArrowSchema* schema, const ArrowDeviceArray* array,
                           qe_batch** out);
int qe_batch_destroy(qe_batch* batch);
int qe_batch_num_columns(const qe_batch* batch, int32_t* ncols, int64_t* length);
/* View of column i (valid while the batch lives); *name (may be NULL) is the field name. */
int qe_batch_column(const qe_batch* batch, int32_t i, qe_column* out, const char** name);
/* Device columns (equal lengths) -> host struct array + schema (all fields nullable, K:31).
 * The consumer owns both and calls their release callbacks (Arrow C data interface rules). */
int qe_batch_export(qe_ctx* ctx, const qe_column* cols, int32_t ncols, const char* const* names,
                    ArrowSchema* out_schema, ArrowArray* out_array);

/* ---- GPU CSV scan (CsvDataSource / ReaderIterator, K:204-357) ------------------
 * Tokenises a CSV file that is already in HBM into Utf8 columns (grammar in qe_csv.hip and
 * oracle/csv_ref.py: quotes with "" escapes, \n / \r\n / \r records, blank and '#' lines
 * skipped, values trimmed as K:263 does, missing trailing fields read as ""). The host resolves
 * the header (first kept record) and the projection to field positions. */
typedef struct qe_csv_options {
  int32_t delimiter;          /* field delimiter byte (the reference detects it; the host passes it) */
  int32_t has_header;         /* 1: the first kept record is the header and yields no row */
  int32_t nfields;            /* number of projected fields (1..32) */
  int32_t flags;              /* QE_CSV_PARTIAL_TAIL: more of the file follows these bytes */
  const int32_t* field_index; /* host array of nfields 0-based field positions (< 1024) */
} qe_csv_options;
/* flags: the bytes after the last record terminator are the start of a record that continues
 * past `nbytes` (a chunk of a larger file): they are not parsed, and qe_csv_consumed reports where
 * the next chunk must start (0: no complete record yet; extend the chunk). A chunk that ends
 * between a '\r' and its '\n' reads the '\r' as the terminator and the next chunk's leading
 * '\n' as a blank line, which is skipped: the records are the same as one parse of the file. */
#define QE_CSV_PARTIAL_TAIL 1
typedef struct qe_csv_table qe_csv_table;
int qe_csv_parse(qe_ctx* ctx, const uint8_t* data, int64_t nbytes, const qe_csv_options* opt,
                 qe_csv_table** out);
int qe_csv_rows(const qe_csv_table* table, int64_t* rows);
/* Bytes of the input covered by the parsed records (== nbytes without QE_CSV_PARTIAL_TAIL). */
int qe_csv_consumed(const qe_csv_table* table, int64_t* bytes);
/* `data` must stay valid until every wanted column has been built (column_copy / column).
 * View of projected column i (UTF8, no validity), built into table-owned memory on first request
 * and valid while the table lives. */
int qe_csv_column(const qe_csv_table* table, int32_t i, qe_column* out);
/* Bytes of projected column i, and building it straight into caller buffers (offsets for
 * rows+1 entries, values >= qe_csv_column_bytes; stream-ordered, no synchronisation). */
int qe_csv_column_bytes(const qe_csv_table* table, int32_t i, int64_t* nbytes);
int qe_csv_column_copy(const qe_csv_table* table, int32_t i, qe_column* dst);
/* Length in bytes of projected column i's longest value (known at parse time, no device work):
 * lets a caller take qe_strdict_encode_packed for short keys. */
int qe_csv_column_max_len(const qe_csv_table* table, int32_t i, int64_t* nbytes);
int qe_csv_destroy(qe_csv_table* table);
/* Streaming a file larger than one device batch (ReaderIterator's batches, K:239-252): host bytes
 * data[0, nbytes) that start at a record boundary are cut after their last complete record.
 * *cut = the end of the last record terminator outside quotes (a '\r' at the very end does not
 * count: a '\n' may follow), 0 if there is none (the caller reads more), nbytes when eof != 0.
 * Host only; the bytes [*cut, nbytes) begin the next chunk. */
int qe_csv_record_end(const uint8_t* data, int64_t nbytes, int32_t eof, int64_t* cut);

#ifdef __cplusplus
}
#endif
#endif /* QE_HIP_H */
