// NativeEngine.kt — the Kotlin declarations of libqe_jni.so (qe_jni.c, same directory).
//
// One `external fun` per JNI entry point; handles are Longs owned by the caller (free them with
// the matching *Free / *Destroy). A failing call throws what kquerydiy/src/Main.kt throws for the
// same condition (NumberFormatException for a bad CAST, K:791; IllegalArgumentException, K:49;
// IllegalStateException for unsupported types or plans, K:195 / K:677 / K:799; RuntimeException
// for device errors). Built only where a JDK is present (no JVM in this image): the C side is
// tested through tests/native/jni_harness.c, which calls every function the way these
// declarations do.

object NativeEngine {
    init {
        System.loadLibrary("qe_jni") // libqe_jni.so next to libqe_hip.so (RPATH $ORIGIN)
    }

    // column types (qe_hip.h QE_TYPE_*)
    const val INT64 = 1
    const val FLOAT64 = 2
    const val BOOL = 3
    const val UTF8 = 4
    const val INT32 = 5
    const val UINT8 = 6
    const val DATE32 = 7

    // binary operators (QE_OP_*)
    const val ADD = 1; const val SUB = 2; const val MUL = 3; const val DIV = 4
    const val EQ = 10; const val NE = 11; const val LT = 12; const val LE = 13; const val GT = 14; const val GE = 15
    const val AND = 20; const val OR = 21; const val NOT = 22; const val IS_NULL = 23; const val IS_NOT_NULL = 24

    // aggregate functions (QE_AGG_*); MAX follows MaxAccumulator (K:538-561)
    const val SUM = 1; const val MIN = 2; const val MAX = 3; const val COUNT = 4; const val COUNT_STAR = 5; const val AVG = 6

    // postfix program tokens (QE_TOK_*)
    const val TOK_COL = 1; const val TOK_LIT = 2; const val TOK_ADD = 3; const val TOK_SUB = 4; const val TOK_MUL = 5; const val TOK_DIV = 6

    const val DETERMINISTIC = 1 // aggCreate flag: exact fixed-point fp64 SUM / AVG

    @JvmStatic external fun abiVersion(): Int

    // context: one per thread (an ExecutionContext per coroutine worker, K:1309-1313)
    @JvmStatic external fun ctxCreate(device: Int): Long
    @JvmStatic external fun ctxDestroy(ctx: Long)
    @JvmStatic external fun ctxSynchronize(ctx: Long)

    // columns (ColumnVector, K:24-27)
    @JvmStatic external fun columnAllocate(ctx: Long, type: Int, rows: Long, utf8Bytes: Long, nullable: Boolean): Long
    @JvmStatic external fun columnFree(col: Long)
    @JvmStatic external fun columnLength(col: Long): Long
    @JvmStatic external fun columnType(col: Long): Int
    @JvmStatic external fun columnNullable(col: Long): Boolean
    @JvmStatic external fun columnFromLongs(ctx: Long, type: Int, values: LongArray, validity: ByteArray?): Long
    @JvmStatic external fun columnFromDoubles(ctx: Long, values: DoubleArray, validity: ByteArray?): Long
    @JvmStatic external fun columnFromUtf8(ctx: Long, offsets: IntArray, data: ByteArray, validity: ByteArray?): Long
    @JvmStatic external fun columnToLongs(ctx: Long, col: Long, out: LongArray)
    @JvmStatic external fun columnToDoubles(ctx: Long, col: Long, out: DoubleArray)
    @JvmStatic external fun columnValidity(ctx: Long, col: Long): ByteArray?
    @JvmStatic external fun columnUtf8Offsets(ctx: Long, col: Long): IntArray
    @JvmStatic external fun columnUtf8Bytes(ctx: Long, col: Long): ByteArray
    @JvmStatic external fun generate(ctx: Long, type: Int, rows: Long, dist: Int, param: Long, seed: Long, colId: Long,
                                     row0: Long, nullPermille: Int): Long

    // RecordBatch over the Arrow C Data Interface (org.apache.arrow.c.ArrowSchema / ArrowArray addresses)
    @JvmStatic external fun importBatch(ctx: Long, schemaAddr: Long, arrayAddr: Long): Long
    @JvmStatic external fun batchDestroy(batch: Long)
    @JvmStatic external fun batchNumColumns(batch: Long): Int
    @JvmStatic external fun batchColumn(batch: Long, i: Int): Long
    @JvmStatic external fun batchColumnName(batch: Long, i: Int): String
    @JvmStatic external fun exportColumns(ctx: Long, cols: LongArray, names: Array<String>, schemaAddr: Long, arrayAddr: Long)

    // Expression.evaluate (K:448-450): rhs = 0 means the literal (litType, litBits, litNull)
    @JvmStatic external fun evalArith(ctx: Long, op: Int, lhs: Long, rhs: Long, litType: Int, litBits: Long, litNull: Boolean): Long
    @JvmStatic external fun evalCmp(ctx: Long, op: Int, lhs: Long, rhs: Long, litType: Int, litBits: Long, litNull: Boolean): Long
    @JvmStatic external fun evalBool(ctx: Long, op: Int, lhs: Long, rhs: Long): Long
    @JvmStatic external fun castToDouble(ctx: Long, input: Long): Long

    // SelectionExec
    @JvmStatic external fun filterCount(ctx: Long, mask: Long): Long
    @JvmStatic external fun filter(ctx: Long, mask: Long, inputs: LongArray): LongArray

    // global aggregate: {rows, count, type, valid, sum, min, max, avg bits}
    @JvmStatic external fun aggGlobal(ctx: Long, col: Long, mask: Long): LongArray

    // fused plans
    @JvmStatic external fun fusedSpec(maskCol: Int, termCol: IntArray, termOp: IntArray, termRhsCol: IntArray,
                                      termLitType: IntArray, termLitBits: LongArray, keyCols: IntArray, progLen: IntArray,
                                      tokOp: IntArray, tokArg: IntArray, tokLitType: IntArray, tokLitBits: LongArray): Long
    @JvmStatic external fun selectSpec(maskCol: Int, termCol: IntArray, termOp: IntArray, termRhsCol: IntArray,
                                       termLitType: IntArray, termLitBits: LongArray, progLen: IntArray, tokOp: IntArray,
                                       tokArg: IntArray, tokLitType: IntArray, tokLitBits: LongArray): Long
    @JvmStatic external fun specFree(spec: Long)

    // HashAggregateExec (K:605-660). keyTypes may hold UTF8: the state keeps the dictionaries, updates
    // take the Utf8 key columns, aggFinalize returns Utf8 key columns, aggMergeInto / aggExchange
    // merge by key content.
    @JvmStatic external fun aggCreate(ctx: Long, keyTypes: IntArray, fns: IntArray, inputTypes: IntArray,
                                      expectedGroups: Long, flags: Int): Long
    @JvmStatic external fun aggDestroy(agg: Long)
    @JvmStatic external fun aggReset(agg: Long)
    @JvmStatic external fun aggSetAsync(agg: Long, enable: Boolean)
    @JvmStatic external fun aggSetRowBase(agg: Long, rowBase: Long)
    @JvmStatic external fun aggUpdate(agg: Long, keyCols: LongArray, inputCols: LongArray, maskCol: Long)
    @JvmStatic external fun aggUpdateFused(agg: Long, cols: LongArray, spec: Long)
    @JvmStatic external fun aggNumGroups(agg: Long): Long
    @JvmStatic external fun aggFinalize(agg: Long): LongArray
    @JvmStatic external fun aggMergeInto(owner: Long, partial: Long)
    @JvmStatic external fun aggLastKernelMs(agg: Long): Double

    // ProjectionExec over SelectionExec, pipelined (K:582-603)
    @JvmStatic external fun selectAllocateOutputs(ctx: Long, spec: Long, cols: LongArray): LongArray
    @JvmStatic external fun selectProjectAsync(ctx: Long, cols: LongArray, spec: Long, outs: LongArray): Long
    @JvmStatic external fun selectProjectWait(pending: Long, outs: LongArray): Long

    // Utf8 codes for callers that encode keys themselves (K:620-627); aggregates need none of these
    @JvmStatic external fun dictCreate(ctx: Long, expected: Long): Long
    @JvmStatic external fun dictDestroy(dict: Long)
    @JvmStatic external fun dictEncode(ctx: Long, dict: Long, input: Long): Long
    @JvmStatic external fun dictDecode(ctx: Long, dict: Long, codes: Long): Long

    // CsvDataSource.scan on the device (K:276-357)
    @JvmStatic external fun csvParse(ctx: Long, data: java.nio.ByteBuffer, nbytes: Long, delimiter: Int, hasHeader: Boolean,
                                     fields: IntArray): Long
    @JvmStatic external fun csvRecordEnd(data: java.nio.ByteBuffer, nbytes: Long, eof: Boolean): Long
    @JvmStatic external fun csvRows(table: Long): Long
    @JvmStatic external fun csvColumn(table: Long, i: Int): Long
    @JvmStatic external fun csvDestroy(table: Long)

    // main()'s partial -> final merge across GPUs over RCCL (K:1309-1325)
    @JvmStatic external fun commUniqueId(): ByteArray
    @JvmStatic external fun commCreate(ctx: Long, world: Int, rank: Int, id: ByteArray): Long
    @JvmStatic external fun commDestroy(comm: Long)
    @JvmStatic external fun aggExchange(comm: Long, partial: Long, owner: Long, slotRecords: Long): Long
}
