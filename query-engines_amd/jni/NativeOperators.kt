// NativeOperators.kt — the device-backed operators, to be APPENDED to kquerydiy/src/Main.kt.
//
// The reference's operator API is file-private (ColumnVector K:24, RecordBatch K:56,
// DataSource K:63, PhysicalPlan K:442, Expression K:448, AggregateExpression K:514), so these
// classes live in the same file. They keep the reference's interfaces and only replace the
// evaluation inside them by NativeEngine calls (libqe_jni.so -> libqe_hip.so). Selection point:
// ExecutionContext.execute (K:415-419) calls createNativePhysicalPlan instead of
// createPhysicalPlan; ExecutionContext.csv (K:395-397) may register NativeCsvDataSource.
//
// Columns stay in HBM between operators: a RecordBatch of NativeColumnVector carries device
// handles; only getValue (printQueryResult, K:1344-1353) copies a column to the host, once.
// Device memory is released by a java.lang.ref.Cleaner when a vector becomes unreachable
// (qe_device_free may run on the cleaner's thread: the allocator is locked and the block is
// reused only after the work queued on its stream). Names outside Main.kt's import block
// (K:1-17) are written fully qualified, so this text appends as is.

private object Native {
    val cleaner: java.lang.ref.Cleaner = java.lang.ref.Cleaner.create()

    // one HIP context (and stream) per thread: the reference runs one ExecutionContext per
    // coroutine worker (K:1309-1313, K:1333), and a native ctx must not be shared between threads
    private val perThread = ThreadLocal.withInitial { NativeEngine.ctxCreate(0) }
    fun ctx(): Long = perThread.get()

    fun typeOf(t: ArrowType): Int = when {
        t == ArrowTypes.DoubleType -> NativeEngine.FLOAT64
        t == ArrowTypes.StringType -> NativeEngine.UTF8
        t is ArrowType.Int && t.bitWidth == 64 -> NativeEngine.INT64
        t is ArrowType.Int && t.bitWidth == 32 -> NativeEngine.INT32
        t is ArrowType.Int && t.bitWidth == 8 && !t.isSigned -> NativeEngine.UINT8
        t is ArrowType.Bool -> NativeEngine.BOOL
        t is ArrowType.Date -> NativeEngine.DATE32
        else -> throw IllegalStateException("no device type for $t") // K:469
    }
}

// ColumnVector (K:24-27) over a device column handle. `owner` keeps alive what a view points into
// (a device batch or CSV table); columnFree releases an owned handle's device blocks, only the
// handle of a view.
private class NativeColumnVector(val handle: Long, private val owner: Any? = null) : ColumnVector {
    val type: Int = NativeEngine.columnType(handle)
    private val n: Int = NativeEngine.columnLength(handle).toInt()
    private val host: Array<Any?> by lazy { download() }

    init {
        val h = handle
        Native.cleaner.register(this) { NativeEngine.columnFree(h) } // frees only the struct for a view
    }

    override fun getValue(i: Int): Any? = host[i]
    override fun size(): Int = n

    // the values ArrowFieldVector.getValue returns (K:178-197): Double, String, else the boxed value
    private fun download(): Array<Any?> {
        val ctx = Native.ctx()
        val valid = NativeEngine.columnValidity(ctx, handle)
        fun ok(i: Int) = valid == null || ((valid[i shr 3].toInt() shr (i and 7)) and 1) == 1
        return when (type) {
            NativeEngine.FLOAT64 -> DoubleArray(n).also { NativeEngine.columnToDoubles(ctx, handle, it) }
                .let { v -> Array(n) { i -> if (ok(i)) v[i] else null } }
            NativeEngine.UTF8 -> {
                val off = NativeEngine.columnUtf8Offsets(ctx, handle)
                val bytes = NativeEngine.columnUtf8Bytes(ctx, handle)
                Array(n) { i -> if (ok(i)) String(bytes, off[i], off[i + 1] - off[i]) else null }
            }
            else -> LongArray(n).also { NativeEngine.columnToLongs(ctx, handle, it) }
                .let { v -> Array(n) { i -> if (ok(i)) (if (type == NativeEngine.BOOL) v[i] != 0L else v[i]) else null } }
        }
    }
}

// Any ColumnVector -> a device column handle: a NativeColumnVector as is, a host Arrow vector
// (ArrowFieldVector, K:176) through the Arrow C Data Interface, one H2D copy.
private fun toDevice(v: ColumnVector): NativeColumnVector = when (v) {
    is NativeColumnVector -> v
    is ArrowFieldVector -> {
        val root = VectorSchemaRoot(listOf1(v.field))
        val batch = DeviceBatch.import(root)
        batch.column(0)
    }
    else -> throw IllegalStateException("cannot move ${v.javaClass.name} to the device")
}

// A RecordBatch's Arrow vectors in HBM (qe_batch_import); columns are views that keep it alive.
private class DeviceBatch private constructor(val handle: Long) {
    init {
        val h = handle
        Native.cleaner.register(this) { NativeEngine.batchDestroy(h) }
    }

    fun column(i: Int) = NativeColumnVector(NativeEngine.batchColumn(handle, i), this)

    companion object {
        fun import(root: VectorSchemaRoot): DeviceBatch {
            val alloc = RootAllocator(Long.MAX_VALUE)
            org.apache.arrow.c.ArrowArray.allocateNew(alloc).use { array ->
                org.apache.arrow.c.ArrowSchema.allocateNew(alloc).use { schema ->
                    org.apache.arrow.c.Data.exportVectorSchemaRoot(alloc, root, null, array, schema)
                    try { // qe_batch_import copies to HBM; the producer's structs are released here
                        return DeviceBatch(NativeEngine.importBatch(Native.ctx(), schema.memoryAddress(), array.memoryAddress()))
                    } finally {
                        array.release()
                        schema.release()
                    }
                }
            }
        }
    }
}

// CastExpression (K:772-805) on the device: Utf8 -> Double with Double.parseDouble semantics;
// a bad string throws NumberFormatException like `vv.toDouble()` (K:791).
private class NativeCastExpression(private val expr: Expression, private val dataType: ArrowType) : Expression {
    override fun evaluate(input: RecordBatch): ColumnVector {
        if (dataType != ArrowTypes.DoubleType) throw IllegalStateException("Cast to $dataType is not supported") // K:799
        val v = toDevice(expr.evaluate(input))
        if (v.type != NativeEngine.UTF8) throw IllegalStateException("Cannot cast value to Double") // K:792
        return NativeColumnVector(NativeEngine.castToDouble(Native.ctx(), v.handle))
    }

    override fun toString() = "CAST($expr AS $dataType)"
}

// Arithmetic (ADD..DIV) or comparison (EQ..GE) of a column with a column or a literal (build-
// defined; the reference's expression set has none, SURVEY §0). int64 wraps like Long, x / 0 is
// null, an fp64 operand promotes; a comparison gives a BOOL column.
private class NativeBinaryExpression(
    private val op: Int, private val l: Expression, private val r: Expression?, private val literal: Any? = null,
) : Expression {
    override fun evaluate(input: RecordBatch): ColumnVector {
        val ctx = Native.ctx()
        val lv = toDevice(l.evaluate(input))
        val rv = r?.let { toDevice(it.evaluate(input)) }
        val litType = if (literal is Double) NativeEngine.FLOAT64 else NativeEngine.INT64
        val litBits = when (literal) {
            is Double -> java.lang.Double.doubleToRawLongBits(literal)
            is Number -> literal.toLong()
            else -> 0L
        }
        val rh = rv?.handle ?: 0L
        val out = if (op >= NativeEngine.EQ) NativeEngine.evalCmp(ctx, op, lv.handle, rh, litType, litBits, r == null && literal == null)
                  else NativeEngine.evalArith(ctx, op, lv.handle, rh, litType, litBits, r == null && literal == null)
        return NativeColumnVector(out)
    }
}

// HashAggregateExec (K:605-660) on the device: every input batch is one aggregate update, then ONE
// output batch (K:649-650). Utf8 keys go in as they are: the native state keeps their dictionaries
// (a lone Utf8 key like K:1336's VendorID gets wide codes — values of up to 7 bytes are their own
// code, and a CSV column's length bound lets them skip the dictionary entirely) and finalize hands
// the strings back. MAX follows MaxAccumulator (K:538-561). A MAX over a Utf8 column is the
// reference's own operator: its accumulator keeps the first String of a group with no type check
// and throws UnsupportedOperationException at the second (K:541-550), row-order behaviour the
// device has no use for; that row loop reads these batches through NativeColumnVector.getValue.
// (Called directly, aggCreate throws the same UnsupportedOperationException for a Utf8 MAX input.)
private class NativeHashAggregateExec(
    private val input: PhysicalPlan,
    private val groupExpr: List<Expression>,
    private val aggregateExpr: List<AggregateExpression>,
    val schema: Schema,
) : PhysicalPlan {
    override fun schema() = schema

    override fun execute(): Sequence<RecordBatch> {
        val inSchema = input.schema()
        if (aggregateExpr.any { e ->
                val x = e.inputExpression()
                e is MaxExpression && x is ColumnExpression && inSchema.fields[x.i].dataType == ArrowTypes.StringType
            }) return HashAggregateExec(input, groupExpr, aggregateExpr, schema).execute() // K:615-651
        val ctx = Native.ctx()
        val fns = IntArray(aggregateExpr.size) { i ->
            when (aggregateExpr[i]) {
                is MaxExpression -> NativeEngine.MAX
                else -> throw IllegalStateException("Unsupported aggregate function: ${aggregateExpr[i]}") // K:696
            }
        }
        var agg = 0L
        try {
            input.execute().forEach { batch ->
                val keys = groupExpr.map { toDevice(it.evaluate(batch)) }
                val inputs = aggregateExpr.map { toDevice(it.inputExpression().evaluate(batch)) }
                if (agg == 0L) {
                    agg = NativeEngine.aggCreate(ctx, IntArray(keys.size) { keys[it].type }, fns,
                                                 IntArray(inputs.size) { inputs[it].type }, 0, 0)
                }
                NativeEngine.aggUpdate(agg, LongArray(keys.size) { keys[it].handle },
                                       LongArray(inputs.size) { inputs[it].handle }, 0)
            }
            if (agg == 0L) return sequenceOf(RecordBatch(schema, schema.fields.map { emptyColumn(ctx, it.dataType) }))
            return sequenceOf(RecordBatch(schema, NativeEngine.aggFinalize(agg).map { NativeColumnVector(it) }))
        } finally {
            if (agg != 0L) NativeEngine.aggDestroy(agg)
        }
    }

    private fun emptyColumn(ctx: Long, t: ArrowType) =
        NativeColumnVector(NativeEngine.columnAllocate(ctx, Native.typeOf(t), 0, 0, true))

    override fun children() = listOf1(input)
    override fun toString() = "NativeHashAggregateExec: groupExpr=$groupExpr, aggrExpr=$aggregateExpr"
}

// Projection(Selection(Scan)) as one fused select-project per batch, pipelined one batch ahead:
// batch i+1's kernels are queued before batch i's row count is read (K:582-603 over a filter).
// `spec` comes from NativeEngine.selectSpec (predicate terms over column slots + output programs).
private class NativeSelectProjectExec(
    private val input: PhysicalPlan, private val spec: Long, val schema: Schema,
) : PhysicalPlan {
    override fun schema() = schema

    override fun execute(): Sequence<RecordBatch> = sequence {
        val ctx = Native.ctx()
        var ahead: Triple<Long, LongArray, List<NativeColumnVector>>? = null // (pending, outputs, inputs kept alive)
        fun finish(p: Triple<Long, LongArray, List<NativeColumnVector>>): RecordBatch {
            NativeEngine.selectProjectWait(p.first, p.second)
            return RecordBatch(schema, p.second.map { NativeColumnVector(it) })
        }
        for (batch in input.execute()) {
            val cols = batch.fields.map { toDevice(it) }
            val handles = LongArray(cols.size) { cols[it].handle }
            val outs = NativeEngine.selectAllocateOutputs(ctx, spec, handles)
            val pending = NativeEngine.selectProjectAsync(ctx, handles, spec, outs)
            ahead?.let { yield(finish(it)) }
            ahead = Triple(pending, outs, cols)
        }
        ahead?.let { yield(finish(it)) }
    }

    override fun children() = listOf1(input)
}

// CsvDataSource (K:276-357) scanned on the device: the file goes to HBM in chunks of whole records
// and is tokenised, trimmed and unquoted there. The header and delimiter come from the reference's
// own CsvDataSource (univocity detection, K:290-297, K:332-356). Like ReaderIterator (K:239-252)
// the scan streams: a chunk of up to chunkBytes is cut after its last complete record
// (csvRecordEnd, quote-aware), parsed on the device as one batch, and its tail begins the next
// chunk; sizes are Long, so files past 2 GiB stream (the reference's monthly tripdata, K:1335).
// A record longer than the buffer doubles it. Each batch's columns are zero-copy views of its
// chunk's parsed table.
private class NativeCsvDataSource(private val filename: String, private val hasHeaders: Boolean) : DataSource {
    private val host = CsvDataSource(filename, hasHeaders, 1000, null)
    private val chunkBytes = 256 shl 20

    override fun schema(): Schema = host.schema()

    override fun scan(projection: List<String>): Sequence<RecordBatch> {
        val file = File(filename)
        if (!file.exists()) throw FileNotFoundException(file.absolutePath) // K:306-308
        val readSchema = if (projection.isNotEmpty()) schema().select(projection) else schema()
        val fields = readSchema.fields.map { f -> schema().fields.indexOfFirst { it.name == f.name } }.toIntArray()
        val delimiter = detectDelimiter(file)
        return sequence {
            java.nio.channels.FileChannel.open(file.toPath(), java.nio.file.StandardOpenOption.READ).use { ch ->
                var buf = java.nio.ByteBuffer.allocateDirect(chunkBytes)
                var header = hasHeaders // the header record is in the first chunk
                var eof = false
                while (true) {
                    while (!eof && buf.hasRemaining()) if (ch.read(buf) < 0) eof = true
                    val have = buf.position().toLong()
                    if (have == 0L) break
                    val cut = NativeEngine.csvRecordEnd(buf, have, eof)
                    if (cut == 0L) { // one record longer than the buffer
                        val bigger = java.nio.ByteBuffer.allocateDirect(Math.multiplyExact(buf.capacity(), 2))
                        buf.flip()
                        bigger.put(buf)
                        buf = bigger
                        continue
                    }
                    val table = parseChunk(buf, cut, delimiter.code, header, fields)
                    header = false
                    if (NativeEngine.csvRows(table.handle) > 0) {
                        yield(RecordBatch(readSchema, fields.indices.map { table.column(it) }))
                    }
                    buf.limit(have.toInt()) // the bytes past the cut begin the next chunk
                    buf.position(cut.toInt())
                    buf.compact()
                }
            }
        }
    }

    private fun detectDelimiter(file: File): Char {
        val head = file.bufferedReader().use { r -> generateSequence { r.readLine() }.firstOrNull { it.isNotBlank() && !it.startsWith("#") } ?: "" }
        return listOf(',', ';', '\t', '|').firstOrNull { head.contains(it) } ?: ','
    }

    // A chunk's table lives until its batch's columns are unreachable (a consumer may keep batches,
    // as toList() does), so only the Cleaner may free it. The JVM side of a table is a few objects,
    // so the heap alone need not trigger a collection while the device holds GBs of parsed chunks:
    // the device bytes of tables not yet freed are counted, and a scan that finds more than two
    // chunks' worth still held asks for a collection before parsing the next chunk; a device OOM
    // collects, waits for the Cleaner, and retries once. A streaming consumer thus stays at about
    // two chunks of device memory (ADVICE r04).
    private fun parseChunk(buf: java.nio.ByteBuffer, cut: Long, delim: Int, header: Boolean, fields: IntArray): CsvTable {
        if (CsvTable.held.get() > 2L * chunkBytes) System.gc()
        val h = try {
            NativeEngine.csvParse(Native.ctx(), buf, cut, delim, header, fields)
        } catch (e: OutOfMemoryError) {
            System.gc()
            val deadline = System.nanoTime() + 2_000_000_000L
            val before = CsvTable.held.get()
            while (CsvTable.held.get() >= before && before > 0 && System.nanoTime() < deadline) Thread.sleep(10)
            NativeEngine.csvParse(Native.ctx(), buf, cut, delim, header, fields)
        }
        return CsvTable(h, cut)
    }

    private class CsvTable(val handle: Long, bytes: Long) {
        init {
            val h = handle
            held.addAndGet(bytes)
            Native.cleaner.register(this) { NativeEngine.csvDestroy(h); held.addAndGet(-bytes) }
        }

        fun column(i: Int) = NativeColumnVector(NativeEngine.csvColumn(handle, i), this)

        companion object {
            val held = java.util.concurrent.atomic.AtomicLong() // device bytes of tables not yet freed
        }
    }
}

// createPhysicalExpr / createPhysicalPlan (K:662-706) with the device operators.
private fun createNativePhysicalExpr(expr: LogicalExpr, input: LogicalPlan): Expression = when (expr) {
    is CastExpr -> NativeCastExpression(createNativePhysicalExpr(expr.expr, input), expr.dataType)
    is Alias -> createNativePhysicalExpr(expr.expr, input)
    else -> createPhysicalExpr(expr, input) // Column / ColumnIndex: zero-copy ColumnExpression
}

private fun createNativePhysicalPlan(plan: LogicalPlan): PhysicalPlan = when (plan) {
    is Scan -> ScanExec(plan.dataSource, plan.projection)
    is Projection -> ProjectionExec(
        createNativePhysicalPlan(plan.input),
        Schema(plan.expr.map { it.toField(plan.input) }),
        plan.expr.map { createNativePhysicalExpr(it, plan.input) },
    )
    is Aggregate -> NativeHashAggregateExec(
        createNativePhysicalPlan(plan.input),
        plan.groupExpr.map { createNativePhysicalExpr(it, plan.input) },
        plan.aggExpr.map {
            when (it) {
                is Max -> MaxExpression(createNativePhysicalExpr(it.expr, plan.input))
                else -> throw IllegalStateException("Unsupported aggregate function: $it")
            }
        },
        plan.schema(),
    )
    else -> throw IllegalStateException("Unknown physical plan")
}
