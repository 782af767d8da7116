package electionguard.gpu

import electionguard.core.ElementModP
import electionguard.core.ElementModQ
import electionguard.core.GroupContext
import java.lang.ref.Cleaner
import java.lang.ref.WeakReference
import java.lang.reflect.InvocationTargetException
import java.lang.reflect.Proxy
import java.math.BigInteger

/**
 * The L1 drop-in: an upstream `GroupContext` (electionguard-kotlin-multiplatform-jvm 1.0-SNAPSHOT,
 * build.gradle.kts:55) whose mod-p arithmetic runs on one MI355X, returned by
 * `KUtils.productionGroup()` (src/main/java/electionguard/util/KUtils.java:10-12) in place of
 * `productionGroup(LOW_MEMORY_USE, Mode4096)`.
 *
 * Kotlin interface delegation (`by base`) keeps every member of the upstream interfaces that is not on
 * the hot path (constants, mod-q arithmetic, serialisation, dLog) on the upstream production objects,
 * so only the members overridden here have to match the jar:
 *   - `GroupContext.gPowP`, `Iterable<ElementModP>.multP()`;
 *   - `ElementModP.powP`, `times`, `multInv`, `div`, `acceleratePow`, `isValidResidue`, `compareTo`;
 *   - the element constructors and constants, which wrap, so that every ElementModP reachable from
 *     this context is a [GpuElementModP].
 *
 * Upstream calls the group one element at a time from 11 threads (RunRemoteWorkflowTest.java:140-141,
 * 179-181), and a result is usually consumed a few calls later (by a product, then a hash).  So these
 * calls are DEFERRED, as in the C++ mirror (host/electionguard.hpp `Deferred`): each returns at once an
 * element holding an expression `(b_1 ... b_k)^e * F0^f0 * F1^f1` over resolved values and registered
 * fixed-base tables (g's; an accelerated element's, `acceleratePow`, e.g. the election key), and
 * products / powers combine on the host where that is exact:
 *   - `x * y` merges fixed-base terms (a base in both adds its exponents mod q when it has order q) and
 *     variable parts (two products, or two powers with the same exponent): g^v * alpha^c is ONE job;
 *   - `x powP e` on a pure fixed-base expression of order-q bases multiplies its exponents by e mod q;
 *     on a product without an exponent it sets the exponent (the contest aggregate (prod alpha)^c);
 *   - otherwise the operand is resolved and the result starts a new expression.
 * The first time a thread needs a value (`byteArray()`, a comparison, any upstream member, a hash of
 * the elements), every expression it created and has not merged is submitted (`eg_mexp_submit`: one
 * job each, coalesced with the other threads' into one launch) and it waits for the one it needs: one
 * GPU round trip per point where upstream's code looks at a value.  Results are the same integers.
 * `multInv` / `div` of a value that is not a fixed-base expression stay on the upstream element (host
 * BigInteger), as does everything off the hot path.  Measured through the same API in C++
 * (tests/cpp/percall_workflow.cpp, final library profiles/r05zs_percall_workflow.json): encrypt 2.2x,
 * verify 2.3x, the one-thread tally 6.9x the CPU port on 11 threads; the caller's thread count
 * (nthreads = 11 at RunRemoteWorkflowTest.java:140,180) against the batch rate: INTEGRATION.md §1.
 *
 * A trustee's context ([trustee]) runs every exponentiation on the constant-time schedules
 * (`eg_ctx_set_ct_pow`): its secret shares s_i, P_l(x_i) reach `powP` through this adapter
 * (RunRemoteDecryptingTrustee.java:189-193,227-232).
 *
 * ConvertCommonProto.java:46-47,55-56 constructs elements with `new ProductionElementModP(elem,
 * (ProductionGroupContext) group)`; with this context it calls `group.binaryToElementModP(bytes)`
 * instead (INTEGRATION.md §1): the cast is the one reference line the swap changes.
 *
 * UNBUILT: there is no JDK or kotlinc in the image, so this source has never been compiled against the
 * upstream jar; tests/test_kotlin_adapter.py checks its overrides against the member list restated in
 * tests/golden/upstream_group_api.json and that every hot-path member reaches the deferred algebra.
 */
class GpuProductionGroupContext(val base: GroupContext, val gpu: GpuGroupContext) : GroupContext by base {

    companion object {
        /** KUtils.productionGroup(): the reference's group on `device`. */
        @JvmStatic
        fun production(base: GroupContext, device: Int = 0): GpuProductionGroupContext =
            GpuProductionGroupContext(base, GpuGroupContext(base, GpuGroupContext.ProductionMode.Mode4096, device))

        /** A DecryptingTrustee's group: every exponentiation on the constant-time schedules. */
        @JvmStatic
        fun trustee(base: GroupContext, device: Int = 0): GpuProductionGroupContext =
            production(base, device).also { it.gpu.setConstantTime(true) }

        private const val P_BYTES = 512
        private const val MAX_JOB_BASES = 16
        private val CLEANER: Cleaner = Cleaner.create()
    }

    internal val q: BigInteger = BigInteger(1, gpu.qBytes())
    internal val p: BigInteger = BigInteger(1, gpu.pBytes())
    private val gBytes: ByteArray = GpuGroupContext.fixed(base.G_MOD_P.byteArray(), P_BYTES)
    private val accelerated = java.util.concurrent.ConcurrentHashMap<BigInteger, GpuGroupContext.Table>()
    private val pending = ThreadLocal.withInitial { ArrayList<WeakReference<Deferred>>() }

    /** false: every per-element call resolves at once (one blocking GPU round trip each). */
    @Volatile
    var deferred: Boolean = true

    internal fun wrap(e: ElementModP): GpuElementModP = if (e is GpuElementModP) e else GpuElementModP(Cell.value(e), this)

    override val ONE_MOD_P: ElementModP get() = wrap(base.ONE_MOD_P)
    override val G_MOD_P: ElementModP get() = wrap(base.G_MOD_P)
    override val GINV_MOD_P: ElementModP get() = wrap(base.GINV_MOD_P)
    override val G_SQUARED_MOD_P: ElementModP get() = wrap(base.G_SQUARED_MOD_P)

    override fun isCompatible(ctx: GroupContext): Boolean =
        base.isCompatible(if (ctx is GpuProductionGroupContext) ctx.base else ctx)

    override fun binaryToElementModP(b: ByteArray): ElementModP? = base.binaryToElementModP(b)?.let { wrap(it) }

    /** g^e: one fixed-base job over g's 16-bit table when the value is first needed. */
    override fun gPowP(e: ElementModQ): ElementModP = wrap(defer(Form.fixed(gpu.gTable(), big(e))))

    /** The product of the elements (1 for none): one product-tree launch (eg_prod_reduce). */
    override fun Iterable<ElementModP>.multP(): ElementModP = wrap(gpu.prodP(this.map { wrap(it).inner }))

    override fun dLogG(p: ElementModP, maxResult: Int): Int? = base.dLogG(wrap(p).inner, maxResult)

    override fun equals(other: Any?): Boolean =
        other is GpuProductionGroupContext && other.base == base && other.gpu.device() == gpu.device()

    override fun hashCode(): Int = base.hashCode()
    override fun toString(): String = "GpuProductionGroupContext(" + base + ", device " + gpu.device() + ")"

    /** Resolve several values with one flush: they share the library's next batch (a hash's inputs). */
    fun resolveAll(xs: List<ElementModP>) {
        flushThread()
        for (x in xs) (x as? GpuElementModP)?.cell?.deferred?.submitIfNew()
        for (x in xs) x.byteArray()
    }

    // ---------------------------------------------------------------- the deferred algebra
    private fun big(e: ElementModQ): BigInteger = BigInteger(1, e.byteArray())

    internal fun powP(x: GpuElementModP, e: ElementModQ): GpuElementModP {
        val eb = big(e)
        val (f, expr) = formOf(x)
        if (f.nb == 0 && f.tabs.isNotEmpty()) {
            if (f.tabs.size == 1 && f.fes[0] == BigInteger.ONE) return consumeAnd(x, expr, Form(null, 0, null, f.tabs, listOf(eb)))
            if (f.tabs.all { it.orderQ })
                return consumeAnd(x, expr, Form(null, 0, null, f.tabs, f.fes.map { it.mod(q).multiply(eb.mod(q)).mod(q) }))
        } else if (f.nb > 0 && f.tabs.isEmpty() && f.exp == null) {
            return consumeAnd(x, expr, Form(f.buf, f.nb, eb, f.tabs, f.fes))
        }
        return defer(Form.value(x.valueBytes()).withExp(eb))
    }

    internal fun times(a: GpuElementModP, b: GpuElementModP): GpuElementModP {
        val (fa, ea) = formOf(a)
        val (fb, eb) = formOf(b)
        val m = merge(fa, fb)
        if (m != null) {
            if (ea) a.cell.deferred?.consume()
            if (eb) b.cell.deferred?.consume()
            return defer(m)
        }
        return defer(Form.value(a.valueBytes()).append(Form.value(b.valueBytes())))
    }

    /** a^-1: a pure fixed-base expression of order-q bases negates its exponents; else upstream's. */
    internal fun multInv(x: GpuElementModP): GpuElementModP {
        val (f, expr) = formOf(x)
        if (f.nb == 0 && f.tabs.isNotEmpty() && f.tabs.all { it.orderQ })
            return consumeAnd(x, expr, Form(null, 0, null, f.tabs, f.fes.map { q.subtract(it.mod(q)).mod(q) }))
        return wrap(x.inner.multInv())
    }

    /** 0 <= x < p and x^q == 1, the power deferred with this thread's other jobs. */
    internal fun isValidResidue(x: GpuElementModP): Boolean {
        val v = x.valueBytes()
        if (BigInteger(1, v) >= p) return false
        return BigInteger(1, defer(Form.value(v).withExp(q)).valueBytes()) == BigInteger.ONE
    }

    /** acceleratePow(): a 16-bit table of x's value (cached by value), its order checked. */
    internal fun accelerate(x: GpuElementModP): GpuElementModP {
        val inner = x.inner
        val t = accelerated.computeIfAbsent(BigInteger(1, x.valueBytes())) { gpu.table(inner, 16) }
        return GpuElementModP(Cell.value(inner), this, t)
    }

    // x as an expression (and whether that is x's own deferred expression, to mark it merged): an
    // accelerated value and g are their table to the power 1
    private fun formOf(x: GpuElementModP): Pair<Form, Boolean> {
        x.accel?.let { return Pair(Form.fixed(it, BigInteger.ONE), false) }
        val d = x.cell.deferred
        if (d != null && (!x.cell.isResolved() || d.form.nb == 0)) return Pair(d.form, true)
        val v = x.valueBytes()
        if (v.contentEquals(gBytes)) return Pair(Form.fixed(gpu.gTable(), BigInteger.ONE), false)
        return Pair(Form.value(v), false)
    }

    private fun consumeAnd(x: GpuElementModP, expr: Boolean, f: Form): GpuElementModP {
        if (expr) x.cell.deferred?.consume()
        return defer(f)
    }

    private fun merge(x: Form, y: Form): Form? {
        if (x.nb > 0 && y.nb > 0 && x.exp != y.exp) return null
        val tabs = ArrayList(x.tabs)
        val fes = ArrayList(x.fes)
        for (t in y.tabs.indices) {
            val k = tabs.indexOf(y.tabs[t])
            if (k >= 0) {
                if (!tabs[k].orderQ) return null
                fes[k] = fes[k].mod(q).add(y.fes[t].mod(q)).mod(q)
            } else {
                if (tabs.size == 2) return null
                tabs.add(y.tabs[t])
                fes.add(y.fes[t])
            }
        }
        return when {
            y.nb == 0 -> Form(x.buf, x.nb, x.exp, tabs, fes)
            x.nb == 0 -> Form(y.buf, y.nb, y.exp, tabs, fes)
            else -> Form(x.buf, x.nb, x.exp, tabs, fes).append(y)
        }
    }

    internal fun defer(f0: Form): GpuElementModP {
        val f = if (f0.nb == 0 && f0.exp != null) Form(null, 0, null, f0.tabs, f0.fes) else f0  // 1^e = 1
        if (f.nb == 0 && f.tabs.isEmpty()) return wrap(base.ONE_MOD_P)
        if (f.nb == 1 && f.exp == null && f.tabs.isEmpty())
            return wrap(base.binaryToElementModP(f.bases()[0]) ?: throw ArithmeticException("not an ElementModP"))
        val d = Deferred(this, f)
        val e = GpuElementModP(Cell.deferred(d), this)
        if (!deferred) {
            e.inner
            return e
        }
        val queue = pending.get()
        queue.add(WeakReference(d))
        if (queue.size >= 4096 && queue.size % 4096 == 0)
            queue.removeAll { w -> w.get()?.let { !it.isNew() || it.consumed } ?: true }
        return e
    }

    internal fun resolve(d: Deferred): ElementModP {
        flushThread()
        return d.value()
    }

    private fun flushThread() {
        val queue = pending.get()
        for (w in queue) {
            val d = w.get() ?: continue
            if (!d.consumed && !d.form.pureProduct) d.submitIfNew()
        }
        queue.clear()
    }

    // one eg_mexp_submit job for a form (> 16 bases are folded first with eg_prod_reduce)
    internal fun submit(f: Form): Long {
        var bases = f.bases()
        if (bases.size > MAX_JOB_BASES)
            bases = listOf(GpuGroupContext.fixed(gpu.prodP(bases.map { wrap(base.binaryToElementModP(it)!!).inner }).byteArray(), P_BYTES))
        val packed = ByteArray(bases.size * P_BYTES)
        for (i in bases.indices) System.arraycopy(bases[i], 0, packed, i * P_BYTES, P_BYTES)
        fun q32(x: BigInteger?): ByteArray? = x?.let { GpuGroupContext.fixed(it.toByteArray(), 32) }
        return gpu.submitJob(packed, bases.size, q32(f.exp), f.tabs.getOrNull(0), q32(f.fes.getOrNull(0)),
            f.tabs.getOrNull(1), q32(f.fes.getOrNull(1)))
    }

    internal fun waitJob(ticket: Long): ElementModP =
        base.binaryToElementModP(gpu.waitJob(ticket)) ?: throw ArithmeticException("result is not an ElementModP")

    internal fun cleaner(): Cleaner = CLEANER
}

/** The bases of product expressions: appended in place while the tail is unshared (an accumulator). */
internal class Bases {
    val list = ArrayList<ByteArray>()
}

/** (bases[0, nb))^exp * prod_t tabs[t]^fes[t]; immutable (a shared buffer is only ever appended). */
internal class Form(
    val buf: Bases?, val nb: Int, val exp: BigInteger?,
    val tabs: List<GpuGroupContext.Table>, val fes: List<BigInteger>,
) {
    companion object {
        fun fixed(t: GpuGroupContext.Table, e: BigInteger) = Form(null, 0, null, listOf(t), listOf(e))
        fun value(v: ByteArray): Form {
            val b = Bases()
            b.list.add(v)
            return Form(b, 1, null, emptyList(), emptyList())
        }
    }

    val pureProduct: Boolean get() = exp == null && tabs.isEmpty()

    fun withExp(e: BigInteger) = Form(buf, nb, e, tabs, fes)

    fun bases(): List<ByteArray> = if (buf == null) emptyList() else synchronized(buf) { ArrayList(buf.list.subList(0, nb)) }

    /** this's bases then y's (in place when nobody extended this's buffer yet) */
    fun append(y: Form): Form {
        val ys = y.bases()
        val b = buf!!
        synchronized(b) {
            if (b.list.size == nb) {
                b.list.addAll(ys)
                return Form(b, nb + ys.size, exp, tabs, fes)
            }
            val nbuf = Bases()
            nbuf.list.addAll(b.list.subList(0, nb))
            nbuf.list.addAll(ys)
            return Form(nbuf, nb + ys.size, exp, tabs, fes)
        }
    }
}

/** A job's ticket; waited exactly once, by the value or (if the value was never read) by the cleaner. */
internal class Ticket(@Volatile var t: Long) : Runnable {
    fun take(): Long = synchronized(this) { val v = t; t = 0; v }
    override fun run() {
        val x = take()
        if (x != 0L) EgHip.ticketWait(x, ByteArray(512))
    }
}

/** The evaluation state of one deferred expression. */
internal class Deferred(val ctx: GpuProductionGroupContext, val form: Form) {
    private var state = 0  // 0 expression, 1 submitted, 2 value, 3 failed
    @Volatile
    var consumed = false
        private set
    private val ticket = Ticket(0)
    private var result: ElementModP? = null
    private var failure: RuntimeException? = null

    @Synchronized
    fun isNew(): Boolean = state == 0

    @Synchronized
    fun consume() {
        if (state == 0) consumed = true
    }

    @Synchronized
    fun submitIfNew() {
        if (state == 0) submit()
    }

    private fun submit() {
        try {
            ticket.t = ctx.submit(form)
            ctx.cleaner().register(this, ticket)
            state = 1
        } catch (e: RuntimeException) {
            failure = e
            state = 3
        }
    }

    @Synchronized
    fun value(): ElementModP {
        if (state == 0) submit()
        if (state == 1) {
            state = try {
                result = ctx.waitJob(ticket.take())
                2
            } catch (e: RuntimeException) {
                failure = e
                3
            }
        }
        failure?.let { throw it }
        return result!!
    }
}

/** A value, or a deferred expression and (once read) its value. */
internal class Cell private constructor(@Volatile private var v: ElementModP?, val deferred: Deferred?) {
    companion object {
        fun value(e: ElementModP) = Cell(e, null)
        fun deferred(d: Deferred) = Cell(null, d)
    }

    fun isResolved(): Boolean = v != null

    fun value(): ElementModP {
        v?.let { return it }
        val d = deferred!!
        val r = d.ctx.resolve(d)
        v = r
        return r
    }
}

/** An ElementModP whose every (non-overridden) member resolves the value and asks the upstream element. */
internal fun forwarding(cell: Cell): ElementModP =
    Proxy.newProxyInstance(ElementModP::class.java.classLoader, arrayOf(ElementModP::class.java)) { _, m, args ->
        try {
            m.invoke(cell.value(), *(args ?: arrayOf()))
        } catch (e: InvocationTargetException) {
            throw e.targetException
        }
    } as ElementModP

/**
 * An upstream ElementModP whose mod-p operations run through the GPU context, deferred: the value, its
 * bytes (`byteArray()`, the wire layout of ConvertCommonProto.java:117-121) and every other member are
 * the upstream element's once resolved.
 */
class GpuElementModP internal constructor(
    internal val cell: Cell,
    private val ctx: GpuProductionGroupContext,
    internal val accel: GpuGroupContext.Table? = null,
) : ElementModP by forwarding(cell) {
    /** The upstream element holding the value (resolving a deferred one). */
    val inner: ElementModP get() = cell.value()

    internal fun valueBytes(): ByteArray = GpuGroupContext.fixed(inner.byteArray(), 512)

    override val context: GroupContext get() = ctx

    /** this^e: a fixed-base job for g, an accelerated element or a fixed-base expression; else base^e. */
    override infix fun powP(e: ElementModQ): ElementModP = ctx.wrap(ctx.powP(this, e))

    /** this * other: merged into one job where exact (g^v * alpha^c), else a product job. */
    override operator fun times(other: ElementModP): ElementModP = ctx.wrap(ctx.times(this, ctx.wrap(other)))

    /** this^-1: exponent negation for a fixed-base expression, else upstream's (host BigInteger). */
    override fun multInv(): ElementModP = ctx.wrap(ctx.multInv(this))

    override infix operator fun div(denominator: ElementModP): ElementModP = this * ctx.wrap(denominator).multInv()

    /** A registered fixed-base table of this value: its powP is then a fixed-base job (the election key). */
    override fun acceleratePow(): ElementModP = ctx.wrap(ctx.accelerate(this))

    override fun isValidResidue(): Boolean = ctx.isValidResidue(this)

    override fun byteArray(): ByteArray = inner.byteArray()

    override fun compareTo(other: ElementModP): Int = inner.compareTo(ctx.wrap(other).inner)

    override fun equals(other: Any?): Boolean = other is ElementModP && inner == ctx.wrap(other).inner
    override fun hashCode(): Int = inner.hashCode()
    override fun toString(): String = inner.toString()
}
