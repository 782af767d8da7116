package electionguard.gpu

import electionguard.core.ElementModP
import electionguard.core.ElementModQ
import electionguard.core.GroupContext

/**
 * The L1 drop-in: an upstream `GroupContext` (electionguard-kotlin-multiplatform-jvm 1.0-SNAPSHOT,
 * build.gradle.kts:55) whose mod-p arithmetic runs on one MI355X, returned by
 * `KUtils.productionGroup()` (src/main/java/electionguard/util/KUtils.java:10-12) in place of
 * `productionGroup(LOW_MEMORY_USE, Mode4096)`.
 *
 * Kotlin interface delegation (`by base`, `by inner`) keeps every member of the upstream interfaces
 * that is not on the hot path (constants, mod-q arithmetic, serialisation, dLog, the residue test)
 * on the upstream production objects, so only the members overridden here have to match the jar:
 *   - `GroupContext.gPowP`, `Iterable<ElementModP>.multP()`;
 *   - `ElementModP.powP`, `times`, `multInv`, `div`, `acceleratePow`, `compareTo`;
 *   - the element constructors and constants, which wrap, so that every ElementModP reachable from
 *     this context is a [GpuElementModP] (upstream's ProductionElementModP.times would reject one
 *     of ours as an argument, see `unwrap`).
 * Each per-element call goes through the library's coalescer (eg_powp_one / eg_gpowp_one /
 * eg_multp_one): the upstream 11-thread loops (RunRemoteWorkflowTest.java:140,180) share GPU
 * batches without being rewritten, and batches that fit one resident round run on the
 * latency-shaped kernels (include/eg_hip.h, eg_powp_one).  Batch callers keep
 * [GpuGroupContext]'s list and ballot entry points, reachable as [gpu].
 *
 * ConvertCommonProto.java:46-47,55-56 constructs elements with `new ProductionElementModP(elem,
 * (ProductionGroupContext) group)`; with this context it calls `group.binaryToElementModP(bytes)`
 * instead (INTEGRATION.md §1): the cast is the one reference line the swap changes.
 *
 * Not compiled here (no JDK or kotlinc in the image); tests/test_kotlin_adapter.py checks the
 * overrides against the member list in tests/golden/reference_signatures.json and that every
 * hot-path member reaches the GPU context.
 */
class GpuProductionGroupContext(val base: GroupContext, val gpu: GpuGroupContext) : GroupContext by base {

    /** KUtils.productionGroup(): the reference's group on `device`. */
    companion object {
        @JvmStatic
        fun production(base: GroupContext, device: Int = 0): GpuProductionGroupContext =
            GpuProductionGroupContext(base, GpuGroupContext(base, GpuGroupContext.ProductionMode.Mode4096, device))
    }

    internal fun wrap(e: ElementModP): GpuElementModP = if (e is GpuElementModP) e else GpuElementModP(e, this)

    override val ONE_MOD_P: ElementModP get() = wrap(base.ONE_MOD_P)
    override val G_MOD_P: ElementModP get() = wrap(base.G_MOD_P)
    override val GINV_MOD_P: ElementModP get() = wrap(base.GINV_MOD_P)
    override val G_SQUARED_MOD_P: ElementModP get() = wrap(base.G_SQUARED_MOD_P)

    override fun isCompatible(ctx: GroupContext): Boolean =
        base.isCompatible(if (ctx is GpuProductionGroupContext) ctx.base else ctx)

    override fun binaryToElementModP(b: ByteArray): ElementModP? = base.binaryToElementModP(b)?.let { wrap(it) }

    /** g^e on the fixed-base table of g (eg_gpowp_one). */
    override fun gPowP(e: ElementModQ): ElementModP = wrap(gpu.gPowP(e))

    /** Π of the elements, one product-tree launch (eg_prod_reduce); 1 for an empty iterable. */
    override fun Iterable<ElementModP>.multP(): ElementModP = wrap(gpu.prodP(this.map { unwrap(it) }))

    override fun dLogG(p: ElementModP, maxResult: Int): Int? = base.dLogG(unwrap(p), maxResult)

    override fun equals(other: Any?): Boolean =
        other is GpuProductionGroupContext && other.base == base && other.gpu.device() == gpu.device()

    override fun hashCode(): Int = base.hashCode()
    override fun toString(): String = "GpuProductionGroupContext(" + base + ", device " + gpu.device() + ")"
}

/** The upstream element under a GPU element: arguments of upstream operations must be theirs. */
internal fun unwrap(e: ElementModP): ElementModP = if (e is GpuElementModP) e.inner else e

/**
 * An upstream ElementModP whose mod-p operations run through the GPU context; the value, its
 * bytes (`byteArray()`, the wire layout of ConvertCommonProto.java:117-121) and every other member
 * are the upstream element's.
 */
class GpuElementModP(val inner: ElementModP, private val ctx: GpuProductionGroupContext) : ElementModP by inner {
    override val context: GroupContext get() = ctx

    /** this^e (eg_powp_one: coalesced with the other threads' calls into one GPU batch). */
    override infix fun powP(e: ElementModQ): ElementModP = ctx.wrap(ctx.gpu.powP(inner, e))

    /** this * other mod p (eg_multp_one). */
    override operator fun times(other: ElementModP): ElementModP = ctx.wrap(ctx.gpu.multP(inner, unwrap(other)))

    /** this^(p-2) (eg_multinv_batch; 0 maps to 0 like BigInteger.modPow). */
    override fun multInv(): ElementModP = ctx.wrap(ctx.gpu.multInv(listOf(inner))[0])

    override infix operator fun div(denominator: ElementModP): ElementModP = this * denominator.multInv()

    /** The GPU's tables are per context (g, the election key), not per element: nothing to build. */
    override fun acceleratePow(): ElementModP = this

    override fun compareTo(other: ElementModP): Int = inner.compareTo(unwrap(other))

    override fun equals(other: Any?): Boolean = other is ElementModP && inner == unwrap(other)
    override fun hashCode(): Int = inner.hashCode()
    override fun toString(): String = inner.toString()
}
