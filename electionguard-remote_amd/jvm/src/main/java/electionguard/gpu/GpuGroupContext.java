package electionguard.gpu;

import electionguard.core.ElGamalCiphertext;
import electionguard.core.ElementModP;
import electionguard.core.ElementModQ;
import electionguard.core.GroupContext;

import java.math.BigInteger;
import java.util.ArrayList;
import java.util.List;

/**
 * GPU-backed batch operations of the upstream GroupContext / ElementModP / ElementModQ
 * (electionguard-kotlin-multiplatform-jvm 1.0-SNAPSHOT, build.gradle.kts:55), for the drop-in
 * at KUtils.productionGroup() (src/main/java/electionguard/util/KUtils.java:10-12).
 *
 * The upstream context keeps constructing and serialising elements (binaryToElementModP,
 * byteArray(): the reference's wire layout, ConvertCommonProto.java:46-56,111-121); every
 * mod-p exponentiation / product of a batch runs on one MI355X through {@link EgHip}.
 * Elements are imported unchecked, like ConvertCommonProto.importElementModP; bases are
 * reduced mod p and results are canonical (java.math.BigInteger semantics, include/eg_hip.h).
 * One instance per device; calls are thread-safe (the library serialises them per context).
 */
public final class GpuGroupContext implements AutoCloseable {
  private final GroupContext group;
  private final ProductionMode mode;
  private final int device;
  private long ctx;

  /** Upstream ProductionMode (KUtils.java:5,11) plus the named EG 2.0 group. */
  public enum ProductionMode { Mode4096, Mode4096_V2 }

  /**
   * @param group the upstream context of the same group (productionGroup(LOW_MEMORY_USE, Mode4096)
   *              for Mode4096): constructs the ElementModP / ElementModQ results
   */
  public GpuGroupContext(GroupContext group, ProductionMode mode, int device) {
    this.group = group;
    this.mode = mode;
    this.device = device;
    final boolean v2 = mode == ProductionMode.Mode4096_V2;
    this.ctx = EgHip.ctxCreate(hex(v2 ? EgConstants.P_HEX_V2 : EgConstants.P_HEX, EgHip.P_BYTES),
        hex(v2 ? EgConstants.Q_HEX_V2 : EgConstants.Q_HEX, EgHip.Q_BYTES),
        hex(v2 ? EgConstants.G_HEX_V2 : EgConstants.G_HEX, EgHip.P_BYTES), device);
    // the upstream context must be the same group: its generator bytes equal ours
    if (!java.util.Arrays.equals(group.getG_MOD_P().byteArray(),
        hex(v2 ? EgConstants.G_HEX_V2 : EgConstants.G_HEX, EgHip.P_BYTES))) {
      close();
      throw new IllegalArgumentException("upstream GroupContext is not the " + mode + " group");
    }
  }

  /** KUtils.productionGroup() for device 0 with the reference's group. */
  public static GpuGroupContext production(GroupContext group) {
    return new GpuGroupContext(group, ProductionMode.Mode4096, 0);
  }

  public GroupContext group() { return group; }
  public ProductionMode mode() { return mode; }
  public int device() { return device; }
  long handle() { return ctx; }

  @Override
  public synchronized void close() {
    if (gTable16 != null) {
      gTable16.close();
      gTable16 = null;
    }
    if (ctx != 0) {
      EgHip.ctxDestroy(ctx);
      ctx = 0;
    }
  }

  // ------------------------------------------------------------------ wire packing

  /** width big-endian bytes of be (BigInteger.toByteArray() / ElementModP.byteArray() forms). */
  public static byte[] fixed(byte[] be, int width) {
    byte[] out = new byte[width];
    put(out, 0, be, width);
    return out;
  }

  static byte[] hex(String h, int width) {
    byte[] out = new byte[width];
    byte[] v = new BigInteger(h, 16).toByteArray();
    int n = Math.min(v.length, width);
    System.arraycopy(v, v.length - n, out, width - n, n);
    return out;
  }

  /** Fixed-width big-endian bytes of an element (left-padded; a leading sign byte dropped). */
  static void put(byte[] dst, int off, byte[] be, int width) {
    int skip = 0;
    while (be.length - skip > width && be[skip] == 0) skip++;
    if (be.length - skip > width) throw new IllegalArgumentException("element wider than " + width + " bytes");
    System.arraycopy(be, skip, dst, off + width - (be.length - skip), be.length - skip);
  }

  static byte[] packP(List<ElementModP> xs) {
    byte[] out = new byte[xs.size() * EgHip.P_BYTES];
    for (int i = 0; i < xs.size(); i++) put(out, i * EgHip.P_BYTES, xs.get(i).byteArray(), EgHip.P_BYTES);
    return out;
  }

  static byte[] packQ(List<ElementModQ> xs) {
    byte[] out = new byte[xs.size() * EgHip.Q_BYTES];
    for (int i = 0; i < xs.size(); i++) put(out, i * EgHip.Q_BYTES, xs.get(i).byteArray(), EgHip.Q_BYTES);
    return out;
  }

  static byte[] packTexts(List<ElGamalCiphertext> ts) {
    byte[] out = new byte[ts.size() * 2 * EgHip.P_BYTES];
    for (int i = 0; i < ts.size(); i++) {
      put(out, (2 * i) * EgHip.P_BYTES, ts.get(i).getPad().byteArray(), EgHip.P_BYTES);
      put(out, (2 * i + 1) * EgHip.P_BYTES, ts.get(i).getData().byteArray(), EgHip.P_BYTES);
    }
    return out;
  }

  ElementModP elementP(byte[] buf, int index) {
    byte[] b = java.util.Arrays.copyOfRange(buf, index * EgHip.P_BYTES, (index + 1) * EgHip.P_BYTES);
    ElementModP e = group.binaryToElementModP(b);
    if (e == null) throw new ArithmeticException("result is not an ElementModP");
    return e;
  }

  ElementModQ elementQ(byte[] buf, int offset) {
    byte[] b = java.util.Arrays.copyOfRange(buf, offset, offset + EgHip.Q_BYTES);
    ElementModQ e = group.binaryToElementModQ(b);
    if (e == null) throw new ArithmeticException("result is not an ElementModQ");
    return e;
  }

  List<ElementModP> unpackP(byte[] buf, int n) {
    List<ElementModP> out = new ArrayList<>(n);
    for (int i = 0; i < n; i++) out.add(elementP(buf, i));
    return out;
  }

  // ------------------------------------------------------------------ batched group ops

  /** out[i] = bases[i].powP(exps[i]) (ElementModP.powP, variable base). */
  public List<ElementModP> powP(List<ElementModP> bases, List<ElementModQ> exps) {
    if (bases.size() != exps.size()) throw new IllegalArgumentException("bases/exps length mismatch");
    final int n = bases.size();
    byte[] out = new byte[n * EgHip.P_BYTES];
    EgHip.powpBatch(ctx, packP(bases), packQ(exps), out, n);
    return unpackP(out, n);
  }

  /** out[i] = g^exps[i] (GroupContext.gPowP, fixed-base table of g). */
  public List<ElementModP> gPowP(List<ElementModQ> exps) {
    final int n = exps.size();
    byte[] out = new byte[n * EgHip.P_BYTES];
    EgHip.fbPowBatch(EgHip.gTable(ctx), packQ(exps), out, n);
    return unpackP(out, n);
  }

  /** out[i] = a[i].times(b[i]). */
  public List<ElementModP> multP(List<ElementModP> a, List<ElementModP> b) {
    if (a.size() != b.size()) throw new IllegalArgumentException("length mismatch");
    final int n = a.size();
    byte[] out = new byte[n * EgHip.P_BYTES];
    EgHip.multpBatch(ctx, packP(a), packP(b), out, n);
    return unpackP(out, n);
  }

  /** Iterable<ElementModP>.multP(): the product of all elements (1 for an empty list). */
  public ElementModP prodP(List<ElementModP> xs) {
    byte[] out = new byte[EgHip.P_BYTES];
    EgHip.prodReduce(ctx, packP(xs), 1, xs.size(), out);
    return elementP(out, 0);
  }

  /** out[i] = xs[i].multInv() (0 maps to 0, as x^(p-2)). */
  public List<ElementModP> multInv(List<ElementModP> xs) {
    final int n = xs.size();
    byte[] out = new byte[n * EgHip.P_BYTES];
    EgHip.multinvBatch(ctx, packP(xs), out, n);
    return unpackP(out, n);
  }

  // ------------------------------------------------------------------ per-element (coalesced)
  // The upstream API's call pattern: one element per call, from many threads.  Concurrent calls
  // join one GPU batch inside the library (eg_powp_one / eg_gpowp_one / eg_multp_one); a thread
  // that has several independent elements submits them all first (powPAsync) and then waits.

  /** base.powP(e) (ElementModP.powP, variable base). */
  public ElementModP powP(ElementModP base, ElementModQ e) {
    byte[] b = new byte[EgHip.P_BYTES], x = new byte[EgHip.Q_BYTES], out = new byte[EgHip.P_BYTES];
    put(b, 0, base.byteArray(), EgHip.P_BYTES);
    put(x, 0, e.byteArray(), EgHip.Q_BYTES);
    EgHip.powpOne(ctx, b, x, out);
    return elementP(out, 0);
  }

  /** g^e (GroupContext.gPowP). */
  public ElementModP gPowP(ElementModQ e) {
    byte[] x = new byte[EgHip.Q_BYTES], out = new byte[EgHip.P_BYTES];
    put(x, 0, e.byteArray(), EgHip.Q_BYTES);
    EgHip.gpowpOne(ctx, x, out);
    return elementP(out, 0);
  }

  /** a.times(b). */
  public ElementModP multP(ElementModP a, ElementModP b) {
    byte[] x = new byte[EgHip.P_BYTES], y = new byte[EgHip.P_BYTES], out = new byte[EgHip.P_BYTES];
    put(x, 0, a.byteArray(), EgHip.P_BYTES);
    put(y, 0, b.byteArray(), EgHip.P_BYTES);
    EgHip.multpOne(ctx, x, y, out);
    return elementP(out, 0);
  }

  /**
   * base.powP(e) queued now, completed by the library's next batch.  The waits run on this context's
   * own daemon threads (never ForkJoinPool.commonPool: many outstanding waits there would starve
   * unrelated parallel streams and CompletableFutures of the JVM).
   */
  public java.util.concurrent.CompletableFuture<ElementModP> powPAsync(ElementModP base, ElementModQ e) {
    byte[] b = new byte[EgHip.P_BYTES], x = new byte[EgHip.Q_BYTES];
    put(b, 0, base.byteArray(), EgHip.P_BYTES);
    put(x, 0, e.byteArray(), EgHip.Q_BYTES);
    final long t = EgHip.powpSubmit(ctx, b, x);
    return java.util.concurrent.CompletableFuture.supplyAsync(() -> {
      byte[] out = new byte[EgHip.P_BYTES];
      EgHip.ticketWait(t, out);
      return elementP(out, 0);
    }, waiters);
  }

  // the threads that wait for submitted tickets (a blocked wait holds one; idle ones exit after 30 s)
  private final java.util.concurrent.ExecutorService waiters = java.util.concurrent.Executors.newCachedThreadPool(r -> {
    Thread th = new Thread(r, "eg-hip-ticket-wait");
    th.setDaemon(true);
    return th;
  });

  // ------------------------------------------------------------------ per-element jobs (deferred)
  // The L1 adapter (GpuProductionGroupContext.kt) defers per-element calls into expressions and
  // submits each as ONE library job when a value is first needed (eg_mexp_submit).

  /** A fixed-base radix table of one base (eg_fixed_base_create); orderQ: base^q == 1 was checked. */
  public static final class Table implements AutoCloseable {
    private long fb;
    public final boolean orderQ;
    private final boolean owned;

    Table(long fb, boolean orderQ, boolean owned) { this.fb = fb; this.orderQ = orderQ; this.owned = owned; }

    long handle() { return fb; }

    @Override
    public synchronized void close() {
      if (owned && fb != 0) EgHip.fixedBaseDestroy(fb);
      fb = 0;
    }
  }

  /** A table of base's value (window_bits wide), its order checked (acceleratePow). */
  public Table table(ElementModP base, int windowBits) {
    byte[] b = new byte[EgHip.P_BYTES];
    put(b, 0, base.byteArray(), EgHip.P_BYTES);
    final long fb = EgHip.fixedBaseCreate(ctx, b, windowBits);
    return new Table(fb, hasOrderQ(b), true);
  }

  private Table gTable16;

  /** g's table for the per-element calls: 16 bits (15 multiplies per g^e, split over 4 waves), built once. */
  public synchronized Table gTable() {
    if (gTable16 == null) gTable16 = table(group.getG_MOD_P(), 16);
    return gTable16;
  }

  private boolean hasOrderQ(byte[] base512) {
    byte[] out = new byte[EgHip.P_BYTES];
    EgHip.powpBatch(ctx, base512, qBytes(), out, 1);
    for (int i = 0; i < EgHip.P_BYTES - 1; i++) if (out[i] != 0) return false;
    return out[EgHip.P_BYTES - 1] == 1;
  }

  public byte[] qBytes() {
    return hex(mode == ProductionMode.Mode4096_V2 ? EgConstants.Q_HEX_V2 : EgConstants.Q_HEX, EgHip.Q_BYTES);
  }

  public byte[] pBytes() {
    return hex(mode == ProductionMode.Mode4096_V2 ? EgConstants.P_HEX_V2 : EgConstants.P_HEX, EgHip.P_BYTES);
  }

  /**
   * Queue one job: (bases[0..nbases))^exp * t0^e0 * t1^e1 mod p (eg_mexp_submit); exp / t0 / t1 may
   * be null.  Returns the ticket for {@link #waitJob}, which must be called exactly once.
   */
  public long submitJob(byte[] bases, int nbases, byte[] exp32, Table t0, byte[] e0, Table t1, byte[] e1) {
    return EgHip.mexpSubmit(ctx, bases, nbases, exp32, t0 == null ? 0 : t0.handle(), e0,
        t1 == null ? 0 : t1.handle(), e1);
  }

  /** The 512-byte result of a submitted job (frees the ticket). */
  public byte[] waitJob(long ticket) {
    byte[] out = new byte[EgHip.P_BYTES];
    EgHip.ticketWait(ticket, out);
    return out;
  }

  /** Constant-time exponentiation for secret exponents (a trustee's context; eg_ctx_set_ct_pow). */
  public void setConstantTime(boolean on) { EgHip.setCtPow(ctx, on); }

  /** Batch window of the per-element calls (defaults: 16384 elements, 100 us). */
  public void setCoalescing(long maxBatch, int windowUs) { EgHip.setCoalescing(ctx, maxBatch, windowUs); }

  /** Hash pre-image hex form: 0 = fixed width (default), 1 = minimal (eg_ctx_set_hash_format). */
  public void setHashFormat(int format) { EgHip.setHashFormat(ctx, format); }

  /**
   * Response convention (0: v = u - c x, 1: v = u + c x) and challenge pre-image order (0 message
   * first, 1 commitments first, 2 public key first) of every proof made or checked on this context;
   * tools/pin_format.py finds the combination an upstream record uses (eg_ctx_set_proof_format).
   */
  public void setProofFormat(int response, int preimage) { EgHip.setProofFormat(ctx, response, preimage); }

  // ------------------------------------------------------------------ ballots

  /** Verdicts and tally of {@link #verifyBallots}. */
  public static final class BallotVerification {
    public final byte[] okSelection;   // nb * nsel, 1 = valid (proof + residues + bounds)
    public final byte[] okContest;     // nb * ncontests
    public final byte[] tally;         // ncontests * (spc - placeholders) * (pad, data) * 512 B, or null

    BallotVerification(byte[] s, byte[] c, byte[] t) { okSelection = s; okContest = c; tally = t; }

    public boolean allValid() {
      for (byte b : okSelection) if (b == 0) return false;
      for (byte b : okContest) if (b == 0) return false;
      return true;
    }
  }

  /**
   * Verifier(record, 11).verify()'s ballot proofs + runAccumulateBallots (RunRemoteWorkflowTest.java:151,179-182)
   * over a whole batch in the include/eg_hip.h wire layout (cts, rproof, cproof).
   */
  public BallotVerification verifyBallots(ElementModP jointKey, ElementModQ qbar, int nb, int ncontests, int spc,
                                          int placeholders, int limit, byte[] cts, byte[] rproof, byte[] cproof,
                                          boolean withTally) {
    return verifyBallots(jointKey, qbar, nb, ncontests, spc, placeholders, limit, cts, rproof, cproof, null, withTally);
  }

  /**
   * Same, with a cast flag per ballot (0 = spoiled: verified but not tallied; the spoiled ballots
   * are decrypted one by one, RunRemoteDecryptor.java:264-269), or null for all cast.
   */
  public BallotVerification verifyBallots(ElementModP jointKey, ElementModQ qbar, int nb, int ncontests, int spc,
                                          int placeholders, int limit, byte[] cts, byte[] rproof, byte[] cproof,
                                          byte[] cast, boolean withTally) {
    byte[] k = new byte[EgHip.P_BYTES], qb = new byte[EgHip.Q_BYTES];
    put(k, 0, jointKey.byteArray(), EgHip.P_BYTES);
    put(qb, 0, qbar.byteArray(), EgHip.Q_BYTES);
    final int nsel = ncontests * spc;
    byte[] okS = new byte[nb * nsel], okC = new byte[nb * ncontests];
    byte[] tally = withTally ? new byte[ncontests * (spc - placeholders) * 2 * EgHip.P_BYTES] : null;
    EgHip.verifyBallots(ctx, k, qb, nb, ncontests, spc, placeholders, limit, cts, rproof, cproof, cast, okS, okC,
        tally);
    return new BallotVerification(okS, okC, tally);
  }

  /** batchEncryption(..., CheckType.None) (RunRemoteWorkflowTest.java:140-141) with injected nonces. */
  public byte[][] encryptBallots(ElementModP jointKey, int keyWindowBits, ElementModQ qbar, int nb, int ncontests,
                                 int spc, byte[] votes, byte[] selNonces, byte[] contestNonces) {
    byte[] k = new byte[EgHip.P_BYTES], qb = new byte[EgHip.Q_BYTES];
    put(k, 0, jointKey.byteArray(), EgHip.P_BYTES);
    put(qb, 0, qbar.byteArray(), EgHip.Q_BYTES);
    EgHip.setElectionKey(ctx, k, keyWindowBits);
    final int nsel = ncontests * spc;
    byte[] cts = new byte[nb * nsel * 1024], rp = new byte[nb * nsel * 128], cp = new byte[nb * ncontests * 64];
    EgHip.encryptBallots(ctx, k, qb, nb, ncontests, spc, votes, selNonces, contestNonces, cts, rp, cp);
    return new byte[][] {cts, rp, cp};
  }
}
