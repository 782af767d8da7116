package electionguard.gpu;

/**
 * JNI binding of libeg_hip.so: one native method per export of include/eg_hip.h (the C ABI
 * of the MI355X path).  Native side: ../c/eg_hip_jni.c (build: see INTEGRATION.md §2).
 *
 * Conventions (the reference's wire layout, src/main/proto/common.proto:6-16):
 *   - element arrays are n fixed-width big-endian values concatenated: ElementModP 512 B,
 *     ElementModQ 32 B, ElGamalCiphertext (pad, data) 1024 B;
 *   - {@code long} handles are eg_ctx* / eg_fixed_base*; {@code long} d* arguments of the *Dev
 *     methods are device (HBM) pointers, e.g. from another native HIP allocation;
 *   - a non-zero status throws {@link ArithmeticException} with eg_last_error(), the mapping the
 *     reference's callers expect from upstream arithmetic (RunRemoteDecryptingTrustee.java:200-204
 *     turns any Throwable into the RPC's error string).
 *
 * JDK 17 target (.idea/misc.xml:3): JNI, not Panama FFM (FFM is final only from JDK 22).
 * No JDK exists in the build container, so this file and the C side are not compiled there.
 */
public final class EgHip {
  static {
    System.loadLibrary("eg_hip_jni"); // links libeg_hip.so (rpath / LD_LIBRARY_PATH)
  }

  private EgHip() {}

  public static final int P_BYTES = 512;
  public static final int Q_BYTES = 32;

  // ---- library / context (KUtils.productionGroup, KUtils.java:10-12) ----
  public static native String version();

  public static native long ctxCreate(byte[] p512, byte[] q32, byte[] g512, int device);

  public static native void ctxDestroy(long ctx);

  public static native void ctxSync(long ctx);

  public static native void profileBegin(long ctx);

  /**
   * @return {kernel ms, Montgomery ops, of which squarings, launches, shader clock GHz (median per
   *     workgroup; 0 if no record was usable), clock records used, clock records dropped} of the
   *     dominant kernel.
   */
  public static native double[] profileEnd(long ctx);

  /** eg_clock_median over (shader ticks, 100 MHz real-time ticks) pairs: {GHz, used, dropped}. */
  public static native double[] clockMedian(long[] recs);

  /** The fixed-base table of g built at ctxCreate (owned by the context: do not destroy). */
  public static native long gTable(long ctx);

  /** Fiat-Shamir pre-image hex form: HASH_FIXED_WIDTH (default) or HASH_MINIMAL (eg_hip.h). */
  public static final int HASH_FIXED_WIDTH = 0;
  public static final int HASH_MINIMAL = 1;

  public static native void setHashFormat(long ctx, int format);

  /** Response convention (0 = v = u - c x, 1 = v = u + c x) and challenge pre-image order
   *  (0 message first, 1 commitments first, 2 public key first): eg_ctx_set_proof_format. */
  public static native void setProofFormat(long ctx, int response, int preimage);

  // ---- fixed-base tables (PowRadix / acceleratePow; LOW_MEMORY_USE = 8-bit windows) ----
  public static native long fixedBaseCreate(long ctx, byte[] base512, int windowBits);

  public static native void fixedBaseDestroy(long fb);

  // ---- batched group ops: ElementModP.powP / gPowP / times / multP() / multInv ----
  public static native void powpBatch(long ctx, byte[] bases, byte[] exps, byte[] out, int n);

  public static native void fbPowBatch(long fb, byte[] exps, byte[] out, int n);

  public static native void powpBatchDev(long ctx, long dBases, long dExps, long dOut, long n);

  public static native void fbPowBatchDev(long fb, long dExps, long dOut, long n);

  public static native void multpBatch(long ctx, byte[] a, byte[] b, byte[] out, int n);

  /** out[g] = prod_k elems[g*len + k] (Iterable<ElementModP>.multP(); runAccumulateBallots). */
  public static native void prodReduce(long ctx, byte[] elems, int groups, int len, byte[] out);

  public static native void multinvBatch(long ctx, byte[] a, byte[] out, int n);

  // ---- ballots: Verifier(record, 11).verify() + runAccumulateBallots, batchEncryption ----
  // (RunRemoteWorkflowTest.java:140-141,151,179-182).  Layouts: include/eg_hip.h.
  /** cast: one byte per ballot (0 = spoiled: verified, not tallied), or null for all cast. */
  public static native void verifyBallots(long ctx, byte[] K512, byte[] qbar32, int nb, int nc, int spc,
                                          int placeholders, int limit, byte[] cts, byte[] rproof, byte[] cproof,
                                          byte[] cast, byte[] okSel, byte[] okContest, byte[] tally);

  public static native void setElectionKey(long ctx, byte[] K512, int windowBits);

  public static native void verifyBallotsDev(long ctx, byte[] K512, byte[] qbar32, long nb, long nc, long spc,
                                             long placeholders, int limit, long dCts, long dRproof, long dCproof,
                                             long dCast, long dOkSel, long dOkContest, long dTally);

  public static native void encryptBallots(long ctx, byte[] K512, byte[] qbar32, int nb, int nc, int spc, byte[] votes,
                                           byte[] selNonces, byte[] contestNonces, byte[] cts, byte[] rproof,
                                           byte[] cproof);

  public static native void encryptBallotsDev(long ctx, byte[] K512, byte[] qbar32, long nb, long nc, long spc,
                                              long dVotes, long dSelNonces, long dContestNonces, long dCts,
                                              long dRproof, long dCproof);

  /** Constant-time encryption (masked scans of small tables; eg_ctx_set_ct_encrypt). */
  public static native void setCtEncrypt(long ctx, boolean on);

  // ---- trustee (DecryptingTrusteeIF, RunRemoteDecryptingTrustee.java:189-193,227-232) ----
  public static native void trusteeDecryptBatch(long ctx, byte[] secret32, byte[] qbar32, byte[] texts, byte[] nonces,
                                                int n, byte[] outM, byte[] outProof);

  /** Mediator side of Decryption.decrypt (RunRemoteDecryptor.java:261-262): share-proof checks. */
  public static native void verifyShares(long ctx, byte[] qbar32, byte[] Ki, byte[] texts, byte[] M, byte[] proof,
                                         int n, byte[] ok);

  // ---- per-element calls, coalesced across threads into GPU batches (eg_powp_one & co.) ----
  // The upstream pattern: ElementModP.powP / times, GroupContext.gPowP one element per call from
  // 11 threads (RunRemoteWorkflowTest.java:140,180).
  public static native void setCoalescing(long ctx, long maxBatch, int windowUs);

  public static native void powpOne(long ctx, byte[] base512, byte[] exp32, byte[] out512);

  public static native void gpowpOne(long ctx, byte[] exp32, byte[] out512);

  public static native void multpOne(long ctx, byte[] a512, byte[] b512, byte[] out512);

  /** Asynchronous forms: a handle to pass to {@link #ticketWait} exactly once. */
  public static native long powpSubmit(long ctx, byte[] base512, byte[] exp32);

  public static native long gpowpSubmit(long ctx, byte[] exp32);

  public static native long multpSubmit(long ctx, byte[] a512, byte[] b512);

  public static native void ticketWait(long ticket, byte[] out512);

  /**
   * The general per-element job (eg_mexp_submit): (bases[0] * ... * bases[nbases-1])^exp *
   * fb0^e0 * fb1^e1 mod p, e.g. g^v * alpha^c in one job; exp / e0 / e1 may be null (exponent 1 /
   * no term; fb 0 with a null exponent).  At most 16 bases.
   */
  public static native long mexpSubmit(long ctx, byte[] bases, int nbases, byte[] exp32, long fb0, byte[] e0,
                                       long fb1, byte[] e1);

  public static native void mexpOne(long ctx, byte[] bases, int nbases, byte[] exp32, long fb0, byte[] e0,
                                    long fb1, byte[] e1, byte[] out512);

  /** An accelerated element's powP over its table (acceleratePow, e.g. the election key K.powP(R)). */
  public static native long fbPowSubmit(long fb, byte[] exp32);

  public static native void fbPowOne(long fb, byte[] exp32, byte[] out512);

  /** Constant-time exponentiation schedules for secret exponents (eg_ctx_set_ct_pow). */
  public static native void setCtPow(long ctx, boolean on);

  // ---- device memory through libeg_hip's own HIP runtime (eg_dev_*): handles are HBM addresses ----
  public static native long devAlloc(long ctx, long bytes);

  public static native void devFree(long ctx, long d);

  public static native void memcpyHtoD(long ctx, long dDst, byte[] src, long srcOff, long bytes);

  public static native void memcpyDtoH(long ctx, byte[] dst, long dstOff, long dSrc, long bytes);

  public static native void memsetDev(long ctx, long d, int value, long bytes);

  /** Every one of n flag bytes in HBM non-zero (the verifier's ok_sel / ok_contest). */
  public static native boolean allNonzeroDev(long ctx, long dFlags, long n);

  // ---- multi-GPU tally exchange (SURVEY 8e): RCCL inside libeg_hip, one rank per GPU ----
  /** Rank 0 makes the 128-byte id; the caller sends it to every rank (any host channel). */
  public static native void commUniqueId(byte[] out128);

  public static native void commInit(long ctx, byte[] id128, int world, int rank);

  public static native void commDestroy(long ctx);

  /** min over ranks of ok (the verdict all-reduce). */
  public static native boolean commAllValid(long ctx, boolean ok);

  /** Every rank's nparts x n partial-tally rows (HBM, 512 B each) folded mod p into out on root. */
  /** Ranks of the ctx's RCCL communicator as RCCL reports them (0 without one), and this rank. */
  public static native int commRanks(long ctx);

  public static native int commRank(long ctx);

  public static native void tallyAllgatherFold(long ctx, long dParts, long nparts, long n, int root, byte[] out);
}
