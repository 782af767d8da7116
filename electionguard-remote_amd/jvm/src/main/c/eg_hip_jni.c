/* eg_hip_jni.c -- JNI side of electionguard.gpu.EgHip (../java/electionguard/gpu/EgHip.java):
 * every export of include/eg_hip.h, with array-length checks before any pointer reaches the
 * library (IllegalArgumentException) and status -> ArithmeticException(eg_last_error()).
 *
 * Build (JDK 17; not available in the build container, so not compiled there):
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I include \
 *       electionguard-remote_amd/jvm/src/main/c/eg_hip_jni.c \
 *       -L electionguard-remote_amd/electionguard/lib -leg_hip -Wl,-rpath,'$ORIGIN' -o libeg_hip_jni.so
 *
 * Host arrays are taken with Get/ReleaseByteArrayElements, NOT a critical region: a batch call
 * runs for seconds on the GPU, and a critical region would stall the VM's garbage collector (and
 * every allocating thread: gRPC server threads, the reference's 11-thread verifier) for that
 * long.  A NULL from Get*Elements (the VM is out of memory and has thrown) ends the call before
 * the library is reached.  Inputs are released with JNI_ABORT (no copy back), outputs with 0.
 * Device pointers (the *Dev methods) are passed through as jlong.
 *
 * tests/jni/jni_harness.c compiles this file against a stand-in JNIEnv (tests/jni/jni.h) and calls
 * every function: short arrays -> IllegalArgumentException, a null ctx / handle ->
 * ArithmeticException(eg_last_error()).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "eg_hip.h"

static void throw_named(JNIEnv* env, const char* cls, const char* msg) {
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, msg);
}

static int check_rc(JNIEnv* env, int rc) {
  if (rc == EG_OK) return 0;
  throw_named(env, "java/lang/ArithmeticException", eg_last_error());
  return 1;
}

/* length check: array a must hold at least `need` bytes (a == NULL allowed when optional) */
static int need_len(JNIEnv* env, jbyteArray a, size_t need, int optional, const char* what) {
  if (a == NULL) {
    if (optional) return 0;
    throw_named(env, "java/lang/NullPointerException", what);
    return 1;
  }
  if ((size_t)(*env)->GetArrayLength(env, a) < need) {
    throw_named(env, "java/lang/IllegalArgumentException", what);
    return 1;
  }
  return 0;
}

/* Elements of a byte[] (NULL array -> NULL, no error); *ok cleared when the VM could not provide
 * them (it has thrown OutOfMemoryError), so the caller releases what it got and returns. */
static uint8_t* pin(JNIEnv* env, jbyteArray a, int* ok) {
  if (!a) return NULL;
  uint8_t* p = (uint8_t*)(*env)->GetByteArrayElements(env, a, NULL);
  if (!p) *ok = 0;
  return p;
}
/* a negative count from Java is an IllegalArgumentException, never a silent no-op */
static int neg(JNIEnv* env, jlong n, const char* what) {
  if (n >= 0) return 0;
  throw_named(env, "java/lang/IllegalArgumentException", what);
  return 1;
}
#define PIN(a) pin(env, (a), &pinned)
#define UNPIN_IN(a, p) \
  do { if ((a) && (p)) (*env)->ReleaseByteArrayElements(env, (a), (jbyte*)(p), JNI_ABORT); } while (0)
#define UNPIN_OUT(a, p) \
  do { if ((a) && (p)) (*env)->ReleaseByteArrayElements(env, (a), (jbyte*)(p), 0); } while (0)
/* the library status when every PIN succeeded, else EG_OK without calling it (the VM has thrown) */
#define CALL_IF_PINNED(expr) (pinned ? (expr) : EG_OK)

/* ---------------------------------------------------------------- library / context */

JNIEXPORT jstring JNICALL Java_electionguard_gpu_EgHip_version(JNIEnv* env, jclass cls) {
  char buf[256];
  if (check_rc(env, eg_version(buf, sizeof buf))) return NULL;
  return (*env)->NewStringUTF(env, buf);
}

JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_ctxCreate(JNIEnv* env, jclass cls, jbyteArray p, jbyteArray q,
                                                               jbyteArray g, jint device) {
  if (need_len(env, p, EG_P_BYTES, 0, "p: 512 bytes") || need_len(env, q, EG_Q_BYTES, 0, "q: 32 bytes") ||
      need_len(env, g, EG_P_BYTES, 0, "g: 512 bytes"))
    return 0;
  uint8_t pb[EG_P_BYTES], qb[EG_Q_BYTES], gb[EG_P_BYTES];
  (*env)->GetByteArrayRegion(env, p, 0, EG_P_BYTES, (jbyte*)pb);
  (*env)->GetByteArrayRegion(env, q, 0, EG_Q_BYTES, (jbyte*)qb);
  (*env)->GetByteArrayRegion(env, g, 0, EG_P_BYTES, (jbyte*)gb);
  eg_ctx* ctx = NULL;
  if (check_rc(env, eg_ctx_create(pb, qb, gb, device, &ctx))) return 0;
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_ctxDestroy(JNIEnv* env, jclass cls, jlong ctx) {
  check_rc(env, eg_ctx_destroy((eg_ctx*)(intptr_t)ctx));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_ctxSync(JNIEnv* env, jclass cls, jlong ctx) {
  check_rc(env, eg_ctx_sync((eg_ctx*)(intptr_t)ctx));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_profileBegin(JNIEnv* env, jclass cls, jlong ctx) {
  check_rc(env, eg_ctx_profile_begin((eg_ctx*)(intptr_t)ctx));
}

JNIEXPORT jdoubleArray JNICALL Java_electionguard_gpu_EgHip_profileEnd(JNIEnv* env, jclass cls, jlong ctx) {
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  int launches = 0;
  uint32_t used = 0, dropped = 0;
  if (check_rc(env, eg_ctx_profile_end((eg_ctx*)(intptr_t)ctx, &v[0], &v[1], &v[2], &launches))) return NULL;
  v[3] = (double)launches;
  if (check_rc(env, eg_ctx_profile_clock((eg_ctx*)(intptr_t)ctx, &v[4], &used, &dropped))) return NULL;
  v[5] = (double)used;
  v[6] = (double)dropped;
  jdoubleArray out = (*env)->NewDoubleArray(env, 7);
  if (out) (*env)->SetDoubleArrayRegion(env, out, 0, 7, v);
  return out;
}

JNIEXPORT jdoubleArray JNICALL Java_electionguard_gpu_EgHip_clockMedian(JNIEnv* env, jclass cls, jlongArray recs) {
  if (!recs) {
    throw_named(env, "java/lang/NullPointerException", "recs");
    return NULL;
  }
  const jsize len = (*env)->GetArrayLength(env, recs);
  if (len % 2) {
    throw_named(env, "java/lang/IllegalArgumentException", "recs: (shader ticks, real-time ticks) pairs");
    return NULL;
  }
  jlong* r = (*env)->GetLongArrayElements(env, recs, NULL);
  if (!r) return NULL;
  double v[3] = {0, 0, 0};
  uint32_t used = 0, dropped = 0;
  const int rc = eg_clock_median((const uint64_t*)r, (size_t)len / 2, &v[0], &used, &dropped);
  (*env)->ReleaseLongArrayElements(env, recs, r, JNI_ABORT);
  if (check_rc(env, rc)) return NULL;
  v[1] = (double)used;
  v[2] = (double)dropped;
  jdoubleArray out = (*env)->NewDoubleArray(env, 3);
  if (out) (*env)->SetDoubleArrayRegion(env, out, 0, 3, v);
  return out;
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_setCtEncrypt(JNIEnv* env, jclass cls, jlong ctx, jboolean on) {
  check_rc(env, eg_ctx_set_ct_encrypt((eg_ctx*)(intptr_t)ctx, on ? 1 : 0));
}

JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_gTable(JNIEnv* env, jclass cls, jlong ctx) {
  return (jlong)(intptr_t)eg_ctx_g_table((eg_ctx*)(intptr_t)ctx);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_setHashFormat(JNIEnv* env, jclass cls, jlong ctx, jint format) {
  check_rc(env, eg_ctx_set_hash_format((eg_ctx*)(intptr_t)ctx, format));
}

/* ---------------------------------------------------------------- fixed-base tables */

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_setProofFormat(JNIEnv* env, jclass cls, jlong ctx, jint response,
                                                                   jint preimage) {
  check_rc(env, eg_ctx_set_proof_format((eg_ctx*)(intptr_t)ctx, response, preimage));
}

JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_fixedBaseCreate(JNIEnv* env, jclass cls, jlong ctx,
                                                                     jbyteArray base, jint wbits) {
  if (need_len(env, base, EG_P_BYTES, 0, "base: 512 bytes")) return 0;
  uint8_t b[EG_P_BYTES];
  (*env)->GetByteArrayRegion(env, base, 0, EG_P_BYTES, (jbyte*)b);
  eg_fixed_base* fb = NULL;
  if (check_rc(env, eg_fixed_base_create((eg_ctx*)(intptr_t)ctx, b, wbits, &fb))) return 0;
  return (jlong)(intptr_t)fb;
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_fixedBaseDestroy(JNIEnv* env, jclass cls, jlong fb) {
  check_rc(env, eg_fixed_base_destroy((eg_fixed_base*)(intptr_t)fb));
}

/* ---------------------------------------------------------------- batched group ops */

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_powpBatch(JNIEnv* env, jclass cls, jlong ctx, jbyteArray bases,
                                                              jbyteArray exps, jbyteArray out, jint n) {
  if (neg(env, n, "n < 0") || need_len(env, bases, (size_t)n * EG_P_BYTES, 0, "bases") ||
      need_len(env, exps, (size_t)n * EG_Q_BYTES, 0, "exps") || need_len(env, out, (size_t)n * EG_P_BYTES, 0, "out"))
    return;
  int pinned = 1;
  uint8_t *b = PIN(bases), *e = PIN(exps), *o = PIN(out);
  const int rc = CALL_IF_PINNED(eg_powp_batch((eg_ctx*)(intptr_t)ctx, b, e, o, (size_t)n));
  UNPIN_OUT(out, o);
  UNPIN_IN(exps, e);
  UNPIN_IN(bases, b);
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_fbPowBatch(JNIEnv* env, jclass cls, jlong fb, jbyteArray exps,
                                                               jbyteArray out, jint n) {
  if (neg(env, n, "n < 0") || need_len(env, exps, (size_t)n * EG_Q_BYTES, 0, "exps") ||
      need_len(env, out, (size_t)n * EG_P_BYTES, 0, "out"))
    return;
  int pinned = 1;
  uint8_t *e = PIN(exps), *o = PIN(out);
  const int rc = CALL_IF_PINNED(eg_fb_pow_batch((eg_fixed_base*)(intptr_t)fb, e, o, (size_t)n));
  UNPIN_OUT(out, o);
  UNPIN_IN(exps, e);
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_powpBatchDev(JNIEnv* env, jclass cls, jlong ctx, jlong dBases,
                                                                 jlong dExps, jlong dOut, jlong n) {
  check_rc(env, eg_powp_batch_dev((eg_ctx*)(intptr_t)ctx, (const uint8_t*)(intptr_t)dBases,
                                  (const uint8_t*)(intptr_t)dExps, (uint8_t*)(intptr_t)dOut, (size_t)n));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_fbPowBatchDev(JNIEnv* env, jclass cls, jlong fb, jlong dExps,
                                                                  jlong dOut, jlong n) {
  check_rc(env, eg_fb_pow_batch_dev((eg_fixed_base*)(intptr_t)fb, (const uint8_t*)(intptr_t)dExps,
                                    (uint8_t*)(intptr_t)dOut, (size_t)n));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_multpBatch(JNIEnv* env, jclass cls, jlong ctx, jbyteArray a,
                                                               jbyteArray b, jbyteArray out, jint n) {
  const size_t len = (size_t)n * EG_P_BYTES;
  if (neg(env, n, "n < 0") || need_len(env, a, len, 0, "a") || need_len(env, b, len, 0, "b") || need_len(env, out, len, 0, "out"))
    return;
  int pinned = 1;
  uint8_t *pa = PIN(a), *pb = PIN(b), *o = PIN(out);
  const int rc = CALL_IF_PINNED(eg_multp_batch((eg_ctx*)(intptr_t)ctx, pa, pb, o, (size_t)n));
  UNPIN_OUT(out, o);
  UNPIN_IN(b, pb);
  UNPIN_IN(a, pa);
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_prodReduce(JNIEnv* env, jclass cls, jlong ctx, jbyteArray elems,
                                                               jint groups, jint len, jbyteArray out) {
  if (neg(env, groups, "groups < 0") || neg(env, len, "len < 0") || need_len(env, elems, (size_t)groups * len * EG_P_BYTES, 0, "elems") ||
      need_len(env, out, (size_t)groups * EG_P_BYTES, 0, "out"))
    return;
  int pinned = 1;
  uint8_t *e = PIN(elems), *o = PIN(out);
  const int rc = CALL_IF_PINNED(eg_prod_reduce((eg_ctx*)(intptr_t)ctx, e, (size_t)groups, (size_t)len, o));
  UNPIN_OUT(out, o);
  UNPIN_IN(elems, e);
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_multinvBatch(JNIEnv* env, jclass cls, jlong ctx, jbyteArray a,
                                                                 jbyteArray out, jint n) {
  const size_t len = (size_t)n * EG_P_BYTES;
  if (neg(env, n, "n < 0") || need_len(env, a, len, 0, "a") || need_len(env, out, len, 0, "out")) return;
  int pinned = 1;
  uint8_t *pa = PIN(a), *o = PIN(out);
  const int rc = CALL_IF_PINNED(eg_multinv_batch((eg_ctx*)(intptr_t)ctx, pa, o, (size_t)n));
  UNPIN_OUT(out, o);
  UNPIN_IN(a, pa);
  check_rc(env, rc);
}

/* ---------------------------------------------------------------- ballots */

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_verifyBallots(JNIEnv* env, jclass cls, jlong ctx, jbyteArray K,
                                                                  jbyteArray qbar, jint nb, jint nc, jint spc,
                                                                  jint ph, jint limit, jbyteArray cts,
                                                                  jbyteArray rproof, jbyteArray cproof,
                                                                  jbyteArray cast, jbyteArray okSel,
                                                                  jbyteArray okCon, jbyteArray tally) {
  if (nb < 0 || nc <= 0 || spc <= 0 || ph < 0 || ph >= spc) {
    throw_named(env, "java/lang/IllegalArgumentException", "bad manifest shape");
    return;
  }
  const size_t nsel = (size_t)nc * spc, nreal = (size_t)nc * (spc - ph);
  if (need_len(env, K, EG_P_BYTES, 0, "K") || need_len(env, qbar, EG_Q_BYTES, 0, "qbar") ||
      need_len(env, cts, (size_t)nb * nsel * 1024, 0, "cts") || need_len(env, rproof, (size_t)nb * nsel * 128, 0, "rproof") ||
      need_len(env, cproof, (size_t)nb * nc * 64, 0, "cproof") || need_len(env, okSel, (size_t)nb * nsel, 0, "okSel") ||
      need_len(env, okCon, (size_t)nb * nc, 0, "okContest") || need_len(env, tally, nreal * 2 * EG_P_BYTES, 1, "tally") ||
      need_len(env, cast, (size_t)nb, 1, "cast"))
    return;
  uint8_t kb[EG_P_BYTES], qb[EG_Q_BYTES];
  (*env)->GetByteArrayRegion(env, K, 0, EG_P_BYTES, (jbyte*)kb);
  (*env)->GetByteArrayRegion(env, qbar, 0, EG_Q_BYTES, (jbyte*)qb);
  int pinned = 1;
  uint8_t *c = PIN(cts), *r = PIN(rproof), *p = PIN(cproof), *cs = PIN(cast), *os = PIN(okSel), *oc = PIN(okCon),
          *t = PIN(tally);
  const int rc = CALL_IF_PINNED(eg_verify_ballots((eg_ctx*)(intptr_t)ctx, kb, qb, (size_t)nb, (size_t)nc, (size_t)spc,
                                                  (size_t)ph, (uint32_t)limit, c, r, p, cs, os, oc, t));
  UNPIN_OUT(tally, t);
  UNPIN_OUT(okCon, oc);
  UNPIN_OUT(okSel, os);
  UNPIN_IN(cast, cs);
  UNPIN_IN(cproof, p);
  UNPIN_IN(rproof, r);
  UNPIN_IN(cts, c);
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_setElectionKey(JNIEnv* env, jclass cls, jlong ctx, jbyteArray K,
                                                                   jint wbits) {
  if (need_len(env, K, EG_P_BYTES, 0, "K")) return;
  uint8_t kb[EG_P_BYTES];
  (*env)->GetByteArrayRegion(env, K, 0, EG_P_BYTES, (jbyte*)kb);
  check_rc(env, eg_set_election_key((eg_ctx*)(intptr_t)ctx, kb, wbits));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_verifyBallotsDev(JNIEnv* env, jclass cls, jlong ctx, jbyteArray K,
                                                                     jbyteArray qbar, jlong nb, jlong nc, jlong spc,
                                                                     jlong ph, jint limit, jlong dCts, jlong dRproof,
                                                                     jlong dCproof, jlong dCast, jlong dOkSel,
                                                                     jlong dOkCon, jlong dTally) {
  if (need_len(env, K, EG_P_BYTES, 0, "K") || need_len(env, qbar, EG_Q_BYTES, 0, "qbar")) return;
  uint8_t kb[EG_P_BYTES], qb[EG_Q_BYTES];
  (*env)->GetByteArrayRegion(env, K, 0, EG_P_BYTES, (jbyte*)kb);
  (*env)->GetByteArrayRegion(env, qbar, 0, EG_Q_BYTES, (jbyte*)qb);
  check_rc(env, eg_verify_ballots_dev((eg_ctx*)(intptr_t)ctx, kb, qb, (size_t)nb, (size_t)nc, (size_t)spc, (size_t)ph,
                                      (uint32_t)limit, (const uint8_t*)(intptr_t)dCts,
                                      (const uint8_t*)(intptr_t)dRproof, (const uint8_t*)(intptr_t)dCproof,
                                      (const uint8_t*)(intptr_t)dCast, (uint8_t*)(intptr_t)dOkSel,
                                      (uint8_t*)(intptr_t)dOkCon, (uint8_t*)(intptr_t)dTally));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_encryptBallots(JNIEnv* env, jclass cls, jlong ctx, jbyteArray K,
                                                                   jbyteArray qbar, jint nb, jint nc, jint spc,
                                                                   jbyteArray votes, jbyteArray selNonces,
                                                                   jbyteArray conNonces, jbyteArray cts,
                                                                   jbyteArray rproof, jbyteArray cproof) {
  if (nb < 0 || nc <= 0 || spc <= 0) {
    throw_named(env, "java/lang/IllegalArgumentException", "bad manifest shape");
    return;
  }
  const size_t nsel = (size_t)nc * spc;
  if (need_len(env, K, EG_P_BYTES, 0, "K") || need_len(env, qbar, EG_Q_BYTES, 0, "qbar") ||
      need_len(env, votes, (size_t)nb * nsel, 0, "votes") ||
      need_len(env, selNonces, (size_t)nb * nsel * 128, 0, "selNonces") ||
      need_len(env, conNonces, (size_t)nb * nc * 32, 0, "contestNonces") ||
      need_len(env, cts, (size_t)nb * nsel * 1024, 0, "cts") || need_len(env, rproof, (size_t)nb * nsel * 128, 0, "rproof") ||
      need_len(env, cproof, (size_t)nb * nc * 64, 0, "cproof"))
    return;
  uint8_t kb[EG_P_BYTES], qb[EG_Q_BYTES];
  (*env)->GetByteArrayRegion(env, K, 0, EG_P_BYTES, (jbyte*)kb);
  (*env)->GetByteArrayRegion(env, qbar, 0, EG_Q_BYTES, (jbyte*)qb);
  int pinned = 1;
  uint8_t *v = PIN(votes), *sn = PIN(selNonces), *cn = PIN(conNonces), *c = PIN(cts), *r = PIN(rproof), *p = PIN(cproof);
  const int rc = CALL_IF_PINNED(
      eg_encrypt_ballots((eg_ctx*)(intptr_t)ctx, kb, qb, (size_t)nb, (size_t)nc, (size_t)spc, v, sn, cn, c, r, p));
  UNPIN_OUT(cproof, p);
  UNPIN_OUT(rproof, r);
  UNPIN_OUT(cts, c);
  UNPIN_IN(conNonces, cn);
  UNPIN_IN(selNonces, sn);
  UNPIN_IN(votes, v);
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_encryptBallotsDev(JNIEnv* env, jclass cls, jlong ctx,
                                                                      jbyteArray K, jbyteArray qbar, jlong nb, jlong nc,
                                                                      jlong spc, jlong dVotes, jlong dSelNonces,
                                                                      jlong dConNonces, jlong dCts, jlong dRproof,
                                                                      jlong dCproof) {
  if (need_len(env, K, EG_P_BYTES, 0, "K") || need_len(env, qbar, EG_Q_BYTES, 0, "qbar")) return;
  uint8_t kb[EG_P_BYTES], qb[EG_Q_BYTES];
  (*env)->GetByteArrayRegion(env, K, 0, EG_P_BYTES, (jbyte*)kb);
  (*env)->GetByteArrayRegion(env, qbar, 0, EG_Q_BYTES, (jbyte*)qb);
  check_rc(env, eg_encrypt_ballots_dev((eg_ctx*)(intptr_t)ctx, kb, qb, (size_t)nb, (size_t)nc, (size_t)spc,
                                       (const uint8_t*)(intptr_t)dVotes, (const uint8_t*)(intptr_t)dSelNonces,
                                       (const uint8_t*)(intptr_t)dConNonces, (uint8_t*)(intptr_t)dCts,
                                       (uint8_t*)(intptr_t)dRproof, (uint8_t*)(intptr_t)dCproof));
}

/* ---------------------------------------------------------------- trustee */

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_trusteeDecryptBatch(JNIEnv* env, jclass cls, jlong ctx,
                                                                        jbyteArray secret, jbyteArray qbar,
                                                                        jbyteArray texts, jbyteArray nonces, jint n,
                                                                        jbyteArray outM, jbyteArray outProof) {
  if (neg(env, n, "n < 0") || need_len(env, secret, EG_Q_BYTES, 0, "secret") || need_len(env, qbar, EG_Q_BYTES, 0, "qbar") ||
      need_len(env, texts, (size_t)n * 1024, 0, "texts") || need_len(env, nonces, (size_t)n * 32, 0, "nonces") ||
      need_len(env, outM, (size_t)n * EG_P_BYTES, 0, "outM") || need_len(env, outProof, (size_t)n * 64, 0, "outProof"))
    return;
  uint8_t sb[EG_Q_BYTES], qb[EG_Q_BYTES];
  (*env)->GetByteArrayRegion(env, secret, 0, EG_Q_BYTES, (jbyte*)sb);
  (*env)->GetByteArrayRegion(env, qbar, 0, EG_Q_BYTES, (jbyte*)qb);
  int pinned = 1;
  uint8_t *t = PIN(texts), *u = PIN(nonces), *m = PIN(outM), *pr = PIN(outProof);
  const int rc = CALL_IF_PINNED(eg_trustee_decrypt_batch((eg_ctx*)(intptr_t)ctx, sb, qb, t, u, (size_t)n, m, pr));
  UNPIN_OUT(outProof, pr);
  UNPIN_OUT(outM, m);
  UNPIN_IN(nonces, u);
  UNPIN_IN(texts, t);
  memset(sb, 0, sizeof sb); /* the secret share leaves no copy on this stack frame */
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_verifyShares(JNIEnv* env, jclass cls, jlong ctx, jbyteArray qbar,
                                                                 jbyteArray Ki, jbyteArray texts, jbyteArray M,
                                                                 jbyteArray proof, jint n, jbyteArray ok) {
  if (neg(env, n, "n < 0") || need_len(env, qbar, EG_Q_BYTES, 0, "qbar") || need_len(env, Ki, (size_t)n * EG_P_BYTES, 0, "Ki") ||
      need_len(env, texts, (size_t)n * 1024, 0, "texts") || need_len(env, M, (size_t)n * EG_P_BYTES, 0, "M") ||
      need_len(env, proof, (size_t)n * 64, 0, "proof") || need_len(env, ok, (size_t)n, 0, "ok"))
    return;
  uint8_t qb[EG_Q_BYTES];
  (*env)->GetByteArrayRegion(env, qbar, 0, EG_Q_BYTES, (jbyte*)qb);
  int pinned = 1;
  uint8_t *k = PIN(Ki), *t = PIN(texts), *m = PIN(M), *p = PIN(proof), *o = PIN(ok);
  const int rc = CALL_IF_PINNED(eg_verify_shares((eg_ctx*)(intptr_t)ctx, qb, k, t, m, p, (size_t)n, o));
  UNPIN_OUT(ok, o);
  UNPIN_IN(proof, p);
  UNPIN_IN(M, m);
  UNPIN_IN(texts, t);
  UNPIN_IN(Ki, k);
  check_rc(env, rc);
}

/* ---------------------------------------------------------------- per-element calls (coalesced) */
/* ElementModP.powP / times and GroupContext.gPowP one element per call, from many threads
 * (RunRemoteWorkflowTest.java:140,180): the library gathers concurrent calls into GPU batches.
 * The asynchronous form returns a handle owning a native 512-byte result slot (a Java array may
 * move while the element waits for its batch); ticketWait copies the result out and frees it. */

typedef struct {
  eg_ticket* t;
  uint8_t out[EG_P_BYTES];
} jni_ticket;

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_setCoalescing(JNIEnv* env, jclass cls, jlong ctx, jlong maxBatch,
                                                                  jint windowUs) {
  if (maxBatch <= 0 || windowUs < 0) {
    throw_named(env, "java/lang/IllegalArgumentException", "maxBatch > 0, windowUs >= 0");
    return;
  }
  check_rc(env, eg_ctx_set_coalescing((eg_ctx*)(intptr_t)ctx, (size_t)maxBatch, (uint32_t)windowUs));
}

static int get_fixed(JNIEnv* env, jbyteArray a, size_t n, uint8_t* dst, const char* what) {
  if (need_len(env, a, n, 0, what)) return 1;
  (*env)->GetByteArrayRegion(env, a, 0, (jsize)n, (jbyte*)dst);
  return 0;
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_powpOne(JNIEnv* env, jclass cls, jlong ctx, jbyteArray base,
                                                            jbyteArray exp, jbyteArray out) {
  uint8_t b[EG_P_BYTES], e[EG_Q_BYTES], o[EG_P_BYTES];
  if (get_fixed(env, base, EG_P_BYTES, b, "base: 512 bytes") || get_fixed(env, exp, EG_Q_BYTES, e, "exp: 32 bytes") ||
      need_len(env, out, EG_P_BYTES, 0, "out: 512 bytes"))
    return;
  if (check_rc(env, eg_powp_one((eg_ctx*)(intptr_t)ctx, b, e, o))) return;
  (*env)->SetByteArrayRegion(env, out, 0, EG_P_BYTES, (const jbyte*)o);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_gpowpOne(JNIEnv* env, jclass cls, jlong ctx, jbyteArray exp,
                                                             jbyteArray out) {
  uint8_t e[EG_Q_BYTES], o[EG_P_BYTES];
  if (get_fixed(env, exp, EG_Q_BYTES, e, "exp: 32 bytes") || need_len(env, out, EG_P_BYTES, 0, "out: 512 bytes")) return;
  if (check_rc(env, eg_gpowp_one((eg_ctx*)(intptr_t)ctx, e, o))) return;
  (*env)->SetByteArrayRegion(env, out, 0, EG_P_BYTES, (const jbyte*)o);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_multpOne(JNIEnv* env, jclass cls, jlong ctx, jbyteArray a,
                                                             jbyteArray b, jbyteArray out) {
  uint8_t x[EG_P_BYTES], y[EG_P_BYTES], o[EG_P_BYTES];
  if (get_fixed(env, a, EG_P_BYTES, x, "a: 512 bytes") || get_fixed(env, b, EG_P_BYTES, y, "b: 512 bytes") ||
      need_len(env, out, EG_P_BYTES, 0, "out: 512 bytes"))
    return;
  if (check_rc(env, eg_multp_one((eg_ctx*)(intptr_t)ctx, x, y, o))) return;
  (*env)->SetByteArrayRegion(env, out, 0, EG_P_BYTES, (const jbyte*)o);
}

static jlong submit_done(JNIEnv* env, jni_ticket* jt, int rc) {
  if (check_rc(env, rc)) {
    free(jt);
    return 0;
  }
  return (jlong)(intptr_t)jt;
}

JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_powpSubmit(JNIEnv* env, jclass cls, jlong ctx, jbyteArray base,
                                                                jbyteArray exp) {
  uint8_t b[EG_P_BYTES], e[EG_Q_BYTES];
  if (get_fixed(env, base, EG_P_BYTES, b, "base: 512 bytes") || get_fixed(env, exp, EG_Q_BYTES, e, "exp: 32 bytes"))
    return 0;
  jni_ticket* jt = (jni_ticket*)calloc(1, sizeof(jni_ticket));
  if (!jt) {
    throw_named(env, "java/lang/OutOfMemoryError", "ticket");
    return 0;
  }
  return submit_done(env, jt, eg_powp_submit((eg_ctx*)(intptr_t)ctx, b, e, jt->out, &jt->t));
}

JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_gpowpSubmit(JNIEnv* env, jclass cls, jlong ctx, jbyteArray exp) {
  uint8_t e[EG_Q_BYTES];
  if (get_fixed(env, exp, EG_Q_BYTES, e, "exp: 32 bytes")) return 0;
  jni_ticket* jt = (jni_ticket*)calloc(1, sizeof(jni_ticket));
  if (!jt) {
    throw_named(env, "java/lang/OutOfMemoryError", "ticket");
    return 0;
  }
  return submit_done(env, jt, eg_gpowp_submit((eg_ctx*)(intptr_t)ctx, e, jt->out, &jt->t));
}

JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_multpSubmit(JNIEnv* env, jclass cls, jlong ctx, jbyteArray a,
                                                                 jbyteArray b) {
  uint8_t x[EG_P_BYTES], y[EG_P_BYTES];
  if (get_fixed(env, a, EG_P_BYTES, x, "a: 512 bytes") || get_fixed(env, b, EG_P_BYTES, y, "b: 512 bytes")) return 0;
  jni_ticket* jt = (jni_ticket*)calloc(1, sizeof(jni_ticket));
  if (!jt) {
    throw_named(env, "java/lang/OutOfMemoryError", "ticket");
    return 0;
  }
  return submit_done(env, jt, eg_multp_submit((eg_ctx*)(intptr_t)ctx, x, y, jt->out, &jt->t));
}

/* The general per-element job (eg_mexp_submit): (prod of nbases 512-byte bases)^exp * fb0^e0 * fb1^e1.
 * exp / e0 / e1 may be null (no exponent / no term; a term needs its table handle and its exponent). */
JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_mexpSubmit(JNIEnv* env, jclass cls, jlong ctx, jbyteArray bases,
                                                                jint nbases, jbyteArray exp, jlong fb0, jbyteArray e0,
                                                                jlong fb1, jbyteArray e1) {
  if (nbases < 0 || nbases > 16) {
    throw_named(env, "java/lang/IllegalArgumentException", "nbases in [0, 16]");
    return 0;
  }
  if ((fb0 != 0) != (e0 != NULL) || (fb1 != 0) != (e1 != NULL)) {
    throw_named(env, "java/lang/IllegalArgumentException", "a fixed-base term needs its table and its exponent");
    return 0;
  }
  uint8_t b[16 * EG_P_BYTES], x[EG_Q_BYTES], f0[EG_Q_BYTES], f1[EG_Q_BYTES];
  if (nbases && get_fixed(env, bases, (size_t)nbases * EG_P_BYTES, b, "bases: nbases x 512 bytes")) return 0;
  if (exp && get_fixed(env, exp, EG_Q_BYTES, x, "exp: 32 bytes")) return 0;
  if (e0 && get_fixed(env, e0, EG_Q_BYTES, f0, "e0: 32 bytes")) return 0;
  if (e1 && get_fixed(env, e1, EG_Q_BYTES, f1, "e1: 32 bytes")) return 0;
  jni_ticket* jt = (jni_ticket*)calloc(1, sizeof(jni_ticket));
  if (!jt) {
    throw_named(env, "java/lang/OutOfMemoryError", "ticket");
    return 0;
  }
  return submit_done(env, jt,
                     eg_mexp_submit((eg_ctx*)(intptr_t)ctx, nbases ? b : NULL, (size_t)nbases, exp ? x : NULL,
                                    (eg_fixed_base*)(intptr_t)fb0, e0 ? f0 : NULL, (eg_fixed_base*)(intptr_t)fb1,
                                    e1 ? f1 : NULL, jt->out, &jt->t));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_mexpOne(JNIEnv* env, jclass cls, jlong ctx, jbyteArray bases,
                                                            jint nbases, jbyteArray exp, jlong fb0, jbyteArray e0,
                                                            jlong fb1, jbyteArray e1, jbyteArray out) {
  if (need_len(env, out, EG_P_BYTES, 0, "out: 512 bytes")) return;
  uint8_t b[16 * EG_P_BYTES], x[EG_Q_BYTES], f0[EG_Q_BYTES], f1[EG_Q_BYTES], o[EG_P_BYTES];
  if (nbases < 0 || nbases > 16) {
    throw_named(env, "java/lang/IllegalArgumentException", "nbases in [0, 16]");
    return;
  }
  if (nbases && get_fixed(env, bases, (size_t)nbases * EG_P_BYTES, b, "bases: nbases x 512 bytes")) return;
  if (exp && get_fixed(env, exp, EG_Q_BYTES, x, "exp: 32 bytes")) return;
  if (e0 && get_fixed(env, e0, EG_Q_BYTES, f0, "e0: 32 bytes")) return;
  if (e1 && get_fixed(env, e1, EG_Q_BYTES, f1, "e1: 32 bytes")) return;
  if (check_rc(env, eg_mexp_one((eg_ctx*)(intptr_t)ctx, nbases ? b : NULL, (size_t)nbases, exp ? x : NULL,
                                (eg_fixed_base*)(intptr_t)fb0, e0 ? f0 : NULL, (eg_fixed_base*)(intptr_t)fb1,
                                e1 ? f1 : NULL, o)))
    return;
  (*env)->SetByteArrayRegion(env, out, 0, EG_P_BYTES, (const jbyte*)o);
}

/* an accelerated element's powP over its fixed-base table (acceleratePow: eg_fb_pow_submit) */
JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_fbPowSubmit(JNIEnv* env, jclass cls, jlong fb, jbyteArray exp) {
  uint8_t e[EG_Q_BYTES];
  if (get_fixed(env, exp, EG_Q_BYTES, e, "exp: 32 bytes")) return 0;
  jni_ticket* jt = (jni_ticket*)calloc(1, sizeof(jni_ticket));
  if (!jt) {
    throw_named(env, "java/lang/OutOfMemoryError", "ticket");
    return 0;
  }
  return submit_done(env, jt, eg_fb_pow_submit((eg_fixed_base*)(intptr_t)fb, e, jt->out, &jt->t));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_fbPowOne(JNIEnv* env, jclass cls, jlong fb, jbyteArray exp,
                                                             jbyteArray out) {
  uint8_t e[EG_Q_BYTES], o[EG_P_BYTES];
  if (get_fixed(env, exp, EG_Q_BYTES, e, "exp: 32 bytes") || need_len(env, out, EG_P_BYTES, 0, "out: 512 bytes")) return;
  if (check_rc(env, eg_fb_pow_one((eg_fixed_base*)(intptr_t)fb, e, o))) return;
  (*env)->SetByteArrayRegion(env, out, 0, EG_P_BYTES, (const jbyte*)o);
}

/* constant-time exponentiation for secret exponents (a trustee's context) */
JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_setCtPow(JNIEnv* env, jclass cls, jlong ctx, jboolean on) {
  check_rc(env, eg_ctx_set_ct_pow((eg_ctx*)(intptr_t)ctx, on ? 1 : 0));
}

/* Waits for the element's batch, copies the 512-byte result into out, frees the handle (also when
 * out is too short: the ticket is consumed either way). */
JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_ticketWait(JNIEnv* env, jclass cls, jlong ticket, jbyteArray out) {
  jni_ticket* jt = (jni_ticket*)(intptr_t)ticket;
  if (!jt) {
    check_rc(env, eg_ticket_wait(NULL));
    return;
  }
  const int rc = eg_ticket_wait(jt->t);
  if (!check_rc(env, rc) && !need_len(env, out, EG_P_BYTES, 0, "out: 512 bytes"))
    (*env)->SetByteArrayRegion(env, out, 0, EG_P_BYTES, (const jbyte*)jt->out);
  free(jt);
}

/* ---------------------------------------------------------------- device memory (eg_dev_*) */
/* HBM of the ctx's device through libeg_hip's own runtime; handles are device addresses (jlong). */

JNIEXPORT jlong JNICALL Java_electionguard_gpu_EgHip_devAlloc(JNIEnv* env, jclass cls, jlong ctx, jlong bytes) {
  if (neg(env, bytes, "bytes < 0")) return 0;
  void* d = NULL;
  if (check_rc(env, eg_dev_alloc((eg_ctx*)(intptr_t)ctx, (size_t)bytes, &d))) return 0;
  return (jlong)(intptr_t)d;
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_devFree(JNIEnv* env, jclass cls, jlong ctx, jlong d) {
  check_rc(env, eg_dev_free((eg_ctx*)(intptr_t)ctx, (void*)(intptr_t)d));
}

/* src[srcOff, srcOff + bytes) -> device dDst */
JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_memcpyHtoD(JNIEnv* env, jclass cls, jlong ctx, jlong dDst,
                                                               jbyteArray src, jlong srcOff, jlong bytes) {
  if (neg(env, srcOff, "srcOff < 0") || neg(env, bytes, "bytes < 0") ||
      need_len(env, src, (size_t)srcOff + (size_t)bytes, 0, "src shorter than srcOff + bytes"))
    return;
  int pinned = 1;
  uint8_t* s = PIN(src);
  const int rc = CALL_IF_PINNED(eg_memcpy_htod((eg_ctx*)(intptr_t)ctx, (void*)(intptr_t)dDst, s + srcOff, (size_t)bytes));
  UNPIN_IN(src, s);
  check_rc(env, rc);
}

/* device dSrc -> dst[dstOff, dstOff + bytes) */
JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_memcpyDtoH(JNIEnv* env, jclass cls, jlong ctx, jbyteArray dst,
                                                               jlong dstOff, jlong dSrc, jlong bytes) {
  if (neg(env, dstOff, "dstOff < 0") || neg(env, bytes, "bytes < 0") ||
      need_len(env, dst, (size_t)dstOff + (size_t)bytes, 0, "dst shorter than dstOff + bytes"))
    return;
  int pinned = 1;
  uint8_t* d = PIN(dst);
  const int rc = CALL_IF_PINNED(eg_memcpy_dtoh((eg_ctx*)(intptr_t)ctx, d + dstOff, (const void*)(intptr_t)dSrc, (size_t)bytes));
  UNPIN_OUT(dst, d);
  check_rc(env, rc);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_memsetDev(JNIEnv* env, jclass cls, jlong ctx, jlong d, jint value,
                                                              jlong bytes) {
  if (neg(env, bytes, "bytes < 0")) return;
  check_rc(env, eg_memset_dev((eg_ctx*)(intptr_t)ctx, (void*)(intptr_t)d, value, (size_t)bytes));
}

JNIEXPORT jboolean JNICALL Java_electionguard_gpu_EgHip_allNonzeroDev(JNIEnv* env, jclass cls, jlong ctx, jlong dFlags,
                                                                      jlong n) {
  if (neg(env, n, "n < 0")) return JNI_FALSE;
  int all = 0;
  if (check_rc(env, eg_all_nonzero_dev((eg_ctx*)(intptr_t)ctx, (const uint8_t*)(intptr_t)dFlags, (size_t)n, &all)))
    return JNI_FALSE;
  return all ? JNI_TRUE : JNI_FALSE;
}

/* ---------------------------------------------------------------- multi-GPU tally exchange (eg_comm_*) */

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_commUniqueId(JNIEnv* env, jclass cls, jbyteArray out128) {
  if (need_len(env, out128, EG_COMM_ID_BYTES, 0, "out: 128 bytes")) return;
  uint8_t id[EG_COMM_ID_BYTES];
  if (check_rc(env, eg_comm_unique_id(id))) return;
  (*env)->SetByteArrayRegion(env, out128, 0, EG_COMM_ID_BYTES, (const jbyte*)id);
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_commInit(JNIEnv* env, jclass cls, jlong ctx, jbyteArray id128,
                                                             jint world, jint rank) {
  uint8_t id[EG_COMM_ID_BYTES];
  if (get_fixed(env, id128, EG_COMM_ID_BYTES, id, "id: 128 bytes")) return;
  check_rc(env, eg_comm_init((eg_ctx*)(intptr_t)ctx, id, world, rank));
}

JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_commDestroy(JNIEnv* env, jclass cls, jlong ctx) {
  check_rc(env, eg_comm_destroy((eg_ctx*)(intptr_t)ctx));
}

JNIEXPORT jboolean JNICALL Java_electionguard_gpu_EgHip_commAllValid(JNIEnv* env, jclass cls, jlong ctx, jboolean ok) {
  int all = 0;
  if (check_rc(env, eg_comm_all_valid((eg_ctx*)(intptr_t)ctx, ok ? 1 : 0, &all))) return JNI_FALSE;
  return all ? JNI_TRUE : JNI_FALSE;
}

/* what the RCCL communicator reports (eg_comm_info): its rank count (0 without one) and this rank */
JNIEXPORT jint JNICALL Java_electionguard_gpu_EgHip_commRanks(JNIEnv* env, jclass cls, jlong ctx) {
  int n = 0;
  if (check_rc(env, eg_comm_info((eg_ctx*)(intptr_t)ctx, &n, NULL))) return 0;
  return (jint)n;
}

JNIEXPORT jint JNICALL Java_electionguard_gpu_EgHip_commRank(JNIEnv* env, jclass cls, jlong ctx) {
  int r = 0;
  if (check_rc(env, eg_comm_info((eg_ctx*)(intptr_t)ctx, NULL, &r))) return 0;
  return (jint)r;
}

/* out: n x 512 bytes on the root (may be null on the other ranks) */
JNIEXPORT void JNICALL Java_electionguard_gpu_EgHip_tallyAllgatherFold(JNIEnv* env, jclass cls, jlong ctx, jlong dParts,
                                                                       jlong nparts, jlong n, jint root, jbyteArray out) {
  if (neg(env, nparts, "nparts < 0") || neg(env, n, "n < 0") ||
      need_len(env, out, (size_t)n * EG_P_BYTES, 1, "out: n x 512 bytes"))
    return;
  int pinned = 1;
  uint8_t* o = PIN(out);
  const int rc = CALL_IF_PINNED(eg_tally_allgather_fold((eg_ctx*)(intptr_t)ctx, (const uint8_t*)(intptr_t)dParts,
                                                        (size_t)nparts, (size_t)n, root, o));
  UNPIN_OUT(out, o);
  check_rc(env, rc);
}
