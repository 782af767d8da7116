/* jni_harness.c -- TEST INFRASTRUCTURE ONLY: executes every Java_electionguard_gpu_EgHip_*
 * function of electionguard-remote_amd/jvm/src/main/c/eg_hip_jni.c (included below, compiled
 * unchanged against the stand-in tests/jni/jni.h) with a minimal JNIEnv whose arrays are plain C
 * buffers and whose exceptions are recorded, not thrown.  Checks, without a GPU:
 *   - every array shorter than its count needs    -> IllegalArgumentException (nothing reaches
 *     the library), negative counts likewise, a missing required array -> NullPointerException;
 *   - a null context / handle with well-sized arrays -> ArithmeticException carrying the
 *     library's eg_last_error() text (the status -> exception mapping);
 *   - Get*Elements failing (VM out of memory) -> the library is not called, nothing leaks;
 *   - the pure functions (version, clockMedian) return their values.
 * Build + run: tests/test_jni_harness.py (gcc, links libeg_hip.so). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

typedef struct eg_test_jobject {
  int kind; /* 1 byte[], 2 long[], 3 double[], 4 string, 5 class */
  jsize len;
  void* data;
  char name[96];
} Obj;

static char g_exc[96], g_msg[256], g_last_msg[256];
static int g_fail_pin = 0, g_pins = 0, g_unpins = 0, g_checks = 0, g_errors = 0;

static jclass FindClass_(JNIEnv* env, const char* name) {
  Obj* o = calloc(1, sizeof(Obj));
  o->kind = 5;
  snprintf(o->name, sizeof o->name, "%s", name);
  return o;
}
static jint ThrowNew_(JNIEnv* env, jclass cls, const char* msg) {
  snprintf(g_exc, sizeof g_exc, "%s", cls->name);
  snprintf(g_msg, sizeof g_msg, "%s", msg ? msg : "");
  free(cls);
  return 0;
}
static jsize GetArrayLength_(JNIEnv* env, jarray a) { return a->len; }
static void GetByteArrayRegion_(JNIEnv* env, jbyteArray a, jsize s, jsize n, jbyte* b) {
  memcpy(b, (char*)a->data + s, (size_t)n);
}
static void SetByteArrayRegion_(JNIEnv* env, jbyteArray a, jsize s, jsize n, const jbyte* b) {
  memcpy((char*)a->data + s, b, (size_t)n);
}
static jbyte* GetByteArrayElements_(JNIEnv* env, jbyteArray a, jboolean* c) {
  if (g_fail_pin) {
    snprintf(g_exc, sizeof g_exc, "java/lang/OutOfMemoryError");
    return NULL;
  }
  ++g_pins;
  jbyte* copy = malloc((size_t)a->len + 1); /* HotSpot copies: so does the stand-in */
  memcpy(copy, a->data, (size_t)a->len);
  return copy;
}
static void ReleaseByteArrayElements_(JNIEnv* env, jbyteArray a, jbyte* e, jint mode) {
  ++g_unpins;
  if (mode != JNI_ABORT) memcpy(a->data, e, (size_t)a->len);
  free(e);
}
static jlong* GetLongArrayElements_(JNIEnv* env, jlongArray a, jboolean* c) { return (jlong*)a->data; }
static void ReleaseLongArrayElements_(JNIEnv* env, jlongArray a, jlong* e, jint mode) {}
static jstring NewStringUTF_(JNIEnv* env, const char* s) {
  Obj* o = calloc(1, sizeof(Obj));
  o->kind = 4;
  snprintf(o->name, sizeof o->name, "%s", s);
  return o;
}
static jdoubleArray NewDoubleArray_(JNIEnv* env, jsize n) {
  Obj* o = calloc(1, sizeof(Obj));
  o->kind = 3;
  o->len = n;
  o->data = calloc((size_t)n, sizeof(double));
  return o;
}
static void SetDoubleArrayRegion_(JNIEnv* env, jdoubleArray a, jsize s, jsize n, const jdouble* b) {
  memcpy((double*)a->data + s, b, sizeof(double) * (size_t)n);
}

static const struct JNINativeInterface_ g_fns = {
    FindClass_, ThrowNew_, GetArrayLength_, GetByteArrayRegion_, SetByteArrayRegion_, GetByteArrayElements_,
    ReleaseByteArrayElements_, GetLongArrayElements_, ReleaseLongArrayElements_, NewStringUTF_, NewDoubleArray_,
    SetDoubleArrayRegion_};
static JNIEnv g_envp = &g_fns;
static JNIEnv* env = &g_envp;

#include "../../electionguard-remote_amd/jvm/src/main/c/eg_hip_jni.c"

static Obj* bytes(jsize n) {
  Obj* o = calloc(1, sizeof(Obj));
  o->kind = 1;
  o->len = n;
  o->data = calloc((size_t)n + 1, 1);
  return o;
}
static Obj* longs(const int64_t* v, jsize n) {
  Obj* o = calloc(1, sizeof(Obj));
  o->kind = 2;
  o->len = n;
  o->data = calloc((size_t)n + 1, sizeof(int64_t));
  memcpy(o->data, v, sizeof(int64_t) * (size_t)n);
  return o;
}

static void reset(void) {
  memcpy(g_last_msg, g_msg, sizeof g_msg);  /* EXPECT_MSG reads the message of the last EXPECT */
  g_exc[0] = g_msg[0] = 0;
}
static void expect(const char* what, const char* exc, int line) {
  ++g_checks;
  const int ok = exc ? strcmp(g_exc, exc) == 0 : g_exc[0] == 0;
  if (!ok) {
    ++g_errors;
    fprintf(stderr, "line %d %s: want %s, got %s (%s)\n", line, what, exc ? exc : "no exception",
            g_exc[0] ? g_exc : "no exception", g_msg);
  }
  reset();
}
#define IAE "java/lang/IllegalArgumentException"
#define AE "java/lang/ArithmeticException"
#define NPE "java/lang/NullPointerException"
#define OOM "java/lang/OutOfMemoryError"
#define EXPECT(what, exc) expect(what, exc, __LINE__)
#define EXPECT_MSG(sub)                                                                    \
  do {                                                                                     \
    ++g_checks;                                                                            \
    if (!strstr(g_last_msg, sub) || !g_last_msg[0]) {                                      \
      ++g_errors;                                                                          \
      fprintf(stderr, "line %d: message '%s' lacks '%s'\n", __LINE__, g_last_msg, sub);   \
    }                                                                                      \
  } while (0)

int main(void) {
  const jclass C = NULL;
  const jlong N0 = 0; /* a null handle: every library entry point reports it as an error */
  Obj *p = bytes(512), *q = bytes(32), *sh = bytes(10), *o512 = bytes(512), *b2 = bytes(1024), *e2 = bytes(64);

  /* ---- library / context ---- */
  jstring v = Java_electionguard_gpu_EgHip_version(env, C);
  EXPECT("version", NULL);
  ++g_checks;
  if (!v || !strstr(v->name, "gfx950")) { ++g_errors; fprintf(stderr, "version string\n"); }
  Java_electionguard_gpu_EgHip_ctxCreate(env, C, sh, q, p, 0);
  EXPECT("ctxCreate short p", IAE);
  Java_electionguard_gpu_EgHip_ctxCreate(env, C, p, q, NULL, 0);
  EXPECT("ctxCreate null g", NPE);
  {
    /* an even p is rejected before any device is touched */
    jlong h = Java_electionguard_gpu_EgHip_ctxCreate(env, C, p, q, p, 0);
    EXPECT("ctxCreate bad modulus", AE);
    EXPECT_MSG("odd");
    if (h) Java_electionguard_gpu_EgHip_ctxDestroy(env, C, h);
  }
  Java_electionguard_gpu_EgHip_ctxDestroy(env, C, N0);
  EXPECT("ctxDestroy(0) is a no-op", NULL);
  Java_electionguard_gpu_EgHip_ctxSync(env, C, N0);
  EXPECT("ctxSync(0)", AE);
  EXPECT_MSG("null");
  Java_electionguard_gpu_EgHip_profileBegin(env, C, N0);
  EXPECT("profileBegin(0)", AE);
  Java_electionguard_gpu_EgHip_profileEnd(env, C, N0);
  EXPECT("profileEnd(0)", AE);
  Java_electionguard_gpu_EgHip_gTable(env, C, N0);
  EXPECT("gTable(0)", NULL);
  Java_electionguard_gpu_EgHip_setHashFormat(env, C, N0, 0);
  EXPECT("setHashFormat(0)", AE);
  Java_electionguard_gpu_EgHip_setProofFormat(env, C, N0, 1, 2);
  EXPECT("setProofFormat(0)", AE);
  Java_electionguard_gpu_EgHip_setCtEncrypt(env, C, N0, 1);
  EXPECT("setCtEncrypt(0)", AE);
  {
    const int64_t recs[8] = {220000, 10000, 0, 0, 230000, 10000, 225000, 10000}; /* 2.2, unset, 2.3, 2.25 GHz */
    Obj* r = longs(recs, 8);
    jdoubleArray out = Java_electionguard_gpu_EgHip_clockMedian(env, C, r);
    EXPECT("clockMedian", NULL);
    const double* d = out ? (const double*)out->data : NULL;
    ++g_checks;
    if (!d || d[0] < 2.249 || d[0] > 2.251 || d[1] != 3 || d[2] != 1) {
      ++g_errors;
      fprintf(stderr, "clockMedian values %g %g %g\n", d ? d[0] : -1, d ? d[1] : -1, d ? d[2] : -1);
    }
    Obj* odd = longs(recs, 3);
    Java_electionguard_gpu_EgHip_clockMedian(env, C, odd);
    EXPECT("clockMedian odd length", IAE);
    Java_electionguard_gpu_EgHip_clockMedian(env, C, NULL);
    EXPECT("clockMedian null", NPE);
  }

  /* ---- fixed-base tables ---- */
  Java_electionguard_gpu_EgHip_fixedBaseCreate(env, C, N0, sh, 8);
  EXPECT("fixedBaseCreate short", IAE);
  Java_electionguard_gpu_EgHip_fixedBaseCreate(env, C, N0, p, 8);
  EXPECT("fixedBaseCreate(0)", AE);
  Java_electionguard_gpu_EgHip_fixedBaseDestroy(env, C, N0);
  EXPECT("fixedBaseDestroy(0) is a no-op", NULL);

  /* ---- batched group ops ---- */
  Java_electionguard_gpu_EgHip_powpBatch(env, C, N0, p, e2, b2, 2);
  EXPECT("powpBatch short bases", IAE);
  Java_electionguard_gpu_EgHip_powpBatch(env, C, N0, b2, e2, b2, -1);
  EXPECT("powpBatch n < 0", IAE);
  Java_electionguard_gpu_EgHip_powpBatch(env, C, N0, b2, e2, b2, 2);
  EXPECT("powpBatch(0)", AE);
  EXPECT_MSG("null");
  g_fail_pin = 1;
  {
    const int pins = g_pins, unpins = g_unpins;
    Java_electionguard_gpu_EgHip_powpBatch(env, C, N0, b2, e2, b2, 2);
    EXPECT("powpBatch with the VM out of memory", OOM);
    ++g_checks;
    if (g_pins - pins != g_unpins - unpins) { ++g_errors; fprintf(stderr, "pin leak\n"); }
  }
  g_fail_pin = 0;
  Java_electionguard_gpu_EgHip_fbPowBatch(env, C, N0, q, b2, 2);
  EXPECT("fbPowBatch short exps", IAE);
  Java_electionguard_gpu_EgHip_fbPowBatch(env, C, N0, e2, b2, 2);
  EXPECT("fbPowBatch(0)", AE);
  Java_electionguard_gpu_EgHip_powpBatchDev(env, C, N0, 0, 0, 0, 1);
  EXPECT("powpBatchDev(0)", AE);
  Java_electionguard_gpu_EgHip_fbPowBatchDev(env, C, N0, 0, 0, 1);
  EXPECT("fbPowBatchDev(0)", AE);
  Java_electionguard_gpu_EgHip_multpBatch(env, C, N0, b2, p, b2, 2);
  EXPECT("multpBatch short b", IAE);
  Java_electionguard_gpu_EgHip_multpBatch(env, C, N0, b2, b2, b2, 2);
  EXPECT("multpBatch(0)", AE);
  Java_electionguard_gpu_EgHip_prodReduce(env, C, N0, p, 1, 2, p);
  EXPECT("prodReduce short elems", IAE);
  Java_electionguard_gpu_EgHip_prodReduce(env, C, N0, b2, -1, 2, p);
  EXPECT("prodReduce groups < 0", IAE);
  Java_electionguard_gpu_EgHip_prodReduce(env, C, N0, b2, 1, 2, p);
  EXPECT("prodReduce(0)", AE);
  Java_electionguard_gpu_EgHip_multinvBatch(env, C, N0, p, b2, 2);
  EXPECT("multinvBatch short a", IAE);
  Java_electionguard_gpu_EgHip_multinvBatch(env, C, N0, b2, b2, 2);
  EXPECT("multinvBatch(0)", AE);

  /* ---- ballots: 1 ballot of 1 contest x (1 + 1 placeholder) ---- */
  {
    Obj *cts = bytes(2 * 1024), *rp = bytes(2 * 128), *cp = bytes(64), *os = bytes(2), *oc = bytes(1),
        *tal = bytes(1024), *cast = bytes(1), *votes = bytes(2), *sn = bytes(2 * 128), *cn = bytes(32);
    Java_electionguard_gpu_EgHip_verifyBallots(env, C, N0, p, q, 1, 1, 2, 2, 1, cts, rp, cp, NULL, os, oc, tal);
    EXPECT("verifyBallots placeholders >= spc", IAE);
    Java_electionguard_gpu_EgHip_verifyBallots(env, C, N0, p, q, 1, 1, 2, 1, 1, sh, rp, cp, NULL, os, oc, tal);
    EXPECT("verifyBallots short cts", IAE);
    Java_electionguard_gpu_EgHip_verifyBallots(env, C, N0, p, q, 2, 1, 2, 1, 1, b2, rp, cp, cast, os, oc, tal);
    EXPECT("verifyBallots short cts for 2 ballots", IAE);
    Java_electionguard_gpu_EgHip_verifyBallots(env, C, N0, p, q, 1, 1, 2, 1, 1, cts, rp, cp, cast, os, oc, sh);
    EXPECT("verifyBallots short tally", IAE);
    Java_electionguard_gpu_EgHip_verifyBallots(env, C, N0, p, q, 1, 1, 2, 1, 1, cts, rp, cp, cast, os, oc, tal);
    EXPECT("verifyBallots(0)", AE);
    Java_electionguard_gpu_EgHip_verifyBallots(env, C, N0, p, q, 1, 1, 2, 1, 1, cts, rp, cp, NULL, os, oc, NULL);
    EXPECT("verifyBallots(0) without cast flags or tally", AE);
    Java_electionguard_gpu_EgHip_setElectionKey(env, C, N0, sh, 8);
    EXPECT("setElectionKey short K", IAE);
    Java_electionguard_gpu_EgHip_setElectionKey(env, C, N0, p, 8);
    EXPECT("setElectionKey(0)", AE);
    Java_electionguard_gpu_EgHip_verifyBallotsDev(env, C, N0, sh, q, 1, 1, 2, 1, 1, 0, 0, 0, 0, 0, 0, 0);
    EXPECT("verifyBallotsDev short K", IAE);
    Java_electionguard_gpu_EgHip_verifyBallotsDev(env, C, N0, p, q, 1, 1, 2, 1, 1, 0, 0, 0, 0, 0, 0, 0);
    EXPECT("verifyBallotsDev(0)", AE);
    Java_electionguard_gpu_EgHip_encryptBallots(env, C, N0, p, q, 1, 1, 2, votes, sn, cn, cts, rp, sh);
    EXPECT("encryptBallots short cproof", IAE);
    Java_electionguard_gpu_EgHip_encryptBallots(env, C, N0, p, q, 1, 0, 2, votes, sn, cn, cts, rp, cp);
    EXPECT("encryptBallots no contests", IAE);
    Java_electionguard_gpu_EgHip_encryptBallots(env, C, N0, p, q, 1, 1, 2, votes, sn, cn, cts, rp, cp);
    EXPECT("encryptBallots(0)", AE);
    Java_electionguard_gpu_EgHip_encryptBallotsDev(env, C, N0, p, sh, 1, 1, 2, 0, 0, 0, 0, 0, 0);
    EXPECT("encryptBallotsDev short qbar", IAE);
    Java_electionguard_gpu_EgHip_encryptBallotsDev(env, C, N0, p, q, 1, 1, 2, 0, 0, 0, 0, 0, 0);
    EXPECT("encryptBallotsDev(0)", AE);
  }

  /* ---- trustee ---- */
  {
    Obj *texts = bytes(2 * 1024), *non = bytes(64), *M = bytes(1024), *pr = bytes(128), *ok = bytes(2), *Ki = bytes(1024);
    Java_electionguard_gpu_EgHip_trusteeDecryptBatch(env, C, N0, q, q, texts, non, 2, M, sh);
    EXPECT("trusteeDecryptBatch short proof", IAE);
    Java_electionguard_gpu_EgHip_trusteeDecryptBatch(env, C, N0, q, q, texts, non, -2, M, pr);
    EXPECT("trusteeDecryptBatch n < 0", IAE);
    Java_electionguard_gpu_EgHip_trusteeDecryptBatch(env, C, N0, q, q, texts, non, 2, M, pr);
    EXPECT("trusteeDecryptBatch(0)", AE);
    Java_electionguard_gpu_EgHip_verifyShares(env, C, N0, q, Ki, texts, M, pr, 2, bytes(1));
    EXPECT("verifyShares short ok", IAE);
    Java_electionguard_gpu_EgHip_verifyShares(env, C, N0, q, Ki, texts, M, pr, 2, ok);
    EXPECT("verifyShares(0)", AE);
  }

  /* ---- per-element calls ---- */
  Java_electionguard_gpu_EgHip_setCoalescing(env, C, N0, 0, 100);
  EXPECT("setCoalescing maxBatch 0", IAE);
  Java_electionguard_gpu_EgHip_setCoalescing(env, C, N0, 64, 100);
  EXPECT("setCoalescing(0)", AE);
  Java_electionguard_gpu_EgHip_powpOne(env, C, N0, p, sh, o512);
  EXPECT("powpOne short exp", IAE);
  Java_electionguard_gpu_EgHip_powpOne(env, C, N0, p, q, o512);
  EXPECT("powpOne(0)", AE);
  Java_electionguard_gpu_EgHip_gpowpOne(env, C, N0, q, sh);
  EXPECT("gpowpOne short out", IAE);
  Java_electionguard_gpu_EgHip_gpowpOne(env, C, N0, q, o512);
  EXPECT("gpowpOne(0)", AE);
  Java_electionguard_gpu_EgHip_multpOne(env, C, N0, p, p, o512);
  EXPECT("multpOne(0)", AE);
  {
    jlong t = Java_electionguard_gpu_EgHip_powpSubmit(env, C, N0, p, q);
    EXPECT("powpSubmit(0)", AE);
    ++g_checks;
    if (t) { ++g_errors; fprintf(stderr, "failed submit returned a ticket\n"); }
    Java_electionguard_gpu_EgHip_gpowpSubmit(env, C, N0, sh);
    EXPECT("gpowpSubmit short exp", IAE);
    Java_electionguard_gpu_EgHip_gpowpSubmit(env, C, N0, q);
    EXPECT("gpowpSubmit(0)", AE);
    Java_electionguard_gpu_EgHip_multpSubmit(env, C, N0, p, p);
    EXPECT("multpSubmit(0)", AE);
    Java_electionguard_gpu_EgHip_ticketWait(env, C, 0, o512);
    EXPECT("ticketWait(0)", AE);
    EXPECT_MSG("null");
    /* the general job and the accelerated-element forms */
    Java_electionguard_gpu_EgHip_mexpSubmit(env, C, N0, p, 17, q, 0, NULL, 0, NULL);
    EXPECT("mexpSubmit 17 bases", IAE);
    Java_electionguard_gpu_EgHip_mexpSubmit(env, C, N0, p, 1, q, 7, NULL, 0, NULL);
    EXPECT("mexpSubmit table without exponent", IAE);
    Java_electionguard_gpu_EgHip_mexpSubmit(env, C, N0, sh, 1, q, 0, NULL, 0, NULL);
    EXPECT("mexpSubmit short bases", IAE);
    t = Java_electionguard_gpu_EgHip_mexpSubmit(env, C, N0, p, 1, q, 0, NULL, 0, NULL);
    EXPECT("mexpSubmit(0)", AE);
    ++g_checks;
    if (t) { ++g_errors; fprintf(stderr, "failed mexp submit returned a ticket\n"); }
    Java_electionguard_gpu_EgHip_mexpOne(env, C, N0, p, 1, q, 0, NULL, 0, NULL, sh);
    EXPECT("mexpOne short out", IAE);
    Java_electionguard_gpu_EgHip_mexpOne(env, C, N0, p, 1, q, 0, NULL, 0, NULL, o512);
    EXPECT("mexpOne(0)", AE);
    Java_electionguard_gpu_EgHip_fbPowSubmit(env, C, N0, sh);
    EXPECT("fbPowSubmit short exp", IAE);
    Java_electionguard_gpu_EgHip_fbPowSubmit(env, C, N0, q);
    EXPECT("fbPowSubmit(0)", AE);
    Java_electionguard_gpu_EgHip_fbPowOne(env, C, N0, q, o512);
    EXPECT("fbPowOne(0)", AE);
    Java_electionguard_gpu_EgHip_setCtPow(env, C, N0, 1);
    EXPECT("setCtPow(0)", AE);
    Java_electionguard_gpu_EgHip_commRanks(env, C, N0);
    EXPECT("commRanks(0)", AE);
    Java_electionguard_gpu_EgHip_commRank(env, C, N0);
    EXPECT("commRank(0)", AE);
  }

  /* ---- device memory and the tally exchange ---- */
  Java_electionguard_gpu_EgHip_devAlloc(env, C, N0, -1);
  EXPECT("devAlloc bytes < 0", IAE);
  Java_electionguard_gpu_EgHip_devAlloc(env, C, N0, 64);
  EXPECT("devAlloc(0)", AE);
  EXPECT_MSG("null");
  Java_electionguard_gpu_EgHip_devFree(env, C, N0, 0);
  EXPECT("devFree(0)", AE);
  Java_electionguard_gpu_EgHip_memcpyHtoD(env, C, N0, 0, sh, 4, 8);
  EXPECT("memcpyHtoD past the array", IAE);
  Java_electionguard_gpu_EgHip_memcpyHtoD(env, C, N0, 0, p, 0, 512);
  EXPECT("memcpyHtoD(0)", AE);
  Java_electionguard_gpu_EgHip_memcpyDtoH(env, C, N0, sh, -1, 0, 4);
  EXPECT("memcpyDtoH dstOff < 0", IAE);
  Java_electionguard_gpu_EgHip_memcpyDtoH(env, C, N0, p, 0, 0, 512);
  EXPECT("memcpyDtoH(0)", AE);
  Java_electionguard_gpu_EgHip_memsetDev(env, C, N0, 0, 0, 16);
  EXPECT("memsetDev(0)", AE);
  Java_electionguard_gpu_EgHip_allNonzeroDev(env, C, N0, 0, 16);
  EXPECT("allNonzeroDev(0)", AE);
  Java_electionguard_gpu_EgHip_commUniqueId(env, C, sh);
  EXPECT("commUniqueId short out", IAE);
  Java_electionguard_gpu_EgHip_commInit(env, C, N0, sh, 2, 0);
  EXPECT("commInit short id", IAE);
  {
    Obj* id = bytes(128);
    Java_electionguard_gpu_EgHip_commInit(env, C, N0, id, 2, 0);
    EXPECT("commInit(0)", AE);
  }
  Java_electionguard_gpu_EgHip_commDestroy(env, C, N0);
  EXPECT("commDestroy(0)", AE);
  Java_electionguard_gpu_EgHip_commAllValid(env, C, N0, 1);
  EXPECT("commAllValid(0)", AE);
  Java_electionguard_gpu_EgHip_tallyAllgatherFold(env, C, N0, 0, 1, 2, 0, p);
  EXPECT("tallyAllgatherFold short out", IAE);
  Java_electionguard_gpu_EgHip_tallyAllgatherFold(env, C, N0, 0, 1, 2, 0, b2);
  EXPECT("tallyAllgatherFold(0)", AE);

  printf("jni harness: %d checks, %d errors, %d pins, %d releases\n", g_checks, g_errors, g_pins, g_unpins);
  return g_errors || g_pins != g_unpins ? 1 : 0;
}
