/* eg_oracle_c.c — CPU restatement of the batched modexp path over OpenSSL BN.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/ as a second, independent oracle (next to
 * oracle/eg_oracle.py) and by bench.py's cpu_baseline leg.  The product path never
 * links or calls it.  Parity status: see oracle/eg_oracle.py ("parity unpinned" —
 * the reference's arithmetic lives in electionguard-kotlin-multiplatform-jvm
 * 1.0-SNAPSHOT, build.gradle.kts:55, absent from the container).
 *
 * Algorithms restated (the JVM upstream's):
 *   variable base  : BN_mod_exp_mont (Montgomery sliding window, the algorithm class of
 *                    java.math.BigInteger.oddModPow)
 *   fixed base g, K: 8-bit radix table (PowRadixOption.LOW_MEMORY_USE, KUtils.java:11),
 *                    32 windows x 256 entries, product of 32 table entries
 *   hash           : SHA-256 over "|" + "|".join(upper-case fixed-width hex) + "|", mod q
 *                    (matches eg_oracle.py:hash_elems)
 * Verification (including the valid-residue tests x^q == 1 of every alpha, beta, which also
 * decide each contest's (A, B)) follows eg_oracle.py:verify_range_proof / verify_constant_proof and the
 * tally eg_oracle.py:accumulate_tally (Verifier / runAccumulateBallots at
 * RunRemoteWorkflowTest.java:151,179-182).  Multi-threaded over ballots (pthreads), as
 * the reference's Verifier(record, 11) is over 11 JVM threads.
 */
#include <openssl/bn.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  BIGNUM *p, *q, *g;
  BN_MONT_CTX* mont;
} Group;

typedef struct {
  BIGNUM* t[32][256]; /* Montgomery form: base^(d * 256^k) */
} Radix;

static Group G;
static Radix* RG = NULL;
static Radix* RK = NULL;
static BIGNUM* Kbn = NULL;

static BIGNUM* bn_be(const uint8_t* b, int n) { return BN_bin2bn(b, n, NULL); }

static void radix_free(Radix** R) {
  if (!*R) return;
  for (int k = 0; k < 32; ++k)
    for (int d = 0; d < 256; ++d) BN_free((*R)->t[k][d]);
  free(*R);
  *R = NULL;
}

/* (Re)initialise the group; tables of a previous group are dropped. */
int ego_init(const uint8_t p[512], const uint8_t q[32], const uint8_t g[512]) {
  radix_free(&RG);
  radix_free(&RK);
  if (G.p) {
    BN_free(G.p);
    BN_free(G.q);
    BN_free(G.g);
    BN_MONT_CTX_free(G.mont);
  }
  BN_CTX* ctx = BN_CTX_new();
  G.p = bn_be(p, 512);
  G.q = bn_be(q, 32);
  G.g = bn_be(g, 512);
  G.mont = BN_MONT_CTX_new();
  int ok = BN_MONT_CTX_set(G.mont, G.p, ctx);
  BN_CTX_free(ctx);
  return ok ? 0 : 1;
}

static Radix* radix_build(const BIGNUM* base) {
  Radix* R = (Radix*)calloc(1, sizeof(Radix));
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM* b = BN_new();
  BN_to_montgomery(b, base, G.mont, ctx); /* b = base^(256^k) in Montgomery form */
  for (int k = 0; k < 32; ++k) {
    R->t[k][0] = BN_new();
    BN_to_montgomery(R->t[k][0], BN_value_one(), G.mont, ctx);
    for (int d = 1; d < 256; ++d) {
      R->t[k][d] = BN_new();
      BN_mod_mul_montgomery(R->t[k][d], R->t[k][d - 1], b, G.mont, ctx);
    }
    /* next window base: b^256 = t[k][255] * b */
    BN_mod_mul_montgomery(b, R->t[k][255], b, G.mont, ctx);
  }
  BN_free(b);
  BN_CTX_free(ctx);
  return R;
}

/* out = base^e (normal form) via the radix table */
static void radix_pow(BIGNUM* out, const Radix* R, const uint8_t e[32], BN_CTX* ctx) {
  BN_copy(out, R->t[0][e[31]]);
  for (int k = 1; k < 32; ++k) BN_mod_mul_montgomery(out, out, R->t[k][e[31 - k]], G.mont, ctx);
  BN_from_montgomery(out, out, G.mont, ctx);
}

int ego_set_key(const uint8_t K[512]) {
  if (!RG) RG = radix_build(G.g);
  if (Kbn) BN_free(Kbn);
  Kbn = bn_be(K, 512);
  radix_free(&RK);
  RK = radix_build(Kbn);
  return 0;
}

static void hex_put(SHA256_CTX* s, const BIGNUM* x, int nbytes) {
  static const char H[] = "0123456789ABCDEF";
  uint8_t b[512];
  char hx[1024];
  BN_bn2binpad(x, b, nbytes);
  for (int i = 0; i < nbytes; ++i) {
    hx[2 * i] = H[b[i] >> 4];
    hx[2 * i + 1] = H[b[i] & 15];
  }
  SHA256_Update(s, hx, 2 * nbytes);
  SHA256_Update(s, "|", 1);
}

/* H(qbar, P-elements...) mod q */
static void hash_elems(BIGNUM* out, const BIGNUM* qbar, BIGNUM** elems, int n, BN_CTX* ctx) {
  SHA256_CTX s;
  uint8_t d[32];
  SHA256_Init(&s);
  SHA256_Update(&s, "|", 1);
  hex_put(&s, qbar, 32);
  for (int i = 0; i < n; ++i) hex_put(&s, elems[i], 512);
  SHA256_Final(d, &s);
  BN_bin2bn(d, 32, out);
  BN_nnmod(out, out, G.q, ctx);
}

static void mulp(BIGNUM* r, const BIGNUM* a, const BIGNUM* b, BN_CTX* ctx) { BN_mod_mul(r, a, b, G.p, ctx); }

typedef struct {
  size_t b0, b1, nc, spc, ph;
  uint32_t limit;
  const uint8_t *qbar, *cts, *rproof, *cproof;
  uint8_t *ok_sel, *ok_con;
} Job;

static void* verify_worker(void* arg) {
  Job* J = (Job*)arg;
  BN_CTX* ctx = BN_CTX_new();
  BN_CTX_start(ctx);
  BIGNUM *qbar = bn_be(J->qbar, 32), *al = BN_new(), *be = BN_new(), *t1 = BN_new(), *t2 = BN_new();
  BIGNUM *a0 = BN_new(), *b0 = BN_new(), *a1 = BN_new(), *b1 = BN_new(), *h = BN_new(), *cs = BN_new();
  BIGNUM *c0 = BN_new(), *v0 = BN_new(), *c1 = BN_new(), *v1 = BN_new(), *A = BN_new(), *B = BN_new();
  BIGNUM* el[6];
  uint8_t e[32];
  const size_t nsel = J->nc * J->spc;
  for (size_t b = J->b0; b < J->b1; ++b) {
    for (size_t k = 0; k < J->nc; ++k) {
      BN_one(A);
      BN_one(B);
      int msg_ok = 1; /* every selection's alpha, beta in range and valid residues */
      for (size_t s = 0; s < J->spc; ++s) {
        const size_t i = b * nsel + k * J->spc + s;
        const uint8_t* ct = J->cts + i * 1024;
        const uint8_t* pr = J->rproof + i * 128;
        BN_bin2bn(ct, 512, al);
        BN_bin2bn(ct + 512, 512, be);
        BN_bin2bn(pr, 32, c0);
        BN_bin2bn(pr + 32, 32, v0);
        BN_bin2bn(pr + 64, 32, c1);
        BN_bin2bn(pr + 96, 32, v1);
        int ok = BN_cmp(al, G.p) < 0 && BN_cmp(be, G.p) < 0 && BN_cmp(c0, G.q) < 0 && BN_cmp(v0, G.q) < 0 &&
                 BN_cmp(c1, G.q) < 0 && BN_cmp(v1, G.q) < 0;
        /* valid residues: alpha^q == 1 and beta^q == 1 (eg_oracle.py:is_valid_residue) */
        int res = BN_cmp(al, G.p) < 0 && BN_cmp(be, G.p) < 0;
        BN_mod_exp_mont(t1, al, G.q, G.p, ctx, G.mont);
        res = res && BN_is_one(t1);
        BN_mod_exp_mont(t1, be, G.q, G.p, ctx, G.mont);
        res = res && BN_is_one(t1);
        ok = ok && res;
        msg_ok = msg_ok && res;
        /* a0 = g^v0 al^c0 ; b0 = K^v0 be^c0 ; a1 = g^v1 al^c1 ; b1 = K^v1 be^c1 g^-c1 */
        radix_pow(t1, RG, pr + 32, ctx);
        BN_mod_exp_mont(t2, al, c0, G.p, ctx, G.mont);
        mulp(a0, t1, t2, ctx);
        radix_pow(t1, RK, pr + 32, ctx);
        BN_mod_exp_mont(t2, be, c0, G.p, ctx, G.mont);
        mulp(b0, t1, t2, ctx);
        radix_pow(t1, RG, pr + 96, ctx);
        BN_mod_exp_mont(t2, al, c1, G.p, ctx, G.mont);
        mulp(a1, t1, t2, ctx);
        radix_pow(t1, RK, pr + 96, ctx);
        BN_mod_exp_mont(t2, be, c1, G.p, ctx, G.mont);
        mulp(b1, t1, t2, ctx);
        BN_sub(t1, G.q, c1); /* (q - c1) mod q */
        BN_nnmod(t1, t1, G.q, ctx);
        BN_bn2binpad(t1, e, 32);
        radix_pow(t2, RG, e, ctx);
        mulp(b1, b1, t2, ctx);
        el[0] = al; el[1] = be; el[2] = a0; el[3] = b0; el[4] = a1; el[5] = b1;
        hash_elems(h, qbar, el, 6, ctx);
        BN_mod_add(cs, c0, c1, G.q, ctx);
        ok = ok && BN_cmp(cs, h) == 0;
        J->ok_sel[i] = (uint8_t)ok;
        mulp(A, A, al, ctx);
        mulp(B, B, be, ctx);
      }
      /* contest: a = g^v A^c ; b = K^v B^c g^-Lc */
      const uint8_t* cp = J->cproof + (b * J->nc + k) * 64;
      BN_bin2bn(cp, 32, c0);
      BN_bin2bn(cp + 32, 32, v0);
      /* (A, B) valid: the subgroup is closed under products, so its factors decide
       * (eg_oracle.py:verify_ballot) */
      int ok = msg_ok && BN_cmp(c0, G.q) < 0 && BN_cmp(v0, G.q) < 0;
      radix_pow(t1, RG, cp + 32, ctx);
      BN_mod_exp_mont(t2, A, c0, G.p, ctx, G.mont);
      mulp(a0, t1, t2, ctx);
      radix_pow(t1, RK, cp + 32, ctx);
      BN_mod_exp_mont(t2, B, c0, G.p, ctx, G.mont);
      mulp(b0, t1, t2, ctx);
      BN_set_word(t1, J->limit);
      BN_mod_mul(t1, t1, c0, G.q, ctx);
      BN_sub(t1, G.q, t1);
      BN_nnmod(t1, t1, G.q, ctx);
      BN_bn2binpad(t1, e, 32);
      radix_pow(t2, RG, e, ctx);
      mulp(b0, b0, t2, ctx);
      el[0] = A; el[1] = B; el[2] = a0; el[3] = b0;
      hash_elems(h, qbar, el, 4, ctx);
      J->ok_con[b * J->nc + k] = (uint8_t)(ok && BN_cmp(h, c0) == 0);
    }
  }
  BIGNUM* all[] = {qbar, al, be, t1, t2, a0, b0, a1, b1, h, cs, c0, v0, c1, v1, A, B};
  for (size_t i = 0; i < sizeof(all) / sizeof(all[0]); ++i) BN_free(all[i]);
  BN_CTX_end(ctx);
  BN_CTX_free(ctx);
  return NULL;
}

/* Verify + tally nb ballots (layout as include/eg_hip.h eg_verify_ballots). */
int ego_verify_ballots(const uint8_t qbar[32], size_t nb, size_t nc, size_t spc, size_t ph, uint32_t limit,
                       const uint8_t* cts, const uint8_t* rproof, const uint8_t* cproof, uint8_t* ok_sel,
                       uint8_t* ok_con, uint8_t* tally, int threads) {
  if (!RK) return 1;
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  Job* jobs = (Job*)calloc(threads, sizeof(Job));
  for (int t = 0; t < threads; ++t) {
    Job* J = &jobs[t];
    J->b0 = nb * t / threads;
    J->b1 = nb * (t + 1) / threads;
    J->nc = nc; J->spc = spc; J->ph = ph; J->limit = limit;
    J->qbar = qbar; J->cts = cts; J->rproof = rproof; J->cproof = cproof;
    J->ok_sel = ok_sel; J->ok_con = ok_con;
    pthread_create(&th[t], NULL, verify_worker, J);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  if (tally) {
    /* runAccumulateBallots: per real selection, product over ballots */
    BN_CTX* ctx = BN_CTX_new();
    BIGNUM *acc = BN_new(), *x = BN_new();
    const size_t nsel = nc * spc, nrs = spc - ph;
    for (size_t k = 0; k < nc; ++k)
      for (size_t s = 0; s < nrs; ++s)
        for (int c = 0; c < 2; ++c) {
          BN_one(acc);
          for (size_t b = 0; b < nb; ++b) {
            BN_bin2bn(cts + ((b * nsel + k * spc + s) * 2 + c) * 512, 512, x);
            BN_mod_mul(acc, acc, x, G.p, ctx);
          }
          BN_bn2binpad(acc, tally + ((k * nrs + s) * 2 + c) * 512, 512);
        }
    BN_free(acc);
    BN_free(x);
    BN_CTX_free(ctx);
  }
  return 0;
}

/* Variable-base powP batch (BigInteger.modPow semantics: base reduced mod p). */
int ego_powp(const uint8_t* base, const uint8_t* exp, uint8_t* out, size_t n) {
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *b = BN_new(), *e = BN_new(), *r = BN_new();
  for (size_t i = 0; i < n; ++i) {
    BN_bin2bn(base + i * 512, 512, b);
    BN_nnmod(b, b, G.p, ctx);
    BN_bin2bn(exp + i * 32, 32, e);
    BN_mod_exp_mont(r, b, e, G.p, ctx, G.mont);
    BN_bn2binpad(r, out + i * 512, 512);
  }
  BN_free(b);
  BN_free(e);
  BN_free(r);
  BN_CTX_free(ctx);
  return 0;
}

/* Fixed-base g^e via the 8-bit radix table. */
int ego_gpowp(const uint8_t* exp, uint8_t* out, size_t n) {
  if (!RG) RG = radix_build(G.g);
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM* r = BN_new();
  for (size_t i = 0; i < n; ++i) {
    radix_pow(r, RG, exp + i * 32, ctx);
    BN_bn2binpad(r, out + i * 512, 512);
  }
  BN_free(r);
  BN_CTX_free(ctx);
  return 0;
}

/* ---------------------------------------------------------------------------------------------
 * Encryption with injected nonces (batchEncryption, RunRemoteWorkflowTest.java:140-141), restating
 * eg_oracle.py:encrypt / make_range_proof / make_constant_proof.  Per selection (R, u, c_fake,
 * v_fake): alpha = g^R, beta = K^R g^m; the real branch commits (g^u, K^u), the fake branch is
 * simulated with the known nonce: a_f = g^(v_f + R c_f), b_f = K^(v_f + R c_f) g^(+-c_f) (the
 * values of g^v_f alpha^c_f and K^v_f (beta g^-f)^c_f); c = H(qbar, alpha, beta, a0, b0, a1, b1),
 * c_real = c - c_f, v_real = u - c_real R.  Per contest: (g^u, K^u), c = H(qbar, A, B, a, b),
 * v = u - c R_sum.  Fixed-base terms use the 8-bit radix tables (LOW_MEMORY_USE).
 * --------------------------------------------------------------------------------------------- */
typedef struct {
  size_t b0, b1, nc, spc;
  const uint8_t *qbar, *votes, *sn, *cn;
  uint8_t *cts, *rproof, *cproof;
} EncJob;

static void q_bytes(uint8_t out[32], const BIGNUM* x) { BN_bn2binpad(x, out, 32); }

static void* encrypt_worker(void* arg) {
  EncJob* J = (EncJob*)arg;
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *qbar = bn_be(J->qbar, 32), *al = BN_new(), *be = BN_new(), *t1 = BN_new(), *t2 = BN_new();
  BIGNUM *ar = BN_new(), *br = BN_new(), *af = BN_new(), *bf = BN_new(), *h = BN_new();
  BIGNUM *R = BN_new(), *u = BN_new(), *cf = BN_new(), *vf = BN_new(), *sf = BN_new(), *cr = BN_new(), *vr = BN_new();
  BIGNUM *A = BN_new(), *B = BN_new(), *Rs = BN_new();
  BIGNUM* el[6];
  uint8_t e[32];
  const size_t nsel = J->nc * J->spc;
  for (size_t b = J->b0; b < J->b1; ++b) {
    for (size_t k = 0; k < J->nc; ++k) {
      BN_one(A);
      BN_one(B);
      BN_zero(Rs);
      for (size_t s = 0; s < J->spc; ++s) {
        const size_t i = b * nsel + k * J->spc + s;
        const uint8_t* n4 = J->sn + i * 128;
        const int m = J->votes[i] != 0;
        BN_bin2bn(n4, 32, R);
        BN_bin2bn(n4 + 32, 32, u);
        BN_bin2bn(n4 + 64, 32, cf);
        BN_bin2bn(n4 + 96, 32, vf);
        radix_pow(al, RG, n4, ctx);                 /* alpha = g^R */
        radix_pow(be, RK, n4, ctx);                 /* beta = K^R g^m */
        if (m) mulp(be, be, G.g, ctx);
        radix_pow(ar, RG, n4 + 32, ctx);            /* real branch: g^u, K^u */
        radix_pow(br, RK, n4 + 32, ctx);
        BN_mod_mul(sf, R, cf, G.q, ctx);            /* s_f = v_f + R c_f */
        BN_mod_add(sf, sf, vf, G.q, ctx);
        q_bytes(e, sf);
        radix_pow(af, RG, e, ctx);
        radix_pow(bf, RK, e, ctx);
        if (m) BN_copy(t1, cf);                     /* g^(c_f) for m = 1, g^(-c_f) for m = 0 */
        else {
          BN_sub(t1, G.q, cf);
          BN_nnmod(t1, t1, G.q, ctx);
        }
        q_bytes(e, t1);
        radix_pow(t2, RG, e, ctx);
        mulp(bf, bf, t2, ctx);
        el[0] = al; el[1] = be;
        if (m == 0) { el[2] = ar; el[3] = br; el[4] = af; el[5] = bf; }
        else { el[2] = af; el[3] = bf; el[4] = ar; el[5] = br; }
        hash_elems(h, qbar, el, 6, ctx);
        BN_mod_sub(cr, h, cf, G.q, ctx);            /* c_real = c - c_f */
        BN_mod_mul(t1, cr, R, G.q, ctx);            /* v_real = u - c_real R */
        BN_mod_sub(vr, u, t1, G.q, ctx);
        uint8_t* ct = J->cts + i * 1024;
        BN_bn2binpad(al, ct, 512);
        BN_bn2binpad(be, ct + 512, 512);
        uint8_t* pr = J->rproof + i * 128;
        if (m == 0) { q_bytes(pr, cr); q_bytes(pr + 32, vr); q_bytes(pr + 64, cf); q_bytes(pr + 96, vf); }
        else { q_bytes(pr, cf); q_bytes(pr + 32, vf); q_bytes(pr + 64, cr); q_bytes(pr + 96, vr); }
        mulp(A, A, al, ctx);
        mulp(B, B, be, ctx);
        BN_mod_add(Rs, Rs, R, G.q, ctx);
      }
      const uint8_t* uc = J->cn + (b * J->nc + k) * 32;
      BN_bin2bn(uc, 32, u);
      radix_pow(ar, RG, uc, ctx);
      radix_pow(br, RK, uc, ctx);
      el[0] = A; el[1] = B; el[2] = ar; el[3] = br;
      hash_elems(h, qbar, el, 4, ctx);
      BN_mod_mul(t1, h, Rs, G.q, ctx);              /* v = u - c R_sum */
      BN_mod_sub(vr, u, t1, G.q, ctx);
      uint8_t* cp = J->cproof + (b * J->nc + k) * 64;
      q_bytes(cp, h);
      q_bytes(cp + 32, vr);
    }
  }
  BIGNUM* all[] = {qbar, al, be, t1, t2, ar, br, af, bf, h, R, u, cf, vf, sf, cr, vr, A, B, Rs};
  for (size_t i = 0; i < sizeof(all) / sizeof(all[0]); ++i) BN_free(all[i]);
  BN_CTX_free(ctx);
  return NULL;
}

/* Encrypt nb ballots (layouts as include/eg_hip.h eg_encrypt_ballots). */
int ego_encrypt_ballots(const uint8_t qbar[32], size_t nb, size_t nc, size_t spc, const uint8_t* votes,
                        const uint8_t* sel_nonces, const uint8_t* contest_nonces, uint8_t* cts, uint8_t* rproof,
                        uint8_t* cproof, int threads) {
  if (!RK) return 1;
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  EncJob* jobs = (EncJob*)calloc(threads, sizeof(EncJob));
  for (int t = 0; t < threads; ++t) {
    EncJob* J = &jobs[t];
    J->b0 = nb * t / threads;
    J->b1 = nb * (t + 1) / threads;
    J->nc = nc; J->spc = spc; J->qbar = qbar; J->votes = votes; J->sn = sel_nonces; J->cn = contest_nonces;
    J->cts = cts; J->rproof = rproof; J->cproof = cproof;
    pthread_create(&th[t], NULL, encrypt_worker, J);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}

/* ---------------------------------------------------------------------------------------------
 * Trustee partial decryption (DecryptingTrusteeIF.directDecrypt / compensatedDecrypt,
 * RunRemoteDecryptingTrustee.java:189-193,227-232), restating eg_oracle.py:direct_decrypt: per
 * text, M = pad^s, proof nonce u: a = g^u, b = pad^u, c = H(qbar, pad, data, a, b, M), v = u - c s.
 * --------------------------------------------------------------------------------------------- */
typedef struct {
  size_t i0, i1;
  const uint8_t *secret, *qbar, *texts, *nonces;
  uint8_t *M, *proof;
} TrJob;

static void* trustee_worker(void* arg) {
  TrJob* J = (TrJob*)arg;
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *qbar = bn_be(J->qbar, 32), *s = bn_be(J->secret, 32), *pad = BN_new(), *dat = BN_new(), *M = BN_new();
  BIGNUM *u = BN_new(), *a = BN_new(), *b = BN_new(), *h = BN_new(), *t = BN_new(), *v = BN_new();
  BIGNUM* el[5];
  for (size_t i = J->i0; i < J->i1; ++i) {
    BN_bin2bn(J->texts + i * 1024, 512, pad);
    BN_bin2bn(J->texts + i * 1024 + 512, 512, dat);
    BN_bin2bn(J->nonces + i * 32, 32, u);
    BN_mod_exp_mont(M, pad, s, G.p, ctx, G.mont);
    radix_pow(a, RG, J->nonces + i * 32, ctx);
    BN_mod_exp_mont(b, pad, u, G.p, ctx, G.mont);
    el[0] = pad; el[1] = dat; el[2] = a; el[3] = b; el[4] = M;
    hash_elems(h, qbar, el, 5, ctx);
    BN_mod_mul(t, h, s, G.q, ctx);
    BN_mod_sub(v, u, t, G.q, ctx);
    BN_bn2binpad(M, J->M + i * 512, 512);
    q_bytes(J->proof + i * 64, h);
    q_bytes(J->proof + i * 64 + 32, v);
  }
  BIGNUM* all[] = {qbar, s, pad, dat, M, u, a, b, h, t, v};
  for (size_t i = 0; i < sizeof(all) / sizeof(all[0]); ++i) BN_free(all[i]);
  BN_CTX_free(ctx);
  return NULL;
}

int ego_trustee_decrypt(const uint8_t secret[32], const uint8_t qbar[32], const uint8_t* texts, const uint8_t* nonces,
                        size_t n, uint8_t* out_M, uint8_t* out_proof, int threads) {
  if (!RG) RG = radix_build(G.g);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  TrJob* jobs = (TrJob*)calloc(threads, sizeof(TrJob));
  for (int t = 0; t < threads; ++t) {
    TrJob* J = &jobs[t];
    J->i0 = n * t / threads;
    J->i1 = n * (t + 1) / threads;
    J->secret = secret; J->qbar = qbar; J->texts = texts; J->nonces = nonces; J->M = out_M; J->proof = out_proof;
    pthread_create(&th[t], NULL, trustee_worker, J);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}
