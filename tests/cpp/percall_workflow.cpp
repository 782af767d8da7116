// percall_workflow.cpp -- the reference's per-element call pattern, end to end, through the C++ mirror's
// per-element API only (host/electionguard.hpp: ElementModP.powP / times / isValidResidue,
// GroupContext.gPowP, the accelerated election key K.powP), on 11 threads, against the CPU port on 11
// threads for the same ballots in the same run.
//
// Upstream runs batchEncryption(..., 11, ...) and Verifier(record, 11).verify() one element at a time
// on the group KUtils.productionGroup() makes (RunRemoteWorkflowTest.java:140-141,179-181;
// KUtils.java:10-12), and runAccumulateBallots single-threaded (:151).  This driver restates their
// per-selection call order:
//   encrypt  alpha = g^R, beta = K^R (* g), the real branch (g^u, K^u), the simulated branch
//            g^v * alpha^c and K^v * beta^c (* g^-c), then the Fiat-Shamir hash, then the responses;
//            per contest (g^u, K^u), H(A, B, a, b), v = u - c R_sum  (eg_oracle.py:make_range_proof);
//   verify   g^v0 * alpha^c0, K^v0 * beta^c0, g^v1 * alpha^c1, K^v1 * beta^c1 * g^-c1, the residue
//            tests alpha^q = beta^q = 1, then the hash; per contest g^v * A^c, K^v * B^c * g^-Lc
//            (eg_oracle.py:verify_range_proof / verify_constant_proof);
//   tally    acc = acc * alpha_b, acc' = acc' * beta_b over the ballots, one thread.
// The hash is host SHA-256 (OpenSSL) over the ctx's default pre-image (eg_hip.h
// EG_HASH_FIXED_WIDTH, EG_RESPONSE_MINUS, EG_PREIMAGE_MESSAGE_FIRST); the nonces are injected.
// Bit-exactness: every ciphertext and proof byte against the C oracle's batch encryption of the same
// nonces, every verdict against its verifier, the tally against a BN_mod_mul loop (oracle/eg_oracle_c.c,
// test infrastructure linked into this driver only).
//
//   percall_workflow <nballots> [threads=11] [eager] [ct]   -> one JSON line on stdout; exit 1 on any mismatch
//     eager: GroupContext::setDeferred(false), every per-element call one blocking round trip (the A/B);
//     ct:    eg_ctx_set_ct_pow on
#include <openssl/bn.h>
#include <openssl/sha.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "eg_constants.hpp"
#include "eg_hip.h"
#include "electionguard.hpp"

extern "C" {  // oracle/eg_oracle_c.c (libegoracle.so): the CPU port and checker
int ego_init(const uint8_t p[512], const uint8_t q[32], const uint8_t g[512]);
int ego_set_key(const uint8_t K[512]);
int ego_encrypt_ballots(const uint8_t qbar[32], size_t nb, size_t nc, size_t spc, const uint8_t* votes,
                        const uint8_t* sel_nonces, const uint8_t* contest_nonces, uint8_t* cts, uint8_t* rproof,
                        uint8_t* cproof, int threads);
int ego_verify_ballots(const uint8_t qbar[32], size_t nb, size_t nc, size_t spc, size_t ph, uint32_t limit,
                       const uint8_t* cts, const uint8_t* rproof, const uint8_t* cproof, uint8_t* ok_sel,
                       uint8_t* ok_con, uint8_t* tally, int threads);
int ego_trustee_decrypt(const uint8_t secret[32], const uint8_t qbar[32], const uint8_t* texts, const uint8_t* nonces,
                        size_t n, uint8_t* out_M, uint8_t* out_proof, int threads);
}

using namespace electionguard;
using Clock = std::chrono::steady_clock;
static double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }

constexpr size_t kNC = 4, kSPC = 6, kNSEL = kNC * kSPC;  // 4 contests x (5 selections + 1 placeholder)

// Fiat-Shamir: SHA-256 over "|" + hex(qbar) + "|" + hex(e_1) + "|" ... (upper case, wire widths), mod q.
// Every element is resolved first, together: one GPU round trip for all of them.
static ElementModQ hashElements(const GroupContext& G, const ElementModQ& qbar, std::vector<const ElementModP*> els) {
  G.resolveAll(els);
  static const char H[] = "0123456789ABCDEF";
  SHA256_CTX s;
  SHA256_Init(&s);
  SHA256_Update(&s, "|", 1);
  auto put = [&](const uint8_t* b, size_t n) {
    std::string hx(2 * n, '0');
    for (size_t i = 0; i < n; ++i) {
      hx[2 * i] = H[b[i] >> 4];
      hx[2 * i + 1] = H[b[i] & 15];
    }
    SHA256_Update(&s, hx.data(), hx.size());
    SHA256_Update(&s, "|", 1);
  };
  const auto qb = qbar.byteArray();
  put(qb.data(), 32);
  for (const auto* e : els) put(e->byteArray(), EG_P_BYTES);
  uint8_t d[32];
  SHA256_Final(d, &s);
  return ElementModQ(G.modq().reduce_small(U256::from_be(d)));
}

struct Election {
  const GroupContext* G;
  ElementModP K;  // accelerated (K.acceleratePow())
  ElementModP g;  // G.G(): g's table
  ElementModQ qbar;
  size_t nb;
  std::vector<uint8_t> votes, sn, cn;  // nb*nsel, nb*nsel*4*32, nb*nc*32
};

static ElementModQ q_at(const uint8_t* p) { return ElementModQ::from_be(p); }

// one ballot, upstream's encryption order; writes the eg_hip.h wire layout
static void encryptBallot(const Election& E, size_t b, uint8_t* cts, uint8_t* rp, uint8_t* cp) {
  const GroupContext& G = *E.G;
  for (size_t k = 0; k < kNC; ++k) {
    ElementModP A = G.one(), B = G.one();
    ElementModQ Rsum;
    for (size_t s = 0; s < kSPC; ++s) {
      const size_t i = b * kNSEL + k * kSPC + s;
      const int m = E.votes[i] != 0;
      const uint8_t* n4 = &E.sn[i * 128];
      const ElementModQ R = q_at(n4), u = q_at(n4 + 32), cf = q_at(n4 + 64), vf = q_at(n4 + 96);
      const ElementModP alpha = G.gPowP(R);
      ElementModP beta = E.K.powP(R);
      if (m) beta = beta.times(E.g);
      const ElementModP ar = G.gPowP(u), br = E.K.powP(u);
      const ElementModP af = G.gPowP(vf).times(alpha.powP(cf));
      ElementModP bf = E.K.powP(vf).times(beta.powP(cf));
      if (!m) bf = bf.times(G.gPowP(G.negQ(cf)));
      const ElementModP *a0 = m ? &af : &ar, *b0 = m ? &bf : &br, *a1 = m ? &ar : &af, *b1 = m ? &br : &bf;
      const ElementModQ c = hashElements(G, E.qbar, {&alpha, &beta, a0, b0, a1, b1});
      const ElementModQ cr = G.subQ(c, cf), vr = G.subQ(u, G.mulQ(cr, R));
      std::memcpy(cts + i * 1024, alpha.byteArray(), 512);
      std::memcpy(cts + i * 1024 + 512, beta.byteArray(), 512);
      uint8_t* pr = rp + i * 128;
      const ElementModQ* w[4] = {m ? &cf : &cr, m ? &vf : &vr, m ? &cr : &cf, m ? &vr : &vf};
      for (int j = 0; j < 4; ++j) w[j]->v.to_be(pr + 32 * j);
      A = A.times(alpha);
      B = B.times(beta);
      Rsum = G.addQ(Rsum, R);
    }
    const ElementModQ uc = q_at(&E.cn[(b * kNC + k) * 32]);
    const ElementModP a = G.gPowP(uc), bb = E.K.powP(uc);
    const ElementModQ c = hashElements(G, E.qbar, {&A, &B, &a, &bb});
    const ElementModQ v = G.subQ(uc, G.mulQ(c, Rsum));
    c.v.to_be(cp + (b * kNC + k) * 64);
    v.v.to_be(cp + (b * kNC + k) * 64 + 32);
  }
}

static bool lessThan(const uint8_t* a, const uint8_t* b, size_t n) { return std::memcmp(a, b, n) < 0; }

// one ballot, upstream's verification order -> ok_sel[nsel], ok_con[nc]
static void verifyBallot(const Election& E, size_t b, const uint8_t* cts, const uint8_t* rp, const uint8_t* cp,
                         uint8_t* ok_sel, uint8_t* ok_con) {
  const GroupContext& G = *E.G;
  const auto qb = G.Q().byteArray();
  const ElementModP ONE = G.one();
  for (size_t k = 0; k < kNC; ++k) {
    ElementModP A = G.one(), B = G.one();
    bool msg_ok = true;
    for (size_t s = 0; s < kSPC; ++s) {
      const size_t i = b * kNSEL + k * kSPC + s;
      const ElementModP alpha = G.binaryToElementModP(cts + i * 1024), beta = G.binaryToElementModP(cts + i * 1024 + 512);
      const uint8_t* pr = rp + i * 128;
      const ElementModQ c0 = q_at(pr), v0 = q_at(pr + 32), c1 = q_at(pr + 64), v1 = q_at(pr + 96);
      bool ok = lessThan(alpha.byteArray(), G.P().byteArray(), 512) && lessThan(beta.byteArray(), G.P().byteArray(), 512);
      for (int j = 0; j < 4; ++j) ok = ok && lessThan(pr + 32 * j, qb.data(), 32);
      const ElementModP a0 = G.gPowP(v0).times(alpha.powP(c0));
      const ElementModP b0 = E.K.powP(v0).times(beta.powP(c0));
      const ElementModP a1 = G.gPowP(v1).times(alpha.powP(c1));
      const ElementModP b1 = E.K.powP(v1).times(beta.powP(c1)).times(G.gPowP(G.negQ(c1)));
      // the residue tests (isValidResidue: x^q == 1), deferred like the rest: one round trip per selection
      const ElementModP ra = alpha.powP(G.Q()), rb = beta.powP(G.Q());
      // (hashing resolves this thread's pending jobs -- the four commitments and both residues -- at once)
      const ElementModQ c = hashElements(G, E.qbar, {&alpha, &beta, &a0, &b0, &a1, &b1});
      const bool res = ra == ONE && rb == ONE;
      ok = ok && res && c == G.addQ(c0, c1);
      msg_ok = msg_ok && res;
      ok_sel[i] = ok;
      A = A.times(alpha);
      B = B.times(beta);
    }
    const uint8_t* q2 = cp + (b * kNC + k) * 64;
    const ElementModQ c = q_at(q2), v = q_at(q2 + 32);
    bool ok = msg_ok && lessThan(q2, qb.data(), 32) && lessThan(q2 + 32, qb.data(), 32);
    const ElementModP a = G.gPowP(v).times(A.powP(c));
    const ElementModP bb = E.K.powP(v).times(B.powP(c)).times(G.gPowP(G.negQ(c))  /* L = votesAllowed = 1 */);
    ok = ok && hashElements(G, E.qbar, {&A, &B, &a, &bb}) == c;
    ok_con[b * kNC + k] = ok;
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: percall_workflow <nballots> [threads]\n");
    return 2;
  }
  const size_t nb = (size_t)std::atol(argv[1]);
  const int T = argc > 2 ? std::atoi(argv[2]) : 11;
  bool eager = false, ct = false;
  for (int a = 3; a < argc; ++a) {
    eager |= std::strcmp(argv[a], "eager") == 0;  // every per-element call blocks (no deferral): the A/B
    ct |= std::strcmp(argv[a], "ct") == 0;        // eg_ctx_set_ct_pow on (constant-time schedules)
  }
  GroupContext& G = GroupContext::productionGroup(0);
  G.setDeferred(!eager);
  G.setConstantTime(ct);
  std::mt19937_64 rng(20261018);
  auto [guardians, K] = keyCeremony(G, 3, 3, 7);
  (void)guardians;
  Election E{&G, G.acceleratePow(K), G.G(), G.randomElementModQ(rng), nb, {}, {}, {}};
  E.votes.assign(nb * kNSEL, 0);
  for (size_t b = 0; b < nb; ++b)
    for (size_t k = 0; k < kNC; ++k) E.votes[b * kNSEL + k * kSPC + rng() % kSPC] = 1;  // last = placeholder
  E.sn.resize(nb * kNSEL * 128);
  E.cn.resize(nb * kNC * 32);
  for (size_t i = 0; i < nb * kNSEL * 4; ++i) G.randomElementModQ(rng).v.to_be(&E.sn[i * 32]);
  for (size_t i = 0; i < nb * kNC; ++i) G.randomElementModQ(rng).v.to_be(&E.cn[i * 32]);
  const auto qbar = E.qbar.byteArray();

  // ---- the CPU port (the checker), 11 threads ----
  const auto qb = G.Q().byteArray();
  ego_init(G.P().byteArray(), qb.data(), G.G().byteArray());
  ego_set_key(K.byteArray());
  std::vector<uint8_t> cts_ref(nb * kNSEL * 1024), rp_ref(nb * kNSEL * 128), cp_ref(nb * kNC * 64);
  auto t = Clock::now();
  ego_encrypt_ballots(qbar.data(), nb, kNC, kSPC, E.votes.data(), E.sn.data(), E.cn.data(), cts_ref.data(), rp_ref.data(),
                      cp_ref.data(), T);
  const double cpu_enc_s = secs(t);
  std::vector<uint8_t> oks_ref(nb * kNSEL), okc_ref(nb * kNC);
  t = Clock::now();
  ego_verify_ballots(qbar.data(), nb, kNC, kSPC, 1, 1, cts_ref.data(), rp_ref.data(), cp_ref.data(), oks_ref.data(),
                     okc_ref.data(), nullptr, T);
  const double cpu_ver_s = secs(t);

  long bad = 0;
  auto run_threads = [&](auto&& body) {
    std::vector<std::thread> th;
    auto t0 = Clock::now();
    for (int k = 0; k < T; ++k)
      th.emplace_back([&, k] {
        for (size_t b = (size_t)k; b < nb; b += (size_t)T) body(b);
      });
    for (auto& x : th) x.join();
    return secs(t0);
  };
  // ---- per-element encryption and verification on the GPU, 11 threads ----
  std::vector<uint8_t> cts(nb * kNSEL * 1024), rp(nb * kNSEL * 128), cp(nb * kNC * 64);
  std::atomic<long> errors{0};
  auto guarded = [&](auto&& f) {
    return [&, f](size_t b) {
      try {
        f(b);
      } catch (const std::exception& e) {
        if (errors++ == 0) fprintf(stderr, "ballot %zu: %s\n", b, e.what());
      }
    };
  };
  // warm-up outside the timed loops (upstream builds g's table when the group is made, KUtils.java:10-12;
  // here: g's per-element table, the code objects and the coalescer's buffers): one ballot each way
  if (nb) {
    std::vector<uint8_t> c1(nb * kNSEL * 1024), r1(nb * kNSEL * 128), p1(nb * kNC * 64), o1(nb * kNSEL), o2(nb * kNC);
    encryptBallot(E, 0, c1.data(), r1.data(), p1.data());
    verifyBallot(E, 0, cts_ref.data(), rp_ref.data(), cp_ref.data(), o1.data(), o2.data());
  }
  G.setCoalescing(16384, 0);  // the library defaults (with EG_COALESCE_STATS=1: the warm-up's batch statistics)
  const double gpu_enc_s = run_threads(guarded([&](size_t b) { encryptBallot(E, b, cts.data(), rp.data(), cp.data()); }));
  G.setCoalescing(16384, 0);  // (EG_COALESCE_STATS=1: the encryption phase's statistics)
  const long enc_mis = (long)(cts != cts_ref) + (long)(rp != rp_ref) + (long)(cp != cp_ref);
  std::vector<uint8_t> oks(nb * kNSEL), okc(nb * kNC);
  const double gpu_ver_s =
      run_threads(guarded([&](size_t b) { verifyBallot(E, b, cts_ref.data(), rp_ref.data(), cp_ref.data(), oks.data(), okc.data()); }));
  G.setCoalescing(16384, 0);  // (EG_COALESCE_STATS=1: the verification phase's statistics)
  long ver_mis = 0, invalid = 0;
  for (size_t i = 0; i < oks.size(); ++i) ver_mis += oks[i] != oks_ref[i], invalid += !oks[i];
  for (size_t i = 0; i < okc.size(); ++i) ver_mis += okc[i] != okc_ref[i], invalid += !okc[i];
  // a tampered proof must fail through the same path (one selection's v0 and one contest's c)
  long tamper_mis = 0;
  if (nb) {
    std::vector<uint8_t> rp2 = rp_ref, cp2 = cp_ref, o1(nb * kNSEL), o2(nb * kNC);
    rp2[32 + 31] ^= 1;
    cp2[5] ^= 0x40;
    verifyBallot(E, 0, cts_ref.data(), rp2.data(), cp2.data(), o1.data(), o2.data());
    tamper_mis = (o1[0] != 0) + (o2[0] != 0);
  }

  // ---- the tally loop (runAccumulateBallots, one thread): per-element times against BN_mod_mul ----
  const size_t nreal = kNC * (kSPC - 1);
  std::vector<uint8_t> tal_ref(nreal * 2 * 512), tal(nreal * 2 * 512);
  {
    BN_CTX* bc = BN_CTX_new();
    BIGNUM *p = BN_bin2bn(G.P().byteArray(), 512, nullptr), *acc = BN_new(), *x = BN_new();
    t = Clock::now();
    for (size_t k = 0; k < kNC; ++k)
      for (size_t s = 0; s + 1 < kSPC; ++s)
        for (int c = 0; c < 2; ++c) {
          BN_one(acc);
          for (size_t b = 0; b < nb; ++b) {
            BN_bin2bn(&cts_ref[((b * kNSEL + k * kSPC + s) * 2 + c) * 512], 512, x);
            BN_mod_mul(acc, acc, x, p, bc);
          }
          BN_bn2binpad(acc, &tal_ref[((k * (kSPC - 1) + s) * 2 + c) * 512], 512);
        }
    const double dt = secs(t);
    BN_free(p);
    BN_free(acc);
    BN_free(x);
    BN_CTX_free(bc);
    t = Clock::now();
    std::vector<ElementModP> accs(nreal * 2, G.one());
    for (size_t b = 0; b < nb; ++b)  // ballot-major, as the upstream loop walks the ballots
      for (size_t k = 0; k < kNC; ++k)
        for (size_t s = 0; s + 1 < kSPC; ++s)
          for (int c = 0; c < 2; ++c) {
            auto& a = accs[(k * (kSPC - 1) + s) * 2 + c];
            a = a.times(G.binaryToElementModP(&cts_ref[((b * kNSEL + k * kSPC + s) * 2 + c) * 512]));
          }
    std::vector<const ElementModP*> ps;
    for (auto& a : accs) ps.push_back(&a);
    G.resolveAll(ps);
    for (size_t i = 0; i < accs.size(); ++i) std::memcpy(&tal[i * 512], accs[i].byteArray(), 512);
    const double gt = secs(t);
    const long tal_mis = tal != tal_ref;
    // ---- a trustee's direct decryption shares (DecryptingTrustee.directDecrypt: one thread over the
    //      texts, RunRemoteDecryptingTrustee.java:189-193) through the per-element API with the
    //      constant-time schedules (the secret exponent), against the port on one thread ----
    const size_t nt = std::min<size_t>(nb * kNSEL, 1100);
    const ElementModQ sk = G.randomElementModQ(rng);
    std::vector<uint8_t> tn(nt * 32), tM_ref(nt * 512), tP_ref(nt * 64), tM(nt * 512), tP(nt * 64);
    for (size_t i = 0; i < nt; ++i) G.randomElementModQ(rng).v.to_be(&tn[i * 32]);
    const auto skb = sk.byteArray();
    t = Clock::now();
    ego_trustee_decrypt(skb.data(), qbar.data(), cts_ref.data(), tn.data(), nt, tM_ref.data(), tP_ref.data(), 1);
    const double tr_cpu = secs(t);
    G.setConstantTime(true);
    auto share = [&](size_t i, uint8_t* M_out, uint8_t* P_out) {
      const ElementModP pad = G.binaryToElementModP(&cts_ref[i * 1024]), dat = G.binaryToElementModP(&cts_ref[i * 1024 + 512]);
      const ElementModQ u = q_at(&tn[i * 32]);
      const ElementModP M = pad.powP(sk), a = G.gPowP(u), b = pad.powP(u);
      const ElementModQ c = hashElements(G, E.qbar, {&pad, &dat, &a, &b, &M});
      const ElementModQ v = G.subQ(u, G.mulQ(c, sk));
      std::memcpy(M_out, M.byteArray(), 512);
      c.v.to_be(P_out);
      v.v.to_be(P_out + 32);
    };
    {
      uint8_t m1[512], p1[64];
      share(0, m1, p1);  // warm-up: the constant-time companion of g's table
    }
    t = Clock::now();
    for (size_t i = 0; i < nt; ++i) share(i, &tM[i * 512], &tP[i * 64]);
    const double tr_gpu = secs(t);
    G.setConstantTime(ct);
    const long tr_mis = (long)(tM != tM_ref) + (long)(tP != tP_ref);
    printf("{\"ballots\": %zu, \"threads\": %d, \"deferred\": %s, \"constant_time\": %s, \"selections_per_ballot\": %zu, "
           "\"encrypt_mismatched_arrays\": %ld, \"verify_flag_mismatches\": %ld, \"invalid_flags\": %ld, "
           "\"tamper_not_rejected\": %ld, \"tally_mismatch\": %ld, \"errors\": %ld, "
           "\"encrypt_ballots_per_s\": {\"gpu_per_element\": %.1f, \"cpu_port\": %.1f}, "
           "\"verify_ballots_per_s\": {\"gpu_per_element\": %.1f, \"cpu_port\": %.1f}, "
           "\"tally_ballots_per_s_one_thread\": {\"gpu_per_element\": %.1f, \"cpu_port\": %.1f}, "
           "\"trustee_texts\": %zu, \"trustee_mismatched_arrays\": %ld, "
           "\"trustee_shares_per_s_one_thread\": {\"gpu_per_element_constant_time\": %.1f, \"cpu_port\": %.1f}, "
           "\"cpu_port\": \"oracle/eg_oracle_c.c (OpenSSL BN_mod_exp_mont + 8-bit radix fixed base), %d threads; tally: "
           "BN_mod_mul loop, one thread\"}\n",
           nb, T, eager ? "false" : "true", ct ? "true" : "false", kNSEL, enc_mis, ver_mis, invalid, tamper_mis, tal_mis, errors.load(), nb / gpu_enc_s, nb / cpu_enc_s,
           nb / gpu_ver_s, nb / cpu_ver_s, nb / gt, nb / dt, nt, tr_mis, nt / tr_gpu, nt / tr_cpu, T);
    bad = enc_mis + ver_mis + invalid + tamper_mis + tal_mis + tr_mis + errors.load();
  }
  return bad == 0 ? 0 : 1;
}
