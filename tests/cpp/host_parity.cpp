// host_parity.cpp -- parity driver for the C++ host mirror (electionguard-remote_amd/host/
// electionguard.hpp) over the C ABI.  Run by tests/test_cpp_host.py:
//   host_parity cpu               host-only checks (mod-q arithmetic, constants, ABI info)
//   host_parity gpu <vectors> [V2] golden vectors (tests/golden/<mode>/*.json flattened to text by
//                                 the test) through the C++ API, then a 5-guardian /
//                                 quorum-3 decryption with 2 missing guardians (config 4
//                                 shape) that must recover the exact counts.
// Prints "OK <checks>" and exits 0, or prints the first mismatch and exits 1.
#include <cstdio>
#include <fstream>
#include <random>
#include <iostream>
#include <sstream>

#include "electionguard.hpp"

using namespace electionguard;

static int g_checks = 0;
#define EXPECT(cond, msg)                                             \
  do {                                                                \
    ++g_checks;                                                       \
    if (!(cond)) {                                                    \
      std::cerr << "FAIL " << __LINE__ << ": " << msg << std::endl;   \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

static int run_cpu() {
  char ver[256];
  EXPECT(eg_version(ver, sizeof ver) == EG_OK, "eg_version");
  const ElementModP p = ElementModP::from_hex(constants::kP_HEX);
  const ElementModQ q = ElementModQ::from_hex(constants::kQ_HEX);
  EXPECT(p.be[0] == 0xFF && (p.be[511] & 1), "p: top byte 0xFF and odd");
  // q = 2^256 - 189
  U256 q2;
  U256::sub(q2, U256{{~0ull, ~0ull, ~0ull, ~0ull}}, U256::from_u64(188));
  EXPECT(q.v == q2, "q = 2^256 - 189");
  const ModQ mq{q.v};
  std::mt19937_64 rng(7);
  for (int it = 0; it < 200; ++it) {
    U256 a, b;
    for (auto& w : a.w) w = rng();
    for (auto& w : b.w) w = rng();
    a = mq.reduce_small(a);
    b = mq.reduce_small(b);
    EXPECT(mq.sub(mq.add(a, b), b) == a, "(a+b)-b");
    EXPECT(mq.mul(a, b) == mq.mul(b, a), "ab = ba");
    if (!a.is_zero()) EXPECT(mq.mul(a, mq.inv(a)) == U256::from_u64(1), "a * a^-1");
    EXPECT(mq.add(a, mq.neg(a)).is_zero(), "a + (-a)");
  }
  // known answer: (q-1)^2 = 1 mod q; 2^256 mod q = 189
  U256 qm1;
  U256::sub(qm1, q.v, U256::from_u64(1));
  EXPECT(mq.mul(qm1, qm1) == U256::from_u64(1), "(q-1)^2");
  EXPECT(mq.mul(U256{{0, 0, 0, 1ull << 63}}, U256::from_u64(2)) == U256::from_u64(189), "2^256 mod q");
  // Lagrange: interpolating P at 0 from any quorum of points recovers P(0)
  std::vector<U256> co;
  for (int j = 0; j < 3; ++j) {
    U256 c;
    for (auto& w : c.w) w = rng();
    co.push_back(mq.reduce_small(c));
  }
  auto P = [&](int x) {
    U256 acc;
    for (int j = 2; j >= 0; --j) acc = mq.add(mq.mul(acc, U256::from_u64((uint64_t)x)), co[j]);
    return acc;
  };
  const std::vector<int> xs = {1, 3, 5};
  U256 s;
  for (int xi : xs) {
    U256 num = U256::from_u64(1), den = U256::from_u64(1);
    for (int xj : xs)
      if (xj != xi) {
        num = mq.mul(num, U256::from_u64((uint64_t)xj));
        den = mq.mul(den, mq.sub(U256::from_u64((uint64_t)xj), U256::from_u64((uint64_t)xi)));
      }
    s = mq.add(s, mq.mul(P(xi), mq.mul(num, mq.inv(den))));
  }
  EXPECT(s == co[0], "Lagrange interpolation recovers P(0)");
  // hex round trips at the wire widths
  EXPECT(ElementModP::from_hex(p.hex()) == p, "P hex round trip");
  EXPECT(ElementModQ::from_hex(q.hex()) == q, "Q hex round trip");
  std::cout << "OK " << g_checks << " (" << ver << ")" << std::endl;
  return 0;
}

static std::vector<std::string> split(const std::string& line) {
  std::istringstream is(line);
  std::vector<std::string> t;
  std::string s;
  while (is >> s) t.push_back(s);
  return t;
}

static int run_gpu(const char* path, ProductionMode mode) {
  GroupContext& G = GroupContext::productionGroup(0, mode);
  std::ifstream in(path);
  if (!in) {
    std::cerr << "cannot open " << path << std::endl;
    return 2;
  }
  // batch the group vectors per op so each op is one GPU call, as the drop-in intends
  std::vector<ElementModP> pb, pr, ga, gb, gr, ia, ir;
  std::vector<ElementModQ> pe, ge;
  std::vector<ElementModP> gpr;
  // trustee golden
  struct GuardianIn {
    int x;
    std::vector<ElementModQ> coeffs;
    std::vector<ElementModP> comm;
  };
  std::vector<GuardianIn> guardians;
  ElementModQ qbar;
  std::vector<ElGamalCiphertext> texts;
  std::vector<ElementModQ> nonces;
  std::vector<std::vector<std::string>> direct, comp;
  std::string line;
  while (std::getline(in, line)) {
    const auto t = split(line);
    if (t.empty()) continue;
    const std::string& op = t[0];
    if (op == "powP") {
      pb.push_back(ElementModP::from_hex(t[1], &G));
      pe.push_back(ElementModQ::from_hex(t[2]));
      pr.push_back(ElementModP::from_hex(t[3], &G));
    } else if (op == "gPowP") {
      ge.push_back(ElementModQ::from_hex(t[1]));
      gpr.push_back(ElementModP::from_hex(t[2], &G));
    } else if (op == "multP") {
      ga.push_back(ElementModP::from_hex(t[1], &G));
      gb.push_back(ElementModP::from_hex(t[2], &G));
      gr.push_back(ElementModP::from_hex(t[3], &G));
    } else if (op == "multInv") {
      ia.push_back(ElementModP::from_hex(t[1], &G));
      ir.push_back(ElementModP::from_hex(t[2], &G));
    } else if (op == "format") {  // response convention and pre-image order of what follows
      G.setProofFormat(std::stoi(t[1]), std::stoi(t[2]));
    } else if (op == "prodP") {
      std::vector<ElementModP> xs;
      for (size_t i = 2; i < t.size(); ++i) xs.push_back(ElementModP::from_hex(t[i], &G));
      EXPECT(G.multP(xs) == ElementModP::from_hex(t[1]), "prodP golden, " << xs.size() << " factors");
    } else if (op == "guardian") {
      GuardianIn gi;
      gi.x = std::stoi(t[1]);
      const int nc = std::stoi(t[2]);
      for (int j = 0; j < nc; ++j) gi.coeffs.push_back(ElementModQ::from_hex(t[3 + j]));
      for (int j = 0; j < nc; ++j) gi.comm.push_back(ElementModP::from_hex(t[3 + nc + j], &G));
      guardians.push_back(gi);
    } else if (op == "qbar") {
      qbar = ElementModQ::from_hex(t[1]);
    } else if (op == "text") {
      texts.push_back({ElementModP::from_hex(t[1], &G), ElementModP::from_hex(t[2], &G)});
    } else if (op == "nonce") {
      nonces.push_back(ElementModQ::from_hex(t[1]));
    } else if (op == "direct") {
      direct.push_back(t);
    } else if (op == "compensated") {
      comp.push_back(t);
    } else {
      std::cerr << "unknown vector op " << op << std::endl;
      return 2;
    }
  }
  {
    const auto o = G.powPBatch(pb, pe);
    for (size_t i = 0; i < o.size(); ++i) EXPECT(o[i] == pr[i], "powP golden #" << i);
    const auto og = G.gPowPBatch(ge);
    for (size_t i = 0; i < og.size(); ++i) EXPECT(og[i] == gpr[i], "gPowP golden #" << i);
    const auto om = G.multPBatch(ga, gb);
    for (size_t i = 0; i < om.size(); ++i) EXPECT(om[i] == gr[i], "multP golden #" << i);
    const auto oi = G.multInvBatch(ia);
    for (size_t i = 0; i < oi.size(); ++i) EXPECT(oi[i] == ir[i], "multInv golden #" << i);
    // per-element API agrees with the batch API
    if (!pb.empty()) EXPECT(pb.back().powP(pe.back()) == pr.back(), "ElementModP.powP");
    if (!ga.empty()) EXPECT(ga[0].times(gb[0]) == gr[0], "ElementModP.times");
  }
  // trustee golden: guardian x=1 direct, guardian x=2 compensating for x=3
  if (!guardians.empty()) {
    std::map<std::string, std::vector<ElementModP>> comm;
    std::vector<GuardianKeys> keys;
    for (const auto& gi : guardians) {
      GuardianKeys k;
      k.id = "guardian" + std::to_string(gi.x);
      k.x = gi.x;
      k.coeffs = gi.coeffs;
      k.commitments = gi.comm;
      comm[k.id] = gi.comm;
      keys.push_back(k);
    }
    for (auto& gi : keys)
      for (const auto& gl : keys)
        if (gl.id != gi.id) gi.sharesFrom[gl.id] = polyEval(G, gl.coeffs, gi.x);
    GpuDecryptingTrustee t1(keys[0], comm), t2(keys[1], comm);
    const auto d = t1.directDecrypt(G, texts, qbar, &nonces);
    EXPECT(d.size() == direct.size(), "direct count");
    for (size_t i = 0; i < d.size(); ++i) {
      EXPECT(d[i].partialDecryption == ElementModP::from_hex(direct[i][1]), "direct M #" << i);
      EXPECT(d[i].proof.c == ElementModQ::from_hex(direct[i][2]) && d[i].proof.v == ElementModQ::from_hex(direct[i][3]),
             "direct proof #" << i);
    }
    const auto c = t2.compensatedDecrypt(G, "guardian3", texts, qbar, &nonces);
    EXPECT(c.size() == comp.size(), "compensated count");
    for (size_t i = 0; i < c.size(); ++i) {
      EXPECT(c[i].partialDecryption == ElementModP::from_hex(comp[i][1]), "compensated M #" << i);
      EXPECT(c[i].proof.c == ElementModQ::from_hex(comp[i][2]) && c[i].proof.v == ElementModQ::from_hex(comp[i][3]),
             "compensated proof #" << i);
      EXPECT(c[i].recoveredPublicKeyShare == ElementModP::from_hex(comp[i][4]), "recovery key #" << i);
    }
    // the proxy contract: an unknown missing guardian -> empty list, not a crash
    const auto bad = TrusteeCallOrEmpty([&] { return t2.compensatedDecrypt(G, "nobody", texts, qbar, &nonces); });
    EXPECT(bad.empty(), "failed trustee call yields an empty list");
  }
  // config-4 shape end to end: 5 guardians, quorum 3, guardians 4 and 5 missing
  {
    auto [gs, K] = keyCeremony(G, 5, 3, 424242);
    std::map<std::string, std::vector<ElementModP>> comm;
    for (const auto& g : gs) comm[g.id] = g.commitments;
    std::vector<std::unique_ptr<GpuDecryptingTrustee>> avail;
    std::vector<DecryptingTrusteeIF*> ptrs;
    for (int i = 0; i < 3; ++i) {
      avail.emplace_back(new GpuDecryptingTrustee(gs[i], comm, 1000 + i));
      ptrs.push_back(avail.back().get());
    }
    std::mt19937_64 rng(99);
    const size_t n = 20;
    std::vector<int64_t> counts(n);
    std::vector<ElementModQ> R(n), m(n);
    for (size_t i = 0; i < n; ++i) {
      counts[i] = (int64_t)(rng() % 1001);
      R[i] = G.randomElementModQ(rng);
      m[i] = G.uIntToElementModQ((uint64_t)counts[i]);
    }
    const auto pads = G.gPowPBatch(R);
    const auto gm = G.gPowPBatch(m);
    const auto KR = G.powPBatch(std::vector<ElementModP>(n, K), R);
    const auto datas = G.multPBatch(gm, KR);
    std::vector<ElGamalCiphertext> tally(n);
    for (size_t i = 0; i < n; ++i) tally[i] = {pads[i], datas[i]};
    const ElementModQ qb = G.randomElementModQ(rng);
    Decryption dec(G, qb, ptrs, {"guardian4", "guardian5"});
    const auto got = dec.decrypt(tally, 1000);
    for (size_t i = 0; i < n; ++i) EXPECT(got[i] && *got[i] == counts[i], "decrypted count #" << i);
    // the published decryption record verifies; tampering fails exactly the covering check
    const DecryptionRecord rec = dec.decryptRecord(tally, 1000);
    std::map<std::string, ElementModP> pks;
    for (const auto& g : gs) pks[g.id] = g.publicKey();
    EXPECT(verifyDecryptionRecord(G, qb, rec, pks, comm).all(), "decryption record verifies");
    DecryptionRecord bad = rec;
    bad.counts[3] = *bad.counts[3] + 1;
    auto chk = verifyDecryptionRecord(G, qb, bad, pks, comm);
    EXPECT(!chk.tally && chk.directProofs && chk.compensatedProofs && chk.recoveryKeys, "tampered count flagged");
    bad = rec;
    auto& rk = bad.compensated["guardian4"]["guardian2"][5].recoveredPublicKeyShare;
    rk = G.multPBatch({rk}, {G.gPowP(G.uIntToElementModQ(1))})[0];
    chk = verifyDecryptionRecord(G, qb, bad, pks, comm);
    EXPECT(!chk.recoveryKeys && !chk.compensatedProofs && chk.tally && chk.directProofs, "tampered recovery key flagged");
    // malformed records: flagged, never an exception or an out-of-bounds read
    bad = rec;
    bad.direct.begin()->second.pop_back();
    chk = verifyDecryptionRecord(G, qb, bad, pks, comm);
    EXPECT(!chk.directProofs && !chk.tally, "short direct share list flagged");
    bad = rec;
    bad.compensated.begin()->second.begin()->second.pop_back();
    chk = verifyDecryptionRecord(G, qb, bad, pks, comm);
    EXPECT(!chk.compensatedProofs && !chk.tally, "short compensated share list flagged");
    bad = rec;
    bad.direct["nobody"] = rec.direct.begin()->second;
    chk = verifyDecryptionRecord(G, qb, bad, pks, comm);
    EXPECT(!chk.directProofs && !chk.quorum, "unknown guardian flagged");
    bad = rec;
    bad.compensated["nobody"] = rec.compensated.begin()->second;
    chk = verifyDecryptionRecord(G, qb, bad, pks, comm);
    EXPECT(!chk.recoveryKeys && !chk.compensatedProofs, "unknown missing guardian flagged");
    bad = rec;
    bad.counts[0] = -1;
    chk = verifyDecryptionRecord(G, qb, bad, pks, comm);
    EXPECT(!chk.tally && chk.directProofs, "negative count flagged");
    // dLogG above the bound -> not found
    EXPECT(!G.dLogG(G.gPowP(G.uIntToElementModQ(1500)), 1000).has_value(), "dLogG beyond maxResult");
  }
  {  // device memory and the tally exchange: 3 local parts folded, then RCCL at world size 1
    std::mt19937_64 rng(77);
    const size_t n = 9, nparts = 3;
    std::vector<ElementModP> xs;
    for (size_t i = 0; i < n * nparts; ++i) xs.push_back(G.gPowP(G.randomElementModQ(rng)));
    const auto raw = GroupContext::packP(xs);
    DeviceBuffer d(G, raw.size());
    d.upload(raw.data(), raw.size());
    std::vector<uint8_t> back(raw.size());
    d.download(back.data(), back.size());
    EXPECT(back == raw, "device buffer round trip");
    auto folded = TallyExchange::foldTally(G, d, nparts, n);
    for (size_t k = 0; k < n; ++k)
      EXPECT(folded[k] == G.multP({xs[k], xs[n + k], xs[2 * n + k]}), "local fold of 3 parts, element " << k);
    const auto id = TallyExchange::uniqueId();
    TallyExchange x(G, id.data(), 1, 0);
    EXPECT(x.allValid(true) && !x.allValid(false), "RCCL verdict all-reduce at world 1");
    folded = x.fold(d, nparts, n);
    for (size_t k = 0; k < n; ++k) EXPECT(folded[k] == G.multP({xs[k], xs[n + k], xs[2 * n + k]}), "RCCL fold " << k);
    std::vector<uint8_t> flags(100, 1);
    DeviceBuffer df(G, flags.size());
    df.upload(flags.data(), flags.size());
    EXPECT(df.allNonzero(flags.size()), "flags all set");
    flags[99] = 0;
    df.upload(flags.data(), flags.size());
    EXPECT(!df.allNonzero(flags.size()) && df.allNonzero(99), "a zero flag found");
  }
  G.setProofFormat(EG_RESPONSE_MINUS, EG_PREIMAGE_MESSAGE_FIRST);
  std::cout << "OK " << g_checks << std::endl;
  return 0;
}

int main(int argc, char** argv) {
  try {
    if (argc >= 2 && std::string(argv[1]) == "cpu") return run_cpu();
    if (argc >= 3 && std::string(argv[1]) == "gpu")
      return run_gpu(argv[2], argc >= 4 && std::string(argv[3]) == "V2" ? ProductionMode::Mode4096_V2
                                                                          : ProductionMode::Mode4096);
  } catch (const std::exception& e) {
    std::cerr << "exception: " << e.what() << std::endl;
    return 1;
  }
  std::cerr << "usage: host_parity cpu | gpu <vectors.txt> [V2]" << std::endl;
  return 2;
}
