// electionguard.hpp -- C++17 host mirror of the reference's group layer and trustee
// plugin, above the C ABI of libeg_hip.so (include/eg_hip.h).  Header-only.
//
// The reference is JVM code (JDK 17 + Kotlin dependency electionguard-kotlin-
// multiplatform-jvm:1.0-SNAPSHOT, build.gradle.kts:55); no JDK exists in this image, so
// this is the compiled-language host side a C++ caller (or a JNI shim)
// uses.  Names, argument meaning and error behaviour follow the reference's interfaces:
//
//   GroupContext / ElementModP / ElementModQ  <- KUtils.productionGroup()
//       (src/main/java/electionguard/util/KUtils.java:10-12); elements cross the boundary
//       as fixed-width big-endian bytes (common.proto:6-16), imported unchecked like
//       ConvertCommonProto.importElementModP (ConvertCommonProto.java:41-57) and exported
//       with byteArray() (ConvertCommonProto.java:111-121).
//   DecryptingTrusteeIF                         <- RemoteDecryptingTrusteeProxy.java:30-122
//       id() / xCoordinate() / electionPublicKey() (:33-46), directDecrypt (:48-53),
//       compensatedDecrypt (:84-90); results in text order; a failed remote call yields an
//       EMPTY list (:64-66, :103-105) -- GpuDecryptingTrustee throws, RemoteProxy-style
//       callers catch and return {} (see TrusteeCallOrEmpty).
//   Decryption::decrypt                         <- RunRemoteDecryptor.java:261-262
//   Verifier / batchEncryption / accumulate     <- RunRemoteWorkflowTest.java:140-141,151,179-182
//
// Errors: a non-zero status from the C ABI throws ArithmeticException(eg_last_error()),
// the JNI mapping INTEGRATION.md §2 describes.  Every mod-p operation runs on the GPU (the
// per-element ones deferred and merged into library jobs, see Deferred); 256-bit mod-q scalar
// arithmetic (a few operations per proof / Lagrange coefficient, and the exponent algebra of
// deferred elements) is host arithmetic in U256 below.
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "eg_constants.hpp"
#include "eg_hip.h"

namespace electionguard {

class ArithmeticException : public std::runtime_error {
 public:
  explicit ArithmeticException(const std::string& what) : std::runtime_error(what) {}
};

inline void check(int rc, const char* fn) {
  if (rc != EG_OK) throw ArithmeticException(std::string(fn) + ": " + eg_last_error());
}

// ---------------------------------------------------------------- hex helpers
inline int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  throw std::invalid_argument("bad hex digit");
}

// big-endian hex (any length <= 2n digits, left-padded) -> n bytes
inline void hex_to_be(const std::string& h, uint8_t* out, size_t n) {
  if (h.size() > 2 * n) throw std::invalid_argument("hex value too wide");
  std::memset(out, 0, n);
  size_t off = 2 * n - h.size();
  for (size_t i = 0; i < h.size(); ++i) {
    const size_t d = off + i;
    out[d / 2] |= (uint8_t)(hexval(h[i]) << ((d & 1) ? 0 : 4));
  }
}

inline std::string be_to_hex(const uint8_t* b, size_t n) {
  static const char* k = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = k[b[i] >> 4];
    s[2 * i + 1] = k[b[i] & 15];
  }
  return s;
}

// ---------------------------------------------------------------- U256 (mod-q scalars)
// Little-endian 4 x 64-bit limbs.  Generic modular arithmetic for any modulus < 2^256
// (EG q = 2^256 - 189); speed is irrelevant here (a handful of ops per proof).
struct U256 {
  std::array<uint64_t, 4> w{0, 0, 0, 0};

  static U256 from_u64(uint64_t x) {
    U256 r;
    r.w[0] = x;
    return r;
  }
  static U256 from_be(const uint8_t* b) {
    U256 r;
    for (int i = 0; i < 32; ++i) r.w[3 - i / 8] = (r.w[3 - i / 8] << 8) | b[i];
    return r;
  }
  static U256 from_hex(const std::string& h) {
    uint8_t b[32];
    hex_to_be(h, b, 32);
    return from_be(b);
  }
  void to_be(uint8_t* b) const {
    for (int i = 0; i < 32; ++i) b[i] = (uint8_t)(w[3 - i / 8] >> (8 * (7 - i % 8)));
  }
  std::string hex() const {
    uint8_t b[32];
    to_be(b);
    return be_to_hex(b, 32);
  }
  bool is_zero() const { return (w[0] | w[1] | w[2] | w[3]) == 0; }
  bool bit(int i) const { return (w[i >> 6] >> (i & 63)) & 1; }
  friend bool operator==(const U256& a, const U256& b) { return a.w == b.w; }
  friend bool operator!=(const U256& a, const U256& b) { return !(a == b); }
  friend bool operator<(const U256& a, const U256& b) {
    for (int i = 3; i >= 0; --i)
      if (a.w[i] != b.w[i]) return a.w[i] < b.w[i];
    return false;
  }
  // a + b, returns carry
  static uint64_t add(U256& r, const U256& a, const U256& b) {
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; ++i) {
      c += (unsigned __int128)a.w[i] + b.w[i];
      r.w[i] = (uint64_t)c;
      c >>= 64;
    }
    return (uint64_t)c;
  }
  // a - b, returns borrow
  static uint64_t sub(U256& r, const U256& a, const U256& b) {
    uint64_t br = 0;
    for (int i = 0; i < 4; ++i) {
      const uint64_t ai = a.w[i], bi = b.w[i];
      const uint64_t d = ai - bi - br;
      br = (ai < bi) || (ai == bi && br) ? 1 : 0;
      r.w[i] = d;
    }
    return br;
  }
};

// Modular arithmetic over a fixed modulus m < 2^256 (values kept in [0, m)).
struct ModQ {
  U256 m;
  U256 reduce_small(U256 a) const {  // a < 2^256 -> a mod m by repeated subtraction of m * 2^k
    while (!(a < m)) {
      U256 t = m;
      int sh = 0;
      while (!(t.w[3] >> 63)) {  // largest m*2^k <= a
        U256 t2;
        for (int i = 3; i > 0; --i) t2.w[i] = (t.w[i] << 1) | (t.w[i - 1] >> 63);
        t2.w[0] = t.w[0] << 1;
        if (a < t2) break;
        t = t2;
        ++sh;
      }
      U256::sub(a, a, t);
    }
    return a;
  }
  U256 add(const U256& a, const U256& b) const {
    U256 r;
    const uint64_t c = U256::add(r, a, b);
    if (c || !(r < m)) U256::sub(r, r, m);
    return r;
  }
  U256 sub(const U256& a, const U256& b) const {
    U256 r;
    if (U256::sub(r, a, b)) U256::add(r, r, m);
    return r;
  }
  U256 neg(const U256& a) const { return a.is_zero() ? a : sub(m, a); }
  U256 mul(const U256& a, const U256& b) const {
    // 512-bit product, then bit-serial reduction r = (2r + bit) mod m from the top
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; ++i) {
      unsigned __int128 c = 0;
      for (int j = 0; j < 4; ++j) {
        c += (unsigned __int128)a.w[i] * b.w[j] + t[i + j];
        t[i + j] = (uint64_t)c;
        c >>= 64;
      }
      t[i + 4] = (uint64_t)c;
    }
    U256 r;
    for (int k = 511; k >= 0; --k) {
      const uint64_t top = r.w[3] >> 63;
      for (int i = 3; i > 0; --i) r.w[i] = (r.w[i] << 1) | (r.w[i - 1] >> 63);
      r.w[0] = (r.w[0] << 1) | ((t[k >> 6] >> (k & 63)) & 1);
      if (top || !(r < m)) U256::sub(r, r, m);
    }
    return r;
  }
  U256 pow(U256 b, const U256& e) const {
    U256 r = reduce_small(U256::from_u64(1));
    b = reduce_small(b);
    for (int i = 255; i >= 0; --i) {
      r = mul(r, r);
      if (e.bit(i)) r = mul(r, b);
    }
    return r;
  }
  U256 inv(const U256& a) const {  // m prime (q): a^(m-2)
    if (reduce_small(a).is_zero()) throw ArithmeticException("multInv of 0 mod q");
    U256 e;
    U256::sub(e, m, U256::from_u64(2));
    return pow(a, e);
  }
};

// ---------------------------------------------------------------- elements
class GroupContext;

// Upstream ProductionMode (KUtils.java:5,11): Mode4096 = EG 1.0 (the reference's group);
// Mode4096_V2 = the EG 2.0 group, a named option (eg_constants.hpp).
enum class ProductionMode { Mode4096 = 0, Mode4096_V2 = 1 };

// A fixed-base radix table on the device (eg_fixed_base_create): g's (the context's) or one made by
// GroupContext::acceleratePow for an element upstream accelerates (the election key K,
// ElementModP.acceleratePow()).  orderQ: base^q == 1 was checked, so exponents of this base may be
// added, multiplied and negated mod q (the deferred algebra below).
class FixedBase {
 public:
  FixedBase(eg_fixed_base* fb, bool owned, bool orderQ, const uint8_t* base_be) : fb_(fb), owned_(owned), orderQ_(orderQ) {
    std::memcpy(base_.data(), base_be, EG_P_BYTES);
  }
  FixedBase(const FixedBase&) = delete;
  FixedBase& operator=(const FixedBase&) = delete;
  ~FixedBase() {
    if (owned_ && fb_) eg_fixed_base_destroy(fb_);
  }
  eg_fixed_base* handle() const { return fb_; }
  bool orderQ() const { return orderQ_; }
  const uint8_t* base() const { return base_.data(); }

 private:
  eg_fixed_base* fb_;
  bool owned_, orderQ_;
  std::array<uint8_t, EG_P_BYTES> base_{};
};
using FixedBasePtr = std::shared_ptr<const FixedBase>;

// The deferred value of per-element operations.  Upstream calls the group one element at a time from
// 11 threads (ElementModP.powP / times, GroupContext.gPowP, the accelerated K.powP:
// RunRemoteWorkflowTest.java:140-141,179-181), and each call's result is usually consumed a few calls
// later (by a product, then a hash).  So an operation does not run when it is called: it returns an
// element holding an EXPRESSION
//     (b_1 * ... * b_k)^e * F0^f0 * F1^f1   (b_i resolved values, F_t registered fixed bases)
// and products / powers of expressions are combined on the host where that is exact:
//   * x.times(y) merges the fixed-base terms (a base that appears in both adds its exponents mod q,
//     allowed when it has order q) and the variable parts (two products without an exponent, or two
//     with the same exponent, concatenate their bases): g^v * alpha^c is ONE job;
//   * x.powP(e) on a pure fixed-base expression of order-q bases multiplies its exponents by e mod q:
//     (g^R)^c = g^(R c); on a product without an exponent it sets the exponent: (prod alpha)^c;
//   * otherwise the operand is resolved and the result starts a new expression.
// The first time a value is needed (byteArray, ==, a hash, isValidResidue) every expression this thread
// created and has not merged into another is submitted (eg_mexp_submit: one job each, all in the
// library's next coalesced batch), and the thread waits for the one it needs: one GPU round trip per
// point where upstream's code actually looks at a value, instead of one per call.  Products of more
// than 16 values (a tally accumulator) are reduced with eg_prod_reduce when resolved; pure products
// (no exponent, no fixed base) are not submitted by other values' flushes, so an accumulator grows
// on the host until it is read.  Results are the same integers as eager evaluation.
struct Deferred {
  struct Buf {  // the bases of product expressions; appended in place while the tail is unshared
    std::mutex mu;
    std::vector<std::array<uint8_t, EG_P_BYTES>> v;
  };
  // the expression (immutable after construction)
  std::shared_ptr<Buf> buf;
  size_t nb = 0;  // bases buf->v[0, nb)
  bool hasExp = false;
  U256 exp;
  FixedBasePtr fb[2];
  U256 fe[2];
  int nfb = 0;
  const GroupContext* group = nullptr;
  // evaluation
  std::mutex mu;
  int state = 0;          // 0 expression, 1 submitted, 2 value in out, 3 failed (err)
  bool consumed = false;  // merged into a newer expression: other values' flushes skip it
  eg_ticket* ticket = nullptr;
  std::array<uint8_t, EG_P_BYTES> out{};
  std::string err;
  bool pureProduct() const { return !hasExp && nfb == 0; }
  ~Deferred() {
    if (ticket) eg_ticket_wait(ticket);  // the library may still write `out`
  }
};

// ElementModP: 512-byte big-endian value (common.proto:6-10), unchecked on import; or a deferred one.
struct ElementModP {
  mutable std::array<uint8_t, EG_P_BYTES> be{};
  const GroupContext* group = nullptr;
  // be holds the value.  Written once, under the expression's lock, with release order; a thread that
  // sees it set (acquire) sees the bytes, so one element may be read from several threads at once
  mutable std::atomic<bool> have{true};
  std::shared_ptr<Deferred> def;           // the expression this value came from (kept for the algebra)
  FixedBasePtr accel;                      // a fixed-base table of this value (acceleratePow; g)

  ElementModP() = default;
  ElementModP(const ElementModP& o) : group(o.group), def(o.def), accel(o.accel) { copyValue(o); }
  ElementModP(ElementModP&& o) noexcept : group(o.group), def(std::move(o.def)), accel(std::move(o.accel)) {
    copyValue(o);
  }
  ElementModP& operator=(const ElementModP& o) {
    if (this != &o) {
      group = o.group;
      def = o.def;
      accel = o.accel;
      copyValue(o);
    }
    return *this;
  }
  ElementModP& operator=(ElementModP&& o) noexcept {
    if (this != &o) {
      group = o.group;
      def = std::move(o.def);
      accel = std::move(o.accel);
      copyValue(o);
    }
    return *this;
  }
  ElementModP(const uint8_t* b, const GroupContext* g) : group(g) { std::memcpy(be.data(), b, EG_P_BYTES); }
  static ElementModP from_hex(const std::string& h, const GroupContext* g = nullptr) {
    ElementModP e;
    e.group = g;
    hex_to_be(h, e.be.data(), EG_P_BYTES);
    return e;
  }
  static ElementModP from_u64(uint64_t x, const GroupContext* g = nullptr) {
    ElementModP e;
    e.group = g;
    for (int i = 0; i < 8; ++i) e.be[EG_P_BYTES - 1 - i] = (uint8_t)(x >> (8 * i));
    return e;
  }
  // the value (resolving a deferred one: see Deferred)
  const uint8_t* byteArray() const {
    if (!have.load(std::memory_order_acquire)) resolve();
    return be.data();
  }
  bool pending() const { return !have.load(std::memory_order_acquire); }
  std::string hex() const { return be_to_hex(byteArray(), EG_P_BYTES); }
  friend bool operator==(const ElementModP& a, const ElementModP& b) {
    return std::memcmp(a.byteArray(), b.byteArray(), EG_P_BYTES) == 0;
  }
  friend bool operator!=(const ElementModP& a, const ElementModP& b) { return !(a == b); }

  // upstream per-element API (deferred: see Deferred)
  inline ElementModP powP(const struct ElementModQ& e) const;
  inline ElementModP times(const ElementModP& o) const;
  inline ElementModP multInv() const;
  inline ElementModP div(const ElementModP& o) const;
  inline bool isValidResidue() const;
  inline ElementModP acceleratePow() const;
  inline void resolve() const;

 private:
  void copyValue(const ElementModP& o) {
    const bool h = o.have.load(std::memory_order_acquire);
    if (h) be = o.be;
    have.store(h, std::memory_order_release);
  }
};

// ElementModQ: 256-bit scalar (common.proto:12-16).
struct ElementModQ {
  U256 v;
  ElementModQ() = default;
  explicit ElementModQ(const U256& x) : v(x) {}
  static ElementModQ from_hex(const std::string& h) { return ElementModQ(U256::from_hex(h)); }
  static ElementModQ from_be(const uint8_t* b) { return ElementModQ(U256::from_be(b)); }
  std::array<uint8_t, EG_Q_BYTES> byteArray() const {
    std::array<uint8_t, EG_Q_BYTES> b;
    v.to_be(b.data());
    return b;
  }
  std::string hex() const { return v.hex(); }
  friend bool operator==(const ElementModQ& a, const ElementModQ& b) { return a.v == b.v; }
  friend bool operator!=(const ElementModQ& a, const ElementModQ& b) { return !(a == b); }
};

struct ElGamalCiphertext {  // ConvertCommonProto.java:59-68,123-128
  ElementModP pad, data;
};
struct GenericChaumPedersenProof {  // compact (c, v), common.proto:23-28
  ElementModQ c, v;
};
struct DirectDecryptionAndProof {  // decrypting_trustee_rpc.proto:25-28
  ElementModP partialDecryption;
  GenericChaumPedersenProof proof;
};
struct CompensatedDecryptionAndProof {  // decrypting_trustee_rpc.proto:41-45
  ElementModP partialDecryption;
  GenericChaumPedersenProof proof;
  ElementModP recoveredPublicKeyShare;
};

// ---------------------------------------------------------------- GroupContext
namespace detail {
// An expression as the deferred algebra manipulates it (Deferred's fields, by value).
struct Form {
  std::shared_ptr<Deferred::Buf> buf;
  size_t nb = 0;
  bool hasExp = false;
  U256 exp;
  FixedBasePtr fb[2];
  U256 fe[2];
  int nfb = 0;
};
// the expressions this thread created and has not submitted (Deferred)
inline std::vector<std::weak_ptr<Deferred>>& pendingQueue() {
  thread_local std::vector<std::weak_ptr<Deferred>> q;
  return q;
}
constexpr size_t kMaxJobBases = 16;  // eg_mexp_submit's limit; longer products go through eg_prod_reduce
}  // namespace detail

class GroupContext {
 public:
  GroupContext(const ElementModP& p, const ElementModQ& q, const ElementModP& g, int device = 0)
      : p_(p), g_(g), q_(q), modq_{q.v}, device_(device) {
    const auto qb = q.byteArray();
    check(eg_ctx_create(p.byteArray(), qb.data(), g.byteArray(), device, &ctx_), "eg_ctx_create");
    p_.group = this;
    g_.group = this;
    // g has order q (checked once here), so g-exponents combine mod q; the per-element calls use a
    // 16-bit table of g of their own (gTable), built on first use
    gOrderQ_ = hasOrderQ(g_);
  }
  ~GroupContext() {
    accel_.clear();  // the tables go before the context
    gfb_.reset();
    if (ctx_) eg_ctx_destroy(ctx_);
  }
  GroupContext(const GroupContext&) = delete;
  GroupContext& operator=(const GroupContext&) = delete;

  // KUtils.productionGroup() (KUtils.java:10-12): Mode4096 is the EG 1.0 4096-bit group of the
  // reference's upstream; Mode4096_V2 the EG 2.0 group.  One context per (mode, device).
  static GroupContext& productionGroup(int device = 0, ProductionMode mode = ProductionMode::Mode4096) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::unique_ptr<GroupContext>> groups;
    std::lock_guard<std::mutex> lk(mu);
    auto& slot = groups[{(int)mode, device}];
    if (!slot) {
      const bool v2 = mode == ProductionMode::Mode4096_V2;
      slot.reset(new GroupContext(ElementModP::from_hex(v2 ? constants::kP_HEX_V2 : constants::kP_HEX),
                                  ElementModQ::from_hex(v2 ? constants::kQ_HEX_V2 : constants::kQ_HEX),
                                  ElementModP::from_hex(v2 ? constants::kG_HEX_V2 : constants::kG_HEX), device));
    }
    return *slot;
  }

  eg_ctx* handle() const { return ctx_; }
  int device() const { return device_; }
  // Fiat-Shamir pre-image hex form (EG_HASH_FIXED_WIDTH default / EG_HASH_MINIMAL): upstream's
  // is unpinned, so it is switchable per context (include/eg_hip.h).
  void setHashFormat(int format) const { check(eg_ctx_set_hash_format(ctx_, format), "eg_ctx_set_hash_format"); }
  // response convention (EG_RESPONSE_MINUS / _PLUS) and challenge pre-image order (EG_PREIMAGE_*)
  void setProofFormat(int response, int preimage) const {
    check(eg_ctx_set_proof_format(ctx_, response, preimage), "eg_ctx_set_proof_format");
  }
  const ElementModP& P() const { return p_; }
  const ElementModP& G() const { return g_; }
  const ElementModQ& Q() const { return q_; }
  const ModQ& modq() const { return modq_; }

  ElementModP binaryToElementModP(const uint8_t* b) const { return ElementModP(b, this); }
  ElementModQ binaryToElementModQ(const uint8_t* b) const { return ElementModQ::from_be(b); }
  ElementModQ uIntToElementModQ(uint64_t x) const { return ElementModQ(modq_.reduce_small(U256::from_u64(x))); }
  ElementModP one() const { return ElementModP::from_u64(1, this); }

  // mod-q scalar ops (ElementModQ.plus/minus/times/unaryMinus upstream)
  ElementModQ addQ(const ElementModQ& a, const ElementModQ& b) const { return ElementModQ(modq_.add(a.v, b.v)); }
  ElementModQ subQ(const ElementModQ& a, const ElementModQ& b) const { return ElementModQ(modq_.sub(a.v, b.v)); }
  ElementModQ mulQ(const ElementModQ& a, const ElementModQ& b) const { return ElementModQ(modq_.mul(a.v, b.v)); }
  ElementModQ negQ(const ElementModQ& a) const { return ElementModQ(modq_.neg(a.v)); }
  ElementModQ invQ(const ElementModQ& a) const { return ElementModQ(modq_.inv(a.v)); }
  ElementModQ powQ(const ElementModQ& a, const ElementModQ& e) const { return ElementModQ(modq_.pow(a.v, e.v)); }

  // ---- batched group ops: the drop-in entry points ----
  std::vector<ElementModP> powPBatch(const std::vector<ElementModP>& bases, const std::vector<ElementModQ>& exps) const {
    if (bases.size() != exps.size()) throw std::invalid_argument("powPBatch: bases/exps length mismatch");
    const size_t n = bases.size();
    std::vector<uint8_t> B = packP(bases), E = packQ(exps), O(n * EG_P_BYTES);
    if (n) check(eg_powp_batch(ctx_, B.data(), E.data(), O.data(), n), "eg_powp_batch");
    return unpackP(O, n);
  }
  std::vector<ElementModP> gPowPBatch(const std::vector<ElementModQ>& exps) const {
    const size_t n = exps.size();
    std::vector<uint8_t> E = packQ(exps), O(n * EG_P_BYTES);
    if (n) check(eg_fb_pow_batch(eg_ctx_g_table(ctx_), E.data(), O.data(), n), "eg_fb_pow_batch");
    return unpackP(O, n);
  }
  std::vector<ElementModP> multPBatch(const std::vector<ElementModP>& a, const std::vector<ElementModP>& b) const {
    if (a.size() != b.size()) throw std::invalid_argument("multPBatch: length mismatch");
    const size_t n = a.size();
    std::vector<uint8_t> A = packP(a), Bv = packP(b), O(n * EG_P_BYTES);
    if (n) check(eg_multp_batch(ctx_, A.data(), Bv.data(), O.data(), n), "eg_multp_batch");
    return unpackP(O, n);
  }
  std::vector<ElementModP> multInvBatch(const std::vector<ElementModP>& a) const {
    const size_t n = a.size();
    std::vector<uint8_t> A = packP(a), O(n * EG_P_BYTES);
    if (n) check(eg_multinv_batch(ctx_, A.data(), O.data(), n), "eg_multinv_batch");
    return unpackP(O, n);
  }
  // out[g] = prod_k elems[g*len + k]  (Iterable<ElementModP>.multP(), the tally)
  std::vector<ElementModP> prodPGroups(const std::vector<ElementModP>& elems, size_t groups, size_t len) const {
    if (elems.size() != groups * len) throw std::invalid_argument("prodPGroups: need groups*len elements");
    std::vector<uint8_t> A = packP(elems), O(groups * EG_P_BYTES);
    if (groups) check(eg_prod_reduce(ctx_, A.data(), groups, len, O.data()), "eg_prod_reduce");
    return unpackP(O, groups);
  }

  // ---- per-element API: the upstream call pattern (one element per call, from many threads,
  // RunRemoteWorkflowTest.java:140-141,179-181).  Deferred (see Deferred): each call returns at
  // once; the values are computed as ONE library job each (eg_mexp_submit, coalesced with the other
  // threads' jobs) when the thread first needs one of them ----
  ElementModP gPowP(const ElementModQ& e) const {
    detail::Form f;
    f.nfb = 1;
    f.fb[0] = gTable();
    f.fe[0] = e.v;
    return make(f);
  }
  // The fixed-base table of g the per-element calls use: kElementWindow bits (16: 16 windows of 65,536
  // entries, 671 MB), so g^e costs 15 multiplies (split over 4 waves by the library) instead of the
  // 31 of the context's 8-bit table; built once, on first use.
  FixedBasePtr gTable() const {
    std::call_once(g_once_, [&] {
      eg_fixed_base* fb = nullptr;
      check(eg_fixed_base_create(ctx_, g_.be.data(), kElementWindow, &fb), "eg_fixed_base_create");
      gfb_ = std::make_shared<FixedBase>(fb, true, gOrderQ_, g_.be.data());
    });
    return gfb_;
  }
  static constexpr int kElementWindow = 16;
  // b^e.  An accelerated b (acceleratePow, g) runs on its fixed-base table; a pure fixed-base
  // expression of order-q bases scales its exponents; a product without an exponent takes e.
  ElementModP powP(const ElementModP& b, const ElementModQ& e) const {
    bool expr = false;
    detail::Form f = formOf(b, &expr);
    if (f.nb == 0 && f.nfb > 0) {
      if (f.nfb == 1 && f.fe[0] == U256::from_u64(1)) {  // F^1 -> F^e (any order)
        f.fe[0] = e.v;
        return consumeAndMake(b, expr, f);
      }
      if (allOrderQ(f)) {
        const U256 ee = modq_.reduce_small(e.v);
        for (int t = 0; t < f.nfb; ++t) f.fe[t] = modq_.mul(modq_.reduce_small(f.fe[t]), ee);
        return consumeAndMake(b, expr, f);
      }
    } else if (f.nb > 0 && f.nfb == 0 && !f.hasExp) {
      f.hasExp = true;
      f.exp = e.v;
      return consumeAndMake(b, expr, f);
    }
    detail::Form v = valueForm(b);
    v.hasExp = true;
    v.exp = e.v;
    return make(v);
  }
  // a * b (upstream ElementModP.times): merged into one expression where that is exact, else a
  // product of the two values (one job when read)
  ElementModP multP(const ElementModP& a, const ElementModP& b) const {
    bool ea = false, eb = false;
    const detail::Form fa = formOf(a, &ea), fb = formOf(b, &eb);
    if (auto m = merge(fa, fb)) {
      if (ea) consume(a);
      if (eb) consume(b);
      return make(*m);
    }
    detail::Form p = valueForm(a);
    append(p, valueForm(b));
    return make(p);
  }
  // a^-1: a pure fixed-base expression of order-q bases negates its exponents; else a^(p-2) on the
  // value (eg_multinv_batch, blocking)
  ElementModP multInv(const ElementModP& a) const {
    bool expr = false;
    detail::Form f = formOf(a, &expr);
    if (f.nb == 0 && f.nfb > 0 && allOrderQ(f)) {
      for (int t = 0; t < f.nfb; ++t) f.fe[t] = modq_.neg(modq_.reduce_small(f.fe[t]));
      return consumeAndMake(a, expr, f);
    }
    return multInvBatch({a})[0];
  }
  // upstream ElementModP.isValidResidue(): 0 <= a < p and a^q == 1 (the job joins this thread's
  // pending ones: one round trip resolves them all)
  bool isValidResidue(const ElementModP& a) const {
    const uint8_t* v = a.byteArray();
    if (std::memcmp(v, p_.be.data(), EG_P_BYTES) >= 0) return false;
    ElementModP r = powP(ElementModP(v, this), q_);
    const uint8_t* rv = r.byteArray();
    for (int i = 0; i < EG_P_BYTES - 1; ++i)
      if (rv[i]) return false;
    return rv[EG_P_BYTES - 1] == 1;
  }
  // upstream ElementModP.acceleratePow(): a fixed-base radix table for a's value (window_bits wide,
  // cached by value per context), so a.powP(e) is a fixed-base job; the base's order is checked
  // (a^q == 1) so its exponents may combine mod q
  ElementModP acceleratePow(const ElementModP& a, int windowBits = kElementWindow) const {
    ElementModP out(a.byteArray(), this);
    const std::string key((const char*)out.be.data(), EG_P_BYTES);
    std::lock_guard<std::mutex> lk(accel_mu_);
    auto it = accel_.find(key);
    if (it == accel_.end()) {
      eg_fixed_base* fb = nullptr;
      check(eg_fixed_base_create(ctx_, out.be.data(), windowBits, &fb), "eg_fixed_base_create");
      auto t = std::make_shared<FixedBase>(fb, true, hasOrderQ(out), out.be.data());
      if (accel_.size() >= 8) accel_.erase(accel_.begin());  // a few keys per context
      it = accel_.emplace(key, std::move(t)).first;
    }
    out.accel = it->second;
    return out;
  }
  // off: every per-element call resolves at once (one blocking GPU round trip each; for A/B runs)
  void setDeferred(bool on) const { deferred_ = on; }
  bool deferred() const { return deferred_; }
  // eg_ctx_set_ct_pow: exponentiation on the constant-time schedule (a trustee's secret exponents)
  void setConstantTime(bool on) const { check(eg_ctx_set_ct_pow(ctx_, on ? 1 : 0), "eg_ctx_set_ct_pow"); }
  // batch window of the per-element calls (eg_ctx_set_coalescing)
  void setCoalescing(size_t maxBatch, uint32_t windowUs) const {
    check(eg_ctx_set_coalescing(ctx_, maxBatch, windowUs), "eg_ctx_set_coalescing");
  }

  // Submit every expression this thread created and has not merged or submitted yet (pure products
  // excepted: accumulators stay on the host until read), then wait for x's value.
  void resolve(const ElementModP& x) const {
    if (x.have.load(std::memory_order_acquire)) return;
    flushThread();
    Deferred& d = *x.def;
    std::lock_guard<std::mutex> lk(d.mu);
    if (x.have.load(std::memory_order_acquire)) return;  // another thread resolved this element
    if (d.state == 0) submit(d);
    if (d.state == 1) {
      const int rc = eg_ticket_wait(d.ticket);
      d.ticket = nullptr;
      d.state = rc ? 3 : 2;
      if (rc) d.err = eg_last_error();
    }
    if (d.state == 3) throw ArithmeticException("deferred group operation: " + d.err);
    std::memcpy(x.be.data(), d.out.data(), EG_P_BYTES);
    x.have.store(true, std::memory_order_release);
  }
  // resolve several values with one flush: every one of them (pure products too) is submitted before
  // the first wait, so they share the library's next batch (a hash over them, a tally read out)
  void resolveAll(const std::vector<const ElementModP*>& xs) const {
    flushThread();
    for (const ElementModP* x : xs) {
      if (x->have.load(std::memory_order_acquire)) continue;
      std::lock_guard<std::mutex> lk(x->def->mu);
      if (x->def->state == 0) submit(*x->def);
    }
    for (const ElementModP* x : xs) resolve(*x);
  }
  static void flushThread() {
    auto& q = detail::pendingQueue();
    for (auto& w : q) {
      auto d = w.lock();
      if (!d) continue;
      std::lock_guard<std::mutex> lk(d->mu);
      if (d->state == 0 && !d->consumed && !d->pureProduct()) d->group->submit(*d);
    }
    q.clear();
  }
  ElementModP multP(const std::vector<ElementModP>& xs) const {
    return xs.empty() ? one() : prodPGroups(xs, 1, xs.size())[0];
  }

  // dLogG(T, maxResult) [upstream]: t with g^t = T, 0 <= t <= maxResult, else nullopt.
  // Baby-step giant-step; every exponentiation and product on the GPU.
  std::vector<std::optional<int64_t>> dLogGBatch(const std::vector<ElementModP>& ys, int64_t maxResult) const {
    std::vector<std::optional<int64_t>> out(ys.size());
    if (ys.empty() || maxResult < 0) return out;
    int64_t m = 1;
    while (m * m <= maxResult) ++m;
    std::vector<ElementModQ> be(m), ge(m + 1);
    for (int64_t j = 0; j < m; ++j) be[j] = uIntToElementModQ((uint64_t)j);
    const ElementModQ mq = uIntToElementModQ((uint64_t)m);
    for (int64_t i = 0; i <= m; ++i) ge[i] = negQ(mulQ(mq, uIntToElementModQ((uint64_t)i)));  // g^{-m i}
    const auto baby = gPowPBatch(be), giants = gPowPBatch(ge);
    std::unordered_map<std::string, int64_t> table;
    table.reserve(2 * m);
    for (int64_t j = 0; j < m; ++j)
      table.emplace(std::string((const char*)baby[j].byteArray(), EG_P_BYTES), j);
    std::vector<ElementModP> a, b;
    a.reserve(ys.size() * (m + 1));
    b.reserve(ys.size() * (m + 1));
    for (const auto& y : ys)
      for (int64_t i = 0; i <= m; ++i) {
        a.push_back(y);
        b.push_back(giants[i]);
      }
    const auto prod = multPBatch(a, b);
    for (size_t k = 0; k < ys.size(); ++k)
      for (int64_t i = 0; i <= m; ++i) {
        auto it = table.find(std::string((const char*)prod[k * (m + 1) + i].byteArray(), EG_P_BYTES));
        if (it != table.end()) {
          const int64_t t = i * m + it->second;
          if (t <= maxResult) out[k] = t;
          break;
        }
      }
    return out;
  }
  std::optional<int64_t> dLogG(const ElementModP& y, int64_t maxResult) const { return dLogGBatch({y}, maxResult)[0]; }

  ElementModQ randomElementModQ(std::mt19937_64& rng, bool nonzero = true) const {
    for (;;) {
      U256 x;
      for (auto& w : x.w) w = rng();
      if (x < q_.v && (!nonzero || !x.is_zero())) return ElementModQ(x);
    }
  }

  static std::vector<uint8_t> packP(const std::vector<ElementModP>& v) {
    std::vector<uint8_t> out(v.size() * EG_P_BYTES);
    for (size_t i = 0; i < v.size(); ++i) std::memcpy(&out[i * EG_P_BYTES], v[i].byteArray(), EG_P_BYTES);
    return out;
  }
  static std::vector<uint8_t> packQ(const std::vector<ElementModQ>& v) {
    std::vector<uint8_t> out(v.size() * EG_Q_BYTES);
    for (size_t i = 0; i < v.size(); ++i) v[i].v.to_be(&out[i * EG_Q_BYTES]);
    return out;
  }
  std::vector<ElementModP> unpackP(const std::vector<uint8_t>& b, size_t n) const {
    std::vector<ElementModP> out(n);
    for (size_t i = 0; i < n; ++i) out[i] = ElementModP(&b[i * EG_P_BYTES], this);
    return out;
  }

 private:
  // ---- the deferred algebra (see Deferred) ----
  bool hasOrderQ(const ElementModP& x) const {
    const auto r = powPBatch({x}, {q_});
    const uint8_t* v = r[0].byteArray();
    for (int i = 0; i < EG_P_BYTES - 1; ++i)
      if (v[i]) return false;
    return v[EG_P_BYTES - 1] == 1;
  }
  static bool allOrderQ(const detail::Form& f) {
    for (int t = 0; t < f.nfb; ++t)
      if (!f.fb[t]->orderQ()) return false;
    return true;
  }
  detail::Form valueForm(const ElementModP& x) const {
    detail::Form f;
    f.buf = std::make_shared<Deferred::Buf>();
    f.buf->v.emplace_back();
    std::memcpy(f.buf->v[0].data(), x.byteArray(), EG_P_BYTES);
    f.nb = 1;
    return f;
  }
  // x as an expression: an accelerated value (and g) is its table to the power 1; a deferred one its
  // expression (a resolved one with a variable part: its value, so the work is not redone)
  detail::Form formOf(const ElementModP& x, bool* expr) const {
    *expr = false;
    const bool is_g = !x.accel && !x.def && x.have.load(std::memory_order_acquire) && x.be == g_.be;
    if (x.accel || is_g) {
      detail::Form f;
      f.nfb = 1;
      f.fb[0] = is_g ? gTable() : x.accel;
      f.fe[0] = U256::from_u64(1);
      return f;
    }
    if (x.def && (!x.have.load(std::memory_order_acquire) || x.def->nb == 0)) {
      const Deferred& d = *x.def;
      detail::Form f;
      f.buf = d.buf;
      f.nb = d.nb;
      f.hasExp = d.hasExp;
      f.exp = d.exp;
      f.nfb = d.nfb;
      for (int t = 0; t < d.nfb; ++t) {
        f.fb[t] = d.fb[t];
        f.fe[t] = d.fe[t];
      }
      *expr = true;
      return f;
    }
    return valueForm(x);
  }
  static void consume(const ElementModP& x) {
    if (!x.def) return;
    std::lock_guard<std::mutex> lk(x.def->mu);
    if (x.def->state == 0) x.def->consumed = true;
  }
  ElementModP consumeAndMake(const ElementModP& x, bool expr, const detail::Form& f) const {
    if (expr) consume(x);
    return make(f);
  }
  // y's bases after x's: in place when x's buffer has not been extended by anyone else
  static void append(detail::Form& x, const detail::Form& y) {
    std::vector<std::array<uint8_t, EG_P_BYTES>> ys;
    {
      std::lock_guard<std::mutex> lk(y.buf->mu);
      ys.assign(y.buf->v.begin(), y.buf->v.begin() + (std::ptrdiff_t)y.nb);
    }
    const std::shared_ptr<Deferred::Buf> old = x.buf;  // alive while its lock is held
    std::lock_guard<std::mutex> lk(old->mu);
    if (old->v.size() != x.nb) {  // another expression extended this buffer already: copy the prefix
      auto nb = std::make_shared<Deferred::Buf>();
      nb->v.assign(old->v.begin(), old->v.begin() + (std::ptrdiff_t)x.nb);
      nb->v.insert(nb->v.end(), ys.begin(), ys.end());
      x.nb += ys.size();
      x.buf = nb;
      return;
    }
    old->v.insert(old->v.end(), ys.begin(), ys.end());
    x.nb += ys.size();
  }
  std::optional<detail::Form> merge(const detail::Form& x, const detail::Form& y) const {
    if (x.nb && y.nb && (x.hasExp != y.hasExp || (x.hasExp && x.exp != y.exp))) return std::nullopt;
    detail::Form r = x;
    for (int t = 0; t < y.nfb; ++t) {
      int k = 0;
      while (k < r.nfb && r.fb[k] != y.fb[t]) ++k;
      if (k < r.nfb) {
        if (!r.fb[k]->orderQ()) return std::nullopt;
        r.fe[k] = modq_.add(modq_.reduce_small(r.fe[k]), modq_.reduce_small(y.fe[t]));
      } else {
        if (r.nfb == 2) return std::nullopt;
        r.fb[r.nfb] = y.fb[t];
        r.fe[r.nfb] = y.fe[t];
        ++r.nfb;
      }
    }
    if (y.nb) {
      if (!r.nb) {
        r.buf = y.buf;
        r.nb = y.nb;
        r.hasExp = y.hasExp;
        r.exp = y.exp;
      } else {
        append(r, y);
      }
    }
    return r;
  }
  // a new deferred element for f (a trivial f is a plain value)
  ElementModP make(const detail::Form& f0) const {
    detail::Form f = f0;
    if (f.nb == 0) f.hasExp = false;  // 1^e = 1
    if (f.nb == 0 && f.nfb == 0) return ElementModP::from_u64(1, this);
    if (f.nb == 1 && !f.hasExp && f.nfb == 0) {
      std::lock_guard<std::mutex> lk(f.buf->mu);
      return ElementModP(f.buf->v[0].data(), this);
    }
    auto d = std::make_shared<Deferred>();
    d->buf = f.buf;
    d->nb = f.nb;
    d->hasExp = f.hasExp;
    d->exp = f.exp;
    d->nfb = f.nfb;
    for (int t = 0; t < f.nfb; ++t) {
      d->fb[t] = f.fb[t];
      d->fe[t] = f.fe[t];
    }
    d->group = this;
    ElementModP e;
    e.group = this;
    e.have.store(false, std::memory_order_relaxed);
    e.def = d;
    if (!deferred_) {
      resolve(e);
      return e;
    }
    auto& q = detail::pendingQueue();
    q.push_back(d);
    if (q.size() >= 4096 && (q.size() & 4095) == 0)  // drop the dead and the already-submitted
      q.erase(std::remove_if(q.begin(), q.end(),
                             [](const std::weak_ptr<Deferred>& w) {
                               auto p = w.lock();
                               return !p || p->state != 0 || p->consumed;
                             }),
              q.end());
    return e;
  }
  // d.mu held, d.state == 0: one job (eg_mexp_submit); > 16 bases are folded first (eg_prod_reduce)
  void submit(Deferred& d) const {
    std::vector<uint8_t> bases;
    size_t nb = d.nb;
    if (nb) {
      std::lock_guard<std::mutex> lk(d.buf->mu);
      bases.resize(nb * EG_P_BYTES);
      for (size_t i = 0; i < nb; ++i) std::memcpy(&bases[i * EG_P_BYTES], d.buf->v[i].data(), EG_P_BYTES);
    }
    int rc = EG_OK;
    if (nb > detail::kMaxJobBases) {
      std::vector<uint8_t> one(EG_P_BYTES);
      rc = eg_prod_reduce(ctx_, bases.data(), 1, nb, one.data());
      bases.swap(one);
      nb = 1;
    }
    if (!rc) {
      uint8_t eb[32], f0[32], f1[32];
      d.exp.to_be(eb);
      d.fe[0].to_be(f0);
      d.fe[1].to_be(f1);
      rc = eg_mexp_submit(ctx_, nb ? bases.data() : nullptr, nb, d.hasExp ? eb : nullptr,
                          d.nfb > 0 ? d.fb[0]->handle() : nullptr, f0, d.nfb > 1 ? d.fb[1]->handle() : nullptr, f1,
                          d.out.data(), &d.ticket);
    }
    if (rc) {
      d.state = 3;
      d.err = eg_last_error();
    } else {
      d.state = 1;
    }
  }

  ElementModP p_, g_;
  ElementModQ q_;
  ModQ modq_;
  int device_;
  eg_ctx* ctx_ = nullptr;
  bool gOrderQ_ = false;
  mutable std::once_flag g_once_;
  mutable FixedBasePtr gfb_;
  mutable std::mutex accel_mu_;
  mutable std::map<std::string, FixedBasePtr> accel_;
  mutable std::atomic<bool> deferred_{true};
};

inline const GroupContext& group_of(const ElementModP& e) {
  if (!e.group) throw std::logic_error("ElementModP without a GroupContext");
  return *e.group;
}
inline ElementModP ElementModP::powP(const ElementModQ& e) const { return group_of(*this).powP(*this, e); }
inline ElementModP ElementModP::times(const ElementModP& o) const { return group_of(*this).multP(*this, o); }
inline ElementModP ElementModP::multInv() const { return group_of(*this).multInv(*this); }
inline ElementModP ElementModP::div(const ElementModP& o) const { return times(o.multInv()); }
inline bool ElementModP::isValidResidue() const { return group_of(*this).isValidResidue(*this); }
inline ElementModP ElementModP::acceleratePow() const { return group_of(*this).acceleratePow(*this); }
inline void ElementModP::resolve() const { group_of(*this).resolve(*this); }

// ---------------------------------------------------------------- key material (synthetic)
// The reference's remote key ceremony (RunRemoteKeyCeremony.java:200-233) is out of scope;
// this restates only its outputs: guardian i (x = i) holds P_i of degree quorum-1,
// commitments K_ij = g^{a_ij}, and the shares P_l(x_i) of every other guardian l.
struct GuardianKeys {
  std::string id;
  int x = 0;
  std::vector<ElementModQ> coeffs;       // a_0 = secret
  std::vector<ElementModP> commitments;  // g^{a_j}
  std::map<std::string, ElementModQ> sharesFrom;  // l -> P_l(x)
  const ElementModQ& secret() const { return coeffs.at(0); }
  const ElementModP& publicKey() const { return commitments.at(0); }
};

inline ElementModQ polyEval(const GroupContext& G, const std::vector<ElementModQ>& coeffs, int x) {
  ElementModQ acc;
  const ElementModQ xq = G.uIntToElementModQ((uint64_t)x);
  for (auto it = coeffs.rbegin(); it != coeffs.rend(); ++it) acc = G.addQ(G.mulQ(acc, xq), *it);
  return acc;
}

// -> guardians and the joint key K = prod_i K_i0
inline std::pair<std::vector<GuardianKeys>, ElementModP> keyCeremony(const GroupContext& G, int n, int quorum,
                                                                     uint64_t seed) {
  if (quorum < 1 || quorum > n) throw std::invalid_argument("need 1 <= quorum <= n");
  std::mt19937_64 rng(seed);
  std::vector<GuardianKeys> gs(n);
  std::vector<ElementModQ> flat;
  for (int i = 0; i < n; ++i) {
    gs[i].id = "guardian" + std::to_string(i + 1);
    gs[i].x = i + 1;
    for (int j = 0; j < quorum; ++j) gs[i].coeffs.push_back(G.randomElementModQ(rng));
    flat.insert(flat.end(), gs[i].coeffs.begin(), gs[i].coeffs.end());
  }
  const auto comm = G.gPowPBatch(flat);
  std::vector<ElementModP> pk;
  for (int i = 0; i < n; ++i) {
    gs[i].commitments.assign(comm.begin() + (size_t)i * quorum, comm.begin() + (size_t)(i + 1) * quorum);
    pk.push_back(gs[i].publicKey());
  }
  for (auto& gi : gs)
    for (const auto& gl : gs)
      if (gl.id != gi.id) gi.sharesFrom[gl.id] = polyEval(G, gl.coeffs, gi.x);
  return {gs, G.multP(pk)};
}

// ---------------------------------------------------------------- trustee plugin (B2)
class DecryptingTrusteeIF {  // RemoteDecryptingTrusteeProxy.java:30-122
 public:
  virtual ~DecryptingTrusteeIF() = default;
  virtual std::string id() const = 0;
  virtual int xCoordinate() const = 0;
  virtual ElementModP electionPublicKey() const = 0;
  // nonces: one per text (deterministic proofs in tests) or nullptr (random, as the
  // reference's nonce = null, RunRemoteDecryptingTrustee.java:193)
  virtual std::vector<DirectDecryptionAndProof> directDecrypt(const GroupContext& group,
                                                              const std::vector<ElGamalCiphertext>& texts,
                                                              const ElementModQ& extendedBaseHash,
                                                              const std::vector<ElementModQ>* nonces) = 0;
  virtual std::vector<CompensatedDecryptionAndProof> compensatedDecrypt(
      const GroupContext& group, const std::string& missingGuardianId, const std::vector<ElGamalCiphertext>& texts,
      const ElementModQ& extendedBaseHash, const std::vector<ElementModQ>* nonces) = 0;
};

// One GPU batch: M_i = pad_i^secret with generic CP proofs (eg_trustee_decrypt_batch).
inline std::pair<std::vector<ElementModP>, std::vector<GenericChaumPedersenProof>> partialDecryptBatch(
    const GroupContext& G, const ElementModQ& secret, const ElementModQ& qbar, const std::vector<ElGamalCiphertext>& texts,
    const std::vector<ElementModQ>& nonces) {
  const size_t n = texts.size();
  if (nonces.size() != n) throw std::invalid_argument("one nonce per text");
  std::vector<uint8_t> T(n * 2 * EG_P_BYTES), N = GroupContext::packQ(nonces), M(n * EG_P_BYTES), PR(n * 64);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&T[(2 * i) * EG_P_BYTES], texts[i].pad.byteArray(), EG_P_BYTES);
    std::memcpy(&T[(2 * i + 1) * EG_P_BYTES], texts[i].data.byteArray(), EG_P_BYTES);
  }
  const auto sb = secret.byteArray(), qb = qbar.byteArray();
  if (n)
    check(eg_trustee_decrypt_batch(G.handle(), sb.data(), qb.data(), T.data(), N.data(), n, M.data(), PR.data()),
          "eg_trustee_decrypt_batch");
  std::vector<GenericChaumPedersenProof> pr(n);
  for (size_t i = 0; i < n; ++i) pr[i] = {ElementModQ::from_be(&PR[64 * i]), ElementModQ::from_be(&PR[64 * i + 32])};
  return {G.unpackP(M, n), pr};
}

class GpuDecryptingTrustee : public DecryptingTrusteeIF {
 public:
  // commitments: every guardian's public commitments (for recovery public keys)
  GpuDecryptingTrustee(GuardianKeys keys, std::map<std::string, std::vector<ElementModP>> commitments,
                       uint64_t nonce_seed = std::random_device{}())
      : keys_(std::move(keys)), commitments_(std::move(commitments)), rng_(nonce_seed) {}

  std::string id() const override { return keys_.id; }
  int xCoordinate() const override { return keys_.x; }
  ElementModP electionPublicKey() const override { return keys_.publicKey(); }

  std::vector<DirectDecryptionAndProof> directDecrypt(const GroupContext& G, const std::vector<ElGamalCiphertext>& texts,
                                                      const ElementModQ& qbar,
                                                      const std::vector<ElementModQ>* nonces) override {
    const auto N = nonces ? *nonces : randomNonces(G, texts.size());
    auto [M, pr] = partialDecryptBatch(G, keys_.secret(), qbar, texts, N);
    std::vector<DirectDecryptionAndProof> out(texts.size());
    for (size_t i = 0; i < texts.size(); ++i) out[i] = {M[i], pr[i]};
    return out;
  }

  // g^{P_l(x_i)} = prod_j K_{l,j}^{x_i^j}
  ElementModP recoveryPublicKey(const GroupContext& G, const std::string& missingId) const {
    const auto& comm = commitments_.at(missingId);
    std::vector<ElementModQ> e;
    ElementModQ xj = G.uIntToElementModQ(1);
    const ElementModQ x = G.uIntToElementModQ((uint64_t)keys_.x);
    for (size_t j = 0; j < comm.size(); ++j) {
      e.push_back(xj);
      xj = G.mulQ(xj, x);
    }
    return G.multP(G.powPBatch(comm, e));
  }

  std::vector<CompensatedDecryptionAndProof> compensatedDecrypt(const GroupContext& G, const std::string& missingId,
                                                                const std::vector<ElGamalCiphertext>& texts,
                                                                const ElementModQ& qbar,
                                                                const std::vector<ElementModQ>* nonces) override {
    auto it = keys_.sharesFrom.find(missingId);
    if (it == keys_.sharesFrom.end()) throw ArithmeticException("no share of " + missingId);
    const auto N = nonces ? *nonces : randomNonces(G, texts.size());
    auto [M, pr] = partialDecryptBatch(G, it->second, qbar, texts, N);
    const ElementModP rk = recoveryPublicKey(G, missingId);
    std::vector<CompensatedDecryptionAndProof> out(texts.size());
    for (size_t i = 0; i < texts.size(); ++i) out[i] = {M[i], pr[i], rk};
    return out;
  }

 private:
  std::vector<ElementModQ> randomNonces(const GroupContext& G, size_t n) {
    std::vector<ElementModQ> v(n);
    for (auto& u : v) u = G.randomElementModQ(rng_);
    return v;
  }
  GuardianKeys keys_;
  std::map<std::string, std::vector<ElementModP>> commitments_;
  std::mt19937_64 rng_;
};

// RemoteDecryptingTrusteeProxy behaviour: any failure -> empty list (:64-66, :103-105).
template <class F>
auto TrusteeCallOrEmpty(F&& f) -> decltype(f()) {
  try {
    return f();
  } catch (const std::exception&) {
    return {};
  }
}

// Share-proof verification: a = g^v K_i^c, b = pad^v M^c, c == H(qbar, pad, data, a, b, M).
inline std::vector<bool> verifyShares(const GroupContext& G, const ElementModQ& qbar, const std::vector<ElementModP>& Ki,
                                      const std::vector<ElGamalCiphertext>& texts, const std::vector<ElementModP>& M,
                                      const std::vector<GenericChaumPedersenProof>& proofs) {
  const size_t n = texts.size();
  if (Ki.size() != n || M.size() != n || proofs.size() != n) throw std::invalid_argument("verifyShares: sizes");
  std::vector<uint8_t> K = GroupContext::packP(Ki), T(n * 2 * EG_P_BYTES), Mm = GroupContext::packP(M), PR(n * 64),
                       ok(n, 0);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&T[(2 * i) * EG_P_BYTES], texts[i].pad.byteArray(), EG_P_BYTES);
    std::memcpy(&T[(2 * i + 1) * EG_P_BYTES], texts[i].data.byteArray(), EG_P_BYTES);
    proofs[i].c.v.to_be(&PR[64 * i]);
    proofs[i].v.v.to_be(&PR[64 * i + 32]);
  }
  const auto qb = qbar.byteArray();
  if (n) check(eg_verify_shares(G.handle(), qb.data(), K.data(), T.data(), Mm.data(), PR.data(), n, ok.data()),
               "eg_verify_shares");
  return std::vector<bool>(ok.begin(), ok.end());
}

inline ElementModQ lagrangeCoefficient(const GroupContext& G, const std::vector<int>& xs, int xi) {
  ElementModQ num = G.uIntToElementModQ(1), den = G.uIntToElementModQ(1);
  for (int xj : xs)
    if (xj != xi) {
      num = G.mulQ(num, G.uIntToElementModQ((uint64_t)xj));
      den = G.mulQ(den, G.subQ(G.uIntToElementModQ((uint64_t)xj), G.uIntToElementModQ((uint64_t)xi)));
    }
  return G.mulQ(num, G.invQ(den));
}

// What the mediator publishes for a decrypted tally (the share data the reference's
// Verifier(record, 11).verify() re-checks, RunRemoteWorkflowTest.java:179-182).
struct DecryptionRecord {
  std::vector<ElGamalCiphertext> texts;                                  // encrypted tally
  std::map<std::string, int> xs;                                         // available guardian -> x
  std::map<std::string, std::vector<DirectDecryptionAndProof>> direct;   // available -> n shares
  std::map<std::string, std::map<std::string, std::vector<CompensatedDecryptionAndProof>>> compensated;  // missing -> available -> n
  std::vector<std::optional<int64_t>> counts;
};

// Mediator combine: new Decryption(group, init, trustees, missing).decrypt(tally)
// (RunRemoteDecryptor.java:261-262): verify every share's proof, Lagrange-weight the
// compensated shares, M = prod M_i, T = data / M, t = dLogG(T).
class Decryption {
 public:
  Decryption(const GroupContext& G, ElementModQ qbar, std::vector<DecryptingTrusteeIF*> trustees,
             std::vector<std::string> missing)
      : G_(G), qbar_(qbar), trustees_(std::move(trustees)), missing_(std::move(missing)) {}

  std::vector<std::optional<int64_t>> decrypt(const std::vector<ElGamalCiphertext>& tally, int64_t maxCount) {
    return decryptRecord(tally, maxCount).counts;
  }

  // decrypt() keeping every share and proof (the published decryption record)
  DecryptionRecord decryptRecord(const std::vector<ElGamalCiphertext>& tally, int64_t maxCount) {
    const size_t n = tally.size();
    DecryptionRecord rec;
    rec.texts = tally;
    std::vector<int> xs;
    for (auto* t : trustees_) {
      xs.push_back(t->xCoordinate());
      rec.xs[t->id()] = t->xCoordinate();
    }
    std::vector<std::vector<ElementModP>> parts;
    for (auto* tr : trustees_) {
      auto res = tr->directDecrypt(G_, tally, qbar_, nullptr);
      if (res.size() != n) throw ArithmeticException("trustee " + tr->id() + " returned a short direct list");
      std::vector<ElementModP> M;
      std::vector<GenericChaumPedersenProof> pr;
      for (auto& r : res) {
        M.push_back(r.partialDecryption);
        pr.push_back(r.proof);
      }
      const auto ok = verifyShares(G_, qbar_, std::vector<ElementModP>(n, tr->electionPublicKey()), tally, M, pr);
      if (std::find(ok.begin(), ok.end(), false) != ok.end())
        throw ArithmeticException("invalid direct decryption proof from " + tr->id());
      rec.direct[tr->id()] = res;
      parts.push_back(std::move(M));
    }
    for (const auto& l : missing_)
      for (auto* tr : trustees_) {
        auto res = tr->compensatedDecrypt(G_, l, tally, qbar_, nullptr);
        if (res.size() != n) throw ArithmeticException("trustee " + tr->id() + " returned a short compensated list");
        std::vector<ElementModP> M, rk;
        std::vector<GenericChaumPedersenProof> pr;
        for (auto& r : res) {
          M.push_back(r.partialDecryption);
          pr.push_back(r.proof);
          rk.push_back(r.recoveredPublicKeyShare);
        }
        const auto ok = verifyShares(G_, qbar_, rk, tally, M, pr);
        if (std::find(ok.begin(), ok.end(), false) != ok.end())
          throw ArithmeticException("invalid compensated decryption proof from " + tr->id() + " for " + l);
        rec.compensated[l][tr->id()] = res;
        const ElementModQ w = lagrangeCoefficient(G_, xs, tr->xCoordinate());
        parts.push_back(G_.powPBatch(M, std::vector<ElementModQ>(n, w)));
      }
    const size_t k = parts.size();
    std::vector<ElementModP> stacked;
    stacked.reserve(n * k);
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j < k; ++j) stacked.push_back(parts[j][i]);
    const auto M = G_.prodPGroups(stacked, n, k);
    std::vector<ElementModP> data;
    for (const auto& t : tally) data.push_back(t.data);
    const auto T = G_.multPBatch(data, G_.multInvBatch(M));
    rec.counts = G_.dLogGBatch(T, maxCount);
    return rec;
  }

 private:
  const GroupContext& G_;
  ElementModQ qbar_;
  std::vector<DecryptingTrusteeIF*> trustees_;
  std::vector<std::string> missing_;
};

// Record-level checks of a tally decryption, independent of the mediator that made it (the
// decryption part of Verifier(record, 11).verify(), RunRemoteWorkflowTest.java:179-182);
// same checks as the Python decrypt.verify_decryption_record, every exponentiation on the GPU.
struct DecryptionRecordChecks {
  bool directProofs = true, recoveryKeys = true, compensatedProofs = true, quorum = true, tally = true;
  bool all() const { return directProofs && recoveryKeys && compensatedProofs && quorum && tally; }
};

inline DecryptionRecordChecks verifyDecryptionRecord(const GroupContext& G, const ElementModQ& qbar,
                                                     const DecryptionRecord& rec,
                                                     const std::map<std::string, ElementModP>& publicKeys,
                                                     const std::map<std::string, std::vector<ElementModP>>& commitments) {
  // Malformed (untrusted) records fail their checks instead of throwing or reading out of
  // bounds: unknown guardian ids, short share lists and negative counts are all "false".
  DecryptionRecordChecks out;
  const size_t n = rec.texts.size();
  auto allTrue = [](const std::vector<bool>& v) { return std::find(v.begin(), v.end(), false) == v.end(); };
  for (const auto& [gid, res] : rec.direct) {
    const auto pk = publicKeys.find(gid);
    if (pk == publicKeys.end() || rec.xs.count(gid) == 0) { out.directProofs = out.quorum = false; continue; }
    if (res.size() != n) { out.directProofs = false; continue; }
    std::vector<ElementModP> M;
    std::vector<GenericChaumPedersenProof> pr;
    for (const auto& r : res) { M.push_back(r.partialDecryption); pr.push_back(r.proof); }
    out.directProofs &= allTrue(verifyShares(G, qbar, std::vector<ElementModP>(n, pk->second), rec.texts, M, pr));
  }
  if (rec.counts.size() != n) out.tally = false;
  for (const auto& c : rec.counts) out.tally &= c.has_value() && *c >= 0;
  for (const auto& [l, byAvail] : rec.compensated) {
    out.quorum &= byAvail.size() == rec.direct.size();
    const auto cm = commitments.find(l);
    if (cm == commitments.end()) { out.recoveryKeys = out.compensatedProofs = false; continue; }
    const auto& comm = cm->second;
    for (const auto& [gid, res] : byAvail) {
      out.quorum &= rec.direct.count(gid) == 1;
      const auto xi = rec.xs.find(gid);
      if (xi == rec.xs.end() || xi->second < 0) { out.quorum = false; continue; }
      if (res.size() != n) { out.compensatedProofs = out.recoveryKeys = false; continue; }
      // g^{P_l(x_i)} = prod_j K_{l,j}^{x_i^j}
      std::vector<ElementModQ> e;
      ElementModQ xj = G.uIntToElementModQ(1);
      const ElementModQ x = G.uIntToElementModQ((uint64_t)xi->second);
      for (size_t j = 0; j < comm.size(); ++j) { e.push_back(xj); xj = G.mulQ(xj, x); }
      const ElementModP want = G.multP(G.powPBatch(comm, e));
      std::vector<ElementModP> M, rk;
      std::vector<GenericChaumPedersenProof> pr;
      for (const auto& r : res) {
        out.recoveryKeys &= r.recoveredPublicKeyShare == want;
        M.push_back(r.partialDecryption); pr.push_back(r.proof); rk.push_back(r.recoveredPublicKeyShare);
      }
      out.compensatedProofs &= allTrue(verifyShares(G, qbar, rk, rec.texts, M, pr));
    }
  }
  // every share list must cover every text before the combination indexes them
  bool lengthsOk = true;
  for (const auto& [gid, res] : rec.direct) lengthsOk &= res.size() == n;
  for (const auto& [l, byAvail] : rec.compensated)
    for (const auto& [gid, res] : byAvail) lengthsOk &= res.size() == n;
  if (!lengthsOk) out.tally = false;
  if (!out.quorum || !out.tally || n == 0) return out;
  // B == M g^t with M = prod_i M_i * prod_l prod_i M_{l,i}^{w_i}; Lagrange over the AVAILABLE x's
  std::vector<int> xs;
  for (const auto& [gid, res] : rec.direct) xs.push_back(rec.xs.at(gid));
  std::vector<std::vector<ElementModP>> parts;
  for (const auto& [gid, res] : rec.direct) {
    std::vector<ElementModP> M;
    for (const auto& r : res) M.push_back(r.partialDecryption);
    parts.push_back(std::move(M));
  }
  for (const auto& [l, byAvail] : rec.compensated)
    for (const auto& [gid, res] : byAvail) {
      std::vector<ElementModP> M;
      for (const auto& r : res) M.push_back(r.partialDecryption);
      parts.push_back(G.powPBatch(M, std::vector<ElementModQ>(n, lagrangeCoefficient(G, xs, rec.xs.at(gid)))));
    }
  const size_t k = parts.size();
  std::vector<ElementModP> stacked;
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < k; ++j) stacked.push_back(parts[j][i]);
  const auto M = G.prodPGroups(stacked, n, k);
  std::vector<ElementModQ> t;
  for (const auto& c : rec.counts) t.push_back(G.uIntToElementModQ((uint64_t)*c));
  const auto lhs = G.multPBatch(M, G.gPowPBatch(t));
  for (size_t i = 0; i < n; ++i) out.tally &= lhs[i] == rec.texts[i].data;
  return out;
}

// ---------------------------------------------------------------- ballots (B1 batch users)
struct Manifest {  // synthetic manifest shape (RandomBallotProvider, RunRemoteWorkflowTest.java:133)
  size_t nContests = 4, nSelections = 5, votesAllowed = 1;
  size_t spc() const { return nSelections + votesAllowed; }
  size_t nsel() const { return nContests * spc(); }
  size_t nReal() const { return nContests * nSelections; }
};

// Wire layout of include/eg_hip.h (big-endian, ballot-major).
struct EncryptedBallots {
  size_t n = 0;
  std::vector<uint8_t> cts, rproof, cproof;  // n*nsel*2*512, n*nsel*4*32, n*nc*2*32
};

inline void setElectionKey(const GroupContext& G, const ElementModP& K, int windowBits) {
  check(eg_set_election_key(G.handle(), K.byteArray(), windowBits), "eg_set_election_key");
}

// batchEncryption with injected nonces (RunRemoteWorkflowTest.java:140-141)
inline EncryptedBallots batchEncryption(const GroupContext& G, const ElementModP& K, int windowBits,
                                        const ElementModQ& qbar, const Manifest& man, size_t nb,
                                        const std::vector<uint8_t>& votes, const std::vector<uint8_t>& selNonces,
                                        const std::vector<uint8_t>& contestNonces) {
  if (votes.size() != nb * man.nsel() || selNonces.size() != nb * man.nsel() * 4 * 32 ||
      contestNonces.size() != nb * man.nContests * 32)
    throw std::invalid_argument("batchEncryption: buffer sizes do not match the manifest");
  EncryptedBallots eb;
  eb.n = nb;
  eb.cts.resize(nb * man.nsel() * 2 * EG_P_BYTES);
  eb.rproof.resize(nb * man.nsel() * 4 * 32);
  eb.cproof.resize(nb * man.nContests * 2 * 32);
  setElectionKey(G, K, windowBits);  // K's table at this width (the call itself passes K too)
  const auto qb = qbar.byteArray();
  if (nb)
    check(eg_encrypt_ballots(G.handle(), K.byteArray(), qb.data(), nb, man.nContests, man.spc(), votes.data(),
                             selNonces.data(), contestNonces.data(), eb.cts.data(), eb.rproof.data(), eb.cproof.data()),
          "eg_encrypt_ballots");
  return eb;
}

// Verifier(record, 11).verify() ballot proofs + runAccumulateBallots (:151,179-182)
struct VerifyResult {
  std::vector<uint8_t> okSelection, okContest;
  std::vector<ElGamalCiphertext> tally;  // n_real selections
  bool allValid() const {
    return std::all_of(okSelection.begin(), okSelection.end(), [](uint8_t v) { return v == 1; }) &&
           std::all_of(okContest.begin(), okContest.end(), [](uint8_t v) { return v == 1; });
  }
};

// cast (optional, one flag per ballot, 0 = spoiled): every ballot is verified, only the cast ones
// are tallied; spoiled ballots go to Decryption::decryptBallots (RunRemoteDecryptor.java:264-269)
inline VerifyResult verifyBallots(const GroupContext& G, const ElementModP& K, const ElementModQ& qbar,
                                  const Manifest& man, const EncryptedBallots& eb,
                                  const std::vector<uint8_t>* cast = nullptr) {
  if (cast && cast->size() != eb.n) throw std::invalid_argument("verifyBallots: one cast flag per ballot");
  VerifyResult r;
  r.okSelection.assign(eb.n * man.nsel(), 0);
  r.okContest.assign(eb.n * man.nContests, 0);
  std::vector<uint8_t> tal(man.nReal() * 2 * EG_P_BYTES);
  const auto qb = qbar.byteArray();
  check(eg_verify_ballots(G.handle(), K.byteArray(), qb.data(), eb.n, man.nContests, man.spc(), man.votesAllowed,
                          (uint32_t)man.votesAllowed, eb.cts.data(), eb.rproof.data(), eb.cproof.data(),
                          cast ? cast->data() : nullptr, r.okSelection.data(), r.okContest.data(), tal.data()),
        "eg_verify_ballots");
  for (size_t i = 0; i < man.nReal(); ++i)
    r.tally.push_back({ElementModP(&tal[(2 * i) * EG_P_BYTES], &G), ElementModP(&tal[(2 * i + 1) * EG_P_BYTES], &G)});
  return r;
}

// ---- device memory and the multi-GPU tally exchange (include/eg_hip.h eg_dev_* / eg_comm_*) ----
// HBM on the context's device through the library's own HIP runtime (RAII).
class DeviceBuffer {
 public:
  DeviceBuffer(const GroupContext& G, size_t bytes) : ctx_(G.handle()), bytes_(bytes) {
    check(eg_dev_alloc(ctx_, bytes, &ptr_), "eg_dev_alloc");
  }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  ~DeviceBuffer() { eg_dev_free(ctx_, ptr_); }
  uint8_t* data() const { return (uint8_t*)ptr_; }
  size_t size() const { return bytes_; }
  void upload(const void* src, size_t bytes, size_t offset = 0) {
    if (offset + bytes > bytes_) throw std::out_of_range("DeviceBuffer::upload past the end");
    check(eg_memcpy_htod(ctx_, data() + offset, src, bytes), "eg_memcpy_htod");
  }
  void download(void* dst, size_t bytes, size_t offset = 0) const {
    if (offset + bytes > bytes_) throw std::out_of_range("DeviceBuffer::download past the end");
    check(eg_memcpy_dtoh(ctx_, dst, data() + offset, bytes), "eg_memcpy_dtoh");
  }
  bool allNonzero(size_t n) const {  // the first n bytes are non-zero flags (verifier verdicts)
    int all = 0;
    check(eg_all_nonzero_dev(ctx_, data(), n, &all), "eg_all_nonzero_dev");
    return all != 0;
  }

 private:
  eg_ctx* ctx_;
  void* ptr_ = nullptr;
  size_t bytes_;
};

// One rank's RCCL communicator inside the library: rank 0 makes the id, the caller
// sends it to every rank over any host channel, each rank constructs the exchange (collective).
class TallyExchange {
 public:
  static std::array<uint8_t, EG_COMM_ID_BYTES> uniqueId() {
    std::array<uint8_t, EG_COMM_ID_BYTES> id{};
    check(eg_comm_unique_id(id.data()), "eg_comm_unique_id");
    return id;
  }
  TallyExchange(const GroupContext& G, const uint8_t id[EG_COMM_ID_BYTES], int world, int rank)
      : G_(G), rank_(rank) {
    check(eg_comm_init(G.handle(), id, world, rank), "eg_comm_init");
  }
  TallyExchange(const TallyExchange&) = delete;
  TallyExchange& operator=(const TallyExchange&) = delete;
  ~TallyExchange() { eg_comm_destroy(G_.handle()); }
  bool allValid(bool ok) const {
    int all = 0;
    check(eg_comm_all_valid(G_.handle(), ok ? 1 : 0, &all), "eg_comm_all_valid");
    return all != 0;
  }
  // every rank's nparts x n partial-tally rows in HBM, folded mod p; the product on root, empty elsewhere
  std::vector<ElementModP> fold(const DeviceBuffer& parts, size_t nparts, size_t n, int root = 0) const {
    return foldTally(G_, parts, nparts, n, root, rank_);
  }
  static std::vector<ElementModP> foldTally(const GroupContext& G, const DeviceBuffer& parts, size_t nparts, size_t n,
                                            int root = 0, int rank = 0) {
    if (parts.size() < nparts * n * EG_P_BYTES) throw std::out_of_range("fold: parts shorter than nparts x n");
    std::vector<uint8_t> out(n * EG_P_BYTES);
    check(eg_tally_allgather_fold(G.handle(), parts.data(), nparts, n, root, rank == root ? out.data() : nullptr),
          "eg_tally_allgather_fold");
    if (rank != root) return {};
    std::vector<ElementModP> r(n);
    for (size_t i = 0; i < n; ++i) r[i] = ElementModP(&out[i * EG_P_BYTES], &G);
    return r;
  }

 private:
  const GroupContext& G_;
  int rank_;
};

// Decryption.decryptBallot (RunRemoteDecryptor.java:264-269) over a batch of spoiled ballots:
// every ballot's real selections (placeholders are not part of the plaintext) go to the trustees
// as ONE batch per guardian, then the same share checks, Lagrange combine and dLog (<= votes
// allowed) as the tally.  -> per ballot, its decrypted selections (nullopt: not a valid count).
inline std::vector<std::vector<std::optional<int64_t>>> decryptBallots(Decryption& dec, const Manifest& man,
                                                                        const EncryptedBallots& spoiled,
                                                                        const GroupContext& G,
                                                                        DecryptionRecord* record = nullptr) {
  std::vector<ElGamalCiphertext> texts;
  texts.reserve(spoiled.n * man.nReal());
  for (size_t b = 0; b < spoiled.n; ++b)
    for (size_t c = 0; c < man.nContests; ++c)
      for (size_t s = 0; s < man.nSelections; ++s) {
        const uint8_t* ct = &spoiled.cts[((b * man.nsel()) + c * man.spc() + s) * 2 * EG_P_BYTES];
        texts.push_back({ElementModP(ct, &G), ElementModP(ct + EG_P_BYTES, &G)});
      }
  std::vector<std::vector<std::optional<int64_t>>> out(spoiled.n);
  if (texts.empty()) return out;
  DecryptionRecord rec = dec.decryptRecord(texts, (int64_t)man.votesAllowed);
  for (size_t b = 0; b < spoiled.n; ++b)
    out[b].assign(rec.counts.begin() + b * man.nReal(), rec.counts.begin() + (b + 1) * man.nReal());
  if (record) *record = std::move(rec);
  return out;
}

}  // namespace electionguard
