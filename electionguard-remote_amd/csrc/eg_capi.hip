// eg_capi.hip — host side of libeg_hip.so: the C ABI declared in include/eg_hip.h.
//
// Reference interfaces replaced (file:line under /root/reference):
//   GroupContext construction  KUtils.productionGroup            KUtils.java:10-12
//   element wire import/export ConvertCommonProto                ConvertCommonProto.java:41-57,111-121
//   batchEncryption / runAccumulateBallots / Verifier             RunRemoteWorkflowTest.java:140-141,151,179-182
//   DecryptingTrusteeIF.directDecrypt / compensatedDecrypt       RunRemoteDecryptingTrustee.java:189-193,227-232
// The arithmetic itself is upstream (electionguard-kotlin-multiplatform-jvm, not in
// the container); see DESIGN.md for the restated algorithms.
#include <hip/hip_runtime.h>

#include <algorithm>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/eg_hip.h"
#include "eg_kernels.hpp"
#include "eg_pow16.h"

using namespace eg;

// ------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------
static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess)                                                           \
      return fail(EG_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_));     \
  } while (0)

extern "C" const char* eg_last_error(void) { return g_err.c_str(); }

extern "C" int eg_version(char* buf, size_t len) {
  if (!buf || !len) return fail(EG_ERR_ARG, "null buffer");
  snprintf(buf, len, "eg_hip gfx950 radix2^%d limbs=%d lanes/elem=%d words/elem=%d", kLimbBits, kN, kT, kW);
  return EG_OK;
}

// ------------------------------------------------------------------------------
// host bignum helpers (constants only; 128 little-endian 32-bit words)
// ------------------------------------------------------------------------------
using Big = std::vector<uint32_t>;

static Big be_to_words(const uint8_t* be, int nbytes) {
  Big w((nbytes + 3) / 4, 0);
  for (int i = 0; i < nbytes; ++i) {
    const int bit = (nbytes - 1 - i) * 8;
    w[bit / 32] |= (uint32_t)be[i] << (bit % 32);
  }
  return w;
}
static bool ge(const Big& a, const Big& b) {
  for (int i = (int)a.size() - 1; i >= 0; --i)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}
static void sub_in(Big& a, const Big& b) {
  int64_t c = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    c += (int64_t)a[i] - b[i];
    a[i] = (uint32_t)c;
    c >>= 32;
  }
}
// a = 2a mod m  (a < m, m < 2^(32*size))
static void dbl_mod(Big& a, const Big& m) {
  uint32_t top = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    const uint32_t nt = a[i] >> 31;
    a[i] = (a[i] << 1) | top;
    top = nt;
  }
  if (top || ge(a, m)) sub_in(a, m);
}
// words (LE, 128+) -> device element format (radix 2^kLimbBits limbs, padded lane blocks)
static void words_to_elem(const Big& w, uint32_t* out) {
  std::memset(out, 0, sizeof(uint32_t) * kW);
  for (int a = 0; a < kN; ++a) {
    const int bit = a * kLimbBits;
    uint64_t v = 0;
    for (int k = 0; k < 2; ++k) {  // bit % 32 + 29 <= 60: two words hold the limb (a shift by 64 would be UB)
      const int wi = bit / 32 + k;
      if (wi < (int)w.size()) v |= (uint64_t)w[wi] << (32 * k);
    }
    const uint32_t limb = (uint32_t)(v >> (bit % 32)) & kMask;
    out[(a / kL) * kLP + (a % kL)] = limb;
  }
}

// ------------------------------------------------------------------------------
// context
// ------------------------------------------------------------------------------
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
};

struct ProfRec {
  hipEvent_t a = nullptr, b = nullptr;
  double mm = 0;   // Montgomery operations (multiplies + squarings)
  double sqr = 0;  // of which squarings (symmetric-half schedule)
};
// Per-workgroup clock records of the profiled k_pow launches: one device buffer per profile
// window (allocated by eg_ctx_profile_begin, so nothing is allocated inside the timed launches),
// (s_memtime ticks, s_memrealtime ticks) per workgroup, launches appended in order.
constexpr size_t kClockRecs = (size_t)1 << 20;

// Montgomery operations of one k_pow job, split into squarings and multiplies: counted from
// the job's op program itself (pow_schedule), so the profile's MM totals are the kernel's work.
struct MMCount {
  double mul = 0, sqr = 0;
};
struct SchedBuf {
  const uint32_t* ptr;
  MMCount mm;
};

struct eg_fixed_base {
  eg_ctx* ctx = nullptr;
  uint32_t* d_tab = nullptr;
  int wbits = 0, nwin = 0;
  std::array<uint8_t, 512> base{};  // the base (big-endian), for the constant-time companion table
  // constant-time companion (eg_ctx_set_ct_pow): the same base at a window a masked scan can read
  // (kCtEncWindow bits), built on first constant-time use when wbits > kCtMaxWindow; owned
  eg_fixed_base* ct = nullptr;
  // per-element jobs queued on this table and not yet run (eg_capi_coalesce.inc): eg_fixed_base_destroy
  // waits for them, so a queued batch never reads a freed table
  std::atomic<int> queued{0};
  FbTab tab() const { return FbTab{d_tab, (uint32_t)wbits, (uint32_t)nwin}; }
};

// widest radix table a constant-time fixed-base term scans (2^w entries per multiply)
constexpr uint32_t kCtMaxWindow = 8;
// radix width of the constant-time encryption tables of g and K (eg_ctx_set_ct_encrypt): 43
// windows of 64 entries, 1.76 MB per base (EG_CT_WINDOW=4..8 overrides it at context creation)
constexpr int kCtEncWindow = 6;

enum Slot {
  W_IN0, W_IN1, W_EXP, W_OUT, W_E0, W_E1, W_E2, W_E3, W_JOBS, W_SCR, W_TMP, W_FLAGS, W_SCAL,
  W_BE0, W_BE1, W_BE2, W_OK0, W_OK1, W_OFF, W_H0, W_H1, W_H2, W_H3, W_H4, W_H5, W_H6, W_H7, W_H8, W_EB0, W_EB1, W_EB2, W_EA2, W_YA, W_YB, W_RZ, W_CRF, W_CAST, W_ANY, W_GATHER, W_KBE, W_NSLOT
};

struct eg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  MontConsts h{};
  MontConsts* d = nullptr;
  uint8_t p_be[512], q_be[32], g_be[512];
  uint8_t* d_q = nullptr;
  uint8_t* d_qbar = nullptr;
  eg_fixed_base* gtab = nullptr;
  eg_fixed_base* Ktab = nullptr;  // the current election key's radix table (keys.front().fb)
  uint32_t* d_gcomb = nullptr;  // Lim-Lee comb subset table of g (32 elements) for constant-time g^u
  uint32_t hash_fmt = EG_HASH_FIXED_WIDTH;  // Fiat-Shamir pre-image hex format (eg_ctx_set_hash_format)
  uint32_t resp_plus = 0;  // response convention (eg_ctx_set_proof_format): 0 = v = u - c x, 1 = v = u + c x
  uint32_t pre_order = EG_PREIMAGE_MESSAGE_FIRST;  // challenge pre-image element order
  DevBuf ws[W_NSLOT];
  bool timing = false;
  std::vector<ProfRec> prof;
  uint64_t* d_clk = nullptr;  // kClockRecs x 2 clock records of the open profile window
  size_t clk_used = 0;        // records handed out in this window
  uint32_t clk_used_last = 0, clk_dropped_last = 0;  // of the last closed window (eg_ctx_profile_clock)
  uint8_t K_be[512];  // the current election key (keys.front().K)
  // radix tables of the election keys seen on this ctx, most recently used first (a shared ctx may
  // serve several keys: calls alternating between two keys reuse both tables instead of rebuilding
  // one per call); each entry also holds the key's constant-time encryption table once built
  struct KeyTabs {
    std::array<uint8_t, 512> K;
    eg_fixed_base* fb = nullptr;
    eg_fixed_base* ct = nullptr;
    uint8_t* d_K = nullptr;  // K's 512 big-endian bytes in HBM (the EG_PREIMAGE_WITH_KEY hash element)
  };
  std::vector<KeyTabs> keys;
  std::map<std::string, DevBuf> cache;  // shape-keyed job tables
  std::map<std::string, SchedBuf> sched;  // k_pow op programs per launch shape (pow_schedule_dev)
  uint32_t use_comb = 1;                // two-exponent jobs use the Lim-Lee comb (EG_NO_COMB=1 to disable)
  uint32_t ct_encrypt = 0;              // encryption on k_pow<F, true> with small CT tables (eg_ctx_set_ct_encrypt)
  uint32_t ct_pow = 0;                  // powP / fixed-base / per-element calls constant-time (eg_ctx_set_ct_pow)
  std::atomic<uint32_t> ct_pow_submit{0};  // the same switch as per-element submits read it (no ctx lock)
  int ct_window = kCtEncWindow;         // their radix width
  eg_fixed_base* g_ct = nullptr;  // g's kCtEncWindow-bit table (K's live in keys[].ct)
  uint32_t ct_rows = 4;                 // trustee pair comb rows (EG_CT_ROWS=5: one 32-entry block)
  uint32_t sel_rows = 4;                // verifier selection jobs' comb: 4 = 4 rows x 3 blocks, 0 = 5 rows x 2 blocks (EG_SEL_COMB=52)
  uint32_t sel_blocks = 3;              // its column blocks (EG_SEL_COMB=42 / 44: 4 rows x 2 / 4 blocks, A/B only)
  // k_pow workgroups resident at once (CUs x blocks per CU): the verifier sizes its launch
  // populations so launches end on full rounds (EG_TAIL_SPLIT=0 disables; 0 = unknown)
  size_t pow_slots = 0;
  uint32_t pow_wps = 3;                 // k_pow waves per SIMD at that occupancy
  double prof_clock_ghz = 0;  // shader clock over the last profiled k_pow launches (eg_ctx_profile_clock)
  // fixed-base tables of guardian keys K_i for large share-proof batches (eg_verify_shares),
  // most recently used first
  std::vector<std::pair<std::array<uint8_t, 512>, eg_fixed_base*>> share_keys;
  // per-element calls from many threads gathered into batches (eg_capi_coalesce.inc)
  std::shared_ptr<struct Coalescer> co;  // tickets share it: waiting stays valid after the ctx is gone
  std::mutex co_mu;  // guards the lazy creation of co
  bool co_closed = false;  // set by eg_ctx_destroy (under co_mu)
  // host-pointer verify: uploads of chunk k+1 on their own stream overlap chunk k's kernels
  hipStream_t copy = nullptr;
  hipEvent_t up_ev[2] = {nullptr, nullptr}, done_ev[2] = {nullptr, nullptr};
  void* comm = nullptr;  // RCCL communicator of the multi-GPU exchange (eg_comm_init; eg_capi_comm.inc)
  int comm_world = 1, comm_rank = 0;
  // sticky after a communicator was aborted (a collective that timed out or failed, an init that did):
  // every collective and the fold fail with EG_ERR_STATE until eg_comm_destroy / eg_comm_init, so a
  // retry can never fold the local parts alone and call that the tally
  bool comm_failed = false;
  std::string comm_fail_msg;
  // the latency-shaped powP layouts (eg_pow16.hip) for the coalescer's small batches: one element
  // per wave for batches up to one per SIMD (latw_jobs), 16-lane groups up to one resident round
  // (lat_jobs); EG_LATENCY_POW=0 keeps every batch on the 8-lane layout, =16 skips the per-wave one
  // (A/B runs)
  Pow16Consts* lat = nullptr;
  size_t lat_jobs = 0;
  PowWaveConsts* latw = nullptr;
  size_t latw_jobs = 0;
  // the coalescer runs a batch of up to wave_max jobs on the per-wave kernel (any mix of kinds);
  // larger batches of one plain kind keep the throughput layouts (EG_WAVE_MAX overrides)
  size_t wave_max = 0;
  bool wave_split = true;  // fixed-base windows of a per-element job over 4 waves (EG_WAVE_SPLIT=0: one wave)
  // per-wave batches of at most r2l_max jobs (one per CU) run their variable parts right to left over
  // 4 waves (k_wave_job r2l; EG_WAVE_R2L=n overrides, 0 keeps the one-wave sliding window)
  size_t r2l_max = 0;
  // per-wave batches of at most w8_max jobs without a variable exponent split their fixed-base windows
  // over 8 waves (two per SIMD at one job per CU: n/8 + 3 multiplies of latency instead of n/4 + 2;
  // EG_WAVE_W8=n overrides, 0 keeps 4 waves)
  size_t w8_max = 0;
  // per-wave batches read inputs (1) / write results (2) straight from / into the coalescer's pinned
  // staging; default: results (2), one copy fewer per batch (EG_COALESCE_ZC=0|in|out|inout)
  int co_zc = 2;
  bool fb_lds = false;     // A/B: eg_fb_pow_batch_dev over a 7-bit table on the LDS-staged k_fb_lds (EG_FB_LDS=1)
  int test_fail_jobs = 0;  // EG_TEST_FAIL_JOBS=k: the k-th job-table upload fails (tests of the cache's failure path)
};

static int ws_get(eg_ctx* c, Slot s, size_t bytes, void** out) {
  DevBuf& b = c->ws[s];
  if (b.bytes < bytes) {
    if (b.ptr) HIPCHK(hipFree(b.ptr));
    b.ptr = nullptr;
    b.bytes = 0;
    size_t want = std::max(bytes, (size_t)4096);
    hipError_t e = hipMalloc(&b.ptr, want);
    if (e != hipSuccess) return fail(EG_ERR_NOMEM, "hipMalloc workspace " + std::to_string(want) + " B failed");
    b.bytes = want;
  }
  *out = b.ptr;
  return EG_OK;
}

// launch the Montgomery-friendly or general instantiation of a kernel template
#define LAUNCH_F(c, K, grid, ...)                                                              \
  do {                                                                                        \
    if ((c)->h.friendly)                                                                      \
      hipLaunchKernelGGL(K<true>, grid, dim3(kBlock), 0, (c)->stream, __VA_ARGS__);            \
    else                                                                                      \
      hipLaunchKernelGGL(K<false>, grid, dim3(kBlock), 0, (c)->stream, __VA_ARGS__);           \
  } while (0)

static inline unsigned grid_for(size_t groups) { return (unsigned)((groups + kGroupsPerBlock - 1) / kGroupsPerBlock); }
static inline size_t padded_groups(size_t groups) { return (size_t)grid_for(groups) * kGroupsPerBlock; }

// ---- launch wrappers (ctx stream) ----
static int launch_import(eg_ctx* c, const uint8_t* d_be, size_t n, uint32_t* d_out, uint8_t* d_ltp) {
  if (!n) return EG_OK;
  LAUNCH_F(c, k_import, dim3(grid_for(n)), c->d, d_be, (uint32_t)n, d_out, d_ltp);
  HIPCHK(hipGetLastError());
  return EG_OK;
}
static int launch_export(eg_ctx* c, const uint32_t* d_in, size_t n, uint8_t* d_be) {
  if (!n) return EG_OK;
  LAUNCH_F(c, k_export, dim3(grid_for(n)), c->d, d_in, (uint32_t)n, d_be);
  HIPCHK(hipGetLastError());
  return EG_OK;
}

// Compile a launch shape into k_pow's op program (eg_kernels.hpp, PowOp).  The order of the
// multiplies is the algorithm:
//   window     : table B^0..B^15 (14 MM); per exponent MSB-first 4-bit windows, 4 sq + 1 mul
//   comb       : y_k = B^(2^(52k)) (208 sq, kept in yout for gather jobs), the 32 subset
//                products (26 MM), per exponent 51 x (1 sq + 1 mul) from column digits
//   comb, v = 2: the chain also keeps B^(2^(52r+26)) (to 2^234), two subset tables (52 MM), per
//                exponent 25 x (1 sq + 2 mul): 26 MM fewer per pair when the chain is paid anyway
//   gather     : y_k = prod of the factor jobs' y_k (4 x (gather-1) MM instead of 208 sq)
//   resid      : the chain runs on to z = B^(2^256); w = B^c for the public c = 2^256 - q is the
//                product of the chain's B^(2^k) at c's set bits (kept in free table slots while
//                the chain passes them: popcount(c) - 1 MM, 5 for EG's c = 189), or a
//                left-to-right ladder when c has too many bits; both to rout (k_resid_check)
//   fixed base : radix-table windows of g / K per term; the first one loads instead of multiplying
static std::vector<uint32_t> pow_schedule(const MontConsts& H, const PowShape& S, const FbTab& f0, const FbTab& f1,
                                          MMCount* mm) {
  std::vector<uint32_t> v;
  MMCount n;
  auto op = [&](PowOp k, uint32_t arg = 0) {
    v.push_back(pow_op(k, arg));
    if (k == OP_SQR) n.sqr += 1;
    else if (k != OP_END && k <= kOpMulLast) n.mul += 1;
  };
  const bool comb = S.comb != 0;
  const uint32_t nb = comb ? comb_blocks(S.blocks) : 1u;  // Lim-Lee column blocks
  const uint32_t ch = comb_rows(S.rows), cw = comb_width(S.rows);  // rows, row width (bits)
  const uint32_t bw = comb ? comb_block_width(S.rows, S.blocks) : cw;  // columns per block (last may be shorter)
  if (S.has_base && !(comb && S.shared_comb)) {
    op(OP_LOAD_ONE);
    for (uint32_t t = 0; t < nb; ++t) op(OP_STORE_TBL, t << ch);
    op(OP_LOAD_BASE);
    op(OP_STORE_TBL, 1);
    if (!comb) {
      for (uint32_t k = 2; k < 16; ++k) {
        op(OP_MUL_BASE);
        op(OP_STORE_TBL, k);
      }
    } else {
      if (S.gather) {
        for (uint32_t k = 1; k < (uint32_t)kCombH; ++k) {
          op(OP_LOAD_GATHER, k - 1);
          for (uint32_t i = 1; i < S.gather; ++i) op(OP_MUL_GATHER, i << 2 | (k - 1));
          op(OP_STORE_TBL, 1u << k);
        }
      } else {
        // residue test: c's set bits k >= 1 take table-0 slots that are not comb bases (the
        // composite indices, free until the subset products below)
        std::vector<uint32_t> cslot(256, 0);
        bool chain_c = false;
        if (S.resid) {
          uint32_t pc = 0;
          for (uint32_t k = 1; k < H.qc_bits && k < 256; ++k) pc += (H.qc[k >> 5] >> (k & 31)) & 1u;
          chain_c = H.qc_bits <= 256 && pc <= std::min(16u, (1u << ch) - ch - 1u);
          for (uint32_t k = 1, nx = 3; chain_c && k < H.qc_bits; ++k) {
            if (!((H.qc[k >> 5] >> (k & 31)) & 1u)) continue;
            while ((nx & (nx - 1)) == 0) ++nx;  // skip the comb bases (powers of two)
            cslot[k] = nx++;
          }
        }
        // comb bases B^(2^(cw r + bw t)) -> slot t * 2^h + 2^r (the chain position of each)
        std::vector<uint32_t> bslot(257, 0);
        for (uint32_t r = 0; r < ch; ++r)
          for (uint32_t t = 0; t < nb; ++t) {
            const uint32_t pos = cw * r + bw * t;
            if (pos > 0 && pos <= 256) bslot[pos] = (t << ch) | (1u << r);
          }
        const uint32_t kend = S.resid ? 256u : (ch - 1) * cw + (nb - 1) * bw;
        for (uint32_t k = 1; k <= kend; ++k) {
          op(OP_SQR);
          if (bslot[k]) op(OP_STORE_TBL, bslot[k]);
          // gather powers y_r = B^(2^(52r)) for the contest jobs (their 5-row combs): kept by
          // the 5-row combs and by the verifier's selection jobs (resid) whatever their rows
          if ((ch == (uint32_t)kCombH || S.resid) && k % kCombW == 0 && k / kCombW < (uint32_t)kCombH)
            op(OP_STORE_Y, k / kCombW - 1);
          if (k < 256 && cslot[k]) op(OP_STORE_TBL, cslot[k]);
        }
        if (S.resid) {
          op(OP_STORE_R, 0);  // z = B^(2^256)
          if (chain_c) {
            bool first = true;
            if (H.qc[0] & 1u) { op(OP_LOAD_TBL, 1); first = false; }
            for (uint32_t k = 1; k < 256; ++k) {
              if (!cslot[k]) continue;
              op(first ? OP_LOAD_TBL : OP_MUL_TBL, cslot[k]);
              first = false;
            }
            if (first) op(OP_LOAD_ONE);
          } else {
            op(OP_LOAD_TBL, 1);
            for (int w = (int)H.qc_bits - 2; w >= 0; --w) {
              op(OP_SQR);
              if ((H.qc[w >> 5] >> (w & 31)) & 1u) op(OP_MUL_TBL, 1);
            }
          }
          op(OP_STORE_R, 1);  // w = B^c
        }
      }
      for (uint32_t t = 0; t < nb; ++t) {
        const uint32_t o = t << ch;
        for (uint32_t k = 3; k < (1u << ch); ++k) {
          if ((k & (k - 1)) == 0) continue;
          op(OP_LOAD_TBL, o + (k & (k - 1)));
          op(OP_MUL_TBL, o + (k & (0u - k)));
          op(OP_STORE_TBL, o + k);
        }
      }
    }
  }
  for (uint32_t o = 0; o < S.nout; ++o) {
    bool one = true;
    if (S.has_base) {
      op(OP_EXP, o);
      if (comb) {  // column w of block t is digit t * bw + w (OP_EXP); a short last block skips its missing columns
        op(OP_LOAD_COMB, bw - 1);
        for (uint32_t t = 1; t < nb; ++t)
          if (t * bw + bw - 1 < cw) op(OP_MUL_COMB, t * bw + bw - 1);
        for (int w = (int)bw - 2; w >= 0; --w) {
          op(OP_SQR);
          for (uint32_t t = 0; t < nb; ++t)
            if (t * bw + (uint32_t)w < cw) op(OP_MUL_COMB, t * bw + (uint32_t)w);
        }
      } else {
        op(OP_LOAD_WIN, o);
        for (uint32_t w = 1; w < S.exp_bytes * 2; ++w) {
          for (int i = 0; i < 4; ++i) op(OP_SQR);
          op(OP_MUL_WIN, w | o << 12);
        }
      }
      one = false;
    }
    for (uint32_t t = 0; t < S.nfb[o]; ++t) {
      const uint32_t tab = S.tab[o][t] ? 1u : 0u;
      const FbTab& T = tab ? f1 : f0;
      const uint32_t nw = S.fb_small[o][t] ? 1u : T.nwin;  // a scalar < 2^wbits needs window 0 only
      for (uint32_t kf = 0; kf < nw; ++kf) {
        op(one ? OP_LOAD_FB : OP_MUL_FB, fb_arg(o, t, tab, kf));
        one = false;
      }
    }
    if (one) op(OP_LOAD_ONE);
    op(OP_STORE_OUT, o);
  }
  op(OP_END);
#if !EG_SQR
  n.mul += n.sqr;  // squarings run the plain multiply schedule
  n.sqr = 0;
#endif
  if (mm) *mm = n;
  return v;
}

// The device copy of a shape's op program, compiled once per (shape, tables) and kept for
// the context's lifetime (a few dozen distinct shapes at most).
static int pow_schedule_dev(eg_ctx* c, const PowShape& S, const FbTab& f0, const FbTab& f1, const uint32_t** d_sched,
                            MMCount* mm) {
  std::string key((const char*)&S, sizeof(S));
  key.append((const char*)&f0.nwin, 4).append((const char*)&f1.nwin, 4);
  auto it = c->sched.find(key);
  if (it == c->sched.end()) {
    MMCount n;
    // fb_arg holds the window index in 8 bits: window_bits >= 4 gives at most 64 windows
    if (f0.nwin > 256 || f1.nwin > 256) return fail(EG_ERR_ARG, "fixed-base table has too many windows");
    std::vector<uint32_t> prog = pow_schedule(c->h, S, f0, f1, &n);
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, prog.size() * 4));
    HIPCHK(hipMemcpy(d, prog.data(), prog.size() * 4, hipMemcpyHostToDevice));
    it = c->sched.emplace(key, SchedBuf{(const uint32_t*)d, n}).first;
  }
  *d_sched = it->second.ptr;
  if (mm) *mm = it->second.mm;
  return EG_OK;
}

// Run a homogeneous batch of exponentiation jobs (device job records).
// yout (comb jobs, optional): y_1..y_4 of every job, (kCombH-1) device elements per job, kept for a
// later gather launch; ygat: the y_k array a gather launch (S.gather > 0) multiplies together.
// tail, tail2 (optional): up to two more independent job populations (shapes tail->S, tail2->S)
// appended to the LAST sub-launch so their short jobs fill that launch's tail (PowPart in
// eg_kernels.hpp).
// jobs per k_pow sub-launch (bounds the per-launch scratch: 32 or 64 comb entries per job)
constexpr size_t kPowMaxJobs = (size_t)1 << 18;
// jobs of a last sub-launch together with its tails that a caller may plan for (the verifier's
// beta head in launch 1): bounds that launch's scratch to ~21 GB of 40-KB comb tables
constexpr size_t kPowTailJobs = (size_t)1 << 19;

struct PowTail {
  PowShape S;
  const uint32_t* jobs;
  size_t njobs;
  uint32_t* yout;
  const uint32_t* ygat;
  uint32_t* rout;  // residue pairs (tail->S.resid)
  const uint32_t* ctab;  // shared comb table (tail->S.shared_comb)
};
static size_t pow_scratch_per_group(const PowShape& S) {
  return (S.has_base && !S.shared_comb) ? (size_t)(S.comb ? (comb_blocks(S.blocks) << comb_rows(S.rows)) : 16u) * kW * 4 : 4;
}
// ct = true: the constant-time instantiation k_pow<F, true> for secret exponents (comb shapes
// without fixed-base terms only); ctab: the shared comb table of S.shared_comb jobs.
// scratch (optional): the per-job table space of a batch of at most one workgroup and no tail
// (the caller keeps the tables, e.g. g's shared comb table; it must hold kGroupsPerBlock jobs'
// tables, since idle groups recompute the last job); default the W_SCR workspace.
static int launch_pow(eg_ctx* c, const PowShape& S, const uint32_t* d_jobs, size_t njobs, const uint32_t* d_elems,
                      const uint8_t* d_scal, uint32_t* d_out, FbTab f0, FbTab f1, uint32_t* yout = nullptr,
                      const uint32_t* ygat = nullptr, const PowTail* tail = nullptr, uint32_t* rout = nullptr,
                      bool ct = false, const uint32_t* ctab = nullptr, uint32_t* scratch = nullptr,
                      const PowTail* tail2 = nullptr) {
  if (tail && !tail->njobs) tail = nullptr;
  if (tail2 && !tail2->njobs) tail2 = nullptr;
  if (tail2 && !tail) std::swap(tail, tail2);
  if (scratch && (tail || njobs > kPowMaxJobs || njobs > kGroupsPerBlock))
    return fail(EG_ERR_ARG, "an explicit k_pow scratch takes one workgroup of jobs and no tail");
  // constant-time shapes: a comb or a 4-bit window (masked scans of their tables) without fixed-base
  // terms, or fixed-base terms alone from small-window tables (masked scans of 2^w-entry window columns)
  auto ct_shape = [&](const PowShape& X) {
    if (X.has_base) return !X.gather && !X.nfb[0] && !X.nfb[1];  // a comb or a 4-bit window
    return f0.wbits <= kCtMaxWindow && f1.wbits <= kCtMaxWindow;
  };
  // every population of the launch: its shape and the buffers it needs
  auto check = [&](const PowShape& X, const uint32_t* yg, const uint32_t* ro, const uint32_t* ct_tab) {
    if (X.resid && (!X.comb || X.gather || !ro)) return fail(EG_ERR_ARG, "residue pairs need a plain comb shape and rout");
    if (X.blocks > 1 && (X.blocks > 4 || !X.comb || X.gather || X.shared_comb))
      return fail(EG_ERR_ARG, "two to four column blocks need a plain comb shape");
    if (X.shared_comb && (!X.comb || X.gather || X.resid || !ct_tab)) return fail(EG_ERR_ARG, "shared comb table missing");
    if (X.rows && (X.rows != 4 || !X.comb || X.gather || X.shared_comb))
      return fail(EG_ERR_ARG, "4-row combs are plain comb shapes");
    if (ct && !ct_shape(X)) return fail(EG_ERR_ARG, "constant-time jobs are plain combs or small-window fixed-base terms");
    if (X.gather && (!X.comb || !yg)) return fail(EG_ERR_ARG, "gather launch needs a comb shape and y_k source");
    return (int)EG_OK;
  };
  int src = check(S, ygat, rout, ctab);
  if (!src && tail) src = check(tail->S, tail->ygat, tail->rout, tail->ctab);
  if (!src && tail2) src = check(tail2->S, tail2->ygat, tail2->rout, tail2->ctab);
  if (src) return src;
  if (!njobs && !tail) return EG_OK;
  const size_t per = pow_scratch_per_group(S);
  const size_t per1 = tail ? pow_scratch_per_group(tail->S) : 0;
  const size_t per2 = tail2 ? pow_scratch_per_group(tail2->S) : 0;
  // bound the per-launch scratch (table of 16/32 powers per job)
  const size_t max_jobs = kPowMaxJobs;
  MMCount mm_job, mm_tail, mm_tail2;
  const uint32_t *sched = nullptr, *sched_tail = nullptr, *sched_tail2 = nullptr;
  src = pow_schedule_dev(c, S, f0, f1, &sched, &mm_job);
  if (!src && tail) src = pow_schedule_dev(c, tail->S, f0, f1, &sched_tail, &mm_tail);
  if (!src && tail2) src = pow_schedule_dev(c, tail2->S, f0, f1, &sched_tail2, &mm_tail2);
  if (src) return src;
  size_t off = 0;
  do {
    const size_t nj = std::min(max_jobs, njobs - off);
    const bool last = off + nj >= njobs;
    const size_t nt = (last && tail) ? tail->njobs : 0;
    const size_t nt2 = (last && tail2) ? tail2->njobs : 0;
    uint32_t* scr = scratch;
    if (!scr) {
      const int rc = ws_get(c, W_SCR, padded_groups(nj) * per + padded_groups(nt) * per1 + padded_groups(nt2) * per2,
                            (void**)&scr);
      if (rc) return rc;
    }
    PowPart P0{S, sched, d_jobs + off * kJobWords, (uint32_t)nj, grid_for(nj), scr,
               yout ? yout + off * (kCombH - 1) * kW : nullptr, ygat, rout ? rout + off * 2 * kW : nullptr, ctab};
    PowPart P1{}, P2{};
    if (nt) {
      P1 = PowPart{tail->S, sched_tail, tail->jobs, (uint32_t)nt, grid_for(nt),
                   scr + padded_groups(nj) * per / 4, tail->yout, tail->ygat, tail->rout, tail->ctab};
    }
    if (nt2) {
      P2 = PowPart{tail2->S, sched_tail2, tail2->jobs, (uint32_t)nt2, grid_for(nt2),
                   scr + (padded_groups(nj) * per + padded_groups(nt) * per1) / 4, tail2->yout, tail2->ygat,
                   tail2->rout, tail2->ctab};
    }
    const dim3 grid(P0.nblocks + P1.nblocks + P2.nblocks);
    ProfRec* pr = nullptr;
    uint64_t* clk = nullptr;
    if (c->timing) {
      // the record joins the window before anything can fail, so profile_end / destroy free its events
      c->prof.push_back(ProfRec{nullptr, nullptr,
                                (mm_job.mul + mm_job.sqr) * (double)nj + (mm_tail.mul + mm_tail.sqr) * (double)nt +
                                    (mm_tail2.mul + mm_tail2.sqr) * (double)nt2,
                                mm_job.sqr * (double)nj + mm_tail.sqr * (double)nt + mm_tail2.sqr * (double)nt2});
      pr = &c->prof.back();
      HIPCHK(hipEventCreate(&pr->a));
      HIPCHK(hipEventCreate(&pr->b));
      if (c->d_clk && c->clk_used + grid.x <= kClockRecs) {  // else this launch goes unclocked
        clk = c->d_clk + 2 * c->clk_used;
        c->clk_used += grid.x;
      }
      HIPCHK(hipEventRecord(pr->a, c->stream));
    }
    if (c->h.friendly) {
      if (ct) hipLaunchKernelGGL((k_pow<true, true>), grid, dim3(kBlock), 0, c->stream, c->d, P0, P1, P2, d_elems, d_scal, d_out, f0, f1, clk);
      else hipLaunchKernelGGL((k_pow<true, false>), grid, dim3(kBlock), 0, c->stream, c->d, P0, P1, P2, d_elems, d_scal, d_out, f0, f1, clk);
    } else {
      if (ct) hipLaunchKernelGGL((k_pow<false, true>), grid, dim3(kBlock), 0, c->stream, c->d, P0, P1, P2, d_elems, d_scal, d_out, f0, f1, clk);
      else hipLaunchKernelGGL((k_pow<false, false>), grid, dim3(kBlock), 0, c->stream, c->d, P0, P1, P2, d_elems, d_scal, d_out, f0, f1, clk);
    }
    HIPCHK(hipGetLastError());
    if (pr) HIPCHK(hipEventRecord(pr->b, c->stream));
    off += nj;
  } while (off < njobs);
  return EG_OK;
}

// Product reduction of `groups` groups of `len` device elements (group layout gm,
// element stride `stride`); result -> d_out[g].  Fully asynchronous.
// mask (optional, len bytes): element k takes part only if mask[k] != 0 (first pass only).
static int run_prod(eg_ctx* c, const uint32_t* d_in, GroupMap gm, size_t groups, size_t len, size_t stride,
                    uint32_t* d_out, const uint8_t* mask = nullptr) {
  if (!groups) return EG_OK;
  if (len == 0) return fail(EG_ERR_ARG, "empty product");
  // Short products (contest aggregates, residue pairs: len = spc) run in one pass.  Long ones
  // (the tally: len = ballots) are a tree whose passes are chains of chunk-1 dependent
  // multiplies on a nearly idle GPU after the first pass, so a small fan-in wins: 8 gives
  // ~30 chained MMs for 10,000 ballots against ~71 with 32.
  const uint32_t chunk = len > 32 ? 8u : 32u;
  const size_t maxpart = groups * ((len + chunk - 1) / chunk);
  uint32_t* tmp = nullptr;
  int rc = ws_get(c, W_TMP, std::max<size_t>(1, maxpart) * kW * 4 * 2, (void**)&tmp);
  if (rc) return rc;
  uint32_t* ping[2] = {tmp, tmp + maxpart * kW};
  size_t cur_len = len, cur_stride = stride;
  const uint32_t* src = d_in;
  int pi = 0;
  while (true) {
    const uint32_t nchunk = (uint32_t)((cur_len + chunk - 1) / chunk);
    const uint32_t ch = nchunk == 1 ? (uint32_t)cur_len : chunk;
    uint32_t* dst = (nchunk == 1) ? d_out : ping[pi];
    const size_t njobs = groups * nchunk;
    LAUNCH_F(c, k_prod, dim3(grid_for(njobs)), c->d, src, gm, (uint32_t)groups,
                       (uint32_t)cur_len, (uint32_t)cur_stride, ch, nchunk, dst, mask);
    HIPCHK(hipGetLastError());
    if (nchunk == 1) break;
    mask = nullptr;  // later passes multiply partial products
    // next round: group g's partials are contiguous at g*nchunk
    gm = GroupMap{1, 1, 0, 0, nchunk};
    src = dst;
    cur_len = nchunk;
    cur_stride = 1;
    pi ^= 1;
  }
  return EG_OK;
}

// ---- fixed-base table build ----
static int build_fb(eg_ctx* c, const uint32_t* d_base_mont, int wbits, eg_fixed_base* fb) {
  const int nwin = (256 + wbits - 1) / wbits;
  const size_t entries = (size_t)nwin << wbits;
  HIPCHK(hipMalloc(&fb->d_tab, entries * kW * 4));
  fb->wbits = wbits;
  fb->nwin = nwin;
  // powers base^(2^j), j < nwin*wbits
  uint32_t* P = nullptr;
  const int npow = nwin * wbits;
  HIPCHK(hipMalloc(&P, (size_t)npow * kW * 4));
  LAUNCH_F(c, k_sqr_chain, dim3(1), c->d, d_base_mont, (uint32_t)npow, P);
  HIPCHK(hipGetLastError());
  // entries (k, 0) = one, (k, 2^a) = P[k*wbits + a]
  for (int k = 0; k < nwin; ++k) {
    uint32_t* row = fb->d_tab + ((size_t)k << wbits) * kW;
    HIPCHK(hipMemcpyAsync(row, c->d->one, kW * 4, hipMemcpyDeviceToDevice, c->stream));
    for (int a = 0; a < wbits; ++a)
      HIPCHK(hipMemcpyAsync(row + ((size_t)1 << a) * kW, P + (size_t)(k * wbits + a) * kW, kW * 4,
                            hipMemcpyDeviceToDevice, c->stream));
  }
  for (int a = 1; a < wbits; ++a) {
    const size_t njobs = (size_t)nwin * (((size_t)1 << a) - 1);
    LAUNCH_F(c, k_fb_level, dim3(grid_for(njobs)), c->d, fb->d_tab,
                       (uint32_t)wbits, (uint32_t)nwin, (uint32_t)a);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipFree(P));
  return EG_OK;
}

static int import_one(eg_ctx* c, const uint8_t be[512], uint32_t** d_mont_out) {
  uint8_t* d_be = nullptr;
  uint32_t* d_m = nullptr;
  HIPCHK(hipMalloc(&d_be, 512));
  HIPCHK(hipMalloc(&d_m, kW * 4));
  HIPCHK(hipMemcpyAsync(d_be, be, 512, hipMemcpyHostToDevice, c->stream));
  int rc = launch_import(c, d_be, 1, d_m, nullptr);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipFree(d_be));
  *d_mont_out = d_m;
  return EG_OK;
}

static int fb_create_locked(eg_ctx* c, const uint8_t base_be[512], int wbits, eg_fixed_base** out) {
  if (wbits < 4 || wbits > 22)
    return fail(EG_ERR_ARG, "window_bits must be in [4, 22]");
  uint32_t* d_m = nullptr;
  int rc = import_one(c, base_be, &d_m);
  if (rc) return rc;
  auto* fb = new eg_fixed_base();
  fb->ctx = c;
  std::memcpy(fb->base.data(), base_be, 512);
  rc = build_fb(c, d_m, wbits, fb);
  hipFree(d_m);
  if (rc) {
    delete fb;
    return rc;
  }
  *out = fb;
  return EG_OK;
}

extern "C" int eg_ctx_create(const uint8_t p_be[512], const uint8_t q_be[32], const uint8_t g_be[512], int device,
                             eg_ctx** out) {
  if (!p_be || !q_be || !g_be || !out) return fail(EG_ERR_ARG, "null argument");
  *out = nullptr;
  const Big p = be_to_words(p_be, 512);
  if ((p[0] & 1) == 0) return fail(EG_ERR_MODULUS, "p must be odd");
  if ((p[127] >> 31) == 0) return fail(EG_ERR_MODULUS, "p must be a 4096-bit modulus (top bit set)");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(EG_ERR_ARG, "bad device ordinal " + std::to_string(device));
  HIPCHK(hipSetDevice(device));
  auto* c = new eg_ctx();
  c->device = device;
  std::memcpy(c->p_be, p_be, 512);
  std::memcpy(c->q_be, q_be, 32);
  std::memcpy(c->g_be, g_be, 512);
  // Montgomery constants, R = 2^(kLimbBits * kSteps) (eg_bignum.hpp: 2^4118 at radix 2^29)
  Big P1 = p;
  P1.push_back(0);  // room for doubling
  Big r(129, 0);
  r[0] = 1;
  for (int i = 0; i < kSteps * kLimbBits; ++i) dbl_mod(r, P1);  // R mod p
  Big r2 = r;
  for (int i = 0; i < kSteps * kLimbBits; ++i) dbl_mod(r2, P1);  // R^2 mod p
  words_to_elem(p, c->h.p);
  words_to_elem(r2, c->h.r2);
  words_to_elem(r, c->h.one);
  Big unit(128, 0);
  unit[0] = 1;
  words_to_elem(unit, c->h.unit);
  for (int i = 0; i < 128; ++i) c->h.pw[i] = p[i];
  // n0 = -p^-1 mod 2^kLimbBits (Newton on 32 bits)
  uint32_t inv = 1;
  for (int i = 0; i < 6; ++i) inv *= 2u - p[0] * inv;
  c->h.n0 = (0u - inv) & kMask;
  c->h.friendly = c->h.n0 == 1 ? 1u : 0u;
  c->h.mask = kMask;
  {
    const char* lp = getenv("EG_LATENCY_POW");
    const std::string mode = lp ? lp : "";
    std::string err;
    if (mode != "0" && pow16_consts_create(p.data(), r2.data(), r.data(), c->h.n0, c->h.friendly, &c->lat, &err) == 0)
      c->lat_jobs = pow16_round_jobs(device) / 2;  // at 12,288 elements 16-lane groups ran 8.4 ms, 8-lane 7.3 (r04l)
    if (mode != "0" && mode != "16" &&
        powwave_consts_create(p.data(), r2.data(), r.data(), c->h.n0, c->h.friendly, &c->latw, &err) == 0) {
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess) {
        c->latw_jobs = (size_t)cus * 4;  // one element per SIMD
        c->r2l_max = (size_t)cus;        // one 4-wave job per CU
        c->w8_max = (size_t)cus;         // one 8-wave job per CU
      }
      if (const char* w8 = getenv("EG_WAVE_W8")) c->w8_max = (size_t)std::max(0L, atol(w8));
      if (const char* rl = getenv("EG_WAVE_R2L")) c->r2l_max = (size_t)std::max(0L, atol(rl));
      if (const char* zc = getenv("EG_COALESCE_ZC")) {
        const std::string z = zc;
        c->co_zc = z == "in" ? 1 : z == "out" ? 2 : z == "inout" ? 3 : 0;
      }
      c->wave_max = c->latw_jobs;
      if (const char* wm = getenv("EG_WAVE_MAX")) c->wave_max = (size_t)std::max(0L, atol(wm));
      if (const char* ws = getenv("EG_WAVE_SPLIT")) c->wave_split = ws[0] != '0';
    }
  }
  {  // c = 2^256 - q (mod 2^256) for the residue test x^(2^256) == x^c
    const Big q = be_to_words(q_be, 32);
    int64_t br = 0;
    for (int i = 0; i < 8; ++i) {
      br += -(int64_t)q[i];
      c->h.qc[i] = (uint32_t)br;
      br >>= 32;
    }
    c->h.qc_bits = 0;
    for (int b = 255; b >= 0; --b)
      if ((c->h.qc[b >> 5] >> (b & 31)) & 1u) { c->h.qc_bits = (uint32_t)b + 1; break; }
  }
  if (const char* nc = getenv("EG_NO_COMB")) c->use_comb = (nc[0] == '1') ? 0u : 1u;
  if (const char* cr = getenv("EG_CT_ROWS")) c->ct_rows = (cr[0] == '5') ? 0u : 4u;
  if (const char* sc = getenv("EG_SEL_COMB")) {
    c->sel_rows = (sc[0] == '5') ? 0u : 4u;
    c->sel_blocks = (sc[0] == '5') ? 2u : (sc[1] == '2' ? 2u : (sc[1] == '4' ? 4u : 3u));
  }
  if (const char* tf = getenv("EG_TEST_FAIL_JOBS")) c->test_fail_jobs = atoi(tf);
  if (const char* fl = getenv("EG_FB_LDS")) c->fb_lds = fl[0] == '1';
  if (const char* cw = getenv("EG_CT_WINDOW")) c->ct_window = std::max(4, std::min((int)kCtMaxWindow, atoi(cw)));
  {
    int cus = 0, per_cu = 0;
    const char* ts = getenv("EG_TAIL_SPLIT");
    if (!(ts && ts[0] == '0') && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pow<true, false>, kBlock, 0) == hipSuccess && per_cu > 0) {
      c->pow_slots = (size_t)cus * (size_t)per_cu;
      // waves per SIMD: per_cu workgroups of kBlock / 64 waves over a CU's 4 SIMDs (3 for k_pow)
      c->pow_wps = (uint32_t)std::max(1, per_cu * (kBlock / 64) / 4);
    }
  }
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(EG_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  auto setup = [&]() -> int {
    HIPCHK(hipMalloc(&c->d, sizeof(MontConsts)));
    HIPCHK(hipMemcpy(c->d, &c->h, sizeof(MontConsts), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&c->d_q, 32));
    HIPCHK(hipMemcpy(c->d_q, q_be, 32, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&c->d_qbar, 32));
    std::lock_guard<std::mutex> lk(c->mu);
    return fb_create_locked(c, g_be, 8, &c->gtab);
  };
  const int rc = setup();
  if (rc) {  // the ctx lock is released here; free whatever was allocated, keep the message
    const std::string msg = g_err;
    eg_ctx_destroy(c);
    return fail(rc, msg);
  }
  *out = c;
  return EG_OK;
}

extern "C" int eg_fixed_base_destroy(eg_fixed_base* fb) {
  if (!fb) return EG_OK;
  // jobs still queued on this table run first (the dispatcher needs no lock the caller holds: tables
  // the library destroys under the ctx lock are never queued while it is held)
  while (fb->queued.load(std::memory_order_acquire) > 0) std::this_thread::sleep_for(std::chrono::microseconds(20));
  if (fb->d_tab) hipFree(fb->d_tab);
  eg_fixed_base_destroy(fb->ct);
  delete fb;
  return EG_OK;
}

// The table a constant-time read of fb's base uses: fb itself when a masked scan of its window
// columns is affordable (wbits <= kCtMaxWindow), else its kCtEncWindow-bit companion, built once.
static int ct_table_locked(eg_ctx* c, eg_fixed_base* fb, FbTab* out) {
  if (fb->wbits <= (int)kCtMaxWindow) {
    *out = fb->tab();
    return EG_OK;
  }
  if (!fb->ct) {
    const int rc = fb_create_locked(c, fb->base.data(), kCtEncWindow, &fb->ct);
    if (rc) return rc;
  }
  *out = fb->ct->tab();
  return EG_OK;
}

static void coalescer_stop(eg_ctx* c);  // eg_capi_coalesce.inc
static int comm_destroy_locked(eg_ctx* c);  // eg_capi_comm.inc

extern "C" int eg_ctx_destroy(eg_ctx* c) {
  if (!c) return EG_OK;
  coalescer_stop(c);  // drains pending per-element calls first
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  comm_destroy_locked(c);
  eg_fixed_base_destroy(c->gtab);
  for (auto& k : c->keys) {
    eg_fixed_base_destroy(k.fb);
    eg_fixed_base_destroy(k.ct);
    if (k.d_K) hipFree(k.d_K);
  }
  eg_fixed_base_destroy(c->g_ct);
  for (auto& kv : c->share_keys) eg_fixed_base_destroy(kv.second);
  for (auto& b : c->ws)
    if (b.ptr) hipFree(b.ptr);
  for (auto& kv : c->cache)
    if (kv.second.ptr) hipFree(kv.second.ptr);
  for (auto& kv : c->sched) hipFree(const_cast<uint32_t*>(kv.second.ptr));
  for (auto& r : c->prof) {  // a profile window left open
    if (r.a) hipEventDestroy(r.a);
    if (r.b) hipEventDestroy(r.b);
  }
  if (c->d_clk) hipFree(c->d_clk);
  pow16_consts_destroy(c->lat);
  powwave_consts_destroy(c->latw);
  if (c->d) hipFree(c->d);
  if (c->d_q) hipFree(c->d_q);
  if (c->d_qbar) hipFree(c->d_qbar);
  if (c->d_gcomb) hipFree(c->d_gcomb);
  if (c->copy) {
    hipStreamSynchronize(c->copy);
    hipStreamDestroy(c->copy);
  }
  for (int i = 0; i < 2; ++i) {
    if (c->up_ev[i]) hipEventDestroy(c->up_ev[i]);
    if (c->done_ev[i]) hipEventDestroy(c->done_ev[i]);
  }
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return EG_OK;
}

extern "C" int eg_ctx_sync(eg_ctx* c) {
  if (!c) return fail(EG_ERR_ARG, "null ctx");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  return EG_OK;
}

extern "C" eg_fixed_base* eg_ctx_g_table(eg_ctx* c) { return c ? c->gtab : nullptr; }

extern "C" int eg_ctx_set_hash_format(eg_ctx* c, int format) {
  if (!c) return fail(EG_ERR_ARG, "null ctx");
  if (format != EG_HASH_FIXED_WIDTH && format != EG_HASH_MINIMAL) return fail(EG_ERR_ARG, "unknown hash format");
  std::lock_guard<std::mutex> lk(c->mu);
  c->hash_fmt = (uint32_t)format;
  return EG_OK;
}

extern "C" int eg_ctx_set_proof_format(eg_ctx* c, int response, int preimage) {
  if (!c) return fail(EG_ERR_ARG, "null ctx");
  if (response != EG_RESPONSE_MINUS && response != EG_RESPONSE_PLUS) return fail(EG_ERR_ARG, "unknown response convention");
  if (preimage < EG_PREIMAGE_MESSAGE_FIRST || preimage > EG_PREIMAGE_WITH_KEY)
    return fail(EG_ERR_ARG, "unknown pre-image order");
  std::lock_guard<std::mutex> lk(c->mu);
  c->resp_plus = response == EG_RESPONSE_PLUS ? 1u : 0u;
  c->pre_order = (uint32_t)preimage;
  return EG_OK;
}

extern "C" int eg_fixed_base_create(eg_ctx* c, const uint8_t base_be[512], int wbits, eg_fixed_base** out) {
  if (!c || !base_be || !out) return fail(EG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  return fb_create_locked(c, base_be, wbits, out);
}

// ------------------------------------------------------------------------------
// batched group ops (host buffers)
// ------------------------------------------------------------------------------
struct Locked {
  std::lock_guard<std::mutex> lk;
  explicit Locked(eg_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

static int upload(eg_ctx* c, Slot s, const void* h, size_t bytes, void** d) {
  int rc = ws_get(c, s, bytes, d);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(*d, h, bytes, hipMemcpyHostToDevice, c->stream));
  return EG_OK;
}

// Element and job indices are 32-bit on the device: one call takes at most 2^31 elements.
constexpr size_t kMaxBatch = (size_t)1 << 31;

static int pow_host(eg_ctx* c, const uint8_t* base_be, const uint8_t* exp_be, uint32_t exp_bytes, bool exp_shared,
                    uint8_t* out_be, size_t n, const FbTab* fbonly) {
  if (n > kMaxBatch) return fail(EG_ERR_ARG, "batch too large");
  uint8_t *d_base = nullptr, *d_exp = nullptr, *d_out = nullptr;
  uint32_t *d_e = nullptr, *d_o = nullptr, *d_jobs = nullptr;
  int rc;
  const size_t nexp = exp_shared ? 1 : n;
  if ((rc = upload(c, W_EXP, exp_be, nexp * exp_bytes, (void**)&d_exp))) return rc;
  PowShape S{};
  S.nout = 1;
  S.exp_bytes = exp_bytes;
  std::vector<uint32_t> jobs(n * kJobWords, kNone);
  for (size_t i = 0; i < n; ++i) {
    uint32_t* J = &jobs[i * kJobWords];
    J[0] = fbonly ? kNone : (uint32_t)i;
    J[1] = exp_shared ? 0u : (uint32_t)i;
    J[3] = (uint32_t)i;
    J[5] = (uint32_t)i;
  }
  if (fbonly) {
    S.has_base = 0;
    S.nfb[0] = 1;
    S.tab[0][0] = 0;
  } else {
    S.has_base = 1;
    if ((rc = upload(c, W_IN0, base_be, n * 512, (void**)&d_base))) return rc;
    if ((rc = ws_get(c, W_E0, n * kW * 4, (void**)&d_e))) return rc;
    if ((rc = launch_import(c, d_base, n, d_e, nullptr))) return rc;
  }
  if ((rc = upload(c, W_JOBS, jobs.data(), jobs.size() * 4, (void**)&d_jobs))) return rc;
  if ((rc = ws_get(c, W_E1, n * kW * 4, (void**)&d_o))) return rc;
  FbTab f0 = fbonly ? *fbonly : c->gtab->tab();
  // eg_ctx_set_ct_pow: the window / fixed-base schedule of k_pow<F, true> (a public exponent, the
  // inverse's p - 2, keeps the variable-time instantiation)
  const bool ct = c->ct_pow && exp_bytes == 32;
  if ((rc = launch_pow(c, S, d_jobs, n, d_e, d_exp, d_o, f0, f0, nullptr, nullptr, nullptr, nullptr, ct))) return rc;
  if ((rc = ws_get(c, W_OUT, n * 512, (void**)&d_out))) return rc;
  if ((rc = launch_export(c, d_o, n, d_out))) return rc;
  HIPCHK(hipMemcpyAsync(out_be, d_out, n * 512, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return EG_OK;
}

static bool latency_shaped(const eg_ctx* c, size_t n);  // eg_capi_coalesce.inc
static int pow_latency(eg_ctx* c, const uint8_t* base_be, const uint8_t* exp_be, uint8_t* out_be, size_t n);
static int fb_latency(eg_ctx* c, const FbTab& t, const uint8_t* exp_be, uint8_t* out_be, size_t n);

extern "C" int eg_powp_batch(eg_ctx* c, const uint8_t* base_be, const uint8_t* exp_be, uint8_t* out_be, size_t n) {
  if (!c || (n && (!base_be || !exp_be || !out_be))) return fail(EG_ERR_ARG, "null argument");
  if (!n) return EG_OK;
  Locked L(c);
  // small batches on the latency layouts: up to one element per SIMD one element per wave (1.7-1.8
  // against 3.7 ms on 8-lane groups), up to half a round 16-lane groups (3.2 against 3.8 ms at 4,096;
  // profiles/r04m_coalesce_shapes.json)
  if (latency_shaped(c, n)) return pow_latency(c, base_be, exp_be, out_be, n);
  return pow_host(c, base_be, exp_be, 32, false, out_be, n, nullptr);
}

extern "C" int eg_fb_pow_batch(eg_fixed_base* fb, const uint8_t* exp_be, uint8_t* out_be, size_t n) {
  if (!fb || (n && (!exp_be || !out_be))) return fail(EG_ERR_ARG, "null argument");
  if (!n) return EG_OK;
  eg_ctx* c = fb->ctx;
  Locked L(c);
  FbTab t = fb->tab();
  if (c->ct_pow) {
    const int rc = ct_table_locked(c, fb, &t);
    if (rc) return rc;
  }
  if (c->latw && n <= c->latw_jobs) return fb_latency(c, t, exp_be, out_be, n);  // one element per wave
  return pow_host(c, nullptr, exp_be, 32, false, out_be, n, &t);
}

static int multp_host(eg_ctx* c, const uint8_t* a_be, const uint8_t* b_be, uint8_t* out_be, size_t n);

// a^-1 mod p (BigInteger.modInverse; 0 -> 0).  The elements of a ballot record and a tally lie in the
// order-q subgroup, where a^-1 = a^(q-1): a 256-bit exponent instead of p - 2's 4096 bits (~16x fewer
// Montgomery operations).  Every candidate r is checked (r * a == 1 mod p, one multiply): the
// elements that fail -- outside the subgroup, or 0 -- take a^(p-2), so the result is the inverse for
// every input.
extern "C" int eg_multinv_batch(eg_ctx* c, const uint8_t* a_be, uint8_t* out_be, size_t n) {
  if (!c || (n && (!a_be || !out_be))) return fail(EG_ERR_ARG, "null argument");
  if (!n) return EG_OK;
  if (n > kMaxBatch) return fail(EG_ERR_ARG, "batch too large");
  Locked L(c);
  int rc;
  uint8_t eq[32];
  std::memcpy(eq, c->q_be, 32);
  for (int i = 31, borrow = 1; borrow && i >= 0; --i) {  // q - 1 (q is odd: only the low byte changes)
    borrow = eq[i] == 0;
    eq[i] = (uint8_t)(eq[i] - 1);
  }
  if (latency_shaped(c, n)) {  // a few elements (a per-element multInv): the latency layouts
    std::vector<uint8_t> es(n * 32);
    for (size_t k = 0; k < n; ++k) std::memcpy(&es[k * 32], eq, 32);
    if ((rc = pow_latency(c, a_be, es.data(), out_be, n))) return rc;
  } else if ((rc = pow_host(c, a_be, eq, 32, true, out_be, n, nullptr))) {
    return rc;
  }
  std::vector<uint8_t> chk(n * 512);
  if ((rc = multp_host(c, a_be, out_be, chk.data(), n))) return rc;
  std::vector<size_t> redo;
  for (size_t k = 0; k < n; ++k) {
    const uint8_t* v = &chk[k * 512];
    bool one = v[511] == 1;
    for (int i = 0; i < 511 && one; ++i) one = v[i] == 0;
    if (!one) redo.push_back(k);
  }
  if (redo.empty()) return EG_OK;
  // a^(p-2) for the rest: p is odd and > 2, so subtracting 2 only touches the low word(s)
  uint8_t e[512];
  std::memcpy(e, c->p_be, 512);
  int i = 511;
  uint32_t borrow = 2;
  while (borrow && i >= 0) {
    const uint32_t v = e[i];
    e[i] = (uint8_t)(v - borrow);
    borrow = v < borrow ? 1 : 0;
    --i;
  }
  std::vector<uint8_t> in(redo.size() * 512), out(redo.size() * 512);
  for (size_t k = 0; k < redo.size(); ++k) std::memcpy(&in[k * 512], a_be + redo[k] * 512, 512);
  if ((rc = pow_host(c, in.data(), e, 512, true, out.data(), redo.size(), nullptr))) return rc;
  for (size_t k = 0; k < redo.size(); ++k) std::memcpy(out_be + redo[k] * 512, &out[k * 512], 512);
  return EG_OK;
}

extern "C" int eg_multp_batch(eg_ctx* c, const uint8_t* a_be, const uint8_t* b_be, uint8_t* out_be, size_t n) {
  if (!c || (n && (!a_be || !b_be || !out_be))) return fail(EG_ERR_ARG, "null argument");
  if (!n) return EG_OK;
  if (n > kMaxBatch) return fail(EG_ERR_ARG, "batch too large");
  Locked L(c);
  return multp_host(c, a_be, b_be, out_be, n);
}

static int multp_host(eg_ctx* c, const uint8_t* a_be, const uint8_t* b_be, uint8_t* out_be, size_t n) {
  uint8_t *d_a = nullptr, *d_b = nullptr, *d_out = nullptr;
  uint32_t *ea = nullptr, *eb = nullptr;
  int rc;
  if ((rc = upload(c, W_IN0, a_be, n * 512, (void**)&d_a))) return rc;
  if ((rc = upload(c, W_IN1, b_be, n * 512, (void**)&d_b))) return rc;
  if ((rc = ws_get(c, W_E0, n * kW * 4, (void**)&ea))) return rc;
  if ((rc = ws_get(c, W_E1, n * kW * 4, (void**)&eb))) return rc;
  if ((rc = launch_import(c, d_a, n, ea, nullptr))) return rc;
  if ((rc = launch_import(c, d_b, n, eb, nullptr))) return rc;
  LAUNCH_F(c, k_mul, dim3(grid_for(n)), c->d, ea, 1u, eb, 1u, (uint32_t)n, ea, 1u);
  HIPCHK(hipGetLastError());
  if ((rc = ws_get(c, W_OUT, n * 512, (void**)&d_out))) return rc;
  if ((rc = launch_export(c, ea, n, d_out))) return rc;
  HIPCHK(hipMemcpyAsync(out_be, d_out, n * 512, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return EG_OK;
}

extern "C" int eg_prod_reduce(eg_ctx* c, const uint8_t* elems_be, size_t groups, size_t len, uint8_t* out_be) {
  if (!c || (groups && (!elems_be || !out_be))) return fail(EG_ERR_ARG, "null argument");
  if (!groups) return EG_OK;
  Locked L(c);
  if (len == 0) {
    // empty product = 1
    std::memset(out_be, 0, groups * 512);
    for (size_t g = 0; g < groups; ++g) out_be[g * 512 + 511] = 1;
    return EG_OK;
  }
  if (groups > kMaxBatch || len > kMaxBatch || groups * len > kMaxBatch) return fail(EG_ERR_ARG, "batch too large");
  const size_t n = groups * len;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  uint32_t *e = nullptr, *o = nullptr;
  int rc;
  if ((rc = upload(c, W_IN0, elems_be, n * 512, (void**)&d_in))) return rc;
  if ((rc = ws_get(c, W_E0, n * kW * 4, (void**)&e))) return rc;
  if ((rc = launch_import(c, d_in, n, e, nullptr))) return rc;
  if ((rc = ws_get(c, W_E1, groups * kW * 4, (void**)&o))) return rc;
  if ((rc = run_prod(c, e, GroupMap{1, 1, 0, 0, (uint32_t)len}, groups, len, 1, o))) return rc;
  if ((rc = ws_get(c, W_OUT, groups * 512, (void**)&d_out))) return rc;
  if ((rc = launch_export(c, o, groups, d_out))) return rc;
  HIPCHK(hipMemcpyAsync(out_be, d_out, groups * 512, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return EG_OK;
}

// In-kernel clock of a profile window (MI355X_MICROARCH.md 'DVFS give-back' item 6): each record
// is one workgroup's (s_memtime ticks, s_memrealtime ticks), the latter at a fixed 100 MHz; the
// clock is the MEDIAN of the per-workgroup ratios.  Records that are unset (0), wrapped (a
// negative difference reads as >= 2^63), shorter than 10 us (too coarse at 100 MHz) or whose
// ratio lies outside [0.5, 3.5] GHz are dropped and counted; a window with no usable record
// yields 0 GHz.  Summing raw ticks instead lets one garbage record dominate the result.
extern "C" int eg_clock_median(const uint64_t* recs, size_t n, double* ghz, uint32_t* used, uint32_t* dropped) {
  if ((n && !recs) || !ghz) return fail(EG_ERR_ARG, "null argument");
  std::vector<double> r;
  r.reserve(n);
  uint32_t drop = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t cyc = recs[2 * i], rt = recs[2 * i + 1];
    if (cyc == 0 || rt < 1000 || cyc >> 62 || rt >> 62) {
      ++drop;
      continue;
    }
    const double g = (double)cyc / (double)rt * 0.1;  // GHz: ticks per 10 ns real-time tick / 10
    if (!(g >= 0.5 && g <= 3.5)) {
      ++drop;
      continue;
    }
    r.push_back(g);
  }
  *ghz = 0;
  if (!r.empty()) {
    const size_t m = r.size() / 2;
    std::nth_element(r.begin(), r.begin() + m, r.end());
    double med = r[m];
    if (r.size() % 2 == 0) med = 0.5 * (med + *std::max_element(r.begin(), r.begin() + m));
    *ghz = med;
  }
  if (used) *used = (uint32_t)r.size();
  if (dropped) *dropped = drop;
  return EG_OK;
}

static void prof_clear(eg_ctx* c) {
  for (auto& r : c->prof) {
    if (r.a) hipEventDestroy(r.a);
    if (r.b) hipEventDestroy(r.b);
  }
  c->prof.clear();
}

extern "C" int eg_ctx_profile_begin(eg_ctx* c) {
  if (!c) return fail(EG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));  // a pending window's launches may still write the records
  prof_clear(c);
  if (!c->d_clk) HIPCHK(hipMalloc(&c->d_clk, kClockRecs * 2 * sizeof(uint64_t)));
  HIPCHK(hipMemsetAsync(c->d_clk, 0, kClockRecs * 2 * sizeof(uint64_t), c->stream));
  c->clk_used = 0;
  c->timing = true;
  return EG_OK;
}

extern "C" int eg_ctx_profile_clock(eg_ctx* c, double* ghz, uint32_t* used, uint32_t* dropped) {
  if (!c || !ghz) return fail(EG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(c->mu);
  *ghz = c->prof_clock_ghz;
  if (used) *used = c->clk_used_last;
  if (dropped) *dropped = c->clk_dropped_last;
  return EG_OK;
}

extern "C" int eg_ctx_profile_end(eg_ctx* c, double* ms, double* mm, double* sqr, int* launches) {
  if (!c) return fail(EG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  double t = 0, m = 0, sq = 0;
  for (auto& r : c->prof) {
    float x = 0;
    HIPCHK(hipEventElapsedTime(&x, r.a, r.b));
    t += x;
    m += r.mm;
    sq += r.sqr;
  }
  c->prof_clock_ghz = 0;
  c->clk_used_last = c->clk_dropped_last = 0;
  if (c->d_clk && c->clk_used) {
    std::vector<uint64_t> h(c->clk_used * 2);
    HIPCHK(hipMemcpy(h.data(), c->d_clk, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    eg_clock_median(h.data(), c->clk_used, &c->prof_clock_ghz, &c->clk_used_last, &c->clk_dropped_last);
    if (c->clk_dropped_last && getenv("EG_DEBUG_CLK"))
      fprintf(stderr, "eg_ctx_profile_end: %u of %zu workgroup clock records dropped\n", c->clk_dropped_last,
              c->clk_used);
  }
  if (ms) *ms = t;
  if (mm) *mm = m;
  if (sqr) *sqr = sq;
  if (launches) *launches = (int)c->prof.size();
  prof_clear(c);
  c->clk_used = 0;
  c->timing = false;
  return EG_OK;
}

#include "eg_capi_ballot.inc"
#include "eg_capi_coalesce.inc"
#include "eg_capi_comm.inc"

// ------------------------------------------------------------------------------
// device-pointer powP / fixed-base powP (asynchronous on the ctx stream): the
// resident-operand form of eg_powp_batch / eg_fb_pow_batch for callers that keep
// elements in HBM across calls (the modexp microbenchmark).  The
// identity job table of a batch size is built once and cached like the verify tables.
// ------------------------------------------------------------------------------
static int identity_pow_jobs(eg_ctx* c, size_t n, bool fbonly, const uint32_t** out) {
  const std::string key = std::string(fbonly ? "fb/" : "pw/") + std::to_string(n);
  if (c->cache.find(key) == c->cache.end()) {
    int rc = cache_bound(c);
    if (rc) return rc;
    auto jobs = new_jobs(n);
    for (size_t i = 0; i < n; ++i) {
      uint32_t* J = &jobs[i * kJobWords];
      J[0] = fbonly ? kNone : (uint32_t)i;
      J[1] = (uint32_t)i;
      J[3] = (uint32_t)i;
      J[5] = (uint32_t)i;
    }
    return cached_jobs(c, key, jobs, out);
  }
  *out = (const uint32_t*)c->cache[key].ptr;
  return EG_OK;
}

static int pow_dev(eg_ctx* c, const uint8_t* d_base_be, const uint8_t* d_exp_be, uint8_t* d_out_be, size_t n,
                   const FbTab* fbonly) {
  if (n > kMaxBatch) return fail(EG_ERR_ARG, "batch too large");
  const uint32_t* d_jobs = nullptr;
  uint32_t *d_e = nullptr, *d_o = nullptr;
  int rc;
  if ((rc = identity_pow_jobs(c, n, fbonly != nullptr, &d_jobs))) return rc;
  PowShape S{};
  S.nout = 1;
  S.exp_bytes = 32;
  if (fbonly) {
    S.nfb[0] = 1;
    S.tab[0][0] = 0;
  } else {
    S.has_base = 1;
    if ((rc = ws_get(c, W_E0, n * kW * 4, (void**)&d_e))) return rc;
    if ((rc = launch_import(c, d_base_be, n, d_e, nullptr))) return rc;
  }
  if ((rc = ws_get(c, W_E1, n * kW * 4, (void**)&d_o))) return rc;
  FbTab f0 = fbonly ? *fbonly : c->gtab->tab();
  if ((rc = launch_pow(c, S, d_jobs, n, d_e, d_exp_be, d_o, f0, f0, nullptr, nullptr, nullptr, nullptr, c->ct_pow != 0)))
    return rc;
  return launch_export(c, d_o, n, d_out_be);
}

extern "C" int eg_powp_batch_dev(eg_ctx* c, const uint8_t* d_base_be, const uint8_t* d_exp_be, uint8_t* d_out_be,
                                 size_t n) {
  if (!c || (n && (!d_base_be || !d_exp_be || !d_out_be))) return fail(EG_ERR_ARG, "null argument");
  if (!n) return EG_OK;
  Locked L(c);
  return pow_dev(c, d_base_be, d_exp_be, d_out_be, n, nullptr);
}

// A/B only (EG_FB_LDS=1, a 7-bit table, variable time): the batch-major LDS-staged kernel k_fb_lds
static int fb_lds_dev(eg_ctx* c, const FbTab& t, const uint8_t* d_exp_be, uint8_t* d_out_be, size_t n) {
  if (n > kMaxBatch) return fail(EG_ERR_ARG, "batch too large");
  uint32_t* d_o = nullptr;
  int rc;
  if ((rc = ws_get(c, W_E1, n * kW * 4, (void**)&d_o))) return rc;
  const dim3 grid((unsigned)((n + kLdsGroups - 1) / kLdsGroups));
  if (c->h.friendly)
    hipLaunchKernelGGL(k_fb_lds<true>, grid, dim3(kLdsBlock), 0, c->stream, c->d, t.data, t.nwin, d_exp_be, (uint32_t)n, d_o);
  else
    hipLaunchKernelGGL(k_fb_lds<false>, grid, dim3(kLdsBlock), 0, c->stream, c->d, t.data, t.nwin, d_exp_be, (uint32_t)n, d_o);
  HIPCHK(hipGetLastError());
  return launch_export(c, d_o, n, d_out_be);
}

extern "C" int eg_fb_pow_batch_dev(eg_fixed_base* fb, const uint8_t* d_exp_be, uint8_t* d_out_be, size_t n) {
  if (!fb || (n && (!d_exp_be || !d_out_be))) return fail(EG_ERR_ARG, "null argument");
  if (!n) return EG_OK;
  eg_ctx* c = fb->ctx;
  Locked L(c);
  FbTab t = fb->tab();
  if (!c->ct_pow && fb->wbits == kLdsWin && c->fb_lds) return fb_lds_dev(c, t, d_exp_be, d_out_be, n);
  if (c->ct_pow) {
    const int rc = ct_table_locked(c, fb, &t);
    if (rc) return rc;
  }
  return pow_dev(c, nullptr, d_exp_be, d_out_be, n, &t);
}
