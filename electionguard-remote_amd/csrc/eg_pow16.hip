// eg_pow16.hip — the latency-shaped instantiation of the device core: the same kernels as the
// throughput path (eg_kernels.hpp: k_import, the op-program k_pow, k_export) compiled with 16 lanes
// per element (EG_T = 16) in namespace eg16.  A 4096-bit exponentiation is ~330 Montgomery
// operations in sequence; an 8-lane group runs each in ~12 us (L = 18 limbs per lane: 142 CIOS
// steps of 36 MACs + glue), a 16-lane group in about half (L = 9, and the quotient broadcast is one
// row_newbcast move), so a batch that fits one resident round finishes in about half the time.
// That is what a blocking per-element caller waits for (eg_capi_coalesce.inc); large batches keep
// the 8-lane layout, which does ~12% more work per lane-cycle.  See eg_pow16.h.
#define EG_T 16
#define eg eg16
#include "eg_kernels.hpp"
#undef eg

#pragma clang diagnostic ignored "-Wunused-value"
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "eg_pow16.h"

using namespace eg16;

struct Pow16Consts {
  MontConsts* d = nullptr;
};

// little-endian 32-bit words -> the 16-lane device element (radix 2^29 limbs, padded lane blocks)
static void words_to_elem16(const uint32_t* w, int nw, uint32_t* out) {
  std::memset(out, 0, sizeof(uint32_t) * kW);
  for (int a = 0; a < kN; ++a) {
    const int bit = a * kLimbBits;
    uint64_t v = 0;
    for (int k = 0; k < 2; ++k) {  // bit % 32 + 29 <= 60: two words hold the limb (a shift by 64 would be UB)
      const int wi = bit / 32 + k;
      if (wi < nw) v |= (uint64_t)w[wi] << (32 * k);
    }
    out[(a / kL) * kLP + (a % kL)] = (uint32_t)(v >> (bit % 32)) & kMask;
  }
}

int pow16_consts_create(const uint32_t* p, const uint32_t* r2, const uint32_t* one, uint32_t n0, uint32_t friendly,
                        Pow16Consts** out, std::string* err) {
  MontConsts h{};
  words_to_elem16(p, 128, h.p);
  words_to_elem16(r2, 129, h.r2);
  words_to_elem16(one, 129, h.one);
  const uint32_t unit[1] = {1};
  words_to_elem16(unit, 1, h.unit);
  std::memcpy(h.pw, p, sizeof(h.pw));
  h.n0 = n0;
  h.friendly = friendly;
  h.mask = kMask;
  auto* c = new Pow16Consts();
  hipError_t e = hipMalloc(&c->d, sizeof(MontConsts));
  if (e == hipSuccess) e = hipMemcpy(c->d, &h, sizeof(MontConsts), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (c->d) hipFree(c->d);
    delete c;
    *err = std::string("pow16 constants: ") + hipGetErrorString(e);
    return 1;
  }
  *out = c;
  return 0;
}

void pow16_consts_destroy(Pow16Consts* c) {
  if (!c) return;
  if (c->d) hipFree(c->d);
  delete c;
}

size_t pow16_elem_bytes() { return (size_t)kW * 4; }

static size_t padded16(size_t n) { return (n + kGroupsPerBlock - 1) / kGroupsPerBlock * kGroupsPerBlock; }

size_t pow16_scratch_bytes(size_t n) { return padded16(n) * 16 * (size_t)kW * 4; }

size_t pow16_round_jobs(int device) {
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pow<true, false>, kBlock, 0) != hipSuccess)
    return 0;
  return (size_t)cus * (size_t)per_cu * kGroupsPerBlock;
}

int pow16_powp(const Pow16Consts* C, bool friendly, bool ct, hipStream_t s, const uint32_t* sched, const uint32_t* jobs,
               const uint8_t* base_be, const uint8_t* exp_be, uint8_t* out_be, size_t n, uint32_t* elems,
               uint32_t* outs, uint32_t* scratch, std::string* err) {
  if (!n) return 0;
  const unsigned grid = (unsigned)((n + kGroupsPerBlock - 1) / kGroupsPerBlock);
  PowShape S{};
  S.has_base = 1;
  S.nout = 1;
  S.exp_bytes = 32;
  PowPart P0{S, sched, jobs, (uint32_t)n, grid, scratch, nullptr, nullptr, nullptr, nullptr};
  PowPart none{};
  const FbTab nofb{nullptr, 0, 0};
  if (friendly) {
    hipLaunchKernelGGL(k_import<true>, dim3(grid), dim3(kBlock), 0, s, C->d, base_be, (uint32_t)n, elems, nullptr);
    if (ct)
      hipLaunchKernelGGL((k_pow<true, true>), dim3(grid), dim3(kBlock), 0, s, C->d, P0, none, none, elems, exp_be, outs,
                         nofb, nofb, nullptr);
    else
      hipLaunchKernelGGL((k_pow<true, false>), dim3(grid), dim3(kBlock), 0, s, C->d, P0, none, none, elems, exp_be, outs,
                         nofb, nofb, nullptr);
    hipLaunchKernelGGL(k_export<true>, dim3(grid), dim3(kBlock), 0, s, C->d, outs, (uint32_t)n, out_be);
  } else {
    hipLaunchKernelGGL(k_import<false>, dim3(grid), dim3(kBlock), 0, s, C->d, base_be, (uint32_t)n, elems, nullptr);
    if (ct)
      hipLaunchKernelGGL((k_pow<false, true>), dim3(grid), dim3(kBlock), 0, s, C->d, P0, none, none, elems, exp_be,
                         outs, nofb, nofb, nullptr);
    else
      hipLaunchKernelGGL((k_pow<false, false>), dim3(grid), dim3(kBlock), 0, s, C->d, P0, none, none, elems, exp_be,
                         outs, nofb, nofb, nullptr);
    hipLaunchKernelGGL(k_export<false>, dim3(grid), dim3(kBlock), 0, s, C->d, outs, (uint32_t)n, out_be);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = std::string("pow16 launch: ") + hipGetErrorString(e);
    return 1;
  }
  return 0;
}

// =================================================================================================
// One element per wave (egw): the latency shape for the smallest per-element batches.
//   * 144 limbs of 2^29 over lanes 0-47, three per lane (lane l holds limbs 3l .. 3l+2), lanes
//     48-63 hold zeros in x, y, p and the accumulator, so every lane runs the same code and the
//     idle ones only ever pass zeros (the shift into lane 47 reads lane 48's zero, the final carry
//     out of lane 47 is zero because the result is < 2p < R);
//   * CIOS as eg_bignum.hpp's mont_mul_impl (the same rotating accumulator registers and the same
//     split of the lowest column), but the quotient digit is ONE v_readlane of lane 0 (the whole
//     wave is one element: no DPP broadcast), the multiplier digit y_s is a v_readlane of the lane
//     that holds it, and the limb shift a wave_shl:1 DPP move;
//   * the exponent is read by the whole wave (one element per wave), so a 5-bit sliding window
//     (16 odd powers in LDS, ~314 Montgomery operations per 256-bit exponent against 329 for the
//     fixed 4-bit window) keeps every branch wave-uniform.
// =================================================================================================
namespace egw {
constexpr int kBits = 29, kLimbs = 144, kLL = 3, kLanes = 48, kRow = 64 * kLL;
constexpr uint32_t kM = (1u << kBits) - 1u;
static_assert(kLanes * kLL == kLimbs, "48 lanes x 3 limbs");
// the Montgomery domain of eg_bignum.hpp (R = 2^(29 * kSteps), 142 steps): limbs 142 and 143 of every
// operand are zero, so the multiply stops two steps early; the result then sits at rotation kRot
constexpr int kSteps = eg16::kSteps, kSkip = kLimbs - kSteps, kRot = kSteps % kLL;
constexpr int kTrips = kSteps / kLL, kRem = kSteps % kLL;  // 47 full trips of 3 steps + 1 step
static_assert(kSkip >= 0 && kSkip < kLL && kSteps * kBits >= 4098, "Montgomery R must exceed 4p");

struct Consts {
  uint32_t p[kRow], r2[kRow], one[kRow];  // limb i at [i], zeros from 144 on
  // p + 1 with its limbs shifted down by 2 (pd) and by 1 (pd1): the delayed-quotient multiply
  uint32_t pd[kRow], pd1[kRow];
  uint32_t n0;
  uint32_t mask;  // 2^29 - 1, read at run time so the AND folds into the DPP limb shift (v_and_b32_dpp)
};

__device__ __forceinline__ uint32_t lane64() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t wnext(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x130 /*wave_shl:1*/, 0xF, 0xF, true); }
__device__ __forceinline__ uint32_t wprev(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x138 /*wave_shr:1*/, 0xF, 0xF, true); }

// x <- x * y * R^-1 mod p (R = 2^4118: kSteps = 142 steps), result < 2p with limbs < 2^29 + small; y may alias x
template <bool F>
__device__ __forceinline__ void mul(uint32_t (&x)[kLL], const uint32_t (&y)[kLL], const uint32_t (&p)[kLL], uint32_t n0,
                                    uint32_t mv) {
  uint64_t acc[kLL] = {0, 0, 0};
  // kSteps steps: full trips in the loop (multiplier limbs 3q .. 3q+2 live in lane q), then the last
  // trip's first kLL - kSkip steps
  auto trip = [&](const int q, auto NR) {
    constexpr int nr = decltype(NR)::value;
#pragma unroll
    for (int r = 0; r < nr; ++r) {
      const uint32_t yi = __builtin_amdgcn_readlane(y[r], q);
#pragma unroll
      for (int j = 0; j < kLL; ++j) {
        uint64_t& A = acc[(j + r) % kLL];
        A = (uint64_t)x[j] * yi + A;
      }
      uint32_t t0 = __builtin_amdgcn_readlane((uint32_t)acc[r], 0);  // the lowest column (lane 0)
      if (!F) t0 *= n0;
      const uint32_t m = t0 & kM;
#pragma unroll
      for (int j = 0; j < kLL; ++j) {
        uint64_t& A = acc[(j + r) % kLL];
        A = (uint64_t)p[j] * m + A;
      }
      uint64_t& A0 = acc[r];
      acc[(r + 1) % kLL] += A0 >> kBits;         // the carry stays in this lane's next column
      A0 = (uint64_t)(wnext((uint32_t)A0) & mv);  // the low bits move to the lane below's top column
    }
  };
  constexpr int kFullTrips = kSkip ? kLanes - 1 : kLanes;
#pragma unroll 1
  for (int q = 0; q < kFullTrips; ++q) trip(q, std::integral_constant<int, kLL>{});
  if constexpr (kSkip > 0) trip(kLanes - 1, std::integral_constant<int, kLL - kSkip>{});
  // two carry passes (limb j of the result is register (kRot + j) % 3: 142 steps = 47 x 3 + 1)
  uint64_t d[kLL];
  {
    const uint64_t top = acc[(kRot + kLL - 1) % kLL] >> kBits;
    const uint64_t c_in = (uint64_t)wprev((uint32_t)top) | ((uint64_t)wprev((uint32_t)(top >> 32)) << 32);
#pragma unroll
    for (int j = 0; j < kLL; ++j)
      d[j] = (uint64_t)((uint32_t)acc[(kRot + j) % kLL] & kM) + (j == 0 ? c_in : (acc[(kRot + j - 1) % kLL] >> kBits));
  }
  const uint32_t c_in = wprev((uint32_t)(d[kLL - 1] >> kBits));
#pragma unroll
  for (int j = 0; j < kLL; ++j) x[j] = ((uint32_t)d[j] & kM) + (j == 0 ? c_in : (uint32_t)(d[j - 1] >> kBits));
}

// The same product for p = -1 mod 2^58 (both production groups: p = -1 mod 2^256), with the quotient
// digit off the step's dependency chain.  With p~ = p + 1 (limbs 0 and 1 zero), m*p = m*p~ - m, and the
// "- m" is the retiring column's low 29 bits (= m), which the wave_shl drops anyway; m_i * p~_j lands in
// column i + j >= i + 2, so it is applied two steps late (m_{i-2} against p~ shifted down by two limbs,
// pd) and never feeds the next quotient's column: each step's chain is the lowest column's
// MAC -> carry shift -> add, the readlane of the quotient runs beside it.  The quotient digits are the
// standard CIOS ones (the m-terms of columns < i + 8 telescope to multiples of 2^29 for this p), so
// the result is the same integer as mul<true>.  The last two digits are applied after the loop.
// The multiplier's digits reach the MACs as LDS broadcasts (the wave's own copy of y, read a trip
// ahead, two register sets in turn) instead of one v_readlane per step.
__device__ __forceinline__ void mul_d2(uint32_t (&x)[kLL], const uint32_t (&y)[kLL], const uint32_t (&pd)[kLL],
                                       const uint32_t (&pd1)[kLL], uint32_t mv) {
  __shared__ __align__(16) uint32_t s_yb[8][kRow + 8];  // per wave of the workgroup (W <= 8)
  uint32_t* yb = s_yb[threadIdx.x >> 6];
  const uint32_t ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  __builtin_amdgcn_wave_barrier();  // the previous multiply's reads of yb are done (in-order LDS)
#pragma unroll
  for (int j = 0; j < kLL; ++j) yb[kLL * ln + j] = y[j];
  __builtin_amdgcn_wave_barrier();
  uint64_t acc[kLL] = {0, 0, 0};
  uint32_t m1 = 0, m2 = 0;  // quotient digits of the previous two steps
  // one CIOS step at rotation R (a compile-time constant) with multiplier digit yi
  auto step = [&](auto R, const uint32_t yi) {
    constexpr int r = decltype(R)::value;
#pragma unroll
    for (int j = 0; j < kLL; ++j) {
      uint64_t& A = acc[(j + r) % kLL];
      A = (uint64_t)x[j] * yi + A;
    }
    // keep one v_mad_u64_u32 per product: without the barrier the compiler re-associates the
    // early-known m2 terms into separate products plus 64-bit adds (r04h: 25% slower)
#pragma unroll
    for (int j = 0; j < kLL; ++j) asm volatile("" : "+v"(acc[j]));
    asm volatile("" : "+s"(m2));  // a 32-bit SGPR: otherwise the loop carries it widened to 64 bits (two MACs)
#pragma unroll
    for (int j = 0; j < kLL; ++j) {
      uint64_t& A = acc[(j + r) % kLL];
      A = (uint64_t)pd[j] * m2 + A;
    }
    uint64_t& A0 = acc[r];
    const uint32_t m = __builtin_amdgcn_readlane((uint32_t)A0, 0) & kM;
    acc[(r + 1) % kLL] += A0 >> kBits;
    A0 = (uint64_t)(wnext((uint32_t)A0) & mv);
    m2 = m1;
    m1 = m;
  };
  // three CIOS steps with the multiplier digits yc (limbs 3q .. 3q + 2)
  auto steps = [&](const uint32_t (&yc)[kLL]) {
    step(std::integral_constant<int, 0>{}, yc[0]);
    step(std::integral_constant<int, 1>{}, yc[1]);
    step(std::integral_constant<int, 2>{}, yc[2]);
  };
  uint32_t ya[kLL] = {yb[0], yb[1], yb[2]}, yz[kLL];
#pragma unroll 1
  for (int q = 0; q + 1 < kTrips; q += 2) {
    const uint32_t* yq = yb + kLL * q;
#pragma unroll
    for (int r = 0; r < kLL; ++r) yz[r] = yq[kLL + r];  // trip q + 1's digits
#pragma unroll
    for (int r = 0; r < kLL; ++r) asm volatile("" : "+v"(ya[r]));  // VGPR operands (no readfirstlane)
    steps(ya);
#pragma unroll
    for (int r = 0; r < kLL; ++r) ya[r] = yq[2 * kLL + r];  // trip q + 2's (yb[144..146]: 0)
#pragma unroll
    for (int r = 0; r < kLL; ++r) asm volatile("" : "+v"(yz[r]));
    steps(yz);
  }
  if constexpr (kTrips % 2 == 1) steps(ya);  // the odd last full trip (trip 46: prefetched as "q + 2")
  if constexpr (kRem >= 1) step(std::integral_constant<int, 0>{}, yb[kLL * kTrips]);  // step 141
  if constexpr (kRem >= 2) step(std::integral_constant<int, 1>{}, yb[kLL * kTrips + 1]);
  // the last two digits: after kSteps steps position P (register (kRot + P) % 3 of its lane) holds
  // column kSteps + P; m_{kSteps-2} * p~_J belongs to P = J - 2 (pd) and m_{kSteps-1} * p~_J to P = J - 1 (pd1)
#pragma unroll
  for (int j = 0; j < kLL; ++j) acc[(kRot + j) % kLL] = (uint64_t)pd[j] * m2 + acc[(kRot + j) % kLL];
#pragma unroll
  for (int j = 0; j < kLL; ++j) acc[(kRot + j) % kLL] = (uint64_t)pd1[j] * m1 + acc[(kRot + j) % kLL];
  uint64_t d[kLL];
  {
    const uint64_t top = acc[(kRot + kLL - 1) % kLL] >> kBits;
    const uint64_t c_in = (uint64_t)wprev((uint32_t)top) | ((uint64_t)wprev((uint32_t)(top >> 32)) << 32);
#pragma unroll
    for (int j = 0; j < kLL; ++j)
      d[j] = (uint64_t)((uint32_t)acc[(kRot + j) % kLL] & kM) + (j == 0 ? c_in : (acc[(kRot + j - 1) % kLL] >> kBits));
  }
  const uint32_t c_in = wprev((uint32_t)(d[kLL - 1] >> kBits));
#pragma unroll
  for (int j = 0; j < kLL; ++j) x[j] = ((uint32_t)d[j] & kM) + (j == 0 ? c_in : (uint32_t)(d[j - 1] >> kBits));
}

// MODE 0: general p, 1: p = -1 mod 2^29 (n0 = 1), 2: p = -1 mod 2^58 (delayed quotient, mul_d2)
template <int MODE>
__device__ __forceinline__ void mulm(uint32_t (&x)[kLL], const uint32_t (&y)[kLL], const uint32_t (&p)[kLL],
                                     const uint32_t (&pd)[kLL], const uint32_t (&pd1)[kLL], uint32_t n0, uint32_t mv) {
  if constexpr (MODE == 2) mul_d2(x, y, pd, pd1, mv);
  else mul<MODE == 1>(x, y, p, n0, mv);
}

// canonical form of a value in [0, p] (limbs as mul leaves them): carries rippled up through the
// lanes until none is left (wave-uniform loop), then p -> 0
__device__ __forceinline__ void normalize(uint32_t (&x)[kLL], const uint32_t (&p)[kLL], uint32_t ln) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kLL; ++j) {
    const uint32_t v = x[j] + c;
    x[j] = v & kM;
    c = v >> kBits;
  }
  for (int round = 0; round < 64; ++round) {
    uint32_t cin = wprev(c);
    if (__ballot(cin != 0) == 0) break;
    c = 0;
    if (cin) {
#pragma unroll
      for (int j = 0; j < kLL; ++j) {
        const uint32_t v = x[j] + cin;
        x[j] = v & kM;
        cin = v >> kBits;
      }
      c = cin;
    }
  }
  bool eq = true;
#pragma unroll
  for (int j = 0; j < kLL; ++j) eq &= x[j] == p[j];
  if (__ballot(!eq) == 0) {
#pragma unroll
    for (int j = 0; j < kLL; ++j) x[j] = 0;
  }
  (void)ln;
}

// LDS staging below is one wave's (wave 0 of a job's workgroup): in-order LDS within a wave, so a
// compiler barrier suffices between a lane's store and another lane's load
__device__ __forceinline__ void wsync() { __builtin_amdgcn_wave_barrier(); }

// 512 big-endian bytes -> this lane's three limbs, staged through s_w (the whole wave takes part)
__device__ __forceinline__ void import_be(const uint8_t* __restrict__ be, uint32_t (&x)[kLL], uint32_t* s_w, uint32_t ln) {
  const uint32_t* be32 = reinterpret_cast<const uint32_t*>(be);
  wsync();  // s_w may still be read by the previous import
  for (uint32_t k = ln; k < 128; k += 64) s_w[127 - k] = __builtin_bswap32(be32[k]);
  wsync();
#pragma unroll
  for (int j = 0; j < kLL; ++j) {
    const int bit = kBits * (kLL * (int)ln + j), wi = bit >> 5, sh = bit & 31;
    const uint32_t lo = (ln < kLanes && wi < 128) ? s_w[wi] : 0u;
    const uint32_t hi = (ln < kLanes && wi + 1 < 128) ? s_w[wi + 1] : 0u;
    x[j] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & kM;
  }
}

// canonical limbs (normalize) -> 512 big-endian bytes
__device__ __forceinline__ void export_be(const uint32_t (&x)[kLL], uint8_t* __restrict__ out_be, uint32_t* s_w,
                                          uint32_t ln) {
  wsync();
#pragma unroll
  for (int j = 0; j < kLL; ++j) s_w[kLL * ln + j] = x[j];
  wsync();
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out_be);
  for (uint32_t b = ln; b < 128; b += 64) {  // big-endian word b = little-endian word 127 - b
    const int bitpos = 32 * (127 - (int)b), a = bitpos / kBits, sh = bitpos - a * kBits;
    auto limb = [&](int k) -> uint64_t { return k < kLimbs ? (uint64_t)s_w[k] : 0ull; };
    const uint64_t v = (limb(a) >> sh) | (limb(a + 1) << (kBits - sh)) | (limb(a + 2) << (2 * kBits - sh));
    out32[b] = __builtin_bswap32((uint32_t)v);
  }
}

// wave-uniform read of bits [bit, bit + w) of a little-endian exponent staged in LDS (9 words, the
// last one zero, so a window that runs past bit 255 reads zeros)
__device__ __forceinline__ uint32_t exp_digit(const uint32_t* s_x, uint32_t bit, uint32_t w) {
  const uint32_t wi = bit >> 5;
  // (readfirstlane returns int: widen through uint32_t, not with sign extension)
  const uint64_t v = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(s_x[wi + 1]) << 32) |
                     (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(s_x[wi]);
  return (uint32_t)(v >> (bit & 31)) & ((1u << w) - 1u);
}

// x <- x^e for the exponent staged in s_x (256 bits).  Variable time: a 5-bit sliding window
// over the odd powers x^1, x^3, ..., x^31 (16 LDS entries, ~314 Montgomery operations for a random
// 256-bit exponent, every branch wave-uniform).  Constant time (CT): x^0 .. x^15 in LDS and a fixed
// 4-bit window, 14 + 63 x (4 squarings + 1 multiply) operations for every exponent, every table
// read a masked scan of all 16 entries (neither the schedule nor an address depends on e).
template <int MODE, bool CT>
__device__ __forceinline__ void pow_var(uint32_t (&x)[kLL], const uint32_t* s_x, uint32_t (*s_tab)[kRow],
                                        const Consts* __restrict__ C, const uint32_t (&p)[kLL],
                                        const uint32_t (&pd)[kLL], const uint32_t (&pd1)[kLL], uint32_t n0,
                                        uint32_t mv, uint32_t ln) {
  uint32_t y[kLL];
  if constexpr (CT) {
    wsync();  // s_tab may still be read by a previous exponentiation
#pragma unroll
    for (int j = 0; j < kLL; ++j) {
      s_tab[0][kLL * ln + j] = C->one[kLL * ln + j];
      s_tab[1][kLL * ln + j] = x[j];
      y[j] = x[j];
    }
#pragma unroll 1
    for (int k = 2; k < 16; ++k) {
      mulm<MODE>(y, x, p, pd, pd1, n0, mv);
#pragma unroll
      for (int j = 0; j < kLL; ++j) s_tab[k][kLL * ln + j] = y[j];
    }
    wsync();
    auto select = [&](uint32_t (&dst)[kLL], uint32_t d) {
#pragma unroll
      for (int j = 0; j < kLL; ++j) dst[j] = 0u;
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t m = 0u - (uint32_t)(k == d);
#pragma unroll
        for (int j = 0; j < kLL; ++j) dst[j] |= s_tab[k][kLL * ln + j] & m;
      }
    };
    select(x, exp_digit(s_x, 252, 4));
#pragma unroll 1
    for (int w = 62; w >= 0; --w) {
#pragma unroll 1
      for (int s = 0; s < 4; ++s) mulm<MODE>(x, x, p, pd, pd1, n0, mv);
      select(y, exp_digit(s_x, (uint32_t)(4 * w), 4));
      mulm<MODE>(x, y, p, pd, pd1, n0, mv);
    }
  } else {
    uint32_t x2[kLL] = {x[0], x[1], x[2]};
    mulm<MODE>(x2, x, p, pd, pd1, n0, mv);
    wsync();
#pragma unroll
    for (int j = 0; j < kLL; ++j) s_tab[0][kLL * ln + j] = x[j];
#pragma unroll 1
    for (int k = 1; k < 16; ++k) {
      mulm<MODE>(x, x2, p, pd, pd1, n0, mv);
#pragma unroll
      for (int j = 0; j < kLL; ++j) s_tab[k][kLL * ln + j] = x[j];
    }
    wsync();
    auto bit = [&](int i) -> uint32_t { return (__builtin_amdgcn_readfirstlane(s_x[i >> 5]) >> (i & 31)) & 1u; };
    int i = 255;
    while (i >= 0 && !bit(i)) --i;
    if (i < 0) {
#pragma unroll
      for (int j = 0; j < kLL; ++j) x[j] = C->one[kLL * ln + j];  // x^0 = 1 (also 0^0)
      return;
    }
    bool started = false;
    while (i >= 0) {
      if (!bit(i)) {
        mulm<MODE>(x, x, p, pd, pd1, n0, mv);
        --i;
        continue;
      }
      int l = i - 4 < 0 ? 0 : i - 4;
      while (!bit(l)) ++l;  // the window [i, l] ends on a set bit: an odd value
      uint32_t val = 0;
      for (int k = i; k >= l; --k) val = val << 1 | bit(k);
      if (started)
        for (int k = 0; k < i - l + 1; ++k) mulm<MODE>(x, x, p, pd, pd1, n0, mv);
#pragma unroll
      for (int j = 0; j < kLL; ++j) y[j] = s_tab[val >> 1][kLL * ln + j];
      if (started) {
        mulm<MODE>(x, y, p, pd, pd1, n0, mv);
      } else {
#pragma unroll
        for (int j = 0; j < kLL; ++j) x[j] = y[j];
        started = true;
      }
      i = l - 1;
    }
  }
}

// x <- x * the job's fixed-base window kk (or x <- that factor when !started).  The windows are T0's
// nw0 windows then T1's, each one multiply of a radix-table entry (eg_fixed_base_create: entries in
// the Montgomery domain, 8-lane element layout, limb i at word (i / 18) * 20 + i % 18 of a 160-word
// entry) selected by that window's digit of the term's exponent (s_x[1 + t]).  Variable time: a zero
// digit skips its window.  CT: every window is multiplied in, its entry a masked scan of the window's
// whole column (tables of <= 8 bits only).
template <int MODE, bool CT>
__device__ __forceinline__ void fixed_window(uint32_t (&x)[kLL], bool& started, const WaveTab& T0, const WaveTab& T1,
                                             uint32_t nw0, uint32_t kk, const uint32_t (*s_x)[9],
                                             const uint32_t (&p)[kLL], const uint32_t (&pd)[kLL],
                                             const uint32_t (&pd1)[kLL], uint32_t n0, uint32_t mv, uint32_t ln) {
  uint32_t y[kLL];
  uint32_t idx[kLL];
#pragma unroll
  for (int j = 0; j < kLL; ++j) {
    const uint32_t i = kLL * ln + j;
    idx[j] = (i / 18) * 20 + i % 18;
  }
  const bool live = ln < (uint32_t)kLanes;
  const bool second = kk >= nw0;
  const WaveTab& T = second ? T1 : T0;
  const uint32_t k = second ? kk - nw0 : kk;
  const uint32_t d = exp_digit(s_x[second ? 2 : 1], k * T.wbits, T.wbits);
  const uint32_t* col = T.data + ((size_t)k << T.wbits) * 160;
  if constexpr (CT) {
#pragma unroll
    for (int j = 0; j < kLL; ++j) y[j] = 0u;
    const uint32_t nent = 1u << T.wbits;
#pragma unroll 4
    for (uint32_t e = 0; e < nent; ++e) {
      const uint32_t m = 0u - (uint32_t)(e == d);
      const uint32_t* ent = col + (size_t)e * 160;
#pragma unroll
      for (int j = 0; j < kLL; ++j) y[j] |= (live ? ent[idx[j]] : 0u) & m;
    }
  } else {
    if (d == 0) return;
    const uint32_t* ent = col + (size_t)d * 160;
#pragma unroll
    for (int j = 0; j < kLL; ++j) y[j] = live ? ent[idx[j]] : 0u;
  }
  if (started) {
    mulm<MODE>(x, y, p, pd, pd1, n0, mv);
  } else {
#pragma unroll
    for (int j = 0; j < kLL; ++j) x[j] = y[j];
    started = true;
  }
}

// windows [k0, k1) of fixed_window
template <int MODE, bool CT>
__device__ __forceinline__ void pow_fixed(uint32_t (&x)[kLL], bool& started, const WaveTab& T0, const WaveTab& T1,
                                          uint32_t nw0, uint32_t k0, uint32_t k1, const uint32_t (*s_x)[9],
                                          const uint32_t (&p)[kLL], const uint32_t (&pd)[kLL],
                                          const uint32_t (&pd1)[kLL], uint32_t n0, uint32_t mv, uint32_t ln) {
#pragma unroll 1
  for (uint32_t kk = k0; kk < k1; ++kk) fixed_window<MODE, CT>(x, started, T0, T1, nw0, kk, s_x, p, pd, pd1, n0, mv, ln);
}

// One job per workgroup of W waves (eg_pow16.h WaveJob): out = (prod of the job's bases)^exp * T0^f0 *
// T1^f1 mod p.  Every per-element group operation is a special case: powP (one base, an exponent),
// gPowP and an accelerated K.powP (one fixed-base term), times (two bases, no exponent), g^v * alpha^c
// (one base, an exponent, one fixed-base term), the contest aggregate (A = prod alpha)^c.
// Wave 0 runs the variable part (the bases' product and its exponentiation: a sequential chain); the
// fixed-base windows, each an independent factor, are split over the other waves (all W waves when the
// job has no variable part), each multiplying its share into a partial product; the partials meet in
// LDS and fold in a log2(W) tree: a fixed-base term of n windows costs ~n/W + log2(W) multiplies of
// latency instead of n.  jobs == nullptr: job e is `dflt` with its rows offset by e (the batch entry
// points: element e of every input array).
// r2l (W > 1, a job with an exponent): the variable part runs right to left instead.
// Wave 0 only squares, x_i = x^(2^i) for i up to the exponent's top bit, W - 1 squarings per round,
// and leaves each round's powers in a double-buffered LDS ring; in the next round wave k (1 <= k < W)
// multiplies x_i with i = (round - 1)(W - 1) + k - 1 into its partial when bit i is set, then takes one
// of its fixed-base windows.  A wave does at most 2 multiplies while wave 0 does W - 1 = 3 squarings,
// so the chain never waits: the latency is the top bit + ~4 operations against ~16 (window table) +
// the top bit + ~43 (window multiplies) for the left-to-right sliding window (one SIMD per wave: the
// waves issue side by side).  The host enables it for batches of at most one job per CU.  CT: the chain
// runs all 255 squarings and every multiplying wave multiplies in every round, by x_i or by 1 (a
// masked select of the two), and takes its fixed-base windows as masked scans: the same operations
// for every exponent.
template <int MODE, bool CT, int W>
__global__ void __launch_bounds__(64 * W) k_wave_job(const Consts* __restrict__ C, const WaveJob* __restrict__ jobs,
                                                     WaveJob dflt, uint32_t njobs, const WaveTab* __restrict__ tabs,
                                                     const uint8_t* __restrict__ bases, const uint8_t* __restrict__ exps,
                                                     uint8_t* __restrict__ out_be, WaveTab t_ident, uint32_t r2l) {
  constexpr int kRing = W > 1 ? 2 * (W - 1) : 1;
  __shared__ uint32_t s_tab[16][kRow];     // window table of the variable-base term (wave 0)
  __shared__ uint32_t s_w[kRow];           // byte <-> limb staging (wave 0)
  __shared__ uint32_t s_x[3][9];           // the exponents (variable, fixed 0, fixed 1), LE words + a zero word
  __shared__ uint32_t s_part[W][kRow];     // the waves' partial products
  __shared__ uint32_t s_has[W];            // ... and whether each has one
  __shared__ uint32_t s_ring[kRing][kRow];  // r2l: two rounds of the squaring chain
  const uint32_t e = blockIdx.x;        // one job per workgroup; the grid is exactly njobs
  if (e >= njobs) return;
  WaveJob J;
  if (jobs) {
    J = jobs[e];
  } else {  // the batch entry points
    J = dflt;
    if (J.nbase) J.base = e;
    if (J.exp != kWaveNone) J.exp = e;
    if (J.tab[0] != kWaveNone) J.fexp[0] = e;
    J.out = e;
  }
  const uint32_t wv = W > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u;
  const uint32_t ln = lane64();
  const uint32_t n0 = C->n0;
  uint32_t mv;  // in a VGPR: v_and_b32_dpp takes its second operand from one
  asm volatile("v_mov_b32 %0, %1" : "=v"(mv) : "s"(C->mask));
  uint32_t p[kLL], x[kLL], y[kLL], pd[kLL], pd1[kLL];
#pragma unroll
  for (int j = 0; j < kLL; ++j) {
    p[j] = C->p[kLL * ln + j];
    pd[j] = MODE == 2 ? C->pd[kLL * ln + j] : 0u;
    pd1[j] = MODE == 2 ? C->pd1[kLL * ln + j] : 0u;
  }
  if (wv == 0) {
    const uint32_t rows[3] = {J.exp, J.fexp[0], J.fexp[1]};
    if (ln < 24) {
      const uint32_t s = ln >> 3, w = ln & 7u, r = rows[s];
      const bool used = r != kWaveNone && (s == 0 || J.tab[s - 1] != kWaveNone);
      s_x[s][7 - w] = used ? __builtin_bswap32(reinterpret_cast<const uint32_t*>(exps + (size_t)r * 32)[w]) : 0u;
    }
    if (ln < 3) s_x[ln][8] = 0u;
  }
  const WaveTab T0 = J.tab[0] != kWaveNone ? (jobs ? tabs[J.tab[0]] : t_ident) : WaveTab{nullptr, 0, 0};
  const WaveTab T1 = J.tab[1] != kWaveNone ? tabs[J.tab[1]] : WaveTab{nullptr, 0, 0};
  const uint32_t nw0 = J.tab[0] != kWaveNone ? T0.nwin : 0u, nw = nw0 + (J.tab[1] != kWaveNone ? T1.nwin : 0u);
  // an exponent on an empty product: 1^e = 1 (no variable part)
  const bool has_var = J.nbase > 0;
  // right to left over W waves (wave-uniform: the same for every wave of the job)
  const bool split = W > 1 && r2l && has_var && J.exp != kWaveNone;
  __syncthreads();  // s_x
  bool started = false;
  if (wv == 0 && has_var) {
    // the product of the bases, each taken into the Montgomery domain (limbs * R^2 * R^-1; a base
    // >= p is reduced here: the result is < 2p)
#pragma unroll 1
    for (uint32_t k = 0; k < J.nbase; ++k) {
      import_be(bases + (size_t)(J.base + k) * 512, y, s_w, ln);
      uint32_t r2[kLL];
#pragma unroll
      for (int j = 0; j < kLL; ++j) r2[j] = C->r2[kLL * ln + j];
      mulm<MODE>(y, r2, p, pd, pd1, n0, mv);
      if (started) {
        mulm<MODE>(x, y, p, pd, pd1, n0, mv);
      } else {
#pragma unroll
        for (int j = 0; j < kLL; ++j) x[j] = y[j];
        started = true;
      }
    }
    if (J.exp != kWaveNone && !split) pow_var<MODE, CT>(x, s_x[0], s_tab, C, p, pd, pd1, n0, mv, ln);
  }
  if constexpr (W > 1) {
    if (split) {
      auto bit = [&](int i) -> uint32_t { return (__builtin_amdgcn_readfirstlane(s_x[0][i >> 5]) >> (i & 31)) & 1u; };
      int top = 255;
      if constexpr (!CT)
        while (top >= 0 && !bit(top)) --top;
      if constexpr (CT) {  // every multiplying wave holds a factor from the start: 1
        if (wv) {
#pragma unroll
          for (int j = 0; j < kLL; ++j) x[j] = C->one[kLL * ln + j];
          started = true;
        }
      }
      constexpr int K = W - 1;
      const int rounds = top < 0 ? 0 : top / K + 1;
      const uint32_t widx = wv - 1;
      uint32_t kk = wv ? widx * nw / K : 0u;
      const uint32_t k1 = wv ? (widx + 1) * nw / K : 0u;
#pragma unroll 1
      for (int r = 0; r <= rounds; ++r) {
        if (wv == 0) {
          // x_i for i = rK .. rK + K - 1 (x holds x_(rK - 1) squared K - 1 times ago ... x_0 = x)
#pragma unroll 1
          for (int k = 0; k < K; ++k) {
            const int i = r * K + k;
            if (r == rounds || i > top) break;
            if (i > 0) mulm<MODE>(x, x, p, pd, pd1, n0, mv);
#pragma unroll
            for (int j = 0; j < kLL; ++j) s_ring[(r & 1) * K + k][kLL * ln + j] = x[j];
          }
        } else {
          const int i = (r - 1) * K + (int)widx;
          if constexpr (CT) {
            if (r > 0 && i <= top) {  // x *= bit i ? x_i : 1, the same multiply either way
              uint32_t msk = 0u - bit(i);
              asm volatile("" : "+s"(msk));
#pragma unroll
              for (int j = 0; j < kLL; ++j)
                y[j] = (s_ring[((r - 1) & 1) * K + widx][kLL * ln + j] & msk) | (C->one[kLL * ln + j] & ~msk);
              mulm<MODE>(x, y, p, pd, pd1, n0, mv);
            }
          } else if (r > 0 && i <= top && bit(i)) {
#pragma unroll
            for (int j = 0; j < kLL; ++j) y[j] = s_ring[((r - 1) & 1) * K + widx][kLL * ln + j];
            if (started) {
              mulm<MODE>(x, y, p, pd, pd1, n0, mv);
            } else {
#pragma unroll
              for (int j = 0; j < kLL; ++j) x[j] = y[j];
              started = true;
            }
          }
          if (kk < k1) fixed_window<MODE, CT>(x, started, T0, T1, nw0, kk++, s_x, p, pd, pd1, n0, mv, ln);
        }
        __syncthreads();  // round r's powers are in the ring; round r - 1's slots are free again
      }
      if (wv) {
        pow_fixed<MODE, CT>(x, started, T0, T1, nw0, kk, k1, s_x, p, pd, pd1, n0, mv, ln);
      } else {
        started = false;  // the chain itself is not a factor
      }
    }
  }
  // this wave's share of the fixed-base windows (W = 1: all of them, after the variable part)
  if (!split) {
    const uint32_t workers = (W > 1 && has_var) ? W - 1 : W;
    const uint32_t widx = (W > 1 && has_var) ? wv - 1 : wv;
    if (!(W > 1 && has_var && wv == 0) && nw)
      pow_fixed<MODE, CT>(x, started, T0, T1, nw0, widx * nw / workers, (widx + 1) * nw / workers, s_x, p, pd,
                          pd1, n0, mv, ln);
  }
  if constexpr (W > 1) {
    // fold the partials: a log2(W) tree through LDS, every wave at every barrier
#pragma unroll
    for (int j = 0; j < kLL; ++j) s_part[wv][kLL * ln + j] = x[j];
    if (ln == 0) s_has[wv] = started ? 1u : 0u;
    __syncthreads();
#pragma unroll 1
    for (uint32_t stride = 1; stride < (uint32_t)W; stride *= 2) {
      if (wv % (2 * stride) == 0 && wv + stride < (uint32_t)W) {
        if (__builtin_amdgcn_readfirstlane(s_has[wv + stride])) {
#pragma unroll
          for (int j = 0; j < kLL; ++j) y[j] = s_part[wv + stride][kLL * ln + j];
          if (started) {
            mulm<MODE>(x, y, p, pd, pd1, n0, mv);
          } else {
#pragma unroll
            for (int j = 0; j < kLL; ++j) x[j] = y[j];
            started = true;
          }
#pragma unroll
          for (int j = 0; j < kLL; ++j) s_part[wv][kLL * ln + j] = x[j];
          if (ln == 0) s_has[wv] = started ? 1u : 0u;
        }
      }
      __syncthreads();
    }
    if (wv != 0) return;
  }
  if (!started) {
#pragma unroll
    for (int j = 0; j < kLL; ++j) x[j] = C->one[kLL * ln + j];
  }
  // leave the Montgomery domain (x * 1 * R^-1: a value in [0, p]) and write canonical bytes
#pragma unroll
  for (int j = 0; j < kLL; ++j) y[j] = (ln == 0 && j == 0) ? 1u : 0u;
  mulm<MODE>(x, y, p, pd, pd1, n0, mv);
  normalize(x, p, ln);
  export_be(x, out_be + (size_t)J.out * 512, s_w, ln);
}
}  // namespace egw

struct PowWaveConsts {
  egw::Consts* d = nullptr;
  bool d2 = false;  // p = -1 mod 2^58: the delayed-quotient multiply (EG_POWWAVE_D2=0 keeps mul<true>)
};

int powwave_consts_create(const uint32_t* p, const uint32_t* r2, const uint32_t* one, uint32_t n0, uint32_t friendly,
                          PowWaveConsts** out, std::string* err) {
  (void)friendly;
  egw::Consts h{};
  auto limbs = [](const uint32_t* w, int nw, uint32_t* o) {
    for (int a = 0; a < egw::kLimbs; ++a) {
      const int bit = a * egw::kBits;
      uint64_t v = 0;
      for (int k = 0; k < 2; ++k) {  // bit % 32 + 29 <= 60: two words hold the limb (a shift by 64 would be UB)
        const int wi = bit / 32 + k;
        if (wi < nw) v |= (uint64_t)w[wi] << (32 * k);
      }
      o[a] = (uint32_t)(v >> (bit % 32)) & egw::kM;
    }
  };
  limbs(p, 128, h.p);
  limbs(r2, 129, h.r2);
  limbs(one, 129, h.one);
  // p + 1 (129 words: the carry out of the top word is zero for p < 2^4096 - 1) in limbs, shifted down
  // by two and by one limb for the delayed-quotient multiply
  {
    uint32_t p1[129];
    uint64_t c = 1;
    for (int k = 0; k < 128; ++k) {
      c += p[k];
      p1[k] = (uint32_t)c;
      c >>= 32;
    }
    p1[128] = (uint32_t)c;
    uint32_t pt[egw::kRow];
    std::memset(pt, 0, sizeof pt);
    limbs(p1, 129, pt);
    for (int a = 0; a < egw::kRow; ++a) {
      h.pd[a] = a + 2 < egw::kLimbs ? pt[a + 2] : 0u;
      h.pd1[a] = a + 1 < egw::kLimbs ? pt[a + 1] : 0u;
    }
  }
  h.n0 = n0;
  h.mask = egw::kM;
  auto* c = new PowWaveConsts();
  {
    const char* env = std::getenv("EG_POWWAVE_D2");
    c->d2 = p[0] == 0xFFFFFFFFu && (p[1] & 0x03FFFFFFu) == 0x03FFFFFFu && !(env && env[0] == '0');
  }
  hipError_t e = hipMalloc(&c->d, sizeof(egw::Consts));
  if (e == hipSuccess) e = hipMemcpy(c->d, &h, sizeof(egw::Consts), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (c->d) hipFree(c->d);
    delete c;
    *err = std::string("powwave constants: ") + hipGetErrorString(e);
    return 1;
  }
  *out = c;
  return 0;
}

void powwave_consts_destroy(PowWaveConsts* c) {
  if (!c) return;
  if (c->d) hipFree(c->d);
  delete c;
}

int powwave_jobs(const PowWaveConsts* C, bool friendly, bool ct, int waves, bool r2l, hipStream_t s,
                 const WaveJob* d_jobs, WaveJob dflt, uint32_t njobs, const WaveTab* d_tabs, WaveTab t_ident,
                 const uint8_t* d_bases, const uint8_t* d_exps, uint8_t* d_out, std::string* err) {
  if (!njobs) return 0;
  if (!d_jobs && dflt.tab[0] != kWaveNone &&
      (t_ident.wbits < 1 || t_ident.wbits > 24 || (uint64_t)t_ident.nwin * t_ident.wbits < 256 ||
       (uint64_t)(t_ident.nwin - 1) * t_ident.wbits >= 256 || (ct && t_ident.wbits > 8))) {
    *err = "powwave: fixed-base table shape";
    return 1;
  }
  const dim3 grid(njobs);
  // fixed-base windows split over 4 waves per job when the batch has any (waves > 1), over 8 (two per
  // SIMD) for waves >= 8 on the Montgomery-friendly p; r2l (4 waves): the variable part right to left
  // over the 4 waves (CT: the constant-time schedule of it)
  const int mode = (friendly && C->d2) ? 2 : (friendly ? 1 : 0);
  const int W = (waves >= 8 && mode == 2 && !r2l) ? 8 : waves > 1 ? 4 : 1;
  const uint32_t r2l_on = (r2l && W == 4) ? 1u : 0u;
#define EGW_LAUNCH(M, CTV, WV)                                                                                    \
  hipLaunchKernelGGL((egw::k_wave_job<M, CTV, WV>), grid, dim3(64 * WV), 0, s, C->d, d_jobs, dflt, njobs, d_tabs, \
                     d_bases, d_exps, d_out, t_ident, r2l_on)
#define EGW_LAUNCH_W(M, CTV) \
  do {                       \
    if (W == 4)              \
      EGW_LAUNCH(M, CTV, 4); \
    else                     \
      EGW_LAUNCH(M, CTV, 1); \
  } while (0)
  if (W == 8) {
    if (ct) EGW_LAUNCH(2, true, 8);
    else EGW_LAUNCH(2, false, 8);
  } else if (ct) {
    if (mode == 2) EGW_LAUNCH_W(2, true);
    else if (mode == 1) EGW_LAUNCH_W(1, true);
    else EGW_LAUNCH_W(0, true);
  } else {
    if (mode == 2) EGW_LAUNCH_W(2, false);
    else if (mode == 1) EGW_LAUNCH_W(1, false);
    else EGW_LAUNCH_W(0, false);
  }
#undef EGW_LAUNCH_W
#undef EGW_LAUNCH
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = std::string("powwave launch: ") + hipGetErrorString(e);
    return 1;
  }
  return 0;
}

int powwave_powp(const PowWaveConsts* C, bool friendly, bool ct, bool r2l, hipStream_t s, const uint8_t* base_be,
                 const uint8_t* exp_be, uint8_t* out_be, size_t n, std::string* err) {
  const WaveJob d{0, 1, 0, {kWaveNone, kWaveNone}, {kWaveNone, kWaveNone}, 0};
  const bool rl = r2l;
  return powwave_jobs(C, friendly, ct, rl ? 4 : 1, rl, s, nullptr, d, (uint32_t)n, nullptr, WaveTab{nullptr, 0, 0},
                      base_be, exp_be, out_be, err);
}

int powwave_fbpow(const PowWaveConsts* C, bool friendly, bool ct, hipStream_t s, const WaveTab& t,
                  const uint8_t* exp_be, uint8_t* out_be, size_t n, std::string* err) {
  const WaveJob d{0, 0, kWaveNone, {0, kWaveNone}, {0, kWaveNone}, 0};
  return powwave_jobs(C, friendly, ct, 4, false, s, nullptr, d, (uint32_t)n, nullptr, t, nullptr, exp_be, out_be, err);
}
