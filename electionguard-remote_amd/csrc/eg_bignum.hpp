// eg_bignum.hpp — CDNA4 (gfx950) device core for 4096-bit Montgomery arithmetic.
//
// Replaces the upstream GroupContext / ElementModP arithmetic reached through
// KUtils.productionGroup() (src/main/java/electionguard/util/KUtils.java:10-12):
// ElementModP.times / multP and the powP built from them.  Results are the unique
// integers mod p, i.e. identical to java.math.BigInteger.modPow / multiply+mod.
//
// Representation (MI355X-first):
//   * radix 2^29, N = 144 limbs (4176 bits) per element, Montgomery R = 2^(29 * 142) = 2^4118 > 4p
//     (142 CIOS steps: kSteps below), so the CIOS loop never needs a final subtraction (values stay
//     < 2p between ops);
//     (EG_RADIX=27 keeps the first design: N = 152, R = 2^4104);
//   * every accumulator register takes ONE v_mad_u64_u32 per limb product with no
//     carry-out handling: a register enters its lane's top position with a 29-bit limb,
//     takes <= 2 products per CIOS step for L = 18 steps and is split when it reaches
//     the bottom: 36 x (2^29 + 2^6)^2 + 2^35 < 2^63.2 (squarings: 18 x (2^59 + 2^58)
//     < 2^63.8); the gfx950 microbenchmark (profiles/r01_ubench_isa.txt)
//     shows v_mad_u64_u32 issues at the same rate as a 32-bit add, so the cost of a
//     Montgomery multiply is its instruction count;
//   * one element is owned by a group of T = EG_T consecutive lanes (a DPP quad or
//     half-row); lane l of the group holds limbs [l*L, l*L+L), L = N/T, in VGPRs;
//   * the multiplier operand y is read from a per-group LDS slot (group-uniform
//     broadcast read), the modulus limbs p live in VGPRs, the accumulator t in
//     L 64-bit VGPR pairs whose register names rotate by one per step (unrolled L
//     steps), so the CIOS "shift by one limb" costs one DPP row_shl:1 per step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#ifndef EG_T
#define EG_T 8
#endif

namespace eg {

#ifndef EG_RADIX
#define EG_RADIX 29
#endif
constexpr int kLimbBits = EG_RADIX;
constexpr uint32_t kMask = (1u << kLimbBits) - 1u;
constexpr int kN = EG_RADIX == 29 ? 144 : (EG_RADIX == 28 ? 148 : 152);  // limbs per element (the layout; R: kSteps)
constexpr int kT = EG_T;              // lanes per element
constexpr int kL = kN / kT;           // limbs per lane
constexpr int kLP = (kL + 3) & ~3;    // padded limbs per lane (16-B aligned lane blocks)
constexpr int kW = kT * kLP;          // words per device element (160 for T=4 and T=8)
constexpr int kYStride = kW + 4;      // LDS words per group slot (bank spread)
constexpr int kWave = 64;
constexpr int kGroupsPerWave = kWave / kT;
static_assert(kN % kT == 0, "limbs must split evenly over the group");
static_assert(EG_RADIX >= 27 && EG_RADIX <= 29, "radix 2^27 (152 limbs), 2^28 (148) or 2^29 (144 limbs)");
static_assert(kN * kLimbBits >= 4098, "the element format must hold values < 2p");
// CIOS steps per Montgomery operation: the fewest radix-2^b digits whose R = 2^(b * steps) exceeds 4p
// (p < 2^4096, values < 2p), 142 at radix 2^29, against the 144 limbs the 8-lane layout holds.  An
// operand's limbs 142 and 143 are always zero (< 2p < 2^4097 = bit 4118 and above clear), so the two
// steps whose multiplier digits they would be only run the m * p half; stopping after 142 steps is
// Montgomery's multiply for R = 2^4118 (eg_capi.hip sets R mod p and R^2 mod p to match).  The last
// trip stops kSkip steps early and the result sits in the accumulator at rotation kRot.
#ifndef EG_CIOS_FULL
#define EG_CIOS_FULL 0  // 1: all kN steps (R = 2^(kN * b), rounds 1-5's domain; A/B builds only)
#endif
constexpr int kSteps = EG_CIOS_FULL ? kN : (4098 + kLimbBits - 1) / kLimbBits;
constexpr int kSkip = kN - kSteps;
static_assert(kSteps * kLimbBits >= 4098, "R must exceed 4p (lazy reduction: values stay < 2p)");
static_assert(kSkip >= 0 && kSkip < kL, "the skipped steps fit in the last trip");
constexpr int kRot = (kL - kSkip) % kL;  // accumulator rotation after kSteps steps
// Accumulator headroom: a register lives L steps in its lane and takes <= 2 products per step
// (x*y + m*p; with SQR one doubled x*x product + m*p).  Radix 2^29 needs L <= 18.
static_assert((unsigned __int128)2 * kL * (((1ull << kLimbBits) + 64) * ((1ull << kLimbBits) + 64)) < ((unsigned __int128)1 << 64), "radix 2^29 overflows the 64-bit columns above 18 limbs per lane");
// kT = 16 (one DPP row per element, 9 limbs per lane) is the latency-shaped instantiation of
// eg_pow16.hip (the per-element coalescer's small batches); its element format is 192 words
static_assert(kT == 4 || kT == 8 || kT == 16, "EG_T must be 4, 8 or 16");
static_assert(kW == (kT == 16 ? 192 : 160), "device element format is 160 words (192 for T = 16)");

// Device constants of one group context (filled by the host, eg_capi.hip).
struct MontConsts {
  uint32_t p[kW];      // modulus limbs, device element format (radix 2^kLimbBits)
  uint32_t r2[kW];     // R^2 mod p (normal form)        -> to-Montgomery multiplier
  uint32_t one[kW];    // R mod p (Montgomery form of 1)
  uint32_t unit[kW];   // the integer 1 (limb 0 = 1)      -> from-Montgomery multiplier
  uint32_t pw[128];    // p as 128 little-endian 32-bit words (final compare / subtract)
  uint32_t n0;         // -p^-1 mod 2^kLimbBits
  uint32_t friendly;   // n0 == 1 (p = -1 mod 2^kLimbBits): EG production group
  uint32_t mask;       // 2^kLimbBits - 1 (read at run time so AND can fuse into DPP moves)
  // Subgroup (residue) test x^q == 1, evaluated as x^(2^256) == x^c with c = 2^256 - q
  // (x != 0): c is public, 189 for the EG q = 2^256 - 189 (8 bits, 7 sq + 5 mul).
  uint32_t qc[8];      // c = 2^256 - q, little-endian words
  uint32_t qc_bits;    // bit length of c
};

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ int glane() { return lane_id() & (kT - 1); }   // lane within element group
__device__ __forceinline__ int gslot() { return lane_id() / kT; }        // group index within wave

#ifndef EG_BCAST
#define EG_BCAST 0  // 0: DPP (VALU), 1: ds_swizzle (LDS pipe, no VALU issue slot)
#endif
#ifndef EG_PLDS
#define EG_PLDS 1   // 1: modulus limbs read from LDS instead of VGPRs (frees 19 VGPRs: 3 waves/SIMD)
#endif

// Broadcast group-lane 0's value to the whole group.
__device__ __forceinline__ uint32_t bcast_g0(uint32_t v) {
#if EG_BCAST == 1
  // bit-mode swizzle within 32 lanes: lane' = lane & and_mask (clears the in-group bits)
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, kT == 8 ? 0x0018 : 0x001C);
#else
  if constexpr (kT == 16) return __builtin_amdgcn_mov_dpp(v, 0x150 /*row_newbcast:0*/, 0xF, 0xF, false);
  uint32_t a = __builtin_amdgcn_mov_dpp(v, 0x00 /*quad_perm [0,0,0,0]*/, 0xF, 0xF, false);
  if constexpr (kT == 8) {
    // lanes 4-7 / 12-15 of every row take the value 4 lanes below (the group's lane 0)
    a = __builtin_amdgcn_update_dpp(a, a, 0x114 /*row_shr:4*/, 0xF, 0xA, false);
  }
  return a;
#endif
}

#ifndef EG_ASM_DPP
#define EG_ASM_DPP 0  // 1: AND fused into the DPP moves by inline asm (v_and_b32_dpp)
#endif

// (v & mask) of group-lane 0, broadcast to the group  (fused form)
__device__ __forceinline__ uint32_t bcast_g0_and(uint32_t v, uint32_t mask) {
#if EG_ASM_DPP && EG_BCAST == 0
  uint32_t r;
  // s_nop 1: a VALU-written VGPR read through DPP needs 2 wait states
  if constexpr (kT == 8) {
    asm volatile(
        "s_nop 1\n\t"
        "v_and_b32_dpp %0, %1, %2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_mov_b32_dpp %0, %0 row_shr:4 row_mask:0xf bank_mask:0xa"
        : "=&v"(r) : "v"(v), "v"(mask));
  } else {
    asm volatile(
        "s_nop 1\n\t"
        "v_and_b32_dpp %0, %1, %2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf"
        : "=v"(r) : "v"(v), "v"(mask));
  }
  return r;
#elif EG_BCAST == 1
  return bcast_g0(v) & mask;
#else
  // T = 16: the group is a DPP row, one row_newbcast:0 move (gfx90a+) broadcasts its lane 0
  if constexpr (kT == 16) return __builtin_amdgcn_mov_dpp(v, 0x150 /*row_newbcast:0*/, 0xF, 0xF, true) & mask;
  // AND first on the full-mask quad_perm move (the DPP combiner folds it into
  // v_and_b32_dpp when mask is a VGPR), then the half-row move for T = 8
  uint32_t a = __builtin_amdgcn_mov_dpp(v, 0x00 /*quad_perm [0,0,0,0]*/, 0xF, 0xF, true) & mask;
  if constexpr (kT == 8) a = __builtin_amdgcn_update_dpp(a, a, 0x114 /*row_shr:4*/, 0xF, 0xA, false);
  return a;
#endif
}

// (v & mask) from lane+1 within the DPP row (0 at the row end)  (fused form)
__device__ __forceinline__ uint32_t from_next_and(uint32_t v, uint32_t mask) {
#if EG_ASM_DPP
  uint32_t r;
  asm volatile(
      "s_nop 1\n\t"
      "v_and_b32_dpp %0, %1, %2 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "=v"(r) : "v"(v), "v"(mask));
  return r;
#else
  return __builtin_amdgcn_mov_dpp(v, 0x101 /*row_shl:1*/, 0xF, 0xF, true) & mask;
#endif
}

// value from lane+1 within the DPP row (0 at the row end)
__device__ __forceinline__ uint32_t from_next(uint32_t v) {
  return __builtin_amdgcn_mov_dpp(v, 0x101 /*row_shl:1*/, 0xF, 0xF, true);
}
// value from lane-1 within the DPP row (0 at the row start)
__device__ __forceinline__ uint32_t from_prev(uint32_t v) {
  return __builtin_amdgcn_mov_dpp(v, 0x111 /*row_shr:1*/, 0xF, 0xF, true);
}

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): compile-time rotation indices
template <int I, int N, class F>
__device__ __forceinline__ void rsteps_from(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    rsteps_from<I + 1, N>(f);
  }
}
template <int N, class F>
__device__ __forceinline__ void rsteps(F& f) { rsteps_from<0, N>(f); }

// Montgomery multiply  x <- x * y * R^-1 mod p  (result < 2p, limbs < 2^b + 2^(64-2b)+1).
//   x : this lane's L limbs (in/out), any value < 2p, limbs <= 2^b + 2^(64-2b) + 1
//   y : the group's LDS slot (kW words, device element format), value < 2p
//   p : this lane's L modulus limbs (VGPRs or LDS)
// CIOS, one radix-2^b digit of y per step; 2L v_mad_u64_u32 + ~7 VALU per step.
//
// SQR = true computes x^2 with y == x (the slot must hold x): the x*x part of each step
// uses the symmetric half.  Pair {a, b} of limb indices (register indices ja, jb) is
// added once, doubled, at the row whose register index is cyclically 1..h behind the
// other ((jb - ja) mod L in [1, h] -> row a, h = (L-1)/2); for even L the pairs at
// distance L/2 go to the row with the smaller register index (r < L/2); pairs with
// ja == jb go to the smaller limb index and the diagonal x_a^2 once.  At row i (register
// r = i mod L, outer block s) every lane therefore touches the SAME register indices
// r..r+h (mod L): doubled products from 2x held in registers, and the diagonal register
// whose multiplier is 2x_r (lanes > s), x_r (lane s) or 0 (lanes < s) -- one v_bfe_u32
// with per-lane (offset, width).  L = 18: 9.5 MACs + 1 VALU instead of 18.  All contributions
// to column c still arrive by step c (each pair is added at row <= c), so the CIOS
// quotient digits are unchanged.
// One CIOS step at register rotation r (multiplier digit yi): t += x * yi, then t += m * p and
// the lowest column's split.  FIRST: the multiply's very first step, whose accumulator is
// implicitly zero -- the products are written instead of added (no zeroing pass; for SQR the
// registers the half-row leaves untouched are first written by the m * p half).
template <bool FRIENDLY, bool SQR, bool FIRST, class PT>
__device__ __forceinline__ void cios_step(uint64_t (&acc)[kL], const uint32_t (&x)[kL], const int r, const uint32_t yi,
                                          const PT& p, uint32_t n0, uint32_t mask, uint32_t doff, uint32_t dwid) {
  // t += x * y_i     (logical position j lives in register (j + r) % L)
  int jmax = 0;
  if constexpr (SQR) {
    {
      const uint32_t d = __builtin_amdgcn_ubfe(x[r], doff, dwid);
      uint64_t& A = acc[(r + r) % kL];
      A = FIRST ? (uint64_t)d * yi : (uint64_t)d * yi + A;
    }
    // odd L: offsets 1..(L-1)/2; even L: offsets 1..L/2-1, plus the offset-L/2 pair
    // at the row with the smaller register index (r < L/2)
    constexpr int kHalf = (kL - 1) / 2;
    jmax = (kL % 2 == 1) ? kHalf : (r < kL / 2 ? kL / 2 : kL / 2 - 1);
#pragma unroll
    for (int jj = 1; jj <= jmax; ++jj) {
      const int j = (r + jj) % kL;
      uint64_t& A = acc[(j + r) % kL];
      A = FIRST ? (uint64_t)x[j] * yi : (uint64_t)x[j] * yi + A;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      uint64_t& A = acc[(j + r) % kL];
      A = FIRST ? (uint64_t)x[j] * yi : (uint64_t)x[j] * yi + A;
    }
  }
  // quotient digit from the group's lowest limb
  uint32_t t0 = (uint32_t)acc[r % kL];
  if constexpr (!FRIENDLY) t0 *= n0;
  const uint32_t m = bcast_g0_and(t0, mask);
  // t += m * p   (FIRST, SQR: registers (r + 1 + jmax .. r + L - 1) % L are still unwritten;
  // with r = 0 those are the ones whose register index exceeds jmax)
#pragma unroll
  for (int j = 0; j < kL; ++j) {
    uint64_t& A = acc[(j + r) % kL];
    const bool fresh = FIRST && SQR && ((j + r) % kL) > r + jmax;
    A = fresh ? (uint64_t)p[j] * m : (uint64_t)p[j] * m + A;
  }
  // split the lowest column: carry stays in this lane (next position),
  // low 27 bits shift into lane-1's top position (0 for the group's lane 0)
  uint64_t& A0 = acc[r % kL];
  acc[(r + 1) % kL] += A0 >> kLimbBits;
  A0 = (uint64_t)from_next_and((uint32_t)A0, mask);
}

template <bool FRIENDLY, bool SQR, class PT>
__device__ __forceinline__ void mont_mul_impl(uint32_t (&x)[kL], const uint32_t* __restrict__ y,
                                              const PT& p, uint32_t n0, uint32_t mask) {
  uint64_t acc[kL];
  if constexpr (SQR) {
#pragma unroll
    for (int j = 0; j < kL; ++j) x[j] <<= 1;  // 2x < 2^(b+1) + 2^(65-2b) < 2^31
  }
  // SQR: the diagonal multiplier of outer block s is x_r (own row: (2x_r) >> 1) on lane s,
  // 2x_r on the lanes above and 0 below (width 0); carried from trip to trip
  const int gl = glane();
  uint32_t doff = SQR && gl == 0 ? 1u : 0u, dwid = SQR ? 31u : 0u;
  // the first step runs peeled (no accumulator zeroing); every trip s then runs its steps
  // 1..L-1 and the next trip's step 0 (same register rotation: r = 0 follows r = L-1)
  cios_step<FRIENDLY, SQR, true>(acc, x, 0, y[0], p, n0, mask, doff, dwid);
  // full trips in the loop (each a whole register rotation, so the loop carries no register moves);
  // with kSkip > 0 the last trip is straight-line code after it that stops after step kSteps - 1
  constexpr int kFull = kSkip ? kT - 1 : kT;
#pragma unroll 1
  for (int s = 0; s < kFull; ++s) {
    const uint32_t* ys = y + s * kLP;
#pragma unroll
    for (int r = 1; r < kL; ++r) cios_step<FRIENDLY, SQR, false>(acc, x, r, ys[r], p, n0, mask, doff, dwid);
    if (s + 1 < kT) {
      if constexpr (SQR) {
        doff = (gl == s + 1) ? 1u : 0u;
        dwid = (gl >= s + 1) ? 31u : 0u;
      }
      cios_step<FRIENDLY, SQR, false>(acc, x, 0, ys[kLP], p, n0, mask, doff, dwid);
    }
  }
  if constexpr (kSkip > 0) {  // the last trip (its step 0 ran at the end of the loop)
    const uint32_t* ys = y + (kT - 1) * kLP;
#pragma unroll
    for (int r = 1; r < kL - kSkip; ++r) cios_step<FRIENDLY, SQR, false>(acc, x, r, ys[r], p, n0, mask, doff, dwid);
  }
  // two parallel carry passes -> limbs < 2^27 + 2^11 (enough headroom for the next op); limb j of the
  // result is accumulator register (kRot + j) % kL
  uint64_t d[kL];
  {
    const uint64_t top = acc[(kRot + kL - 1) % kL];
    uint64_t c_in = ((uint64_t)from_prev((uint32_t)(top >> kLimbBits)) |
                     ((uint64_t)from_prev((uint32_t)(top >> (kLimbBits + 32))) << 32));
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      const uint64_t c = (j == 0) ? c_in : (acc[(kRot + j - 1) % kL] >> kLimbBits);
      d[j] = (uint64_t)((uint32_t)acc[(kRot + j) % kL] & mask) + c;
    }
  }
  {
    const uint32_t c_in = from_prev((uint32_t)(d[kL - 1] >> kLimbBits));
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      const uint32_t c = (j == 0) ? c_in : (uint32_t)(d[j - 1] >> kLimbBits);
      x[j] = ((uint32_t)d[j] & mask) + c;
    }
  }
}

// Montgomery reduction  x <- x * R^-1 mod p  (leaving the Montgomery domain; result in [0, p]
// for x < 2p).  The CIOS schedule of mont_mul_impl with y = 1: its only product step adds x
// into the accumulator, so the accumulator starts as x and every step is the m * p half alone
// (18 v_mad_u64_u32 per step instead of 36).  Bit-identical to mont_mul(x, 1).
template <bool FRIENDLY, class PT>
__device__ __forceinline__ void mont_redc_impl(uint32_t (&x)[kL], const PT& p, uint32_t n0, uint32_t mask) {
  uint64_t acc[kL];
#pragma unroll
  for (int j = 0; j < kL; ++j) acc[j] = x[j];
  // one reduction step at rotation r (compile-time)
  auto rstep = [&](auto R) {
    constexpr int r = decltype(R)::value;
    uint32_t t0 = (uint32_t)acc[r % kL];
    if constexpr (!FRIENDLY) t0 *= n0;
    const uint32_t m = bcast_g0_and(t0, mask);
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      uint64_t& A = acc[(j + r) % kL];
      A = (uint64_t)p[j] * m + A;
    }
    uint64_t& A0 = acc[r % kL];
    acc[(r + 1) % kL] += A0 >> kLimbBits;
    A0 = (uint64_t)from_next_and((uint32_t)A0, mask);
  };
  // kSteps steps (R = 2^(b * kSteps)): full trips in the loop, then the last trip's first kL - kSkip
  constexpr int kFull = kSkip ? kT - 1 : kT;
#pragma unroll 1
  for (int s = 0; s < kFull; ++s) {
    rsteps<kL>(rstep);
  }
  if constexpr (kSkip > 0) rsteps<kL - kSkip>(rstep);
  uint64_t d[kL];
  {
    const uint64_t top = acc[(kRot + kL - 1) % kL];
    uint64_t c_in = ((uint64_t)from_prev((uint32_t)(top >> kLimbBits)) |
                     ((uint64_t)from_prev((uint32_t)(top >> (kLimbBits + 32))) << 32));
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      const uint64_t c = (j == 0) ? c_in : (acc[(kRot + j - 1) % kL] >> kLimbBits);
      d[j] = (uint64_t)((uint32_t)acc[(kRot + j) % kL] & mask) + c;
    }
  }
  {
    const uint32_t c_in = from_prev((uint32_t)(d[kL - 1] >> kLimbBits));
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      const uint32_t c = (j == 0) ? c_in : (uint32_t)(d[j - 1] >> kLimbBits);
      x[j] = ((uint32_t)d[j] & mask) + c;
    }
  }
}

template <bool FRIENDLY, class PT>
__device__ __forceinline__ void mont_mul(uint32_t (&x)[kL], const uint32_t* __restrict__ y,
                                         const PT& p, uint32_t n0, uint32_t mask) {
  mont_mul_impl<FRIENDLY, false>(x, y, p, n0, mask);
}

// ---- element I/O between VGPRs, LDS slots and the device element format ----

__device__ __forceinline__ void load_elem(uint32_t (&x)[kL], const uint32_t* __restrict__ src) {
  const uint32_t* s = src + glane() * kLP;
#pragma unroll
  for (int j = 0; j < kL; ++j) x[j] = s[j];
}

__device__ __forceinline__ void store_elem(uint32_t* __restrict__ dst, const uint32_t (&x)[kL]) {
  uint32_t* s = dst + glane() * kLP;
#pragma unroll
  for (int j = 0; j < kL; ++j) s[j] = x[j];
#pragma unroll
  for (int j = kL; j < kLP; ++j) s[j] = 0;
}

// copy a device element (global) into the group's LDS slot, each lane its block
__device__ __forceinline__ void elem_to_lds(uint32_t* __restrict__ slot, const uint32_t* __restrict__ src) {
  const int o = glane() * kLP;
  static_assert(kLP % 4 == 0, "");
#pragma unroll
  for (int j = 0; j < kLP; j += 4) {
    *reinterpret_cast<uint4*>(slot + o + j) = *reinterpret_cast<const uint4*>(src + o + j);
  }
}

__device__ __forceinline__ void regs_to_lds(uint32_t* __restrict__ slot, const uint32_t (&x)[kL]) {
  uint32_t* s = slot + glane() * kLP;
#pragma unroll
  for (int j = 0; j < kL; ++j) s[j] = x[j];
}

// ---- conversion between 512-byte big-endian (common.proto:6-10) and limbs ----

// Read bits [b, b+kLimbBits) of a little-endian word array of 128 words (zero above 4096).
__device__ __forceinline__ uint32_t bits_limb(const uint32_t* __restrict__ w, int b) {
  const int wi = b >> 5, sh = b & 31;
  const uint32_t lo = (wi < 128) ? w[wi] : 0u;
  const uint32_t hi = (wi + 1 < 128) ? w[wi + 1] : 0u;
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  return (uint32_t)(v >> sh) & kMask;
}

}  // namespace eg
