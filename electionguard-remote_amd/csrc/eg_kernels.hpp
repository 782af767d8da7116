// eg_kernels.hpp — HIP kernels for the batched ElectionGuard group path on gfx950.
//
// All kernels run one element per group of kT lanes (eg_bignum.hpp) with 256-thread
// workgroups and keep every Montgomery multiply WAVE-UNIFORM: per-launch shape
// parameters are kernel arguments and tail groups recompute a clamped element
// instead of branching out, so the DPP lane exchanges inside mont_mul never read
// a disabled lane.
#pragma once
#include "eg_bignum.hpp"
#include "eg_sha256.hpp"

namespace eg {

constexpr int kBlock = 256;
#ifndef EG_SQR
#define EG_SQR 1  // squarings use the symmetric-half CIOS (eg_bignum.hpp)
#endif
#ifndef EG_MASK_RT
#define EG_MASK_RT 2  // 2: limb mask pinned in a VGPR so both per-step ANDs fold into v_and_b32_dpp
#endif
#ifndef EG_TRAFFIC_X2
#define EG_TRAFFIC_X2 0  // A/B probe: extra HBM traffic at equal VALU count (never in production builds)
#endif
#ifndef EG_MIN_WAVES
#define EG_MIN_WAVES 3  // k_pow: 3 waves/SIMD (<= 168 VGPRs; a few squaring-loop spills, measured +1.3..1.6%)
#endif
constexpr int kGroupsPerBlock = kBlock / kT;
constexpr uint32_t kNone = 0xFFFFFFFFu;

struct FbTab {
  const uint32_t* data;  // (nwin << wbits) device elements, entry (k, d) = base^(d * 2^(wbits*k))
  uint32_t wbits;
  uint32_t nwin;
};

// Per-thread constants of the modulus (loaded once per kernel).  F = p is
// Montgomery-friendly (n0 == 1); every kernel is instantiated for both and the host
// picks one per context, so only one Montgomery body is inlined per kernel.
template <bool F>
struct Mont {
#if EG_PLDS
  const uint32_t* p;  // this lane's modulus block in LDS
#else
  uint32_t p[kL];
#endif
  uint32_t n0, mask;
  // Must be called by every thread of the block (EG_PLDS stages p with a barrier).
  __device__ __forceinline__ void load(const MontConsts* __restrict__ C) {
#if EG_PLDS
    __shared__ uint32_t s_p[kW];
    for (int i = threadIdx.x; i < kW; i += blockDim.x) s_p[i] = C->p[i];
    __syncthreads();
    p = s_p + glane() * kLP;
#else
    const uint32_t* s = C->p + glane() * kLP;
#pragma unroll
    for (int j = 0; j < kL; ++j) p[j] = s[j];
#endif
    n0 = C->n0;
#if EG_MASK_RT == 2
    mask = kMask;
    asm volatile("" : "+v"(mask));  // pin the mask in a VGPR (VOP2-DPP needs a VGPR src1)
#elif EG_MASK_RT
    mask = C->mask;  // run-time mask: lets the DPP combiner fold AND into v_and_b32_dpp
#else
    mask = kMask;
#endif
  }
  __device__ __forceinline__ void mul(uint32_t (&x)[kL], const uint32_t* y) const {
    mont_mul_impl<F, false>(x, y, p, n0, mask);
  }
  // x <- x * R^-1 (leave the Montgomery domain; no multiplier operand)
  __device__ __forceinline__ void redc(uint32_t (&x)[kL]) const { mont_redc_impl<F>(x, p, n0, mask); }
  // x <- x^2 (the slot must hold x); symmetric-half schedule (EG_SQR) or plain CIOS
  __device__ __forceinline__ void sqr(uint32_t (&x)[kL], const uint32_t* y) const {
#if EG_SQR
    mont_mul_impl<F, true>(x, y, p, n0, mask);
#else
    mont_mul_impl<F, false>(x, y, p, n0, mask);
#endif
  }
};

__device__ __forceinline__ uint32_t* group_slot() {
  __shared__ uint32_t s_slots[kGroupsPerBlock * kYStride];
  return s_slots + (threadIdx.x / kT) * kYStride;
}
__device__ __forceinline__ uint32_t group_id() { return blockIdx.x * kGroupsPerBlock + threadIdx.x / kT; }

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// x <- x * x
template <bool F>
__device__ __forceinline__ void msqr(const Mont<F>& M, uint32_t (&x)[kL], uint32_t* slot) {
  regs_to_lds(slot, x);
  wave_sync();
  M.sqr(x, slot);
  wave_sync();
}
// x <- x * E  (E a device element in global memory)
template <bool F>
__device__ __forceinline__ void mmul_g(const Mont<F>& M, uint32_t (&x)[kL], uint32_t* slot,
                                       const uint32_t* __restrict__ E) {
  elem_to_lds(slot, E);
  wave_sync();
  M.mul(x, slot);
  wave_sync();
}

// ---------------------------------------------------------------------------------
// Big-endian bytes <-> Montgomery form.
// ---------------------------------------------------------------------------------

// Stage one 512-byte big-endian element into the group slot as 128 LE words.
__device__ __forceinline__ void stage_be(uint32_t* slot, const uint8_t* __restrict__ be) {
  constexpr int kPer = 32 / kT;  // uint4 per lane
  const uint4* src = reinterpret_cast<const uint4*>(be);
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int idx = glane() * kPer + k;  // BE words 4idx..4idx+3
    const uint4 v = src[idx];
    slot[127 - 4 * idx] = __builtin_bswap32(v.x);
    slot[126 - 4 * idx] = __builtin_bswap32(v.y);
    slot[125 - 4 * idx] = __builtin_bswap32(v.z);
    slot[124 - 4 * idx] = __builtin_bswap32(v.w);
  }
}

// out[i] = be[i] * R mod p (Montgomery form); lt_p[i] = (be[i] < p) if lt_p != null
template <bool F>
__global__ void __launch_bounds__(kBlock) k_import(const MontConsts* __restrict__ C,
                                                   const uint8_t* __restrict__ be, uint32_t n,
                                                   uint32_t* __restrict__ out, uint8_t* __restrict__ lt_p) {
  const uint32_t gid = group_id();
  const uint32_t e = gid < n ? gid : n - 1;
  uint32_t* slot = group_slot();
  Mont<F> M;
  M.load(C);
  stage_be(slot, be + (size_t)e * 512);
  wave_sync();
  uint32_t x[kL];
#pragma unroll
  for (int j = 0; j < kL; ++j) x[j] = bits_limb(slot, kLimbBits * (glane() * kL + j));
  if (lt_p != nullptr) {
    // be < p: each lane compares its 128/kT words from the top; the most significant lane
    // that differs decides
    constexpr int kWords = 128 / kT;
    int cmp = 0;
#pragma unroll
    for (int i = kWords - 1; i >= 0; --i) {
      const int w = glane() * kWords + i;
      const uint32_t a = slot[w], b = C->pw[w];
      if (cmp == 0) cmp = a < b ? -1 : (a > b ? 1 : 0);
    }
    const uint32_t sh = gslot() * kT;
    const uint32_t lt = (uint32_t)(__ballot(cmp < 0) >> sh) & ((1u << kT) - 1u);
    const uint32_t ne = (uint32_t)(__ballot(cmp != 0) >> sh) & ((1u << kT) - 1u);
    if (glane() == 0 && gid < n) lt_p[gid] = ne ? (uint8_t)((lt >> (31 - __builtin_clz(ne))) & 1u) : 0;
  }
  wave_sync();
  elem_to_lds(slot, C->r2);
  wave_sync();
  M.mul(x, slot);
  if (gid < n) store_elem(out + (size_t)gid * kW, x);
}

// Canonical form of a value in [0, p] held in registers (this lane's kL limbs, limbs below
// 2^b + 2^(64-2b) + 1 as mont_mul leaves them): limbs < 2^b, and p -> 0.  The kT lanes of the
// group work in parallel: a local carry pass, then the carries between lanes ripple upward
// (a carry crosses a lane only through saturated limbs, so one round nearly always settles
// it; the loop runs until no lane receives a carry, at most kT rounds, and its exit is
// wave-uniform), then a group-wide equality test against p's limbs.
template <bool F>
__device__ __forceinline__ void regs_normalize(const Mont<F>& M, uint32_t (&x)[kL]) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kL; ++j) {
    const uint32_t v = x[j] + c;
    x[j] = v & kMask;
    c = v >> kLimbBits;
  }
  const bool g0 = glane() == 0;
  for (int round = 0; round < kT; ++round) {
    uint32_t cin = from_prev(c);  // carry out of the lane below (the group's top carry is 0: value < R)
    if (g0) cin = 0;
    if (__ballot(cin != 0) == 0) break;
    c = 0;
    if (cin) {
#pragma unroll
      for (int j = 0; j < kL; ++j) {
        const uint32_t v = x[j] + cin;
        x[j] = v & kMask;
        cin = v >> kLimbBits;
      }
      c = cin;
    }
  }
  bool eq = true;
#pragma unroll
  for (int j = 0; j < kL; ++j) eq &= x[j] == M.p[j];
  const uint64_t gmask = (uint64_t)((1u << kT) - 1u) << (gslot() * kT);
  if ((__ballot(!eq) & gmask) == 0) {
#pragma unroll
    for (int j = 0; j < kL; ++j) x[j] = 0;
  }
}

// 512 big-endian bytes of a canonical value held in the group slot (regs_normalize'd).
__device__ __forceinline__ void slot_to_be(uint32_t* slot, uint8_t* __restrict__ dst, bool do_store) {
  constexpr int kPer = 128 / kT;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int b = glane() * kPer + k;  // BE word index
    const int w = 127 - b;             // LE word index
    const int bit = 32 * w;
    const int a = bit / kLimbBits, sh = bit - a * kLimbBits;
    auto limb = [&](int i) -> uint64_t {
      return i < kN ? (uint64_t)slot[(i / kL) * kLP + (i % kL)] : 0ull;
    };
    const uint64_t v = (limb(a) >> sh) | (limb(a + 1) << (kLimbBits - sh)) |
                       (limb(a + 2) << (2 * kLimbBits - sh));
    if (do_store) reinterpret_cast<uint32_t*>(dst)[b] = __builtin_bswap32((uint32_t)v);
  }
}

template <bool F>
__global__ void __launch_bounds__(kBlock) k_export(const MontConsts* __restrict__ C,
                                                   const uint32_t* __restrict__ in, uint32_t n,
                                                   uint8_t* __restrict__ be) {
  const uint32_t gid = group_id();
  const uint32_t e = gid < n ? gid : n - 1;
  uint32_t* slot = group_slot();
  Mont<F> M;
  M.load(C);
  uint32_t x[kL];
  load_elem(x, in + (size_t)e * kW);
  M.redc(x);  // leave the Montgomery domain: value in [0, p]
  regs_normalize(M, x);
  regs_to_lds(slot, x);
  wave_sync();
  slot_to_be(slot, be + (size_t)gid * 512, gid < n);
}

// Canonical value in [0, p) of a lazy Montgomery-domain value in [0, 2p) held in registers
// (limbs as mont_mul leaves them): the carry passes of regs_normalize, then x >= p decided by
// the group's most significant differing limb (each lane compares its own limbs from the top,
// the highest lane with a difference decides; no difference = equal), and a group-uniform
// subtraction of p whose borrows ripple between lanes like the carries.
template <bool F>
__device__ __forceinline__ void regs_reduce_lazy(const Mont<F>& M, uint32_t (&x)[kL]) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kL; ++j) {
    const uint32_t v = x[j] + c;
    x[j] = v & kMask;
    c = v >> kLimbBits;
  }
  const bool g0 = glane() == 0;
  for (int round = 0; round < kT; ++round) {
    uint32_t cin = from_prev(c);
    if (g0) cin = 0;
    if (__ballot(cin != 0) == 0) break;
    c = 0;
    if (cin) {
#pragma unroll
      for (int j = 0; j < kL; ++j) {
        const uint32_t v = x[j] + cin;
        x[j] = v & kMask;
        cin = v >> kLimbBits;
      }
      c = cin;
    }
  }
  bool ne = false, gt = false;
#pragma unroll
  for (int j = 0; j < kL; ++j) {  // ascending: the last (most significant) difference wins
    if (x[j] != M.p[j]) { ne = true; gt = x[j] > M.p[j]; }
  }
  const uint32_t sh = gslot() * kT;
  const uint32_t nem = (uint32_t)(__ballot(ne) >> sh) & ((1u << kT) - 1u);
  const uint32_t gtm = (uint32_t)(__ballot(gt) >> sh) & ((1u << kT) - 1u);
  const bool ge = nem == 0 || ((gtm >> (31 - __builtin_clz(nem))) & 1u);
  if (__ballot(ge) == 0) return;  // no group of the wave needs the subtraction
  uint32_t b = 0;
  if (ge) {
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      const uint32_t v = x[j] - M.p[j] - b;
      x[j] = v & kMask;
      b = v >> 31;  // limbs < 2^29: a borrow leaves the top bit set
    }
  }
  for (int round = 0; round < kT; ++round) {
    uint32_t bin = from_prev(b);  // borrow out of the lane below (none out of the top: x >= p)
    if (g0) bin = 0;
    if (__ballot(bin != 0) == 0) break;
    b = 0;
    if (bin) {
#pragma unroll
      for (int j = 0; j < kL; ++j) {
        const uint32_t v = x[j] - bin;
        x[j] = v & kMask;
        bin = v >> 31;
      }
      b = bin;
    }
  }
}

// Residue (subgroup) test of n bases from their k_pow residue pairs (PowShape::resid):
//   pair i = (z, w) = (B^(2^256), B^c) in Montgomery form;  B^q == 1  <=>  z == w and B != 0
// (B^(2^256) = B^q * B^c, and B is invertible unless B == 0, where z = w = 0).  zR == wR (mod p)
// iff z == w, and zR == 0 iff z == 0, so the test runs on the Montgomery forms reduced to
// [0, p) with no multiply.  flags[i * fstride] &= verdict — the per-element range flag of the
// verifier (k_import).  Cost: two lane-parallel reductions per base (no MM).
template <bool F>
__global__ void __launch_bounds__(kBlock) k_resid_check(const MontConsts* __restrict__ C,
                                                        const uint32_t* __restrict__ pairs, uint32_t n,
                                                        uint8_t* __restrict__ flags, uint32_t fstride) {
  const uint32_t gid = group_id();
  const uint32_t e = gid < n ? gid : n - 1;
  Mont<F> M;
  M.load(C);
  uint32_t z[kL], x[kL];
  load_elem(z, pairs + (size_t)e * 2 * kW);
  load_elem(x, pairs + ((size_t)e * 2 + 1) * kW);
  regs_reduce_lazy(M, z);
  regs_reduce_lazy(M, x);
  bool eq = true, nz = false;
#pragma unroll
  for (int j = 0; j < kL; ++j) {
    eq &= z[j] == x[j];
    nz |= z[j] != 0;
  }
  const uint64_t neq = __ballot(!eq), nzb = __ballot(nz);
  const uint64_t gmask = (uint64_t)((1u << kT) - 1u) << (gslot() * kT);
  if (glane() == 0 && gid < n) {
    const bool ok = (neq & gmask) == 0 && (nzb & gmask) != 0;
    if (!ok) flags[(size_t)gid * fstride] = 0;
  }
}

// A contest's message flags (A, B) = (prod alpha_i, prod beta_i) from its selections' flags: the
// order-q subgroup is closed under products, so A is a valid residue when every alpha_i is one
// (range + residue flags, k_import / k_resid_check), and a contest with an invalid selection is
// rejected with it.  One thread per (contest, component); flags[(j spc + s) * 2 + comp].
__global__ void __launch_bounds__(kBlock) k_contest_flags(const uint8_t* __restrict__ sel_flags, uint32_t ncn,
                                                          uint32_t spc, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ncn * 2) return;
  const size_t base = (size_t)(i >> 1) * spc * 2 + (i & 1u);
  uint8_t ok = 1;
  for (uint32_t s = 0; s < spc; ++s) ok &= sel_flags[base + (size_t)s * 2];
  out[i] = ok;
}

// out[i*so] = a[i*sa] * b[i*sb]  (Montgomery form; strides in elements)
template <bool F>
__global__ void __launch_bounds__(kBlock) k_mul(const MontConsts* __restrict__ C,
                                                const uint32_t* __restrict__ a, uint32_t sa,
                                                const uint32_t* __restrict__ b, uint32_t sb, uint32_t n,
                                                uint32_t* __restrict__ out, uint32_t so) {
  const uint32_t gid = group_id();
  const uint32_t e = gid < n ? gid : n - 1;
  uint32_t* slot = group_slot();
  Mont<F> M;
  M.load(C);
  uint32_t x[kL];
  load_elem(x, a + (size_t)e * sa * kW);
  mmul_g(M, x, slot, b + (size_t)e * sb * kW);
  if (gid < n) store_elem(out + (size_t)gid * so * kW, x);
}

// ---------------------------------------------------------------------------------
// Exponentiation jobs.
//   job record (kJobWords u32): base, e0, e1, out0, out1, f00, f01, f10, f11
//   base    : element index of the variable base (kNone = no variable part)
//   e0/e1   : scalar indices (32-B BE) of the variable-base exponents
//   out0/1  : output element indices
//   fXY     : scalar index of fixed-base term Y of output X
// Launch-uniform shape: nout (1|2), nfb0/nfb1 (0..2), tab[X][Y] in {0,1} = which FbTab.
// Variable part: fixed 4-bit window, table base^0..base^15 in per-group scratch.
// ---------------------------------------------------------------------------------
constexpr int kJobWords = 9;

struct PowShape {
  uint32_t has_base, nout, nfb[2], tab[2][2];
  uint32_t exp_bytes;  // variable-base exponent length (32, or 512 for inverses)
  uint32_t comb;       // 1: Lim-Lee comb (h = 5) shared by the job's exponents (32-byte only)
  uint32_t gather;     // comb jobs whose base is a PRODUCT of `gather` earlier comb bases (the contest
                       // aggregates A = prod alpha, B = prod beta): y_k = prod of their y_k (ygat,
                       // job J[2] onwards) instead of 208 squarings; 0 = none
  uint32_t resid;      // comb jobs (not gather): also write the residue-test pair of the base B,
                       // z = B^(2^256) (the squaring chain run to the end) and w = B^c, c = 2^256 - q, to
                       // rout[2 gid], rout[2 gid + 1]; B^q == 1 iff z == w and B != 0 (k_resid_check)
  uint32_t shared_comb;  // comb jobs whose 32-entry subset table is PowPart::ctab (one table for every
                         // job, e.g. the trustee's g^u): no per-job precompute
  uint32_t blocks;     // Lim-Lee column blocks v of a plain comb (0/1: one block of cw columns, one
                       // 2^h-entry table; 2 or 3: blocks of ceil(cw / v) columns, tables of
                       // B^(2^(cw r + bw t)), v * 2^h entries).  v > 1 pays when the squaring chain
                       // runs to 2^256 anyway (resid)
  uint32_t rows;       // Lim-Lee rows h of a plain comb (0: kCombH = 5 rows of 52 bits, 32-entry
                       // tables; 4: rows of 64 bits, 16-entry tables -- the constant-time trustee
                       // pair, whose masked scans read every entry of a table, and the EG_SEL_COMB=43
                       // selection jobs, 4 rows x 3 blocks)
  uint32_t fb_small[2][2];  // fixed-base term [o][t] whose scalar is < 2^wbits (the vote m of
                            // beta = K^R g^m): only radix window 0 is applied (host schedule only)
};

// Constant-time table read for secret digits (k_pow<F, CT = true>, the trustee's shares):
// every entry of the table is read and the wanted one kept with a mask, so the addresses a
// job touches do not depend on the digit d.  Each lane selects its own 20-word block.
__device__ __forceinline__ void ct_select_to_lds(uint32_t* __restrict__ slot, const uint32_t* __restrict__ tbl,
                                                 uint32_t h, uint32_t d) {
  // d = block << h | digit: the column block is public (fixed by the column index), so only
  // its 2^h entries are scanned; the digit selects among them by mask
  const int nent = 1 << h;
  tbl += (size_t)(d >> h << h) * kW;
  d &= (uint32_t)nent - 1u;
  const int o = glane() * kLP;
  uint4 acc[kLP / 4];
#pragma unroll
  for (int j = 0; j < kLP / 4; ++j) acc[j] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll 1
  for (int e = 0; e < nent; ++e) {
    const uint32_t m = 0u - (uint32_t)((uint32_t)e == d);
    const uint4* src = reinterpret_cast<const uint4*>(tbl + (size_t)e * kW + o);
#pragma unroll
    for (int j = 0; j < kLP / 4; ++j) {
      const uint4 v = src[j];
      acc[j].x |= v.x & m;
      acc[j].y |= v.y & m;
      acc[j].z |= v.z & m;
      acc[j].w |= v.w & m;
    }
  }
#pragma unroll
  for (int j = 0; j < kLP / 4; ++j) *reinterpret_cast<uint4*>(slot + o + 4 * j) = acc[j];
}

// Lim-Lee comb parameters for 256-bit exponents: 5 rows of 52 bits (PowShape::rows = 4: 4 rows of 64).
constexpr int kCombH = 5;
constexpr int kCombW = 52;
__host__ __device__ constexpr uint32_t comb_rows(uint32_t rows) { return rows ? rows : (uint32_t)kCombH; }
__host__ __device__ constexpr uint32_t comb_width(uint32_t rows) { return (256u + comb_rows(rows) - 1u) / comb_rows(rows); }
// Lim-Lee column blocks v (PowShape::blocks: 0 or 1 = one table, 2 or 3 tables of 2^h entries)
// and the columns per block, ceil(cw / v) (the last block may be shorter)
__host__ __device__ constexpr uint32_t comb_blocks(uint32_t blocks) { return blocks > 1 ? blocks : 1u; }
__host__ __device__ constexpr uint32_t comb_block_width(uint32_t rows, uint32_t blocks) {
  return (comb_width(rows) + comb_blocks(blocks) - 1u) / comb_blocks(blocks);
}

__device__ __forceinline__ uint32_t be_digit(const uint8_t* __restrict__ e, int nbytes, int bit, int wb) {
  uint32_t v = 0;
  const int b0 = bit >> 3;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = nbytes - 1 - (b0 + i);
    if (idx >= 0) v |= (uint32_t)e[idx] << (8 * i);
  }
  return (v >> (bit & 7)) & ((1u << wb) - 1u);
}

// A k_pow job is a straight-line program over one register element x (its group's 8 lanes):
// the host compiles every launch shape into a list of op words (pow_schedule in eg_capi.hip),
// the same list for every job of the launch, and k_pow interprets it.  The op word is read
// with a scalar load and every branch is wave-uniform; only the operands differ per job
// (the base J[0], exponents J[1..2], fixed-base scalars J[5..8] and outputs J[3..4]).
// Keeping the control state to one program counter (instead of a phase state machine)
// leaves the multiply bodies with fewer live registers and no per-multiply bookkeeping.
//   op = kind | arg << kOpShift
enum PowOp : uint32_t {
  OP_END = 0,
  OP_SQR,         // x <- x^2
  OP_MUL_BASE,    // x <- x * B
  OP_MUL_TBL,     // x <- x * tbl[arg]
  OP_MUL_WIN,     // x <- x * tbl[nibble w of exponent J[1 + o]], arg = w | o << 12 (4-bit window, MSB first)
  OP_MUL_COMB,    // x <- x * tbl[dig[arg]]                      (Lim-Lee column arg)
  OP_MUL_GATHER,  // x <- x * y_{k}(job J[2] + i), arg = i << 2 | (k - 1)
  OP_MUL_FB,      // x <- x * T[kf][digit kf of scalar J[5 + 2o + t]], arg = fb_arg(o, t, tab, kf)
  OP_LOAD_ONE,    // x <- R mod p
  OP_LOAD_BASE,   // x <- B
  OP_LOAD_TBL,    // x <- tbl[arg]
  OP_LOAD_WIN,    // x <- tbl[nibble 0 of exponent J[1 + arg]]
  OP_LOAD_COMB,   // x <- tbl[dig[arg]]
  OP_LOAD_GATHER, // x <- y_{arg + 1}(job J[2])
  OP_LOAD_FB,     // x <- T[kf][digit], arg as OP_MUL_FB
  OP_STORE_TBL,   // tbl[arg] <- x
  OP_STORE_Y,     // yout[job][arg] <- x                         (if the part has yout)
  OP_STORE_R,     // rout[job][arg] <- x                         (residue pair)
  OP_STORE_OUT,   // out[J[3 + arg]] <- x
  OP_EXP,         // comb shapes: spread the column digits of exponent J[1 + arg] to dig[]
};
constexpr uint32_t kOpShift = 5;
constexpr uint32_t kOpMulLast = OP_MUL_FB;
__host__ __device__ constexpr uint32_t pow_op(PowOp k, uint32_t arg = 0) { return (uint32_t)k | (arg << kOpShift); }
// fixed-base operand: window kf (< 256) of term t (< 2) of output o (< 2) from table tab (0 = fb0)
__host__ __device__ constexpr uint32_t fb_arg(uint32_t o, uint32_t t, uint32_t tab, uint32_t kf) {
  return kf | (t << 8) | (o << 9) | (tab << 10);
}

// One launch may carry up to three job populations of different shapes (e.g. the beta jobs,
// the contest-A jobs that only depend on the previous launch and the contest-B jobs whose
// betas the previous launch finished): part 0 owns the first P0.nblocks workgroups, part 1 the
// next P1.nblocks, part 2 the rest, so the short jobs of parts 1-2 fill the tail of part 0
// instead of running as a separate, under-filled launch.  The shape stays workgroup-uniform.
struct PowPart {
  PowShape S;
  const uint32_t* sched;  // the shape's op program (pow_schedule), OP_END-terminated
  const uint32_t* jobs;
  uint32_t njobs;
  uint32_t nblocks;   // workgroups of this part
  uint32_t* scratch;  // per-group table (comb: 32 elements, window: 16)
  uint32_t* yout;     // comb y_1..y_4 per job (optional)
  const uint32_t* ygat;  // gather source (S.gather > 0)
  uint32_t* rout;        // residue-test pairs (S.resid), 2 device elements per job
  const uint32_t* ctab;  // shared comb subset table (S.shared_comb), 32 device elements
};

// CT = true: the constant-time instantiation for secret exponents (trustee shares s_i and
// P_l(x_i), proof nonces u; encryption nonces R, u and the vote with eg_ctx_set_ct_encrypt).
// Comb shapes, 4-bit window shapes (variable-base powP with eg_ctx_set_ct_pow: the window
// schedule is fixed, 4 squarings + 1 multiply per nibble, a zero nibble multiplies by tbl[0] = 1)
// and small-window radix fixed-base terms: every comb- or window-table read is ct_select_to_lds
// over the block's whole table, every fixed-base read over the window's whole column, and the
// square/multiply schedule is fixed by the shape, so neither time nor addresses depend on
// exponent bits.
template <bool F, bool CT>
__global__ void __launch_bounds__(kBlock, EG_MIN_WAVES) k_pow(const MontConsts* __restrict__ C, PowPart P0,
                                                PowPart P1, PowPart P2, const uint32_t* __restrict__ elems,
                                                const uint8_t* __restrict__ scalars,
                                                uint32_t* __restrict__ out, FbTab fb0, FbTab fb1,
                                                uint64_t* __restrict__ clk) {
  __shared__ uint8_t s_dig[kGroupsPerBlock][64];
  // clk (profiling only): per workgroup, shader-clock ticks (s_memtime) and 100 MHz real-time
  // ticks (s_memrealtime) from its start to its end; the host reports the median per-workgroup
  // ratio (eg_clock_median), the in-kernel clock of MI355X_MICROARCH.md 'DVFS give-back' item 6
  const uint64_t cyc0 = clk ? __builtin_amdgcn_s_memtime() : 0, wall0 = clk ? __builtin_amdgcn_s_memrealtime() : 0;
  const uint32_t b01 = P0.nblocks + P1.nblocks;
  const uint32_t part = blockIdx.x < P0.nblocks ? 0u : (blockIdx.x < b01 ? 1u : 2u);
  // kernarg memory: shape fields stay scalar loads
  const PowPart& P = part == 0 ? P0 : (part == 1 ? P1 : P2);
  const PowShape& S = P.S;
  // the op program is read-only for the kernel's lifetime: through the constant address space
  // its words are scalar loads (s_load), not vector loads plus readfirstlane
  typedef __attribute__((address_space(4))) const uint32_t const_u32;
  const const_u32* sched = (const const_u32*)P.sched;
  const uint32_t njobs = P.njobs;
  const uint32_t gid0 = (blockIdx.x - (part == 0 ? 0u : (part == 1 ? P0.nblocks : b01))) * kGroupsPerBlock;  // wave-uniform
  uint32_t* slot = group_slot();
  uint8_t* dig = s_dig[threadIdx.x / kT];
  Mont<F> M;
  M.load(C);
  uint32_t x[kL];
  const uint32_t ch = comb_rows(S.rows);  // comb rows: table entries per column block = 2^ch
  const uint32_t tsize = S.comb ? (comb_blocks(S.blocks) << ch) : 16u;
  const uint32_t gid = gid0 + threadIdx.x / kT;
  const bool live = gid < njobs;  // tail groups recompute job njobs-1 and store nothing
  const uint32_t* J = P.jobs + (size_t)(live ? gid : njobs - 1) * kJobWords;
  // shared comb table (read-only: the schedule has no precompute) or the job's scratch table
  uint32_t* tbl = (S.comb && S.shared_comb) ? const_cast<uint32_t*>(P.ctab) : P.scratch + (size_t)gid * tsize * kW;
  const uint32_t* B = (S.has_base && !S.shared_comb) ? elems + (size_t)J[0] * kW : nullptr;

  // Outer loop: one Montgomery multiply (or square) per trip, at a single inlined site; the
  // inner loop runs the program's loads, stores and digit spreads up to the next multiply.
  uint32_t pc = 0;
  while (true) {
    uint32_t op = sched[pc++];
    uint32_t kind = op & ((1u << kOpShift) - 1u), arg = op >> kOpShift;
    // loads, stores and digit spreads up to the next multiply; the multiply kinds (OP_SQR ..
    // OP_MUL_FB) leave this loop without passing through any handler that rewrites x, so the
    // multiply site keeps x in the registers the handlers use (no copies on the hot path)
    while (kind > kOpMulLast) {
      if (kind == OP_LOAD_FB) {
        const FbTab& T = (arg >> 10) ? fb1 : fb0;
        const uint32_t kf = arg & 255u;
        const uint32_t d = be_digit(scalars + (size_t)J[5 + 2 * ((arg >> 9) & 1u) + ((arg >> 8) & 1u)] * 32, 32,
                                    kf * T.wbits, T.wbits);
        if constexpr (CT) {
          // secret scalar (encryption nonces, the vote): masked scan of the window's whole
          // column of 2^wbits entries (small tables only, eg_ctx_set_ct_encrypt)
          ct_select_to_lds(slot, T.data + (size_t)(kf << T.wbits) * kW, T.wbits, d);
          wave_sync();
          load_elem(x, slot);
          wave_sync();
        } else {
          load_elem(x, T.data + ((size_t)(kf << T.wbits) + d) * kW);
        }
      } else {
        switch (kind) {
          case OP_LOAD_ONE: load_elem(x, C->one); break;
          case OP_LOAD_BASE: load_elem(x, B); break;
          case OP_LOAD_TBL: load_elem(x, tbl + (size_t)arg * kW); break;
          case OP_LOAD_WIN: {
            const uint32_t d = scalars[(size_t)J[1 + arg] * S.exp_bytes] >> 4;
            if constexpr (CT) {  // secret exponent (eg_ctx_set_ct_pow): masked scan of the 16-entry table
              ct_select_to_lds(slot, tbl, 4, d);
              wave_sync();
              load_elem(x, slot);
              wave_sync();
            } else {
              load_elem(x, tbl + (size_t)d * kW);
            }
            break;
          }
          case OP_LOAD_COMB:
            if constexpr (CT) {
              ct_select_to_lds(slot, tbl, ch, dig[arg]);
              wave_sync();
              load_elem(x, slot);
              wave_sync();
            } else {
              load_elem(x, tbl + (size_t)dig[arg] * kW);
            }
            break;
          case OP_LOAD_GATHER: load_elem(x, P.ygat + ((size_t)J[2] * (kCombH - 1) + arg) * kW); break;
          case OP_STORE_TBL: store_elem(tbl + (size_t)arg * kW, x); break;
          case OP_STORE_Y:
            if (P.yout != nullptr && live) store_elem(P.yout + ((size_t)gid * (kCombH - 1) + arg) * kW, x);
            break;
          case OP_STORE_R:
            if (live) store_elem(P.rout + ((size_t)gid * 2 + arg) * kW, x);
            break;
          case OP_STORE_OUT:
            if (live) store_elem(out + (size_t)J[3 + arg] * kW, x);
            break;
          case OP_EXP:
            if (S.comb) {
              // column digits of exponent J[1 + arg]: bit j of each of the h rows (cw bits each);
              // with v column blocks of bw = ceil(cw / v) columns, column j indexes table j / bw
              // (entry (j / bw) * 2^h + digit)
              const uint8_t* e = scalars + (size_t)J[1 + arg] * 32;
              const int cw = (int)comb_width(S.rows);
              const int bw = (int)comb_block_width(S.rows, S.blocks);
              wave_sync();
              for (int j = glane(); j < cw; j += kT) {
                uint32_t d = (uint32_t)(j / bw) << ch;
#pragma unroll
                for (int r = 0; r < kCombH; ++r) {
                  const int bit = r * cw + j;
                  if (r < (int)ch && bit < 256) d |= (((uint32_t)e[31 - (bit >> 3)] >> (bit & 7)) & 1u) << r;
                }
                dig[j] = (uint8_t)d;
              }
              wave_sync();
            }
            break;
          default: break;
        }
      }
      op = sched[pc++];
      kind = op & ((1u << kOpShift) - 1u);
      arg = op >> kOpShift;
    }
    if (kind == OP_END) break;
    // the multiply's operand: nullptr = square
    const uint32_t* ysrc = nullptr;
    const uint32_t* fb_col = nullptr;  // CT: the fixed-base window column the multiply scans
    uint32_t fb_h = 0, fb_d = 0;
    if (kind == OP_MUL_BASE) ysrc = B;
    else if (kind == OP_MUL_TBL) ysrc = tbl + (size_t)arg * kW;
    else if (kind == OP_MUL_WIN) {  // arg = w | o << 12
      const uint32_t w = arg & 4095u;
      const uint32_t byte = scalars[(size_t)J[1 + (arg >> 12)] * S.exp_bytes + (w >> 1)];
      ysrc = tbl + (size_t)((w & 1) ? (byte & 15u) : (byte >> 4)) * kW;
      fb_d = (w & 1) ? (byte & 15u) : (byte >> 4);  // CT: the window digit the masked scan selects
    } else if (kind == OP_MUL_COMB) ysrc = tbl + (size_t)dig[arg] * kW;
    else if (kind == OP_MUL_GATHER) ysrc = P.ygat + ((size_t)(J[2] + (arg >> 2)) * (kCombH - 1) + (arg & 3u)) * kW;
    else if (kind == OP_MUL_FB) {
      const FbTab& T = (arg >> 10) ? fb1 : fb0;
      const uint32_t kf = arg & 255u;
      const uint32_t d = be_digit(scalars + (size_t)J[5 + 2 * ((arg >> 9) & 1u) + ((arg >> 8) & 1u)] * 32, 32,
                                  kf * T.wbits, T.wbits);
      fb_col = T.data + (size_t)(kf << T.wbits) * kW;
      fb_h = T.wbits;
      fb_d = d;
      ysrc = fb_col + (CT ? 0 : (size_t)d * kW);
    }
    // ---- the one Montgomery multiply (or square) ----
    if (ysrc) {
      if constexpr (CT) {
        if (kind == OP_MUL_COMB) ct_select_to_lds(slot, tbl, ch, dig[arg]);  // secret digit
        else if (kind == OP_MUL_FB) ct_select_to_lds(slot, fb_col, fb_h, fb_d);
        else if (kind == OP_MUL_WIN) ct_select_to_lds(slot, tbl, 4, fb_d);  // secret nibble
        else elem_to_lds(slot, ysrc);
      } else {
        elem_to_lds(slot, ysrc);
#if EG_TRAFFIC_X2
        // A/B probe only (tools/ab_mm.py): every comb multiply also reads the same entry of the
        // table of a job 7 workgroups away (an L2 miss) into a discarded LDS block, adding ~60%
        // HBM traffic at nearly equal VALU count
        if (kind == OP_MUL_COMB && !S.shared_comb) {
          __shared__ uint32_t s_sink[kGroupsPerBlock * kT];
          const uint32_t ngr = P.nblocks * kGroupsPerBlock;
          const uint32_t og = (gid + 7u * kGroupsPerBlock) % ngr;
          const uint32_t* far = P.scratch + (size_t)og * tsize * kW + (size_t)dig[arg] * kW;
          const uint32_t* src = far + glane() * kLP;
          uint32_t acc = 0;
#pragma unroll 1
          for (int j = 0; j < kLP; j += 4) acc ^= src[j] ^ src[j + 1] ^ src[j + 2] ^ src[j + 3];
          reinterpret_cast<volatile uint32_t*>(s_sink)[threadIdx.x] = acc;
        }
#endif
      }
      wave_sync();
      M.mul(x, slot);
    } else {
      regs_to_lds(slot, x);
      wave_sync();
      M.sqr(x, slot);
    }
    wave_sync();
  }
  if (clk && threadIdx.x == 0) {
    clk[2 * (size_t)blockIdx.x] = __builtin_amdgcn_s_memtime() - cyc0;
    clk[2 * (size_t)blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - wall0;
  }
}

// ---------------------------------------------------------------------------------
// Product reduction.  Group g is addressed by a mixed-radix decomposition
//   g = (d2 * R1 + d1) * R0 + d0,  offset(g) = d2*M2 + d1*M1 + d0*M0   (elements)
// and its k-th element sits at offset(g) + k*stride.  Job j -> group j / nchunk,
// chunk j % nchunk; every job runs exactly `chunk`-1 multiplies (missing elements
// are R mod p, the Montgomery one) so all groups of a wave stay in lock-step.
// mask (optional): element k of every group takes part only if mask[k] != 0, else it counts
// as the Montgomery one (the tally over CAST ballots: k = ballot, mask = the cast flags); the
// selection only picks the operand's address, so the wave stays uniform.
// ---------------------------------------------------------------------------------
struct GroupMap {
  uint32_t R0, R1, M0, M1, M2;
  __device__ __forceinline__ size_t offset(uint32_t g) const {
    const uint32_t d0 = g % R0, t = g / R0;
    const uint32_t d1 = t % R1, d2 = t / R1;
    return (size_t)d2 * M2 + (size_t)d1 * M1 + (size_t)d0 * M0;
  }
};

template <bool F>
__global__ void __launch_bounds__(kBlock) k_prod(const MontConsts* __restrict__ C,
                                                 const uint32_t* __restrict__ in, GroupMap gm, uint32_t ngroups,
                                                 uint32_t len, uint32_t stride, uint32_t chunk,
                                                 uint32_t nchunk, uint32_t* __restrict__ out,
                                                 const uint8_t* __restrict__ mask) {
  const uint32_t gid = group_id();
  const uint32_t njobs = ngroups * nchunk;
  const uint32_t jb = gid < njobs ? gid : njobs - 1;
  const uint32_t g = jb / nchunk, c = jb % nchunk;
  uint32_t* slot = group_slot();
  Mont<F> M;
  M.load(C);
  uint32_t x[kL];
  const size_t base = gm.offset(g);
  const uint32_t k0 = c * chunk;
  const bool in0 = k0 < len && (mask == nullptr || mask[k0] != 0);
  load_elem(x, in0 ? in + (base + (size_t)k0 * stride) * kW : C->one);
#pragma unroll 1
  for (uint32_t k = 1; k < chunk; ++k) {
    const uint32_t kk = k0 + k;
    const bool use = kk < len && (mask == nullptr || mask[kk] != 0);
    const uint32_t* E = use ? in + (base + (size_t)kk * stride) * kW : C->one;
    mmul_g(M, x, slot, E);
  }
  if (gid < njobs) store_elem(out + (size_t)gid * kW, x);
}

// ---------------------------------------------------------------------------------
// Fixed-base table construction.
// k_sqr_chain: one group; P[j] = base^(2^j), j = 0..count-1 (Montgomery form).
// k_fb_level : entries (k, 2^a + b) = (k, 2^a) * (k, b) for b in [1, 2^a).
// ---------------------------------------------------------------------------------
template <bool F>
__global__ void __launch_bounds__(kBlock) k_sqr_chain(const MontConsts* __restrict__ C,
                                                      const uint32_t* __restrict__ base, uint32_t count,
                                                      uint32_t* __restrict__ P) {
  uint32_t* slot = group_slot();
  Mont<F> M;
  M.load(C);
  uint32_t x[kL];
  load_elem(x, base);
  const bool leader = group_id() == 0;
  if (leader) store_elem(P, x);
#pragma unroll 1
  for (uint32_t j = 1; j < count; ++j) {
    msqr(M, x, slot);
    if (leader) store_elem(P + (size_t)j * kW, x);
  }
}

template <bool F>
__global__ void __launch_bounds__(kBlock) k_fb_level(const MontConsts* __restrict__ C, uint32_t* __restrict__ tab,
                                                     uint32_t wbits, uint32_t nwin, uint32_t a) {
  const uint32_t per = (1u << a) - 1u;
  const uint32_t njobs = nwin * per;
  const uint32_t gid = group_id();
  const uint32_t jb = gid < njobs ? gid : njobs - 1;
  const uint32_t k = jb / per, b = 1 + jb % per;
  uint32_t* slot = group_slot();
  Mont<F> M;
  M.load(C);
  uint32_t x[kL];
  uint32_t* row = tab + ((size_t)k << wbits) * kW;
  load_elem(x, row + ((size_t)1 << a) * kW);
  mmul_g(M, x, slot, row + (size_t)b * kW);
  if (gid < njobs) store_elem(row + (size_t)((1u << a) + b) * kW, x);
}

// ---------------------------------------------------------------------------------
// LDS-staged fixed-base powP (A/B only: EG_FB_LDS=1 on eg_fb_pow_batch_dev with a 7-bit table).
// The north_star's plan for fixed-base g / K, batch-major: a workgroup of 96 element
// groups walks the radix windows in order; for window k the whole workgroup first copies the
// window's table slice (2^7 entries x 640 B = 80 KiB) from HBM / L2 into LDS, then every group
// multiplies its accumulator by the entry its digit selects, straight out of LDS (the multiplier
// operand of mont_mul is the LDS entry: no per-multiply copy).  Every group multiplies in every
// window (entry 0 is the Montgomery one) so the wave stays uniform.  One workgroup per CU (the
// slice fills half the LDS and a second would not fit beside the first's modulus copy).
// ---------------------------------------------------------------------------------
constexpr int kLdsWin = 7;
constexpr int kLdsBlock = 768;                  // 12 waves: 3 per SIMD at k_pow's register budget
constexpr int kLdsGroups = kLdsBlock / kT;      // 96 elements per workgroup
template <bool F>
__global__ void __launch_bounds__(kLdsBlock, 1) k_fb_lds(const MontConsts* __restrict__ C,
                                                       const uint32_t* __restrict__ tab, uint32_t nwin,
                                                       const uint8_t* __restrict__ exps, uint32_t n,
                                                       uint32_t* __restrict__ out) {
  __shared__ uint4 s_slice[((size_t)1 << kLdsWin) * kW / 4];
  Mont<F> M;
  M.load(C);
  const uint32_t g = blockIdx.x * kLdsGroups + threadIdx.x / kT;
  const bool live = g < n;
  const uint8_t* e = exps + (size_t)(live ? g : n - 1) * 32;
  const uint32_t* slice = reinterpret_cast<const uint32_t*>(s_slice);
  uint32_t x[kL];
#pragma unroll 1
  for (uint32_t k = 0; k < nwin; ++k) {
    __syncthreads();  // every group is done with the previous slice
    const uint4* src = reinterpret_cast<const uint4*>(tab + ((size_t)k << kLdsWin) * kW);
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < ((uint32_t)1 << kLdsWin) * kW / 4; i += kLdsBlock) s_slice[i] = src[i];
    __syncthreads();
    const uint32_t d = be_digit(e, 32, (int)(k * kLdsWin), kLdsWin);
    if (k == 0) {
      load_elem(x, slice + (size_t)d * kW);
    } else {
      M.mul(x, slice + (size_t)d * kW);
    }
  }
  if (live) store_elem(out + (size_t)g * kW, x);
}

// ---------------------------------------------------------------------------------
// 256-bit scalar helpers (one thread per scalar).  Scalars are 32-B big-endian.
// ---------------------------------------------------------------------------------
struct U256 {
  uint32_t w[8];  // little-endian words
};
__device__ __forceinline__ U256 ld256(const uint8_t* __restrict__ be) {
  U256 r;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(be);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = __builtin_bswap32(s[7 - i]);
  return r;
}
__device__ __forceinline__ void st256(uint8_t* __restrict__ be, const U256& a) {
  uint32_t* d = reinterpret_cast<uint32_t*>(be);
#pragma unroll
  for (int i = 0; i < 8; ++i) d[7 - i] = __builtin_bswap32(a.w[i]);
}
// The mod-q helpers below are branch-free in their operands (trustee responses v = u - c s and
// the encryption's R c_fake touch secrets): a < b is the borrow of a - b, selections are masks.
__device__ __forceinline__ bool lt256(const U256& a, const U256& b) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (int64_t)a.w[i] - (int64_t)b.w[i];
    c >>= 32;
  }
  return c != 0;
}
__device__ __forceinline__ U256 sel256(uint32_t mask, const U256& a, const U256& b) {  // mask ? a : b
  U256 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = (a.w[i] & mask) | (b.w[i] & ~mask);
  return r;
}
__device__ __forceinline__ uint32_t add256(U256& a, const U256& b) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.w[i] + b.w[i];
    a.w[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}
__device__ __forceinline__ uint32_t sub256(U256& a, const U256& b) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (int64_t)a.w[i] - (int64_t)b.w[i];
    a.w[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)(c & 1);
}
// (a + b) mod q for a, b < q
__device__ __forceinline__ U256 addmod256(U256 a, const U256& b, const U256& q) {
  const uint32_t carry = add256(a, b);
  U256 t = a;
  const uint32_t borrow = sub256(t, q);
  return sel256(0u - (carry | (borrow ^ 1u)), t, a);  // subtract q iff a + b >= q
}
// (L * a) mod q for a < q, L < 2^32  (schoolbook + repeated subtraction-free fold)
__device__ __forceinline__ U256 mulsmall_mod(const U256& a, uint32_t L, const U256& q) {
  // r = L*a as 288-bit, then reduce by long division on the top word
  uint32_t r[9];
  uint64_t c = 0;
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.w[i] * L;
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  r[8] = (uint32_t)c;
  U256 x;
  for (int i = 0; i < 8; ++i) x.w[i] = r[i];
  // subtract hi * q repeatedly: value = r8*2^256 + x; x < 2^256, r8 < L
  // reduce via q's structure-free approach: while (r8 || x >= q) x -= q (with borrow into r8)
  uint32_t hi = r[8];
  while (hi != 0 || !lt256(x, q)) {
    const uint32_t borrow = sub256(x, q);
    hi -= borrow;
  }
  return x;
}
__device__ __forceinline__ U256 negmod(const U256& a, const U256& q) {  // (q - a) mod q, branch-free
  uint32_t nz = 0;
  for (int i = 0; i < 8; ++i) nz |= a.w[i];
  U256 r = q;
  sub256(r, a);
  return sel256(0u - (uint32_t)(nz != 0), r, a);
}

// (a - b) mod q for a, b < q
__device__ __forceinline__ U256 submod256(U256 a, const U256& b, const U256& q) {
  const uint32_t borrow = sub256(a, b);
  U256 t = a;
  add256(t, q);
  return sel256(0u - borrow, t, a);
}
// (a * b) mod q for a, b < q: left-to-right double-and-always-add with a masked select (one
// thread; per proof, not per limb), so neither operand's bits steer the control flow
__device__ __noinline__ U256 mulmod256(const U256& a, const U256& b, const U256& q) {
  U256 r;
  for (int k = 0; k < 8; ++k) r.w[k] = 0;
  for (int bit = 255; bit >= 0; --bit) {
    r = addmod256(r, r, q);
    const U256 t = addmod256(r, b, q);
    r = sel256(0u - ((a.w[bit >> 5] >> (bit & 31)) & 1u), t, r);
  }
  return r;
}

// Encryption scalars, one thread per selection (nonces n = (R, u, c_fake, v_fake)):
//   s_fake = v_fake + R*c_fake, s_gneg = m ? c_fake : -c_fake, mscal = m   (mod q)
// (known-nonce simulation of the fake branch: a_f = g^s_fake, b_f = K^s_fake g^(+-c_fake)).
// plus (eg_ctx_set_proof_format EG_RESPONSE_PLUS: a = g^v X^-c): s_fake = v_fake - R*c_fake and
// s_gneg = m ? -c_fake : c_fake.  The response convention is public; the vote stays masked.
__global__ void k_enc_prep(const uint8_t* __restrict__ q_be, const uint8_t* __restrict__ votes,
                           const uint8_t* __restrict__ nonces, uint32_t n, uint8_t* __restrict__ derived,
                           uint32_t plus) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const U256 q = ld256(q_be);
  const U256 R = ld256(nonces + ((size_t)i * 4 + 0) * 32);
  const U256 cf = ld256(nonces + ((size_t)i * 4 + 2) * 32);
  const U256 vf = ld256(nonces + ((size_t)i * 4 + 3) * 32);
  const uint32_t m = votes[i] ? 1u : 0u;
  const U256 Rc = mulmod256(R, cf, q);
  const U256 sf = plus ? submod256(vf, Rc, q) : addmod256(vf, Rc, q);
  // (m xor plus) ? c_fake : -c_fake, branch-free in the (secret) vote
  const U256 sg = sel256((0u - m) ^ (0u - (plus & 1u)), cf, negmod(cf, q));
  U256 ms;
  for (int k = 0; k < 8; ++k) ms.w[k] = 0;
  ms.w[0] = m;
  st256(derived + ((size_t)i * 3 + 0) * 32, ms);
  st256(derived + ((size_t)i * 3 + 1) * 32, sf);
  st256(derived + ((size_t)i * 3 + 2) * 32, sg);
}

// R_sum per contest (one thread per contest): sum of the spc selection nonces R
__global__ void k_enc_rsum(const uint8_t* __restrict__ q_be, const uint8_t* __restrict__ nonces, uint32_t ncon,
                           uint32_t spc, uint8_t* __restrict__ rsum) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ncon) return;
  const U256 q = ld256(q_be);
  U256 r;
  for (int k = 0; k < 8; ++k) r.w[k] = 0;
  for (uint32_t s = 0; s < spc; ++s) r = addmod256(r, ld256(nonces + (((size_t)j * spc + s) * 4) * 32), q);
  st256(rsum + (size_t)j * 32, r);
}

// Finish the range proofs: c_real = c - c_fake, v_real = u - c_real*R (plus: u + c_real*R); arrange by m.
__global__ void k_enc_finish(const uint8_t* __restrict__ q_be, const uint8_t* __restrict__ votes,
                             const uint8_t* __restrict__ nonces, const uint8_t* __restrict__ chal, uint32_t n,
                             uint8_t* __restrict__ rproof, uint32_t plus) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const U256 q = ld256(q_be);
  const U256 R = ld256(nonces + ((size_t)i * 4 + 0) * 32);
  const U256 u = ld256(nonces + ((size_t)i * 4 + 1) * 32);
  const U256 cf = ld256(nonces + ((size_t)i * 4 + 2) * 32);
  const U256 vf = ld256(nonces + ((size_t)i * 4 + 3) * 32);
  const U256 c = ld256(chal + (size_t)i * 32);
  const U256 cr = submod256(c, cf, q);
  const U256 cR = mulmod256(cr, R, q);
  const U256 vr = plus ? addmod256(u, cR, q) : submod256(u, cR, q);
  uint8_t* o = rproof + (size_t)i * 4 * 32;
  const uint32_t mk = 0u - (uint32_t)(votes[i] != 0);  // the branch order follows the vote: masked
  st256(o + 0, sel256(mk, cf, cr));
  st256(o + 32, sel256(mk, vf, vr));
  st256(o + 64, sel256(mk, cr, cf));
  st256(o + 96, sel256(mk, vr, vf));
}

// Encryption commitments are computed vote-independently, real branch (a, b) in slots 0-1 and
// the simulated branch in slots 2-3 of each selection's 4 commitment elements; this puts them in
// proof order (branch 0 first), i.e. swaps the pairs where the vote is 1, with masks (the vote
// is secret).  One thread per 4-word column of a selection's pair.
__global__ void k_enc_order(uint32_t* __restrict__ comm, const uint8_t* __restrict__ votes, uint32_t n) {
  constexpr uint32_t kQuads = 2 * kW / 4;  // a pair of elements, in uint4
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n * kQuads) return;
  const uint32_t i = (uint32_t)(t / kQuads), k = (uint32_t)(t % kQuads);
  const uint32_t mk = 0u - (uint32_t)(votes[i] != 0);
  uint4* lo = reinterpret_cast<uint4*>(comm + (size_t)i * 4 * kW) + k;
  uint4* hi = lo + kQuads;
  const uint4 a = *lo, b = *hi;
  *lo = make_uint4((a.x & ~mk) | (b.x & mk), (a.y & ~mk) | (b.y & mk), (a.z & ~mk) | (b.z & mk),
                   (a.w & ~mk) | (b.w & mk));
  *hi = make_uint4((b.x & ~mk) | (a.x & mk), (b.y & ~mk) | (a.y & mk), (b.z & ~mk) | (a.z & mk),
                   (b.w & ~mk) | (a.w & mk));
}

// Generic response v = u - c*x mod q (plus: u + c*x; x per item or shared when x_stride == 0);
// writes proof (c, v) as 2 x 32 B.
__global__ void k_response(const uint8_t* __restrict__ q_be, const uint8_t* __restrict__ u_be,
                           const uint8_t* __restrict__ chal, const uint8_t* __restrict__ x_be, uint32_t x_stride,
                           uint32_t n, uint8_t* __restrict__ proof, uint32_t plus) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const U256 q = ld256(q_be);
  const U256 u = ld256(u_be + (size_t)i * 32);
  const U256 c = ld256(chal + (size_t)i * 32);
  const U256 x = ld256(x_be + (size_t)i * x_stride);
  const U256 cx = mulmod256(c, x, q);
  const U256 v = plus ? addmod256(u, cx, q) : submod256(u, cx, q);
  st256(proof + (size_t)i * 64, c);
  st256(proof + (size_t)i * 64 + 32, v);
}

// scalar derivation for the verifier (one thread per selection / contest)
//   sel: out[i] = (q - c1_i) mod q  ; ok[i] = all of c0,v0,c1,v1 < q
//   con: out[i] = (q - L*c_i mod q) ; ok[i] = c,v < q
// plus (EG_RESPONSE_PLUS, a = g^v X^-c): out[i] = L*c_i mod q, and the proof words in neg_mask
// (the challenges the variable bases are raised to) are negated in place, so the same job tables
// compute X^-c; the Fiat-Shamir check then reads the caller's unmodified proofs.
__global__ void k_scalar_prep(const uint8_t* __restrict__ q_be, uint8_t* __restrict__ proofs,
                              uint32_t n, uint32_t words_per, uint32_t neg_idx, uint32_t L,
                              uint8_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t plus,
                              uint32_t neg_mask) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const U256 q = ld256(q_be);
  bool good = true;
  for (uint32_t k = 0; k < words_per; ++k) good &= lt256(ld256(proofs + ((size_t)i * words_per + k) * 32), q);
  U256 c = ld256(proofs + ((size_t)i * words_per + neg_idx) * 32);
  if (good) {
    if (L != 1) c = mulsmall_mod(c, L, q);
    if (!plus) c = negmod(c, q);
    if (plus)
      for (uint32_t k = 0; k < words_per; ++k)
        if ((neg_mask >> k) & 1u) {
          uint8_t* w = proofs + ((size_t)i * words_per + k) * 32;
          st256(w, negmod(ld256(w), q));
        }
  } else {
    for (int k = 0; k < 8; ++k) c.w[k] = 0;
  }
  st256(out + (size_t)i * 32, c);
  ok[i] = good ? 1 : 0;
}

// ---------------------------------------------------------------------------------
// Fiat-Shamir hash + compare (one thread per proof).
//   H = SHA256("|" + hex(e_0) + "|" + ... + "|") mod q, hex upper-case, fixed width or
//   minimal-length per hash_minimal (eg_ctx_set_hash_format).
//   selection: elements (qbar, alpha, beta, a0, b0, a1, b1), expect (c0 + c1) mod q
//   contest  : elements (qbar, A, B, a, b),                   expect c
// (the elements after qbar in the ctx's pre-image order, eg_ctx_set_proof_format; up to 8 sources;
// a source of stride 0 is one element shared by every proof, e.g. the election key K)
// ---------------------------------------------------------------------------------
struct HashSrc {
  const uint8_t* ptr;  // base pointer
  uint32_t bytes;      // element width (32 or 512)
  uint32_t stride;     // bytes between consecutive proofs' elements
};

__global__ void __launch_bounds__(kBlock) k_hash_check(const uint8_t* __restrict__ q_be,
                                                       const uint8_t* __restrict__ qbar_be, uint32_t n,
                                                       uint32_t nsrc, HashSrc s0, HashSrc s1, HashSrc s2,
                                                       HashSrc s3, HashSrc s4, HashSrc s5, HashSrc s6, HashSrc s7,
                                                       const uint8_t* __restrict__ proofs,
                                                       uint32_t proof_words, uint32_t cidx0, uint32_t cidx1,
                                                       const uint8_t* __restrict__ pre_ok,
                                                       const uint8_t* __restrict__ pre_ok2, uint32_t pre2_div,
                                                       uint8_t* __restrict__ ok, uint8_t* __restrict__ out_h,
                                                       uint32_t hash_minimal) {
  // one 64-B block buffer per thread, at a 68-B stride: with a 64-B stride every lane's
  // byte k sits in the same LDS bank and each buffer access is a 32-way conflict
  constexpr int kBufStride = 17;
  __shared__ uint32_t s_buf[kBlock * kBufStride];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Sha256 H;
  H.init(s_buf + threadIdx.x * kBufStride);
  H.put('|');
  H.put_hex(qbar_be, 32, hash_minimal != 0);
  H.put('|');
  const HashSrc src[8] = {s0, s1, s2, s3, s4, s5, s6, s7};
  for (uint32_t k = 0; k < nsrc; ++k) {
    H.put_hex(src[k].ptr + (size_t)i * src[k].stride, src[k].bytes, hash_minimal != 0);
    H.put('|');
  }
  uint32_t dig[8];
  H.finish(dig);
  const U256 q = ld256(q_be);
  U256 h;
  for (int k = 0; k < 8; ++k) h.w[k] = dig[7 - k];
  if (!lt256(h, q)) sub256(h, q);
  if (out_h) st256(out_h + (size_t)i * 32, h);
  if (!ok) return;
  U256 c = ld256(proofs + ((size_t)i * proof_words + cidx0) * 32);
  if (cidx1 != kNone) c = addmod256(c, ld256(proofs + ((size_t)i * proof_words + cidx1) * 32), q);
  bool good = true;
  for (int k = 0; k < 8; ++k) good &= (c.w[k] == h.w[k]);
  if (pre_ok) good &= pre_ok[i] != 0;
  if (pre_ok2) {
    // pre_ok2 indexed per element pair: both pad/data of selection i must be < p
    good &= pre_ok2[(size_t)i * pre2_div] != 0 && pre_ok2[(size_t)i * pre2_div + 1] != 0;
  }
  ok[i] = good ? 1 : 0;
}

}  // namespace eg
