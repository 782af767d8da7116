// eg_pow16.h — host interface of eg_pow16.hip, the latency-shaped instantiation of the device core
// (16 lanes per element: one DPP row, 9 limbs of 2^29 per lane) that runs the per-element
// coalescer's small variable-base batches (ElementModP.powP called element by element from 11
// threads, RunRemoteWorkflowTest.java:140,180, on the group of KUtils.java:10-12).  It lives in its
// own translation unit (namespace eg16) because the element format is a compile-time layout; the
// handles below are opaque to eg_capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

struct Pow16Consts;  // the modulus constants in the 16-lane element layout (device memory)

// p, r2 = R^2 mod p, one = R mod p as little-endian 32-bit words (128, 129, 129 of them; R = 2^4176,
// the same Montgomery radix as the 8-lane layout); n0 = -p^-1 mod 2^29; friendly = (n0 == 1)
int pow16_consts_create(const uint32_t* p, const uint32_t* r2, const uint32_t* one, uint32_t n0, uint32_t friendly,
                        Pow16Consts** out, std::string* err);
void pow16_consts_destroy(Pow16Consts* c);
size_t pow16_elem_bytes();                 // one device element (192 words)
size_t pow16_scratch_bytes(size_t n);      // the 16-entry window tables of a batch of n
// elements one resident round of the 16-lane k_pow holds on `device` (0 when unknown)
size_t pow16_round_jobs(int device);
// out_be[i] = base_be[i]^exp_be[i] mod p for n elements, device pointers, asynchronous on `s`:
// import -> k_pow (the 4-bit window op program `sched`, identity job records `jobs`) -> export;
// ct: k_pow's constant-time instantiation (every window-table read a masked scan of its 16 entries).
// elems / outs: n device elements each; scratch: pow16_scratch_bytes(n).
int pow16_powp(const Pow16Consts* C, bool friendly, bool ct, hipStream_t s, const uint32_t* sched, const uint32_t* jobs,
               const uint8_t* base_be, const uint8_t* exp_be, uint8_t* out_be, size_t n, uint32_t* elems,
               uint32_t* outs, uint32_t* scratch, std::string* err);

// One job per WAVE or per workgroup of 4 waves (eg_pow16.hip, namespace egw): 48 lanes x 3 limbs of 2^29 (the same 144 limbs and
// Montgomery radix), lanes 48-63 holding zeros, the quotient digit broadcast with v_readlane and the
// limb shift a wave_shl:1 DPP move.  A batch of up to one job per SIMD runs every job on its own
// SIMD: the shortest latency a blocking per-element caller can get (the coalescer's batches).
struct PowWaveConsts;
int powwave_consts_create(const uint32_t* p, const uint32_t* r2, const uint32_t* one, uint32_t n0, uint32_t friendly,
                          PowWaveConsts** out, std::string* err);
void powwave_consts_destroy(PowWaveConsts* c);

// A fixed-base radix table as the per-wave kernel reads it (eg_fixed_base_create: (nwin << wbits)
// 8-lane device elements in the Montgomery domain).
struct WaveTab {
  const uint32_t* data;
  uint32_t wbits, nwin;
};
constexpr uint32_t kWaveNone = 0xFFFFFFFFu;  // an absent row / table
constexpr uint32_t kWaveMaxBases = 16;       // bases one job multiplies together
// One per-wave job: out row `out` = (prod of base rows [base, base + nbase))^(exp row `exp`)
//   * tabs[tab[0]]^(exp row fexp[0]) * tabs[tab[1]]^(exp row fexp[1])  mod p.
// Base rows are 512-byte big-endian elements (any value: reduced mod p), exp rows 32-byte big-endian
// exponents; exp = kWaveNone: the product itself (exponent 1); tab[t] = kWaveNone: no fixed-base term;
// nbase = 0 with an exponent: 1.  x^0 = 1 (also 0^0).
struct WaveJob {
  uint32_t base, nbase, exp, tab[2], fexp[2], out;
};
// Run njobs jobs (device pointers, asynchronous on s).  d_jobs == nullptr: job e is `dflt` with its base,
// exp, fexp[0] and out rows set to e and its fixed-base term (if any) over t_ident -- element e of every
// input array.  ct: the constant-time instantiation (fixed 4-bit windows with masked LDS scans for the
// variable-base term, masked scans of every window column and no zero-digit skip for fixed-base terms,
// whose tables must then have wbits <= 8).
// waves > 1: four waves per job, the fixed-base windows split over them (eg_pow16.hip k_wave_job); with
// r2l the variable part runs right to left over the four waves too (the latency shape for batches of at
// most one job per CU; with ct its constant-time schedule).  waves >= 8 without r2l on the
// Montgomery-friendly p: eight waves per job (the fixed-base windows over seven or eight of them).
int powwave_jobs(const PowWaveConsts* C, bool friendly, bool ct, int waves, bool r2l, hipStream_t s,
                 const WaveJob* d_jobs, WaveJob dflt, uint32_t njobs, const WaveTab* d_tabs, WaveTab t_ident,
                 const uint8_t* d_bases, const uint8_t* d_exps, uint8_t* d_out, std::string* err);
// out_be[i] = base_be[i]^exp_be[i] mod p (device pointers, asynchronous on s; no scratch); r2l: four
// waves per element, right to left
int powwave_powp(const PowWaveConsts* C, bool friendly, bool ct, bool r2l, hipStream_t s, const uint8_t* base_be,
                 const uint8_t* exp_be, uint8_t* out_be, size_t n, std::string* err);
// out_be[i] = base^exp_be[i] mod p over a fixed-base radix table, one element per wave
int powwave_fbpow(const PowWaveConsts* C, bool friendly, bool ct, hipStream_t s, const WaveTab& t,
                  const uint8_t* exp_be, uint8_t* out_be, size_t n, std::string* err);
