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
// import -> k_pow (the 4-bit window op program `sched`, identity job records `jobs`) -> export.
// elems / outs: n device elements each; scratch: pow16_scratch_bytes(n).
int pow16_powp(const Pow16Consts* C, bool friendly, hipStream_t s, const uint32_t* sched, const uint32_t* jobs,
               const uint8_t* base_be, const uint8_t* exp_be, uint8_t* out_be, size_t n, uint32_t* elems,
               uint32_t* outs, uint32_t* scratch, std::string* err);

// One element per WAVE (eg_pow16.hip, namespace egw): 48 lanes x 3 limbs of 2^29 (the same 144
// limbs and Montgomery radix), lanes 48-63 holding zeros, the quotient digit broadcast with
// v_readlane and the limb shift a wave_shl:1 DPP move, 5-bit sliding-window exponent.  A batch of
// up to one element per SIMD runs every element on its own SIMD: the shortest latency a blocking
// per-element caller can get (the coalescer's smallest batches).
struct PowWaveConsts;
int powwave_consts_create(const uint32_t* p, const uint32_t* r2, const uint32_t* one, uint32_t n0, uint32_t friendly,
                          PowWaveConsts** out, std::string* err);
void powwave_consts_destroy(PowWaveConsts* c);
// out_be[i] = base_be[i]^exp_be[i] mod p (device pointers, asynchronous on s; no scratch)
int powwave_powp(const PowWaveConsts* C, bool friendly, hipStream_t s, const uint8_t* base_be, const uint8_t* exp_be,
                 uint8_t* out_be, size_t n, std::string* err);
// out_be[i] = base^exp_be[i] mod p over a fixed-base radix table (eg_fixed_base_create: (nwin << wbits)
// 8-lane device elements in the Montgomery domain), one element per wave (device pointers, async on s)
int powwave_fbpow(const PowWaveConsts* C, bool friendly, hipStream_t s, const uint32_t* tab, uint32_t wbits,
                  uint32_t nwin, const uint8_t* exp_be, uint8_t* out_be, size_t n, std::string* err);
