// Separated product-then-REDC against the interleaved CIOS multiply of k_pow.
//
// A one-level Karatsuba multiply can only exist in the SEPARATED form: the full 288-limb product
// T = x * y first (where Karatsuba replaces the 144 x 144 schoolbook by three 72 x 72 products),
// then Montgomery's REDC(T) = (T_low + m p) / R + T_high, with m taken from T_low alone.  The CIOS
// multiply of eg_bignum.hpp interleaves the two halves digit by digit in ONE rotating accumulator,
// so the product half costs no glue of its own.  This benchmark measures what the separation alone
// costs on the same 8-lane layout -- the price Karatsuba's MAC saving would first have to repay:
//
//   mode 0  CIOS multiply            x <- x * y * R^-1    (eg_bignum.hpp mont_mul_impl, as k_pow)
//   mode 1  CIOS squaring            x <- x^2 * R^-1      (the symmetric-half schedule)
//   mode 2  separated multiply       product phase: 144 steps of 18 MACs into the rotating window, the
//                                    finished low column of each step leaves through LDS (T_low); REDC
//                                    phase: T_low back into the window, 144 steps of m * p; + T_high
//   mode 3  separated squaring       the same with the symmetric-half product
//
// Every mode runs `iters` dependent operations per element on the production group (EG 1.0 p) at
// k_pow's shape (256-thread workgroups, 3 waves per SIMD, p in LDS); the separated results are
// checked against CIOS's as integers (both are the exact (x y + m p) / R).  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -o _ub/ubench_karatsuba tools/ubench_karatsuba.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../electionguard-remote_amd/csrc/eg_kernels.hpp"
#include "../electionguard-remote_amd/host/eg_constants.hpp"

using namespace eg;

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "HIP %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int kTStride = kN + 4;  // LDS words per group for T_low (the group's lane 0 writes column i at step i)

// One product step of the separated multiply: t += x * y_i in the rotating window (no m * p), then
// the lowest column splits: its carry stays in this lane, its low 29 bits go to lane - 1's top
// position; the group's lane 0 emits them (column i of T is final after step i) into the group's T
// buffer (an exec-masked ds_write).  mask_in: the limb mask, 0 on lane 7 (whose DPP neighbour is the
// next group's lane 0, which here is not 0 mod 2^29 as it is in CIOS).
template <bool SQR>
__device__ __forceinline__ void prod_step(uint64_t (&acc)[kL], const uint32_t (&x)[kL], const int r, const uint32_t yi,
                                          uint32_t mask, uint32_t mask_in, uint32_t doff, uint32_t dwid,
                                          uint32_t* __restrict__ tl, bool emit) {
  if constexpr (SQR) {
    {
      const uint32_t d = __builtin_amdgcn_ubfe(x[r], doff, dwid);
      uint64_t& A = acc[(r + r) % kL];
      A = (uint64_t)d * yi + A;
    }
    constexpr int kHalf = (kL - 1) / 2;
    const int jmax = (kL % 2 == 1) ? kHalf : (r < kL / 2 ? kL / 2 : kL / 2 - 1);
#pragma unroll
    for (int jj = 1; jj <= jmax; ++jj) {
      const int j = (r + jj) % kL;
      uint64_t& A = acc[(j + r) % kL];
      A = (uint64_t)x[j] * yi + A;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      uint64_t& A = acc[(j + r) % kL];
      A = (uint64_t)x[j] * yi + A;
    }
  }
  uint64_t& A0 = acc[r % kL];
  acc[(r + 1) % kL] += A0 >> kLimbBits;
  if (emit) tl[r] = (uint32_t)A0 & mask;
  A0 = (uint64_t)from_next_and((uint32_t)A0, mask_in);
}

// x <- x * y * R^-1 (SQR: x^2 R^-1, the slot holding x), separated: product, then REDC.  Exact same
// integer as mont_mul_impl (m depends on T mod R only).
template <bool SQR>
__device__ __forceinline__ void sep_mul(const Mont<true>& M, uint32_t (&x)[kL], const uint32_t* __restrict__ y,
                                        uint32_t* __restrict__ tbuf) {
  const int gl = glane();
  const uint32_t mask = M.mask;
  const uint32_t mask_in = gl == kT - 1 ? 0u : mask;
  const bool emit = gl == 0;
  uint64_t acc[kL];
#pragma unroll
  for (int j = 0; j < kL; ++j) acc[j] = 0;
  if constexpr (SQR) {
#pragma unroll
    for (int j = 0; j < kL; ++j) x[j] <<= 1;
  }
  uint32_t doff = SQR && gl == 0 ? 1u : 0u, dwid = SQR ? 31u : 0u;
#pragma unroll 1
  for (int s = 0; s < kT; ++s) {
    if constexpr (SQR) {
      doff = (gl == s) ? 1u : 0u;
      dwid = (gl >= s) ? 31u : 0u;
    }
    const uint32_t* ys = y + s * kLP;
    uint32_t* ts = tbuf + s * kL;
#pragma unroll
    for (int r = 0; r < kL; ++r) prod_step<SQR>(acc, x, r, ys[r], mask, mask_in, doff, dwid, ts, emit);
  }
  // the window now holds T_high: lane l register k = column 144 + 18 l + k (64-bit, unnormalised)
  uint64_t th[kL];
#pragma unroll
  for (int j = 0; j < kL; ++j) th[j] = acc[j];
  __builtin_amdgcn_wave_barrier();
  // REDC over T_low (this lane's 18 limbs, written by lane 0 as the columns finished)
  const uint32_t* tlo = tbuf + gl * kL;
#pragma unroll
  for (int j = 0; j < kL; ++j) acc[j] = tlo[j];
#pragma unroll 1
  for (int s = 0; s < kT; ++s) {
#pragma unroll
    for (int r = 0; r < kL; ++r) {
      const uint32_t m = bcast_g0_and((uint32_t)acc[r % kL], mask);  // friendly p: n0 = 1
#pragma unroll
      for (int j = 0; j < kL; ++j) {
        uint64_t& A = acc[(j + r) % kL];
        A = (uint64_t)M.p[j] * m + A;
      }
      uint64_t& A0 = acc[r % kL];
      acc[(r + 1) % kL] += A0 >> kLimbBits;
      A0 = (uint64_t)from_next_and((uint32_t)A0, mask);
    }
  }
#pragma unroll
  for (int j = 0; j < kL; ++j) acc[j] += th[j];
  // the CIOS epilogue: two parallel carry passes
  uint64_t d[kL];
  {
    uint64_t c_in = ((uint64_t)from_prev((uint32_t)(acc[kL - 1] >> kLimbBits)) |
                     ((uint64_t)from_prev((uint32_t)(acc[kL - 1] >> (kLimbBits + 32))) << 32));
#pragma unroll
    for (int j = 0; j < kL; ++j) {
      const uint64_t c = (j == 0) ? c_in : (acc[j - 1] >> kLimbBits);
      d[j] = (uint64_t)((uint32_t)acc[j] & mask) + c;
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
  __builtin_amdgcn_wave_barrier();
}

template <int MODE>
__global__ void __launch_bounds__(kBlock, 3) k_bench(const MontConsts* __restrict__ C, const uint32_t* __restrict__ xin,
                                                     const uint32_t* __restrict__ yin, uint32_t* __restrict__ xout,
                                                     int iters) {
  Mont<true> M;
  M.load(C);
  __shared__ uint32_t s_t[kGroupsPerBlock * kTStride];
  uint32_t* slot = group_slot();
  uint32_t* tbuf = s_t + (threadIdx.x / kT) * kTStride;
  const uint32_t gid = group_id();
  uint32_t x[kL];
  load_elem(x, xin + (size_t)gid * kW);
  if (MODE == 0 || MODE == 2) {
    elem_to_lds(slot, yin + (size_t)gid * kW);
    wave_sync();
  }
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
      M.mul(x, slot);
    } else if constexpr (MODE == 1) {
      msqr(M, x, slot);
    } else if constexpr (MODE == 2) {
      sep_mul<false>(M, x, slot, tbuf);
    } else {
      regs_to_lds(slot, x);
      wave_sync();
      sep_mul<true>(M, x, slot, tbuf);
    }
  }
  store_elem(xout + (size_t)gid * kW, x);
}

// ---- host: the production p in the device element format, Montgomery constants, checks ----
static std::vector<uint32_t> hex_words_le(const char* hex) {  // 4096-bit big-endian hex -> 128 LE words
  std::string h(hex);
  std::vector<uint32_t> w(128, 0);
  for (size_t i = 0; i < h.size(); ++i) {
    const char c = h[h.size() - 1 - i];
    const uint32_t v = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
    w[i / 8] |= v << (4 * (i % 8));
  }
  return w;
}

static uint32_t bits_at(const std::vector<uint32_t>& w, int b) {
  const int wi = b >> 5, sh = b & 31;
  const uint64_t lo = wi < (int)w.size() ? w[wi] : 0, hi = wi + 1 < (int)w.size() ? w[wi + 1] : 0;
  return (uint32_t)(((hi << 32) | lo) >> sh) & kMask;
}

static void to_device_format(const std::vector<uint32_t>& w, uint32_t* out) {  // kW words
  std::memset(out, 0, kW * 4);
  for (int k = 0; k < kN; ++k) out[(k / kL) * kLP + k % kL] = bits_at(w, k * kLimbBits);
}

// integer value of a device element (lazy limbs may exceed 29 bits) as 132 LE words
static std::vector<uint32_t> value_of(const uint32_t* e) {
  std::vector<uint64_t> acc(140, 0);
  for (int k = 0; k < kN; ++k) {
    const uint64_t v = e[(k / kL) * kLP + k % kL];
    const int b = k * kLimbBits;
    acc[b >> 5] += (v << (b & 31)) & 0xFFFFFFFFull;
    acc[(b >> 5) + 1] += (v << (b & 31)) >> 32;
  }
  std::vector<uint32_t> out(140);
  uint64_t c = 0;
  for (int i = 0; i < 140; ++i) {
    c += acc[i];
    out[i] = (uint32_t)c;
    c >>= 32;
  }
  return out;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 128;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 3 * 2;  // 3 waves per SIMD (one 4-wave block per SIMD quadruple), two rounds
  const size_t groups = (size_t)blocks * kGroupsPerBlock;
  MontConsts hc{};
  const auto pw = hex_words_le(electionguard::constants::kP_HEX);
  to_device_format(pw, hc.p);
  for (int i = 0; i < 128; ++i) hc.pw[i] = pw[i];
  hc.n0 = 1;
  hc.friendly = 1;
  hc.mask = kMask;
  // inputs: < p (top limb cleared), deterministic
  std::vector<uint32_t> hx(groups * kW), hy(groups * kW);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto rnd = [&] {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return (uint32_t)s;
  };
  for (size_t g = 0; g < groups; ++g) {
    std::vector<uint32_t> a(128), b(128);
    for (int i = 0; i < 127; ++i) a[i] = rnd(), b[i] = rnd();
    to_device_format(a, &hx[g * kW]);
    to_device_format(b, &hy[g * kW]);
  }
  MontConsts* dC;
  uint32_t *dx, *dy, *dout[4];
  CHK(hipMalloc(&dC, sizeof(MontConsts)));
  CHK(hipMemcpy(dC, &hc, sizeof(MontConsts), hipMemcpyHostToDevice));
  CHK(hipMalloc(&dx, groups * kW * 4));
  CHK(hipMalloc(&dy, groups * kW * 4));
  for (auto& o : dout) CHK(hipMalloc(&o, groups * kW * 4));
  CHK(hipMemcpy(dx, hx.data(), groups * kW * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dy, hy.data(), groups * kW * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  // every mode at k_pow's occupancy, 3 workgroups (3 waves per SIMD) per CU: dynamic LDS pads each
  // workgroup to 44 KB, so a 4th never fits (160 KB per CU) even where the registers would allow it
  size_t lds_static[4];
  {
    hipFuncAttributes fa;
    const void* fns[4] = {(const void*)k_bench<0>, (const void*)k_bench<1>, (const void*)k_bench<2>, (const void*)k_bench<3>};
    for (int m = 0; m < 4; ++m) {
      CHK(hipFuncGetAttributes(&fa, fns[m]));
      lds_static[m] = fa.sharedSizeBytes;
    }
  }
  auto pad = [&](int m) -> size_t { return 44 * 1024 > lds_static[m] ? 44 * 1024 - lds_static[m] : 0; };
  auto launch = [&](int mode) -> float {
    CHK(hipEventRecord(e0));
    switch (mode) {
      case 0: hipLaunchKernelGGL(k_bench<0>, dim3(blocks), dim3(kBlock), pad(0), 0, dC, dx, dy, dout[0], iters); break;
      case 1: hipLaunchKernelGGL(k_bench<1>, dim3(blocks), dim3(kBlock), pad(1), 0, dC, dx, dy, dout[1], iters); break;
      case 2: hipLaunchKernelGGL(k_bench<2>, dim3(blocks), dim3(kBlock), pad(2), 0, dC, dx, dy, dout[2], iters); break;
      default: hipLaunchKernelGGL(k_bench<3>, dim3(blocks), dim3(kBlock), pad(3), 0, dC, dx, dy, dout[3], iters); break;
    }
    CHK(hipGetLastError());
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  for (int m = 0; m < 4; ++m) launch(m);  // warm-up (code objects, clocks)
  std::vector<std::vector<float>> ms(4);
  for (int r = 0; r < rounds; ++r)
    for (int m = 0; m < 4; ++m) ms[m].push_back(launch(m));  // interleaved
  CHK(hipDeviceSynchronize());
  // checks: separated == CIOS as integers, per element
  long mism[2] = {0, 0};
  std::vector<uint32_t> o[4];
  for (int m = 0; m < 4; ++m) {
    o[m].resize(groups * kW);
    CHK(hipMemcpy(o[m].data(), dout[m], groups * kW * 4, hipMemcpyDeviceToHost));
  }
  for (size_t g = 0; g < groups; ++g) {
    mism[0] += value_of(&o[0][g * kW]) != value_of(&o[2][g * kW]);
    mism[1] += value_of(&o[1][g * kW]) != value_of(&o[3][g * kW]);
  }
  const char* names[4] = {"cios_mul", "cios_sqr", "separated_mul", "separated_sqr"};
  printf("{\"groups\": %zu, \"iters\": %d, \"rounds\": %d, \"cus\": %d", groups, iters, rounds, cus);
  double best[4];
  for (int m = 0; m < 4; ++m) {
    best[m] = 1e30;
    for (float v : ms[m]) best[m] = v < best[m] ? v : best[m];
    printf(", \"%s\": {\"best_ms\": %.4f, \"mm_per_s\": %.4g, \"ms\": [", names[m], best[m],
           groups * (double)iters / (best[m] / 1e3));
    for (size_t i = 0; i < ms[m].size(); ++i) printf("%s%.4f", i ? ", " : "", ms[m][i]);
    printf("]}");
  }
  printf(", \"separated_over_cios_time\": {\"mul\": %.4f, \"sqr\": %.4f}", best[2] / best[0], best[3] / best[1]);
  printf(", \"mismatched_elements\": {\"mul\": %ld, \"sqr\": %ld}}\n", mism[0], mism[1]);
  return (mism[0] || mism[1]) ? 1 : 0;
}
