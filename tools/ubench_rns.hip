// Cost model microbenchmark for an RNS Montgomery multiply on MFMA ("the next
// large lever"): the shape planned there, measured before any of the path is rebuilt.
//   * 16 jobs per wave, 4 lanes per job, two waves per SIMD (512-thread workgroups, one per CU):
//     the state of a wave's jobs is emulated by kLive live VGPRs per lane (x in both bases,
//     packed 16-bit channels) that every tile touches, so the compiler keeps them resident;
//   * each base extension is 18 output tiles of 16 channel rows; a tile is 20
//     v_mfma_i32_16x16x64_i8: four byte products (cl.ql, cl.qh, ch.ql, ch.qh) over 5 K-blocks of
//     64 channel digits, three shift classes; the job digits (B operands) sit in registers, the
//     constant fragments (A operands, 2 x 5 KB per tile) come from a double-buffered LDS ring
//     that the CU's 8 waves fill together from L2 while they compute (one barrier per stage
//     of RNS_SUB tiles);
//   * every tile also runs the channel VALU work the design counts per job-MM (~20k lane-ops:
//     f32 magic-number Barrett reductions, shift-class recombination, byte packing), spread
//     evenly: kValuPerTile real modular operations on live data per lane.
// The figure of merit is SIMD-cycles per job-MM, against 2,700 for today's CIOS k_pow
// (21.6k SIMD-cycles per wave-MM, 8 jobs per wave).  Timing only: the arithmetic is real but
// the data are synthetic (the exact RNS algorithm is not implemented here).
//   hipcc --offload-arch=gfx950 -O3 [-DRNS_SUB=3] [-DRNS_VALU=0 | -DRNS_MFMA=0] -o tools/_ubench_rns tools/ubench_rns.hip
// Results: profiles/r03u_ubench_rns*.txt (1.62 ns per job-MM against 1.18 for the CIOS k_pow).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

#ifndef RNS_LIVE
#define RNS_LIVE 120  // emulated per-lane state (x in B and B', 16-bit packed: ~144 in the design)
#endif
#ifndef RNS_VALU
#define RNS_VALU 12  // elementwise channel products per lane per tile (x 6 ops each): ~10.7k lane-ops per job-MM
#endif
constexpr int kSlices = 10;  // live-state slices the tiles rotate through (RNS_VALU x 10 >= RNS_LIVE)
#ifndef RNS_MFMA
#define RNS_MFMA 1
#endif
#ifndef RNS_SUB
#define RNS_SUB 1  // output tiles per LDS stage (one barrier per stage)
#endif
constexpr int kLive = RNS_LIVE;
constexpr int kKB = 5;          // K-blocks of 64 digits per digit plane (288 channels padded to 320)
constexpr int kTileBytes = 2 * kKB * 16 * 64;  // cl and ch fragments of one 16-row output tile
constexpr int kStageBytes = RNS_SUB * kTileBytes;
constexpr int kTiles = 36;      // 18 output tiles per extension, two extensions per MM

// one channel product reduced mod m: f32 magic-number Barrett (p < 2^24 exact in f32)
__device__ __forceinline__ int modmul(int a, int b, int m, float inv) {
  const int pr = __mul24(a, b);                // a*b, |a|,|b| < 2^12 here
  const float q = __builtin_fmaf((float)pr, inv, 12582912.0f);  // round(pr / m) + 1.5 * 2^23
  const int qi = __builtin_bit_cast(int, q) - 0x4B400000;
  return pr - __mul24(qi, m);
}

__global__ void __launch_bounds__(512, 1) k_rns(const uint8_t* __restrict__ consts, const int* __restrict__ digits,
                                                 int* __restrict__ out, int mms, uint32_t seed) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[2][kStageBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  // job digits: 2 planes x kKB K-blocks, 16 bytes per lane each
  v4i ql[kKB], qh[kKB];
  const int* dj = digits + ((size_t)blockIdx.x * 512 + tid) * 8 * kKB;
#pragma unroll
  for (int k = 0; k < kKB; ++k) {
    ql[k] = v4i{dj[8 * k], dj[8 * k + 1], dj[8 * k + 2], dj[8 * k + 3]};
    qh[k] = v4i{dj[8 * k + 4], dj[8 * k + 5], dj[8 * k + 6], dj[8 * k + 7]};
  }
  int live[kLive];
#pragma unroll
  for (int i = 0; i < kLive; ++i) live[i] = (int)(seed * (i + 1) + tid) & 0x7FF;
  const int m = 32003 - 2 * (lane & 15);
  const float inv = 1.0f / (float)m;
  // prologue: tile 0 into ring 0
  const uint4* csrc = reinterpret_cast<const uint4*>(consts);
  constexpr int kVec = kStageBytes / 16;  // uint4 per stage
  for (int i = tid; i < kVec; i += 512) reinterpret_cast<uint4*>(s_ring[0])[i] = csrc[i];
  __syncthreads();
  int acc_x = 0;
  for (int it = 0; it < mms * kTiles / RNS_SUB; ++it) {
    const int cur = it & 1, tile = it % (kTiles / RNS_SUB);
    // fill the other ring slot with the next stage's constants (the 36 tiles cycle through L2)
    const int nt = (tile + 1) % (kTiles / RNS_SUB);
    uint4 pre[(kVec + 511) / 512];
#pragma unroll
    for (int r = 0; r < (kVec + 511) / 512; ++r) {
      const int i = tid + r * 512;
      if (i < kVec) pre[r] = csrc[(size_t)nt * kVec + i];
    }
#pragma unroll
    for (int sub = 0; sub < RNS_SUB; ++sub) {
    v4i s0 = {0, 0, 0, 0}, s1 = {0, 0, 0, 0}, s2 = {0, 0, 0, 0};
#if RNS_MFMA
    const uint8_t* ring = s_ring[cur] + sub * kTileBytes;
#pragma unroll
    for (int k = 0; k < kKB; ++k) {
      const v4i cl = *reinterpret_cast<const v4i*>(ring + (k * 16 * 64) + lane * 16);
      const v4i ch = *reinterpret_cast<const v4i*>(ring + kTileBytes / 2 + (k * 16 * 64) + lane * 16);
      s0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(cl, ql[k], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(cl, qh[k], s1, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ch, ql[k], s1, 0, 0, 0);
      s2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ch, qh[k], s2, 0, 0, 0);
    }
#endif
    // channel work: the tile's 4 output channels per lane (recombination of the classes) and
    // this tile's share of the elementwise products, on live state
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int r2 = modmul(s2[c] & 0xFFF, 2731, m, inv);
      const int r1 = modmul(s1[c] & 0xFFF, 1999, m, inv);
      const int v = (s0[c] & 0xFFFFF) + (r1 << 8) + __mul24(r2, 677);
      acc_x ^= modmul(v & 0xFFF, 1021, m, inv);
    }
    }
    // elementwise share: RNS_VALU channel products on a compile-time slice of the live state,
    // the slice chosen by the tile (a wave-uniform switch, no dynamic register indexing)
    const int key = (acc_x & 0x7FF) | 1;
    switch ((it * RNS_SUB) % kSlices) {
#define RNS_SLICE(S)                                                      \
  case S:                                                                 \
    _Pragma("unroll") for (int j = 0; j < RNS_VALU * RNS_SUB; ++j) {                \
      int& v = live[(S * RNS_VALU * RNS_SUB + j) % kLive];                          \
      v = modmul(v, key, m, inv) & 0xFFF;                                 \
    }                                                                     \
    break;
      RNS_SLICE(0) RNS_SLICE(1) RNS_SLICE(2) RNS_SLICE(3) RNS_SLICE(4)
      RNS_SLICE(5) RNS_SLICE(6) RNS_SLICE(7) RNS_SLICE(8) RNS_SLICE(9)
#undef RNS_SLICE
    }
    // publish the next tile's constants, then swap
#pragma unroll
    for (int r = 0; r < (kVec + 511) / 512; ++r) {
      const int i = tid + r * 512;
      if (i < kVec) reinterpret_cast<uint4*>(s_ring[cur ^ 1])[i] = pre[r];
    }
    __syncthreads();
  }
  int sink = acc_x;
#pragma unroll
  for (int i = 0; i < kLive; ++i) sink += live[i];
  out[(size_t)blockIdx.x * 512 + tid] = sink;
}

int main(int argc, char** argv) {
  const int mms = argc > 1 ? atoi(argv[1]) : 40;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus;  // one 512-thread workgroup (8 waves, 2 per SIMD) per CU
  std::vector<uint8_t> consts((size_t)kTiles * kTileBytes);
  for (auto& v : consts) v = (uint8_t)(rand() & 0x7F);
  std::vector<int> dig((size_t)blocks * 512 * 8 * kKB);
  for (auto& v : dig) v = rand() & 0x3F3F3F3F;
  uint8_t* dc;
  int *dd, *dout;
  CHK(hipMalloc(&dc, consts.size()));
  CHK(hipMalloc(&dd, dig.size() * 4));
  CHK(hipMalloc(&dout, (size_t)blocks * 512 * 4));
  CHK(hipMemcpy(dc, consts.data(), consts.size(), hipMemcpyHostToDevice));
  CHK(hipMemcpy(dd, dig.data(), dig.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_rns, dim3(blocks), dim3(512), 0, 0, dc, dd, dout, 2, 1u);
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL(k_rns, dim3(blocks), dim3(512), 0, 0, dc, dd, dout, mms, 7u);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  hipFuncAttributes fa{};
  CHK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_rns)));
  const double jobs = (double)blocks * 8 * 16;  // 16 jobs per wave
  const double job_mm = jobs * mms;
  const double ns_per_job_mm = ms * 1e6 / job_mm;
  const double mfma = (double)blocks * 8 * mms * kTiles * 4 * kKB;
  const double clk = 2.2e9;  // for SIMD-cycles: the clock k_pow holds under load (2.1-2.3 GHz)
  const double simd_cyc = ms * 1e-3 * clk * cus * 4 / job_mm;
  printf("sub %d live %d valu/tile %d mfma %d | regs %d | %d CUs x 1 WG x 8 waves, %d MMs: %.3f ms, %.4f ns per job-MM, "
         "%.0f SIMD-cycles per job-MM at 2.2 GHz (CIOS k_pow: 2,700), i8 MFMA %.2f P MAC/s\n",
         RNS_SUB, kLive, RNS_VALU, RNS_MFMA, fa.numRegs, blocks, mms, ms, ns_per_job_mm, simd_cyc,
         mfma * 16384.0 / (ms * 1e-3) / 1e15);
  return 0;
}
