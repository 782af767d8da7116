// Feasibility microbenchmark for an i8-MFMA Barrett reduction: the two
// reduction products of a Barrett step, q = hi(T_hi * mu) and lo(q * p), are Toeplitz GEMMs
// over a block's 32 jobs with a SHARED constant operand (mu or p), in radix-2^7 digits so
// both operands are non-negative i8 (586 digits per 4097-bit value).
//   part 1: operand/result lane maps of v_mfma_i32_32x32x32_i8, checked with exact integers;
//   part 2: one Toeplitz GEMM (the high half of T_hi * mu, 19 column tiles of 32) per block of
//           32 jobs: A digits (per job) held in VGPRs, B fragments (Toeplitz of the constant)
//           read from 16 byte-shifted LDS copies, one ds_read_b128 per MFMA; checked against
//           the CPU, then timed.  The figure of merit is GPU time per job per GEMM against the
//           1.19 ns per job-MM of the current CIOS k_pow (841 M MM/s).
//   hipcc --offload-arch=gfx950 -O3 -o tools/_ubench_toeplitz tools/ubench_toeplitz.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// ---------------- part 1: lane maps ----------------
// map 0: lane l (r = l & 31, h = l >> 5) holds A[r][16h + j], B[16h + j][r], j = 0..15
// map 1: lane l holds A[r][8h + (j & 7) + 16 (j >> 3)], same for B
__device__ __host__ inline int kmap(int map, int h, int j) { return map == 0 ? 16 * h + j : 8 * h + (j & 7) + 16 * (j >> 3); }

__global__ void k_layout(const int8_t* A, const int8_t* B, int* D, int map) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[r * 32 + kmap(map, h, j)];
    b[j] = B[kmap(map, h, j) * 32 + r];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

// ---------------- part 2: Toeplitz GEMM ----------------
constexpr int kDig = 586;                 // radix-2^7 digits of a 4097-bit value
constexpr int kKB = (kDig + 31) / 32;     // 19 k-blocks
constexpr int kKPad = kKB * 32;           // 608
constexpr int kT0 = 18, kT1 = 37;         // column tiles of the high half: columns [576, 1184)
constexpr int kP = 680, kMurLen = 768;    // MUR[t] = mu[kP - t]

template <int MAP>
__global__ void __launch_bounds__(256) k_toeplitz(const uint8_t* __restrict__ digits, const uint8_t* __restrict__ mu,
                                                  int* __restrict__ out, int iters, int check) {
  __shared__ __attribute__((aligned(16))) uint8_t s_a[32][kKPad];
  __shared__ __attribute__((aligned(16))) uint8_t s_mur[16][kMurLen];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, r = l & 31, h = l >> 5;
  const uint8_t* src = digits + (size_t)blockIdx.x * 32 * kKPad;
  for (int i = tid; i < 32 * kKPad; i += 256) s_a[i / kKPad][i % kKPad] = src[i];
  for (int i = tid; i < 16 * kMurLen; i += 256) {
    const int s = i / kMurLen, u = i % kMurLen, t = u + s, mi = kP - t;
    s_mur[s][u] = (mi >= 0 && mi < kDig) ? mu[mi] : 0;
  }
  __syncthreads();
  // A fragments of all k-blocks in VGPRs (19 x 4)
  v4i af[kKB];
#pragma unroll
  for (int kb = 0; kb < kKB; ++kb) {
    if (MAP == 0) {
      af[kb] = *reinterpret_cast<const v4i*>(&s_a[r][kb * 32 + 16 * h]);
    } else {
      const uint2 lo = *reinterpret_cast<const uint2*>(&s_a[r][kb * 32 + 8 * h]);
      const uint2 hi = *reinterpret_cast<const uint2*>(&s_a[r][kb * 32 + 16 + 8 * h]);
      af[kb] = v4i{(int)lo.x, (int)lo.y, (int)hi.x, (int)hi.y};
    }
  }
  int sink = 0;
  constexpr int kPerWave = (kT1 - kT0 + 3) / 4;  // column tiles per wave (tile kT0 + wave + 4m)
  for (int it = 0; it < iters; ++it) {
    v16i acc[kPerWave];
#pragma unroll
    for (int m = 0; m < kPerWave; ++m) acc[m] = v16i{};
    // k-block outer (its A fragment is a static register), the wave's tiles inner; a tile takes
    // the k-blocks whose Toeplitz band meets it (0 <= c - k < kDig): a wave-uniform branch
#pragma unroll
    for (int kb = 0; kb < kKB; ++kb) {
#pragma unroll
      for (int m = 0; m < kPerWave; ++m) {
        const int ct = kT0 + wave + 4 * m;
        const int c0 = ct * 32, D = c0 - kb * 32;
        if (ct < kT1 && D + 31 >= 0 && D - 31 < kDig) {
          const int t0 = kP - D - r + (MAP == 0 ? 16 * h : 8 * h);
          v4i bf;
          if (MAP == 0) {
            const int s = t0 & 15;
            bf = *reinterpret_cast<const v4i*>(&s_mur[s][t0 - s]);
          } else {
            const int s0 = t0 & 7, s1 = (t0 + 16) & 7;
            const uint2 lo = *reinterpret_cast<const uint2*>(&s_mur[s0][t0 - s0]);
            const uint2 hi = *reinterpret_cast<const uint2*>(&s_mur[s1][t0 + 16 - s1]);
            bf = v4i{(int)lo.x, (int)lo.y, (int)hi.x, (int)hi.y};
          }
          acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[kb], bf, acc[m], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < kPerWave; ++m) {
      const int ct = kT0 + wave + 4 * m;
      if (ct >= kT1) continue;
      if (check && it == 0) {
        for (int i = 0; i < 16; ++i)
          out[((size_t)blockIdx.x * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * 1184 + ct * 32 + r] = acc[m][i];
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) sink += acc[m][i];
    }
  }
  if (sink == 0x7fffffff) out[0] = sink;
}

// Diagonal reuse: B[k][c] of a Toeplitz operand depends on c - k only, so one B fragment
// (diagonal d = tile - k-block) serves every tile of the wave on that diagonal.  Each wave owns
// a static run of kRun column tiles (template W), loads each diagonal's fragment once and
// issues up to kRun MFMAs with it.
constexpr int kRun = (kT1 - kT0 + 3) / 4;  // 5 tiles per wave
template <int W>
__device__ __forceinline__ int diag_body(const uint8_t (*s_mur)[kMurLen], const v4i (&af)[kKB], int r, int h,
                                         int* out, int check, int it) {
  v16i acc[kRun];
#pragma unroll
  for (int m = 0; m < kRun; ++m) acc[m] = v16i{};
  constexpr int ct0 = kT0 + W * kRun;
#pragma unroll
  for (int d = ct0 - (kKB - 1); d <= ct0 + kRun - 1; ++d) {
    const int D = d * 32;
    if (!(D + 31 >= 0 && D - 31 < kDig)) continue;
    const int t0 = kP - D - r + 16 * h;
    const int s = t0 & 15;
    const v4i bf = *reinterpret_cast<const v4i*>(&s_mur[s][t0 - s]);
#pragma unroll
    for (int m = 0; m < kRun; ++m) {
      const int kb = ct0 + m - d;
      if (ct0 + m < kT1 && kb >= 0 && kb < kKB) acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[kb], bf, acc[m], 0, 0, 0);
    }
  }
  int sink = 0;
#pragma unroll
  for (int m = 0; m < kRun; ++m) {
    if (ct0 + m >= kT1) continue;
    if (check && it == 0)
      for (int i = 0; i < 16; ++i)
        out[((size_t)blockIdx.x * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * 1184 + (ct0 + m) * 32 + r] = acc[m][i];
#pragma unroll
    for (int i = 0; i < 16; ++i) sink += acc[m][i];
  }
  return sink;
}

__global__ void __launch_bounds__(256) k_toeplitz_diag(const uint8_t* __restrict__ digits, const uint8_t* __restrict__ mu,
                                                       int* __restrict__ out, int iters, int check) {
  __shared__ __attribute__((aligned(16))) uint8_t s_a[32][kKPad];
  __shared__ __attribute__((aligned(16))) uint8_t s_mur[16][kMurLen];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, r = l & 31, h = l >> 5;
  const uint8_t* src = digits + (size_t)blockIdx.x * 32 * kKPad;
  for (int i = tid; i < 32 * kKPad; i += 256) s_a[i / kKPad][i % kKPad] = src[i];
  for (int i = tid; i < 16 * kMurLen; i += 256) {
    const int s = i / kMurLen, u = i % kMurLen, t = u + s, mi = kP - t;
    s_mur[s][u] = (mi >= 0 && mi < kDig) ? mu[mi] : 0;
  }
  __syncthreads();
  v4i af[kKB];
#pragma unroll
  for (int kb = 0; kb < kKB; ++kb) af[kb] = *reinterpret_cast<const v4i*>(&s_a[r][kb * 32 + 16 * h]);
  int sink = 0;
  for (int it = 0; it < iters; ++it) {
    if (wave == 0) sink += diag_body<0>(s_mur, af, r, h, out, check, it);
    else if (wave == 1) sink += diag_body<1>(s_mur, af, r, h, out, check, it);
    else if (wave == 2) sink += diag_body<2>(s_mur, af, r, h, out, check, it);
    else sink += diag_body<3>(s_mur, af, r, h, out, check, it);
  }
  if (sink == 0x7fffffff) out[0] = sink;
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 768 * 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  int dev_cus = 0;
  CHK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
  srand(7);
  // part 1
  {
    std::vector<int8_t> A(1024), B(1024);
    for (auto& v : A) v = (int8_t)(rand() % 256 - 128);
    for (auto& v : B) v = (int8_t)(rand() % 256 - 128);
    std::vector<int> ref(1024, 0);
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j)
        for (int k = 0; k < 32; ++k) ref[i * 32 + j] += A[i * 32 + k] * B[k * 32 + j];
    int8_t *dA, *dB;
    int* dD;
    CHK(hipMalloc(&dA, 1024));
    CHK(hipMalloc(&dB, 1024));
    CHK(hipMalloc(&dD, 4096));
    CHK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    for (int map = 0; map < 2; ++map) {
      hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD, map);
      CHK(hipDeviceSynchronize());
      std::vector<int> D(1024);
      CHK(hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int i = 0; i < 1024; ++i) bad += D[i] != ref[i];
      printf("layout map %d: %d / 1024 mismatches\n", map, bad);
    }
  }
  // part 2
  const size_t nj = (size_t)blocks * 32;
  std::vector<uint8_t> dig(nj * kKPad, 0), mu(kDig);
  for (size_t j = 0; j < nj; ++j)
    for (int k = 0; k < kDig; ++k) dig[j * kKPad + k] = (uint8_t)(rand() & 127);
  for (auto& v : mu) v = (uint8_t)(rand() & 127);
  uint8_t *d_dig, *d_mu;
  int* d_out;
  CHK(hipMalloc(&d_dig, dig.size()));
  CHK(hipMalloc(&d_mu, kDig));
  CHK(hipMalloc(&d_out, nj * 1184 * 4));
  CHK(hipMemcpy(d_dig, dig.data(), dig.size(), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_mu, mu.data(), kDig, hipMemcpyHostToDevice));
  for (int map = 0; map < 3; ++map) {
    auto kern = map == 0 ? k_toeplitz<0> : map == 1 ? k_toeplitz<1> : k_toeplitz_diag;
    CHK(hipMemset(d_out, 0, nj * 1184 * 4));
    hipLaunchKernelGGL(kern, dim3(2), dim3(256), 0, 0, d_dig, d_mu, d_out, 1, 1);
    CHK(hipDeviceSynchronize());
    std::vector<int> o(64 * 1184);
    CHK(hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0, checked = 0;
    for (int j = 0; j < 64; ++j)
      for (int c = kT0 * 32; c < kT1 * 32; ++c) {
        long s = 0;
        for (int k = 0; k < kDig; ++k) {
          const int mi = c - k;
          if (mi >= 0 && mi < kDig) s += (long)dig[j * kKPad + k] * mu[mi];
        }
        bad += o[j * 1184 + c] != s;
        ++checked;
      }
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_dig, d_mu, d_out, 2, 0);
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_dig, d_mu, d_out, iters, 0);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    long mfma = 0;
    for (int ct = kT0; ct < kT1; ++ct)
      for (int kb = 0; kb < kKB; ++kb) {
        const int D = ct * 32 - kb * 32;
        mfma += (D + 31 >= 0 && D - 31 < kDig);
      }
    const double jobs = (double)nj * iters;
    printf("map %d: check %d / %d mismatches; %d blocks x %d iters: %.3f ms, %.4f ns per job-GEMM "
           "(%ld MFMA 32x32x32 per 32 jobs, %.2f P i8-MAC/s), CUs %d\n",
           map, bad, checked, blocks, iters, ms, ms * 1e6 / jobs, mfma,
           (double)mfma * 32768.0 * blocks * iters / (ms * 1e-3) / 1e15, dev_cus);
  }
  return 0;
}
