// Co-execution microbenchmark for the planned Barrett + i8-MFMA reduction:
// can an MFMA-heavy wave (v_mfma_i32_16x16x64_i8 fed by one ds_read_b128 per MFMA, the
// Toeplitz B-fragment rate) run beside a VALU-heavy wave (v_mad_u64_u32 chains, the CIOS
// product) on the same SIMD without slowing it?
//   mode 0: every wave VALU      mode 1: every wave MFMA      mode 2: half VALU, half MFMA
// 512-thread workgroups (2 waves per SIMD), 2 workgroups per CU.  In mode 2 waves 0-3 run the
// VALU loop and waves 4-7 the MFMA loop, so every SIMD holds both kinds.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_coexec tools/ubench_coexec.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

template <int MODE, int VOP, int LDSB>
__global__ void __launch_bounds__(512) kco(uint32_t* out, int iv, int im, uint32_t seed) {
  __shared__ v4i s_b[1024];
  for (int i = threadIdx.x; i < 1024; i += 512) s_b[i] = v4i{(int)(i * 7 + seed), i ^ 0x55, i * 3, (int)seed};
  __syncthreads();
  const int wave = threadIdx.x / 64;
  const bool valu = MODE == 0 || (MODE == 2 && wave < 4);
  uint32_t res = 0;
  if (valu) {
    uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
    uint64_t acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = a + k;
    for (int it = 0; it < iv; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if constexpr (VOP == 0)
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b) : "vcc");
        else if constexpr (VOP == 1)
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(*(uint32_t*)&acc[k]) : "v"(b));
        else
          asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(*(uint32_t*)&acc[k]) : "v"(b));
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) res += (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32);
  } else {
    v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const v4i a = {(int)threadIdx.x, (int)seed, 3, 5};
    int idx = threadIdx.x & 63;
    for (int it = 0; it < im; ++it) {
      v4i b0 = a, b1 = a, b2 = a, b3 = a;
      if constexpr (LDSB) {
        b0 = s_b[(idx + 0) & 1023];
        b1 = s_b[(idx + 64) & 1023];
        b2 = s_b[(idx + 128) & 1023];
        b3 = s_b[(idx + 192) & 1023];
      }
      c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b0, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b2, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b3, c3, 0, 0, 0);
      idx += 256;
    }
    res = c0.x + c1.y + c2.z + c3.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = res;
}

template <int MODE, int VOP, int LDSB>
float run(uint32_t* out, int blocks, int iv, int im) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  kco<MODE, VOP, LDSB><<<blocks, 512>>>(out, iv, im, 1);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  kco<MODE, VOP, LDSB><<<blocks, 512>>>(out, iv, im, 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 2;  // 2 x 512-thread workgroups per CU -> 4 waves per SIMD
  uint32_t* out;
  CHK(hipMalloc(&out, (size_t)blocks * 512 * 4));
  const int iv = 2048 * 16, im = 1024 * 16;  // per wave: 256k VALU ops, 64k MFMA 16x16x64 i8
  const double waves = blocks * 8.0;
  printf("device %s  CUs %d\n", prop.gcnArchName, cus);
  auto report = [&](const char* name, float t0, float t1, float t2) {
    printf("%-34s valu %.3f ms (%.2f T lane-op/s)  mfma %.3f ms (%.2f P MAC/s)  mixed %.3f ms  co-exec eff %.2f\n",
           name, t0, waves * iv * 8 * 64 / t0 / 1e9, t1, waves * im * 4 * 16384.0 / t1 / 1e12, t2,
           ((t0 + t1) / 2 - t2) / ((t0 + t1) / 2 - (t0 > t1 ? t0 : t1) / 2));
  };
  report("v_mad_u64_u32 + mfma(LDS B)", run<0, 0, 1>(out, blocks, iv, im), run<1, 0, 1>(out, blocks, iv, im),
         run<2, 0, 1>(out, blocks, iv, im));
  report("v_mad_u64_u32 + mfma(reg B)", run<0, 0, 0>(out, blocks, iv, im), run<1, 0, 0>(out, blocks, iv, im),
         run<2, 0, 0>(out, blocks, iv, im));
  report("v_add_u32     + mfma(reg B)", run<0, 1, 0>(out, blocks, iv, im), run<1, 1, 0>(out, blocks, iv, im),
         run<2, 1, 0>(out, blocks, iv, im));
  report("v_mul_lo_u32  + mfma(reg B)", run<0, 2, 0>(out, blocks, iv, im), run<1, 2, 0>(out, blocks, iv, im),
         run<2, 2, 0>(out, blocks, iv, im));
  return 0;
}
