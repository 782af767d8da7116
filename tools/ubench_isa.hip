// Instruction-throughput microbenchmark for the integer / fp64 ops a 4096-bit
// Montgomery multiply can be built from on gfx950.  Each thread runs 8
// independent chains so issue (not latency) is measured.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int OP>
__global__ void __launch_bounds__(256) kbench(uint32_t* out, uint32_t seed, unsigned long long* clk) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t b = a ^ 0x9e3779b9u;
  uint64_t acc[8];
  double facc[8];
  uint32_t u[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { acc[k] = a + k; facc[k] = (double)(a + k); u[k] = a * (k + 3); }
  double fa = (double)a, fb = (double)b * 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (OP == 0) {  // v_mad_u64_u32
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b) : "vcc");
      } else if constexpr (OP == 1) {  // v_mul_lo_u32
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[k]) : "v"(b));
      } else if constexpr (OP == 2) {  // v_mul_hi_u32
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[k]) : "v"(b));
      } else if constexpr (OP == 3) {  // v_add_co_u32
        asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(u[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 4) {  // v_addc_co_u32
        asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(u[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 5) {  // v_fma_f64
        asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(facc[k]) : "v"(fa), "v"(fb));
      } else if constexpr (OP == 6) {  // v_mad_u32_u24
        asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(u[k]) : "v"(b), "v"(a));
      } else if constexpr (OP == 7) {  // v_mul_hi_u32_u24
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(u[k]) : "v"(b));
      } else if constexpr (OP == 8) {  // v_dot2_u32_u16
        asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(u[k]) : "v"(a), "v"(b));
      } else if constexpr (OP == 9) {  // v_lshl_add_u64 (gfx940+)
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"((uint64_t)b));
      } else if constexpr (OP == 10) {  // v_add3_u32
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(u[k]) : "v"(a), "v"(b));
      } else if constexpr (OP == 11) {  // v_mad_u64_u32 with SGPR multiplicand
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "s"(seed), "v"(b) : "vcc");
      } else if constexpr (OP == 12) {  // DPP row_shr:1 mov
        asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(u[k]));
      } else if constexpr (OP == 13) {  // v_mul_f64
        asm volatile("v_mul_f64 %0, %0, %1" : "+v"(facc[k]) : "v"(fb));
      } else if constexpr (OP == 14) {  // v_cndmask-free carry capture: v_addc_co_u32 hi, vcc, hi, 0, vcc
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_addc_co_u32 %3, vcc, %3, 0, vcc" : "+v"(acc[k]), "+v"(u[k]) : "v"(a), "v"(b) : "vcc");
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += acc[k] + (uint64_t)facc[k] + u[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int OP>
int run(const char* name, int insts_per_iter) {
  int blocks = 256 * 8, threads = 256;
  uint32_t* out; unsigned long long* clk;
  CHK(hipMalloc(&out, blocks * threads * 4));
  CHK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  kbench<OP><<<blocks, threads>>>(out, 1, clk);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  kbench<OP><<<blocks, threads>>>(out, 2, clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long c[2]; CHK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double insts = (double)blocks * threads * ITERS * 8 * insts_per_iter;  // lane-instructions
  double rate = insts / (ms * 1e-3);
  double clk_ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  // lanes per clock per CU at the measured in-kernel clock
  double lpc = rate / (256.0 * clk_ghz * 1e9);
  printf("%-28s %8.3f ms  %9.3f Tlane-op/s  clk %.2f GHz  %6.1f lane-op/clk/CU  (%.2f cyc/wave-instr/SIMD)\n",
         name, ms, rate / 1e12, clk_ghz, lpc, 64.0 * 4.0 / lpc);
  CHK(hipFree(out)); CHK(hipFree(clk));
  return 0;
}

int main() {
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  printf("device %s  CUs %d  clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  run<0>("v_mad_u64_u32", 1);
  run<11>("v_mad_u64_u32 (sgpr src)", 1);
  run<14>("mad_u64_u32+addc pair", 2);
  run<1>("v_mul_lo_u32", 1);
  run<2>("v_mul_hi_u32", 1);
  run<3>("v_add_co_u32", 1);
  run<4>("v_addc_co_u32", 1);
  run<10>("v_add3_u32", 1);
  run<9>("v_lshl_add_u64", 1);
  run<5>("v_fma_f64", 1);
  run<13>("v_mul_f64", 1);
  run<6>("v_mad_u32_u24", 1);
  run<7>("v_mul_hi_u32_u24", 1);
  run<8>("v_dot2_u32_u16", 1);
  run<12>("v_mov_b32_dpp row_shr", 1);
  return 0;
}
