// One-wave latency microbenchmark (gfx950): the per-element multiply runs ONE wave per SIMD, so
// its speed is set by dependency latency, not issue.  One workgroup of 64 lanes; each case runs K
// independent dependency chains of one instruction and reports core clocks per instruction per
// chain (s_memtime counts core clocks: checked against s_memrealtime's 100 MHz).
//   hipcc --offload-arch=gfx950 -O3 -o _ub/ubench_lat tools/ubench_lat.hip && _ub/ubench_lat
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 2048
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int OP, int K>
__global__ void __launch_bounds__(1024) klat(uint32_t* out, uint32_t seed, unsigned long long* clk) {
  __shared__ uint32_t s_l[256];
  const uint32_t ln = threadIdx.x & 63;
  uint32_t a = ln * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_l[i] = (i * 7u) & 255u;
  __syncthreads();
  uint64_t acc[K];
  uint32_t u[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { acc[k] = a + k; u[k] = (a + k) & 255u; }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if constexpr (OP == 0) {  // v_mad_u64_u32 acc = a*b + acc
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b) : "vcc");
      } else if constexpr (OP == 1) {  // carry split: acc = (acc >> 29) + acc  (v_lshrrev_b64 + v_lshl_add_u64)
        uint64_t t;
        asm volatile("v_lshrrev_b64 %0, 29, %1\n\tv_lshl_add_u64 %1, %1, 0, %0" : "=&v"(t), "+v"(acc[k]));
      } else if constexpr (OP == 2) {  // DPP wave_shl:1
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %0 wave_shl:1 row_mask:0xf bank_mask:0xf" : "+v"(u[k]));
      } else if constexpr (OP == 3) {  // readlane -> add
        uint32_t s;
        asm volatile("v_readlane_b32 %0, %1, 0\n\ts_nop 3\n\tv_add_u32 %1, %0, %1" : "=&s"(s), "+v"(u[k]));
      } else if constexpr (OP == 4) {  // LDS load whose address is the previous value
        asm volatile("v_lshlrev_b32 %0, 2, %0\n\tds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)" : "+v"(u[k]) :: "memory");
      } else if constexpr (OP == 5) {  // v_add_u32
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[k]) : "v"(b));
      } else if constexpr (OP == 7) {  // a MAC and an independent add in turn (does the add hide under the MAC?)
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_add_u32 %1, %1, %3" : "+v"(acc[k]), "+v"(u[k]) : "v"(a), "v"(b) : "vcc");
      } else if constexpr (OP == 6) {  // 64-bit add via lshl_add
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"((uint64_t)b));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) s += acc[k] + u[k];
  out[threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32) ^ s_l[ln];
  if (threadIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
  if (ln == 0) { clk[2 + 2 * (threadIdx.x >> 6)] = t0; clk[3 + 2 * (threadIdx.x >> 6)] = t1; }
}

// waves: the workgroup's waves (4 SIMDs per CU: 4 waves = one per SIMD, 8 = two per SIMD, ...)
template <int OP, int K>
int run(const char* name, int insts, int waves = 1) {
  uint32_t* out;
  unsigned long long* clk;
  CHK(hipMalloc(&out, 1024 * 4));
  CHK(hipMalloc(&clk, 16 * 36));
  klat<OP, K><<<1, 64 * waves>>>(out, 1, clk);
  CHK(hipDeviceSynchronize());
  klat<OP, K><<<1, 64 * waves>>>(out, 2, clk);
  CHK(hipDeviceSynchronize());
  unsigned long long c[36];
  CHK(hipMemcpy(c, clk, 8 * (2 + 2 * waves), hipMemcpyDeviceToHost));
  unsigned long long lo = ~0ull, hi = 0;
  for (int w = 0; w < waves; ++w) { lo = c[2 + 2 * w] < lo ? c[2 + 2 * w] : lo; hi = c[3 + 2 * w] > hi ? c[3 + 2 * w] : hi; }
  // all waves together: clocks per wave-instruction per SIMD (waves spread over 4 SIMDs)
  const double simd = (double)(hi - lo) / ((double)ITERS * insts * K * waves / (waves < 4 ? waves : 4));
  const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  const double per_chain = (double)c[0] / ITERS / insts;   // clocks per instruction along one chain
  const double per_issue = per_chain / K;                   // clocks per issued instruction
  printf("%-34s W=%-2d K=%-2d %7.2f clk/instr on a chain  %6.2f clk/instr issued  %6.2f clk/instr per SIMD, all waves  (clk %.2f GHz)\n",
         name, waves, K, per_chain, per_issue, simd, ghz);
  CHK(hipFree(out));
  CHK(hipFree(clk));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  printf("device %s  CUs %d\n", p.gcnArchName, p.multiProcessorCount);
  run<0, 1>("v_mad_u64_u32 acc chain", 1);
  run<0, 2>("v_mad_u64_u32 acc chain", 1);
  run<0, 3>("v_mad_u64_u32 acc chain", 1);
  run<0, 4>("v_mad_u64_u32 acc chain", 1);
  run<0, 6>("v_mad_u64_u32 acc chain", 1);
  run<0, 8>("v_mad_u64_u32 acc chain", 1);
  run<0, 12>("v_mad_u64_u32 acc chain", 1);
  run<1, 1>("lshr64+lshl_add64 carry chain", 2);
  run<1, 4>("lshr64+lshl_add64 carry chain", 2);
  run<6, 1>("v_lshl_add_u64 chain", 1);
  run<6, 4>("v_lshl_add_u64 chain", 1);
  run<5, 1>("v_add_u32 chain", 1);
  run<5, 4>("v_add_u32 chain", 1);
  run<2, 1>("dpp wave_shl (+s_nop 1) chain", 2);
  run<2, 4>("dpp wave_shl (+s_nop 1) chain", 2);
  run<3, 1>("readlane+nop3+add chain", 3);
  run<4, 1>("ds_read addr chain", 3);
  run<4, 4>("ds_read addr chain", 3);
  // per-wave MAC rate against waves per SIMD (the workgroup's waves spread over the CU's 4 SIMDs)
  run<0, 8>("v_mad_u64_u32 acc chain", 1, 2);
  run<0, 8>("v_mad_u64_u32 acc chain", 1, 4);
  run<0, 8>("v_mad_u64_u32 acc chain", 1, 8);
  run<0, 8>("v_mad_u64_u32 acc chain", 1, 12);
  run<0, 8>("v_mad_u64_u32 acc chain", 1, 16);
  run<5, 4>("v_add_u32 chain", 1, 8);
  run<7, 8>("mad_u64_u32 + add_u32 pairs", 2);
  return 0;
}
