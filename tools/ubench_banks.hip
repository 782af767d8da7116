// VGPR-bank microbenchmark for v_mad_u64_u32, the CIOS multiply-accumulate.
// The VGPR file has 4 banks (register index mod 4).  One v_mad_u64_u32 reads src0, src1 and a
// 64-bit src2 pair (two consecutive registers = two banks).  The question is whether operands
// that share a bank slow the issue rate, i.e. whether a bank-aware register assignment of the
// CIOS step (accumulator pairs in banks {0,1}, x / y / m / p in banks {2,3}) would pay.
// Every variant runs 8 independent accumulator chains per lane with explicitly named VGPRs.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_banks tools/ubench_banks.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 8192
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define CLOB "v2", "v3", "v4", "v5", "v6", "v7", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", \
  "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", \
  "v41", "v42", "v43", "v44", "v45", "v46", "v47", "vcc"

// acc pairs at v[16+4k : 17+4k] -> banks (0,1); src0 v2 (bank 2), src1 v3 (bank 3): conflict-free
#define FREE8 \
  "v_mad_u64_u32 v[16:17], vcc, v2, v3, v[16:17]\n\t" "v_mad_u64_u32 v[20:21], vcc, v2, v3, v[20:21]\n\t" \
  "v_mad_u64_u32 v[24:25], vcc, v2, v3, v[24:25]\n\t" "v_mad_u64_u32 v[28:29], vcc, v2, v3, v[28:29]\n\t" \
  "v_mad_u64_u32 v[32:33], vcc, v2, v3, v[32:33]\n\t" "v_mad_u64_u32 v[36:37], vcc, v2, v3, v[36:37]\n\t" \
  "v_mad_u64_u32 v[40:41], vcc, v2, v3, v[40:41]\n\t" "v_mad_u64_u32 v[44:45], vcc, v2, v3, v[44:45]\n\t"
// same pairs, src0 v2 and src1 v6 both in bank 2: src0/src1 conflict
#define SRCCONF8 \
  "v_mad_u64_u32 v[16:17], vcc, v2, v6, v[16:17]\n\t" "v_mad_u64_u32 v[20:21], vcc, v2, v6, v[20:21]\n\t" \
  "v_mad_u64_u32 v[24:25], vcc, v2, v6, v[24:25]\n\t" "v_mad_u64_u32 v[28:29], vcc, v2, v6, v[28:29]\n\t" \
  "v_mad_u64_u32 v[32:33], vcc, v2, v6, v[32:33]\n\t" "v_mad_u64_u32 v[36:37], vcc, v2, v6, v[36:37]\n\t" \
  "v_mad_u64_u32 v[40:41], vcc, v2, v6, v[40:41]\n\t" "v_mad_u64_u32 v[44:45], vcc, v2, v6, v[44:45]\n\t"
// acc pairs at v[18+4k : 19+4k] -> banks (2,3): both sources collide with the accumulator
#define ACCCONF8 \
  "v_mad_u64_u32 v[18:19], vcc, v2, v3, v[18:19]\n\t" "v_mad_u64_u32 v[22:23], vcc, v2, v3, v[22:23]\n\t" \
  "v_mad_u64_u32 v[26:27], vcc, v2, v3, v[26:27]\n\t" "v_mad_u64_u32 v[30:31], vcc, v2, v3, v[30:31]\n\t" \
  "v_mad_u64_u32 v[34:35], vcc, v2, v3, v[34:35]\n\t" "v_mad_u64_u32 v[38:39], vcc, v2, v3, v[38:39]\n\t" \
  "v_mad_u64_u32 v[42:43], vcc, v2, v3, v[42:43]\n\t" "v_mad_u64_u32 v[46:47], vcc, v2, v3, v[46:47]\n\t"
// the kernel's typical pattern: even src0 / src1 (banks 0/2) against alternating pairs
#define MIXED8 \
  "v_mad_u64_u32 v[16:17], vcc, v2, v4, v[16:17]\n\t" "v_mad_u64_u32 v[18:19], vcc, v2, v4, v[18:19]\n\t" \
  "v_mad_u64_u32 v[20:21], vcc, v2, v4, v[20:21]\n\t" "v_mad_u64_u32 v[22:23], vcc, v2, v4, v[22:23]\n\t" \
  "v_mad_u64_u32 v[24:25], vcc, v2, v4, v[24:25]\n\t" "v_mad_u64_u32 v[26:27], vcc, v2, v4, v[26:27]\n\t" \
  "v_mad_u64_u32 v[28:29], vcc, v2, v4, v[28:29]\n\t" "v_mad_u64_u32 v[30:31], vcc, v2, v4, v[30:31]\n\t"

template <int V, int OCC>
__global__ void __launch_bounds__(256, OCC) kbank(uint32_t* out, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (V == 0) asm volatile(FREE8 ::: CLOB);
    else if constexpr (V == 1) asm volatile(SRCCONF8 ::: CLOB);
    else if constexpr (V == 2) asm volatile(ACCCONF8 ::: CLOB);
    else asm volatile(MIXED8 ::: CLOB);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)t1;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int V, int OCC>
int run(const char* name, int blocks_per_cu) {
  const int blocks = 256 * blocks_per_cu, threads = 256;
  uint32_t* out; unsigned long long* clk;
  CHK(hipMalloc(&out, (size_t)blocks * threads * 4));
  CHK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  kbank<V, OCC><<<blocks, threads>>>(out, clk);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  kbank<V, OCC><<<blocks, threads>>>(out, clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long c[2]; CHK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  const double insts = (double)blocks * threads * ITERS * 8;  // lane-instructions
  const double clk_ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  const double lpc = insts / (ms * 1e-3) / (256.0 * clk_ghz * 1e9);
  printf("%-44s waves/SIMD %d  %7.3f ms  clk %.2f GHz  %5.1f lane-op/clk/CU  %.2f cyc/wave-instr/SIMD\n", name,
         blocks_per_cu, ms, clk_ghz, lpc, 64.0 * 4.0 / lpc);
  CHK(hipFree(out)); CHK(hipFree(clk));
  return 0;
}

int main() {
  for (int bpc : {1, 3}) {  // waves per SIMD (4 waves per 256-thread block, one per SIMD)
    run<0, 1>("conflict-free (acc b01, src b2/b3)", bpc);
    run<1, 1>("src0/src1 same bank", bpc);
    run<2, 1>("both sources collide with acc pair", bpc);
    run<3, 1>("kernel-like (even srcs, alternating pairs)", bpc);
  }
  return 0;
}
