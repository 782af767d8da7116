// Issue rate of v_mad_u64_u32 against waves per SIMD and independent chains per wave
// ("Where the cycles go").  k_pow runs 3 waves per SIMD (VGPR-limited); this
// asks whether the measured 4.4 cycles per wave-instruction is the pipe's rate or a latency
// that more waves (a smaller register budget) or more independent accumulators would hide.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_ubench_occ tools/ubench_occ.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 32768
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define CLOB "v2", "v3", "v4", "v5", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", \
  "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", \
  "v43", "v44", "v45", "v46", "v47", "vcc"

#define M(a) "v_mad_u64_u32 v[" #a "], vcc, v2, v3, v[" #a "]\n\t"
// 4 chains: each accumulator is re-read 4 instructions later
#define C4 M(16:17) M(18:19) M(20:21) M(22:23)
// 8 chains
#define C8 C4 M(24:25) M(26:27) M(28:29) M(30:31)
// 16 chains
#define C16 C8 M(32:33) M(34:35) M(36:37) M(38:39) M(40:41) M(42:43) M(44:45) M(46:47)
// 32-bit adds, 16 chains (the glue's rate)
#define A(a) "v_add_u32 v" #a ", v2, v" #a "\n\t"
#define A16 A(16) A(17) A(18) A(19) A(20) A(21) A(22) A(23) A(24) A(25) A(26) A(27) A(28) A(29) A(30) A(31)
// the CIOS step's mix: 4 MACs then one 32-bit op, 16 chains
#define MIX M(16:17) M(18:19) M(20:21) M(22:23) A(4) M(24:25) M(26:27) M(28:29) M(30:31) A(5) \
  M(32:33) M(34:35) M(36:37) M(38:39) A(4) M(40:41) M(42:43) M(44:45) M(46:47) A(5)
// 8 MACs : 1 add (about the CIOS step's 36 : 5)
#define MIX8 C8 A(4) M(32:33) M(34:35) M(36:37) M(38:39) M(40:41) M(42:43) M(44:45) M(46:47) A(5)
// 1 MAC : 1 add
#define MIX1 M(16:17) A(4) M(18:19) A(5) M(20:21) A(4) M(22:23) A(5) M(24:25) A(4) M(26:27) A(5) M(28:29) A(4) \
  M(30:31) A(5)
// 8 MACs : 1 DPP move
#define D(a) "v_mov_b32_dpp v" #a ", v3 row_shl:1 row_mask:0xf bank_mask:0xf\n\t"
#define MIXD C8 D(4) M(32:33) M(34:35) M(36:37) M(38:39) M(40:41) M(42:43) M(44:45) M(46:47) D(5)

template <int V>
__global__ void __launch_bounds__(256) kocc(uint32_t* out, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (V == 0) asm volatile(C4 C4 C4 C4 ::: CLOB);
    else if constexpr (V == 1) asm volatile(C8 C8 ::: CLOB);
    else if constexpr (V == 2) asm volatile(C16 ::: CLOB);
    else if constexpr (V == 3) asm volatile(A16 ::: CLOB);
    else if constexpr (V == 4) asm volatile(MIX ::: CLOB);
    else if constexpr (V == 5) asm volatile(MIX8 ::: CLOB);
    else if constexpr (V == 6) asm volatile(MIX1 ::: CLOB);
    else asm volatile(MIXD ::: CLOB);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)t1;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int V>
int run(const char* name, int per_iter, int bpc) {
  const int blocks = 256 * bpc, threads = 256;
  uint32_t* out; unsigned long long* clk;
  CHK(hipMalloc(&out, (size_t)blocks * threads * 4));
  CHK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  kocc<V><<<blocks, threads>>>(out, clk);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  kocc<V><<<blocks, threads>>>(out, clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long c[2]; CHK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  const double insts = (double)blocks * threads * ITERS * per_iter;  // lane-instructions
  const double clk_ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  const double lpc = insts / (ms * 1e-3) / (256.0 * clk_ghz * 1e9);
  // one wave's own cycle count: all bpc waves of its SIMD run beside it for the whole loop
  const double wave_cyc = (double)c[0] / ((double)ITERS * per_iter * bpc);
  printf("%-28s waves/SIMD %d  %7.3f ms  clk %.2f GHz  %5.1f lane-op/clk/CU  %.2f cyc/wave-instr/SIMD (event)  "
         "%.2f (wave clock)\n", name, bpc, ms, clk_ghz, lpc, 64.0 * 4.0 / lpc, wave_cyc);
  CHK(hipFree(out)); CHK(hipFree(clk));
  CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
  return 0;
}

int main() {
  for (int bpc : {1, 2, 3, 4, 6, 8}) {  // waves per SIMD (a 256-thread block puts one wave on each SIMD)
    if (run<0>("mad, 4 chains", 16, bpc)) return 1;
    if (run<1>("mad, 8 chains", 16, bpc)) return 1;
    if (run<2>("mad, 16 chains", 16, bpc)) return 1;
    if (run<3>("add_u32, 16 chains", 16, bpc)) return 1;
    if (run<4>("4 mad : 1 add, 16 chains", 20, bpc)) return 1;
    if (run<5>("8 mad : 1 add", 18, bpc)) return 1;
    if (run<6>("1 mad : 1 add", 16, bpc)) return 1;
    if (run<7>("8 mad : 1 dpp mov", 18, bpc)) return 1;
  }
  return 0;
}
