// eg_pow16.hip — the latency-shaped instantiation of the device core: the same kernels as the
// throughput path (eg_kernels.hpp: k_import, the op-program k_pow, k_export) compiled with 16 lanes
// per element (EG_T = 16) in namespace eg16.  A 4096-bit exponentiation is ~330 Montgomery
// operations in sequence; an 8-lane group runs each in ~12 us (L = 18 limbs per lane: 144 CIOS
// steps of 36 MACs + glue), a 16-lane group in about half (L = 9, and the quotient broadcast is one
// row_newbcast move), so a batch that fits one resident round finishes in about half the time.
// That is what a blocking per-element caller waits for (eg_capi_coalesce.inc); large batches keep
// the 8-lane layout, which does ~12% more work per lane-cycle.  See eg_pow16.h.
#define EG_T 16
#define eg eg16
#include "eg_kernels.hpp"
#undef eg

#pragma clang diagnostic ignored "-Wunused-value"
#include <cstring>
#include <vector>

#include "eg_pow16.h"

using namespace eg16;

struct Pow16Consts {
  MontConsts* d = nullptr;
};

// little-endian 32-bit words -> the 16-lane device element (radix 2^29 limbs, padded lane blocks)
static void words_to_elem16(const uint32_t* w, int nw, uint32_t* out) {
  std::memset(out, 0, sizeof(uint32_t) * kW);
  for (int a = 0; a < kN; ++a) {
    const int bit = a * kLimbBits;
    uint64_t v = 0;
    for (int k = 0; k < 3; ++k) {
      const int wi = bit / 32 + k;
      if (wi < nw) v |= (uint64_t)w[wi] << (32 * k);
    }
    out[(a / kL) * kLP + (a % kL)] = (uint32_t)(v >> (bit % 32)) & kMask;
  }
}

int pow16_consts_create(const uint32_t* p, const uint32_t* r2, const uint32_t* one, uint32_t n0, uint32_t friendly,
                        Pow16Consts** out, std::string* err) {
  MontConsts h{};
  words_to_elem16(p, 128, h.p);
  words_to_elem16(r2, 129, h.r2);
  words_to_elem16(one, 129, h.one);
  const uint32_t unit[1] = {1};
  words_to_elem16(unit, 1, h.unit);
  std::memcpy(h.pw, p, sizeof(h.pw));
  h.n0 = n0;
  h.friendly = friendly;
  h.mask = kMask;
  auto* c = new Pow16Consts();
  hipError_t e = hipMalloc(&c->d, sizeof(MontConsts));
  if (e == hipSuccess) e = hipMemcpy(c->d, &h, sizeof(MontConsts), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (c->d) hipFree(c->d);
    delete c;
    *err = std::string("pow16 constants: ") + hipGetErrorString(e);
    return 1;
  }
  *out = c;
  return 0;
}

void pow16_consts_destroy(Pow16Consts* c) {
  if (!c) return;
  if (c->d) hipFree(c->d);
  delete c;
}

size_t pow16_elem_bytes() { return (size_t)kW * 4; }

static size_t padded16(size_t n) { return (n + kGroupsPerBlock - 1) / kGroupsPerBlock * kGroupsPerBlock; }

size_t pow16_scratch_bytes(size_t n) { return padded16(n) * 16 * (size_t)kW * 4; }

size_t pow16_round_jobs(int device) {
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pow<true, false>, kBlock, 0) != hipSuccess)
    return 0;
  return (size_t)cus * (size_t)per_cu * kGroupsPerBlock;
}

int pow16_powp(const Pow16Consts* C, bool friendly, hipStream_t s, const uint32_t* sched, const uint32_t* jobs,
               const uint8_t* base_be, const uint8_t* exp_be, uint8_t* out_be, size_t n, uint32_t* elems,
               uint32_t* outs, uint32_t* scratch, std::string* err) {
  if (!n) return 0;
  const unsigned grid = (unsigned)((n + kGroupsPerBlock - 1) / kGroupsPerBlock);
  PowShape S{};
  S.has_base = 1;
  S.nout = 1;
  S.exp_bytes = 32;
  PowPart P0{S, sched, jobs, (uint32_t)n, grid, scratch, nullptr, nullptr, nullptr, nullptr};
  PowPart none{};
  const FbTab nofb{nullptr, 0, 0};
  if (friendly) {
    hipLaunchKernelGGL(k_import<true>, dim3(grid), dim3(kBlock), 0, s, C->d, base_be, (uint32_t)n, elems, nullptr);
    hipLaunchKernelGGL((k_pow<true, false>), dim3(grid), dim3(kBlock), 0, s, C->d, P0, none, none, elems, exp_be, outs,
                       nofb, nofb, nullptr);
    hipLaunchKernelGGL(k_export<true>, dim3(grid), dim3(kBlock), 0, s, C->d, outs, (uint32_t)n, out_be);
  } else {
    hipLaunchKernelGGL(k_import<false>, dim3(grid), dim3(kBlock), 0, s, C->d, base_be, (uint32_t)n, elems, nullptr);
    hipLaunchKernelGGL((k_pow<false, false>), dim3(grid), dim3(kBlock), 0, s, C->d, P0, none, none, elems, exp_be,
                       outs, nofb, nofb, nullptr);
    hipLaunchKernelGGL(k_export<false>, dim3(grid), dim3(kBlock), 0, s, C->d, outs, (uint32_t)n, out_be);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = std::string("pow16 launch: ") + hipGetErrorString(e);
    return 1;
  }
  return 0;
}
