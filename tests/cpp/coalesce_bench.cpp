// coalesce_bench.cpp -- per-element group calls from 11 threads through the C ABI's coalescer
// (eg_powp_one / eg_multp_one / eg_gpowp_one and the submit/wait form, include/eg_hip.h), the
// reference's call pattern: upstream ElementModP.powP / times and GroupContext.gPowP one element per
// call from the 11 encryptor / verifier threads (RunRemoteWorkflowTest.java:140,180) on the context
// KUtils.productionGroup() makes (KUtils.java:10-12).
//
//   coalesce_bench <vectors.bin> [threads]
// vectors.bin (written by tests/test_gpu_coalesce.py from CPython pow, the oracle): u32 n, then n
// records of base[512] exp[32] powp[512] b[512] multp[512] gpowp[512] (big-endian).  Checks every
// result bit-exact and prints one JSON line: the rates of eg_powp_batch (one call), of blocking
// per-element powP calls, of submit-all-then-wait per-element calls, and the mismatch count.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "eg_constants.hpp"
#include "eg_hip.h"
#include "electionguard.hpp"

using namespace electionguard;
using Clock = std::chrono::steady_clock;

static double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: coalesce_bench vectors.bin [threads]\n");
    return 2;
  }
  const int nthreads = argc > 2 ? std::atoi(argv[2]) : 11;
  std::ifstream f(argv[1], std::ios::binary);
  uint32_t n = 0;
  f.read((char*)&n, 4);
  constexpr size_t kRec = 512 + 32 + 512 + 512 + 512 + 512;
  std::vector<uint8_t> v((size_t)n * kRec);
  f.read((char*)v.data(), (std::streamsize)v.size());
  if (!f || n == 0) {
    fprintf(stderr, "bad vector file\n");
    return 2;
  }
  auto rec = [&](uint32_t i) { return v.data() + (size_t)i * kRec; };
  GroupContext& G = GroupContext::productionGroup(0);
  eg_ctx* ctx = G.handle();
  std::atomic<long> bad{0};

  // 1. one batch call over all n (the batched entry point; warm up first)
  std::vector<uint8_t> B(n * 512), E(n * 32), O(n * 512);
  for (uint32_t i = 0; i < n; ++i) {
    std::memcpy(&B[i * 512], rec(i), 512);
    std::memcpy(&E[i * 32], rec(i) + 512, 32);
  }
  check(eg_powp_batch(ctx, B.data(), E.data(), O.data(), n), "eg_powp_batch");
  auto t0 = Clock::now();
  check(eg_powp_batch(ctx, B.data(), E.data(), O.data(), n), "eg_powp_batch");
  const double batch_s = secs(t0);
  for (uint32_t i = 0; i < n; ++i) bad += std::memcmp(&O[i * 512], rec(i) + 544, 512) != 0;

  // 2. blocking per-element calls from nthreads threads (element i on thread i % nthreads)
  auto per_element = [&](int kind) {
    std::vector<std::thread> th;
    auto t = Clock::now();
    for (int k = 0; k < nthreads; ++k)
      th.emplace_back([&, k] {
        uint8_t out[512];
        for (uint32_t i = (uint32_t)k; i < n; i += (uint32_t)nthreads) {
          const uint8_t* r = rec(i);
          int rc;
          if (kind == 0) rc = eg_powp_one(ctx, r, r + 512, out);
          else if (kind == 1) rc = eg_multp_one(ctx, r, r + 1056, out);
          else rc = eg_gpowp_one(ctx, r + 512, out);
          const uint8_t* want = r + (kind == 0 ? 544 : kind == 1 ? 1568 : 2080);
          if (rc || std::memcmp(out, want, 512) != 0) ++bad;
        }
      });
    for (auto& x : th) x.join();
    return secs(t);
  };
  const double one_powp_s = per_element(0);
  const double one_multp_s = per_element(1);
  const double one_gpowp_s = per_element(2);

  // 3. submit-all-then-wait per-element calls (futures), nthreads threads
  std::vector<uint8_t> O2(n * 512);
  std::vector<std::thread> th;
  auto t3 = Clock::now();
  for (int k = 0; k < nthreads; ++k)
    th.emplace_back([&, k] {
      std::vector<eg_ticket*> ts;
      for (uint32_t i = (uint32_t)k; i < n; i += (uint32_t)nthreads) {
        eg_ticket* t = nullptr;
        if (eg_powp_submit(ctx, rec(i), rec(i) + 512, &O2[i * 512], &t)) {
          ++bad;
          continue;
        }
        ts.push_back(t);
      }
      for (auto* t : ts) bad += eg_ticket_wait(t) != EG_OK;
    });
  for (auto& x : th) x.join();
  const double async_s = secs(t3);
  for (uint32_t i = 0; i < n; ++i) bad += std::memcmp(&O2[i * 512], rec(i) + 544, 512) != 0;

  // 4. the C++ mirror's per-element API takes the same path (ElementModP::powP)
  {
    const ElementModP b(rec(0), &G);
    const ElementModQ e = ElementModQ::from_be(rec(0) + 512);
    bad += std::memcmp(b.powP(e).byteArray(), rec(0) + 544, 512) != 0;
  }
  // 5. batch latency sweep: one submit-all-then-wait batch of m elements through the coalescer
  // (max_batch = m: dispatched as soon as the m-th arrives) and one eg_powp_batch call of m, best of 3
  std::string sweep;
  for (uint32_t m : {1u, 11u, 64u, 256u, 1024u, 4096u, 12288u}) {
    if (m > n) m = n;
    std::vector<uint8_t> O3((size_t)m * 512);
    double co_best = 1e9, b_best = 1e9;
    check(eg_ctx_set_coalescing(ctx, m, 1000000), "eg_ctx_set_coalescing");
    for (int rep = 0; rep < 4; ++rep) {  // the first is a warm-up (job tables, buffers)
      std::vector<eg_ticket*> ts(m);
      auto t = Clock::now();
      for (uint32_t i = 0; i < m; ++i) check(eg_powp_submit(ctx, rec(i % n), rec(i % n) + 512, &O3[(size_t)i * 512], &ts[i]), "submit");
      for (auto* x : ts) bad += eg_ticket_wait(x) != EG_OK;
      if (rep) co_best = std::min(co_best, secs(t));
      t = Clock::now();
      check(eg_powp_batch(ctx, B.data(), E.data(), O.data(), m), "eg_powp_batch");
      if (rep) b_best = std::min(b_best, secs(t));
    }
    for (uint32_t i = 0; i < m; ++i) bad += std::memcmp(&O3[(size_t)i * 512], rec(i % n) + 544, 512) != 0;
    char buf[160];
    snprintf(buf, sizeof buf, "%s{\"m\": %u, \"coalesced_ms\": %.3f, \"batch_call_ms\": %.3f}", sweep.empty() ? "" : ", ", m,
             co_best * 1e3, b_best * 1e3);
    sweep += buf;
    if (m == n) break;
  }
  check(eg_ctx_set_coalescing(ctx, 16384, 0), "eg_ctx_set_coalescing");  // the adaptive default
  printf("{\"n\": %u, \"threads\": %d, \"mismatches\": %ld, \"sweep\": [%s], \"powp_batch_per_s\": %.1f, "
         "\"powp_one_blocking_per_s\": %.1f, \"multp_one_blocking_per_s\": %.1f, \"gpowp_one_blocking_per_s\": %.1f, "
         "\"powp_submit_wait_per_s\": %.1f}\n",
         n, nthreads, bad.load(), sweep.c_str(), n / batch_s, n / one_powp_s, n / one_multp_s, n / one_gpowp_s, n / async_s);
  return bad.load() == 0 ? 0 : 1;
}
