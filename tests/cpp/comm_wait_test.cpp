// CPU test of the deadline-bounded collective wait (electionguard-remote_amd/csrc/eg_comm_wait.hpp),
// the code libeg_hip.so runs after every RCCL collective in place of a bare hipStreamSynchronize.
// Fake communicators stand in for RCCL: their "completion" is a callable, so the cases a real
// multi-GPU run can only show by accident -- a peer that never arrives, a communicator that fails
// mid-collective -- run here on any host.  Prints one JSON line; exit 0 when every case holds.
//
//   g++ -std=c++17 -O2 -pthread -I electionguard-remote_amd/csrc tests/cpp/comm_wait_test.cpp
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "eg_comm_wait.hpp"

using egcomm::Wait;
using clk = std::chrono::steady_clock;

static double secs_since(clk::time_point t) { return std::chrono::duration<double>(clk::now() - t).count(); }

int main(int argc, char** argv) {
  const double deadline = argc > 1 ? atof(argv[1]) : 0.5;
  int failures = 0;
  printf("{");
  // 1. the completion never arrives (a peer died after the enqueue): kTimedOut at the deadline
  {
    const auto t = clk::now();
    long polls = 0;
    const Wait w = egcomm::wait_with_deadline([&] { ++polls; return 0; }, [] { return 0; }, deadline);
    const double s = secs_since(t);
    const bool ok = w == Wait::kTimedOut && s >= deadline && s < deadline + 2.5;  // (slack for a loaded host)
    failures += !ok;
    printf("\"never_completes\": {\"result\": \"%s\", \"seconds\": %.3f, \"deadline\": %.3f, \"polls\": %ld, \"ok\": %s}",
           egcomm::wait_name(w), s, deadline, polls, ok ? "true" : "false");
  }
  // 2. the communicator reports an asynchronous error while the collective is pending: kCommError at once
  {
    const auto t = clk::now();
    int polls = 0, code = 0;
    const Wait w = egcomm::wait_with_deadline([] { return 0; }, [&] { return ++polls >= 10 ? 6 : 0; }, 60.0, &code);
    const double s = secs_since(t);
    const bool ok = w == Wait::kCommError && code == 6 && polls == 10 && s < 3.0;
    failures += !ok;
    printf(", \"async_error\": {\"result\": \"%s\", \"code\": %d, \"polls\": %d, \"seconds\": %.4f, \"ok\": %s}",
           egcomm::wait_name(w), code, polls, s, ok ? "true" : "false");
  }
  // 3. the completion arrives from another thread after 20 ms (a healthy collective): kDone
  {
    std::atomic<bool> flag{false};
    std::thread th([&] {
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      flag = true;
    });
    const auto t = clk::now();
    const Wait w = egcomm::wait_with_deadline([&] { return flag.load() ? 1 : 0; }, [] { return 0; }, 60.0);
    const double s = secs_since(t);
    th.join();
    const bool ok = w == Wait::kDone && s >= 0.019 && s < 3.0;
    failures += !ok;
    printf(", \"completes\": {\"result\": \"%s\", \"seconds\": %.4f, \"ok\": %s}", egcomm::wait_name(w), s,
           ok ? "true" : "false");
  }
  // 4. the stream reports an error (hipEventQuery other than success / not ready): kStreamError
  {
    const Wait w = egcomm::wait_with_deadline([] { return -1; }, [] { return 0; }, 60.0);
    const bool ok = w == Wait::kStreamError;
    failures += !ok;
    printf(", \"stream_error\": {\"result\": \"%s\", \"ok\": %s}", egcomm::wait_name(w), ok ? "true" : "false");
  }
  // 5. completion wins over a late error: a collective that completed is done even if the deadline is 0
  {
    const Wait w = egcomm::wait_with_deadline([] { return 1; }, [] { return 6; }, 0.0);
    const bool ok = w == Wait::kDone;
    failures += !ok;
    printf(", \"done_first\": {\"result\": \"%s\", \"ok\": %s}", egcomm::wait_name(w), ok ? "true" : "false");
  }
  printf(", \"failures\": %d}\n", failures);
  return failures ? 1 : 0;
}
