// eg_comm_wait.hpp — the deadline-bounded wait behind every RCCL collective of libeg_hip.so.
//
// A collective on a non-blocking communicator returns once it is ENQUEUED; the wait for the peers
// happens on the GPU.  A bare hipStreamSynchronize after it would hang forever on a peer that died
// after the enqueue, so eg_capi_comm.inc records a hipEvent behind the collective and
// waits here instead: poll the event, and between polls ask RCCL whether the communicator failed
// (ncclCommGetAsyncError), until the event completes or the deadline (EG_COMM_TIMEOUT_S) passes.
// The caller aborts the communicator (ncclCommAbort) on anything but kDone.
//
// Header-only and free of HIP / RCCL types, so the CPU test suite drives the same code with fake
// completions (tests/cpp/comm_wait_test.cpp: a completion that never arrives returns kTimedOut at the
// deadline; an async error returns kCommError at once).
#pragma once
#include <chrono>
#include <thread>

namespace egcomm {

enum class Wait { kDone, kTimedOut, kCommError, kStreamError };

// done():        > 0 complete, 0 not yet, < 0 the stream reported an error
// async_error(): 0 while the communicator is healthy (or still in progress), else its error code
// The first ~2,000 polls only yield (a healthy collective completes in tens of microseconds); after
// that the poll sleeps 50 us, so a long wait costs no host core.
template <class Done, class AsyncErr>
Wait wait_with_deadline(Done done, AsyncErr async_error, double timeout_s, int* err_code = nullptr) {
  using clock = std::chrono::steady_clock;
  const auto end = clock::now() + std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(timeout_s));
  for (unsigned it = 0;; ++it) {
    const int d = done();
    if (d > 0) return Wait::kDone;
    if (d < 0) return Wait::kStreamError;
    const int e = async_error();
    if (e != 0) {
      if (err_code) *err_code = e;
      return Wait::kCommError;
    }
    if (clock::now() > end) return Wait::kTimedOut;
    if (it < 2000)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

inline const char* wait_name(Wait w) {
  switch (w) {
    case Wait::kDone: return "done";
    case Wait::kTimedOut: return "timed out";
    case Wait::kCommError: return "communicator error";
    case Wait::kStreamError: return "stream error";
  }
  return "?";
}

}  // namespace egcomm
