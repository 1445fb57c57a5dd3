// Bounded waits for the data-parallel drivers (collective watchdog).
//
// The reference's MPI program returns 111 from one rank without
// MPI_Abort/MPI_Finalize (cnnmpi.c:443-453,509-519, defect D9): the other
// ranks then block in MPI_Allreduce forever.  On the RCCL path the same
// failure is a rank that dies (or faults) with collectives in flight: the
// survivors' RCCL kernels spin on xGMI and a plain hipStreamSynchronize never
// returns.  Every host-side wait of cnn_dist therefore goes through
// bounded_wait(): it polls the completion predicate and the communicator's
// asynchronous error state, sleeping with a short back-off, and gives up at a
// deadline (MCC_COMM_TIMEOUT seconds, default 300) so the caller can
// ncclCommAbort and exit 111.  Header-only and GPU-free so the policy is unit
// tested on the CPU (build/bin/test_watchdog).
#pragma once

#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>

namespace mcc {

enum class WaitStatus { Done, Error, Timeout };

// done(): true once the awaited work has completed.
// error(): non-zero once the communicator reports an asynchronous error.
template <class Done, class ErrorFn>
WaitStatus bounded_wait(Done&& done, ErrorFn&& error, double timeout_s) {
  using clock = std::chrono::steady_clock;
  const auto deadline = clock::now() + std::chrono::duration<double>(timeout_s);
  int sleep_us = 20;
  while (true) {
    if (done()) return WaitStatus::Done;
    if (error() != 0) return WaitStatus::Error;
    if (clock::now() >= deadline) return WaitStatus::Timeout;
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    if (sleep_us < 1000) sleep_us *= 2;
  }
}

// Deadline of one collective wait: MCC_COMM_TIMEOUT (seconds), default 300.
inline double comm_timeout_s() {
  const char* v = std::getenv("MCC_COMM_TIMEOUT");
  const double t = v && *v ? std::atof(v) : 300.0;
  return t > 0 ? t : 300.0;
}

// Deadline of the post-training agreement that waits for rank 0's test
// phase (evaluation + weight save can outlast a collective deadline):
// MCC_TEST_TIMEOUT seconds, default 3600, never below the collective one.
inline double test_phase_timeout_s() {
  const char* v = std::getenv("MCC_TEST_TIMEOUT");
  const double t = v && *v ? std::atof(v) : 3600.0;
  const double c = comm_timeout_s();
  return t > c ? t : c;
}

// Failure path of a bounded wait: abort the communicator FIRST (so the RCCL
// kernels spinning on a dead peer are torn down), then throw.  Throwing first
// would run the destructors of the caller's device buffers while those
// kernels still spin; hipFree synchronises the device, so the rank would hang
// instead of exiting 111.  `Err` is the exception type thrown.
template <class Err, class AbortFn>
[[noreturn]] void collective_fail(AbortFn&& abort_now, const std::string& msg) {
  abort_now(msg.c_str());
  throw Err(msg);
}

}  // namespace mcc
