// CPU unit test of the collective watchdog policy (csrc/apps/watchdog.h):
// completion, asynchronous-error and deadline branches.  Run by
// tests/test_watchdog.py; exits non-zero on the first failed check.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "watchdog.h"

using namespace mcc;

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                     \
    }                                                               \
  } while (0)

int main() {
  using clock = std::chrono::steady_clock;
  // completes after a few polls
  int polls = 0;
  CHECK(bounded_wait([&] { return ++polls >= 5; }, [] { return 0; }, 10.0) == WaitStatus::Done);
  CHECK(polls == 5);
  // the communicator reports an async error: returned at once, not at the deadline
  auto t0 = clock::now();
  int checks = 0;
  CHECK(bounded_wait([] { return false; }, [&] { return ++checks >= 3 ? 7 : 0; }, 10.0) == WaitStatus::Error);
  CHECK(std::chrono::duration<double>(clock::now() - t0).count() < 1.0);
  // never completes, no error: times out at the deadline (not before, not much after)
  t0 = clock::now();
  CHECK(bounded_wait([] { return false; }, [] { return 0; }, 0.3) == WaitStatus::Timeout);
  const double el = std::chrono::duration<double>(clock::now() - t0).count();
  CHECK(el >= 0.3 && el < 1.5);
  // completion wins over a simultaneous error
  CHECK(bounded_wait([] { return true; }, [] { return 1; }, 1.0) == WaitStatus::Done);
  // MCC_COMM_TIMEOUT parsing
  setenv("MCC_COMM_TIMEOUT", "12.5", 1);
  CHECK(comm_timeout_s() == 12.5);
  setenv("MCC_COMM_TIMEOUT", "-3", 1);
  CHECK(comm_timeout_s() == 300.0);
  unsetenv("MCC_COMM_TIMEOUT");
  CHECK(comm_timeout_s() == 300.0);
  // MCC_TEST_TIMEOUT: default 3600, never below the collective deadline
  CHECK(test_phase_timeout_s() == 3600.0);
  setenv("MCC_COMM_TIMEOUT", "5000", 1);
  CHECK(test_phase_timeout_s() == 5000.0);
  unsetenv("MCC_COMM_TIMEOUT");
  setenv("MCC_TEST_TIMEOUT", "900", 1);
  CHECK(test_phase_timeout_s() == 900.0);
  unsetenv("MCC_TEST_TIMEOUT");
  // failure path: the communicator abort runs BEFORE the caller's device
  // buffers are released (their destructors run while the exception unwinds)
  {
    std::string order;
    struct DeviceBuffer {  // stands for a DevBuf / arena whose hipFree syncs the device
      std::string* o;
      ~DeviceBuffer() { *o += "free;"; }
    };
    bool thrown = false;
    try {
      DeviceBuffer buf{&order};
      (void)buf;
      collective_fail<std::runtime_error>([&](const char*) { order += "abort;"; }, "peer gone");
    } catch (const std::runtime_error& e) {
      thrown = std::string(e.what()) == "peer gone";
    }
    CHECK(thrown);
    CHECK(order == "abort;free;");
  }
  std::printf("watchdog ok\n");
  return 0;
}
