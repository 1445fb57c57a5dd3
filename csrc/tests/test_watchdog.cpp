// CPU unit test of the collective watchdog policy (csrc/apps/watchdog.h):
// completion, asynchronous-error and deadline branches.  Run by
// tests/test_watchdog.py; exits non-zero on the first failed check.
#include <chrono>
#include <cstdio>
#include <cstdlib>

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
  std::printf("watchdog ok\n");
  return 0;
}
