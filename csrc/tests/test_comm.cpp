// CPU tests of the native multi-process rendezvous and host collectives
// (bootstrap.cpp, shm_group.cpp) with real forked processes:
//   * the TCP bootstrap serves one blob to 3 clients (world 4), and both of its
//     timeout branches (a client that never comes, a server that never comes)
//     end with an mcc::Error within the deadline;
//   * ShmGroup at world 4: sums bit-identical on every rank and equal to the
//     fixed-rank-order reference, max with NaN, broadcast, 300 back-to-back
//     collectives; a rank that stops participating makes the others' next
//     collective fail within the deadline; poison() fails peers immediately.
// Exit 0 and "comm ok" on success.
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "bootstrap.h"
#include "mcc/common.h"
#include "shm_group.h"

using namespace mcc;
using Clock = std::chrono::steady_clock;

#define CHECK(c)                                                                \
  do {                                                                          \
    if (!(c)) {                                                                 \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::_Exit(1);                                                            \
    }                                                                           \
  } while (0)

static int free_port() {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  sa.sin_port = 0;
  ::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa));
  socklen_t len = sizeof(sa);
  ::getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &len);
  ::close(fd);
  return ntohs(sa.sin_port);
}

// fork `n` children running fn(i); returns their exit codes
template <class F>
static std::vector<int> run_procs(int n, F fn) {
  std::vector<pid_t> pids;
  for (int i = 0; i < n; ++i) {
    pid_t p = ::fork();
    if (p == 0) {
      int rc = 1;
      try {
        rc = fn(i);
      } catch (const std::exception& e) {
        std::fprintf(stderr, "proc %d: %s\n", i, e.what());
        rc = 2;
      }
      std::_Exit(rc);
    }
    pids.push_back(p);
  }
  std::vector<int> rcs;
  for (pid_t p : pids) {
    int st = 0;
    ::waitpid(p, &st, 0);
    rcs.push_back(WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st));
  }
  return rcs;
}

static void test_bootstrap_world4() {
  BootstrapAddr a;
  a.port = free_port();
  a.timeout_s = 20;
  unsigned char blob[128];
  std::mt19937 g(7);
  for (auto& b : blob) b = (unsigned char)g();
  int fds[2];
  CHECK(::pipe(fds) == 0);
  auto rcs = run_procs(4, [&](int r) {
    unsigned char got[128] = {};
    if (r == 0) std::memcpy(got, blob, sizeof(got));
    bootstrap_blob(got, sizeof(got), r, 4, a);
    if (r > 0) CHECK(::write(fds[1], got, sizeof(got)) == (ssize_t)sizeof(got));
    return 0;
  });
  ::close(fds[1]);
  for (int rc : rcs) CHECK(rc == 0);
  for (int i = 0; i < 3; ++i) {
    unsigned char got[128];
    size_t k = 0;
    while (k < sizeof(got)) {
      ssize_t m = ::read(fds[0], got + k, sizeof(got) - k);
      CHECK(m > 0);
      k += (size_t)m;
    }
    CHECK(std::memcmp(got, blob, sizeof(blob)) == 0);
  }
  ::close(fds[0]);
  std::printf("bootstrap world 4 ok\n");
}

static void test_bootstrap_timeouts() {
  BootstrapAddr a;
  a.port = free_port();
  a.timeout_s = 1.0;
  // server expects 2 clients, only 1 comes
  auto rcs = run_procs(2, [&](int r) {
    char b[16] = "token";
    if (r == 0) {
      const auto t0 = Clock::now();
      try {
        serve_blob(b, sizeof(b), 2, a);
      } catch (const Error& e) {
        const double s = std::chrono::duration<double>(Clock::now() - t0).count();
        CHECK(std::strstr(e.what(), "timed out waiting for ranks"));
        CHECK(s >= 0.9 && s < 5.0);
        return 0;
      }
      return 3;  // must not succeed
    }
    fetch_blob(b, sizeof(b), 1, a);
    return 0;
  });
  CHECK(rcs[0] == 0 && rcs[1] == 0);
  // client with no server
  BootstrapAddr c;
  c.port = free_port();
  c.timeout_s = 0.5;
  const auto t0 = Clock::now();
  bool threw = false;
  try {
    char b[16];
    fetch_blob(b, sizeof(b), 1, c);
  } catch (const Error& e) {
    threw = std::strstr(e.what(), "timed out connecting") != nullptr;
  }
  const double s = std::chrono::duration<double>(Clock::now() - t0).count();
  CHECK(threw && s < 5.0);
  std::printf("bootstrap timeouts ok\n");
}

// Stray connectors (connect + close, a garbage hello, an out-of-range rank)
// do not take the slots of real ranks: world 3 still serves ranks 1 and 2.
static void test_bootstrap_stray_connections() {
  BootstrapAddr a;
  a.port = free_port();
  a.timeout_s = 20;
  auto rcs = run_procs(4, [&](int r) {
    char b[16] = {};
    if (r == 0) {
      std::strcpy(b, "token");
      serve_blob(b, sizeof(b), 2, a);
      return 0;
    }
    if (r == 3) {  // the stray
      for (int k = 0; k < 3; ++k) {
        for (int t = 0; t < 400; ++t) {
          int fd = ::socket(AF_INET, SOCK_STREAM, 0);
          sockaddr_in sa{};
          sa.sin_family = AF_INET;
          sa.sin_port = htons((uint16_t)a.port);
          sa.sin_addr.s_addr = htonl(0x7f000001);
          if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) {
            const int32_t bad[2] = {k == 1 ? 0x4243434d : 1234, k == 1 ? 99 : 1};
            if (k > 0) (void)!::write(fd, bad, sizeof(bad));
            char junk[16];
            const ssize_t got = ::read(fd, junk, sizeof(junk));  // the server must not send the blob
            ::close(fd);
            if (got > 0) return 6;
            break;
          }
          ::close(fd);
          ::usleep(5000);
        }
      }
      return 0;
    }
    ::usleep(300000);  // the real ranks arrive after the strays
    fetch_blob(b, sizeof(b), r, a);
    return std::strcmp(b, "token") == 0 ? 0 : 4;
  });
  for (int rc : rcs) CHECK(rc == 0);
  std::printf("bootstrap stray connections ok\n");
}

// Silent connectors (connect, send nothing, hold the socket) must not stall
// the real ranks: hellos are awaited concurrently, each for at most 2 s.
static void test_bootstrap_silent_connectors() {
  BootstrapAddr a;
  a.port = free_port();
  a.timeout_s = 20;
  constexpr int kSilent = 5;
  auto rcs = run_procs(3 + kSilent, [&](int r) {
    char b[16] = {};
    if (r == 0) {
      std::strcpy(b, "token");
      serve_blob(b, sizeof(b), 2, a);
      return 0;
    }
    if (r >= 3) {  // a silent connector: holds its connection for 6 s
      for (int t = 0; t < 400; ++t) {
        int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in sa{};
        sa.sin_family = AF_INET;
        sa.sin_port = htons((uint16_t)a.port);
        sa.sin_addr.s_addr = htonl(0x7f000001);
        if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) {
          ::usleep(6000000);
          ::close(fd);
          return 0;
        }
        ::close(fd);
        ::usleep(5000);
      }
      return 0;
    }
    ::usleep(300000);  // the real ranks arrive after the silent ones
    const auto t0 = Clock::now();
    fetch_blob(b, sizeof(b), r, a);
    const double s = std::chrono::duration<double>(Clock::now() - t0).count();
    if (s > 3.0) return 7;  // served behind the silent connectors
    return std::strcmp(b, "token") == 0 ? 0 : 4;
  });
  for (int rc : rcs) CHECK(rc == 0);
  std::printf("bootstrap silent connectors ok\n");
}

static uint64_t token() {
  std::random_device rd;
  return ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)::getpid();
}

static void test_shm_collectives() {
  const int W = 4;
  const size_t n = 3000;
  const uint64_t tok = token();
  // per-rank inputs: values of very different magnitude, so the summation
  // order matters in fp32 and a wrong order shows up as a bit difference
  auto input = [&](int r, int it, size_t i) {
    const float big = (i % 3 == 0) ? 1e7f : 1.f;
    return (float)((r + 1) * 0.1f + it * 1e-3f) * big * ((i & 1) ? -1.f : 1.f) + (float)i * 1e-4f;
  };
  int fds[2];
  CHECK(::pipe(fds) == 0);
  auto rcs = run_procs(W, [&](int r) {
    ShmGroup g(tok, r, W, n * sizeof(float), 20.0);
    std::vector<float> v(n);
    double h = 0;
    for (int it = 0; it < 100; ++it) {
      for (size_t i = 0; i < n; ++i) v[i] = input(r, it, i);
      CHECK(g.sum_f32(v.data(), v.data(), n));
      for (size_t i = 0; i < n; ++i) {
        float ref = input(0, it, i);
        for (int q = 1; q < W; ++q) ref += input(q, it, i);
        CHECK(std::memcmp(&ref, &v[i], 4) == 0);
        h = h * 1.0000001 + v[i];
      }
      double m[2] = {(double)r, r == 2 && it == 7 ? NAN : -1.0 * r};
      CHECK(g.max_f64(m, m, 2));
      CHECK(m[0] == W - 1);
      CHECK(it == 7 ? std::isnan(m[1]) : m[1] == 0.0);
      int payload[4] = {r, r, r, r};
      CHECK(g.broadcast(payload, payload, sizeof(payload), it % W));
      CHECK(payload[0] == it % W && payload[3] == it % W);
    }
    CHECK(g.collectives() == 1 + 300);  // attach barrier + 3 per iteration
    bool threw = false;
    try {
      std::vector<float> big(n + 64);
      g.sum_f32(big.data(), big.data(), n + 64);
    } catch (const Error&) {
      threw = true;
    }
    CHECK(threw);
    CHECK(::write(fds[1], &h, sizeof(h)) == (ssize_t)sizeof(h));
    return 0;
  });
  ::close(fds[1]);
  for (int rc : rcs) CHECK(rc == 0);
  double h0 = 0;
  for (int i = 0; i < W; ++i) {
    double h;
    CHECK(::read(fds[0], &h, sizeof(h)) == (ssize_t)sizeof(h));
    if (i == 0) h0 = h;
    CHECK(std::memcmp(&h, &h0, sizeof(h)) == 0);  // bit-identical on every rank
  }
  ::close(fds[0]);
  char path[96];
  std::snprintf(path, sizeof(path), "/dev/shm/mcc_%016llx", (unsigned long long)tok);
  CHECK(::access(path, F_OK) != 0);  // name unlinked after attach
  std::printf("shm collectives world 4 ok\n");
}

static void test_shm_dead_peer_and_poison() {
  const uint64_t tok = token();
  auto rcs = run_procs(3, [&](int r) {
    ShmGroup g(tok, r, 3, 1024, 1.0);
    float x = 1.f;
    CHECK(g.sum_f32(&x, &x, 1) && x == 3.f);
    if (r == 2) return 0;  // stops participating
    const auto t0 = Clock::now();
    CHECK(!g.sum_f32(&x, &x, 1));
    const double s = std::chrono::duration<double>(Clock::now() - t0).count();
    CHECK(s >= 0.9 && s < 5.0);
    return 0;
  });
  for (int rc : rcs) CHECK(rc == 0);
  const uint64_t tok2 = token();
  rcs = run_procs(2, [&](int r) {
    ShmGroup g(tok2, r, 2, 1024, 30.0);
    if (r == 1) {
      g.poison();
      return 0;
    }
    const auto t0 = Clock::now();
    CHECK(!g.barrier());
    CHECK(std::chrono::duration<double>(Clock::now() - t0).count() < 5.0);
    return 0;
  });
  for (int rc : rcs) CHECK(rc == 0);
  // a rank that never attaches: the others' constructor times out
  const uint64_t tok3 = token();
  rcs = run_procs(1, [&](int) {
    try {
      ShmGroup g(tok3, 0, 2, 1024, 0.5);
    } catch (const Error& e) {
      return std::strstr(e.what(), "attach") ? 0 : 4;
    }
    return 3;
  });
  CHECK(rcs[0] == 0);
  std::printf("shm dead peer / poison / attach timeout ok\n");
}

int main() {
  test_bootstrap_world4();
  test_bootstrap_timeouts();
  test_bootstrap_stray_connections();
  test_bootstrap_silent_connectors();
  test_shm_collectives();
  test_shm_dead_peer_and_poison();
  std::printf("comm ok\n");
  return 0;
}
