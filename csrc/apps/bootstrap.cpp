// TCP rendezvous (bootstrap.h).  Host-only code: built into cnn_dist and the
// CPU test binary test_comm (csrc/tests/test_comm.cpp).
#include "bootstrap.h"

#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <set>
#include <thread>
#include <vector>

#include "mcc/common.h"

namespace mcc {
namespace {

using Clock = std::chrono::steady_clock;
constexpr int32_t kHelloMagic = 0x4243434d;  // "MCCB"

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

int ms_left(Clock::time_point deadline) {
  const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
  return ms > 0 ? (int)std::min<long long>(ms, 1 << 30) : 0;
}

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, char* p, size_t n, Clock::time_point deadline) {
  while (n) {
    pollfd pf{fd, POLLIN, 0};
    const int left = ms_left(deadline);
    if (left <= 0 || ::poll(&pf, 1, left) <= 0) return false;
    const ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

struct Fd {
  int fd;
  explicit Fd(int f) : fd(f) {}
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

}  // namespace

BootstrapAddr bootstrap_addr_from_env() {
  BootstrapAddr a;
  if (const char* h = std::getenv("MASTER_ADDR"); h && *h) a.host = h;
  a.port = env_int("MCC_BOOTSTRAP_PORT", -1);
  if (a.port < 0) a.port = env_int("MASTER_PORT", 29500) + 1;
  a.timeout_s = env_int("MCC_BOOTSTRAP_TIMEOUT", 300);
  return a;
}

void serve_blob(const void* blob, size_t n, int clients, const BootstrapAddr& addr) {
  const auto deadline = Clock::now() + std::chrono::milliseconds((long long)(addr.timeout_s * 1000));
  Fd srv(::socket(AF_INET, SOCK_STREAM, 0));
  if (srv.fd < 0) throw Error("bootstrap: socket() failed");
  int one = 1;
  ::setsockopt(srv.fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = htonl(INADDR_ANY);
  sa.sin_port = htons((uint16_t)addr.port);
  if (::bind(srv.fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(srv.fd, clients + 4) != 0)
    throw Error("bootstrap: cannot listen on port " + std::to_string(addr.port));
  // A client first sends {kHelloMagic, rank}; only a well-formed hello from
  // a rank in [1, clients] that has not been served yet counts.  A stray
  // connection (no or a malformed hello) is dropped without the blob, and a
  // rank that reconnects (e.g. after its own receive timed out) gets the blob
  // again without taking another rank's slot.
  //
  // Connections are served concurrently: every accepted socket waits for its
  // hello in one poll() set with the listening socket (at most 2 s each), so
  // silent connectors (port scanners, leftovers of a dead job) cannot hold up
  // the real ranks queued behind them.
  struct Pending {
    int fd;
    Clock::time_point until;
    int32_t hello[2];
    size_t got;
  };
  std::vector<Pending> pend;
  auto drop = [&](size_t i) {
    ::close(pend[i].fd);
    pend[i] = pend.back();
    pend.pop_back();
  };
  std::set<int32_t> served;
  try {
    while ((int)served.size() < clients) {
      const int left = ms_left(deadline);
      if (left <= 0)
        throw Error("bootstrap: timed out waiting for ranks (" + std::to_string(served.size()) + " of " +
                    std::to_string(clients) + " served)");
      std::vector<pollfd> pf(1 + pend.size());
      pf[0] = pollfd{srv.fd, POLLIN, 0};
      int wait = std::min(left, 100);
      for (size_t i = 0; i < pend.size(); ++i) {
        pf[1 + i] = pollfd{pend[i].fd, POLLIN, 0};
        wait = std::max(0, std::min(wait, ms_left(pend[i].until)));
      }
      ::poll(pf.data(), pf.size(), wait);
      // hellos first (indices shift on drop: walk backwards)
      for (size_t i = pend.size(); i-- > 0;) {
        Pending& q = pend[i];
        if (pf[1 + i].revents & (POLLIN | POLLHUP | POLLERR)) {
          const ssize_t k = ::recv(q.fd, reinterpret_cast<char*>(q.hello) + q.got, sizeof(q.hello) - q.got, 0);
          if (k <= 0) { drop(i); continue; }
          q.got += (size_t)k;
          if (q.got == sizeof(q.hello)) {
            if (q.hello[0] == kHelloMagic && q.hello[1] >= 1 && q.hello[1] <= clients &&
                send_all(q.fd, static_cast<const char*>(blob), n))
              served.insert(q.hello[1]);
            drop(i);
            continue;
          }
        }
        if (Clock::now() >= q.until) drop(i);
      }
      if (pf[0].revents & POLLIN) {
        const int c = ::accept(srv.fd, nullptr, nullptr);
        if (c >= 0) pend.push_back(Pending{c, std::min(deadline, Clock::now() + std::chrono::seconds(2)), {0, -1}, 0});
      }
    }
  } catch (...) {
    for (auto& q : pend) ::close(q.fd);
    throw;
  }
  for (auto& q : pend) ::close(q.fd);
}

void fetch_blob(void* blob, size_t n, int rank, const BootstrapAddr& addr) {
  const auto deadline = Clock::now() + std::chrono::milliseconds((long long)(addr.timeout_s * 1000));
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(addr.host.c_str(), std::to_string(addr.port).c_str(), &hints, &res) != 0 || !res)
    throw Error("bootstrap: cannot resolve MASTER_ADDR " + addr.host);
  std::unique_ptr<addrinfo, void (*)(addrinfo*)> guard(res, ::freeaddrinfo);
  while (true) {
    {
      Fd fd(::socket(AF_INET, SOCK_STREAM, 0));
      const int32_t hello[2] = {kHelloMagic, (int32_t)rank};
      if (fd.fd >= 0 && ::connect(fd.fd, res->ai_addr, res->ai_addrlen) == 0 &&
          send_all(fd.fd, reinterpret_cast<const char*>(hello), sizeof(hello)) &&
          recv_all(fd.fd, static_cast<char*>(blob), n, deadline))
        return;
    }
    if (Clock::now() >= deadline) throw Error("bootstrap: timed out connecting to rank 0 at " + addr.host + ":" +
                                              std::to_string(addr.port));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

}  // namespace mcc
