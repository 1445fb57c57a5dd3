// `cnn_dist`: data-parallel multi-GPU trainer, one process per GPU, gradient
// sync over RCCL (xGMI).  Replaces cnnmpi.c / CUDAMPI.c's per-sample, per-layer
// blocking MPI_Allreduce of the wrong buffer (cnnmpi.c:487-498, defects D4-D7)
// with one mean-gradient all-reduce per step, bucketed and overlapped with
// backward (see trainer.cpp), and an initial weight broadcast from rank 0.
//
// Launch (any of):
//   torchrun --no-python --nproc-per-node N --master-addr 127.0.0.1 build/bin/cnn_dist <4 IDX> [flags]
//   python -m mpi_cuda_cnn_amd.launch -n N build/bin/cnn_dist <4 IDX> [flags]
//   mpiexec -n N build/bin/cnn_dist ...            (PMI_RANK/PMI_SIZE or OMPI_* env)
// Rendezvous: rank 0 creates the RCCL unique id and serves it over TCP on
// MASTER_ADDR:(MCC_BOOTSTRAP_PORT or MASTER_PORT+1); every wait is bounded
// (MCC_BOOTSTRAP_TIMEOUT seconds, default 300) so a dead rank cannot hang
// the others forever (defect D9).  After the rendezvous every host-side wait
// goes through the collective watchdog (watchdog.h: ncclCommGetAsyncError +
// deadline MCC_COMM_TIMEOUT); on expiry the rank aborts its communicator and
// exits 111.
//
// The RCCL communicator is created at every world size, 1 included, so a
// single-GPU run executes the same broadcast, bucketed all-reduce on the comm
// stream and graph-captured collectives as an 8-GPU one.  MCC_AB=local_comm
// (world 1 only) swaps in the collective-free LocalComm for A/B runs.
#include "mcc/ab.h"
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "cli.h"
#include "trainer.h"
#include "watchdog.h"

namespace mcc {
namespace {

#define NCCLCHK(expr)                                                                            \
  do {                                                                                           \
    ncclResult_t _r = (expr);                                                                    \
    if (_r != ncclSuccess) throw Error(std::string("RCCL: ") + ncclGetErrorString(_r) + " @ " + #expr); \
  } while (0)

int env_int(const char* const* names, int dflt) {
  for (int i = 0; names[i]; ++i)
    if (const char* v = std::getenv(names[i])) return std::atoi(v);
  return dflt;
}

bool send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, void* buf, size_t n, int timeout_ms) {
  char* p = static_cast<char*>(buf);
  while (n) {
    pollfd pf{fd, POLLIN, 0};
    if (::poll(&pf, 1, timeout_ms) <= 0) return false;
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

void bootstrap_id(ncclUniqueId& id, int rank, int world) {
  const char* addr = std::getenv("MASTER_ADDR");
  std::string host = addr ? addr : "127.0.0.1";
  int port = env_int((const char*[]){"MCC_BOOTSTRAP_PORT", nullptr}, -1);
  if (port < 0) port = env_int((const char*[]){"MASTER_PORT", nullptr}, 29500) + 1;
  const int timeout_s = env_int((const char*[]){"MCC_BOOTSTRAP_TIMEOUT", nullptr}, 300);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  if (rank == 0) {
    NCCLCHK(ncclGetUniqueId(&id));
    if (world == 1) return;  // nobody to serve
    int srv = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    sa.sin_port = htons((uint16_t)port);
    if (::bind(srv, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(srv, world) != 0) {
      ::close(srv);
      throw Error("bootstrap: cannot listen on port " + std::to_string(port));
    }
    for (int served = 1; served < world;) {
      pollfd pf{srv, POLLIN, 0};
      const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
      if (left <= 0 || ::poll(&pf, 1, left) <= 0) { ::close(srv); throw Error("bootstrap: timed out waiting for ranks"); }
      int c = ::accept(srv, nullptr, nullptr);
      if (c < 0) continue;
      const bool ok = send_all(c, &id, sizeof(id));
      ::close(c);
      if (ok) ++served;
    }
    ::close(srv);
    return;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw Error("bootstrap: cannot resolve MASTER_ADDR " + host);
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      const bool ok = recv_all(fd, &id, sizeof(id), 60000);
      ::close(fd);
      if (ok) break;
    } else {
      ::close(fd);
    }
    if (std::chrono::steady_clock::now() > deadline) {
      ::freeaddrinfo(res);
      throw Error("bootstrap: timed out connecting to rank 0");
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  ::freeaddrinfo(res);
}

struct RcclComm : Comm {
  int rank_ = 0, world_ = 1, local_ = 0;
  ncclComm_t comm_ = nullptr;
  float* dummy_ = nullptr;
  hipStream_t bs_ = nullptr;  // barrier stream
  hipEvent_t bev_ = nullptr;
  double timeout_s_ = comm_timeout_s();

  RcclComm(int rank, int world, int local) : rank_(rank), world_(world), local_(local) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) throw Error("no GPU");
    if (hipSetDevice(local_ % ndev) != hipSuccess) throw Error("hipSetDevice failed");
    ncclUniqueId id;
    bootstrap_id(id, rank_, world_);
    NCCLCHK(ncclCommInitRank(&comm_, world_, id, rank_));
    if (hipMalloc(&dummy_, 64) != hipSuccess) throw Error("hipMalloc failed");
    if (hipStreamCreateWithFlags(&bs_, hipStreamNonBlocking) != hipSuccess) throw Error("hipStreamCreate failed");
    if (hipEventCreateWithFlags(&bev_, hipEventDisableTiming) != hipSuccess) throw Error("hipEventCreate failed");
  }
  ~RcclComm() override {
    if (bev_) (void)hipEventDestroy(bev_);
    if (bs_) (void)hipStreamDestroy(bs_);
    if (dummy_) (void)hipFree(dummy_);
    if (comm_) ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  int local_rank() const override { return local_; }
  const char* name() const override { return "rccl"; }
  bool collective() const override { return true; }
  void allreduce_sum_f32(float* buf, int64_t n, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, comm_, s));
  }
  void allreduce_max_f64(double* buf, int64_t n, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(buf, buf, (size_t)n, ncclFloat64, ncclMax, comm_, s));
  }
  void broadcast_f32(float* buf, int64_t n, int root, hipStream_t s) override {
    NCCLCHK(ncclBroadcast(buf, buf, (size_t)n, ncclFloat32, root, comm_, s));
  }
  // Collective watchdog: poll the event and the communicator's async error
  // state until the deadline (watchdog.h).
  void wait(hipEvent_t ev) override { wait_for(ev, timeout_s_, "MCC_COMM_TIMEOUT"); }
  void wait_long(hipEvent_t ev) override { wait_for(ev, test_phase_timeout_s(), "MCC_TEST_TIMEOUT"); }
  // On a timeout or an asynchronous error the communicator is aborted here,
  // before the exception unwinds the caller's device buffers (collective_fail).
  void wait_for(hipEvent_t ev, double timeout_s, const char* knob) {
    ncclResult_t async = ncclSuccess;
    hipError_t herr = hipSuccess;
    const WaitStatus st = bounded_wait(
        [&] {
          herr = hipEventQuery(ev);
          return herr != hipErrorNotReady;
        },
        [&] {
          if (herr != hipSuccess && herr != hipErrorNotReady) return 1;
          if (comm_ && ncclCommGetAsyncError(comm_, &async) == ncclSuccess && async != ncclSuccess &&
              async != ncclInProgress)
            return 2;
          return 0;
        },
        timeout_s);
    if (st == WaitStatus::Done && herr == hipSuccess) return;
    auto abort_now = [this](const char* why) { abort(why); };
    if (st == WaitStatus::Timeout)
      collective_fail<Error>(abort_now, "collective watchdog: no progress within " + std::to_string(timeout_s) + " s (" +
                                            knob + "); a peer rank is gone or hung");
    if (herr != hipSuccess && herr != hipErrorNotReady)
      collective_fail<Error>(abort_now, std::string("HIP: ") + hipGetErrorString(herr));
    collective_fail<Error>(abort_now, std::string("RCCL async error: ") + ncclGetErrorString(async));
  }
  void barrier() override {
    NCCLCHK(ncclAllReduce(dummy_, dummy_, 1, ncclFloat32, ncclSum, comm_, bs_));
    if (hipEventRecord(bev_, bs_) != hipSuccess) throw Error("hipEventRecord failed");
    wait(bev_);
  }
  void abort(const char* why) override {
    std::fprintf(stderr, "rank %d aborting: %s\n", rank_, why);
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
};

}  // namespace
}  // namespace mcc

int main(int argc, char** argv) {
  mcc::CliArgs a;
  if (mcc::parse_cli(argc, argv, a) != 0) return 100;
  const int rank = mcc::env_int((const char*[]){"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", nullptr}, 0);
  const int world = mcc::env_int((const char*[]){"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", nullptr}, 1);
  const int local =
      mcc::env_int((const char*[]){"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", nullptr}, rank);
  std::unique_ptr<mcc::Comm> comm;
  try {
    if (world == 1 && mcc::ab_flag("local_comm")) comm.reset(new mcc::LocalComm());
    else comm.reset(new mcc::RcclComm(rank, world, local));
  } catch (const mcc::Error& e) {
    std::fprintf(stderr, "rank %d: %s\n", rank, e.what());
    return 111;
  }
  int rc = 111;
  try {
    rc = mcc::run_gpu_training(a, *comm, "cnn_dist");
  } catch (const mcc::Error& e) {
    std::fprintf(stderr, "rank %d error: %s\n", rank, e.what());
    comm->abort(e.what());
    rc = 111;
  }
  if (rc != 0) comm->abort("non-zero exit");
  return rc;
}
