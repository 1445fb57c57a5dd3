// HostComm (host_comm.h): Comm over host shared memory for several ranks on
// one GPU.  Each collective is three stream-ordered operations on the stream
// it is issued on -- a device->host copy into a pinned staging buffer, a host
// function (hipLaunchHostFunc) that runs the ShmGroup collective, a
// host->device copy of the result -- so it is ordered exactly like an RCCL
// call and is captured into the step's hipGraph the same way (memcpy + host
// nodes instead of a collective kernel).  Messages larger than the staging
// slot are chunked.  Collectives must be issued in one global order on every
// rank (the trainer's event fork/join guarantees it), which is also what
// RCCL requires.
#include "host_comm.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <deque>
#include <random>

#include "bootstrap.h"
#include "shm_group.h"
#include "watchdog.h"

namespace mcc {
namespace {

#define HCHK(expr)                                                                              \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess) throw Error(std::string("HIP: ") + hipGetErrorString(_e) + " @ " + #expr); \
  } while (0)

constexpr size_t kSlotBytes = 4 << 20;  // per-rank staging slot (/dev/shm use: world x 4 MiB)

struct HostComm : Comm {
  enum Kind { kSum, kMax, kBcast };
  struct Op {
    HostComm* c;
    Kind kind;
    size_t bytes;
    int root;
    std::atomic<bool> done{false};  // eager ops: the host function has run (slot reusable)
    Op(HostComm* c_, Kind k, size_t b, int r) : c(c_), kind(k), bytes(b), root(r) {}
  };

  int rank_, world_, local_;
  std::unique_ptr<ShmGroup> g_;
  char* in_ = nullptr;   // pinned staging: device -> host
  char* out_ = nullptr;  // pinned staging: host -> device
  // Host-node arguments need stable addresses.  Ops recorded into a graph
  // are kept for the communicator's lifetime (every replay calls the same
  // host nodes again); eager ops are released once their host function has
  // run, so an eager run (--no-graph, --profile) does not grow this per step.
  std::deque<Op> graph_ops_;
  std::deque<Op> eager_ops_;
  std::atomic<bool> failed_{false};
  double timeout_s_ = comm_timeout_s();

  HostComm(int rank, int world, int local) : rank_(rank), world_(world), local_(local) {
    int ndev = 0;
    HCHK(hipGetDeviceCount(&ndev));
    if (ndev < 1) throw Error("no GPU");
    HCHK(hipSetDevice(local_ % ndev));
    // rank 0 draws the segment token and serves it over the TCP bootstrap
    uint64_t token = 0;
    if (rank_ == 0) {
      std::random_device rd;
      token = ((uint64_t)rd() << 32) ^ rd() ^ ((uint64_t)::getpid() << 16);
    }
    bootstrap_blob(&token, sizeof(token), rank_, world_, bootstrap_addr_from_env());
    // The host functions may wait as long as the test-phase agreement; the
    // host-side watchdog (wait) bounds every step and poisons the group.
    g_ = std::make_unique<ShmGroup>(token, rank_, world_, kSlotBytes, test_phase_timeout_s());
    HCHK(hipHostMalloc(reinterpret_cast<void**>(&in_), kSlotBytes, hipHostMallocDefault));
    HCHK(hipHostMalloc(reinterpret_cast<void**>(&out_), kSlotBytes, hipHostMallocDefault));
  }
  ~HostComm() override {
    if (in_) (void)hipHostFree(in_);
    if (out_) (void)hipHostFree(out_);
  }
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  int local_rank() const override { return local_; }
  const char* name() const override { return "host"; }
  bool collective() const override { return true; }

  static void run_op(void* p) {
    Op& o = *static_cast<Op*>(p);
    HostComm& c = *o.c;
    if (c.failed_.load()) return;
    bool ok = false;
    switch (o.kind) {
      case kSum:
        ok = c.g_->sum_f32(reinterpret_cast<const float*>(c.in_), reinterpret_cast<float*>(c.out_), o.bytes / 4);
        break;
      case kMax:
        ok = c.g_->max_f64(reinterpret_cast<const double*>(c.in_), reinterpret_cast<double*>(c.out_), o.bytes / 8);
        break;
      case kBcast:
        ok = c.g_->broadcast(c.in_, c.out_, o.bytes, o.root);
        break;
    }
    if (!ok) c.failed_.store(true);
    o.done.store(true, std::memory_order_release);
  }

  void issue(void* dev, size_t bytes, size_t elem, Kind kind, int root, hipStream_t s) {
    const size_t chunk = kSlotBytes / elem * elem;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HCHK(hipStreamIsCapturing(s, &cap));
    std::deque<Op>& ops = cap == hipStreamCaptureStatusNone ? eager_ops_ : graph_ops_;
    // host functions run in issue order (one stream order per collective
    // sequence), so the finished eager ops are a prefix of the deque
    while (!eager_ops_.empty() && eager_ops_.front().done.load(std::memory_order_acquire)) eager_ops_.pop_front();
    for (size_t off = 0; off < bytes; off += chunk) {
      const size_t len = std::min(chunk, bytes - off);
      char* d = static_cast<char*>(dev) + off;
      HCHK(hipMemcpyAsync(in_, d, len, hipMemcpyDeviceToHost, s));
      ops.emplace_back(this, kind, len, root);
      HCHK(hipLaunchHostFunc(s, &HostComm::run_op, &ops.back()));
      HCHK(hipMemcpyAsync(d, out_, len, hipMemcpyHostToDevice, s));
    }
  }
  void allreduce_sum_f32(float* buf, int64_t n, hipStream_t s) override { issue(buf, (size_t)n * 4, 4, kSum, 0, s); }
  void allreduce_max_f64(double* buf, int64_t n, hipStream_t s) override { issue(buf, (size_t)n * 8, 8, kMax, 0, s); }
  void broadcast_f32(float* buf, int64_t n, int root, hipStream_t s) override {
    issue(buf, (size_t)n * 4, 4, kBcast, root, s);
  }

  void wait(hipEvent_t ev) override { wait_for(ev, timeout_s_, "MCC_COMM_TIMEOUT"); }
  void wait_long(hipEvent_t ev) override { wait_for(ev, test_phase_timeout_s(), "MCC_TEST_TIMEOUT"); }
  void wait_for(hipEvent_t ev, double timeout_s, const char* knob) {
    hipError_t herr = hipSuccess;
    const WaitStatus st = bounded_wait(
        [&] {
          herr = hipEventQuery(ev);
          return herr != hipErrorNotReady;
        },
        [&] { return (herr != hipSuccess && herr != hipErrorNotReady) || failed_.load() || g_->poisoned() ? 1 : 0; },
        timeout_s);
    if (st == WaitStatus::Done && herr == hipSuccess && !failed_.load()) return;
    auto abort_now = [this](const char* why) { abort(why); };
    if (st == WaitStatus::Timeout)
      collective_fail<Error>(abort_now, "collective watchdog: no progress within " + std::to_string(timeout_s) + " s (" +
                                            knob + "); a peer rank is gone or hung");
    if (herr != hipSuccess && herr != hipErrorNotReady)
      collective_fail<Error>(abort_now, std::string("HIP: ") + hipGetErrorString(herr));
    collective_fail<Error>(abort_now, "host collective failed: a peer rank aborted, died or timed out");
  }
  void barrier() override {
    if (!g_->barrier()) {
      abort("barrier failed");
      throw Error("host comm: barrier failed (a peer rank is gone)");
    }
  }
  void abort(const char* why) override {
    if (!failed_.exchange(true)) std::fprintf(stderr, "rank %d aborting: %s\n", rank_, why);
    // peers' pending and future collectives fail at once; our own host
    // functions return, so the streams drain and device frees cannot hang
    g_->poison();
  }
};

}  // namespace

std::unique_ptr<Comm> make_host_comm(int rank, int world, int local) {
  return std::make_unique<HostComm>(rank, world, local);
}

}  // namespace mcc
