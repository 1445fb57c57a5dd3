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
// stream and graph-captured collectives as an 8-GPU one.  --comm local
// (world 1 only) swaps in the collective-free LocalComm for A/B runs;
// --comm host runs several ranks on ONE GPU with host shared-memory
// collectives (host_comm.h) -- the multi-rank rehearsal of the test box.
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "bootstrap.h"
#include "cli.h"
#include "host_comm.h"
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

void bootstrap_id(ncclUniqueId& id, int rank, int world) {
  if (rank == 0) NCCLCHK(ncclGetUniqueId(&id));
  bootstrap_blob(&id, sizeof(id), rank, world, bootstrap_addr_from_env());
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
    if (a.comm == "local") {
      if (world != 1) throw mcc::Error("--comm local needs world size 1");
      comm.reset(new mcc::LocalComm());
    } else if (a.comm == "host") {
      comm = mcc::make_host_comm(rank, world, local);
    } else if (a.comm == "rccl") {
      comm.reset(new mcc::RcclComm(rank, world, local));
    } else {
      throw mcc::Error("--comm must be rccl, host or local");
    }
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
