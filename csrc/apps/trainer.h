// Native GPU training driver shared by `cnn_hip` (1 GPU) and `cnn_dist`
// (one process per GPU, RCCL over xGMI).  Reference counterparts: the serial
// main (cnn.c:406-531), the MPI main (cnnmpi.c:412-560) and the intended
// hybrid CUDAMPI.c + CUDAMPI.cu program (which never compiled).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "cli.h"
#include "mcc/common.h"

namespace mcc {

// Collective interface of the data-parallel driver.  Implementations:
// LocalComm (no collectives: cnn_hip, or cnn_dist --comm local), HostComm (host_comm.h: several ranks on one GPU) and
// RcclComm (cnn_dist.cpp, any world size including 1).  Every collective is
// enqueued on the given stream; the host blocks only in wait() and barrier(),
// which RcclComm bounds with the collective watchdog (watchdog.h).
struct Comm {
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual int local_rank() const { return rank(); }
  virtual const char* name() const = 0;
  // true when the collectives really execute (RCCL, even at world 1)
  virtual bool collective() const = 0;
  // Block until `ev` has completed (throws mcc::Error on a communicator
  // error or when the watchdog deadline passes).
  virtual void wait(hipEvent_t ev) {
    if (hipEventSynchronize(ev) != hipSuccess) throw Error("hipEventSynchronize failed");
  }
  // wait() with the longer deadline of the post-training agreement, which
  // covers rank 0's test phase (MCC_TEST_TIMEOUT)
  virtual void wait_long(hipEvent_t ev) { wait(ev); }
  virtual void allreduce_sum_f32(float* buf, int64_t n, hipStream_t s) = 0;
  virtual void allreduce_max_f64(double* buf, int64_t n, hipStream_t s) = 0;
  virtual void broadcast_f32(float* buf, int64_t n, int root, hipStream_t s) = 0;
  virtual void barrier() = 0;
  virtual void abort(const char* why) = 0;
};

struct LocalComm : Comm {
  int rank() const override { return 0; }
  int size() const override { return 1; }
  const char* name() const override { return "local"; }
  bool collective() const override { return false; }
  void allreduce_sum_f32(float*, int64_t, hipStream_t) override {}
  void allreduce_max_f64(double*, int64_t, hipStream_t) override {}
  void broadcast_f32(float*, int64_t, int, hipStream_t) override {}
  void barrier() override {}
  void abort(const char*) override {}
};

// Runs the full program (train + test + optional save) and returns the exit code.
int run_gpu_training(const CliArgs& args, Comm& comm, const char* program);

}  // namespace mcc
