// `cnn_hip`: single-GPU trainer with the reference CLI (cnn.c:406-531),
// every layer on the framework's gfx950 kernels.  This is what CUDAcnn.cu
// (one fp64 conv-forward offload with per-call cudaMalloc, never compiled)
// was meant to be.
//
//   cnn_hip train-images train-labels test-images test-labels [--model lenet5 --batch 4096 ...]
//
// --dtype bf16|fp32 runs the GpuNet engine (device-resident data, hipGraph
// step); --dtype fp64 runs the reference program's own loop at its own
// precision on GpuNet64 (with --ref-compat: its D1/D10 semantics and
// per-sample updates), printing the same log as `cnn`.
#include <cstdio>
#include <memory>

#include "cli.h"
#include "mcc/net64.h"
#include "serial_loop.h"
#include "trainer.h"

namespace mcc {
void net_set_params(GpuNet64& n, const std::vector<double>& p) { n.set_params(p.data()); }
std::vector<double> net_get_params(GpuNet64& n) {
  std::vector<double> p(n.nparams());
  n.get_params(p.data());
  return p;
}
}  // namespace mcc

int main(int argc, char** argv) {
  mcc::CliArgs a;
  if (mcc::parse_cli(argc, argv, a) != 0) return 100;
  try {
    if (a.dtype == "fp64") {
      const int max_batch = std::max(a.ref_compat ? 1 : a.batch, 256);  // 256: the test loop's batch
      return mcc::run_serial<double>(a, "cnn_hip", [&](const mcc::ModelSpec& s) {
        return std::make_unique<mcc::GpuNet64>(s, a.ref_compat, max_batch);
      });
    }
    mcc::LocalComm comm;
    return mcc::run_gpu_training(a, comm, "cnn_hip");
  } catch (const mcc::Error& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 111;
  }
}
