// `cnn_hip`: single-GPU trainer with the reference CLI (cnn.c:406-531),
// every layer on the framework's gfx950 kernels.  This is what CUDAcnn.cu
// (one fp64 conv-forward offload with per-call cudaMalloc, never compiled)
// was meant to be.
//
//   cnn_hip train-images train-labels test-images test-labels [--model lenet5 --batch 4096 ...]
#include <cstdio>

#include "cli.h"
#include "trainer.h"

int main(int argc, char** argv) {
  mcc::CliArgs a;
  if (mcc::parse_cli(argc, argv, a) != 0) return 100;
  try {
    mcc::LocalComm comm;
    return mcc::run_gpu_training(a, comm, "cnn_hip");
  } catch (const mcc::Error& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 111;
  }
}
