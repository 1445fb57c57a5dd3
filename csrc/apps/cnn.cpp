// `cnn`: serial CPU trainer / evaluator (reference cnn.c:406-531).
//
//   cnn train-images train-labels test-images test-labels [flags]
//
// --ref-compat reproduces the reference program: glibc srand(seed) init, the
// shared-slice conv indexing (D1), batch-1 backprop with the update applied
// whenever i % batch == 0 at rate/batch, sampling with replacement rand() % N
// (cnn.c:451-474) — so its stderr log can be diffed line by line against the
// original.  The default mode fixes D1 and uses true mean-gradient minibatches
// (same sampling and log format).
#include <cstdio>

#include "serial_loop.h"

using namespace mcc;

template <typename T>
static int run(const CliArgs& a) {
  return run_serial<T>(a, "cnn", [&](const ModelSpec& s) { return std::make_unique<CpuNet<T>>(s, a.ref_compat); });
}

int main(int argc, char** argv) {
  CliArgs a;
  if (parse_cli(argc, argv, a) != 0) return 100;
  try {
    return a.fp32 ? run<float>(a) : run<double>(a);
  } catch (const Error& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 111;
  }
}
