// Common host/device definitions for the MI355X CNN framework (mcc).
//
// Everything here is gfx950 (CDNA4) specific: 64-lane waves, bf16 MFMA,
// 16-byte vector staging.  No CUDA compatibility layer exists anywhere.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace mcc {

enum class DType : int { F32 = 0, BF16 = 1, F64 = 2 };

inline const char* dtype_name(DType d) {
  switch (d) {
    case DType::F32: return "fp32";
    case DType::BF16: return "bf16";
    case DType::F64: return "fp64";
  }
  return "?";
}

inline size_t dtype_size(DType d) {
  switch (d) {
    case DType::F32: return 4;
    case DType::BF16: return 2;
    case DType::F64: return 8;
  }
  return 0;
}

// Errors carry a message; bindings translate them to Python exceptions and the
// native drivers to exit code 111 (reference convention, cnn.c:432).
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define MCC_CHECK(cond, msg)                                                   \
  do {                                                                         \
    if (!(cond)) {                                                             \
      throw ::mcc::Error(std::string("mcc check failed: ") + (msg) + " [" +    \
                         __FILE__ + ":" + std::to_string(__LINE__) + "]");     \
    }                                                                          \
  } while (0)

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

}  // namespace mcc
