// Data and weight I/O.
//
// IDX reader: same header checks as the reference IdxFile_read (cnn.c:345-383:
// u16 magic == 0, u8 type == 0x08, u8 ndims >= 1, big-endian u32 dims, u8
// payload) but the payload is always read (defect D3, cnnmpi.c:382) and a
// short file is an error instead of uninitialised memory.
//
// Weight file ("MCNNW"): the reference keeps weights only in memory
// (Layer.weights/biases, cnn.c:26-30) and has no file format; this is the
// framework's serialisation of exactly those arrays, in the reference's
// layouts and precision (fp64), in layer order.  Little-endian:
//   char[8] magic "MCNNW\0\0\0"; u32 version(=2); u32 byte-order mark
//   0x01020304 (version 2; absent in version 1); u32 nlayers; u64 nparams
//   per layer: i32 ltype (0 input, 1 full, 2 conv — cnn.c:8-12 — 3 maxpool),
//              i32 depth, width, height, kernsize, padding, stride, act;
//              i64 nbiases, nweights
//   per layer: f64 biases[nbiases], f64 weights[nweights]
// The loader re-derives every layer's shapes and parameter counts from the
// stored geometry and rejects a file whose stored nbiases / nweights / act
// disagree, a big-endian file, or a truncated / oversized payload.
#pragma once

#include <string>
#include <vector>

#include "mcc/model.h"

namespace mcc {

struct IdxFile {
  std::vector<uint32_t> dims;
  std::vector<uint8_t> data;
  int64_t count() const { return dims.empty() ? 0 : dims[0]; }
  int64_t item_size() const {
    int64_t n = 1;
    for (size_t i = 1; i < dims.size(); ++i) n *= dims[i];
    return n;
  }
};

IdxFile idx_read(const std::string& path);  // throws mcc::Error
// Labels are used as indices by the loss kernels (the reference only ever
// compared j == label, cnn.c:462): reject any of the first n labels that is
// not a valid class.  Throws mcc::Error naming the file and the offender.
void check_labels(const IdxFile& labels, int64_t n, int num_classes, const std::string& what);
void idx_write(const std::string& path, const std::vector<uint32_t>& dims, const uint8_t* data);

// Synthetic, learnable, MNIST/CIFAR/ImageNet-shaped data: a noisy background
// (0..39) plus a bright class-indexed horizontal stripe (SURVEY.md §6 recipe).
// images: [N][H][W][C] u8 (== [N][C][H][W] when C == 1); labels: [N] u8.
void synth_dataset(int64_t N, int C, int H, int W, int num_classes, uint64_t seed,
                   std::vector<uint8_t>& images, std::vector<uint8_t>& labels);

void save_weights(const std::string& path, const ModelSpec& spec, const double* params);
// Returns the model stored in the file and fills params (canonical, fp64).
ModelSpec load_weights(const std::string& path, std::vector<double>& params);

}  // namespace mcc
