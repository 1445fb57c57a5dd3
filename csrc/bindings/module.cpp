// Python bindings (pybind11) for the native core.  Tensors cross the boundary
// as raw device pointers + HIP stream handles (torch's data_ptr() and
// current_stream().cuda_stream), so this translation unit needs no torch
// headers and the same engine serves the native drivers and Python.
#include <cstring>
#include <limits>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime_api.h>

#include "kernels.h"
#include "mcc/cpu_net.h"
#include "mcc/engine.h"
#include "mcc/io.h"
#include "mcc/model.h"
#include "mcc/net64.h"

namespace py = pybind11;
using namespace mcc;

namespace {

template <typename T>
T* ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::dict layer_dict(const LayerSpec& L) {
  py::dict d;
  d["kind"] = layer_kind_name(L.kind);
  d["C"] = L.C; d["H"] = L.H; d["W"] = L.W;
  d["inC"] = L.inC; d["inH"] = L.inH; d["inW"] = L.inW;
  d["ks"] = L.ks; d["stride"] = L.stride; d["pad"] = L.pad;
  d["act"] = act_name(L.act);
  d["init_std"] = L.init_std;
  d["w_off"] = L.w_off; d["b_off"] = L.b_off; d["nweights"] = L.nweights; d["nbiases"] = L.nbiases;
  return d;
}

DType parse_dtype(const std::string& s) {
  if (s == "bf16" || s == "bfloat16") return DType::BF16;
  if (s == "fp32" || s == "float32" || s == "f32") return DType::F32;
  if (s == "fp64" || s == "float64" || s == "f64") return DType::F64;
  throw Error("unknown dtype '" + s + "'");
}

template <typename T>
void bind_cpu_net(py::module_& m, const char* name) {
  using Net = CpuNet<T>;
  py::class_<Net>(m, name)
      .def(py::init<const ModelSpec&, bool>(), py::arg("spec"), py::arg("ref_compat") = false)
      .def_property_readonly("nparams", &Net::nparams)
      .def_property_readonly("ref_compat", &Net::ref_compat)
      .def("get_params", [](const Net& n) { return py::array_t<T>(n.params.size(), n.params.data()); })
      .def("get_grads", [](const Net& n) { return py::array_t<T>(n.grads.size(), n.grads.data()); })
      .def("set_params",
           [](Net& n, py::array_t<T, py::array::c_style | py::array::forcecast> a) {
             MCC_CHECK((int64_t)a.size() == n.nparams(), "set_params: size mismatch");
             std::copy(a.data(), a.data() + a.size(), n.params.begin());
           })
      .def("set_grads",
           [](Net& n, py::array_t<T, py::array::c_style | py::array::forcecast> a) {
             MCC_CHECK((int64_t)a.size() == n.nparams(), "set_grads: size mismatch");
             std::copy(a.data(), a.data() + a.size(), n.grads.begin());
           })
      .def("forward",
           [](Net& n, py::array_t<T, py::array::c_style | py::array::forcecast> x) {
             const int64_t in = n.spec().input_nodes();
             MCC_CHECK(x.size() % in == 0, "forward: input size not a multiple of the input shape");
             const int B = (int)(x.size() / in);
             {
               py::gil_scoped_release rel;
               n.forward(x.data(), B);
             }
             const int nc = n.spec().num_classes();
             return py::array_t<T>({B, nc}, n.probs());
           })
      .def("backward",
           [](Net& n, py::array_t<int, py::array::c_style | py::array::forcecast> labels, double scale) {
             StepStats s;
             {
               py::gil_scoped_release rel;
               s = n.backward(labels.data(), (T)scale);
             }
             py::dict d;
             d["loss_sum"] = s.loss_sum; d["mse_sum"] = s.mse_sum; d["correct"] = s.correct; d["count"] = s.count;
             return d;
           },
           py::arg("labels"), py::arg("scale") = 1.0)
      .def("evaluate",
           [](const Net& n, py::array_t<int, py::array::c_style | py::array::forcecast> labels) {
             StepStats s = n.evaluate(labels.data());
             py::dict d;
             d["loss_sum"] = s.loss_sum; d["mse_sum"] = s.mse_sum; d["correct"] = s.correct; d["count"] = s.count;
             return d;
           })
      .def("sgd", [](Net& n, double lr) { n.sgd((T)lr); })
      .def("zero_grads", &Net::zero_grads);
}

// Minimal DLPack (v0.8 ABI) so torch can alias engine-owned device buffers
// (torch.utils.dlpack.from_dlpack) — e.g. the flat gradient buffer that
// torch.distributed all-reduces in place.  The capsule does not own memory.
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data; DLDevice device; int32_t ndim; DLDataType dtype;
  int64_t* shape; int64_t* strides; uint64_t byte_offset;
};
struct DLManagedTensor { DLTensor dl_tensor; void* manager_ctx; void (*deleter)(DLManagedTensor*); };
struct DLHolder { DLManagedTensor t; int64_t shape[1]; int64_t strides[1]; };

void dl_deleter(DLManagedTensor* t) { delete reinterpret_cast<DLHolder*>(t->manager_ctx); }

py::capsule dlpack_wrap(uintptr_t p, int64_t numel, const std::string& dtype, int device) {
  auto* h = new DLHolder();
  h->shape[0] = numel;
  h->strides[0] = 1;
  h->t.dl_tensor.data = reinterpret_cast<void*>(p);
  h->t.dl_tensor.device = DLDevice{10 /* kDLROCM */, device};
  h->t.dl_tensor.ndim = 1;
  if (dtype == "float32") h->t.dl_tensor.dtype = DLDataType{2, 32, 1};
  else if (dtype == "bfloat16") h->t.dl_tensor.dtype = DLDataType{4, 16, 1};
  else if (dtype == "uint8") h->t.dl_tensor.dtype = DLDataType{1, 8, 1};
  else if (dtype == "int32") h->t.dl_tensor.dtype = DLDataType{0, 32, 1};
  else if (dtype == "int64") h->t.dl_tensor.dtype = DLDataType{0, 64, 1};
  else { delete h; throw Error("dlpack_wrap: unsupported dtype " + dtype); }
  h->t.dl_tensor.shape = h->shape;
  h->t.dl_tensor.strides = h->strides;
  h->t.dl_tensor.byte_offset = 0;
  h->t.manager_ctx = h;
  h->t.deleter = dl_deleter;
  return py::capsule(&h->t, "dltensor", [](PyObject* cap) {
    // Only free if torch never consumed it (consumed capsules are renamed).
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (t && t->deleter) t->deleter(t);
    }
  });
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native CNN framework core (HIP/CDNA4 kernels + C++ runtime)";
  py::register_exception<Error>(m, "MccError", PyExc_RuntimeError);

  // ---------------------------------------------------------------- model
  py::class_<ModelSpec>(m, "ModelSpec")
      .def_readonly("name", &ModelSpec::name)
      .def_readonly("nparams", &ModelSpec::nparams)
      .def("describe", &ModelSpec::describe)
      .def("macs_per_sample", &ModelSpec::macs_per_sample)
      .def("num_classes", &ModelSpec::num_classes)
      .def("input_shape", [](const ModelSpec& s) {
        return py::make_tuple(s.input().C, s.input().H, s.input().W);
      })
      .def("layers", [](const ModelSpec& s) {
        py::list l;
        for (const auto& L : s.layers) l.append(layer_dict(L));
        return l;
      });
  m.def("make_model", &make_model, py::arg("name"));
  m.def("model_names", &model_names);
  m.def("parse_model_spec", &parse_model_spec, py::arg("text"), py::arg("name") = "custom");
  m.def("plan_buckets",
        [](const ModelSpec& s, int64_t bytes) {
          py::list l;
          for (const auto& b : plan_buckets(s, bytes)) l.append(py::make_tuple(b.stage_hi, b.stage_lo, b.off, b.count));
          return l;
        },
        py::arg("spec"), py::arg("bucket_bytes"));
  m.def("init_params",
        [](const ModelSpec& s, uint64_t seed, const std::string& mode) {
          py::array_t<double> out(s.nparams);
          init_params(s, out.mutable_data(), seed, mode == "fast" ? InitMode::Fast : InitMode::GlibcRef);
          return out;
        },
        py::arg("spec"), py::arg("seed") = 0, py::arg("mode") = "glibc");

  // ------------------------------------------------------------------- io
  m.def("idx_read", [](const std::string& path) {
    IdxFile f = idx_read(path);
    std::vector<py::ssize_t> shape(f.dims.begin(), f.dims.end());
    py::array_t<uint8_t> a(shape);
    std::copy(f.data.begin(), f.data.end(), a.mutable_data());
    return a;
  });
  m.def("idx_write", [](const std::string& path, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
    std::vector<uint32_t> dims;
    for (py::ssize_t i = 0; i < a.ndim(); ++i) dims.push_back((uint32_t)a.shape(i));
    idx_write(path, dims, a.data());
  });
  m.def("synth_dataset",
        [](int64_t N, int C, int H, int W, int classes, uint64_t seed) {
          std::vector<uint8_t> img, lab;
          {
            py::gil_scoped_release rel;
            synth_dataset(N, C, H, W, classes, seed, img, lab);
          }
          py::array_t<uint8_t> a({(py::ssize_t)N, (py::ssize_t)H, (py::ssize_t)W, (py::ssize_t)C});
          std::copy(img.begin(), img.end(), a.mutable_data());
          py::array_t<uint8_t> b((py::ssize_t)N);
          std::copy(lab.begin(), lab.end(), b.mutable_data());
          return py::make_tuple(a, b);
        },
        py::arg("n"), py::arg("c"), py::arg("h"), py::arg("w"), py::arg("classes") = 10, py::arg("seed") = 0);
  m.def("save_weights", [](const std::string& path, const ModelSpec& s,
                           py::array_t<double, py::array::c_style | py::array::forcecast> p) {
    MCC_CHECK((int64_t)p.size() == s.nparams, "save_weights: size mismatch");
    save_weights(path, s, p.data());
  });
  m.def("load_weights", [](const std::string& path) {
    std::vector<double> p;
    ModelSpec s = load_weights(path, p);
    return py::make_tuple(s, py::array_t<double>(p.size(), p.data()));
  });

  bind_cpu_net<double>(m, "CpuNet64");
  bind_cpu_net<float>(m, "CpuNet32");

  // fp64 on the GPU, CpuNet64's API (host arrays in and out) plus device
  // pointers for zero-copy use
  auto stats_dict = [](const StepStats& s) {
    py::dict d;
    d["loss_sum"] = s.loss_sum; d["mse_sum"] = s.mse_sum; d["correct"] = s.correct; d["count"] = s.count;
    return d;
  };
  using F64 = py::array_t<double, py::array::c_style | py::array::forcecast>;
  py::class_<GpuNet64>(m, "GpuNet64")
      .def(py::init<const ModelSpec&, bool, int, int>(), py::arg("spec"), py::arg("ref_compat") = false,
           py::arg("max_batch") = 256, py::arg("device") = -1)
      .def_property_readonly("nparams", &GpuNet64::nparams)
      .def_property_readonly("ref_compat", &GpuNet64::ref_compat)
      .def_property_readonly("max_batch", &GpuNet64::max_batch)
      .def_property_readonly("device_bytes", &GpuNet64::device_bytes)
      .def_property_readonly("params_ptr", [](const GpuNet64& n) { return reinterpret_cast<uintptr_t>(n.device_params()); })
      .def_property_readonly("grads_ptr", [](const GpuNet64& n) { return reinterpret_cast<uintptr_t>(n.device_grads()); })
      .def_property_readonly("stream", [](const GpuNet64& n) { return reinterpret_cast<uintptr_t>(n.stream()); })
      .def("forward_u8",
           [](GpuNet64& n, uintptr_t data, uintptr_t labels, uintptr_t idx, int B) {
             n.forward_u8(reinterpret_cast<const uint8_t*>(data), reinterpret_cast<const uint8_t*>(labels),
                          reinterpret_cast<const int32_t*>(idx), B);
           },
           py::arg("data"), py::arg("labels"), py::arg("idx"), py::arg("B"),
           "device-resident batch: rows idx[0..B) of the u8 dataset (/255) and their labels; no host sync")
      .def("backward_device", &GpuNet64::backward_device, py::arg("scale"),
           "backward of the last forward_u8 with device labels; per-sample stats stay on the device")
      .def("loss_sum",
           [](const GpuNet64& n) {
             // sum of -log p_label over the last backward's batch (synchronises)
             std::vector<double> st(3 * (size_t)n.batch());
             if (hipDeviceSynchronize() != hipSuccess) throw Error("hipDeviceSynchronize failed");
             if (hipMemcpy(st.data(), n.device_stats(), 8 * st.size(), hipMemcpyDeviceToHost) != hipSuccess)
               throw Error("hipMemcpy failed");
             double s = 0.0;
             for (int b = 0; b < n.batch(); ++b) s += st[3 * b];
             return s;
           })
      .def("get_params", [](const GpuNet64& n) { py::array_t<double> a(n.nparams()); n.get_params(a.mutable_data()); return a; })
      .def("get_grads", [](const GpuNet64& n) { py::array_t<double> a(n.nparams()); n.get_grads(a.mutable_data()); return a; })
      .def("set_params", [](GpuNet64& n, F64 a) {
        MCC_CHECK((int64_t)a.size() == n.nparams(), "set_params: size mismatch");
        n.set_params(a.data());
      })
      .def("set_grads", [](GpuNet64& n, F64 a) {
        MCC_CHECK((int64_t)a.size() == n.nparams(), "set_grads: size mismatch");
        n.set_grads(a.data());
      })
      .def("forward", [](GpuNet64& n, F64 x) {
        const int64_t in = n.spec().input_nodes();
        MCC_CHECK(x.size() % in == 0, "forward: input size not a multiple of the input shape");
        const int B = (int)(x.size() / in);
        const double* p;
        {
          py::gil_scoped_release rel;
          n.forward(x.data(), B);
          p = n.probs();
        }
        return py::array_t<double>({B, n.spec().num_classes()}, p);
      })
      .def("forward_device", [](GpuNet64& n, uintptr_t x, int B) { n.forward_device(ptr<const double>(x), B); },
           py::arg("x"), py::arg("B"))
      .def("backward", [stats_dict](GpuNet64& n, py::array_t<int, py::array::c_style | py::array::forcecast> labels,
                                    double scale) {
        MCC_CHECK(labels.size() >= n.batch(), "backward: fewer labels than the forward batch");
        StepStats s;
        {
          py::gil_scoped_release rel;
          s = n.backward(labels.data(), scale);
        }
        return stats_dict(s);
      }, py::arg("labels"), py::arg("scale") = 1.0)
      .def("evaluate", [stats_dict](GpuNet64& n, py::array_t<int, py::array::c_style | py::array::forcecast> labels) {
        MCC_CHECK(labels.size() >= n.batch(), "evaluate: fewer labels than the forward batch");
        return stats_dict(n.evaluate(labels.data()));
      })
      .def("sgd", [](GpuNet64& n, double lr) { n.sgd(lr); })
      .def("zero_grads", &GpuNet64::zero_grads);

  // --------------------------------------------------------------- engine
  py::class_<GpuNet>(m, "GpuNet")
      .def(py::init([](const ModelSpec& s, const std::string& dtype, int max_batch, int device) {
             return new GpuNet(s, parse_dtype(dtype), max_batch, device);
           }),
           py::arg("spec"), py::arg("dtype") = "bf16", py::arg("max_batch") = 1024, py::arg("device") = -1)
      .def("plan", &GpuNet::plan)
      .def_property_readonly("nparams", &GpuNet::nparams)
      .def_property_readonly("num_stages", &GpuNet::num_stages)
      .def_property_readonly("max_batch", &GpuNet::max_batch)
      .def_property_readonly("arena_bytes", &GpuNet::arena_bytes)
      .def_property_readonly("params_ptr", [](const GpuNet& n) { return (uintptr_t)n.params(); })
      .def_property_readonly("grads_ptr", [](const GpuNet& n) { return (uintptr_t)n.grads(); })
      .def_property_readonly("stats_ptr", [](const GpuNet& n) { return (uintptr_t)n.stats(); })
      .def_property_readonly("logits_ptr", [](const GpuNet& n) { return (uintptr_t)n.logits(); })
      .def_property_readonly("logits_ld", &GpuNet::logits_ld)
      .def("set_params",
           [](GpuNet& n, py::array_t<float, py::array::c_style | py::array::forcecast> a) {
             MCC_CHECK((int64_t)a.size() == n.nparams(), "set_params: size mismatch");
             n.set_params(a.data());
           })
      .def("get_params",
           [](const GpuNet& n) {
             py::array_t<float> a(n.nparams());
             n.get_params(a.mutable_data());
             return a;
           })
      .def("get_grads",
           [](const GpuNet& n) {
             py::array_t<float> a(n.nparams());
             n.get_grads(a.mutable_data());
             return a;
           })
      .def("get_logits",
           [](const GpuNet& n, int B) {
             MCC_CHECK(B > 0 && B <= n.max_batch(), "get_logits: bad batch");
             // forward() may have been enqueued on any (non-blocking) stream:
             // the deferred FC forward runs on the null stream only after the
             // whole device is idle, and is itself waited for before the copy
             if (hipDeviceSynchronize() != hipSuccess) throw Error("hipDeviceSynchronize failed");
             n.flush_forward(nullptr);
             const int nc = n.spec().num_classes(), ld = n.logits_ld();
             std::vector<float> tmp((size_t)B * ld);
             if (hipDeviceSynchronize() != hipSuccess) throw Error("hipDeviceSynchronize failed");
             if (hipMemcpy(tmp.data(), n.logits(), 4 * tmp.size(), hipMemcpyDeviceToHost) != hipSuccess)
               throw Error("hipMemcpy failed");
             py::array_t<float> a({B, nc});
             for (int b = 0; b < B; ++b)
               for (int j = 0; j < nc; ++j) a.mutable_at(b, j) = tmp[(size_t)b * ld + j];
             return a;
           })
      .def("stage_output",
           [](const GpuNet& n, int stage, int B) {
             // (float32 copy of the stored activation, argmax bytes or None)
             MCC_CHECK(B > 0 && B <= n.max_batch(), "stage_output: bad batch");
             // a deferred LeNet-5 FC forward (forward() alone) is run first, on
             // the null stream after the device is idle, so stages 2-4 are current
             if (hipDeviceSynchronize() != hipSuccess) throw Error("hipDeviceSynchronize failed");
             n.flush_forward(nullptr);
             int64_t per = 0;
             const uint8_t* arg = nullptr;
             const void* y = n.stage_output(stage, per, &arg);
             const size_t cnt = (size_t)B * per, es = n.dtype() == DType::BF16 ? 2 : 4;
             std::vector<uint8_t> raw(cnt * es);
             if (hipDeviceSynchronize() != hipSuccess) throw Error("hipDeviceSynchronize failed");
             if (hipMemcpy(raw.data(), y, raw.size(), hipMemcpyDeviceToHost) != hipSuccess) throw Error("hipMemcpy failed");
             py::array_t<float> a((py::ssize_t)cnt);
             float* d = a.mutable_data();
             for (size_t i = 0; i < cnt; ++i) {
               if (es == 4) std::memcpy(d + i, raw.data() + 4 * i, 4);
               else {
                 const uint32_t bits = (uint32_t)(raw[2 * i] | (raw[2 * i + 1] << 8)) << 16;
                 std::memcpy(d + i, &bits, 4);
               }
             }
             if (!arg) return py::tuple(py::make_tuple(a, py::none()));
             py::array_t<uint8_t> g((py::ssize_t)cnt);
             if (hipMemcpy(g.mutable_data(), arg, cnt, hipMemcpyDeviceToHost) != hipSuccess) throw Error("hipMemcpy failed");
             return py::tuple(py::make_tuple(a, g));
           })
      .def("get_stats",
           [](const GpuNet& n) {
             unsigned long long h[4];
             if (hipDeviceSynchronize() != hipSuccess) throw Error("hipDeviceSynchronize failed");
             if (hipMemcpy(h, n.stats(), 32, hipMemcpyDeviceToHost) != hipSuccess) throw Error("hipMemcpy failed");
             py::dict d;
             const double nan = std::numeric_limits<double>::quiet_NaN();
             d["loss_sum"] = h[gpu::kStatNaN] ? nan : (double)h[0] / gpu::kStatScale;
             d["mse_sum"] = h[gpu::kStatNaN] ? nan : (double)h[1] / gpu::kStatScale;
             d["correct"] = (double)h[2];
             return d;
           })
      .def("forward",
           [](GpuNet& n, uintptr_t images, uintptr_t idx, int B, uintptr_t s) {
             n.forward(ptr<const uint8_t>(images), ptr<const int32_t>(idx), B, stream_of(s));
           },
           py::arg("images"), py::arg("idx"), py::arg("batch"), py::arg("stream") = 0)
      .def("loss",
           [](GpuNet& n, uintptr_t labels, uintptr_t idx, float scale, bool backward, uintptr_t s, uintptr_t pred) {
             n.loss(ptr<const uint8_t>(labels), ptr<const int32_t>(idx), scale, backward, stream_of(s),
                    ptr<int32_t>(pred));
           },
           py::arg("labels"), py::arg("idx"), py::arg("scale"), py::arg("backward") = true, py::arg("stream") = 0,
           py::arg("pred") = 0)
      .def("zero_stats", [](GpuNet& n, uintptr_t s) { n.zero_stats(stream_of(s)); }, py::arg("stream") = 0)
      .def("backward", [](GpuNet& n, int hi, int lo, uintptr_t s) { n.backward(hi, lo, stream_of(s)); },
           py::arg("stage_hi"), py::arg("stage_lo"), py::arg("stream") = 0)
      .def("backward_all", [](GpuNet& n, uintptr_t s) { n.backward_all(stream_of(s)); }, py::arg("stream") = 0)
      .def("sgd",
           [](GpuNet& n, float lr, float mu, float wd, uintptr_t s) { n.sgd(lr, mu, wd, stream_of(s)); },
           py::arg("lr"), py::arg("momentum") = 0.f, py::arg("weight_decay") = 0.f, py::arg("stream") = 0)
      .def("sgd_range",
           [](GpuNet& n, float lr, float mu, float wd, int64_t off, int64_t cnt, uintptr_t s) {
             n.sgd_range(lr, mu, wd, off, cnt, stream_of(s));
           },
           py::arg("lr"), py::arg("momentum"), py::arg("weight_decay"), py::arg("off"), py::arg("count"),
           py::arg("stream") = 0)
      .def("pack", [](GpuNet& n, uintptr_t s) { n.pack(stream_of(s)); }, py::arg("stream") = 0)
      .def("stage_param_range",
           [](const GpuNet& n, int s) {
             int64_t off, cnt;
             n.stage_param_range(s, off, cnt);
             return py::make_tuple(off, cnt);
           })
      .def("buckets", [](const GpuNet& n, int64_t bytes) {
        py::list l;
        for (const auto& b : n.buckets(bytes)) l.append(py::make_tuple(b.stage_hi, b.stage_lo, b.off, b.count));
        return l;
      });

  // ------------------------------------------------- raw kernels (tests)
  py::module_ k = m.def_submodule("kernels", "raw gfx950 kernel entry points (device pointers)");
  k.def("gemm",
        [](const std::string& dt, int M, int N, int K, uintptr_t A, int lda, bool ta, uintptr_t B, int ldb, bool tb,
           int ones_col, int epi, int act, uintptr_t bias, uintptr_t aux, int ldaux, uintptr_t C, int ldc,
           uintptr_t Cf, int splitk, int64_t pstride, uintptr_t s) {
          gpu::GemmParams p;
          p.M = M; p.N = N; p.K = K;
          p.A = ptr<void>(A); p.lda = lda; p.ta = ta;
          p.B = ptr<void>(B); p.ldb = ldb; p.tb = tb;
          p.ones_col = ones_col; p.epi = epi; p.act = act;
          p.bias = ptr<float>(bias); p.aux = ptr<void>(aux); p.ldaux = ldaux;
          p.C = ptr<void>(C); p.ldc = ldc; p.Cf = ptr<float>(Cf);
          p.splitk = splitk; p.partial_stride = pstride;
          gpu::gemm(parse_dtype(dt), p, stream_of(s));
        },
        py::arg("dtype"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"), py::arg("ta"),
        py::arg("B"), py::arg("ldb"), py::arg("tb"), py::arg("ones_col") = -1, py::arg("epi") = 0,
        py::arg("act") = 0, py::arg("bias") = 0, py::arg("aux") = 0, py::arg("ldaux") = 0, py::arg("C") = 0,
        py::arg("ldc") = 0, py::arg("Cf") = 0, py::arg("splitk") = 1, py::arg("pstride") = 0,
        py::arg("stream") = 0);
  // the engine's FC forward for long-K layers (VGG-11 FC1): split-K partials
  // into `scratch` + the finishing bias / activation pass; splitk < 1 = the
  // engine's own rule (gemm_fwd_splitk)
  k.def("gemm_fwd_splitk", &gpu::gemm_fwd_splitk, py::arg("M"), py::arg("N"), py::arg("K"));
  k.def("gemm_splitk_fwd",
        [](const std::string& dt, int M, int N, int K, uintptr_t A, int lda, uintptr_t W, int ldw, int act,
           uintptr_t bias, uintptr_t C, int ldc, uintptr_t scratch, int splitk, uintptr_t s) {
          gpu::GemmParams p;
          p.M = M; p.N = N; p.K = K;
          p.A = ptr<void>(A); p.lda = lda;
          p.B = ptr<void>(W); p.ldb = ldw;
          p.bias = ptr<float>(bias);
          p.epi = gpu::EPI_BIAS_ACT; p.act = act; p.C = ptr<void>(C); p.ldc = ldc;
          const int sk = splitk >= 1 ? splitk : gpu::gemm_fwd_splitk(M, N, K);
          gpu::gemm_splitk_fwd(parse_dtype(dt), p, ptr<float>(scratch), sk, stream_of(s));
          return sk;
        },
        py::arg("dtype"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"), py::arg("W"),
        py::arg("ldw"), py::arg("act"), py::arg("bias"), py::arg("C"), py::arg("ldc"), py::arg("scratch"),
        py::arg("splitk") = 0, py::arg("stream") = 0);
  k.def("fc",
        [](int M, int N, int K, uintptr_t A, int lda, uintptr_t W, int ldw, int epi, int act, uintptr_t bias,
           uintptr_t aux, int ldaux, uintptr_t C, int ldc, uintptr_t Cf, uintptr_t dbg, uintptr_t s) {
          gpu::FcParams p;
          p.M = M; p.N = N; p.K = K;
          p.A = ptr<void>(A); p.lda = lda; p.W = ptr<void>(W); p.ldw = ldw;
          p.epi = epi; p.act = act; p.bias = ptr<float>(bias); p.aux = ptr<void>(aux); p.ldaux = ldaux;
          p.C = ptr<void>(C); p.ldc = ldc; p.Cf = ptr<float>(Cf);
          p.dbg = ptr<long long>(dbg);
          gpu::fc_forward(p, stream_of(s));
        },
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"), py::arg("W"), py::arg("ldw"),
        py::arg("epi") = 0, py::arg("act") = 0, py::arg("bias") = 0, py::arg("aux") = 0, py::arg("ldaux") = 0,
        py::arg("C") = 0, py::arg("ldc") = 0, py::arg("Cf") = 0, py::arg("dbg") = 0, py::arg("stream") = 0);
  k.def("fc_supported", &gpu::fc_supported);
  k.def("igemm_conv_supported", &gpu::igemm_conv_supported);
  k.def("igemm_conv",
        [](int B, int H, int W, int C, int N, int KS, int stride, int pad, uintptr_t in, uintptr_t w, int ldw,
           uintptr_t bias, bool bias_act, int act, uintptr_t out, int ldo, uintptr_t out_arg, int tile,
           uintptr_t s) {
          gpu::IgemmParams p;
          p.B = B; p.H = H; p.W = W; p.C = C; p.N = N; p.KS = KS; p.stride = stride; p.pad = pad;
          p.OH = (H + 2 * pad - KS) / stride + 1; p.OW = (W + 2 * pad - KS) / stride + 1;
          p.M = B * p.OH * p.OW; p.K = KS * KS * C;
          p.in = ptr<void>(in); p.w = ptr<void>(w); p.ldw = ldw;
          p.bias = ptr<float>(bias); p.epi_bias_act = bias_act; p.act = act;
          p.out = ptr<void>(out); p.ldo = ldo;
          p.pool = out_arg != 0; p.out_arg = ptr<uint8_t>(out_arg); p.tile = tile;
          gpu::igemm_conv(p, stream_of(s));
        },
        py::arg("B"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("N"), py::arg("KS"), py::arg("stride"),
        py::arg("pad"), py::arg("input"), py::arg("w"), py::arg("ldw"), py::arg("bias") = 0,
        py::arg("bias_act") = true, py::arg("act") = 0, py::arg("out") = 0, py::arg("ldo") = 0,
        py::arg("out_arg") = 0, py::arg("tile") = -1, py::arg("stream") = 0);
  k.def("igemm_dw_splitk", &gpu::igemm_dw_splitk, py::arg("M"), py::arg("Cout"), py::arg("kf"), py::arg("tile") = -1);
  k.def("igemm_dw",
        [](int B, int H, int W, int C, int Cout, int KS, int stride, int pad, uintptr_t dz, int ldz, uintptr_t in,
           uintptr_t slab, int64_t slab_stride, int splitk, uintptr_t gw, uintptr_t gb, float beta, int tile,
           uintptr_t s) {
          gpu::IgemmDwParams p;
          p.B = B; p.H = H; p.W = W; p.C = C; p.Cout = Cout; p.KS = KS; p.stride = stride; p.pad = pad;
          p.OH = (H + 2 * pad - KS) / stride + 1; p.OW = (W + 2 * pad - KS) / stride + 1;
          p.M = B * p.OH * p.OW; p.kf = KS * KS * C;
          p.dz = ptr<void>(dz); p.ldz = ldz; p.in = ptr<void>(in);
          p.slab = ptr<float>(slab); p.slab_stride = slab_stride; p.splitk = splitk; p.tile = tile;
          gpu::igemm_dw(p, ptr<float>(gw), ptr<float>(gb), beta, stream_of(s));
        },
        py::arg("B"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("Cout"), py::arg("KS"), py::arg("stride"),
        py::arg("pad"), py::arg("dz"), py::arg("ldz"), py::arg("input"), py::arg("slab"), py::arg("slab_stride"),
        py::arg("splitk"), py::arg("gw"), py::arg("gb"), py::arg("beta") = 0.f, py::arg("tile") = -1,
        py::arg("stream") = 0);
  // LeNet-5 conv block (lenet.hip): raw launches for the kernel unit tests
  k.def("lenet_forward",
        [](int B, uintptr_t x, uintptr_t idx, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2, uintptr_t y1,
           uintptr_t a1, uintptr_t y2, uintptr_t a2, uintptr_t s) {
          gpu::LenetFwdParams p;
          p.B = B; p.x = ptr<const uint8_t>(x); p.idx = ptr<const int32_t>(idx);
          p.w1 = ptr<const float>(w1); p.b1 = ptr<const float>(b1); p.w2 = ptr<const float>(w2); p.b2 = ptr<const float>(b2);
          p.y1 = ptr<void>(y1); p.a1 = ptr<uint8_t>(a1); p.y2 = ptr<void>(y2); p.a2 = ptr<uint8_t>(a2);
          gpu::lenet_forward(p, stream_of(s));
        },
        py::arg("B"), py::arg("x"), py::arg("idx"), py::arg("w1"), py::arg("b1"), py::arg("w2"), py::arg("b2"),
        py::arg("y1"), py::arg("a1"), py::arg("y2"), py::arg("a2"), py::arg("stream") = 0);
  k.def("lenet_backward",
        [](int B, uintptr_t x, uintptr_t idx, uintptr_t w2, uintptr_t dy2, uintptr_t a2, uintptr_t y1, uintptr_t a1,
           uintptr_t slab, uintptr_t gw1, uintptr_t gb1, uintptr_t gw2, uintptr_t gb2, uintptr_t s) {
          gpu::LenetBwdParams p;
          p.B = B; p.x = ptr<const uint8_t>(x); p.idx = ptr<const int32_t>(idx); p.w2 = ptr<const float>(w2);
          p.dy2 = ptr<const void>(dy2); p.a2 = ptr<const uint8_t>(a2); p.y1 = ptr<const void>(y1);
          p.a1 = ptr<const uint8_t>(a1); p.slab = ptr<float>(slab);
          p.gw1 = ptr<float>(gw1); p.gb1 = ptr<float>(gb1); p.gw2 = ptr<float>(gw2); p.gb2 = ptr<float>(gb2);
          gpu::lenet_backward(p, stream_of(s));
        },
        py::arg("B"), py::arg("x"), py::arg("idx"), py::arg("w2"), py::arg("dy2"), py::arg("a2"), py::arg("y1"),
        py::arg("a1"), py::arg("slab"), py::arg("gw1"), py::arg("gb1"), py::arg("gw2"), py::arg("gb2"),
        py::arg("stream") = 0);
  // reference-model conv block (refnet.hip): raw launches for the kernel unit tests
  k.def("ref_forward",
        [](int B, uintptr_t x, uintptr_t idx, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2, uintptr_t y2,
           uintptr_t s, bool f32) {
          gpu::RefFwdParams p;
          p.B = B; p.x = reinterpret_cast<const uint8_t*>(x); p.idx = reinterpret_cast<const int32_t*>(idx);
          p.w1 = reinterpret_cast<const float*>(w1); p.b1 = reinterpret_cast<const float*>(b1);
          p.w2 = reinterpret_cast<const float*>(w2); p.b2 = reinterpret_cast<const float*>(b2);
          p.y2 = reinterpret_cast<void*>(y2);
          p.f32 = f32;
          gpu::ref_forward(p, stream_of(s));
        },
        py::arg("B"), py::arg("x"), py::arg("idx"), py::arg("w1"), py::arg("b1"), py::arg("w2"), py::arg("b2"),
        py::arg("y2"), py::arg("stream"), py::arg("f32") = false);
  k.def("ref_backward",
        [](int B, uintptr_t x, uintptr_t idx, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t y2, uintptr_t dy2,
           uintptr_t slab, uintptr_t gw1, uintptr_t gb1, uintptr_t gw2, uintptr_t gb2, uintptr_t s, bool f32) {
          gpu::RefBwdParams p;
          p.f32 = f32;
          p.B = B; p.x = reinterpret_cast<const uint8_t*>(x); p.idx = reinterpret_cast<const int32_t*>(idx);
          p.w1 = reinterpret_cast<const float*>(w1); p.b1 = reinterpret_cast<const float*>(b1);
          p.w2 = reinterpret_cast<const float*>(w2);
          p.y2 = reinterpret_cast<const void*>(y2); p.dy2 = reinterpret_cast<const void*>(dy2);
          p.slab = reinterpret_cast<float*>(slab);
          p.gw1 = reinterpret_cast<float*>(gw1); p.gb1 = reinterpret_cast<float*>(gb1);
          p.gw2 = reinterpret_cast<float*>(gw2); p.gb2 = reinterpret_cast<float*>(gb2);
          gpu::ref_backward(p, stream_of(s));
        },
        py::arg("B"), py::arg("x"), py::arg("idx"), py::arg("w1"), py::arg("b1"), py::arg("w2"), py::arg("y2"),
        py::arg("dy2"), py::arg("slab"), py::arg("gw1"), py::arg("gb1"), py::arg("gw2"), py::arg("gb2"),
        py::arg("stream"), py::arg("f32") = false);
  k.def("ref_slab_bytes", &gpu::ref_slab_bytes, py::arg("f32") = false);
  k.def("lenet_slab_bytes", &gpu::lenet_slab_bytes);
  // device minibatch sampler (rand() % N semantics, cnn.c:455) with the step
  // counter in device memory: graph-capturable (a replay draws fresh indices)
  k.def("sample_indices",
        [](uintptr_t idx, int B, int64_t lo, int64_t hi, uint64_t seed, uintptr_t step, uintptr_t s) {
          gpu::sample_indices(ptr<int32_t>(idx), B, lo, hi, seed, ptr<const uint64_t>(step), stream_of(s));
        },
        py::arg("idx"), py::arg("B"), py::arg("lo"), py::arg("hi"), py::arg("seed"), py::arg("step"),
        py::arg("stream") = 0);
  k.def("advance_counter", [](uintptr_t step, uintptr_t s) { gpu::advance_counter(ptr<uint64_t>(step), stream_of(s)); },
        py::arg("step"), py::arg("stream") = 0);
  // both in one launch: step -> int64[2] (counter, ticket; zero-initialised)
  k.def("sample_indices_advance",
        [](uintptr_t idx, int B, int64_t lo, int64_t hi, uint64_t seed, uintptr_t step, uintptr_t s) {
          gpu::sample_indices_advance(ptr<int32_t>(idx), B, lo, hi, seed, ptr<uint64_t>(step), stream_of(s));
        },
        py::arg("idx"), py::arg("B"), py::arg("lo"), py::arg("hi"), py::arg("seed"), py::arg("step"),
        py::arg("stream") = 0);
  k.def("sgd_update",
        [](uintptr_t p, uintptr_t g, uintptr_t v, int64_t n, float lr, float mu, float wd, uintptr_t s) {
          gpu::sgd_update(ptr<float>(p), ptr<const float>(g), ptr<float>(v), n, lr, mu, wd, stream_of(s));
        },
        py::arg("params"), py::arg("grads"), py::arg("mom"), py::arg("n"), py::arg("lr"), py::arg("momentum") = 0.f,
        py::arg("weight_decay") = 0.f, py::arg("stream") = 0);
  k.def("softmax_xent",
        [](const std::string& dt, int M, int N, uintptr_t logits, int ldl, uintptr_t labels, uintptr_t idx,
           uintptr_t dlogits, int ldd, float scale, uintptr_t stats, uintptr_t probs, uintptr_t pred, uintptr_t s) {
          gpu::XentParams p;
          p.M = M; p.N = N; p.logits = ptr<const float>(logits); p.ldl = ldl;
          p.labels = ptr<const uint8_t>(labels); p.labels_idx = ptr<const int32_t>(idx);
          p.dlogits = ptr<void>(dlogits); p.ldd = ldd; p.scale = scale;
          p.stats = ptr<unsigned long long>(stats); p.probs = ptr<float>(probs); p.pred = ptr<int32_t>(pred);
          gpu::softmax_xent(parse_dtype(dt), p, stream_of(s));
        },
        py::arg("dtype"), py::arg("M"), py::arg("N"), py::arg("logits"), py::arg("ldl"), py::arg("labels"),
        py::arg("idx") = 0, py::arg("dlogits") = 0, py::arg("ldd") = 0, py::arg("scale") = 1.f, py::arg("stats") = 0,
        py::arg("probs") = 0, py::arg("pred") = 0, py::arg("stream") = 0);
  k.def(
      "fc_tall",
      [](int M, int N, int K, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t bias, int act, uintptr_t out,
         int ldo, uintptr_t s, bool f32) {
        gpu::FcTallParams p;
        p.M = M; p.N = N; p.K = K; p.f32 = f32;
        p.A = reinterpret_cast<const void*>(A); p.lda = lda;
        p.W = reinterpret_cast<const void*>(W); p.ldw = ldw;
        p.bias = reinterpret_cast<const float*>(bias); p.act = act;
        p.out = reinterpret_cast<void*>(out); p.ldo = ldo;
        gpu::fc_tall(p, stream_of(s));
      },
      py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"), py::arg("W"), py::arg("ldw"),
      py::arg("bias"), py::arg("act"), py::arg("out"), py::arg("ldo"), py::arg("stream") = 0, py::arg("f32") = false);
  k.def(
      "fc_wres",
      [](int M, int N, int K, uintptr_t A, int lda, uintptr_t W, int ldw, int act, uintptr_t aux, int ldaux,
         uintptr_t out, int ldo, uintptr_t s, bool f32) {
        gpu::FcTallParams p;
        p.M = M; p.N = N; p.K = K; p.f32 = f32;
        p.A = reinterpret_cast<const void*>(A); p.lda = lda;
        p.W = reinterpret_cast<const void*>(W); p.ldw = ldw;
        p.act = act;
        p.out = reinterpret_cast<void*>(out); p.ldo = ldo;
        gpu::fc_wres(p, reinterpret_cast<const void*>(aux), ldaux, stream_of(s));
      },
      py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"), py::arg("W"), py::arg("ldw"),
      py::arg("act"), py::arg("aux"), py::arg("ldaux"), py::arg("out"), py::arg("ldo"), py::arg("stream") = 0,
      py::arg("f32") = false);
  k.def("fc_wres_supported", &gpu::fc_wres_supported, py::arg("f32"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("act"));
  k.def(
      "cu_hold", [](int nwg, int lds_bytes, double usec, uintptr_t s) { gpu::cu_hold(nwg, lds_bytes, usec, stream_of(s)); },
      py::arg("nwg"), py::arg("lds_bytes"), py::arg("usec"), py::arg("stream") = 0);
  k.attr("EPI_BIAS_ACT") = (int)gpu::EPI_BIAS_ACT;
  k.attr("EPI_LOGITS") = (int)gpu::EPI_LOGITS;
  k.attr("EPI_DACT") = (int)gpu::EPI_DACT;
  k.attr("EPI_PARTIAL") = (int)gpu::EPI_PARTIAL;
  k.attr("ACT_NONE") = (int)gpu::ACT_NONE;
  k.attr("ACT_RELU") = (int)gpu::ACT_RELU;
  k.attr("ACT_TANH") = (int)gpu::ACT_TANH;

  m.def("dlpack_wrap", &dlpack_wrap, py::arg("ptr"), py::arg("numel"), py::arg("dtype"), py::arg("device"));
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("synchronize", []() {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) throw Error(std::string("HIP error: ") + hipGetErrorString(e));
  });
}
