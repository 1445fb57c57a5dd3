// Native GPU training driver (see trainer.h).
//
// One step = device-side sampling from the rank's shard -> fused forward ->
// softmax-CE -> backward bucket by bucket, each bucket's RCCL all-reduce
// issued on a comm stream as soon as its gradients are final (event
// fork/join, overlapped with the remaining backward) -> SGD + repack.  The
// whole step is captured once into a hipGraph and replayed (the sampler reads
// its step counter from device memory, so replays draw fresh indices).
#include "trainer.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <memory>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "kernels.h"
#include "mcc/cpu_net.h"
#include "mcc/engine.h"
#include "mcc/io.h"

namespace mcc {

#define HIPCHK(expr)                                                                        \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) throw Error(std::string("HIP: ") + hipGetErrorString(_e) + " @ " + #expr); \
  } while (0)

namespace {

struct DevBuf {
  void* p = nullptr;
  explicit DevBuf(size_t bytes) { HIPCHK(hipMalloc(&p, bytes ? bytes : 1)); }
  ~DevBuf() { if (p) (void)hipFree(p); }
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

// Host -> device upload of a dataset through two pinned 32 MiB staging
// buffers (a pageable hipMemcpy is staged by the runtime one small chunk at a
// time): memcpy into one buffer while the DMA engine drains the other.
void upload_pinned(void* dst, const void* src, size_t bytes) {
  constexpr size_t kChunk = 32u << 20;
  if (bytes <= (1u << 20)) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return;
  }
  char* pin[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  hipStream_t s = nullptr;
  auto cleanup = [&] {
    if (s) (void)hipStreamSynchronize(s);
    for (int i = 0; i < 2; ++i) {
      if (pin[i]) (void)hipHostFree(pin[i]);
      if (done[i]) (void)hipEventDestroy(done[i]);
    }
    if (s) (void)hipStreamDestroy(s);
  };
  try {
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&pin[i]), kChunk, hipHostMallocDefault));
      HIPCHK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
    }
    for (size_t off = 0, k = 0; off < bytes; off += kChunk, ++k) {
      const int b = (int)(k & 1);
      const size_t len = std::min(kChunk, bytes - off);
      if (k >= 2) HIPCHK(hipEventSynchronize(done[b]));  // buffer b's previous copy has drained
      std::memcpy(pin[b], static_cast<const char*>(src) + off, len);
      HIPCHK(hipMemcpyAsync(static_cast<char*>(dst) + off, pin[b], len, hipMemcpyHostToDevice, s));
      HIPCHK(hipEventRecord(done[b], s));
    }
    HIPCHK(hipStreamSynchronize(s));
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
}

struct PhaseTimer {
  bool on;
  hipEvent_t ev[5];
  double ms[4] = {0, 0, 0, 0};
  int n = 0;
  explicit PhaseTimer(bool enabled) : on(enabled) {
    if (on) for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  }
  ~PhaseTimer() {
    if (on) for (auto& e : ev) (void)hipEventDestroy(e);
  }
  // hipEvent per-phase timing plus a roctx range per phase, so a
  // `rocprofv3 --marker-trace` run attributes kernels to fwd/bwd/sync/update
  // (the reference has no instrumentation at all).
  static constexpr const char* kPhase[4] = {"mcc.forward+loss", "mcc.backward+allreduce", "mcc.allreduce_join", "mcc.sgd"};
  void mark(int i, hipStream_t s) {
    if (!on) return;
    HIPCHK(hipEventRecord(ev[i], s));
    if (i > 0) roctxRangePop();
    if (i < 4) roctxRangePush(kPhase[i]);
  }
  void collect() {
    if (!on) return;
    HIPCHK(hipEventSynchronize(ev[4]));
    for (int i = 0; i < 4; ++i) {
      float t = 0;
      HIPCHK(hipEventElapsedTime(&t, ev[i], ev[i + 1]));
      ms[i] += t;
    }
    ++n;
  }
};

}  // namespace

int run_gpu_training(const CliArgs& a, Comm& comm, const char* program) {
  const int rank = comm.rank(), world = comm.size();
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (ndev < 1) { std::fprintf(stderr, "%s: no GPU\n", program); return 111; }
  HIPCHK(hipSetDevice(comm.local_rank() % ndev));
  MCC_CHECK(a.dtype == "bf16" || a.dtype == "fp32",
            "--dtype " + a.dtype + ": the data-parallel engine runs bf16 | fp32 (fp64: cnn_hip --dtype fp64)");
  const DType dt = a.dtype == "fp32" ? DType::F32 : DType::BF16;

  // ---- model + initial weights (identical on every rank, then broadcast) ----
  ModelSpec spec;
  std::vector<double> p64;
  try {
    if (!a.load.empty()) spec = load_weights(a.load, p64);
    else {
      spec = make_model(a.model);
      p64.resize(spec.nparams);
      init_params(spec, p64.data(), a.seed, InitMode::GlibcRef);
    }
  } catch (const Error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 111;
  }

  // ---- data (IDX, device resident) ----
  IdxFile tr_img, tr_lab, te_img, te_lab;
  try {
    tr_img = load_idx(a.train_images, spec);
    tr_lab = load_idx(a.train_labels, spec);
  } catch (const Error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 111;
  }
  const int64_t in_nodes = spec.input_nodes();
  if (tr_img.item_size() != in_nodes || tr_lab.count() < tr_img.count()) {
    std::fprintf(stderr, "train set shape does not match the model input\n");
    return 111;
  }
  int64_t N = tr_img.count();
  if (a.max_train > 0 && a.max_train < N) N = a.max_train;
  // contiguous per-rank shard (cnnmpi.c:457-458)
  const int64_t shard_lo = N / world * rank, shard_hi = N / world * (rank + 1);
  if (world > 1) std::fprintf(stderr, "%d %lld %lld\n", rank, (long long)shard_lo, (long long)shard_hi);

  // Each rank trains b = floor(B / world) samples per step: the effective
  // global batch (the SGD mean, the sample count and img/s) is b * world.
  const int b = std::max(1, a.batch / world);
  const int B_eff = b * world;
  if (rank == 0 && B_eff != a.batch)
    std::fprintf(stderr, "note: --batch %d is not a multiple of %d ranks; global batch %d\n", a.batch, world, B_eff);
  // evaluation batch: >= 1024 small images per forward; large images (VGG
  // @224: ~50 MB of activations per image) evaluate at the training batch
  const int eval_b = spec.input().H * spec.input().W > 64 * 64 ? b : std::max(b, 1024);
  GpuNet net(spec, dt, eval_b);
  {
    std::vector<float> p32(p64.begin(), p64.end());
    net.set_params(p32.data());
  }
  DevBuf d_img((size_t)N * in_nodes), d_lab((size_t)N);
  upload_pinned(d_img.p, tr_img.data.data(), (size_t)N * in_nodes);
  upload_pinned(d_lab.p, tr_lab.data.data(), (size_t)N);
  DevBuf d_idx(4 * (size_t)eval_b), d_step(8);
  DevBuf d_red(64);  // log / timing / exit-code reductions (no allocation in the loop)
  // pinned host side of those reductions: floats [0, 16), doubles from byte 64.
  // Every device->host copy lands here and is read only after an event the
  // watchdog waits on (a pageable hipMemcpyAsync would block, unbounded).
  float* h_red = nullptr;
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h_red), 128, hipHostMallocDefault));
  std::unique_ptr<float, hipError_t (*)(void*)> h_red_guard(h_red, hipHostFree);
  double* h_dbl = reinterpret_cast<double*>(h_red + 16);
  HIPCHK(hipMemset(d_step.p, 0, 8));

  // Comm stream C from the high-priority pool: HIP spreads streams over
  // GPU_MAX_HW_QUEUES hardware queues per priority, so a normal-priority C
  // can share S's queue and serialise every all-reduce behind backward.
  int prio_lo = 0, prio_hi = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  hipStream_t S, C;
  auto make_streams = [&] {
    HIPCHK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithPriority(&C, hipStreamNonBlocking, prio_hi));
  };
  make_streams();
  const bool coll = comm.collective();
  // identical weights on every rank (fixes D6: srand(rank), no broadcast)
  comm.broadcast_f32(net.params(), net.nparams(), 0, S);
  net.pack(S);
  hipEvent_t ev_sync;
  HIPCHK(hipEventCreateWithFlags(&ev_sync, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ev_sync, S));
  comm.wait(ev_sync);

  const auto buckets = net.buckets((int64_t)(a.bucket_mb * (1 << 20)));
  std::vector<hipEvent_t> ev_b(buckets.size());
  hipEvent_t ev_join;
  for (auto& e : ev_b) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // per-bucket SGD (default at world > 1): bucket k's parameters are updated
  // as soon as ITS all-reduce has landed, so the FC update of LeNet-5 / the
  // reference model overlaps the conv block's (last, small) collective
  const bool split_sgd = coll && buckets.size() > 1 && (a.split_sgd == 1 || (a.split_sgd < 0 && world > 1));
  std::vector<hipEvent_t> ev_done(buckets.size());
  for (auto& e : ev_done) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
  // The loss is scaled by 1/(b*world) and the bucket all-reduce sums over
  // ranks, so the update uses the global-batch mean.  (ncclAvg is a
  // pre-multiplied sum in RCCL: at one rank it still streams the whole bucket
  // through a "oneRankReduce" kernel, while an in-place one-rank SUM is elided.)
  const float grad_scale = 1.0f / ((float)b * (float)world);
  PhaseTimer timer(a.profile);
  const bool seq_sampler = a.sampler == "seq";

  auto step = [&](bool timed) {
    if (seq_sampler)
      gpu::seq_sample_indices(d_idx.as<int32_t>(), b, (int64_t)rank * b, B_eff, N, d_step.as<uint64_t>(), S);
    else
      gpu::sample_indices(d_idx.as<int32_t>(), b, shard_lo, shard_hi, a.seed * 7919ull + rank, d_step.as<uint64_t>(), S);
    if (timed) timer.mark(0, S);
    net.forward(d_img.as<uint8_t>(), d_idx.as<int32_t>(), b, S);
    net.loss(d_lab.as<uint8_t>(), d_idx.as<int32_t>(), grad_scale, true, S);
    if (timed) timer.mark(1, S);
    for (size_t k = 0; k < buckets.size(); ++k) {
      net.backward(buckets[k].stage_hi, buckets[k].stage_lo, S);
      if (coll) {
        // fork: the bucket's all-reduce runs on the comm stream C while S
        // continues with the earlier stages' backward
        HIPCHK(hipEventRecord(ev_b[k], S));
        HIPCHK(hipStreamWaitEvent(C, ev_b[k], 0));
        comm.allreduce_sum_f32(net.grads() + buckets[k].off, buckets[k].count, C);
        if (split_sgd) HIPCHK(hipEventRecord(ev_done[k], C));
      }
    }
    if (timed) timer.mark(2, S);
    if (split_sgd) {
      // join bucket by bucket (the comm stream runs them in issue order)
      for (size_t k = 0; k < buckets.size(); ++k) {
        HIPCHK(hipStreamWaitEvent(S, ev_done[k], 0));
        if (timed && k == 0) timer.mark(3, S);
        net.sgd_range((float)a.lr, (float)a.momentum, (float)a.weight_decay, buckets[k].off, buckets[k].count, S);
      }
    } else {
      if (coll) {  // join before the update
        HIPCHK(hipEventRecord(ev_join, C));
        HIPCHK(hipStreamWaitEvent(S, ev_join, 0));
      }
      if (timed) timer.mark(3, S);
      net.sgd((float)a.lr, (float)a.momentum, (float)a.weight_decay, S);
    }
    gpu::advance_counter(d_step.as<uint64_t>(), S);
    if (timed) timer.mark(4, S);
  };

  const int64_t total = (int64_t)a.epochs * N;
  const int64_t steps = (total + B_eff - 1) / B_eff;
  if (rank == 0) std::fprintf(stderr, "training...\n");
  net.zero_stats(S);

  // Capture one step into a hipGraph (skipped with --profile: timers need
  // host-visible event records between phases).  With RCCL the captured
  // graph holds the bucket fork/join and the ncclAllReduce nodes.
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  bool use_graph = !a.profile && steps > 2 && !a.no_graph;
  if (a.momentum != 0.0) net.ensure_momentum();  // no allocation inside capture
  if (use_graph) {
    HIPCHK(hipStreamSynchronize(S));
    if (hipStreamBeginCapture(S, hipStreamCaptureModeRelaxed) == hipSuccess) {
      bool ok = true;
      try { step(false); } catch (const Error&) { ok = false; }
      hipError_t e = hipStreamEndCapture(S, &graph);
      if (!ok || e != hipSuccess || hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0) != hipSuccess) {
        use_graph = false;
        (void)hipGetLastError();
        // a failed capture can leave the stream unusable: start from fresh streams
        (void)hipStreamDestroy(S);
        (void)hipStreamDestroy(C);
        make_streams();
        if (rank == 0) std::fprintf(stderr, "note: hipGraph capture unavailable, running eagerly\n");
      }
    } else {
      use_graph = false;
      (void)hipGetLastError();
    }
  }

  // At most kInFlight steps are queued ahead of the host: before enqueueing
  // step it, the host waits (bounded, watchdog) for step it - kInFlight.  A
  // hung collective is then detected within the deadline instead of the
  // host blocking forever inside a full launch queue.
  constexpr int kInFlight = 4;
  hipEvent_t ev_step[kInFlight];
  for (auto& e : ev_step) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  int64_t seen = 0, last_log = 0;
  // fault injection for the rank-death tests (same variables as train.py):
  // MCC_FAULT_RANK=r MCC_FAULT_STEP=k makes rank r die abruptly before step k
  const char* fr = std::getenv("MCC_FAULT_RANK");
  const char* fs = std::getenv("MCC_FAULT_STEP");
  const int64_t fault_step = fr && fs && std::atoi(fr) == rank ? std::atoll(fs) : -1;
  for (int64_t it = 0; it < steps; ++it) {
    if (it == fault_step) {
      std::fprintf(stderr, "rank %d: injected fault before step %lld\n", rank, (long long)it);
      std::_Exit(9);
    }
    if (it >= kInFlight) comm.wait(ev_step[it % kInFlight]);
    if (use_graph) HIPCHK(hipGraphLaunch(gexec, S));
    else step(a.profile);
    HIPCHK(hipEventRecord(ev_step[it % kInFlight], S));
    if (a.profile) timer.collect();
    const int64_t prev = seen;
    seen += B_eff;
    // log at i = 0 and every log_every samples (cnn.c:470-473)
    const int64_t mark = (prev + a.log_every - 1) / a.log_every * a.log_every;
    if (!a.quiet && (mark < seen || it == steps - 1)) {
      // [mse sum of this rank, samples of this rank]; summed over ranks
      float* d = d_red.as<float>();
      gpu::stats_to_f32(net.stats(), d + 2, S);  // d[3] = this rank's mse sum
      HIPCHK(hipMemcpyAsync(d, d + 3, 4, hipMemcpyDeviceToDevice, S));
      h_red[1] = (float)((seen - last_log) / world);
      HIPCHK(hipMemcpyAsync(d + 1, h_red + 1, 4, hipMemcpyHostToDevice, S));
      comm.allreduce_sum_f32(d, 2, S);
      HIPCHK(hipMemcpyAsync(h_red, d, 8, hipMemcpyDeviceToHost, S));
      HIPCHK(hipEventRecord(ev_sync, S));
      comm.wait(ev_sync);
      if (rank == 0 && mark < seen)
        std::fprintf(stderr, "i=%lld, error=%.4f\n", (long long)mark, h_red[0] / std::max(1.0f, h_red[1]));
      net.zero_stats(S);
      last_log = seen;
    }
  }
  HIPCHK(hipEventRecord(ev_sync, S));
  comm.wait(ev_sync);
  double train_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (coll) {  // the slowest rank's time
    double* d = d_red.as<double>();
    h_dbl[0] = train_s;
    HIPCHK(hipMemcpyAsync(d, h_dbl, 8, hipMemcpyHostToDevice, S));
    comm.allreduce_max_f64(d, 1, S);
    HIPCHK(hipMemcpyAsync(h_dbl + 1, d, 8, hipMemcpyDeviceToHost, S));
    HIPCHK(hipEventRecord(ev_sync, S));
    comm.wait(ev_sync);
    train_s = h_dbl[1];
  }
  for (auto& e : ev_step) (void)hipEventDestroy(e);
  if (gexec) (void)hipGraphExecDestroy(gexec);
  if (graph) (void)hipGraphDestroy(graph);

  // ---- test (rank 0; every rank holds identical weights) ----
  int rc = 0;
  int64_t ntests = 0, ncorrect = 0;
  double test_s = 0;
  // --save PATH saves rank 0's weights; a PATH containing "{rank}" makes
  // every rank save its own replica (the multi-rank tests compare them)
  const size_t rk = a.save.find("{rank}");
  if (rank != 0 && rk != std::string::npos) {
    std::vector<float> p32(net.nparams());
    net.get_params(p32.data());
    std::vector<double> pd(p32.begin(), p32.end());
    std::string path = a.save;
    path.replace(rk, 6, std::to_string(rank));
    try {
      save_weights(path, spec, pd.data());
    } catch (const Error& e) {
      std::fprintf(stderr, "%s\n", e.what());
      rc = 111;
    }
  }
  if (rank == 0) {
    try {
      te_img = load_idx(a.test_images, spec);
      te_lab = load_idx(a.test_labels, spec);
      if (te_img.item_size() != in_nodes || te_lab.count() < te_img.count())
        throw Error("test set shape does not match the model input");
      std::fprintf(stderr, "testing...\n");
      ntests = te_img.count();
      DevBuf t_img((size_t)ntests * in_nodes), t_lab((size_t)ntests);
      upload_pinned(t_img.p, te_img.data.data(), (size_t)ntests * in_nodes);
      upload_pinned(t_lab.p, te_lab.data.data(), (size_t)ntests);
      net.zero_stats(S);
      const auto t1 = std::chrono::steady_clock::now();
      for (int64_t i = 0; i < ntests; i += eval_b) {
        const int nb = (int)std::min<int64_t>(eval_b, ntests - i);
        gpu::iota_i32(d_idx.as<int32_t>(), nb, i, S);
        net.forward(t_img.as<uint8_t>(), d_idx.as<int32_t>(), nb, S);
        net.loss(t_lab.as<uint8_t>(), d_idx.as<int32_t>(), 1.f, false, S);
        for (int64_t j = i; j < i + nb; ++j)
          if (j % 1000 == 0) std::fprintf(stderr, "i=%lld\n", (long long)j);
      }
      gpu::stats_to_f32(net.stats(), d_red.as<float>(), S);
      HIPCHK(hipMemcpyAsync(h_red, d_red.as<float>(), 12, hipMemcpyDeviceToHost, S));
      HIPCHK(hipStreamSynchronize(S));
      test_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
      ncorrect = (int64_t)std::llround(h_red[2]);
      std::fprintf(stderr, "ntests=%lld, ncorrect=%lld\n", (long long)ntests, (long long)ncorrect);
      if (!a.save.empty()) {
        std::vector<float> p32(net.nparams());
        net.get_params(p32.data());
        std::vector<double> pd(p32.begin(), p32.end());
        std::string path = a.save;
        if (rk != std::string::npos) path.replace(rk, 6, "0");
        save_weights(path, spec, pd.data());
      }
    } catch (const Error& e) {
      std::fprintf(stderr, "%s\n", e.what());
      rc = 111;
    }
  }
  // every rank leaves with rank 0's verdict (a failed test phase must not
  // leave the others in the final barrier; advisor finding, D9)
  if (coll) {
    // the other ranks wait here while rank 0 evaluates and saves: the longer
    // test-phase deadline, not the per-collective one
    double* d = d_red.as<double>();
    h_dbl[0] = rc;
    HIPCHK(hipMemcpyAsync(d, h_dbl, 8, hipMemcpyHostToDevice, S));
    comm.allreduce_max_f64(d, 1, S);
    HIPCHK(hipMemcpyAsync(h_dbl + 1, d, 8, hipMemcpyDeviceToHost, S));
    HIPCHK(hipEventRecord(ev_sync, S));
    comm.wait_long(ev_sync);
    rc = (int)h_dbl[1];
  }
  if (rank == 0 && !a.log_json.empty()) {
    FILE* f = a.log_json == "-" ? stdout : std::fopen(a.log_json.c_str(), "w");
    if (f) {
      const double img_s = (double)steps * B_eff / std::max(train_s, 1e-9);
      std::fprintf(f,
                   "{\"program\": \"%s\", \"model\": \"%s\", \"dtype\": \"%s\", \"world\": %d, \"global_batch\": %d, "
                   "\"steps\": %lld, \"train_s\": %.6f, \"train_img_per_s\": %.1f, \"hipgraph\": %s, "
                   "\"comm\": \"%s\", \"buckets\": %d, "
                   "\"test_img_per_s\": %.1f, \"ntests\": %lld, \"ncorrect\": %lld",
                   program, spec.name.c_str(), dtype_name(dt), world, B_eff, (long long)steps, train_s, img_s,
                   use_graph ? "true" : "false", comm.name(), (int)buckets.size(), ntests / std::max(test_s, 1e-9),
                   (long long)ntests, (long long)ncorrect);
      if (timer.on && timer.n > 0)
        std::fprintf(f, ", \"phase_ms\": {\"forward_loss\": %.4f, \"backward_allreduce_issue\": %.4f, "
                        "\"allreduce_wait\": %.4f, \"sgd\": %.4f}",
                     timer.ms[0] / timer.n, timer.ms[1] / timer.n, timer.ms[2] / timer.n, timer.ms[3] / timer.n);
      std::fprintf(f, "}\n");
      if (f != stdout) std::fclose(f);
    }
  }
  comm.barrier();
  for (auto& e : ev_b) (void)hipEventDestroy(e);
  for (auto& e : ev_done) (void)hipEventDestroy(e);
  (void)hipEventDestroy(ev_join);
  (void)hipEventDestroy(ev_sync);
  (void)hipStreamDestroy(S);
  (void)hipStreamDestroy(C);
  return rc;
}

}  // namespace mcc
