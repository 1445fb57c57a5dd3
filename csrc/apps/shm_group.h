// Host shared-memory collectives among the processes of one node: the
// reduction core of HostComm (cnn_dist --comm host), which rehearses the
// multi-rank data-parallel driver with several ranks on ONE GPU (RCCL refuses
// two ranks per device).  Not a performance path: every collective is staged
// through host memory.
//
// Segment: POSIX shm "/mcc_<token>" (the random token travels over the TCP
// bootstrap, so a stale segment of an earlier run is never attached), a
// header of monotonic arrive/depart counters and one slot per rank.  One
// collective k (every rank issues the same sequence):
//   copy in -> slot[rank];  arrive += 1;  wait arrive >= k * world
//   out = f(slot[0], slot[1], ..., slot[world-1])   (fixed rank order: the
//         result is bit-identical on every rank)
//   depart += 1;  wait depart >= k * world          (slots reusable)
// Every wait is bounded (timeout_s) and watches a shared error word, so a
// dead or aborting peer ends the others' collectives with `false`.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace mcc {

class ShmGroup {
 public:
  // Rank 0 creates the segment, the others attach (retrying until the
  // deadline); the constructor ends with a barrier, after which rank 0
  // unlinks the name (no /dev/shm leftovers even if a rank dies later).
  // Throws mcc::Error on failure / timeout.
  ShmGroup(uint64_t token, int rank, int world, size_t slot_bytes, double timeout_s);
  ~ShmGroup();
  ShmGroup(const ShmGroup&) = delete;
  ShmGroup& operator=(const ShmGroup&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  size_t slot_bytes() const { return slot_; }

  // in and out may alias; n * element size <= slot_bytes().  Return false on
  // timeout or when a peer has raised the error word.
  bool sum_f32(const float* in, float* out, size_t n);
  bool max_f64(const double* in, double* out, size_t n);
  bool broadcast(const void* in, void* out, size_t bytes, int root);
  bool barrier();
  // Raise the shared error word: every peer's current and next wait fails.
  void poison();
  bool poisoned() const;
  uint64_t collectives() const { return seq_; }

 private:
  struct Header;
  template <class F>
  bool run(const void* in, size_t bytes, F&& combine);
  bool wait_count(std::atomic<uint64_t>& c, uint64_t target);
  char* slot(int r) const { return base_ + kHeaderBytes + (size_t)r * slot_; }

  static constexpr size_t kHeaderBytes = 4096;
  int rank_, world_;
  size_t slot_;
  double timeout_s_;
  std::string name_;
  char* base_ = nullptr;
  size_t bytes_ = 0;
  Header* hdr_ = nullptr;
  uint64_t seq_ = 0;
};

}  // namespace mcc
