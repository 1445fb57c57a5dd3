// Host shared-memory collectives (shm_group.h).  Host-only code: built into
// cnn_dist (HostComm) and the CPU test binary test_comm.
#include "shm_group.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <new>
#include <thread>

#include "mcc/common.h"

namespace mcc {

struct ShmGroup::Header {
  std::atomic<uint64_t> arrive;
  std::atomic<uint64_t> depart;
  std::atomic<int> error;
  std::atomic<uint32_t> ready;  // magic once rank 0 has initialised the header
  uint32_t world;
  uint64_t slot;
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics need lock-free u64");

namespace {
constexpr uint32_t kMagic = 0x4D434321u;
using Clock = std::chrono::steady_clock;
}  // namespace

ShmGroup::ShmGroup(uint64_t token, int rank, int world, size_t slot_bytes, double timeout_s)
    : rank_(rank), world_(world), slot_((slot_bytes + 63) / 64 * 64), timeout_s_(timeout_s) {
  if (world < 1 || rank < 0 || rank >= world) throw Error("ShmGroup: bad rank/world");
  char nm[64];
  std::snprintf(nm, sizeof(nm), "/mcc_%016llx", (unsigned long long)token);
  name_ = nm;
  bytes_ = kHeaderBytes + (size_t)world * slot_;
  const auto deadline = Clock::now() + std::chrono::milliseconds((long long)(timeout_s * 1000));
  int fd = -1;
  if (rank == 0) {
    fd = ::shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw Error("ShmGroup: shm_open(" + name_ + ") failed");
    if (::ftruncate(fd, (off_t)bytes_) != 0) {
      ::close(fd);
      ::shm_unlink(name_.c_str());
      throw Error("ShmGroup: ftruncate failed (is /dev/shm large enough?)");
    }
  } else {
    while (true) {
      fd = ::shm_open(name_.c_str(), O_RDWR, 0600);
      struct stat st {};
      if (fd >= 0 && ::fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes_) break;
      if (fd >= 0) ::close(fd);
      if (Clock::now() >= deadline) throw Error("ShmGroup: timed out attaching " + name_);
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  void* p = ::mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) {
    if (rank == 0) ::shm_unlink(name_.c_str());
    throw Error("ShmGroup: mmap failed");
  }
  base_ = static_cast<char*>(p);
  if (rank == 0) {
    hdr_ = new (base_) Header();
    hdr_->arrive.store(0);
    hdr_->depart.store(0);
    hdr_->error.store(0);
    hdr_->world = (uint32_t)world;
    hdr_->slot = slot_;
    hdr_->ready.store(kMagic, std::memory_order_release);
  } else {
    hdr_ = reinterpret_cast<Header*>(base_);
    while (hdr_->ready.load(std::memory_order_acquire) != kMagic) {
      if (Clock::now() >= deadline) {
        ::munmap(base_, bytes_);
        throw Error("ShmGroup: timed out waiting for rank 0 to initialise " + name_);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (hdr_->world != (uint32_t)world || hdr_->slot != slot_) {
      ::munmap(base_, bytes_);
      throw Error("ShmGroup: segment geometry mismatch");
    }
  }
  const bool ok = barrier();  // everyone attached
  if (rank == 0) ::shm_unlink(name_.c_str());
  if (!ok) {
    ::munmap(base_, bytes_);
    throw Error("ShmGroup: timed out waiting for all ranks to attach");
  }
}

ShmGroup::~ShmGroup() {
  if (base_) ::munmap(base_, bytes_);
}

void ShmGroup::poison() {
  if (hdr_) hdr_->error.store(1, std::memory_order_release);
}

bool ShmGroup::poisoned() const { return hdr_ && hdr_->error.load(std::memory_order_acquire) != 0; }

bool ShmGroup::wait_count(std::atomic<uint64_t>& c, uint64_t target) {
  const auto deadline = Clock::now() + std::chrono::milliseconds((long long)(timeout_s_ * 1000));
  for (int spin = 0;; ++spin) {
    if (c.load(std::memory_order_acquire) >= target) return true;
    if (hdr_->error.load(std::memory_order_acquire)) return false;
    if (spin > 256) {
      if ((spin & 255) == 0 && Clock::now() >= deadline) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

template <class F>
bool ShmGroup::run(const void* in, size_t bytes, F&& combine) {
  if (bytes > slot_) throw Error("ShmGroup: message larger than the slot");
  const uint64_t k = ++seq_;
  if (bytes) std::memcpy(slot(rank_), in, bytes);
  hdr_->arrive.fetch_add(1, std::memory_order_acq_rel);
  if (!wait_count(hdr_->arrive, k * (uint64_t)world_)) return false;
  combine();
  hdr_->depart.fetch_add(1, std::memory_order_acq_rel);
  return wait_count(hdr_->depart, k * (uint64_t)world_);
}

bool ShmGroup::sum_f32(const float* in, float* out, size_t n) {
  return run(in, n * sizeof(float), [&] {
    const float* s0 = reinterpret_cast<const float*>(slot(0));
    for (size_t i = 0; i < n; ++i) {
      float acc = s0[i];
      for (int r = 1; r < world_; ++r) acc += reinterpret_cast<const float*>(slot(r))[i];
      out[i] = acc;
    }
  });
}

bool ShmGroup::max_f64(const double* in, double* out, size_t n) {
  return run(in, n * sizeof(double), [&] {
    for (size_t i = 0; i < n; ++i) {
      double m = reinterpret_cast<const double*>(slot(0))[i];
      for (int r = 1; r < world_; ++r) {
        const double v = reinterpret_cast<const double*>(slot(r))[i];
        m = v > m || v != v ? v : m;  // NaN wins, as a verdict must not hide it
      }
      out[i] = m;
    }
  });
}

bool ShmGroup::broadcast(const void* in, void* out, size_t bytes, int root) {
  return run(in, bytes, [&] { std::memmove(out, slot(root), bytes); });
}

bool ShmGroup::barrier() {
  return run(nullptr, 0, [] {});
}

}  // namespace mcc
