// TCP rendezvous of the native multi-process drivers: rank 0 serves a small
// blob (the RCCL ncclUniqueId, or the host-comm segment token) to the other
// world-1 ranks.  Every wait is bounded by a deadline, so a rank that never
// shows up (or a rank 0 that died) ends the others with an mcc::Error instead
// of a hang (reference defect D9: cnnmpi.c:443-453 returns early from rank 0
// and leaves the peers blocked in MPI forever).
#pragma once

#include <chrono>
#include <cstddef>
#include <string>

namespace mcc {

struct BootstrapAddr {
  std::string host = "127.0.0.1";
  int port = 29501;
  double timeout_s = 300.0;
};

// From the environment: MASTER_ADDR, MCC_BOOTSTRAP_PORT (else MASTER_PORT + 1),
// MCC_BOOTSTRAP_TIMEOUT (seconds, default 300).
BootstrapAddr bootstrap_addr_from_env();

// Rank 0: serve the n-byte blob to ranks 1..clients on addr.port.  Each
// client identifies itself with its rank first; stray or duplicate
// connections do not count.  Throws mcc::Error if not every rank has been
// served by the deadline.
void serve_blob(const void* blob, size_t n, int clients, const BootstrapAddr& addr);

// Other ranks: connect to addr (retrying until the deadline), send this
// rank's id and receive the n-byte blob.  Throws mcc::Error on timeout.
void fetch_blob(void* blob, size_t n, int rank, const BootstrapAddr& addr);

// Collective form: rank 0 serves `blob` (already filled), others receive it.
inline void bootstrap_blob(void* blob, size_t n, int rank, int world, const BootstrapAddr& addr) {
  if (world <= 1) return;
  if (rank == 0) serve_blob(blob, n, world - 1, addr);
  else fetch_blob(blob, n, rank, addr);
}

}  // namespace mcc
