// HostComm: the Comm of `cnn_dist --comm host` -- several ranks on ONE GPU
// (RCCL refuses two ranks per device), collectives staged through host shared
// memory (shm_group.h).  It exists to execute the multi-rank driver paths
// (TCP bootstrap at world > 1, per-rank shards and sampler ranges, bucketed
// fork/join with graph capture, multi-rank log reduction, time / exit-code MAX,
// rank-death detection) on the one-GPU test box; it is not a performance path.
#pragma once

#include <memory>

#include "trainer.h"

namespace mcc {

std::unique_ptr<Comm> make_host_comm(int rank, int world, int local);

}  // namespace mcc
