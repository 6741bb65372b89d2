// tsdf_internal.h -- library-internal entry points shared between the engine and the group layer
// (not part of the public C ABI in include/disinfect_tsdf.h).
#pragma once
#include <stdint.h>

#include "disinfect_tsdf.h"

extern "C" {
// tsdf_integrate_shard_pipe whose update writes this shard's candidate slot into each of the ndst
// slots listed at dsts_dev (a device array; dsts_host: the same pointers on the host) -- this shard's
// slot of every shard's inbox -- instead of one outgoing slot (tsdf_group_*)
int tsdf_integrate_shard_pipe_fanout(tsdf_engine* e, const tsdf_frame* f, const tsdf_intrinsics* K,
                                     const tsdf_pose* pose, float max_depth, const void* cands_in,
                                     void* const* dsts_dev, void* const* dsts_host, int ndst, int32_t cand_cap,
                                     int32_t* pending);
// the message tsdf_last_error returns (this thread)
void tsdf_set_last_error(const char* what);
}
