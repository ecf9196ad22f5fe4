// rt_rccl.h — RCCL communicators and the frame gather (rt_rccl.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

namespace rt {

// Communicators over devs (rank q on device devs[q], ncclCommInitAll), made
// once per device list and kept until rccl_release.  0, or -1 with err set.
int rccl_comms(const std::vector<int>& devs, std::string& err);
// ncclGather of `count` doubles from send[q] (on devs[q], stream streams[q])
// into recv on rank 0 (q * count doubles apart), the ranks' calls in one
// group.  Enqueued only (stream-ordered).  0, or -1 with err set.
int rccl_gather(const std::vector<int>& devs, const std::vector<const void*>& send, void* recv, size_t count,
                const std::vector<hipStream_t>& streams, std::string& err);
// Destroys the communicators (rt_shutdown).
void rccl_release();
// "RCCL x.y.z (path)" once loaded.
std::string rccl_describe();

}  // namespace rt
