// comm.hpp -- the multi-GPU exchange of one rank's sharded apply inside the library
// (DESIGN.md §5): the tier-0 root all-gather between the two phases and the halo
// all-to-all of the iterate, enqueued by the library itself on the apply's stream, so
// one C call runs a whole sharded block matvec with no host round trip between its
// phases.  Two implementations of the three collectives it needs:
//   RCCL       -- ncclAllGather / grouped ncclSend+ncclRecv / ncclAllReduce on the
//                 stream (RCCL over xGMI; the library binds the process's librccl.so.1
//                 at run time, the copy PyTorch-ROCm already loaded);
//   callbacks  -- caller-supplied functions (aniso_collectives): a host-staged
//                 transport such as gloo, which rehearses the same orchestration with
//                 several ranks sharing one GPU (RCCL refuses two ranks per device).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "../../include/aniso_mi355x.h"

namespace aniso {

class Collectives {
  public:
    virtual ~Collectives() = default;
    // recv (nranks x count doubles) = every rank's send (count doubles); device buffers
    virtual void allgather(const double* send, double* recv, size_t count, hipStream_t s) = 0;
    // per-peer variable all-to-all of doubles (device buffers, host counts / offsets)
    virtual void alltoallv(const double* send, const int64_t* scount, const int64_t* soff, double* recv,
                           const int64_t* rcount, const int64_t* roff, hipStream_t s) = 0;
    // buf (count doubles, device) = its sum over the ranks
    virtual void allreduce(double* buf, size_t count, hipStream_t s) = 0;
    // development: no peers (make_loopback_collectives); commInit then builds the
    // peers' exchange lists from their plans instead of gathering them
    virtual bool loopback() const { return false; }
    int nranks = 1, rank = 0;
};

std::unique_ptr<Collectives> make_rccl_collectives(const unsigned char* uniqueId, int nranks, int rank);
std::unique_ptr<Collectives> make_callback_collectives(const aniso_collectives& c, int nranks, int rank);
// development: a rank's schedule with the other ranks' data left out (timing on one GPU)
std::unique_ptr<Collectives> make_loopback_collectives(int nranks, int rank);
void rccl_unique_id(unsigned char* out);

}  // namespace aniso
