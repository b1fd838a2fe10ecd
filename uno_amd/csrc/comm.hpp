// comm.hpp -- inter-GPU transport of the distributed (subtree-partitioned) factorization.
//
// independent elimination subtrees are factored on different GPUs; the only data
// exchanges are the contribution blocks (factor) and update vectors (forward solve) of the subtree
// roots, sent to the rank that owns the top of the assembly tree, the broadcast of the top rows of
// the solution (backward solve), and small reductions (equilibration of the separator rows, the
// null-pivot norm, inertia counters).  Three implementations:
//   RcclTransport  -- one process per GPU, RCCL point-to-point + collectives over xGMI;
//   LocalTransport -- several handles in one process (threads), device-to-device copies; used to run
//                     and test the distributed algorithm on a single GPU;
//   HostTransport  -- one process per rank, the caller's host-side exchange (callbacks) through
//                     page-locked staging buffers.
// The reference has no multi-process path (MUMPS par=1, MUMPSSolver.cpp:17); this is new.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

namespace ukkt {

enum class RedOp { SumU64, MaxU64, MaxF64, SumF64 };

class Transport {
public:
    virtual ~Transport() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // point-to-point, stream-ordered; a batch of sends/recvs is bracketed by group_begin/group_end
    virtual hipError_t group_begin() { return hipSuccess; }
    virtual hipError_t group_end() { return hipSuccess; }
    virtual hipError_t send(const void* buf, size_t bytes, int peer, hipStream_t s) = 0;
    virtual hipError_t recv(void* buf, size_t bytes, int peer, hipStream_t s) = 0;
    // in-place all-reduce of `count` elements of a device buffer
    virtual hipError_t allreduce(void* buf, size_t count, RedOp op, hipStream_t s) = 0;
    // in-place broadcast of a device buffer from `root`
    virtual hipError_t broadcast(void* buf, size_t bytes, int root, hipStream_t s) = 0;
    virtual std::string describe() const = 0;
};

// Local (in-process) group: create once with the world size, attach one handle per rank; every rank
// must be driven by its own host thread (collectives block until all ranks have arrived).
struct LocalGroup;
LocalGroup* local_group_create(int world);
void local_group_destroy(LocalGroup* g);
Transport* make_local_transport(LocalGroup* g, int rank);

// Host-staged: the caller's exchange on host buffers (callbacks, e.g. torch.distributed over gloo or
// MPI); device data goes through page-locked staging buffers.  For one process per rank when RCCL is
// not available (several ranks on one GPU: RCCL refuses duplicate devices), and for tests of the
// multi-process orchestration.
struct HostComm {
    void* ctx;
    int (*send)(void* ctx, const void* buf, size_t bytes, int peer);
    int (*recv)(void* ctx, void* buf, size_t bytes, int peer);
    int (*group_end)(void* ctx);
    int (*allreduce)(void* ctx, void* buf, size_t count, int op);
    int (*broadcast)(void* ctx, void* buf, size_t bytes, int root);
};
Transport* make_host_transport(const HostComm& cb, int rank, int world);

// Tracing decorator (option comm_trace, tests): forwards every call to `inner` (owned) and records it as
// (op, peer / root, bytes, reduction op), op: 0 send, 1 recv, 2 allreduce, 3 broadcast, 4 group_begin,
// 5 group_end.  The library issues the same sequence whatever the transport, so a trace taken through the
// host or local transport is the sequence the RCCL transport would see (ncclSend / ncclRecv sizes, peers,
// grouping, collective order).
Transport* make_tracing_transport(Transport* inner);
// stream-order probe of a tracing transport: called with the stream of every send / recv / collective, it returns
// (the call is on the handle's main stream, the side streams whose launches are not yet joined into it as a bit
// mask); the transport records it as an op 6 record (peer = on-main flag, bytes = mask) right before the call.  An
// exchange is ordered after every producing launch iff it is on the main stream with mask 0.
void comm_trace_set_probe(Transport* t, std::function<std::pair<int, int>(hipStream_t)> probe);
// the records of a tracing transport (empty for any other transport); clear: start a new trace
bool comm_trace_records(Transport* t, std::vector<int64_t>& out, bool clear);

// RCCL: unique id from rank 0 (NCCL_UNIQUE_ID_BYTES = 128), then every rank attaches with it.
int rccl_unique_id(unsigned char out[128]);
Transport* make_rccl_transport(const unsigned char id[128], int rank, int world, int device, std::string& err);

}  // namespace ukkt
