// comm.h -- the collectives of the band frame (csrc/band_frame.cpp, include/rsd.h rsd_comm_*).
//
// each GPU renders a screen band; the frame needs three exchanges per rank -- an
// all-gather of a small count row, point-to-point transfers of the sparse interval / SD halos and an
// all-gather of the AO bands (the reference renders on one GPU; its single-GPU geometry is
// SVAO.cpp:700-723, VAOData.slang:44).  Two implementations behind one interface, both
// stream-ordered (no host wait for the GPU):
//   RcclComm   one process per GPU: ncclAllGather / ncclSend / ncclRecv inside ncclGroupStart/End on
//              the caller's stream (librccl.so.1, the copy torch already loaded when there is one);
//   LocalComm  `world` host threads of one process sharing a GPU (one stream each): device-to-device
//              copies ordered by events, a rendezvous on a condition variable -- the same stream
//              semantics, for one-GPU tests of the whole N > 1 frame.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rsd.h"

namespace rsd {

struct Xfer {
    void* buf;
    uint64_t bytes;
    uint32_t peer;
};

class Comm {
public:
    virtual ~Comm() = default;
    virtual uint32_t kind() const = 0;
    uint32_t rank() const { return rank_; }
    uint32_t world() const { return world_; }
    // recv = world x bytes: rank k's send at offset k x bytes
    virtual rsd_status all_gather(const void* send, void* recv, uint64_t bytes, hipStream_t s) = 0;
    // one group of point-to-point transfers; both sides agree on every size beforehand
    virtual rsd_status exchange(const Xfer* sends, uint32_t ns, const Xfer* recvs, uint32_t nr, hipStream_t s) = 0;

protected:
    uint32_t rank_ = 0, world_ = 1;
};

// a batch of device-to-device byte copies in one launch (halo.hip)
struct CopySeg {
    const void* src;
    void* dst;
    uint64_t bytes;
};
// zero (optional): zero_n 64-bit words set to 0 by the same launch (a side job, e.g. the band frame's count row)
rsd_status copy_segments(const CopySeg* segs, uint32_t n, hipStream_t s, uint64_t* zero = nullptr, uint32_t zero_n = 0);
constexpr uint32_t kMaxCopySegs = 16;

}  // namespace rsd

struct rsd_comm {
    rsd::Comm* impl = nullptr;
};
