// comm.cpp -- rsd_comm: RCCL and in-process communicators of the band frame (comm.h, include/rsd.h).
#include "comm.h"

#include <dlfcn.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "rsd_internal.h"

// RCCL's types only (the functions are resolved at run time: librsd loads without RCCL, and in a process
// that imported torch it binds the librccl.so.1 torch already loaded -- one RCCL per process)
#include <rccl/rccl.h>

namespace rsd {
namespace {

struct Rccl {
    void* so = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mutex;
Rccl g_rccl;

rsd_status rccl_load(const Rccl** out) {
    std::lock_guard<std::mutex> lock(g_rccl_mutex);
    if (!g_rccl.so) {
        void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, when loaded
        if (!so) so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) {
            set_error(std::string("rsd_comm: cannot load librccl.so.1: ") + dlerror());
            return RSD_ERR_UNSUPPORTED;
        }
        Rccl r;
        r.so = so;
        bool ok = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(so, name));
            ok = ok && fn != nullptr;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.AllGather, "ncclAllGather");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.GetErrorString, "ncclGetErrorString");
        if (!ok) {
            set_error("rsd_comm: librccl.so.1 lacks a symbol (ncclSend / ncclRecv / ncclAllGather / ...)");
            return RSD_ERR_UNSUPPORTED;
        }
        g_rccl = r;
    }
    *out = &g_rccl;
    return RSD_OK;
}

rsd_status nccl_fail(const Rccl* r, ncclResult_t e, const char* what) {
    set_error(std::string(what) + ": " + (r && r->GetErrorString ? r->GetErrorString(e) : "RCCL error"));
    return RSD_ERR_HIP;
}

class RcclComm final : public Comm {
public:
    RcclComm(const Rccl* r, ncclComm_t c, uint32_t rank, uint32_t world) : r_(r), c_(c) {
        rank_ = rank;
        world_ = world;
    }
    ~RcclComm() override { (void)r_->CommDestroy(c_); }
    uint32_t kind() const override { return RSD_COMM_RCCL; }

    rsd_status all_gather(const void* send, void* recv, uint64_t bytes, hipStream_t s) override {
        if (bytes == 0) return RSD_OK;
        ncclResult_t e = r_->AllGather(send, recv, bytes, ncclInt8, c_, s);
        return e == ncclSuccess ? RSD_OK : nccl_fail(r_, e, "ncclAllGather");
    }

    rsd_status exchange(const Xfer* sends, uint32_t ns, const Xfer* recvs, uint32_t nr, hipStream_t s) override {
        ncclResult_t e = r_->GroupStart();
        if (e != ncclSuccess) return nccl_fail(r_, e, "ncclGroupStart");
        for (uint32_t i = 0; i < ns && e == ncclSuccess; ++i)
            if (sends[i].bytes) e = r_->Send(sends[i].buf, sends[i].bytes, ncclInt8, (int)sends[i].peer, c_, s);
        for (uint32_t i = 0; i < nr && e == ncclSuccess; ++i)
            if (recvs[i].bytes) e = r_->Recv(recvs[i].buf, recvs[i].bytes, ncclInt8, (int)recvs[i].peer, c_, s);
        const ncclResult_t g = r_->GroupEnd();  // always close the group
        if (e != ncclSuccess) return nccl_fail(r_, e, "ncclSend / ncclRecv");
        return g == ncclSuccess ? RSD_OK : nccl_fail(r_, g, "ncclGroupEnd");
    }

private:
    const Rccl* r_;
    ncclComm_t c_;
};

}  // namespace

// ---- in-process communicator ------------------------------------------------------------------
// A collective is a rendezvous of all ranks under a sequence number: every rank posts what it offers
// (device pointers) with an event recorded on its stream, then reads what it needs from the others'
// posts after making its stream wait for their events, posts a "done" event, and makes its stream wait
// for every reader's done event before the call returns (so a later kernel of the writer cannot
// overwrite a buffer a reader's copy has not consumed yet).  One data and one done event per rank
// suffice: a rank re-records them only in its next collective, which no rank can enter before every
// rank has issued its waits on the previous ones.
struct LocalPost {
    const void* send = nullptr;              // all-gather
    std::vector<Xfer> sends;                 // exchange
    hipEvent_t ev = nullptr;
    bool posted = false;
    hipEvent_t done = nullptr;
    bool finished = false;
};
struct LocalSlot {
    std::vector<LocalPost> p;
    uint32_t left = 0;  // ranks that have not yet left the collective
};

}  // namespace rsd

struct rsd_comm_hub {
    uint32_t world = 0;
    std::mutex m;
    std::condition_variable cv;
    std::map<uint64_t, rsd::LocalSlot> slots;
};

namespace rsd {
namespace {

class LocalComm final : public Comm {
public:
    LocalComm(rsd_comm_hub* hub, uint32_t rank) : hub_(hub) {
        rank_ = rank;
        world_ = hub->world;
    }
    ~LocalComm() override {
        if (ev_) (void)hipEventDestroy(ev_);
        if (done_) (void)hipEventDestroy(done_);
    }
    rsd_status init() {
        RSD_HIP(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
        RSD_HIP(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
        return RSD_OK;
    }
    uint32_t kind() const override { return RSD_COMM_LOCAL; }

    rsd_status all_gather(const void* send, void* recv, uint64_t bytes, hipStream_t s) override {
        LocalPost mine;
        mine.send = send;
        std::vector<LocalPost> got;
        rsd_status st = post_and_wait(mine, s, got);
        if (st != RSD_OK) return st;
        std::vector<CopySeg> segs;
        for (uint32_t k = 0; k < world_; ++k) {
            if (k != rank_) RSD_HIP(hipStreamWaitEvent(s, got[k].ev, 0));
            if (bytes) segs.push_back({got[k].send, static_cast<char*>(recv) + k * bytes, bytes});
        }
        st = copy_all(segs, s);
        if (st != RSD_OK) return st;
        return finish(s);
    }

    rsd_status exchange(const Xfer* sends, uint32_t ns, const Xfer* recvs, uint32_t nr, hipStream_t s) override {
        LocalPost mine;
        mine.sends.assign(sends, sends + ns);
        std::vector<LocalPost> got;
        rsd_status st = post_and_wait(mine, s, got);
        if (st != RSD_OK) return st;
        std::vector<CopySeg> segs;
        for (uint32_t i = 0; i < nr; ++i) {
            const Xfer& r = recvs[i];
            if (!r.bytes) continue;
            if (r.peer >= world_) {
                set_error("rsd_comm_exchange: peer out of range");
                return RSD_ERR_INVALID_ARG;
            }
            const Xfer* src = nullptr;
            for (const Xfer& x : got[r.peer].sends)
                if (x.peer == rank_) src = &x;
            if (!src || src->bytes != r.bytes) {
                set_error("rsd_comm_exchange (local): rank " + std::to_string(rank_) + " expects " +
                          std::to_string(r.bytes) + " bytes from rank " + std::to_string(r.peer) +
                          ", which sends " + std::to_string(src ? src->bytes : 0));
                return RSD_ERR_INVALID_ARG;
            }
            if (r.peer != rank_) RSD_HIP(hipStreamWaitEvent(s, got[r.peer].ev, 0));
            segs.push_back({src->buf, r.buf, r.bytes});
        }
        st = copy_all(segs, s);
        if (st != RSD_OK) return st;
        return finish(s);
    }

private:
    rsd_status copy_all(const std::vector<CopySeg>& segs, hipStream_t s) {
        for (size_t i = 0; i < segs.size(); i += kMaxCopySegs) {
            rsd_status st = copy_segments(segs.data() + i, (uint32_t)std::min<size_t>(kMaxCopySegs, segs.size() - i), s);
            if (st != RSD_OK) return st;
        }
        return RSD_OK;
    }

    rsd_status post_and_wait(LocalPost& mine, hipStream_t s, std::vector<LocalPost>& got) {
        RSD_HIP(hipEventRecord(ev_, s));
        mine.ev = ev_;
        mine.posted = true;
        cur_ = seq_++;
        std::unique_lock<std::mutex> lock(hub_->m);
        LocalSlot& sl = slot_locked(cur_);
        const std::vector<Xfer> keep = mine.sends;
        sl.p[rank_].send = mine.send;
        sl.p[rank_].sends = keep;
        sl.p[rank_].ev = mine.ev;
        sl.p[rank_].posted = true;
        hub_->cv.notify_all();
        const bool ok = hub_->cv.wait_for(lock, std::chrono::seconds(120), [&] {
            for (const LocalPost& p : hub_->slots[cur_].p)
                if (!p.posted) return false;
            return true;
        });
        if (!ok) {
            set_error("rsd_comm (local): rank " + std::to_string(rank_) + " timed out waiting for the other ranks");
            return RSD_ERR_HIP;
        }
        got = hub_->slots[cur_].p;  // copies: the slot is erased by the last rank to leave
        return RSD_OK;
    }

    rsd_status finish(hipStream_t s) {
        RSD_HIP(hipEventRecord(done_, s));
        std::unique_lock<std::mutex> lock(hub_->m);
        LocalSlot& sl = hub_->slots[cur_];
        sl.p[rank_].done = done_;
        sl.p[rank_].finished = true;
        hub_->cv.notify_all();
        const bool ok = hub_->cv.wait_for(lock, std::chrono::seconds(120), [&] {
            for (const LocalPost& p : hub_->slots[cur_].p)
                if (!p.finished) return false;
            return true;
        });
        if (!ok) {
            set_error("rsd_comm (local): rank " + std::to_string(rank_) + " timed out waiting for the readers");
            return RSD_ERR_HIP;
        }
        std::vector<hipEvent_t> done;
        for (uint32_t k = 0; k < world_; ++k)
            if (k != rank_) done.push_back(hub_->slots[cur_].p[k].done);
        if (--hub_->slots[cur_].left == 0) hub_->slots.erase(cur_);
        lock.unlock();
        for (hipEvent_t e : done) RSD_HIP(hipStreamWaitEvent(s, e, 0));
        return RSD_OK;
    }

    LocalSlot& slot_locked(uint64_t seq) {
        auto it = hub_->slots.find(seq);
        if (it == hub_->slots.end()) {
            LocalSlot sl;
            sl.p.resize(world_);
            sl.left = world_;
            it = hub_->slots.emplace(seq, std::move(sl)).first;
        }
        return it->second;
    }

    rsd_comm_hub* hub_;
    hipEvent_t ev_ = nullptr, done_ = nullptr;
    uint64_t seq_ = 0, cur_ = 0;
};

// moves nothing (host-cost probes of one rank's frame, tools/halo_host_profile.py): the all-gather writes
// only the caller's own block, the exchange returns at once
class NullComm final : public Comm {
public:
    NullComm(uint32_t rank, uint32_t world) {
        rank_ = rank;
        world_ = world;
    }
    uint32_t kind() const override { return RSD_COMM_NULL; }
    rsd_status all_gather(const void* send, void* recv, uint64_t bytes, hipStream_t s) override {
        if (!bytes) return RSD_OK;
        const CopySeg c{send, static_cast<char*>(recv) + rank_ * bytes, bytes};
        return copy_segments(&c, 1, s);
    }
    rsd_status exchange(const Xfer*, uint32_t, const Xfer*, uint32_t, hipStream_t) override { return RSD_OK; }
};

rsd_status check_comm(const rsd_comm* c, const char* who) {
    if (!c || !c->impl) {
        set_error(std::string(who) + ": null communicator");
        return RSD_ERR_INVALID_ARG;
    }
    return RSD_OK;
}

}  // namespace
}  // namespace rsd

using namespace rsd;

extern "C" rsd_status rsd_comm_rccl_available(void) {
    const Rccl* r = nullptr;
    return rccl_load(&r);
}

extern "C" rsd_status rsd_comm_rccl_unique_id(uint8_t id[RSD_COMM_UNIQUE_ID_BYTES]) {
    if (!id) {
        set_error("rsd_comm_rccl_unique_id: null output");
        return RSD_ERR_INVALID_ARG;
    }
    const Rccl* r = nullptr;
    rsd_status st = rccl_load(&r);
    if (st != RSD_OK) return st;
    ncclUniqueId u;
    ncclResult_t e = r->GetUniqueId(&u);
    if (e != ncclSuccess) return nccl_fail(r, e, "ncclGetUniqueId");
    static_assert(sizeof(u) == RSD_COMM_UNIQUE_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return RSD_OK;
}

extern "C" rsd_status rsd_comm_rccl_create(const uint8_t id[RSD_COMM_UNIQUE_ID_BYTES], uint32_t world, uint32_t rank,
                                           rsd_comm** out) {
    if (!id || !out || world == 0 || rank >= world) {
        set_error("rsd_comm_rccl_create: null argument or rank >= world");
        return RSD_ERR_INVALID_ARG;
    }
    const Rccl* r = nullptr;
    rsd_status st = rccl_load(&r);
    if (st != RSD_OK) return st;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    ncclResult_t e = r->CommInitRank(&c, (int)world, u, (int)rank);  // collective: every rank calls it
    if (e != ncclSuccess) return nccl_fail(r, e, "ncclCommInitRank");
    *out = new rsd_comm{new RcclComm(r, c, rank, world)};
    return RSD_OK;
}

extern "C" rsd_status rsd_comm_hub_create(uint32_t world, rsd_comm_hub** out) {
    if (!out || world == 0 || world > 64) {
        set_error("rsd_comm_hub_create: world must be 1..64");
        return RSD_ERR_INVALID_ARG;
    }
    rsd_comm_hub* h = new rsd_comm_hub();
    h->world = world;
    *out = h;
    return RSD_OK;
}

extern "C" void rsd_comm_hub_release(rsd_comm_hub* hub) { delete hub; }

extern "C" rsd_status rsd_comm_local_create(rsd_comm_hub* hub, uint32_t rank, rsd_comm** out) {
    if (!hub || !out || rank >= hub->world) {
        set_error("rsd_comm_local_create: null hub / output or rank >= world");
        return RSD_ERR_INVALID_ARG;
    }
    LocalComm* c = new LocalComm(hub, rank);
    rsd_status st = c->init();
    if (st != RSD_OK) {
        delete c;
        return st;
    }
    *out = new rsd_comm{c};
    return RSD_OK;
}

extern "C" rsd_status rsd_comm_null_create(uint32_t world, uint32_t rank, rsd_comm** out) {
    if (!out || world == 0 || world > 64 || rank >= world) {
        set_error("rsd_comm_null_create: world must be 1..64 and rank < world");
        return RSD_ERR_INVALID_ARG;
    }
    *out = new rsd_comm{new NullComm(rank, world)};
    return RSD_OK;
}

extern "C" void rsd_comm_release(rsd_comm* c) {
    if (!c) return;
    delete c->impl;
    delete c;
}

extern "C" rsd_status rsd_comm_info(const rsd_comm* c, uint32_t* kind, uint32_t* rank, uint32_t* world) {
    rsd_status st = check_comm(c, "rsd_comm_info");
    if (st != RSD_OK) return st;
    if (kind) *kind = c->impl->kind();
    if (rank) *rank = c->impl->rank();
    if (world) *world = c->impl->world();
    return RSD_OK;
}

extern "C" rsd_status rsd_comm_all_gather(rsd_comm* c, const void* d_send, void* d_recv, uint64_t bytes,
                                          rsd_stream stream) {
    rsd_status st = check_comm(c, "rsd_comm_all_gather");
    if (st != RSD_OK) return st;
    if (bytes && (!d_send || !d_recv)) {
        set_error("rsd_comm_all_gather: null buffer");
        return RSD_ERR_INVALID_ARG;
    }
    return c->impl->all_gather(d_send, d_recv, bytes, (hipStream_t)stream);
}

extern "C" rsd_status rsd_comm_exchange(rsd_comm* c, const rsd_comm_xfer* sends, uint32_t n_sends,
                                        const rsd_comm_xfer* recvs, uint32_t n_recvs, rsd_stream stream) {
    rsd_status st = check_comm(c, "rsd_comm_exchange");
    if (st != RSD_OK) return st;
    if ((n_sends && !sends) || (n_recvs && !recvs)) {
        set_error("rsd_comm_exchange: null transfer list");
        return RSD_ERR_INVALID_ARG;
    }
    std::vector<Xfer> s(n_sends), r(n_recvs);
    for (uint32_t i = 0; i < n_sends; ++i) {
        if (sends[i].peer >= c->impl->world() || (sends[i].bytes && !sends[i].buf)) {
            set_error("rsd_comm_exchange: send peer out of range or null buffer");
            return RSD_ERR_INVALID_ARG;
        }
        s[i] = {sends[i].buf, sends[i].bytes, sends[i].peer};
    }
    for (uint32_t i = 0; i < n_recvs; ++i) {
        if (recvs[i].peer >= c->impl->world() || (recvs[i].bytes && !recvs[i].buf)) {
            set_error("rsd_comm_exchange: receive peer out of range or null buffer");
            return RSD_ERR_INVALID_ARG;
        }
        r[i] = {recvs[i].buf, recvs[i].bytes, recvs[i].peer};
    }
    return c->impl->exchange(s.data(), n_sends, r.data(), n_recvs, (hipStream_t)stream);
}
