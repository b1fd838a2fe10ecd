// comm.cpp -- RCCL and in-process transports (see comm.hpp).
#include "comm.hpp"

#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <vector>

namespace ukkt {

// ------------------------------------------------------------------------------------------------
// in-process group
// ------------------------------------------------------------------------------------------------
struct LocalGroup {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    struct Msg {
        const void* buf;
        size_t bytes;
        hipEvent_t ev;
    };
    std::vector<std::deque<Msg>> box;  // src * world + dst
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<std::vector<uint64_t>> contrib;
    std::vector<uint64_t> result;
    const void* bptr = nullptr;
    hipEvent_t bev = nullptr;
    explicit LocalGroup(int w) : world(w), box((size_t)w * w), contrib(w) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

LocalGroup* local_group_create(int world) { return world > 0 ? new LocalGroup(world) : nullptr; }
void local_group_destroy(LocalGroup* g) { delete g; }

namespace {

class LocalTransport final : public Transport {
public:
    LocalTransport(LocalGroup* g, int r) : g_(g), r_(r) {}
    int rank() const override { return r_; }
    int size() const override { return g_->world; }
    std::string describe() const override { return "local(in-process, " + std::to_string(g_->world) + " ranks)"; }

    hipError_t send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
        hipEvent_t ev;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        if ((e = hipEventRecord(ev, s)) != hipSuccess) return e;
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            g_->box[(size_t)r_ * g_->world + peer].push_back({buf, bytes, ev});
        }
        g_->cv.notify_all();
        return hipSuccess;
    }
    hipError_t recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
        LocalGroup::Msg m;
        {
            std::unique_lock<std::mutex> lk(g_->mu);
            auto& q = g_->box[(size_t)peer * g_->world + r_];
            g_->cv.wait(lk, [&] { return !q.empty(); });
            m = q.front();
            q.pop_front();
        }
        if (m.bytes != bytes) return hipErrorInvalidValue;
        hipError_t e = hipStreamWaitEvent(s, m.ev, 0);
        if (e == hipSuccess && bytes) e = hipMemcpyAsync(buf, m.buf, bytes, hipMemcpyDefault, s);
        hipEventDestroy(m.ev);
        return e;
    }
    hipError_t allreduce(void* buf, size_t count, RedOp op, hipStream_t s) override {
        std::vector<uint64_t> mine(count);
        hipError_t e = hipStreamSynchronize(s);
        if (e == hipSuccess && count) e = hipMemcpy(mine.data(), buf, count * 8, hipMemcpyDeviceToHost);
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            g_->contrib[r_] = std::move(mine);
        }
        g_->barrier();
        std::vector<uint64_t> out(g_->contrib[0]);
        for (int q = 1; q < g_->world; ++q) {  // rank order: deterministic
            const auto& c = g_->contrib[q];
            for (size_t i = 0; i < count && i < c.size(); ++i) {
                switch (op) {
                    case RedOp::SumU64: out[i] += c[i]; break;
                    case RedOp::MaxU64: out[i] = out[i] > c[i] ? out[i] : c[i]; break;
                    case RedOp::MaxF64:
                    case RedOp::SumF64: {
                        double a, b;
                        memcpy(&a, &out[i], 8);
                        memcpy(&b, &c[i], 8);
                        a = op == RedOp::SumF64 ? a + b : (a > b ? a : b);
                        memcpy(&out[i], &a, 8);
                    } break;
                }
            }
        }
        g_->barrier();  // every rank has read every contribution
        if (e == hipSuccess && count) e = hipMemcpy(buf, out.data(), count * 8, hipMemcpyHostToDevice);
        return e;
    }
    hipError_t broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        hipError_t e = hipSuccess;
        hipEvent_t ev = nullptr;
        if (r_ == root) {
            e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventRecord(ev, s);
            std::lock_guard<std::mutex> lk(g_->mu);
            g_->bptr = buf;
            g_->bev = ev;
        }
        g_->barrier();
        if (r_ != root && bytes) {
            e = hipStreamWaitEvent(s, g_->bev, 0);
            if (e == hipSuccess) e = hipMemcpyAsync(buf, g_->bptr, bytes, hipMemcpyDefault, s);
        }
        g_->barrier();  // every copy is enqueued behind the event
        if (ev) hipEventDestroy(ev);
        return e;
    }

private:
    LocalGroup* g_;
    int r_;
};

// ------------------------------------------------------------------------------------------------
// RCCL
// ------------------------------------------------------------------------------------------------
class RcclTransport final : public Transport {
public:
    RcclTransport(ncclComm_t c, int r, int w) : c_(c), r_(r), w_(w) {}
    ~RcclTransport() override { ncclCommDestroy(c_); }
    int rank() const override { return r_; }
    int size() const override { return w_; }
    std::string describe() const override { return "rccl(" + std::to_string(w_) + " ranks)"; }
    hipError_t group_begin() override { return st(ncclGroupStart()); }
    hipError_t group_end() override { return st(ncclGroupEnd()); }
    hipError_t send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
        return st(ncclSend(buf, bytes, ncclUint8, peer, c_, s));
    }
    hipError_t recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
        return st(ncclRecv(buf, bytes, ncclUint8, peer, c_, s));
    }
    hipError_t allreduce(void* buf, size_t count, RedOp op, hipStream_t s) override {
        ncclDataType_t t = (op == RedOp::SumU64 || op == RedOp::MaxU64) ? ncclUint64 : ncclFloat64;
        ncclRedOp_t o = (op == RedOp::SumU64 || op == RedOp::SumF64) ? ncclSum : ncclMax;
        return st(ncclAllReduce(buf, buf, count, t, o, c_, s));
    }
    hipError_t broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        return st(ncclBroadcast(buf, buf, bytes, ncclUint8, root, c_, s));
    }

private:
    static hipError_t st(ncclResult_t r) { return r == ncclSuccess ? hipSuccess : hipErrorLaunchFailure; }
    ncclComm_t c_;
    int r_, w_;
};

// ------------------------------------------------------------------------------------------------
// host-staged (caller's callbacks on host buffers)
// ------------------------------------------------------------------------------------------------
class HostTransport final : public Transport {
public:
    HostTransport(const HostComm& cb, int r, int w) : cb_(cb), r_(r), w_(w) {}
    ~HostTransport() override {
        for (auto& p : pend_) hipHostFree(p.host);
    }
    int rank() const override { return r_; }
    int size() const override { return w_; }
    std::string describe() const override { return "host-staged(" + std::to_string(w_) + " ranks)"; }
    hipError_t group_begin() override {
        in_group_ = true;
        return hipSuccess;
    }
    hipError_t group_end() override {
        in_group_ = false;
        return complete();
    }
    hipError_t send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
        if (bytes == 0) return hipSuccess;
        void* hb = nullptr;
        hipError_t e = stage(bytes, &hb);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipMemcpy(hb, buf, bytes, hipMemcpyDeviceToHost);
        pend_.push_back({hb, nullptr, 0});
        if (e == hipSuccess && cb_.send(cb_.ctx, hb, bytes, peer) != 0) e = hipErrorLaunchFailure;
        return (e != hipSuccess || in_group_) ? e : complete();
    }
    hipError_t recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
        if (bytes == 0) return hipSuccess;
        void* hb = nullptr;
        hipError_t e = stage(bytes, &hb);
        if (e == hipSuccess) e = hipStreamSynchronize(s);  // earlier work on `buf` is done before it is overwritten
        pend_.push_back({hb, buf, bytes});
        if (e == hipSuccess && cb_.recv(cb_.ctx, hb, bytes, peer) != 0) e = hipErrorLaunchFailure;
        return (e != hipSuccess || in_group_) ? e : complete();
    }
    hipError_t allreduce(void* buf, size_t count, RedOp op, hipStream_t s) override {
        if (count == 0) return hipSuccess;
        void* hb = nullptr;
        hipError_t e = stage(count * 8, &hb);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipMemcpy(hb, buf, count * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess && cb_.allreduce(cb_.ctx, hb, count, (int)op) != 0) e = hipErrorLaunchFailure;
        if (e == hipSuccess) e = hipMemcpy(buf, hb, count * 8, hipMemcpyHostToDevice);
        hipHostFree(hb);
        return e;
    }
    hipError_t broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        if (bytes == 0) return hipSuccess;
        void* hb = nullptr;
        hipError_t e = stage(bytes, &hb);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess && r_ == root) e = hipMemcpy(hb, buf, bytes, hipMemcpyDeviceToHost);
        if (e == hipSuccess && cb_.broadcast(cb_.ctx, hb, bytes, root) != 0) e = hipErrorLaunchFailure;
        if (e == hipSuccess && r_ != root) e = hipMemcpy(buf, hb, bytes, hipMemcpyHostToDevice);
        hipHostFree(hb);
        return e;
    }

private:
    struct Pending {
        void* host;
        void* dev;  // receives: destination, copied after the exchange completes
        size_t bytes;
    };
    static hipError_t stage(size_t bytes, void** hb) { return hipHostMalloc(hb, bytes, hipHostMallocDefault); }
    // every posted send / receive is finished by the caller, then received data goes to the device
    hipError_t complete() {
        hipError_t e = cb_.group_end(cb_.ctx) == 0 ? hipSuccess : hipErrorLaunchFailure;
        for (auto& p : pend_) {
            if (e == hipSuccess && p.dev) e = hipMemcpy(p.dev, p.host, p.bytes, hipMemcpyHostToDevice);
            hipHostFree(p.host);
        }
        pend_.clear();
        return e;
    }
    HostComm cb_;
    int r_, w_;
    bool in_group_ = false;
    std::vector<Pending> pend_;
};

}  // namespace

Transport* make_host_transport(const HostComm& cb, int rank, int world) {
    if (!cb.send || !cb.recv || !cb.group_end || !cb.allreduce || !cb.broadcast || rank < 0 || rank >= world) return nullptr;
    return new HostTransport(cb, rank, world);
}

Transport* make_local_transport(LocalGroup* g, int rank) {
    if (!g || rank < 0 || rank >= g->world) return nullptr;
    return new LocalTransport(g, rank);
}

int rccl_unique_id(unsigned char out[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "NCCL_UNIQUE_ID_BYTES");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
    memcpy(out, &id, 128);
    return 0;
}

Transport* make_rccl_transport(const unsigned char id[128], int rank, int world, int device, std::string& err) {
    ncclUniqueId uid;
    memcpy(&uid, id, 128);
    if (hipSetDevice(device) != hipSuccess) { err = "hipSetDevice failed"; return nullptr; }
    ncclComm_t c;
    ncclResult_t r = ncclCommInitRank(&c, world, uid, rank);
    if (r != ncclSuccess) { err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r); return nullptr; }
    return new RcclTransport(c, rank, world);
}

// ------------------------------------------------------------------------------------------------
// tracing decorator (option comm_trace)
// ------------------------------------------------------------------------------------------------
namespace {
class TracingTransport final : public Transport {
public:
    explicit TracingTransport(Transport* inner) : in_(inner) {}
    ~TracingTransport() override { delete in_; }
    int rank() const override { return in_->rank(); }
    int size() const override { return in_->size(); }
    std::string describe() const override { return "trace(" + in_->describe() + ")"; }
    hipError_t group_begin() override { rec(4, -1, 0, -1); return in_->group_begin(); }
    hipError_t group_end() override { rec(5, -1, 0, -1); return in_->group_end(); }
    hipError_t send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
        order(s);
        rec(0, peer, bytes, -1);
        return in_->send(buf, bytes, peer, s);
    }
    hipError_t recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
        order(s);
        rec(1, peer, bytes, -1);
        return in_->recv(buf, bytes, peer, s);
    }
    hipError_t allreduce(void* buf, size_t count, RedOp op, hipStream_t s) override {
        order(s);
        rec(2, -1, count * 8, (int)op);
        return in_->allreduce(buf, count, op, s);
    }
    hipError_t broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        order(s);
        rec(3, root, bytes, -1);
        return in_->broadcast(buf, bytes, root, s);
    }
    std::vector<int64_t> log;
    std::function<std::pair<int, int>(hipStream_t)> probe;

private:
    void order(hipStream_t s) {
        if (!probe) return;
        const std::pair<int, int> o = probe(s);
        rec(6, o.first, (size_t)o.second, -1);
    }
    void rec(int op, int peer, size_t bytes, int red) {
        log.push_back(op);
        log.push_back(peer);
        log.push_back((int64_t)bytes);
        log.push_back(red);
    }
    Transport* in_;
};
}  // namespace

Transport* make_tracing_transport(Transport* inner) { return inner ? new TracingTransport(inner) : nullptr; }

void comm_trace_set_probe(Transport* t, std::function<std::pair<int, int>(hipStream_t)> probe) {
    if (auto* tt = dynamic_cast<TracingTransport*>(t)) tt->probe = std::move(probe);
}

bool comm_trace_records(Transport* t, std::vector<int64_t>& out, bool clear) {
    auto* tt = dynamic_cast<TracingTransport*>(t);
    if (!tt) return false;
    out = tt->log;
    if (clear) tt->log.clear();
    return true;
}

}  // namespace ukkt
