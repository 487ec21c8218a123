// comm.cpp -- the collectives of the library's own multi-GPU exchange (comm.hpp).
#include "comm.hpp"
#include "kernels.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace aniso {

[[noreturn]] void throw_hip(hipError_t e, const char* file, int line);

namespace {

// The RCCL entry points, bound at run time to the process's librccl.so.1 (the copy
// PyTorch-ROCm loaded, same SONAME, so the library and torch.distributed share one
// RCCL): no link-time dependency, and single-GPU use never loads it.
struct Rccl {
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char* (*errorString)(ncclResult_t) = nullptr;

    static Rccl& get() {
        static Rccl r;
        static std::once_flag once;
        static std::string err;
        std::call_once(once, [] {
            void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
            if (!h) {
                err = std::string("RCCL not found (librccl.so.1): ") + dlerror();
                return;
            }
            auto sym = [&](const char* n) {
                void* f = dlsym(h, n);
                if (!f) err = std::string("RCCL symbol missing: ") + n;
                return f;
            };
            r.getUniqueId = reinterpret_cast<decltype(r.getUniqueId)>(sym("ncclGetUniqueId"));
            r.commInitRank = reinterpret_cast<decltype(r.commInitRank)>(sym("ncclCommInitRank"));
            r.commDestroy = reinterpret_cast<decltype(r.commDestroy)>(sym("ncclCommDestroy"));
            r.allGather = reinterpret_cast<decltype(r.allGather)>(sym("ncclAllGather"));
            r.allReduce = reinterpret_cast<decltype(r.allReduce)>(sym("ncclAllReduce"));
            r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
            r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
            r.groupStart = reinterpret_cast<decltype(r.groupStart)>(sym("ncclGroupStart"));
            r.groupEnd = reinterpret_cast<decltype(r.groupEnd)>(sym("ncclGroupEnd"));
            r.errorString = reinterpret_cast<decltype(r.errorString)>(sym("ncclGetErrorString"));
        });
        if (!err.empty()) throw std::runtime_error(err);
        return r;
    }
    void check(ncclResult_t e, const char* what) const {
        if (e != ncclSuccess)
            throw std::runtime_error(std::string("RCCL ") + what + " failed: " + (errorString ? errorString(e) : "?"));
    }
};

class RcclCollectives : public Collectives {
  public:
    RcclCollectives(const unsigned char* id, int n, int r) {
        nranks = n;
        rank = r;
        Rccl& R = Rccl::get();
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, sizeof(uid.internal));
        R.check(R.commInitRank(&comm_, n, uid, r), "ncclCommInitRank");
    }
    ~RcclCollectives() override {
        if (comm_) (void)Rccl::get().commDestroy(comm_);
    }
    void allgather(const double* send, double* recv, size_t count, hipStream_t s) override {
        Rccl& R = Rccl::get();
        R.check(R.allGather(send, recv, count, ncclFloat64, comm_, s), "ncclAllGather");
    }
    void alltoallv(const double* send, const int64_t* sc, const int64_t* so, double* recv, const int64_t* rc,
                   const int64_t* ro, hipStream_t s) override {
        Rccl& R = Rccl::get();
        R.check(R.groupStart(), "ncclGroupStart");
        for (int p = 0; p < nranks; ++p) {
            if (p == rank) continue;
            if (sc[p] > 0) R.check(R.send(send + so[p], (size_t)sc[p], ncclFloat64, p, comm_, s), "ncclSend");
            if (rc[p] > 0) R.check(R.recv(recv + ro[p], (size_t)rc[p], ncclFloat64, p, comm_, s), "ncclRecv");
        }
        R.check(R.groupEnd(), "ncclGroupEnd");
    }
    void allreduce(double* buf, size_t count, hipStream_t s) override {
        Rccl& R = Rccl::get();
        R.check(R.allReduce(buf, buf, count, ncclFloat64, ncclSum, comm_, s), "ncclAllReduce");
    }
  private:
    ncclComm_t comm_ = nullptr;
};

// Caller-supplied collectives: the stream is drained before each call, so a host-staged
// transport sees complete device buffers, and the caller returns after its copies.
class CallbackCollectives : public Collectives {
  public:
    CallbackCollectives(const aniso_collectives& c, int n, int r) : c_(c) {
        nranks = n;
        rank = r;
        if (!c_.allgather || !c_.alltoallv || !c_.allreduce)
            throw std::invalid_argument("aniso_collectives: every callback must be set");
    }
    void allgather(const double* send, double* recv, size_t count, hipStream_t s) override {
        sync(s);
        if (c_.allgather(c_.ctx, send, recv, count, s)) throw std::runtime_error("allgather callback failed");
    }
    void alltoallv(const double* send, const int64_t* sc, const int64_t* so, double* recv, const int64_t* rc,
                   const int64_t* ro, hipStream_t s) override {
        sync(s);
        if (c_.alltoallv(c_.ctx, send, sc, so, recv, rc, ro, s)) throw std::runtime_error("alltoallv callback failed");
    }
    void allreduce(double* buf, size_t count, hipStream_t s) override {
        sync(s);
        if (c_.allreduce(c_.ctx, buf, count, s)) throw std::runtime_error("allreduce callback failed");
    }

  private:
    static void sync(hipStream_t s) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) throw_hip(e, __FILE__, __LINE__);
    }
    aniso_collectives c_;
};

// Development: one rank's exchange with the others' data left out -- its own part of
// the all-gather copied into place on the stream, nothing sent or received.  Times a
// rank's schedule (streams, events, kernels) on one GPU; its results are not the
// sharded operator's.
class LoopbackCollectives : public Collectives {
  public:
    LoopbackCollectives(int n, int r) {
        nranks = n;
        rank = r;
    }
    void allgather(const double* send, double* recv, size_t count, hipStream_t s) override {
        const hipError_t e = hipMemcpyAsync(recv + (size_t)rank * count, send, count * sizeof(double),
                                            hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) throw_hip(e, __FILE__, __LINE__);
    }
    // ANISO_LOOPBACK_XCHG_US: a stand-in for the exchange's latency over xGMI (a spin
    // kernel of that duration on 8 workgroups), so a rank's schedule is timed with the
    // exchange in its critical path
    void alltoallv(const double*, const int64_t*, const int64_t*, double*, const int64_t*, const int64_t*,
                   hipStream_t s) override {
        static const int us = [] {
            const char* e = std::getenv("ANISO_LOOPBACK_XCHG_US");
            return e ? std::atoi(e) : 0;
        }();
        launch_spin_us(us, 8, s);
    }
    void allreduce(double*, size_t, hipStream_t) override {}
    bool loopback() const override { return true; }
};

}  // namespace

std::unique_ptr<Collectives> make_loopback_collectives(int nranks, int rank) {
    return std::unique_ptr<Collectives>(new LoopbackCollectives(nranks, rank));
}

std::unique_ptr<Collectives> make_rccl_collectives(const unsigned char* uniqueId, int nranks, int rank) {
    return std::unique_ptr<Collectives>(new RcclCollectives(uniqueId, nranks, rank));
}

std::unique_ptr<Collectives> make_callback_collectives(const aniso_collectives& c, int nranks, int rank) {
    return std::unique_ptr<Collectives>(new CallbackCollectives(c, nranks, rank));
}

void rccl_unique_id(unsigned char* out) {
    Rccl& R = Rccl::get();
    ncclUniqueId uid;
    R.check(R.getUniqueId(&uid), "ncclGetUniqueId");
    std::memcpy(out, uid.internal, sizeof(uid.internal));
}

}  // namespace aniso
