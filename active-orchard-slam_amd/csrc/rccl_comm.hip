// aos_comm over RCCL: the communicator of a tiled frame when every rank is its own
// process on its own GPU (torch.distributed-style launch). The library owns the exchange buffers
// in HBM; the all-gather of the halo strips / final tiles is one ncclAllGather over xGMI, and the
// max-reduction of the thinning flags one ncclAllReduce(ncclMax) of a small int32 array.
//
// RCCL is opened at run time (dlopen of librccl.so.1), so libaos_gpu.so loads without it and a
// process that never asks for the communicator never initialises RCCL. The aos_comm callbacks are
// collective and synchronous (aos_comm contract, include/aos_gpu.h): each one enqueues on the
// communicator's own stream and waits for it. A tiled frame that recognises this communicator
// (rccl_stream_coll) enqueues the same collectives on its own stream instead (StreamColl: no host wait),
// plus two point-to-point forms: the halo strips to the neighbouring tiles only, the final tiles to the root.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "aos_ctx.h"

namespace aos {

namespace {
struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId *);
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*group_start)();
    ncclResult_t (*group_end)();
    ncclResult_t (*comm_destroy)(ncclComm_t);
    const char *(*error_string)(ncclResult_t);
};

const RcclApi &rccl_api() {
    static RcclApi api{};
    static std::string err;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) { err = std::string("cannot load librccl.so.1: ") + dlerror(); return; }
        auto sym = [&](const char *name) {
            void *p = dlsym(h, name);
            if (!p && err.empty()) err = std::string("librccl.so.1 lacks ") + name;
            return p;
        };
        api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(sym("ncclGetUniqueId"));
        api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(sym("ncclCommInitRank"));
        api.all_gather = reinterpret_cast<decltype(api.all_gather)>(sym("ncclAllGather"));
        api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(sym("ncclAllReduce"));
        api.send = reinterpret_cast<decltype(api.send)>(sym("ncclSend"));
        api.recv = reinterpret_cast<decltype(api.recv)>(sym("ncclRecv"));
        api.group_start = reinterpret_cast<decltype(api.group_start)>(sym("ncclGroupStart"));
        api.group_end = reinterpret_cast<decltype(api.group_end)>(sym("ncclGroupEnd"));
        api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(sym("ncclCommDestroy"));
        api.error_string = reinterpret_cast<decltype(api.error_string)>(sym("ncclGetErrorString"));
    });
    if (!err.empty()) throw CommError{err};
    return api;
}

void rccl_check(const RcclApi &api, ncclResult_t r, const char *what) {
    if (r != ncclSuccess) throw CommError{std::string(what) + ": " + api.error_string(r)};
}
}  // namespace

}  // namespace aos

struct aos_rccl {   // the C-ABI's opaque communicator
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    int device = 0;
    aos::DevBuf send, recv, red;
    aos_comm c{};
};

namespace aos {

void rccl_unique_id(uint8_t *id) {
    const RcclApi &api = rccl_api();
    ncclUniqueId u;
    rccl_check(api, api.get_unique_id(&u), "ncclGetUniqueId");
    static_assert(sizeof(u) == NCCL_UNIQUE_ID_BYTES, "unique id size");
    std::memcpy(id, &u, sizeof(u));
}

static void sc_all_gather(void *impl, uint64_t bytes, hipStream_t s);
static void sc_all_to_all(void *impl, const uint64_t *counts, hipStream_t s);

// the aos_comm callbacks: the stream-ordered collectives below on the communicator's own stream, then a wait
static int rc_all_gather(void *user, uint64_t bytes) {
    aos_rccl *r = static_cast<aos_rccl *>(user);
    try {
        DeviceScope ds(r->device);
        if (bytes > r->c.buf_bytes) return 1;
        sc_all_gather(r, bytes, r->stream);
        return hipStreamSynchronize(r->stream) == hipSuccess ? 0 : 1;
    } catch (...) {
        return 1;
    }
}

// point-to-point blocks of the personalised exchange: one ncclGroupStart / ncclGroupEnd around a send and a
// receive per peer (the own block is a device copy); every link of the xGMI mesh carries its pair at once
static int rc_all_to_all(void *user, const uint64_t *counts) {
    aos_rccl *r = static_cast<aos_rccl *>(user);
    try {
        DeviceScope ds(r->device);
        sc_all_to_all(r, counts, r->stream);
        return hipStreamSynchronize(r->stream) == hipSuccess ? 0 : 1;
    } catch (...) {
        return 1;
    }
}

static int rc_all_reduce_max(void *user, int32_t *v, int32_t n) {
    aos_rccl *r = static_cast<aos_rccl *>(user);
    try {
        const RcclApi &api = rccl_api();
        DeviceScope ds(r->device);
        if (n <= 0) return 0;
        int32_t *d = static_cast<int32_t *>(r->red.ensure(sizeof(int32_t) * (size_t)n));
        AOS_HIP(hipMemcpyAsync(d, v, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, r->stream));
        rccl_check(api, api.all_reduce(d, d, (size_t)n, ncclInt32, ncclMax, r->comm, r->stream), "ncclAllReduce");
        AOS_HIP(hipMemcpyAsync(v, d, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, r->stream));
        return hipStreamSynchronize(r->stream) == hipSuccess ? 0 : 1;
    } catch (...) {
        return 1;
    }
}

// ---- the same collectives enqueued on the caller's stream (StreamColl, aos_internal.h): no host wait; the frame's
// kernels before and after them are ordered by the stream. RCCL takes any stream of the communicator's device.
static void sc_all_gather(void *impl, uint64_t bytes, hipStream_t s) {
    aos_rccl *r = static_cast<aos_rccl *>(impl);
    const RcclApi &api = rccl_api();
    DeviceScope ds(r->device);
    if (bytes > r->c.buf_bytes) throw CommError{"all_gather larger than the RCCL buffers"};
    rccl_check(api, api.all_gather(r->send.p, r->recv.p, bytes, ncclUint8, r->comm, s), "ncclAllGather");
}

// rank q's send_buf[0, bytes) -> the root's recv_buf[q * bytes, ...): each rank sends one block, only the root
// receives (W - 1 blocks; its own block is a device copy)
static void sc_gather(void *impl, uint64_t bytes, int root, hipStream_t s) {
    aos_rccl *r = static_cast<aos_rccl *>(impl);
    const RcclApi &api = rccl_api();
    DeviceScope ds(r->device);
    const int W = r->c.world, me = r->c.rank;
    if (bytes > r->c.buf_bytes) throw CommError{"gather larger than the RCCL buffers"};
    if (root < 0 || root >= W) throw CommError{"gather: root outside the communicator"};
    if (!bytes) return;
    char *rb = static_cast<char *>(r->recv.p);
    if (me == root) AOS_HIP(hipMemcpyAsync(rb + (uint64_t)me * bytes, r->send.p, bytes, hipMemcpyDeviceToDevice, s));
    if (W == 1) return;
    rccl_check(api, api.group_start(), "ncclGroupStart");
    if (me == root) {
        for (int q = 0; q < W; ++q)
            if (q != me) rccl_check(api, api.recv(rb + (uint64_t)q * bytes, bytes, ncclUint8, q, r->comm, s), "ncclRecv");
    } else {
        rccl_check(api, api.send(r->send.p, bytes, ncclUint8, root, r->comm, s), "ncclSend");
    }
    rccl_check(api, api.group_end(), "ncclGroupEnd");
}

static void sc_max_dev(void *impl, int32_t *d, int n, hipStream_t s) {
    aos_rccl *r = static_cast<aos_rccl *>(impl);
    const RcclApi &api = rccl_api();
    DeviceScope ds(r->device);
    if (n > 0) rccl_check(api, api.all_reduce(d, d, (size_t)n, ncclInt32, ncclMax, r->comm, s), "ncclAllReduce");
}

static void sc_all_to_all(void *impl, const uint64_t *counts, hipStream_t s) {
    aos_rccl *r = static_cast<aos_rccl *>(impl);
    const RcclApi &api = rccl_api();
    DeviceScope ds(r->device);
    const int W = r->c.world, me = r->c.rank;
    uint64_t soff = 0, roff = 0;
    std::vector<uint64_t> so(W), ro(W);
    for (int q = 0; q < W; ++q) {
        so[q] = soff; soff += counts[(size_t)me * W + q];
        ro[q] = roff; roff += counts[(size_t)q * W + me];
    }
    if (soff > r->c.buf_bytes || roff > r->c.buf_bytes * (uint64_t)W) throw CommError{"all_to_all larger than the RCCL buffers"};
    const char *sb = static_cast<const char *>(r->send.p);
    char *rb = static_cast<char *>(r->recv.p);
    if (const uint64_t n = counts[(size_t)me * W + me]) AOS_HIP(hipMemcpyAsync(rb + ro[me], sb + so[me], n, hipMemcpyDeviceToDevice, s));
    if (W == 1) return;
    rccl_check(api, api.group_start(), "ncclGroupStart");
    for (int q = 0; q < W; ++q) {
        if (q == me) continue;
        if (const uint64_t n = counts[(size_t)me * W + q]) rccl_check(api, api.send(sb + so[q], n, ncclUint8, q, r->comm, s), "ncclSend");
        if (const uint64_t n = counts[(size_t)q * W + me]) rccl_check(api, api.recv(rb + ro[q], n, ncclUint8, q, r->comm, s), "ncclRecv");
    }
    rccl_check(api, api.group_end(), "ncclGroupEnd");
}

// the halo exchange: this rank's strips to each peer, each peer's strips into its block (grouped point-to-point:
// a rank receives its 3-8 neighbours' strips instead of every rank's)
static void sc_exchange(void *impl, uint64_t bytes, const uint8_t *peer, hipStream_t s) {
    aos_rccl *r = static_cast<aos_rccl *>(impl);
    const RcclApi &api = rccl_api();
    DeviceScope ds(r->device);
    const int W = r->c.world, me = r->c.rank;
    if (bytes > r->c.buf_bytes) throw CommError{"exchange larger than the RCCL buffers"};
    if (!bytes || W == 1) return;
    char *rb = static_cast<char *>(r->recv.p);
    rccl_check(api, api.group_start(), "ncclGroupStart");
    for (int q = 0; q < W; ++q) {
        if (q == me || !peer[q]) continue;
        rccl_check(api, api.send(r->send.p, bytes, ncclUint8, q, r->comm, s), "ncclSend");
        rccl_check(api, api.recv(rb + (uint64_t)q * bytes, bytes, ncclUint8, q, r->comm, s), "ncclRecv");
    }
    rccl_check(api, api.group_end(), "ncclGroupEnd");
}

bool rccl_stream_coll(const aos_comm &cm, StreamColl &out) {
    if (cm.all_gather != rc_all_gather || !cm.user) return false;   // (a caller's communicator: its callbacks)
    out.impl = cm.user;
    out.all_gather = sc_all_gather;
    out.gather = sc_gather;
    out.max_dev = sc_max_dev;
    out.all_to_all = sc_all_to_all;
    out.exchange = sc_exchange;
    return true;
}

aos_rccl *rccl_create(const uint8_t *id, int rank, int world, int device, uint64_t buf_bytes) {
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("aos_rccl_create: bad rank / world");
    if (buf_bytes == 0) throw std::invalid_argument("aos_rccl_create: buf_bytes = 0");
    const RcclApi &api = rccl_api();
    DeviceScope ds(device);
    auto *r = new aos_rccl();
    try {
        r->device = device;
        AOS_HIP(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
        r->send.ensure(buf_bytes);
        r->recv.ensure(buf_bytes * (uint64_t)world);
        r->red.ensure(4096);
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        rccl_check(api, api.comm_init_rank(&r->comm, world, u, rank), "ncclCommInitRank");
    } catch (...) {
        rccl_destroy(r);
        throw;
    }
    r->c.user = r;
    r->c.rank = rank;
    r->c.world = world;
    r->c.send_buf = r->send.p;
    r->c.recv_buf = r->recv.p;
    r->c.buf_bytes = buf_bytes;
    r->c.all_gather = rc_all_gather;
    r->c.all_reduce_max = rc_all_reduce_max;
    r->c.all_to_all = rc_all_to_all;
    return r;
}

const aos_comm *rccl_comm(aos_rccl *r) { return &r->c; }

void rccl_destroy(aos_rccl *r) {
    if (!r) return;
    DeviceScope ds(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    if (r->comm) (void)rccl_api().comm_destroy(r->comm);
    r->send.release();
    r->recv.release();
    r->red.release();
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
}

}  // namespace aos
