// In-process multi-GPU tiled frame (aos_group_*, SURVEY §8b's multi-GPU handle): one map cut into
// tiles_x x tiles_y tiles, one aos_ctx per tile on its own device (devices may repeat), the ranks
// driven by one thread each inside the library. Their aos_comm is local: the all-gather pulls every
// rank's registered send buffer into each rank's receive buffer with peer copies (xGMI between
// MI355X devices; a device-to-device copy when two ranks share a GPU), and the max all-reduce runs
// on host ints. A barrier with an abort flag keeps one failing rank from hanging the others.
// The frame itself is aos_tiled_seedgen_process on every rank (tiled.hip), so the root rank's
// outputs are byte-identical to aos_seedgen_process on the whole cloud.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <thread>
#include <vector>

#include "aos_ctx.h"

namespace aos {
namespace {

struct LocalGroup;

struct Member {
    LocalGroup *g = nullptr;
    int rank = 0, device = 0;
    hipStream_t stream = nullptr;     // copies of the all-gather
    DevBuf send, recv;
};

struct LocalGroup {
    int world = 0;
    std::vector<std::unique_ptr<Member>> m;   // (DevBuf is not movable)
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t phase = 0;
    bool aborted = false;
    std::vector<std::vector<int32_t>> red;   // all-reduce slots
    // AOS_GROUP_SERIAL=1 (measurement: tools/tiling_overhead.py): one rank at a time has GPU work in flight. A rank
    // holds `gpu` from its frame's start to its next collective (whose caller has drained its stream) and again
    // around the collective's own copies, so the ranks' kernels never overlap on a shared GPU and a kernel trace
    // sums each rank's work as it would run alone.
    bool serial = false;
    std::mutex gpu;
    void hold() { if (serial) gpu.lock(); }
    void drop() { if (serial) gpu.unlock(); }

    // returns false if the group was aborted (or a rank stalled for 10 minutes)
    bool barrier() {
        std::unique_lock<std::mutex> l(mu);
        if (aborted) return false;
        const uint64_t my = phase;
        if (++arrived == world) {
            arrived = 0;
            ++phase;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(l, std::chrono::minutes(10), [&] { return phase != my || aborted; });
        if (!ok) aborted = true;
        if (aborted) { cv.notify_all(); return false; }
        return true;
    }
    void abort() {
        std::lock_guard<std::mutex> l(mu);
        aborted = true;
        cv.notify_all();
    }
};

// (serial groups: the caller holds the GPU token when a collective starts and gets it back when it returns)
struct SerialGap {
    LocalGroup &g;
    explicit SerialGap(LocalGroup &grp) : g(grp) { g.drop(); }
    ~SerialGap() { g.hold(); }
};

int local_all_gather(void *user, uint64_t bytes) {
    Member &me = *static_cast<Member *>(user);
    LocalGroup &g = *me.g;
    SerialGap gap(g);
    if (!g.barrier()) return -1;   // every rank's send buffer is packed
    std::unique_lock<std::mutex> tok(g.gpu, std::defer_lock);
    if (g.serial) tok.lock();
    if (hipSetDevice(me.device) != hipSuccess) { g.abort(); return -1; }
    for (int r = 0; r < g.world; ++r) {
        const Member &src = *g.m[r];
        char *dst = static_cast<char *>(me.recv.p) + (size_t)r * bytes;
        const hipError_t e = src.device == me.device
                                 ? hipMemcpyAsync(dst, src.send.p, bytes, hipMemcpyDeviceToDevice, me.stream)
                                 : hipMemcpyPeerAsync(dst, me.device, src.send.p, src.device, bytes, me.stream);
        if (e != hipSuccess) { g.abort(); return -1; }
    }
    if (hipStreamSynchronize(me.stream) != hipSuccess) { g.abort(); return -1; }
    if (tok.owns_lock()) tok.unlock();
    return g.barrier() ? 0 : -1;   // nobody repacks its send buffer before every rank has read it
}

// every rank pulls the blocks addressed to it out of the others' send buffers (peer copies over xGMI)
int local_all_to_all(void *user, const uint64_t *counts) {
    Member &me = *static_cast<Member *>(user);
    LocalGroup &g = *me.g;
    SerialGap gap(g);
    if (!g.barrier()) return -1;   // every rank's send buffer is packed
    std::unique_lock<std::mutex> tok(g.gpu, std::defer_lock);
    if (g.serial) tok.lock();
    if (hipSetDevice(me.device) != hipSuccess) { g.abort(); return -1; }
    const int W = g.world;
    uint64_t roff = 0;
    for (int r = 0; r < W; ++r) {
        const Member &src = *g.m[r];
        uint64_t soff = 0;   // rank r's block for me in its send buffer
        for (int q = 0; q < me.rank; ++q) soff += counts[(size_t)r * W + q];
        const uint64_t n = counts[(size_t)r * W + me.rank];
        if (n) {
            char *dst = static_cast<char *>(me.recv.p) + roff;
            const char *sp = static_cast<const char *>(src.send.p) + soff;
            const hipError_t e = src.device == me.device
                                     ? hipMemcpyAsync(dst, sp, n, hipMemcpyDeviceToDevice, me.stream)
                                     : hipMemcpyPeerAsync(dst, me.device, sp, src.device, n, me.stream);
            if (e != hipSuccess) { g.abort(); return -1; }
        }
        roff += n;
    }
    if (hipStreamSynchronize(me.stream) != hipSuccess) { g.abort(); return -1; }
    if (tok.owns_lock()) tok.unlock();
    return g.barrier() ? 0 : -1;
}

int local_all_reduce_max(void *user, int32_t *v, int32_t n) {
    Member &me = *static_cast<Member *>(user);
    LocalGroup &g = *me.g;
    SerialGap gap(g);
    g.red[me.rank].assign(v, v + n);
    if (!g.barrier()) return -1;
    for (int r = 0; r < g.world; ++r) {
        if ((int)g.red[r].size() != n) { g.abort(); return -1; }
        for (int i = 0; i < n; ++i) v[i] = std::max(v[i], g.red[r][i]);
    }
    return g.barrier() ? 0 : -1;
}

}  // namespace
}  // namespace aos

using namespace aos;

struct aos_group {
    int tiles_x = 1, tiles_y = 1, root = 0;
    std::vector<aos_ctx *> ranks;
    LocalGroup g;
    std::vector<aos_tile_plan> plans;
    Poly poly;
    bool poly_set = false;
};

extern "C" {

int aos_group_create(const aos_params *p, const int32_t *devices, int32_t tiles_x, int32_t tiles_y, aos_group **out) {
    if (!p || !devices || !out) { set_error("aos_group_create: null argument"); return AOS_E_INVALID; }
    *out = nullptr;
    if (tiles_x < 1 || tiles_y < 1 || tiles_x > kMaxTiles || tiles_y > kMaxTiles) {
        set_error("aos_group_create: tiles_x / tiles_y out of range");
        return AOS_E_INVALID;
    }
    auto *G = new (std::nothrow) aos_group();
    if (!G) { set_error("out of host memory"); return AOS_E_NOMEM; }
    G->tiles_x = tiles_x;
    G->tiles_y = tiles_y;
    const int world = tiles_x * tiles_y;
    G->g.world = world;
    {
        const char *e = getenv("AOS_GROUP_SERIAL");
        G->g.serial = e && atoi(e) != 0;
    }
    for (int r = 0; r < world; ++r) G->g.m.emplace_back(new Member());
    G->g.red.resize(world);
    for (int r = 0; r < world; ++r) {
        aos_ctx *c = nullptr;
        const int rc = aos_create(p, devices[r], &c);
        if (rc != AOS_OK) { for (aos_ctx *x : G->ranks) aos_destroy(x); delete G; return rc; }
        G->ranks.push_back(c);
        Member &m = *G->g.m[r];
        m.g = &G->g;
        m.rank = r;
        m.device = devices[r];
    }
    try {
        for (int r = 0; r < world; ++r) {
            Member &m = *G->g.m[r];
            DeviceScope dev(m.device);
            AOS_HIP(hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking));
            for (int q = 0; q < world; ++q) {   // peer access for the all-gather pulls (xGMI)
                const int d = devices[q];
                int can = 0;
                if (d != m.device && hipDeviceCanAccessPeer(&can, m.device, d) == hipSuccess && can) {
                    const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) AOS_HIP(e);
                    (void)hipGetLastError();
                }
            }
        }
    } catch (const HipError &e) {
        set_error(std::string("aos_group_create: HIP error ") + hipGetErrorString(e.e) + ": " + e.what);
        aos_group_destroy(G);
        return AOS_E_HIP;
    }
    *out = G;
    return AOS_OK;
}

void aos_group_destroy(aos_group *G) {
    if (!G) return;
    for (size_t r = 0; r < G->g.m.size(); ++r) {
        Member &m = *G->g.m[r];
        if (m.stream) {
            (void)hipSetDevice(m.device);
            (void)hipStreamDestroy(m.stream);
        }
        m.send.release();
        m.recv.release();
    }
    for (aos_ctx *c : G->ranks) aos_destroy(c);
    delete G;
}

int aos_group_set_polygon(aos_group *G, const double *xy, uint32_t n) {
    if (!G) { set_error("aos_group_set_polygon: null handle"); return AOS_E_INVALID; }
    for (aos_ctx *c : G->ranks) {
        const int rc = aos_set_polygon(c, xy, n);
        if (rc != AOS_OK) return rc;
    }
    return AOS_OK;
}

int aos_group_plan(aos_group *G, int32_t rank, aos_tile_plan *out) {
    if (!G || !out || rank < 0 || rank >= (int)G->ranks.size()) { set_error("aos_group_plan: bad argument"); return AOS_E_INVALID; }
    aos_ctx *c = G->ranks[rank];
    std::vector<double> xy;
    for (const auto &q : c->poly) { xy.push_back(q.first); xy.push_back(q.second); }
    return aos_tile_plan_compute(&c->P, xy.data(), (uint32_t)(xy.size() / 2), G->tiles_x, G->tiles_y, rank, out);
}

aos_ctx *aos_group_rank(aos_group *G, int32_t rank) {
    if (!G || rank < 0 || rank >= (int)G->ranks.size()) return nullptr;
    return G->ranks[rank];
}

}  // extern "C"

// Runs frame(rank, comm, out) on every rank (one thread each, plans and communicator buffers sized for
// the current geometry); the first failing rank aborts the others' collectives.
template <class F>
static int group_run(aos_group *G, int32_t root, aos_seedgen_out *root_out, const char *what, F frame) {
    const int world = (int)G->ranks.size();
    if (root < 0 || root >= world) { set_error(std::string(what) + ": bad root"); return AOS_E_INVALID; }
    std::vector<aos_comm> comms(world);
    for (int r = 0; r < world; ++r) {
        aos_tile_plan plan{};
        const int rc = aos_group_plan(G, r, &plan);
        if (rc != AOS_OK) return rc;
        Member &m = *G->g.m[r];
        try {
            DeviceScope dev(m.device);
            m.send.ensure(std::max<uint64_t>(plan.exchange_bytes, 1));
            m.recv.ensure((size_t)world * std::max<uint64_t>(plan.exchange_bytes, 1));
        } catch (const HipError &e) {
            set_error(std::string(what) + ": HIP error " + hipGetErrorString(e.e));
            return AOS_E_HIP;
        }
        comms[r] = aos_comm{&m, r, world, m.send.p, m.recv.p, plan.exchange_bytes, local_all_gather, local_all_reduce_max,
                            local_all_to_all};
    }
    {
        std::lock_guard<std::mutex> l(G->g.mu);
        G->g.aborted = false;
        G->g.arrived = 0;
    }
    std::vector<aos_seedgen_out> outs(world);
    std::mutex fail_mu;
    int fail_rank = -1, fail_rc = AOS_OK;
    std::string fail_msg;
    auto run = [&](int r) {
        G->g.hold();   // (serial groups: the frame's first GPU work; the collectives hand the token on)
        const int rc = frame(r, &comms[r], &outs[r]);
        if (G->g.serial) {   // (its last work is done before the token goes: the next rank's trace starts clean)
            DeviceScope dev(G->g.m[r]->device);
            (void)hipDeviceSynchronize();
        }
        G->g.drop();
        if (rc != AOS_OK) {
            {
                std::lock_guard<std::mutex> l(fail_mu);
                if (fail_rank < 0) { fail_rank = r; fail_rc = rc; fail_msg = aos_last_error(); }   // the root cause
            }
            G->g.abort();   // the other ranks leave their next collective
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < world; ++r) th.emplace_back(run, r);
    run(0);
    for (auto &t : th) t.join();
    if (fail_rank >= 0) {
        set_error(std::string(what) + ": rank " + std::to_string(fail_rank) + ": " + fail_msg);
        return fail_rc;
    }
    *root_out = outs[root];
    return AOS_OK;
}

extern "C" {

int aos_group_process(aos_group *G, const aos_cloud_view *clouds, int32_t root, int want_host, aos_seedgen_out *root_out) {
    if (!G || !clouds || !root_out) { set_error("aos_group_process: null argument"); return AOS_E_INVALID; }
    return group_run(G, root, root_out, "aos_group_process", [&](int r, const aos_comm *cm, aos_seedgen_out *o) {
        return aos_tiled_seedgen_process(G->ranks[r], cm, G->tiles_x, G->tiles_y, root, &clouds[r], r == root ? want_host : 0, o);
    });
}

int aos_group_map_reset(aos_group *G, uint64_t reserve_points) {
    if (!G) { set_error("aos_group_map_reset: null handle"); return AOS_E_INVALID; }
    for (aos_ctx *c : G->ranks) {
        const int rc = aos_map_reset(c, reserve_points);
        if (rc != AOS_OK) return rc;
    }
    return AOS_OK;
}

int aos_group_map_append(aos_group *G, const aos_cloud_view *scan, int32_t root, int want_host, aos_seedgen_out *root_out) {
    if (!G || !scan || !root_out) { set_error("aos_group_map_append: null argument"); return AOS_E_INVALID; }
    return group_run(G, root, root_out, "aos_group_map_append", [&](int r, const aos_comm *cm, aos_seedgen_out *o) {
        return aos_tiled_map_append(G->ranks[r], cm, G->tiles_x, G->tiles_y, root, scan, r == root ? want_host : 0, o);
    });
}

}  // extern "C"
