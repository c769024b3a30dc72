// Tiled multi-GPU seed-gen frame (BASELINE.json configs[3]: 8192^2 in 2 x 4 tiles).
//
// One map, tiles_x x tiles_y tiles, one rank per tile; a rank is a handle on its own GPU plus an
// aos_comm (all-gather + max all-reduce: RCCL over xGMI in production). A rank runs a1-a7 on a
// window = its own tile plus a halo of G rows and G/64 words per side, clamped at the map edge,
// with the single-GPU kernels unchanged. A window edge that is not a map edge acts as an image
// border. That can only corrupt cells from the edge inward: R cells for the inflation, 2 for the
// opening and 1 per Zhang-Suen sub-iteration. Before the damage reaches the tile, the halo is
// refreshed from the neighbours' exact border strips (each tile's strips to its 3-8 neighbouring tiles; an
// all-gather through a communicator without point-to-point collectives):
//   ROR + raster (own cells) -> exchange -> inflate -> open -> thin (G - R - 2 sub-iterations)
//   -> [exchange -> thin (G sub-iterations)]* until converged.
// Convergence is global: each rank flags the iterations that deleted one of its OWN cells, the
// flags are max-reduced over ranks and the ximgproc stopping rule runs on the reduced flags. After
// the first iteration that deletes nothing anywhere the map is a fixed point, so the extra
// iterations of the last period change no own cell. Finally the bit-packed skeleton and inflated
// tiles go to the frame's root, which finishes the frame (a6, a16, seeds) on the whole map exactly like
// aos_seedgen_process, with a8-a10 shared over the ranks (cluster_dist.hip): every output is
// byte-identical to the single-GPU frame. With the library's RCCL communicator the collectives are
// enqueued on the frame's stream (FrameComm / StreamColl): the host waits once per thinning period.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "aos_ctx.h"

namespace aos {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

TilePlan make_tile_plan(const FrameGeom &g, float margin, int tiles_x, int tiles_y, int rank) {
    if (tiles_x < 1 || tiles_y < 1 || tiles_x > kMaxTiles || tiles_y > kMaxTiles)
        throw std::invalid_argument("tiles_x and tiles_y must be in [1, 16]");
    if (rank < 0 || rank >= tiles_x * tiles_y) throw std::invalid_argument("rank outside the tiling");
    TilePlan t{};
    t.tiles_x = tiles_x; t.tiles_y = tiles_y; t.rank = rank;
    t.tx = rank % tiles_x; t.ty = rank / tiles_x;
    // halo: inflation (R) + opening (2) + one thinning launch (2 KIT sub-iterations) before the
    // first refresh, in whole words so that tile edges stay word-aligned
    t.gw = (g.R + 2 + 2 * kThinItersPerLaunch + 63) / 64;
    t.G = 64 * t.gw;
    t.hy = tiles_y > 1 ? t.G : 0;
    t.hw = tiles_x > 1 ? t.gw : 0;
    for (int i = 0; i <= tiles_y; ++i) t.rs[i] = (int)((long long)g.H * i / tiles_y);
    for (int i = 0; i <= tiles_x; ++i) t.cs[i] = (int)((long long)g.WW * i / tiles_x);
    for (int y = 0; y < tiles_y; ++y)
        for (int x = 0; x < tiles_x; ++x) {
            const long long nr = t.rs[y + 1] - t.rs[y], nc = t.cs[x + 1] - t.cs[x];
            if (nr < std::max(t.hy, 1) || nc < std::max(t.hw, 1))
                throw std::invalid_argument("tile smaller than its halo: " + std::to_string(nr) + " rows x " +
                                            std::to_string(nc) + " words, halo " + std::to_string(t.G) + " cells");
            t.max_border = std::max(t.max_border, 2LL * t.hy * nc + 2LL * nr * t.hw);
            t.max_own = std::max(t.max_own, nr * nc);
        }
    t.y0 = t.rs[t.ty]; t.y1 = t.rs[t.ty + 1]; t.c0 = t.cs[t.tx]; t.c1 = t.cs[t.tx + 1];
    t.wy0 = std::max(0, t.y0 - t.hy); t.wy1 = std::min(g.H, t.y1 + t.hy);
    t.wc0 = std::max(0, t.c0 - t.hw); t.wc1 = std::min(g.WW, t.c1 + t.hw);
    t.lg = g;
    t.lg.W = std::min(g.W, 64 * t.wc1) - 64 * t.wc0;
    t.lg.H = t.wy1 - t.wy0;
    t.lg.WW = t.wc1 - t.wc0;
    // points whose (truncated) cell can be an own cell, one cell of slack, and their ROR neighbours
    const int x0 = 64 * t.c0, x1 = std::min(g.W, 64 * t.c1);
    t.box[0] = (float)(g.origin_x + (double)(x0 - 1) * g.res) - margin;
    t.box[1] = (float)(g.origin_y + (double)(t.y0 - 1) * g.res) - margin;
    t.box[2] = (float)(g.origin_x + (double)(x1 + 1) * g.res) + margin;
    t.box[3] = (float)(g.origin_y + (double)(t.y1 + 1) * g.res) + margin;
    t.exchange_bytes = 8ull * (uint64_t)std::max(t.max_border, 2 * t.max_own);
    return t;
}

// Kernel view of the tiling; stride = words per rank in the gathered buffer.
struct TileSplit {
    int tiles_x, tiles_y, hy, hw;
    int rs[kMaxTiles + 1], cs[kMaxTiles + 1];
    long long stride;
};
static TileSplit split_of(const TilePlan &t, long long stride) {
    TileSplit S{};
    S.tiles_x = t.tiles_x; S.tiles_y = t.tiles_y; S.hy = t.hy; S.hw = t.hw; S.stride = stride;
    std::memcpy(S.rs, t.rs, sizeof(S.rs));
    std::memcpy(S.cs, t.cs, sizeof(S.cs));
    return S;
}
__device__ __forceinline__ int tile_row(const TileSplit &S, int gy) {
    int ty = 0;
    while (ty + 1 < S.tiles_y && gy >= S.rs[ty + 1]) ++ty;
    return ty;
}
__device__ __forceinline__ int tile_col(const TileSplit &S, int gc) {
    int tx = 0;
    while (tx + 1 < S.tiles_x && gc >= S.cs[tx + 1]) ++tx;
    return tx;
}

// A tile's border strips, one rank's chunk: top [hy][nc], bottom [hy][nc], left [nr][hw], right [nr][hw].
__global__ void k_pack_border(const uint64_t *win, int WWl, int oy, int oc, int nr, int nc, int hy, int hw,
                              uint64_t *out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long a = (long long)hy * nc, b = (long long)nr * hw;
    if (i >= 2 * (a + b)) return;
    long long r, k;
    if (i < a) { r = i / nc; k = i % nc; }
    else if (i < 2 * a) { const long long j = i - a; r = nr - hy + j / nc; k = j % nc; }
    else if (i < 2 * a + b) { const long long j = i - 2 * a; r = j / hw; k = j % hw; }
    else { const long long j = i - 2 * a - b; r = j / hw; k = nc - hw + j % hw; }
    out[i] = win[(oy + r) * WWl + oc + k];
}

// Halo words of the window <- their owners' border strips in the gathered buffer. A halo word lies
// within hy rows / hw words of this tile, i.e. inside the facing strip of a neighbour.
__global__ void k_unpack_halo(uint64_t *win, int WWl, int Hl, int wy0, int wc0, int y0, int y1, int c0, int c1,
                              TileSplit S, const uint64_t *recv) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
    if (k >= WWl || r >= Hl) return;
    const int gy = wy0 + r, gc = wc0 + k;
    if (gy >= y0 && gy < y1 && gc >= c0 && gc < c1) return;   // own word
    const int ty = tile_row(S, gy), tx = tile_col(S, gc);
    const int ty0 = S.rs[ty], ty1 = S.rs[ty + 1], tc0 = S.cs[tx], tc1 = S.cs[tx + 1];
    const long long nr = ty1 - ty0, nc = tc1 - tc0, a = (long long)S.hy * nc;
    const uint64_t *b = recv + (long long)(ty * S.tiles_x + tx) * S.stride;
    long long i;
    if (gy < ty0 + S.hy) i = (long long)(gy - ty0) * nc + (gc - tc0);
    else if (gy >= ty1 - S.hy) i = a + (long long)(gy - (ty1 - S.hy)) * nc + (gc - tc0);
    else if (gc < tc0 + S.hw) i = 2 * a + (long long)(gy - ty0) * S.hw + (gc - tc0);
    else i = 2 * a + nr * S.hw + (long long)(gy - ty0) * S.hw + (gc - (tc1 - S.hw));
    win[(long long)r * WWl + k] = b[i];
}

// Own words of two window grids -> [nr][nc] blocks, a then b.
__global__ void k_pack_own2(const uint64_t *a, const uint64_t *b, int WWl, int oy, int oc, int nr, int nc,
                            uint64_t *out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x, n = (long long)nr * nc;
    if (i >= n) return;
    const long long r = i / nc, k = i % nc, w = (oy + r) * WWl + oc + k;
    out[i] = a[w];
    out[n + i] = b[w];
}

// Gathered tiles -> the two whole-map grids.
__global__ void k_unpack_full2(const uint64_t *recv, TileSplit S, int WW, int H, uint64_t *a, uint64_t *b) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (c >= WW || y >= H) return;
    const int ty = tile_row(S, y), tx = tile_col(S, c);
    const long long nc = S.cs[tx + 1] - S.cs[tx], n = (long long)(S.rs[ty + 1] - S.rs[ty]) * nc;
    const uint64_t *src = recv + (long long)(ty * S.tiles_x + tx) * S.stride;
    const long long i = (long long)(y - S.rs[ty]) * nc + (c - S.cs[tx]);
    a[(long long)y * WW + c] = src[i];
    b[(long long)y * WW + c] = src[n + i];
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// ------------------------------------------------------------------ FrameComm (aos_internal.h)
FrameComm::FrameComm(const aos_comm &cm, std::vector<hipEvent_t> &pool, DevBuf &scratch) : c(cm), ev(pool), red(scratch) {
    rccl_stream_coll(cm, sc);
}

namespace {
// events around one enqueued collective (the pool grows once, then is reused frame after frame); a pair that
// cannot be created or recorded is left out of the timing, never half-counted
struct EnqTimer {
    FrameComm &f;
    hipStream_t s;
    bool ok = false;
    EnqTimer(FrameComm &fc, hipStream_t st) : f(fc), s(st) {
        while ((int)f.ev.size() < f.ev_used + 2) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return;   // (timing only)
            f.ev.push_back(e);
        }
        ok = hipEventRecord(f.ev[f.ev_used], s) == hipSuccess;
    }
    ~EnqTimer() {
        if (ok && hipEventRecord(f.ev[f.ev_used + 1], s) == hipSuccess) f.ev_used += 2;
    }
};
}  // namespace

float FrameComm::ms_enqueued() {
    if (ev_used < 2) return 0.0f;
    (void)hipEventSynchronize(ev[ev_used - 1]);
    float tot = 0.0f;
    for (int i = 0; i + 1 < ev_used; i += 2) {
        float v = 0.0f;
        if (hipEventElapsedTime(&v, ev[i], ev[i + 1]) == hipSuccess) tot += v;
    }
    return tot;
}

void FrameComm::all_gather(uint64_t bytes, hipStream_t s) {
    ++n_gather;
    bytes_sent += bytes;
    bytes_recv += (uint64_t)(c.world - 1) * bytes;
    if (ordered()) {
        EnqTimer t(*this, s);
        sc.all_gather(sc.impl, bytes, s);
        return;
    }
    AOS_HIP(hipStreamSynchronize(s));   // (the callbacks run with the stream idle: the send buffer is packed)
    const auto t0 = std::chrono::steady_clock::now();
    const int r = c.all_gather(c.user, bytes);
    ms_gather += ms_since(t0);
    if (r != 0) throw CommError{"aos_comm.all_gather failed"};
}

void FrameComm::neighbour_exchange(uint64_t bytes, const uint8_t *peer, hipStream_t s) {
    if (!ordered() || !sc.exchange) return all_gather(bytes, s);
    ++n_gather;
    for (int r = 0; r < c.world; ++r)
        if (r != c.rank && peer[r]) { bytes_sent += bytes; bytes_recv += bytes; }
    EnqTimer t(*this, s);
    sc.exchange(sc.impl, bytes, peer, s);
}

void FrameComm::all_to_all(const uint64_t *counts, hipStream_t s) {
    ++n_gather;
    for (int d = 0; d < c.world; ++d)
        if (d != c.rank) {
            bytes_sent += counts[(size_t)c.rank * c.world + d];
            bytes_recv += counts[(size_t)d * c.world + c.rank];
        }
    if (ordered()) {
        EnqTimer t(*this, s);
        sc.all_to_all(sc.impl, counts, s);
        return;
    }
    if (!c.all_to_all) throw std::logic_error("FrameComm::all_to_all without aos_comm.all_to_all");
    AOS_HIP(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    const int r = c.all_to_all(c.user, counts);
    ms_gather += ms_since(t0);
    if (r != 0) throw CommError{"aos_comm.all_to_all failed"};
}

void FrameComm::gather(uint64_t bytes, int root, hipStream_t s) {
    if (ordered()) {
        ++n_gather;
        bytes_sent += c.rank == root ? 0 : bytes;
        bytes_recv += c.rank == root ? (uint64_t)(c.world - 1) * bytes : 0;
        EnqTimer t(*this, s);
        sc.gather(sc.impl, bytes, root, s);
        return;
    }
    if (!c.all_to_all) return all_gather(bytes, s);
    // the personalised exchange with one non-zero column: every rank's block to the root (its own included),
    // landing at block r of the root's recv_buf as an all-gather would put it
    std::vector<uint64_t> counts((size_t)c.world * c.world, 0);
    for (int r = 0; r < c.world; ++r) counts[(size_t)r * c.world + root] = bytes;
    all_to_all(counts.data(), s);
}

void FrameComm::max_host(int32_t *v, int n) {
    ++n_reduce;
    const auto t0 = std::chrono::steady_clock::now();
    const int r = c.all_reduce_max(c.user, v, n);
    ms_reduce += ms_since(t0);
    if (r != 0) throw CommError{"aos_comm.all_reduce_max failed"};
}

void FrameComm::max_flags(const int *d, int32_t *h, int n, hipStream_t s) {
    if (ordered()) {   // the reduction on the device, then one read-back and one wait
        ++n_reduce;
        int32_t *dr = static_cast<int32_t *>(red.ensure(sizeof(int32_t) * (size_t)std::max(n, 1)));
        AOS_HIP(hipMemcpyAsync(dr, d, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToDevice, s));
        {
            EnqTimer t(*this, s);
            sc.max_dev(sc.impl, dr, n, s);
        }
        AOS_HIP(hipMemcpyAsync(h, dr, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        return;
    }
    AOS_HIP(hipMemcpyAsync(h, d, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
    AOS_HIP(hipStreamSynchronize(s));
    max_host(h, n);
}

}  // namespace aos

using namespace aos;

// Refresh the halo of a window grid (in place) from the neighbours' border strips.
void aos_ctx::tile_halo_exchange(uint64_t *win, const TilePlan &t, FrameComm &fc) {
    if (!t.hy && !t.hw) return;
    const int nr = t.y1 - t.y0, nc = t.c1 - t.c0;
    const long long n = 2LL * t.hy * nc + 2LL * nr * t.hw;
    k_pack_border<<<cdiv(n, 256), 256, 0, stream>>>(win, t.lg.WW, t.y0 - t.wy0, t.c0 - t.wc0, nr, nc, t.hy, t.hw,
                                                    static_cast<uint64_t *>(fc.c.send_buf));
    AOS_HIP(hipGetLastError());
    // the strips go to the tiles next to this one only (8-neighbourhood: a halo word lies in an adjacent tile,
    // the plan keeps every tile at least as large as the halo); symmetric, so every rank pairs its sends
    std::vector<uint8_t> peer((size_t)fc.c.world, 0);
    for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
            const int x = t.tx + dx, y = t.ty + dy;
            if ((dx || dy) && x >= 0 && x < t.tiles_x && y >= 0 && y < t.tiles_y) peer[(size_t)y * t.tiles_x + x] = 1;
        }
    fc.neighbour_exchange(8ull * (uint64_t)t.max_border, peer.data(), stream);
    const TileSplit S = split_of(t, t.max_border);
    dim3 grid(cdiv(t.lg.WW, 64), t.lg.H);
    k_unpack_halo<<<grid, 64, 0, stream>>>(win, t.lg.WW, t.lg.H, t.wy0, t.wc0, t.y0, t.y1, t.c0, t.c1, S,
                                           static_cast<const uint64_t *>(fc.c.recv_buf));
    AOS_HIP(hipGetLastError());
}

void aos_ctx::run_tiled(const aos_comm &cm, int tiles_x, int tiles_y, int root, bool want_host, aos_seedgen_out &out) {
    FrameComm fc(cm, coll_ev, coll_red);
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t skipped0 = ror_skipped;
    auto record = [&]() {
        tstats = aos_tiled_stats{};
        tstats.ms_frame = (float)ms_since(t0);
        tstats.ms_comm_gather = (float)fc.ms_gather;
        tstats.ms_comm_reduce = (float)fc.ms_reduce;
        if (fc.ordered()) tstats.ms_comm_gather += fc.ms_enqueued();   // (device time of the enqueued ones)
        tstats.n_gather = fc.n_gather;
        tstats.n_reduce = fc.n_reduce;
        tstats.bytes_gather = fc.bytes_sent;
        tstats.bytes_recv = fc.bytes_recv;
        tstats.ms_cluster_local = cdist_stats.ms_local;
        tstats.ms_cluster_global = cdist_stats.ms_global;
        tstats.ms_replay = cdist_stats.ms_replay;
        tstats.n_replayed = cdist_stats.n_replayed_here;
        tstats.ror_skipped = ror_skipped != skipped0 ? 1 : 0;
        tstats.is_root = cm.rank == root ? 1 : 0;
    };
    try {
        run_tiled_frame(fc, tiles_x, tiles_y, root, want_host, out);
    } catch (...) {
        record();
        throw;
    }
    record();
    tstats.ms_ror = out.ms_ror;
    tstats.ms_thin = out.ms_thin;
    tstats.ms_cluster = out.ms_cluster;
    tstats.ms_seeds = out.ms_seeds;
}

void aos_ctx::run_tiled_frame(FrameComm &fc, int tiles_x, int tiles_y, int root, bool want_host, aos_seedgen_out &out) {
    const aos_comm &cm = fc.c;
    std::memset(&out, 0, sizeof(out));
    have_frame = false;
    tiled_frame = true;
    infl_bits_sent = false;
    skel_bits = nullptr;
    const FrameGeom g = frame_geom(poly, P);
    geom = g;
    if (g.R > 63) throw std::runtime_error("inflation radius > 63 cells is not supported by the bit-packed kernel");
    if ((size_t)g.W * g.H > (size_t)1 << 31) throw std::runtime_error("grid larger than 2^31 cells");
    if (cm.world != tiles_x * tiles_y) throw std::invalid_argument("aos_comm.world != tiles_x * tiles_y");
    if (root < 0 || root >= cm.world) throw std::invalid_argument("root outside the tiling");
    const TilePlan t = make_tile_plan(g, ror_margin(P), tiles_x, tiles_y, cm.rank);
    if (!cm.all_gather || !cm.all_reduce_max || !cm.send_buf || !cm.recv_buf || cm.buf_bytes < t.exchange_bytes)
        throw std::invalid_argument("aos_comm: a callback or buffer is missing, or buf_bytes < exchange_bytes = " +
                                    std::to_string(t.exchange_bytes));
    hipStream_t s = stream;
    const FrameGeom &lg = t.lg;
    const size_t Cwl = (size_t)lg.WW * lg.H;
    AOS_HIP(hipEventRecord(ev[0], s));

    // ---- a1-a4 for the candidates whose cell is an own cell, rastered into the window
    RorOwn own{64 * t.c0, t.y0, std::min(g.W, 64 * t.c1), t.y1, 64 * t.wc0, t.wy0, lg.W, lg.H, true,
               {t.box[0], t.box[1], t.box[2], t.box[3]}};
    uint64_t *d_rbits = static_cast<uint64_t *>(raster_bits.ensure(Cwl * 8));
    ror_stage(g, own, d_rbits, false);   // sized by a read-back: a rank cannot redo a frame alone
    AOS_HIP(hipEventRecord(ev[1], s));

    // ---- raster halo from the neighbours, a5 inflation on the window
    uint64_t *d_ibits = static_cast<uint64_t *>(infl_bits.ensure(Cwl * 8));
    tile_halo_exchange(d_rbits, t, fc);
    launch_inflate(d_rbits, d_ibits, lg, s);
    AOS_HIP(hipEventRecord(ev[2], s));

    // ---- a7 opening + Zhang-Suen in halo periods
    uint64_t *d_open = static_cast<uint64_t *>(open_bits.ensure(Cwl * 8));
    uint64_t *bufs[2] = {static_cast<uint64_t *>(thin_a.ensure(Cwl * 8)), static_cast<uint64_t *>(thin_b.ensure(Cwl * 8))};
    const int K = kThinItersPerLaunch;
    const int max_iters = std::max(g.W, g.H) + 4;
    const bool halo = t.hy || t.hw;
    const int nflags = 2 + max_iters + t.G / 2 + 4 * K;   // a period may run G / 2 iterations past T
    int *d_flags = static_cast<int *>(flags.ensure(sizeof(int) * nflags));
    launch_open(d_ibits, d_open, lg, s, d_flags, nflags);   // (the opening clears the flags: no fill launch)
    int *h_flags = static_cast<int *>(h_small.ensure(sizeof(int) * nflags));
    const ThinOwn mine{t.y0 - t.wy0, t.y1 - t.wy0, t.c0 - t.wc0, t.c1 - t.wc0, 0};
    uint64_t *cur = d_open;
    int launched = 0, T = 0;
    long long budget = halo ? t.G - g.R - 2 : LLONG_MAX;   // sub-iterations the halo still supports
    std::vector<int32_t> fl;
    for (int period = 0;; ++period) {
        int nl = halo ? (int)(budget / (2 * K)) : (period == 0 ? 3 : 4);
        if (nl < 1) throw std::logic_error("tile halo too small for one thinning launch");
        // the first period stops where the last frame's T says the thinning ends (as the single-GPU frame sizes
        // its first batch): a tiled launch cannot skip itself past convergence, so a spare one costs a full pass
        if (period == 0) nl = std::min(nl, std::max(2, (thin_iters + 2 + K - 1) / K));
        for (int j = 0; j < nl; ++j) {
            uint64_t *dst = bufs[launched & 1];
            launch_thin_block(cur, dst, lg, launched * K, d_flags, mine, s);
            cur = dst;
            ++launched;
        }
        if (halo) budget -= 2LL * K * nl;
        const int nf = 1 + launched * K;
        fc.max_flags(d_flags, h_flags, nf, s);   // (the period's one host wait: the stop rule runs on the host)
        fl.assign(h_flags, h_flags + nf);
        T = thin_iterations(fl.data(), launched * K);
        if (T) break;
        if (launched * K > max_iters) throw std::runtime_error("thinning did not converge");
        if (halo) {
            tile_halo_exchange(cur, t, fc);
            budget = t.G;
        }
    }
    thin_iters = T;
    AOS_HIP(hipEventRecord(ev[3], s));

    // ---- kept candidates over all tiles: each rank fills its own slot, max = sum of the slots
    unsigned long long *h_cnt = static_cast<unsigned long long *>(h_stats.ensure(64 + 8 * kRorCounters)) + 8;
    AOS_HIP(hipMemcpyAsync(h_cnt, counters.p, 8 * kRorCounters, hipMemcpyDeviceToHost, s));
    AOS_HIP(hipStreamSynchronize(s));
    // (sized by a read-back, so no staging overflow is expected; a streaming store's merge can still
    // overflow a stale size: the bits travel with the counts and every rank fails the frame together)
    if (g_debug_stuck_rank.load(std::memory_order_relaxed) == cm.rank)   // (tests: this rank's column scan "got stuck")
        reinterpret_cast<unsigned long long *>(static_cast<int *>(h_stats.p) + 4)[1] |= 4;
    const bool ror_over = ror_collect(false);   // (bit 4, a stuck look-back, travels with the others)
    const int ror_bits = ror_over ? (int)reinterpret_cast<const unsigned long long *>(static_cast<const int *>(h_stats.p) + 4)[1] : 0;
    uint64_t mine_cnt = 0;
    for (int i = 0; i < kRorCounters; ++i) mine_cnt += h_cnt[i];
    std::vector<int32_t> slots(2 * (size_t)cm.world + 1, 0);
    slots[2 * cm.rank] = (int32_t)(mine_cnt & 0x7fffffff);
    slots[2 * cm.rank + 1] = (int32_t)(mine_cnt >> 31);
    slots[2 * cm.world] = ror_bits;
    fc.max_host(slots.data(), (int)slots.size());
    if (slots[2 * cm.world])
        throw std::runtime_error("tiled frame: ROR stage overflow on a rank (bits " + std::to_string(slots[2 * cm.world]) +
                                 ": 1 staged capacity / store merge, 2 a tile beyond the LDS capacity, 4 a stuck look-back "
                                 "wait in the ROR column scan)");
    uint64_t total = 0;
    for (int r = 0; r < cm.world; ++r) total += (uint64_t)slots[2 * r] | ((uint64_t)slots[2 * r + 1] << 31);

    // ---- the own skeleton + inflated words to the root, which finishes the frame on the whole map (only the root
    // receives them when the communicator has a personalised exchange: the other ranks need no whole-map grid)
    const int nr = t.y1 - t.y0, nc = t.c1 - t.c0;
    k_pack_own2<<<cdiv((long long)nr * nc, 256), 256, 0, s>>>(cur, d_ibits, lg.WW, t.y0 - t.wy0, t.c0 - t.wc0, nr,
                                                               nc, static_cast<uint64_t *>(cm.send_buf));
    AOS_HIP(hipGetLastError());
    fc.gather(16ull * (uint64_t)t.max_own, root, s);
    uint64_t *fs = nullptr;
    if (cm.rank == root) {
        const size_t Cw = (size_t)g.WW * g.H;
        fs = static_cast<uint64_t *>(full_skel.ensure(Cw * 8));
        uint64_t *fi = static_cast<uint64_t *>(full_infl.ensure(Cw * 8));
        const TileSplit S = split_of(t, 2 * t.max_own);
        k_unpack_full2<<<dim3(cdiv(g.WW, 64), g.H), 64, 0, s>>>(static_cast<const uint64_t *>(cm.recv_buf), S, g.WW,
                                                                g.H, fs, fi);
        AOS_HIP(hipGetLastError());
        int8_t *d_occ = static_cast<int8_t *>(occ_bytes.ensure((size_t)g.W * g.H));
        launch_bits_to_bytes(fi, d_occ, g, 5, s);   // a6 /occupancy_grid
    }

    // ---- a8-a10 over the ranks: own-tile labelling, border union-find, shared statistics / replays
    AOS_HIP(hipEventRecord(ev[6], s));
    PreClusters pre;
    cluster_dist(cdist, fc, t, g, poly, static_cast<float>(P.cluster_min_length), cur, root, s, pre, cdist_stats);
    if (cm.rank == root) {
        skel_bits = fs;
        finish_frame(g, want_host, &total, out, &pre);
        return;
    }
    n_clipped = total;
    out.info = aos_grid_info{g.origin_x, g.origin_y, g.res, (uint32_t)g.W, (uint32_t)g.H};
    out.thin_iters = T;
    out.n_input = (d_cloud == map_buf.as<uint8_t>() && n_points == map_n) ? map_total : n_points;
    out.n_clipped = total;
    auto ms = [&](int a, int b) { float v = 0; (void)hipEventElapsedTime(&v, ev[a], ev[b]); return v; };
    AOS_HIP(hipEventRecord(ev[4], s));
    AOS_HIP(hipEventSynchronize(ev[4]));
    out.ms_ror = ms(0, 1); out.ms_grid = ms(1, 2); out.ms_thin = ms(2, 3); out.ms_cluster = ms(6, 4);
    out.ms_total = ms(0, 4);
    out.n_binned = static_cast<const int *>(h_stats.p)[0];
    out.ms_ror_count = out.n_binned ? ms(10, 11) : 0.0f;
    out.ms_ror_bin = out.n_binned ? ms(12, 13) : 0.0f;
    out.ms_ror_scatter = out.n_binned ? ms(14, 10) : 0.0f;
    out.n_ror_read = ror_read;
}
