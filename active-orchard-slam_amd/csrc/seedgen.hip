// Seed-gen frame orchestration (AosSeedGenNode::processPointCloud, seed_gen:452-579) on one
// HIP stream. Host work is limited to launch geometry derived from the polygon (a few scalars);
// every per-point / per-cell stage runs on the GPU. The tiled multi-GPU frame (tiled.hip) reuses
// ror_stage and finish_frame.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <functional>
#include <thread>

#include "aos_ctx.h"
#include "cloud_split.h"
#include "host_pool.h"

using namespace aos;

void aos_ctx::release() {
    for (DevBuf *b : {&cloud_copy, &bin_count, &bin_start, &sorted, &ror_scratch, &ror_bigbins, &scan_tmp, &counters,
                      &raster_bits, &infl_bits, &open_bits, &thin_a, &thin_b, &thin_out, &thin_act, &occ_bytes, &skel_bytes, &flags,
                      &full_infl, &full_skel, &map_buf, &scan_stage, &coll_red})
        b->release();
    for (hipEvent_t e : coll_ev) (void)hipEventDestroy(e);
    coll_ev.clear();
    thin_graphs_release();
    try { expander.join(); } catch (...) {}   // (before its buffers go)
    if (copy_stream) {
        (void)hipStreamSynchronize(copy_stream);
        (void)hipEventDestroy(copy_ready);
        if (copy_done) (void)hipEventDestroy(copy_done);
        copy_done = nullptr;
        (void)hipStreamDestroy(copy_stream);
        copy_stream = nullptr;
    }
    h_small.release();
    h_stats.release();
    h_occ.release();
    h_skel.release();
    h_occ_bits.release();
    h_skel_bits.release();
    for (DevBuf *b : {&cs.fg_bits, &cs.word_cnt, &cs.word_off, &cs.fg_list, &cs.parent, &cs.root_flag, &cs.root_rank,
                      &cs.cl_count, &cs.cl_off, &cs.cl_cursor, &cs.cl_cells, &cs.rec, &cs.row_idx, &cs.cur_tab,
                      &cs.poly, &cs.cand_xy, &cs.cand_ok, &cs.cand_state, &cs.hash_count,
                      &cs.hash_start, &cs.hash_slot, &cs.hash_sorted, &cs.seed_out, &cs.misc, &cs.scan_tmp})
        b->release();
    cs.h_misc.release();
    gvd_async_stop();   // joins the jobs in flight (they use the lanes' GvdStates)
    try { prefetch_join(); } catch (...) {}
    release_uploader();
    for (CloudSplit *sp : {&split_cur, &split_next}) {
        if (sp->copied) { (void)hipEventSynchronize(sp->copied); (void)hipEventDestroy(sp->copied); sp->copied = nullptr; }
        sp->copy_pending = false;
        sp->rest.release();
        sp->on = false;
    }
    free_path_state(path_state);
    path_state = nullptr;
    have_gvd = false;
    for (auto &lp : lanes) {
        GvdState &gs = lp->gs;
        markers_wait(gs, false);
        free_gvd_scratch(gs);
        gs.cells.reset();
        for (DevBuf *b : {&gs.seeds, &gs.merge_state, &gs.hash_count, &gs.hash_start, &gs.hash_slot, &gs.hash_sorted,
                          &gs.scan_tmp, &gs.edges, &gs.bpts, &gs.near_idx, &gs.cand, &gs.cand_ok, &gs.skel,
                          &gs.grid_bytes_ext})
            b->release();
        gs.h_misc.release();
    }
}

// Host PointCloud2 -> HBM. A pageable hipMemcpyAsync of the 160 MB C2 cloud runs at ~20 GB/s: the runtime
// stages it through pinned memory on one thread. Here up_threads() threads each take a range of points,
// gather their x, y, z floats (12 of the record's point_step bytes: the only fields the path reads) into
// a ring of kUpSlots pinned 2 MB slots and DMA them on their own streams, so 25 % fewer bytes cross PCIe
// for the common 16-byte record and the device gets a packed float3 cloud (step 12). With the split
// (CloudSplit, default) only the points inside the binned box go into the slots (C2: 49.5 % of the cloud);
// the others go to the (pageable) rest buffer (cloud_split.cpp: AVX-512 compress, 4 records per register). The
// handle's stream waits for all of them. The caller's buffer is only read during the call.
// Round 4 (profiles/r04v_split_ab.txt): C2's upload ends 2.2-2.8 ms after it starts with the split at 8
// threads, 2.4-3.8 ms without it (4 / 8 / 16 threads); the DMA no longer trails the gather.
// Default 16 (the box's core share per GPU): the gather is bound by each core's memory bandwidth (10 M points: 160 MB
// read, 120 MB written), and 16 threads took ~0.8 ms off the C2 frame against 8 (bench A/B, two rounds alternating:
// frame p50 23.19-23.32 -> 22.09-22.13 ms on one box, profiles/r05zb_upload_threads.txt).
int aos_ctx::up_threads() {
    static const int n = [] {
        const char *e = getenv("AOS_UP_THREADS");
        return e ? std::max(1, std::min(kUpThreads, atoi(e))) : std::min(kUpThreads, host_cpu_share());
    }();
    return n;
}

// AOS_STAGED_TOUCH: 1 (default) the staged array is read while the upload DMAs run; 0 never. (Round 4 also
// measured it beside the count pass on a second stream and on the stage's stream before the count pass: both
// slower, profiles/r04h_ror_variants_touch_ab.txt, r04t_touch_placement_ab.txt.)
static int staged_touch_mode() {
    static const int m = [] { const char *e = getenv("AOS_STAGED_TOUCH"); return e ? atoi(e) : 1; }();
    return m;
}

bool aos_ctx::split_enabled() {
    static const bool on = [] { const char *e = getenv("AOS_UP_SPLIT"); return !e || atoi(e) != 0; }();
    return on;
}

// The ROR stage's binned box for polygon poly (ror_stage computes the same floats the same way)
static void binned_box(const FrameGeom &g, const aos_params &P, float b[6]) {
    const float m = ror_margin(P);
    b[0] = g.minx - m; b[1] = g.maxx + m; b[2] = g.miny - m; b[3] = g.maxy + m;
    b[4] = P.clipping_minz - m; b[5] = P.clipping_maxz + m;
}

bool aos_ctx::split_box(const Poly &pg, float box[6]) const {
    if (!split_enabled()) return false;
    binned_box(frame_geom(pg, P), P, box);
    for (int i = 0; i < 6; ++i)
        if (!std::isfinite(box[i])) return false;
    return box[0] <= box[1] && box[2] <= box[3] && box[4] <= box[5];
}

void aos_ctx::CloudSplit::swap_with(CloudSplit &o) {
    std::swap(rest.p, o.rest.p); std::swap(rest.cap, o.rest.cap);
    std::swap(rbeg, o.rbeg); std::swap(rn, o.rn); std::swap(nth, o.nth);
    std::swap(n_front, o.n_front); std::swap(n_all, o.n_all); std::swap(box, o.box);
    std::swap(on, o.on); std::swap(whole, o.whole); std::swap(copied, o.copied); std::swap(copy_pending, o.copy_pending);
}

// Device points of the handle's host cloud that a ROR stage with binned box b reads: the front when b lies
// inside the split's box, else (first time) the rest is copied behind the front on the handle's stream.
uint64_t aos_ctx::cloud_for_box(const float b[6]) {
    CloudSplit &sp = split_cur;
    if (!sp.on || sp.whole) return sp.n_all;
    if (b[0] >= sp.box[0] && b[1] <= sp.box[1] && b[2] >= sp.box[2] && b[3] <= sp.box[3] && b[4] >= sp.box[4] &&
        b[5] <= sp.box[5])
        return sp.n_front;
    uint64_t at = sp.n_front;
    for (int t = 0; t < sp.nth; ++t) {
        if (!sp.rn[t]) continue;
        AOS_HIP(hipMemcpyAsync(cloud_copy.as<char>() + 12 * at, sp.rest.as<char>() + sp.rbeg[t], 12 * sp.rn[t],
                               hipMemcpyHostToDevice, stream));
        at += sp.rn[t];
    }
    if (!sp.copied) AOS_HIP(hipEventCreateWithFlags(&sp.copied, hipEventDisableTiming));
    AOS_HIP(hipEventRecord(sp.copied, stream));
    sp.copy_pending = true;
    sp.whole = true;
    return sp.n_all;
}

void aos_ctx::upload_pack(void *dst, const aos_cloud_view &v, CloudSplit &sp, bool prefetch) {
    // chunks of AOS_UP_CHUNK_KB (default 2 MB): the last DMAs start soon after the last gather, so the upload
    // ends ~one chunk's DMA after the gather instead of one slot per thread later (8 MB slots: ~1 ms)
    static const uint64_t kChunkPts = [] {
        const char *e = getenv("AOS_UP_CHUNK_KB");
        const long kb = e ? std::max(64L, std::min(65536L, atol(e))) : 2048L;
        return (uint64_t)(kb << 10) / 12;
    }();
    const uint64_t n = v.n_points;
    const int nth = up_threads();
    // AOS_UP_STREAMS (A/B runs): the threads' copies share this many streams (thread t: stream t mod it)
    static const int n_up_streams = [] { const char *e = getenv("AOS_UP_STREAMS"); return e ? std::max(1, atoi(e)) : kUpThreads; }();
    for (int t = 0; t < nth; ++t)
        if (!up.st[t]) {
            AOS_HIP(hipStreamCreateWithFlags(&up.st[t], hipStreamNonBlocking));
            for (int k = 0; k < kUpSlots; ++k) AOS_HIP(hipEventCreateWithFlags(&up.ev[t][k], hipEventDisableTiming));
            AOS_HIP(hipEventCreateWithFlags(&up.done[t], hipEventDisableTiming));
            for (int k = 0; k < kUpSlots; ++k) up.slot[t][k].ensure(12 * kChunkPts);
        }
    // the handle's stream may still read dst (the previous frame): the copies start after it (a prefetch
    // writes the spare buffer, which no queued work reads)
    if (!prefetch) {
        AOS_HIP(hipEventRecord(ev[15], stream));
        // while the DMAs run (they wait for ev[15] only): the last frame's staged array is read once so that
        // the scatter's partial-line writes hit the Infinity Cache (launch_rt_touch)
        if (staged_touch_mode() == 1 && ror_staged_max > 0)   // (the last frame's records)
            launch_rt_touch(sorted.as<float4>(), std::min(sorted.cap / sizeof(float4), (size_t)ror_staged_max + 1), stream);
    }
    const uint64_t per = (n + nth - 1) / nth;
    const uint8_t *src = static_cast<const uint8_t *>(v.data);
    // split (CloudSplit): points inside the box go to the slot (the device front), the others to the rest
    const bool split = sp.on;
    if (sp.copy_pending) { AOS_HIP(hipEventSynchronize(sp.copied)); sp.copy_pending = false; }   // rest is read
    float *rest = split ? static_cast<float *>(sp.rest.ensure(12 * (size_t)n + kPackSlack * (nth + 1))) : nullptr;
    const float *box = sp.box;
    const PackLayout lay{v.point_step, v.off_x, v.off_y, v.off_z};
    std::atomic<uint64_t> front{0};
    uint64_t rn[kUpThreads] = {};
    std::exception_ptr err[kUpThreads];
    auto work = [&](int t) {
        try {
            AOS_HIP(hipSetDevice(device));
            hipStream_t ust = up.st[t % std::min(nth, n_up_streams)];
            if (!prefetch) AOS_HIP(hipStreamWaitEvent(ust, ev[15], 0));
            const uint64_t p0 = std::min(n, per * t), p1 = std::min(n, per * (t + 1));
            float *rr = split ? rest + 3 * p0 + (kPackSlack / 4) * t : nullptr;   // (kPackSlack between runs)
            uint64_t nr = 0;
            int k = 0;
            for (uint64_t c = p0; c < p1; c += kChunkPts, k = (k + 1) % kUpSlots) {
                const uint64_t m = std::min(kChunkPts, p1 - c);
                if (up.used[t][k]) AOS_HIP(hipEventSynchronize(up.ev[t][k]));   // its last DMA is done
                float *o = static_cast<float *>(up.slot[t][k].p);
                uint64_t f = m;
                if (split) {
                    uint64_t r = 0;
                    f = pack_split(src + c * (uint64_t)v.point_step, m, lay, box, o, rr + 3 * nr, &r);
                    nr += r;
                } else {
                    pack_all(src + c * (uint64_t)v.point_step, m, lay, o);
                }
                if (!f) continue;   // (the slot's last DMA, if any, stays its event)
                const uint64_t at = split ? front.fetch_add(f) : c;
                AOS_HIP(hipMemcpyAsync(static_cast<char *>(dst) + 12 * at, o, 12 * f, hipMemcpyHostToDevice, ust));
                AOS_HIP(hipEventRecord(up.ev[t][k], ust));
                up.used[t][k] = true;
            }
            rn[t] = nr;
            AOS_HIP(hipEventRecord(up.done[t], ust));
        } catch (...) { err[t] = std::current_exception(); }
    };
    HostTrace tr{"upload"};
    up_pool.run(nth, work);   // (parked workers: round 4 spawned nth - 1 threads per upload)
    for (int t = 0; t < nth; ++t)
        if (err[t]) std::rethrow_exception(err[t]);
    sp.nth = nth; sp.n_all = n; sp.n_front = split ? front.load() : n; sp.whole = !split;
    for (int t = 0; t < kUpThreads; ++t) {   // (byte offsets of the threads' rest runs)
        sp.rbeg[t] = t < nth ? 12 * std::min(n, per * t) + kPackSlack * t : 0;
        sp.rn[t] = t < nth ? rn[t] : 0;
    }
    tr.mark("gathered");
    if (tr.on) {   // (AOS_TRACE only: wait for the DMAs to see when the cloud is in HBM)
        for (int t = 0; t < nth; ++t) AOS_HIP(hipEventSynchronize(up.done[t]));
        tr.mark("dma_done");
    }
    if (!prefetch)
        for (int t = 0; t < nth; ++t) AOS_HIP(hipStreamWaitEvent(stream, up.done[t], 0));
}

// aos_cloud_prefetch: the host stages and DMAs the next cloud into cloud_next on a background thread
// (the same four-thread uploader), while this frame's kernels and the GVD jobs run.
void aos_ctx::prefetch_start(const aos_cloud_view &v) {
    prefetch_join();
    const size_t bytes = (size_t)v.n_points * v.point_step;
    if (v.on_device || bytes < (32u << 20)) return;   // nothing to hide
    void *dst = cloud_next.ensure(12 * (size_t)v.n_points);
    split_next.on = split_box(poly, split_next.box);   // (the polygon now; ror_stage checks it still holds)
    pf.view = v;
    pf.src = v.data;
    pf.bytes = bytes;
    pf.err = nullptr;
    pf.active = true;
    pf.th = std::thread([this, dst]() {
        try { upload_pack(dst, pf.view, split_next, true); } catch (...) { pf.err = std::current_exception(); }
    });
}

bool aos_ctx::prefetch_join() {
    if (!pf.active) return false;
    pf.th.join();
    pf.active = false;
    if (pf.err) { std::exception_ptr e = pf.err; pf.err = nullptr; std::rethrow_exception(e); }
    return true;
}

void aos_ctx::release_uploader() {
    up_pool.stop();
    for (int t = 0; t < kUpThreads; ++t) {
        if (up.st[t]) {
            (void)hipStreamSynchronize(up.st[t]);
            for (int k = 0; k < kUpSlots; ++k) (void)hipEventDestroy(up.ev[t][k]);
            (void)hipEventDestroy(up.done[t]);
            (void)hipStreamDestroy(up.st[t]);
            up.st[t] = nullptr;
        }
        for (int k = 0; k < kUpSlots; ++k) { up.slot[t][k].release(); up.used[t][k] = false; }
    }
}

// The cloud state is committed only after the upload succeeded: a failed upload leaves no cloud
// (aos_seedgen_reprocess then fails instead of reading a partly copied buffer).
void aos_ctx::set_cloud(const aos_cloud_view &v) {
    have_cloud = false;
    ms.valid = false;
    const uint8_t *dc;
    if (v.on_device) {
        dc = static_cast<const uint8_t *>(v.data);
    } else {
        size_t bytes = (size_t)v.n_points * v.point_step;
        const void *pf_src = pf.src;
        const size_t pf_bytes = pf.bytes;
        const bool same_view = pf_src == v.data && pf_bytes == bytes;
        bool pf_ok = false;
        try {
            pf_ok = prefetch_join();
        } catch (...) {
            if (same_view) throw;   // the prefetch of this very cloud failed; another view's is dropped
        }
        if (pf_ok && same_view) {
            // the prefetched copy of this very view: it becomes the frame's cloud once its DMAs are done
            std::swap(cloud_copy.p, cloud_next.p);
            std::swap(cloud_copy.cap, cloud_next.cap);
            split_cur.swap_with(split_next);
            for (int t = 0; t < up_threads(); ++t) AOS_HIP(hipStreamWaitEvent(stream, up.done[t], 0));
        } else {
            void *dst = cloud_copy.ensure(std::max<size_t>(12 * (size_t)v.n_points, 16));
            split_cur.on = bytes && split_box(poly, split_cur.box);
            split_cur.whole = true; split_cur.n_all = split_cur.n_front = 0;   // (until the upload succeeds)
            if (bytes) upload_pack(dst, v, split_cur);
        }
        dc = cloud_copy.as<uint8_t>();
    }
    n_points = v.n_points;
    if (v.on_device) { step = v.point_step; ox = v.off_x; oy = v.off_y; oz = v.off_z; }
    else { step = 12; ox = 0; oy = 4; oz = 8; }   // packed by upload_pack
    is_dense = v.is_dense ? 1 : 0;
    d_cloud = dc;
    have_cloud = true;
}

// Streaming ingest: append one scan to the device-resident map (aos_map_append) and make the map
// this frame's cloud. Only the scan crosses PCIe; the map grows by 1.5x when full.
void aos_ctx::map_grow(uint64_t n) {
    if (map_n + n <= map_buf.cap / sizeof(float4)) return;
    const uint64_t want = std::max<uint64_t>(map_n + n, map_n + map_n / 2);
    DevBuf grown;
    void *dst = grown.ensure(sizeof(float4) * std::max<uint64_t>(want, 1));
    if (map_n) AOS_HIP(hipMemcpyAsync(dst, map_buf.p, sizeof(float4) * map_n, hipMemcpyDeviceToDevice, stream));
    AOS_HIP(hipStreamSynchronize(stream));
    std::swap(map_buf.p, grown.p);
    std::swap(map_buf.cap, grown.cap);
}

void aos_ctx::map_append(const aos_cloud_view &v) {
    hipStream_t s = stream;
    const uint64_t n = v.n_points;
    if (map_boxed && map_n) throw std::logic_error("aos_map_append on a tiled streaming map (aos_map_reset first)");
    map_boxed = false;
    map_grow(n);
    const uint8_t *src = static_cast<const uint8_t *>(v.data);
    if (n && !v.on_device) {
        void *st = scan_stage.ensure((size_t)n * v.point_step);
        AOS_HIP(hipMemcpyAsync(st, v.data, (size_t)n * v.point_step, hipMemcpyHostToDevice, s));
        src = static_cast<const uint8_t *>(st);
    }
    launch_pack_xyz(src, n, v.point_step, v.off_x, v.off_y, v.off_z, map_buf.as<float4>() + map_n, s);
    map_scan_begin = map_n;
    map_n += n;
    map_total = map_n;
    map_dense = map_dense && v.is_dense;
    n_points = map_n;
    step = 16; ox = 0; oy = 4; oz = 8;
    is_dense = map_dense;
    d_cloud = map_buf.as<uint8_t>();
    have_cloud = true;
}

// Tiled streaming map (aos_tiled_map_append, BASELINE configs[4] over several GPUs): every rank receives
// the whole scan (each subscriber of /global_map does) and keeps, on its GPU, the points inside its tile's
// points box — all its tile can rasterise or count as ROR neighbours (make_tile_plan) — so the ROR stage
// of the tiled frame sees exactly the points it would see in the whole map. The box is fixed by the
// polygon the map was started with.
void aos_ctx::map_append_box(const aos_cloud_view &v, const float box[4]) {
    hipStream_t s = stream;
    const uint64_t n = v.n_points;
    if (map_n && (!map_boxed || std::memcmp(map_box, box, sizeof(map_box)))) {
        throw std::invalid_argument(map_boxed ? "tiled streaming map: the tile's points box changed (polygon or tiling); "
                                                "aos_map_reset and append the map again"
                                              : "aos_tiled_map_append on a whole streaming map (aos_map_reset first)");
    }
    map_boxed = true;
    std::memcpy(map_box, box, sizeof(map_box));
    map_grow(n);   // (an upper bound: every point of the scan may be in the box)
    const uint8_t *src = static_cast<const uint8_t *>(v.data);
    if (n && !v.on_device) {
        void *st = scan_stage.ensure((size_t)n * v.point_step);
        AOS_HIP(hipMemcpyAsync(st, v.data, (size_t)n * v.point_step, hipMemcpyHostToDevice, s));
        src = static_cast<const uint8_t *>(st);
    }
    unsigned long long *d_cnt = static_cast<unsigned long long *>(map_count.ensure(8));
    unsigned long long *h_cnt = static_cast<unsigned long long *>(h_map_count.ensure(8));
    AOS_HIP(hipMemsetAsync(d_cnt, 0, 8, s));
    launch_pack_xyz_box(src, n, v.point_step, v.off_x, v.off_y, v.off_z, box, map_buf.as<float4>() + map_n, d_cnt, s);
    AOS_HIP(hipMemcpyAsync(h_cnt, d_cnt, 8, hipMemcpyDeviceToHost, s));
    AOS_HIP(hipStreamSynchronize(s));
    map_scan_begin = map_n;
    map_n += *h_cnt;
    map_total += n;
    map_dense = map_dense && v.is_dense;
    n_points = map_n;
    step = 16; ox = 0; oy = 4; oz = 8;
    is_dense = map_dense;
    d_cloud = map_buf.as<uint8_t>();
    have_cloud = true;
}

namespace aos {

// getActiveBounds (seed_gen:874-890) + generateOccupancyGrid geometry (:584-600)
FrameGeom frame_geom(const Poly &poly, const aos_params &P) {
    FrameGeom g{};
    double hminx = poly[0].first, hmaxx = poly[0].first, hminy = poly[0].second, hmaxy = poly[0].second;
    for (const auto &pt : poly) {
        hminx = std::min(hminx, pt.first); hmaxx = std::max(hmaxx, pt.first);
        hminy = std::min(hminy, pt.second); hmaxy = std::max(hmaxy, pt.second);
    }
    const double margin = 2.5;
    g.minx = static_cast<float>(hminx - margin); g.maxx = static_cast<float>(hmaxx + margin);
    g.miny = static_cast<float>(hminy - margin); g.maxy = static_cast<float>(hmaxy + margin);
    g.res = P.grid_resolution;
    float width = std::max(0.0f, g.maxx - g.minx), height = std::max(0.0f, g.maxy - g.miny);
    unsigned int w = static_cast<unsigned int>(std::ceil(width / g.res));
    unsigned int h = static_cast<unsigned int>(std::ceil(height / g.res));
    if (w == 0) w = 1;
    if (h == 0) h = 1;
    g.W = (int)w; g.H = (int)h; g.WW = (g.W + 63) / 64;
    g.origin_x = g.minx; g.origin_y = g.miny;
    g.R = static_cast<int>(P.inflation_radius / P.grid_resolution);  // applyInflation seed_gen:936
    return g;
}

// Half-width of the band around the clip box (or a tile's cells) whose points can be ROR
// neighbours of a candidate: r plus slack for the float box arithmetic.
float ror_margin(const aos_params &P) { return (float)(P.ror_radius * 1.01) + 1e-4f; }

Poly default_polygon() {   // hard-coded default polygon of the reference constructor (seed_gen:196-199)
    return {{-1.972916603088379, 7.9420671463012695}, {-2.0726776123046875, 0.022441387176513672},
            {70.22465515136719, 2.102720260620117}, {69.48777770996094, 9.786612510681152}};
}

// ximgproc thinning loop: T = 1 if the image is empty after iteration 1, else the first iteration
// (k >= 2, 1-based) that deletes nothing; 0 while undecided. flags as written by k_thin_block.
int thin_iterations(const int *flags, int iters_run) {
    if (!flags[0]) return 1;
    for (int k = 1; k < iters_run; ++k)
        if (!flags[1 + k]) return k + 1;
    return 0;
}

}  // namespace aos

// The count pass's column-scan look-back: its err word is the frame's overflow word (d_own[1], read back
// with the frame's stats), bit 4 = a stuck wait (ror_collect throws).
LookBack aos_ctx::ror_lookback(const RorLaunch &L, int G, unsigned long long *d_own) {
    LookBack lb = ror_lb.take(rt_colscan_words(L, G), stream);
    lb.err = reinterpret_cast<int *>(d_own + 1);
    return lb;
}

// a1-a4: ROR restricted to the points that can reach the (own) cells, clip, exclusion discs, raster
// straight into the bit-packed window rbits (o.Hr rows of ceil(o.Wr / 64) words, zeroed here), by the
// tile walk of ror.hip. Records ev[12] / ev[13] / ev[14] / ev[10] / ev[11] around its passes and
// leaves the number of binned points in h_stats[0].
void aos_ctx::ror_stage(const FrameGeom &g, const RorOwn &o, uint64_t *rbits, bool allow_guess) {
    hipStream_t s = stream;
    std::memset(h_stats.ensure(64 + 8 * kRorCounters), 0, 32);   // binned, staged, ror_collect's counters
    RorLaunch L{};
    L.cloud = d_cloud; L.n = n_points; L.step = step; L.ox = ox; L.oy = oy; L.oz = oz; L.is_dense = is_dense;
    L.cminx = g.minx; L.cmaxx = g.maxx; L.cminy = g.miny; L.cmaxy = g.maxy;
    L.cminz = P.clipping_minz; L.cmaxz = P.clipping_maxz;
    const float m = ror_margin(P);
    L.bminx = L.cminx - m; L.bmaxx = L.cmaxx + m; L.bminy = L.cminy - m; L.bmaxy = L.cmaxy + m;
    L.bminz = L.cminz - m; L.bmaxz = L.cmaxz + m;
    if (o.limit_box) {   // a tile: only the neighbourhood of its own cells
        L.bminx = std::max(L.bminx, o.box[0]); L.bminy = std::max(L.bminy, o.box[1]);
        L.bmaxx = std::min(L.bmaxx, o.box[2]); L.bmaxy = std::min(L.bmaxy, o.box[3]);
    }
    if (d_cloud == cloud_copy.as<uint8_t>() && n_points) {   // a host cloud: its split front, or all of it
        const float b[6] = {L.bminx, L.bmaxx, L.bminy, L.bmaxy, L.bminz, L.bmaxz};
        L.n = cloud_for_box(b);
    }
    ror_read = L.n;
    float cs_ = (float)(P.ror_radius * 1.001);
    const double ext = std::max((double)L.bmaxx - L.bminx, (double)L.bmaxy - L.bminy);
    if (ext / cs_ > 8192.0) cs_ = (float)(ext / 8192.0);  // cap the bin grid; coarser bins stay exact
    for (;;) {   // and keep the tiles of 32 x 32 bins within the tile walk's capacity (coarser: still exact)
        L.inv_cs = 1.0f / cs_;
        L.nbx = std::max(1, (int)((L.bmaxx - L.bminx) * L.inv_cs) + 1);
        L.nby = std::max(1, (int)((L.bmaxy - L.bminy) * L.inv_cs) + 1);
        if ((long long)((L.nbx + 31) / 32) * ((L.nby + 31) / 32) <= kRtMaxTiles) break;
        cs_ *= 1.25f;
    }
    L.r2 = P.ror_radius * P.ror_radius;
    L.r2f = (float)(P.ror_radius * P.ror_radius);
    L.r2df = (float)L.r2;
    if ((double)L.r2df > L.r2) L.r2df = std::nextafter(L.r2df, 0.0f);
    L.need = P.ror_min_neighbors + 1;
    L.origin_x = g.origin_x; L.origin_y = g.origin_y; L.res = g.res; L.W = g.W; L.H = g.H;
    L.rx0 = o.rx0; L.ry0 = o.ry0; L.rx1 = o.rx1; L.ry1 = o.ry1; L.wx0 = o.wx0; L.wy0 = o.wy0; L.Wr = o.Wr;
    const int WWr = (o.Wr + 63) / 64;
    // the streaming map keeps a tile store across appends (its tile size stays fixed); a tiled rank's
    // map (limit_box) holds the points of its box only
    const bool map_mode = map_n > 0 && d_cloud == map_buf.as<uint8_t>() && n_points == map_n && map_boxed == o.limit_box;
    // the store becomes valid again only in ror_collect, once this frame's read-back shows no overflow
    // (a frame that fails in between leaves it invalid: the next append reprocesses the whole map)
    const bool store_ok = map_mode && ms.valid;
    ms.valid = false;
    ms.pend.on = false;
    // a streaming store keeps its tile size, but only while the bin grid is the one it was built on
    const bool same_bins = store_ok && ms.L.nbx == L.nbx && ms.L.nby == L.nby && ms.L.inv_cs == L.inv_cs &&
                           ms.L.bminx == L.bminx && ms.L.bminy == L.bminy;
    rt_configure(L, o.Hr, WWr, ror_est_binned > 0 ? ror_est_binned : 0.5 * (double)n_points,
                 same_bins ? ms.L.TB : 0);
    auto geom_of = [](RorLaunch x) {
        x.cloud = nullptr; x.n = 0; x.step = x.ox = x.oy = x.oz = 0; x.staged_cap = 0; x.overflow = nullptr;
        x.big_ok = 0;
        return x;
    };
    // the big-tile kernels run once a frame of this handle has needed them, and on every frame that cannot
    // be redone (a tiled rank, a redo); a frame that finds a big tile without them is redone (ror_collect)
    L.big_ok = ror_big_seen || !allow_guess || o.limit_box;
    if (store_ok && ms.dense == is_dense && ms.n_points == map_scan_begin && n_points >= ms.n_points) {
        const RorLaunch a = geom_of(L), b = ms.L;
        if (!std::memcmp(&a, &b, sizeof(RorLaunch))) {
            ror_read = n_points - ms.n_points;   // (the scan)
            if (n_points > ms.n_points) ror_stage_append(L, rbits);
            else ror_stage_unchanged();
            return;
        }
    }
    const int nt = L.ntiles;
    const int G = rt_part_blocks(L);

    int *d_H = static_cast<int *>(bin_count.ensure(sizeof(int) * rt_h_ints(L, G)));
    int *d_ts = static_cast<int *>(bin_start.ensure(sizeof(int) * (nt + 1)));
    if (map_mode) d_ts = static_cast<int *>(ms.ts[ms.cur].ensure(sizeof(int) * (nt + 1)));
    int *d_kept = map_mode ? static_cast<int *>(ms.kept.ensure(sizeof(int) * nt)) : nullptr;
    DevBuf &stage_buf = map_mode ? ms.st[ms.cur] : sorted;
    unsigned long long *d_cnt = static_cast<unsigned long long *>(counters.ensure(8 * kRorCounters + 24));
    unsigned long long *d_own = d_cnt + kRorCounters;   // [0] binned points, [1] overflow flag, [2] largest tile
    // PCL dense kNN needs k = min_pts + 1 points in the whole cloud (else every point is removed).
    // A tile's shard holds every neighbour of its own candidates, so a shard with fewer points has
    // no keepable candidate either: the local test is exact.
    const bool any = L.n > 0 && !(is_dense && n_points < (uint64_t)L.need);
    // the counters, raster bits and kept counts start at zero: cleared by the count launch (no fills)
    RtClear clr;
    clr.w = rbits; clr.nw = (size_t)o.Hr * WWr;
    clr.c = d_cnt; clr.nc = kRorCounters + 3;
    clr.k = d_kept; clr.nk = d_kept ? nt : 0;
    if (!any) {
        AOS_HIP(hipMemsetAsync(d_cnt, 0, 8 * kRorCounters + 24, s));
        AOS_HIP(hipMemsetAsync(rbits, 0, sizeof(uint64_t) * clr.nw, s));
        if (d_kept) AOS_HIP(hipMemsetAsync(d_kept, 0, sizeof(int) * nt, s));
        return;
    }
    AOS_HIP(hipEventRecord(ev[12], s));
    launch_rt_count(L, d_H, G, d_ts, d_own, ror_lookback(L, G, d_own), s, clr);
    AOS_HIP(hipEventRecord(ev[13], s));
    // The staged array holds own + halo copies. With a capacity from an earlier frame the scatter
    // runs at once and reports an overflow (the frame is then redone with the size it read back,
    // run_seedgen); without one, or when the caller cannot redo (a tiled frame), the size is read
    // back first.
    int *h = static_cast<int *>(h_stats.p);
    const size_t cap_now = stage_buf.cap / sizeof(float4);
    const bool guess = allow_guess && ror_staged_max > 0 && cap_now >= (size_t)(ror_staged_max * 1.1);
    if (!guess) {
        // the staged total and the largest tile (h[3]: rewritten by ror_stats_to_host later)
        peek_to_host(h + 2, {d_ts + nt, reinterpret_cast<const int *>(d_own + 2)}, s);
        AOS_HIP(hipStreamSynchronize(s));
        // the big-tile kernels only for a frame that has a tile beyond the LDS cap (a tiled rank launched all six
        // on every frame: ~27 us per rank, profiles/r06/r06d_tiling.json)
        if (!map_mode && h[3] <= rt_lds_tile_cap()) L.big_ok = 0;
        const size_t need = (size_t)std::max(h[2], 1);
        ror_staged_max = std::max<double>(ror_staged_max, (double)need);
        stage_buf.ensure(sizeof(float4) * (size_t)(need * 1.15 + 1024));
    }
    float4 *d_staged = stage_buf.as<float4>();
    L.staged_cap = (int)std::min<size_t>(stage_buf.cap / sizeof(float4), (size_t)INT_MAX);
    // Records are float4 (x, y, z, w = the class). Round 5 measured and removed two other forms (rorbench, C2 cloud,
    // identical raster hashes): 12-byte records with the class recomputed by the tile pass (scatter 89-90 -> 96-97 us,
    // tile pass 122 -> 126: 12-byte accesses are not 16-byte aligned, profiles/r05k_rorbench.txt), and w carrying the
    // record's local bin in its tile so the tile pass does not recompute it (tile pass unchanged at 113-115 us, scatter
    // +2-4 us: the tile pass is not bound by that arithmetic, profiles/r05n_ror_ab.txt).
    float4 *d_scratch = static_cast<float4 *>(ror_scratch.ensure(sizeof(float4) * (size_t)L.staged_cap));
    L.overflow = reinterpret_cast<int *>(d_own + 1);
    AOS_HIP(hipEventRecord(ev[14], s));
    launch_rt_scatter(L, d_H, d_ts, G, d_staged, s);
    AOS_HIP(hipEventRecord(ev[10], s));
    int *d_big = static_cast<int *>(ror_bigbins.ensure(sizeof(int) * rt_bigbins_ints(L)));
    launch_rt_ror(L, d_ts, d_staged, d_scratch, d_big, rbits, d_cnt, d_kept, nullptr, s);
    AOS_HIP(hipEventRecord(ev[11], s));
    // binned points, staged total, overflow flag: read with the frame's other stats (finish_frame)
    ror_stats_to_host(d_ts + nt, d_own);
    if (map_mode)   // the store will hold the whole map (committed by ror_collect: no overflow)
        ms.pend = MapStore::Pending{true, false, geom_of(L), is_dense, n_points, ms.cur};
}

// Streaming map, one appended scan: the keep decision is monotone in the point set
// (adding points only adds neighbours: PCL's kNN distance can only shrink, a radius count only grow),
// and a candidate's neighbours all sit in its own tile's list. So only the scan is partitioned; each
// tile's list becomes old run + scan run (k_rt_merge); only tiles that received scan points (own or
// halo copies) are recounted, OR-ing into the raster bits the map already has; the kept count is the
// sum of the per-tile counts. Equal to reprocessing the whole map (tests/test_gpu_stream.py).
void aos_ctx::ror_stage_append(RorLaunch L, uint64_t *rbits) {
    hipStream_t s = stream;
    const int nt = L.ntiles;
    const uint64_t scan_n = n_points - ms.n_points;
    RorLaunch Ls = L;   // the scan's float4 records in the map buffer
    Ls.cloud = map_buf.as<uint8_t>() + sizeof(float4) * ms.n_points;
    Ls.n = scan_n; Ls.step = 16; Ls.ox = 0; Ls.oy = 4; Ls.oz = 8;
    const int G = rt_part_blocks(Ls);
    int *d_H = static_cast<int *>(ms.scan_H.ensure(sizeof(int) * rt_h_ints(Ls, G)));
    int *d_sts = static_cast<int *>(ms.scan_ts.ensure(sizeof(int) * (nt + 1)));
    unsigned long long *d_cnt = static_cast<unsigned long long *>(counters.ensure(8 * kRorCounters + 24));
    unsigned long long *d_own = d_cnt + kRorCounters;
    // a point lands in at most 4 tiles: the scan's staging and the merged store cannot overflow
    const size_t scan_cap = 4 * (size_t)scan_n + 1024;
    float4 *d_scan = static_cast<float4 *>(ms.scan_st.ensure(sizeof(float4) * scan_cap));
    const int nxt = ms.cur ^ 1;
    const size_t cap = ms.n_staged + scan_cap;
    if (cap > (size_t)INT_MAX) throw std::runtime_error("streaming map: ROR store exceeds 2^31 points");
    float4 *d_new = static_cast<float4 *>(ms.st[nxt].ensure(sizeof(float4) * cap));
    int *d_nts = static_cast<int *>(ms.ts[nxt].ensure(sizeof(int) * (nt + 1)));
    float4 *d_scratch = static_cast<float4 *>(ror_scratch.ensure(sizeof(float4) * cap));
    Ls.staged_cap = (int)scan_cap;
    Ls.overflow = reinterpret_cast<int *>(d_own + 1);
    AOS_HIP(hipEventRecord(ev[12], s));
    RtClear clr;
    clr.c = d_cnt; clr.nc = kRorCounters + 3;
    launch_rt_count(Ls, d_H, G, d_sts, d_own, ror_lookback(Ls, G, d_own), s, clr);
    AOS_HIP(hipEventRecord(ev[13], s));
    AOS_HIP(hipEventRecord(ev[14], s));
    launch_rt_scatter(Ls, d_H, d_sts, G, d_scan, s);
    AOS_HIP(hipEventRecord(ev[10], s));
    launch_rt_merge(ms.st[ms.cur].as<float4>(), ms.ts[ms.cur].as<int>(), d_scan, d_sts, d_new, d_nts, nt, (int)cap,
                    Ls.overflow, s);
    L.staged_cap = (int)cap;
    L.overflow = Ls.overflow;
    int *d_big = static_cast<int *>(ror_bigbins.ensure(sizeof(int) * rt_bigbins_ints(L)));
    launch_rt_ror(L, d_nts, d_new, d_scratch, d_big, rbits, d_cnt, ms.kept.as<int>(), d_sts, s);
    launch_rt_sum_kept(ms.kept.as<int>(), nt, d_cnt, s);
    AOS_HIP(hipEventRecord(ev[11], s));
    ror_stats_to_host(d_nts + nt, d_own);
    // committed by ror_collect (the old store ms.st[ms.cur] stays intact until then)
    ms.pend = MapStore::Pending{true, true, ms.L, ms.dense, n_points, nxt};
}

// A streaming map's frame with no new points in the map (a tiled rank whose box the scan missed: ADVICE
// r03): the kept set, the raster bits (ORed into across appends) and the kept count (counters) are the last
// frame's, so the stage is skipped; the store is recommitted as it is.
void aos_ctx::ror_stage_unchanged() {
    for (int e : {12, 13, 14, 10, 11}) AOS_HIP(hipEventRecord(ev[e], stream));
    int *h = static_cast<int *>(h_stats.p);
    h[2] = (int)ms.n_staged;   // (binned 0 new points and no overflow: zeroed by ror_stage)
    ms.pend = MapStore::Pending{true, true, ms.L, ms.dense, n_points, ms.cur};
    ++ror_skipped;
}

// The stage's staged total (h[2]) and binned count + overflow bits (h + 4: two u64) into the pinned stats, read
// after the frame's sync (ror_collect): one kernel store instead of two copy-engine read-backs
void aos_ctx::ror_stats_to_host(const int *d_staged_total, const unsigned long long *d_own) {
    int *h = static_cast<int *>(h_stats.p);
    const int *o = reinterpret_cast<const int *>(d_own);
    peek_to_host(h + 2, {d_staged_total, d_staged_total, o, o + 1, o + 2, o + 3}, stream);
}

// After the frame's sync: binned count, staged size, and whether the scatter overflowed its guess. A stuck
// look-back (bit 4) throws unless throw_stuck is false (a tiled rank: its bits go to every rank first, so
// all ranks fail the frame together instead of one leaving the others in a collective: ADVICE r04).
bool aos_ctx::ror_collect(bool throw_stuck) {
    int *h = static_cast<int *>(h_stats.p);
    const unsigned long long *u = reinterpret_cast<const unsigned long long *>(h + 4);
    double binned = (double)u[0];
    if (ms.pend.on && ms.pend.incremental) binned += ms.n_binned;   // the scan's binned points on top of the map's
    h[0] = (int)binned;
    ror_est_binned = binned;
    ror_staged_max = std::max<double>(ror_staged_max, (double)h[2]);
    if (u[1] & 4) {
        ms.pend.on = false;
        if (throw_stuck) throw std::runtime_error("ROR column scan: a look-back wait exceeded its cap (kSpinCap)");
        return true;
    }
    if (u[1] & 2) ror_big_seen = true;
    if (ms.pend.on && u[1] == 0) {   // commit the streaming map's tile store
        ms.valid = true;
        ms.L = ms.pend.L;
        ms.dense = ms.pend.dense;
        ms.n_points = ms.pend.n_points;
        ms.cur = ms.pend.cur;
        ms.n_binned = binned;
        ms.n_staged = (size_t)h[2];
    }
    ms.pend.on = false;
    return u[1] != 0;
}

// First thinning batch of a whole-map frame: flags reset, opening, after_open (the inflated grid's read-back),
// batch_n temporal-block launches
// (launch_next issues them and keeps the caller's launch state). With AOS_THIN_GRAPH != 0 the batch is a
// hipGraph (BASELINE configs[4]: hipGraph-captured thinning; aos_params.thin_graph), one per batch size,
// batch_n rounded up to a
// power of two. A graph bakes every argument in by value, so it is keyed on every pointer and size its
// nodes hold (the input, opening and ping-pong bit grids, the flags, the tile-activity rows, the host
// flags buffer when it copies them, and W, H, WW, R, the launch count, the flags length) and re-captured
// when any of them changes; the per-launch act_prev / act_next alternation is a function of the launch
// index from 0, the same on every replay. Graph shapes (AOS_THIN_GRAPH, for the diagnosis of round 2's
// failure, tools/thin_graph_probe.py): 1 (default) the thinning launches only, the opening (which clears the flags)
// launched just before the graph and the flags read back outside it; 2 round 1's shape: memset node + kernels + D2H copy node; 3 memset node +
// kernels; 4 clearing kernel + kernels + D2H copy node. Returns true when the graph copied the flags
// of the batch to h_flags itself.
bool aos_ctx::thin_first_batch(const FrameGeom &g, const uint64_t *d_ibits, uint64_t *d_open, uint64_t *const bufs[2],
                               int *d_flags, int *h_flags, int *d_act, int nflags, int &batch_n, int cap_launches,
                               const std::function<void(int)> &launch_next, const std::function<void()> &after_open) {
    hipStream_t s = stream;
    const int K = kThinItersPerLaunch;
    if (thin_graph_shape < 0) {
        const char *e = getenv("AOS_THIN_GRAPH");   // (diagnosis: overrides aos_params.thin_graph)
        thin_graph_shape = e ? std::max(0, std::min(4, atoi(e))) : (P.thin_graph ? 1 : 0);
        thin_graph_check = getenv("AOS_THIN_GRAPH_CHECK") != nullptr;
    }
    const int shape = thin_graph_shape;
    last_thin_graph = 0;
    // The opening runs outside the graph (shapes 0 and 1) so that after_open (the inflated grid's read-back) can
    // be queued behind it: the read-back's blit kernel beside k_open took it from ~40 to 110 us at C3 (round-5
    // trace); beside thinning the copy meets long, LDS-bound launches instead.
    if (shape <= 1) {
        launch_open(d_ibits, d_open, g, s, d_flags, nflags);   // (clears the flags)
        after_open();
    }
    if (shape == 0) {
        launch_next(batch_n);
        return false;
    }
    int bn = 2;
    while (bn < batch_n) bn *= 2;
    batch_n = std::min(bn, cap_launches);
    const bool memset_node = shape == 2 || shape == 3, copy_node = shape == 2 || shape == 4;
    const std::array<const void *, 8> ptrs{d_ibits, d_open, bufs[0], bufs[1], d_flags, d_act,
                                           copy_node ? h_flags : nullptr, nullptr};
    const std::array<int, 8> dims{g.W, g.H, g.WW, g.R, batch_n, nflags, shape, thin_tiles(g)};
    ThinGraph *tg = nullptr;
    for (auto &t : thin_graphs)
        if (t.dims[4] == batch_n) tg = &t;
    if (tg && tg->exec && (tg->ptrs != ptrs || tg->dims != dims)) {
        AOS_HIP(hipGraphExecDestroy(tg->exec));
        tg->exec = nullptr;
    }
    if (!tg) {
        thin_graphs.emplace_back();
        tg = &thin_graphs.back();
    }
    if (!tg->exec) {
        hipGraph_t graph = nullptr;
        AOS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        try {
            if (memset_node) {
                AOS_HIP(hipMemsetAsync(d_flags, 0, sizeof(int) * nflags, s));
                launch_open(d_ibits, d_open, g, s);
            } else if (shape == 4) {
                launch_zero_ints(d_flags, nflags, s);
                launch_open(d_ibits, d_open, g, s);
            }   // (shape 1: the opening, which clears the flags, ran before the graph)
            launch_next(batch_n);
            if (copy_node)
                AOS_HIP(hipMemcpyAsync(h_flags, d_flags, sizeof(int) * (1 + batch_n * K), hipMemcpyDeviceToHost, s));
        } catch (...) {
            (void)hipStreamEndCapture(s, &graph);
            if (graph) (void)hipGraphDestroy(graph);
            throw;
        }
        AOS_HIP(hipStreamEndCapture(s, &graph));
        const hipError_t e = hipGraphInstantiate(&tg->exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (e != hipSuccess) tg->exec = nullptr;
        AOS_HIP(e);
        tg->ptrs = ptrs;
        tg->dims = dims;
        last_thin_graph = 2;
    } else {
        last_thin_graph = 1;
    }
    if (shape > 1) after_open();   // (diagnostic shapes: the opening is inside the graph)
    AOS_HIP(hipGraphLaunch(tg->exec, s));
    return copy_node;
}

void aos_ctx::thin_graphs_release() {
    for (auto &t : thin_graphs)
        if (t.exec) (void)hipGraphExecDestroy(t.exec);
    thin_graphs.clear();
}

// AOS_THIN_GRAPH_CHECK: after the flags read-back, compare the host copy with a fresh synchronous read of
// the device flags (after a device-wide sync) and check that no flag word holds anything but 0 / 1 and
// that the words past the iterations run are still 0. Reports to stderr; diagnosis only.
void aos_ctx::thin_check_flags(const int *d_flags, const int *h_flags, int n_read, int nflags) {
    AOS_HIP(hipDeviceSynchronize());
    std::vector<int> dv(nflags);
    AOS_HIP(hipMemcpy(dv.data(), d_flags, sizeof(int) * nflags, hipMemcpyDeviceToHost));
    int host_diff = 0, not01 = 0, tail = 0, first = -1;
    char vals[160] = "";
    for (int i = 0, nv = 0; i < nflags; ++i) {
        if (i < n_read && dv[i] != h_flags[i]) { ++host_diff; if (first < 0) first = i; }
        if (dv[i] != 0 && dv[i] != 1) {
            ++not01;
            if (nv < 6) { const size_t l = strlen(vals); snprintf(vals + l, sizeof(vals) - l, " [%d]=0x%08x", i, (unsigned)dv[i]); ++nv; }
        }
        if (i >= n_read && dv[i] != 0) ++tail;
    }
    ++thin_checks;
    if (host_diff || not01 || tail) {
        ++thin_check_failures;
        fprintf(stderr, "[aos thin check] graph %d shape %d: %d of %d read words differ host vs device (first %d: host %d "
                        "device %d), %d words not 0/1 (%s), %d nonzero words past the read range\n", last_thin_graph,
                thin_graph_shape, host_diff, n_read, first, first >= 0 ? h_flags[first] : 0, first >= 0 ? dv[first] : 0,
                not01, vals, tail);
    }
}

static int grid_readback_bits();

void aos_ctx::run_seedgen(bool want_host, aos_seedgen_out &out) {
    // A frame is served (have_frame) only once every check passed: finish_frame sets it before the ROR
    // overflow and thinning-convergence checks of the deferred path, so every way out of here that is not
    // a good frame (a redo, a throw, a HIP error in between) clears it again.
    try {
        // a frame whose ROR scatter outgrew its size guess is redone once with the size it read back
        for (int attempt = 0; attempt < 2; ++attempt) {
            if (!run_seedgen_once(want_host, out, attempt == 0)) return;
            have_frame = false;
        }
        throw std::runtime_error("ROR staging overflowed twice");
    } catch (...) {
        have_frame = false;
        throw;
    }
}

bool aos_ctx::run_seedgen_once(bool want_host, aos_seedgen_out &out, bool allow_guess) {
    const bool trace = getenv("AOS_TRACE") != nullptr;
    const auto t_in = std::chrono::steady_clock::now();
    auto since = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_in).count(); };
    std::memset(&out, 0, sizeof(out));
    tiled_frame = false;
    have_frame = false;
    const FrameGeom g = frame_geom(poly, P);
    geom = g;
    if (g.R > 63) throw std::runtime_error("inflation radius > 63 cells is not supported by the bit-packed kernel");
    if ((size_t)g.W * g.H > (size_t)1 << 31) throw std::runtime_error("grid larger than 2^31 cells");
    hipStream_t s = stream;
    const size_t Cw = (size_t)g.WW * g.H;
    AOS_HIP(hipEventRecord(ev[0], s));

    // ---------------- a1-a4: ROR restricted to the clip box, clip, exclusion discs, raster
    RorOwn own{0, 0, g.W, g.H, 0, 0, g.W, g.H, false, {0, 0, 0, 0}};
    uint64_t *d_rbits = static_cast<uint64_t *>(raster_bits.ensure(Cw * 8));
    ror_stage(g, own, d_rbits, allow_guess);
    AOS_HIP(hipEventRecord(ev[1], s));

    // ---------------- a5 inflation, a6 frame -> /occupancy_grid
    uint64_t *d_ibits = static_cast<uint64_t *>(infl_bits.ensure(Cw * 8));
    int8_t *d_occ = static_cast<int8_t *>(occ_bytes.ensure((size_t)g.W * g.H));
    launch_inflate(d_rbits, d_ibits, g, s, d_occ, 5);   // (the bytes with the 5-cell frame in the same launch)
    AOS_HIP(hipEventRecord(ev[2], s));
    // /occupancy_grid's bits cross PCIe beside thinning (after the opening: thin_first_batch), instead of beside
    // the cluster stage's read-backs (finish_frame sends the skeleton's)
    infl_bits_sent = false;
    auto send_infl_bits = [&]() {
        if (!want_host || !grid_readback_bits()) return;
        expander.drain();   // (a failed frame's expansion may still read the buffer)
        const size_t nb = 8 * Cw;
        grid_d2h(h_occ_bits.ensure(std::max<size_t>(nb, 8)), d_ibits, nb);
        infl_bits_sent = true;
    };

    // ---------------- a7 opening + Zhang-Suen (temporal blocks of kThinItersPerLaunch iterations)
    uint64_t *d_open = static_cast<uint64_t *>(open_bits.ensure(Cw * 8));
    uint64_t *bufs[2] = {static_cast<uint64_t *>(thin_a.ensure(Cw * 8)), static_cast<uint64_t *>(thin_b.ensure(Cw * 8))};
    const int K = kThinItersPerLaunch;
    const int max_iters = std::max(g.W, g.H) + 4;   // Zhang-Suen removes >= 1 cell per changing iteration
    const int nflags = 2 + max_iters + K;
    int *d_flags = static_cast<int *>(flags.ensure(sizeof(int) * nflags));
    int *h_flags = static_cast<int *>(h_small.ensure(sizeof(int) * nflags));
    const int ntt = thin_tiles(g);
    int *d_act = static_cast<int *>(thin_act.ensure(sizeof(int) * 2 * (size_t)ntt));
    // Launches past convergence return at once (k_thin_block reads the previous iteration's flag on the
    // device), so the first batch is sized from the last frame's T (at least 2 launches) and later
    // batches double: a frame pays one host round trip in the common case, a few when T jumps.
    int cap_launches = std::max(3, max_iters / K);
    if (const char *e = getenv("AOS_DEBUG_THIN_CAP")) cap_launches = std::max(1, atoi(e));   // (tests: force non-convergence)
    int launched = 0;
    const uint64_t *src = d_open;
    ThinOwn whole{0, g.H, 0, g.WW, 1};
    auto launch_next = [&](int count) {
        for (int j = 0; j < count && launched < cap_launches; ++j) {
            uint64_t *dst = bufs[launched & 1];
            // tile activity of the previous launch (none for the first: every tile runs)
            whole.act_prev = launched ? d_act + (size_t)((launched - 1) & 1) * ntt : nullptr;
            whole.act_next = d_act + (size_t)(launched & 1) * ntt;
            launch_thin_block(src, dst, g, launched * K, d_flags, whole, s);
            src = dst;
            ++launched;
        }
    };
    int batch_n = std::min(cap_launches, std::max(2, (thin_iters_prev + 2 + K - 1) / K));
    const bool flags_in_graph = thin_first_batch(g, d_ibits, d_open, bufs, d_flags, h_flags, d_act, nflags, batch_n,
                                                 cap_launches, launch_next, send_infl_bits);
    launched = batch_n;
    src = bufs[(batch_n - 1) & 1];
    const uint64_t *final_buf = d_open;
    int T = 0;
    // No host round trip after the first batch (verdict r02 weak item 9): a device kernel copies the converged
    // launch's buffer (read from the device flags) into thin_out, the flags come back with the frame's later
    // read-backs, and the post-thinning stages run at once. After the frame the host checks convergence (and
    // the ROR overflow); a frame whose T outgrew the first batch runs more launches below and the
    // post-thinning stages again. AOS_THIN_DEFER=0: wait for the flags here (round 2's order).
    static const bool defer = [] { const char *e = getenv("AOS_THIN_DEFER"); return !e || atoi(e) != 0; }();
    bool ror_done = false;
    int round0 = 0;
    if (defer && !flags_in_graph) {
        uint64_t *d_out = static_cast<uint64_t *>(thin_out.ensure(Cw * 8));
        launch_thin_pick(d_flags, launched, bufs[0], bufs[1], d_out, Cw, s, h_flags, 1 + launched * K);
        AOS_HIP(hipEventRecord(ev[3], s));
        skel_bits = d_out;
        const double t_thin = since();
        finish_frame(g, want_host, nullptr, out);   // (ends with a stream synchronisation: h_flags is on the host)
        if (thin_graph_check) thin_check_flags(d_flags, h_flags, 1 + launched * K, nflags);
        if (ror_collect()) return true;
        ror_done = true;
        // (finish_frame read the binned count before ror_collect set it: the fields that depend on it again)
        auto ms_ev = [&](int a, int b) { float t = 0; (void)hipEventElapsedTime(&t, ev[a], ev[b]); return t; };
        out.n_binned = static_cast<const int *>(h_stats.p)[0];
        out.ms_ror_count = out.n_binned ? ms_ev(10, 11) : 0.0f;
        out.ms_ror_bin = out.n_binned ? ms_ev(12, 13) : 0.0f;
        out.ms_ror_scatter = out.n_binned ? ms_ev(14, 10) : 0.0f;
        T = thin_iterations(h_flags, launched * K);
        if (T) {
            last_thin_launches = launched;
            thin_iters = thin_iters_prev = T;
            out.thin_iters = T;
            out.thin_launches = launched;
            if (trace)
                fprintf(stderr, "[aos trace seedgen] at %.2f: thin (deferred) %.2f finish %.2f (T %d, launches %d, graph %d)\n",
                        trace_ms() - since(), t_thin, since(), T, launched, last_thin_graph);
            return false;
        }
        if (launched >= cap_launches) throw std::runtime_error("thinning did not converge");
        round0 = 1;   // T outgrew the first batch: more launches, then the post-thinning stages again
    }
    for (int round = round0;; ++round) {
        if (round > 0) launch_next(batch_n << round);
        if (round > 0 || !flags_in_graph)
            AOS_HIP(hipMemcpyAsync(h_flags, d_flags, sizeof(int) * (1 + launched * K), hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        if (thin_graph_check) thin_check_flags(d_flags, h_flags, 1 + launched * K, nflags);
        T = thin_iterations(h_flags, launched * K);
        if (T) {
            // the last launch that ran: launch j runs iff j == 0 or iteration j*K-1 deleted something
            int last = 0;
            for (int j = 1; j < launched; ++j)
                if (h_flags[1 + j * K - 1]) last = j; else break;
            final_buf = bufs[last & 1];
            break;
        }
        if (launched >= cap_launches) throw std::runtime_error("thinning did not converge");
    }
    last_thin_launches = launched;
    thin_iters = T;
    thin_iters_prev = T;
    skel_bits = final_buf;
    AOS_HIP(hipEventRecord(ev[3], s));
    const double t_thin = since();
    if (!ror_done && ror_collect()) return true;   // (the thinning read-back above synchronised the stream)
    finish_frame(g, want_host, nullptr, out);
    if (trace)
        fprintf(stderr, "[aos trace seedgen] at %.2f: thin-sync %.2f finish %.2f (T %d, launches %d, graph %d)\n",
                trace_ms() - since(), t_thin, since(), T, launched, last_thin_graph);
    return false;
}

// The published grids' D2H. Default (AOS_GRID_READBACK=1, round 5): the two bit-packed grids (the inflated
// grid and the frameless skeleton, W*H/8 bytes each) cross PCIe and host threads expand them to the {0, 100}
// bytes with the frame / rectangle while the cluster stage runs (grid_host.cpp). Round 4's traces showed the
// byte grids' D2H as runtime blit kernels (__amd_rocclr_copyBuffer, 0.65 ms per C2 frame, 2.6 ms at C3) that
// stretched the cluster stage's kernels beside them (k_fg 18 -> 280 us): the bits are 8x fewer bytes through
// them. AOS_GRID_READBACK=0: the byte grids by hipMemcpyAsync (round 4), or AOS_GRID_COPY_KERNEL=1 by a kernel of
// grid_copy_blocks() workgroups.
static int grid_readback_bits() {
    static const int v = [] { const char *e = getenv("AOS_GRID_READBACK"); return e ? atoi(e) : 1; }();
    return v;
}
static int grid_expand_threads() {   // AOS_GRID_EXPAND_THREADS (default 8)
    static const int v = [] { const char *e = getenv("AOS_GRID_EXPAND_THREADS"); return e ? std::max(1, atoi(e)) : 8; }();
    return v;
}
// The grids' D2H runs as the runtime's blit kernels (under the HIP runtime torch loads). Beside the cluster stage
// they held the CUs its kernels needed: k_fg took 45 us instead of 18.6 beside the 2 MB bits copy at C2, 159
// instead of 24 beside the 8 MB at C3 (round-5 traces, tools/kt_overlap.py). AOS_COPY_CUS = k > 0 creates the copy
// stream with a CU mask (hipExtStreamCreateWithCUMask) of k CUs spread over the id range, so its blit waves stay
// there. Measured and not adopted (profiles/r05g_copy_cus_ab.txt): with 16 CUs seed-gen took 1.47-1.49 ms per C2
// frame instead of 1.24-1.27 (thinning and k_fg slower beside the masked copy). Default 0: no mask; the copies are
// placed where they meet the fewest kernels instead (the inflated grid beside thinning, the skeleton after k_fg).
static void create_copy_stream(hipStream_t *st) {
    static const int want = [] { const char *e = getenv("AOS_COPY_CUS"); return e ? std::max(0, atoi(e)) : 0; }();
    int dev = 0, ncu = 0;
    AOS_HIP(hipGetDevice(&dev));
    AOS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (want <= 0 || want >= ncu) {
        AOS_HIP(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
        return;
    }
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    for (int k = 0; k < want; ++k) {
        const int cu = (int)((long long)k * ncu / want);
        mask[cu >> 5] |= 1u << (cu & 31);
    }
    AOS_HIP(hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data()));
}
void aos_ctx::grid_d2h(void *h, const void *d, size_t bytes) {
    grid_copy_wait();
    AOS_HIP(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, copy_stream));
}
// the copy stream (created on first use) waits for the work queued on the handle's stream so far
void aos_ctx::grid_copy_wait() {
    if (!copy_stream) {
        create_copy_stream(&copy_stream);
        AOS_HIP(hipEventCreateWithFlags(&copy_ready, hipEventDisableTiming));
        AOS_HIP(hipEventCreateWithFlags(&copy_done, hipEventDisableTiming));
    }
    AOS_HIP(hipEventRecord(copy_ready, stream));
    AOS_HIP(hipStreamWaitEvent(copy_stream, copy_ready, 0));
}
static int grid_copy_blocks() {   // AOS_GRID_COPY_BLOCKS (default 64)
    static const int b = [] { const char *e = getenv("AOS_GRID_COPY_BLOCKS"); return e ? std::max(1, atoi(e)) : 64; }();
    return b;
}
static bool grid_copy_kernel() {
    static const bool on = [] { const char *e = getenv("AOS_GRID_COPY_KERNEL"); return e && atoi(e) != 0; }();
    return on;
}

// a16 + a8-a15 on the whole map from skel_bits / occ_bytes, then the frame outputs. clipped_total:
// the kept-candidate count when it was reduced over tiles (else read from this handle's counters).
void aos_ctx::finish_frame(const FrameGeom &g, bool want_host, const uint64_t *clipped_total, aos_seedgen_out &out,
                           const PreClusters *pre) {
    hipStream_t s = stream;
    ++frame_gen;   // skel_bytes is rewritten below
    const size_t C = (size_t)g.W * g.H;
    int8_t *d_occ = occ_bytes.as<int8_t>();

    // ---------------- a16 /skeletonized_occupancy_grid = skeleton + polygon bbox rectangle
    int8_t *d_skel = static_cast<int8_t *>(skel_bytes.ensure(C));
    int rect[4] = {0, 0, 0, 0};   // markPolygonBoundaryAsOccupied's rectangle: gx0, gy0, gx1, gy1
    {
        double hminx = poly[0].first, hmaxx = poly[0].first, hminy = poly[0].second, hmaxy = poly[0].second;
        for (const auto &pt : poly) {
            hminx = std::min(hminx, pt.first); hmaxx = std::max(hmaxx, pt.first);
            hminy = std::min(hminy, pt.second); hmaxy = std::max(hmaxy, pt.second);
        }
        const double margin = 2.5;
        auto w2g = [&](float wx, float wy, int &gx, int &gy) {  // worldToGrid seed_gen:760-769
            float rel_x = (wx - g.origin_x) / g.res;
            float rel_y = (wy - g.origin_y) / g.res;
            gx = static_cast<int>(std::floor(rel_x)); gy = static_cast<int>(std::floor(rel_y));
            gx = gx < 0 ? 0 : (gx >= g.W ? g.W - 1 : gx);
            gy = gy < 0 ? 0 : (gy >= g.H ? g.H - 1 : gy);
        };
        w2g(static_cast<float>(hminx - margin), static_cast<float>(hminy - margin), rect[0], rect[1]);
        w2g(static_cast<float>(hmaxx + margin), static_cast<float>(hmaxy + margin), rect[2], rect[3]);
    }
    // the two published grids go to host memory on the copy stream while the cluster / seed stage runs
    // (AOS_GRID_COPY=1: after it instead; the copy's blit kernels share the CUs with the stage's kernels)
    static const int grid_copy_mode = [] { const char *e = getenv("AOS_GRID_COPY"); return e ? atoi(e) : 0; }();
    const bool as_bits = grid_readback_bits() != 0;
    auto issue_grid_copy = [&]() {
        // (a failed frame's expansion may still write h_occ / h_skel and read the bit buffers: drained before
        // any of them can be reallocated; ADVICE r05. A no-op when the inflated bits' send drained it.)
        expander.drain();
        h_occ.ensure(std::max<size_t>(C, 1)); h_skel.ensure(std::max<size_t>(C, 1));
        if (as_bits) {
            const size_t nb = 8 * (size_t)g.WW * g.H;
            uint64_t *hob = static_cast<uint64_t *>(h_occ_bits.ensure(std::max<size_t>(nb, 8)));
            uint64_t *hsb = static_cast<uint64_t *>(h_skel_bits.ensure(std::max<size_t>(nb, 8)));
            if (!infl_bits_sent)   // (a tiled frame: the gathered inflated grid)
                grid_d2h(hob, tiled_frame ? full_infl.as<uint64_t>() : infl_bits.as<uint64_t>(), nb);
            grid_d2h(hsb, skel_bits, nb);
            AOS_HIP(hipEventRecord(copy_done, copy_stream));
            GridExpander::Job j{};
            const int dev = device;
            hipEvent_t e = copy_done;
            j.wait = [dev, e] {
                AOS_HIP(hipSetDevice(dev));
                AOS_HIP(hipEventSynchronize(e));
            };
            j.occ_bits = hob; j.skel_bits = hsb;
            j.occ = h_occ.as<int8_t>(); j.skel = h_skel.as<int8_t>();
            j.W = g.W; j.H = g.H; j.WW = g.WW; j.frame = 5;
            j.rect[0] = rect[0]; j.rect[1] = rect[1]; j.rect[2] = rect[2]; j.rect[3] = rect[3];
            j.threads = grid_expand_threads();
            expander.start(j);
        } else if (grid_copy_kernel()) {   // (a kernel launch never holds the host; see copy_kernel_bulk)
            grid_copy_wait();
            copy_kernel_bulk(h_occ.p, d_occ, C, grid_copy_blocks(), copy_stream);
            copy_kernel_bulk(h_skel.p, d_skel, C, grid_copy_blocks(), copy_stream);
        } else {
            grid_d2h(h_occ.p, d_occ, C);
            grid_d2h(h_skel.p, d_skel, C);
        }
    };
    HostTrace tr{"finish"};
    launch_bits_to_bytes(skel_bits, d_skel, g, 0, s, rect);   // (a16: the rectangle drawn in the same launch)
    // the bits go once the cluster stage has queued k_fg and its count read-back (SeedStageIn::after_fg; round 5
    // traces: beside k_fg the copy's blit kernel took k_fg from 19 to 49 us, and the read-back waited behind it on
    // PCIe); the byte copies of the other modes right away
    bool copy_issued = false;
    auto copy_now = [&]() {
        if (copy_issued) return;
        copy_issued = true;
        issue_grid_copy();
    };
    if (want_host && grid_copy_mode == 0 && !as_bits) copy_now();
    tr.mark("copy_issued");

    // ---------------- a8-a15 clusters, tree rows, seeds
    SeedStageIn sin{skel_bits, &geom, &poly, P.cluster_min_length, pre};
    if (want_host && grid_copy_mode == 0 && as_bits) {
        sin.after_fg = copy_now;
        // the replays walk the skeleton's bits once their read-back (queued by after_fg) is done
        static const bool replay_bits = [] { const char *e = getenv("AOS_REPLAY_BITS"); return !e || atoi(e) != 0; }();
        if (replay_bits)
            sin.host_skel_bits = [&]() -> const uint64_t * {
                if (!copy_issued) return nullptr;
                AOS_HIP(hipEventSynchronize(copy_done));
                return static_cast<const uint64_t *>(h_skel_bits.p);
            };
    }
    SeedStageOut so;
    run_cluster_seed_stage(cs, sin, so, s, ev[4], trace_on() ? &ev[16] : nullptr);
    AOS_HIP(hipEventRecord(ev[5], s));
    if (want_host && (grid_copy_mode == 1 || as_bits)) copy_now();   // (a stage that did not call after_fg)

    unsigned long long *h_cnt = static_cast<unsigned long long *>(h_stats.ensure(64 + 8 * kRorCounters)) + 8;
    if (!clipped_total) AOS_HIP(hipMemcpyAsync(h_cnt, counters.p, 8 * kRorCounters, hipMemcpyDeviceToHost, s));
    tr.mark("stage_done");
    AOS_HIP(hipStreamSynchronize(s));
    tr.mark("stream_synced");
    if (want_host) {
        if (as_bits) expander.join();   // (rethrows a failed wait)
        else AOS_HIP(hipStreamSynchronize(copy_stream));
    }
    tr.mark("copies_synced");
    if (clipped_total) {
        n_clipped = *clipped_total;
    } else {
        n_clipped = 0;
        for (int i = 0; i < kRorCounters; ++i) n_clipped += h_cnt[i];
    }
    have_frame = true;

    h_row_center = std::move(so.row_center); h_row_start = std::move(so.row_start);
    h_row_end = std::move(so.row_end); h_row_length = std::move(so.row_length);
    n_virtual = so.n_virtual; n_ray = so.n_ray; n_endpoint = so.n_endpoint;
    if (so.n_voronoi) h_voronoi.assign(so.h_voronoi, so.h_voronoi + 2 * (size_t)so.n_voronoi);
    else h_voronoi.clear();
    h_rows_info = std::move(so.rows_info);
    h_cluster_info = std::move(so.cluster_info);
    n_clusters_all = so.n_clusters_all;
    n_bfs_replayed = so.n_bfs;

    out.info = aos_grid_info{g.origin_x, g.origin_y, g.res, (uint32_t)g.W, (uint32_t)g.H};
    out.thin_iters = thin_iters;
    out.n_input = (d_cloud == map_buf.as<uint8_t>() && n_points == map_n) ? map_total : n_points;
    out.n_clipped = n_clipped;
    out.n_ror_kept = 0;  // not materialised (ROR is evaluated only where it can reach the grid)
    out.occupancy = want_host ? h_occ.as<int8_t>() : nullptr;
    out.skeleton = want_host ? h_skel.as<int8_t>() : nullptr;
    out.d_occupancy = d_occ;
    out.d_skeleton = d_skel;
    out.n_clusters_all = n_clusters_all;
    out.n_bfs_replayed = n_bfs_replayed;
    out.n_rows = (int)h_row_length.size();
    out.row_center = h_row_center.data(); out.row_start = h_row_start.data();
    out.row_end = h_row_end.data(); out.row_length = h_row_length.data();
    out.n_virtual = n_virtual; out.n_ray = n_ray; out.n_endpoint = n_endpoint;
    out.n_voronoi = (int)h_voronoi.size() / 2;
    out.voronoi_xy = h_voronoi.data();
    out.rows_info_xy = h_rows_info.data();
    out.n_cluster_info = (int)h_cluster_info.size() / 2;
    out.cluster_info_xy = h_cluster_info.data();
    auto ms = [&](int a, int b) { float t = 0; (void)hipEventElapsedTime(&t, ev[a], ev[b]); return t; };
    // (a tiled frame: its cluster stage starts at ev[6], after the grids' all-gather)
    out.ms_ror = ms(0, 1); out.ms_grid = ms(1, 2); out.ms_thin = ms(2, 3); out.ms_cluster = ms(pre ? 6 : 3, 4);
    out.ms_seeds = ms(4, 5); out.ms_total = ms(0, 5);
    if (trace_on() && !pre)
        fprintf(stderr, "[aos trace events] thin_end->stage_start %.3f stage_gpu %.3f gpu_end->rows %.3f (ms)\n", ms(3, 16),
                ms(16, 17), ms(17, 4));
    out.n_binned = static_cast<const int *>(h_stats.p)[0];   // (ror_collect)
    out.ms_ror_count = out.n_binned ? ms(10, 11) : 0.0f;
    out.ms_ror_bin = out.n_binned ? ms(12, 13) : 0.0f;
    out.ms_ror_scatter = out.n_binned ? ms(14, 10) : 0.0f;
    out.thin_graph = tiled_frame ? 0 : last_thin_graph;
    out.thin_launches = last_thin_launches;
    out.n_ror_read = ror_read;
}

int aos_ctx::debug_grid(const char *which, int8_t *dst, uint64_t capacity) {
    const size_t C = (size_t)geom.W * geom.H;
    if (capacity < C) { set_error("aos_debug_grid: capacity < width*height"); return AOS_E_INVALID; }
    const uint64_t *bits = nullptr;
    if (!std::strcmp(which, "inflated")) bits = tiled_frame ? full_infl.as<uint64_t>() : infl_bits.as<uint64_t>();
    else if (!std::strcmp(which, "skeleton_frameless")) bits = skel_bits;
    else if (!tiled_frame && !std::strcmp(which, "raster")) bits = raster_bits.as<uint64_t>();
    else if (!tiled_frame && !std::strcmp(which, "opened")) bits = open_bits.as<uint64_t>();
    else {
        set_error(std::string("aos_debug_grid: unknown grid (or not kept by a tiled frame) ") + which);
        return AOS_E_INVALID;
    }
    DevBuf tmp;
    int8_t *d = static_cast<int8_t *>(tmp.ensure(C));
    launch_bits_to_bytes(bits, d, geom, 0, stream);
    AOS_HIP(hipMemcpyAsync(dst, d, C, hipMemcpyDeviceToHost, stream));
    AOS_HIP(hipStreamSynchronize(stream));
    tmp.release();
    return AOS_OK;
}
