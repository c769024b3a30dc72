// Per-handle state of libaos_gpu.so. Not part of the ABI.
#pragma once
#include <array>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "aos_internal.h"
#include "cluster_seed.h"
#include "grid_host.h"
#include "host_pool.h"

struct aos_ctx {
    aos_params P{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::array<hipEvent_t, 18> ev{};   // (16, 17: AOS_TRACE splits of the cluster stage)
    aos::Poly poly;

    // ---- last cloud (reprocess reuses it: seed_gen:244, 283-285)
    bool have_cloud = false, have_frame = false;
    const uint8_t *d_cloud = nullptr;  // device view (own copy or caller's device buffer)
    uint64_t n_points = 0;
    uint32_t step = 16, ox = 0, oy = 4, oz = 8;
    int is_dense = 1;

    // ---- streaming map (aos_map_append): float4 x, y, z, 0
    aos::DevBuf map_buf, scan_stage;
    uint64_t map_n = 0;
    int map_dense = 1;
    // tiled streaming map (aos_tiled_map_append): the rank's map holds only the points of its points
    // box; map_total counts every point appended (the frame's n_input, as on one GPU)
    bool map_boxed = false;
    float map_box[4] = {0, 0, 0, 0};
    uint64_t map_total = 0;
    aos::DevBuf map_count;
    aos::PinnedBuf h_map_count;
    // ---- tile store of the streaming map (incremental ROR, seedgen.hip ror_stage): the map's binned
    // points partitioned by ROR tile (own + halo copies, ping-pong), tile starts, kept candidates per
    // tile; valid while the geometry, density and raster bits are the ones it was built with
    struct MapStore {
        bool valid = false;
        aos::RorLaunch L{};          // geometry it was built with (pointers / counts cleared)
        aos::DevBuf st[2], ts[2], kept, scan_st, scan_H, scan_ts;
        int cur = 0, dense = 1;
        uint64_t n_points = 0;       // map points it covers
        double n_binned = 0;         // binned (own) points it holds
        size_t n_staged = 0;         // staged copies it holds
        // what this frame's ROR stage built, committed by ror_collect after the read-back
        struct Pending {
            bool on = false, incremental = false;
            aos::RorLaunch L{};
            int dense = 1;
            uint64_t n_points = 0;
            int cur = 0;
        } pend;
    } ms;
    uint64_t map_scan_begin = 0;     // map points before the last aos_map_append

    // ---- device buffers
    aos::DevBuf cloud_copy, bin_count, bin_start, sorted, ror_scratch, ror_bigbins, scan_tmp, counters;
    aos::DevBuf raster_bits, infl_bits, open_bits, thin_a, thin_b, thin_act, occ_bytes, skel_bytes, flags;
    aos::DevBuf thin_out;   // the converged skeleton bits, picked on the device (launch_thin_pick)
    aos::LookBackScratch ror_lb;           // look-back words of the ROR column scan (k_rt_colscan)
    aos::DevBuf full_infl, full_skel;      // tiled frames: the whole map, assembled on the root rank
    aos::PinnedBuf h_small, h_stats;
    // Host -> device upload of a large pageable buffer (a PointCloud2 message): kUpThreads host
    // threads copy 2 MB chunks into rings of pinned slots, each DMA'd on the thread's stream (tools/upload_ab.py:
    // 4-8 threads and 1-8 MB chunks all upload C2's 120 MB in 3-4 ms on the box, the H2D DMA's ~40 GB/s).
    static constexpr int kUpThreads = 16;   // capacity; up_threads() of them gather (AOS_UP_THREADS, default 16)
    static int up_threads();
    static constexpr int kUpSlots = 4;      // pinned slots per thread (a ring: gather one while others DMA)
    struct Uploader {
        aos::PinnedBuf slot[kUpThreads][kUpSlots];
        hipStream_t st[kUpThreads] = {};
        hipEvent_t ev[kUpThreads][kUpSlots] = {}, done[kUpThreads] = {};
        bool used[kUpThreads][kUpSlots] = {};
    } up;
    aos::HostPool up_pool;                  // the gather threads (upload_pack)
    // A host cloud is split while it is gathered (upload_pack): the points inside `box`, the ROR stage's
    // binned box for the polygon and parameters current at upload time (ror_stage: no point outside it
    // can be binned), go to the device, packed at the front of the cloud buffer in chunk-arrival order (the
    // ROR results do not depend on point order); the others stay in `rest` (pageable host memory: it is copied
    // only when the polygon grows, so it holds no page-locked memory — 2 x 12 n bytes at C2 with a prefetch —
    // ADVICE r04; thread t's run at byte rbeg[t], rn[t] points). A frame whose binned box is not inside `box`
    // (the polygon changed: aos_seedgen_reprocess) first copies the rest behind the front (cloud_for_box).
    struct CloudSplit {
        aos::HostBuf rest;
        uint64_t rbeg[kUpThreads] = {}, rn[kUpThreads] = {};
        int nth = 0;
        uint64_t n_front = 0, n_all = 0;
        float box[6] = {};          // bminx, bmaxx, bminy, bmaxy, bminz, bmaxz
        bool on = false;            // split (else all n_all points are on the device)
        bool whole = false;         // the rest was copied behind the front
        hipEvent_t copied = nullptr;   // that copy (recorded on the handle's stream; rest is rewritten after it)
        bool copy_pending = false;
        void swap_with(CloudSplit &o);
    } split_cur, split_next;
    static bool split_enabled();    // AOS_UP_SPLIT (default 1)
    bool split_box(const aos::Poly &poly, float box[6]) const;   // false: do not split
    uint64_t cloud_for_box(const float b[6]);   // device points the ROR stage reads for binned box b
    // prefetch = true (aos_cloud_prefetch): dst is not read by queued work and the handle's stream is not
    // made to wait; the consumer waits for up.done[] (set_cloud). sp: the split's state (box[] and on set
    // by the caller; on = false: no split)
    void upload_pack(void *dst, const aos_cloud_view &v, CloudSplit &sp, bool prefetch = false);
    void release_uploader();
    // aos_cloud_prefetch: the next frame's cloud uploaded into cloud_next on a background thread
    struct Prefetch {
        std::thread th;
        aos_cloud_view view{};
        const void *src = nullptr;
        size_t bytes = 0;
        bool active = false;
        std::exception_ptr err;
        float box[6] = {};
        bool split = false;
    } pf;
    aos::DevBuf cloud_next;
    void prefetch_start(const aos_cloud_view &v);
    bool prefetch_join();   // true: a prefetch was in flight and succeeded
    const uint64_t *skel_bits = nullptr;   // final thinning buffer (thin_a / thin_b, or full_skel)
    aos::FrameGeom geom{};                 // the whole map
    bool tiled_frame = false;
    int thin_iters = 0, thin_iters_prev = 0;   // (the previous frame's T sizes the first thinning batch)
    // First thinning batch (n temporal-block launches; the opening, which clears the flags, runs just before it so the
    // inflated grid's read-back can be queued behind it) as hipGraphs, one per batch
    // size n (a power of two), captured on first use and replayed while every pointer and size baked into
    // the graph is unchanged (seedgen.hip thin_first_batch). Graph shape: AOS_THIN_GRAPH (see there).
    struct ThinGraph {
        hipGraphExec_t exec = nullptr;
        std::array<const void *, 8> ptrs{};   // every device / host pointer a node holds
        std::array<int, 8> dims{};            // W, H, WW, R, launches, flag ints, shape, tiles
    };
    std::vector<ThinGraph> thin_graphs;
    int thin_graph_shape = -1;                // AOS_THIN_GRAPH at create (default 1)
    int last_thin_graph = 0, last_thin_launches = 0;
    bool thin_graph_check = false;            // AOS_THIN_GRAPH_CHECK (diagnosis)
    long thin_checks = 0, thin_check_failures = 0;
    void thin_graphs_release();
    bool thin_first_batch(const aos::FrameGeom &g, const uint64_t *d_ibits, uint64_t *d_open, uint64_t *const bufs[2],
                          int *d_flags, int *h_flags, int *d_act, int nflags, int &batch_n, int cap_launches,
                          const std::function<void(int)> &launch_next, const std::function<void()> &after_open);
    void thin_check_flags(const int *d_flags, const int *h_flags, int n_read, int nflags);
    uint64_t n_ror_kept = 0, n_clipped = 0;
    double ror_est_binned = 0;             // binned points of the last frame (sizes the ROR tiles)
    double ror_staged_max = 0;             // largest staged (own + halo) count seen (sizes the scatter)
    bool ror_big_seen = false;             // a frame had a ROR tile beyond the LDS capacity (ror.hip big_ok)

    // ---- cluster / row / seed stage (cluster_seed.hip); tiled frames: distributed a8-a10 (cluster_dist.hip)
    aos::ClusterSeedState cs;
    aos::ClusterDistState cdist;
    aos::ClusterDistStats cdist_stats;

    // ---- host-side outputs of the last frame
    aos::PinnedBuf h_occ, h_skel;   // the two OccupancyGrids (pinned: the D2H runs at DMA speed)
    aos::PinnedBuf h_occ_bits, h_skel_bits;   // their bit-packed device grids (the default read-back, grid_host.h)
    aos::GridExpander expander;               // expands them on host threads beside the cluster / seed stage
    hipStream_t copy_stream = nullptr;   // their D2H, beside the cluster / seed stage
    hipEvent_t copy_ready = nullptr, copy_done = nullptr;
    bool infl_bits_sent = false;         // this frame's inflated-grid bits are already on the copy stream
    void grid_d2h(void *h, const void *d, size_t bytes);   // on the copy stream, after the work queued so far
    void grid_copy_wait();
    std::vector<double> h_row_center, h_row_start, h_row_end, h_row_length, h_voronoi, h_rows_info, h_cluster_info;
    int n_virtual = 0, n_ray = 0, n_endpoint = 0, n_clusters_all = 0, n_bfs_replayed = 0;

    // ---- GVD (gvd.hip)
    bool have_gvd = false, gvd_from_frame = false;
    uint64_t frame_gen = 0, gvd_frame_gen = 0, gvd_gen = 0;   // seed-gen frames / GVD calls so far
    const int8_t *gvd_skel = nullptr;                          // the skeleton the last GVD call used
    aos_grid_info gvd_info{};

    // ---- pipelined GVD (aos_gvd_from_seedgen_async): the reference runs seed-gen and the GVD as two
    // nodes, so frame k + 1's seed-gen overlaps frame k's graph. The GVD of a snapshot of the frame
    // (seeds, rows, skeleton) runs on a lane: a GvdState with a persistent worker thread and its own
    // stream. Frames are independent, so up to gvd_depth jobs may be in flight on gvd_depth lanes
    // (aos_gvd_pipeline_depth); one more lane holds the handle's current result (markers, planning).
    struct AsyncGvd {
        std::thread worker;
        std::mutex mu;
        std::condition_variable cv;
        bool busy = false, quit = false, pub = false, done = false, prefix = false;
        std::exception_ptr err;
        hipStream_t stream = nullptr;
        std::array<hipEvent_t, 16> ev{};
        hipEvent_t ready = nullptr;               // the snapshot copy on the seed-gen stream
        std::vector<double> seeds, rows;          // snapshot of h_voronoi / h_rows_info
        aos_grid_info info{};
        aos_params P{};                           // the handle's parameters when the job started (markers incl.)
        bool applied = false;                     // its result was made current by a settle (gvd_view_settle)
    };
    struct alignas(128) GvdLane {
        aos::GvdState gs;
        AsyncGvd ag;
    };
    std::vector<std::unique_ptr<GvdLane>> lanes{};   // lanes[cur_lane] holds the current result
    int cur_lane = 0, gvd_depth = 1;
    hipStream_t gvd_stream = nullptr;                // the lanes' shared GPU stream
    std::deque<int> inflight;                        // lanes with uncollected jobs, oldest first
    bool view_newest = false;                        // no aos_gvd_wait since the last job started
    aos::GvdState &gs() { return lanes[cur_lane]->gs; }
    void gvd_lanes_ensure();
    void gvd_async_start();
    bool gvd_async_wait(bool rethrow);   // aos_gvd_wait: collect the oldest job; false if none
    void gvd_view_settle();              // markers / planning: settle which result is current
    void gvd_async_drop();               // a synchronous GVD call supersedes every job in flight
    void gvd_async_stop();
    void lane_join(int l);               // waits for lane l's job (no bookkeeping)
    void lane_apply(int l);              // lane l's finished job becomes the current result

    // ---- path planning (path.hip)
    void *path_state = nullptr;   // aos::PathState

    // Cells a frame rasterises / counts: [rx0, rx1) x [ry0, ry1) (clamped cell), stored into the
    // Wr x Hr bit window at cell (wx0, wy0), wx0 a multiple of 64; limit_box: bin only points in box
    // (a tile's shard).
    struct RorOwn { int rx0, ry0, rx1, ry1, wx0, wy0, Wr, Hr; bool limit_box; float box[4]; };

    void set_cloud(const aos_cloud_view &v);
    void map_append(const aos_cloud_view &scan);
    void map_append_box(const aos_cloud_view &scan, const float box[4]);   // tiled streaming map
    void map_grow(uint64_t n);
    void ror_stage(const aos::FrameGeom &g, const RorOwn &o, uint64_t *rbits, bool allow_guess);
    bool ror_collect(bool throw_stuck = true);
    void ror_stats_to_host(const int *d_staged_total, const unsigned long long *d_own);   // after the stream synchronised: true if the ROR scatter overflowed
    void ror_stage_append(aos::RorLaunch L, uint64_t *rbits);   // streaming map: one scan on the tile store
    aos::LookBack ror_lookback(const aos::RorLaunch &L, int G, unsigned long long *d_own);
    void ror_stage_unchanged();   // streaming map: no new points since the committed store
    uint64_t ror_skipped = 0;     // frames that skipped the ROR stage that way
    uint64_t ror_read = 0;        // points this frame's partition passes read (aos_seedgen_out::n_ror_read)
    void finish_frame(const aos::FrameGeom &g, bool want_host, const uint64_t *clipped_total, aos_seedgen_out &out,
                      const aos::PreClusters *pre = nullptr);
    void run_seedgen(bool want_host, aos_seedgen_out &out);
    bool run_seedgen_once(bool want_host, aos_seedgen_out &out, bool allow_guess);   // true: redo
    void run_tiled(const aos_comm &cm, int tiles_x, int tiles_y, int root, bool want_host, aos_seedgen_out &out);
    void run_tiled_frame(aos::FrameComm &fc, int tiles_x, int tiles_y, int root, bool want_host, aos_seedgen_out &out);
    aos_tiled_stats tstats{};   // the last tiled frame's breakdown (aos_tiled_stats_get)
    std::vector<hipEvent_t> coll_ev;   // FrameComm: begin / end events of the frame's enqueued collectives
    aos::DevBuf coll_red;              // FrameComm: the reduced thinning flags
    aos::LookBackScratch debug_lb;     // aos_debug_scan
    void tile_halo_exchange(uint64_t *win, const aos::TilePlan &t, aos::FrameComm &fc);
    void run_gvd_external(const aos_gvd_in &in, aos_gvd_out &out);
    void run_gvd_from_frame(aos_gvd_out &out);
    void run_path_plan(const aos_path_graph *graph, const int8_t *skeleton, int skeleton_on_device,
                       const aos_grid_info *info, const aos_path_query &q, aos_path_out &out);
    int debug_grid(const char *which, int8_t *dst, uint64_t capacity);
    void release();
};

namespace aos {
// aos_gvd_wait: collects the pipelined GVD job's graph into out; 0 if no job was started (gvd.hip)
int gvd_wait_out(aos_ctx *c, aos_gvd_out *out);
}  // namespace aos
