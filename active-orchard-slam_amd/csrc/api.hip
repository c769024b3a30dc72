// libaos_gpu.so — C ABI + per-handle orchestration of the seed-gen / GVD hot path on MI355X.
// One handle = one device + one HIP stream; all stage buffers stay resident in HBM.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>

#include "aos_ctx.h"

namespace aos {

thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

static const auto g_epoch = std::chrono::steady_clock::now();
double trace_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_epoch).count(); }
bool trace_on() {
    static const bool on = getenv("AOS_TRACE") != nullptr;
    return on;
}
void trace_alloc(const char *kind, size_t bytes, double t0) {
    fprintf(stderr, "[aos trace alloc] %s %.1f MB at %.2f ms took %.2f ms\n", kind, bytes / 1e6, t0, trace_ms() - t0);
}

}  // namespace aos

using namespace aos;

#define AOS_GUARD_BEGIN try {
#define AOS_GUARD_END                                                                                         \
    }                                                                                                         \
    catch (const HipError &e) {                                                                               \
        set_error(std::string("HIP error ") + hipGetErrorString(e.e) + " at api line " + std::to_string(e.line) + \
                  ": " + e.what);                                                                             \
        return AOS_E_HIP;                                                                                     \
    }                                                                                                         \
    catch (const std::bad_alloc &) {                                                                          \
        set_error("out of host memory");                                                                      \
        return AOS_E_NOMEM;                                                                                   \
    }                                                                                                         \
    catch (const CommError &e) {                                                                              \
        set_error("communicator error: " + e.what);                                                           \
        return AOS_E_RCCL;                                                                                    \
    }                                                                                                         \
    catch (const std::invalid_argument &e) {                                                                  \
        set_error(std::string("invalid argument: ") + e.what());                                              \
        return AOS_E_INVALID;                                                                                 \
    }                                                                                                         \
    catch (const std::exception &e) {                                                                         \
        set_error(std::string("error: ") + e.what());                                                         \
        return AOS_E_STATE;                                                                                   \
    }

namespace aos {
std::atomic<int> g_debug_stuck_rank{-1};
std::atomic<uint64_t> g_debug_a2a_round{0};
std::atomic<int> g_debug_replay_min{-1};
std::atomic<int> g_debug_replay_ring{0};
std::atomic<bool> g_debug_replay_all{false};
}  // namespace aos

extern "C" {

const char *aos_last_error(void) { return g_err.c_str(); }

void aos_default_params(aos_params *p) {
    p->clipping_minz = -0.4f; p->clipping_maxz = 0.5f;
    p->clipping_minx = -5.0f; p->clipping_maxx = 72.0f;
    p->clipping_miny = -10.0f; p->clipping_maxy = 20.0f;
    p->grid_resolution = 0.05f;
    p->inflation_radius = 0.8f;
    p->cluster_min_length = 2.0;
    p->ror_radius = 0.2;
    p->ror_min_neighbors = 2;
    p->subdiv_rect_mode = 0;
    p->max_graph_publish_rate = 10.0;
    p->gvd_markers = 1;
    p->thin_graph = 1;
    p->gvd_count_evals = 0;
}

int aos_create(const aos_params *p, int device, aos_ctx **out) {
    if (!p || !out) { set_error("aos_create: null argument"); return AOS_E_INVALID; }
    *out = nullptr;
    AOS_GUARD_BEGIN
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("aos_create: no HIP device visible (libaos_gpu has no CPU fallback)");
        return AOS_E_HIP;
    }
    if (device < 0 || device >= ndev) { set_error("aos_create: bad device index"); return AOS_E_INVALID; }
    hipDeviceProp_t prop;
    AOS_HIP(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
        set_error(std::string("aos_create: device is ") + prop.gcnArchName + ", this build targets gfx950 only");
        return AOS_E_HIP;
    }
    auto *c = new aos_ctx();
    c->P = *p;
    c->device = device;
    DeviceScope dev_scope(device);
    AOS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (auto &e : c->ev) AOS_HIP(hipEventCreate(&e));
    c->poly = default_polygon();
    c->gvd_lanes_ensure();
    *out = c;
    return AOS_OK;
    AOS_GUARD_END
}

void aos_destroy(aos_ctx *c) {
    if (!c) return;
    DeviceScope dev_scope(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->release();
    for (auto &e : c->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

void *aos_stream(aos_ctx *c) { return c ? (void *)c->stream : nullptr; }

void aos_debug_faults(int32_t ror_stuck_rank, uint64_t a2a_round_bytes) {
    aos::g_debug_stuck_rank.store(ror_stuck_rank, std::memory_order_relaxed);
    aos::g_debug_a2a_round.store(a2a_round_bytes, std::memory_order_relaxed);
}

void aos_debug_replay(int32_t gpu_min_clusters, int32_t ring_cap, int32_t replay_all) {
    aos::g_debug_replay_all.store(replay_all != 0, std::memory_order_relaxed);
    aos::g_debug_replay_min.store(gpu_min_clusters < 0 ? -1 : gpu_min_clusters, std::memory_order_relaxed);
    aos::g_debug_replay_ring.store(ring_cap > 0 ? ring_cap : 0, std::memory_order_relaxed);
}

int aos_replay_counts(aos_ctx *c, int32_t out[4]) {
    if (!c || !out) { set_error("aos_replay_counts: null argument"); return AOS_E_INVALID; }
    out[0] = c->n_bfs_replayed;
    out[1] = c->cs.n_replay_gpu;
    out[2] = c->cs.n_replay_from_bits;
    out[3] = c->cs.n_replay_cells;
    return AOS_OK;
}

void aos_comm_init(aos_comm *comm) {
    if (comm) std::memset(comm, 0, sizeof(*comm));
}

int aos_set_polygon(aos_ctx *c, const double *xy, uint32_t n) {
    if (!c) { set_error("null handle"); return AOS_E_INVALID; }
    if (!xy || n < 3) return AOS_OK;  // explorationAreaCallback ignores < 3 points (seed_gen:253)
    c->poly.clear();
    for (uint32_t i = 0; i < n; ++i) c->poly.push_back({xy[2 * i], xy[2 * i + 1]});
    return AOS_OK;
}

static bool cloud_layout_ok(const aos_cloud_view *cloud) {
    if (!cloud->n_points) return true;
    return cloud->data && cloud->point_step >= 12 && !(cloud->point_step & 3) && !(cloud->off_x & 3) &&
           !(cloud->off_y & 3) && !(cloud->off_z & 3) && cloud->off_x + 4 <= cloud->point_step &&
           cloud->off_y + 4 <= cloud->point_step && cloud->off_z + 4 <= cloud->point_step;
}

int aos_seedgen_process(aos_ctx *c, const aos_cloud_view *cloud, int want_host, aos_seedgen_out *out) {
    if (!c || !cloud || !out) { set_error("aos_seedgen_process: null argument"); return AOS_E_INVALID; }
    if (!cloud_layout_ok(cloud)) {
        set_error("aos_seedgen_process: invalid PointCloud2 layout (float32 x/y/z, 4-byte aligned)");
        return AOS_E_INVALID;
    }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->set_cloud(*cloud);
    c->run_seedgen(want_host != 0, *out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_seedgen_reprocess(aos_ctx *c, int want_host, aos_seedgen_out *out) {
    if (!c || !out) { set_error("aos_seedgen_reprocess: null argument"); return AOS_E_INVALID; }
    if (!c->have_cloud) { std::memset(out, 0, sizeof(*out)); return AOS_OK; }  // last_cloud empty (:283)
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->run_seedgen(want_host != 0, *out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_map_reset(aos_ctx *c, uint64_t reserve_points) {
    if (!c) { set_error("aos_map_reset: null handle"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->map_n = 0;
    c->map_total = 0;
    c->map_boxed = false;
    c->ms.valid = false;
    c->map_dense = 1;
    if (reserve_points) c->map_buf.ensure(sizeof(float4) * reserve_points);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_map_append(aos_ctx *c, const aos_cloud_view *scan, int want_host, aos_seedgen_out *out) {
    if (!c || !scan || !out) { set_error("aos_map_append: null argument"); return AOS_E_INVALID; }
    if (!cloud_layout_ok(scan)) {
        set_error("aos_map_append: invalid PointCloud2 layout (float32 x/y/z, 4-byte aligned)");
        return AOS_E_INVALID;
    }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->map_append(*scan);
    c->run_seedgen(want_host != 0, *out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_gvd_process(aos_ctx *c, const aos_gvd_in *in, aos_gvd_out *out) {
    if (!c || !in || !out) { set_error("aos_gvd_process: null argument"); return AOS_E_INVALID; }
    // counts and their arrays (an empty seed or row list is the callbacks' early return, not an error)
    if (in->n_seeds < 0 || in->n_rows_poses < 0 || (in->n_seeds > 0 && !in->seeds_xy) ||
        (in->n_rows_poses > 0 && !in->rows_info_xy) || ((size_t)in->info.width * in->info.height > 0 && !in->skeleton)) {
        set_error("aos_gvd_process: negative count, or a null array for a non-empty seed / row list or skeleton grid");
        return AOS_E_INVALID;
    }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->run_gvd_external(*in, *out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_gvd_from_seedgen(aos_ctx *c, aos_gvd_out *out) {
    if (!c || !out) { set_error("aos_gvd_from_seedgen: null argument"); return AOS_E_INVALID; }
    if (!c->have_frame) { set_error("aos_gvd_from_seedgen: no seed-gen frame yet"); return AOS_E_STATE; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->run_gvd_from_frame(*out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_cloud_prefetch(aos_ctx *c, const aos_cloud_view *cloud) {
    if (!c) { set_error("aos_cloud_prefetch: null handle"); return AOS_E_INVALID; }
    if (cloud && !cloud_layout_ok(cloud)) { set_error("aos_cloud_prefetch: invalid PointCloud2 layout"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    if (cloud) c->prefetch_start(*cloud);
    else c->prefetch_join();   // wait for (and drop) the prefetch in flight
    return AOS_OK;
    AOS_GUARD_END
}

int aos_seedgen_grids_copy(aos_ctx *c, int8_t *occupancy, int8_t *skeleton) {
    if (!c) { set_error("aos_seedgen_grids_copy: null handle"); return AOS_E_INVALID; }
    if (!c->have_frame) { set_error("aos_seedgen_grids_copy: no seed-gen frame yet"); return AOS_E_STATE; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    const size_t C = (size_t)c->geom.W * c->geom.H;
    if (occupancy) AOS_HIP(hipMemcpyAsync(occupancy, c->occ_bytes.p, C, hipMemcpyDeviceToHost, c->stream));
    if (skeleton) AOS_HIP(hipMemcpyAsync(skeleton, c->skel_bytes.p, C, hipMemcpyDeviceToHost, c->stream));
    AOS_HIP(hipStreamSynchronize(c->stream));
    return AOS_OK;
    AOS_GUARD_END
}

int aos_gvd_from_seedgen_async(aos_ctx *c) {
    if (!c) { set_error("aos_gvd_from_seedgen_async: null handle"); return AOS_E_INVALID; }
    if (!c->have_frame) { set_error("aos_gvd_from_seedgen_async: no seed-gen frame yet"); return AOS_E_STATE; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->gvd_async_start();
    return AOS_OK;
    AOS_GUARD_END
}

int aos_gvd_wait(aos_ctx *c, aos_gvd_out *out) {
    if (!c || !out) { set_error("aos_gvd_wait: null argument"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    if (!gvd_wait_out(c, out)) { set_error("aos_gvd_wait: no GVD job started since the last wait"); return AOS_E_STATE; }
    return AOS_OK;
    AOS_GUARD_END
}

int aos_rccl_unique_id(uint8_t *id) {
    if (!id) { set_error("aos_rccl_unique_id: null argument"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    rccl_unique_id(id);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_rccl_create(const uint8_t *id, int32_t rank, int32_t world, int32_t device, uint64_t buf_bytes,
                    aos_rccl **out) {
    if (!id || !out) { set_error("aos_rccl_create: null argument"); return AOS_E_INVALID; }
    *out = nullptr;
    AOS_GUARD_BEGIN
    *out = rccl_create(id, rank, world, device, buf_bytes);
    return AOS_OK;
    AOS_GUARD_END
}

const aos_comm *aos_rccl_comm(aos_rccl *r) { return r ? rccl_comm(r) : nullptr; }

void aos_rccl_destroy(aos_rccl *r) { rccl_destroy(r); }

int aos_gvd_set_markers(aos_ctx *c, int32_t on) {
    if (!c) { set_error("aos_gvd_set_markers: null handle"); return AOS_E_INVALID; }
    c->P.gvd_markers = on ? 1 : 0;
    return AOS_OK;
}

int aos_gvd_set_count_evals(aos_ctx *c, int32_t on) {
    if (!c) { set_error("aos_gvd_set_count_evals: null handle"); return AOS_E_INVALID; }
    c->P.gvd_count_evals = on ? 1 : 0;
    return AOS_OK;
}

int aos_gvd_evals_get(aos_ctx *c, aos_gvd_evals *out) {
    if (!c || !out) { set_error("aos_gvd_evals_get: null argument"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->gvd_view_settle();   // (the result aos_gvd_wait collected last, as markers and planning use)
    *out = c->gs().evals;
    return AOS_OK;
    AOS_GUARD_END
}

int aos_gvd_pipeline_depth(aos_ctx *c, int32_t depth) {
    if (!c) { set_error("aos_gvd_pipeline_depth: null handle"); return AOS_E_INVALID; }
    if (depth < 1 || depth > 16) { set_error("aos_gvd_pipeline_depth: depth must be in [1, 16]"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->gvd_depth = depth;
    c->gvd_lanes_ensure();
    return AOS_OK;
    AOS_GUARD_END
}

int aos_tile_plan_compute(const aos_params *p, const double *poly_xy, uint32_t n_poly, int32_t tiles_x,
                          int32_t tiles_y, int32_t rank, aos_tile_plan *out) {
    if (!p || !out) { set_error("aos_tile_plan_compute: null argument"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    Poly poly = default_polygon();
    if (poly_xy && n_poly >= 3) {
        poly.clear();
        for (uint32_t i = 0; i < n_poly; ++i) poly.push_back({poly_xy[2 * i], poly_xy[2 * i + 1]});
    }
    const FrameGeom g = frame_geom(poly, *p);
    const TilePlan t = make_tile_plan(g, ror_margin(*p), tiles_x, tiles_y, rank);
    std::memset(out, 0, sizeof(*out));
    out->tiles_x = tiles_x; out->tiles_y = tiles_y; out->rank = rank; out->tile_x = t.tx; out->tile_y = t.ty;
    out->halo_rows = t.hy; out->halo_words = t.hw;
    out->row0 = t.y0; out->row1 = t.y1; out->word0 = t.c0; out->word1 = t.c1;
    out->win_row0 = t.wy0; out->win_row1 = t.wy1; out->win_word0 = t.wc0; out->win_word1 = t.wc1;
    for (int i = 0; i < 4; ++i) out->points_box[i] = t.box[i];
    out->exchange_bytes = t.exchange_bytes;
    out->info = aos_grid_info{g.origin_x, g.origin_y, g.res, (uint32_t)g.W, (uint32_t)g.H};
    return AOS_OK;
    AOS_GUARD_END
}

int aos_tiled_seedgen_process(aos_ctx *c, const aos_comm *comm, int32_t tiles_x, int32_t tiles_y, int32_t root,
                              const aos_cloud_view *cloud, int want_host, aos_seedgen_out *out) {
    if (!c || !comm || !cloud || !out) { set_error("aos_tiled_seedgen_process: null argument"); return AOS_E_INVALID; }
    if (!cloud_layout_ok(cloud)) {
        set_error("aos_tiled_seedgen_process: invalid PointCloud2 layout (float32 x/y/z, 4-byte aligned)");
        return AOS_E_INVALID;
    }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->set_cloud(*cloud);
    c->run_tiled(*comm, tiles_x, tiles_y, root, want_host != 0, *out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_tiled_map_append(aos_ctx *c, const aos_comm *comm, int32_t tiles_x, int32_t tiles_y, int32_t root,
                         const aos_cloud_view *scan, int want_host, aos_seedgen_out *out) {
    if (!c || !comm || !scan || !out) { set_error("aos_tiled_map_append: null argument"); return AOS_E_INVALID; }
    if (!cloud_layout_ok(scan)) {
        set_error("aos_tiled_map_append: invalid PointCloud2 layout (float32 x/y/z, 4-byte aligned)");
        return AOS_E_INVALID;
    }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    const FrameGeom g = frame_geom(c->poly, c->P);
    const TilePlan t = make_tile_plan(g, ror_margin(c->P), tiles_x, tiles_y, comm->rank);
    c->map_append_box(*scan, t.box);
    c->run_tiled(*comm, tiles_x, tiles_y, root, want_host != 0, *out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_tiled_stats_get(aos_ctx *c, aos_tiled_stats *out) {
    if (!c || !out) { set_error("aos_tiled_stats_get: null argument"); return AOS_E_INVALID; }
    *out = c->tstats;
    return AOS_OK;
}

// settle = true: the handle's newest result (a job started since the last aos_gvd_wait is waited for);
// false: the frame last returned by aos_gvd_wait / a synchronous GVD call, even with newer jobs in flight
static int markers_get(aos_ctx *c, aos_gvd_markers *out, bool settle) {
    if (!c || !out) { set_error("aos_gvd_markers_get: null argument"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    if (settle) c->gvd_view_settle();
    markers_wait(c->gs(), true);   // the cells run on after the graph is returned
    // a frame whose GVD ran with markers off (aos_gvd_set_markers): computed now, as publishMarkers
    // does for the frames the node publishes (gvd:306-314)
    if (!c->gs().have_markers && c->gs().graph_ok) markers_on_demand(c->gs());
    AOS_GUARD_END
    GvdState &G = c->gs();
    if (!G.have_markers || !G.cells) {
        set_error("aos_gvd_markers_get: no markers (gvd_markers = 0 or no GVD frame)");
        return AOS_E_STATE;
    }
    const CellsWork &W = *G.cells;
    std::memset(out, 0, sizeof(*out));
    out->n_seeds = (int32_t)(G.merged_xy.size() / 2); out->seeds_xy = G.merged_xy.data();
    out->n_rows = (int32_t)(G.row_label_valid.size() / 4);
    out->row_label_xy = G.row_label_xy.data(); out->row_label_valid = G.row_label_valid.data();
    out->n_cells = (int32_t)W.cell_off.size() - 1;
    out->cell_offsets = W.cell_off.data(); out->cell_xy = W.cell_xy.data();
    out->cell_center_xy = W.cell_center.data(); out->cell_rgba = W.cell_rgba.data();
    out->ms_cells = W.ms;
    return AOS_OK;
}

int aos_gvd_markers_get(aos_ctx *c, aos_gvd_markers *out) { return markers_get(c, out, true); }

int aos_gvd_collected_markers_get(aos_ctx *c, aos_gvd_markers *out) { return markers_get(c, out, false); }

int aos_path_plan(aos_ctx *c, const aos_path_graph *graph, const int8_t *skeleton, int skeleton_on_device,
                  const aos_grid_info *info, const aos_path_query *query, aos_path_out *out) {
    if (!c || !query || !out) { set_error("aos_path_plan: null argument"); return AOS_E_INVALID; }
    if (skeleton && !info) { set_error("aos_path_plan: skeleton without grid info"); return AOS_E_INVALID; }
    if (skeleton && (info->width == 0 || info->height == 0 || !(info->resolution > 0.0f))) {
        set_error("aos_path_plan: empty skeleton grid or resolution <= 0");
        return AOS_E_INVALID;
    }
    if (graph && (graph->num_nodes < 0 || graph->num_edges < 0 || graph->n_label_entries < 0 ||
                  (graph->num_nodes && (!graph->nodes_xy || !graph->node_labels || !graph->node_cluster_indices ||
                                        !graph->node_label_counts)) ||
                  (graph->num_edges && (!graph->edges || !graph->edge_lengths)) ||
                  (graph->n_label_entries && (!graph->node_label_clusters || !graph->node_label_types)))) {
        set_error("aos_path_plan: inconsistent graph arrays");
        return AOS_E_INVALID;
    }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    c->run_path_plan(graph, skeleton, skeleton_on_device, info, *query, *out);
    return AOS_OK;
    AOS_GUARD_END
}

int aos_debug_scan(aos_ctx *c, int32_t *d_in, int32_t *d_out, int32_t n, int zero_in) {
    if (!c || (n > 0 && (!d_in || !d_out)) || n < 0) { set_error("aos_debug_scan: bad argument"); return AOS_E_INVALID; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    aos::scan_1p(c->debug_lb, d_in, d_out, n, zero_in != 0, c->stream);
    int *err = c->debug_lb.err_word(c->stream);
    int h = 0;
    AOS_HIP(hipMemcpyAsync(&h, err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    AOS_HIP(hipStreamSynchronize(c->stream));
    if (h) { set_error("aos_debug_scan: look-back error word " + std::to_string(h)); return AOS_E_HIP; }
    return AOS_OK;
    AOS_GUARD_END
}

int aos_debug_grid(aos_ctx *c, const char *which, int8_t *dst, uint64_t capacity) {
    if (!c || !which || !dst) { set_error("aos_debug_grid: null argument"); return AOS_E_INVALID; }
    if (!c->have_frame) { set_error("aos_debug_grid: no frame"); return AOS_E_STATE; }
    AOS_GUARD_BEGIN
    DeviceScope dev_scope(c->device);
    return c->debug_grid(which, dst, capacity);
    AOS_GUARD_END
}

}  // extern "C"
