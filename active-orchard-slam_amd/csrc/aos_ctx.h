// Per-handle state of libaos_gpu.so. Not part of the ABI.
#pragma once
#include <array>
#include <vector>

#include "aos_internal.h"
#include "cluster_seed.h"

struct aos_ctx {
    aos_params P{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::array<hipEvent_t, 12> ev{};
    aos::Poly poly;

    // ---- last cloud (reprocess reuses it: seed_gen:244, 283-285)
    bool have_cloud = false, have_frame = false;
    const uint8_t *d_cloud = nullptr;  // device view (own copy or caller's device buffer)
    uint64_t n_points = 0;
    uint32_t step = 16, ox = 0, oy = 4, oz = 8;
    int is_dense = 1;

    // ---- device buffers
    aos::DevBuf cloud_copy, bin_count, bin_start, pt_binslot, sorted, scan_tmp, counters;
    aos::DevBuf raster_bytes, raster_bits, infl_bits, open_bits, thin_a, thin_b, occ_bytes, skel_bytes, flags;
    aos::PinnedBuf h_small, h_stats;
    const uint64_t *skel_bits = nullptr;   // final thinning buffer (thin_a or thin_b)
    aos::FrameGeom geom{};
    int thin_iters = 0;
    uint64_t n_ror_kept = 0, n_clipped = 0;

    // ---- cluster / row / seed stage (cluster_seed.hip)
    aos::ClusterSeedState cs;

    // ---- host-side outputs of the last frame
    std::vector<int8_t> h_occ, h_skel;
    std::vector<double> h_row_center, h_row_start, h_row_end, h_row_length, h_voronoi, h_rows_info, h_cluster_info;
    int n_virtual = 0, n_ray = 0, n_endpoint = 0, n_clusters_all = 0, n_bfs_replayed = 0;

    // ---- GVD (gvd.hip)
    aos::GvdState gs;

    void set_cloud(const aos_cloud_view &v);
    void run_seedgen(bool want_host, aos_seedgen_out &out);
    void run_gvd_external(const aos_gvd_in &in, aos_gvd_out &out);
    void run_gvd_from_frame(aos_gvd_out &out);
    int debug_grid(const char *which, int8_t *dst, uint64_t capacity);
    void release();
};
