/*
 * aos_gpu.h — C ABI of libaos_gpu.so, the MI355X (gfx950) implementation of the AOS
 * seed-gen + GVD hot path.
 *
 * The reference has no plugin/FFI boundary: the path is two rclcpp nodes wired by topics.
 * Each entry point below replaces one reference callback; the rclcpp drop-in wrapper
 * (active-orchard-slam_amd/node/) maps the same topics, QoS and parameter
 * names onto these calls.
 *
 *   aos_seedgen_process   <- AosSeedGenNode::globalMapCallback   src/aos_seed_gen_node.cpp:230-248
 *   aos_set_polygon       <- AosSeedGenNode::explorationAreaCallback (polygon part) :250-277
 *   aos_seedgen_reprocess <- explorationAreaCallback -> processPointCloud(last_cloud) :282-285
 *   aos_gvd_process       <- AosGvdNode::processGraph on the settled inputs of
 *                            voronoiSeedsCallback :84-128, explorationTreeRowsInfoCallback :130-150,
 *                            skeletonizedGridCallback :173-177  (src/aos_gvd_node.cpp:255-318)
 *   aos_gvd_from_seedgen  <- the same, fed directly from this handle's last seed-gen frame
 *                            (device-resident, no serialisation) — the fused pipeline.
 *
 * Conventions
 *  - Plain C types only; no torch / HIP types cross this boundary.
 *  - Status: 0 = OK, < 0 = error (AOS_E_*); aos_last_error() returns a thread-local message.
 *    No C++ exception crosses the ABI. Empty input -> empty outputs with status 0, mirroring the
 *    reference's early returns (gvd:257-259, 273-275, 284-287).
 *  - Inputs are caller-owned and only read during the call. Output arrays are library-owned and
 *    valid until the next call on the same handle or aos_destroy.
 *  - One handle = one device + one HIP stream; a handle is not re-entrant, different handles may
 *    run concurrently (one per GPU).
 *  - There is no CPU fallback: without a usable gfx950 device aos_create fails.
 */
#ifndef AOS_GPU_H
#define AOS_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AOS_OK 0
#define AOS_E_INVALID -1
#define AOS_E_NOMEM -2
#define AOS_E_HIP -3
#define AOS_E_STATE -4
#define AOS_E_RCCL -5

/* Parameters: names and defaults of the reference nodes (seed_gen:69-100, gvd:26,
 * config/aos_planner_params.yaml:55-89). */
typedef struct aos_params {
    float clipping_minz, clipping_maxz;      /* -0.4, 0.5  (seed-gen node override)     */
    float clipping_minx, clipping_maxx;      /* -5, 72    (only used without polygon)   */
    float clipping_miny, clipping_maxy;      /* -10, 20                                  */
    float grid_resolution;                   /* 0.05                                     */
    float inflation_radius;                  /* 0.8                                      */
    double cluster_min_length;               /* 2.0                                      */
    double ror_radius;                       /* 0.2 (hard-coded, seed_gen:238)           */
    int32_t ror_min_neighbors;               /* 2   (hard-coded, seed_gen:239)           */
    int32_t subdiv_rect_mode;                /* 0: Subdiv2D(Rect2f); 1: Rect2f->Rect      */
    double max_graph_publish_rate;           /* 10 Hz (throttle is the wrapper's job)    */
    int32_t gvd_markers;                     /* 1: also publishMarkers' Voronoi cells (gvd:1098-1194),
                                                a second Subdiv2D on its own host thread */
    int32_t thin_graph;                      /* 1 (default): the first thinning batch of a frame is a
                                                replayed hipGraph; 0: plain kernel launches */
    int32_t gvd_count_evals;                 /* 0 (default); 1: the GVD graph phase counts the work of its
                                                searches (aos_gvd_evals_get; a few atomics per workgroup) */
} aos_params;

void aos_default_params(aos_params *p);

typedef struct aos_ctx aos_ctx;

/* PointCloud2 view (fields x, y, z float32 at the given byte offsets). */
typedef struct aos_cloud_view {
    const void *data;        /* n_points * point_step bytes                                   */
    uint64_t n_points;
    uint32_t point_step, off_x, off_y, off_z;
    int32_t is_dense;        /* PointCloud2.is_dense: selects PCL's kNN vs radius ROR branch   */
    int32_t on_device;       /* 1: data is a device pointer on this handle's GPU (no H2D copy) */
} aos_cloud_view;

/* OccupancyGrid.info subset. */
typedef struct aos_grid_info {
    double origin_x, origin_y;
    float resolution;
    uint32_t width, height;
} aos_grid_info;

/* Seed-gen frame outputs. Host arrays are filled only when want_host != 0 (aos_seedgen_process
 * argument); device arrays are always valid (HBM, library-owned). */
typedef struct aos_seedgen_out {
    aos_grid_info info;
    int32_t thin_iters;                  /* Zhang-Suen iterations incl. the final no-change pass */
    uint64_t n_input, n_ror_kept, n_clipped;
    /* grids, int8 {0,100}, row-major x + y*width */
    const int8_t *occupancy;             /* /occupancy_grid (inflated + 5-cell frame)            */
    const int8_t *skeleton;              /* /skeletonized_occupancy_grid (with polygon frame)    */
    const int8_t *d_occupancy, *d_skeleton;
    /* clusters after the length filter, discovery order */
    int32_t n_clusters_all;              /* before the length filter                             */
    int32_t n_bfs_replayed;              /* clusters without the order-free certificate (exact BFS) */
    int32_t n_rows;                      /* tree rows (all_tree_rows order)                      */
    const double *row_center, *row_start, *row_end, *row_length;  /* 2, 2, 2, 1 per row         */
    /* /voronoi_seeds = virtual ++ real(empty) ++ ray ++ endpoint seeds (x, y) */
    int32_t n_virtual, n_ray, n_endpoint, n_voronoi;
    const double *voronoi_xy;
    /* /exploration_tree_rows_info: sorted (start.x, start.y, end.x, end.y) per row */
    const double *rows_info_xy;
    /* /cluster_info: exploration cluster centres sorted by y */
    int32_t n_cluster_info;
    const double *cluster_info_xy;
    /* per-stage device time (ms), HIP events */
    float ms_ror, ms_grid, ms_thin, ms_cluster, ms_seeds, ms_total;
    /* ROR stage (ror.hip): points it binned (near the clip box); device time of the per-tile
     * neighbour counts (k_rt_ror + the big-tile kernels), of the count pass + tile scan (ms_ror_bin)
     * and of the scatter pass (ms_ror_scatter), HIP events on the handle's stream */
    uint64_t n_binned;
    float ms_ror_count;
    float ms_ror_bin, ms_ror_scatter;
    /* thinning launches of this frame: thin_graph = 0 plain launches, 1 the first batch replayed from
     * a hipGraph, 2 that graph captured this frame (then launched); thin_launches = k_thin_block
     * launches issued (8 Zhang-Suen iterations each, launches past convergence return at once) */
    int32_t thin_graph, thin_launches;
    /* points the ROR stage's partition passes read: a host cloud's upload keeps on the device only the
     * points near the clip box of the polygon current at upload time (the others stay in pinned host
     * memory until a frame's box needs them); otherwise every point of the cloud / map */
    uint64_t n_ror_read;
} aos_seedgen_out;

/* GVD inputs when not fed from this handle's seed-gen frame. */
typedef struct aos_gvd_in {
    const double *seeds_xy; int32_t n_seeds;          /* /voronoi_seeds poses (x, y)            */
    const double *rows_info_xy; int32_t n_rows_poses;  /* /exploration_tree_rows_info poses      */
    aos_grid_info info;
    const int8_t *skeleton;                            /* /skeletonized_occupancy_grid data      */
} aos_gvd_in;

/* msg/GvdGraph.msg fields. */
typedef struct aos_gvd_out {
    int32_t published;                   /* 0 when processGraph returns early                   */
    double resolution, origin_x, origin_y;
    int32_t num_nodes, num_edges;
    const double *nodes_xy;
    const int32_t *node_labels, *node_cluster_indices, *node_label_counts;
    int32_t n_label_entries;
    const int32_t *node_label_clusters, *node_label_types;
    const int32_t *edges;                /* 2 per edge                                          */
    const float *edge_lengths, *edge_clearances;
    int32_t n_merged_seeds, n_voronoi_edges, n_boundary_points;
    float ms_merge, ms_delaunay, ms_graph, ms_total;
    float ms_cells;                      /* always 0: the cells finish after the call returns;
                                            see aos_gvd_markers.ms_cells                          */
} aos_gvd_out;

const char *aos_last_error(void);
int aos_create(const aos_params *p, int device, aos_ctx **out);
void aos_destroy(aos_ctx *ctx);
int aos_set_polygon(aos_ctx *ctx, const double *xy, uint32_t n_points);  /* n < 3: ignored (:253) */
int aos_seedgen_process(aos_ctx *ctx, const aos_cloud_view *cloud, int want_host, aos_seedgen_out *out);
int aos_seedgen_reprocess(aos_ctx *ctx, int want_host, aos_seedgen_out *out);
/* aos_gvd_process: AOS_E_INVALID for a negative count or a null array behind a non-empty seed / row list or
 * grid; empty lists are processGraph's early returns (status 0, published 0); non-finite seeds are filtered. */
int aos_gvd_process(aos_ctx *ctx, const aos_gvd_in *in, aos_gvd_out *out);
int aos_gvd_from_seedgen(aos_ctx *ctx, aos_gvd_out *out);
/* Pipelined form: the reference runs seed-gen and the GVD as two nodes, so frame k + 1's seed-gen
 * overlaps frame k's graph. _async snapshots the last seed-gen frame's GVD inputs (seeds, rows,
 * skeleton) and starts the GVD on a worker thread and its own stream; aos_seedgen_process /
 * aos_map_append may run meanwhile. aos_gvd_wait returns that graph (the same as
 * aos_gvd_from_seedgen would have). A synchronous GVD call supersedes every job in flight.
 * Frames are independent, so up to `depth` jobs (aos_gvd_pipeline_depth, default 1) may be in flight,
 * each replaying its Subdiv2D on its own host thread; aos_gvd_wait collects them in start order, and
 * starting one more than `depth` supersedes the oldest. aos_gvd_markers_get / aos_path_plan on the
 * handle's graph use the job aos_gvd_wait collected last, or the newest job if none was collected
 * since it started (they wait for it without collecting it). */
/* Starts copying a host PointCloud2 to the device in the background (a node can start as soon as the
 * message arrives, while the previous frame is processed). The next aos_seedgen_process with a host view
 * joins it: the same view (same data pointer and size) uses that copy instead of uploading (a failed
 * prefetch of it is raised there); another host view drops it (and any error it had) and uploads
 * normally. aos_cloud_prefetch (another cloud or NULL) joins it too and raises its error; aos_destroy
 * joins and drops it;
 * aos_seedgen_process with a device view and aos_map_append leave it in flight. The caller keeps the
 * bytes unchanged until it is joined. Device views and clouds under 32 MB are ignored.
 * cloud = NULL waits for the prefetch in flight and drops it. */
int aos_cloud_prefetch(aos_ctx *ctx, const aos_cloud_view *cloud);
/* The last seed-gen frame's two published OccupancyGrids (W*H bytes each, x + y*width), copied from HBM
 * straight into caller memory — e.g. the data vectors of the outgoing nav_msgs/OccupancyGrid messages
 * (seed_gen:552-577), so a frame run with want_host = 0 publishes without the library's host copies.
 * Either pointer may be null. */
int aos_seedgen_grids_copy(aos_ctx *ctx, int8_t *occupancy, int8_t *skeleton);
int aos_gvd_from_seedgen_async(aos_ctx *ctx);
int aos_gvd_wait(aos_ctx *ctx, aos_gvd_out *out);
int aos_gvd_pipeline_depth(aos_ctx *ctx, int32_t depth);   /* 1..16 GVD jobs in flight */
/* publishMarkers' cells for the GVD calls that follow (aos_params.gvd_markers): 1 = computed in the
 * background after each graph, 0 = not computed. The reference throttles publishGraph + publishMarkers
 * (gvd:306-314, max_graph_publish_rate): a wrapper that publishes 1 frame in n turns them on for the
 * published frames only. A background job keeps the value it had when it started. With 0,
 * aos_gvd_markers_get computes the cells of the current frame on demand (synchronously). */
int aos_gvd_set_markers(aos_ctx *ctx, int32_t on);
/* SURVEY §8d's GVD figure, "pair evaluations": the distance / sample evaluations of the graph phase's searches
 * in the last GVD call that ran with aos_params.gvd_count_evals = 1 (aos_gvd_set_count_evals). ref_* are what
 * the reference evaluates for the same inputs: findNearestBoundaryPoint scans every boundary point for each of
 * the 2E edge ends (gvd:812-824), the pair loop every i < j (gvd:861-894), findVoronoiBoundaryPointNearEndpoint
 * every filtered node once per radius it tries (gvd:686-790); gpu_* are the candidates this build's kernels
 * examined (k_nearest, k_pairs' two passes, k_occupancy's grid samples, k_label_points). */
typedef struct aos_gvd_evals {
    int32_t counted;                      /* 1: the last GVD call counted                                  */
    int32_t n_label_jobs;                 /* 4 per exploration row                                         */
    uint64_t edge_ends, boundary_points, filtered_nodes;   /* 2E, M, M'                                   */
    uint64_t ref_nearest, ref_pairs, ref_labels;
    uint64_t gpu_nearest, gpu_pairs, gpu_samples, gpu_labels;
} aos_gvd_evals;
int aos_gvd_set_count_evals(aos_ctx *ctx, int32_t on);
int aos_gvd_evals_get(aos_ctx *ctx, aos_gvd_evals *out);

/* ---------------------------------------------------------------------------------------------
 * Streaming ingest (BASELINE.json configs[4]). The handle keeps the global
 * map device-resident. Each aos_map_append call uploads only the new scan (packed to x, y, z float4
 * on the GPU), then processes the frame on the whole accumulated map. The outputs equal
 * aos_seedgen_process on the concatenation of the scans (the reference reprocesses its whole
 * global map on every callback, seed_gen:230-248). The map is dense iff every scan was.
 * ------------------------------------------------------------------------------------------- */
int aos_map_reset(aos_ctx *ctx, uint64_t reserve_points);
int aos_map_append(aos_ctx *ctx, const aos_cloud_view *scan, int want_host, aos_seedgen_out *out);

/* ---------------------------------------------------------------------------------------------
 * Multi-GPU tiled frame (BASELINE.json configs[3]: 8192^2 in 2 x 4 tiles).
 * One map is split into tiles_x x tiles_y tiles, one rank (process or thread) per tile, each with
 * its own handle on its own GPU. Ranks refresh the halos of their bit-packed grids by all-gathering
 * every tile's border strips, and max-reduce the thinning convergence flags. After thinning, the
 * skeleton and inflated tiles are all-gathered and the root rank finishes the frame on the whole
 * map. The root's outputs are byte-identical to aos_seedgen_process on the whole cloud. The
 * reference has no counterpart: its node processes the whole map on one core (seed_gen:230-248).
 * ------------------------------------------------------------------------------------------- */

/* Communicator supplied by the caller: RCCL over xGMI in production (torch.distributed 'nccl', or
 * ncclAllGather / ncclAllReduce on the same buffers). send_buf / recv_buf are device memory on
 * this rank's GPU, registered once; the library packs into send_buf and reads recv_buf. Both
 * callbacks are collective (every rank makes the same calls in the same order), are called with
 * the handle's stream idle, and must have completed when they return. Return 0 on success.
 * The library calls every non-NULL callback, including the optional ones at the end: fill the struct
 * from a zeroed one (aos_comm_init, or `aos_comm c = {0};`) so that a caller built against an older
 * header leaves the newer fields NULL. aos_rccl_comm's communicator is the library's own: with it, a
 * tiled frame enqueues its collectives on the handle's stream instead (no host wait around them). */
typedef struct aos_comm {
    void *user;
    int32_t rank, world;                 /* world = tiles_x * tiles_y; rank r = tile (r % tiles_x, r / tiles_x) */
    void *send_buf;                      /* >= buf_bytes                                       */
    void *recv_buf;                      /* >= world * buf_bytes                               */
    uint64_t buf_bytes;                  /* >= aos_tile_plan.exchange_bytes                    */
    /* recv_buf[r * bytes, (r + 1) * bytes) = send_buf[0, bytes) of rank r, for every rank r */
    int (*all_gather)(void *user, uint64_t bytes);
    /* element-wise max over ranks of n int32 values in host memory, in place */
    int (*all_reduce_max)(void *user, int32_t *values, int32_t n);
    /* Optional (NULL: the library routes through all_gather instead). Personalised exchange:
     * counts[s * world + d] = bytes rank s sends to rank d, the same world x world matrix on every rank.
     * send_buf holds this rank's blocks for d = 0, 1, ... back to back; on return recv_buf holds the blocks
     * addressed to this rank from s = 0, 1, ... back to back. The library keeps every row sum <= buf_bytes
     * and every column sum <= world * buf_bytes (larger exchanges are split into rounds). RCCL: grouped
     * ncclSend / ncclRecv; torch.distributed: all_to_all_single. Used by the distributed cluster stage to
     * send each long cluster's cells to the one rank that measures (and replays) it. */
    int (*all_to_all)(void *user, const uint64_t *counts);
} aos_comm;
void aos_comm_init(aos_comm *comm);   /* all fields zero / NULL */

/* RCCL communicator (one process per GPU, e.g. a torch.distributed launch): an aos_comm whose
 * exchange buffers live in HBM, all-gather = ncclAllGather over xGMI, max all-reduce =
 * ncclAllReduce(ncclMax) of the int32 flags. Rank 0 makes the id (NCCL_UNIQUE_ID_BYTES = 128 bytes)
 * and hands it to every rank out of band; aos_rccl_create is collective (every rank, at once).
 * RCCL (librccl.so.1) is loaded at run time by aos_rccl_unique_id / aos_rccl_create only. This
 * replaces the in-process group's peer copies when the ranks are separate processes. */
typedef struct aos_rccl aos_rccl;
int aos_rccl_unique_id(uint8_t *id128);
int aos_rccl_create(const uint8_t *id128, int32_t rank, int32_t world, int32_t device, uint64_t buf_bytes,
                    aos_rccl **out);
const aos_comm *aos_rccl_comm(aos_rccl *comm);   /* valid until aos_rccl_destroy */
void aos_rccl_destroy(aos_rccl *comm);

typedef struct aos_tile_plan {
    int32_t tiles_x, tiles_y, rank, tile_x, tile_y;
    int32_t halo_rows, halo_words;       /* halo depth (0 along an untiled dimension)          */
    int32_t row0, row1, word0, word1;    /* own rows and 64-cell words of the map              */
    int32_t win_row0, win_row1, win_word0, win_word1;   /* own tile + halo, clamped to the map */
    double points_box[4];                /* xmin, ymin, xmax, ymax: the points this rank needs  */
    uint64_t exchange_bytes;             /* minimum aos_comm.buf_bytes                         */
    aos_grid_info info;                  /* the whole map                                      */
} aos_tile_plan;

/* Host arithmetic only (no device needed): the tile of `rank` for this polygon (n_poly < 3: the
 * reference's default polygon, seed_gen:196-199) and these parameters. */
int aos_tile_plan_compute(const aos_params *p, const double *poly_xy, uint32_t n_poly, int32_t tiles_x,
                          int32_t tiles_y, int32_t rank, aos_tile_plan *out);
/* One tiled frame on this rank (uses the handle's polygon, see aos_set_polygon). `cloud` must hold
 * every point inside this rank's points_box; points outside it are ignored, so the whole cloud
 * also works. Root: the full aos_seedgen_out, and aos_gvd_from_seedgen works afterwards. Other
 * ranks: info, thin_iters, n_clipped (whole map) and timings only. */
int aos_tiled_seedgen_process(aos_ctx *ctx, const aos_comm *comm, int32_t tiles_x, int32_t tiles_y, int32_t root,
                              const aos_cloud_view *cloud, int want_host, aos_seedgen_out *out);

/* Streaming ingest on a tiled map (BASELINE.json configs[4] over several GPUs). Every rank keeps its own
 * device-resident map of the points inside its tile's points_box (aos_map_reset on the rank's handle
 * starts it) and its own incremental ROR tile store. Each call hands every rank the whole scan (as every
 * subscriber of /global_map receives it); the rank keeps its box's points on the GPU, then runs the tiled
 * frame on its map (halo all-gathers, global thinning convergence, root finishes the frame). The root's
 * outputs equal aos_map_append of the same scans on one GPU (n_input counts every appended point). The
 * box follows from the polygon and the tiling: changing either needs aos_map_reset and a new map. */
int aos_tiled_map_append(aos_ctx *ctx, const aos_comm *comm, int32_t tiles_x, int32_t tiles_y, int32_t root,
                         const aos_cloud_view *scan, int want_host, aos_seedgen_out *out);

/* Where this rank's last tiled frame (aos_tiled_seedgen_process / aos_tiled_map_append) spent its time
 * (no reference counterpart: the reference runs one map on one core). Host wall clock; a collective's
 * time includes the wait for the slowest rank. */
typedef struct aos_tiled_stats {
    float ms_frame;            /* the whole call on this rank                                        */
    float ms_comm_gather;      /* inside aos_comm.all_gather / all_to_all (halo strips, tables, the final
                                  grids, the long clusters' cells)                                    */
    float ms_comm_reduce;      /* inside aos_comm.all_reduce_max (thinning flags, counts, sizes)     */
    int32_t n_gather, n_reduce;
    uint64_t bytes_gather;     /* all-gather / all-to-all payload sent by this rank                  */
    float ms_ror, ms_thin;     /* device stage times (HIP events), as aos_seedgen_out                */
    float ms_cluster;          /* cluster stage, from the final all-gather (device events)           */
    float ms_seeds;            /* root: rows + seeds                                                 */
    float ms_cluster_local;    /* own-tile labelling and piece tables (host clock)                   */
    float ms_cluster_global;   /* union-find, long-cluster statistics and replays (incl. collectives) */
    float ms_replay;           /* of which: this rank's exact BFS replays                            */
    int32_t n_replayed;        /* clusters replayed on this rank                                     */
    int32_t ror_skipped;       /* streaming: 1 if no new point reached this rank's box (stage skipped) */
    int32_t is_root;
    uint64_t bytes_recv;       /* payload this rank received (halo strips, tables, the final tiles on the root, the
                                  owned clusters' cells, records)                                     */
} aos_tiled_stats;
int aos_tiled_stats_get(aos_ctx *ctx, aos_tiled_stats *out);

/* Border union-find of per-tile cluster pieces: the numbering step of the tiled frame's distributed
 * cluster stage (csrc/cluster_dist.hip; it replaces clusterOccupiedCells' whole-map raster scan + BFS
 * labelling, aos_seed_gen_node.cpp:970-1049, for clusters that cross tiles). Host code: no GPU needed.
 * A piece is a tile's 8-connected component of foreground cells, named by its first cell in raster
 * order (y * width + x, distinct over pieces); border_cell[i] (a piece's cell on its tile's edge)
 * belongs to the piece named border_root[i]. Two pieces are one cluster iff two of their border cells
 * are 8-adjacent. piece_cluster[i] = the cluster of piece i, clusters numbered in raster order of
 * their first cell (the reference's discovery order); *n_clusters = their number. */
int aos_cluster_union(int32_t width, int32_t height, int32_t n_pieces, const int32_t *piece_root, int32_t n_border,
                      const int32_t *border_cell, const int32_t *border_root, int32_t *piece_cluster,
                      int32_t *n_clusters);

/* One map over several GPUs from one process (SURVEY §8b's multi-GPU handle). The group owns one
 * handle per tile (devices[r] for rank r = tile (r % tiles_x, r / tiles_x); devices may repeat) and
 * drives the ranks with its own threads and an in-process aos_comm (peer copies over xGMI, host
 * max-reduction). clouds[r] must hold every point in rank r's points_box (aos_group_plan); the whole
 * cloud works too. The root's outputs equal aos_seedgen_process on the whole cloud; aos_group_rank
 * returns a rank's handle for aos_gvd_from_seedgen, markers and path planning on the root. */
typedef struct aos_group aos_group;
int aos_group_create(const aos_params *p, const int32_t *devices, int32_t tiles_x, int32_t tiles_y, aos_group **out);
void aos_group_destroy(aos_group *group);
int aos_group_set_polygon(aos_group *group, const double *xy, uint32_t n_points);
int aos_group_plan(aos_group *group, int32_t rank, aos_tile_plan *out);
aos_ctx *aos_group_rank(aos_group *group, int32_t rank);
int aos_group_process(aos_group *group, const aos_cloud_view *clouds, int32_t root, int want_host,
                      aos_seedgen_out *root_out);
/* The group's tiled streaming map (aos_tiled_map_append on every rank with the same scan). */
int aos_group_map_reset(aos_group *group, uint64_t reserve_points_per_rank);
int aos_group_map_append(aos_group *group, const aos_cloud_view *scan, int32_t root, int want_host,
                         aos_seedgen_out *root_out);

/* /gvd/markers content of the last GVD call (publishMarkers gvd:1012-1591) that is not already in
 * aos_gvd_out; the wrapper adds styles, ids and text. Needs aos_params.gvd_markers = 1.
 * The reference publishes the graph before the markers (gvd:310-313). Likewise a GVD call returns
 * once the graph is ready, and the cells (a second Subdiv2D) finish on a background thread: this
 * call waits for them, and raises their error if they failed. They overlap the next seed-gen
 * frame; the next GVD call and aos_destroy wait for them. The pointers stay valid until then. */
typedef struct aos_gvd_markers {
    int32_t n_seeds; const double *seeds_xy;   /* /gvd_voronoi_seeds: the merged seeds (gvd:1019-1041)        */
    int32_t n_rows;                            /* exploration rows (sorted rows_info pairs)                   */
    const double *row_label_xy;                /* TL, TR, BL, BR boundary points per row, (x, y) x 4          */
    const int32_t *row_label_valid;            /* 4 per row (gvd:1370-1450 draws the valid ones)             */
    int32_t n_cells;                           /* VoronoiDiagram::extractCellBoundaries voronoi_diagram.cpp:209-311 */
    const int32_t *cell_offsets;               /* n_cells + 1, into cell_xy points                            */
    const double *cell_xy;                     /* cell boundary, closed when its ends are > 1 cm apart        */
    const double *cell_center_xy;              /* seeds_[i]: the centre publishMarkers pairs with cell i      */
    const float *cell_rgba;                    /* /gvd_voronoi_cells i colour: HSV(i / n_cells, 0.7, 0.9), a 0.4 */
    float ms_cells;                            /* host time of the cells' Subdiv2D + facets (parallel thread) */
} aos_gvd_markers;
int aos_gvd_markers_get(aos_ctx *ctx, aos_gvd_markers *out);
/* The markers of the frame last returned by aos_gvd_wait (or the last synchronous GVD call), without
 * waiting for the jobs started since: a pipelined caller collects a frame's cells one step later,
 * while the next frames' jobs run (aos_gvd_markers_get would wait for the newest job). */
int aos_gvd_collected_markers_get(aos_ctx *ctx, aos_gvd_markers *out);

/* ---------------------------------------------------------------------------------------------
 * Path planning over the GvdGraph (aos_path_gen_node): graphCallback
 * (path_gen:418-579) = cluster waypoint mapping (:704-765) + waypoint sequence (:588-702) + target
 * restore (:496-560), then planAndPublishPath (:976-1567): weighted A* (:800-896) from the 5 nodes
 * nearest the start (:914-932), the straight 0.2 m segments, orientations, and
 * trimPathNearOccupiedRegions (:1570-1630) on the skeleton. The node's state goes in as
 * aos_path_query; the published /path poses, the status and the indices come out.
 * ------------------------------------------------------------------------------------------- */
typedef struct aos_path_graph {          /* msg/GvdGraph.msg */
    int32_t num_nodes; const double *nodes_xy;
    const int32_t *node_labels, *node_cluster_indices, *node_label_counts;
    int32_t n_label_entries; const int32_t *node_label_clusters, *node_label_types;
    int32_t num_edges; const int32_t *edges; const float *edge_lengths;
} aos_path_graph;

typedef struct aos_path_query {
    int32_t initial_waypoint_reached;    /* 0: straight line (0, 0) -> initial waypoint (:983-1031) */
    double initial_waypoint_xy[2];       /* (8, 0) in the reference (:81-83)                      */
    int32_t target_waypoint_index;       /* current_target_waypoint_index_ before this graph (-1)  */
    int32_t have_saved_target;           /* that index was valid: its position follows            */
    double saved_target_xy[2];
    int32_t previous_waypoint_index;     /* previous_waypoint_index_ (-1: start at the initial waypoint) */
    int32_t use_current_position;        /* service call with a received position (:1062-1066)    */
    double current_xy[2];
    int32_t exploration_completed;       /* the origin (0, 0) ends the sequence (node -1, :1096-1280);
                                            modelled as this graph's sequence plus the origin      */
} aos_path_query;

typedef struct aos_path_out {
    int32_t status;                      /* publishPlanningStatus: 1 "Success", 0 "Failed"          */
    int32_t target_waypoint_index;       /* after the restore                                       */
    int32_t cluster_index;               /* calculateClusterIndex (:1633-1652)                      */
    int32_t n_clusters;                  /* cluster_waypoint_nodes_, ascending cluster id           */
    const int32_t *cluster_ids, *cluster_nodes;   /* 4 per cluster: TL, TR, BL, BR node (-1: none) */
    int32_t n_waypoints; const double *waypoints_xy; const int32_t *waypoint_nodes;
    int32_t n_node_path; const int32_t *node_path;   /* the chosen A* node path                   */
    int32_t n_poses; const double *poses;            /* x, y, qz, qw per /path pose (z = 0)       */
    int32_t trimmed_from;                /* pose count before the trim, or -1                       */
    float ms_plan;
} aos_path_out;

/* graph: NULL = this handle's last GVD graph. skeleton: /skeletonized_occupancy_grid bytes, host
 * memory (skeleton_on_device = 0) or device memory on the handle's GPU (1), with `info`; NULL = the
 * skeleton that graph was built on (AOS_E_STATE if a later seed-gen frame replaced it). On
 * "Failed" the outputs hold no poses: the node republishes its last path. */
int aos_path_plan(aos_ctx *ctx, const aos_path_graph *graph, const int8_t *skeleton, int skeleton_on_device,
                  const aos_grid_info *info, const aos_path_query *query, aos_path_out *out);

/* Diagnostics: copy an internal device grid of the last frame to host as int8 {0,100}.
 * which: "raster", "inflated", "opened", "skeleton_frameless". */
int aos_debug_grid(aos_ctx *ctx, const char *which, int8_t *dst, uint64_t capacity);
/* Diagnostics: the library's single-pass exclusive scan (its counting sorts' and compactions' primitive) on the
 * handle's stream: d_out[i] = d_in[0] + ... + d_in[i - 1] for i in [0, n] (n + 1 outputs), device int32 arrays on
 * the handle's GPU; zero_in: d_in is left zero. Returns once done. */
int aos_debug_scan(aos_ctx *ctx, int32_t *d_in, int32_t *d_out, int32_t n, int zero_in);
/* Stream of the handle (hipStream_t as void*) for callers that time with their own events. */
void *aos_stream(aos_ctx *ctx);
/* Test hooks (fault injection for the tiled path's error tests; process-wide, not for production use):
 * ror_stuck_rank >= 0: that tiled rank reports a stuck look-back wait in its ROR column scan (every rank
 * must then fail the frame together); a2a_round_bytes > 0: the distributed cluster stage's personalised
 * exchange moves at most that many bytes per rank pair and round. (-1, 0) turns both off (the default). */
void aos_debug_faults(int32_t ror_stuck_rank, uint64_t a2a_round_bytes);
/* Test hook (process-wide): a seed-gen frame replays its clusters without the order-free certificate on the GPU
 * (one wave per cluster) once it has at least gpu_min_clusters of them, else on host threads. -1: the default
 * (never: the host walk is faster); 0: always on the GPU (where a cluster's box fits the wave's LDS
 * bitmap).
 * ring_cap in [1, 63]: the GPU walk gives a cluster up to the host once more than that many cells are queued
 * (default 0: 64), so tests reach the fallback. replay_all != 0: every cluster is replayed, also those with the
 * order-free certificate (whose records the replay must reproduce). (-1, 0, 0): the defaults. */
void aos_debug_replay(int32_t gpu_min_clusters, int32_t ring_cap, int32_t replay_all);
/* Diagnostics: the last single-GPU seed-gen frame's exact BFS replays: out[0] = all of them (n_bfs_replayed),
 * out[1] = on the GPU, out[2] = on host threads over the skeleton bits, out[3] = on host threads from the clusters'
 * cells. */
int aos_replay_counts(aos_ctx *ctx, int32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif /* AOS_GPU_H */
