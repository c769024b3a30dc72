// Cluster / tree-row / seed stage and GVD stage state. Not part of the ABI.
#pragma once
#include <climits>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "aos_internal.h"
#include "dev_prims.h"
#include "host_pool.h"
#include "subdiv2d.h"

namespace aos {

// Per-cluster result of the cluster-statistics kernel (a8-a10).
struct ClusterRec {
    long long sx, sy;        // exact integer sums of cell coordinates
    int n;                   // cells
    int maxd2;               // max pairwise squared distance (grid units)
    float cx, cy;            // cluster.center_x / center_y (grid units, float)
    float length;            // cluster.length (m)
    int flags;               // bit0: row (length >= min && centre in polygon); bit1: needs BFS order
    double2 center, start, end;  // world (double from float)
    int bx0, by0, bx1, by1;  // bounding box (cells, inclusive)
    int first;               // first raster cell (y * W + x): where clusterOccupiedCells' BFS starts
    int pad_;
};

// ------------------------------------------------------------------ greedy first-come de-duplication
// Keeps candidate i iff no earlier KEPT candidate conflicts with it (the reference's
// "if no existing within d: push_back" loops) = the lexicographically-first maximal independent
// set of the conflict graph; decided on the GPU by one fused kernel over a hashed cell index (greedy.hip).
enum ConflictMode {
    kConflictLess = 0,     // sqrt(dx*dx + dy*dy) <  thr  (seed dedups, seed_gen:2076-2085 ...)
    kConflictLessEq = 1,   // sqrt(dx*dx + dy*dy) <= thr  (GVD seed merge, gvd:107-115)
    kConflictKeyOrSq = 2,  // same (int)(x*100),(int)(y*100) key, or dx*dx + dy*dy < thr (extractBoundaryPoints)
};
// Waits for the work queued so far on a stream through an event of the caller's own: a GVD lane's host
// thread waits for its own work only, not for other lanes' work queued on the shared GVD stream.
struct SyncEvent {
    hipEvent_t e = nullptr;
    SyncEvent() = default;
    SyncEvent(const SyncEvent &) = delete;
    SyncEvent &operator=(const SyncEvent &) = delete;
    ~SyncEvent() { if (e) (void)hipEventDestroy(e); }
    void sync(hipStream_t s) {
        if (!e) AOS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        AOS_HIP(hipEventRecord(e, s));
        AOS_HIP(hipEventSynchronize(e));
    }
};

struct DedupScratch {
    CellScratch cells;
    CellIdx ci{};          // the cell index of the last de-duplication (the GVD merge finds members through it)
    LookBackScratch lb;
    DevBuf state, misc;
    unsigned epoch = 0;    // of the state words
    SyncEvent sev;
};
// Enqueues one de-duplication (no host synchronisation): cand / ok (nullable: all ok) device arrays of n
// entries, h a hash with cells >= the conflict radius and a bounded bucket count (make_hash_n); the kept
// points in order -> out, their indices -> kept_index (nullable), the kept count -> *d_count (device).
// owner (nullable): per candidate, the smallest kept candidate it conflicts with (itself if kept, INT_MAX
// if not ok): the members of each merged seed (gvd:93-125). pos_of (nullable): per candidate, its position
// in out or -1 (the GVD graph finds boundary points through the de-duplication's own index, S.ci).
void greedy_dedup_async(DedupScratch &S, const double2 *cand, const int *ok, int n, int mode, double thr, const HashG &h,
                        double2 *out, int *kept_index, int *owner, int *d_count, hipStream_t s, int *pos_of = nullptr);
// The same, then waits and returns the kept count (h_scalar: 2 pinned ints).
int greedy_dedup(DedupScratch &S, const double2 *cand, const int *ok, int n, int mode, double thr, const HashG &h,
                 double2 *out, int *kept_index_out, hipStream_t s, int *h_scalar);
// Problems of at most kSmallMax candidates (up to 2 per launch), one workgroup each, the index and the
// rounds in LDS: one launch. h: small_hash (at most 2048 buckets).
constexpr int kSmallMax = 4096;
struct SmallProb { const double2 *p; const int *ok; int n; HashG h; double2 *out; int *count; };
struct SmallDedup { SmallProb prob[2]; int mode; double thr; int *err; };
void greedy_dedup_small(DedupScratch &S, SmallDedup A, int nprob, hipStream_t s);
HashG small_hash(double minx, double maxx, double miny, double maxy, double cell);
// The device error word of S's launches (0 = fine) and the check of its value once read back.
int *dedup_err(DedupScratch &S, hipStream_t s);
void dedup_check(DedupScratch &S, int err_word);

struct ClusterSeedState {
    DedupScratch dedup;
    DevBuf fg_bits, word_cnt, word_off, fg_list, parent, root_flag, root_rank, cl_count, cl_off, cl_cursor, cl_cells;
    DevBuf ccl_edges;   // k_ccl_local's cross-chunk links: count, pad, then (i, j) pairs
    DevBuf rec, row_idx, poly, cur_tab;
    DevBuf cand_xy, cand_ok, cand_state, hash_count, hash_start, hash_slot, hash_sorted, seed_out, misc, scan_tmp;
    LookBackScratch lb;           // the stage's single-pass scans
    bool cl_count_dirty = true;   // cl_count (cluster sizes) not known to be zero
    PinnedBuf h_recbuf, h_up_poly, h_up_rows;   // cluster records read back; host -> device staging
    std::vector<double> poly_up;                 // the polygon in `poly` (uploaded again only when it changes)
    PinnedBuf h_seeds;   // the frame's seeds (one DMA into pinned memory: no staging copy, no page faults)
    PinnedBuf h_cells;   // the replayed clusters' cells (one DMA; round 3's zeroed pageable vector cost ~1.5 ms at C3)
    PinnedBuf h_misc;
    int n_fg = 0, n_clusters = 0, n_rows = 0, n_cur_tab = 0;
    int n_replay_from_bits = 0;   // the last frame's exact replays that walked the host skeleton bits
    int n_replay_gpu = 0;         // ... that ran on the GPU (replay_gpu.hip)
    int n_replay_cells = 0;       // ... that replayed from the clusters' cells on the host
    DevBuf replay_ids, replay_order;   // the GPU replays' cluster list and their BFS orders
    PinnedBuf h_replay;                // the list's upload staging and the replays' status words
    double cur_tab_amax = -1.0;
    std::vector<ClusterRec> h_rec;
    HostPool replay_pool;   // the BFS replays' host threads (replay_clusters)
};

// a8-a10 computed elsewhere (the tiled frame's distributed cluster stage, cluster_dist.hip): every
// cluster's record in cluster order, exactly as the whole-map stage makes it.
struct PreClusters {
    std::vector<ClusterRec> rec;
    int n_fg = 0, n_bfs = 0;
};

// Everything the seed stage needs from the frame.
struct SeedStageIn {
    const uint64_t *skel_bits;   // frameless skeleton
    const FrameGeom *g;
    const Poly *poly;
    double cluster_min_length;
    const PreClusters *pre = nullptr;   // set: skip a8-a10 (labelling, statistics, replays)
    // called once the foreground count's read-back is queued (at the start with pre): the published grids'
    // D2H goes there, after k_fg, so the copy shares neither k_fg's CUs nor PCIe with that read-back
    std::function<void()> after_fg;
    // (nullable) the frameless skeleton's bits in host memory, WW words per row, once they are there (waits for
    // their read-back; returns null when they are not sent): the exact BFS replays walk them (cluster_host.cpp)
    std::function<const uint64_t *()> host_skel_bits;
};

struct GridC;
// k_cluster_stats over clusters given as runs of raster-ordered cells (off[n_clusters + 1], cells)
void launch_cluster_stats(const int *off, const int *cells, int n_clusters, const GridC &g, const double *poly, int np,
                          float min_length, ClusterRec *rec, hipStream_t s,
                          ClusterRec *hrec = nullptr);   // hrec: pinned host copy of the records, same launch
// exact FIFO-BFS replays (host, parallel over clusters; cluster_host.cpp); cells of a job in any order (the BFS
// starts from the smallest), n of them
// cells == nullptr: from bits (the frameless skeleton in host memory, WW words per row) over the record's box from its
// first cell; a job whose bits do not give its cluster (the polygon cuts the box) leaves its record unchanged and its
// index goes to *failed (the caller replays it from its cells)
struct ReplayJob { int c; const int *cells; int n; const uint64_t *bits = nullptr; };
void replay_clusters(const std::vector<ReplayJob> &jobs, const GridC &g, const double *poly, int np, float min_len,
                     ClusterRec *rec, HostPool *pool = nullptr, std::vector<int> *failed = nullptr);
// The same replays on the GPU (replay_gpu.hip), one wave per cluster, for frames with many of them: d_ids (device)
// lists n_jobs clusters whose bordered box bitmap takes at most lds_words 32-bit words (replay_bitmap_words; -1: not
// on the GPU), walked over the foreground bits fg (g.WW words per row); order: nf ints of scratch (cluster c at
// off[c]). A replayed cluster's record is updated in rec and hrec (pinned) and h_status[j] = 0; a cluster the GPU
// leaves (frontier wider than 64 cells, records that disagree with the grid) keeps its records and h_status[j] = 1.
constexpr size_t kReplayLdsBytes = 64 * 1024;
// Not by default: a wave walks ~0.5 us per cell (C3's 215 row replays: 5.2 ms on the GPU, 1.4 ms on 16 host threads,
// profiles/r06/r06g_*), so the host threads replay every frame's clusters unless a test asks (aos_debug_replay).
constexpr int kGpuReplayMin = INT_MAX;
long long replay_bitmap_words(const ClusterRec &r);
void launch_gpu_replays(const int *d_ids, int n_jobs, int lds_words, const int *off, const uint64_t *fg, ClusterRec *rec,
                        ClusterRec *hrec, int *h_status, int *order, const GridC &g, const double *poly, int np,
                        float min_length, hipStream_t s, long long *h_prof = nullptr);
void print_replay_prof(const long long *prof, int n_jobs);   // (AOS_REPLAY_PROF=1: h_prof's phase counters)
// aos_debug_replay (tests): the flagged-cluster count from which a frame replays on the GPU (-1: kGpuReplayMin), and
// a smaller queue ring for the GPU walk (0: 64), so that wide frontiers reach the host fallback
extern std::atomic<int> g_debug_replay_min, g_debug_replay_ring;
extern std::atomic<bool> g_debug_replay_all;   // ... and every cluster replayed, certified or not

// a tree row as the seed kernels take it: start / end (world), k base seeds, first virtual-seed slot
struct RowDev { double sx, sy, ex, ey; int k; int slot0; };

struct SeedStageOut {
    int n_clusters_all = 0;
    int n_bfs = 0;
    std::vector<double> row_center, row_start, row_end, row_length;  // all_tree_rows order
    std::vector<double> rows_info, cluster_info;
    // the concatenated seeds (virtual, ray, endpoint): device copy, and the host copy in the stage's pinned
    // buffer (valid until the stage runs again)
    const double *d_voronoi = nullptr, *h_voronoi = nullptr;
    int n_voronoi = 0, n_virtual = 0, n_ray = 0, n_endpoint = 0;
};

void run_cluster_seed_stage(ClusterSeedState &S, const SeedStageIn &in, SeedStageOut &out, hipStream_t stream,
                            hipEvent_t ev_mid, const hipEvent_t *ev_split = nullptr);
// the row arrays, the rows' seed slots and the sorted cluster_info / rows_info (host; cluster_host.cpp)
void assemble_rows(const std::vector<ClusterRec> &rec, SeedStageOut &out, std::vector<RowDev> &rows);

// ------------------------------------------------------------------ distributed a8-a10 (cluster_dist.hip)
// The union-find labelling of a foreground (bits, g.WW words x g.H rows; off: the exclusive scan of the words'
// popcounts, off[Cw] = nf, made by the producer with B.lb) into the raster-ordered list of its cells (local
// raster indices), parent[i] = list index of the first cell of i's component and rank[] = the exclusive scan of
// the roots (rank[nf] = components, left on the device): the whole-map stage's kernels (cluster_seed.hip).
// Returns nf (one host wait); *err = the scans' error word.
struct GridC;
struct CclScratch {
    DevBuf off, list, parent, isroot, rank, edges;
    LookBackScratch lb;
    int *list_p = nullptr, *parent_p = nullptr, *rank_p = nullptr;
};
int ccl_label(CclScratch &B, const uint64_t *fg, const int *off, const GridC &g, hipStream_t s, int *h_pinned2, int *err);

struct ClusterDistState {
    CclScratch ccl;
    DevBuf poly, fg, cnt, pieces, pid, prank, border, counts, blob, poff, sendbuf, landing, segs, cells, coff, rec;
    PinnedBuf h, h_poly, h_poff, h_segs, h_coff, h_rec, h_cells, h_out, h_tab, h_all;   // (one per upload / read-back)
    PinnedBuf h_recv;   // gather_bytes: a chunk's receive buffer in host memory (one read-back per chunk)
};
struct ClusterDistStats {
    int n_pieces = 0, n_border = 0, n_long = 0, long_cells = 0, n_replayed_here = 0;
    float ms_local = 0, ms_global = 0;   // own labelling / tables, union-find, long-cluster statistics and replays
    float ms_replay = 0;                 // (of ms_global) this rank's exact BFS replays
};
// The tiled frame's cluster stage on one rank (collective over the tile ranks): win = the rank's
// window skeleton (own cells exact). The root receives every cluster's record in pre.
int cluster_union(int W, int H, int n_pieces, const int *piece_root, int n_border, const int *bcell, const int *broot,
                  int *piece_cluster);
void cluster_dist(ClusterDistState &D, FrameComm &fc, const TilePlan &t, const FrameGeom &g, const Poly &poly,
                  float min_len, const uint64_t *win, int root, hipStream_t s, PreClusters &pre, ClusterDistStats &st);

// ------------------------------------------------------------------ GVD
// publishMarkers' Voronoi cells, computed by a worker thread next to the main Subdiv2D replay. It
// lives in its own cache-line-aligned heap object: the two replays write their state on every step,
// and sharing lines with the main replay's fields slowed both down by ~40 % on the EPYC host.
// Device buffers of the facet builder (calcVoronoi + getVoronoiFacetList on the GPU, gvd.hip).
// raw = the exported Subdiv2D state in one buffer (quad-edges | points | firstEdge | type), one H2D copy
struct FacetBufs { DevBuf raw, face, cnt, off, scan_tmp; LookBackScratch lb; PinnedBuf h_stage; int *qe = nullptr, *vf = nullptr, *vt = nullptr; };

struct alignas(128) CellsWork {
    Subdiv2D sd;                               // extractCellBoundaries' Subdiv2D
    std::vector<double> seeds;                 // VoronoiDiagram::seeds_ (finite merged seeds)
    std::vector<double> cell_xy, cell_center;
    std::vector<int32_t> cell_off;
    std::vector<float> cell_rgba;
    float ms = 0;
    // its facets are built on the GPU too, on the worker's own stream
    int device = 0;
    hipStream_t stream = nullptr;
    FacetBufs fb;
    DevBuf edges;
    PinnedBuf h;
    // One persistent worker per handle: it sleeps between frames and keeps its core (and the
    // replay's ~6 MB of quad-edges in that core's caches); a thread per frame landed on a cold core.
    std::thread worker;
    std::mutex mu;
    std::condition_variable cv;
    bool busy = false, quit = false;
    int rect_mode = 0;
    std::exception_ptr err;     // the last job's error (markers_wait raises or discards it)
    CellsWork() = default;
    CellsWork(const CellsWork &) = delete;
    CellsWork &operator=(const CellsWork &) = delete;
    ~CellsWork() {
        if (worker.joinable()) {
            { std::lock_guard<std::mutex> l(mu); quit = true; }
            cv.notify_all();
            worker.join();
        }
        if (stream) (void)hipStreamDestroy(stream);
    }
};

struct GvdState {
    DedupScratch dedup;
    DevBuf seeds, merge_state, hash_count, hash_start, hash_slot, hash_sorted, scan_tmp, misc;
    DevBuf edges, bpts, near_idx, cand, cand_ok, skel, grid_bytes_ext;
    PinnedBuf h_misc;
    void *scratch = nullptr;   // GvdScratch (gvd.hip), freed by free_gvd_scratch
    PinnedBuf h_seeds;   // seeds in / merged seeds out (g1)
    PinnedBuf h_out;     // the GvdGraph arrays, gathered into it by one kernel (k_gather_words)
    PinnedBuf h_evals;   // the graph searches' work counters (aos_params.gvd_count_evals)
    aos_gvd_evals evals{};
    SyncEvent sev;       // host waits of this state's GVD calls (the stream may be shared by several lanes)
    Subdiv2D subdiv;   // host insert replay; kept across frames to reuse its allocations
    // host outputs
    std::vector<double> nodes_xy;
    std::vector<int32_t> labels, cluster_idx, label_counts, label_clusters, label_types, edges_out;
    std::vector<float> lengths, clearances;
    int n_merged = 0, n_vor_edges = 0, n_bpts = 0;
    int pairs_cap = 0;   // capacity of the g6 pair lists (from the last frame's pair count)
    float ms_merge = 0, ms_delaunay = 0, ms_graph = 0, ms_total = 0;
    // markers (aos_gvd_markers)
    bool have_markers = false;
    bool graph_ok = false;     // the last GVD call produced a graph (markers can be computed on demand)
    int rect_mode = 0;         // its Subdiv2D rectangle mode
    std::vector<double> merged_xy, row_label_xy;
    std::vector<int32_t> row_label_valid;
    std::unique_ptr<CellsWork> cells;   // the worker thread's own heap object (no false sharing)
};

struct GvdStageIn {
    const double *seeds_host;  int n_seeds;     // /voronoi_seeds (x, y)
    const double *rows_info;   int n_rows_poses;
    aos_grid_info info;
    const int8_t *d_skeleton;                   // framed skeleton bytes on device
    // called once the merged seeds are on the host, when the GPU prefix is done and the host
    // Subdiv2D replay starts (the pipelined caller lets the next seed-gen frame go from here)
    void (*on_host_phase)(void *) = nullptr;
    void *hook_arg = nullptr;
};
bool run_gvd_stage(GvdState &G, const aos_params &P, const GvdStageIn &in, hipStream_t stream, hipEvent_t *ev);
void free_gvd_scratch(GvdState &G);
// Joins the markers' cells job of the last GVD call; rethrow: raise its error (else discard it).
void markers_wait(GvdState &G, bool rethrow);
// aos_gvd_markers_get on a frame whose GVD ran without markers: compute them now (and wait)
void markers_on_demand(GvdState &G);

}  // namespace aos
