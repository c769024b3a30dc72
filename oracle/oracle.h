/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A single-threaded CPU restatement of the AOS seed-gen + GVD hot path
 * (reference: /root/reference/src/aos_seed_gen_node.cpp, src/aos_gvd_node.cpp,
 * src/utils/voronoi_diagram.cpp) plus the third-party semantics it depends on
 * (PCL RadiusOutlierRemoval / PassThrough, OpenCV morphologyEx + getStructuringElement,
 * opencv_contrib ximgproc::thinning(ZHANGSUEN), OpenCV Subdiv2D), restated in oracle/NOTES.md.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline. The product (libaos_gpu.so) never links or calls it.
 *
 * Parity status: the reference publishes no tests, fixtures or golden vectors for this path
 *  and cannot be built or imported here (ROS 2 / PCL / OpenCV absent), so
 * this oracle is pinned only by hand-derived known-answer tests and independent scipy
 * cross-checks (tests/test_oracle_*.py): PARITY UNPINNED against the reference binary.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_params {
    float clip_minz, clip_maxz, clip_minx, clip_maxx, clip_miny, clip_maxy;  /* seed_gen:69-74 */
    float grid_resolution;                                                   /* seed_gen:75    */
    float inflation_radius;                                                  /* seed_gen:76    */
    double cluster_min_length;                                               /* seed_gen:83    */
    double ror_radius;                /* seed_gen:238 (hard-coded 0.2)  */
    int32_t ror_min_neighbors;        /* seed_gen:239 (hard-coded 2)    */
    int32_t subdiv_rect_mode;         /* 0: Subdiv2D(Rect2f); 1: Rect2f -> Rect (cvRound) conversion */
    int32_t faithful_dead_work;       /* 1: also run work whose result is never read (CPU-cost parity) */
    int32_t markers;                  /* 1: also publishMarkers' extractCellBoundaries (gvd:1098-1194) */
} orc_params;

void orc_default_params(orc_params *p);

/* ---------- seed gen (aos_seed_gen_node) ---------- */
typedef struct orc_seedgen_out {
    double origin_x, origin_y;
    float resolution;
    uint32_t width, height;
    int32_t thin_iters;
    uint64_t n_input, n_ror_kept, n_clipped;
    const int8_t *raster;            /* generateOccupancyGrid          */
    const int8_t *inflated;          /* applyInflation                 */
    const int8_t *occupancy;         /* + markBoundariesAsOccupied -> /occupancy_grid */
    const uint8_t *opened;           /* morphologyEx OPEN result, 0/1  */
    const int8_t *skeleton;          /* skeletonizeOccupancyGrid (frameless) */
    const int8_t *skeleton_framed;   /* markPolygonBoundaryAsOccupied -> /skeletonized_occupancy_grid */
    const uint8_t *ror_keep;         /* per input point                */
    int32_t n_clusters;              /* all clusters (before length filter), discovery order */
    const int32_t *cluster_offsets;  /* n_clusters + 1                 */
    const int32_t *cluster_cells;    /* (x, y) pairs in BFS order      */
    const float *cluster_center;     /* (cx, cy) in grid units         */
    const float *cluster_length;
    int32_t n_rows;                  /* all_tree_rows (convertClustersToTreeRows order) */
    const double *row_center, *row_start, *row_end, *row_length;  /* 2,2,2,1 per row */
    int32_t n_virtual, n_ray, n_endpoint, n_voronoi;
    const double *virtual_xy, *ray_xy, *endpoint_xy, *voronoi_xy;
    const double *rows_info_xy;      /* sorted: (start.x, start.y, end.x, end.y) per row */
    int32_t n_cluster_info;
    const double *cluster_info_xy;
} orc_seedgen_out;

/* cloud: PointCloud2 data bytes (x/y/z float32 at the given offsets). poly: (x, y) doubles, n>=3
 * replaces the hard-coded default polygon (seed_gen:196-199) like explorationAreaCallback. */
void *orc_seedgen_run(const orc_params *p, const uint8_t *cloud, uint64_t n_points, uint32_t point_step,
                      uint32_t off_x, uint32_t off_y, uint32_t off_z, int32_t is_dense,
                      const double *poly_xy, int32_t n_poly, orc_seedgen_out *out);

/* ---------- GVD (aos_gvd_node) ---------- */
typedef struct orc_gvd_in {
    const double *seeds_xy; int32_t n_seeds;          /* /voronoi_seeds poses          */
    const double *rows_info_xy; int32_t n_rows_poses;  /* /exploration_tree_rows_info   */
    double origin_x, origin_y; float resolution; uint32_t width, height;
    const int8_t *skeleton;                            /* /skeletonized_occupancy_grid */
} orc_gvd_in;

typedef struct orc_gvd_out {
    int32_t published;
    double resolution, origin_x, origin_y;
    int32_t n_merged; const double *merged_xy;
    int32_t n_vor_edges; const double *vor_edges;      /* 4 doubles per edge */
    int32_t n_boundary_raw; const double *boundary_raw;
    int32_t n_vertices_dead;                           /* VoronoiDiagram vertex dedup (never read) */
    int32_t num_nodes; const double *nodes_xy;
    const int32_t *node_labels, *node_cluster_indices, *node_label_counts;
    int32_t n_label_entries; const int32_t *node_label_clusters, *node_label_types;
    int32_t num_edges; const int32_t *edges; const float *edge_lengths, *edge_clearances;
    int32_t n_label_rows; const double *row_label_pts; const int32_t *row_label_valid;
    /* markers (p->markers): extractCellBoundaries + the /gvd_voronoi_cells colours and centres */
    int32_t n_cells; const int32_t *cell_offsets; const double *cell_xy, *cell_center_xy; const float *cell_rgba;
} orc_gvd_out;

void *orc_gvd_run(const orc_params *p, const orc_gvd_in *in, orc_gvd_out *out);

/* ---------- path planning over the GvdGraph (aos_path_gen_node) ---------- */
typedef struct orc_path_graph {      /* msg/GvdGraph.msg */
    int32_t num_nodes; const double *nodes_xy;
    const int32_t *node_labels, *node_cluster_indices, *node_label_counts;
    int32_t n_label_entries; const int32_t *node_label_clusters, *node_label_types;
    int32_t num_edges; const int32_t *edges; const float *edge_lengths;
} orc_path_graph;

typedef struct orc_path_query {      /* the node's state when the graph arrives */
    int32_t initial_waypoint_reached; double initial_waypoint_xy[2];
    int32_t target_waypoint_index;    /* current_target_waypoint_index_ before the graph (-1: none) */
    int32_t have_saved_target; double saved_target_xy[2];   /* its position in the old sequence */
    int32_t previous_waypoint_index;
    int32_t use_current_position; double current_xy[2];
    int32_t exploration_completed;    /* with the origin (0, 0) as the last waypoint (node -1) */
} orc_path_query;

typedef struct orc_path_out {
    int32_t status;                   /* publishPlanningStatus: 1 Success, 0 Failed */
    int32_t target_waypoint_index, cluster_index;
    int32_t n_clusters; const int32_t *cluster_ids, *cluster_nodes;   /* 4 per cluster: TL TR BL BR */
    int32_t n_waypoints; const double *waypoints_xy; const int32_t *waypoint_nodes;
    int32_t n_node_path; const int32_t *node_path;   /* the chosen A* path */
    int32_t n_poses; const double *poses;            /* x, y, qz, qw per pose (published /path) */
    int32_t trimmed_from;             /* poses before trimPathNearOccupiedRegions, or -1 */
} orc_path_out;

void *orc_path_plan(const orc_path_graph *g, const int8_t *skeleton, double origin_x, double origin_y,
                    float resolution, uint32_t width, uint32_t height, const orc_path_query *q, orc_path_out *out);
void orc_free_path(void *handle);

void orc_free_seedgen(void *handle);
void orc_free_gvd(void *handle);
void orc_free_facets(void *handle);
void orc_free_subdiv_state(void *handle);

/* ---------- single-stage entry points (KATs / cross-checks) ---------- */
void orc_ror(const float *xyz, uint64_t n, int32_t is_dense, double radius, int32_t min_pts, uint8_t *keep);
void orc_inflate(const int8_t *in, uint32_t w, uint32_t h, int32_t cells, int8_t *out);
void orc_open_cross(const uint8_t *in01, uint32_t w, uint32_t h, uint8_t *out01);
int32_t orc_thin(const uint8_t *in01, uint32_t w, uint32_t h, uint8_t *out01);
/* Subdiv2D facets: returns handle; facets flattened (x,y floats), offsets n_facets+1. */
/* Test hook: raw Subdiv2D state after inserting xy (float pairs) into Subdiv2D(rect = x, y, w, h). */
void *orc_subdiv_state(const float *xy, int32_t n, const float *rect, int32_t rect_mode, int32_t *n_q, const int32_t **qe,
                       int32_t *n_v, const int32_t **vfirst, const int32_t **vtype, const float **vxy, const int32_t **inserted,
                       int32_t *n_facets, const int32_t **offsets, const float **pts);
void *orc_subdiv_facets(const double *seeds_xy, int32_t n, double min_x, double max_x, double min_y,
                        double max_y, int32_t rect_mode, int32_t *n_facets, const int32_t **offsets,
                        const float **pts, const float **centers);

#ifdef __cplusplus
}
#endif
