// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h): extern "C" entry points for ctypes.
#include <cstring>
#include <new>

#include "oracle_internal.h"

using namespace orc;

// (x, y) doubles of a V2 vector; null when empty (taking ->x of an empty vector's data() is UB)
template <class V> static const double *xy_of(const V &v) { return v.empty() ? nullptr : &v[0].x; }

extern "C" {

void orc_default_params(orc_params *p) {
    // seed_gen:69-83 defaults overridden by config/aos_planner_params.yaml:55-89 (seed gen node)
    p->clip_minz = -0.4f; p->clip_maxz = 0.5f;
    p->clip_minx = -5.0f; p->clip_maxx = 72.0f; p->clip_miny = -10.0f; p->clip_maxy = 20.0f;
    p->grid_resolution = 0.05f;
    p->inflation_radius = 0.8f;
    p->cluster_min_length = 2.0;
    p->ror_radius = 0.2;
    p->ror_min_neighbors = 2;
    p->subdiv_rect_mode = 0;
    p->faithful_dead_work = 0;
    p->markers = 0;
}

void *orc_seedgen_run(const orc_params *p, const uint8_t *cloud, uint64_t n, uint32_t point_step, uint32_t ox,
                      uint32_t oy, uint32_t oz, int32_t is_dense, const double *poly_xy, int32_t n_poly,
                      orc_seedgen_out *out) {
    auto *R = new (std::nothrow) SeedGenResult();
    if (!R) return nullptr;
    // pcl::fromROSMsg: copy x, y, z by field offset (seed_gen:232-233)
    std::vector<float> xyz(3 * n);
    for (uint64_t i = 0; i < n; ++i) {
        std::memcpy(&xyz[3 * i + 0], cloud + i * point_step + ox, 4);
        std::memcpy(&xyz[3 * i + 1], cloud + i * point_step + oy, 4);
        std::memcpy(&xyz[3 * i + 2], cloud + i * point_step + oz, 4);
    }
    Poly poly;
    if (poly_xy && n_poly >= 3) {
        for (int i = 0; i < n_poly; ++i) poly.push_back({poly_xy[2 * i], poly_xy[2 * i + 1]});
    } else {  // hard-coded default polygon seed_gen:196-199
        poly = {{-1.972916603088379, 7.9420671463012695}, {-2.0726776123046875, 0.022441387176513672},
                {70.22465515136719, 2.102720260620117}, {69.48777770996094, 9.786612510681152}};
    }
    seedgen(*p, xyz.data(), n, is_dense != 0, poly, *R);

    std::memset(out, 0, sizeof(*out));
    out->origin_x = R->info.origin_x; out->origin_y = R->info.origin_y;
    out->resolution = R->info.resolution; out->width = R->info.width; out->height = R->info.height;
    out->thin_iters = R->thin_iters;
    out->n_input = R->n_input; out->n_ror_kept = R->n_ror_kept; out->n_clipped = R->n_clipped;
    out->raster = R->raster.data(); out->inflated = R->inflated.data(); out->occupancy = R->occupancy.data();
    out->opened = R->opened.data(); out->skeleton = R->skeleton.data(); out->skeleton_framed = R->skeleton_framed.data();
    out->ror_keep = R->ror_keep.data();
    R->cl_off.push_back(0);
    for (const auto &c : R->clusters) {
        for (const auto &cell : c.cells) { R->cl_cells.push_back(cell.first); R->cl_cells.push_back(cell.second); }
        R->cl_off.push_back((int32_t)(R->cl_cells.size() / 2));
        R->cl_center.push_back(c.center_x); R->cl_center.push_back(c.center_y);
        R->cl_length.push_back(c.length);
    }
    out->n_clusters = (int32_t)R->clusters.size();
    out->cluster_offsets = R->cl_off.data(); out->cluster_cells = R->cl_cells.data();
    out->cluster_center = R->cl_center.data(); out->cluster_length = R->cl_length.data();
    for (const auto &r : R->rows) {
        R->row_center.push_back(r.center.x); R->row_center.push_back(r.center.y);
        R->row_start.push_back(r.start.x); R->row_start.push_back(r.start.y);
        R->row_end.push_back(r.end.x); R->row_end.push_back(r.end.y);
        R->row_length.push_back(r.length);
    }
    out->n_rows = (int32_t)R->rows.size();
    out->row_center = R->row_center.data(); out->row_start = R->row_start.data();
    out->row_end = R->row_end.data(); out->row_length = R->row_length.data();
    out->n_virtual = (int32_t)R->virtual_seeds.size(); out->virtual_xy = xy_of(R->virtual_seeds);
    out->n_ray = (int32_t)R->ray_seeds.size(); out->ray_xy = xy_of(R->ray_seeds);
    out->n_endpoint = (int32_t)R->endpoint_seeds.size(); out->endpoint_xy = xy_of(R->endpoint_seeds);
    out->n_voronoi = (int32_t)R->voronoi_seeds.size(); out->voronoi_xy = xy_of(R->voronoi_seeds);
    out->rows_info_xy = xy_of(R->rows_info);
    out->n_cluster_info = (int32_t)R->cluster_info.size(); out->cluster_info_xy = xy_of(R->cluster_info);
    return R;
}

struct GvdHandle { GvdResult R; };

void *orc_gvd_run(const orc_params *p, const orc_gvd_in *in, orc_gvd_out *out) {
    auto *H = new (std::nothrow) GvdHandle();
    if (!H) return nullptr;
    GvdInput gin;
    for (int i = 0; i < in->n_seeds; ++i) gin.seeds.push_back(V2{in->seeds_xy[2 * i], in->seeds_xy[2 * i + 1]});
    for (int i = 0; i < in->n_rows_poses; ++i) gin.rows_info.push_back(V2{in->rows_info_xy[2 * i], in->rows_info_xy[2 * i + 1]});
    gin.info = GridInfo{in->origin_x, in->origin_y, in->resolution, in->width, in->height};
    gin.skeleton = in->skeleton;
    gvd(*p, gin, H->R);
    GvdResult &R = H->R;
    std::memset(out, 0, sizeof(*out));
    out->published = R.published;
    out->resolution = R.resolution; out->origin_x = R.origin_x; out->origin_y = R.origin_y;
    for (auto &v : R.merged) { R.flat_merged.push_back(v.x); R.flat_merged.push_back(v.y); }
    for (auto &e : R.vor_edges) { R.flat_edges.push_back(e.start.x); R.flat_edges.push_back(e.start.y); R.flat_edges.push_back(e.end.x); R.flat_edges.push_back(e.end.y); }
    for (auto &v : R.boundary_raw) { R.flat_braw.push_back(v.x); R.flat_braw.push_back(v.y); }
    for (auto &v : R.nodes) { R.flat_nodes.push_back(v.x); R.flat_nodes.push_back(v.y); }
    out->n_merged = (int32_t)R.merged.size(); out->merged_xy = R.flat_merged.data();
    out->n_vor_edges = (int32_t)R.vor_edges.size(); out->vor_edges = R.flat_edges.data();
    out->n_boundary_raw = (int32_t)R.boundary_raw.size(); out->boundary_raw = R.flat_braw.data();
    out->n_vertices_dead = R.n_vertices_dead;
    out->num_nodes = (int32_t)R.nodes.size(); out->nodes_xy = R.flat_nodes.data();
    out->node_labels = R.labels.data(); out->node_cluster_indices = R.cluster_idx.data(); out->node_label_counts = R.label_counts.data();
    out->n_label_entries = (int32_t)R.label_clusters.size();
    out->node_label_clusters = R.label_clusters.data(); out->node_label_types = R.label_types.data();
    out->num_edges = (int32_t)R.lengths.size(); out->edges = R.edges.data();
    out->edge_lengths = R.lengths.data(); out->edge_clearances = R.clearances.data();
    out->n_label_rows = (int32_t)(R.row_label_valid.size() / 4);
    out->row_label_pts = R.row_label_pts.data(); out->row_label_valid = R.row_label_valid.data();
    out->n_cells = R.cell_off.empty() ? 0 : (int32_t)R.cell_off.size() - 1;
    out->cell_offsets = R.cell_off.data(); out->cell_xy = R.cell_xy.data();
    out->cell_center_xy = R.cell_center.data(); out->cell_rgba = R.cell_rgba.data();
    return H;
}

struct FacetHandle { Facets F; std::vector<int32_t> off; std::vector<float> pts, centers; };

void *orc_subdiv_facets(const double *seeds_xy, int32_t n, double min_x, double max_x, double min_y, double max_y,
                        int32_t rect_mode, int32_t *n_facets, const int32_t **offsets, const float **pts,
                        const float **centers) {
    auto *H = new (std::nothrow) FacetHandle();
    std::vector<V2> s;
    for (int i = 0; i < n; ++i) s.push_back(V2{seeds_xy[2 * i], seeds_xy[2 * i + 1]});
    subdiv_voronoi_facets(s, min_x, max_x, min_y, max_y, rect_mode, H->F);
    H->off.push_back(0);
    for (auto &f : H->F.facets) {
        for (auto &p : f) { H->pts.push_back(p.first); H->pts.push_back(p.second); }
        H->off.push_back((int32_t)(H->pts.size() / 2));
    }
    for (auto &c : H->F.centers) { H->centers.push_back(c.first); H->centers.push_back(c.second); }
    *n_facets = (int32_t)H->F.facets.size();
    *offsets = H->off.data(); *pts = H->pts.data(); *centers = H->centers.data();
    return H;
}

// qe: next[4] of every quad-edge, then pt[4] of every quad-edge (n_q of each); vertices: firstEdge, type, xy
struct SubdivStateHandle { std::vector<int> qe, vfirst, vtype, inserted; std::vector<float> vxy; FacetHandle f; };
void *orc_subdiv_state(const float *xy, int32_t n, const float *rect, int32_t rect_mode, int32_t *n_q, const int32_t **qe,
                       int32_t *n_v, const int32_t **vfirst, const int32_t **vtype, const float **vxy, const int32_t **inserted,
                       int32_t *n_facets, const int32_t **offsets, const float **pts) {
    auto *H = new (std::nothrow) SubdivStateHandle();
    subdiv_raw_state(xy, n, rect, rect_mode, H->qe, H->vfirst, H->vtype, H->vxy, H->f.F, H->inserted);
    *n_q = (int32_t)(H->qe.size() / 8);
    *qe = H->qe.data();
    *n_v = (int32_t)H->vfirst.size();
    *vfirst = H->vfirst.data(); *vtype = H->vtype.data(); *vxy = H->vxy.data(); *inserted = H->inserted.data();
    H->f.off.push_back(0);
    for (auto &fc : H->f.F.facets) {
        for (auto &p : fc) { H->f.pts.push_back(p.first); H->f.pts.push_back(p.second); }
        H->f.off.push_back((int32_t)(H->f.pts.size() / 2));
    }
    *n_facets = (int32_t)H->f.F.facets.size();
    *offsets = H->f.off.data(); *pts = H->f.pts.data();
    return H;
}
void orc_free_subdiv_state(void *h) { delete static_cast<SubdivStateHandle *>(h); }

void orc_free_seedgen(void *h) { delete static_cast<SeedGenResult *>(h); }
void orc_free_gvd(void *h) { delete static_cast<GvdHandle *>(h); }
void orc_free_facets(void *h) { delete static_cast<FacetHandle *>(h); }

void orc_ror(const float *xyz, uint64_t n, int32_t is_dense, double radius, int32_t min_pts, uint8_t *keep) {
    ror(xyz, n, is_dense != 0, radius, min_pts, keep);
}
void orc_inflate(const int8_t *in, uint32_t w, uint32_t h, int32_t cells, int8_t *out) { inflate(in, (int)w, (int)h, cells, out); }
void orc_open_cross(const uint8_t *in01, uint32_t w, uint32_t h, uint8_t *out01) { open_cross(in01, (int)w, (int)h, out01); }
int32_t orc_thin(const uint8_t *in01, uint32_t w, uint32_t h, uint8_t *out01) { return thin(in01, (int)w, (int)h, out01); }

}  // extern "C"
