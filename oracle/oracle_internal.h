// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
#pragma once
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

#include "oracle.h"

namespace orc {

typedef orc_params Params;
typedef std::vector<std::pair<double, double>> Poly;

// Eigen::Vector2d semantics used by the reference (Eigen 3.4, no FMA): squaredNorm = x*x + y*y,
// norm = sqrt(squaredNorm), normalized = v / norm (if squaredNorm > 0), dot = x*x' + y*y'.
struct V2 { double x, y; };
inline V2 operator-(V2 a, V2 b) { return V2{a.x - b.x, a.y - b.y}; }
inline V2 operator+(V2 a, V2 b) { return V2{a.x + b.x, a.y + b.y}; }
inline V2 operator-(V2 a) { return V2{-a.x, -a.y}; }
inline V2 operator*(double s, V2 a) { return V2{s * a.x, s * a.y}; }
inline V2 operator*(V2 a, double s) { return V2{a.x * s, a.y * s}; }
inline double squared_norm(V2 a) { return a.x * a.x + a.y * a.y; }
inline double norm(V2 a) { return std::sqrt(squared_norm(a)); }
inline double dot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
inline V2 normalized(V2 a) {
    double z = squared_norm(a);
    if (z > 0.0) { double s = std::sqrt(z); return V2{a.x / s, a.y / s}; }
    return a;
}

// The reference is built without optimisation (colcon without CMAKE_BUILD_TYPE; CMakeLists.txt:12):
// sin and cos are separate libm calls, never fused into one sincos (which can differ by an ulp).
__attribute__((noinline)) inline double lib_sin(double a) { return std::sin(a); }
__attribute__((noinline)) inline double lib_cos(double a) { return std::cos(a); }

struct GridInfo { double origin_x, origin_y; float resolution; uint32_t width, height; };

struct Cluster {
    std::vector<std::pair<int, int>> cells;
    float center_x = 0.0f, center_y = 0.0f;
    int size = 0;
    float length = 0.0f;
};

struct TreeRow { V2 center, start, end; double length; };

struct SeedGenResult {
    GridInfo info{};
    uint64_t n_input = 0, n_ror_kept = 0, n_clipped = 0;
    std::vector<uint8_t> ror_keep, opened;
    std::vector<int8_t> raster, inflated, occupancy, skeleton, skeleton_framed;
    int thin_iters = 0;
    std::vector<Cluster> clusters;
    std::vector<TreeRow> rows;
    std::vector<V2> virtual_seeds, ray_seeds, endpoint_seeds, voronoi_seeds, rows_info, cluster_info;
    // flattened views for the C API
    std::vector<int32_t> cl_off, cl_cells;
    std::vector<float> cl_center, cl_length;
    std::vector<double> row_center, row_start, row_end, row_length;
};

void ror(const float *xyz, uint64_t n, bool is_dense, double radius, int min_pts, uint8_t *keep);
void inflate(const int8_t *in, int w, int h, int cells, int8_t *out);
void open_cross(const uint8_t *in, int w, int h, uint8_t *out);
int thin(const uint8_t *in, int w, int h, uint8_t *out);
bool point_in_polygon(double px, double py, const Poly &polygon);
void seedgen(const Params &P, const float *xyz, uint64_t n, bool is_dense, const Poly &poly, SeedGenResult &R);

// ---- GVD ----
struct VEdge { V2 start, end; };
struct EdgeRecord { int from, to; double length_m; float min_clearance_m; };

struct GvdResult {
    bool published = false;
    double resolution = 0, origin_x = 0, origin_y = 0;
    std::vector<V2> merged, boundary_raw, nodes;
    std::vector<VEdge> vor_edges;
    int n_vertices_dead = 0;
    std::vector<int32_t> labels, cluster_idx, label_counts, label_clusters, label_types, edges;
    std::vector<float> lengths, clearances;
    std::vector<double> row_label_pts;
    std::vector<int32_t> row_label_valid;
    std::vector<double> flat_merged, flat_edges, flat_braw, flat_nodes;
    // publishMarkers (P.markers): cells of extractCellBoundaries, closed like the reference
    std::vector<int32_t> cell_off;
    std::vector<double> cell_xy, cell_center;
    std::vector<float> cell_rgba;
};

struct GvdInput {
    std::vector<V2> seeds;
    std::vector<V2> rows_info;  // poses
    GridInfo info;
    const int8_t *skeleton;
};

// OpenCV Subdiv2D facets (restatement; NOTES.md §5)
struct Facets {
    std::vector<std::vector<std::pair<float, float>>> facets;
    std::vector<std::pair<float, float>> centers;
};
void subdiv_raw_state(const float *xy, int n, const float rect[4], int rect_mode, std::vector<int> &qe,
                      std::vector<int> &vfirst, std::vector<int> &vtype, std::vector<float> &vxy, Facets &facets,
                      std::vector<int> &inserted);
void subdiv_voronoi_facets(const std::vector<V2> &seeds, double min_x, double max_x, double min_y, double max_y,
                           int rect_mode, Facets &out, float *rect_out = nullptr);
void voronoi_compute(const std::vector<V2> &seeds, double min_x, double max_x, double min_y, double max_y, int rect_mode,
                     bool dead_work, std::vector<VEdge> &edges, int &n_vertices);
void gvd(const Params &P, const GvdInput &in, GvdResult &R);

}  // namespace orc
