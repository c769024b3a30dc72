// Incremental Delaunay / Voronoi facets with OpenCV 4.5.4 cv::Subdiv2D semantics
// (modules/imgproc/src/subdivision2d.cpp, used by aos::VoronoiDiagram::compute,
// src/utils/voronoi_diagram.cpp:51-94).
//
// Why on the host: insertion is inherently sequential and history-dependent — the quad-edge
// numbering, vtx[].firstEdge (which decides where each facet starts) and which edge pair computes
// each circumcentre (float rounding) all depend on the exact locate walk and flip order. GvdGraph
// node numbering follows that order, so bit-identical topology needs this exact replay; the
// GPU takes over from the facet list on (boundary points, graph, labels).
//
// Layout: one 32-byte record per quad-edge ({next[4], pt[4]}, one cache line holds two) and one
// 8-byte float2 per vertex: the flip walk (~115 iterations per insert on orchard seed rows, where
// a new row line briefly fans out to the whole previous line) is pure pointer chasing.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace aos {

class Subdiv2D {
  public:
    // rect: Subdiv2D(Rect2f) (mode 0) or the implicit Rect2f -> Rect conversion (mode 1)
    void init_delaunay(float rx, float ry, float rw, float rh, int rect_mode);
    // Subdiv2D::insert; returns false where OpenCV throws (the reference catches and skips).
    bool insert(float x, float y);
    // getVoronoiFacetList(idx = {}): per real vertex (in vertex order) the facet polygon.
    // Emits the reference's edge list directly: (p_i, p_{i+1 mod n}) for facets with >= 2 points
    // (voronoi_diagram.cpp:97-114), as float x0, y0, x1, y1.
    void voronoi_edges(std::vector<float> &edges);
    size_t num_vertices() const { return vp.size(); }
    // Raw quad-edge state after the inserts, for the GPU facet builder (gvd.hip k_vor_faces /
    // k_facet_*): qe = 8 ints per quad-edge {next[4], pt[4]}, vp = float2 per vertex.
    struct Raw { const int *qe; int n_rec; const float *vp; const int *vfirst, *vtype; int n_vtx; };
    Raw raw() const {
        return Raw{reinterpret_cast<const int *>(qe.data()), (int)qe.size(), reinterpret_cast<const float *>(vp.data()),
                   vfirst.data(), vtype.data(), (int)vp.size()};
    }
    void reserve(size_t n_points);

  private:
    enum { NEXT_AROUND_LEFT = 0x13, NEXT_AROUND_RIGHT = 0x31, PREV_AROUND_ORG = 0x11, PREV_AROUND_DST = 0x33 };
    struct alignas(32) QE { int next[4]; int pt[4]; };
    struct V2f { float x, y; };
    struct V2d { double x, y, n2, pad; };
    std::vector<V2f> vp;
    std::vector<V2d> vd;   // exact double copies of vp plus x*x + y*y, for the flip-loop predicates
    std::vector<int> vfirst, vtype;   // type: -1 free, 0 real, 1 virtual
    std::vector<QE> qe;
    int free_q = 0, free_p = 0, recent = 0;
    float tlx = 0, tly = 0, brx = 0, bry = 0;

    int next_e(int e) const { return qe[e >> 2].next[e & 3]; }
    static int rot(int e, int r) { return (e & ~3) + ((e + r) & 3); }
    int get_e(int e, int t) const { e = qe[e >> 2].next[(e + t) & 3]; return (e & ~3) + ((e + (t >> 4)) & 3); }
    int org(int e) const { return qe[e >> 2].pt[e & 3]; }
    int dst(int e) const { return qe[e >> 2].pt[(e + 2) & 3]; }
    int right_of(float px, float py, int e) const;
    int new_edge();
    int new_point(float x, float y, int type);
    void splice(int a, int b);
    void set_pts(int e, int o, int d);
    int connect(int a, int b);
    void swap_edge(int e);
    void delete_edge(int e);
    int locate(float px, float py, int &edge, int &vertex);
    void calc_voronoi();
};

}  // namespace aos
