// Incremental Delaunay / Voronoi facets with OpenCV 4.5.4 cv::Subdiv2D semantics
// (modules/imgproc/src/subdivision2d.cpp, used by aos::VoronoiDiagram::compute,
// src/utils/voronoi_diagram.cpp:51-94).
//
// Why on the host: insertion is inherently sequential and history-dependent — the quad-edge
// numbering, vtx[].firstEdge (which decides where each facet starts) and which edge pair computes
// each circumcentre (float rounding) all depend on the exact locate walk and flip order. Each
// insert's locate walk starts where the previous one ended, so there is no independent work to
// spread. GvdGraph node order follows that history, so bit-identical topology needs this exact
// replay; the GPU takes over from the facet list on (gvd.hip: k_vor_faces, k_facet_*).
//
// Representation: OpenCV stores all four rotations of a quad-edge (primal and dual rings). Only the
// primal rings are stored here, doubly linked (onext and its inverse oprev per directed edge), with
// the same quad-edge ids (directed edge e = 4q + {0, 2}). Every navigation the algorithm uses is an
// identity of the edge algebra (Oprev = Rot Onext Rot):
//   Lnext(e) = Oprev(Sym e),  Dprev(e) = Sym Oprev(Sym e),  Lprev(e) = Sym Onext(e),
// and splice(a, b) = swap(Onext a, Onext b) plus the two inverse links: two independent loads and
// four stores instead of OpenCV's two-level dependent chain through the dual ring. The dual links
// are recovered when the structure is exported (Onext(Rot e) = Rot^-1 Oprev(e)). On orchard seed rows
// an insert performs ~56 swaps (~115 flip-loop steps) as each new seed on the next tree line takes
// over the fan of the previous one, so these constant factors are the replay's cost.
//
// Cavity form of the swap loop (insert_cavity). Every triangle the swap loop tests lies across a
// link edge from the new point p, so it is never incident to p: it is an *old* triangle, untouched
// when it is tested. Each test is therefore a pure function of the triangulation before the insert,
// and the loop is a depth-first pre-order walk of the cavity tree (children in clockwise order
// around p). A read-only DFS over the old structure replays exactly the same tests with the same
// arguments, then the outcome is written in one pass:
//   * the internal edge e through which the walk entered cavity triangle T (directed as the loop's
//     curr_edge) becomes T's apex -> p with pt[dir(e)] = apex (setEdgePoints in swapEdges);
//   * vtx[apex].firstEdge = e, and vtx[p].firstEdge = Sym of the last swap in walk order;
//   * the rings are the cyclic orders of the final star, which the walk order of the boundary
//     (link) edges fixes; the unique onext/oprev values are stored directly.
// The swap loop stays as the reference path (on-edge inserts, and any walk that meets an apex that is
// already a cavity vertex). tools/sdcheck compares the two paths' complete state after every insert.
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <vector>

namespace aos {

// per-phase counters of a build with -DAOS_SD_PROF (tools/sdcheck/sdprof.cpp); TSC ticks
struct SdProf { unsigned long long t_locate = 0, t_dfs = 0, t_write = 0, loc_iters = 0, dfs_steps = 0; };
extern SdProf g_sdprof;

class Subdiv2D {
  public:
    Subdiv2D();
    // rect: Subdiv2D(Rect2f) (mode 0) or the implicit Rect2f -> Rect conversion (mode 1)
    void init_delaunay(float rx, float ry, float rw, float rh, int rect_mode);
    // Subdiv2D::insert; returns false where OpenCV throws (the reference catches and skips).
    bool insert(float x, float y);
    // 0: cavity DFS + bulk write (default); 1: always OpenCV's swap loop (reference / cross-check)
    void set_swap_loop(bool on) { force_loop = on; }
    void set_simd(bool on) { use_avx2 = on && simd_ok(); }   // batched boundary flip tests on AVX2 (off by default)
    static bool simd_ok() {
#if defined(__x86_64__)
        return __builtin_cpu_supports("avx2");
#else
        return false;
#endif
    }
    // full internal state (for the equivalence checker): rings, end points, firstEdge, recentEdge
    bool same_state(const Subdiv2D &o) const;
    long n_cavity = 0, n_loop = 0;   // inserts done by each path
    // getVoronoiFacetList(idx = {}): per real vertex (in vertex order) the facet polygon.
    // Emits the reference's edge list directly: (p_i, p_{i+1 mod n}) for facets with >= 2 points
    // (voronoi_diagram.cpp:97-114), as float x0, y0, x1, y1. Host reference of the GPU builder.
    void voronoi_edges(std::vector<float> &edges);
    // getVoronoiFacetList(idx = {}) as polygons: facet f (real vertices in vertex order) is the float
    // points xy[2 * off[f] .. 2 * off[f + 1]) (extractCellBoundaries, voronoi_diagram.cpp:288-290).
    void voronoi_facets(std::vector<int> &off, std::vector<float> &xy);
    size_t num_vertices() const { return vp.size(); }
    void reserve(size_t n_points);
    // OpenCV-layout quad-edge state after the inserts, for the GPU facet builder:
    // qe = 8 ints per quad-edge {next[4], pt[4]} (free quad-edges have next[0] = 0), vp = float2.
    struct Raw { const int *qe; int n_rec; const float *vp; const int *vfirst, *vtype; int n_vtx; };
    Raw raw();
    // the same state written straight into dst (raw_bytes() bytes: qe | vp | vfirst | vtype), e.g. the
    // pinned staging buffer of the GPU facet builder: no zero-fill, export buffer or second copy
    size_t raw_bytes() const { return (8 * sizeof(int) * rec.size()) + (sizeof(V2f) + 2 * sizeof(int)) * vp.size(); }
    // written(offset, bytes): called after each chunk_recs records but the last, so that the caller can start
    // copying what is written (the rest, from the last call's end to raw_bytes(), once raw_into returns)
    Raw raw_into(void *dst, int chunk_recs = 0, const std::function<void(size_t, size_t)> &written = {}) const;

  private:
    // (32-byte aligned: a record or a vertex never straddles two cache lines; the C2 replay 26.3-27.0 ->
    // 26.0-26.6 ms on the box, profiles/r04z_replay_dfs.txt)
    // A quad-edge's record holds its two primal directed edges, 16 bytes each: directed edge e (always even, 4q or
    // 4q + 2) sits at byte 8 e of the array, so a field is one load at [base + 8 e + field] with no index arithmetic
    // (round 5: the replay's field accessors took 3-4 instructions each in the {on[2], op[2], org[2]} layout)
    struct alignas(16) Half { int on, op, org, x; };   // x: the free-list link in half 0 of a free record
    struct alignas(32) Rec { Half h[2]; };
    struct V2f { float x, y; };
    struct alignas(32) V2d { double x, y, n2; int stamp, spoke; };   // stamp / spoke: insert_cavity scratch
    std::vector<Rec> rec;
    std::vector<V2f> vp;
    std::vector<V2d> vd;   // exact double copies of vp plus x*x + y*y, for the predicates
    std::vector<int> vfirst, vtype;   // type: -1 free, 0 real, 1 virtual
    std::vector<int> qx;              // export buffer (Raw::qe)
    int free_q = 0, free_p = 0, recent = 0;
    bool force_loop = false, use_avx2 = false;
    // cavity DFS scratch: stack of link edges, boundary edges in walk order (with their origins); per
    // vertex (V2d) the spoke, valid while its stamp is this insert's
    std::vector<int> dfs_stack, cav_bnd, cav_bu;
    int stamp = 0;
    float tlx = 0, tly = 0, brx = 0, bry = 0;

    static int sym(int e) { return e ^ 2; }
    static int dir(int e) { return (e >> 1) & 1; }
    int *ri() { return reinterpret_cast<int *>(rec.data()); }
    const int *ri() const { return reinterpret_cast<const int *>(rec.data()); }
    int &on(int e) { return ri()[2 * (ptrdiff_t)e]; }
    int &op(int e) { return ri()[2 * (ptrdiff_t)e + 1]; }
    int &orgr(int e) { return ri()[2 * (ptrdiff_t)e + 2]; }
    int onext(int e) const { return ri()[2 * (ptrdiff_t)e]; }
    int oprev(int e) const { return ri()[2 * (ptrdiff_t)e + 1]; }
    int org(int e) const { return ri()[2 * (ptrdiff_t)e + 2]; }
    int dst(int e) const { return ri()[2 * (ptrdiff_t)(e ^ 2) + 2]; }
    int lnext(int e) const { return oprev(sym(e)); }          // NEXT_AROUND_LEFT
    int dprev(int e) const { return sym(oprev(sym(e))); }     // PREV_AROUND_DST
    int lprev(int e) const { return sym(onext(e)); }          // PREV_AROUND_LEFT
    int right_of(float px, float py, int e) const;
    int new_edge();
    int new_point(float x, float y, int type);
    void splice(int a, int b) {
        const int an = on(a), bn = on(b);
        on(a) = bn; on(b) = an;
        op(bn) = a; op(an) = b;
    }
    void set_pts(int e, int o, int d);
    int connect(int a, int b);
    void swap_edge(int e);
    void delete_edge(int e);
    int locate(float px, float py, int &edge, int &vertex);
    void swap_loop(int curr_edge, int first_point, int curr_point);
    void flip_tests_scalar(const int *es, int n, const V2d &P, int *out) const;
    void flip_tests_avx2(const int *es, int n, const V2d &P, int *out) const;
    template <bool SIMD> bool insert_cavity(int e0, int curr_point);
    void calc_voronoi();   // calcVoronoi on the exported layout (qx), creating the virtual vertices
    int facet_next(int e) const;
};

}  // namespace aos
