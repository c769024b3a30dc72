// Host Delaunay with cv::Subdiv2D semantics — see subdiv2d.h. Compiled -ffp-contract=off.
#include "subdiv2d.h"

#include <algorithm>
#include <cfloat>
#include <cmath>

namespace aos {

namespace {
// triangleArea (double from float coordinates)
inline double tri_area(float ax, float ay, float bx, float by, float cx, float cy) {
    return ((double)bx - ax) * ((double)cy - ay) - ((double)by - ay) * ((double)cx - ax);
}
// computeVoronoiPoint; returns false for det == 0 or a huge result (the vertex is not created)
inline bool voronoi_point(float o0x, float o0y, float d0x, float d0y, float o1x, float o1y, float d1x, float d1y,
                          float &rx, float &ry) {
    double a0 = d0x - o0x, b0 = d0y - o0y;
    double c0 = -0.5 * (a0 * (d0x + o0x) + b0 * (d0y + o0y));
    double a1 = d1x - o1x, b1 = d1y - o1y;
    double c1 = -0.5 * (a1 * (d1x + o1x) + b1 * (d1y + o1y));
    double det = a0 * b1 - a1 * b0;
    if (det != 0) {
        det = 1. / det;
        rx = (float)((b0 * c1 - b1 * c0) * det);
        ry = (float)((a1 * c0 - a0 * c1) * det);
        return std::abs(rx) < FLT_MAX * 0.5 && std::abs(ry) < FLT_MAX * 0.5;
    }
    return false;
}
}  // namespace

void Subdiv2D::reserve(size_t n) {
    vp.reserve(2 * n + 8); vd.reserve(2 * n + 8); vfirst.reserve(2 * n + 8); vtype.reserve(2 * n + 8);
    rec.reserve(3 * n + 8);
}

int Subdiv2D::right_of(float px, float py, int e) const {   // isRightOf: sign of triangleArea(p, dst, org)
    const V2d &o = vd[org(e)], &d = vd[dst(e)];
    const double x = px, y = py;
    const double cw = (d.x - x) * (o.y - y) - (d.y - y) * (o.x - x);
    return (cw > 0) - (cw < 0);
}

// newEdge: a fresh quad-edge whose primal edges are singleton rings; free quad-edges are reused LIFO
int Subdiv2D::new_edge() {
    if (free_q <= 0) {
        rec.push_back(Rec{{0, 0}, {0, 0}, {0, 0}, 0, 0});
        free_q = (int)rec.size() - 1;
    }
    const int q = free_q, e = q * 4;
    free_q = rec[q].link;
    rec[q] = Rec{{e, e + 2}, {e, e + 2}, {0, 0}, 0, 0};
    return e;
}

int Subdiv2D::new_point(float x, float y, int type) {
    if (free_p == 0) {
        vp.push_back(V2f{0.f, 0.f}); vfirst.push_back(0); vtype.push_back(-1);
        free_p = (int)vp.size() - 1;
    }
    const int v = free_p;
    free_p = vfirst[v];
    vp[v] = V2f{x, y}; vfirst[v] = 0; vtype[v] = type;
    if (vd.size() < vp.size()) vd.resize(vp.size());
    vd[v] = V2d{(double)x, (double)y, (double)x * x + (double)y * y, 0.0};
    return v;
}

void Subdiv2D::set_pts(int e, int o, int d) {   // setEdgePoints
    rec[e >> 2].org[dir(e)] = o;
    rec[e >> 2].org[dir(e) ^ 1] = d;
    vfirst[o] = e;
    vfirst[d] = sym(e);
}

int Subdiv2D::connect(int a, int b) {   // connectEdges
    const int e = new_edge();
    splice(e, lnext(a));
    splice(sym(e), b);
    set_pts(e, dst(a), org(b));
    return e;
}

void Subdiv2D::swap_edge(int e) {   // swapEdges
    const int se = sym(e);
    const int a = oprev(e), b = oprev(se);
    splice(e, a);
    splice(se, b);
    set_pts(e, dst(a), dst(b));
    splice(e, lnext(a));
    splice(se, lnext(b));
}

void Subdiv2D::delete_edge(int e) {   // deleteEdge
    splice(e, oprev(e));
    const int se = sym(e);
    splice(se, oprev(se));
    const int q = e >> 2;
    rec[q].on[0] = 0;          // free marker (OpenCV: next[0] = 0)
    rec[q].link = free_q;
    free_q = q;
}

void Subdiv2D::init_delaunay(float rx, float ry, float rw, float rh, int rect_mode) {
    if (rect_mode == 1) {  // Rect_<float> -> Rect_<int>: saturate_cast<int> = cvRound (nearest even)
        rx = (float)(int)std::lrint(rx); ry = (float)(int)std::lrint(ry);
        rw = (float)(int)std::lrint(rw); rh = (float)(int)std::lrint(rh);
    }
    const float big = 3.f * std::max(rw, rh);
    vp.clear(); vd.clear(); vfirst.clear(); vtype.clear(); rec.clear();
    recent = 0;
    tlx = rx; tly = ry; brx = rx + rw; bry = ry + rh;
    vp.push_back(V2f{0.f, 0.f}); vd.push_back(V2d{0.0, 0.0, 0.0, 0.0}); vfirst.push_back(0); vtype.push_back(-1);
    rec.push_back(Rec{{0, 0}, {0, 0}, {0, 0}, 0, 0});                          // quad-edge 0 (NULL)
    free_q = 0; free_p = 0;
    const int pA = new_point(rx + big, ry, 0), pB = new_point(rx, ry + big, 0), pC = new_point(rx - big, ry - big, 0);
    const int eAB = new_edge(), eBC = new_edge(), eCA = new_edge();
    set_pts(eAB, pA, pB); set_pts(eBC, pB, pC); set_pts(eCA, pC, pA);
    splice(eAB, sym(eCA)); splice(eBC, sym(eAB)); splice(eCA, sym(eBC));
    recent = eAB;
}

// Subdiv2D::locate: 0 inside, 1 vertex, 2 on edge, -1 outside rect, -2 error
int Subdiv2D::locate(float px, float py, int &out_edge, int &out_vertex) {
    int vertex = 0;
    const int max_edges = (int)rec.size() * 4;
    if (px < tlx || py < tly || px >= brx || py >= bry) return -1;
    int edge = recent;
    int location = -2;
    int roc = right_of(px, py, edge);
    if (roc > 0) { edge = sym(edge); roc = -roc; }
    for (int i = 0; i < max_edges; i++) {
        const int on_ = onext(edge);
        const int dp = dprev(edge);
        const int ron = right_of(px, py, on_);
        const int rod = right_of(px, py, dp);
        if (rod > 0) {
            if (ron > 0 || (ron == 0 && roc == 0)) { location = 0; break; }
            roc = ron; edge = on_;
        } else {
            if (ron > 0) {
                if (rod == 0 && roc == 0) { location = 0; break; }
                roc = rod; edge = dp;
            } else if (roc == 0 && right_of(vp[dst(on_)].x, vp[dst(on_)].y, edge) >= 0) {
                edge = sym(edge);
            } else {
                roc = ron; edge = on_;
            }
        }
    }
    recent = edge;
    if (location == 0) {
        const int o = org(edge), d = dst(edge);
        const float ox = vp[o].x, oy = vp[o].y, dx = vp[d].x, dy = vp[d].y;
        double t1 = std::fabs(px - ox); t1 += std::fabs(py - oy);
        double t2 = std::fabs(px - dx); t2 += std::fabs(py - dy);
        double t3 = std::fabs(ox - dx); t3 += std::fabs(oy - dy);
        if (t1 < FLT_EPSILON) { location = 1; vertex = o; edge = 0; }
        else if (t2 < FLT_EPSILON) { location = 1; vertex = d; edge = 0; }
        else if ((t1 < t3 || t2 < t3) && std::fabs(tri_area(px, py, ox, oy, dx, dy)) < FLT_EPSILON) { location = 2; vertex = 0; }
    }
    if (location == -2) { edge = 0; vertex = 0; }
    out_edge = edge; out_vertex = vertex;
    return location;
}

bool Subdiv2D::insert(float x, float y) {
    int curr_edge = 0, curr_point = 0;
    const int loc = locate(x, y, curr_edge, curr_point);
    if (loc < 0) return false;        // PTLOC_ERROR (CV_StsBadSize) / outside rect (CV_StsOutOfRange)
    if (loc == 1) return true;        // existing vertex: nothing inserted
    if (loc == 2) {
        const int deleted = curr_edge;
        recent = curr_edge = oprev(curr_edge);
        delete_edge(deleted);
    }
    if (curr_edge == 0) return false;  // CV_Assert
    curr_point = new_point(x, y, 0);
    int base = new_edge();
    const int first_point = org(curr_edge);
    set_pts(base, first_point, curr_point);
    splice(base, curr_edge);
    do {
        base = connect(curr_edge, sym(base));
        curr_edge = oprev(base);
    } while (dst(curr_edge) != first_point);
    curr_edge = oprev(base);
    const int max_edges = (int)rec.size() * 4;
    // Swap loop with the predicates written out on exact double copies of the float coordinates
    // (the float -> double conversions are exact, so every product and sum rounds as in
    // triangleArea / isPtInCircle3, and |p|^2 is formed once per vertex in the same order).
    const V2d P = vd[curr_point];
    auto area = [](const V2d &a, const V2d &b, const V2d &c) { return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x); };
    for (int i = 0; i < max_edges; i++) {
        const int temp = oprev(curr_edge);
        const int tdst = dst(temp), corg = org(curr_edge), cdst = dst(curr_edge);
        const V2d &T = vd[tdst], &O = vd[corg], &D = vd[cdst];
        bool flip = false;
        if (area(T, D, O) > 0) {   // isRightOf(temp_dst, curr_edge) > 0
            // isPtInCircle3(pt = org, a = temp_dst, b = dst, c = new point) < 0, eps = FLT_EPSILON / 8
            double val = T.n2 * area(D, P, O);
            val -= D.n2 * area(T, P, O);
            val += P.n2 * area(T, D, O);
            val -= O.n2 * area(T, D, P);
            flip = val < -(FLT_EPSILON * 0.125);
        }
        if (flip) {
            swap_edge(curr_edge);
            curr_edge = oprev(curr_edge);
        } else if (corg == first_point) {
            break;
        } else {
            curr_edge = lprev(onext(curr_edge));
        }
    }
    return true;
}

// OpenCV quad-edge layout: next[r] = Onext of rotation r of quad-edge q. Primal rotations come
// straight from the rings; Onext(Rot e) = Rot^-1 Oprev(e) gives the dual ones. pt[0] / pt[2] are
// the primal end points; the dual pt[1] / pt[3] (Voronoi vertices) start unset (calcVoronoi).
Subdiv2D::Raw Subdiv2D::raw() {
    const int n = (int)rec.size();
    qx.assign(8 * (size_t)n, 0);
    auto rot3 = [](int x) { return (x & ~3) + ((x + 3) & 3); };
    for (int q = 1; q < n; ++q) {
        const Rec &r = rec[q];
        int *o = &qx[8 * (size_t)q];
        if (r.on[0] <= 0) continue;   // free
        o[0] = r.on[0]; o[1] = rot3(r.op[0]); o[2] = r.on[1]; o[3] = rot3(r.op[1]);
        o[4] = r.org[0]; o[6] = r.org[1];
    }
    return Raw{qx.data(), n, reinterpret_cast<const float *>(vp.data()), vfirst.data(), vtype.data(), (int)vp.size()};
}

// calcVoronoi on the exported layout (host reference of gvd.hip's builder): quad-edges from #4;
// the first quad-edge touching a triangle computes its circumcentre (pt[3] left face, pt[1] right).
int Subdiv2D::facet_next(int e) const {   // getEdge(e, NEXT_AROUND_LEFT = 0x13) on the exported layout
    const int x = qx[8 * (size_t)(e >> 2) + ((e + 3) & 3)];
    return (x & ~3) + ((x + 1) & 3);
}

void Subdiv2D::calc_voronoi() {
    raw();
    const int total = (int)rec.size();
    auto next = [&](int e) { return qx[8 * (size_t)(e >> 2) + (e & 3)]; };
    auto get_e = [&](int e, int t) { const int x = next((e & ~3) + ((e + t) & 3)); return (x & ~3) + ((x + (t >> 4)) & 3); };
    auto pt = [&](int e) -> int & { return qx[8 * (size_t)(e >> 2) + 4 + (e & 3)]; };
    for (size_t i = 0; i < vp.size(); ++i)
        if (vtype[i] > 0) { vfirst[i] = free_p; vtype[i] = -1; free_p = (int)i; }
    for (int q = 4; q < total; q++) {
        if (qx[8 * (size_t)q] <= 0) continue;  // free
        const int e0 = q * 4;
        if (!pt(e0 + 3)) {   // left face
            const int e1 = get_e(e0, 0x13), e2 = get_e(e1, 0x13);
            const V2f a = vp[pt(e0)], b = vp[pt(e0 + 2)], c = vp[pt(e1)], d = vp[pt(e1 ^ 2)];
            float rx, ry;
            if (voronoi_point(a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y, rx, ry)) {
                const int p = new_point(rx, ry, 1);
                pt(e0 + 3) = p;
                qx[8 * (size_t)(e1 >> 2) + 4 + 3 - (e1 & 2)] = p;
                qx[8 * (size_t)(e2 >> 2) + 4 + 3 - (e2 & 2)] = p;
            }
        }
        if (!pt(e0 + 1)) {   // right face
            const int e1 = get_e(e0, 0x31), e2 = get_e(e1, 0x31);
            const V2f a = vp[pt(e0)], b = vp[pt(e0 + 2)], c = vp[pt(e1)], d = vp[pt(e1 ^ 2)];
            float rx, ry;
            if (voronoi_point(a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y, rx, ry)) {
                const int p = new_point(rx, ry, 1);
                pt(e0 + 1) = p;
                qx[8 * (size_t)(e1 >> 2) + 4 + 1 + (e1 & 2)] = p;
                qx[8 * (size_t)(e2 >> 2) + 4 + 1 + (e2 & 2)] = p;
            }
        }
    }
}

// getVoronoiFacetList: per real vertex (vertex order) the ring of Voronoi points, starting at
// rotateEdge(firstEdge, 1) and walking NEXT_AROUND_LEFT; vtx[edgeOrg(t)] (index 0 = the (0,0)
// NULL vertex when a circumcentre was not created).
void Subdiv2D::voronoi_facets(std::vector<int> &off, std::vector<float> &xy) {
    calc_voronoi();
    off.assign(1, 0);
    xy.clear();
    const size_t nv = vp.size();
    for (size_t k = 4; k < nv; k++) {
        if (vtype[k] != 0) continue;  // free or virtual
        const int f = vfirst[k], start = (f & ~3) + ((f + 1) & 3);
        int t = start;
        do {
            const int p = qx[8 * (size_t)(t >> 2) + 4 + (t & 3)];
            xy.push_back(vp[p].x); xy.push_back(vp[p].y);
            t = facet_next(t);
        } while (t != start);
        off.push_back((int)(xy.size() / 2));
    }
}

void Subdiv2D::voronoi_edges(std::vector<float> &edges) {
    std::vector<int> off;
    std::vector<float> xy;
    voronoi_facets(off, xy);
    edges.clear();
    for (size_t f = 0; f + 1 < off.size(); ++f) {
        const int b = off[f], n = off[f + 1] - b;
        if (n < 2) continue;
        for (int i = 0; i < n; ++i) {
            const int a = b + i, c = b + (i + 1) % n;
            edges.push_back(xy[2 * a]); edges.push_back(xy[2 * a + 1]); edges.push_back(xy[2 * c]); edges.push_back(xy[2 * c + 1]);
        }
    }
}

}  // namespace aos
