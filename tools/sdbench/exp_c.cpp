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
// computeVoronoiPoint; returns false for det == 0 (FLT_MAX marker)
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
    qe.reserve(3 * n + 8);
}

int Subdiv2D::right_of(float px, float py, int e) const {
    const QE &q = qe[e >> 2];
    const V2d &o = vd[q.pt[e & 3]], &d = vd[q.pt[(e + 2) & 3]];
    const double x = px, y = py;
    double cw = (d.x - x) * (o.y - y) - (d.y - y) * (o.x - x);
    return (cw > 0) - (cw < 0);
}

int Subdiv2D::new_edge() {
    if (free_q <= 0) {
        qe.push_back(QE{{0, 0, 0, 0}, {0, 0, 0, 0}});
        free_q = (int)qe.size() - 1;
    }
    int e = free_q * 4;
    QE &q = qe[free_q];
    free_q = q.next[1];
    q.next[0] = e; q.next[1] = e + 3; q.next[2] = e + 2; q.next[3] = e + 1;
    q.pt[0] = q.pt[1] = q.pt[2] = q.pt[3] = 0;
    return e;
}

int Subdiv2D::new_point(float x, float y, int type) {
    if (free_p == 0) {
        vp.push_back(V2f{0.f, 0.f}); vfirst.push_back(0); vtype.push_back(-1);
        free_p = (int)vp.size() - 1;
    }
    int v = free_p;
    free_p = vfirst[v];
    vp[v] = V2f{x, y}; vfirst[v] = 0; vtype[v] = type;
    if (vd.size() < vp.size()) vd.resize(vp.size());
    vd[v] = V2d{(double)x, (double)y, (double)x * x + (double)y * y, 0.0};
    return v;
}

void Subdiv2D::splice(int a, int b) {
    int &an = qe[a >> 2].next[a & 3], &bn = qe[b >> 2].next[b & 3];
    int ar = rot(an, 1), br = rot(bn, 1);
    int &arn = qe[ar >> 2].next[ar & 3], &brn = qe[br >> 2].next[br & 3];
    std::swap(an, bn);
    std::swap(arn, brn);
}

void Subdiv2D::set_pts(int e, int o, int d) {
    qe[e >> 2].pt[e & 3] = o;
    qe[e >> 2].pt[(e + 2) & 3] = d;
    vfirst[o] = e;
    vfirst[d] = e ^ 2;
}

int Subdiv2D::connect(int a, int b) {
    int e = new_edge();
    splice(e, get_e(a, NEXT_AROUND_LEFT));
    splice(e ^ 2, b);
    set_pts(e, dst(a), org(b));
    return e;
}

void Subdiv2D::swap_edge(int e) {
    int se = e ^ 2;
    int a = get_e(e, PREV_AROUND_ORG), b = get_e(se, PREV_AROUND_ORG);
    splice(e, a);
    splice(se, b);
    set_pts(e, dst(a), dst(b));
    splice(e, get_e(a, NEXT_AROUND_LEFT));
    splice(se, get_e(b, NEXT_AROUND_LEFT));
}

void Subdiv2D::delete_edge(int e) {
    splice(e, get_e(e, PREV_AROUND_ORG));
    int se = e ^ 2;
    splice(se, get_e(se, PREV_AROUND_ORG));
    int q = e >> 2;
    qe[q].next[0] = 0;
    qe[q].next[1] = free_q;
    free_q = q;
}

void Subdiv2D::init_delaunay(float rx, float ry, float rw, float rh, int rect_mode) {
    if (rect_mode == 1) {  // Rect_<float> -> Rect_<int>: saturate_cast<int> = cvRound (nearest even)
        rx = (float)(int)std::lrint(rx); ry = (float)(int)std::lrint(ry);
        rw = (float)(int)std::lrint(rw); rh = (float)(int)std::lrint(rh);
    }
    const float big = 3.f * std::max(rw, rh);
    vp.clear(); vd.clear(); vfirst.clear(); vtype.clear(); qe.clear();
    recent = 0;
    tlx = rx; tly = ry; brx = rx + rw; bry = ry + rh;
    vp.push_back(V2f{0.f, 0.f}); vfirst.push_back(0); vtype.push_back(-1);   // vtx[0]
    qe.push_back(QE{{0, 0, 0, 0}, {0, 0, 0, 0}});                             // qedges[0]
    free_q = 0; free_p = 0;
    int pA = new_point(rx + big, ry, 0), pB = new_point(rx, ry + big, 0), pC = new_point(rx - big, ry - big, 0);
    int eAB = new_edge(), eBC = new_edge(), eCA = new_edge();
    set_pts(eAB, pA, pB); set_pts(eBC, pB, pC); set_pts(eCA, pC, pA);
    splice(eAB, eCA ^ 2); splice(eBC, eAB ^ 2); splice(eCA, eBC ^ 2);
    recent = eAB;
}

// Subdiv2D::locate: 0 inside, 1 vertex, 2 on edge, -1 outside rect, -2 error
int Subdiv2D::locate(float px, float py, int &out_edge, int &out_vertex) {
    int vertex = 0;
    const int max_edges = (int)qe.size() * 4;
    if (px < tlx || py < tly || px >= brx || py >= bry) return -1;
    int edge = recent;
    int location = -2;
    int roc = right_of(px, py, edge);
    if (roc > 0) { edge ^= 2; roc = -roc; }
    for (int i = 0; i < max_edges; i++) {
        int onext = next_e(edge);
        int dprev = get_e(edge, PREV_AROUND_DST);
        int ron = right_of(px, py, onext);
        int rod = right_of(px, py, dprev);
        if (rod > 0) {
            if (ron > 0 || (ron == 0 && roc == 0)) { location = 0; break; }
            roc = ron; edge = onext;
        } else {
            if (ron > 0) {
                if (rod == 0 && roc == 0) { location = 0; break; }
                roc = rod; edge = dprev;
            } else if (roc == 0 && right_of(vp[dst(onext)].x, vp[dst(onext)].y, edge) >= 0) {
                edge ^= 2;
            } else {
                roc = ron; edge = onext;
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
    int loc = locate(x, y, curr_edge, curr_point);
    if (loc < 0) return false;        // PTLOC_ERROR (CV_StsBadSize) / outside rect (CV_StsOutOfRange)
    if (loc == 1) return true;        // existing vertex: nothing inserted
    if (loc == 2) {
        int deleted = curr_edge;
        recent = curr_edge = get_e(curr_edge, PREV_AROUND_ORG);
        delete_edge(deleted);
    }
    if (curr_edge == 0) return false;  // CV_Assert
    curr_point = new_point(x, y, 0);
    int base = new_edge();
    const int first_point = org(curr_edge);
    set_pts(base, first_point, curr_point);
    splice(base, curr_edge);
    do {
        base = connect(curr_edge, base ^ 2);
        curr_edge = get_e(base, PREV_AROUND_ORG);
    } while (dst(curr_edge) != first_point);
    curr_edge = get_e(base, PREV_AROUND_ORG);
    const int max_edges = (int)qe.size() * 4;
    // Swap loop with the predicates written out on exact double copies of the float coordinates
    // (the float -> double conversions are exact, so every product and sum rounds as in
    // triangleArea / isPtInCircle3, and |p|^2 is formed once per vertex in the same order).
    const V2d P = vd[curr_point];
    auto area = [](const V2d &a, const V2d &b, const V2d &c) { return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x); };
    for (int i = 0; i < max_edges; i++) {
        int temp = get_e(curr_edge, PREV_AROUND_ORG);
        int tdst = dst(temp), corg = org(curr_edge), cdst = dst(curr_edge);
        const V2d T = vd[tdst], O = vd[corg], D = vd[cdst];
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
            curr_edge = get_e(curr_edge, PREV_AROUND_ORG);
        } else if (corg == first_point) {
            break;
        } else {
            curr_edge = get_e(next_e(curr_edge), 0x20 /* PREV_AROUND_LEFT */);
        }
    }
    return true;
}

// calcVoronoi: quad-edges from #4 (#0 is NULL, #1-#3 the outer triangle); the first quad-edge
// touching a triangle computes its circumcentre (pt[3] = left face, pt[1] = right face).
void Subdiv2D::calc_voronoi() {
    const int total = (int)qe.size();
    for (int q = 0; q < total; ++q) qe[q].pt[1] = qe[q].pt[3] = 0;
    for (size_t i = 0; i < vp.size(); ++i)
        if (vtype[i] > 0) { vfirst[i] = free_p; vtype[i] = -1; free_p = (int)i; }
    for (int q = 4; q < total; q++) {
        if (qe[q].next[0] <= 0) continue;  // free
        const int e0 = q * 4;
        if (!qe[q].pt[3]) {
            int e1 = get_e(e0, NEXT_AROUND_LEFT), e2 = get_e(e1, NEXT_AROUND_LEFT);
            const V2f a = vp[org(e0)], b = vp[dst(e0)], c = vp[org(e1)], d = vp[dst(e1)];
            float rx, ry;
            if (voronoi_point(a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y, rx, ry)) {
                int p = new_point(rx, ry, 1);
                qe[q].pt[3] = qe[e1 >> 2].pt[3 - (e1 & 2)] = qe[e2 >> 2].pt[3 - (e2 & 2)] = p;
            }
        }
        if (!qe[q].pt[1]) {
            int e1 = get_e(e0, NEXT_AROUND_RIGHT), e2 = get_e(e1, NEXT_AROUND_RIGHT);
            const V2f a = vp[org(e0)], b = vp[dst(e0)], c = vp[org(e1)], d = vp[dst(e1)];
            float rx, ry;
            if (voronoi_point(a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y, rx, ry)) {
                int p = new_point(rx, ry, 1);
                qe[q].pt[1] = qe[e1 >> 2].pt[1 + (e1 & 2)] = qe[e2 >> 2].pt[1 + (e2 & 2)] = p;
            }
        }
    }
}

void Subdiv2D::voronoi_edges(std::vector<float> &edges) {
    calc_voronoi();
    edges.clear();
    std::vector<int> facet;
    const size_t total = vp.size();
    for (size_t k = 4; k < total; k++) {
        if (vtype[k] != 0) continue;  // free or virtual
        const int start = rot(vfirst[k], 1);
        int t = start;
        facet.clear();
        do {
            facet.push_back(org(t));   // vtx[edgeOrg(t)] (index 0 = the (0,0) NULL vertex)
            t = get_e(t, NEXT_AROUND_LEFT);
        } while (t != start);
        const size_t n = facet.size();
        if (n < 2) continue;
        for (size_t i = 0; i < n; ++i) {
            int a = facet[i], b = facet[(i + 1) % n];
            edges.push_back(vp[a].x); edges.push_back(vp[a].y); edges.push_back(vp[b].x); edges.push_back(vp[b].y);
        }
    }
}

}  // namespace aos
