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
// isPtInCircle3, eps = FLT_EPSILON / 8
inline int in_circle(float px, float py, float ax, float ay, float bx, float by, float cx, float cy) {
    const double eps = FLT_EPSILON * 0.125;
    double val = ((double)ax * ax + (double)ay * ay) * tri_area(bx, by, cx, cy, px, py);
    val -= ((double)bx * bx + (double)by * by) * tri_area(ax, ay, cx, cy, px, py);
    val += ((double)cx * cx + (double)cy * cy) * tri_area(ax, ay, bx, by, px, py);
    val -= ((double)px * px + (double)py * py) * tri_area(ax, ay, bx, by, cx, cy);
    return val > eps ? 1 : val < -eps ? -1 : 0;
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

int Subdiv2D::right_of(float px, float py, int e) const {
    int o = org(e), d = dst(e);
    double cw = tri_area(px, py, vx[d], vy[d], vx[o], vy[o]);
    return (cw > 0) - (cw < 0);
}

int Subdiv2D::new_edge() {
    if (free_q <= 0) {
        qnext.resize(qnext.size() + 4, 0);
        qpt.resize(qpt.size() + 4, 0);
        free_q = (int)(qnext.size() / 4) - 1;
    }
    int e = free_q * 4;
    free_q = qnext[e + 1];
    qnext[e] = e; qnext[e + 1] = e + 3; qnext[e + 2] = e + 2; qnext[e + 3] = e + 1;
    qpt[e] = qpt[e + 1] = qpt[e + 2] = qpt[e + 3] = 0;
    return e;
}

int Subdiv2D::new_point(float x, float y, int type) {
    if (free_p == 0) {
        vx.push_back(0.f); vy.push_back(0.f); vfirst.push_back(0); vtype.push_back(-1);
        free_p = (int)vx.size() - 1;
    }
    int v = free_p;
    free_p = vfirst[v];
    vx[v] = x; vy[v] = y; vfirst[v] = 0; vtype[v] = type;
    return v;
}

void Subdiv2D::splice(int a, int b) {
    int &an = qnext[a], &bn = qnext[b];
    int ar = rot(an, 1), br = rot(bn, 1);
    int &arn = qnext[ar], &brn = qnext[br];
    std::swap(an, bn);
    std::swap(arn, brn);
}

void Subdiv2D::set_pts(int e, int o, int d) {
    qpt[e] = o;
    qpt[(e & ~3) + ((e + 2) & 3)] = d;
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
    qnext[4 * q] = 0;
    qnext[4 * q + 1] = free_q;
    free_q = q;
}

void Subdiv2D::init_delaunay(float rx, float ry, float rw, float rh, int rect_mode) {
    if (rect_mode == 1) {  // Rect_<float> -> Rect_<int>: saturate_cast<int> = cvRound (nearest even)
        rx = (float)(int)std::lrint(rx); ry = (float)(int)std::lrint(ry);
        rw = (float)(int)std::lrint(rw); rh = (float)(int)std::lrint(rh);
    }
    const float big = 3.f * std::max(rw, rh);
    vx.clear(); vy.clear(); vfirst.clear(); vtype.clear(); qnext.clear(); qpt.clear();
    recent = 0;
    tlx = rx; tly = ry; brx = rx + rw; bry = ry + rh;
    vx.push_back(0.f); vy.push_back(0.f); vfirst.push_back(0); vtype.push_back(-1);   // vtx[0]
    qnext.assign(4, 0); qpt.assign(4, 0);                                             // qedges[0]
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
    const int max_edges = (int)qnext.size();  // qedges.size() * 4
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
            } else if (roc == 0 && right_of(vx[dst(onext)], vy[dst(onext)], edge) >= 0) {
                edge ^= 2;
            } else {
                roc = ron; edge = onext;
            }
        }
    }
    recent = edge;
    if (location == 0) {
        const int o = org(edge), d = dst(edge);
        const float ox = vx[o], oy = vy[o], dx = vx[d], dy = vy[d];
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
    const int max_edges = (int)qnext.size();
    for (int i = 0; i < max_edges; i++) {
        int temp = get_e(curr_edge, PREV_AROUND_ORG);
        int tdst = dst(temp), corg = org(curr_edge), cdst = dst(curr_edge);
        if (right_of(vx[tdst], vy[tdst], curr_edge) > 0 &&
            // isPtInCircle3(pt = org, a = temp_dst, b = dst, c = new point)
            in_circle(vx[corg], vy[corg], vx[tdst], vy[tdst], vx[cdst], vy[cdst], vx[curr_point], vy[curr_point]) < 0) {
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
    const int total = (int)(qnext.size() / 4);
    for (int q = 0; q < total; ++q) qpt[4 * q + 1] = qpt[4 * q + 3] = 0;
    for (size_t i = 0; i < vx.size(); ++i)
        if (vtype[i] > 0) { vfirst[i] = free_p; vtype[i] = -1; free_p = (int)i; }
    for (int q = 4; q < total; q++) {
        if (qnext[4 * q] <= 0) continue;  // free
        const int e0 = q * 4;
        if (!qpt[e0 + 3]) {
            int e1 = get_e(e0, NEXT_AROUND_LEFT), e2 = get_e(e1, NEXT_AROUND_LEFT);
            float rx, ry;
            if (voronoi_point(vx[org(e0)], vy[org(e0)], vx[dst(e0)], vy[dst(e0)], vx[org(e1)], vy[org(e1)], vx[dst(e1)],
                              vy[dst(e1)], rx, ry)) {
                int p = new_point(rx, ry, 1);
                qpt[e0 + 3] = qpt[(e1 & ~3) + 3 - (e1 & 2)] = qpt[(e2 & ~3) + 3 - (e2 & 2)] = p;
            }
        }
        if (!qpt[e0 + 1]) {
            int e1 = get_e(e0, NEXT_AROUND_RIGHT), e2 = get_e(e1, NEXT_AROUND_RIGHT);
            float rx, ry;
            if (voronoi_point(vx[org(e0)], vy[org(e0)], vx[dst(e0)], vy[dst(e0)], vx[org(e1)], vy[org(e1)], vx[dst(e1)],
                              vy[dst(e1)], rx, ry)) {
                int p = new_point(rx, ry, 1);
                qpt[e0 + 1] = qpt[(e1 & ~3) + 1 + (e1 & 2)] = qpt[(e2 & ~3) + 1 + (e2 & 2)] = p;
            }
        }
    }
}

void Subdiv2D::voronoi_edges(std::vector<float> &edges) {
    calc_voronoi();
    edges.clear();
    std::vector<int> facet;
    const size_t total = vx.size();
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
            edges.push_back(vx[a]); edges.push_back(vy[a]); edges.push_back(vx[b]); edges.push_back(vy[b]);
        }
    }
}

}  // namespace aos
