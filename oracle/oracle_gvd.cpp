// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). Build: g++ -O2 -ffp-contract=off.
// CPU restatement of aos_gvd_node (reference src/aos_gvd_node.cpp) and aos::VoronoiDiagram
// (src/utils/voronoi_diagram.cpp), including a restatement of OpenCV 4.5.4 cv::Subdiv2D
// (modules/imgproc/src/subdivision2d.cpp; not vendored in the reference, NOTES.md §5).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>
#include <set>
#include <unordered_set>

#include "oracle_internal.h"

namespace orc {

// =============================================================== cv::Subdiv2D restatement
namespace {
struct P2f { float x, y; };

class Subdiv {
  public:
    enum { PTLOC_ERROR = -2, PTLOC_OUTSIDE_RECT = -1, PTLOC_INSIDE = 0, PTLOC_VERTEX = 1, PTLOC_ON_EDGE = 2 };
    enum { NEXT_AROUND_ORG = 0x00, NEXT_AROUND_DST = 0x22, PREV_AROUND_ORG = 0x11, PREV_AROUND_DST = 0x33,
           NEXT_AROUND_LEFT = 0x13, NEXT_AROUND_RIGHT = 0x31, PREV_AROUND_LEFT = 0x20, PREV_AROUND_RIGHT = 0x02 };
    struct Vertex { int firstEdge = 0; int type = -1; P2f pt{0.f, 0.f}; bool isvirtual() const { return type > 0; } bool isfree() const { return type < 0; } };
    struct QuadEdge {
        int next[4] = {0, 0, 0, 0};
        int pt[4] = {0, 0, 0, 0};
        QuadEdge() {}
        explicit QuadEdge(int e) { next[0] = e; next[1] = e + 3; next[2] = e + 2; next[3] = e + 1; }
        bool isfree() const { return next[0] <= 0; }
    };
    std::vector<Vertex> vtx;
    std::vector<QuadEdge> qedges;
    int freeQEdge = 0, freePoint = 0, recentEdge = 0;
    bool validGeometry = false;
    P2f topLeft{0, 0}, bottomRight{0, 0};

    int nextEdge(int e) const { return qedges[e >> 2].next[e & 3]; }
    static int rotateEdge(int e, int r) { return (e & ~3) + ((e + r) & 3); }
    static int symEdge(int e) { return e ^ 2; }
    int getEdge(int e, int t) const {
        e = qedges[e >> 2].next[(e + t) & 3];
        return (e & ~3) + ((e + (t >> 4)) & 3);
    }
    int edgeOrg(int e, P2f *p = nullptr) const { int v = qedges[e >> 2].pt[e & 3]; if (p) *p = vtx[v].pt; return v; }
    int edgeDst(int e, P2f *p = nullptr) const { int v = qedges[e >> 2].pt[(e + 2) & 3]; if (p) *p = vtx[v].pt; return v; }

    static double triangleArea(P2f a, P2f b, P2f c) {
        return ((double)b.x - a.x) * ((double)c.y - a.y) - ((double)b.y - a.y) * ((double)c.x - a.x);
    }
    int isRightOf(P2f pt, int edge) const {
        P2f org, dst;
        edgeOrg(edge, &org); edgeDst(edge, &dst);
        double cw = triangleArea(pt, dst, org);
        return (cw > 0) - (cw < 0);
    }
    static int isPtInCircle3(P2f pt, P2f a, P2f b, P2f c) {
        const double eps = FLT_EPSILON * 0.125;
        double val = ((double)a.x * a.x + (double)a.y * a.y) * triangleArea(b, c, pt);
        val -= ((double)b.x * b.x + (double)b.y * b.y) * triangleArea(a, c, pt);
        val += ((double)c.x * c.x + (double)c.y * c.y) * triangleArea(a, b, pt);
        val -= ((double)pt.x * pt.x + (double)pt.y * pt.y) * triangleArea(a, b, c);
        return val > eps ? 1 : val < -eps ? -1 : 0;
    }

    int newEdge() {
        if (freeQEdge <= 0) { qedges.push_back(QuadEdge()); freeQEdge = (int)(qedges.size() - 1); }
        int edge = freeQEdge * 4;
        freeQEdge = qedges[edge >> 2].next[1];
        qedges[edge >> 2] = QuadEdge(edge);
        return edge;
    }
    void splice(int a, int b) {
        int &a_next = qedges[a >> 2].next[a & 3];
        int &b_next = qedges[b >> 2].next[b & 3];
        int a_rot = rotateEdge(a_next, 1), b_rot = rotateEdge(b_next, 1);
        int &a_rot_next = qedges[a_rot >> 2].next[a_rot & 3];
        int &b_rot_next = qedges[b_rot >> 2].next[b_rot & 3];
        std::swap(a_next, b_next);
        std::swap(a_rot_next, b_rot_next);
    }
    void deleteEdge(int edge) {
        splice(edge, getEdge(edge, PREV_AROUND_ORG));
        int sedge = symEdge(edge);
        splice(sedge, getEdge(sedge, PREV_AROUND_ORG));
        edge >>= 2;
        qedges[edge].next[0] = 0;
        qedges[edge].next[1] = freeQEdge;
        freeQEdge = edge;
    }
    int newPoint(P2f pt, bool isvirtual, int firstEdge = 0) {
        if (freePoint == 0) { vtx.push_back(Vertex()); freePoint = (int)(vtx.size() - 1); }
        int vidx = freePoint;
        freePoint = vtx[vidx].firstEdge;
        vtx[vidx].firstEdge = firstEdge; vtx[vidx].type = (int)isvirtual; vtx[vidx].pt = pt;
        return vidx;
    }
    void deletePoint(int vidx) { vtx[vidx].firstEdge = freePoint; vtx[vidx].type = -1; freePoint = vidx; }
    void setEdgePoints(int edge, int o, int d) {
        qedges[edge >> 2].pt[edge & 3] = o;
        qedges[edge >> 2].pt[(edge + 2) & 3] = d;
        vtx[o].firstEdge = edge;
        vtx[d].firstEdge = edge ^ 2;
    }
    int connectEdges(int a, int b) {
        int edge = newEdge();
        splice(edge, getEdge(a, NEXT_AROUND_LEFT));
        splice(symEdge(edge), b);
        setEdgePoints(edge, edgeDst(a), edgeOrg(b));
        return edge;
    }
    void swapEdges(int edge) {
        int sedge = symEdge(edge);
        int a = getEdge(edge, PREV_AROUND_ORG);
        int b = getEdge(sedge, PREV_AROUND_ORG);
        splice(edge, a);
        splice(sedge, b);
        setEdgePoints(edge, edgeDst(a), edgeDst(b));
        splice(edge, getEdge(a, NEXT_AROUND_LEFT));
        splice(sedge, getEdge(b, NEXT_AROUND_LEFT));
    }

    // initDelaunay(Rect2f) / initDelaunay(Rect)
    void init(float rx, float ry, float rw, float rh) {
        float big_coord = 3.f * std::max(rw, rh);
        vtx.clear(); qedges.clear();
        recentEdge = 0; validGeometry = false;
        topLeft = P2f{rx, ry};
        bottomRight = P2f{rx + rw, ry + rh};
        P2f ppA{rx + big_coord, ry}, ppB{rx, ry + big_coord}, ppC{rx - big_coord, ry - big_coord};
        vtx.push_back(Vertex());
        qedges.push_back(QuadEdge());
        freeQEdge = 0; freePoint = 0;
        int pA = newPoint(ppA, false), pB = newPoint(ppB, false), pC = newPoint(ppC, false);
        int eAB = newEdge(), eBC = newEdge(), eCA = newEdge();
        setEdgePoints(eAB, pA, pB); setEdgePoints(eBC, pB, pC); setEdgePoints(eCA, pC, pA);
        splice(eAB, symEdge(eCA)); splice(eBC, symEdge(eAB)); splice(eCA, symEdge(eBC));
        recentEdge = eAB;
    }

    // returns location; throws are modelled by PTLOC_ERROR / OUTSIDE (caller skips the seed)
    int locate(P2f pt, int &_edge, int &_vertex) {
        int vertex = 0;
        int maxEdges = (int)(qedges.size() * 4);
        if (pt.x < topLeft.x || pt.y < topLeft.y || pt.x >= bottomRight.x || pt.y >= bottomRight.y) return PTLOC_OUTSIDE_RECT;
        int edge = recentEdge;
        int location = PTLOC_ERROR;
        int right_of_curr = isRightOf(pt, edge);
        if (right_of_curr > 0) { edge = symEdge(edge); right_of_curr = -right_of_curr; }
        for (int i = 0; i < maxEdges; i++) {
            int onext_edge = nextEdge(edge);
            int dprev_edge = getEdge(edge, PREV_AROUND_DST);
            int right_of_onext = isRightOf(pt, onext_edge);
            int right_of_dprev = isRightOf(pt, dprev_edge);
            if (right_of_dprev > 0) {
                if (right_of_onext > 0 || (right_of_onext == 0 && right_of_curr == 0)) { location = PTLOC_INSIDE; break; }
                else { right_of_curr = right_of_onext; edge = onext_edge; }
            } else {
                if (right_of_onext > 0) {
                    if (right_of_dprev == 0 && right_of_curr == 0) { location = PTLOC_INSIDE; break; }
                    else { right_of_curr = right_of_dprev; edge = dprev_edge; }
                } else if (right_of_curr == 0 && isRightOf(vtx[edgeDst(onext_edge)].pt, edge) >= 0) {
                    edge = symEdge(edge);
                } else { right_of_curr = right_of_onext; edge = onext_edge; }
            }
        }
        recentEdge = edge;
        if (location == PTLOC_INSIDE) {
            P2f org_pt, dst_pt;
            edgeOrg(edge, &org_pt); edgeDst(edge, &dst_pt);
            double t1 = std::fabs(pt.x - org_pt.x); t1 += std::fabs(pt.y - org_pt.y);
            double t2 = std::fabs(pt.x - dst_pt.x); t2 += std::fabs(pt.y - dst_pt.y);
            double t3 = std::fabs(org_pt.x - dst_pt.x); t3 += std::fabs(org_pt.y - dst_pt.y);
            if (t1 < FLT_EPSILON) { location = PTLOC_VERTEX; vertex = edgeOrg(edge); edge = 0; }
            else if (t2 < FLT_EPSILON) { location = PTLOC_VERTEX; vertex = edgeDst(edge); edge = 0; }
            else if ((t1 < t3 || t2 < t3) && std::fabs(triangleArea(pt, org_pt, dst_pt)) < FLT_EPSILON) { location = PTLOC_ON_EDGE; vertex = 0; }
        }
        if (location == PTLOC_ERROR) { edge = 0; vertex = 0; }
        _edge = edge; _vertex = vertex;
        return location;
    }

    // insert(Point2f); returns false where OpenCV throws (the reference catches and skips)
    bool insert(P2f pt) {
        int curr_point = 0, curr_edge = 0, deleted_edge = 0;
        int location = locate(pt, curr_edge, curr_point);
        if (location == PTLOC_ERROR || location == PTLOC_OUTSIDE_RECT) return false;
        if (location == PTLOC_VERTEX) return true;
        if (location == PTLOC_ON_EDGE) {
            deleted_edge = curr_edge;
            recentEdge = curr_edge = getEdge(curr_edge, PREV_AROUND_ORG);
            deleteEdge(deleted_edge);
        }
        if (curr_edge == 0) return false;  // CV_Assert
        validGeometry = false;
        curr_point = newPoint(pt, false);
        int base_edge = newEdge();
        int first_point = edgeOrg(curr_edge);
        setEdgePoints(base_edge, first_point, curr_point);
        splice(base_edge, curr_edge);
        do {
            base_edge = connectEdges(curr_edge, symEdge(base_edge));
            curr_edge = getEdge(base_edge, PREV_AROUND_ORG);
        } while (edgeDst(curr_edge) != first_point);
        curr_edge = getEdge(base_edge, PREV_AROUND_ORG);
        int max_edges = (int)(qedges.size() * 4);
        for (int i = 0; i < max_edges; i++) {
            int temp_edge = getEdge(curr_edge, PREV_AROUND_ORG);
            int temp_dst = edgeDst(temp_edge), curr_org = edgeOrg(curr_edge), curr_dst = edgeDst(curr_edge);
            if (isRightOf(vtx[temp_dst].pt, curr_edge) > 0 &&
                isPtInCircle3(vtx[curr_org].pt, vtx[temp_dst].pt, vtx[curr_dst].pt, vtx[curr_point].pt) < 0) {
                swapEdges(curr_edge);
                curr_edge = getEdge(curr_edge, PREV_AROUND_ORG);
            } else if (curr_org == first_point) {
                break;
            } else {
                curr_edge = getEdge(nextEdge(curr_edge), PREV_AROUND_LEFT);
            }
        }
        return true;
    }

    static P2f computeVoronoiPoint(P2f org0, P2f dst0, P2f org1, P2f dst1) {
        double a0 = dst0.x - org0.x;
        double b0 = dst0.y - org0.y;
        double c0 = -0.5 * (a0 * (dst0.x + org0.x) + b0 * (dst0.y + org0.y));
        double a1 = dst1.x - org1.x;
        double b1 = dst1.y - org1.y;
        double c1 = -0.5 * (a1 * (dst1.x + org1.x) + b1 * (dst1.y + org1.y));
        double det = a0 * b1 - a1 * b0;
        if (det != 0) {
            det = 1. / det;
            return P2f{(float)((b0 * c1 - b1 * c0) * det), (float)((a1 * c0 - a0 * c1) * det)};
        }
        return P2f{FLT_MAX, FLT_MAX};
    }
    void clearVoronoi() {
        for (auto &q : qedges) q.pt[1] = q.pt[3] = 0;
        for (size_t i = 0; i < vtx.size(); i++) if (vtx[i].isvirtual()) deletePoint((int)i);
        validGeometry = false;
    }
    void calcVoronoi() {
        if (validGeometry) return;
        clearVoronoi();
        int total = (int)qedges.size();
        for (int i = 4; i < total; i++) {
            QuadEdge &quadedge = qedges[i];
            if (quadedge.isfree()) continue;
            int edge0 = i * 4;
            P2f org0, dst0, org1, dst1;
            if (!quadedge.pt[3]) {
                int edge1 = getEdge(edge0, NEXT_AROUND_LEFT);
                int edge2 = getEdge(edge1, NEXT_AROUND_LEFT);
                edgeOrg(edge0, &org0); edgeDst(edge0, &dst0); edgeOrg(edge1, &org1); edgeDst(edge1, &dst1);
                P2f vp = computeVoronoiPoint(org0, dst0, org1, dst1);
                if (std::abs(vp.x) < FLT_MAX * 0.5 && std::abs(vp.y) < FLT_MAX * 0.5) {
                    int np = newPoint(vp, true);
                    qedges[i].pt[3] = qedges[edge1 >> 2].pt[3 - (edge1 & 2)] = qedges[edge2 >> 2].pt[3 - (edge2 & 2)] = np;
                }
            }
            if (!qedges[i].pt[1]) {
                int edge1 = getEdge(edge0, NEXT_AROUND_RIGHT);
                int edge2 = getEdge(edge1, NEXT_AROUND_RIGHT);
                edgeOrg(edge0, &org0); edgeDst(edge0, &dst0); edgeOrg(edge1, &org1); edgeDst(edge1, &dst1);
                P2f vp = computeVoronoiPoint(org0, dst0, org1, dst1);
                if (std::abs(vp.x) < FLT_MAX * 0.5 && std::abs(vp.y) < FLT_MAX * 0.5) {
                    int np = newPoint(vp, true);
                    qedges[i].pt[1] = qedges[edge1 >> 2].pt[1 + (edge1 & 2)] = qedges[edge2 >> 2].pt[1 + (edge2 & 2)] = np;
                }
            }
        }
        validGeometry = true;
    }
    void getVoronoiFacetList(Facets &out) {
        calcVoronoi();
        out.facets.clear(); out.centers.clear();
        size_t total = vtx.size();
        for (size_t k = 4; k < total; k++) {
            if (vtx[k].isfree() || vtx[k].isvirtual()) continue;
            int edge = rotateEdge(vtx[k].firstEdge, 1), t = edge;
            std::vector<std::pair<float, float>> buf;
            do {
                P2f p = vtx[edgeOrg(t)].pt;
                buf.push_back({p.x, p.y});
                t = getEdge(t, NEXT_AROUND_LEFT);
            } while (t != edge);
            out.facets.push_back(std::move(buf));
            out.centers.push_back({vtx[k].pt.x, vtx[k].pt.y});
        }
    }
};

static inline int cv_round(float v) { return (int)std::lrint(v); }
}  // namespace

// Test hook (known-answer tests, tests/test_subdiv_host.py): a Subdiv2D on the rectangle as given
// (mode 1: the implicit Rect2f -> Rect conversion), the points inserted in order, then the raw state in
// OpenCV's layout: per quad-edge next[4] + pt[4] (before calcVoronoi: pt[1] = pt[3] = 0), per vertex
// firstEdge / type / point, and getVoronoiFacetList's facets (which runs calcVoronoi).
void subdiv_raw_state(const float *xy, int n, const float rect[4], int rect_mode, std::vector<int> &qe,
                      std::vector<int> &vfirst, std::vector<int> &vtype, std::vector<float> &vxy, Facets &facets,
                      std::vector<int> &inserted) {
    Subdiv sd;
    float rx = rect[0], ry = rect[1], rw = rect[2], rh = rect[3];
    if (rect_mode == 1) { rx = (float)cv_round(rx); ry = (float)cv_round(ry); rw = (float)cv_round(rw); rh = (float)cv_round(rh); }
    sd.init(rx, ry, rw, rh);
    inserted.clear();
    for (int i = 0; i < n; ++i) inserted.push_back(sd.insert(P2f{xy[2 * i], xy[2 * i + 1]}) ? 1 : 0);
    auto dump = [&]() {
        qe.clear(); vfirst.clear(); vtype.clear(); vxy.clear();
        for (const auto &q : sd.qedges)
            for (int k = 0; k < 4; ++k) qe.push_back(q.next[k]);
        for (size_t i = 0; i < sd.qedges.size(); ++i)
            for (int k = 0; k < 4; ++k) qe.push_back(sd.qedges[i].pt[k]);
        for (const auto &v : sd.vtx) { vfirst.push_back(v.firstEdge); vtype.push_back(v.type); vxy.push_back(v.pt.x); vxy.push_back(v.pt.y); }
    };
    dump();   // the insert state (no Voronoi points)
    sd.getVoronoiFacetList(facets);
}

// VoronoiDiagram::compute voronoi_diagram.cpp:16-94 up to the facet list
void subdiv_voronoi_facets(const std::vector<V2> &seeds, double min_x, double max_x, double min_y, double max_y,
                           int rect_mode, Facets &out, float *rect_out) {
    out.facets.clear(); out.centers.clear();
    if (seeds.empty()) return;
    if (!std::isfinite(min_x) || !std::isfinite(max_x) || !std::isfinite(min_y) || !std::isfinite(max_y)) return;
    if (min_x > max_x) std::swap(min_x, max_x);
    if (min_y > max_y) std::swap(min_y, max_y);
    const double min_size = 1.0;
    if (max_x - min_x < min_size) { double c = (min_x + max_x) / 2.0; min_x = c - min_size / 2.0; max_x = c + min_size / 2.0; }
    if (max_y - min_y < min_size) { double c = (min_y + max_y) / 2.0; min_y = c - min_size / 2.0; max_y = c + min_size / 2.0; }
    float rx = static_cast<float>(min_x - 1.0), ry = static_cast<float>(min_y - 1.0);
    float rw = static_cast<float>(std::abs(max_x - min_x) + 2.0), rh = static_cast<float>(std::abs(max_y - min_y) + 2.0);
    if (rect_out) { rect_out[0] = rx; rect_out[1] = ry; rect_out[2] = rw; rect_out[3] = rh; }
    if (rw <= 0 || rh <= 0) return;
    Subdiv sd;
    if (rect_mode == 1) {  // implicit Rect2f -> Rect (saturate_cast<int> = cvRound)
        int ix = cv_round(rx), iy = cv_round(ry), iw = cv_round(rw), ih = cv_round(rh);
        sd.init((float)ix, (float)iy, (float)iw, (float)ih);
    } else {
        sd.init(rx, ry, rw, rh);
    }
    for (const auto &s : seeds) {
        if (!std::isfinite(s.x) || !std::isfinite(s.y)) continue;
        float x = static_cast<float>(s.x), y = static_cast<float>(s.y);
        const float margin = 0.1f;
        x = std::max(rx + margin, std::min(rx + rw - margin, x));
        y = std::max(ry + margin, std::min(ry + rh - margin, y));
        sd.insert(P2f{x, y});
    }
    sd.getVoronoiFacetList(out);
}

void voronoi_compute(const std::vector<V2> &seeds, double min_x, double max_x, double min_y, double max_y, int rect_mode,
                     bool dead_work, std::vector<VEdge> &edges, int &n_vertices) {
    edges.clear();
    n_vertices = 0;
    Facets f;
    subdiv_voronoi_facets(seeds, min_x, max_x, min_y, max_y, rect_mode, f);
    for (const auto &facet : f.facets) {  // voronoi_diagram.cpp:97-114
        if (facet.size() < 2) continue;
        for (size_t i = 0; i < facet.size(); ++i) {
            size_t ni = (i + 1) % facet.size();
            edges.push_back(VEdge{V2{facet[i].first, facet[i].second}, V2{facet[ni].first, facet[ni].second}});
        }
    }
    if (dead_work) {  // voronoi_diagram.cpp:117-146 (result never read by the GVD node)
        std::vector<V2> vs;
        const double th = 0.01;
        for (const auto &e : edges) {
            bool sf = false;
            for (auto &v : vs) if (norm(v - e.start) < th) { sf = true; break; }
            if (!sf) vs.push_back(e.start);
            bool ef = false;
            for (auto &v : vs) if (norm(v - e.end) < th) { ef = true; break; }
            if (!ef) vs.push_back(e.end);
        }
        n_vertices = (int)vs.size();
    }
}

// VoronoiDiagram::extractCellBoundaries voronoi_diagram.cpp:209-311: a second Subdiv2D over the
// seeds' own bounding box; cell i = facet i (i < seeds, facets) with >= 3 points, closed when its
// ends are more than 1 cm apart. publishMarkers (gvd:1098-1194) pairs cell i with seeds_[i] and
// colours it from hue = i / max(1, cells) (HSV, s = 0.7, v = 0.9, alpha 0.4), all in float.
static void cell_markers(const std::vector<V2> &seeds, int rect_mode, GvdResult &R) {
    R.cell_off.assign(1, 0);
    if (seeds.empty()) return;
    double min_x = std::numeric_limits<double>::max(), max_x = std::numeric_limits<double>::lowest();
    double min_y = std::numeric_limits<double>::max(), max_y = std::numeric_limits<double>::lowest();
    for (const auto &s : seeds)
        if (std::isfinite(s.x) && std::isfinite(s.y)) {
            min_x = std::min(min_x, s.x); max_x = std::max(max_x, s.x);
            min_y = std::min(min_y, s.y); max_y = std::max(max_y, s.y);
        }
    if (min_x > max_x || min_y > max_y) return;
    Facets f;
    subdiv_voronoi_facets(seeds, min_x, max_x, min_y, max_y, rect_mode, f);   // same rect rules as compute()
    std::vector<std::vector<V2>> cells;
    for (size_t i = 0; i < seeds.size() && i < f.facets.size(); ++i) {
        std::vector<V2> cp;
        for (const auto &pt : f.facets[i]) cp.push_back(V2{pt.first, pt.second});
        if (cp.size() >= 3) {
            if (norm(cp.front() - cp.back()) > 0.01) cp.push_back(cp.front());
            cells.push_back(cp);
        }
    }
    for (size_t i = 0; i < cells.size(); ++i) {
        for (const auto &v : cells[i]) { R.cell_xy.push_back(v.x); R.cell_xy.push_back(v.y); }
        R.cell_off.push_back((int32_t)(R.cell_xy.size() / 2));
        R.cell_center.push_back(seeds[i].x); R.cell_center.push_back(seeds[i].y);
        float hue = static_cast<float>(i) / std::max(1.0f, static_cast<float>(cells.size()));
        float saturation = 0.7f, value = 0.9f;
        float c = value * saturation;
        float x = c * (1.0f - std::abs(std::fmod(hue * 6.0f, 2.0f) - 1.0f));
        float m = value - c;
        float r = 0.0f, g = 0.0f, b = 0.0f;
        if (hue < 1.0f / 6.0f) { r = c; g = x; b = 0.0f; }
        else if (hue < 2.0f / 6.0f) { r = x; g = c; b = 0.0f; }
        else if (hue < 3.0f / 6.0f) { r = 0.0f; g = c; b = x; }
        else if (hue < 4.0f / 6.0f) { r = 0.0f; g = x; b = c; }
        else if (hue < 5.0f / 6.0f) { r = x; g = 0.0f; b = c; }
        else { r = c; g = 0.0f; b = x; }
        R.cell_rgba.push_back(r + m); R.cell_rgba.push_back(g + m); R.cell_rgba.push_back(b + m); R.cell_rgba.push_back(0.4f);
    }
}

// extractBoundaryPoints voronoi_diagram.cpp:149-207
static std::vector<V2> extract_boundary_points(const std::vector<VEdge> &edges) {
    std::vector<V2> bp;
    std::set<std::pair<int, int>> keys;
    const double threshold = 0.05;
    auto consider = [&](V2 p) {
        int ix = static_cast<int>(p.x * 100), iy = static_cast<int>(p.y * 100);
        std::pair<int, int> key{ix, iy};
        if (keys.find(key) != keys.end()) return;
        for (const auto &e : bp) {
            double dx = e.x - p.x, dy = e.y - p.y;
            if (dx * dx + dy * dy < threshold * threshold) return;
        }
        keys.insert(key);
        bp.push_back(p);
    };
    for (const auto &e : edges) { consider(e.start); consider(e.end); }
    return bp;
}

namespace {
struct GridView {
    GridInfo gi; const int8_t *data;
    double minx() const { return gi.origin_x; }
    double maxx() const { return gi.origin_x + gi.width * gi.resolution; }
    double miny() const { return gi.origin_y; }
    double maxy() const { return gi.origin_y + gi.height * gi.resolution; }
    bool occupied_trunc(V2 p) const {
        const double resolution = gi.resolution;
        int mx = static_cast<int>((p.x - gi.origin_x) / resolution);
        int my = static_cast<int>((p.y - gi.origin_y) / resolution);
        if (mx >= 0 && mx < (int)gi.width && my >= 0 && my < (int)gi.height) return data[mx + my * (int)gi.width] == 100;
        return false;
    }
};
}  // namespace

// edgePassesThroughOccupiedPixels gvd:320-359
static bool edge_through_occupied(const GridView &g, V2 start, V2 end) {
    const double resolution = g.gi.resolution;
    double edge_length = norm(end - start);
    if (edge_length < 1e-6) return false;
    const double sample_step = resolution * 0.5;
    int num_samples = static_cast<int>(edge_length / sample_step) + 1;
    V2 dir = normalized(end - start);
    for (int i = 0; i <= num_samples; ++i) {
        double t = (i == num_samples) ? 1.0 : (static_cast<double>(i) / static_cast<double>(num_samples));
        V2 sp = start + (t * dir) * edge_length;
        if (g.occupied_trunc(sp)) return true;
    }
    return false;
}

// castRay gvd:558-684
static V2 cast_ray(const GridView &g, V2 start_point, V2 other, double angle_offset_deg, double min_distance) {
    V2 e2o = other - start_point;
    double d = norm(e2o);
    if (d < 1e-6) e2o = V2{1.0, 0.0}; else e2o = normalized(e2o);
    V2 outward = -e2o;
    V2 perp{-e2o.y, e2o.x};
    double a = angle_offset_deg * M_PI / 180.0;
    V2 ray;
    if (angle_offset_deg > 0) ray = lib_cos(a) * outward + lib_sin(a) * perp;
    else ray = lib_cos(-a) * outward + lib_sin(-a) * (-perp);
    ray = normalized(ray);
    auto inside = [&](V2 p) { return p.x >= g.minx() && p.x <= g.maxx() && p.y >= g.miny() && p.y <= g.maxy(); };
    double step_size = g.gi.resolution * 0.5;
    if (step_size < 0.01) step_size = 0.01;
    double current = min_distance;
    double gw = g.gi.width * g.gi.resolution, gh = g.gi.height * g.gi.resolution;
    double amax = std::sqrt(gw * gw + gh * gh) * 3.0;
    while (current <= amax) {
        V2 cp = start_point + ray * current;
        if (!inside(cp)) return V2{std::max(g.minx(), std::min(g.maxx(), cp.x)), std::max(g.miny(), std::min(g.maxy(), cp.y))};
        if (g.occupied_trunc(cp)) return cp;
        current += step_size;
    }
    V2 fp = start_point + ray * amax;
    if (!inside(fp)) { fp.x = std::max(g.minx(), std::min(g.maxx(), fp.x)); fp.y = std::max(g.miny(), std::min(g.maxy(), fp.y)); }
    return fp;
}

// findVoronoiBoundaryPointNearEndpoint gvd:686-790
static void find_label_point(const GridView &g, const std::vector<V2> &pts, V2 endpoint, V2 other, double target_deg,
                             V2 &point, bool &valid) {
    valid = false;
    const double min_distance = 0.5, max_distance = 5.0;
    V2 main_dir = other - endpoint;
    double ml = norm(main_dir);
    if (ml < 1e-6) main_dir = V2{1.0, 0.0}; else main_dir = normalized(main_dir);
    V2 outward = -main_dir;
    V2 perp{-main_dir.y, main_dir.x};
    const bool m90 = std::abs(target_deg - (-90.0)) < 1e-6, p90 = std::abs(target_deg - 90.0) < 1e-6;
    double gw = g.gi.width * g.gi.resolution, gh = g.gi.height * g.gi.resolution;
    double max_radius = std::sqrt(gw * gw + gh * gh) * 2.0;
    const double radii[4] = {max_distance, 7.0, 9.0, max_radius};
    for (double sr : radii) {
        std::vector<V2> cand;
        for (const auto &vp : pts) {
            V2 dir = vp - endpoint;
            double dist = norm(dir);
            if (dist < min_distance || dist > sr) continue;
            dir = normalized(dir);
            double dwo = dot(outward, dir);
            if (dwo < 0.0) continue;
            double dwp = dot(perp, dir);
            if (m90) { if (dwp > 0.0) continue; }
            else if (p90) { if (dwp < 0.0) continue; }
            cand.push_back(vp);
        }
        if (!cand.empty()) {
            double md = std::numeric_limits<double>::max();
            size_t mi = 0;
            for (size_t i = 0; i < cand.size(); ++i) {
                double dd = norm(cand[i] - endpoint);
                if (dd < md) { md = dd; mi = i; }
            }
            point = cand[mi];
            valid = true;
            return;
        }
    }
    point = cast_ray(g, endpoint, other, target_deg, min_distance);
    valid = true;
}

// processGraph gvd:255-318 on the settled state (all inputs from one seed-gen frame)
void gvd(const Params &P, const GvdInput &in, GvdResult &R) {
    R = GvdResult();
    // voronoiSeedsCallback gvd:84-128: greedy non-transitive merge within 0.5 m
    const size_t S = in.seeds.size();
    std::vector<bool> used(S, false);
    for (size_t i = 0; i < S; ++i) {
        if (used[i]) continue;
        std::vector<size_t> ci{i};
        used[i] = true;
        for (size_t j = i + 1; j < S; ++j) {
            if (used[j]) continue;
            if (norm(in.seeds[i] - in.seeds[j]) <= 0.5) { ci.push_back(j); used[j] = true; }
        }
        V2 m{0.0, 0.0};
        for (size_t idx : ci) m = m + in.seeds[idx];
        m = V2{m.x / static_cast<double>(ci.size()), m.y / static_cast<double>(ci.size())};
        R.merged.push_back(m);
    }
    // explorationTreeRowsInfoCallback gvd:130-150
    std::vector<std::pair<V2, V2>> rows;
    for (size_t i = 0; i + 1 < in.rows_info.size(); i += 2) {
        V2 s = in.rows_info[i], e = in.rows_info[i + 1];
        if (s.x > e.x) std::swap(s, e);
        rows.push_back({s, e});
    }
    GridView g{in.info, in.skeleton};
    R.resolution = in.info.resolution; R.origin_x = in.info.origin_x; R.origin_y = in.info.origin_y;
    if (R.merged.empty()) return;
    std::vector<V2> all;
    for (const auto &s : R.merged) if (std::isfinite(s.x) && std::isfinite(s.y)) all.push_back(s);
    if (all.empty()) return;
    double minx = g.minx(), maxx = g.maxx(), miny = g.miny(), maxy = g.maxy();
    if (!std::isfinite(minx) || !std::isfinite(maxx) || !std::isfinite(miny) || !std::isfinite(maxy)) return;
    voronoi_compute(all, minx, maxx, miny, maxy, P.subdiv_rect_mode, P.faithful_dead_work != 0, R.vor_edges, R.n_vertices_dead);
    if (P.markers) cell_markers(all, P.subdiv_rect_mode, R);
    std::vector<V2> bp = extract_boundary_points(R.vor_edges);
    R.boundary_raw = bp;

    // buildGraphFromBoundaryPoints gvd:794-895
    const int M = (int)bp.size();
    std::vector<EdgeRecord> er;
    if (M > 0 && !R.vor_edges.empty()) {
        auto nearest = [&](V2 q) {
            int ni = -1;
            double md = std::numeric_limits<double>::max();
            for (int i = 0; i < M; ++i) { double d = norm(bp[i] - q); if (d < md) { md = d; ni = i; } }
            return ni;
        };
        std::unordered_set<int64_t> added;
        for (const auto &ve : R.vor_edges) {
            int si = nearest(ve.start), ei = nearest(ve.end);
            if (si >= 0 && ei >= 0 && si != ei) {
                V2 sp = bp[si], ep = bp[ei];
                int a = si, b = ei;
                if (a > b) std::swap(a, b);
                int64_t key = (static_cast<int64_t>(a) << 32) ^ static_cast<uint32_t>(b);
                if (added.find(key) == added.end()) {
                    if (edge_through_occupied(g, sp, ep)) continue;
                    added.insert(key);
                    er.push_back(EdgeRecord{a, b, norm(ep - sp), 0.0f});
                }
            }
        }
        for (int i = 0; i < M; ++i)
            for (int j = i + 1; j < M; ++j) {
                double dist = norm(bp[i] - bp[j]);
                if (dist <= 0.5 && dist > 1e-6) {
                    int64_t key = (static_cast<int64_t>(i) << 32) ^ static_cast<uint32_t>(j);
                    if (added.find(key) == added.end()) {
                        if (edge_through_occupied(g, bp[i], bp[j])) continue;
                        added.insert(key);
                        er.push_back(EdgeRecord{i, j, dist, 0.0f});
                    }
                }
            }
    }
    // filterNodesAndEdgesOutsideGrid gvd:420-483
    std::vector<V2> fp;
    std::vector<int> o2n(bp.size(), -1);
    for (size_t i = 0; i < bp.size(); ++i) {
        const V2 &p = bp[i];
        if (p.x >= minx && p.x <= maxx && p.y >= miny && p.y <= maxy) { o2n[i] = (int)fp.size(); fp.push_back(p); }
    }
    std::vector<EdgeRecord> fer;
    for (const auto &e : er) {
        int nf = o2n[e.from], nt = o2n[e.to];
        if (nf >= 0 && nt >= 0 && nf != nt) {
            const V2 &a = fp[nf], &b = fp[nt];
            if (a.x >= minx && a.x <= maxx && a.y >= miny && a.y <= maxy && b.x >= minx && b.x <= maxx && b.y >= miny && b.y <= maxy) {
                int x = nf, y = nt;
                if (x > y) std::swap(x, y);
                fer.push_back(EdgeRecord{x, y, norm(b - a), e.min_clearance_m});
            }
        }
    }
    R.nodes = fp;
    // findClusterEndpointVoronoiBoundaryPoints gvd:485-556
    struct CV { V2 p[4]; bool v[4]; };
    std::vector<CV> cvs;
    if (!fp.empty()) {
        for (const auto &row : rows) {
            CV c;
            find_label_point(g, fp, row.first, row.second, -90.0, c.p[0], c.v[0]);
            find_label_point(g, fp, row.first, row.second, 90.0, c.p[1], c.v[1]);
            find_label_point(g, fp, row.second, row.first, -90.0, c.p[2], c.v[2]);
            find_label_point(g, fp, row.second, row.first, 90.0, c.p[3], c.v[3]);
            cvs.push_back(c);
        }
    }
    for (const auto &c : cvs)
        for (int k = 0; k < 4; ++k) { R.row_label_pts.push_back(c.p[k].x); R.row_label_pts.push_back(c.p[k].y); R.row_label_valid.push_back(c.v[k]); }
    // publishGraph gvd:897-1010
    R.published = true;
    for (const auto &p : fp) {
        int mask = 0, cidx = -1, cnt = 0;
        for (size_t cid = 0; cid < cvs.size(); ++cid)
            for (int k = 0; k < 4; ++k) {
                if (cvs[cid].v[k] && norm(p - cvs[cid].p[k]) < 0.1) {
                    mask |= (1 << k);
                    R.label_clusters.push_back((int)cid);
                    R.label_types.push_back(k);
                    ++cnt;
                    if (cidx == -1) cidx = (int)cid;
                }
            }
        R.labels.push_back(mask);
        R.cluster_idx.push_back(cidx);
        R.label_counts.push_back(cnt);
    }
    for (const auto &e : fer) {
        R.edges.push_back(e.from); R.edges.push_back(e.to);
        R.lengths.push_back(static_cast<float>(e.length_m));
        R.clearances.push_back(e.min_clearance_m);
    }
}

}  // namespace orc
