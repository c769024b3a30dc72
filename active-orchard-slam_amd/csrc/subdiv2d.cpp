// Host Delaunay with cv::Subdiv2D semantics — see subdiv2d.h. Compiled -ffp-contract=off.
#include "subdiv2d.h"

#include <immintrin.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <functional>

// AOS_SD_PROF (tools/sdcheck/sdprof.cpp only): per-phase TSC accumulators of the insert path
#ifdef AOS_SD_PROF
#include <x86intrin.h>
namespace aos { SdProf g_sdprof; }
#define SDP_T0(v) const unsigned long long v = __rdtsc()
#define SDP_ADD(field, t0) (aos::g_sdprof.field += __rdtsc() - (t0))
#define SDP_INC(field) (++aos::g_sdprof.field)
#else
#define SDP_T0(v)
#define SDP_ADD(field, t0)
#define SDP_INC(field)
#endif

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
        rec.push_back(Rec{});
        free_q = (int)rec.size() - 1;
    }
    const int q = free_q, e = q * 4;
    free_q = rec[q].h[0].x;
    rec[q] = Rec{{Half{e, e, 0, 0}, Half{e + 2, e + 2, 0, 0}}};
    return e;
}

int Subdiv2D::new_point(float x, float y, int type) {
    if (free_p == 0) {
        vp.push_back(V2f{0.f, 0.f}); vfirst.push_back(0); vtype.push_back(-1); vd.push_back(V2d{0.0, 0.0, 0.0, 0, 0});
        free_p = (int)vp.size() - 1;
    }
    const int v = free_p;
    free_p = vfirst[v];
    vp[v] = V2f{x, y}; vfirst[v] = 0; vtype[v] = type;
    vd[v] = V2d{(double)x, (double)y, (double)x * x + (double)y * y, 0, 0};
    return v;
}

void Subdiv2D::set_pts(int e, int o, int d) {   // setEdgePoints
    orgr(e) = o;
    orgr(sym(e)) = d;
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
    rec[q].h[0].on = 0;        // free marker (OpenCV: next[0] = 0)
    rec[q].h[0].x = free_q;
    free_q = q;
}

// The batched AVX2 tests are exact but not faster on the EPYC 9575F host (the 4 x 4 transposes take
// the FP pipes the scalar tests use): off by default, kept for tools/sdcheck and set_simd().
Subdiv2D::Subdiv2D() = default;

void Subdiv2D::init_delaunay(float rx, float ry, float rw, float rh, int rect_mode) {
    if (rect_mode == 1) {  // Rect_<float> -> Rect_<int>: saturate_cast<int> = cvRound (nearest even)
        rx = (float)(int)std::lrint(rx); ry = (float)(int)std::lrint(ry);
        rw = (float)(int)std::lrint(rw); rh = (float)(int)std::lrint(rh);
    }
    const float big = 3.f * std::max(rw, rh);
    vp.clear(); vd.clear(); vfirst.clear(); vtype.clear(); rec.clear();
    recent = 0;
    tlx = rx; tly = ry; brx = rx + rw; bry = ry + rh;
    vp.push_back(V2f{0.f, 0.f}); vd.push_back(V2d{0.0, 0.0, 0.0, 0, 0}); vfirst.push_back(0); vtype.push_back(-1);
    rec.push_back(Rec{});                                                      // quad-edge 0 (NULL)
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
    SDP_T0(t_loc);
    // The walk carries the current edge's end points o = Org(edge), d = Dst(edge): Onext(edge) keeps the origin and
    // Dprev(edge) the destination, and both end at the left face's third vertex a (Dst Onext = Org Dprev), so a step
    // loads one vertex. right_of(p, x -> y) is the sign of (y.x - p.x) (x.y - p.y) - (y.y - p.y) (x.x - p.x), as before.
    // (Checked against the round-4 walk on every locate of tools/sdcheck's 241 cases and the C2 seeds: same location,
    // edge, vertex and recentEdge; the C2 replay 17.4 -> 17.1 ms on the box, profiles/r05s_sdprof.txt.)
    const double x = px, y = py;
    auto rof = [&](int oi, int di) {
        const V2d &o = vd[oi], &d = vd[di];
        const double cw = (d.x - x) * (o.y - y) - (d.y - y) * (o.x - x);
        return (cw > 0) - (cw < 0);
    };
    int edge = recent;
    int location = -2;
    int o = org(edge), d = dst(edge);
    int roc = rof(o, d);
    if (roc > 0) { edge = sym(edge); roc = -roc; std::swap(o, d); }
    for (int i = 0; i < max_edges; i++) {
        SDP_INC(loc_iters);
        const int on_ = onext(edge);
        const int a = dst(on_);
        const int ron = rof(o, a);   // Onext: o -> a
        const int rod = rof(a, d);   // Dprev: a -> d
        if (rod > 0) {
            if (ron > 0 || (ron == 0 && roc == 0)) { location = 0; break; }
            roc = ron; edge = on_; d = a;
        } else {
            if (ron > 0) {
                if (rod == 0 && roc == 0) { location = 0; break; }
                roc = rod; edge = dprev(edge); o = a;
            } else if (roc == 0 && right_of(vp[a].x, vp[a].y, edge) >= 0) {
                edge = sym(edge); std::swap(o, d);
            } else {
                roc = ron; edge = on_; d = a;
            }
        }
    }
    recent = edge;
    if (location == 0) {
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
    SDP_ADD(t_locate, t_loc);
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
    if (loc == 0 && !force_loop &&
        (use_avx2 ? insert_cavity<true>(curr_edge, curr_point) : insert_cavity<false>(curr_edge, curr_point))) {
        ++n_cavity;
        return true;
    }
    ++n_loop;
    int base = new_edge();
    const int first_point = org(curr_edge);
    set_pts(base, first_point, curr_point);
    splice(base, curr_edge);
    do {
        base = connect(curr_edge, sym(base));
        curr_edge = oprev(base);
    } while (dst(curr_edge) != first_point);
    swap_loop(oprev(base), first_point, curr_point);
    return true;
}

// OpenCV's swap loop (Subdiv2D::insert after the connects), the reference path.
void Subdiv2D::swap_loop(int curr_edge, int first_point, int curr_point) {
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
}

// The swap loop's flip test for link edges es[0..n) (n <= 4) against the new point P, written into
// out[] (1 = swap): isRightOf(temp_dst, e) > 0 && isPtInCircle3(org, temp_dst, dst, P) < -eps, with
// temp_dst = Dst(Oprev e). Same operands and operation order as swap_loop in every lane.
void Subdiv2D::flip_tests_scalar(const int *es, int n, const V2d &P, int *out) const {
    auto area = [](const V2d &a, const V2d &b, const V2d &c) { return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x); };
    for (int i = 0; i < n; ++i) {
        const int e = es[i];
        const V2d &T = vd[dst(oprev(e))], &O = vd[org(e)], &D = vd[dst(e)];
        bool flip = false;
        if (area(T, D, O) > 0) {
            double val = T.n2 * area(D, P, O);
            val -= D.n2 * area(T, P, O);
            val += P.n2 * area(T, D, O);
            val -= O.n2 * area(T, D, P);
            flip = val < -(FLT_EPSILON * 0.125);
        }
        out[i] = flip;
    }
}

// Four tests at once on AVX2 (one lane each; every lane rounds exactly like the scalar form: plain
// IEEE double sub / mul in the same order, no FMA).
#define AOS_AVX2 __attribute__((target("avx2")))
AOS_AVX2 static inline void transpose3(const __m256d *r, __m256d &X, __m256d &Y, __m256d &N) {
    const __m256d t0 = _mm256_unpacklo_pd(r[0], r[1]), t1 = _mm256_unpackhi_pd(r[0], r[1]);
    const __m256d t2 = _mm256_unpacklo_pd(r[2], r[3]), t3 = _mm256_unpackhi_pd(r[2], r[3]);
    X = _mm256_permute2f128_pd(t0, t2, 0x20);
    N = _mm256_permute2f128_pd(t0, t2, 0x31);
    Y = _mm256_permute2f128_pd(t1, t3, 0x20);
}
AOS_AVX2 static inline __m256d area4(__m256d ax, __m256d ay, __m256d bx, __m256d by, __m256d cx, __m256d cy) {
    return _mm256_sub_pd(_mm256_mul_pd(_mm256_sub_pd(bx, ax), _mm256_sub_pd(cy, ay)),
                         _mm256_mul_pd(_mm256_sub_pd(by, ay), _mm256_sub_pd(cx, ax)));
}

AOS_AVX2 void Subdiv2D::flip_tests_avx2(const int *es, int n, const V2d &P, int *out) const {
    __m256d rT[4], rO[4], rD[4];
    for (int i = 0; i < 4; ++i) {
        const int e = es[i < n ? i : 0];
        rT[i] = _mm256_loadu_pd(&vd[dst(oprev(e))].x);
        rO[i] = _mm256_loadu_pd(&vd[org(e)].x);
        rD[i] = _mm256_loadu_pd(&vd[dst(e)].x);
    }
    __m256d Tx, Ty, Tn, Ox, Oy, On, Dx, Dy, Dn;
    transpose3(rT, Tx, Ty, Tn);
    transpose3(rO, Ox, Oy, On);
    transpose3(rD, Dx, Dy, Dn);
    const __m256d Px = _mm256_set1_pd(P.x), Py = _mm256_set1_pd(P.y), Pn = _mm256_set1_pd(P.n2);
    const __m256d aTDO = area4(Tx, Ty, Dx, Dy, Ox, Oy);
    __m256d val = _mm256_mul_pd(Tn, area4(Dx, Dy, Px, Py, Ox, Oy));
    val = _mm256_sub_pd(val, _mm256_mul_pd(Dn, area4(Tx, Ty, Px, Py, Ox, Oy)));
    val = _mm256_add_pd(val, _mm256_mul_pd(Pn, aTDO));
    val = _mm256_sub_pd(val, _mm256_mul_pd(On, area4(Tx, Ty, Dx, Dy, Px, Py)));
    const __m256d right = _mm256_cmp_pd(aTDO, _mm256_setzero_pd(), _CMP_GT_OQ);
    const __m256d inside = _mm256_cmp_pd(val, _mm256_set1_pd(-(FLT_EPSILON * 0.125)), _CMP_LT_OQ);
    const int mask = _mm256_movemask_pd(_mm256_and_pd(right, inside));
    for (int i = 0; i < n; ++i) out[i] = (mask >> i) & 1;
}

// The ring pass of insert_cavity over plain restrict pointers (the Rec / V2d layouts as ints: a record is on[2],
// op[2], org[2], link, pad; a vertex's spoke sits at int 7 of its 32 bytes): one pass over the boundary L_k
// (k in walk order) writes every field of spoke S_k = x_k -> p (on / op / org in both directions), the two ring
// links of the boundary edges next to it and vtx[x_k].firstEdge = S_k. In a function of its own the compiler keeps
// the loop's values in registers (round 5 on the box: the replay's write phase 7.9 -> 5.3 ms with the certification
// change below, profiles/r05s_sdprof.txt).
__attribute__((noinline)) static void ring_pass(int *__restrict R, int *__restrict vfirst, const int *__restrict spoke,
                                                const int *__restrict bd, const int *__restrict bu, int m, int p) {
    // directed edge e's fields at R[2 e] (onext), R[2 e + 1] (oprev), R[2 e + 2] (origin)
    auto sp = [&](int x) { return spoke[8 * (size_t)x]; };
    int Sm = sp(bu[m - 1]), S = sp(bu[0]);
    for (int k = 0; k < m; ++k) {
        const int k1 = k + 1 == m ? 0 : k + 1;
        const int L = bd[k], Ln = bd[k1], x = bu[k], Sn = sp(bu[k1]);
        const int sLn = Ln ^ 2, sS = S ^ 2;
        R[2 * (ptrdiff_t)L] = S;                                       // Onext(L_k) = S_k
        R[2 * (ptrdiff_t)sLn + 1] = S;                                 // Oprev(Sym L_k+1) = S_k
        int *a = R + 2 * (ptrdiff_t)S, *b = R + 2 * (ptrdiff_t)sS;
        a[0] = sLn; a[1] = L; a[2] = x;                                // S_k: x_k -> p
        b[0] = Sm ^ 2; b[1] = Sn ^ 2; b[2] = p;                        // Sym S_k: around p, counter-clockwise
        vfirst[x] = S;
        Sm = S; S = Sn;
    }
}

// Cavity form of an INSIDE insert (subdiv2d.h). e0 = locate's edge: p lies left of it, inside the
// triangle (e0, Lnext e0, Lnext^2 e0). Returns false, having changed nothing but the scratch, when
// the DFS cannot certify the cavity; the caller then runs the connects and the swap loop.
template <bool SIMD>
bool Subdiv2D::insert_cavity(int e0, int p) {
    // the marks live in the vertex's own line (V2d::stamp / spoke): the DFS reads them right after the
    // vertex's coordinates (C2 replay 25.3-26.1 -> 25.1-25.9 ms on the box, profiles/r04z_replay_dfs.txt)
    if (++stamp >= (1 << 29)) { for (V2d &x : vd) x.stamp = 0; stamp = 1; }
    const int sA = 2 * stamp;   // this insert's mark: a cavity vertex (the three corners and every apex)
    const int eB = lnext(e0), eA = lnext(eB);          // root link edges in walk order: eA, eB, e0
    if (lnext(eA) != e0) return false;
    const int first = org(e0), v1 = org(eB), v2 = org(eA);
    if (first == v1 || v1 == v2 || v2 == first) return false;
    vd[first].stamp = vd[v1].stamp = vd[v2].stamp = sA;

    const V2d P = vd[p];
    auto area = [](const V2d &a, const V2d &b, const V2d &c) { return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x); };
    // scratch sized for the worst case: every swap adds one apex, one stacked edge and one boundary edge
    const size_t cap = vp.size() + 8;
    if (dfs_stack.size() < cap) {
        dfs_stack.resize(2 * cap); cav_bnd.resize(2 * cap);
        cav_bu.resize(2 * cap);
    }
    int *const stk = dfs_stack.data(), *const bd = cav_bnd.data(), *const bu = cav_bu.data();
    // The stack and the boundary lists are bumped pointers and no flip counter is kept (last_flip < 0: no flip): with
    // fewer live values the walk keeps them in registers (the flip path had reloaded four spilled base pointers and
    // incremented a counter in memory; round 5 on the box: walk 11.7-13.3 -> 10.5-10.6 ms, the C2 replay 17.0-17.7 ->
    // 15.8-16.2 ms, profiles/r05zq_sdprof.txt).
    int *top = stk, *bdp = bd, *bup = bu;
    int last_flip = -1;
    *top++ = e0; *top++ = eB;
    int e = eA;
    // Pre-order walk; every test reads the old triangle right of the link edge (never incident to p).
    // The first child (w -> v) is walked at once; the second (u -> w) waits on the stack. Once the walk
    // reaches a boundary edge it pops the stacked edges, whose tests are independent of each other (the SIMD
    // instantiation, off by default, evaluates them four at a time until one swaps).
    // The test is evaluated whole and combined without a branch: the orientation test is nearly always true
    // and the in-circle sum's operands are already loaded (box A/B: 28.0-28.6 -> 26.1-26.5 ms for the C2
    // seeds together with the SIMD batches compiled out of the default path, profiles/r04z_replay_dfs.txt).
    int known = -1;   // 1: e is known to swap (decided in a batch; SIMD only)
    SDP_T0(t_dfs);
    for (;;) {
        SDP_INC(dfs_steps);
        const int t = oprev(e), w = dst(t);
        bool flip;
        if (SIMD && known == 1) {
            flip = true;
        } else {
            const V2d &T = vd[w], &O = vd[org(e)], &D = vd[dst(e)];
            const double aTDO = area(T, D, O);   // same expressions and order as swap_loop
            double val = T.n2 * area(D, P, O);
            val -= D.n2 * area(T, P, O);
            val += P.n2 * aTDO;
            val -= O.n2 * area(T, D, P);
            flip = (aTDO > 0) & (val < -(FLT_EPSILON * 0.125));
        }
        known = -1;
        if (flip) {
            // the cavity would wrap a vertex. (w is never p: p has no edge yet. The scratch cannot overflow: every
            // swap adds a distinct vertex, so the swaps are fewer than the vertices <= cap - 8.)
            V2d &W = vd[w];
            if (W.stamp == sA) return false;
            W.stamp = sA;
            W.spoke = e;                                       // e becomes w -> p
            last_flip = e;
            *top++ = t;                                        // u -> w, after the w -> v subtree
            e = sym(onext(sym(e)));                            // w -> v
            continue;
        }
        *bdp++ = e; *bup++ = org(e);
        if (SIMD) {
            int d[4];
            while (top - stk >= 4) {
                const int b[4] = {top[-1], top[-2], top[-3], top[-4]};
                flip_tests_avx2(b, 4, P, d);
                int i = 0;
                for (; i < 4 && !d[i]; ++i) {
                    const int x = b[i];
                    *bdp++ = x; *bup++ = org(x);
                }
                top -= i;
                if (i < 4) { known = 1; break; }
            }
        }
        if (top == stk) break;
        e = *--top;
    }
    const int nb = (int)(bdp - bd);
    SDP_ADD(t_dfs, t_dfs);
    SDP_T0(t_wr);
    // Why no certification of the boundary is needed (round 4 checked it after the walk): by induction over the walk,
    // a tested edge u -> v emits boundary edges forming a chain from v back to u (a leaf emits itself; a swapped
    // edge with apex w emits the chain of w -> v, then that of u -> w), whose origins are u and the apexes below it.
    // So the three root chains always close into one cycle of 3 + (swaps) edges, and its vertices are distinct exactly
    // when every apex is new, which the walk checks at each swap (the C2 replay 25.6-26.4 -> 22.6-23.1 ms on the
    // box with ring_pass; tools/sdcheck still compares every insert's full state with the swap loop).
    const int m = nb;
    // ---- the outcome. OpenCV's two connectEdges (after the first newEdge + splice) number the three new quad-edges
    // first -> p, v1 -> p, v2 -> p in that order; everything else they write (the rings of first, v1, v2 and p next to
    // the new edges, their end points, firstEdge) is rewritten by ring_pass, which sets every field of every spoke and
    // the ring links of the boundary edges on both sides of it. So only their allocations are kept (the C2 replay
    // 22.6-23.1 -> 21.8-22.2 ms on the box; tools/sdcheck: identical full state after every insert).
    const int c0 = new_edge(), c1 = new_edge(), c2 = new_edge();   // first -> p, v1 -> p, v2 -> p
    vd[first].spoke = c0; vd[v1].spoke = c1; vd[v2].spoke = c2;
    vfirst[p] = sym(last_flip >= 0 ? last_flip : c2);   // the last setEdgePoints with p as destination
    // swapEdges' setEdgePoints(e, apex, p) and vtx[apex].firstEdge = e, and the rings of the final star: ring_pass
    static_assert(sizeof(Rec) == 32 && sizeof(Half) == 16 && offsetof(Half, op) == 4 && offsetof(Half, org) == 8, "ring_pass: Rec layout");
    static_assert(sizeof(V2d) == 32 && offsetof(V2d, spoke) == 28, "ring_pass: V2d layout");
    ring_pass(ri(), vfirst.data(), &vd[0].spoke, bd, bu, m, p);
    SDP_ADD(t_write, t_wr);
    return true;
}

bool Subdiv2D::same_state(const Subdiv2D &o) const {
    if (rec.size() != o.rec.size() || vp.size() != o.vp.size() || recent != o.recent || free_q != o.free_q ||
        free_p != o.free_p)
        return false;
    for (size_t q = 0; q < rec.size(); ++q)
        for (int d = 0; d < 2; ++d)
            if (rec[q].h[d].on != o.rec[q].h[d].on || rec[q].h[d].op != o.rec[q].h[d].op || rec[q].h[d].org != o.rec[q].h[d].org)
                return false;
    for (size_t v = 0; v < vp.size(); ++v)
        if (vfirst[v] != o.vfirst[v] || vtype[v] != o.vtype[v] || vp[v].x != o.vp[v].x || vp[v].y != o.vp[v].y)
            return false;
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
        if (r.h[0].on <= 0) continue;   // free
        o[0] = r.h[0].on; o[1] = rot3(r.h[0].op); o[2] = r.h[1].on; o[3] = rot3(r.h[1].op);
        o[4] = r.h[0].org; o[6] = r.h[1].org;
    }
    return Raw{qx.data(), n, reinterpret_cast<const float *>(vp.data()), vfirst.data(), vtype.data(), (int)vp.size()};
}

// Records [q0, q1) in OpenCV's layout {next[4], pt[4]} (free ones and #0 as zeros). The AVX2 form moves a record
// with one load, one permute and one store (round 5: the export is on the frame's path between the last insert and
// the GPU facet builder).
static void export_recs_scalar(const int *R, int *out, int q0, int q1) {
    auto rot3 = [](int x) { return (x & ~3) + ((x + 3) & 3); };
    for (int q = q0; q < q1; ++q) {
        const int *r = R + 8 * (size_t)q;   // {on, op, org, x} of Sym-direction 0, then 1
        int o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (q > 0 && r[0] > 0) {
            o[0] = r[0]; o[1] = rot3(r[1]); o[2] = r[4]; o[3] = rot3(r[5]);
            o[4] = r[2]; o[6] = r[6];
        }
        std::memcpy(out + 8 * (size_t)q, o, sizeof(o));
    }
}
AOS_AVX2 static void export_recs_avx2(const int *R, int *out, int q0, int q1) {
    if (q0 == 0 && q1 > 0) { export_recs_scalar(R, out, 0, 1); q0 = 1; }
    const __m256i perm = _mm256_setr_epi32(0, 1, 4, 5, 2, 0, 6, 0);   // on0 op0 on1 op1 org0 . org1 .
    const __m256i keep = _mm256_setr_epi32(-1, -1, -1, -1, -1, 0, -1, 0);
    const __m256i m3 = _mm256_set1_epi32(3), not3 = _mm256_set1_epi32(~3), zero = _mm256_setzero_si256();
    for (int q = q0; q < q1; ++q) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(R + 8 * (size_t)q));
        const __m256i w = _mm256_permutevar8x32_epi32(v, perm);
        const __m256i rot = _mm256_add_epi32(_mm256_and_si256(w, not3), _mm256_and_si256(_mm256_add_epi32(w, m3), m3));
        __m256i o = _mm256_and_si256(_mm256_blend_epi32(w, rot, 0x0a), keep);
        const __m256i live = _mm256_cmpgt_epi32(_mm256_permutevar8x32_epi32(v, zero), zero);   // on0 > 0
        o = _mm256_and_si256(o, live);
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(out + 8 * (size_t)q), o);
    }
}

Subdiv2D::Raw Subdiv2D::raw_into(void *dst, int chunk_recs, const std::function<void(size_t, size_t)> &written) const {
    const int n = (int)rec.size(), nv = (int)vp.size();
    int *qe = static_cast<int *>(dst);
    static const bool avx2 = simd_ok();
    const int step = chunk_recs > 0 ? chunk_recs : std::max(n, 1);
    for (int q0 = 0; q0 < n; q0 += step) {
        const int q1 = std::min(n, q0 + step);
        if (avx2) export_recs_avx2(ri(), qe, q0, q1);
        else export_recs_scalar(ri(), qe, q0, q1);
        if (written && q1 < n) written(sizeof(int) * 8 * (size_t)q0, sizeof(int) * 8 * (size_t)(q1 - q0));
    }
    char *p = reinterpret_cast<char *>(qe + 8 * (size_t)n);
    float *vpo = reinterpret_cast<float *>(p);
    std::memcpy(vpo, vp.data(), sizeof(V2f) * (size_t)nv);
    int *vf = reinterpret_cast<int *>(p + sizeof(V2f) * (size_t)nv), *vt = vf + nv;
    std::memcpy(vf, vfirst.data(), sizeof(int) * (size_t)nv);
    std::memcpy(vt, vtype.data(), sizeof(int) * (size_t)nv);
    return Raw{qe, n, vpo, vf, vt, nv};
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
