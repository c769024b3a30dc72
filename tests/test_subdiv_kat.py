"""Hand-traced known answers for Subdiv2D (OpenCV 4.5.4 modules/imgproc/src/subdivision2d.cpp, used by
VoronoiDiagram::compute, src/utils/voronoi_diagram.cpp:51-114): the quad-edge ids, vtx[k].firstEdge and
each Voronoi facet's start vertex and point order, which decide GvdGraph node order.

Every expected value below was derived BY HAND from OpenCV's algorithm (initDelaunay, locate, insert with
its swap loop, connectEdges, swapEdges, deleteEdge, calcVoronoi, getVoronoiFacetList), not produced by
tools/make_golden.py or by either implementation; the comments are the traces. Both the oracle's
restatement (oracle/oracle_gvd.cpp) and the product's replay (active-orchard-slam_amd/csrc/subdiv2d.cpp)
must reproduce them, in both rectangle modes (Subdiv2D(Rect2f), and the implicit Rect2f -> Rect cvRound
conversion). Verdict r03 "missing 1".

Notation: rect (0, 0, 10, 10) -> big = 3 * 10 = 30: vertices 1 A(30, 0), 2 B(0, 30), 3 C(-30, -30);
quad-edge q holds directed edges 4q (org pt[0] -> dst pt[2]), 4q + 2 (its Sym), 4q + 1 / 4q + 3 (duals).
next[r] = Onext of rotation r (OpenCV's QuadEdge::next). Initially q1 = AB (4), q2 = BC (8), q3 = CA (12).
"""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "active-orchard-slam_amd", "csrc", "subdiv2d.cpp")

# ---------------------------------------------------------------------------------------------- case 1
# insert P = (5, 5) (vertex 4). locate from recentEdge 4 (A->B): isRightOf(P, 4) = sign(-600) = -1; onext = 14
# (A->C), dprev = 10 (C->B); right_of_onext = +1 (1050), right_of_dprev = +1 (1050) -> INSIDE at edge 4 (t1 =
# t2 = 30 >= FLT_EPSILON, |area| = 600). newEdge -> 16; setEdgePoints(16, A, P); splice(16, 4): q1.next[0] = 16,
# q4.next = [14, 7, ...]. connectEdges(4, 18) -> 20 = B->P (Lnext(4) = 8), curr = Oprev(20) = 8; connectEdges(8,
# 22) -> 24 = C->P (Lnext(8) = 12), curr = 12, dst A == first point. Swap loop: 12 (C->A): B not right of it; 8:
# A not right of it; 4: C not right of it, org A == first -> done, no flips.
CASE1_NEXT = [[0, 0, 0, 0], [16, 13, 8, 23], [20, 5, 12, 27], [24, 9, 4, 19], [14, 7, 22, 25], [6, 11, 26, 17],
              [10, 15, 18, 21]]
CASE1_ENDS = [[0, 0], [1, 2], [2, 3], [3, 1], [1, 4], [2, 4], [3, 4]]   # pt[0], pt[2]
CASE1_FIRST = [0, 16, 20, 24, 26]   # setEdgePoints order: v1 14 -> 16; v2 8 -> 20; v3 12 -> 24; v4 18 -> 22 -> 26
# calcVoronoi: q4 left face (A, P, C): a0 = -25, b0 = 5, c0 = 425; a1 = b1 = -35, c1 = -875; det = 1050 ->
# (10500 / 1050, -36750 / 1050) = (10, -35) = vtx 5; q4 right face (A, P, B) -> (12750 / 600) = (21.25, 21.25) =
# vtx 6; q5 right face (B, C, P) -> (-36750 / 1050, 10500 / 1050) = (-35, 10) = vtx 7; q6 has both faces.
# Facet of P: rotate(firstEdge 26, 1) = 27 -> pt[3] of q6 = vtx 7, Lnext -> 19 (q4.pt[3] = 5), -> 23 (q5.pt[3]
# = 6), -> 27.
CASE1_FACETS = [[(-35.0, 10.0), (10.0, -35.0), (21.25, 21.25)]]

# ---------------------------------------------------------------------------------------------- case 2
# then Q = (6, 2) (vertex 5). locate from 4: right_of_curr -1 (-660); onext 16: -1 (-70), dprev 22: +1 (10) ->
# edge = 16; onext 14: +1 (840), dprev 24: +1 (140) -> INSIDE at 16 (A->P), triangle (A, P, C); recentEdge = 16.
# newEdge 28 = A->Q, splice(28, 16); connectEdges(16, 30) -> 32 = P->Q (Lnext(16) = 26), curr 26; connectEdges(26,
# 34) -> 36 = C->Q (Lnext(26) = 12), curr 12 (dst A). Swap loop: 12: B left of C->A; 26 (P->C): B right (1050),
# isPtInCircle3(P, B, C, Q) = +126000 -> keep; 16 (A->P): B right (600), isPtInCircle3(A, B, P, Q) = 900*70 -
# 50*660 + 40*600 - 900*10 = +45000 -> keep; org A == first -> done, no flips.
CASE2_NEXT = [[0, 0, 0, 0], [16, 13, 8, 23], [20, 5, 12, 27], [36, 9, 4, 31], [28, 7, 22, 35], [6, 11, 26, 17],
              [10, 39, 32, 21], [14, 19, 34, 37], [18, 25, 38, 29], [24, 15, 30, 33]]
CASE2_ENDS = [[0, 0], [1, 2], [2, 3], [3, 1], [1, 4], [2, 4], [3, 4], [1, 5], [4, 5], [3, 5]]
CASE2_FIRST = [0, 28, 20, 36, 32, 38]
# calcVoronoi: q4 left (A, P, Q): a0 = -25, b0 = 5, c0 = 425; a1 = 1, b1 = -3, c1 = 5; det = 70 -> (1300 / 70,
# 550 / 70) = vtx 6; q4 right (A, P, B) = (21.25, 21.25) vtx 7; q5 right (B, C, P) = (-35, 10) vtx 8; q6 right (C,
# Q, P): a0 = b0 = 35, c0 = 875; a1 = -36, b1 = -32, c1 = -880; det = 140 -> (-2800 / 140, -700 / 140) = (-20, -5)
# vtx 9; q7 left (A, Q, C): a0 = -24, b0 = 2, c0 = 430; det = 840 -> (12000 / 840, -36600 / 840) vtx 10.
# Facet P: rotate(32, 1) = 33 -> q8.pt[1] = 9, 19 -> 6, 23 -> 7, 27 -> 8; facet Q: rotate(38, 1) = 39 -> q9.pt[3] =
# 9, 31 -> 10, 35 -> 6.
V_APQ = (1300.0 / 70.0, 550.0 / 70.0)
V_AQC = (12000.0 / 840.0, -36600.0 / 840.0)
CASE2_FACETS = [[(-20.0, -5.0), V_APQ, (21.25, 21.25), (-35.0, 10.0)],
                [(-20.0, -5.0), V_AQC, V_APQ]]

# ---------------------------------------------------------------------------------------------- case 3
# then R = (8, 8) (vertex 6): one flip. locate from 16: right_of_curr = +1 (90) -> edge 18 (P->A); onext 22 (P->B):
# +1 (90), dprev 6 (B->A): +1 (420) -> INSIDE at 18, triangle (P, A, B); recentEdge = 18. newEdge 40 = P->R; connect
# 44 = A->R (Lnext(18) = 4), curr 4; connect 48 = B->R (Lnext(4) = 20), curr 20 (dst P). Swap loop: 20 (B->P): C right
# (1050), isPtInCircle3(B, C, P, R) = +239400 (C, P, R collinear) -> keep; 4: C left; 18 (P->A): Q right (70),
# isPtInCircle3(P, Q, A, R) = 40*90 - 900*12 + 128*70 - 50*148 = -5640 < 0 -> swapEdges(18): a = Oprev(18) = 32,
# b = Oprev(16) = 44; edge 18 becomes Q->R (q4 = R->Q), vtx[5].firstEdge = 18, vtx[6].firstEdge = 16; curr = 30
# (Q->A): C right (840), +465120 -> keep; 32 (P->Q): C right (140), +31920 -> keep; org P == first -> done.
CASE3_NEXT = [[0, 0, 0, 0], [44, 13, 8, 51], [20, 5, 12, 27], [36, 9, 4, 31], [46, 41, 34, 29], [48, 11, 26, 43],
              [10, 39, 32, 21], [14, 47, 18, 37], [40, 25, 38, 17], [24, 15, 30, 33], [22, 35, 16, 49],
              [28, 7, 50, 19], [6, 23, 42, 45]]
CASE3_ENDS = [[0, 0], [1, 2], [2, 3], [3, 1], [6, 5], [2, 4], [3, 4], [1, 5], [4, 5], [3, 5], [4, 6], [1, 6], [2, 6]]
CASE3_FIRST = [0, 44, 48, 36, 40, 18, 16]
# calcVoronoi: q4 left (R, Q, A): a0 = -2, b0 = -6, c0 = 44; a1 = 24, b1 = -2, c1 = -430; det = 148 -> (2668 / 148,
# 196 / 148) vtx 7; q4 right (R, Q, P): a1 = b1 = 3, c1 = -39; det = 12 -> (102 / 12, 54 / 12) = (8.5, 4.5) vtx 8; q5
# left (B, P, R): det = 90 -> (-300 / 90, 1470 / 90) vtx 9; q5 right (-35, 10) vtx 10; q6 right (-20, -5) vtx 11;
# q7 left (A, Q, C) vtx 12; q11 right (A, B, R): a0 = -22, b0 = 8, c0 = 386; a1 = 30, b1 = -30, c1 = -0.0; det = 420
# -> (11580 / 420, 11580 / 420) vtx 13.
V_RQA = (2668.0 / 148.0, 196.0 / 148.0)
V_BPR = (-300.0 / 90.0, 1470.0 / 90.0)
V_ABR = (11580.0 / 420.0, 11580.0 / 420.0)
CASE3_FACETS = [[(8.5, 4.5), V_BPR, (-35.0, 10.0), (-20.0, -5.0)],       # P: 41, 23, 27, 33
                [V_RQA, (8.5, 4.5), (-20.0, -5.0), V_AQC],               # Q: 19, 35, 39, 31
                [(8.5, 4.5), V_RQA, V_ABR, V_BPR]]                       # R: 17, 47, 51, 43

# ---------------------------------------------------------------------------------------------- case 4
# then S = (5, 4) (vertex 7), exactly on the circumcircle of (P, Q, R) (centre (8.5, 4.5), r^2 = 12.5): the
# co-circular test must keep the edge. locate from 18 (now Q->R): -1 (-10); onext 34 (Q->P): -1, dprev 40: +1 ->
# edge 34; onext 38 (Q->C): +1 (104), dprev 24 (C->P): +1 (35) -> INSIDE at 34, triangle (Q, P, C). newEdge 52 =
# Q->S; connect 56 = P->S (Lnext(34) = 26), curr 26; connect 60 = C->S (Lnext(26) = 36), curr 36 (dst Q). Swap loop:
# 36 (C->Q): A right (840), +171240 -> keep; 26 (P->C): B right, isPtInCircle3(P, B, C, S) = +11550 -> keep (S is
# 1636 > 1625 from (-35, 10)); 34 (Q->P): R right (12), isPtInCircle3(Q, R, P, S) = 128*1 - 50*10 + 41*12 - 40*3 =
# 0 exactly -> not < 0, keep; org Q == first -> done.
CASE4_NEXT = [[0, 0, 0, 0], [44, 13, 8, 51], [20, 5, 12, 27], [36, 9, 4, 31], [46, 41, 34, 29], [48, 11, 26, 43],
              [10, 63, 56, 21], [14, 47, 18, 37], [40, 59, 52, 17], [60, 15, 30, 55], [22, 35, 16, 49],
              [28, 7, 50, 19], [6, 23, 42, 45], [38, 33, 58, 61], [32, 25, 62, 53], [24, 39, 54, 57]]
CASE4_ENDS = CASE3_ENDS + [[5, 7], [4, 7], [3, 7]]
CASE4_FIRST = [0, 44, 48, 60, 56, 52, 16, 62]
# calcVoronoi: vtx 8 = V_RQA (q4 left), vtx 9 = (8.5, 4.5) (q4 right, from R->Q), 10 = V_BPR, 11 = (-35, 10), q6
# right (C, S, P): a1 = -35, b1 = -34, c1 = -879.5; det = 35 -> (-1032.5 / 35, 157.5 / 35) = (-29.5, 4.5) vtx 12,
# 13 = V_AQC, q8 right (P, S, Q): a0 = 1, b0 = -3, c0 = 5; a1 = 0, b1 = 1, c1 = -4.5; det = 1 -> (8.5, 4.5) again,
# a second vertex (vtx 14); q9 left (C, Q, S): det = 104 -> (-1776 / 104, -862 / 104) vtx 15; 16 = V_ABR.
# The two co-circular triangles give two facet points at the same place (a zero-length Voronoi edge).
V_CQS = (-1776.0 / 104.0, -862.0 / 104.0)
CASE4_FACETS = [[(-29.5, 4.5), (8.5, 4.5), (8.5, 4.5), V_BPR, (-35.0, 10.0)],   # P: 57 (14), 33 (14), 41 (9), 23, 27
                [(8.5, 4.5), V_CQS, V_AQC, V_RQA, (8.5, 4.5)],                  # Q: 53 (14), 39, 31, 19, 35 (9)
                [(8.5, 4.5), V_RQA, V_ABR, V_BPR],                              # R: unchanged
                [(-29.5, 4.5), V_CQS, (8.5, 4.5)]]                              # S: 63, 55, 59

# ---------------------------------------------------------------------------------------------- case 5
# P = (5, 5), then T = (8.125, 4.375) exactly on edge P-A (area 0 in double). locate from 4: -1; onext 16: 0,
# dprev 22: +1 -> (onext 0 but right_of_curr -1) edge = 16, right_of_curr = 0; onext 14: +1, dprev 24: +1 -> INSIDE
# at 16 (A->P): t1 = 26.25, t2 = 3.75, t3 = 30, |area| = 0 < FLT_EPSILON -> PTLOC_ON_EDGE. insert: curr = Oprev(16) =
# 4 (recentEdge = 4), deleteEdge(16): q4 freed (next[0] = 0, freeQEdge = 4); vtx[1].firstEdge stays 16. T = vtx 5;
# newEdge reuses quad-edge 4: 16 = A->T; connect 28 = B->T (Lnext(4) = 20), curr 20; connect 32 = P->T (Lnext(20)
# = 26), curr 26; connect 36 = C->T (Lnext(26) = 12), curr 12 (dst A). Swap loop: 12: B left; 26 (P->C): B right,
# isPtInCircle3(P, B, C, T) = +279726.5625 -> keep; 20 (B->P): C right, +279726.5625 -> keep; 4: C left, org A ->
# done.
CASE5_NEXT = [[0, 0, 0, 0], [16, 13, 8, 31], [20, 5, 12, 27], [36, 9, 4, 19], [14, 7, 30, 37], [28, 11, 26, 35],
              [10, 39, 32, 21], [6, 23, 34, 17], [22, 25, 38, 29], [24, 15, 18, 33]]
CASE5_ENDS = [[0, 0], [1, 2], [2, 3], [3, 1], [1, 5], [2, 4], [3, 4], [2, 5], [4, 5], [3, 5]]
CASE5_FIRST = [0, 16, 28, 36, 32, 38]

RECT = (0.0, 0.0, 10.0, 10.0)
RECT_ROUNDS_TO_IT = (0.3, 0.2, 9.6, 9.7)   # cvRound -> (0, 0, 10, 10): mode 1 must give the same answers
CASES = {
    "one_seed": ([(5, 5)], CASE1_NEXT, CASE1_ENDS, CASE1_FIRST, CASE1_FACETS),
    "two_seeds": ([(5, 5), (6, 2)], CASE2_NEXT, CASE2_ENDS, CASE2_FIRST, CASE2_FACETS),
    "three_seeds_one_flip": ([(5, 5), (6, 2), (8, 8)], CASE3_NEXT, CASE3_ENDS, CASE3_FIRST, CASE3_FACETS),
    "cocircular": ([(5, 5), (6, 2), (8, 8), (5, 4)], CASE4_NEXT, CASE4_ENDS, CASE4_FIRST, CASE4_FACETS),
    "on_edge": ([(5, 5), (8.125, 4.375)], CASE5_NEXT, CASE5_ENDS, CASE5_FIRST, None),
}

SHIM = r"""
#include "subdiv2d.h"
#include <cstring>
#include <vector>
extern "C" int subdiv_state(const float* xy, int n, const float* rect, int mode, int* qe, int cap_q, int* vfirst,
                            int* vtype, int cap_v, int* n_v, int* foff, float* fxy, int cap_f, int* n_f) {
    aos::Subdiv2D sd;
    sd.init_delaunay(rect[0], rect[1], rect[2], rect[3], mode);
    for (int i = 0; i < n; ++i) sd.insert(xy[2 * i], xy[2 * i + 1]);
    aos::Subdiv2D::Raw r = sd.raw();   // the insert state (no Voronoi points yet)
    if (r.n_rec > cap_q || r.n_vtx > cap_v) return -1;
    std::memcpy(qe, r.qe, sizeof(int) * 8 * r.n_rec);
    std::memcpy(vfirst, r.vfirst, sizeof(int) * r.n_vtx);
    std::memcpy(vtype, r.vtype, sizeof(int) * r.n_vtx);
    *n_v = r.n_vtx;
    const int nq = r.n_rec;
    std::vector<int> off;
    std::vector<float> pts;
    sd.voronoi_facets(off, pts);
    if ((int)off.size() > cap_f || (int)pts.size() > 2 * cap_f) return -1;
    std::memcpy(foff, off.data(), sizeof(int) * off.size());
    std::memcpy(fxy, pts.data(), sizeof(float) * pts.size());
    *n_f = (int)off.size() - 1;
    return nq;
}
"""
_lib = None


def product_lib():
    global _lib
    if _lib is None:
        d = tempfile.mkdtemp(prefix="subdiv_kat_")
        src = os.path.join(d, "shim.cpp")
        open(src, "w").write(SHIM)
        so = os.path.join(d, "libshim.so")
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-shared", "-I",
                               os.path.dirname(SRC), "-o", so, src, SRC])
        _lib = ctypes.CDLL(so)
        _lib.subdiv_state.restype = ctypes.c_int
    return _lib


def product_state(points, rect, mode):
    xy = np.ascontiguousarray(points, np.float32).reshape(-1)
    r = np.ascontiguousarray(rect, np.float32)
    cap = 256
    qe = np.zeros(8 * cap, np.int32)
    vf, vt = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    foff, fxy = np.zeros(cap, np.int32), np.zeros(2 * cap, np.float32)
    nv, nf = ctypes.c_int(), ctypes.c_int()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    nq = product_lib().subdiv_state(p(xy), xy.size // 2, p(r), mode, p(qe), cap, p(vf), p(vt), cap, ctypes.byref(nv),
                                    p(foff), p(fxy), cap, ctypes.byref(nf))
    assert nq > 0
    q = qe[:8 * nq].reshape(-1, 8)
    facets = [fxy.reshape(-1, 2)[foff[i]:foff[i + 1]] for i in range(nf.value)]
    return {"next": q[:, :4], "pt": q[:, 4:], "first_edge": vf[:nv.value], "type": vt[:nv.value], "facets": facets}


def oracle_state(points, rect, mode):
    return O.subdiv_state(points, rect, mode)


def _expect_facets(got, want):
    assert len(got) == len(want)
    for f, w in zip(got, want):
        w = np.array(w, np.float64).astype(np.float32)   # computeVoronoiPoint casts to float
        assert f.shape == w.shape, (f, w)
        assert np.array_equal(f, w), (f, w)


@pytest.mark.parametrize("impl", ["oracle", "product"])
@pytest.mark.parametrize("rect,mode", [(RECT, 0), (RECT, 1), (RECT_ROUNDS_TO_IT, 1)])
@pytest.mark.parametrize("case", sorted(CASES))
def test_subdiv_known_answers(case, rect, mode, impl):
    points, nxt, ends, first, facets = CASES[case]
    st = (oracle_state if impl == "oracle" else product_state)(points, rect, mode)
    assert st["next"].tolist() == nxt
    assert st["pt"][:, [0, 2]].tolist() == ends
    assert st["first_edge"][:len(first)].tolist() == first
    assert st["type"][:len(first)].tolist() == [-1] + [0] * (len(first) - 1)
    if case == "on_edge":   # the deleted quad-edge's id is reused by the first new edge (freeQEdge = 4)
        assert st["first_edge"][1] == 16 and st["next"][4][0] == 14
    if facets is not None:
        _expect_facets(st["facets"], facets)


@pytest.mark.parametrize("case", sorted(set(CASES) - {"on_edge"}))
def test_subdiv_rect_modes_agree_on_topology(case):
    """Subdiv2D(Rect2f) on a fractional rectangle moves the super-triangle by < 1 unit: the hand-traced
    topology (ids, end points, firstEdge) of cases 1-4 holds there too, on both implementations (every
    predicate sign above stays the same). Not case 5: T is exactly on P-A only for A = (30, 0)."""
    points, nxt, ends, first, _ = CASES[case]
    for impl in (oracle_state, product_state):
        st = impl(points, RECT_ROUNDS_TO_IT, 0)
        assert st["next"].tolist() == nxt
        assert st["pt"][:, [0, 2]].tolist() == ends
        assert st["first_edge"][:len(first)].tolist() == first
