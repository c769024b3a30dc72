// GVD construction (AosGvdNode::processGraph, src/aos_gvd_node.cpp:255-318) on gfx950.
//
//  g1 seed merge (gvd:84-128)                 GPU  greedy LFMIS (<= 0.5 m) + ordered member sums
//  g4 Subdiv2D inserts                       host sequential replay (subdiv2d.h explains why)
//     calcVoronoi + facet list               GPU  k_vor_faces / k_facet_count / k_facet_emit
//  g5 extractBoundaryPoints                   GPU  greedy LFMIS (1 cm key or < 5 cm)
//  g6 buildGraphFromBoundaryPoints            GPU  hashed nearest snap + pair search + occupancy
//                                                  sampling + first-passing-occurrence selection
//  g7 filterNodesAndEdgesOutsideGrid          GPU  compaction
//  g8 TL/TR/BL/BR label points                GPU  per (row, label) arg-min / castRay
//  g9 publishGraph labels                     GPU  per node
#include <algorithm>
#include <chrono>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <exception>
#include <limits>
#include <thread>

#include "aos_ctx.h"
#include "dev_prims_device.h"
#include "subdiv2d.h"

namespace aos {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
template <class T> static T *dev(DevBuf &b, size_t n) { return static_cast<T *>(b.ensure(sizeof(T) * std::max<size_t>(n, 1))); }

struct GridG {
    double ox, oy, res;             // info.origin, (double)info.resolution
    int W, H;
    double minx, maxx, miny, maxy;  // origin + width * resolution (float product) gvd:278-281
    double diag2;                   // sqrt(gw^2 + gh^2) * 2 (findVoronoiBoundaryPointNearEndpoint)
    double diag3;                   // * 3 (castRay)
    double step;                    // castRay step: max(0.01, res * 0.5)
};

__device__ __forceinline__ bool occ_trunc(const int8_t *sk, const GridG &g, double px, double py) {
    double fx = (px - g.ox) / g.res, fy = (py - g.oy) / g.res;
    // static_cast<int>: x86 gives INT_MIN out of range; either way such samples are outside
    if (!(fx > -1.0 && fx < (double)g.W) || !(fy > -1.0 && fy < (double)g.H)) return false;
    int mx = (int)fx, my = (int)fy;
    if (mx >= 0 && mx < g.W && my >= 0 && my < g.H) return sk[(size_t)my * g.W + mx] == 100;
    return false;
}

// ------------------------------------------------------------------ g1 merge
// merged seed r = the mean of its leader's members (owner == leader, the leader first), summed in index
// order as voronoiSeedsCallback does (gvd:116-123). Members conflict with the leader (<= 0.5 m), so they
// sit in its 3 x 3 cells of the de-duplication's index: taken in increasing index, one pass each.
// (h_merged / h_sc: pinned host copies of the means, and of the count and the merge's error word (h_sc[0], [1]),
// stored by the same launch: no copy-engine read-backs)
__global__ void k_merge_members(const double2 *raw, CellIdx ci, const int *owner, const int *leaders, const int *count,
                                double2 *merged, double2 *h_merged, int *h_sc, const int *err) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r == 0) { h_sc[0] = *count; h_sc[1] = *err; }
    if (r >= *count) return;
    const int L = leaders[r];
    const double2 pl = raw[L];
    int cx, cy;
    hash_cell(ci.h, pl.x, pl.y, cx, cy);
    double sx = 0.0, sy = 0.0;
    int cnt = 0, cur = -1;
    for (;;) {
        int nxt = INT_MAX;
        for (int yy = max(cy - 1, 0); yy <= min(cy + 1, ci.h.ny - 1); ++yy) {
            int k0, k1;
            ci_row(ci, yy, cx, k0, k1);
            for (int k = k0; k < k1; ++k) {
                const int j = ci.items[k];
                if (j > cur && j < nxt && owner[j] == L) nxt = j;
            }
        }
        if (nxt == INT_MAX) break;
        const double2 q = raw[nxt];
        sx += q.x; sy += q.y;
        ++cnt;
        cur = nxt;
    }
    merged[r] = h_merged[r] = make_double2(sx / (double)cnt, sy / (double)cnt);
}

// ------------------------------------------------------------------ g5/g6 helpers
// Sizes the host has not read stay on the device: M boundary points (*M_dev, <= no), P pairs
// (poff[no]), Mn nodes, ... Kernels are launched over host-known upper bounds and return past the
// device count; the per-item arrays the scans read are zero there.

// findNearestBoundaryPoint (gvd:812-824): first strict minimum of |bp_i - q| over i = the (distance, i)
// lexicographic minimum. The boundary points are the kept candidates of the extractBoundaryPoints
// de-duplication (pos_of[c] = their index), found through its cell index (cells >= 0.5 m). The nearest
// lies within 5 cm (extractBoundaryPoints kept it or a conflicting point within 5 cm / the same 1 cm
// key), inside q's 3 x 3 cells; brute force otherwise.
// evals (nullable, aos_params.gvd_count_evals): the number of candidates examined, added per thread
__device__ __forceinline__ void eval_add(unsigned long long *evals, int k, long long v) {
    if (evals && v > 0) atomicAdd(&evals[k], (unsigned long long)v);
}
__global__ void k_nearest(const double2 *occ, int n_occ, CellIdx ci, const int *pos_of, const double2 *bp, const int *M_dev,
                          int *near_out, unsigned long long *evals) {   // near_out: the ft array's first 2E ints
    int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_occ) return;
    const double2 q = occ[o];
    int cx, cy;
    hash_cell(ci.h, q.x, q.y, cx, cy);
    double best = 1.7976931348623157e308;
    int bi = -1;
    long long ne = 0;
    struct PosPt { int i; double2 p; };
    for (int yy = max(cy - 1, 0); yy <= min(cy + 1, ci.h.ny - 1); ++yy) {
        int k0, k1;
        ci_row(ci, yy, cx, k0, k1);
        ne += k1 - k0;
        walk_items<8>(ci.items, k0, k1, [&](int c) { return PosPt{pos_of[c], occ[c]}; }, [&](int, const PosPt &v) {
            if (v.i < 0) return true;
            double dx = v.p.x - q.x, dy = v.p.y - q.y, d = sqrt(dx * dx + dy * dy);
            if (d < best || (d == best && v.i < bi)) { best = d; bi = v.i; }
            return true;
        });
    }
    if (!(best < 0.05)) {  // safety net: exact brute force
        const int M = *M_dev;
        best = 1.7976931348623157e308; bi = -1;
        for (int i = 0; i < M; ++i) {
            double dx = bp[i].x - q.x, dy = bp[i].y - q.y, d = sqrt(dx * dx + dy * dy);
            if (d < best) { best = d; bi = i; }
        }
        ne += M;
    }
    near_out[o] = bi;
    eval_add(evals, 0, ne);
}

// all pairs i < j with 1e-6 < |bp_i - bp_j| <= 0.5 (gvd:861-894), CSR per i, j ascending (count pass:
// poff == nullptr; entries past cap are dropped and flag the caller, who reruns with the exact size)
// (poff == nullptr: the count pass, with the pairs' exclusive scan fused: pcount = the offsets, [no] = total)
template <bool COUNT>
__device__ __forceinline__ int pairs_of(int i, const double2 *bp, CellIdx ci, const int *pos_of, const double2 *occ,
                                        const int *poff, int2 *plist, int cap, unsigned long long *evals) {
    const double2 p = bp[i];
    int cx, cy;
    hash_cell(ci.h, p.x, p.y, cx, cy);
    int c = 0, w = COUNT ? 0 : poff[i];
    long long ne = 0;
    struct PosPt { int j; double2 q; };
    for (int yy = max(cy - 1, 0); yy <= min(cy + 1, ci.h.ny - 1); ++yy) {
        int k0, k1;
        ci_row(ci, yy, cx, k0, k1);
        ne += k1 - k0;
        walk_items<8>(ci.items, k0, k1, [&](int cc) { return PosPt{pos_of[cc], occ[cc]}; }, [&](int, const PosPt &v) {
            const int j = v.j;
            if (j <= i) return true;
            double dx = p.x - v.q.x, dy = p.y - v.q.y, d = sqrt(dx * dx + dy * dy);
            if (d <= 0.5 && d > 1e-6) {
                if (!COUNT && w + c < cap) {  // insertion into the sorted run
                    int pos = w + c;
                    while (pos > w && plist[pos - 1].y > j) { plist[pos] = plist[pos - 1]; --pos; }
                    plist[pos] = make_int2(i, j);
                }
                ++c;
            }
            return true;
        });
    }
    eval_add(evals, 1, ne);
    return c;
}
__global__ void k_pairs_count(const double2 *bp, int no, const int *M_dev, CellIdx ci, const int *pos_of, const double2 *occ,
                              int *pcount, unsigned long long *evals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= no) return;
    pcount[i] = i < *M_dev ? pairs_of<true>(i, bp, ci, pos_of, occ, nullptr, nullptr, 0, evals) : 0;
}
__global__ void k_pairs(const double2 *bp, int no, const int *M_dev, CellIdx ci, const int *pos_of, const double2 *occ,
                        const int *poff, int2 *plist, int cap, unsigned long long *evals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= no || i >= *M_dev) return;
    (void)pairs_of<false>(i, bp, ci, pos_of, occ, poff, plist, cap, evals);
}

// Candidate edge occurrences ft: [0, E) the Voronoi edges (k_nearest writes both ends' nearest boundary
// points: ft[c] = (near(2c), near(2c + 1))), [E, E + P) the pairs (P = poff[no] <= cap; k_pairs writes (i, j),
// j ascending per i). from/to keep the direction in which the reference samples the segment.

// edgePassesThroughOccupiedPixels (gvd:320-359) on the framed skeleton. Samples whose t-range
// cannot touch the grid are skipped (they read no cell), which keeps far hull edges cheap. A passing
// occurrence (a != b, both valid, no occupied sample) is counted in the group of its smaller node
// (grank: its rank there) for the first-occurrence selection.
// Round 5: the samples of a block's occurrences are flattened and spread over all of its threads (an
// exclusive scan of the per-occurrence sample counts in LDS), each thread taking kOccPer consecutive samples per
// round (one binary search for the first one's occurrence) whose lookups are in flight together, and a sample
// of an occurrence already hit is skipped.
// Round 4 walked each occurrence's samples on one lane, 16 per round: a wave waited for its longest edge (a
// passing edge between two tree rows: every sample read), ~90 us per C2 frame. The hit test is an OR over
// the samples, so the order they are read in never shows.
constexpr int kOccTB = 256, kOccPer = 8;
__global__ __launch_bounds__(kOccTB) void k_occupancy(const int2 *ft, const int *poff, int no, int ne, int cap,
                                                      const double2 *bp, const int8_t *sk, GridG g, int *pass, int *gcnt,
                                                      int *grank, unsigned long long *evals) {
    __shared__ int pre[kOccTB + 1], hit_s[kOccTB], wsum[kOccTB / 64], tot_s;
    __shared__ double sx_s[kOccTB], sy_s[kOccTB], ux_s[kOccTB], uy_s[kOccTB], len_s[kOccTB];
    __shared__ int num_s[kOccTB], i0_s[kOccTB];
    const int tid = threadIdx.x, c = blockIdx.x * kOccTB + tid;
    const int nocc = ne + min(poff[no], cap);
    int2 e2 = make_int2(-1, -1);
    bool valid = false;
    int nsamp = 0;
    if (c < nocc) {
        e2 = ft[c];
        valid = e2.x >= 0 && e2.y >= 0 && e2.x != e2.y;
    }
    if (valid) {
        const double2 s = bp[e2.x], e = bp[e2.y];
        double ex = e.x - s.x, ey = e.y - s.y;
        double len = sqrt(ex * ex + ey * ey);
        if (len >= 1e-6) {
            const double step = g.res * 0.5;
            double q = len / step;
            int num = (q > -2147483649.0 && q < 2147483647.0) ? (int)q + 1 : INT_MIN + 1;  // x86 int conversion
            // candidate sample window: cells exist only for world x in (ox - res, ox + W res), same for y
            int i0 = 0, i1 = num;
            if (num > 64) {
                double lo_t = 0.0, hi_t = 1.0;
                const double gx0 = g.ox - 2 * g.res, gx1 = g.ox + (g.W + 2) * g.res;
                const double gy0 = g.oy - 2 * g.res, gy1 = g.oy + (g.H + 2) * g.res;
                auto clip = [&](double p0, double dp, double a, double b) {
                    if (dp == 0.0) { if (p0 < a || p0 > b) { lo_t = 1.0; hi_t = 0.0; } return; }
                    double t0 = (a - p0) / dp, t1 = (b - p0) / dp;
                    if (t0 > t1) { double t = t0; t0 = t1; t1 = t; }
                    lo_t = fmax(lo_t, t0); hi_t = fmin(hi_t, t1);
                };
                clip(s.x, ex, gx0, gx1);
                clip(s.y, ey, gy0, gy1);
                if (lo_t > hi_t) { i0 = 1; i1 = 0; }
                else { i0 = max(0, (int)floor(lo_t * num) - 2); i1 = min(num, (int)ceil(hi_t * num) + 2); }
            }
            if (num >= 0 && i1 >= i0) nsamp = i1 - i0 + 1;
            sx_s[tid] = s.x; sy_s[tid] = s.y; ux_s[tid] = ex / len; uy_s[tid] = ey / len; len_s[tid] = len;
            num_s[tid] = num; i0_s[tid] = i0;
        }
    }
    hit_s[tid] = 0;
    const int before = block_excl_scan<kOccTB>(nsamp, wsum, &tot_s);   // (synchronises)
    pre[tid] = before;
    if (tid == 0) pre[kOccTB] = tot_s;
    __syncthreads();
    const int T = pre[kOccTB];
    long long nread = 0;
    for (int q0 = 0; q0 < T; q0 += kOccTB * kOccPer) {
        bool h[kOccPer];
        int oo[kOccPer];
        // the thread's kOccPer consecutive samples: one search for the first one's occurrence, then forward
        const int qb = q0 + tid * kOccPer;
        int o = 0;
        if (qb < T) {
            int lo = 0, hi = kOccTB - 1;   // the occurrence o with pre[o] <= qb < pre[o + 1]
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (pre[mid] <= qb) lo = mid; else hi = mid - 1;
            }
            o = lo;
        }
#pragma unroll
        for (int u = 0; u < kOccPer; ++u) {
            const int q = qb + u;
            h[u] = false;
            oo[u] = -1;
            if (q >= T) continue;
            while (pre[o + 1] <= q) ++o;   // (q < T = pre[kOccTB]: o stays below kOccTB)
            if (hit_s[o]) continue;
            oo[u] = o;
            const int i = i0_s[o] + (q - pre[o]), num = num_s[o];
            const double t = (i == num) ? 1.0 : ((double)i / (double)num);
            const double len = len_s[o];
            const double px = sx_s[o] + (t * ux_s[o]) * len, py = sy_s[o] + (t * uy_s[o]) * len;
            h[u] = occ_trunc(sk, g, px, py);
            ++nread;
        }
#pragma unroll
        for (int u = 0; u < kOccPer; ++u)
            if (h[u]) hit_s[oo[u]] = 1;
        __syncthreads();
    }
    if (evals) {
        for (int o = 32; o > 0; o >>= 1) nread += __shfl_xor(nread, o);
        if ((tid & 63) == 0) eval_add(evals, 2, nread);
    }
    if (c >= nocc) return;
    if (!valid) { pass[c] = 0; return; }
    const bool hit = hit_s[tid] != 0;
    pass[c] = hit ? 0 : 1;
    if (!hit) grank[c] = atomicAdd(&gcnt[min(e2.x, e2.y)], 1);
}
// The edge of key (a < b) is added by its first passing occurrence (gvd:840-857): a passing occurrence
// is selected iff no smaller passing occurrence in its group (smaller node a) has the same larger node.
__global__ void k_group_scatter(const int2 *ft, const int *pass, const int *poff, int no, int ne, int cap, const int *goff,
                                const int *grank, int *glist) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ne + min(poff[no], cap) || !pass[c]) return;
    glist[goff[min(ft[c].x, ft[c].y)] + grank[c]] = c;
}
__global__ void k_select(const int2 *ft, const int *pass, const int *poff, int no, int ne, int cap, const int *goff,
                         const int *glist, int *selected) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ne + cap) return;
    int sel = 0;
    if (c < ne + min(poff[no], cap) && pass[c]) {
        const int a = min(ft[c].x, ft[c].y), b = max(ft[c].x, ft[c].y);
        sel = 1;
        for (int k = goff[a]; k < goff[a + 1]; ++k) {
            const int c2 = glist[k];
            if (c2 < c && max(ft[c2].x, ft[c2].y) == b) { sel = 0; break; }
        }
    }
    selected[c] = sel;
}

// ------------------------------------------------------------------ g7 filter
__global__ void k_inside(const double2 *bp, int no, const int *M_dev, GridG g, int *f) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= no) return;
    int v = 0;
    if (i < *M_dev) {
        double2 p = bp[i];
        v = p.x >= g.minx && p.x <= g.maxx && p.y >= g.miny && p.y <= g.maxy;
    }
    f[i] = v;
}
// selected candidate c -> record (a<b); keep if both nodes stay (and stay distinct); 0 past the candidates
// (and the kept nodes gathered, nodes[pos[i]] = bp[i] for i < no: k_gather_nodes folded in)
__global__ void k_edge_keep(const int *selected, const int2 *ft, int ncap, const int *inside, const int *pos, int *keep,
                            const double2 *bp, int no, double2 *nodes) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < no && inside[c]) nodes[pos[c]] = bp[c];
    int k = 0;
    if (c < ncap && selected[c]) {
        int a = min(ft[c].x, ft[c].y), b = max(ft[c].x, ft[c].y);
        k = inside[a] && inside[b] && pos[a] != pos[b];
    }
    if (c < ncap) keep[c] = k;
}
__global__ void k_edge_emit(const int *keep, const int *kpos, const int2 *ft, int ncap, const int *pos, const double2 *nodes,
                            int *edges, float *len) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncap || !keep[c]) return;
    int a = pos[min(ft[c].x, ft[c].y)], b = pos[max(ft[c].x, ft[c].y)];
    if (a > b) { int t = a; a = b; b = t; }
    double dx = nodes[b].x - nodes[a].x, dy = nodes[b].y - nodes[a].y;  // (to - from).norm()
    int r = kpos[c];
    edges[2 * r] = a; edges[2 * r + 1] = b;
    len[r] = (float)sqrt(dx * dx + dy * dy);
}

// ------------------------------------------------------------------ g8 label points
struct LabelRow { double ex, ey, ox, oy; double deg, cs, sn; };  // endpoint, other endpoint, angle, host cos/sin
// one workgroup per (row, label): arg-min over the filtered nodes (gvd:731-774); castRay fallback (:788)
// Pass 0 reads only the nodes of the 3 x 3 cells (of >= 5.01 m: the cell index cn over the nodes)
// around the endpoint, which hold every node with z <= 25 (1 + 1e-12); a job scanned all ~10^5 nodes
// before (≈ 177 us per C2 frame).
__global__ __launch_bounds__(256) void k_label_points(const LabelRow *jobs, int nj, const double2 *nodes, const int *Mn_dev,
                                                      GridG g, const int8_t *sk, CellIdx cn, double2 *pts, int *valid,
                                                      unsigned long long *evals) {
    const int jb = blockIdx.x;
    if (jb >= nj) return;
    const int Mn = *Mn_dev;
    const LabelRow J = jobs[jb];
    double mdx = J.ox - J.ex, mdy = J.oy - J.ey;
    double ml = sqrt(mdx * mdx + mdy * mdy);
    if (ml < 1e-6) { mdx = 1.0; mdy = 0.0; }
    else { mdx = mdx / ml; mdy = mdy / ml; }
    const double outx = -mdx, outy = -mdy, perx = -mdy, pery = mdx;
    const bool m90 = fabs(J.deg - (-90.0)) < 1e-6, p90 = fabs(J.deg - 90.0) < 1e-6;
    // The reference returns the nearest valid candidate of the first radius in {5, 7, 9, diag2} that
    // has one, i.e. the arg-min (first strict minimum) over all valid candidates. Pass 0 evaluates
    // the exact test only for nodes with z <= 25 (1 + 1e-12) (a superset of dist <= 5); if it finds a
    // candidate, the global arg-min is among them. Pass 1 tests every node of the 5 x 5 cells around the
    // endpoint: a node outside them is at least 2 cells (>= 10 m) away, so a candidate nearer than that
    // is the arg-min. Pass 2 (rare) scans everything. (Round 3 went from pass 0 straight to the full
    // scan: 472 us of k_label_points at C3, where many endpoints have their node 5-10 m away.)
    __shared__ double sb[256];
    __shared__ int si[256];
    int cx, cy;
    hash_cell(cn.h, J.ex, J.ey, cx, cy);
    const double two_cells = 2.0 / cn.h.inv * (1.0 - 1e-9);
    long long ntest = 0;
    for (int pass = 0; pass < 3; ++pass) {
        double best = 1.7976931348623157e308;
        int bi = INT_MAX;
        auto test = [&](int i) {
            ++ntest;
            double dx = nodes[i].x - J.ex, dy = nodes[i].y - J.ey;
            double z = dx * dx + dy * dy;
            if (pass == 0 && !(z <= 25.0 * (1.0 + 1e-12))) return;
            double dist = sqrt(z);
            if (dist < 0.5 || dist > fmax(9.0, g.diag2)) return;
            double nx = dx, ny = dy;
            if (z > 0.0) { double s = sqrt(z); nx = dx / s; ny = dy / s; }
            if (outx * nx + outy * ny < 0.0) return;
            double dp = perx * nx + pery * ny;
            if (m90) { if (dp > 0.0) return; }
            else if (p90) { if (dp < 0.0) return; }
            if (dist < best || (dist == best && i < bi)) { best = dist; bi = i; }
        };
        if (pass == 0) {
            for (int yy = max(cy - 1, 0); yy <= min(cy + 1, cn.h.ny - 1); ++yy) {
                int k0, k1;
                ci_row(cn, yy, cx, k0, k1);
                for (int k = k0 + threadIdx.x; k < k1; k += blockDim.x) test(cn.items[k]);
            }
        } else if (pass == 1) {
            for (int yy = max(cy - 2, 0); yy <= min(cy + 2, cn.h.ny - 1); ++yy) {
                const int b = yy * cn.h.nx;
                const int k0 = cn.start[b + max(cx - 2, 0)], k1 = cn.start[b + min(cx + 2, cn.h.nx - 1) + 1];
                for (int k = k0 + threadIdx.x; k < k1; k += blockDim.x) test(cn.items[k]);
            }
        } else {
            for (int i = threadIdx.x; i < Mn; i += blockDim.x) test(i);
        }
        sb[threadIdx.x] = best; si[threadIdx.x] = bi;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (threadIdx.x < o) {
                double b2 = sb[threadIdx.x + o]; int i2 = si[threadIdx.x + o];
                if (b2 < sb[threadIdx.x] || (b2 == sb[threadIdx.x] && i2 < si[threadIdx.x])) { sb[threadIdx.x] = b2; si[threadIdx.x] = i2; }
            }
            __syncthreads();
        }
        // (uniform: every thread reads the same shared values)
        if (si[0] != INT_MAX && (pass != 1 || sb[0] < two_cells)) break;
        __syncthreads();
    }
    eval_add(evals, 3, ntest);
    if (threadIdx.x != 0) return;
    if (evals) {   // the radii the reference scans all nodes for: 5, 7, 9, 2 diag until one has a candidate
        const double r[4] = {5.0, 7.0, 9.0, g.diag2};
        int scans = 4;
        if (si[0] != INT_MAX)
            for (int k = 0; k < 4; ++k)
                if (sb[0] <= r[k]) { scans = k + 1; break; }
        atomicAdd(&evals[4], (unsigned long long)scans);
    }
    if (si[0] != INT_MAX) { pts[jb] = nodes[si[0]]; valid[jb] = 1; return; }
    // castRay gvd:558-684 (angles +-90: cos/sin from the host table in J.deg's sign)
    double ex = J.ox - J.ex, ey = J.oy - J.ey;
    double d = sqrt(ex * ex + ey * ey);
    if (d < 1e-6) { ex = 1.0; ey = 0.0; } else { ex = ex / d; ey = ey / d; }
    double ox_ = -ex, oy_ = -ey, px = -ey, py = ex;
    double rx, ry;
    const double cs = J.cs, sn = J.sn;  // std::cos/std::sin of the angle, evaluated by the host libm
    if (J.deg > 0) { rx = cs * ox_ + sn * px; ry = cs * oy_ + sn * py; }
    else { rx = cs * ox_ + sn * (-px); ry = cs * oy_ + sn * (-py); }
    { double z = rx * rx + ry * ry; if (z > 0.0) { double q = sqrt(z); rx = rx / q; ry = ry / q; } }
    double cur = 0.5;  // min_distance passed by findVoronoiBoundaryPointNearEndpoint
    double resx = 0, resy = 0;
    bool done = false, ended = false;
    while (!done && !ended) {
        double px[16], py[16];
        bool valid[16], ins[16], occ[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            valid[j] = cur <= g.diag3;
            px[j] = J.ex + rx * cur; py[j] = J.ey + ry * cur;
            cur += g.step;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            ins[j] = px[j] >= g.minx && px[j] <= g.maxx && py[j] >= g.miny && py[j] <= g.maxy;
            occ[j] = valid[j] && ins[j] && occ_trunc(sk, g, px[j], py[j]);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (done || ended) continue;
            if (!valid[j]) { ended = true; continue; }
            if (!ins[j]) { resx = fmax(g.minx, fmin(g.maxx, px[j])); resy = fmax(g.miny, fmin(g.maxy, py[j])); done = true; continue; }
            if (occ[j]) { resx = px[j]; resy = py[j]; done = true; }
        }
    }
    if (!done) {
        double fx = J.ex + rx * g.diag3, fy = J.ey + ry * g.diag3;
        if (!(fx >= g.minx && fx <= g.maxx && fy >= g.miny && fy <= g.maxy)) {
            fx = fmax(g.minx, fmin(g.maxx, fx)); fy = fmax(g.miny, fmin(g.maxy, fy));
        }
        resx = fx; resy = fy;
    }
    pts[jb] = make_double2(resx, resy);
    valid[jb] = 1;
}

// ------------------------------------------------------------------ g9 node labels (publishGraph gvd:920-995)
// A node matches label point j iff |dx|, |dy| < 0.1 (and the reference's distance test), so only the
// label points of its 3 x 3 cells of the label points' cell index cq (cells >= 0.1 m) can match; the
// matches are put back in (r, k) order. More than kNodeMatch matches: the plain loop over every label
// point. Count pass (off == nullptr) over [0, no): 0 past the Mn nodes.
constexpr int kNodeMatch = 16;
// node i's label mask, first matching row and number of (row, type) entries; off != nullptr: the entries too
__device__ __forceinline__ int node_labels_of(int i, const double2 *nodes, const double2 *lp, const int *lv, int n_rows,
                                              const CellIdx &cq, int &mask_out, int &cidx_out, const int *off, int *lcl,
                                              int *lty) {
    const double2 p = nodes[i];
    int m = 0, ci = -1, cnt = 0;
    const int w = off ? off[i] : 0;
    {
        int js[kNodeMatch], nm = 0;
        bool over = false;
        int cx, cy;
        hash_cell(cq.h, p.x, p.y, cx, cy);
        for (int yy = max(cy - 1, 0); yy <= min(cy + 1, cq.h.ny - 1); ++yy) {
            int k0, k1;
            ci_row(cq, yy, cx, k0, k1);
            for (int q = k0; q < k1; ++q) {
                const int j = cq.items[q];
                double dx = p.x - lp[j].x, dy = p.y - lp[j].y;
                if (!(fabs(dx) < 0.1) || !(fabs(dy) < 0.1)) continue;
                if (sqrt(dx * dx + dy * dy) < 0.1) {
                    if (nm < kNodeMatch) js[nm++] = j;
                    else over = true;
                }
            }
        }
        if (!over) {
            for (int a = 1; a < nm; ++a)   // (r, k) order
                for (int b = a; b > 0 && js[b - 1] > js[b]; --b) { const int t = js[b]; js[b] = js[b - 1]; js[b - 1] = t; }
            for (int a = 0; a < nm; ++a) {
                const int r = js[a] >> 2, k = js[a] & 3;
                m |= 1 << k;
                if (off) { lcl[w + cnt] = r; lty[w + cnt] = k; }
                ++cnt;
                if (ci == -1) ci = r;
            }
            mask_out = m; cidx_out = ci;
            return cnt;
        }
    }
    for (int r = 0; r < n_rows; ++r)
        for (int k = 0; k < 4; ++k) {
            if (!lv[4 * r + k]) continue;
            double dx = p.x - lp[4 * r + k].x, dy = p.y - lp[4 * r + k].y;
            // exact prefilter: |dx| >= 0.1 implies fl(sqrt(fl(dx*dx) + fl(dy*dy))) >= sqrt(fl(0.1*0.1)) = 0.1
            // (monotone rounding), so the reference's test below is false anyway
            if (!(fabs(dx) < 0.1) || !(fabs(dy) < 0.1)) continue;
            if (sqrt(dx * dx + dy * dy) < 0.1) {
                m |= 1 << k;
                if (off) { lcl[w + cnt] = r; lty[w + cnt] = k; }
                ++cnt;
                if (ci == -1) ci = r;
            }
        }
    mask_out = m; cidx_out = ci;
    return cnt;
}
// count pass over [0, no) (0 past the Mn nodes)
__global__ void k_node_labels_count(const double2 *nodes, int no, const int *Mn_dev, const double2 *lp, const int *lv, int n_rows,
                                    CellIdx cq, int *mask, int *cidx, int *count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= no) return;
    int cnt = 0;
    if (i < *Mn_dev) {
        int m = 0, ci = -1;
        cnt = node_labels_of(i, nodes, lp, lv, n_rows, cq, m, ci, nullptr, nullptr, nullptr);
        mask[i] = m; cidx[i] = ci;
    }
    count[i] = cnt;
}
// fill pass over the Mn nodes: the (row, type) entries at off[i]
__global__ void k_node_labels_fill(const double2 *nodes, int Mn, const double2 *lp, const int *lv, int n_rows, CellIdx cq,
                                   const int *off, int *lcl, int *lty) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Mn) return;
    int m, ci;
    (void)node_labels_of(i, nodes, lp, lv, n_rows, cq, m, ci, off, lcl, lty);
}

// ------------------------------------------------------------------ output gather
// The GvdGraph arrays (4-byte words) packed back to back into the state's pinned host buffer by one launch (no
// device staging buffer and no copy-engine read-back).
constexpr int kMaxSegs = 12;
struct SegList { const int *src[kMaxSegs]; long long off[kMaxSegs + 1]; int n; };
// (four words per thread, one 16-byte store: host memory is written across PCIe, where 4-byte stores ran at
// ~20 GB/s, 59 us for the C2 graph)
__global__ void k_gather_words(SegList L, int *dst) {
    const long long i0 = 4 * ((long long)blockIdx.x * blockDim.x + threadIdx.x), n = L.off[L.n];
    if (i0 >= n) return;
    int v[4];
    int k = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long long i = i0 + u;
        v[u] = 0;
        if (i >= n) continue;
        while (i >= L.off[k + 1]) ++k;
        v[u] = L.src[k][i - L.off[k]];
    }
    if (i0 + 4 <= n) {
        *reinterpret_cast<int4 *>(dst + i0) = make_int4(v[0], v[1], v[2], v[3]);
    } else {
        for (int u = 0; u < 4 && i0 + u < n; ++u) dst[i0 + u] = v[u];
    }
}

// ------------------------------------------------------------------ g4 facets (calcVoronoi + getVoronoiFacetList)
// The Subdiv2D inserts are replayed on the host; the facets they imply are built here from the raw
// quad-edge arrays (8 ints per quad-edge: next[4], pt[4]). calcVoronoi (subdivision2d.cpp) walks
// quad-edges q = 4.. in id order, left face of q*4 before its right face, and the first of those
// that touches a triangle computes its circumcentre (computeVoronoiPoint from that edge and its
// NEXT_AROUND_LEFT / NEXT_AROUND_RIGHT successor). A failed computation (det = 0 or huge) leaves the
// face unset for the next edge of the triangle. So a face's value is: over its 3 boundary edges in
// that key order (key = 2*q + right), the first successful computation; (0, 0) = vtx[0] if none.
__device__ __forceinline__ int q_get(const int *qe, int e, int t) {
    const int x = qe[(e >> 2) * 8 + ((e + t) & 3)];
    return (x & ~3) + ((x + (t >> 4)) & 3);
}
__device__ __forceinline__ int q_org(const int *qe, int e) { return qe[(e >> 2) * 8 + 4 + (e & 3)]; }
__device__ __forceinline__ int q_dst(const int *qe, int e) { return qe[(e >> 2) * 8 + 4 + ((e + 2) & 3)]; }

__device__ bool d_voronoi_point(float2 o0, float2 d0, float2 o1, float2 d1, float2 &r) {
    double a0 = d0.x - o0.x, b0 = d0.y - o0.y;
    double c0 = -0.5 * (a0 * (d0.x + o0.x) + b0 * (d0.y + o0.y));
    double a1 = d1.x - o1.x, b1 = d1.y - o1.y;
    double c1 = -0.5 * (a1 * (d1.x + o1.x) + b1 * (d1.y + o1.y));
    double det = a0 * b1 - a1 * b0;
    if (det == 0) return false;
    det = 1. / det;
    r.x = (float)((b0 * c1 - b1 * c0) * det);
    r.y = (float)((a1 * c0 - a0 * c1) * det);
    return fabsf(r.x) < FLT_MAX * 0.5f && fabsf(r.y) < FLT_MAX * 0.5f;
}

// face[2*q + side]: side 0 = left face of q*4 (pt[3]), side 1 = right face (pt[1])
__global__ void k_vor_faces(const int *qe, int n_rec, const float2 *vp, float2 *face, int *err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *err = 0;   // (k_facet_count's flag, launched after this kernel)
    if (i >= 2 * n_rec) return;
    const int q = i >> 1, side = i & 1;
    float2 res = make_float2(0.f, 0.f);
    if (q >= 1 && qe[q * 8] > 0) {   // allocated quad-edge
        const int d1 = q * 4 + 2 * side, d2 = q_get(qe, d1, 0x13), d3 = q_get(qe, d2, 0x13);
        int k[3];
        const int ds[3] = {d1, d2, d3};
#pragma unroll
        for (int j = 0; j < 3; ++j) k[j] = (ds[j] >> 2) < 4 ? INT_MAX : 2 * (ds[j] >> 2) + ((ds[j] & 2) ? 1 : 0);
        if (k[0] > k[1]) { int t = k[0]; k[0] = k[1]; k[1] = t; }
        if (k[1] > k[2]) { int t = k[1]; k[1] = k[2]; k[2] = t; }
        if (k[0] > k[1]) { int t = k[0]; k[0] = k[1]; k[1] = t; }
        for (int j = 0; j < 3 && k[j] != INT_MAX; ++j) {
            const int e0 = (k[j] >> 1) * 4, e1 = (k[j] & 1) ? q_get(qe, e0, 0x31) : q_get(qe, e0, 0x13);
            float2 r;
            if (d_voronoi_point(vp[q_org(qe, e0)], vp[q_dst(qe, e0)], vp[q_org(qe, e1)], vp[q_dst(qe, e1)], r)) { res = r; break; }
        }
    }
    face[i] = res;
}

// getVoronoiFacetList({}) + VoronoiDiagram edges (voronoi_diagram.cpp:97-114): for each real vertex
// k >= 4 in id order, walk t = rotate(firstEdge, 1) by NEXT_AROUND_LEFT; a facet of n >= 2 points
// gives the edges (p_i, p_(i+1 mod n)).
constexpr int kMaxFacet = 1 << 16;
__device__ __forceinline__ float2 dual_face(const float2 *face, int t) { return face[2 * (t >> 2) + ((t & 3) == 1 ? 1 : 0)]; }

// (the facet sizes' exclusive scan is fused: off[k] = edges before vertex k, off[nv] = the total)
__global__ __launch_bounds__(256) void k_facet_count(const int *qe, const int *vfirst, const int *vtype, int nv, int *cnt,
                                                     int *off, int *err, LookBack L) {
    __shared__ int sh_vid;
    __shared__ LbScanShared sh;
    const int vid = lb_block_id(L, &sh_vid);
    const int k = vid * 256 + (int)threadIdx.x;
    int c = 0;
    if (k < nv && k >= 4 && vtype[k] == 0) {
        const int f = vfirst[k], start = (f & ~3) + ((f + 1) & 3);
        int t = start;
        do { ++c; t = q_get(qe, t, 0x13); } while (t != start && c < kMaxFacet);
        if (c >= kMaxFacet) atomicOr(err, 1);
        if (c < 2) c = 0;
    }
    if (k < nv) cnt[k] = c;
    lb_scan_store<256>(L, vid, c, nv, off, sh);
}
// OCC: the edges' ends straight as the g5 boundary-point candidates (double: edge k -> occ[2k] start, occ[2k + 1]
// end; the GVD's edges_ are double from the float facet points), else float4 edges (the markers' cells)
template <bool OCC>
__global__ void k_facet_emit(const int *qe, const int *vfirst, const int *off, const int *cnt, int nv, const float2 *face,
                             float4 *edges, double2 *occ) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nv || cnt[k] == 0) return;
    const int f = vfirst[k], start = (f & ~3) + ((f + 1) & 3), n = cnt[k];
    const int o = off[k];
    auto put = [&](int i, float2 a, float2 b) {
        if (OCC) {
            occ[2 * (size_t)(o + i)] = make_double2((double)a.x, (double)a.y);
            occ[2 * (size_t)(o + i) + 1] = make_double2((double)b.x, (double)b.y);
        } else {
            edges[o + i] = make_float4(a.x, a.y, b.x, b.y);
        }
    };
    const float2 first = dual_face(face, start);
    float2 prev = first;
    int t = q_get(qe, start, 0x13);
    for (int i = 1; i < n; ++i) {
        const float2 cur = dual_face(face, t);
        put(i - 1, prev, cur);
        prev = cur;
        t = q_get(qe, t, 0x13);
    }
    put(n - 1, prev, first);
}

// ------------------------------------------------------------------ orchestration
struct GvdScratch {
    DevBuf raw, ok, leaders, merged, owner, oidx, sowner, sidx, tmp, edges_f, occ, occ_ok, bp, kept_occ, keys, idx, skeys,
        sidx2, near_idx, pk, pidx, pskeys, psidx, pcount, poff, plist, ft, ckey, cvalid, pass, k2, occ_idx, sk2, socc, selected,
        inside, ipos, nodes, keep, kpos, edges, lens, jobs, nkeys, nidx, qkeys, qidx, lpts, lval, lmask, lcidx, lcount, loff, lcl, lty, scan_tmp,
        misc, gcnt, goff, glist, evals;
    bool gcnt_dirty = true;           // gcnt (edge groups' counts) not known to be zero
    CellScratch ci_nodes, ci_labels;  // g8 / g9 indices (g5 / g6 use the de-duplication's own)
    CellIdx cq{};
    LookBackScratch lb;               // the graph's single-pass scans
    FacetBufs fb;
};
static GvdScratch &scratch(GvdState &G) {
    if (!G.scratch) G.scratch = new GvdScratch();
    return *static_cast<GvdScratch *>(G.scratch);
}
void free_gvd_scratch(GvdState &G) {
    delete static_cast<GvdScratch *>(G.scratch);   // DevBuf members free themselves
    G.scratch = nullptr;
}

// Facets of a replayed Subdiv2D on the GPU: uploads the quad-edge state, computes every face's
// circumcentre (k_vor_faces) and the per-vertex facet sizes (k_facet_count, 0 below 2 points), and
// scans them into edge offsets. Returns the edge total (F.cnt / F.off stay on the device); h_sc =
// 2 pinned ints. The caller launches k_facet_emit into a buffer of that many float4.
static int facets_count(FacetBufs &F, const Subdiv2D &sd, Subdiv2D::Raw &R, int *h_sc, hipStream_t s, SyncEvent &sev) {
    // the quad-edge export (~6 MB at C2) is written straight into the builder's own pinned buffer (a
    // pageable copy is staged by the runtime through its own buffers and blocks the calling thread) and
    // goes up as one copy
    // (in chunks of kRawChunk records: each goes up while the next is written; one copy took ~0.15 ms after the
    // whole export at C2)
    constexpr int kRawChunk = 16384;
    const size_t total = sd.raw_bytes();
    char *hs = static_cast<char *>(F.h_stage.ensure(total));
    char *d = static_cast<char *>(F.raw.ensure(total));
    size_t sent = 0;
    R = sd.raw_into(hs, kRawChunk, [&](size_t off, size_t bytes) {
        AOS_HIP(hipMemcpyAsync(d + off, hs + off, bytes, hipMemcpyHostToDevice, s));
        sent = off + bytes;
    });
    const size_t bq = sizeof(int) * 8 * (size_t)R.n_rec, bv = sizeof(float2) * R.n_vtx, bi = sizeof(int) * R.n_vtx;
    if (bq + bv + 2 * bi != total) throw std::logic_error("Subdiv2D export: size mismatch");
    AOS_HIP(hipMemcpyAsync(d + sent, hs + sent, total - sent, hipMemcpyHostToDevice, s));
    F.qe = reinterpret_cast<int *>(d);
    const float2 *d_vp = reinterpret_cast<const float2 *>(d + bq);
    F.vf = reinterpret_cast<int *>(d + bq + bv);
    F.vt = reinterpret_cast<int *>(d + bq + bv + bi);
    float2 *d_face = dev<float2>(F.face, 2 * (size_t)R.n_rec);
    int *d_cnt = dev<int>(F.cnt, R.n_vtx + 1), *d_off = dev<int>(F.off, R.n_vtx + 2);   // off[n_vtx + 1]: walk error
    k_vor_faces<<<cdiv(2 * R.n_rec, 256), 256, 0, s>>>(F.qe, R.n_rec, d_vp, d_face, d_off + R.n_vtx + 1);
    {
        const int blocks = cdiv((long long)R.n_vtx + 1, 256);
        k_facet_count<<<blocks, 256, 0, s>>>(F.qe, F.vf, F.vt, R.n_vtx, d_cnt, d_off, d_off + R.n_vtx + 1,
                                             F.lb.take(blocks, s));
    }
    peek_to_host(h_sc, {d_off + R.n_vtx, d_off + R.n_vtx + 1, F.lb.err_word(s)}, s);
    sev.sync(s);
    if (h_sc[1]) throw std::runtime_error("Subdiv2D facet walk did not close");
    if (h_sc[2]) throw std::runtime_error("Subdiv2D facets: single-pass scan failed on the device");
    return h_sc[0];
}
static void facets_emit(FacetBufs &F, const Subdiv2D::Raw &R, float4 *edges, hipStream_t s, double2 *occ = nullptr) {
    if (occ)
        k_facet_emit<true><<<cdiv(R.n_vtx, 256), 256, 0, s>>>(F.qe, F.vf, F.off.as<int>(), F.cnt.as<int>(), R.n_vtx,
                                                             F.face.as<float2>(), nullptr, occ);
    else
        k_facet_emit<false><<<cdiv(R.n_vtx, 256), 256, 0, s>>>(F.qe, F.vf, F.off.as<int>(), F.cnt.as<int>(), R.n_vtx,
                                                              F.face.as<float2>(), edges, nullptr);
}

// publishMarkers' Voronoi cells (gvd:1098-1194): VoronoiDiagram::extractCellBoundaries
// (voronoi_diagram.cpp:209-311), a second Subdiv2D over the finite merged seeds with their own
// bounding box as the rectangle, then cell i = facet i (i < seeds, facets) with >= 3 points, closed
// when its ends are more than 1 cm apart, paired with seeds_[i] and coloured from hue = i / cells.
// Pure host work on the merged seeds: it runs on a worker thread next to the main replay.
static void cells_colours(CellsWork &W, const std::vector<double> &seeds, int ncell);
static bool markers_gpu_facets() {   // AOS_MARKERS_GPU_FACETS=1: the markers' facets on the GPU builder
    static const bool on = getenv("AOS_MARKERS_GPU_FACETS") != nullptr;
    return on;
}

static void compute_cells(CellsWork &W, int rect_mode) {
    const auto t0 = std::chrono::steady_clock::now();
    struct CellTrace {
        const double t = trace_on() ? trace_ms() : 0.0;
        ~CellTrace() { if (trace_on()) fprintf(stderr, "[aos trace cells] %.2f -> %.2f\n", t, trace_ms()); }
    } ctr;
    W.cell_off.assign(1, 0);
    W.cell_xy.clear(); W.cell_center.clear(); W.cell_rgba.clear();
    const std::vector<double> &seeds = W.seeds;   // VoronoiDiagram::seeds_ = the finite merged seeds
    const int ns = (int)seeds.size() / 2;
    if (ns == 0) return;
    double min_x = std::numeric_limits<double>::max(), max_x = std::numeric_limits<double>::lowest();
    double min_y = min_x, max_y = max_x;
    for (int i = 0; i < ns; ++i) {
        min_x = std::min(min_x, seeds[2 * i]); max_x = std::max(max_x, seeds[2 * i]);
        min_y = std::min(min_y, seeds[2 * i + 1]); max_y = std::max(max_y, seeds[2 * i + 1]);
    }
    if (max_x - min_x < 1.0) { double cx = (min_x + max_x) / 2.0; min_x = cx - 0.5; max_x = cx + 0.5; }
    if (max_y - min_y < 1.0) { double cy = (min_y + max_y) / 2.0; min_y = cy - 0.5; max_y = cy + 0.5; }
    const float rx = static_cast<float>(min_x - 1.0), ry = static_cast<float>(min_y - 1.0);
    const float rw = static_cast<float>(std::abs(max_x - min_x) + 2.0), rh = static_cast<float>(std::abs(max_y - min_y) + 2.0);
    if (rw <= 0 || rh <= 0) return;
    Subdiv2D &sd = W.sd;
    sd.reserve(ns);
    sd.init_delaunay(rx, ry, rw, rh, rect_mode);
    const float margin = 0.1f;
    for (int i = 0; i < ns; ++i) {
        float x = static_cast<float>(seeds[2 * i]), y = static_cast<float>(seeds[2 * i + 1]);
        x = std::max(rx + margin, std::min(rx + rw - margin, x));
        y = std::max(ry + margin, std::min(ry + rh - margin, y));
        sd.insert(x, y);   // insertion failures are skipped (voronoi_diagram.cpp:280-285)
    }
    if (!markers_gpu_facets()) {
        // getVoronoiFacetList on the worker's own core (calcVoronoi + the facet walk of subdiv2d.cpp, the
        // host reference of the GPU builder, bit-identical to it): the markers job then needs no stream,
        // pinned buffers or GPU time of its own; the walk costs the worker a few ms next to its replay
        std::vector<int> off;
        std::vector<float> xy;
        sd.voronoi_facets(off, xy);
        int ncell = 0;
        for (size_t f = 0; f + 1 < off.size() && (int)f < ns; ++f) {
            const int b0 = off[f], n = off[f + 1] - b0;
            if (n < 3) continue;
            for (int j = 0; j < n; ++j) { W.cell_xy.push_back(xy[2 * (b0 + j)]); W.cell_xy.push_back(xy[2 * (b0 + j) + 1]); }
            const double dx = (double)xy[2 * b0] - (double)xy[2 * (b0 + n - 1)];
            const double dy = (double)xy[2 * b0 + 1] - (double)xy[2 * (b0 + n - 1) + 1];
            if (std::sqrt(dx * dx + dy * dy) > 0.01) { W.cell_xy.push_back(xy[2 * b0]); W.cell_xy.push_back(xy[2 * b0 + 1]); }
            W.cell_off.push_back((int32_t)(W.cell_xy.size() / 2));
            ++ncell;
        }
        cells_colours(W, seeds, ncell);
        W.ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return;
    }
    // getVoronoiFacetList on the GPU (the builder of the main graph, on the worker's stream): the
    // facet of real vertex k is the start points of its k_facet_emit edges, cnt[k] of them (0 for a
    // facet of fewer than 2 points: never a cell).
    AOS_HIP(hipSetDevice(W.device));
    if (!W.stream) AOS_HIP(hipStreamCreateWithFlags(&W.stream, hipStreamNonBlocking));
    int *h_sc = static_cast<int *>(W.h.ensure(4096));
    SyncEvent sev;
    Subdiv2D::Raw R{};
    const int ne = facets_count(W.fb, sd, R, h_sc, W.stream, sev);
    const size_t need = sizeof(float4) * (size_t)std::max(ne, 1) + sizeof(int) * (size_t)R.n_vtx;
    float4 *d_e = dev<float4>(W.edges, std::max(ne, 1));
    if (ne) facets_emit(W.fb, R, d_e, W.stream);
    char *hb = static_cast<char *>(W.h.ensure(need + 4096)) + 4096;   // h_sc stays in the first 4 KiB
    const float4 *he = reinterpret_cast<const float4 *>(hb);
    const int *hcnt = reinterpret_cast<const int *>(hb + sizeof(float4) * (size_t)std::max(ne, 1));
    if (ne) AOS_HIP(hipMemcpyAsync(const_cast<float4 *>(he), d_e, sizeof(float4) * (size_t)ne, hipMemcpyDeviceToHost, W.stream));
    AOS_HIP(hipMemcpyAsync(const_cast<int *>(hcnt), W.fb.cnt.p, sizeof(int) * (size_t)R.n_vtx, hipMemcpyDeviceToHost, W.stream));
    AOS_HIP(hipStreamSynchronize(W.stream));
    int ncell = 0;
    size_t b = 0;
    for (int k = 4, i = 0; k < R.n_vtx && i < ns; ++k) {
        if (R.vtype[k] != 0) continue;
        const int n = hcnt[k];
        const size_t b0 = b;
        b += (size_t)n;
        ++i;
        if (n < 3) continue;
        for (int j = 0; j < n; ++j) { W.cell_xy.push_back(he[b0 + j].x); W.cell_xy.push_back(he[b0 + j].y); }
        const float4 f = he[b0], l = he[b0 + n - 1];
        const double dx = (double)f.x - (double)l.x, dy = (double)f.y - (double)l.y;
        if (std::sqrt(dx * dx + dy * dy) > 0.01) { W.cell_xy.push_back(f.x); W.cell_xy.push_back(f.y); }
        W.cell_off.push_back((int32_t)(W.cell_xy.size() / 2));
        ++ncell;
    }
    cells_colours(W, seeds, ncell);
    W.ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// cell i's centre and colour (gvd:1117-1145, float arithmetic as written)
static void cells_colours(CellsWork &W, const std::vector<double> &seeds, int ncell) {
    for (int i = 0; i < ncell; ++i) {
        W.cell_center.push_back(seeds[2 * i]); W.cell_center.push_back(seeds[2 * i + 1]);
        float hue = static_cast<float>(i) / std::max(1.0f, static_cast<float>(ncell));
        float saturation = 0.7f, value = 0.9f;
        float cc = value * saturation;
        float x = cc * (1.0f - std::abs(std::fmod(hue * 6.0f, 2.0f) - 1.0f));
        float m = value - cc;
        float r = 0.0f, g = 0.0f, b = 0.0f;
        if (hue < 1.0f / 6.0f) { r = cc; g = x; b = 0.0f; }
        else if (hue < 2.0f / 6.0f) { r = x; g = cc; b = 0.0f; }
        else if (hue < 3.0f / 6.0f) { r = 0.0f; g = cc; b = x; }
        else if (hue < 4.0f / 6.0f) { r = 0.0f; g = x; b = cc; }
        else if (hue < 5.0f / 6.0f) { r = x; g = 0.0f; b = cc; }
        else { r = cc; g = 0.0f; b = x; }
        W.cell_rgba.push_back(r + m); W.cell_rgba.push_back(g + m); W.cell_rgba.push_back(b + m); W.cell_rgba.push_back(0.4f);
    }
}

// The cells' worker thread. publishMarkers runs after publishGraph (gvd:310-313), so the graph is
// returned as soon as it is ready and the cells finish in the background: aos_gvd_markers_get, the
// next GVD call and release() join the job (markers_wait). An error of the job is raised by
// aos_gvd_markers_get; a job nobody asked about is discarded by the next call.
static void markers_start(GvdState &G, int rect_mode) {
    if (!G.cells) G.cells.reset(new CellsWork());
    CellsWork &W = *G.cells;
    AOS_HIP(hipGetDevice(&W.device));
    W.seeds.clear();
    for (size_t i = 0; i + 1 < G.merged_xy.size(); i += 2)
        if (std::isfinite(G.merged_xy[i]) && std::isfinite(G.merged_xy[i + 1])) {
            W.seeds.push_back(G.merged_xy[i]); W.seeds.push_back(G.merged_xy[i + 1]);
        }
    if (!W.worker.joinable())
        W.worker = std::thread([&W]() {
            std::unique_lock<std::mutex> l(W.mu);
            for (;;) {
                W.cv.wait(l, [&W] { return W.busy || W.quit; });
                if (W.quit) return;
                l.unlock();
                std::exception_ptr e;
                try { compute_cells(W, W.rect_mode); } catch (...) { e = std::current_exception(); }
                l.lock();
                W.err = e;
                W.busy = false;
                W.cv.notify_all();
            }
        });
    {
        std::lock_guard<std::mutex> l(W.mu);
        W.rect_mode = rect_mode;
        W.err = nullptr;
        W.busy = true;
    }
    W.cv.notify_all();
}

void markers_on_demand(GvdState &G) {
    markers_start(G, G.rect_mode);
    markers_wait(G, true);
    G.have_markers = true;
}

void markers_wait(GvdState &G, bool rethrow) {
    if (!G.cells) return;
    CellsWork &W = *G.cells;
    std::unique_lock<std::mutex> l(W.mu);
    W.cv.wait(l, [&W] { return !W.busy; });
    if (W.err) {
        std::exception_ptr e = W.err;
        W.err = nullptr;
        G.have_markers = false;
        if (rethrow) std::rethrow_exception(e);
    }
}


bool run_gvd_stage(GvdState &G, const aos_params &P, const GvdStageIn &in, hipStream_t s, hipEvent_t *ev) {
    HostTrace tr{"gvd"};
    GvdScratch &S = scratch(G);
    G.nodes_xy.clear(); G.labels.clear(); G.cluster_idx.clear(); G.label_counts.clear();
    G.label_clusters.clear(); G.label_types.clear(); G.edges_out.clear(); G.lengths.clear(); G.clearances.clear();
    G.n_merged = G.n_vor_edges = G.n_bpts = 0;
    G.ms_merge = G.ms_delaunay = G.ms_graph = G.ms_total = 0;
    markers_wait(G, false);
    tr.mark("markers_wait");
    G.have_markers = false;
    G.graph_ok = false;
    G.rect_mode = P.subdiv_rect_mode;
    G.merged_xy.clear(); G.row_label_xy.clear(); G.row_label_valid.clear();
    if (G.cells) { G.cells->cell_off.assign(1, 0); G.cells->ms = 0; }
    int *h_sc = static_cast<int *>(G.h_misc.ensure(4096));
    const int n = in.n_seeds;
    AOS_HIP(hipEventRecord(ev[6], s));
    if (n <= 0) return false;  // processGraph: voronoi_seeds_.empty() -> return (gvd:257)

    GridG g{};
    g.ox = in.info.origin_x; g.oy = in.info.origin_y; g.res = (double)in.info.resolution;
    g.W = (int)in.info.width; g.H = (int)in.info.height;
    g.minx = in.info.origin_x; g.maxx = g.minx + in.info.width * in.info.resolution;
    g.miny = in.info.origin_y; g.maxy = g.miny + in.info.height * in.info.resolution;
    {
        double gw = in.info.width * in.info.resolution, gh = in.info.height * in.info.resolution;
        g.diag2 = std::sqrt(gw * gw + gh * gh) * 2.0;
        g.diag3 = std::sqrt(gw * gw + gh * gh) * 3.0;
        g.step = in.info.resolution * 0.5;
        if (g.step < 0.01) g.step = 0.01;
    }

    // ---- g1 merge
    double2 *d_raw = dev<double2>(S.raw, n);
    // seeds in and merged seeds out through the state's pinned buffer (a pageable copy is staged by the
    // runtime and, measured on the streaming map, could stall ~20 ms behind unrelated copy traffic)
    double *h_seeds = static_cast<double *>(G.h_seeds.ensure(sizeof(double2) * (size_t)n));
    std::memcpy(h_seeds, in.seeds_host, sizeof(double2) * (size_t)n);
    AOS_HIP(hipMemcpyAsync(d_raw, h_seeds, sizeof(double2) * n, hipMemcpyHostToDevice, s));
    tr.mark("h2d");
    const HashG hm = make_hash_n(g.minx - 60.0, g.maxx + 60.0, g.miny - 60.0, g.maxy + 60.0, 0.5, n);
    double2 *d_merged = dev<double2>(S.merged, n);
    int *d_leaders = dev<int>(S.leaders, n), *d_owner = dev<int>(S.owner, n);
    int *d_cnt = dev<int>(S.misc, 8);
    // leaders (the kept seeds) -> d_merged, overwritten in leader order by their means
    greedy_dedup_async(G.dedup, d_raw, nullptr, n, kConflictLessEq, 0.5, hm, d_merged, d_leaders, d_owner, d_cnt, s);
    // (the means and the count come back from the same launch: one host wait)
    k_merge_members<<<cdiv(n, 128), 128, 0, s>>>(d_raw, G.dedup.ci, d_owner, d_leaders, d_cnt, d_merged,
                                                 reinterpret_cast<double2 *>(h_seeds), h_sc, dedup_err(G.dedup, s));
    G.sev.sync(s);
    dedup_check(G.dedup, h_sc[1]);
    tr.mark("merge");
    const int nl = h_sc[0];
    std::vector<double> merged(2 * (size_t)nl);
    std::memcpy(merged.data(), h_seeds, sizeof(double2) * (size_t)nl);
    G.n_merged = nl;
    AOS_HIP(hipEventRecord(ev[7], s));
    G.merged_xy = merged;
    if (P.gvd_markers) markers_start(G, P.subdiv_rect_mode);
    if (in.on_host_phase) in.on_host_phase(in.hook_arg);

    // ---- g3/g4 finite filter, bounds, Subdiv2D inserts (host replay) -> facets / Voronoi edges (GPU)
    auto t0 = std::chrono::steady_clock::now();
    int ne = 0;
    double2 *d_occ = nullptr;
    {
        double min_x = g.minx, max_x = g.maxx, min_y = g.miny, max_y = g.maxy;
        if (!std::isfinite(min_x) || !std::isfinite(max_x) || !std::isfinite(min_y) || !std::isfinite(max_y)) return false;
        bool any_finite = false;
        for (int i = 0; i < nl; ++i) any_finite |= std::isfinite(merged[2 * i]) && std::isfinite(merged[2 * i + 1]);
        if (!any_finite) return false;  // gvd:273-275
        // VoronoiDiagram::compute voronoi_diagram.cpp:27-89
        if (min_x > max_x) std::swap(min_x, max_x);
        if (min_y > max_y) std::swap(min_y, max_y);
        if (max_x - min_x < 1.0) { double c = (min_x + max_x) / 2.0; min_x = c - 0.5; max_x = c + 0.5; }
        if (max_y - min_y < 1.0) { double c = (min_y + max_y) / 2.0; min_y = c - 0.5; max_y = c + 0.5; }
        float rx = static_cast<float>(min_x - 1.0), ry = static_cast<float>(min_y - 1.0);
        float rw = static_cast<float>(std::abs(max_x - min_x) + 2.0), rh = static_cast<float>(std::abs(max_y - min_y) + 2.0);
        if (!(rw <= 0 || rh <= 0)) {
            Subdiv2D &sd = G.subdiv;
            sd.reserve(nl);
            sd.init_delaunay(rx, ry, rw, rh, P.subdiv_rect_mode);
            const float margin = 0.1f;
            for (int i = 0; i < nl; ++i) {
                const double sx = merged[2 * i], sy = merged[2 * i + 1];
                if (!std::isfinite(sx) || !std::isfinite(sy)) continue;
                float x = static_cast<float>(sx), y = static_cast<float>(sy);
                x = std::max(rx + margin, std::min(rx + rw - margin, x));
                y = std::max(ry + margin, std::min(ry + rh - margin, y));
                sd.insert(x, y);
            }
            tr.mark("inserts");
            Subdiv2D::Raw R{};
            ne = facets_count(S.fb, sd, R, h_sc, s, G.sev);
            tr.mark("facets");
            d_occ = dev<double2>(S.occ, 2 * (size_t)std::max(ne, 1));   // (g5's candidates: the edge ends)
            if (ne) facets_emit(S.fb, R, nullptr, s, d_occ);
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    G.ms_delaunay = std::chrono::duration<float, std::milli>(t1 - t0).count();
    G.n_vor_edges = ne;
    AOS_HIP(hipEventRecord(ev[8], s));
    if (ne == 0) {   // no boundary points: an empty graph is still published
        G.have_markers = P.gvd_markers != 0;
        G.graph_ok = true;
        return true;
    }

    // ---- g5 boundary points: the 2E edge ends, de-duplicated (1 cm key or < 5 cm) through a cell index of
    // cells >= 0.5 m, which g6 reuses for its nearest-point and pair searches (pos_of: ends -> points)
    const int no = 2 * ne;
    const HashG h5 = make_hash_n(g.minx - 10.0, g.maxx + 10.0, g.miny - 10.0, g.maxy + 10.0, 0.5, no);
    double2 *d_bp = dev<double2>(S.bp, no);
    int *d_pos_of = dev<int>(S.kept_occ, no);
    int *d_sc = dev<int>(S.misc, 16);   // [0] M
    const double thr5 = 0.05 * 0.05;
    greedy_dedup_async(G.dedup, d_occ, nullptr, no, kConflictKeyOrSq, thr5, h5, d_bp, nullptr, nullptr, d_sc, s, d_pos_of);
    const CellIdx cio = G.dedup.ci;
    const int *d_M = d_sc;

    // ---- g6 graph edges
    unsigned long long *d_evals = nullptr;   // (aos_params.gvd_count_evals)
    if (P.gvd_count_evals) {
        d_evals = dev<unsigned long long>(S.evals, 8);
        AOS_HIP(hipMemsetAsync(d_evals, 0, 8 * sizeof(unsigned long long), s));
    }
    int *d_pcount = dev<int>(S.pcount, no), *d_poff = dev<int>(S.poff, no + 1);
    // The pair lists get a capacity from the last frame (P is read back only with the frame's sizes below);
    // a frame with more pairs runs the rest again with the exact size.
    int cap = G.pairs_cap > 0 ? G.pairs_cap : std::max(1024, 2 * no);
    k_pairs_count<<<cdiv(no, 256), 256, 0, s>>>(d_bp, no, d_M, cio, d_pos_of, d_occ, d_pcount, d_evals);
    scan_1p(S.lb, d_pcount, d_poff, no, false, s);
    int Mn = 0, Ne = 0, n_entries = 0;
    const int nrows = in.n_rows_poses / 2;
    const int nj = 4 * nrows;
    std::vector<LabelRow> jobs;
    for (int r = 0; r < nrows; ++r) {   // the exploration rows' label jobs (gvd:130-150, 485-556)
        double sx = in.rows_info[4 * r], sy = in.rows_info[4 * r + 1], ex = in.rows_info[4 * r + 2], ey = in.rows_info[4 * r + 3];
        if (sx > ex) { std::swap(sx, ex); std::swap(sy, ey); }
        // castRay angle terms (gvd:574-581): +90 -> cos(a), sin(a); -90 -> cos(-a), sin(-a)
        const double am = -90.0 * M_PI / 180.0, ap = 90.0 * M_PI / 180.0;
        const double cm = std::cos(-am), sm = std::sin(-am), cp = std::cos(ap), sp = std::sin(ap);
        jobs.push_back({sx, sy, ex, ey, -90.0, cm, sm});
        jobs.push_back({sx, sy, ex, ey, 90.0, cp, sp});
        jobs.push_back({ex, ey, sx, sy, -90.0, cm, sm});
        jobs.push_back({ex, ey, sx, sy, 90.0, cp, sp});
    }
    LabelRow *d_jobs = dev<LabelRow>(S.jobs, nj);
    if (nj) AOS_HIP(hipMemcpyAsync(d_jobs, jobs.data(), sizeof(LabelRow) * nj, hipMemcpyHostToDevice, s));
    double2 *d_lp = dev<double2>(S.lpts, nj);
    int *d_lv = dev<int>(S.lval, nj);
    double2 *d_nodes = dev<double2>(S.nodes, no);
    int *d_in = dev<int>(S.inside, no), *d_ipos = dev<int>(S.ipos, no + 1);
    int *d_mask = dev<int>(S.lmask, no), *d_cidx = dev<int>(S.lcidx, no), *d_lcnt = dev<int>(S.lcount, no),
        *d_loff = dev<int>(S.loff, no + 1);
    int *d_edges = nullptr, *d_lcl = nullptr, *d_lty = nullptr;
    float *d_lens = nullptr;
    int *h_sz = h_sc + 8;
    for (int attempt = 0;; ++attempt) {
        const int ncap = ne + cap;
        int2 *d_ft = dev<int2>(S.ft, ncap);
        unsigned long long *ev_k = attempt ? nullptr : d_evals;   // (a rerun with the exact pair capacity is not counted)
        // (round 5 measured k_nearest on a second stream beside the pair count, scan and lists: no gain, r05l)
        k_nearest<<<cdiv(no, 256), 256, 0, s>>>(d_occ, no, cio, d_pos_of, d_bp, d_M, reinterpret_cast<int *>(d_ft), ev_k);
        k_pairs<<<cdiv(no, 256), 256, 0, s>>>(d_bp, no, d_M, cio, d_pos_of, d_occ, d_poff, d_ft + ne, cap, ev_k);
        int *d_pass = dev<int>(S.pass, ncap), *d_grank = dev<int>(S.occ_idx, ncap), *d_sel = dev<int>(S.selected, ncap);
        const size_t gc0 = S.gcnt.cap;
        int *d_gcnt = dev<int>(S.gcnt, no);
        if (S.gcnt.cap != gc0 || S.gcnt_dirty) AOS_HIP(hipMemsetAsync(d_gcnt, 0, S.gcnt.cap, s));
        S.gcnt_dirty = true;
        int *d_goff = dev<int>(S.goff, no + 1), *d_glist = dev<int>(S.glist, ncap);
        k_occupancy<<<cdiv(ncap, kOccTB), kOccTB, 0, s>>>(d_ft, d_poff, no, ne, cap, d_bp, in.d_skeleton, g, d_pass, d_gcnt, d_grank,
                                                  ev_k);
        scan_1p(S.lb, d_gcnt, d_goff, no, true, s);   // (leaves the group counts zero)
        S.gcnt_dirty = false;
        k_group_scatter<<<cdiv(ncap, 256), 256, 0, s>>>(d_ft, d_pass, d_poff, no, ne, cap, d_goff, d_grank, d_glist);
        k_select<<<cdiv(ncap, 256), 256, 0, s>>>(d_ft, d_pass, d_poff, no, ne, cap, d_goff, d_glist, d_sel);

        // ---- g7 filter
        k_inside<<<cdiv(no, 256), 256, 0, s>>>(d_bp, no, d_M, g, d_in);
        scan_1p(S.lb, d_in, d_ipos, no, false, s);
        int *d_keep = dev<int>(S.keep, ncap), *d_kpos = dev<int>(S.kpos, ncap + 1);
        k_edge_keep<<<cdiv(std::max(ncap, no), 256), 256, 0, s>>>(d_sel, d_ft, ncap, d_in, d_ipos, d_keep, d_bp, no, d_nodes);
        scan_1p(S.lb, d_keep, d_kpos, ncap, false, s);
        d_edges = dev<int>(S.edges, 2 * (size_t)ncap);
        d_lens = dev<float>(S.lens, ncap);
        k_edge_emit<<<cdiv(ncap, 256), 256, 0, s>>>(d_keep, d_kpos, d_ft, ncap, d_ipos, d_nodes, d_edges, d_lens);
        const int *d_Mn = d_ipos + no;

        // ---- g8 label points for the exploration rows: the nodes in cells of >= 5.01 m
        if (nj) {
            const HashG hl = make_hash_n(g.minx - 10.0, g.maxx + 10.0, g.miny - 10.0, g.maxy + 10.0, 5.01, no);
            const CellIdx cn = cell_index_build(S.ci_nodes, d_nodes, nullptr, no, hl, s, d_Mn);
            k_label_points<<<nj, 256, 0, s>>>(d_jobs, nj, d_nodes, d_Mn, g, in.d_skeleton, cn, d_lp, d_lv, ev_k);
        }
        // ---- g9 node labels: the valid label points in cells of >= 0.1 m
        const HashG hq = make_hash_n(g.minx - 1.0, g.maxx + 1.0, g.miny - 1.0, g.maxy + 1.0, 0.1, nj);
        const CellIdx cq = S.cq = cell_index_build(S.ci_labels, d_lp, d_lv, nj, hq, s);
        k_node_labels_count<<<cdiv(no, 256), 256, 0, s>>>(d_nodes, no, d_Mn, d_lp, d_lv, nrows, cq, d_mask, d_cidx, d_lcnt);
        scan_1p(S.lb, d_lcnt, d_loff, no, false, s);
        // the frame's sizes and error words: one read-back
        peek_to_host(h_sz, {d_M, d_poff + no, d_Mn, d_kpos + ncap, d_loff + no, dedup_err(G.dedup, s), S.lb.err_word(s),
                            S.ci_nodes.lb.err_word(s)}, s);
        G.sev.sync(s);
        if (h_sz[5] || h_sz[6] || h_sz[7]) {
            if (h_sz[6] || h_sz[7]) throw std::runtime_error("GVD graph: single-pass scan failed on the device");
            dedup_check(G.dedup, h_sz[5]);
        }
        const int P_ = h_sz[1];
        G.pairs_cap = std::max(1024, P_ + P_ / 4);
        if (P_ <= cap) {
            G.n_bpts = h_sz[0];
            Mn = h_sz[2]; Ne = h_sz[3]; n_entries = h_sz[4];
            break;
        }
        if (attempt) throw std::runtime_error("GVD graph: pair lists overflowed twice");
        cap = G.pairs_cap;
    }
    tr.mark("graph");
    const int nj_out = Mn > 0 ? nj : 0;   // (no nodes: no label jobs, gvd:485-556 finds nothing to label)
    d_lcl = dev<int>(S.lcl, n_entries);
    d_lty = dev<int>(S.lty, n_entries);
    if (n_entries)
        k_node_labels_fill<<<cdiv(Mn, 256), 256, 0, s>>>(d_nodes, Mn, d_lp, d_lv, nrows, S.cq, d_loff, d_lcl, d_lty);

    // ---- outputs: one gather kernel, one D2H copy into the state's pinned buffer, host copies out
    G.nodes_xy.resize(2 * (size_t)Mn); G.labels.resize(Mn); G.cluster_idx.resize(Mn); G.label_counts.resize(Mn);
    G.label_clusters.resize(n_entries); G.label_types.resize(n_entries);
    G.edges_out.resize(2 * (size_t)Ne); G.lengths.resize(Ne); G.clearances.assign(Ne, 0.0f);
    G.row_label_xy.resize(2 * (size_t)nj_out); G.row_label_valid.resize(nj_out);
    struct Out { const void *d; void *h; long long words; };
    const Out outs[] = {{d_nodes, G.nodes_xy.data(), 4LL * Mn}, {d_mask, G.labels.data(), Mn}, {d_cidx, G.cluster_idx.data(), Mn},
                        {d_lcnt, G.label_counts.data(), Mn}, {d_lcl, G.label_clusters.data(), n_entries},
                        {d_lty, G.label_types.data(), n_entries}, {d_edges, G.edges_out.data(), 2LL * Ne},
                        {d_lens, G.lengths.data(), Ne}, {d_lp, G.row_label_xy.data(), 4LL * nj_out},
                        {d_lv, G.row_label_valid.data(), nj_out}};
    SegList sl{};
    for (const Out &o : outs) {
        if (o.words <= 0) continue;
        sl.src[sl.n] = static_cast<const int *>(o.d);
        sl.off[sl.n + 1] = sl.off[sl.n] + o.words;
        ++sl.n;
    }
    const long long total = sl.off[sl.n];
    int *h_out = static_cast<int *>(G.h_out.ensure(sizeof(int) * (size_t)std::max(total, 1LL)));
    if (total) k_gather_words<<<cdiv(cdiv(total, 4), 256), 256, 0, s>>>(sl, h_out);   // (straight into the pinned buffer)
    unsigned long long *h_ev = d_evals ? static_cast<unsigned long long *>(G.h_evals.ensure(8 * sizeof(unsigned long long))) : nullptr;
    if (d_evals) AOS_HIP(hipMemcpyAsync(h_ev, d_evals, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    AOS_HIP(hipEventRecord(ev[9], s));
    G.sev.sync(s);
    tr.mark("out");
    G.evals = aos_gvd_evals{};
    if (h_ev) {   // the work of the searches (SURVEY §8d "pair evaluations"), the reference's beside the GPU's
        aos_gvd_evals &E = G.evals;
        const uint64_t M = (uint64_t)G.n_bpts;
        E.counted = 1;
        E.n_label_jobs = nj_out;
        E.edge_ends = (uint64_t)no; E.boundary_points = M; E.filtered_nodes = (uint64_t)Mn;
        E.ref_nearest = (uint64_t)no * M;                        // gvd:812-824 per edge end, every boundary point
        E.ref_pairs = M ? M * (M - 1) / 2 : 0;                   // gvd:861-894
        E.ref_labels = nj_out ? h_ev[4] * (uint64_t)Mn : 0;      // gvd:731-774, once per radius tried
        E.gpu_nearest = h_ev[0]; E.gpu_pairs = h_ev[1]; E.gpu_samples = h_ev[2]; E.gpu_labels = h_ev[3];
    }
    for (const Out &o : outs)
        if (o.words > 0) { std::memcpy(o.h, h_out, sizeof(int) * (size_t)o.words); h_out += o.words; }
    G.have_markers = P.gvd_markers != 0;
    G.graph_ok = true;
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, ev[6], ev[7]);
    (void)hipEventElapsedTime(&b, ev[8], ev[9]);
    G.ms_merge = a; G.ms_graph = b;
    (void)hipEventElapsedTime(&G.ms_total, ev[6], ev[9]);
    return true;
}

}  // namespace aos

// ------------------------------------------------------------------ handle methods
using namespace aos;

static void fill_gvd_out(const aos_ctx &c, const GvdState &G, const aos_grid_info &info, bool published, aos_gvd_out &out) {
    std::memset(&out, 0, sizeof(out));
    out.published = published ? 1 : 0;
    out.resolution = info.resolution;  // GvdGraph.resolution = skeleton info.resolution (gvd:903)
    out.origin_x = info.origin_x; out.origin_y = info.origin_y;
    out.num_nodes = (int32_t)G.labels.size();
    out.num_edges = (int32_t)G.lengths.size();
    out.nodes_xy = G.nodes_xy.data();
    out.node_labels = G.labels.data(); out.node_cluster_indices = G.cluster_idx.data();
    out.node_label_counts = G.label_counts.data();
    out.n_label_entries = (int32_t)G.label_clusters.size();
    out.node_label_clusters = G.label_clusters.data(); out.node_label_types = G.label_types.data();
    out.edges = G.edges_out.data(); out.edge_lengths = G.lengths.data(); out.edge_clearances = G.clearances.data();
    out.n_merged_seeds = G.n_merged; out.n_voronoi_edges = G.n_vor_edges; out.n_boundary_points = G.n_bpts;
    out.ms_merge = G.ms_merge; out.ms_delaunay = G.ms_delaunay; out.ms_graph = G.ms_graph; out.ms_total = G.ms_total;
    out.ms_cells = 0.0f;   // the cells job may still run: aos_gvd_markers.ms_cells
    (void)c;
}

void aos_ctx::run_gvd_external(const aos_gvd_in &in, aos_gvd_out &out) {
    gvd_async_drop();
    GvdState &G = gs();
    const size_t C = (size_t)in.info.width * in.info.height;
    int8_t *d_sk = static_cast<int8_t *>(G.skel.ensure(std::max<size_t>(C, 1)));
    if (C && in.skeleton) AOS_HIP(hipMemcpyAsync(d_sk, in.skeleton, C, hipMemcpyHostToDevice, stream));
    GvdStageIn gi{in.seeds_xy, in.n_seeds, in.rows_info_xy, in.n_rows_poses, in.info, d_sk};
    have_gvd = false;
    const bool pub = run_gvd_stage(G, P, gi, stream, ev.data());
    have_gvd = true; gvd_from_frame = false; gvd_skel = d_sk; gvd_info = in.info; ++gvd_gen;
    fill_gvd_out(*this, G, in.info, pub, out);
}

void aos_ctx::run_gvd_from_frame(aos_gvd_out &out) {
    gvd_async_drop();
    GvdState &G = gs();
    aos_grid_info info{geom.origin_x, geom.origin_y, geom.res, (uint32_t)geom.W, (uint32_t)geom.H};
    GvdStageIn gi{h_voronoi.data(), (int)(h_voronoi.size() / 2), h_rows_info.data(), (int)(h_rows_info.size() / 2), info,
                  skel_bytes.as<int8_t>()};
    have_gvd = false;
    const bool pub = run_gvd_stage(G, P, gi, stream, ev.data());
    have_gvd = true; gvd_from_frame = true; gvd_frame_gen = frame_gen; gvd_skel = gi.d_skeleton; gvd_info = info; ++gvd_gen;
    fill_gvd_out(*this, G, info, pub, out);
}

// ------------------------------------------------------------------ pipelined GVD
// aos_gvd_from_seedgen_async: snapshot the frame's GVD inputs (host seeds and rows, a device copy of
// the skeleton ordered on the seed-gen stream) into a free lane, whose worker runs the same
// run_gvd_stage on the lane's stream. The next seed-gen frame may run meanwhile; it rewrites only
// seed-gen state. Frames are independent, so with aos_gvd_pipeline_depth(D) up to D jobs run at once
// (each Subdiv2D replay on its own host core); aos_gvd_wait collects them in start order.
void aos_ctx::gvd_lanes_ensure() {
    if (lanes.empty()) lanes.emplace_back(new GvdLane());
    while ((int)lanes.size() < gvd_depth + 1) lanes.emplace_back(new GvdLane());
}

void aos_ctx::lane_join(int l) {
    AsyncGvd &A = lanes[l]->ag;
    if (!A.worker.joinable()) return;
    std::unique_lock<std::mutex> lk(A.mu);
    A.cv.wait(lk, [&A] { return !A.busy; });
}

void aos_ctx::lane_apply(int l) {
    lanes[l]->ag.applied = true;
    cur_lane = l;
    have_gvd = true; gvd_from_frame = false; gvd_skel = lanes[l]->gs.skel.as<int8_t>(); gvd_info = lanes[l]->ag.info;
    ++gvd_gen;
}

void aos_ctx::gvd_async_start() {
    gvd_lanes_ensure();
    // D jobs in flight already: the oldest is superseded (joined, its result dropped)
    while ((int)inflight.size() >= gvd_depth) {
        const int l = inflight.front();
        inflight.pop_front();
        lane_join(l);
        std::lock_guard<std::mutex> lk(lanes[l]->ag.mu);
        lanes[l]->ag.done = false;
        lanes[l]->ag.err = nullptr;
    }
    int L = -1;   // a lane that holds neither the current result nor a job
    for (int i = 0; i < (int)lanes.size() && L < 0; ++i)
        if (i != cur_lane && std::find(inflight.begin(), inflight.end(), i) == inflight.end()) L = i;
    if (L < 0) throw std::logic_error("gvd_async_start: no free lane");
    GvdLane &ln = *lanes[L];
    AsyncGvd &A = ln.ag;
    if (!gvd_stream) AOS_HIP(hipStreamCreateWithFlags(&gvd_stream, hipStreamNonBlocking));
    if (!A.stream) {
        // every lane queues its GPU work on the handle's one GVD stream (few streams for the GPU's 4 hardware
        // queues: no false dependencies behind unrelated streams); each lane waits on its own events
        A.stream = gvd_stream;
        for (auto &e : A.ev) AOS_HIP(hipEventCreate(&e));
        AOS_HIP(hipEventCreateWithFlags(&A.ready, hipEventDisableTiming));
    }
    A.seeds = h_voronoi;
    A.rows = h_rows_info;
    A.P = P;   // snapshot on the caller's thread: aos_gvd_set_markers may change P while the job runs
    A.applied = false;
    A.info = aos_grid_info{geom.origin_x, geom.origin_y, geom.res, (uint32_t)geom.W, (uint32_t)geom.H};
    const size_t C = (size_t)geom.W * geom.H;
    int8_t *d_sk = static_cast<int8_t *>(ln.gs.skel.ensure(std::max<size_t>(C, 1)));
    AOS_HIP(hipMemcpyAsync(d_sk, skel_bytes.p, C, hipMemcpyDeviceToDevice, stream));
    AOS_HIP(hipEventRecord(A.ready, stream));
    AOS_HIP(hipStreamWaitEvent(A.stream, A.ready, 0));
    if (!A.worker.joinable())
        A.worker = std::thread([this, &ln]() {
            AsyncGvd &W = ln.ag;
            std::unique_lock<std::mutex> l(W.mu);
            for (;;) {
                W.cv.wait(l, [&W] { return W.busy || W.quit; });
                if (W.quit) return;
                l.unlock();
                std::exception_ptr e;
                bool pub = false;
                try {
                    AOS_HIP(hipSetDevice(device));
                    GvdStageIn gi{W.seeds.data(), (int)(W.seeds.size() / 2), W.rows.data(), (int)(W.rows.size() / 2),
                                  W.info, ln.gs.skel.as<int8_t>()};
                    gi.hook_arg = &W;
                    gi.on_host_phase = [](void *p) {
                        AsyncGvd *A = static_cast<AsyncGvd *>(p);
                        { std::lock_guard<std::mutex> g(A->mu); A->prefix = true; }
                        A->cv.notify_all();
                    };
                    pub = run_gvd_stage(ln.gs, W.P, gi, W.stream, W.ev.data());
                } catch (...) { e = std::current_exception(); }
                l.lock();
                W.err = e;
                W.pub = pub;
                W.busy = false;
                W.done = true;
                W.cv.notify_all();
            }
        });
    {
        std::lock_guard<std::mutex> l(A.mu);
        A.err = nullptr;
        A.done = false;
        A.prefix = false;
        A.busy = true;
    }
    A.cv.notify_all();
    inflight.push_back(L);
    view_newest = true;
    // Return once the job's short GPU prefix (seed merge) is done and its host replay runs: a
    // seed-gen frame launched earlier would occupy the GPU and hold the prefix back, and the replay
    // would start late instead of overlapping it.
    std::unique_lock<std::mutex> l(A.mu);
    A.cv.wait(l, [&A] { return A.prefix || !A.busy; });
}

// aos_gvd_wait: collects the oldest job in flight (raising its error if rethrow); its lane becomes
// the handle's current result (markers, planning).
bool aos_ctx::gvd_async_wait(bool rethrow) {
    if (inflight.empty()) return false;
    const int l = inflight.front();
    inflight.pop_front();
    view_newest = false;
    lane_join(l);
    AsyncGvd &A = lanes[l]->ag;
    std::exception_ptr e;
    {
        std::lock_guard<std::mutex> lk(A.mu);
        A.done = false;
        e = A.err;
        A.err = nullptr;
    }
    if (e) {
        if (rethrow) std::rethrow_exception(e);
        return false;
    }
    // a settle (markers / planning before this wait) already made this lane current: same graph, so the
    // path planner's graph cache (keyed on gvd_gen) stays valid
    if (!(cur_lane == l && A.applied && have_gvd)) lane_apply(l);
    return true;
}

// Markers and planning on the handle's own graph: right after aos_gvd_wait they see the collected
// job; with no wait since the last start they see the newest job (waited for, still collectable).
void aos_ctx::gvd_view_settle() {
    if (!view_newest || inflight.empty()) return;
    const int l = inflight.back();
    lane_join(l);
    AsyncGvd &A = lanes[l]->ag;
    bool ok;
    {
        std::lock_guard<std::mutex> lk(A.mu);
        ok = A.done && !A.err;
    }
    if (ok && (cur_lane != l || !have_gvd)) lane_apply(l);
}

// A synchronous GVD call (or the handle's release) supersedes every job in flight.
void aos_ctx::gvd_async_drop() {
    gvd_lanes_ensure();
    for (int l : inflight) {
        lane_join(l);
        std::lock_guard<std::mutex> lk(lanes[l]->ag.mu);
        lanes[l]->ag.done = false;
        lanes[l]->ag.err = nullptr;
    }
    inflight.clear();
    view_newest = false;
}

void aos_ctx::gvd_async_stop() {
    for (auto &lp : lanes) {
        AsyncGvd &A = lp->ag;
        if (A.worker.joinable()) {
            { std::lock_guard<std::mutex> l(A.mu); A.quit = true; }
            A.cv.notify_all();
            A.worker.join();
        }
        if (A.stream) {
            (void)hipStreamSynchronize(A.stream);
            for (auto &e : A.ev) (void)hipEventDestroy(e);
            (void)hipEventDestroy(A.ready);
            A.stream = nullptr;   // (the shared gvd_stream)
        }
    }
    if (gvd_stream) {
        (void)hipStreamDestroy(gvd_stream);
        gvd_stream = nullptr;
    }
    inflight.clear();
    view_newest = false;
}

int aos::gvd_wait_out(aos_ctx *c, aos_gvd_out *out) {   // aos_gvd_wait (api.hip)
    if (!c->gvd_async_wait(true)) return 0;
    const aos_ctx::GvdLane &ln = *c->lanes[c->cur_lane];
    fill_gvd_out(*c, ln.gs, ln.ag.info, ln.ag.pub, *out);
    return 1;
}
