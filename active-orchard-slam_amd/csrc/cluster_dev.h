// Grid view and device helpers shared by the whole-map cluster stage (cluster_seed.hip) and the
// tiled frame's distributed labelling (cluster_dist.hip). Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "aos_internal.h"
#include "cluster_geom.h"

namespace aos {

// isPointInPolygon for every cell of one grid row: the crossing abscissa of an edge,
// (pjx - pix) * (py - piy) / dy + pix, does not depend on px, so a workgroup whose cells share py
// computes the crossings of the edges that straddle py once (LDS) and a cell's test is its parity of
// px < crossing: the same double operations and comparisons as d_pip. Polygons with more than
// kRowCrossMax straddling edges fall back to d_pip.
constexpr int kRowCrossMax = 256;
__device__ inline bool row_crossings(const double *poly, int n, double py, double *xc, int *nxc) {
    if (threadIdx.x == 0) *nxc = 0;
    __syncthreads();
    if (n >= 3)
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int j = i == 0 ? n - 1 : i - 1;
            const double pix = poly[2 * i], piy = poly[2 * i + 1], pjx = poly[2 * j], pjy = poly[2 * j + 1];
            const double dy = pjy - piy;
            if (fabs(dy) > 1e-9 && ((piy > py) != (pjy > py))) {
                const int k = atomicAdd(nxc, 1);
                if (k < kRowCrossMax) xc[k] = (pjx - pix) * (py - piy) / dy + pix;
            }
        }
    __syncthreads();
    return *nxc <= kRowCrossMax;
}
__device__ __forceinline__ bool pip_row(double px, const double *xc, int nxc) {
    bool inside = false;
    for (int k = 0; k < nxc; ++k) inside ^= px < xc[k];
    return inside;
}
// pip_row for the 64 cells x0 .. x0 + 63 of a row at once: bit b set iff pip_row(cell_world(ox, x0 + b, res), ...).
// cell_world is non-decreasing in x (each of its roundings is monotone), so "px < xc[k]" holds on a prefix of the
// word, found by a binary search over its 64 cells; the mask is the XOR of the prefixes (round 6: words with many
// set cells, the skeleton's rectangle rows, took one test per cell: 64 per word set k_fg's time, 15-19 us blocks at C2)
constexpr int kPipWordMin = 8;   // set cells from which a word is tested this way
__device__ __forceinline__ uint64_t pip_row_word(double ox, float res, int x0, const double *xc, int nxc) {
    uint64_t inside = 0;
    for (int k = 0; k < nxc; ++k) {
        const double t = xc[k];
        int lo = 0, hi = 64;   // the first cell with !(px < t)
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((double)cell_world(ox, x0 + mid, res) < t) lo = mid + 1;
            else hi = mid;
        }
        inside ^= lo == 64 ? ~0ull : ((1ull << lo) - 1);
    }
    return inside;
}

__device__ __forceinline__ bool bit_at(const uint64_t *bits, int WW, int x, int y) {
    return (bits[(size_t)y * WW + (x >> 6)] >> (x & 63)) & 1ull;
}

// ------------------------------------------------------------------ union-find (8-connectivity CCL)
__device__ __forceinline__ int ld_parent(int *parent, int i) {
    return __hip_atomic_load(&parent[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// root of x. (Round 4 measured path halving here, ECL-CC style: the C2 flatten got shallower trees,
// 53 -> 23 us, but the halving stores made the union kernel 139 -> 247 us: every walker's agent-scope
// store and load goes past the XCD's L2. Not adopted.)
__device__ __forceinline__ int uf_find(int *parent, int x) {
    while (true) {
        int p = ld_parent(parent, x);
        if (p == x) return x;
        x = p;
    }
}
// links the components of list entries i and j; the smaller index becomes the root
__device__ __forceinline__ void uf_union(int *parent, int i, int j) {
    int a = uf_find(parent, i), b = uf_find(parent, j);
    while (a != b) {
        if (a < b) { int t = a; a = b; b = t; }
        int old = atomicCAS(&parent[a], a, b);  // link the larger root under the smaller
        if (old == a) break;
        a = uf_find(parent, old);
        b = uf_find(parent, b);
    }
}

}  // namespace aos
