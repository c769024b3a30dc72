// Grid view and device helpers shared by the whole-map cluster stage (cluster_seed.hip) and the
// tiled frame's distributed labelling (cluster_dist.hip). Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "aos_internal.h"

namespace aos {

struct GridC {
    double ox, oy;       // origin
    float res;
    int W, H, WW;
    double minx, maxx, miny, maxy;  // origin + W * res (float product), seed_gen:1807-1810
    double amax;         // castRayFromEndpoint absolute max distance, seed_gen:1838-1840
};

// The whole map's view, bounds formed as the reference forms them (uint32 * float -> float, then
// double add).
inline GridC make_gridc(const FrameGeom &fg) {
    GridC g{};
    g.ox = fg.origin_x; g.oy = fg.origin_y; g.res = fg.res; g.W = fg.W; g.H = fg.H; g.WW = fg.WW;
    const uint32_t W = (uint32_t)fg.W, H = (uint32_t)fg.H;
    const float res = fg.res;
    g.minx = fg.origin_x; g.maxx = g.minx + W * res;
    g.miny = fg.origin_y; g.maxy = g.miny + H * res;
    const double gw = W * res, gh = H * res;
    g.amax = std::sqrt(gw * gw + gh * gh) * 3.0;
    return g;
}

// isPointInPolygon seed_gen:1231-1255
__host__ __device__ inline bool d_pip(double px, double py, const double *poly, int n) {
    if (n < 3) return false;
    bool inside = false;
    int j = n - 1;
    for (int i = 0; i < n; ++i) {
        double pix = poly[2 * i], piy = poly[2 * i + 1], pjx = poly[2 * j], pjy = poly[2 * j + 1];
        double dy = pjy - piy;
        if (fabs(dy) > 1e-9) {
            if (((piy > py) != (pjy > py)) && (px < (pjx - pix) * (py - piy) / dy + pix)) inside = !inside;
        }
        j = i;
    }
    return inside;
}

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

// float world coordinate of a cell: origin + float(x) * res (float product, double add, to float)
__host__ __device__ __forceinline__ float cell_world(double o, int i, float res) { return (float)(o + (double)((float)i * res)); }

__host__ __device__ __forceinline__ double2 cell_w(const GridC &g, int p) {
    int y = p / g.W, x = p - y * g.W;
    return make_double2((double)cell_world(g.ox, x, g.res), (double)cell_world(g.oy, y, g.res));
}

__device__ __forceinline__ bool bit_at(const uint64_t *bits, int WW, int x, int y) {
    return (bits[(size_t)y * WW + (x >> 6)] >> (x & 63)) & 1ull;
}

// ------------------------------------------------------------------ union-find (8-connectivity CCL)
__device__ __forceinline__ int ld_parent(int *parent, int i) {
    return __hip_atomic_load(&parent[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
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
