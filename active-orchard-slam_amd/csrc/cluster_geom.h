// Grid view and the host/device geometry helpers of the cluster stage (world points of cells, the polygon
// test): host-compilable (cluster_host.cpp, the sanitizer build); cluster_dev.h adds the device-only helpers.
// Not part of the ABI.
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

// float world coordinate of a cell: origin + float(x) * res (float product, double add, to float)
__host__ __device__ __forceinline__ float cell_world(double o, int i, float res) { return (float)(o + (double)((float)i * res)); }

__host__ __device__ __forceinline__ double2 cell_w(const GridC &g, int p) {
    int y = p / g.W, x = p - y * g.W;
    return make_double2((double)cell_world(g.ox, x, g.res), (double)cell_world(g.oy, y, g.res));
}

}  // namespace aos
