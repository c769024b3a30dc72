// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). Build: g++ -O2 -ffp-contract=off.
// CPU restatement of aos_seed_gen_node (reference src/aos_seed_gen_node.cpp); every function
// cites the reference lines it follows. Float/double promotions are kept expression by
// expression because they decide grid indices and seed coordinates.
#include "oracle_internal.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <queue>
#include <utility>
#include <vector>

namespace orc {

// ---------------------------------------------------------------- a1: PCL RadiusOutlierRemoval
// seed_gen:236-242 -> PCL 1.12 RadiusOutlierRemoval::applyFilterIndices (NOTES.md §1).
// dense cloud  : kNN k = min_pts + 1 (incl. the query), keep iff k found and
//                nn_dists[k-1] <= radius^2 (double compare of the float distance).
// !dense cloud : radius search (FLANN: dist < float(radius^2)), keep iff count > min_pts.
// FLANN L2_Simple distance: ((0 + dx*dx) + dy*dy) + dz*dz in float.
// Non-finite points are never neighbours and are always removed.
void ror(const float *xyz, uint64_t n, bool is_dense, double radius, int min_pts, uint8_t *keep) {
    if (n) std::memset(keep, 0, n);
    const double cell = radius * 1.0001;
    double mnx = 1e300, mny = 1e300, mnz = 1e300, mxx = -1e300, mxy = -1e300, mxz = -1e300;
    uint64_t nfin = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const float *p = xyz + 3 * i;
        if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
        ++nfin;
        mnx = std::min(mnx, (double)p[0]); mxx = std::max(mxx, (double)p[0]);
        mny = std::min(mny, (double)p[1]); mxy = std::max(mxy, (double)p[1]);
        mnz = std::min(mnz, (double)p[2]); mxz = std::max(mxz, (double)p[2]);
    }
    if (nfin == 0) return;
    // 3-D binning, coarsened if the extent is huge (coarser cells stay correct).
    double cs = cell;
    auto dims = [&](double c, int64_t &bx, int64_t &by, int64_t &bz) {
        bx = (int64_t)((mxx - mnx) / c) + 1; by = (int64_t)((mxy - mny) / c) + 1; bz = (int64_t)((mxz - mnz) / c) + 1;
    };
    int64_t bx, by, bz;
    dims(cs, bx, by, bz);
    while ((double)bx * by * bz > 6.0e7) { cs *= 1.5; dims(cs, bx, by, bz); }
    const int64_t ncell = bx * by * bz;
    std::vector<uint32_t> start(ncell + 1, 0);
    std::vector<int64_t> cid(n, -1);
    for (uint64_t i = 0; i < n; ++i) {
        const float *p = xyz + 3 * i;
        if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
        int64_t ix = (int64_t)(((double)p[0] - mnx) / cs), iy = (int64_t)(((double)p[1] - mny) / cs),
                iz = (int64_t)(((double)p[2] - mnz) / cs);
        cid[i] = (iz * by + iy) * bx + ix;
        start[cid[i] + 1]++;
    }
    for (int64_t c = 0; c < ncell; ++c) start[c + 1] += start[c];
    std::vector<uint32_t> fill(start.begin(), start.end() - 1), order(nfin);
    for (uint64_t i = 0; i < n; ++i)
        if (cid[i] >= 0) order[fill[cid[i]]++] = (uint32_t)i;
    const double r2 = radius * radius;             // nn_dists_max (double)
    const float r2f = (float)(radius * radius);    // FLANN radius argument (float)
    const int need = min_pts + 1;
    if (is_dense && nfin < (uint64_t)need) return;  // k < mean_k for every query
    for (uint64_t i = 0; i < n; ++i) {
        if (cid[i] < 0) continue;
        const float *p = xyz + 3 * i;
        int64_t c = cid[i];
        int64_t ix = c % bx, iy = (c / bx) % by, iz = c / (bx * by);
        int cnt = 0;
        for (int64_t z = std::max<int64_t>(0, iz - 1); z <= std::min(bz - 1, iz + 1) && cnt < need; ++z)
            for (int64_t y = std::max<int64_t>(0, iy - 1); y <= std::min(by - 1, iy + 1) && cnt < need; ++y)
                for (int64_t x = std::max<int64_t>(0, ix - 1); x <= std::min(bx - 1, ix + 1) && cnt < need; ++x) {
                    int64_t cc = (z * by + y) * bx + x;
                    for (uint32_t k = start[cc]; k < start[cc + 1]; ++k) {
                        const float *q = xyz + 3 * (uint64_t)order[k];
                        float dx = p[0] - q[0], dy = p[1] - q[1], dz = p[2] - q[2];
                        float d2 = 0.0f;
                        d2 += dx * dx; d2 += dy * dy; d2 += dz * dz;
                        bool in = is_dense ? ((double)d2 <= r2) : (d2 < r2f);
                        if (in && ++cnt >= need) break;
                    }
                }
        keep[i] = (uint8_t)(cnt >= need);
    }
}

// ---------------------------------------------------------------- a3: getActiveBounds seed_gen:874-890
static void active_bounds(const Poly &poly, float &minx, float &maxx, float &miny, float &maxy) {
    double hminx = poly[0].first, hmaxx = poly[0].first, hminy = poly[0].second, hmaxy = poly[0].second;
    for (const auto &pt : poly) {  // seed_gen:263-273
        hminx = std::min(hminx, pt.first); hmaxx = std::max(hmaxx, pt.first);
        hminy = std::min(hminy, pt.second); hmaxy = std::max(hmaxy, pt.second);
    }
    const double margin = 2.5;
    minx = static_cast<float>(hminx - margin); maxx = static_cast<float>(hmaxx + margin);
    miny = static_cast<float>(hminy - margin); maxy = static_cast<float>(hmaxy + margin);
}

// isPointInPolygon seed_gen:1231-1255 (even-odd, double)
bool point_in_polygon(double px, double py, const Poly &polygon) {
    if (polygon.size() < 3) return false;
    bool inside = false;
    size_t j = polygon.size() - 1;
    for (size_t i = 0; i < polygon.size(); ++i) {
        const auto &pi = polygon[i];
        const auto &pj = polygon[j];
        double dy = pj.second - pi.second;
        if (std::abs(dy) > 1e-9) {
            if (((pi.second > py) != (pj.second > py)) && (px < (pj.first - pi.first) * (py - pi.second) / dy + pi.first))
                inside = !inside;
        }
        j = i;
    }
    return inside;
}

// ---------------------------------------------------------------- a5 applyInflation seed_gen:933-967
void inflate(const int8_t *in, int w, int h, int cells, int8_t *out) {
    std::memcpy(out, in, (size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            if (in[x + y * w] != 100) continue;
            for (int dy = -cells; dy <= cells; dy++)
                for (int dx = -cells; dx <= cells; dx++) {
                    if (dx * dx + dy * dy <= cells * cells) {
                        int nx = x + dx, ny = y + dy;
                        if (nx >= 0 && nx < w && ny >= 0 && ny < h) out[nx + ny * w] = 100;
                    }
                }
        }
}

// markBoundariesAsOccupied seed_gen:708-757 (5-cell frame)
static void mark_boundaries(int8_t *g, int w, int h) {
    const int t = 5;
    for (int y = 0; y < t && y < h; y++) for (int x = 0; x < w; x++) g[x + y * w] = 100;
    for (int y = std::max(0, h - t); y < h; y++) for (int x = 0; x < w; x++) g[x + y * w] = 100;
    for (int x = 0; x < t && x < w; x++) for (int y = 0; y < h; y++) g[x + y * w] = 100;
    for (int x = std::max(0, w - t); x < w; x++) for (int y = 0; y < h; y++) g[x + y * w] = 100;
}

// ---------------------------------------------------------------- a7 skeletonize seed_gen:672-705
// morphologyEx(OPEN, getStructuringElement(MORPH_ELLIPSE, 3x3)) — the 3x3 ellipse is a cross.
// BORDER_CONSTANT with the default morphology border value: erode sees 255 outside, dilate 0.
void open_cross(const uint8_t *in, int w, int h, uint8_t *out) {
    std::vector<uint8_t> er((size_t)w * h);
    auto at1 = [&](const uint8_t *g, int x, int y, uint8_t outside) -> uint8_t {
        return (x < 0 || y < 0 || x >= w || y >= h) ? outside : g[(size_t)y * w + x];
    };
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            er[(size_t)y * w + x] = at1(in, x, y, 1) & at1(in, x - 1, y, 1) & at1(in, x + 1, y, 1) &
                                    at1(in, x, y - 1, 1) & at1(in, x, y + 1, 1);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            out[(size_t)y * w + x] = at1(er.data(), x, y, 0) | at1(er.data(), x - 1, y, 0) | at1(er.data(), x + 1, y, 0) |
                                     at1(er.data(), x, y - 1, 0) | at1(er.data(), x, y + 1, 0);
}

// ximgproc::thinning(THINNING_ZHANGSUEN) (opencv_contrib 4.5.4, NOTES.md §4): repeat
// {sub-iteration 0, sub-iteration 1} until an iteration changes nothing. Each sub-iteration
// computes its marks on a snapshot (Jacobi); rows/cols 0 and last are never examined.
static void thin_iter(std::vector<uint8_t> &img, std::vector<uint8_t> &marker, int w, int h, int iter) {
    std::fill(marker.begin(), marker.end(), 0);
    for (int i = 1; i < h - 1; i++) {
        for (int j = 1; j < w - 1; j++) {
            const uint8_t *r0 = &img[(size_t)(i - 1) * w], *r1 = &img[(size_t)i * w], *r2 = &img[(size_t)(i + 1) * w];
            int p2 = r0[j], p3 = r0[j + 1], p4 = r1[j + 1], p5 = r2[j + 1];
            int p6 = r2[j], p7 = r2[j - 1], p8 = r1[j - 1], p9 = r0[j - 1];
            int A = (p2 == 0 && p3 == 1) + (p3 == 0 && p4 == 1) + (p4 == 0 && p5 == 1) + (p5 == 0 && p6 == 1) +
                    (p6 == 0 && p7 == 1) + (p7 == 0 && p8 == 1) + (p8 == 0 && p9 == 1) + (p9 == 0 && p2 == 1);
            int B = p2 + p3 + p4 + p5 + p6 + p7 + p8 + p9;
            int m1 = iter == 0 ? (p2 * p4 * p6) : (p2 * p4 * p8);
            int m2 = iter == 0 ? (p4 * p6 * p8) : (p2 * p6 * p8);
            if (A == 1 && (B >= 2 && B <= 6) && m1 == 0 && m2 == 0) marker[(size_t)i * w + j] = 1;
        }
    }
    for (size_t k = 0; k < img.size(); ++k) img[k] &= (uint8_t)~marker[k];
}

int thin(const uint8_t *in, int w, int h, uint8_t *out) {
    std::vector<uint8_t> img(in, in + (size_t)w * h), prev((size_t)w * h, 0), marker((size_t)w * h);
    int iters = 0;
    bool diff;
    do {
        thin_iter(img, marker, w, h, 0);
        thin_iter(img, marker, w, h, 1);
        ++iters;
        diff = std::memcmp(img.data(), prev.data(), img.size()) != 0;
        prev = img;
    } while (diff);
    std::memcpy(out, img.data(), img.size());
    return iters;
}

// worldToGrid seed_gen:760-769 (float rel, floor, clamp; uses the node's grid_resolution)
static void world_to_grid(const GridInfo &gi, float grid_resolution, float wx, float wy, int &gx, int &gy) {
    float rel_x = (wx - gi.origin_x) / grid_resolution;
    float rel_y = (wy - gi.origin_y) / grid_resolution;
    gx = static_cast<int>(std::floor(rel_x));
    gy = static_cast<int>(std::floor(rel_y));
    if (gx < 0) gx = 0; else if (gx >= static_cast<int>(gi.width)) gx = static_cast<int>(gi.width) - 1;
    if (gy < 0) gy = 0; else if (gy >= static_cast<int>(gi.height)) gy = static_cast<int>(gi.height) - 1;
}

// drawLineInGrid seed_gen:828-870 (Bresenham)
static void draw_line(int8_t *g, int width, int height, int x0, int y0, int x1, int y1) {
    x0 = std::max(0, std::min(width - 1, x0)); y0 = std::max(0, std::min(height - 1, y0));
    x1 = std::max(0, std::min(width - 1, x1)); y1 = std::max(0, std::min(height - 1, y1));
    int dx = std::abs(x1 - x0), dy = std::abs(y1 - y0);
    int sx = (x0 < x1) ? 1 : -1, sy = (y0 < y1) ? 1 : -1;
    int err = dx - dy, x = x0, y = y0;
    while (true) {
        int index = x + y * width;
        if (index >= 0 && index < width * height) g[index] = 100;
        if (x == x1 && y == y1) break;
        int e2 = 2 * err;
        if (e2 > -dy) { err -= dy; x += sx; }
        if (e2 < dx) { err += dx; y += sy; }
    }
}

// ---------------------------------------------------------------- a8 clusterOccupiedCells seed_gen:970-1083
static std::vector<Cluster> cluster_cells(const int8_t *grid, const GridInfo &gi, float res, const Poly &poly) {
    std::vector<Cluster> clusters;
    const int W = (int)gi.width, H = (int)gi.height;
    std::vector<uint8_t> visited((size_t)W * H, 0);
    const int dxs[] = {-1, -1, -1, 0, 0, 1, 1, 1};
    const int dys[] = {-1, 0, 1, -1, 1, -1, 0, 1};
    for (int y = 0; y < H; y++) {
        for (int x = 0; x < W; x++) {
            int index = x + y * W;
            if (grid[index] != 100 || visited[index]) continue;
            float world_x = gi.origin_x + static_cast<float>(x) * res;
            float world_y = gi.origin_y + static_cast<float>(y) * res;
            if (!point_in_polygon(world_x, world_y, poly)) { visited[index] = 1; continue; }
            Cluster cluster;
            std::queue<std::pair<int, int>> q;
            q.push({x, y});
            visited[index] = 1;
            while (!q.empty()) {
                auto cur = q.front(); q.pop();
                int cx = cur.first, cy = cur.second;
                cluster.cells.push_back({cx, cy});
                for (int i = 0; i < 8; i++) {
                    int nx = cx + dxs[i], ny = cy + dys[i];
                    if (nx >= 0 && nx < W && ny >= 0 && ny < H) {
                        int ni = nx + ny * W;
                        if (!visited[ni] && grid[ni] == 100) {
                            float nwx = gi.origin_x + static_cast<float>(nx) * res;
                            float nwy = gi.origin_y + static_cast<float>(ny) * res;
                            if (!point_in_polygon(nwx, nwy, poly)) { visited[ni] = 1; continue; }
                            visited[ni] = 1;
                            q.push({nx, ny});
                        }
                    }
                }
            }
            float sum_x = 0.0f, sum_y = 0.0f;
            for (const auto &c : cluster.cells) { sum_x += c.first; sum_y += c.second; }
            cluster.center_x = sum_x / cluster.cells.size();
            cluster.center_y = sum_y / cluster.cells.size();
            cluster.size = (int)cluster.cells.size();
            float max_distance = 0.0f;  // O(n^2) exactly as seed_gen:1063-1073
            for (size_t i = 0; i < cluster.cells.size(); i++)
                for (size_t j = i + 1; j < cluster.cells.size(); j++) {
                    int ddx = cluster.cells[i].first - cluster.cells[j].first;
                    int ddy = cluster.cells[i].second - cluster.cells[j].second;
                    float distance = std::sqrt(ddx * ddx + ddy * ddy) * res;
                    if (distance > max_distance) max_distance = distance;
                }
            cluster.length = max_distance;
            clusters.push_back(std::move(cluster));
        }
    }
    return clusters;
}

// ---------------------------------------------------------------- rays
// raycastToOccupiedCell seed_gen:1730-1771
static bool raycast_to_occupied(const int8_t *g, const GridInfo &gi, float grid_resolution, double start_x, double start_y,
                                double dir_x, double dir_y, double max_distance, double &hit_x, double &hit_y) {
    const double step_size = grid_resolution * 0.5;
    const int max_steps = static_cast<int>(max_distance / step_size);
    const double min_distance = 1.0;
    double cx = start_x, cy = start_y;
    const int size = (int)(gi.width * gi.height);
    for (int i = 0; i < max_steps; ++i) {
        cx += dir_x * step_size;
        cy += dir_y * step_size;
        double dx = cx - start_x, dy = cy - start_y;
        double distance = std::sqrt(dx * dx + dy * dy);
        if (distance < min_distance) continue;
        int gx, gy;
        world_to_grid(gi, grid_resolution, static_cast<float>(cx), static_cast<float>(cy), gx, gy);
        int index = gx + gy * (int)gi.width;
        if (index >= 0 && index < size && g[index] == 100) { hit_x = cx; hit_y = cy; return true; }
    }
    return false;
}

// castRayFromEndpoint seed_gen:1774-1891
static V2 cast_ray_from_endpoint(V2 start, V2 other, double angle_offset_deg, const int8_t *g, const GridInfo &gi,
                                 double min_distance) {
    V2 e2o = other - start;
    double dist_to_other = norm(e2o);
    if (dist_to_other < 1e-6) e2o = V2{1.0, 0.0}; else e2o = normalized(e2o);
    V2 outward = -e2o;
    V2 perp{-e2o.y, e2o.x};
    double a = angle_offset_deg * M_PI / 180.0;
    V2 ray;
    if (angle_offset_deg > 0) ray = lib_cos(a) * outward + lib_sin(a) * perp;
    else ray = lib_cos(-a) * outward + lib_sin(-a) * (-perp);
    ray = normalized(ray);
    const double minx = gi.origin_x, maxx = minx + gi.width * gi.resolution;
    const double miny = gi.origin_y, maxy = miny + gi.height * gi.resolution;
    auto inside = [&](V2 p) { return p.x >= minx && p.x <= maxx && p.y >= miny && p.y <= maxy; };
    auto occupied = [&](V2 p) {
        const double resolution = gi.resolution;
        int mx = static_cast<int>((p.x - gi.origin_x) / resolution);
        int my = static_cast<int>((p.y - gi.origin_y) / resolution);
        if (mx >= 0 && mx < (int)gi.width && my >= 0 && my < (int)gi.height) return g[mx + my * (int)gi.width] == 100;
        return false;
    };
    const double step_size = 0.1;
    double current = min_distance;
    double gw = gi.width * gi.resolution, gh = gi.height * gi.resolution;
    double amax = std::sqrt(gw * gw + gh * gh) * 3.0;
    while (current <= amax) {
        V2 cp = start + ray * current;
        if (!inside(cp)) return V2{std::max(minx, std::min(maxx, cp.x)), std::max(miny, std::min(maxy, cp.y))};
        if (occupied(cp)) return cp;
        current += step_size;
    }
    V2 fp = start + ray * amax;
    if (!inside(fp)) { fp.x = std::max(minx, std::min(maxx, fp.x)); fp.y = std::max(miny, std::min(maxy, fp.y)); }
    return fp;
}

static inline bool near_any(const std::vector<V2> &list, V2 p) {  // sqrt(pow+pow) < 0.5 (seed_gen:2076-2085 ...)
    for (const auto &e : list) {
        double dist = std::sqrt(std::pow(e.x - p.x, 2) + std::pow(e.y - p.y, 2));
        if (dist < 0.5) return true;
    }
    return false;
}

// generateVirtualSeeds seed_gen:1987-2268 (real_seeds_ is always empty: convertVirtualSeedsToReal
// never finds a confirmed tree, seed_gen:2277-2278)
static std::vector<V2> virtual_seeds(const std::vector<TreeRow> &rows, const int8_t *skel, const GridInfo &gi, float res,
                                     const Poly &poly) {
    std::vector<V2> seeds;
    const double interval = 1.0;
    for (size_t r = 0; r < rows.size(); ++r) {
        const TreeRow &row = rows[r];
        if (!point_in_polygon(row.center.x, row.center.y, poly)) continue;
        double dx = row.end.x - row.start.x, dy = row.end.y - row.start.y;
        double distance = std::sqrt(dx * dx + dy * dy);
        if (distance < interval) continue;
        double nrm = std::sqrt(dx * dx + dy * dy);
        if (nrm < 1e-6) continue;
        double rdx = dx / nrm, rdy = dy / nrm;
        double p1x = -rdy, p1y = rdx, p2x = rdy, p2y = -rdx;
        int num = static_cast<int>(std::floor(distance / interval));
        for (int i = 1; i <= num; ++i) {
            double t = static_cast<double>(i) / (num + 1);
            double bx = row.start.x + t * dx, by = row.start.y + t * dy;
            V2 base{bx, by};
            if (!near_any(seeds, base)) seeds.push_back(base);
            const double maxd = 4.0;
            for (int side = 0; side < 2; ++side) {
                double pdx = side == 0 ? p1x : p2x, pdy = side == 0 ? p1y : p2y;
                double hx, hy, sx, sy;
                if (raycast_to_occupied(skel, gi, res, bx, by, pdx, pdy, maxd, hx, hy)) { sx = hx; sy = hy; }
                else { sx = bx + pdx * maxd; sy = by + pdy * maxd; }
                if (point_in_polygon(sx, sy, poly)) continue;
                V2 s{sx, sy};
                if (!near_any(seeds, s)) seeds.push_back(s);
            }
        }
    }
    return seeds;
}

// generateRayPointsFromEndpoints seed_gen:1894-1982
static std::vector<V2> endpoint_ray_seeds(const std::vector<TreeRow> &rows, const int8_t *skel, const GridInfo &gi,
                                          const Poly &poly) {
    std::vector<V2> out;
    const double minx = gi.origin_x, maxx = minx + gi.width * gi.resolution;
    const double miny = gi.origin_y, maxy = miny + gi.height * gi.resolution;
    for (const auto &row : rows) {
        V2 ep1 = row.start, ep2 = row.end;
        V2 pts[6] = {cast_ray_from_endpoint(ep1, ep2, 0.0, skel, gi, 1.0), cast_ray_from_endpoint(ep1, ep2, -90.0, skel, gi, 1.0),
                     cast_ray_from_endpoint(ep1, ep2, 90.0, skel, gi, 1.0), cast_ray_from_endpoint(ep2, ep1, 0.0, skel, gi, 1.0),
                     cast_ray_from_endpoint(ep2, ep1, -90.0, skel, gi, 1.0), cast_ray_from_endpoint(ep2, ep1, 90.0, skel, gi, 1.0)};
        for (const V2 &p : pts) {
            if (!(std::isfinite(p.x) && std::isfinite(p.y))) continue;
            if (!(p.x >= minx && p.x <= maxx && p.y >= miny && p.y <= maxy)) continue;
            if (point_in_polygon(p.x, p.y, poly)) continue;
            if (!near_any(out, p)) out.push_back(p);
        }
    }
    return out;
}

// ---------------------------------------------------------------- processPointCloud seed_gen:452-579
void seedgen(const Params &P, const float *xyz, uint64_t n, bool is_dense, const Poly &poly, SeedGenResult &R) {
    R.n_input = n;
    R.ror_keep.assign(n, 0);
    ror(xyz, n, is_dense, P.ror_radius, P.ror_min_neighbors, R.ror_keep.data());
    R.n_ror_kept = 0;
    for (uint64_t i = 0; i < n; ++i) R.n_ror_kept += R.ror_keep[i];

    float use_minx, use_maxx, use_miny, use_maxy;
    active_bounds(poly, use_minx, use_maxx, use_miny, use_maxy);
    const float res = P.grid_resolution;

    // generateOccupancyGrid seed_gen:581-622
    float width = std::max(0.0f, use_maxx - use_minx);
    float height = std::max(0.0f, use_maxy - use_miny);
    unsigned int w_cells = static_cast<unsigned int>(std::ceil(width / res));
    unsigned int h_cells = static_cast<unsigned int>(std::ceil(height / res));
    if (w_cells == 0) w_cells = 1;
    if (h_cells == 0) h_cells = 1;
    GridInfo gi{(double)use_minx, (double)use_miny, res, w_cells, h_cells};
    R.info = gi;
    const size_t C = (size_t)w_cells * h_cells;
    R.raster.assign(C, 0);

    // PassThrough z, x, y (inclusive, non-finite dropped) + exclusion discs seed_gen:459-525
    struct Ex { float x, y, radius; };
    static const Ex excl[] = {{0.646417f, 3.83918f, 1.0f},  {2.0405f, 3.62485f, 1.0f},  {65.3711f, 2.09755f, 1.0f},
                              {66.9094f, 2.07515f, 1.0f},  {-1.61309f, 5.69933f, 1.0f}, {-1.97349f, 4.77329f, 1.0f},
                              {-2.11365f, 3.74464f, 1.0f}, {-2.26381f, 2.70848f, 1.0f}, {-2.66426f, 1.72738f, 1.0f},
                              {68.0229f, 2.31687f, 1.0f},  {65.4647f, 2.18653f, 1.0f}};
    R.n_clipped = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (!R.ror_keep[i]) continue;
        const float px = xyz[3 * i], py = xyz[3 * i + 1], pz = xyz[3 * i + 2];
        if (!std::isfinite(px) || !std::isfinite(py) || !std::isfinite(pz)) continue;
        if (pz < P.clip_minz || pz > P.clip_maxz) continue;
        if (px < use_minx || px > use_maxx) continue;
        if (py < use_miny || py > use_maxy) continue;
        bool exclude = false;
        for (const auto &e : excl) {
            float dx = px - e.x, dy = py - e.y;
            float dist_sq = dx * dx + dy * dy;
            if (dist_sq <= e.radius * e.radius) { exclude = true; break; }
        }
        if (exclude) continue;
        ++R.n_clipped;
        int grid_x = static_cast<int>((px - gi.origin_x) / res);
        int grid_y = static_cast<int>((py - gi.origin_y) / res);
        if (grid_x >= 0 && grid_x < (int)w_cells && grid_y >= 0 && grid_y < (int)h_cells)
            R.raster[grid_x + (size_t)grid_y * w_cells] = 100;
    }

    // a5 inflation
    int inflation_cells = static_cast<int>(P.inflation_radius / res);
    R.inflated.assign(C, 0);
    inflate(R.raster.data(), (int)w_cells, (int)h_cells, inflation_cells, R.inflated.data());
    // a6 frame -> /occupancy_grid
    R.occupancy = R.inflated;
    mark_boundaries(R.occupancy.data(), (int)w_cells, (int)h_cells);

    // a7 skeleton of the frameless inflated grid
    std::vector<uint8_t> bin(C);
    for (size_t k = 0; k < C; ++k) bin[k] = R.inflated[k] == 100 ? 1 : 0;
    R.opened.assign(C, 0);
    open_cross(bin.data(), (int)w_cells, (int)h_cells, R.opened.data());
    std::vector<uint8_t> sk(C);
    R.thin_iters = thin(R.opened.data(), (int)w_cells, (int)h_cells, sk.data());
    R.skeleton.assign(C, 0);
    for (size_t k = 0; k < C; ++k) R.skeleton[k] = sk[k] ? 100 : 0;

    // a8/a9 clustering + length filter seed_gen:1258-1306
    R.clusters = cluster_cells(R.skeleton.data(), gi, res, poly);
    std::vector<const Cluster *> filtered;
    float min_length = static_cast<float>(P.cluster_min_length);
    for (const auto &c : R.clusters)
        if (c.length >= min_length) filtered.push_back(&c);
    // exploration clusters -> publishClusterInfo seed_gen:1515-1565 (sorted by centre y)
    {
        struct CI { size_t index; float cx, cy; };
        std::vector<CI> infos;
        for (const Cluster *c : filtered) {
            if (c->cells.empty()) continue;
            float cx = gi.origin_x + c->center_x * res, cy = gi.origin_y + c->center_y * res;
            if (point_in_polygon(cx, cy, poly)) infos.push_back({infos.size(), cx, cy});
        }
        std::sort(infos.begin(), infos.end(), [](const CI &a, const CI &b) { return a.cy < b.cy; });
        R.cluster_info.clear();
        for (const auto &ci : infos) R.cluster_info.push_back(V2{ci.cx, ci.cy});
    }

    // a10 convertClustersToTreeRows seed_gen:1309-1406
    R.rows.clear();
    for (const Cluster *cl : filtered) {
        if (cl->cells.empty()) continue;
        float center_x = gi.origin_x + cl->center_x * res;
        float center_y = gi.origin_y + cl->center_y * res;
        if (!point_in_polygon(center_x, center_y, poly)) continue;
        TreeRow row;
        row.center = V2{center_x, center_y};
        std::vector<V2> wp;
        wp.reserve(cl->cells.size());
        for (const auto &cell : cl->cells) {
            float wx = gi.origin_x + cell.first * res;
            float wy = gi.origin_y + cell.second * res;
            wp.push_back(V2{wx, wy});
        }
        double max_dist_sq = 0.0;
        size_t first_idx = 0;
        V2 first_dir{0.0, 0.0};
        for (size_t i = 0; i < wp.size(); ++i) {
            V2 diff = wp[i] - row.center;
            double d2 = squared_norm(diff);
            if (d2 > max_dist_sq) { max_dist_sq = d2; first_idx = i; first_dir = normalized(diff); }
        }
        double max_opp = 0.0;
        size_t second_idx = 0;
        for (size_t i = 0; i < wp.size(); ++i) {
            if (i == first_idx) continue;
            V2 diff = wp[i] - row.center;
            double d2 = squared_norm(diff);
            double dp = dot(normalized(diff), first_dir);
            if (dp < 0.0 && d2 > max_opp) { max_opp = d2; second_idx = i; }
        }
        if (max_opp == 0.0) {
            max_opp = 0.0;
            for (size_t i = 0; i < wp.size(); ++i) {
                if (i == first_idx) continue;
                double d2 = squared_norm(wp[i] - wp[first_idx]);
                if (d2 > max_opp) { max_opp = d2; second_idx = i; }
            }
        }
        row.start = wp[first_idx];
        row.end = wp[second_idx];
        row.length = cl->length;
        R.rows.push_back(row);
    }

    // a11-a12 seeds (frameless skeleton, seed_gen:1436-1448)
    R.virtual_seeds = virtual_seeds(R.rows, R.skeleton.data(), gi, res, poly);
    R.ray_seeds = endpoint_ray_seeds(R.rows, R.skeleton.data(), gi, poly);
    // endpoint seeds seed_gen:1451-1496
    R.endpoint_seeds.clear();
    for (const auto &row : R.rows) {
        if (!near_any(R.endpoint_seeds, row.start)) R.endpoint_seeds.push_back(row.start);
        if (!near_any(R.endpoint_seeds, row.end)) R.endpoint_seeds.push_back(row.end);
    }
    // a13 /voronoi_seeds = virtual ++ real (empty) ++ ray ++ endpoint seed_gen:1670-1710
    R.voronoi_seeds = R.virtual_seeds;
    R.voronoi_seeds.insert(R.voronoi_seeds.end(), R.ray_seeds.begin(), R.ray_seeds.end());
    R.voronoi_seeds.insert(R.voronoi_seeds.end(), R.endpoint_seeds.begin(), R.endpoint_seeds.end());

    // a14 /exploration_tree_rows_info seed_gen:2546-2582 (std::sort with the reference comparator)
    std::vector<TreeRow> sorted = R.rows;
    std::sort(sorted.begin(), sorted.end(), [](const TreeRow &a, const TreeRow &b) {
        if (std::abs(a.center.y - b.center.y) < 1e-6) return a.center.x < b.center.x;
        return a.center.y < b.center.y;
    });
    R.rows_info.clear();
    for (const auto &r : sorted) { R.rows_info.push_back(r.start); R.rows_info.push_back(r.end); }

    // a16 markPolygonBoundaryAsOccupied seed_gen:772-825 -> /skeletonized_occupancy_grid
    R.skeleton_framed = R.skeleton;
    {
        double hminx = poly[0].first, hmaxx = poly[0].first, hminy = poly[0].second, hmaxy = poly[0].second;
        for (const auto &pt : poly) {
            hminx = std::min(hminx, pt.first); hmaxx = std::max(hmaxx, pt.first);
            hminy = std::min(hminy, pt.second); hmaxy = std::max(hmaxy, pt.second);
        }
        const double margin = 2.5;
        int gx0, gy0, gx1, gy1;
        world_to_grid(gi, res, static_cast<float>(hminx - margin), static_cast<float>(hminy - margin), gx0, gy0);
        world_to_grid(gi, res, static_cast<float>(hmaxx + margin), static_cast<float>(hmaxy + margin), gx1, gy1);
        int8_t *g = R.skeleton_framed.data();
        draw_line(g, (int)w_cells, (int)h_cells, gx0, gy0, gx1, gy0);
        draw_line(g, (int)w_cells, (int)h_cells, gx0, gy1, gx1, gy1);
        draw_line(g, (int)w_cells, (int)h_cells, gx0, gy0, gx0, gy1);
        draw_line(g, (int)w_cells, (int)h_cells, gx1, gy0, gx1, gy1);
    }
}

}  // namespace orc
