// Path planning over the GvdGraph: aos_path_gen_node's graphCallback + planAndPublishPath
// (src/aos_path_gen_node.cpp:418-1652), behind aos_path_plan.
//
// What runs where:
//   nearest / 5 nearest nodes (:898-932)   GPU  k_nearest_k: one 512-thread workgroup keeps a
//                                              (distance, index)-ordered top-k per thread, then
//                                              merges them pairwise in LDS (the order std::sort
//                                              gives the first k pairs)
//   trimPathNearOccupiedRegions (:1570-1630) GPU  k_trim_check on the device skeleton: one thread
//                                              per pose, the first pose >= 1 within 0.2 m of an
//                                              occupied cell wins (atomicMin); the 16.8 MB grid
//                                              never crosses PCIe
//   weighted A* (:800-896)                   host: a serial best-first search; the edge cost that
//                                              the reference finds by scanning the edge list
//                                              (O(E) per relaxation) is an O(1) lookup of the first
//                                              edge of that node pair, the same edge
//   waypoints, segments, orientations        host: a few hundred poses of libm atan2/cos/sin,
//                                              bit-identical to the reference's host arithmetic
// The std::priority_queue, its comparator and its push order are the reference's, so ties pop in
// the same order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <queue>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "aos_ctx.h"

namespace aos {

// ------------------------------------------------------------------ kernels
constexpr int kNearThreads = 512, kNearK = 5;

__device__ __forceinline__ bool di_less(double da, int ia, double db, int ib) { return da < db || (da == db && ia < ib); }

// out[0..k) = indices of the k smallest (distance, index) pairs, -1 past n. distance(a, b) of the
// reference: dx = a.x - b.x, dy = a.y - b.y, sqrt(dx * dx + dy * dy) (correctly rounded sqrt).
__global__ void __launch_bounds__(kNearThreads) k_nearest_k(const double2 *nodes, int n, double px, double py, int k,
                                                             int *out) {
    __shared__ double sd[kNearThreads * kNearK];
    __shared__ int si[kNearThreads * kNearK];
    double d[kNearK];
    int id[kNearK];
#pragma unroll
    for (int j = 0; j < kNearK; ++j) { d[j] = INFINITY; id[j] = INT_MAX; }
    for (int i = threadIdx.x; i < n; i += kNearThreads) {
        const double2 q = nodes[i];
        const double dx = px - q.x, dy = py - q.y;
        const double v = sqrt(dx * dx + dy * dy);
        if (!di_less(v, i, d[k - 1], id[k - 1])) continue;
        int j = k - 1;
        while (j > 0 && di_less(v, i, d[j - 1], id[j - 1])) { d[j] = d[j - 1]; id[j] = id[j - 1]; --j; }
        d[j] = v; id[j] = i;
    }
    for (int j = 0; j < k; ++j) { sd[threadIdx.x * kNearK + j] = d[j]; si[threadIdx.x * kNearK + j] = id[j]; }
    __syncthreads();
    for (int s = kNearThreads / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const int a = threadIdx.x * kNearK, b = (threadIdx.x + s) * kNearK;
            double md[kNearK];
            int mi[kNearK];
            int ia = 0, ib = 0;
            for (int j = 0; j < k; ++j) {
                if (di_less(sd[b + ib], si[b + ib], sd[a + ia], si[a + ia])) { md[j] = sd[b + ib]; mi[j] = si[b + ib]; ++ib; }
                else { md[j] = sd[a + ia]; mi[j] = si[a + ia]; ++ia; }
            }
            for (int j = 0; j < k; ++j) { sd[a + j] = md[j]; si[a + j] = mi[j]; }
        }
        __syncthreads();
    }
    if (threadIdx.x < k) out[threadIdx.x] = si[threadIdx.x] == INT_MAX ? -1 : si[threadIdx.x];
}

// trimPathNearOccupiedRegions: pose i (>= 1) is cut when a cell within `safety` of it, sampled at
// (x + dx * res, y + dy * res) for |dx|, |dy| <= rc, holds 100. first = min such i.
__global__ void k_trim_check(const double2 *pts, int n, const int8_t *grid, int W, int H, double ox, double oy, double res,
                             int rc, double safety, int *first) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 1 || i >= n) return;
    const double2 p = pts[i];
    for (int dx = -rc; dx <= rc; ++dx) {
        for (int dy = -rc; dy <= rc; ++dy) {
            const double cx = p.x + dx * res;
            const double cy = p.y + dy * res;
            const double dist = sqrt((double)(dx * dx + dy * dy)) * res;
            if (dist > safety) continue;
            const double fx = (cx - ox) / res, fy = (cy - oy) / res;
            // static_cast<int> of an out-of-range double is INT_MIN on x86 (cvttsd2si): never in the grid
            const int mx = (fx > -2147483649.0 && fx < 2147483648.0) ? (int)fx : INT_MIN;
            const int my = (fy > -2147483649.0 && fy < 2147483648.0) ? (int)fy : INT_MIN;
            if (mx >= 0 && mx < W && my >= 0 && my < H && grid[(size_t)mx + (size_t)my * W] == 100) {
                atomicMin(first, i);
                return;
            }
        }
    }
}

// ------------------------------------------------------------------ host planner
namespace {

struct Pt { double x, y; };
struct Pose { double x, y, qz, qw; };

// The reference is built without optimisation (colcon without CMAKE_BUILD_TYPE; CMakeLists.txt:12),
// so sin and cos are separate libm calls. An optimising compiler fuses sin(y) and cos(y) of the same
// argument into one sincos call, whose result can differ by an ulp: keep them in separate functions.
__attribute__((noinline)) double half_sin(double yaw) { return std::sin(yaw / 2.0); }
__attribute__((noinline)) double half_cos(double yaw) { return std::cos(yaw / 2.0); }

double distance(Pt a, Pt b) {   // path_gen:781-785
    double dx = a.x - b.x;
    double dy = a.y - b.y;
    return std::sqrt(dx * dx + dy * dy);
}

}  // namespace

struct PathState {
    // graph in CSR form (adjacency in the reference's push order, :440-454) + first edge per pair
    const void *graph_key = nullptr;
    uint64_t graph_gen = ~0ull;
    int n = 0;
    std::vector<Pt> nodes;
    std::vector<int> off, adj;
    std::unordered_map<uint64_t, int> first_edge;
    std::vector<float> lengths;
    DevBuf d_nodes, d_pts, d_grid, d_res;
    PinnedBuf h;
    // outputs
    std::vector<int32_t> cluster_ids, cluster_nodes, waypoint_nodes, node_path;
    std::vector<double> waypoints_xy, poses;
};

void free_path_state(void *p) { delete static_cast<PathState *>(p); }

namespace {

struct Planner {
    PathState &S;
    const aos_path_graph &g;
    hipStream_t s;
    const int8_t *d_grid;
    aos_grid_info info;
    std::unordered_map<int, std::vector<int>> cwn;   // cluster_waypoint_nodes_
    std::vector<Pt> wps;
    std::vector<int> wpn;
    std::vector<int> best;
    std::vector<Pose> path;
    int target = -1, prev = -1, status = 0, trimmed_from = -1;
    bool initial_reached = false, completed = false, have_current = false;
    Pt initial{8.0, 0.0}, current{0.0, 0.0};

    Planner(PathState &S_, const aos_path_graph &g_, hipStream_t s_, const int8_t *grid, const aos_grid_info &inf)
        : S(S_), g(g_), s(s_), d_grid(grid), info(inf) {}

    double edge_cost(int a, int b) const {   // the edge-list scan of :862-879 / :945-962
        const uint64_t key = ((uint64_t)(uint32_t)std::min(a, b) << 32) | (uint32_t)std::max(a, b);
        auto it = S.first_edge.find(key);
        if (it == S.first_edge.end()) return std::numeric_limits<double>::max();
        return (double)S.lengths[it->second];
    }
    double heuristic(int n, int goal, double w) const {   // :789-797
        if (n < 0 || n >= S.n || goal < 0 || goal >= S.n) return std::numeric_limits<double>::max();
        return distance(S.nodes[n], S.nodes[goal]) * w;
    }
    struct NodeCost {
        int node_idx; double g_cost, f_cost;
        bool operator>(const NodeCost &o) const { return f_cost > o.f_cost; }
    };
    std::vector<int> astar(int start, int goal) const {   // :800-896
        if (start < 0 || start >= S.n || goal < 0 || goal >= S.n) return {};
        if (start == goal) return {start};
        if (S.off[start] == S.off[start + 1] || S.off[goal] == S.off[goal + 1]) return {};
        const double W = 3.0;
        std::priority_queue<NodeCost, std::vector<NodeCost>, std::greater<NodeCost>> pq;
        std::vector<double> gc(S.n, std::numeric_limits<double>::max());
        std::vector<int> parent(S.n, -1);
        std::vector<uint8_t> visited(S.n, 0);
        gc[start] = 0.0;
        pq.push({start, 0.0, heuristic(start, goal, W)});
        while (!pq.empty()) {
            const NodeCost cur = pq.top();
            pq.pop();
            if (visited[cur.node_idx]) continue;
            visited[cur.node_idx] = 1;
            if (cur.node_idx == goal) {
                std::vector<int> p;
                for (int v = goal; v != -1; v = parent[v]) p.push_back(v);
                std::reverse(p.begin(), p.end());
                return p;
            }
            for (int k = S.off[cur.node_idx]; k < S.off[cur.node_idx + 1]; ++k) {
                const int nb = S.adj[k];
                if (visited[nb]) continue;
                const double ng = gc[cur.node_idx] + edge_cost(cur.node_idx, nb);
                if (ng < gc[nb]) {
                    gc[nb] = ng;
                    parent[nb] = cur.node_idx;
                    pq.push({nb, ng, ng + heuristic(nb, goal, W)});
                }
            }
        }
        return {};
    }
    double path_cost(const std::vector<int> &np) const {   // :935-973
        if (np.size() < 2) return 0.0;
        double total = 0.0;
        for (size_t i = 0; i + 1 < np.size(); ++i) {
            double c = edge_cost(np[i], np[i + 1]);
            if (c == std::numeric_limits<double>::max()) c = distance(S.nodes[np[i]], S.nodes[np[i + 1]]);
            total += c;
        }
        return total;
    }
    std::vector<int> nearest_k(Pt p, int k) {   // findKNearestNodes (:914-932), findNearestNode (k = 1)
        if (S.n == 0) return {};
        int *d_out = static_cast<int *>(S.d_res.ensure(64));
        k_nearest_k<<<1, kNearThreads, 0, s>>>(S.d_nodes.as<double2>(), S.n, p.x, p.y, k, d_out + 1);
        int *h = static_cast<int *>(S.h.ensure(4096));
        AOS_HIP(hipMemcpyAsync(h, d_out + 1, sizeof(int) * k, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        std::vector<int> r;
        for (int j = 0; j < k; ++j) if (h[j] >= 0) r.push_back(h[j]);
        return r;
    }

    void build_mapping() {   // :704-765
        const int n = g.num_nodes;
        if (n == 0 || g.n_label_entries == 0) {   // counts / clusters / types empty: the old bitmask method
            for (int i = 0; i < n; ++i) {
                const int mask = g.node_labels[i], ci = g.node_cluster_indices[i];
                if (ci >= 0 && mask > 0) {
                    if (cwn.find(ci) == cwn.end()) cwn[ci] = std::vector<int>(4, -1);
                    for (int b = 0; b < 4; ++b)
                        if (mask & (1 << b)) cwn[ci][b] = i;
                }
            }
            return;
        }
        int k = 0;
        for (int i = 0; i < n; ++i) {
            const int cnt = g.node_label_counts[i];
            for (int j = 0; j < cnt; ++j) {
                if (k + j < g.n_label_entries) {
                    const int ci = g.node_label_clusters[k + j], t = g.node_label_types[k + j];
                    if (ci >= 0 && t >= 0 && t <= 3) {
                        if (cwn.find(ci) == cwn.end()) cwn[ci] = std::vector<int>(4, -1);
                        if (cwn[ci][t] < 0) cwn[ci][t] = i;
                    }
                }
            }
            k += cnt;
        }
    }
    void build_sequence() {   // :588-702
        wps.clear(); wpn.clear();
        if (cwn.empty()) return;
        std::vector<int> ids;
        for (const auto &kv : cwn) ids.push_back(kv.first);
        std::sort(ids.begin(), ids.end());
        std::vector<Pt> tw;
        std::vector<int> tn;
        const bool last_odd = ids.back() >= 0 && ids.back() % 2 == 1;
        auto add = [&](int v) { if (v >= 0 && v < S.n) { tw.push_back(S.nodes[v]); tn.push_back(v); } };
        for (size_t i = 0; i < ids.size(); ++i) {
            const int ci = ids[i];
            const bool last = i == ids.size() - 1;
            const std::vector<int> &w = cwn[ci];
            if (ci % 2 == 0) { add(w[3]); add(w[2]); if (last && !last_odd) add(w[1]); }
            else { add(w[0]); add(w[1]); if (last && last_odd) add(w[2]); }
        }
        if (!tw.empty()) {
            wps.push_back(tw[0]); wpn.push_back(tn[0]);
            for (size_t i = 1; i < tw.size(); ++i)
                if (distance(tw[i], wps.back()) > 0.2) { wps.push_back(tw[i]); wpn.push_back(tn[i]); }
        }
    }
    // graphCallback :456-560; completion is modelled as this graph's sequence plus the origin
    void on_graph(bool have_saved, Pt saved_pos) {
        build_mapping();
        const int saved_index = target;
        build_sequence();
        if (completed) {
            const Pt origin{0.0, 0.0};
            if (wps.empty() || distance(origin, wps.back()) > 0.2) { wps.push_back(origin); wpn.push_back(-1); }
        }
        const int nw = (int)wps.size();
        if (have_saved && nw > 0) {
            int bi = -1;
            double m = std::numeric_limits<double>::max();
            for (int i = 0; i < nw; ++i) {
                const double d = distance(saved_pos, wps[i]);
                if (d < m) { m = d; bi = i; }
            }
            if (bi >= 0 && m < 0.5) target = bi;
            else if (saved_index >= 0 && saved_index < nw) target = saved_index;
            else if (!completed) { if (target < 0) target = 0; }
            else target = nw - 1;
        } else if (completed) {
            if (saved_index >= 0 && saved_index < nw) target = saved_index;
            else if (nw > 0) target = nw - 1;
        } else {
            if (saved_index >= 0 && saved_index < nw) target = saved_index;
            else if (nw > 0 && target < 0) target = 0;
        }
    }

    void trim() {   // :1570-1630 on the device skeleton
        if (!d_grid || path.empty()) return;
        const int n = (int)path.size();
        double2 *h = static_cast<double2 *>(S.h.ensure(sizeof(double2) * (size_t)n + 4096));
        for (int i = 0; i < n; ++i) h[i] = make_double2(path[i].x, path[i].y);
        double2 *d_pts = static_cast<double2 *>(S.d_pts.ensure(sizeof(double2) * (size_t)n));
        int *d_first = static_cast<int *>(S.d_res.ensure(64));
        const int big = INT_MAX;
        AOS_HIP(hipMemcpyAsync(d_pts, h, sizeof(double2) * (size_t)n, hipMemcpyHostToDevice, s));
        AOS_HIP(hipMemcpyAsync(d_first, &big, sizeof(int), hipMemcpyHostToDevice, s));
        const double res = (double)info.resolution, safety = 0.2;
        const int rc = static_cast<int>(std::ceil(safety / res));
        k_trim_check<<<(n + 127) / 128, 128, 0, s>>>(d_pts, n, d_grid, (int)info.width, (int)info.height, info.origin_x,
                                                     info.origin_y, res, rc, safety, d_first);
        int *hf = reinterpret_cast<int *>(reinterpret_cast<char *>(h) + sizeof(double2) * (size_t)n);
        AOS_HIP(hipMemcpyAsync(hf, d_first, sizeof(int), hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        if (*hf != INT_MAX) { trimmed_from = n; path.resize(*hf); }
    }
    void straight(Pt from, Pt to, int first_step) {   // :989-1010, :1228-1250
        const double dx = to.x - from.x, dy = to.y - from.y;
        const double total = std::sqrt(dx * dx + dy * dy);
        const int steps = static_cast<int>(std::ceil(total / 0.2));
        for (int i = first_step; i <= steps; i++) {
            const double t = static_cast<double>(i) / steps;
            const double yaw = std::atan2(dy, dx);
            path.push_back({from.x + t * dx, from.y + t * dy, half_sin(yaw), half_cos(yaw)});
        }
    }
    size_t add_node_path(const std::vector<int> &bp, Pt start, bool &start_added) {   // :1172-1225, :1397-1455
        start_added = false;
        if (!bp.empty() && bp[0] >= 0 && bp[0] < S.n) {
            if (distance(start, S.nodes[bp[0]]) > 0.1) { path.push_back({start.x, start.y, 0.0, 1.0}); start_added = true; }
        } else {
            path.push_back({start.x, start.y, 0.0, 1.0});
            start_added = true;
        }
        size_t added = 0;
        for (int v : bp) {
            if (v < 0 || v >= S.n) continue;
            const double d = path.empty() ? 0.0 : distance(Pt{path.back().x, path.back().y}, S.nodes[v]);
            if (path.empty() || d > 0.001 || d > 0.0) { path.push_back({S.nodes[v].x, S.nodes[v].y, 0.0, 1.0}); added++; }
        }
        return added;
    }
    std::vector<int> best_of(const std::vector<int> &cands, int goal, Pt start, bool &found) const {
        std::vector<int> bp;
        double mc = std::numeric_limits<double>::max();
        found = false;
        for (int c : cands) {
            if (c == goal) continue;
            const std::vector<int> np = astar(c, goal);
            if (np.size() > 1) {
                found = true;
                const double total = distance(start, S.nodes[c]) + path_cost(np);
                if (total < mc) { mc = total; bp = np; }
            }
        }
        return bp;
    }
    void orient_all(bool last_too, double last_yaw) {
        for (size_t i = 0; i < path.size(); ++i) {
            if (i + 1 < path.size()) {
                const double yaw = std::atan2(path[i + 1].y - path[i].y, path[i + 1].x - path[i].x);
                path[i].qw = half_cos(yaw);
                path[i].qz = half_sin(yaw);
            } else if (last_too) {
                path[i].qw = half_cos(last_yaw);
                path[i].qz = half_sin(last_yaw);
            }
        }
    }
    void plan() {   // planAndPublishPath :976-1567
        path.clear();
        if (!initial_reached) {
            straight(Pt{0.0, 0.0}, initial, 0);
            if (!path.empty()) { path.back().x = initial.x; path.back().y = initial.y; }
            trim();
            status = 1;
            return;
        }
        if (wps.empty() || target < 0 || target >= (int)wps.size()) return;
        Pt start = initial;
        if (have_current) start = current;
        else if (prev >= 0 && prev < (int)wps.size()) start = wps[prev];
        const Pt tgt = wps[target];
        const int tnode = wpn[target];
        if (tnode < 0) {   // origin return :1096-1280
            const std::vector<int> nn = nearest_k(tgt, 1);
            if (nn.empty()) return;
            const std::vector<int> cands = nearest_k(start, kNearK);
            if (cands.empty()) return;
            bool found;
            const std::vector<int> bp = best_of(cands, nn[0], start, found);
            if (!found || bp.empty()) return;
            best = bp;
            bool sa;
            add_node_path(bp, start, sa);
            if (!path.empty()) straight(Pt{path.back().x, path.back().y}, tgt, 1);
            if (!path.empty()) { path.back().x = tgt.x; path.back().y = tgt.y; }
            orient_all(false, 0.0);
            trim();
            status = 1;
            return;
        }
        const std::vector<int> cands = nearest_k(start, kNearK);   // :1283
        if (cands.empty() || tnode >= S.n) return;
        bool found;
        const std::vector<int> bp = best_of(cands, tnode, start, found);
        if (!found || bp.empty()) return;
        best = bp;
        bool sa;
        const size_t added = add_node_path(bp, start, sa);
        if ((added == 0 && !sa) || path.empty()) return;
        if (distance(Pt{path.back().x, path.back().y}, tgt) > 0.01) path.push_back({tgt.x, tgt.y, 0.0, 1.0});
        else { path.back().x = tgt.x; path.back().y = tgt.y; }
        double last_yaw = 0.0;
        if (target < (int)wps.size() - 1) {
            const Pt nt = wps[target + 1];
            last_yaw = std::atan2(nt.y - path.back().y, nt.x - path.back().x);
        } else if (path.size() > 1) {
            const Pose &pp = path[path.size() - 2], &lp = path.back();
            last_yaw = std::atan2(lp.y - pp.y, lp.x - pp.x);
        }
        orient_all(true, last_yaw);
        trim();
        status = 1;
    }
    int cluster_index() const {   // :1633-1658
        const int total = (int)cwn.size();
        if (target < 0 || total <= 0) return -1;
        int c = 0, wp = 0;
        for (int i = 0; i < total; i++) {
            const int k = (i == total - 1) ? 3 : 2;
            if (target < wp + k) { c = i; break; }
            wp += k;
        }
        return c;
    }
};

// CSR adjacency + first-edge table, rebuilt when the graph changes (graphCallback :440-454).
void load_graph(PathState &S, const aos_path_graph &g, const void *key, uint64_t gen, hipStream_t s) {
    if (key && key == S.graph_key && gen == S.graph_gen) return;
    const int n = g.num_nodes, ne = g.num_edges;
    S.n = n;
    S.nodes.resize(n);
    for (int i = 0; i < n; ++i) S.nodes[i] = {g.nodes_xy[2 * i], g.nodes_xy[2 * i + 1]};
    S.lengths.assign(g.edge_lengths, g.edge_lengths + ne);
    S.off.assign(n + 1, 0);
    for (int e = 0; e < ne; ++e) {
        const int a = g.edges[2 * e], b = g.edges[2 * e + 1];
        if (a >= 0 && a < n && b >= 0 && b < n) { S.off[a + 1]++; S.off[b + 1]++; }
    }
    for (int i = 0; i < n; ++i) S.off[i + 1] += S.off[i];
    S.adj.resize(S.off[n]);
    std::vector<int> cur(S.off.begin(), S.off.end() - 1);
    S.first_edge.clear();
    S.first_edge.reserve(2 * (size_t)ne);
    for (int e = 0; e < ne; ++e) {
        const int a = g.edges[2 * e], b = g.edges[2 * e + 1];
        if (a >= 0 && a < n && b >= 0 && b < n) {
            S.adj[cur[a]++] = b;
            S.adj[cur[b]++] = a;
            const uint64_t k = ((uint64_t)(uint32_t)std::min(a, b) << 32) | (uint32_t)std::max(a, b);
            S.first_edge.emplace(k, e);   // keeps the first edge of the pair
        }
    }
    double2 *d = static_cast<double2 *>(S.d_nodes.ensure(sizeof(double2) * (size_t)std::max(n, 1)));
    if (n) AOS_HIP(hipMemcpyAsync(d, g.nodes_xy, sizeof(double2) * (size_t)n, hipMemcpyHostToDevice, s));
    AOS_HIP(hipStreamSynchronize(s));
    S.graph_key = key;
    S.graph_gen = gen;
}

}  // namespace

}  // namespace aos

using namespace aos;

void aos_ctx::run_path_plan(const aos_path_graph *graph, const int8_t *skeleton, int skeleton_on_device,
                            const aos_grid_info *info, const aos_path_query &q, aos_path_out &out) {
    const auto t0 = std::chrono::steady_clock::now();
    gvd_view_settle();
    if (!path_state) path_state = new PathState();
    PathState &S = *static_cast<PathState *>(path_state);
    // the graph
    aos_path_graph own{};
    const void *key = nullptr;
    uint64_t gen = 0;
    if (!graph) {
        if (!have_gvd) throw std::runtime_error("aos_path_plan: no GVD graph on this handle");
        GvdState &gs = this->gs();
        markers_wait(gs, false);
        own.num_nodes = (int32_t)gs.labels.size(); own.nodes_xy = gs.nodes_xy.data();
        own.node_labels = gs.labels.data(); own.node_cluster_indices = gs.cluster_idx.data();
        own.node_label_counts = gs.label_counts.data();
        own.n_label_entries = (int32_t)gs.label_clusters.size();
        own.node_label_clusters = gs.label_clusters.data(); own.node_label_types = gs.label_types.data();
        own.num_edges = (int32_t)gs.lengths.size(); own.edges = gs.edges_out.data(); own.edge_lengths = gs.lengths.data();
        graph = &own;
        key = &gs;
        gen = gvd_gen;
    }
    // the skeleton (device)
    const int8_t *d_grid = nullptr;
    aos_grid_info gi{};
    if (skeleton) {
        gi = *info;
        const size_t C = (size_t)gi.width * gi.height;
        if (skeleton_on_device) d_grid = skeleton;
        else {
            int8_t *d = static_cast<int8_t *>(S.d_grid.ensure(std::max<size_t>(C, 1)));
            if (C) AOS_HIP(hipMemcpyAsync(d, skeleton, C, hipMemcpyHostToDevice, stream));
            d_grid = d;
        }
    } else {
        if (!have_gvd) throw std::runtime_error("aos_path_plan: no skeleton given and no GVD call on this handle");
        if (gvd_from_frame && gvd_frame_gen != frame_gen)
            throw std::runtime_error("aos_path_plan: the GVD graph's skeleton was replaced by a later seed-gen frame; pass it");
        d_grid = gvd_skel;
        gi = gvd_info;
    }
    load_graph(S, *graph, key, gen, stream);

    Planner pl(S, *graph, stream, d_grid, gi);
    pl.initial_reached = q.initial_waypoint_reached != 0;
    pl.initial = {q.initial_waypoint_xy[0], q.initial_waypoint_xy[1]};
    pl.target = q.target_waypoint_index;
    pl.prev = q.previous_waypoint_index;
    pl.have_current = q.use_current_position != 0;
    pl.current = {q.current_xy[0], q.current_xy[1]};
    pl.completed = q.exploration_completed != 0;
    pl.on_graph(q.have_saved_target != 0, {q.saved_target_xy[0], q.saved_target_xy[1]});
    pl.plan();
    if (!pl.status) { pl.path.clear(); pl.best.clear(); pl.trimmed_from = -1; }   // the node republishes its last path

    S.cluster_ids.clear(); S.cluster_nodes.clear();
    std::map<int, std::vector<int>> sorted(pl.cwn.begin(), pl.cwn.end());
    for (const auto &kv : sorted) {
        S.cluster_ids.push_back(kv.first);
        for (int t = 0; t < 4; ++t) S.cluster_nodes.push_back(kv.second[t]);
    }
    S.waypoints_xy.clear();
    for (const auto &w : pl.wps) { S.waypoints_xy.push_back(w.x); S.waypoints_xy.push_back(w.y); }
    S.waypoint_nodes.assign(pl.wpn.begin(), pl.wpn.end());
    S.node_path.assign(pl.best.begin(), pl.best.end());
    S.poses.clear();
    for (const auto &p : pl.path) { S.poses.push_back(p.x); S.poses.push_back(p.y); S.poses.push_back(p.qz); S.poses.push_back(p.qw); }
    std::memset(&out, 0, sizeof(out));
    out.status = pl.status;
    out.target_waypoint_index = pl.target;
    out.cluster_index = pl.cluster_index();
    out.n_clusters = (int32_t)S.cluster_ids.size();
    out.cluster_ids = S.cluster_ids.data(); out.cluster_nodes = S.cluster_nodes.data();
    out.n_waypoints = (int32_t)pl.wps.size(); out.waypoints_xy = S.waypoints_xy.data(); out.waypoint_nodes = S.waypoint_nodes.data();
    out.n_node_path = (int32_t)S.node_path.size(); out.node_path = S.node_path.data();
    out.n_poses = (int32_t)pl.path.size(); out.poses = S.poses.data();
    out.trimmed_from = pl.trimmed_from;
    out.ms_plan = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
