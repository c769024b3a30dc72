// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
// CPU restatement of aos_path_gen_node's planning over the GvdGraph:
//   graphCallback                      src/aos_path_gen_node.cpp:418-579
//   buildWaypointSequence              :588-702
//   buildClusterWaypointMapping        :704-765
//   distance / heuristic / astar       :781-896   (edge cost by a linear scan of the edge list, as written)
//   findNearestNode / findKNearestNodes :898-932
//   calculatePathCost                  :935-973
//   planAndPublishPath                 :976-1567
//   trimPathNearOccupiedRegions        :1570-1630
//   calculateClusterIndex              :1633-1652
// The node's ROS state (current target, previous waypoint, current position, completion) comes in
// as orc_path_query; the published /path poses, the status and the indices go out.
#include <algorithm>
#include <cmath>
#include <functional>
#include <limits>
#include <map>
#include <new>
#include <queue>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "oracle.h"

namespace {

struct Pt { double x, y; };
struct Pose { double x, y, qz, qw; };

// The reference is built without optimisation (colcon without CMAKE_BUILD_TYPE; CMakeLists.txt:12),
// so sin and cos are separate libm calls. An optimising compiler fuses sin(y) and cos(y) of the same
// argument into one sincos call, whose result can differ by an ulp: keep them in separate functions.
__attribute__((noinline)) double half_sin(double yaw) { return std::sin(yaw / 2.0); }
__attribute__((noinline)) double half_cos(double yaw) { return std::cos(yaw / 2.0); }

struct Planner {
    // graph (graphCallback :420-454)
    std::vector<Pt> nodes;
    std::vector<int> edges;
    std::vector<float> lengths;
    std::vector<int> labels, cluster_indices, label_clusters, label_types, label_counts;
    std::vector<std::vector<int>> adj;
    // skeleton (skeletonizedGridCallback :345-347)
    const int8_t *grid = nullptr;
    double origin_x = 0, origin_y = 0, resolution = 0;
    int width = 0, height = 0;
    // state
    std::unordered_map<int, std::vector<int>> cluster_waypoint_nodes;
    std::vector<Pt> waypoints;
    std::vector<int> waypoint_nodes;
    int current_target = -1, previous_waypoint = -1;
    bool initial_reached = false, exploration_completed = false, have_current = false;
    Pt initial{8.0, 0.0}, current{0, 0};
    // result
    int status = 0;
    std::vector<int> best_path_out;
    std::vector<Pose> path;
    int trimmed_from = -1;

    static double distance(Pt a, Pt b) {   // :781-785
        double dx = a.x - b.x;
        double dy = a.y - b.y;
        return std::sqrt(dx * dx + dy * dy);
    }
    double heuristic(int n, int goal, double w) {   // :789-797
        if (n < 0 || n >= (int)nodes.size() || goal < 0 || goal >= (int)nodes.size())
            return std::numeric_limits<double>::max();
        return distance(nodes[n], nodes[goal]) * w;
    }
    double edge_cost(int a, int b) {   // the scan inside astar :862-879 and calculatePathCost :945-962
        double c = std::numeric_limits<double>::max();
        for (size_t i = 0; i < edges.size(); i += 2) {
            if (i + 1 < edges.size()) {
                int from = edges[i], to = edges[i + 1];
                if ((from == a && to == b) || (from == b && to == a)) {
                    size_t e = i / 2;
                    c = e < lengths.size() ? (double)lengths[e] : distance(nodes[a], nodes[b]);
                    break;
                }
            }
        }
        return c;
    }

    struct NodeCost {
        int node_idx; double g_cost, f_cost;
        bool operator>(const NodeCost &o) const { return f_cost > o.f_cost; }
    };
    std::vector<int> astar(int start, int goal) {   // :800-896
        if (start < 0 || start >= (int)nodes.size() || goal < 0 || goal >= (int)nodes.size()) return {};
        if (start == goal) return {start};
        if (adj[start].empty()) return {};
        if (adj[goal].empty()) return {};
        const double W = 3.0;
        std::priority_queue<NodeCost, std::vector<NodeCost>, std::greater<NodeCost>> pq;
        std::vector<double> g(nodes.size(), std::numeric_limits<double>::max());
        std::vector<int> parent(nodes.size(), -1);
        std::unordered_set<int> visited;
        g[start] = 0.0;
        pq.push({start, 0.0, heuristic(start, goal, W)});
        while (!pq.empty()) {
            NodeCost cur = pq.top();
            pq.pop();
            if (visited.find(cur.node_idx) != visited.end()) continue;
            visited.insert(cur.node_idx);
            if (cur.node_idx == goal) {
                std::vector<int> p;
                for (int n = goal; n != -1; n = parent[n]) p.push_back(n);
                std::reverse(p.begin(), p.end());
                return p;
            }
            for (int nb : adj[cur.node_idx]) {
                if (visited.find(nb) != visited.end()) continue;
                double c = edge_cost(cur.node_idx, nb);
                double ng = g[cur.node_idx] + c;
                if (ng < g[nb]) {
                    g[nb] = ng;
                    parent[nb] = cur.node_idx;
                    double h = heuristic(nb, goal, W);
                    pq.push({nb, ng, ng + h});
                }
            }
        }
        return {};
    }
    int nearest(Pt p) {   // :898-911
        int best = -1;
        double m = std::numeric_limits<double>::max();
        for (size_t i = 0; i < nodes.size(); ++i) {
            double d = distance(p, nodes[i]);
            if (d < m) { m = d; best = (int)i; }
        }
        return best;
    }
    std::vector<int> k_nearest(Pt p, int k) {   // :914-932
        std::vector<std::pair<double, int>> nd;
        for (size_t i = 0; i < nodes.size(); ++i) nd.push_back({distance(p, nodes[i]), (int)i});
        std::sort(nd.begin(), nd.end());
        std::vector<int> r;
        for (size_t i = 0; i < std::min((size_t)k, nd.size()); ++i) r.push_back(nd[i].second);
        return r;
    }
    double path_cost(const std::vector<int> &np) {   // :935-973
        if (np.size() < 2) return 0.0;
        double total = 0.0;
        for (size_t i = 0; i + 1 < np.size(); ++i) {
            double c = edge_cost(np[i], np[i + 1]);
            if (c == std::numeric_limits<double>::max()) c = distance(nodes[np[i]], nodes[np[i + 1]]);
            total += c;
        }
        return total;
    }

    void build_mapping() {   // :704-765
        cluster_waypoint_nodes.clear();
        if (label_counts.empty() || label_clusters.empty() || label_types.empty()) {
            for (size_t i = 0; i < labels.size(); ++i) {
                int mask = labels[i], ci = cluster_indices[i];
                if (ci >= 0 && mask > 0) {
                    if (cluster_waypoint_nodes.find(ci) == cluster_waypoint_nodes.end())
                        cluster_waypoint_nodes[ci] = std::vector<int>(4, -1);
                    for (int b = 0; b < 4; ++b)
                        if (mask & (1 << b)) cluster_waypoint_nodes[ci][b] = (int)i;
                }
            }
        } else {
            int k = 0;
            for (size_t i = 0; i < label_counts.size(); ++i) {
                int cnt = label_counts[i];
                for (int j = 0; j < cnt; ++j) {
                    if (k + j < (int)label_clusters.size() && k + j < (int)label_types.size()) {
                        int ci = label_clusters[k + j], t = label_types[k + j];
                        if (ci >= 0 && t >= 0 && t <= 3) {
                            if (cluster_waypoint_nodes.find(ci) == cluster_waypoint_nodes.end())
                                cluster_waypoint_nodes[ci] = std::vector<int>(4, -1);
                            if (cluster_waypoint_nodes[ci][t] < 0) cluster_waypoint_nodes[ci][t] = (int)i;
                        }
                    }
                }
                k += cnt;
            }
        }
    }

    void build_sequence() {   // :588-702
        waypoints.clear();
        waypoint_nodes.clear();
        if (cluster_waypoint_nodes.empty()) return;
        std::vector<int> ids;
        for (const auto &kv : cluster_waypoint_nodes) ids.push_back(kv.first);
        std::sort(ids.begin(), ids.end());
        std::vector<Pt> tw;
        std::vector<int> tn;
        int max_id = ids.empty() ? -1 : ids.back();
        bool last_odd = (max_id >= 0 && max_id % 2 == 1);
        auto add = [&](int n) {
            if (n >= 0 && n < (int)nodes.size()) { tw.push_back(nodes[n]); tn.push_back(n); }
        };
        for (size_t i = 0; i < ids.size(); ++i) {
            int ci = ids[i];
            bool last = (i == ids.size() - 1);
            const std::vector<int> &w = cluster_waypoint_nodes[ci];
            if (ci % 2 == 0) {
                add(w[3]); add(w[2]);
                if (last && !last_odd) add(w[1]);
            } else {
                add(w[0]); add(w[1]);
                if (last && last_odd) add(w[2]);
            }
        }
        const double min_d = 0.2;
        if (!tw.empty()) {
            waypoints.push_back(tw[0]);
            waypoint_nodes.push_back(tn[0]);
            for (size_t i = 1; i < tw.size(); ++i)
                if (distance(tw[i], waypoints.back()) > min_d) { waypoints.push_back(tw[i]); waypoint_nodes.push_back(tn[i]); }
        }
    }

    // graphCallback :456-560 (saved_position: the current target's position in the old sequence).
    // After completion the reference keeps its old sequence (:483-485), which ends at the origin; this
    // restatement has no old sequence and models it as the sequence of this graph plus the origin.
    void on_graph(bool have_saved, Pt saved_pos) {
        build_mapping();
        bool had_origin = false;
        Pt saved_origin{0, 0};
        if (exploration_completed) {   // the frozen sequence ended with the origin: rebuilt, origin re-appended
            had_origin = true;
        }
        const int saved_index = current_target;
        build_sequence();
        if (exploration_completed && had_origin) {
            if (waypoints.empty() || distance(saved_origin, waypoints.back()) > 0.2) {
                waypoints.push_back(saved_origin);
                waypoint_nodes.push_back(-1);
            }
        }
        const int nw = (int)waypoints.size();
        if (have_saved && !waypoints.empty()) {
            int best = -1;
            double m = std::numeric_limits<double>::max();
            for (int i = 0; i < nw; ++i) {
                double d = distance(saved_pos, waypoints[i]);
                if (d < m) { m = d; best = i; }
            }
            if (best >= 0 && m < 0.5) {
                current_target = best;
            } else if (saved_index >= 0 && saved_index < nw) {
                current_target = saved_index;
            } else if (!exploration_completed) {
                if (current_target < 0) current_target = 0;
            } else {
                current_target = nw - 1;
            }
        } else if (exploration_completed) {
            if (saved_index >= 0 && saved_index < nw) current_target = saved_index;
            else if (!waypoints.empty()) current_target = nw - 1;
        } else {
            if (saved_index >= 0 && saved_index < nw) current_target = saved_index;
            else if (!waypoints.empty() && current_target < 0) current_target = 0;
        }
    }

    void trim() {   // :1570-1630
        if (!grid || path.empty()) return;
        const double safety = 0.2;
        for (size_t i = 0; i < path.size(); ++i) {
            const Pose p = path[i];
            bool too_close = false;
            int rc = static_cast<int>(std::ceil(safety / resolution));
            for (int dx = -rc; dx <= rc && !too_close; ++dx) {
                for (int dy = -rc; dy <= rc && !too_close; ++dy) {
                    double cx = p.x + dx * resolution;
                    double cy = p.y + dy * resolution;
                    double dist = std::sqrt(dx * dx + dy * dy) * resolution;
                    if (dist > safety) continue;
                    int mx = static_cast<int>((cx - origin_x) / resolution);
                    int my = static_cast<int>((cy - origin_y) / resolution);
                    if (mx >= 0 && mx < width && my >= 0 && my < height) {
                        long long idx = (long long)mx + (long long)my * width;
                        if (idx >= 0 && idx < (long long)width * height && grid[idx] == 100) { too_close = true; break; }
                    }
                }
            }
            if (too_close && i > 0) {
                trimmed_from = (int)path.size();
                path.resize(i);
                break;
            }
        }
    }

    void straight(Pt from, Pt to, int first_step) {   // the 0.2 m straight-line segments (:989-1010, :1228-1250)
        double dx = to.x - from.x, dy = to.y - from.y;
        double total = std::sqrt(dx * dx + dy * dy);
        const double step = 0.2;
        int n = static_cast<int>(std::ceil(total / step));
        for (int i = first_step; i <= n; i++) {
            double t = static_cast<double>(i) / n;
            double yaw = std::atan2(dy, dx);
            path.push_back({from.x + t * dx, from.y + t * dy, half_sin(yaw), half_cos(yaw)});
        }
    }

    // appends start point + node path (:1172-1225 and :1397-1455); returns nodes added
    size_t add_node_path(const std::vector<int> &bp, Pt start, bool &start_added) {
        start_added = false;
        if (!bp.empty() && bp[0] >= 0 && bp[0] < (int)nodes.size()) {
            if (distance(start, nodes[bp[0]]) > 0.1) { path.push_back({start.x, start.y, 0.0, 1.0}); start_added = true; }
        } else {
            path.push_back({start.x, start.y, 0.0, 1.0});
            start_added = true;
        }
        size_t added = 0;
        for (size_t j = 0; j < bp.size(); ++j) {
            int n = bp[j];
            if (n < 0 || n >= (int)nodes.size()) continue;
            Pose p{nodes[n].x, nodes[n].y, 0.0, 1.0};
            double d = 0.0;
            if (!path.empty()) d = distance(Pt{path.back().x, path.back().y}, nodes[n]);
            if (path.empty()) { path.push_back(p); added++; }
            else if (d > 0.001) { path.push_back(p); added++; }
            else if (d > 0.0) { path.push_back(p); added++; }
        }
        return added;
    }

    std::vector<int> best_of(const std::vector<int> &cands, int goal, Pt start, bool skip_single, bool &found) {
        std::vector<int> best;
        double mc = std::numeric_limits<double>::max();
        found = false;
        for (int c : cands) {
            if (c == goal) continue;
            std::vector<int> np = astar(c, goal);
            if (skip_single && !np.empty() && np.size() <= 1) continue;
            if (!np.empty() && np.size() > 1) {
                found = true;
                double total = distance(start, nodes[c]) + path_cost(np);
                if (total < mc) { mc = total; best = np; }
            }
        }
        return best;
    }

    void plan() {   // planAndPublishPath(use_current_position) :976-1567
        path.clear();
        if (!initial_reached) {
            straight(Pt{0.0, 0.0}, initial, 0);
            if (!path.empty()) { path.back().x = initial.x; path.back().y = initial.y; }
            trim();
            status = 1;
            return;
        }
        if (waypoints.empty()) { status = 0; return; }
        if (current_target < 0 || current_target >= (int)waypoints.size()) { status = 0; return; }
        Pt start;
        if (have_current) start = current;
        else if (previous_waypoint >= 0 && previous_waypoint < (int)waypoints.size()) start = waypoints[previous_waypoint];
        else start = initial;
        const Pt target = waypoints[current_target];
        const int target_node = waypoint_nodes[current_target];
        if (target_node < 0) {   // origin return :1096-1280
            int goal = nearest(target);
            if (goal < 0 || goal >= (int)nodes.size()) { status = 0; return; }
            std::vector<int> cands = k_nearest(start, 5);
            if (cands.empty()) { status = 0; return; }
            bool found;
            std::vector<int> bp = best_of(cands, goal, start, false, found);
            if (!found || bp.empty()) { status = 0; return; }
            best_path_out = bp;
            bool sa;
            add_node_path(bp, start, sa);
            if (!path.empty()) {
                // :1229 binds a reference to the last pose and then appends to the same vector; the
                // values it reads are the node's position, copied here
                const Pt last{path.back().x, path.back().y};
                straight(last, target, 1);
            }
            if (!path.empty()) { path.back().x = target.x; path.back().y = target.y; }
            for (size_t i = 0; i + 1 < path.size(); ++i) {
                double dx = path[i + 1].x - path[i].x, dy = path[i + 1].y - path[i].y;
                double yaw = std::atan2(dy, dx);
                path[i].qw = half_cos(yaw);
                path[i].qz = half_sin(yaw);
            }
            trim();
            status = 1;
            return;
        }
        std::vector<int> cands = k_nearest(start, 5);   // :1283
        if (cands.empty()) { status = 0; return; }
        if (target_node < 0 || target_node >= (int)nodes.size()) { status = 0; return; }
        bool found;
        std::vector<int> bp = best_of(cands, target_node, start, true, found);
        if (!found || bp.empty()) { status = 0; return; }
        best_path_out = bp;
        bool sa;
        size_t added = add_node_path(bp, start, sa);
        if (added == 0 && !sa) { path.clear(); status = 0; return; }
        if (path.empty()) { status = 0; return; }
        if (distance(Pt{path.back().x, path.back().y}, target) > 0.01) path.push_back({target.x, target.y, 0.0, 1.0});
        else { path.back().x = target.x; path.back().y = target.y; }
        double last_yaw = 0.0;
        if (current_target < (int)waypoints.size() - 1) {
            const Pt nt = waypoints[current_target + 1];
            last_yaw = std::atan2(nt.y - path.back().y, nt.x - path.back().x);
        } else if (path.size() > 1) {
            const Pose &pp = path[path.size() - 2], &lp = path.back();
            last_yaw = std::atan2(lp.y - pp.y, lp.x - pp.x);
        }
        for (size_t i = 0; i < path.size(); ++i) {
            if (i + 1 < path.size()) {
                double yaw = std::atan2(path[i + 1].y - path[i].y, path[i + 1].x - path[i].x);
                path[i].qw = half_cos(yaw);
                path[i].qz = half_sin(yaw);
            } else {
                path[i].qw = half_cos(last_yaw);
                path[i].qz = half_sin(last_yaw);
            }
        }
        trim();
        status = 1;
    }

    int cluster_index() const {   // calculateClusterIndex :1633-1652 via publishPlanningStatus :1655-1658
        const int total = (int)cluster_waypoint_nodes.size();
        if (current_target < 0 || total <= 0) return -1;
        int c = 0, wp = 0;
        for (int i = 0; i < total; i++) {
            int n = (i == total - 1) ? 3 : 2;
            if (current_target < wp + n) { c = i; break; }
            wp += n;
        }
        return c;
    }

    // outputs
    std::vector<int> out_cluster_ids, out_cluster_nodes;
    std::vector<double> out_wp, out_poses;
};

}  // namespace

extern "C" {

void *orc_path_plan(const orc_path_graph *g, const int8_t *skeleton, double origin_x, double origin_y, float resolution,
                    uint32_t width, uint32_t height, const orc_path_query *q, orc_path_out *out) {
    auto *P = new (std::nothrow) Planner();
    if (!P) return nullptr;
    const int n = g->num_nodes;
    for (int i = 0; i < n; ++i) P->nodes.push_back({g->nodes_xy[2 * i], g->nodes_xy[2 * i + 1]});
    P->edges.assign(g->edges, g->edges + 2 * (size_t)g->num_edges);
    P->lengths.assign(g->edge_lengths, g->edge_lengths + g->num_edges);
    P->labels.assign(g->node_labels, g->node_labels + n);
    P->cluster_indices.assign(g->node_cluster_indices, g->node_cluster_indices + n);
    P->label_counts.assign(g->node_label_counts, g->node_label_counts + n);
    P->label_clusters.assign(g->node_label_clusters, g->node_label_clusters + g->n_label_entries);
    P->label_types.assign(g->node_label_types, g->node_label_types + g->n_label_entries);
    P->adj.assign(n, {});
    for (size_t i = 0; i < P->edges.size(); i += 2) {   // :440-454
        if (i + 1 < P->edges.size()) {
            int from = P->edges[i], to = P->edges[i + 1];
            if (from >= 0 && from < n && to >= 0 && to < n) { P->adj[from].push_back(to); P->adj[to].push_back(from); }
        }
    }
    P->grid = skeleton;
    P->origin_x = origin_x; P->origin_y = origin_y; P->resolution = (double)resolution;
    P->width = (int)width; P->height = (int)height;
    P->initial_reached = q->initial_waypoint_reached != 0;
    P->initial = {q->initial_waypoint_xy[0], q->initial_waypoint_xy[1]};
    P->current_target = q->target_waypoint_index;
    P->previous_waypoint = q->previous_waypoint_index;
    P->have_current = q->use_current_position != 0;
    P->current = {q->current_xy[0], q->current_xy[1]};
    P->exploration_completed = q->exploration_completed != 0;
    P->on_graph(q->have_saved_target != 0, Pt{q->saved_target_xy[0], q->saved_target_xy[1]});
    P->plan();
    if (!P->status) { P->path.clear(); P->best_path_out.clear(); P->trimmed_from = -1; }   // keeps the last path

    std::map<int, std::vector<int>> sorted(P->cluster_waypoint_nodes.begin(), P->cluster_waypoint_nodes.end());
    for (const auto &kv : sorted) {
        P->out_cluster_ids.push_back(kv.first);
        for (int t = 0; t < 4; ++t) P->out_cluster_nodes.push_back(kv.second[t]);
    }
    for (const Pt &w : P->waypoints) { P->out_wp.push_back(w.x); P->out_wp.push_back(w.y); }
    for (const Pose &p : P->path) { P->out_poses.push_back(p.x); P->out_poses.push_back(p.y); P->out_poses.push_back(p.qz); P->out_poses.push_back(p.qw); }
    out->status = P->status;
    out->target_waypoint_index = P->current_target;
    out->cluster_index = P->cluster_index();
    out->n_clusters = (int32_t)P->out_cluster_ids.size();
    out->cluster_ids = P->out_cluster_ids.data(); out->cluster_nodes = P->out_cluster_nodes.data();
    out->n_waypoints = (int32_t)P->waypoints.size();
    out->waypoints_xy = P->out_wp.data(); out->waypoint_nodes = P->waypoint_nodes.data();
    out->n_node_path = (int32_t)P->best_path_out.size(); out->node_path = P->best_path_out.data();
    out->n_poses = (int32_t)P->path.size(); out->poses = P->out_poses.data();
    out->trimmed_from = P->trimmed_from;
    return P;
}

void orc_free_path(void *h) { delete static_cast<Planner *>(h); }

}  // extern "C"
