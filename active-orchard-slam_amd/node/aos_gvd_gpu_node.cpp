// Drop-in rclcpp node for aos_gvd_node's graph build on MI355X.
// Same parameters, topics and QoS as src/aos_gvd_node.cpp:26-78; processGraph (gvd:255-318) is
// aos_gvd_process on the latest inputs. The throttle (max_graph_publish_rate, gvd:306-314) stays
// here. The reference computes the graph even when the throttle suppresses publishing; the graph
// is then unobservable, so this node skips that work. /gvd/markers (publishMarkers gvd:1012-1591)
// is built from aos_gvd_out + aos_gvd_markers_get (merged seeds, Voronoi cells, label points); the
// styles (namespaces, ids, scales, colours) are the reference's.
//
// Not built in this repository's image (no ROS 2); see INTEGRATION.md for the ament recipe.
#include <geometry_msgs/msg/pose_array.hpp>
#include <nav_msgs/msg/occupancy_grid.hpp>
#include <rclcpp/rclcpp.hpp>
#include <visualization_msgs/msg/marker_array.hpp>

#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <vector>

#include "aos/msg/gvd_graph.hpp"
#include "aos_gpu.h"

class AosGvdGpuNode : public rclcpp::Node {
  public:
    AosGvdGpuNode() : Node("aos_gvd_node") {
        rate_ = declare_parameter("max_graph_publish_rate", 10.0);
        const auto seeds_t = declare_parameter("voronoi_seeds_topic", std::string("/voronoi_seeds"));
        const auto rows_t = declare_parameter("exploration_tree_rows_info_topic", std::string("/exploration_tree_rows_info"));
        const auto all_rows_t = declare_parameter("tree_rows_all_topic", std::string("/tree_rows_all"));
        const auto skel_t = declare_parameter("skeletonized_occupancy_grid_topic", std::string("/skeletonized_occupancy_grid"));
        declare_parameter("occupancy_grid_topic", std::string("/occupancy_grid"));   // trigger only (gvd:181)
        declare_parameter("robot_position_topic", std::string("/Local/utm"));        // no effect on GvdGraph
        aos_params p;
        aos_default_params(&p);
        p.max_graph_publish_rate = rate_;
        if (aos_create(&p, declare_parameter<int>("gpu_device", 0), &ctx_) != AOS_OK) throw std::runtime_error(aos_last_error());
        // markers only for the published frames: publish_markers asks for them (computed on demand), as
        // publishMarkers runs inside the publish throttle (gvd:306-314)
        aos_gvd_set_markers(ctx_, 0);

        rclcpp::QoS reliable(10);   // gvd:44-45
        reliable.reliable();
        sub_seeds_ = create_subscription<geometry_msgs::msg::PoseArray>(seeds_t, reliable,
            [this](geometry_msgs::msg::PoseArray::SharedPtr m) {            // voronoiSeedsCallback gvd:84-128
                seeds_.clear();
                for (const auto &p : m->poses) { seeds_.push_back(p.position.x); seeds_.push_back(p.position.y); }
                process();
            });
        sub_rows_ = create_subscription<geometry_msgs::msg::PoseArray>(rows_t, reliable,
            [this](geometry_msgs::msg::PoseArray::SharedPtr m) {            // gvd:130-150
                rows_.clear();
                for (const auto &p : m->poses) { rows_.push_back(p.position.x); rows_.push_back(p.position.y); }
                process();
            });
        sub_all_rows_ = create_subscription<visualization_msgs::msg::MarkerArray>(all_rows_t, reliable,
            [this](visualization_msgs::msg::MarkerArray::SharedPtr) { process(); });   // trigger (gvd:152-171)
        sub_skel_ = create_subscription<nav_msgs::msg::OccupancyGrid>(skel_t, reliable,
            [this](nav_msgs::msg::OccupancyGrid::SharedPtr m) { skel_ = m; process(); });   // gvd:173-177
        pub_graph_ = create_publisher<aos::msg::GvdGraph>("/gvd/graph", reliable);
        pub_markers_ = create_publisher<visualization_msgs::msg::MarkerArray>("/gvd/markers", reliable);
    }
    ~AosGvdGpuNode() override { aos_destroy(ctx_); }

  private:
    void process() {
        if (seeds_.empty() || !skel_) return;   // gvd:257-259
        aos_gvd_in in{};
        in.seeds_xy = seeds_.data(); in.n_seeds = (int32_t)(seeds_.size() / 2);
        in.rows_info_xy = rows_.data(); in.n_rows_poses = (int32_t)(rows_.size() / 2);
        in.info.origin_x = skel_->info.origin.position.x;
        in.info.origin_y = skel_->info.origin.position.y;
        in.info.resolution = skel_->info.resolution;
        in.info.width = skel_->info.width;
        in.info.height = skel_->info.height;
        in.skeleton = skel_->data.data();
        aos_gvd_out o{};
        if (aos_gvd_process(ctx_, &in, &o) != AOS_OK) {
            RCLCPP_ERROR(get_logger(), "Error computing Voronoi diagram: %s", aos_last_error());   // gvd:315-317
            return;
        }
        if (!o.published) return;
        // The graph is built on every callback; only publishing is throttled, with the time taken
        // after the graph is built and measured from construction (gvd:80, 306-314).
        const auto now = std::chrono::steady_clock::now();
        if (std::chrono::duration<double>(now - last_).count() < 1.0 / rate_) return;
        aos::msg::GvdGraph g;                  // publishGraph gvd:897-1010
        g.header.frame_id = "map";
        g.header.stamp = this->now();
        g.resolution = o.resolution; g.origin_x = o.origin_x; g.origin_y = o.origin_y;
        g.num_nodes = o.num_nodes; g.num_edges = o.num_edges;
        g.nodes.resize(o.num_nodes);
        for (int i = 0; i < o.num_nodes; ++i) { g.nodes[i].x = o.nodes_xy[2 * i]; g.nodes[i].y = o.nodes_xy[2 * i + 1]; }
        g.node_labels.assign(o.node_labels, o.node_labels + o.num_nodes);
        g.node_cluster_indices.assign(o.node_cluster_indices, o.node_cluster_indices + o.num_nodes);
        g.node_label_counts.assign(o.node_label_counts, o.node_label_counts + o.num_nodes);
        g.node_label_clusters.assign(o.node_label_clusters, o.node_label_clusters + o.n_label_entries);
        g.node_label_types.assign(o.node_label_types, o.node_label_types + o.n_label_entries);
        g.edges.assign(o.edges, o.edges + 2 * o.num_edges);
        g.edge_lengths.assign(o.edge_lengths, o.edge_lengths + o.num_edges);
        g.edge_clearances.assign(o.edge_clearances, o.edge_clearances + o.num_edges);
        pub_graph_->publish(g);
        publish_markers(g.header, o);
        last_ = now;
    }

    // publishMarkers gvd:1012-1591 (content from the library, styles as in the reference)
    void publish_markers(const std_msgs::msg::Header &h, const aos_gvd_out &o) {
        aos_gvd_markers m{};
        if (aos_gvd_markers_get(ctx_, &m) != AOS_OK) return;
        using visualization_msgs::msg::Marker;
        visualization_msgs::msg::MarkerArray ma;
        Marker del;
        del.action = Marker::DELETEALL;
        ma.markers.push_back(del);
        auto mk = [&](const char *ns, int id, int type, double scale, float r, float gg, float b, float a) {
            Marker k;
            k.header = h; k.ns = ns; k.id = id; k.type = type; k.action = Marker::ADD;
            k.scale.x = k.scale.y = k.scale.z = scale;
            k.color.r = r; k.color.g = gg; k.color.b = b; k.color.a = a;
            return k;
        };
        auto pt = [](double x, double y, double z = 0.0) { geometry_msgs::msg::Point q; q.x = x; q.y = y; q.z = z; return q; };
        if (m.n_seeds > 0) {                                                       // gvd:1019-1041
            Marker s = mk("/gvd_voronoi_seeds", 0, Marker::SPHERE_LIST, 0.2, 1.0f, 1.0f, 0.0f, 1.0f);
            for (int i = 0; i < m.n_seeds; ++i) s.points.push_back(pt(m.seeds_xy[2 * i], m.seeds_xy[2 * i + 1]));
            ma.markers.push_back(s);
        }
        Marker nodes = mk("/gvd_voronoi_nodes", 0, Marker::SPHERE_LIST, 0.15, 0.8f, 0.0f, 0.8f, 1.0f);   // :1044-1064
        for (int i = 0; i < o.num_nodes; ++i) nodes.points.push_back(pt(o.nodes_xy[2 * i], o.nodes_xy[2 * i + 1]));
        ma.markers.push_back(nodes);
        Marker edges = mk("/gvd_voronoi_edges", 0, Marker::LINE_LIST, 0.08, 0.0f, 0.8f, 1.0f, 1.0f);     // :1067-1094
        for (int e = 0; e < o.num_edges; ++e)
            for (int k = 0; k < 2; ++k) {
                const int v = o.edges[2 * e + k];
                edges.points.push_back(pt(o.nodes_xy[2 * v], o.nodes_xy[2 * v + 1]));
            }
        ma.markers.push_back(edges);
        for (int i = 0; i < m.n_cells; ++i) {                                      // :1098-1194
            const int b = m.cell_offsets[i], n = m.cell_offsets[i + 1] - b;
            if (n < 3) continue;
            const float *rgba = m.cell_rgba + 4 * i;
            Marker cell = mk("/gvd_voronoi_cells", i, Marker::TRIANGLE_LIST, 1.0, rgba[0], rgba[1], rgba[2], rgba[3]);
            const auto c = pt(m.cell_center_xy[2 * i], m.cell_center_xy[2 * i + 1]);
            for (int j = 0; j < n; ++j) {
                const int a = b + j, z = b + (j + 1) % n;
                cell.points.push_back(c);
                cell.points.push_back(pt(m.cell_xy[2 * a], m.cell_xy[2 * a + 1]));
                cell.points.push_back(pt(m.cell_xy[2 * z], m.cell_xy[2 * z + 1]));
            }
            ma.markers.push_back(cell);
            Marker line = mk("/gvd_voronoi_cell_boundaries", i, Marker::LINE_STRIP, 0.05, 0.0f, 0.0f, 0.0f, 0.8f);
            for (int j = 0; j < n; ++j) line.points.push_back(pt(m.cell_xy[2 * (b + j)], m.cell_xy[2 * (b + j) + 1]));
            line.points.push_back(pt(m.cell_xy[2 * b], m.cell_xy[2 * b + 1]));
            ma.markers.push_back(line);
        }
        // labelled nodes and their texts (:1196-1380): the mask is GvdGraph's node_labels
        static const char *kText[4] = {"TL", "TR", "BL", "BR"};
        static const float kRgb[4][3] = {{0.0f, 1.0f, 1.0f}, {1.0f, 0.5f, 0.0f}, {0.0f, 1.0f, 1.0f}, {1.0f, 0.5f, 0.0f}};
        Marker ln = mk("/gvd_labeled_nodes", 0, Marker::SPHERE_LIST, 0.3, 0.0f, 0.0f, 0.0f, 1.0f);
        int text_id = 0;
        std::vector<Marker> texts;
        for (int i = 0; i < o.num_nodes; ++i) {
            const int mask = o.node_labels[i];
            if (!mask) continue;
            ln.points.push_back(pt(o.nodes_xy[2 * i], o.nodes_xy[2 * i + 1], 0.1));
            float r = 0.0f, gg = 0.0f, bb = 0.0f;
            int cnt = 0;
            for (int k = 0; k < 4; ++k)
                if (mask & (1 << k)) { r += kRgb[k][0]; gg += kRgb[k][1]; bb += kRgb[k][2]; ++cnt; }
            std_msgs::msg::ColorRGBA col;
            col.r = r / cnt; col.g = gg / cnt; col.b = bb / cnt; col.a = 1.0f;
            ln.colors.push_back(col);
            double z_offset = 0.3;
            for (int k = 0; k < 4; ++k) {
                if (!(mask & (1 << k))) continue;
                Marker t = mk("/gvd_node_labels", text_id++, Marker::TEXT_VIEW_FACING, 0.0, kRgb[k][0], kRgb[k][1],
                              kRgb[k][2], 1.0f);
                t.scale.z = 0.5;   // text height only (gvd:1335)
                t.pose.position = pt(o.nodes_xy[2 * i], o.nodes_xy[2 * i + 1], z_offset);
                t.pose.orientation.w = 1.0;
                t.text = kText[k];
                texts.push_back(t);
                z_offset += 0.1;
            }
        }
        if (!ln.points.empty()) ma.markers.push_back(ln);
        ma.markers.insert(ma.markers.end(), texts.begin(), texts.end());
        // cluster endpoints and their TL/TR/BL/BR boundary points (:1382-1591): rows are the
        // (start, end) pairs of /exploration_tree_rows_info, swapped so start.x <= end.x (gvd:130-150)
        for (int i = 0; i < m.n_rows; ++i) {
            double sx = rows_[4 * i], sy = rows_[4 * i + 1], ex = rows_[4 * i + 2], ey = rows_[4 * i + 3];
            if (sx > ex) { std::swap(sx, ex); std::swap(sy, ey); }
            Marker e1 = mk("/gvd_cluster_endpoints", 2 * i, Marker::SPHERE, 0.5, 1.0f, 0.0f, 0.0f, 1.0f);
            e1.pose.position = pt(sx, sy); e1.pose.orientation.w = 1.0;
            Marker e2 = mk("/gvd_cluster_endpoints", 2 * i + 1, Marker::SPHERE, 0.5, 0.0f, 0.0f, 1.0f, 1.0f);
            e2.pose.position = pt(ex, ey); e2.pose.orientation.w = 1.0;
            ma.markers.push_back(e1);
            ma.markers.push_back(e2);
        }
        for (int i = 0; i < m.n_rows; ++i) {
            double ep[2][2] = {{rows_[4 * i], rows_[4 * i + 1]}, {rows_[4 * i + 2], rows_[4 * i + 3]}};
            if (ep[0][0] > ep[1][0]) std::swap(ep[0], ep[1]);
            for (int k = 0; k < 4; ++k) {
                if (!m.row_label_valid[4 * i + k]) continue;
                Marker v = mk(k < 2 ? "/gvd_ep1_voronoi_boundary" : "/gvd_ep2_voronoi_boundary", 4 * i + k, Marker::SPHERE,
                              0.3, kRgb[k][0], kRgb[k][1], kRgb[k][2], 1.0f);
                v.pose.position = pt(m.row_label_xy[8 * i + 2 * k], m.row_label_xy[8 * i + 2 * k + 1]);
                v.pose.orientation.w = 1.0;
                ma.markers.push_back(v);
            }
            for (int e = 0; e < 2; ++e) {
                Marker l = mk(e == 0 ? "/gvd_ep1_voronoi_lines" : "/gvd_ep2_voronoi_lines", 2 * i + e, Marker::LINE_LIST,
                              0.03, 0.0f, 0.8f, 0.8f, 0.7f);
                for (int k = 2 * e; k < 2 * e + 2; ++k) {
                    if (!m.row_label_valid[4 * i + k]) continue;
                    l.points.push_back(pt(ep[e][0], ep[e][1]));
                    l.points.push_back(pt(m.row_label_xy[8 * i + 2 * k], m.row_label_xy[8 * i + 2 * k + 1]));
                }
                if (!l.points.empty()) ma.markers.push_back(l);
            }
        }
        pub_markers_->publish(ma);
    }

    aos_ctx *ctx_ = nullptr;
    double rate_ = 10.0;
    std::chrono::steady_clock::time_point last_ = std::chrono::steady_clock::now();   // gvd:80
    std::vector<double> seeds_, rows_;
    nav_msgs::msg::OccupancyGrid::SharedPtr skel_;
    rclcpp::Subscription<geometry_msgs::msg::PoseArray>::SharedPtr sub_seeds_, sub_rows_;
    rclcpp::Subscription<visualization_msgs::msg::MarkerArray>::SharedPtr sub_all_rows_;
    rclcpp::Subscription<nav_msgs::msg::OccupancyGrid>::SharedPtr sub_skel_;
    rclcpp::Publisher<aos::msg::GvdGraph>::SharedPtr pub_graph_;
    rclcpp::Publisher<visualization_msgs::msg::MarkerArray>::SharedPtr pub_markers_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    rclcpp::spin(std::make_shared<AosGvdGpuNode>());
    rclcpp::shutdown();
    return 0;
}
