// Drop-in rclcpp node for aos_gvd_node's graph build on MI355X.
// Same parameters, topics and QoS as src/aos_gvd_node.cpp:26-78; processGraph (gvd:255-318) is
// aos_gvd_process on the latest inputs. The throttle (max_graph_publish_rate, gvd:306-314) stays
// here. The reference computes the graph even when the throttle suppresses publishing; the graph
// is then unobservable, so this node skips that work. /gvd/markers (publishMarkers) is out of scope.
//
// Not built in this repository's image (no ROS 2); see INTEGRATION.md for the ament recipe.
#include <geometry_msgs/msg/pose_array.hpp>
#include <nav_msgs/msg/occupancy_grid.hpp>
#include <rclcpp/rclcpp.hpp>
#include <visualization_msgs/msg/marker_array.hpp>

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
    }
    ~AosGvdGpuNode() override { aos_destroy(ctx_); }

  private:
    void process() {
        if (seeds_.empty() || !skel_) return;   // gvd:257-259
        const auto now = std::chrono::steady_clock::now();
        if (std::chrono::duration<double>(now - last_).count() < 1.0 / rate_) return;
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
        last_ = now;
    }

    aos_ctx *ctx_ = nullptr;
    double rate_ = 10.0;
    std::chrono::steady_clock::time_point last_{};
    std::vector<double> seeds_, rows_;
    nav_msgs::msg::OccupancyGrid::SharedPtr skel_;
    rclcpp::Subscription<geometry_msgs::msg::PoseArray>::SharedPtr sub_seeds_, sub_rows_;
    rclcpp::Subscription<visualization_msgs::msg::MarkerArray>::SharedPtr sub_all_rows_;
    rclcpp::Subscription<nav_msgs::msg::OccupancyGrid>::SharedPtr sub_skel_;
    rclcpp::Publisher<aos::msg::GvdGraph>::SharedPtr pub_graph_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    rclcpp::spin(std::make_shared<AosGvdGpuNode>());
    rclcpp::shutdown();
    return 0;
}
