// Drop-in rclcpp node for aos_seed_gen_node's hot path on MI355X.
// Same node name, parameter names/defaults, topics and QoS as src/aos_seed_gen_node.cpp:60-190;
// the computation is libaos_gpu.so (include/aos_gpu.h). Visualisation-only MarkerArrays are out of
// scope except /tree_rows_all, which the GVD node uses as a trigger (gvd:361-373).
//
// Not built in this repository's image (no ROS 2); see INTEGRATION.md for the ament recipe.
#include <geometry_msgs/msg/polygon_stamped.hpp>
#include <geometry_msgs/msg/pose_array.hpp>
#include <nav_msgs/msg/occupancy_grid.hpp>
#include <rclcpp/rclcpp.hpp>
#include <sensor_msgs/msg/point_cloud2.hpp>
#include <visualization_msgs/msg/marker_array.hpp>

#include <cstring>
#include <stdexcept>
#include <string>

#include "aos_gpu.h"

namespace {

uint32_t field_offset(const sensor_msgs::msg::PointCloud2 &m, const char *name) {
    for (const auto &f : m.fields)
        if (f.name == name && f.datatype == sensor_msgs::msg::PointField::FLOAT32) return f.offset;
    throw std::runtime_error(std::string("PointCloud2 has no float32 field ") + name);
}

// header and info of a published grid; the data vector is sized here and filled by aos_seedgen_grids_copy
// straight from HBM (no intermediate host copy)
void grid_header(nav_msgs::msg::OccupancyGrid &g, const aos_grid_info &info, const rclcpp::Time &t) {
    g.header.frame_id = "map";   // seed_gen:542-576
    g.header.stamp = t;
    g.info.resolution = info.resolution;
    g.info.width = info.width;
    g.info.height = info.height;
    g.info.origin.position.x = info.origin_x;
    g.info.origin.position.y = info.origin_y;
    g.info.origin.orientation.w = 1.0;
    g.data.resize((size_t)info.width * info.height);
}

geometry_msgs::msg::PoseArray poses(const double *xy, int n, const rclcpp::Time &t) {
    geometry_msgs::msg::PoseArray pa;
    pa.header.frame_id = "map";
    pa.header.stamp = t;
    pa.poses.resize(n);
    for (int i = 0; i < n; ++i) {
        pa.poses[i].position.x = xy[2 * i];
        pa.poses[i].position.y = xy[2 * i + 1];
        pa.poses[i].orientation.w = 1.0;
    }
    return pa;
}

}  // namespace

class AosSeedGenGpuNode : public rclcpp::Node {
  public:
    AosSeedGenGpuNode() : Node("aos_seed_gen_node") {
        aos_params p;
        aos_default_params(&p);
        // seed_gen:69-100 (same names and defaults)
        p.clipping_minz = declare_parameter<float>("clipping_minz", -0.4);
        p.clipping_maxz = declare_parameter<float>("clipping_maxz", 0.5);
        p.clipping_minx = declare_parameter<float>("clipping_minx", -5.0);
        p.clipping_maxx = declare_parameter<float>("clipping_maxx", 72.0);
        p.clipping_miny = declare_parameter<float>("clipping_miny", -10.0);
        p.clipping_maxy = declare_parameter<float>("clipping_maxy", 20.0);
        p.grid_resolution = declare_parameter<float>("grid_resolution", 0.05);
        p.inflation_radius = declare_parameter<float>("inflation_radius", 0.8);
        p.cluster_min_length = declare_parameter<double>("cluster_min_length", 2.0);
        const int device = declare_parameter<int>("gpu_device", 0);
        if (aos_create(&p, device, &ctx_) != AOS_OK) throw std::runtime_error(aos_last_error());

        rclcpp::QoS reliable(10);   // seed_gen:120-123
        reliable.reliable().durability(rclcpp::DurabilityPolicy::TransientLocal).history(rclcpp::HistoryPolicy::KeepLast);
        pub_occ_ = create_publisher<nav_msgs::msg::OccupancyGrid>("occupancy_grid", reliable);
        pub_skel_ = create_publisher<nav_msgs::msg::OccupancyGrid>("skeletonized_occupancy_grid", reliable);
        pub_cluster_info_ = create_publisher<geometry_msgs::msg::PoseArray>("cluster_info", reliable);
        pub_seeds_ = create_publisher<geometry_msgs::msg::PoseArray>("voronoi_seeds", reliable);
        pub_rows_info_ = create_publisher<geometry_msgs::msg::PoseArray>("exploration_tree_rows_info", reliable);
        pub_rows_all_ = create_publisher<visualization_msgs::msg::MarkerArray>("tree_rows_all", reliable);

        const auto map_topic = declare_parameter<std::string>("global_map_topic", "/lio_sam/mapping/global_map");
        const auto area_topic = declare_parameter<std::string>("exploration_area_topic", "/aos_planner/exploration_area");
        declare_parameter<std::string>("robot_position_topic", "/Local/utm");   // no effect on outputs
        sub_map_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            map_topic, 10, [this](sensor_msgs::msg::PointCloud2::SharedPtr m) { on_map(*m); });
        sub_area_ = create_subscription<geometry_msgs::msg::PolygonStamped>(
            area_topic, 10, [this](geometry_msgs::msg::PolygonStamped::SharedPtr m) { on_area(*m); });
    }
    ~AosSeedGenGpuNode() override { aos_destroy(ctx_); }

  private:
    // globalMapCallback seed_gen:230-248
    void on_map(const sensor_msgs::msg::PointCloud2 &m) {
        aos_cloud_view v{};
        v.data = m.data.data();
        v.n_points = (uint64_t)m.width * m.height;
        v.point_step = m.point_step;
        v.off_x = field_offset(m, "x");
        v.off_y = field_offset(m, "y");
        v.off_z = field_offset(m, "z");
        v.is_dense = m.is_dense;
        v.on_device = 0;
        aos_seedgen_out out{};
        if (aos_seedgen_process(ctx_, &v, 0, &out) != AOS_OK) {   // grids: aos_seedgen_grids_copy in publish()
            RCLCPP_ERROR(get_logger(), "seed gen failed: %s", aos_last_error());
            return;
        }
        publish(out);
    }
    // explorationAreaCallback seed_gen:250-286: new polygon (>= 3 points) -> reprocess the last cloud
    void on_area(const geometry_msgs::msg::PolygonStamped &m) {
        std::vector<double> xy;
        for (const auto &p : m.polygon.points) { xy.push_back(p.x); xy.push_back(p.y); }
        if (aos_set_polygon(ctx_, xy.data(), (uint32_t)m.polygon.points.size()) != AOS_OK) return;
        aos_seedgen_out out{};
        const int rc = aos_seedgen_reprocess(ctx_, 0, &out);
        if (rc == AOS_OK) publish(out);
        else if (rc != AOS_E_STATE) RCLCPP_ERROR(get_logger(), "reprocess failed: %s", aos_last_error());
    }
    void publish(const aos_seedgen_out &o) {
        const rclcpp::Time t = now();
        nav_msgs::msg::OccupancyGrid occ, skel;
        grid_header(occ, o.info, t);
        grid_header(skel, o.info, t);
        if (aos_seedgen_grids_copy(ctx_, occ.data.data(), skel.data.data()) != AOS_OK) {
            RCLCPP_ERROR(get_logger(), "grid copy failed: %s", aos_last_error());
            return;
        }
        pub_occ_->publish(occ);
        pub_skel_->publish(skel);
        pub_cluster_info_->publish(poses(o.cluster_info_xy, o.n_cluster_info, t));
        visualization_msgs::msg::MarkerArray rows;   // publishTreeRowsAllFromClusters :1567-1611
        visualization_msgs::msg::Marker del;
        del.header.frame_id = "map"; del.header.stamp = t;
        del.action = visualization_msgs::msg::Marker::DELETEALL;
        rows.markers.push_back(del);
        for (int i = 0; i < o.n_rows; ++i) {
            visualization_msgs::msg::Marker l;
            l.header = del.header; l.ns = "tree_rows_all"; l.id = i;
            l.type = visualization_msgs::msg::Marker::LINE_STRIP;
            l.action = visualization_msgs::msg::Marker::ADD;
            l.pose.orientation.w = 1.0; l.scale.x = 0.1; l.color.a = 1.0; l.color.g = 1.0;
            geometry_msgs::msg::Point a, b;
            a.x = o.row_start[2 * i]; a.y = o.row_start[2 * i + 1];
            b.x = o.row_end[2 * i]; b.y = o.row_end[2 * i + 1];
            l.points = {a, b};
            rows.markers.push_back(l);
        }
        pub_rows_all_->publish(rows);
        pub_seeds_->publish(poses(o.voronoi_xy, o.n_voronoi, t));
        pub_rows_info_->publish(poses(o.rows_info_xy, 2 * o.n_rows, t));
    }

    aos_ctx *ctx_ = nullptr;
    rclcpp::Publisher<nav_msgs::msg::OccupancyGrid>::SharedPtr pub_occ_, pub_skel_;
    rclcpp::Publisher<geometry_msgs::msg::PoseArray>::SharedPtr pub_cluster_info_, pub_seeds_, pub_rows_info_;
    rclcpp::Publisher<visualization_msgs::msg::MarkerArray>::SharedPtr pub_rows_all_;
    rclcpp::Subscription<sensor_msgs::msg::PointCloud2>::SharedPtr sub_map_;
    rclcpp::Subscription<geometry_msgs::msg::PolygonStamped>::SharedPtr sub_area_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    rclcpp::spin(std::make_shared<AosSeedGenGpuNode>());
    rclcpp::shutdown();
    return 0;
}
