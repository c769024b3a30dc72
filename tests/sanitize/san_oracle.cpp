// Host sanitizer driver (ASan + UBSan, tests/sanitize/Makefile; run by tests/test_sanitize.py).
// Runs the CPU code that has no GPU in it under -fsanitize=address,undefined: the oracle's whole
// path (seed-gen, GVD with the markers' second Subdiv2D, path planning) on the C0 scene, a non-dense
// copy with NaN points and a custom point layout, and empty / tiny clouds; plus the synthetic
// orchard generator it reads. The product's host Subdiv2D is covered by sdcheck built the same way.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../oracle/oracle.h"

extern "C" {
typedef struct orchard_cfg {
    uint64_t seed, n_points;
    int32_t grid_n;
    float res;
    int32_t max_rows;
    double row_x_end, outlier_frac;
} orchard_cfg;
int64_t orchard_num_trees(const orchard_cfg *c);
int64_t orchard_tree_centres(const orchard_cfg *c, double *tree_x, double *tree_y, int64_t cap);
void orchard_polygon(const orchard_cfg *c, double *poly_xy);
void orchard_generate_range(const orchard_cfg *c, const double *tree_x, const double *tree_y, int64_t n_trees,
                            uint64_t begin, uint64_t end, uint8_t *out);
}

static int frame(const char *name, const orc_params &p, const std::vector<uint8_t> &cloud, uint64_t n, uint32_t step,
                 uint32_t ox, uint32_t oy, uint32_t oz, int dense, const double *poly) {
    orc_seedgen_out s;
    std::memset(&s, 0, sizeof(s));
    void *hs = orc_seedgen_run(&p, cloud.data(), n, step, ox, oy, oz, dense, poly, 4, &s);
    if (!hs) { printf("FAIL %s: seed-gen returned null\n", name); return 1; }
    orc_gvd_in gi{s.voronoi_xy, s.n_voronoi, s.rows_info_xy, s.n_rows > 0 ? 2 * s.n_rows : 0,
                  s.origin_x, s.origin_y, s.resolution, s.width, s.height, s.skeleton_framed};
    gi.n_rows_poses = 0;
    for (int i = 0; i < s.n_rows; ++i) gi.n_rows_poses += 2;
    orc_gvd_out g;
    std::memset(&g, 0, sizeof(g));
    void *hg = orc_gvd_run(&p, &gi, &g);
    int paths = 0;
    if (hg && g.num_nodes > 0) {
        orc_path_graph pg{g.num_nodes, g.nodes_xy, g.node_labels, g.node_cluster_indices, g.node_label_counts,
                          g.n_label_entries, g.node_label_clusters, g.node_label_types, g.num_edges, g.edges,
                          g.edge_lengths};
        for (int t = 0; t < 4; ++t) {
            orc_path_query q;
            std::memset(&q, 0, sizeof(q));
            q.target_waypoint_index = t;
            q.previous_waypoint_index = t - 1;
            q.initial_waypoint_reached = t > 0;
            orc_path_out po;
            std::memset(&po, 0, sizeof(po));
            void *hp = orc_path_plan(&pg, s.skeleton_framed, s.origin_x, s.origin_y, s.resolution, s.width, s.height,
                                     &q, &po);
            paths += po.n_poses;
            orc_free_path(hp);
        }
    }
    printf("ok   %-10s n=%-7llu %ux%u T=%d rows=%d seeds=%d nodes=%d edges=%d cells=%d path poses=%d\n", name,
           (unsigned long long)n, s.width, s.height, s.thin_iters, s.n_rows, s.n_voronoi, hg ? g.num_nodes : -1,
           hg ? g.num_edges : -1, hg ? g.n_cells : -1, paths);
    if (hg) orc_free_gvd(hg);
    orc_free_seedgen(hs);
    return 0;
}

int main() {
    orchard_cfg c{1, 100000, 512, 0.2f, 5, 95.0, 0.01};   // tools/orchard.py CONFIGS["C0"]
    const int64_t nt = orchard_num_trees(&c);
    std::vector<double> tx(nt), ty(nt);
    orchard_tree_centres(&c, tx.data(), ty.data(), nt);
    std::vector<uint8_t> cloud(16 * c.n_points);
    orchard_generate_range(&c, tx.data(), ty.data(), nt, 0, c.n_points, cloud.data());
    double poly[8];
    orchard_polygon(&c, poly);
    orc_params p;
    orc_default_params(&p);
    p.grid_resolution = c.res;
    p.markers = 1;
    p.faithful_dead_work = 1;
    int fails = frame("C0", p, cloud, c.n_points, 16, 0, 4, 8, 1, poly);
    // non-dense: 24-byte records (x at 8, y at 0, z at 16), every 97th point NaN
    std::vector<uint8_t> nd(24 * c.n_points, 0);
    for (uint64_t i = 0; i < c.n_points; ++i) {
        float xyz[3];
        std::memcpy(xyz, &cloud[16 * i], 12);
        if (i % 97 == 0) xyz[i % 3] = NAN;
        std::memcpy(&nd[24 * i + 8], &xyz[0], 4);
        std::memcpy(&nd[24 * i + 0], &xyz[1], 4);
        std::memcpy(&nd[24 * i + 16], &xyz[2], 4);
    }
    fails += frame("non-dense", p, nd, c.n_points, 24, 8, 0, 16, 0, poly);
    p.subdiv_rect_mode = 1;
    fails += frame("rect-mode1", p, cloud, c.n_points / 4, 16, 0, 4, 8, 1, poly);
    p.subdiv_rect_mode = 0;
    fails += frame("tiny", p, cloud, 3, 16, 0, 4, 8, 1, poly);
    fails += frame("empty", p, cloud, 0, 16, 0, 4, 8, 1, poly);
    printf("%s\n", fails ? "FAILED" : "all frames ok");
    return fails ? 1 : 0;
}
