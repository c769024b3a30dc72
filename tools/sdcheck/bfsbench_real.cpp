// Exact BFS replay timing (cluster_host.cpp) on real skeleton clusters (tools/sdcheck/dump_clusters.py: the oracle's C1
// row clusters), one cluster at a time on one thread: bfs_order alone, then the whole replay with the endpoint search.
// Built against the product file and against exp/cluster_host_r06.cpp by bfs_real.sh.
#include "cluster_host.cpp"
#include <chrono>
#include <cstdio>
using namespace aos;
int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb"); int hdr[3]; fread(hdr, 4, 3, f);
    GridC g{}; g.ox = -10.5; g.oy = 3.25; g.res = 0.1f; g.W = hdr[0]; g.H = hdr[1]; g.WW = (hdr[0] + 63) / 64;
    std::vector<std::vector<int>> cl(hdr[2]);
    for (auto &v : cl) { int n; fread(&n, 4, 1, f); v.resize(n); fread(v.data(), 4, n, f); }
    std::vector<XY> q; std::vector<int> tab; std::vector<uint64_t> bm;
    double poly[8] = {-1e4, -1e4, 1e4, -1e4, 1e4, 1e4, -1e4, 1e4};
    size_t tot = 0; for (auto &v : cl) tot += v.size();
    for (int rep = 0; rep < 5; ++rep) {
        float sx, sy; double acc = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (auto &v : cl) { bfs_order(v.data(), (int)v.size(), g, q, tab, bm, sx, sy); acc += sx + sy; }
        auto t1 = std::chrono::steady_clock::now();
        for (auto &v : cl) { ClusterRec r{}; r.length = 100.f; host_bfs_replay(v.data(), nullptr, (int)v.size(), g, poly, 4, 1.f, r, q, tab, bm); acc += r.start.x + r.end.y + r.cx; }
        auto t2 = std::chrono::steady_clock::now();
        printf("order %.2f ns/cell  replay(row) %.2f ns/cell  check %.17g\n", std::chrono::duration<double, std::nano>(t1 - t0).count() / tot,
               std::chrono::duration<double, std::nano>(t2 - t1).count() / tot, acc);
    }
}
