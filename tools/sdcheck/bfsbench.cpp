// BFS-replay timing (the cluster stage's exact replays, cluster_host.cpp) on synthetic row clusters of ~9 k cells:
// the product vs the round-6 form (tools/sdcheck/exp/cluster_host_r06.cpp), one cluster at a time on one thread.
// Env: STRAIGHT=1 rows within two cells of a line (bitmap path), NOROW=1 centres only (no endpoint search).
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
#include <set>
#include <cstdlib>
#include "cluster_geom.h"
#include "cluster_seed.h"
namespace aos_old { void replay_clusters(const std::vector<aos::ReplayJob> &, const aos::GridC &, const double *, int, float, aos::ClusterRec *, aos::HostPool *, std::vector<int> *); }
int main() {
    aos::GridC g{}; g.ox = -10.5; g.oy = 3.25; g.res = 0.1f; g.W = 8192; g.H = 8192; g.WW = 128;
    double poly[8] = {-1e4, -1e4, 1e4, -1e4, 1e4, 1e4, -1e4, 1e4};
    // 64 row-like clusters: a 1-2 cell wide line 8000 cells long with short side branches
    std::mt19937 rng(3);
    std::vector<std::vector<int>> cl;
    for (int c = 0; c < 64; ++c) {
        std::vector<int> v; int y = 100 + c * 120;
        for (int x = 50; x < 8050; ++x) { if (rng() % 5 == 0) y += (rng() % 3) - 1; if (getenv("STRAIGHT")) y = 100 + c * 120 + (rng() % 2); v.push_back(y * g.W + x); if (rng() % 7 == 0) v.push_back((y + 1) * g.W + x); }
        std::set<int> s(v.begin(), v.end()); cl.emplace_back(s.begin(), s.end());
    }
    std::vector<aos::ReplayJob> jobs; for (int c = 0; c < 64; ++c) jobs.push_back({c, cl[c].data(), (int)cl[c].size()});
    std::vector<aos::ClusterRec> a(64), b(64); const float L0 = getenv("NOROW") ? 0.f : 100.f; for (auto &r : a) r.length = L0; for (auto &r : b) r.length = L0;
    for (int rep = 0; rep < 5; ++rep) {
        // one thread each: jobs one at a time
        auto t0 = std::chrono::steady_clock::now();
        for (auto &j : jobs) { std::vector<aos::ReplayJob> one{{0, j.cells, j.n}}; aos::replay_clusters(one, g, poly, 4, 1.f, &a[j.c], nullptr); }
        auto t1 = std::chrono::steady_clock::now();
        for (auto &j : jobs) { std::vector<aos::ReplayJob> one{{0, j.cells, j.n}}; aos_old::replay_clusters(one, g, poly, 4, 1.f, &b[j.c], nullptr, nullptr); }
        auto t2 = std::chrono::steady_clock::now();
        for (int c = 0; c < 64; ++c)
            if (a[c].cx != b[c].cx || a[c].cy != b[c].cy || a[c].start.x != b[c].start.x || a[c].end.y != b[c].end.y || a[c].flags != b[c].flags) {
                printf("MISMATCH cluster %d\n", c); return 1;
            }
        printf("new %.1f us/cluster  old %.1f us/cluster (n ~ %zu)\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 64,
               std::chrono::duration<double, std::micro>(t2 - t1).count() / 64, cl[0].size());
    }
}
