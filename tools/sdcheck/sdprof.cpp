// Subdiv2D replay timing on the host CPU: the product's insert path (cavity DFS) over a seed file, best of R
// runs, with the per-phase split (locate walk, cavity DFS, bulk write) when built with -DAOS_SD_PROF, and the
// facet-edge hash (variants must print the same one).
// usage: sdprof seeds.bin [reps]     (seeds.bin: int n, n double pairs, 4 double bounds; as sdcheck)
#include "subdiv2d.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <x86intrin.h>

int main(int argc, char **argv) {
    if (argc < 2) { printf("usage: sdprof seeds.bin [reps]\n"); return 2; }
    const int reps = argc > 2 ? atoi(argv[2]) : 7;
    FILE *f = fopen(argv[1], "rb");
    int n = 0;
    if (!f || fread(&n, 4, 1, f) != 1) { printf("cannot read %s\n", argv[1]); return 2; }
    std::vector<double> s(2 * (size_t)n);
    double b[4];
    if (fread(s.data(), 8, s.size(), f) != s.size() || fread(b, 8, 4, f) != 4) { printf("short %s\n", argv[1]); return 2; }
    fclose(f);
    const float rx = (float)(b[0] - 1.0), ry = (float)(b[2] - 1.0);
    const float rw = (float)(std::abs(b[1] - b[0]) + 2.0), rh = (float)(std::abs(b[3] - b[2]) + 2.0);
    double best = 1e30, best_ticks_per_ms = 0;
    uint64_t hash = 0;
    aos::SdProf bestp{};
    for (int rep = 0; rep < reps; ++rep) {
#ifdef AOS_SD_PROF
        aos::g_sdprof = aos::SdProf{};
#endif
        aos::Subdiv2D sd;
        sd.reserve(n);
        const auto t0 = std::chrono::steady_clock::now();
        const unsigned long long c0 = __rdtsc();
        sd.init_delaunay(rx, ry, rw, rh, 0);
        for (int i = 0; i < n; ++i) {
            float x = (float)s[2 * i], y = (float)s[2 * i + 1];
            x = std::max(rx + 0.1f, std::min(rx + rw - 0.1f, x));
            y = std::max(ry + 0.1f, std::min(ry + rh - 0.1f, y));
            sd.insert(x, y);
        }
        const unsigned long long c1 = __rdtsc();
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms < best) {
            best = ms;
            best_ticks_per_ms = (double)(c1 - c0) / ms;
#ifdef AOS_SD_PROF
            bestp = aos::g_sdprof;
#endif
        }
        std::vector<float> e;
        sd.voronoi_edges(e);
        hash = 1469598103934665603ull;
        for (float v : e) { uint32_t u; memcpy(&u, &v, 4); hash = (hash ^ u) * 1099511628211ull; }
    }
    printf("inserts %d: best %.2f ms of %d; facet-edge hash %016llx", n, best, reps, (unsigned long long)hash);
#ifdef AOS_SD_PROF
    const double k = 1.0 / best_ticks_per_ms;   // ticks -> ms
    printf(" | locate %.2f ms (%.2f steps/insert), dfs %.2f ms (%.2f steps/insert), write %.2f ms, rest %.2f ms",
           bestp.t_locate * k, (double)bestp.loc_iters / n, bestp.t_dfs * k, (double)bestp.dfs_steps / n, bestp.t_write * k,
           best - (bestp.t_locate + bestp.t_dfs + bestp.t_write) * k);
#endif
    printf("\n");
    return 0;
}
