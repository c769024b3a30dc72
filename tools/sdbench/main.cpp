#include "subdiv2d.h"
#include <chrono>
#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>
#include <cstring>
int main(int argc, char**argv) {
    FILE *f = fopen("seeds.bin", "rb"); int n; if (fread(&n, 4, 1, f)!=1) return 1;
    std::vector<double> s(2 * n); if (fread(s.data(), 8, 2 * n, f)!=(size_t)2*n) return 1; double b[4]; if (fread(b, 8, 4, f)!=4) return 1; fclose(f);
    float rx = (float)(b[0] - 1.0), ry = (float)(b[2] - 1.0);
    float rw = (float)(std::abs(b[1] - b[0]) + 2.0), rh = (float)(std::abs(b[3] - b[2]) + 2.0);
    double best = 1e9; unsigned long long h = 0;
    for (int rep = 0; rep < 15; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        aos::Subdiv2D sd; sd.reserve(n);
        sd.init_delaunay(rx, ry, rw, rh, 0);
        for (int i = 0; i < n; ++i) {
            float x = (float)s[2 * i], y = (float)s[2 * i + 1];
            x = std::max(rx + 0.1f, std::min(rx + rw - 0.1f, x)); y = std::max(ry + 0.1f, std::min(ry + rh - 0.1f, y));
            sd.insert(x, y);
        }
        auto t1 = std::chrono::steady_clock::now();
        std::vector<float> e; sd.voronoi_edges(e);
        best = std::min(best, std::chrono::duration<double, std::milli>(t1 - t0).count());
        h = 1469598103934665603ull; for (float v : e) { unsigned u; memcpy(&u, &v, 4); h = (h ^ u) * 1099511628211ull; }
    }
    printf("insert best %.2f ms  edges-hash %016llx\n", best, h);
}
