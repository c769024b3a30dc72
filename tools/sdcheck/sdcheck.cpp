// Equivalence checker for aos::Subdiv2D's cavity insert (subdiv2d.h): the same seeds go into two
// instances, one forced onto OpenCV's swap loop, and the complete internal state (rings, end points,
// firstEdge, recentEdge, free lists) must be equal after every insert. Also times both paths.
// usage: sdcheck [seeds.bin]   (seeds.bin: int n, n double pairs, 4 double bounds)
#include "subdiv2d.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static uint64_t sm_state;
static uint64_t splitmix() {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double uni() { return (splitmix() >> 11) * (1.0 / 9007199254740992.0); }

struct Case { const char *name; std::vector<double> s; double b[4]; };

static bool check(const Case &c, bool verbose, bool simd) {
    float rx = (float)(c.b[0] - 1.0), ry = (float)(c.b[2] - 1.0);
    float rw = (float)(std::abs(c.b[1] - c.b[0]) + 2.0), rh = (float)(std::abs(c.b[3] - c.b[2]) + 2.0);
    aos::Subdiv2D a, r;
    a.set_simd(simd);
    r.set_swap_loop(true);
    const int n = (int)c.s.size() / 2;
    a.reserve(n); r.reserve(n);
    a.init_delaunay(rx, ry, rw, rh, 0); r.init_delaunay(rx, ry, rw, rh, 0);
    for (int i = 0; i < n; ++i) {
        float x = (float)c.s[2 * i], y = (float)c.s[2 * i + 1];
        x = std::max(rx + 0.1f, std::min(rx + rw - 0.1f, x)); y = std::max(ry + 0.1f, std::min(ry + rh - 0.1f, y));
        const bool ka = a.insert(x, y), kr = r.insert(x, y);
        if (ka != kr || !a.same_state(r)) {
            printf("FAIL %s: state differs after insert %d of %d (%.9g, %.9g)\n", c.name, i, n, x, y);
            return false;
        }
    }
    std::vector<float> ea, er;
    a.voronoi_edges(ea); r.voronoi_edges(er);
    if (ea.size() != er.size() || memcmp(ea.data(), er.data(), ea.size() * 4)) {
        printf("FAIL %s: facet edges differ\n", c.name);
        return false;
    }
    if (verbose) printf("ok   %-22s n=%-7d cavity inserts %ld, swap-loop inserts %ld\n", c.name, n, a.n_cavity, a.n_loop);
    return true;
}

static double time_inserts(const Case &c, bool loop, bool simd, uint64_t &hash) {
    float rx = (float)(c.b[0] - 1.0), ry = (float)(c.b[2] - 1.0);
    float rw = (float)(std::abs(c.b[1] - c.b[0]) + 2.0), rh = (float)(std::abs(c.b[3] - c.b[2]) + 2.0);
    const int n = (int)c.s.size() / 2;
    double best = 1e30;
    for (int rep = 0; rep < 7; ++rep) {
        aos::Subdiv2D sd;
        sd.set_swap_loop(loop);
        sd.set_simd(simd);
        sd.reserve(n);
        auto t0 = std::chrono::steady_clock::now();
        sd.init_delaunay(rx, ry, rw, rh, 0);
        for (int i = 0; i < n; ++i) {
            float x = (float)c.s[2 * i], y = (float)c.s[2 * i + 1];
            x = std::max(rx + 0.1f, std::min(rx + rw - 0.1f, x)); y = std::max(ry + 0.1f, std::min(ry + rh - 0.1f, y));
            sd.insert(x, y);
        }
        auto t1 = std::chrono::steady_clock::now();
        best = std::min(best, std::chrono::duration<double, std::milli>(t1 - t0).count());
        std::vector<float> e;
        sd.voronoi_edges(e);
        hash = 1469598103934665603ull;
        for (float v : e) { uint32_t u; memcpy(&u, &v, 4); hash = (hash ^ u) * 1099511628211ull; }
    }
    return best;
}

int main(int argc, char **argv) {
    std::vector<Case> cases;
    // random uniform, lattices (co-circular everywhere), lattice rows in row-by-row order (orchard-like),
    // jittered lattices, duplicates / near-duplicates, collinear runs, tiny clusters
    const char *reps_env = getenv("AOS_SDCHECK_REPS");   // (the sanitizer build runs a few repetitions)
    const int reps = reps_env ? atoi(reps_env) : 40;
    for (int rep = 0; rep < reps; ++rep) {
        sm_state = 1000 + rep;
        Case u{"uniform", {}, {0, 50, 0, 50}};
        const int n = 200 + (int)(uni() * 3000);
        for (int i = 0; i < n; ++i) { u.s.push_back(uni() * 50); u.s.push_back(uni() * 50); }
        cases.push_back(u);
        Case g{"lattice", {}, {0, 30, 0, 30}};
        const double sp = 0.25 + uni();
        for (double y = 0; y <= 30; y += sp) for (double x = 0; x <= 30; x += sp) { g.s.push_back(x); g.s.push_back(y); }
        cases.push_back(g);
        Case o{"orchard-rows", {}, {0, 120, 0, 60}};
        const double dx = 0.3 + 0.7 * uni(), dy = 1.5 + 2.5 * uni();
        for (double y = 1; y < 60; y += dy) {
            const bool rev = uni() < 0.5;
            for (double x0 = 1; x0 < 119; x0 += dx) {
                const double x = rev ? 120 - x0 : x0;
                o.s.push_back(x + (uni() < 0.2 ? 0.05 * (uni() - 0.5) : 0)); o.s.push_back(y + (uni() < 0.3 ? 0.3 * (uni() - 0.5) : 0));
                if (uni() < 0.3) { o.s.push_back(x); o.s.push_back(y + dy * 0.5); }
            }
        }
        cases.push_back(o);
        Case j{"jitter-lattice", {}, {0, 40, 0, 40}};
        for (double y = 0; y <= 40; y += 0.5) for (double x = 0; x <= 40; x += 0.5) {
            j.s.push_back(x + 1e-6 * (uni() - 0.5)); j.s.push_back(y + 1e-6 * (uni() - 0.5));
        }
        cases.push_back(j);
        Case d{"dups-collinear", {}, {0, 20, 0, 20}};
        for (int i = 0; i < 1500; ++i) {
            const double r = uni();
            if (r < 0.2 && d.s.size() >= 2) { size_t k = 2 * (size_t)(uni() * (d.s.size() / 2)); d.s.push_back(d.s[k] + (uni() < 0.5 ? 0 : 1e-7)); d.s.push_back(d.s[k + 1]); }
            else if (r < 0.5) { d.s.push_back(uni() * 20); d.s.push_back(10.0); }
            else if (r < 0.6) { const double t = uni() * 20; d.s.push_back(t); d.s.push_back(t); }
            else { d.s.push_back(uni() * 20); d.s.push_back(uni() * 20); }
        }
        cases.push_back(d);
        Case c{"clamped-border", {}, {0, 10, 0, 10}};
        for (int i = 0; i < 800; ++i) { c.s.push_back(uni() * 14 - 2); c.s.push_back(uni() * 14 - 2); }
        cases.push_back(c);
    }
    Case file{"seeds.bin", {}, {0, 0, 0, 0}};
    const char *path = argc > 1 ? argv[1] : nullptr;
    if (path) {
        FILE *f = fopen(path, "rb");
        int n = 0;
        if (!f || fread(&n, 4, 1, f) != 1) { printf("cannot read %s\n", path); return 2; }
        file.s.resize(2 * (size_t)n);
        if (fread(file.s.data(), 8, 2 * (size_t)n, f) != 2 * (size_t)n || fread(file.b, 8, 4, f) != 4) { printf("short %s\n", path); return 2; }
        fclose(f);
        cases.push_back(file);
    }
    int fails = 0;
    const bool simd = aos::Subdiv2D::simd_ok();
    for (int pass = 0; pass < (simd ? 2 : 1); ++pass) {
        for (size_t i = 0; i < cases.size(); ++i) fails += !check(cases[i], pass == 0 && (i < 6 || i + 1 == cases.size()), pass == 0 && simd);
        printf("%zu cases (%s flip tests), %d failed so far\n", cases.size(), pass == 0 && simd ? "AVX2" : "scalar", fails);
    }
    if (path) {
        uint64_t ha = 0, hs = 0, hr = 0;
        const double ta = time_inserts(file, false, simd, ha), ts = time_inserts(file, false, false, hs),
                     tr = time_inserts(file, true, false, hr);
        printf("%s inserts: cavity+%s %.2f ms, cavity+scalar %.2f ms, swap loop %.2f ms (x%.2f); facet-edge hash %016llx %s\n",
               path, simd ? "AVX2" : "scalar", ta, ts, tr, tr / ta, (unsigned long long)ha,
               ha == hr && hs == hr ? "equal" : "DIFFERENT");
        if (ha != hr || hs != hr) fails++;
    }
    return fails ? 1 : 0;
}
