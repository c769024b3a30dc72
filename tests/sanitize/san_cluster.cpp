// ASan/UBSan driver of the product's host cluster code (active-orchard-slam_amd/csrc/cluster_host.cpp:
// cluster_union, replay_clusters, assemble_rows), built by tests/sanitize/Makefile and run by
// tests/test_sanitize.py on inputs the test writes (binary, little endian):
//   san_cluster U <in> <out>   in: W H n_pieces piece_root[] n_border bcell[] broot[] (int32)
//                              out: n_clusters piece_cluster[] (int32)
//   san_cluster R <in> <out>   in: ox oy (f64) res (f32) W H np (i32) poly[2 np] (f64) min_len (f32) n_clusters (i32),
//                                  then per cluster: n (i32) length (f32) cells[n] (i32, any order)
//                              out: per cluster flags (i32) cx cy (f32) center start end (f64 x 2 each);
//                                   then n_rows (i32) rows_info[4 n_rows] cluster_info[2 n_rows] (f64)
//   san_cluster B <in> <out>   in: as R, then n_extra (i32) extra[n_extra] (i32: skeleton cells outside every cluster)
//                              the replays walk a skeleton bit grid (every cluster's cells + the extra cells) over
//                              each cluster's box from its first cell; the ones that fail replay from their cells
//                              out: as R, then n_failed (i32)
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "cluster_geom.h"
#include "cluster_seed.h"

namespace {
struct In {
    FILE *f;
    template <class T> T get() {
        T v;
        if (fread(&v, sizeof(T), 1, f) != 1) throw std::runtime_error("short input");
        return v;
    }
    template <class T> std::vector<T> vec(size_t n) {
        std::vector<T> v(n);
        if (n && fread(v.data(), sizeof(T), n, f) != n) throw std::runtime_error("short input");
        return v;
    }
};
template <class T> void put(FILE *f, const T &v) { fwrite(&v, sizeof(T), 1, f); }
template <class T> void put(FILE *f, const std::vector<T> &v) { if (!v.empty()) fwrite(v.data(), sizeof(T), v.size(), f); }
}  // namespace

int main(int argc, char **argv) {
    if (argc != 4) { fprintf(stderr, "usage: san_cluster U|R in out\n"); return 2; }
    FILE *fi = fopen(argv[2], "rb"), *fo = fopen(argv[3], "wb");
    if (!fi || !fo) { fprintf(stderr, "cannot open files\n"); return 2; }
    In in{fi};
    const std::string mode = argv[1];
    if (mode == "U") {
        const int W = in.get<int32_t>(), H = in.get<int32_t>(), np = in.get<int32_t>();
        const std::vector<int32_t> root = in.vec<int32_t>(np);
        const int nb = in.get<int32_t>();
        const std::vector<int32_t> bcell = in.vec<int32_t>(nb), broot = in.vec<int32_t>(nb);
        std::vector<int32_t> pc(np);
        const int ncl = aos::cluster_union(W, H, np, root.data(), nb, bcell.data(), broot.data(), pc.data());
        put(fo, (int32_t)ncl);
        put(fo, pc);
    } else if (mode == "R" || mode == "B") {
        aos::GridC g{};
        g.ox = in.get<double>(); g.oy = in.get<double>(); g.res = in.get<float>();
        g.W = in.get<int32_t>(); g.H = in.get<int32_t>();
        g.WW = (g.W + 63) / 64;
        const int np = in.get<int32_t>();
        const std::vector<double> poly = in.vec<double>(2 * (size_t)np);
        const float min_len = in.get<float>();
        const int ncl = in.get<int32_t>();
        std::vector<std::vector<int32_t>> cells(ncl);
        std::vector<aos::ClusterRec> rec(ncl);
        std::vector<aos::ReplayJob> jobs;
        for (int c = 0; c < ncl; ++c) {
            const int n = in.get<int32_t>();
            rec[c].n = n;
            rec[c].length = in.get<float>();
            cells[c] = in.vec<int32_t>(n);
        }
        int n_failed = 0;
        if (mode == "B") {
            const int nx = in.get<int32_t>();
            const std::vector<int32_t> extra = in.vec<int32_t>(nx);
            std::vector<uint64_t> bits((size_t)g.WW * g.H, 0ull);
            auto set = [&](int p) { const int y = p / g.W, x = p - y * g.W; bits[(size_t)y * g.WW + x / 64] |= 1ull << (x % 64); };
            for (int c = 0; c < ncl; ++c) {
                aos::ClusterRec &r = rec[c];
                r.bx0 = r.by0 = INT32_MAX; r.bx1 = r.by1 = -1; r.first = INT32_MAX;
                for (int p : cells[c]) {
                    set(p);
                    const int y = p / g.W, x = p - y * g.W;
                    r.bx0 = std::min(r.bx0, x); r.bx1 = std::max(r.bx1, x);
                    r.by0 = std::min(r.by0, y); r.by1 = std::max(r.by1, y);
                    r.first = std::min(r.first, p);
                }
            }
            for (int p : extra) set(p);
            for (int c = 0; c < ncl; ++c) jobs.push_back({c, nullptr, (int)cells[c].size(), bits.data()});
            std::vector<int> failed;
            aos::replay_clusters(jobs, g, poly.data(), np, min_len, rec.data(), nullptr, &failed);
            n_failed = (int)failed.size();
            jobs.clear();
            for (int i : failed) jobs.push_back({i, cells[i].data(), (int)cells[i].size()});
        } else {
            for (int c = 0; c < ncl; ++c) jobs.push_back({c, cells[c].data(), (int)cells[c].size()});
        }
        aos::replay_clusters(jobs, g, poly.data(), np, min_len, rec.data());
        for (const auto &r : rec) {
            put(fo, (int32_t)r.flags); put(fo, r.cx); put(fo, r.cy);
            for (const double2 &d : {r.center, r.start, r.end}) { put(fo, d.x); put(fo, d.y); }
        }
        aos::SeedStageOut so;
        std::vector<aos::RowDev> rows;
        aos::assemble_rows(rec, so, rows);
        put(fo, (int32_t)rows.size());
        put(fo, so.rows_info);
        put(fo, so.cluster_info);
        if (mode == "B") put(fo, (int32_t)n_failed);
    } else {
        fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    fclose(fi);
    fclose(fo);
    printf("san_cluster %s ok\n", mode.c_str());
    return 0;
}
