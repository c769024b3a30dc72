// Round-6 form of active-orchard-slam_amd/csrc/cluster_host.cpp (namespace aos_old), kept for tools/sdcheck/bfsbench.cpp A/B only.
// Host-side parts of the cluster stage (a8-a10), kept in a plain C++ file so the sanitizer build
// (tests/sanitize: ASan + UBSan, no GPU) runs exactly the code the product links:
//   * host_bfs_replay / replay_clusters: clusterOccupiedCells' FIFO BFS (seed_gen:1007-1049) and its
//     order-dependent statistics, for the clusters without the GPU's order-free certificate;
//   * cluster_union: the border union-find of the tiled frame's distributed cluster stage (aos_cluster_union);
//   * assemble_rows: convertClustersToTreeRows' row arrays (seed_gen:1329-1406) and the std::sort-ed
//     cluster_info / rows_info outputs (seed_gen:1515-1565, 2546-2582).
#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <thread>
#include <unordered_map>
#include <vector>

#include "cluster_geom.h"
#include "cluster_seed.h"

namespace aos_old { using namespace aos;

constexpr int kReplayThreads = 16;   // host threads for the exact BFS replays of one frame (the box share: 16 cores)



// ------------------------------------------------------------------ exact BFS replay
// clusterOccupiedCells' FIFO BFS (seed_gen:1007-1049) and the order-dependent statistics that follow
// (float centre sums :1030-1046, first-strict-maximum endpoints :1354-1395) for the rare clusters
// without the order-free certificate. This is a serial chain of dependent steps: it runs on the host
// core next to the GPU (the cluster's cells come over in raster order), ~10 ns per step.
// Raster id -> (x, y) without an integer division per cell (~25 cycles each; round 4's replay divided 5-6 times per
// cell): the double quotient is within a few ulps of p / W, so its truncation is the quotient or one off.
struct DivW {
    int W; double inv;
    explicit DivW(int w) : W(w), inv(1.0 / (double)w) {}
    void xy(int p, int &x, int &y) const {
        long long q = (long long)((double)p * inv);
        if (q * W > p) --q; else if ((q + 1) * W <= p) ++q;
        y = (int)q; x = p - (int)q * W;
    }
};
struct XY { int x, y; };

// The FIFO BFS over the cluster's cells from its smallest (first raster) cell, into q as (x, y). Membership and the
// visited marks live in a bitmap over the cluster's bounding box when that box is small against n (row clusters: a
// few cells wide), else in an open-addressing hash of the cells: the same order either way.
// Round 5: the bitmap has a zero border of one cell, so a popped cell reads its 3 x 3 neighbourhood as three 3-bit
// fields (unaligned 64-bit loads of a byte array) into one mask in the reference's neighbour order, and walks only the
// set bits; the queue holds (x, y), so no division at all (C3's ~450 replays: profiles/r05y_*).
static const int kDxs[8] = {-1, -1, -1, 0, 0, 1, 1, 1}, kDys[8] = {-1, 0, 1, -1, 1, -1, 0, 1};

// The FIFO walk over a bordered box bitmap B (RW words per row; a set bit = in the cluster, not yet queued; bit c of
// row r = cell (x0 + c - 1, y0 + r - 1)) from (sx, sy), whose bit is already clear. Q receives the cells in pop
// order; at most cap of them (returns -1 past it), else their number. The centre sums ride along in pop order (the
// float additions of seed_gen:1030-1046 in the same order).
static long long bfs_walk(uint64_t *B, long long RW, int x0, int y0, int sx, int sy, XY *Q, long long cap, float &sum_x,
                          float &sum_y) {
    auto win3 = [&](long long r, long long c) {   // bits c, c + 1, c + 2 of row r (c >= 0: the border)
        const uint64_t *w = B + r * RW + (c >> 6);
        const unsigned __int128 v = ((unsigned __int128)w[1] << 64) | w[0];
        return (unsigned)(v >> (c & 63)) & 7u;
    };
    Q[0] = XY{sx, sy};
    long long head = 0, tail = 1;
    float ax = 0.0f, ay = 0.0f;
    while (head < tail) {
        const XY c = Q[head++];
        ax += (float)c.x; ay += (float)c.y;
        const long long r = c.y - y0 + 1, cc = c.x - x0 + 1;
        const unsigned rm = win3(r - 1, cc - 1), r0 = win3(r, cc - 1), rp = win3(r + 1, cc - 1);
        // the neighbour order (dx, dy) of kDxs / kDys: column x - 1 (rows y - 1, y, y + 1), column x (y - 1, y + 1),
        // column x + 1 (y - 1, y, y + 1)
        unsigned m = (rm & 1u) | (r0 & 1u) << 1 | (rp & 1u) << 2 | (rm & 2u) << 2 | (rp & 2u) << 3 | (rm & 4u) << 3 |
                     (r0 & 4u) << 4 | (rp & 4u) << 5;
        while (m) {
            const int i = __builtin_ctz(m);
            m &= m - 1;
            const long long nr = r + kDys[i], nc = cc + kDxs[i];
            B[nr * RW + (nc >> 6)] &= ~(1ull << (nc & 63));
            if (tail >= cap) return -1;
            Q[tail++] = XY{c.x + kDxs[i], c.y + kDys[i]};
        }
    }
    sum_x = ax; sum_y = ay;
    return tail;
}

static void bfs_order(const int *cells, int n, const GridC &g, std::vector<XY> &q, std::vector<int> &tab,
                      std::vector<uint64_t> &bm, float &sum_x, float &sum_y) {
    static const int *const dxs = kDxs, *const dys = kDys;
    const DivW dw(g.W);
    q.resize(n);
    // the cells' (x, y) go to the queue's storage first: the bitmap pass below reads them back instead of dividing again
    XY *const Q = q.data();
    int start = cells[0], x0 = INT_MAX, x1 = INT_MIN, y0 = INT_MAX, y1 = INT_MIN;
    for (int k = 0; k < n; ++k) {
        const int p = cells[k];
        int x, y;
        dw.xy(p, x, y);
        Q[k] = XY{x, y};
        start = std::min(start, p);
        x0 = std::min(x0, x); x1 = std::max(x1, x); y0 = std::min(y0, y); y1 = std::max(y1, y);
    }
    int sx, sy;
    dw.xy(start, sx, sy);
    const long long bw = (long long)x1 - x0 + 1, area = bw * ((long long)y1 - y0 + 1);
    static const bool force_hash = [] { const char *e = getenv("AOS_REPLAY_HASH"); return e && atoi(e) != 0; }();
    if (!force_hash && area <= std::max<long long>(64ll * n, 1 << 16)) {   // (AOS_REPLAY_HASH=1: tests)
        // rows of RW 64-bit words over the box plus a one-cell zero border (and one spare word per row, so a 3-bit
        // window is always inside two words); a set bit = in the cluster, not yet queued. Every access is an aligned
        // 64-bit word: a queued cell's bit is cleared by a word store that later word loads of the same address read
        // forwarded (round-5 first form: byte stores under unaligned 8-byte loads, which wait for the stores to retire).
        const long long pw = bw + 2, ph = (long long)y1 - y0 + 3;
        const long long RW = (pw + 63) / 64 + 1;
        bm.assign((size_t)(RW * ph), 0ull);
        uint64_t *B = bm.data();
        auto setb = [&](long long r, long long c) { B[r * RW + (c >> 6)] |= 1ull << (c & 63); };
        for (int k = 0; k < n; ++k) setb(Q[k].y - y0 + 1, Q[k].x - x0 + 1);
        {
            const long long r = sy - y0 + 1, c = sx - x0 + 1;
            B[r * RW + (c >> 6)] &= ~(1ull << (c & 63));
        }
        const long long tail = bfs_walk(B, RW, x0, y0, sx, sy, Q, n, sum_x, sum_y);
        if (tail != n) throw std::runtime_error("BFS replay: cluster is not 8-connected (or its cells repeat)");
        return;
    }
    int cap = 64;
    while (cap < 2 * n) cap <<= 1;
    const unsigned mask = (unsigned)cap - 1;
    tab.assign(cap, -1);
    auto slot_of = [&](int key) -> int {   // key present -> its slot, else -1
        unsigned h = ((unsigned)key * 2654435761u) & mask;
        for (;;) {
            int v = tab[h];
            if (v == -1) return -1;
            if ((v & 0x7fffffff) == key) return (int)h;
            h = (h + 1) & mask;
        }
    };
    for (int k = 0; k < n; ++k) {
        unsigned h = ((unsigned)cells[k] * 2654435761u) & mask;
        while (tab[h] != -1) h = (h + 1) & mask;
        tab[h] = cells[k];
    }
    tab[slot_of(start)] |= (int)0x80000000;   // (start: the first raster cell; the cells come in any order)
    q[0] = XY{sx, sy};
    int head = 0, tail = 1;
    while (head < tail) {
        const XY c = q[head++];
        for (int i = 0; i < 8; ++i) {
            const int nx = c.x + dxs[i], ny = c.y + dys[i];
            if (nx < 0 || nx >= g.W || ny < 0 || ny >= g.H) continue;
            const int h = slot_of(ny * g.W + nx);
            if (h < 0 || tab[h] < 0) continue;
            tab[h] |= (int)0x80000000;
            if (tail >= n) throw std::runtime_error("BFS replay: cluster cells repeat");
            q[tail++] = XY{nx, ny};
        }
    }
    if (tail != n) throw std::runtime_error("BFS replay: cluster is not 8-connected");
    float ax = 0.0f, ay = 0.0f;
    for (int k = 0; k < n; ++k) { ax += (float)q[k].x; ay += (float)q[k].y; }
    sum_x = ax; sum_y = ay;
}

// The same walk over the frameless skeleton's bits in host memory (the published grid's read-back, bit x of word
// y * WW + x / 64), restricted to the cluster's bounding box, from its first raster cell: no copy of the cluster's
// cells. Inside the box the skeleton's cells reachable from the first cell are the cluster's cells unless the polygon
// cuts the box (skeleton cells outside it are not foreground): then the walk meets more than n cells and returns
// false (the caller replays that cluster from its cells).
static bool bfs_order_bits(const uint64_t *bits, const GridC &g, const ClusterRec &r, std::vector<XY> &q,
                           std::vector<uint64_t> &bm, float &sum_x, float &sum_y) {
    const int n = r.n, x0 = r.bx0, x1 = r.bx1, y0 = r.by0, y1 = r.by1;
    const int sy = r.first / g.W, sx = r.first - sy * g.W;
    if (n <= 0 || x0 > x1 || y0 > y1 || sx < x0 || sx > x1 || sy < y0 || sy > y1) return false;
    const long long bw = (long long)x1 - x0 + 1, pw = bw + 2, ph = (long long)y1 - y0 + 3;
    const long long RW = (pw + 63) / 64 + 1;
    bm.assign((size_t)(RW * ph), 0ull);
    uint64_t *B = bm.data();
    // row y of the box -> bitmap row y - y0 + 1, bit c <- cell x0 + c - 1 for c in [1, bw]; the border stays zero
    auto src64 = [&](const uint64_t *row, long long sb) -> uint64_t {   // cells sb .. sb + 63 of a skeleton row
        const long long w = sb >> 6;   // (sb >= -1: arithmetic shift)
        const int o = (int)(sb & 63);
        const uint64_t lo = (w >= 0 && w < g.WW) ? row[w] : 0ull;
        const uint64_t hi = (w + 1 >= 0 && w + 1 < g.WW) ? row[w + 1] : 0ull;
        return o ? (lo >> o) | (hi << (64 - o)) : lo;
    };
    for (int y = y0; y <= y1; ++y) {
        const uint64_t *row = bits + (size_t)y * g.WW;
        uint64_t *out = B + (long long)(y - y0 + 1) * RW;
        for (long long k = 0; k * 64 < pw; ++k) {
            uint64_t v = src64(row, (long long)x0 - 1 + 64 * k);
            const long long c0 = 64 * k;   // bitmap bits [c0, c0 + 64): keep c in [1, bw]
            if (c0 == 0) v &= ~1ull;
            if (c0 + 64 > bw + 1) {
                const long long keep = bw + 1 - c0;   // bits below keep
                v = keep <= 0 ? 0ull : (keep >= 64 ? v : v & ((1ull << keep) - 1));
            }
            out[k] = v;
        }
    }
    {
        const long long rr = sy - y0 + 1, c = sx - x0 + 1;
        if (!(B[rr * RW + (c >> 6)] >> (c & 63) & 1)) return false;   // (not a skeleton cell: records and bits disagree)
        B[rr * RW + (c >> 6)] &= ~(1ull << (c & 63));
    }
    q.resize((size_t)n);
    return bfs_walk(B, RW, x0, y0, sx, sy, q.data(), n, sum_x, sum_y) == n;
}

// cells != nullptr: replay from the cluster's cells; else from the skeleton bits (returns false when they do not give
// the cluster, see bfs_order_bits)
static bool host_bfs_replay(const int *cells, const uint64_t *bits, int n, const GridC &g, const double *poly, int np,
                            float min_length, ClusterRec &r, std::vector<XY> &q, std::vector<int> &tab,
                            std::vector<uint64_t> &bm) {
    float sum_x, sum_y;
    if (cells) bfs_order(cells, n, g, q, tab, bm, sum_x, sum_y);
    else if (!bfs_order_bits(bits, g, r, q, bm, sum_x, sum_y)) return false;
    r.cx = sum_x / (float)n;
    r.cy = sum_y / (float)n;
    bool row = false;
    if (r.length >= min_length) {
        float cwx = (float)(g.ox + (double)(r.cx * g.res)), cwy = (float)(g.oy + (double)(r.cy * g.res));
        r.center = make_double2(cwx, cwy);
        row = d_pip(cwx, cwy, poly, np);
    }
    if (row) {
        auto cw = [&](int k) {   // cell_w of the k-th BFS cell
            return make_double2((double)cell_world(g.ox, q[k].x, g.res), (double)cell_world(g.oy, q[k].y, g.res));
        };
        // the first strict maximum of d2, then its direction (the reference normalises at every new maximum; only the
        // last one's values survive, and they are the same operations on the same operands)
        double mx = 0.0; int fi = 0; double fx = 0, fy = 0;
        for (int k = 0; k < n; ++k) {
            double2 w = cw(k);
            double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            if (d2 > mx) { mx = d2; fi = k; }
        }
        if (mx > 0.0) {
            double2 w = cw(fi);
            double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            double s = std::sqrt(d2); fx = dx / s; fy = dy / s;
        }
        double mo = 0.0; int si = 0;
        for (int k = 0; k < n; ++k) {
            if (k == fi) continue;
            double2 w = cw(k);
            double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            if (!(d2 > mo)) continue;   // (the same test, its cheap half first: the normalisation only for a new max)
            // the sign of the normalised dot product nx fx + ny fy is that of dx fx + dy fy whenever the latter is not
            // within rounding of zero (both round within a few ulps of |dx fx| + |dy fy|, over s > 0); near zero the
            // reference's own expression decides
            const double pa = dx * fx, pb = dy * fy, dd = pa + pb;
            bool opposite;
            if (std::fabs(dd) > 1e-12 * (std::fabs(pa) + std::fabs(pb))) {
                opposite = dd < 0.0;
            } else {
                double nx = dx, ny = dy;
                if (d2 > 0.0) { double s = std::sqrt(d2); nx = dx / s; ny = dy / s; }
                opposite = nx * fx + ny * fy < 0.0;
            }
            if (opposite) { mo = d2; si = k; }
        }
        if (mo == 0.0) {
            double2 wf = cw(fi);
            for (int k = 0; k < n; ++k) {
                if (k == fi) continue;
                double2 w = cw(k);
                double dx = w.x - wf.x, dy = w.y - wf.y, d2 = dx * dx + dy * dy;
                if (d2 > mo) { mo = d2; si = k; }
            }
        }
        r.start = cw(fi);
        r.end = cw(si);
    }
    r.flags = (row ? 1 : 0) | 4;  // 4: replayed
    return true;
}

// The exact replays of a frame, in parallel over clusters on up to kReplayThreads host threads (each
// writes only its own record): the pool's parked workers when one is given (no thread start per frame).
void replay_clusters(const std::vector<ReplayJob> &jobs, const GridC &g, const double *poly, int np, float min_len,
                     ClusterRec *rec, HostPool *pool, std::vector<int> *failed) {
    if (jobs.empty()) return;
    std::vector<char> bad(jobs.size(), 0);
    std::atomic<int> next{0};
    std::exception_ptr err;
    std::mutex mu;
    auto work = [&](int) {
        std::vector<XY> q;
        std::vector<int> tab;
        std::vector<uint64_t> bm;
        for (int i; (i = next.fetch_add(1)) < (int)jobs.size();) {
            const ReplayJob &j = jobs[i];
            try {
                if (!host_bfs_replay(j.cells, j.bits, j.n, g, poly, np, min_len, rec[j.c], q, tab, bm)) bad[i] = 1;
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu);
                if (!err) err = std::current_exception();
            }
        }
    };
    const int nt = std::min<int>((int)jobs.size(), std::min(kReplayThreads, host_cpu_share()));
    if (pool) {
        pool->run(nt, work);
    } else {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
        work(0);
        for (auto &t : th) t.join();
    }
    if (err) std::rethrow_exception(err);
    for (size_t i = 0; i < jobs.size(); ++i) {
        if (!bad[i]) continue;
        if (!failed) throw std::logic_error("replay_clusters: a skeleton-bits replay failed without a fallback");
        failed->push_back((int)i);
    }
}

// ------------------------------------------------------------------ host union-find over pieces
int cluster_union(int W, int H, int n_pieces, const int *piece_root, int n_border, const int *bcell, const int *broot,
                  int *piece_cluster) {
    if (W <= 0 || H <= 0 || n_pieces < 0 || n_border < 0) throw std::invalid_argument("cluster_union: bad sizes");
    // pieces by root cell (roots are distinct: a cell belongs to one piece)
    std::vector<std::pair<int, int>> by_root((size_t)n_pieces);
    for (int i = 0; i < n_pieces; ++i) by_root[i] = {piece_root[i], i};
    std::sort(by_root.begin(), by_root.end());
    for (int i = 1; i < n_pieces; ++i)
        if (by_root[i].first == by_root[i - 1].first) throw std::invalid_argument("cluster_union: duplicate piece root");
    auto piece_of_root = [&](int r) {
        auto it = std::lower_bound(by_root.begin(), by_root.end(), std::make_pair(r, INT_MIN));
        if (it == by_root.end() || it->first != r) throw std::invalid_argument("cluster_union: border cell of an unknown piece");
        return it->second;
    };
    std::vector<int> parent((size_t)n_pieces);
    std::iota(parent.begin(), parent.end(), 0);
    auto find = [&](int x) {
        while (parent[x] != x) { parent[x] = parent[parent[x]]; x = parent[x]; }
        return x;
    };
    auto unite = [&](int a, int b) {   // the piece with the smaller first cell stays the representative
        a = find(a); b = find(b);
        if (a == b) return;
        if (piece_root[a] < piece_root[b]) parent[b] = a;
        else parent[a] = b;
    };
    std::unordered_map<int, int> cell_piece;
    cell_piece.reserve((size_t)n_border * 2 + 16);
    for (int i = 0; i < n_border; ++i) cell_piece.emplace(bcell[i], piece_of_root(broot[i]));
    // each adjacent pair once, from its smaller cell: E, SW, S, SE
    const int dxs[4] = {1, -1, 0, 1}, dys[4] = {0, 1, 1, 1};
    for (const auto &kv : cell_piece) {
        const int p = kv.first, y = p / W, x = p - y * W;
        for (int k = 0; k < 4; ++k) {
            const int nx = x + dxs[k], ny = y + dys[k];
            if (nx < 0 || nx >= W || ny >= H) continue;
            auto it = cell_piece.find(ny * W + nx);
            if (it != cell_piece.end()) unite(kv.second, it->second);
        }
    }
    // clusters in raster order of their first cell
    std::vector<int> reps;
    for (int i = 0; i < n_pieces; ++i)
        if (find(i) == i) reps.push_back(i);
    std::sort(reps.begin(), reps.end(), [&](int a, int b) { return piece_root[a] < piece_root[b]; });
    std::vector<int> id((size_t)n_pieces, -1);
    for (size_t k = 0; k < reps.size(); ++k) id[reps[k]] = (int)k;
    for (int i = 0; i < n_pieces; ++i) piece_cluster[i] = id[find(i)];
    return (int)reps.size();
}

// convertClustersToTreeRows (seed_gen:1329-1406) over the records in cluster order: the row arrays and
// each row's virtual-seed slots; then cluster_info (publishClusterInfo :1515-1565) and rows_info
// (:2546-2582), std::sort on the host with the reference comparators (same libstdc++ algorithm => same
// order on ties).
void assemble_rows(const std::vector<ClusterRec> &rec, SeedStageOut &out, std::vector<RowDev> &rows) {
    rows.clear();
    int slot = 0;
    for (const auto &r : rec) {
        if (!(r.flags & 1)) continue;
        out.row_center.push_back(r.center.x); out.row_center.push_back(r.center.y);
        out.row_start.push_back(r.start.x); out.row_start.push_back(r.start.y);
        out.row_end.push_back(r.end.x); out.row_end.push_back(r.end.y);
        out.row_length.push_back((double)r.length);
        RowDev d{r.start.x, r.start.y, r.end.x, r.end.y, 0, slot};
        double dx = r.end.x - r.start.x, dy = r.end.y - r.start.y;
        double dist = std::sqrt(dx * dx + dy * dy);
        if (!(dist < 1.0) && !(std::sqrt(dx * dx + dy * dy) < 1e-6)) d.k = static_cast<int>(std::floor(dist / 1.0));
        slot += 3 * d.k;
        rows.push_back(d);
    }
    const size_t n_rows = rows.size();
    struct CI { size_t index; float cx, cy; };
    std::vector<CI> infos;
    for (size_t i = 0; i < n_rows; ++i)
        infos.push_back({i, (float)out.row_center[2 * i], (float)out.row_center[2 * i + 1]});
    std::sort(infos.begin(), infos.end(), [](const CI &a, const CI &b) { return a.cy < b.cy; });
    for (const auto &ci : infos) { out.cluster_info.push_back(ci.cx); out.cluster_info.push_back(ci.cy); }
    struct TR { double cx, cy, sx, sy, ex, ey; };
    std::vector<TR> tr;
    for (size_t i = 0; i < n_rows; ++i)
        tr.push_back({out.row_center[2 * i], out.row_center[2 * i + 1], out.row_start[2 * i], out.row_start[2 * i + 1],
                      out.row_end[2 * i], out.row_end[2 * i + 1]});
    std::sort(tr.begin(), tr.end(), [](const TR &a, const TR &b) {
        if (std::abs(a.cy - b.cy) < 1e-6) return a.cx < b.cx;
        return a.cy < b.cy;
    });
    for (const auto &t : tr) { out.rows_info.insert(out.rows_info.end(), {t.sx, t.sy, t.ex, t.ey}); }
}

}  // namespace aos
