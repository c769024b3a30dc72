// Distributed a8-a10 of the tiled frame: cluster labelling, numbering and statistics
// spread over the tile ranks instead of run on the frame's root over the whole map.
//
// clusterOccupiedCells (seed_gen:970-1049) numbers the 8-connected skeleton clusters in raster order
// of their first cell (its scan + BFS discovery order). Per frame:
//  1. every rank labels the foreground (skeleton inside the polygon) of its OWN cells with the GPU
//     union-find (root = first raster cell): pieces, with n, integer sums and bbox per piece, and the
//     piece of every foreground cell on the tile's edge (border cells);
//  2. the piece tables and border cells are all-gathered; every rank runs the same host union-find
//     (cluster_union): two pieces are one cluster iff two of their border cells are 8-adjacent. A
//     cluster's first cell is the smallest first cell of its pieces, so clusters are numbered exactly
//     as on one GPU;
//  3. n and the exact integer sums add up over pieces; a cluster whose bbox diagonal is shorter than
//     cluster_min_length cannot be a row (length = max pairwise distance <= the diagonal), so its
//     record needs no cells. Only the cells of the other ("long") clusters are all-gathered, as
//     (cluster, cell) keys; every rank sorts them on its GPU and runs the whole-map stage's statistics
//     kernel on them (the same kernel on the same raster-ordered cells => the same records);
//  4. the exact BFS replays (clusters without the order-free certificate, all rows at 8192^2) are
//     split over the ranks' host cores (largest first, to the least loaded rank) and the replayed
//     records are all-gathered.
// The root then goes on with rows and seeds from the records (run_cluster_seed_stage, PreClusters).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <unordered_map>

#include "cluster_dev.h"
#include "cluster_seed.h"

namespace aos {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------ the rank's own cells (device)
// Own region of the window skeleton: rows [y0, y0 + nr), words [c0, c0 + nc) of the map, at row oy /
// word oc of the window (row pitch WWl).
struct TileView {
    int y0, nr, c0, nc, oy, oc, WWl;
    int Wt;   // own width in cells: min(W, 64 (c0 + nc)) - 64 c0
};

__global__ void k_dist_fg(const uint64_t *win, TileView T, GridC g, const double *poly, int np, uint64_t *fg, int *cnt) {
    __shared__ double xc[kRowCrossMax];
    __shared__ int nxc;
    const int k = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
    const int gy = T.y0 + r;
    const double wy = cell_world(g.oy, gy, g.res);
    const bool rowwise = row_crossings(poly, np, wy, xc, &nxc);   // (block-uniform; synchronises)
    if (k >= T.nc || r >= T.nr) return;
    uint64_t w = win[(size_t)(T.oy + r) * T.WWl + T.oc + k], o = 0;
    while (w) {
        const int b = __ffsll((long long)w) - 1;
        w &= w - 1;
        const int gx = 64 * (T.c0 + k) + b;
        if (gx >= g.W) continue;
        const double wx = cell_world(g.ox, gx, g.res);
        if (rowwise ? pip_row(wx, xc, nxc) : d_pip(wx, wy, poly, np)) o |= 1ull << b;
    }
    fg[(size_t)r * T.nc + k] = o;
    cnt[(size_t)r * T.nc + k] = __popcll(o);
}

__global__ void k_dist_list(const uint64_t *fg, const int *off, TileView T, int W, int *list) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
    if (k >= T.nc || r >= T.nr) return;
    const size_t wi = (size_t)r * T.nc + k;
    uint64_t w = fg[wi];
    int j = off[wi];
    while (w) {
        const int b = __ffsll((long long)w) - 1;
        w &= w - 1;
        list[j++] = (T.y0 + r) * W + 64 * (T.c0 + k) + b;   // the map's raster index
    }
}

__device__ __forceinline__ int dist_index(const uint64_t *fg, const int *off, const TileView &T, int lx, int ly) {
    if (lx < 0 || ly < 0 || lx >= T.Wt || ly >= T.nr) return -1;   // (outside the own region)
    const size_t wi = (size_t)ly * T.nc + (lx >> 6);
    const uint64_t w = fg[wi];
    const int b = lx & 63;
    if (!((w >> b) & 1ull)) return -1;
    return off[wi] + __popcll(w & ((1ull << b) - 1));
}

__global__ void k_dist_init(int *parent, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) parent[i] = i;
}
__global__ void k_dist_union(const int *list, int n, const uint64_t *fg, const int *off, TileView T, int W, int *parent) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = list[i], gy = p / W, ly = gy - T.y0, lx = p - gy * W - 64 * T.c0;
    const int ndx[4] = {-1, 0, 1, -1}, ndy[4] = {-1, -1, -1, 0};
    for (int k = 0; k < 4; ++k) {
        const int j = dist_index(fg, off, T, lx + ndx[k], ly + ndy[k]);
        if (j >= 0) uf_union(parent, i, j);
    }
}
__global__ void k_dist_flatten(int *parent, int *is_root, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int x = i;
    while (parent[x] != x) x = parent[x];
    parent[i] = x;
    is_root[i] = (x == i);
}

// pieces: n, sums, bbox by atomics; root = the first cell (the piece's smallest list index)
struct PieceDev { int *n, *root, *box; unsigned long long *sx, *sy; };   // box: minx, maxx, miny, maxy per piece
__global__ void k_dist_piece_init(PieceDev P, int np) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    P.n[i] = 0; P.sx[i] = 0; P.sy[i] = 0;
    P.box[4 * i] = INT_MAX; P.box[4 * i + 1] = INT_MIN; P.box[4 * i + 2] = INT_MAX; P.box[4 * i + 3] = INT_MIN;
}
__global__ void k_dist_piece(const int *list, const int *parent, const int *rank, int n, int W, TileView T, PieceDev P,
                             int2 *border, int *n_border) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = list[i], y = p / W, x = p - y * W, root = parent[i], id = rank[root];
    atomicAdd(&P.n[id], 1);
    atomicAdd(&P.sx[id], (unsigned long long)x);
    atomicAdd(&P.sy[id], (unsigned long long)y);
    atomicMin(&P.box[4 * id], x); atomicMax(&P.box[4 * id + 1], x);
    atomicMin(&P.box[4 * id + 2], y); atomicMax(&P.box[4 * id + 3], y);
    if (root == i) P.root[id] = p;
    const int lx = x - 64 * T.c0, ly = y - T.y0;
    if (lx == 0 || ly == 0 || lx == T.Wt - 1 || ly == T.nr - 1)
        border[atomicAdd(n_border, 1)] = make_int2(p, list[root]);
}

// (long-cluster index << 32 | cell) of the own cells of long clusters (lidx[piece] >= 0)
__global__ void k_dist_keys(const int *list, const int *parent, const int *rank, int n, const int *lidx,
                            unsigned long long *keys, int *n_keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int l = lidx[rank[parent[i]]];
    if (l < 0) return;
    keys[atomicAdd(n_keys, 1)] = ((unsigned long long)l << 32) | (unsigned)list[i];
}

// sorted keys -> cells and the runs of the long clusters
__global__ void k_dist_runs(const unsigned long long *keys, int n, int n_long, int *cells, int *off) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = keys[i];
    const int l = (int)(k >> 32);
    cells[i] = (int)(unsigned)(k & 0xffffffffull);
    if (i == 0 || (int)(keys[i - 1] >> 32) != l) off[l] = i;
    if (i == n - 1) off[n_long] = n;
}

// ------------------------------------------------------------------ collectives of variable size
static void comm_max(const aos_comm &cm, int32_t *v, int n) {
    if (cm.all_reduce_max(cm.user, v, n) != 0) throw CommError{"aos_comm.all_reduce_max failed"};
}
// every rank's byte count (each rank fills its own slot; max = the slot's value)
static std::vector<uint64_t> gather_sizes(const aos_comm &cm, uint64_t mine) {
    std::vector<int32_t> slots(2 * (size_t)cm.world, 0);
    slots[2 * cm.rank] = (int32_t)(mine & 0x7fffffff);
    slots[2 * cm.rank + 1] = (int32_t)(mine >> 31);
    comm_max(cm, slots.data(), (int)slots.size());
    std::vector<uint64_t> sz((size_t)cm.world);
    for (int r = 0; r < cm.world; ++r) sz[r] = (uint64_t)(uint32_t)slots[2 * r] | ((uint64_t)(uint32_t)slots[2 * r + 1] << 31);
    return sz;
}
// All-gather of sizes[r] bytes per rank through the communicator's fixed buffers, in chunks of
// buf_bytes: rank r's bytes land at dst + (sizes[0] + ... + sizes[r - 1]). src / dst: device or host.
static void gather_bytes(const aos_comm &cm, hipStream_t s, const void *src, bool src_dev,
                         const std::vector<uint64_t> &sizes, void *dst, bool dst_dev) {
    const uint64_t B = cm.buf_bytes & ~7ull;
    if (!B) throw CommError{"aos_comm.buf_bytes too small"};
    uint64_t maxb = 0;
    std::vector<uint64_t> at((size_t)cm.world + 1, 0);
    for (int r = 0; r < cm.world; ++r) { maxb = std::max(maxb, sizes[r]); at[r + 1] = at[r] + sizes[r]; }
    const uint64_t mine = sizes[cm.rank];
    for (uint64_t off = 0; off < maxb; off += B) {
        const uint64_t c = std::min(B, maxb - off);
        const uint64_t m = mine > off ? std::min(c, mine - off) : 0;
        if (m)
            AOS_HIP(hipMemcpyAsync(cm.send_buf, static_cast<const uint8_t *>(src) + off, m,
                                   src_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
        AOS_HIP(hipStreamSynchronize(s));
        if (cm.all_gather(cm.user, c) != 0) throw CommError{"aos_comm.all_gather failed"};
        for (int r = 0; r < cm.world; ++r) {
            const uint64_t v = sizes[r] > off ? std::min(c, sizes[r] - off) : 0;
            if (v)
                AOS_HIP(hipMemcpyAsync(static_cast<uint8_t *>(dst) + at[r] + off,
                                       static_cast<const uint8_t *>(cm.recv_buf) + (uint64_t)r * c, v,
                                       dst_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        }
        AOS_HIP(hipStreamSynchronize(s));   // (the next chunk's all-gather rewrites recv_buf)
    }
}

struct PieceRec { int root, n; long long sx, sy; int minx, maxx, miny, maxy; };
struct ReplayOut { int l, pad; ClusterRec r; };

template <class T> static T *dptr(DevBuf &b, size_t n) { return static_cast<T *>(b.ensure(sizeof(T) * std::max<size_t>(n, 1))); }

// ------------------------------------------------------------------ the rank's part of a frame
void cluster_dist(ClusterDistState &D, const aos_comm &cm, const TilePlan &t, const FrameGeom &fg, const Poly &poly,
                  float min_len, const uint64_t *win, int root, hipStream_t s, PreClusters &pre, ClusterDistStats &st) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    pre = PreClusters();
    st = ClusterDistStats();
    const GridC g = make_gridc(fg);
    const int W = g.W;
    const int np = (int)poly.size();
    std::vector<double> hp(2 * (size_t)np);
    for (int i = 0; i < np; ++i) { hp[2 * i] = poly[i].first; hp[2 * i + 1] = poly[i].second; }
    double *d_poly = dptr<double>(D.poly, hp.size());
    AOS_HIP(hipMemcpyAsync(d_poly, hp.data(), sizeof(double) * hp.size(), hipMemcpyHostToDevice, s));
    TileView T{t.y0, t.y1 - t.y0, t.c0, t.c1 - t.c0, t.y0 - t.wy0, t.c0 - t.wc0, t.lg.WW, 0};
    T.Wt = std::min(W, 64 * t.c1) - 64 * t.c0;
    int *h = static_cast<int *>(D.h.ensure(64));

    // ---- 1. own foreground, pieces, border cells
    const size_t Cw = (size_t)T.nc * T.nr;
    uint64_t *d_fg = dptr<uint64_t>(D.fg, Cw);
    int *d_cnt = dptr<int>(D.cnt, Cw + 1), *d_off = dptr<int>(D.off, Cw + 1);
    AOS_HIP(hipMemsetAsync(d_cnt + Cw, 0, sizeof(int), s));
    const dim3 gw(cdiv(T.nc, 64), T.nr);
    k_dist_fg<<<gw, 64, 0, s>>>(win, T, g, d_poly, np, d_fg, d_cnt);
    size_t tb = 0;
    AOS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (int *)nullptr, (int *)nullptr, (int)Cw + 1, s));
    AOS_HIP(hipcub::DeviceScan::ExclusiveSum(D.tmp.ensure(tb), tb, d_cnt, d_off, (int)Cw + 1, s));
    AOS_HIP(hipMemcpyAsync(h, d_off + Cw, sizeof(int), hipMemcpyDeviceToHost, s));
    AOS_HIP(hipStreamSynchronize(s));
    const int nf = h[0];
    int *d_list = dptr<int>(D.list, nf), *d_par = dptr<int>(D.parent, nf);
    int *d_isroot = dptr<int>(D.isroot, (size_t)nf + 1), *d_rank = dptr<int>(D.rank, (size_t)nf + 1);
    int npieces = 0;
    if (nf > 0) {
        k_dist_list<<<gw, 64, 0, s>>>(d_fg, d_off, T, W, d_list);
        k_dist_init<<<cdiv(nf, 256), 256, 0, s>>>(d_par, nf);
        k_dist_union<<<cdiv(nf, 256), 256, 0, s>>>(d_list, nf, d_fg, d_off, T, W, d_par);
        AOS_HIP(hipMemsetAsync(d_isroot + nf, 0, sizeof(int), s));
        k_dist_flatten<<<cdiv(nf, 256), 256, 0, s>>>(d_par, d_isroot, nf);
        size_t tb2 = 0;
        AOS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, (int *)nullptr, (int *)nullptr, nf + 1, s));
        AOS_HIP(hipcub::DeviceScan::ExclusiveSum(D.tmp.ensure(std::max(tb, tb2)), tb2, d_isroot, d_rank, nf + 1, s));
        AOS_HIP(hipMemcpyAsync(h, d_rank + nf, sizeof(int), hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        npieces = h[0];
    }
    // piece arrays: n | root | box (4) ints, sx | sy u64; border (cell, root) pairs and their count
    const size_t PI = (size_t)std::max(npieces, 1);
    int *d_pint = dptr<int>(D.pieces, 6 * PI + 4 * PI);   // 6 ints + 2 u64 (= 4 ints) per piece
    PieceDev P{d_pint, d_pint + PI, d_pint + 2 * PI, reinterpret_cast<unsigned long long *>(d_pint + 6 * PI),
               reinterpret_cast<unsigned long long *>(d_pint + 8 * PI)};
    int2 *d_border = dptr<int2>(D.border, (size_t)nf);
    int *d_nb = dptr<int>(D.counts, 2);
    AOS_HIP(hipMemsetAsync(d_nb, 0, 2 * sizeof(int), s));
    std::vector<PieceRec> mine((size_t)npieces);
    std::vector<int> h_n(npieces), h_root(npieces), h_box(4 * (size_t)npieces);
    std::vector<unsigned long long> h_sx(npieces), h_sy(npieces);
    int nb = 0;
    std::vector<int2> h_border;
    if (npieces > 0) {
        k_dist_piece_init<<<cdiv(npieces, 256), 256, 0, s>>>(P, npieces);
        k_dist_piece<<<cdiv(nf, 256), 256, 0, s>>>(d_list, d_par, d_rank, nf, W, T, P, d_border, d_nb);
        AOS_HIP(hipMemcpyAsync(h_n.data(), P.n, sizeof(int) * npieces, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipMemcpyAsync(h_root.data(), P.root, sizeof(int) * npieces, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipMemcpyAsync(h_box.data(), P.box, sizeof(int) * 4 * npieces, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipMemcpyAsync(h_sx.data(), P.sx, 8 * (size_t)npieces, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipMemcpyAsync(h_sy.data(), P.sy, 8 * (size_t)npieces, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipMemcpyAsync(h, d_nb, sizeof(int), hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        nb = h[0];
        h_border.resize(nb);
        if (nb) AOS_HIP(hipMemcpyAsync(h_border.data(), d_border, sizeof(int2) * nb, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        for (int i = 0; i < npieces; ++i)
            mine[i] = PieceRec{h_root[i], h_n[i], (long long)h_sx[i], (long long)h_sy[i], h_box[4 * i], h_box[4 * i + 1],
                               h_box[4 * i + 2], h_box[4 * i + 3]};
    }
    const auto t1 = clk::now();

    // ---- 2. all-gather the tables; the same union-find on every rank
    const std::vector<uint64_t> psz = gather_sizes(cm, sizeof(PieceRec) * (uint64_t)npieces);
    const std::vector<uint64_t> bsz = gather_sizes(cm, sizeof(int2) * (uint64_t)nb);
    uint64_t ptot = 0, btot = 0;
    for (int r = 0; r < cm.world; ++r) { ptot += psz[r]; btot += bsz[r]; }
    std::vector<PieceRec> all(ptot / sizeof(PieceRec));
    std::vector<int2> allb(btot / sizeof(int2));
    gather_bytes(cm, s, mine.data(), false, psz, all.data(), false);
    gather_bytes(cm, s, h_border.data(), false, bsz, allb.data(), false);
    const int NP = (int)all.size();
    std::vector<int> proot(NP), pcl(NP), bc(allb.size()), br(allb.size());
    for (int i = 0; i < NP; ++i) proot[i] = all[i].root;
    for (size_t i = 0; i < allb.size(); ++i) { bc[i] = allb[i].x; br[i] = allb[i].y; }
    const int ncl = cluster_union(W, g.H, NP, proot.data(), (int)allb.size(), bc.data(), br.data(), pcl.data());
    int my0 = 0;   // this rank's first piece in the gathered table
    for (int r = 0; r < cm.rank; ++r) my0 += (int)(psz[r] / sizeof(PieceRec));

    // ---- 3. per-cluster sums; long clusters
    struct Agg { long long sx = 0, sy = 0; int n = 0, minx = INT_MAX, maxx = INT_MIN, miny = INT_MAX, maxy = INT_MIN; };
    std::vector<Agg> agg((size_t)ncl);
    long long n_fg = 0;
    for (int i = 0; i < NP; ++i) {
        Agg &a = agg[pcl[i]];
        const PieceRec &p = all[i];
        a.sx += p.sx; a.sy += p.sy; a.n += p.n;
        a.minx = std::min(a.minx, p.minx); a.maxx = std::max(a.maxx, p.maxx);
        a.miny = std::min(a.miny, p.miny); a.maxy = std::max(a.maxy, p.maxy);
        n_fg += p.n;
    }
    std::vector<int> long_of((size_t)ncl, -1), long_ids;
    long long long_cells = 0;
    for (int c = 0; c < ncl; ++c) {
        const Agg &a = agg[c];
        const long long dx = a.maxx - a.minx, dy = a.maxy - a.miny;
        const float diag = (float)(std::sqrt((double)(dx * dx + dy * dy)) * (double)g.res);
        if (diag >= min_len) { long_of[c] = (int)long_ids.size(); long_ids.push_back(c); long_cells += a.n; }
    }
    const int nlong = (int)long_ids.size();
    std::vector<ClusterRec> lrec((size_t)nlong);
    if (nlong > 0) {
        // ---- own cells of long clusters as keys, all-gathered, sorted: runs of raster-ordered cells
        std::vector<int> lidx((size_t)std::max(npieces, 1), -1);
        long long my_keys = 0;
        for (int i = 0; i < npieces; ++i) {
            lidx[i] = long_of[pcl[my0 + i]];
            if (lidx[i] >= 0) my_keys += mine[i].n;
        }
        int *d_lidx = dptr<int>(D.lidx, lidx.size());
        unsigned long long *d_keys = dptr<unsigned long long>(D.keys, (size_t)my_keys);
        AOS_HIP(hipMemcpyAsync(d_lidx, lidx.data(), sizeof(int) * lidx.size(), hipMemcpyHostToDevice, s));
        if (my_keys > 0) {
            AOS_HIP(hipMemsetAsync(d_nb + 1, 0, sizeof(int), s));
            k_dist_keys<<<cdiv(nf, 256), 256, 0, s>>>(d_list, d_par, d_rank, nf, d_lidx, d_keys, d_nb + 1);
        }
        const std::vector<uint64_t> ksz = gather_sizes(cm, 8ull * (uint64_t)my_keys);
        const int nk = (int)long_cells;
        unsigned long long *d_all = dptr<unsigned long long>(D.keys_all, 2 * (size_t)nk);
        gather_bytes(cm, s, d_keys, true, ksz, d_all, true);
        int bits = 1;
        while ((1 << bits) <= nlong) ++bits;
        size_t tbs = 0;
        AOS_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tbs, d_all, d_all + nk, nk, 0, 32 + bits, s));
        AOS_HIP(hipcub::DeviceRadixSort::SortKeys(D.tmp.ensure(std::max(std::max(tb, tbs), (size_t)64)), tbs, d_all,
                                                  d_all + nk, nk, 0, 32 + bits, s));
        int *d_cells = dptr<int>(D.cells, (size_t)nk), *d_coff = dptr<int>(D.coff, (size_t)nlong + 1);
        k_dist_runs<<<cdiv(nk, 256), 256, 0, s>>>(d_all + nk, nk, nlong, d_cells, d_coff);
        ClusterRec *d_rec = dptr<ClusterRec>(D.rec, (size_t)nlong);
        launch_cluster_stats(d_coff, d_cells, nlong, g, d_poly, np, min_len, d_rec, s);
        AOS_HIP(hipMemcpyAsync(lrec.data(), d_rec, sizeof(ClusterRec) * nlong, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        st.n_long = nlong;
        st.long_cells = nk;

        // ---- 4. replays: largest first, each to the least loaded rank (the same plan on every rank)
        std::vector<int> flagged;
        for (int l = 0; l < nlong; ++l)
            if (lrec[l].flags & 2) flagged.push_back(l);
        std::stable_sort(flagged.begin(), flagged.end(), [&](int a, int b) { return lrec[a].n > lrec[b].n; });
        std::vector<long long> load((size_t)cm.world, 0);
        std::vector<int> my_jobs;
        for (int l : flagged) {
            const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            load[r] += lrec[l].n;
            if (r == cm.rank) my_jobs.push_back(l);
        }
        pre.n_bfs = (int)flagged.size();
        std::vector<long long> coff((size_t)nlong + 1);
        std::vector<int> hoff((size_t)nlong + 1);
        AOS_HIP(hipMemcpyAsync(hoff.data(), d_coff, sizeof(int) * (nlong + 1), hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        long long my_cells = 0;
        for (int l : my_jobs) my_cells += lrec[l].n;
        std::vector<int> hc((size_t)my_cells);
        std::vector<ReplayJob> jobs;
        long long at = 0;
        for (int l : my_jobs) {
            AOS_HIP(hipMemcpyAsync(hc.data() + at, d_cells + hoff[l], sizeof(int) * lrec[l].n, hipMemcpyDeviceToHost, s));
            jobs.push_back({l, hc.data() + at, lrec[l].n});
            at += lrec[l].n;
        }
        AOS_HIP(hipStreamSynchronize(s));
        const auto tr0 = clk::now();
        replay_clusters(jobs, g, hp.data(), np, min_len, lrec.data());
        st.ms_replay = std::chrono::duration<float, std::milli>(clk::now() - tr0).count();
        st.n_replayed_here = (int)my_jobs.size();
        std::vector<ReplayOut> outs;
        for (int l : my_jobs) outs.push_back(ReplayOut{l, 0, lrec[l]});
        const std::vector<uint64_t> rsz = gather_sizes(cm, sizeof(ReplayOut) * (uint64_t)outs.size());
        uint64_t rtot = 0;
        for (int r = 0; r < cm.world; ++r) rtot += rsz[r];
        std::vector<ReplayOut> allr(rtot / sizeof(ReplayOut));
        gather_bytes(cm, s, outs.data(), false, rsz, allr.data(), false);
        for (const auto &o : allr) lrec[o.l] = o.r;
    }
    const auto t2 = clk::now();
    st.n_pieces = npieces;
    st.n_border = nb;
    st.ms_local = std::chrono::duration<float, std::milli>(t1 - t0).count();
    st.ms_global = std::chrono::duration<float, std::milli>(t2 - t1).count();
    if (cm.rank != root) return;

    // ---- the root's records, in cluster order
    pre.rec.assign((size_t)ncl, ClusterRec{});
    pre.n_fg = (int)n_fg;
    for (int c = 0; c < ncl; ++c) {
        if (long_of[c] >= 0) { pre.rec[c] = lrec[long_of[c]]; continue; }
        ClusterRec &r = pre.rec[c];   // not a row: only the certificate is observable (n_bfs)
        const Agg &a = agg[c];
        r.sx = a.sx; r.sy = a.sy; r.n = a.n;
        const bool exact_sums = a.sx <= (1ll << 24) && a.sy <= (1ll << 24);
        r.flags = exact_sums ? 0 : 2;
        if (!exact_sums) ++pre.n_bfs;
    }
}

}  // namespace aos

using namespace aos;

extern "C" int aos_cluster_union(int32_t width, int32_t height, int32_t n_pieces, const int32_t *piece_root,
                                 int32_t n_border, const int32_t *border_cell, const int32_t *border_root,
                                 int32_t *piece_cluster, int32_t *n_clusters) {
    if ((n_pieces > 0 && (!piece_root || !piece_cluster)) || (n_border > 0 && (!border_cell || !border_root)) ||
        !n_clusters) {
        set_error("aos_cluster_union: null array");
        return AOS_E_INVALID;
    }
    try {
        *n_clusters = cluster_union(width, height, n_pieces, piece_root, n_border, border_cell, border_root, piece_cluster);
        return AOS_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return AOS_E_INVALID;
    }
}
