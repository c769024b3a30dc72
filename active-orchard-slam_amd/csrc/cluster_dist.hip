// Distributed a8-a10 of the tiled frame: cluster labelling, numbering and statistics
// spread over the tile ranks instead of run on the frame's root over the whole map.
//
// clusterOccupiedCells (seed_gen:970-1049) numbers the 8-connected skeleton clusters in raster order
// of their first cell (its scan + BFS discovery order). Per frame:
//  1. every rank labels the foreground (skeleton inside the polygon) of its OWN cells with the whole-map
//     stage's union-find kernels (ccl_label: block-local union-find in LDS): pieces, named by their first
//     raster cell. One pass aggregates per piece n, the exact integer sums and the bbox (LDS-combined per
//     workgroup: one global atomic per (workgroup, piece) instead of seven per cell), gives every cell its
//     rank inside its piece, and lists the piece of every foreground cell on an inner tile edge;
//  2. the piece tables and border cells are all-gathered (one size reduction, one all-gather); every rank
//     runs the same host union-find (cluster_union): two pieces are one cluster iff two of their border
//     cells are 8-adjacent. A cluster's first cell is the smallest first cell of its pieces, so clusters are
//     numbered exactly as on one GPU;
//  3. n and the sums add up over pieces; a cluster whose bbox diagonal is shorter than cluster_min_length
//     cannot be a row (length = max pairwise distance <= the diagonal), so its record needs no cells. Every
//     other ("long") cluster gets ONE owner rank, the same plan on every rank (largest first, to the least
//     loaded rank), and its cells go to that rank only: one personalised exchange (aos_comm.all_to_all;
//     without it, through all_gather), whose sizes every rank already knows from the piece table;
//  4. the owner puts each cluster's pieces together (one segment copy), runs the whole-map stage's
//     statistics kernel on them (the same kernel on the same cells => the same record) and, for a cluster
//     without the order-free certificate (every row at 8192^2), the exact BFS replay on its own host cores;
//     then the owners' records are all-gathered.
// The root goes on with rows and seeds from the records (run_cluster_seed_stage, PreClusters).
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>

#include "cluster_dev.h"
#include "cluster_seed.h"
#include "dev_prims_device.h"

namespace aos {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------ the rank's own cells (device)
// Own region of the window skeleton: rows [y0, y0 + nr), words [c0, c0 + nc) of the map, at row oy /
// word oc of the window (row pitch WWl).
struct TileView {
    int y0, nr, c0, nc, oy, oc, WWl;
    int Wt;   // own width in cells: min(W, 64 (c0 + nc)) - 64 c0
};

// own foreground (compact: nc words x nr rows) and its popcount per word
__global__ void k_dist_fg(const uint64_t *win, TileView T, GridC g, const double *poly, int np, uint64_t *fg, int *cnt) {
    __shared__ double xc[kRowCrossMax];
    __shared__ int nxc;
    const int k = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
    const int gy = T.y0 + r;
    const double wy = cell_world(g.oy, gy, g.res);
    const bool rowwise = row_crossings(poly, np, wy, xc, &nxc);   // (block-uniform; synchronises)
    if (k >= T.nc || r >= T.nr) return;
    uint64_t w = win[(size_t)(T.oy + r) * T.WWl + T.oc + k], o = 0;
    const int x0 = 64 * (T.c0 + k);
    if (rowwise && __popcll(w) >= kPipWordMin) {
        const uint64_t valid = g.W - x0 >= 64 ? ~0ull : (1ull << (g.W - x0)) - 1;   // (cells gx < W)
        o = w & valid & pip_row_word(g.ox, g.res, x0, xc, nxc);
    } else {
        while (w) {
            const int b = __ffsll((long long)w) - 1;
            w &= w - 1;
            const int gx = x0 + b;
            if (gx >= g.W) continue;
            const double wx = cell_world(g.ox, gx, g.res);
            if (rowwise ? pip_row(wx, xc, nxc) : d_pip(wx, wy, poly, np)) o |= 1ull << b;
        }
    }
    fg[(size_t)r * T.nc + k] = o;
    cnt[(size_t)r * T.nc + k] = __popcll(o);
}

// piece tables, SoA: n | root | minx | maxx | miny | maxy (ints), sx | sy (u64)
struct PieceDev { int *n, *root, *mnx, *mxx, *mny, *mxy; unsigned long long *sx, *sy; };
struct PieceRec { int root, n; long long sx, sy; int minx, maxx, miny, maxy; };   // 40 B, the gathered table

__global__ void k_piece_init(PieceDev P, const int *n_pieces, int cap, int *n_border) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *n_border = 0;   // (k_piece_agg counts the border cells: no fill launch)
    if (i >= cap || i >= *n_pieces) return;
    P.n[i] = 0; P.sx[i] = 0; P.sy[i] = 0;
    P.mnx[i] = INT_MAX; P.mxx[i] = INT_MIN; P.mny[i] = INT_MAX; P.mxy[i] = INT_MIN;
}

// One workgroup = kPcTB consecutive cells of the raster-ordered list: a handful of pieces. Their counts, sums
// and bboxes are combined in an LDS table first; each workgroup then adds one total per piece to the global
// tables, and the atomicAdd on the piece's n returns the workgroup's base inside the piece, so every cell
// gets a unique rank inside its piece (prank). Border cells: the piece of each foreground cell on an inner
// edge of the own region (a map edge has no neighbour tile).
constexpr int kPcTB = 256, kPcSlots = 512;
__global__ __launch_bounds__(kPcTB) void k_piece_agg(const int *list, const int *parent, const int *rank, int nf, TileView T,
                                                      int W, int H, PieceDev P, int *pid_of, int *prank, int2 *border,
                                                      int *n_border) {
    __shared__ int key[kPcSlots], cnt[kPcSlots], mnx[kPcSlots], mxx[kPcSlots], mny[kPcSlots], mxy[kPcSlots];
    __shared__ unsigned long long ssx[kPcSlots], ssy[kPcSlots];
    const int tid = threadIdx.x, i = blockIdx.x * kPcTB + tid;
    for (int k = tid; k < kPcSlots; k += kPcTB) {
        key[k] = -1; cnt[k] = 0; ssx[k] = 0; ssy[k] = 0;
        mnx[k] = INT_MAX; mxx[k] = INT_MIN; mny[k] = INT_MAX; mxy[k] = INT_MIN;
    }
    __syncthreads();
    int slot = 0, lr = 0;
    if (i < nf) {
        const int l = list[i], ly = l / T.Wt, lx = l - ly * T.Wt;
        const int x = 64 * T.c0 + lx, y = T.y0 + ly;
        const int root = parent[i], pid = rank[root];
        pid_of[i] = pid;
        slot = (int)(((unsigned)pid * 2654435761u) >> 23) & (kPcSlots - 1);
        for (;;) {   // (at most kPcTB distinct ids per workgroup: a free slot always exists)
            const int old = atomicCAS(&key[slot], -1, pid);
            if (old == -1 || old == pid) break;
            slot = (slot + 1) & (kPcSlots - 1);
        }
        lr = atomicAdd(&cnt[slot], 1);
        atomicAdd(&ssx[slot], (unsigned long long)x);
        atomicAdd(&ssy[slot], (unsigned long long)y);
        atomicMin(&mnx[slot], x); atomicMax(&mxx[slot], x);
        atomicMin(&mny[slot], y); atomicMax(&mxy[slot], y);
        if (root == i) P.root[pid] = y * W + x;
        const bool edge = (lx == 0 && T.c0 > 0) || (ly == 0 && T.y0 > 0) || (lx == T.Wt - 1 && x + 1 < W) ||
                          (ly == T.nr - 1 && y + 1 < H);
        if (edge) {
            const int l0 = list[root], ry = T.y0 + l0 / T.Wt, rx = 64 * T.c0 + l0 % T.Wt;
            border[atomicAdd(n_border, 1)] = make_int2(y * W + x, ry * W + rx);
        }
    }
    __syncthreads();
    for (int k = tid; k < kPcSlots; k += kPcTB) {
        const int id = key[k];
        if (id < 0) continue;
        cnt[k] = atomicAdd(&P.n[id], cnt[k]);   // (now the workgroup's base inside the piece)
        atomicAdd(&P.sx[id], ssx[k]);
        atomicAdd(&P.sy[id], ssy[k]);
        atomicMin(&P.mnx[id], mnx[k]); atomicMax(&P.mxx[id], mxx[k]);
        atomicMin(&P.mny[id], mny[k]); atomicMax(&P.mxy[id], mxy[k]);
    }
    __syncthreads();
    if (i < nf) prank[i] = cnt[slot] + lr;
}

// the gathered blob of this rank: PieceRec[n_pieces] then int2 border[n_border]
__global__ void k_piece_pack(PieceDev P, const int *n_pieces, const int2 *border, const int *n_border, int cap,
                             uint8_t *blob) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int np = *n_pieces, nb = *n_border;
    if (i < np && i < cap) {
        PieceRec r{P.root[i], P.n[i], (long long)P.sx[i], (long long)P.sy[i], P.mnx[i], P.mxx[i], P.mny[i], P.mxy[i]};
        reinterpret_cast<PieceRec *>(blob)[i] = r;
    }
    if (i < nb && i < cap) reinterpret_cast<int2 *>(blob + sizeof(PieceRec) * (size_t)np)[i] = border[i];
}

// the cells of long pieces, each to its slot in the send layout (destination-major, then cluster, piece)
__global__ void k_route(const int *list, const int *pid_of, const int *prank, int nf, const int *poff, TileView T, int W,
                        int *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const int o = poff[pid_of[i]];
    if (o < 0) return;
    const int l = list[i], ly = l / T.Wt, lx = l - ly * T.Wt;
    out[o + prank[i]] = (T.y0 + ly) * W + 64 * T.c0 + lx;
}

// one workgroup per segment: landing[src, src + n) -> cells[dst, dst + n) (a cluster's pieces side by side)
struct Seg { long long src, dst; int n, pad; };
__global__ void k_segments(const Seg *segs, const int *landing, int *cells) {
    const Seg s = segs[blockIdx.x];
    for (int k = threadIdx.x; k < s.n; k += blockDim.x) cells[s.dst + k] = landing[s.src + k];
}

// ------------------------------------------------------------------ collectives of variable size
// All-gather of sizes[r] bytes per rank through the communicator's fixed buffers, in chunks of
// buf_bytes: rank r's bytes land at dst + (sizes[0] + ... + sizes[r - 1]). src / dst: device or pinned host
// memory (host ends move by kernel stores: copy_to_host / copy_from_host). Stream-ordered collectives need no
// wait between the chunks (the stream orders each chunk's copies around its all-gather); a host dst is waited for.
static void gather_bytes(FrameComm &fc, hipStream_t s, const void *src, bool src_dev, const std::vector<uint64_t> &sizes,
                         void *dst, bool dst_dev, PinnedBuf &h_recv) {
    const aos_comm &cm = fc.c;
    const uint64_t B = cm.buf_bytes & ~7ull;
    if (!B) throw CommError{"aos_comm.buf_bytes too small"};
    uint64_t maxb = 0;
    std::vector<uint64_t> at((size_t)cm.world + 1, 0);
    for (int r = 0; r < cm.world; ++r) { maxb = std::max(maxb, sizes[r]); at[r + 1] = at[r] + sizes[r]; }
    const uint64_t mine = sizes[cm.rank];
    for (uint64_t off = 0; off < maxb; off += B) {
        const uint64_t c = std::min(B, maxb - off);
        const uint64_t m = mine > off ? std::min(c, mine - off) : 0;
        if (m) {
            const uint8_t *p = static_cast<const uint8_t *>(src) + off;
            if (src_dev) AOS_HIP(hipMemcpyAsync(cm.send_buf, p, m, hipMemcpyDeviceToDevice, s));
            else copy_from_host(cm.send_buf, p, m, s);
        }
        fc.all_gather(c, s);
        if (!dst_dev) {   // the chunk's whole receive buffer in one read-back, then each rank's bytes on the host
            uint64_t last = 0;   // (up to the last rank's bytes in this chunk)
            for (int r = 0; r < cm.world; ++r)
                if (sizes[r] > off) last = (uint64_t)r * c + std::min(c, sizes[r] - off);
            uint8_t *h = static_cast<uint8_t *>(h_recv.ensure(std::max<uint64_t>(last, 16)));
            // (whole 16-byte words while they stay inside recv_buf's world * buf_bytes: the copy kernel's uint4 form)
            copy_to_host(h, cm.recv_buf, std::min<uint64_t>((last + 15) & ~15ull, (uint64_t)cm.world * cm.buf_bytes), s);
            AOS_HIP(hipStreamSynchronize(s));
            for (int r = 0; r < cm.world; ++r) {
                const uint64_t v = sizes[r] > off ? std::min(c, sizes[r] - off) : 0;
                if (v) std::memcpy(static_cast<uint8_t *>(dst) + at[r] + off, h + (uint64_t)r * c, v);
            }
            continue;
        }
        for (int r = 0; r < cm.world; ++r) {
            const uint64_t v = sizes[r] > off ? std::min(c, sizes[r] - off) : 0;
            if (v) AOS_HIP(hipMemcpyAsync(static_cast<uint8_t *>(dst) + at[r] + off,
                                          static_cast<const uint8_t *>(cm.recv_buf) + (uint64_t)r * c, v,
                                          hipMemcpyDeviceToDevice, s));
        }
        if (!fc.ordered()) AOS_HIP(hipStreamSynchronize(s));   // (the next chunk's all-gather rewrites recv_buf)
    }
}

template <class T> static T *dptr(DevBuf &b, size_t n) { return static_cast<T *>(b.ensure(sizeof(T) * std::max<size_t>(n, 1))); }
template <class T> static T *hptr(PinnedBuf &b, size_t n) { return static_cast<T *>(b.ensure(sizeof(T) * std::max<size_t>(n, 1))); }

struct OwnedOut { int l, replayed; ClusterRec r; };

static uint64_t debug_a2a_round_bytes() { return g_debug_a2a_round.load(std::memory_order_relaxed); }   // (aos_debug_faults)

// The personalised exchange of the long clusters' cells. cnt[s * W + d]: bytes rank s sends to rank d (known
// on every rank). send: this rank's route buffer (device, destination-major). Returns the device buffer the
// blocks addressed to this rank landed in and, per source s, where s's block for this rank starts in it.
static const int *exchange_cells(FrameComm &fc, ClusterDistState &D, hipStream_t s, const std::vector<uint64_t> &cnt,
                                 const int *send, std::vector<uint64_t> &src_base) {
    const aos_comm &cm = fc.c;
    const int W = cm.world, me = cm.rank;
    src_base.assign((size_t)W, 0);
    if (W == 1) return send;
    std::vector<uint64_t> row((size_t)W, 0), col((size_t)W, 0);
    for (int a = 0; a < W; ++a)
        for (int b = 0; b < W; ++b) { row[a] += cnt[(size_t)a * W + b]; col[b] += cnt[(size_t)a * W + b]; }
    if (!fc.has_all_to_all()) {   // through all_gather: everyone's route buffer, then this rank's blocks from it
        uint8_t *all = dptr<uint8_t>(D.landing, std::accumulate(row.begin(), row.end(), (uint64_t)0));
        gather_bytes(fc, s, send, true, row, all, true, D.h_recv);
        uint64_t at = 0;
        for (int r = 0; r < W; ++r) {
            uint64_t pre = 0;
            for (int q = 0; q < me; ++q) pre += cnt[(size_t)r * W + q];
            src_base[r] = (at + pre) / 4;
            at += row[r];
        }
        return reinterpret_cast<const int *>(all);
    }
    uint64_t roff = 0;
    for (int r = 0; r < W; ++r) { src_base[r] = roff / 4; roff += cnt[(size_t)r * W + me]; }
    int *land = dptr<int>(D.landing, roff / 4);
    // rounds of at most q bytes per pair keep every row sum <= buf_bytes and column sum <= world * buf_bytes
    uint64_t q = (cm.buf_bytes / (uint64_t)W) & ~7ull;
    const uint64_t q_cap = debug_a2a_round_bytes();   // (tests: force many rounds)
    if (q_cap) q = std::min(q, std::max<uint64_t>(8, q_cap & ~7ull));   // (tests: force many rounds)
    if (!q) throw CommError{"aos_comm.buf_bytes too small for the cluster exchange"};
    uint64_t most = 0;
    for (uint64_t c : cnt) most = std::max(most, c);
    std::vector<uint64_t> so((size_t)W, 0);
    for (int d = 1; d < W; ++d) so[d] = so[d - 1] + cnt[(size_t)me * W + d - 1];
    std::vector<uint64_t> c((size_t)W * W);
    for (uint64_t off = 0; off < std::max<uint64_t>(most, 1); off += q) {
        for (size_t k = 0; k < c.size(); ++k) c[k] = cnt[k] > off ? std::min(q, cnt[k] - off) : 0;
        uint64_t at = 0;
        for (int d = 0; d < W; ++d) {
            const uint64_t n = c[(size_t)me * W + d];
            if (n) AOS_HIP(hipMemcpyAsync(static_cast<uint8_t *>(cm.send_buf) + at,
                                          reinterpret_cast<const uint8_t *>(send) + so[d] + off, n,
                                          hipMemcpyDeviceToDevice, s));
            at += n;
        }
        fc.all_to_all(c.data(), s);
        at = 0;
        for (int r = 0; r < W; ++r) {
            const uint64_t n = c[(size_t)r * W + me];
            if (n) AOS_HIP(hipMemcpyAsync(reinterpret_cast<uint8_t *>(land) + src_base[r] * 4 + off,
                                          static_cast<const uint8_t *>(cm.recv_buf) + at, n, hipMemcpyDeviceToDevice, s));
            at += n;
        }
        if (!fc.ordered()) AOS_HIP(hipStreamSynchronize(s));   // (the next round rewrites recv_buf)
    }
    return land;
}

// ------------------------------------------------------------------ the rank's part of a frame
void cluster_dist(ClusterDistState &D, FrameComm &fc, const TilePlan &t, const FrameGeom &fg, const Poly &poly,
                  float min_len, const uint64_t *win, int root, hipStream_t s, PreClusters &pre, ClusterDistStats &st) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const aos_comm &cm = fc.c;
    pre = PreClusters();
    st = ClusterDistStats();
    const GridC g = make_gridc(fg);
    const int W = g.W, world = cm.world, me = cm.rank;
    const int npoly = (int)poly.size();
    double *hp = hptr<double>(D.h_poly, 2 * (size_t)npoly);
    for (int i = 0; i < npoly; ++i) { hp[2 * i] = poly[i].first; hp[2 * i + 1] = poly[i].second; }
    double *d_poly = dptr<double>(D.poly, 2 * (size_t)npoly);
    copy_from_host(d_poly, hp, sizeof(double) * 2 * npoly, s);
    TileView T{t.y0, t.y1 - t.y0, t.c0, t.c1 - t.c0, t.y0 - t.wy0, t.c0 - t.wc0, t.lg.WW, 0};
    T.Wt = std::min(W, 64 * t.c1) - 64 * t.c0;
    int *h = hptr<int>(D.h, 16);

    // ---- 1. own foreground, pieces, border cells (the whole-map stage's labelling on the own region)
    const size_t Cw = (size_t)T.nc * T.nr;
    uint64_t *d_fg = dptr<uint64_t>(D.fg, Cw);
    int *d_cnt = dptr<int>(D.cnt, Cw), *d_off = dptr<int>(D.ccl.off, Cw + 1);
    k_dist_fg<<<dim3(cdiv(T.nc, 64), T.nr), 64, 0, s>>>(win, T, g, d_poly, npoly, d_fg, d_cnt);
    scan_1p(D.ccl.lb, d_cnt, d_off, (int)Cw, false, s);
    GridC gl{};   // the own region as an image: local raster index = ly * Wt + lx
    gl.W = T.Wt; gl.H = T.nr; gl.WW = T.nc;
    int err = 0;
    const int nf = ccl_label(D.ccl, d_fg, d_off, gl, s, h, &err);
    const int *d_list = D.ccl.list_p, *d_par = D.ccl.parent_p, *d_rank = D.ccl.rank_p;
    const int *d_np = d_rank + nf;   // (pieces: on the device)
    const size_t PC = (size_t)std::max(nf, 1);
    int *pi = dptr<int>(D.pieces, 6 * PC + 4 * PC);
    PieceDev P{pi, pi + PC, pi + 2 * PC, pi + 3 * PC, pi + 4 * PC, pi + 5 * PC,
               reinterpret_cast<unsigned long long *>(pi + 6 * PC), reinterpret_cast<unsigned long long *>(pi + 8 * PC)};
    int *d_pid = dptr<int>(D.pid, PC), *d_prank = dptr<int>(D.prank, PC);
    int2 *d_border = dptr<int2>(D.border, PC);
    int *d_nb = dptr<int>(D.counts, 2);
    uint8_t *d_blob = dptr<uint8_t>(D.blob, (sizeof(PieceRec) + sizeof(int2)) * PC);
    if (nf > 0) {
        k_piece_init<<<cdiv(nf, 256), 256, 0, s>>>(P, d_np, nf, d_nb);
        k_piece_agg<<<cdiv(nf, kPcTB), kPcTB, 0, s>>>(d_list, d_par, d_rank, nf, T, W, g.H, P, d_pid, d_prank, d_border, d_nb);
        k_piece_pack<<<cdiv(nf, 256), 256, 0, s>>>(P, d_np, d_border, d_nb, nf, d_blob);
        AOS_HIP(hipGetLastError());
    }
    peek_to_host(h + 2, {d_np, d_nb, D.ccl.lb.err_word(s)}, s);
    AOS_HIP(hipStreamSynchronize(s));
    const int npieces = nf > 0 ? h[2] : 0, nb = nf > 0 ? h[3] : 0;
    err |= h[4];
    const auto t1 = clk::now();

    // ---- 2. all-gather the tables (every rank's sizes and error word first); the same union-find on every rank
    std::vector<int32_t> slots(2 * (size_t)world + 1, 0);
    slots[2 * me] = npieces;
    slots[2 * me + 1] = nb;
    slots[2 * world] = err ? 1 : 0;
    fc.max_host(slots.data(), (int)slots.size());
    if (slots[2 * world]) throw std::runtime_error("tiled cluster stage: a single-pass scan failed on a rank's device");
    std::vector<uint64_t> bsz((size_t)world);
    std::vector<int> rp0((size_t)world + 1, 0);   // first piece of rank r in the gathered table
    uint64_t btot = 0;
    int NB = 0;
    for (int r = 0; r < world; ++r) {
        bsz[r] = sizeof(PieceRec) * (uint64_t)slots[2 * r] + sizeof(int2) * (uint64_t)slots[2 * r + 1];
        btot += bsz[r];
        rp0[r + 1] = rp0[r] + slots[2 * r];
        NB += slots[2 * r + 1];
    }
    uint8_t *hall = hptr<uint8_t>(D.h_all, btot);
    gather_bytes(fc, s, d_blob, true, bsz, hall, false, D.h_recv);
    const int NP = rp0[world];
    std::vector<PieceRec> all((size_t)NP);
    std::vector<int> proot(NP), pcl(NP), bc((size_t)NB), br((size_t)NB);
    {
        uint64_t at = 0;
        int nbk = 0;
        for (int r = 0; r < world; ++r) {
            const int n_p = slots[2 * r], n_b = slots[2 * r + 1];
            std::memcpy(all.data() + rp0[r], hall + at, sizeof(PieceRec) * (size_t)n_p);
            const int2 *b = reinterpret_cast<const int2 *>(hall + at + sizeof(PieceRec) * (size_t)n_p);
            for (int k = 0; k < n_b; ++k, ++nbk) { bc[nbk] = b[k].x; br[nbk] = b[k].y; }
            at += bsz[r];
        }
    }
    for (int i = 0; i < NP; ++i) proot[i] = all[i].root;
    const int ncl = cluster_union(W, g.H, NP, proot.data(), NB, bc.data(), br.data(), pcl.data());

    // ---- 3. per-cluster sums; long clusters and their owners
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
    st.n_long = nlong;
    st.long_cells = (int)long_cells;
    std::vector<ClusterRec> lrec((size_t)nlong);
    if (nlong > 0) {
        // owners: largest first, each to the least loaded rank (ties: the lowest rank) -- the same on every rank
        std::vector<int> order((size_t)nlong), owner((size_t)nlong);
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return agg[long_ids[a]].n > agg[long_ids[b]].n; });
        std::vector<long long> load((size_t)world, 0);
        for (int l : order) {
            const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            load[r] += agg[long_ids[l]].n;
            owner[l] = r;
        }
        // every rank's send layout: destination, then long cluster, then piece (all ranks compute all of them)
        std::vector<std::vector<int>> lpieces((size_t)nlong);   // the pieces of each long cluster, by table index
        for (int i = 0; i < NP; ++i)
            if (long_of[pcl[i]] >= 0) lpieces[long_of[pcl[i]]].push_back(i);
        std::vector<int> by_owner((size_t)nlong);   // long clusters ordered by (owner, id)
        std::iota(by_owner.begin(), by_owner.end(), 0);
        std::stable_sort(by_owner.begin(), by_owner.end(), [&](int a, int b) { return owner[a] < owner[b]; });
        std::vector<uint64_t> cnt((size_t)world * world, 0);
        std::vector<long long> piece_off((size_t)NP, -1);   // element offset inside its rank's send buffer
        std::vector<long long> rank_at((size_t)world, 0);
        auto rank_of = [&](int i) { return (int)(std::upper_bound(rp0.begin(), rp0.end(), i) - rp0.begin()) - 1; };
        for (int l : by_owner)
            for (int i : lpieces[l]) {
                const int r = rank_of(i);
                piece_off[i] = rank_at[r];
                rank_at[r] += all[i].n;
                cnt[(size_t)r * world + owner[l]] += 4ull * (uint64_t)all[i].n;
            }
        // ---- route the own cells of long pieces into the send layout
        const long long my_send = rank_at[me];
        int *d_send = dptr<int>(D.sendbuf, (size_t)my_send);
        if (my_send > 0) {
            int *hpo = hptr<int>(D.h_poff, (size_t)npieces);
            for (int p = 0; p < npieces; ++p) hpo[p] = (int)piece_off[rp0[me] + p];
            int *d_poff = dptr<int>(D.poff, (size_t)npieces);
            copy_from_host(d_poff, hpo, sizeof(int) * npieces, s);
            k_route<<<cdiv(nf, 256), 256, 0, s>>>(d_list, d_pid, d_prank, nf, d_poff, T, W, d_send);
            AOS_HIP(hipGetLastError());
        }
        // ---- 4. exchange; the owned clusters' pieces side by side; statistics
        std::vector<uint64_t> src_base;
        const int *land = exchange_cells(fc, D, s, cnt, d_send, src_base);
        std::vector<int> mine_l;   // owned long clusters, by id
        for (int l = 0; l < nlong; ++l)
            if (owner[l] == me) mine_l.push_back(l);
        const int nown = (int)mine_l.size();
        // s's block for this rank: s's pieces of the owned clusters by (cluster id, table index) -- the order
        // s routed them in; a cluster's pieces in table order are rank-major, so one walk gives every segment
        std::vector<Seg> segs;
        std::vector<int> coff((size_t)nown + 1, 0);
        {
            std::vector<long long> blk_at((size_t)world, 0);
            long long at = 0;
            for (int j = 0; j < nown; ++j) {
                coff[j] = (int)at;
                for (int i : lpieces[mine_l[j]]) {
                    const int r = rank_of(i);
                    segs.push_back(Seg{(long long)src_base[r] + blk_at[r], at, all[i].n, 0});
                    blk_at[r] += all[i].n;
                    at += all[i].n;
                }
            }
            coff[nown] = (int)at;
        }
        const int n_owned_cells = coff[nown];
        std::vector<int> replayed((size_t)nown, 0);   // the owned clusters replayed here
        if (nown > 0) {
            Seg *hs = hptr<Seg>(D.h_segs, segs.size());
            std::copy(segs.begin(), segs.end(), hs);
            Seg *d_segs = dptr<Seg>(D.segs, segs.size());
            copy_from_host(d_segs, hs, sizeof(Seg) * segs.size(), s);
            int *hco = hptr<int>(D.h_coff, (size_t)nown + 1);
            std::copy(coff.begin(), coff.end(), hco);
            int *d_coff = dptr<int>(D.coff, (size_t)nown + 1);
            copy_from_host(d_coff, hco, sizeof(int) * (nown + 1), s);
            int *d_cells = dptr<int>(D.cells, (size_t)n_owned_cells);
            k_segments<<<(int)segs.size(), 256, 0, s>>>(d_segs, land, d_cells);
            ClusterRec *d_rec = dptr<ClusterRec>(D.rec, (size_t)nown);
            launch_cluster_stats(d_coff, d_cells, nown, g, d_poly, npoly, min_len, d_rec, s);
            ClusterRec *hr = hptr<ClusterRec>(D.h_rec, (size_t)nown);
            copy_to_host(hr, d_rec, sizeof(ClusterRec) * nown, s);
            AOS_HIP(hipStreamSynchronize(s));
            std::vector<ClusterRec> orec(hr, hr + nown);
            std::vector<int> flagged;
            for (int j = 0; j < nown; ++j)
                if (orec[j].flags & 2) { flagged.push_back(j); replayed[j] = 1; }
            if (!flagged.empty()) {   // the owned flagged clusters' cells in one copy, then the exact replays
                // (from a 16-byte boundary in whole 16-byte words: the copy kernel's uint4 form; d_cells has slack)
                const int lo = coff[flagged.front()] & ~3, hi = (coff[flagged.back() + 1] + 3) & ~3;
                int *hc = hptr<int>(D.h_cells, (size_t)(hi - lo));
                copy_to_host(hc, d_cells + lo, sizeof(int) * (size_t)(hi - lo), s);
                AOS_HIP(hipStreamSynchronize(s));
                std::vector<ReplayJob> jobs;
                for (int j : flagged) jobs.push_back({j, hc + (coff[j] - lo), orec[j].n});
                const auto tr0 = clk::now();
                replay_clusters(jobs, g, hp, npoly, min_len, orec.data());
                st.ms_replay = std::chrono::duration<float, std::milli>(clk::now() - tr0).count();
                st.n_replayed_here = (int)flagged.size();
            }
            for (int j = 0; j < nown; ++j) lrec[mine_l[j]] = orec[j];
        }
        // ---- the owners' records to every rank (sizes known: the plan)
        std::vector<uint64_t> rsz((size_t)world, 0);
        for (int l = 0; l < nlong; ++l) rsz[owner[l]] += sizeof(OwnedOut);
        OwnedOut *ho = hptr<OwnedOut>(D.h_out, (size_t)std::max(nown, 1));
        for (int j = 0; j < nown; ++j) ho[j] = OwnedOut{mine_l[j], replayed[j], lrec[mine_l[j]]};
        OwnedOut *ha = hptr<OwnedOut>(D.h_tab, (size_t)nlong);
        gather_bytes(fc, s, ho, false, rsz, ha, false, D.h_recv);
        int n_bfs_long = 0;   // (a replay clears the record's flag: the owners say which they replayed)
        for (int k = 0; k < nlong; ++k) {
            lrec[ha[k].l] = ha[k].r;
            n_bfs_long += ha[k].replayed;
        }
        pre.n_bfs = n_bfs_long;
    }
    const auto t2 = clk::now();
    st.n_pieces = npieces;
    st.n_border = nb;
    st.ms_local = std::chrono::duration<float, std::milli>(t1 - t0).count();
    st.ms_global = std::chrono::duration<float, std::milli>(t2 - t1).count();
    if (me != root) return;

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
