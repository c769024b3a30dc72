// Clusters -> tree rows -> Voronoi seeds (seed_gen:970-1083, 1258-1512, 1730-2268) on gfx950.
//
// a8 clusterOccupiedCells is a raster-order scan + FIFO BFS. Its outputs depend on the BFS
// order only through (i) float sums of cell coordinates and (ii) "first strict maximum"
// tie-breaks. The GPU computes the partition with union-find (root = minimum raster index =
// the reference's discovery order) and every per-cluster statistic order-free, together with a
// certificate: integer coordinate sums <= 2^24 (so every float partial sum is exact in any
// order) and no ties in the three argmax searches. A cluster without the certificate is
// replayed exactly (FIFO BFS with the reference's neighbour order) on the host, in parallel over
// such clusters (host_bfs_replay).
//
// Greedy first-come de-duplications (seeds within 0.5 m) are the lexicographically-first
// maximal independent set of the conflict graph in candidate order; the GPU builds the graph
// with a uniform hash and decides the set in rounds (a candidate is kept once every earlier
// conflicting candidate is removed, removed once one of them is kept).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <stdexcept>

#include "cluster_dev.h"
#include "cluster_seed.h"
#include "dev_prims_device.h"
#include "dev_wave.h"

namespace aos {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------ foreground = skeleton inside polygon
// The foreground words and their popcounts (k_scan_1p turns them into the words' offsets). (Round 5 measured the
// scan fused into this kernel with a decoupled look-back: 117 us instead of 18 + 9 at C2 -- the 4096 one-wave
// blocks waited on their predecessors' work, so few ran at once; the fusion stays only where blocks are
// uniform and short, k_facet_count.)
__global__ void k_fg(const uint64_t *skel, uint64_t *fg, int *cnt, GridC g, const double *poly, int np) {
    __shared__ double xc[kRowCrossMax];
    __shared__ int nxc;
    const int c = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    const double wy = y < g.H ? cell_world(g.oy, y, g.res) : 0.0;
    const bool rowwise = row_crossings(poly, np, wy, xc, &nxc);   // (block-uniform; synchronises)
    if (c >= g.WW || y >= g.H) return;
    size_t wi = (size_t)y * g.WW + c;
    uint64_t w = skel[wi], o = 0;
    if (rowwise && __popcll(w) >= kPipWordMin) {
        o = w & pip_row_word(g.ox, g.res, c * 64, xc, nxc);
    } else {
        while (w) {
            int b = __ffsll((long long)w) - 1;
            w &= w - 1;
            int x = c * 64 + b;
            const double wx = cell_world(g.ox, x, g.res);
            if (rowwise ? pip_row(wx, xc, nxc) : d_pip(wx, wy, poly, np)) o |= 1ull << b;
        }
    }
    fg[wi] = o;
    cnt[wi] = __popcll(o);
}

// (parent != nullptr: also the union-find's initial parents, parent[k] = k; zero != nullptr: *zero = 0, the
// cross-chunk link count of k_ccl_local, without a fill launch)
__global__ void k_fg_list(const uint64_t *fg, const int *off, int *list, GridC g, int *parent, int *zero) {
    int c = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (zero && c == 0 && y == 0) *zero = 0;
    if (c >= g.WW || y >= g.H) return;
    size_t wi = (size_t)y * g.WW + c;
    uint64_t w = fg[wi];
    int k = off[wi];
    while (w) {
        int b = __ffsll((long long)w) - 1;
        w &= w - 1;
        if (parent) parent[k] = k;
        list[k++] = y * g.W + c * 64 + b;
    }
}

__device__ __forceinline__ int fg_index(const uint64_t *fg, const int *off, const GridC &g, int x, int y) {
    if (x < 0 || y < 0 || x >= g.W || y >= g.H) return -1;
    size_t wi = (size_t)y * g.WW + (x >> 6);
    uint64_t w = fg[wi];
    int b = x & 63;
    if (!((w >> b) & 1ull)) return -1;
    return off[wi] + __popcll(w & ((1ull << b) - 1));
}

// ------------------------------------------------------------------ union-find CCL (8-connectivity)
__global__ void k_ccl_init(int *parent, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) parent[i] = i;
}
__global__ void k_ccl_union(const int *list, int n, const uint64_t *fg, const int *off, GridC g, int *parent) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int p = list[i], y = p / g.W, x = p - y * g.W;
    const int ndx[4] = {-1, 0, 1, -1}, ndy[4] = {-1, -1, -1, 0};
    for (int k = 0; k < 4; ++k) {
        int j = fg_index(fg, off, g, x + ndx[k], y + ndy[k]);
        if (j >= 0) uf_union(parent, i, j);
    }
}
// Block-local CCL (round 4): the list is in raster order, so workgroup b's chunk of kCclChunk consecutive
// cells spans a few grid rows and nearly every 8-neighbour link stays inside it. The chunk is labelled by
// union-find in LDS (LDS-latency walks instead of global ones past the XCD's L2); parent[i] becomes the
// global index of its chunk root; links into an earlier chunk are appended to a cross-edge list that
// k_ccl_cross then unions globally (C2: ~10^4 edges instead of ~10^6 global unions). The smaller index is
// always the root, as in k_ccl_union, so the roots and the flattened labels are the same.
// chunk and block size (AOS_CCL_CHUNK / AOS_CCL_TB override them for A/B runs)
static int ccl_chunk() { static const int v = [] { const char *e = getenv("AOS_CCL_CHUNK"); return e ? std::max(64, std::min(16384, atoi(e))) : 2048; }(); return v; }
// (1024 threads: k_ccl_local 77 -> 52 us per C2 frame against 256, 60 with 512; 1024-cell chunks 58, 4096 with 1024
// threads 69: profiles/r05j_ccl_ab.txt)
static int ccl_tb() { static const int v = [] { const char *e = getenv("AOS_CCL_TB"); return e ? std::max(64, std::min(1024, atoi(e))) / 64 * 64 : 1024; }(); return v; }
// capacity of k_ccl_local's cross-chunk link list (AOS_DEBUG_CCL_ECAP, read per call: tests force the overflow
// fallback of k_ccl_cross with a tiny list)
static int ccl_edge_cap(int nf) {
    const char *e = getenv("AOS_DEBUG_CCL_ECAP");
    return e ? std::max(2, atoi(e)) : std::max(4096, nf / 4);
}
constexpr int kCclBatch = 2;        // k_ccl_local: cells per thread whose neighbour lookups are in flight together
constexpr int kCclEdgeLds = 1024;   // k_ccl_local: cross-chunk links gathered per block before the global append
// Root of x with path halving: x is pointed at its grandparent as the walk passes (a parent always has the
// smaller index, so the grandparent is an ancestor and no cycle can form; a root is never written: only entries
// already read as non-roots are). The chunk's unions arrive in no particular order along the skeleton's lines,
// and without halving their chains grew to hundreds of links that every later find walked again. (The global
// union-find keeps its read-only walks: agent-scope stores past the XCD's L2 cost more than they saved, round 4.)
__device__ __forceinline__ int lds_find(int *lp, int x) {
    for (;;) {
        const int p = __hip_atomic_load(&lp[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (p == x) return x;
        const int g = __hip_atomic_load(&lp[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (g == p) return p;
        __hip_atomic_store(&lp[x], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        x = g;
    }
}
__device__ __forceinline__ void lds_union(int *lp, int i, int j) {
    int a = lds_find(lp, i), b = lds_find(lp, j);
    while (a != b) {
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = atomicCAS(&lp[a], a, b);
        if (old == a) break;
        a = lds_find(lp, old);
        b = lds_find(lp, b);
    }
}
struct IMaxOp { __device__ int operator()(int a, int b) const { return a > b ? a : b; } };
// Horizontal runs are labelled before any union (round 6): lp[i] = the first cell of i's run of x-adjacent cells inside
// the chunk, by a max-scan of the run starts (each thread a contiguous segment; DPP wave scan, one barrier). The orchard
// skeleton is long horizontal lines, and linking each cell to its left neighbour by concurrent unions built chains as
// long as the runs (hundreds of cells) that the finds then walked with path halving: C2 50 us, C3 161 us per frame
// (profiles/r06/r06z_kt*_summary.txt). A run's start is its smallest index, so the forest keeps the invariant of the
// unions (a parent has the smaller index) and every component's root is still its smallest cell: the labels are
// unchanged. Only the three upper links go through lookups and unions; a chunk's first cell links left into the
// previous chunk through the cross-edge list, as before. The cross-chunk links (a line's cells link up into the same
// line's previous grid row, ~10^4 links at C3) gather in LDS and reach the global list with one atomic per block: one
// global atomic per link on the one counter had serialised the launch (in-kernel s_memrealtime stamps per block: C3
// blocks waited up to 100 us in their first phase behind it). With batches of 2 cells (42 VGPRs, two 1024-thread
// blocks per CU): C2 50 -> 13 us, C3 161 -> 23 us per frame; chunks of 4096 or 512-thread blocks were slower at C2.
__global__ __launch_bounds__(1024) void k_ccl_local(const int *list, int n, const uint64_t *fg, const int *off, GridC g,
                                                    int *parent, int2 *edges, int *n_edges, int cap, int chunk) {
    extern __shared__ int lp[];   // [chunk]
    __shared__ int wmax[16];
    __shared__ int2 s_edge[kCclEdgeLds];
    __shared__ int s_ne, s_ebase;
    const int base = blockIdx.x * chunk, m = min(chunk, n - base), nt = blockDim.x, tid = threadIdx.x;
    {
        const int S = (m + nt - 1) / nt, s0 = tid * S;
        int run = -1;
        for (int k = 0; k < S; ++k) {
            const int i = s0 + k;
            if (i >= m) break;
            const int p = list[base + i];
            const bool start = i == 0 || p % g.W == 0 || list[base + i - 1] != p - 1;
            if (start) run = i;
            lp[i] = run;
        }
        const int before = wave_scan_excl(run, -1, IMaxOp());
        if ((tid & 63) == 63) wmax[tid >> 6] = max(before, run);
        __syncthreads();
        int carry = before;
        for (int w = 0; w < (tid >> 6); ++w) carry = max(carry, wmax[w]);
        for (int k = 0; k < S; ++k) {
            const int i = s0 + k;
            if (i >= m) break;
            if (lp[i] < 0) lp[i] = carry;   // (cell 0 starts a run: carry >= 0 here)
        }
        if (tid == 0) s_ne = 0;
    }
    __syncthreads();
    // The cross-chunk links gather in LDS and go to the global list with one atomic per block (round 6: one global
    // atomic per link on one counter serialised the C3 launch, ~10^4 links)
    auto cross = [&](int a, int b) {
        const int e = atomicAdd(&s_ne, 1);
        if (e < kCclEdgeLds) {
            s_edge[e] = make_int2(a, b);
        } else {
            const int ge = atomicAdd(n_edges, 1);
            if (ge < cap) edges[ge] = make_int2(a, b);
        }
    };
    if (tid == 0 && base > 0) {   // the chunk's first cell and its left neighbour in the previous chunk
        const int p = list[base];
        if (p % g.W != 0 && list[base - 1] == p - 1) cross(base, base - 1);
    }
    const int ndx[3] = {-1, 0, 1};   // (the row above: raster predecessors, their indices < base + i)
    // kCclBatch cells per thread at a time, their 3 x kCclBatch neighbour lookups issued together (the fg words,
    // then the offsets of the set bits) before any union: round 4 walked each cell's lookups as a chain of
    // dependent global load pairs between LDS unions, so the kernel waited on load latency cell after cell
    constexpr int B = kCclBatch;
    const int S = (m + nt - 1) / nt, s0 = tid * S, s1 = min(s0 + S, m);   // (the segment of the run scan)
    for (int i0 = s0; i0 < s1; i0 += B) {
        int wi[B][3], bit[B][3], jj[B][3];
        uint64_t w[B][3];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int i = i0 + b < s1 ? i0 + b : m;
            const int p = i < m ? list[base + i] : 0, y = p / g.W, x = p - y * g.W;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int nx = x + ndx[k], ny = y - 1;
                const bool ok = i < m && nx >= 0 && ny >= 0 && nx < g.W;
                wi[b][k] = ok ? ny * g.WW + (nx >> 6) : 0;
                bit[b][k] = nx & 63;
                w[b][k] = ok ? fg[wi[b][k]] : 0ull;
            }
        }
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint64_t v = w[b][k];
                jj[b][k] = ((v >> bit[b][k]) & 1ull) ? off[wi[b][k]] + __popcll(v & ((1ull << bit[b][k]) - 1)) : -1;
            }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int i = i0 + b;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int j = jj[b][k];
                if (j < 0) continue;
                if (j >= base) lds_union(lp, i, j - base);
                else cross(base + i, j);
            }
        }
    }
    __syncthreads();
    const int nl = min(s_ne, kCclEdgeLds);
    if (tid == 0 && nl) s_ebase = atomicAdd(n_edges, nl);
    for (int i = tid; i < m; i += nt) parent[base + i] = base + lds_find(lp, i);
    __syncthreads();
    for (int k = tid; k < nl; k += nt)
        if (s_ebase + k < cap) edges[s_ebase + k] = s_edge[k];
}
// The cross-chunk links, unioned globally; when the list overflowed (never at C1-C4) every link of every cell
// again instead (the fallback, in the same launch: round 4's separate k_ccl_union_if returned at once in
// every frame)
__global__ void k_ccl_cross(const int2 *edges, const int *n_edges, int cap, int *parent, const int *list, int n,
                            const uint64_t *fg, const int *off, GridC g) {
    const int stride = gridDim.x * blockDim.x;
    if (*n_edges <= cap) {
        const int ne = *n_edges;
        for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += stride) uf_union(parent, edges[e].x, edges[e].y);
        return;
    }
    const int ndx[4] = {-1, 0, 1, -1}, ndy[4] = {-1, -1, -1, 0};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int p = list[i], y = p / g.W, x = p - y * g.W;
        for (int k = 0; k < 4; ++k) {
            const int j = fg_index(fg, off, g, x + ndx[k], y + ndy[k]);
            if (j >= 0) uf_union(parent, i, j);
        }
    }
}
__global__ void k_ccl_flatten(int *parent, int *is_root, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int x = i;   // (a read-only walk: a halving store into another thread's entry could land after its root)
    for (int p; (p = ld_parent(parent, x)) != x;) x = p;
    __hip_atomic_store(&parent[i], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_root[i] = (x == i);
}
// parent[i] := the root; rank[r] = the cluster id of root r (the roots' raster order = the reference's discovery
// order), rank[n] = the number of clusters
static void ccl_flatten_rank(LookBackScratch &lb, int *parent, int *is_root, int *rank, int n, hipStream_t s) {
    k_ccl_flatten<<<cdiv(n, 256), 256, 0, s>>>(parent, is_root, n);
    scan_1p(lb, is_root, rank, n, false, s);
}
// Counting sort of the foreground cells by cluster id (cluster = rank of the cell's root among the roots,
// i.e. raster order of first cells): per cell its id and its rank inside the cluster. A cluster holds
// thousands of cells and the list is in raster order, so a block's 256 cells touch few clusters: they are
// counted in an LDS table first and each block adds one total per cluster to the global counter.
// The order inside a cluster is the blocks' atomics order; k_cluster_stats is order-free and the BFS
// replay starts from the smallest cell.
constexpr int kClTB = 256, kClSlots = 512;
__global__ __launch_bounds__(kClTB) void k_cluster_count(const int *parent, const int *rank, int n, int *cid_of, int *crank,
                                                       int *cl_cnt) {
    __shared__ int key[kClSlots], cnt[kClSlots];
    const int tid = threadIdx.x, i = blockIdx.x * kClTB + tid;
    for (int k = tid; k < kClSlots; k += kClTB) { key[k] = -1; cnt[k] = 0; }
    __syncthreads();
    int cid = -1, slot = 0, lr = 0;
    if (i < n) {
        cid = rank[parent[i]];
        cid_of[i] = cid;
        slot = (int)(((unsigned)cid * 2654435761u) >> 23) & (kClSlots - 1);
        for (;;) {   // (at most kClTB distinct ids per block: a free slot always exists)
            const int old = atomicCAS(&key[slot], -1, cid);
            if (old == -1 || old == cid) break;
            slot = (slot + 1) & (kClSlots - 1);
        }
        lr = atomicAdd(&cnt[slot], 1);
    }
    __syncthreads();
    for (int k = tid; k < kClSlots; k += kClTB)
        if (key[k] >= 0) cnt[k] = atomicAdd(&cl_cnt[key[k]], cnt[k]);   // the block's base in the cluster
    __syncthreads();
    if (i < n) crank[i] = cnt[slot] + lr;
}
__global__ void k_cluster_scatter(const int *list, const int *cid_of, const int *crank, const int *off, int n, int *cells) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) cells[off[cid_of[i]] + crank[i]] = list[i];
}

// ------------------------------------------------------------------ per-cluster statistics
struct StatArgs {
    const int *off, *cells;
    const int *list;          // fg list (raster order); list[root] = first raster cell of a cluster
    int n_clusters;
    GridC g;
    const double *poly; int np;
    float min_length;
    ClusterRec *rec;
    ClusterRec *hrec;         // nullable: pinned host copy of rec, stored by the same threads
    int lds_cap;              // clusters of at most this many cells are read from global memory once (kStatLds or 0)
};

struct MaxOp { template <class T> __device__ T operator()(T a, T b) const { return a > b ? a : b; } };
struct MinOp { template <class T> __device__ T operator()(T a, T b) const { return a < b ? a : b; } };
struct AddOp { template <class T> __device__ T operator()(T a, T b) const { return a + b; } };

// The strict maximum of a pass (seed_gen:1354-1399's "first cell with a strictly larger value"): the largest value d,
// how many cells reach it and the smallest of them. Order-free: the pass's cells in any order give the same triple.
struct ArgMax {
    double d; int c, a;
    __device__ void add(double v, int p) {
        if (v > d) { d = v; c = 1; a = p; }
        else if (v == d) { ++c; a = min(a, p); }
    }
    template <int CTRL, int RM> __device__ ArgMax dpp(const ArgMax &old) const {
        return ArgMax{dpp_f64<CTRL, RM>(old.d, d), dpp_i32<CTRL, RM>(old.c, c), dpp_i32<CTRL, RM>(old.a, a)};
    }
    __device__ ArgMax lane63() const { return ArgMax{lane63_f64(d), lane63_i32(c), lane63_i32(a)}; }
};
struct ArgMaxOp {
    __device__ ArgMax operator()(const ArgMax &x, const ArgMax &y) const {
        if (y.d > x.d) return y;
        if (x.d > y.d) return x;
        return ArgMax{x.d, x.c + y.c, min(x.a, y.a)};
    }
};
__device__ constexpr ArgMax kArgMaxNone{-1.0, 0, INT_MAX};

__device__ __forceinline__ double2 cell_wxy(const GridC &g, int x, int y) {   // cell_w of the cell (x, y)
    return make_double2((double)cell_world(g.ox, x, g.res), (double)cell_world(g.oy, y, g.res));
}

// One workgroup per cluster, three passes over its cells (a fourth in the rare fallback of the second endpoint):
//  1. from global memory (four loads in flight per thread), kept in LDS as packed (y << 16 | x): the coordinate sums,
//     and min over the keys (x, p), (W - 1 - x, p), (y, p), (H - 1 - y, p) -- the bounding box, the extreme cells of
//     the length bound and (the smallest p) the first cell at once;
//  2. the length candidates and the first endpoint's strict maximum (ArgMax: max, count, smallest cell) around the
//     centre, computed for every cluster (it is used only for rows: seed_gen:1354-1367);
//  3. the second endpoint's strict maximum (seed_gen:1369-1385).
// Reductions run on DPP row moves (dev_wave.h), one barrier each. Before: one pass per maximum and per argument, every
// pass from global memory with a division by W per cell, 18 three-barrier shuffle reductions; 49.7 us per C2 frame
// (round-6 start, profiles/r06/r06t_kt_summary.txt), 36.7 us with the LDS copy alone (r06y), where each pass cost
// ~3-4 us of which ~2 us was its ds_bpermute reduction chains (in-kernel s_memrealtime stamps per pass).
// Clusters beyond the LDS (or grids of 65536 columns or rows and more: lds_cap 0) read global memory in every pass.
constexpr int kStatTB = 512, kStatLds = 16384;   // 64 KB of cells
__global__ __launch_bounds__(kStatTB) void k_cluster_stats(StatArgs A) {
    constexpr int NW = kStatTB / 64;
    __shared__ unsigned cc[kStatLds];
    __shared__ long long s_l[6][NW];
    __shared__ ArgMax s_m[2][NW];
    __shared__ int s_i[NW];
    __shared__ int cand[2048];
    __shared__ int ncand;
    const int cid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int b = A.off[cid], e = A.off[cid + 1], n = e - b;
    const GridC &g = A.g;
    const int W = g.W, H = g.H;
    const bool lds = n <= A.lds_cap;
    auto xy_at = [&](int k, int &x, int &y) {
        if (lds) {
            const unsigned v = cc[k];
            x = (int)(v & 0xffffu); y = (int)(v >> 16);
        } else {
            const int p = A.cells[b + k];
            y = p / W; x = p - y * W;
        }
    };
    auto key = [](int hi, int p) { return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)p); };
    // ---- pass 1
    long long sx = 0, sy = 0;
    long long kx0 = LLONG_MAX, kx1 = LLONG_MAX, ky0 = LLONG_MAX, ky1 = LLONG_MAX;
    for (int k0 = tid; k0 < n; k0 += 4 * kStatTB) {
        int pv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u * kStatTB;
            pv[u] = k < n ? A.cells[b + k] : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int p = pv[u];
            if (p < 0) continue;
            const int y = p / W, x = p - y * W;
            if (lds) cc[k0 + u * kStatTB] = (unsigned)x | ((unsigned)y << 16);
            sx += x; sy += y;
            kx0 = min(kx0, key(x, p)); kx1 = min(kx1, key(W - 1 - x, p));
            ky0 = min(ky0, key(y, p)); ky1 = min(ky1, key(H - 1 - y, p));
        }
    }
    if (tid == 0) ncand = 0;
    sx = wave_reduce(sx, 0ll, AddOp()); sy = wave_reduce(sy, 0ll, AddOp());
    kx0 = wave_reduce(kx0, LLONG_MAX, MinOp()); kx1 = wave_reduce(kx1, LLONG_MAX, MinOp());
    ky0 = wave_reduce(ky0, LLONG_MAX, MinOp()); ky1 = wave_reduce(ky1, LLONG_MAX, MinOp());
    if (lane == 0) {
        s_l[0][wid] = sx; s_l[1][wid] = sy; s_l[2][wid] = kx0; s_l[3][wid] = kx1; s_l[4][wid] = ky0; s_l[5][wid] = ky1;
    }
    __syncthreads();   // (also publishes cc and ncand)
    sx = s_l[0][0]; sy = s_l[1][0]; kx0 = s_l[2][0]; kx1 = s_l[3][0]; ky0 = s_l[4][0]; ky1 = s_l[5][0];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        sx += s_l[0][w]; sy += s_l[1][w];
        kx0 = min(kx0, s_l[2][w]); kx1 = min(kx1, s_l[3][w]); ky0 = min(ky0, s_l[4][w]); ky1 = min(ky1, s_l[5][w]);
    }
    const int mnx = (int)(kx0 >> 32), mxx = W - 1 - (int)(kx1 >> 32), mny = (int)(ky0 >> 32), mxy = H - 1 - (int)(ky1 >> 32);
    const int first = (int)(unsigned)ky0;   // the smallest p has the smallest y
    // ---- max pairwise squared distance (cluster.length, seed_gen:1063-1073), pruned exactly:
    // LB = d^2 between the cells of extreme x / extreme y; a cell can belong to a farther pair only
    // if its distance to the farthest bbox corner reaches LB.
    auto d2p = [&](int p, int q) {
        int py = p / W, px = p - py * W, qy = q / W, qx = q - qy * W;
        int dx = px - qx, dy = py - qy;
        return dx * dx + dy * dy;
    };
    const int LB = max(d2p((int)(unsigned)kx0, (int)(unsigned)kx1), d2p((int)(unsigned)ky0, (int)(unsigned)ky1));
    ClusterRec r{};
    r.sx = sx; r.sy = sy; r.n = n;
    r.bx0 = mnx; r.by0 = mny; r.bx1 = mxx; r.by1 = mxy; r.first = first;
    r.cx = (float)sx / (float)n;       // sum_x / cells.size() (float / float)
    r.cy = (float)sy / (float)n;
    const float cwx = (float)(g.ox + (double)(r.cx * g.res)), cwy = (float)(g.oy + (double)(r.cy * g.res));
    const double2 ctr = make_double2(cwx, cwy);
    // ---- pass 2
    ArgMax m1 = kArgMaxNone;   // |wp - centre|^2
    for (int k = tid; k < n; k += kStatTB) {
        int x, y;
        xy_at(k, x, y);
        const int dxm = max(x - mnx, mxx - x), dym = max(y - mny, mxy - y);
        if (dxm * dxm + dym * dym >= LB) {
            const int s = atomicAdd(&ncand, 1);
            if (s < 2048) cand[s] = y * W + x;
        }
        const double2 w = cell_wxy(g, x, y);
        const double dx = w.x - ctr.x, dy = w.y - ctr.y;
        m1.add(dx * dx + dy * dy, y * W + x);
    }
    m1 = wave_reduce(m1, kArgMaxNone, ArgMaxOp());
    if (lane == 0) s_m[0][wid] = m1;
    __syncthreads();
    int maxd2 = LB;
    const int nc = ncand;
    if (nc <= 2048) {
        for (int i = 0; i < nc; ++i)
            for (int j = i + 1 + tid; j < nc; j += kStatTB) maxd2 = max(maxd2, d2p(cand[i], cand[j]));
    } else {  // too many candidates: exact brute force over all pairs
        for (int i = b; i < e; ++i)
            for (int k = i + 1 + tid; k < e; k += kStatTB) maxd2 = max(maxd2, d2p(A.cells[i], A.cells[k]));
    }
    maxd2 = wave_reduce(maxd2, INT_MIN, MaxOp());
    if (lane == 0) s_i[wid] = maxd2;
    __syncthreads();
    m1 = s_m[0][0];
    maxd2 = s_i[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) { m1 = ArgMaxOp()(m1, s_m[0][w]); maxd2 = max(maxd2, s_i[w]); }
    r.maxd2 = maxd2;
    r.flags = 0;
    const bool exact_sums = sx <= (1ll << 24) && sy <= (1ll << 24);
    r.length = (float)(sqrt((double)maxd2) * (double)g.res);
    bool needs_bfs = !exact_sums;
    bool row = false;
    if (r.length >= A.min_length) {
        r.center = ctr;
        row = d_pip(cwx, cwy, A.poly, A.np);
    }
    if (row && !needs_bfs) {   // (uniform over the block)
        // first endpoint: first cell with strictly maximal |wp - centre|^2 (seed_gen:1354-1367)
        const int arg = m1.a;
        if (!(m1.d > 0.0) || m1.c != 1) needs_bfs = true;
        if (!needs_bfs) {
            const double2 wf = cell_w(g, arg);
            double fdx = wf.x - r.center.x, fdy = wf.y - r.center.y;
            double z = fdx * fdx + fdy * fdy, s = sqrt(z);
            const double fx = fdx / s, fy = fdy / s;  // first_direction = diff.normalized()
            // ---- pass 3: second endpoint, dot(normalized(diff), first_dir) < 0, strictly maximal (seed_gen:1369-1385)
            ArgMax m2 = kArgMaxNone;
            for (int k = tid; k < n; k += kStatTB) {
                int x, y;
                xy_at(k, x, y);
                const int p = y * W + x;
                if (p == arg) continue;
                const double2 w = cell_wxy(g, x, y);
                double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
                double nx = dx, ny = dy;
                if (d2 > 0.0) { double q = sqrt(d2); nx = dx / q; ny = dy / q; }
                if (nx * fx + ny * fy < 0.0) m2.add(d2, p);
            }
            m2 = wave_reduce(m2, kArgMaxNone, ArgMaxOp());
            if (lane == 0) s_m[1][wid] = m2;
            __syncthreads();
            m2 = s_m[1][0];
#pragma unroll
            for (int w = 1; w < NW; ++w) m2 = ArgMaxOp()(m2, s_m[1][w]);
            if (!(m2.d > 0.0)) {  // farthest from the first endpoint (seed_gen:1387-1399)
                __syncthreads();   // (s_m[1] is read above and written again below)
                m2 = kArgMaxNone;
                for (int k = tid; k < n; k += kStatTB) {
                    int x, y;
                    xy_at(k, x, y);
                    const int p = y * W + x;
                    if (p == arg) continue;
                    const double2 w = cell_wxy(g, x, y);
                    double dx = w.x - wf.x, dy = w.y - wf.y;
                    m2.add(dx * dx + dy * dy, p);
                }
                m2 = wave_reduce(m2, kArgMaxNone, ArgMaxOp());
                if (lane == 0) s_m[1][wid] = m2;
                __syncthreads();
                m2 = s_m[1][0];
#pragma unroll
                for (int w = 1; w < NW; ++w) m2 = ArgMaxOp()(m2, s_m[1][w]);
            }
            if (!(m2.d > 0.0) || m2.c != 1) needs_bfs = true;  // (fallback with max 0 keeps index 0 -> BFS replay)
            r.start = wf;
            if (!needs_bfs) r.end = cell_w(g, m2.a);
        }
    }
    r.flags = (row ? 1 : 0) | (needs_bfs ? 2 : 0);
    if (tid == 0) {
        A.rec[cid] = r;
        if (A.hrec) A.hrec[cid] = r;
    }
}

// clusters read from global memory once when they fit the LDS (AOS_DEBUG_STATS_LDS=0, read per call: every pass
// from global memory, the path of larger clusters and of grids of 65536 columns or rows and more)
static int stats_lds_cap(const GridC &g) {
    const char *e = getenv("AOS_DEBUG_STATS_LDS");
    if (e && atoi(e) == 0) return 0;
    return g.W <= 65536 && g.H <= 65536 ? kStatLds : 0;
}

void launch_cluster_stats(const int *off, const int *cells, int n_clusters, const GridC &g, const double *poly, int np,
                          float min_length, ClusterRec *rec, hipStream_t s, ClusterRec *hrec) {
    if (n_clusters <= 0) return;
    StatArgs A{off, cells, nullptr, n_clusters, g, poly, np, min_length, rec, hrec, stats_lds_cap(g)};
    k_cluster_stats<<<n_clusters, kStatTB, 0, s>>>(A);
    AOS_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ rays

// raycastToOccupiedCell seed_gen:1730-1771 on the frameless skeleton
// Marching loops are latency chains of dependent skeleton lookups; the sample positions are not
// (cur += step / cx += dx*step depend only on the arithmetic), so each thread computes kLook
// positions ahead with the reference's exact accumulation, issues their lookups together and then
// resolves them in order.
constexpr int kLook = 16;

__device__ bool d_raycast(const uint64_t *skel, const GridC &g, double sx, double sy, double dx, double dy, double maxd,
                          double &hx, double &hy) {
    const double step = (double)g.res * 0.5;
    const int max_steps = (int)(maxd / step);
    double cx = sx, cy = sy;
    for (int i0 = 0; i0 < max_steps; i0 += kLook) {
        double px[kLook], py[kLook];
        bool hit[kLook];
#pragma unroll
        for (int j = 0; j < kLook; ++j) {
            cx += dx * step;
            cy += dy * step;
            px[j] = cx; py[j] = cy;
        }
#pragma unroll
        for (int j = 0; j < kLook; ++j) {
            // every lookup is issued (clamped cell), the loop conditions only mask the result
            double ddx = px[j] - sx, ddy = py[j] - sy;
            double dist = sqrt(ddx * ddx + ddy * ddy);
            float fx = (float)px[j], fy = (float)py[j];
            float rel_x = (float)(((double)fx - g.ox) / (double)g.res);
            float rel_y = (float)(((double)fy - g.oy) / (double)g.res);
            float flx = floorf(rel_x), fly = floorf(rel_y);
            int gx = !(flx > 0.0f) ? 0 : (flx >= (float)(g.W - 1) ? g.W - 1 : (int)flx);
            int gy = !(fly > 0.0f) ? 0 : (fly >= (float)(g.H - 1) ? g.H - 1 : (int)fly);
            hit[j] = (i0 + j < max_steps && !(dist < 1.0)) && bit_at(skel, g.WW, gx, gy);
        }
#pragma unroll
        for (int j = 0; j < kLook; ++j)
            if (hit[j]) { hx = px[j]; hy = py[j]; return true; }
    }
    return false;
}

// virtual-seed candidates of generateVirtualSeeds (seed_gen:2008-2263): per base seed i of a row,
// slot 3*(i-1) + {0: base, 1: perp_dir1 ray seed, 2: perp_dir2 ray seed}
__global__ void k_virtual_candidates(const RowDev *rows, int n_rows, int n_slots, const uint64_t *skel, GridC g,
                                     const double *poly, int np, double2 *cand, int *ok) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    int lo = 0, hi = n_rows - 1;  // row whose slot range contains s
    while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (rows[mid].slot0 <= s) lo = mid; else hi = mid - 1; }
    const RowDev R = rows[lo];
    const int local = s - R.slot0, i = local / 3 + 1, type = local - (i - 1) * 3;
    double dx = R.ex - R.sx, dy = R.ey - R.sy;
    double nrm = sqrt(dx * dx + dy * dy);
    double rdx = dx / nrm, rdy = dy / nrm;
    double t = (double)i / (R.k + 1);
    double bx = R.sx + t * dx, by = R.sy + t * dy;
    if (type == 0) { cand[s] = make_double2(bx, by); ok[s] = 1; return; }
    double pdx = type == 1 ? -rdy : rdy, pdy = type == 1 ? rdx : -rdx;
    const double maxd = 4.0;
    double hx, hy, sx_, sy_;
    if (d_raycast(skel, g, bx, by, pdx, pdy, maxd, hx, hy)) { sx_ = hx; sy_ = hy; }
    else { sx_ = bx + pdx * maxd; sy_ = by + pdy * maxd; }
    cand[s] = make_double2(sx_, sy_);
    ok[s] = d_pip(sx_, sy_, poly, np) ? 0 : 1;
}

struct RayAngles { double cs[3], sn[3]; int pos_branch[3]; };  // 0, -90, +90 degrees

// castRayFromEndpoint seed_gen:1774-1891 + the filters of generateRayPointsFromEndpoints :1941-1961.
// One wave per ray, 64 consecutive march steps per iteration. The reference's distance sequence
// (current_dist = 1.0; current_dist += 0.1, :1833-1871) is the same for every ray, so the host
// tabulates it once with the same double adds (cur_tab[i] = value at step i; the table ends with the
// first value > absolute_max_distance). Each lane evaluates its step with an unconditional (clamped)
// skeleton load; the first lane with an event (loop end, left the grid, occupied cell) decides.
// (k_endpoint_candidates folded in: the first ray block of row r also writes the row's two endpoint seed
// candidates, start then end, into ecand / eok [2r, 2r + 1] -- seed_gen:1451-1496's order)
__global__ __launch_bounds__(64) void k_endpoint_rays(const RowDev *rows, int n_rows, const uint64_t *skel, GridC g,
                                                      RayAngles ang, const double *poly, int np, const double *cur_tab,
                                                      int n_tab, double2 *cand, int *ok, double2 *ecand, int *eok) {
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= n_rows * 6) return;
    const RowDev R = rows[s / 6];
    if (s % 6 == 0 && lane < 2) {
        ecand[2 * (s / 6) + lane] = lane ? make_double2(R.ex, R.ey) : make_double2(R.sx, R.sy);
        eok[2 * (s / 6) + lane] = 1;
    }
    const int k = s % 6, a = k % 3;
    double stx = k < 3 ? R.sx : R.ex, sty = k < 3 ? R.sy : R.ey;
    double otx = k < 3 ? R.ex : R.sx, oty = k < 3 ? R.ey : R.sy;
    double ex = otx - stx, ey = oty - sty;
    double dist = sqrt(ex * ex + ey * ey);
    if (dist < 1e-6) { ex = 1.0; ey = 0.0; }
    else { ex = ex / dist; ey = ey / dist; }
    double ox_ = -ex, oy_ = -ey, px0 = -ey, py0 = ex;
    double rx, ry;
    if (ang.pos_branch[a]) { rx = ang.cs[a] * ox_ + ang.sn[a] * px0; ry = ang.cs[a] * oy_ + ang.sn[a] * py0; }
    else { rx = ang.cs[a] * ox_ + ang.sn[a] * (-px0); ry = ang.cs[a] * oy_ + ang.sn[a] * (-py0); }
    { double z = rx * rx + ry * ry; if (z > 0.0) { double q = sqrt(z); rx = rx / q; ry = ry / q; } }
    double resx = 0, resy = 0;
    bool done = false;
    // kRayBatch groups of 64 steps per trip, their skeleton loads in flight together, then the groups' events in step
    // order (round 6: one group per trip waited for one load per 64 steps; rays that cross the map run ~100 groups)
    // (C2 41 -> 31 us, C3 87 -> 74 us, profiles/r06/r06zi_kt*_summary.txt; 16 groups were slower, 188 VGPRs and more steps
    // past the event, r06zj; the divisions through the reciprocal changed nothing, r06zk)
    constexpr int kRayBatch = 4;
    for (int base = 0; base < n_tab && !done; base += 64 * kRayBatch) {
        double px[kRayBatch], py[kRayBatch];
        bool valid[kRayBatch], ins[kRayBatch], occ[kRayBatch];
        uint64_t w[kRayBatch];
        int cx[kRayBatch];
#pragma unroll
        for (int u = 0; u < kRayBatch; ++u) {
            const int i = base + 64 * u + lane;
            const double cur = cur_tab[i < n_tab ? i : n_tab - 1];
            valid[u] = i < n_tab && cur <= g.amax;
            px[u] = stx + rx * cur; py[u] = sty + ry * cur;
            ins[u] = px[u] >= g.minx && px[u] <= g.maxx && py[u] >= g.miny && py[u] <= g.maxy;
            bool inr = false;
            int mx = 0, my = 0;
            if (ins[u]) {
                mx = (int)((px[u] - g.ox) / (double)g.res); my = (int)((py[u] - g.oy) / (double)g.res);
                inr = mx >= 0 && mx < g.W && my >= 0 && my < g.H;
            }
            cx[u] = inr ? mx : -1;
            const int cy = inr ? my : 0;
            w[u] = skel[(size_t)cy * g.WW + ((inr ? mx : 0) >> 6)];
        }
#pragma unroll
        for (int u = 0; u < kRayBatch; ++u) {
            occ[u] = cx[u] >= 0 && ((w[u] >> (cx[u] & 63)) & 1ull);
            const bool ev = !valid[u] || !ins[u] || occ[u];
            const unsigned long long m = __ballot(ev);
            if (m) {
                const int j = __ffsll((long long)m) - 1;
                const double qx = __shfl(px[u], j), qy = __shfl(py[u], j);
                const bool qvalid = __shfl((int)valid[u], j), qins = __shfl((int)ins[u], j);
                if (qvalid) {
                    done = true;
                    if (!qins) { resx = fmax(g.minx, fmin(g.maxx, qx)); resy = fmax(g.miny, fmin(g.maxy, qy)); }
                    else { resx = qx; resy = qy; }
                }
                base = n_tab;   // (the walk ends at the first event, found or not)
                break;
            }
        }
    }
    if (!done) {
        double fx = stx + rx * g.amax, fy = sty + ry * g.amax;
        if (!(fx >= g.minx && fx <= g.maxx && fy >= g.miny && fy <= g.maxy)) {
            fx = fmax(g.minx, fmin(g.maxx, fx)); fy = fmax(g.miny, fmin(g.maxy, fy));
        }
        resx = fx; resy = fy;
    }
    if (lane == 0) {
        int good = isfinite(resx) && isfinite(resy) && resx >= g.minx && resx <= g.maxx && resy >= g.miny &&
                   resy <= g.maxy && !d_pip(resx, resy, poly, np);
        cand[s] = make_double2(resx, resy);
        ok[s] = good;
    }
}


// /voronoi_seeds order (seed_gen:1670-1710): virtual, ray, endpoint seeds (counts on the device)
// The seeds and their counts also go straight into pinned host memory (h_out, h_cnt[0..2], h_cnt[3] = the
// de-duplications' error word): one launch and one host wait instead of a count read-back, a wait, a copy and a
// second wait.
__global__ void k_concat3(const double2 *a, const double2 *b, const double2 *c, const int *cnt, double2 *out, double2 *h_out,
                          int *h_cnt, const int *err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int na = cnt[0], nb = cnt[1], nc = cnt[2];
    if (i == 0) { h_cnt[0] = na; h_cnt[1] = nb; h_cnt[2] = nc; h_cnt[3] = *err; }
    double2 v;
    if (i < na) v = a[i];
    else if (i < na + nb) v = b[i - na];
    else if (i < na + nb + nc) v = c[i - na - nb];
    else return;
    out[i] = v;
    h_out[i] = v;
}

// ------------------------------------------------------------------ host orchestration
template <class T> static T *dev(DevBuf &b, size_t n) { return static_cast<T *>(b.ensure(sizeof(T) * std::max<size_t>(n, 1))); }

// The whole-map stage's labelling on any foreground given as bits (the tiled frame's own region, cluster_dist.hip):
// list, block-local union-find in LDS, cross-chunk unions, flatten, root ranks. One host wait (for nf); the
// component count stays on the device at rank + nf. err: the single-pass scans' error word (read with nf).
int ccl_label(CclScratch &B, const uint64_t *fg, const int *off, const GridC &g, hipStream_t s, int *h_pinned2, int *err) {
    const size_t Cw = (size_t)g.WW * g.H;
    const int *d_off = off;
    peek_to_host(h_pinned2, {d_off + Cw, B.lb.err_word(s)}, s);
    AOS_HIP(hipStreamSynchronize(s));
    *err = h_pinned2[1];
    const int nf = *err ? 0 : h_pinned2[0];
    B.list_p = dev<int>(B.list, nf);
    B.parent_p = dev<int>(B.parent, nf);
    B.rank_p = dev<int>(B.rank, (size_t)nf + 1);
    if (nf == 0) {
        AOS_HIP(hipMemsetAsync(B.rank_p, 0, sizeof(int), s));
        return 0;
    }
    const dim3 gw2(cdiv(g.WW, 64), g.H);
    const int ecap = ccl_edge_cap(nf);
    int *d_ne = dev<int>(B.edges, 2 + 2 * (size_t)ecap);
    int2 *d_edges = reinterpret_cast<int2 *>(d_ne + 2);
    k_fg_list<<<gw2, 64, 0, s>>>(fg, d_off, B.list_p, g, nullptr, d_ne);
    const int chunk = ccl_chunk();
    k_ccl_local<<<cdiv(nf, chunk), ccl_tb(), sizeof(int) * chunk, s>>>(B.list_p, nf, fg, d_off, g, B.parent_p, d_edges, d_ne,
                                                                      ecap - 1, chunk);
    k_ccl_cross<<<256, 256, 0, s>>>(d_edges, d_ne, ecap - 1, B.parent_p, B.list_p, nf, fg, d_off, g);
    ccl_flatten_rank(B.lb, B.parent_p, dev<int>(B.isroot, nf), B.rank_p, nf, s);
    AOS_HIP(hipGetLastError());
    return nf;
}

void run_cluster_seed_stage(ClusterSeedState &S, const SeedStageIn &in, SeedStageOut &out, hipStream_t s, hipEvent_t ev_mid,
                            const hipEvent_t *ev_split) {
    HostTrace tr{"cluster"};
    if (ev_split) AOS_HIP(hipEventRecord(ev_split[0], s));   // (AOS_TRACE: the stage's first kernel is next)
    if (in.pre && in.after_fg) in.after_fg();
    const FrameGeom &fg = *in.g;
    const GridC g = make_gridc(fg);
    const Poly &poly = *in.poly;
    const int np = (int)poly.size();
    const size_t pc0 = S.poly.cap;
    double *d_poly = dev<double>(S.poly, 2 * np);
    std::vector<double> hp(2 * np);
    for (int i = 0; i < np; ++i) { hp[2 * i] = poly[i].first; hp[2 * i + 1] = poly[i].second; }
    // host -> device through a pinned staging buffer, only when the polygon (or its buffer) changed
    if (S.poly.cap != pc0 || hp != S.poly_up) {
        double *h_up = static_cast<double *>(S.h_up_poly.ensure(sizeof(double) * 2 * np));
        std::copy(hp.begin(), hp.end(), h_up);
        S.poly_up.clear();   // (until the copy is queued)
        copy_from_host(d_poly, h_up, sizeof(double) * 2 * np, s);
        S.poly_up = hp;
    }
    int *h_sc = static_cast<int *>(S.h_misc.ensure(4096));

    // ---- foreground list (raster order)
    const size_t Cw = (size_t)g.WW * g.H;
    uint64_t *d_fg = nullptr;
    int *d_wo = nullptr;
    const dim3 gw2(cdiv(g.WW, 64), g.H);
    if (!in.pre) {
        d_fg = dev<uint64_t>(S.fg_bits, Cw);
        int *d_wc = dev<int>(S.word_cnt, Cw);
        d_wo = dev<int>(S.word_off, Cw + 1);
        k_fg<<<gw2, 64, 0, s>>>(in.skel_bits, d_fg, d_wc, g, d_poly, np);
        scan_1p(S.lb, d_wc, d_wo, (int)Cw, false, s);
        peek_to_host(h_sc, {d_wo + Cw, S.lb.err_word(s)}, s);
        if (in.after_fg) in.after_fg();
        S.dedup.sev.sync(s);
        tr.mark("fg");
        if (h_sc[1]) throw std::runtime_error("cluster stage: scan failed on the device");
    }
    const int nf = in.pre ? in.pre->n_fg : h_sc[0];
    S.n_fg = nf;
    out = SeedStageOut();
    S.n_clusters = 0;
    S.h_rec.clear();
    S.n_replay_from_bits = S.n_replay_gpu = S.n_replay_cells = 0;
    std::vector<RowDev> rows;
    if (in.pre) {   // labelled and measured by the tile ranks (cluster_dist.hip)
        S.h_rec = in.pre->rec;
        S.n_clusters = (int)S.h_rec.size();
        out.n_bfs = in.pre->n_bfs;
    } else if (nf > 0) {
        int *d_list = dev<int>(S.fg_list, nf);
        int *d_par = dev<int>(S.parent, nf), *d_isroot = dev<int>(S.root_flag, nf), *d_rank = dev<int>(S.root_rank, nf + 1);
        const int ecap = ccl_edge_cap(nf);
        int *d_ne = dev<int>(S.ccl_edges, 2 + 2 * (size_t)ecap);
        int2 *d_edges = reinterpret_cast<int2 *>(d_ne + 2);   // (8-byte aligned: DevBuf bases are)
        k_fg_list<<<gw2, 64, 0, s>>>(d_fg, d_wo, d_list, g, nullptr, d_ne);
        const int chunk = ccl_chunk();
        k_ccl_local<<<cdiv(nf, chunk), ccl_tb(), sizeof(int) * chunk, s>>>(d_list, nf, d_fg, d_wo, g, d_par, d_edges, d_ne,
                                                                          ecap - 1, chunk);
        k_ccl_cross<<<256, 256, 0, s>>>(d_edges, d_ne, ecap - 1, d_par, d_list, nf, d_fg, d_wo, g);
        ccl_flatten_rank(S.lb, d_par, d_isroot, d_rank, nf, s);
        peek_to_host(h_sc, {d_rank + nf, S.lb.err_word(s)}, s);
        S.dedup.sev.sync(s);
        tr.mark("roots");
        if (h_sc[1]) throw std::runtime_error("cluster stage: scan failed on the device");
        const int ncl = h_sc[0];
        S.n_clusters = ncl;
        // bucket the foreground cells by cluster id: counting sort (k_cluster_count)
        const size_t cc0 = S.cl_count.cap;
        int *d_ccnt = dev<int>(S.cl_count, ncl + 1);
        if (S.cl_count.cap != cc0 || S.cl_count_dirty) AOS_HIP(hipMemsetAsync(d_ccnt, 0, S.cl_count.cap, s));
        S.cl_count_dirty = true;
        int *d_off = dev<int>(S.cl_off, ncl + 1);
        int *d_cid = dev<int>(S.cl_cursor, 2 * (size_t)nf), *d_crank = d_cid + nf;
        int *d_cells = dev<int>(S.cl_cells, nf);
        k_cluster_count<<<cdiv(nf, kClTB), kClTB, 0, s>>>(d_par, d_rank, nf, d_cid, d_crank, d_ccnt);
        scan_1p(S.lb, d_ccnt, d_off, ncl, true, s);   // (leaves the counts zero)
        S.cl_count_dirty = false;
        k_cluster_scatter<<<cdiv(nf, 256), 256, 0, s>>>(d_list, d_cid, d_crank, d_off, nf, d_cells);
        ClusterRec *d_rec = dev<ClusterRec>(S.rec, ncl);
        S.h_rec.resize(ncl);
        ClusterRec *hr = static_cast<ClusterRec *>(S.h_recbuf.ensure(sizeof(ClusterRec) * (size_t)ncl));
        launch_cluster_stats(d_off, d_cells, ncl, g, d_poly, np, static_cast<float>(in.cluster_min_length), d_rec, s, hr);
        if (ev_split) AOS_HIP(hipEventRecord(ev_split[1], s));   // (AOS_TRACE: the GPU part ends here)
        S.dedup.sev.sync(s);
        tr.mark("recs");
        std::copy(hr, hr + ncl, S.h_rec.begin());
        if (g_debug_replay_all.load(std::memory_order_relaxed))
            for (auto &r : S.h_rec) r.flags |= 2;
        int n_bfs = 0;
        for (const auto &r : S.h_rec) n_bfs += (r.flags & 2) != 0;
        out.n_bfs = n_bfs;
        if (n_bfs) {
            // Replays are independent (each writes only its own ClusterRec), so they run in parallel over clusters
            // on up to kReplayThreads host threads: at 8192^2 every row cluster needs one (sums > 2^24). When the
            // frameless skeleton's bits come to the host anyway (the published grid's read-back), the replays walk
            // them over each cluster's box: no copy of the clusters' cells (C3: 7.6 MB on PCIe beside the grids'
            // read-back, round-5 traces). The clusters the bits do not give (a polygon cutting the box), and every
            // flagged cluster without the bits, replay from their cells, which come over in one copy.
            std::vector<int> ids;
            for (int c = 0; c < ncl; ++c)
                if (S.h_rec[c].flags & 2) ids.push_back(c);
            const int gpu_min = g_debug_replay_min.load(std::memory_order_relaxed) >= 0
                                    ? g_debug_replay_min.load(std::memory_order_relaxed) : kGpuReplayMin;
            if ((int)ids.size() >= gpu_min) {
                // many replays (C3: every row cluster): all at once on the GPU, one wave each (replay_gpu.hip), from
                // the cells already on the device; the few it leaves go on below
                std::vector<int> gids, rest;
                long long maxw = 0;
                for (int c : ids) {
                    const long long w = replay_bitmap_words(S.h_rec[c]);
                    if (w > 0 && w * 4 <= (long long)kReplayLdsBytes) { gids.push_back(c); maxw = std::max(maxw, w); }
                    else rest.push_back(c);
                }
                if (!gids.empty()) {
                    const int nj = (int)gids.size();
                    static const bool prof = [] { const char *e = getenv("AOS_REPLAY_PROF"); return e && atoi(e) != 0; }();
                    int *h_ids = static_cast<int *>(S.h_replay.ensure(sizeof(int) * 2 * (size_t)nj + (prof ? 64 * (size_t)nj + 64 : 0)));
                    int *h_st = h_ids + nj;
                    long long *h_prof = prof ? reinterpret_cast<long long *>(h_ids + ((2 * (size_t)nj + 1) & ~(size_t)1)) : nullptr;
                    std::copy(gids.begin(), gids.end(), h_ids);
                    std::fill(h_st, h_st + nj, 1);
                    int *d_ids = dev<int>(S.replay_ids, nj);
                    copy_from_host(d_ids, h_ids, sizeof(int) * nj, s);
                    launch_gpu_replays(d_ids, nj, (int)maxw, d_off, d_fg, d_rec, hr, h_st, dev<int>(S.replay_order, nf),
                                       g, d_poly, np, static_cast<float>(in.cluster_min_length), s, h_prof);
                    S.dedup.sev.sync(s);
                    tr.mark("replays_gpu");
                    if (h_prof) print_replay_prof(h_prof, nj);
                    for (int j = 0; j < nj; ++j) {
                        if (h_st[j]) { rest.push_back(gids[j]); continue; }
                        S.h_rec[gids[j]] = hr[gids[j]];
                        ++S.n_replay_gpu;
                    }
                    std::sort(rest.begin(), rest.end());
                }
                ids.swap(rest);
            }
            const uint64_t *hbits = !ids.empty() && in.host_skel_bits ? in.host_skel_bits() : nullptr;
            if (hbits) {
                tr.mark("bits");
                std::vector<ReplayJob> jobs;
                for (int c : ids) jobs.push_back({c, nullptr, S.h_rec[c].n, hbits});
                std::vector<int> failed, rest;
                replay_clusters(jobs, g, hp.data(), np, static_cast<float>(in.cluster_min_length), S.h_rec.data(),
                                &S.replay_pool, &failed);
                tr.mark("replays_bits");
                for (int i : failed) rest.push_back(jobs[i].c);
                S.n_replay_from_bits = (int)(ids.size() - rest.size());
                ids.swap(rest);
            }
            if (!ids.empty()) {
                std::vector<long long> off(ncl + 1, 0);
                for (int c = 0; c < ncl; ++c) off[c + 1] = off[c] + S.h_rec[c].n;
                // from a 16-byte boundary, in whole 16-byte words (the copy kernel's uint4 form); d_cells has slack
                // past nf (DevBuf)
                const long long lo = off[ids.front()] & ~3LL, hi = (off[ids.back() + 1] + 3) & ~3LL;
                int *hc = static_cast<int *>(S.h_cells.ensure(sizeof(int) * (size_t)(hi - lo)));
                copy_to_host(hc, d_cells + lo, sizeof(int) * (hi - lo), s);
                S.dedup.sev.sync(s);
                tr.mark("cells");
                std::vector<ReplayJob> jobs;
                for (int c : ids) jobs.push_back({c, hc + (off[c] - lo), S.h_rec[c].n});
                replay_clusters(jobs, g, hp.data(), np, static_cast<float>(in.cluster_min_length), S.h_rec.data(),
                                &S.replay_pool);
                tr.mark("replays");
                S.n_replay_cells = (int)ids.size();
            }
        }
    }
    assemble_rows(S.h_rec, out, rows);   // (host: cluster_host.cpp)
    tr.mark("rows");
    out.n_clusters_all = S.n_clusters;
    S.n_rows = (int)rows.size();
    if (ev_mid) AOS_HIP(hipEventRecord(ev_mid, s));

    if (rows.empty()) return;

    // ---- seeds: virtual seeds (a11), endpoint-ray seeds (a12) and endpoint seeds (:1451-1496), each a
    // first-come 0.5 m de-duplication of its candidates in order; the three run back to back on the device
    // (the two small ones in one launch) and one kernel concatenates them: two host waits in all
    DedupScratch &scr = S.dedup;
    const int nr = (int)rows.size();
    RowDev *d_rows = dev<RowDev>(S.row_idx, nr);
    {
        RowDev *hr = static_cast<RowDev *>(S.h_up_rows.ensure(sizeof(RowDev) * (size_t)nr));
        std::copy(rows.begin(), rows.end(), hr);
        copy_from_host(d_rows, hr, sizeof(RowDev) * nr, s);
    }
    const int nslots = rows.back().slot0 + 3 * rows.back().k;
    const size_t ncand = (size_t)nslots + 8 * (size_t)nr;
    double2 *d_cand = dev<double2>(S.cand_xy, ncand), *d_rcand = d_cand + nslots, *d_ecand = d_rcand + 6 * nr;
    int *d_ok = dev<int>(S.cand_ok, ncand), *d_rok = d_ok + nslots, *d_eok = d_rok + 6 * nr;
    double2 *d_vout = dev<double2>(S.hash_sorted, ncand), *d_rout = d_vout + nslots, *d_eout = d_rout + 6 * nr;
    double2 *d_seeds = dev<double2>(S.seed_out, ncand);
    int *d_cnt = dev<int>(S.misc, 8);   // kept counts: virtual, ray, endpoint
    const double hx0 = g.minx - 50.0, hx1 = g.maxx + 50.0, hy0 = g.miny - 50.0, hy1 = g.maxy + 50.0;
    RayAngles ang{};
    const double degs[3] = {0.0, -90.0, 90.0};
    for (int a = 0; a < 3; ++a) {  // seed_gen:1796-1803, evaluated with the host libm
        double rad = degs[a] * M_PI / 180.0;
        if (degs[a] > 0) { ang.cs[a] = std::cos(rad); ang.sn[a] = std::sin(rad); ang.pos_branch[a] = 1; }
        else { ang.cs[a] = std::cos(-rad); ang.sn[a] = std::sin(-rad); ang.pos_branch[a] = 0; }
    }
    if (S.cur_tab_amax != g.amax) {   // current_dist sequence of castRayFromEndpoint (:1833-1871)
        std::vector<double> t;
        for (double cur = 1.0;; cur += 0.1) { t.push_back(cur); if (!(cur <= g.amax)) break; }
        S.n_cur_tab = (int)t.size();
        double *d = dev<double>(S.cur_tab, t.size());
        AOS_HIP(hipMemcpyAsync(d, t.data(), sizeof(double) * t.size(), hipMemcpyHostToDevice, s));
        S.dedup.sev.sync(s);
        tr.mark("curtab");
        S.cur_tab_amax = g.amax;
    }
    if (nslots > 0) {
        k_virtual_candidates<<<cdiv(nslots, 128), 128, 0, s>>>(d_rows, nr, nslots, in.skel_bits, g, d_poly, np, d_cand, d_ok);
        greedy_dedup_async(scr, d_cand, d_ok, nslots, kConflictLess, 0.5, make_hash_n(hx0, hx1, hy0, hy1, 0.5, nslots),
                           d_vout, nullptr, nullptr, d_cnt, s);
    } else {
        AOS_HIP(hipMemsetAsync(d_cnt, 0, sizeof(int), s));
    }
    // (Round 5 measured the endpoint-ray chain on a second stream with a hardware queue of its own, beside the
    // virtual-seed chain: the look-back kernels of the one waited longer beside the other, the stage took 0.25 ms
    // instead of 0.21-0.23; profiles/r05l_kt_summary.txt. Serial.)
    k_endpoint_rays<<<6 * nr, 64, 0, s>>>(d_rows, nr, in.skel_bits, g, ang, d_poly, np,
                                          static_cast<const double *>(S.cur_tab.p), S.n_cur_tab, d_rcand, d_rok, d_ecand, d_eok);
    if (6 * nr <= kSmallMax) {
        const HashG hs = small_hash(hx0, hx1, hy0, hy1, 0.5);
        SmallDedup sd{};
        sd.prob[0] = SmallProb{d_rcand, d_rok, 6 * nr, hs, d_rout, d_cnt + 1};
        sd.prob[1] = SmallProb{d_ecand, d_eok, 2 * nr, hs, d_eout, d_cnt + 2};
        sd.mode = kConflictLess;
        sd.thr = 0.5;
        greedy_dedup_small(scr, sd, 2, s);
    } else {
        greedy_dedup_async(scr, d_rcand, d_rok, 6 * nr, kConflictLess, 0.5, make_hash_n(hx0, hx1, hy0, hy1, 0.5, 6 * nr),
                           d_rout, nullptr, nullptr, d_cnt + 1, s);
        greedy_dedup_async(scr, d_ecand, d_eok, 2 * nr, kConflictLess, 0.5, make_hash_n(hx0, hx1, hy0, hy1, 0.5, 2 * nr),
                           d_eout, nullptr, nullptr, d_cnt + 2, s);
    }
    double *hs = static_cast<double *>(S.h_seeds.ensure(sizeof(double2) * std::max<size_t>(ncand, 1)));
    k_concat3<<<cdiv((long long)ncand, 256), 256, 0, s>>>(d_vout, d_rout, d_eout, d_cnt, d_seeds,
                                                          reinterpret_cast<double2 *>(hs), h_sc, dedup_err(scr, s));
    S.dedup.sev.sync(s);
    tr.mark("seeds");
    dedup_check(scr, h_sc[3]);
    const int n_virtual = h_sc[0], n_ray = h_sc[1], n_end = h_sc[2];
    const int ntot = n_virtual + n_ray + n_end;
    out.h_voronoi = hs;
    out.n_virtual = n_virtual; out.n_ray = n_ray; out.n_endpoint = n_end;
    out.d_voronoi = reinterpret_cast<const double *>(d_seeds);
    out.n_voronoi = ntot;
}

}  // namespace aos
