// Exact FIFO-BFS replays on the GPU (a8-a10 for the clusters without the order-free certificate): one wave per
// cluster, all of a frame's replays at once. clusterOccupiedCells' BFS (seed_gen:1007-1049) visits a cluster in
// FIFO order from its first cell with the neighbour order (dx, dy) = (-1,-1) (-1,0) (-1,1) (0,-1) (0,1) (1,-1)
// (1,0) (1,1); the float centre sums (:1030-1046) and the first-strict-maximum endpoints (:1354-1395) depend on
// that order. The host replays (cluster_host.cpp) run ~10 ns per step but only 16 at a time; at 8192^2 every row
// cluster needs one (~450 of ~9,000 cells: 1.4 ms on the host threads, profiles/r06/r06c_c3_cluster_trace.txt).
// Here each cluster's walk is one wave's serial chain:
//   * the cluster's bounding box, with a zero border of one cell, is a bitmap in LDS (a set bit = in the cluster,
//     not yet queued); a popped cell reads its 3 x 3 window as three 3-bit fields of wave-uniform LDS words and
//     makes the same 8-bit neighbour mask as the host walk;
//   * the FIFO queue is a ring of 64 entries in one VGPR, entry i in lane i mod 64: a pop is one v_readlane, and a
//     push is a ballot-ordered append (the lane of entry tail + j takes the j-th set bit of the mask, clears its
//     bitmap bit and stores the cell): no memory round trip on the queue. A frontier wider than 64 cells is a
//     failure (the host replays that cluster);
//   * the centre sums are the float additions of the reference in pop order (wave-uniform values), and the pop
//     order goes to global memory 64 cells at a time (one coalesced store), for the endpoint passes: three
//     parallel first-strict-maximum searches over the order (the maximum, then the smallest BFS index holding it).
// The record is updated exactly as host_bfs_replay updates it; a cluster whose box does not fit the LDS budget, or
// whose frontier overflows the ring, is left to the host (its status word says so).
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdint>
#include <stdexcept>

#include "cluster_geom.h"
#include "cluster_seed.h"

namespace aos {

namespace {

// packed (dx + 1), (dy + 1) of the neighbour order, one nibble per direction
constexpr uint32_t kDxP = 0x22211000u, kDyP = 0x21020210u;

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// (value, index) with the larger value, ties to the smaller index; invalid = (0, INT_MAX)
__device__ __forceinline__ void wave_argmax(double &v, int &k) {
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o);
        const int ok = __shfl_xor(k, o);
        if (ov > v || (ov == v && ok < k)) { v = ov; k = ok; }
    }
}

struct ReplayArgs {
    const int *ids;        // the clusters of this launch
    int n_jobs;
    const int *off, *cells;
    ClusterRec *rec;       // device records (updated)
    ClusterRec *hrec;      // pinned host copy of the updated records
    int *status;           // pinned host: per job, 0 = replayed, 1 = left to the host
    int *order;            // scratch: a cluster's BFS order at order[off[c] ...]
    GridC g;
    const double *poly; int np;
    float min_length;
    int lds_words;         // the launch's bitmap budget (32-bit words)
    int ring_cap;          // queue entries in flight at most (64; tests lower it to reach the host fallback)
};

__global__ __launch_bounds__(64) void k_bfs_replay(ReplayArgs A) {
    extern __shared__ uint32_t bm[];
    const int lane = threadIdx.x;
    const int c = A.ids[blockIdx.x];
    ClusterRec r = A.rec[c];
    const GridC &g = A.g;
    const int n = r.n, o = A.off[c];
    const int bw = r.bx1 - r.bx0 + 1, pw = bw + 2, ph = r.by1 - r.by0 + 3;
    const int RW = (pw + 31) / 32 + 1;
    const int sy = r.first / g.W, sx = r.first - sy * g.W;
    bool fail = n <= 0 || bw <= 0 || ph <= 2 || pw >= 65536 || ph >= 65536 || (long long)RW * ph > A.lds_words ||
                sx < r.bx0 || sx > r.bx1 || sy < r.by0 || sy > r.by1;
    if (!fail) {
        for (int i = lane; i < RW * ph; i += 64) bm[i] = 0u;
        __syncthreads();
        bool bad = false;
        for (int k = lane; k < n; k += 64) {
            const int p = A.cells[o + k], y = p / g.W, x = p - y * g.W;
            const int col = x - r.bx0 + 1, row = y - r.by0 + 1;
            if (col < 1 || col > bw || row < 1 || row > ph - 2) { bad = true; continue; }
            atomicOr(&bm[row * RW + (col >> 5)], 1u << (col & 31));
        }
        fail = __any(bad);
        __syncthreads();
    }
    int head = 0, tail = 0;
    float ax = 0.0f, ay = 0.0f;
    if (!fail) {
        const int scol = sx - r.bx0 + 1, srow = sy - r.by0 + 1;
        const int sw = srow * RW + (scol >> 5);
        const uint32_t sb = 1u << (scol & 31);
        if (!(rfl(bm[sw]) & sb)) fail = true;   // (the first cell is not among the cells: records and cells disagree)
        __syncthreads();
        if (lane == 0) bm[sw] &= ~sb;
        __syncthreads();
        uint32_t qv = (lane == 0) ? ((uint32_t)srow << 16 | (uint32_t)scol) : 0u;   // the ring: entry i in lane i % 64
        uint32_t ov = 0u;                                                           // pop order staging, same layout
        tail = fail ? 0 : 1;
        while (head < tail) {
            const uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)qv, head & 63);
            const int col = (int)(cur & 0xffffu), row = (int)(cur >> 16);
            const int x = r.bx0 + col - 1, y = r.by0 + row - 1;
            ax += (float)x; ay += (float)y;
            if (lane == (head & 63)) ov = (uint32_t)(y * g.W + x);
            ++head;
            if ((head & 63) == 0) A.order[o + head - 64 + lane] = (int)ov;
            // the 3 x 3 window: bits col - 1 .. col + 1 of rows row - 1 .. row + 1 (two words per row: the spare word)
            const int c0 = col - 1, sh = c0 & 31, base = (row - 1) * RW + (c0 >> 5);
            const uint32_t a0 = rfl(bm[base]), a1 = rfl(bm[base + 1]);
            const uint32_t b0 = rfl(bm[base + RW]), b1 = rfl(bm[base + RW + 1]);
            const uint32_t d0 = rfl(bm[base + 2 * RW]), d1 = rfl(bm[base + 2 * RW + 1]);
            const uint32_t rm = (uint32_t)((((uint64_t)a1 << 32) | a0) >> sh) & 7u;
            const uint32_t r0 = (uint32_t)((((uint64_t)b1 << 32) | b0) >> sh) & 7u;
            const uint32_t rp = (uint32_t)((((uint64_t)d1 << 32) | d0) >> sh) & 7u;
            // the neighbour order: column x - 1 (rows y - 1, y, y + 1), column x (y - 1, y + 1), column x + 1 (y - 1, y, y + 1)
            const uint32_t m = (rm & 1u) | (r0 & 1u) << 1 | (rp & 1u) << 2 | (rm & 2u) << 2 | (rp & 2u) << 3 |
                               (rm & 4u) << 3 | (r0 & 4u) << 4 | (rp & 4u) << 5;
            if (m == 0u) continue;
            const int pc = __builtin_popcount(m);
            if (tail + pc - head > A.ring_cap) { fail = true; break; }   // (the frontier outgrew the ring)
            const int j = (lane - tail) & 63;   // this lane takes entry tail + j: the j-th set bit of m
            if (j < pc) {
                uint32_t mm = m;
                for (int t = 0; t < j; ++t) mm &= mm - 1u;
                const int d = __builtin_ctz(mm);
                const int nc = col + (int)((kDxP >> (4 * d)) & 0xfu) - 1, nr = row + (int)((kDyP >> (4 * d)) & 0xfu) - 1;
                atomicAnd(&bm[nr * RW + (nc >> 5)], ~(1u << (nc & 31)));
                qv = (uint32_t)nr << 16 | (uint32_t)nc;
            }
            tail += pc;
        }
        if (!fail && (head & 63)) {
            const int rest = head & 63;
            if (lane < rest) A.order[o + head - rest + lane] = (int)ov;
        }
        if (tail != n) fail = true;   // (not 8-connected, or the cells repeat)
    }
    if (fail) {
        if (lane == 0) A.status[blockIdx.x] = 1;
        return;
    }
    __syncthreads();   // (the order's stores, read back by other lanes below)
    r.cx = ax / (float)n;
    r.cy = ay / (float)n;
    bool row_ok = false;
    if (r.length >= A.min_length) {
        const float cwx = (float)(g.ox + (double)(r.cx * g.res)), cwy = (float)(g.oy + (double)(r.cy * g.res));
        r.center = make_double2(cwx, cwy);
        row_ok = d_pip(cwx, cwy, A.poly, A.np);
    }
    if (row_ok) {
        const int *q = A.order + o;
        // the first strict maximum of |w - centre|^2 over the BFS order (d2 > 0; none: index 0)
        double mx = 0.0; int fi = INT_MAX;
        for (int k = lane; k < n; k += 64) {
            const double2 w = cell_w(g, q[k]);
            const double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            if (d2 > mx) { mx = d2; fi = k; }
        }
        wave_argmax(mx, fi);
        if (fi == INT_MAX) fi = 0;
        double fx = 0.0, fy = 0.0;
        if (mx > 0.0) {
            const double2 w = cell_w(g, q[fi]);
            const double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            const double s = sqrt(d2);
            fx = dx / s; fy = dy / s;
        }
        // the first strict maximum among the cells opposite the first direction (host_bfs_replay's test)
        double mo = 0.0; int si = INT_MAX;
        for (int k = lane; k < n; k += 64) {
            if (k == fi) continue;
            const double2 w = cell_w(g, q[k]);
            const double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            if (!(d2 > mo)) continue;
            const double pa = dx * fx, pb = dy * fy, dd = pa + pb;
            bool opposite;
            if (fabs(dd) > 1e-12 * (fabs(pa) + fabs(pb))) {
                opposite = dd < 0.0;
            } else {
                double nx = dx, ny = dy;
                if (d2 > 0.0) { const double s = sqrt(d2); nx = dx / s; ny = dy / s; }
                opposite = nx * fx + ny * fy < 0.0;
            }
            if (opposite) { mo = d2; si = k; }
        }
        wave_argmax(mo, si);
        if (mo == 0.0) {   // farthest from the first endpoint
            const double2 wf = cell_w(g, q[fi]);
            mo = 0.0; si = INT_MAX;
            for (int k = lane; k < n; k += 64) {
                if (k == fi) continue;
                const double2 w = cell_w(g, q[k]);
                const double dx = w.x - wf.x, dy = w.y - wf.y, d2 = dx * dx + dy * dy;
                if (d2 > mo) { mo = d2; si = k; }
            }
            wave_argmax(mo, si);
        }
        if (si == INT_MAX) si = 0;
        r.start = cell_w(g, q[fi]);
        r.end = cell_w(g, q[si]);
    }
    r.flags = (row_ok ? 1 : 0) | 4;   // 4: replayed
    if (lane == 0) {
        A.rec[c] = r;
        A.hrec[c] = r;
        A.status[blockIdx.x] = 0;
    }
}

}  // namespace

long long replay_bitmap_words(const ClusterRec &r) {
    const long long bw = (long long)r.bx1 - r.bx0 + 1, pw = bw + 2, ph = (long long)r.by1 - r.by0 + 3;
    if (r.n <= 0 || bw <= 0 || ph <= 2 || pw >= 65536 || ph >= 65536) return -1;
    return ((pw + 31) / 32 + 1) * ph;
}

void launch_gpu_replays(const int *d_ids, int n_jobs, int lds_words, const int *off, const int *cells, ClusterRec *rec,
                        ClusterRec *hrec, int *h_status, int *order, const GridC &g, const double *poly, int np,
                        float min_length, hipStream_t s) {
    if (n_jobs <= 0) return;
    if (lds_words <= 0 || (size_t)lds_words * 4 > kReplayLdsBytes)
        throw std::invalid_argument("launch_gpu_replays: bitmap budget out of range");
    const int rc = g_debug_replay_ring.load(std::memory_order_relaxed);
    ReplayArgs A{d_ids, n_jobs, off, cells, rec, hrec, h_status, order, g, poly, np, min_length, lds_words,
                 rc > 0 && rc < 64 ? rc : 64};
    k_bfs_replay<<<n_jobs, 64, (size_t)lds_words * 4, s>>>(A);
    AOS_HIP(hipGetLastError());
}

}  // namespace aos
