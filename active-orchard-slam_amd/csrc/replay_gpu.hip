// Exact FIFO-BFS replays on the GPU (a8-a10 for the clusters without the order-free certificate): one wave per
// cluster, all of a frame's replays at once. clusterOccupiedCells' BFS (seed_gen:1007-1049) visits a cluster in
// FIFO order from its first cell with the neighbour order (dx, dy) = (-1,-1) (-1,0) (-1,1) (0,-1) (0,1) (1,-1)
// (1,0) (1,1); the float centre sums (:1030-1046) and the first-strict-maximum endpoints (:1354-1395) depend on
// that order. The host replays (cluster_host.cpp) run a few ns per cell but only 16 at a time; at 8192^2 every row
// cluster needs one (215 of ~9,000 cells). Here each cluster's walk is one wave's serial chain:
//   * the cluster's bounding box, with a zero border of one cell, is a bitmap in LDS read from the foreground bits
//     (a set bit = foreground, not yet queued; other clusters' cells in the box are never reached); a popped cell
//     reads its 3 x 3 window as three 3-bit fields of wave-uniform LDS words and makes the same 8-bit neighbour
//     mask as the host walk;
//   * runs, as in the host walk: when a step queues only its right neighbour and nothing else is queued, the next
//     k pops each queue just the next cell right (k from bit scans of the row and its neighbours), so they are
//     taken at once: the float sums cell by cell, the order and the bit clears by lanes. A lone wave's general step
//     costs ~0.5 us (one instruction issue per 4 cycles, two LDS round trips), so the runs carry the speed;
//   * the FIFO queue is a ring of 64 entries in one VGPR, entry i in lane i mod 64: a pop is one v_readlane, and a
//     push is a ballot-ordered append (the lane of entry tail + j takes the j-th set bit of the mask, clears its
//     bitmap bit and stores the cell): no memory round trip on the queue. A frontier wider than 64 cells is a
//     failure (the host replays that cluster);
//   * the centre sums are the float additions of the reference in pop order (wave-uniform values), and the pop
//     order goes to global memory as packed box cells, for the endpoint passes: three parallel first-strict-maximum
//     searches over the order (the maximum, then the smallest BFS index holding it), four loads in flight a lane.
// The record is updated exactly as host_bfs_replay updates it; a cluster whose box does not fit the LDS budget, or
// whose frontier overflows the ring, is left to the host (its status word says so).
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdint>
#include <algorithm>
#include <cstdio>
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
    const int *off;        // cluster offsets: cluster c's BFS order goes to order[off[c] ...]
    const uint64_t *fg;    // the foreground bits (skeleton inside the polygon), WW words per row
    ClusterRec *rec;       // device records (updated)
    ClusterRec *hrec;      // pinned host copy of the updated records
    int *status;           // pinned host: per job, 0 = replayed, 1 = left to the host
    int *order;            // scratch: the BFS order as packed box cells (row << 16 | column)
    GridC g;
    const double *poly; int np;
    float min_length;
    int lds_words;         // the launch's bitmap budget (32-bit words)
    int ring_cap;          // queue entries in flight at most (64; tests lower it to reach the host fallback)
    long long *prof;       // (nullable, AOS_REPLAY_PROF=1) per job: kProfWords counters of the phases
};
constexpr int kProfWords = 8;   // realtime ticks: fill, walk, endpoints; cycles of the walk; steps, runs, run cells, n

// 32 bits of a foreground row from grid column gx (gx >= -1; columns outside the row read as 0)
__device__ __forceinline__ uint32_t fg_bits32(const uint64_t *row, long long gx, int WW) {
    const long long wi = gx >= 0 ? gx >> 6 : -1;
    const int o = (int)(gx - 64 * wi);
    const uint64_t lo = (wi >= 0 && wi < WW) ? row[wi] : 0ull;
    const uint64_t hi = (wi + 1 >= 0 && wi + 1 < WW) ? row[wi + 1] : 0ull;
    return (uint32_t)(o ? (lo >> o) | (hi << (64 - o)) : lo);
}

__global__ __launch_bounds__(64) void k_bfs_replay(ReplayArgs A) {
    extern __shared__ uint32_t bm[];
    const int lane = threadIdx.x;
    const int c = A.ids[blockIdx.x];
    ClusterRec r = A.rec[c];
    const GridC &g = A.g;
    const int n = r.n, o = A.off[c];
    int *const ord = A.order + o;
    const int bw = r.bx1 - r.bx0 + 1, pw = bw + 2, ph = r.by1 - r.by0 + 3;
    const int RW = (pw + 31) / 32 + 1;
    const int sy = r.first / g.W, sx = r.first - sy * g.W;
    bool fail = n <= 0 || bw <= 0 || ph <= 2 || pw >= 65536 || ph >= 65536 || (long long)RW * ph > A.lds_words ||
                sx < r.bx0 || sx > r.bx1 || sy < r.by0 || sy > r.by1;
    int head = 0, tail = 0;
    float ax = 0.0f, ay = 0.0f;
    long long t0 = wall_clock64(), t1 = t0, t2 = t0, cyc = 0, n_steps = 0, n_runs = 0, n_runc = 0;
    if (!fail) {
        // the box's foreground rows (bitmap row rr = grid row by0 + rr - 1, bit c = column bx0 + c - 1; the border
        // rows and columns stay 0). Other clusters' cells inside the box are never reached: a foreground cell
        // 8-adjacent to this cluster belongs to it.
        for (int i = lane; i < RW * ph; i += 64) {
            const int rr = i / RW, w = i - rr * RW;
            uint32_t v = 0u;
            if (rr >= 1 && rr <= ph - 2) {
                const int c0 = 32 * w, keep = bw + 1 - c0;   // keep bitmap columns [1, bw]
                if (keep > 0) {
                    v = fg_bits32(A.fg + (size_t)(r.by0 + rr - 1) * g.WW, (long long)r.bx0 - 1 + c0, g.WW);
                    if (c0 == 0) v &= ~1u;
                    if (keep < 32) v &= (1u << keep) - 1u;
                }
            }
            bm[i] = v;
        }
        __syncthreads();
        const int scol = sx - r.bx0 + 1, srow = sy - r.by0 + 1;
        const int sw = srow * RW + (scol >> 5);
        const uint32_t sb = 1u << (scol & 31);
        if (!(rfl(bm[sw]) & sb)) fail = true;   // (the first cell is not foreground: records and grid disagree)
        __syncthreads();
        if (lane == 0) bm[sw] &= ~sb;
        __syncthreads();
        t1 = wall_clock64();
        cyc = clock64();
        uint32_t qv = (lane == 0) ? ((uint32_t)srow << 16 | (uint32_t)scol) : 0u;   // the ring: entry i in lane i % 64
        tail = fail ? 0 : 1;
        while (head < tail) {
            const uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)qv, head & 63);
            const int col = (int)(cur & 0xffffu), row = (int)(cur >> 16);
            ax += (float)(r.bx0 + col - 1); ay += (float)(r.by0 + row - 1);
            if (lane == 0) ord[head] = (int)cur;
            ++head;
            ++n_steps;
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
            if (tail + pc - head > A.ring_cap || tail + pc > n) { fail = true; break; }   // (ring; more cells than n)
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
            // A run (cluster_host.cpp's bfs_walk: a row cluster is a horizontal line walked from its left end with one
            // cell queued): the step queued only its right neighbour e = (col + 1, row), so from e on each pop queues
            // exactly the next cell right while it is set and the cells above and below it are not. Its length k is
            // the trailing ones of row & ~(row - 1 | row + 1) from bitmap column col + 2.
            if (m != (1u << 6) || tail - head != 1) continue;
            int k = 0;
            for (;;) {
                const int s = col + 2 + k, wi = s >> 5, so = s & 31;
                if (wi + 1 >= RW) break;
                auto w32 = [&](int rr) {
                    const uint64_t v = ((uint64_t)rfl(bm[rr * RW + wi + 1]) << 32) | rfl(bm[rr * RW + wi]);
                    return (uint32_t)(v >> so);
                };
                const uint32_t ok = w32(row) & ~(w32(row - 1) | w32(row + 1));
                const int t = ok == ~0u ? 32 : __builtin_ctz(~ok);
                k += t;
                if (t < 32) break;
            }
            if (k == 0) continue;
            ++n_runs; n_runc += k;
            if (head + k + 1 > n) { fail = true; break; }
            // pops e .. e + k - 1 (entries head .. head + k - 1) in order: the float sums cell by cell, the order by
            // lanes; their pushes e + 1 .. e + k: bitmap columns col + 2 .. col + k + 1 cleared by word
            const float fy = (float)(r.by0 + row - 1);
            const int ex = r.bx0 + col;   // e's grid x
            for (int t = 0; t < k; ++t) { ax += (float)(ex + t); ay += fy; }
            for (int t = lane; t < k; t += 64) ord[head + t] = (int)((uint32_t)row << 16 | (uint32_t)(col + 1 + t));
            {
                const int b0 = col + 2, b1 = col + 1 + k;   // inclusive
                for (int w = (b0 >> 5) + lane; w <= (b1 >> 5); w += 64) {
                    const int lo = max(b0, 32 * w) - 32 * w, hi = min(b1, 32 * w + 31) - 32 * w;
                    const uint32_t msk = (hi - lo == 31) ? ~0u : (((1u << (hi - lo + 1)) - 1u) << lo);
                    atomicAnd(&bm[row * RW + w], ~msk);
                }
            }
            head += k;
            tail = head + 1;
            if (lane == (head & 63)) qv = (uint32_t)row << 16 | (uint32_t)(col + 1 + k);
        }
        if (tail != n) fail = true;   // (not 8-connected, or the records disagree)
        cyc = clock64() - cyc;
        t2 = wall_clock64();
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
        auto cw = [&](int v) {   // cell_w of a packed box cell
            const int x = r.bx0 + (v & 0xffff) - 1, y = r.by0 + (v >> 16) - 1;
            return make_double2((double)cell_world(g.ox, x, g.res), (double)cell_world(g.oy, y, g.res));
        };
        // each lane walks k = lane, lane + 64, ... in increasing order, four loads in flight
        auto pass = [&](auto body) {
            for (int b = 0; b < n; b += 256) {
                int v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) { const int k = b + 64 * u + lane; v[u] = k < n ? ord[k] : 0; }
#pragma unroll
                for (int u = 0; u < 4; ++u) { const int k = b + 64 * u + lane; if (k < n) body(k, cw(v[u])); }
            }
        };
        // the first strict maximum of |w - centre|^2 over the BFS order (d2 > 0; none: index 0)
        double mx = 0.0; int fi = INT_MAX;
        pass([&](int k, double2 w) {
            const double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            if (d2 > mx) { mx = d2; fi = k; }
        });
        wave_argmax(mx, fi);
        if (fi == INT_MAX) fi = 0;
        const double2 wf = cw(ord[fi]);
        double fx = 0.0, fy = 0.0;
        if (mx > 0.0) {
            const double dx = wf.x - r.center.x, dy = wf.y - r.center.y, d2 = dx * dx + dy * dy;
            const double s = sqrt(d2);
            fx = dx / s; fy = dy / s;
        }
        // the first strict maximum among the cells opposite the first direction (host_bfs_replay's test)
        double mo = 0.0; int si = INT_MAX;
        pass([&](int k, double2 w) {
            if (k == fi) return;
            const double dx = w.x - r.center.x, dy = w.y - r.center.y, d2 = dx * dx + dy * dy;
            if (!(d2 > mo)) return;
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
        });
        wave_argmax(mo, si);
        if (mo == 0.0) {   // farthest from the first endpoint
            mo = 0.0; si = INT_MAX;
            pass([&](int k, double2 w) {
                if (k == fi) return;
                const double dx = w.x - wf.x, dy = w.y - wf.y, d2 = dx * dx + dy * dy;
                if (d2 > mo) { mo = d2; si = k; }
            });
            wave_argmax(mo, si);
        }
        if (si == INT_MAX) si = 0;
        r.start = wf;
        r.end = cw(ord[si]);
    }
    r.flags = (row_ok ? 1 : 0) | 4;   // 4: replayed
    if (A.prof && lane == 0) {
        long long *pr = A.prof + (size_t)kProfWords * blockIdx.x;
        pr[0] = t1 - t0; pr[1] = t2 - t1; pr[2] = wall_clock64() - t2; pr[3] = cyc;
        pr[4] = n_steps; pr[5] = n_runs; pr[6] = n_runc; pr[7] = n;
    }
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

void launch_gpu_replays(const int *d_ids, int n_jobs, int lds_words, const int *off, const uint64_t *fg, ClusterRec *rec,
                        ClusterRec *hrec, int *h_status, int *order, const GridC &g, const double *poly, int np,
                        float min_length, hipStream_t s, long long *h_prof) {
    if (n_jobs <= 0) return;
    if (lds_words <= 0 || (size_t)lds_words * 4 > kReplayLdsBytes)
        throw std::invalid_argument("launch_gpu_replays: bitmap budget out of range");
    const int rc = g_debug_replay_ring.load(std::memory_order_relaxed);
    ReplayArgs A{d_ids, n_jobs, off, fg, rec, hrec, h_status, order, g, poly, np, min_length, lds_words,
                 rc > 0 && rc < 64 ? rc : 64, h_prof};
    k_bfs_replay<<<n_jobs, 64, (size_t)lds_words * 4, s>>>(A);
    AOS_HIP(hipGetLastError());
}

// AOS_REPLAY_PROF=1 (timing experiments): the per-job phase counters of the last launch on stderr
void print_replay_prof(const long long *p, int n_jobs) {
    long long s[kProfWords] = {}, mx[kProfWords] = {};
    for (int j = 0; j < n_jobs; ++j)
        for (int k = 0; k < kProfWords; ++k) { s[k] += p[kProfWords * j + k]; mx[k] = std::max(mx[k], p[kProfWords * j + k]); }
    fprintf(stderr, "[aos replay prof] jobs %d  fill us avg %.1f max %.1f  walk us avg %.1f max %.1f (cycles/us %.0f)  "
                    "endpoints us avg %.1f max %.1f  steps avg %.0f  runs avg %.0f  run cells avg %.0f  n avg %.0f\n",
            n_jobs, s[0] / 100.0 / n_jobs, mx[0] / 100.0, s[1] / 100.0 / n_jobs, mx[1] / 100.0,
            s[1] ? (double)s[3] / (s[1] / 100.0) : 0.0, s[2] / 100.0 / n_jobs, mx[2] / 100.0, (double)s[4] / n_jobs,
            (double)s[5] / n_jobs, (double)s[6] / n_jobs, (double)s[7] / n_jobs);
}

}  // namespace aos
