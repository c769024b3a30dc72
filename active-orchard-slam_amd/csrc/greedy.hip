// Greedy first-come de-duplication on the GPU (see cluster_seed.h), and the primitives it is built on
// (dev_prims.h): a single-pass look-back scan and a counting-sort cell index.
//
// Reference loops of the form
//   for c in candidates (in order): if no already-kept k conflicts with c: keep c
// (seed_gen:2076-2085, 1964-1974, 1460-1470; gvd:98-125; voronoi_diagram.cpp:156-204) keep exactly
// the lexicographically-first maximal independent set (LFMIS) of the conflict graph. The candidates are
// hashed into cells no smaller than the conflict radius (a counting sort: count, scan, scatter), and one
// fused kernel (k_lfmis) then does the rest:
//   * each thread lists its candidate's EARLIER conflicting candidates (3 x 3 cells) in LDS;
//   * it waits until its list decides it: kept once every listed candidate is removed, removed once one
//     is kept. A candidate waits only for smaller indices, and blocks take their index ranges in launch
//     order (dev_prims.h), so the smallest undecided candidate can always decide: no deadlock, and the
//     set is the LFMIS whatever the timing (decisions are facts about the final set);
//   * the block's kept candidates are compacted in index order with a decoupled look-back over the
//     blocks' kept counts.
// Four launches per de-duplication and no host round trip (round 3: a radix sort, two conflict passes, a
// scan, batches of rounds and a read-back per batch, ~25 launches). Problems of at most kSmallMax
// candidates run in one workgroup each (k_dedup_small: index, rounds and compaction in LDS).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "cluster_seed.h"
#include "dev_prims_device.h"
#include "dev_wave.h"

namespace aos {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

HashG make_hash(double minx, double maxx, double miny, double maxy, double cell) {
    HashG h{};
    h.inv = 1.0 / (cell * (1.0 + 1e-9));
    h.x0 = minx; h.y0 = miny;
    double nx = (maxx - minx) * h.inv + 2.0, ny = (maxy - miny) * h.inv + 2.0;
    // keep nx * ny < 2^31 (clamped far points stay correct, they only share border cells)
    while (nx * ny > 2.0e9) { h.inv *= 0.5; nx = (maxx - minx) * h.inv + 2.0; ny = (maxy - miny) * h.inv + 2.0; }
    h.nx = std::max(1, (int)nx); h.ny = std::max(1, (int)ny);
    return h;
}

static HashG make_hash_cap(double minx, double maxx, double miny, double maxy, double cell, double cap) {
    double c = cell;
    HashG h = make_hash(minx, maxx, miny, maxy, c);
    while ((double)h.nx * (double)h.ny > cap) {
        c *= 1.25;
        h = make_hash(minx, maxx, miny, maxy, c);
    }
    return h;
}

HashG make_hash_n(double minx, double maxx, double miny, double maxy, double cell, long long n, double cells_per_item) {
    return make_hash_cap(minx, maxx, miny, maxy, cell, std::max(4096.0, cells_per_item * (double)std::max(n, 1LL)));
}

// ------------------------------------------------------------------ look-back scratch
LookBack LookBackScratch::take(int blocks, hipStream_t s) {
    const size_t need = sizeof(unsigned long long) * (size_t)std::max(blocks, 1);
    const size_t cap0 = part.cap;
    part.ensure(need);
    if (part.cap != cap0) AOS_HIP(hipMemsetAsync(part.p, 0, part.cap, s));
    if (!ticket.p) {
        ticket.ensure(64);
        AOS_HIP(hipMemsetAsync(ticket.p, 0, 64, s));
    }
    if (++epoch >= (1u << 30)) {   // (30-bit tags: clear the words once per 2^30 launches)
        epoch = 1;
        AOS_HIP(hipMemsetAsync(part.p, 0, part.cap, s));
    }
    return LookBack{part.as<unsigned long long>(), ticket.as<unsigned>(), epoch, err_word(s)};
}

int *LookBackScratch::err_word(hipStream_t s) {
    if (ext_err) return ext_err;
    if (!err.p) {
        err.ensure(64);
        AOS_HIP(hipMemsetAsync(err.p, 0, 64, s));
    }
    return err.as<int>();
}

// ------------------------------------------------------------------ single-pass scan
// out[i] = in[0] + ... + in[i - 1] for i in [0, n] (out[n] = the total); zero_in: in[0, n) is left zero.
// A block scans kScanTile ints. Its loads and stores are lane-contiguous 16-byte words: thread t moves ints
// [4t, 4t + 4) of each of the tile's kScanPer / 4 quarters, so a wave instruction covers 1 KB of consecutive
// memory (round 5 read 8 consecutive ints per lane as dwords at a 32-byte lane stride: 2 KB touched per 256 B
// moved). The quarters are scanned one after another inside the block, then the blocks chain by a decoupled
// look-back. A tile is 8192 ints: the look-back of a block that meets only aggregates walks back 64 blocks per
// step, so the chain's length sets the launch's time (C3 trace, 2048-int tiles: 2.1 M ints in 22.8 us, 1032
// blocks). Problems of at most kScanSmall + 1 ints take one workgroup with a running carry (no ticket, no
// look-back words).
constexpr int kScanTB = 256, kScanPer = 32, kScanTile = kScanTB * kScanPer, kScanQ = kScanPer / 4;
constexpr int kScanSmallTB = 1024, kScanSmall = 64 * 1024;

template <bool VEC>
__device__ __forceinline__ int4 scan_load4(const int *in, long long i, int n) {
    if (VEC && i + 4 <= n) return *reinterpret_cast<const int4 *>(in + i);
    int4 v;
    v.x = i < n ? in[i] : 0;
    v.y = i + 1 < n ? in[i + 1] : 0;
    v.z = i + 2 < n ? in[i + 2] : 0;
    v.w = i + 3 < n ? in[i + 3] : 0;
    return v;
}
// exclusive prefixes of v (starting at acc) -> out[i .. i + 3], the entries <= n
template <bool VEC>
__device__ __forceinline__ void scan_store4(int *out, long long i, int n, int4 v, int acc) {
    int4 o;
    o.x = acc; o.y = o.x + v.x; o.z = o.y + v.y; o.w = o.z + v.z;
    if (VEC && i + 4 <= n + 1) { *reinterpret_cast<int4 *>(out + i) = o; return; }
    if (i <= n) out[i] = o.x;
    if (i + 1 <= n) out[i + 1] = o.y;
    if (i + 2 <= n) out[i + 2] = o.z;
    if (i + 3 <= n) out[i + 3] = o.w;
}
template <bool VEC>
__device__ __forceinline__ void scan_zero4(int *in, long long i, int n) {
    if (VEC && i + 4 <= n) { *reinterpret_cast<int4 *>(in + i) = make_int4(0, 0, 0, 0); return; }
    for (int k = 0; k < 4; ++k)
        if (i + k < n) in[i + k] = 0;
}

// Exclusive prefixes of NQ runs per thread over a block of NT threads, the runs ordered quarter-major (every thread's
// run[0], then every thread's run[1], ...): before[q] = the sum of the runs ahead of (q, thread); returns the sum of all.
// One barrier: each quarter's wave-inclusive scan by shuffles, the NQ x NT / 64 wave totals through LDS (wt), then
// every thread adds up the totals ahead of it (NQ block scans one after another took two barriers each).
template <int NQ, int NT>
__device__ __forceinline__ int block_excl_scan_q(const int (&run)[NQ], int (&before)[NQ], int *wt) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        incl[q] = wave_scan_incl(run[q], 0, IAdd());   // (DPP row moves, dev_wave.h)
        if (lane == 63) wt[q * NW + w] = incl[q];
    }
    __syncthreads();
    int acc = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        int wb = 0, qt = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int x = wt[q * NW + k];
            wb += k < w ? x : 0;
            qt += x;
        }
        before[q] = acc + wb + incl[q] - run[q];
        acc += qt;
    }
    return acc;
}

template <bool VEC>
__global__ __launch_bounds__(kScanTB) void k_scan_1p(int *in, int *out, int n, int zero_in, LookBack L) {
    __shared__ int sh_vid, wt[kScanQ * kScanTB / 64], sh_excl;
    const int vid = lb_block_id(L, &sh_vid);
    const long long base = (long long)vid * kScanTile + 4LL * threadIdx.x;
    int4 v[kScanQ];
    int run[kScanQ];
#pragma unroll
    for (int q = 0; q < kScanQ; ++q) {
        v[q] = scan_load4<VEC>(in, base + (long long)q * 4 * kScanTB, n);
        run[q] = v[q].x + v[q].y + v[q].z + v[q].w;
    }
    if (zero_in)
#pragma unroll
        for (int q = 0; q < kScanQ; ++q) scan_zero4<VEC>(in, base + (long long)q * 4 * kScanTB, n);
    int before[kScanQ];
    const int agg = block_excl_scan_q<kScanQ, kScanTB>(run, before, wt);
    if (threadIdx.x < 64) {
        const unsigned e = lb_exclusive(L, vid, (unsigned)agg);
        if (threadIdx.x == 0) sh_excl = (int)e;
    }
    __syncthreads();
    const int excl = sh_excl;
#pragma unroll
    for (int q = 0; q < kScanQ; ++q) scan_store4<VEC>(out, base + (long long)q * 4 * kScanTB, n, v[q], excl + before[q]);
}

// one workgroup, n + 1 <= kScanSmall + 1: tiles of kScanSmallQ x 4 kScanSmallTB ints with a running carry (the wave
// totals double-buffered: one barrier per tile)
constexpr int kScanSmallQ = 4;
template <bool VEC>
__global__ __launch_bounds__(kScanSmallTB) void k_scan_small(int *in, int *out, int n, int zero_in) {
    __shared__ int wt[2][kScanSmallQ * kScanSmallTB / 64];
    int carry = 0, par = 0;
    for (long long t0 = 0; t0 <= n; t0 += kScanSmallQ * 4 * kScanSmallTB, par ^= 1) {
        const long long i0 = t0 + 4LL * threadIdx.x;
        int4 v[kScanSmallQ];
        int run[kScanSmallQ], before[kScanSmallQ];
#pragma unroll
        for (int q = 0; q < kScanSmallQ; ++q) {
            v[q] = scan_load4<VEC>(in, i0 + (long long)q * 4 * kScanSmallTB, n);
            run[q] = v[q].x + v[q].y + v[q].z + v[q].w;
        }
        if (zero_in)
#pragma unroll
            for (int q = 0; q < kScanSmallQ; ++q) scan_zero4<VEC>(in, i0 + (long long)q * 4 * kScanSmallTB, n);
        const int tot = block_excl_scan_q<kScanSmallQ, kScanSmallTB>(run, before, wt[par]);
#pragma unroll
        for (int q = 0; q < kScanSmallQ; ++q)
            scan_store4<VEC>(out, i0 + (long long)q * 4 * kScanSmallTB, n, v[q], carry + before[q]);
        carry += tot;
    }
}

void scan_1p(LookBackScratch &lb, int *in, int *out, int n, bool zero_in, hipStream_t s) {
    const bool vec = !((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15);
    if (n <= kScanSmall) {
        if (vec) k_scan_small<true><<<1, kScanSmallTB, 0, s>>>(in, out, n, zero_in ? 1 : 0);
        else k_scan_small<false><<<1, kScanSmallTB, 0, s>>>(in, out, n, zero_in ? 1 : 0);
        AOS_HIP(hipGetLastError());
        return;
    }
    const int blocks = cdiv((long long)n + 1, kScanTile);
    const LookBack L = lb.take(blocks, s);
    if (vec) k_scan_1p<true><<<blocks, kScanTB, 0, s>>>(in, out, n, zero_in ? 1 : 0, L);
    else k_scan_1p<false><<<blocks, kScanTB, 0, s>>>(in, out, n, zero_in ? 1 : 0, L);
    AOS_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ cell index (counting sort)
// One atomic per run of equal buckets in a wave (round 6): the points arrive in spatial order (raster-ordered lists,
// rows of seeds), so a wave's lanes mostly share a few buckets and per-lane atomics on one counter were serialised:
// k_ci_count took 10.1 us per launch against k_ci_scatter's 5.1 at C2 and 24.8 against 6.5 at C3 (6 launches per
// frame, profiles/r06/r06za_kt*_summary.txt). A run's head (its bucket differs from the lane before, DPP wave_shr:1)
// adds the run's length and each lane takes head's base + its offset in the run: the ranks inside a bucket stay a
// permutation of 0 .. count - 1 (their order was the atomics' order before, too).
__global__ __launch_bounds__(256) void k_ci_count(const double2 *p, const int *ok, int n, const int *n_dev, HashG h,
                                                  int *cnt, int *rank) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
    int b = -1;   // (no bucket: past n, or not a point)
    if (i < n) {
        if ((ok && !ok[i]) || (n_dev && i >= *n_dev)) {
            rank[i] = -1;
        } else {
            int cx, cy;
            hash_cell(h, p[i].x, p[i].y, cx, cy);
            b = cy * h.nx + cx;
        }
    }
    const int prev = dpp_i32<0x138>(INT_MIN, b);   // wave_shr:1 (lane 0: INT_MIN)
    const unsigned long long heads = __ballot(b != prev);
    const unsigned long long upto = lane == 63 ? ~0ull : (2ull << lane) - 1;
    const int hl = 63 - __clzll((long long)(heads & upto));   // this lane's run head
    int base = 0;
    if (lane == hl && b >= 0) {
        const unsigned long long after = heads & ~upto;
        const int next = after ? __ffsll((long long)after) - 1 : 64;
        base = atomicAdd(&cnt[b], next - lane);
    }
    base = __shfl(base, hl);
    if (b >= 0) rank[i] = base + lane - hl;
}
__global__ void k_ci_scatter(const double2 *p, const int *rank, int n, HashG h, const int *start, int *items) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = rank[i];
    if (r < 0) return;
    int cx, cy;
    hash_cell(h, p[i].x, p[i].y, cx, cy);
    items[start[cy * h.nx + cx] + r] = i;
}

template <class T> static T *dev(DevBuf &b, size_t n) { return static_cast<T *>(b.ensure(sizeof(T) * std::max<size_t>(n, 1))); }

CellIdx cell_index_build(CellScratch &S, const double2 *p, const int *ok, int n, const HashG &h, hipStream_t s,
                         const int *n_dev) {
    const long long nb = (long long)h.nx * h.ny;
    if (nb >= INT_MAX) throw std::runtime_error("cell index: too many buckets");
    const size_t cap0 = S.cnt.cap;
    int *cnt = dev<int>(S.cnt, (size_t)nb + 1);
    if (S.dirty || S.cnt.cap != cap0) AOS_HIP(hipMemsetAsync(cnt, 0, S.cnt.cap, s));
    int *start = dev<int>(S.start, (size_t)nb + 1), *items = dev<int>(S.items, n), *rank = dev<int>(S.rank, n);
    S.dirty = true;
    if (n > 0) k_ci_count<<<cdiv(n, 256), 256, 0, s>>>(p, ok, n, n_dev, h, cnt, rank);
    scan_1p(S.lb, cnt, start, (int)nb, true, s);   // (leaves the counts zero for the next build)
    S.dirty = false;
    if (n > 0) k_ci_scatter<<<cdiv(n, 256), 256, 0, s>>>(p, rank, n, h, start, items);
    AOS_HIP(hipGetLastError());
    return CellIdx{h, start, items};
}

// ------------------------------------------------------------------ conflict tests
// x86-64 cvttsd2si semantics of static_cast<int>(double): out of range / NaN -> INT_MIN
__device__ __forceinline__ int x86_trunc_i32(double v) {
    return (v > -2147483649.0 && v < 2147483648.0) ? (int)v : INT_MIN;
}

__device__ __forceinline__ bool conflict(double2 a, double2 b, int mode, double thr) {
    double dx = a.x - b.x, dy = a.y - b.y;
    if (mode == kConflictKeyOrSq) {
        if (x86_trunc_i32(a.x * 100) == x86_trunc_i32(b.x * 100) && x86_trunc_i32(a.y * 100) == x86_trunc_i32(b.y * 100))
            return true;
        return dx * dx + dy * dy < thr;
    }
    double d = sqrt(dx * dx + dy * dy);
    return mode == kConflictLessEq ? (d <= thr) : (d < thr);
}

// ------------------------------------------------------------------ fused LFMIS + compaction
// state[i] = epoch << 2 | s, s = 1 kept, 2 removed (a word of another epoch: undecided). OWNER (the GVD
// merge, gvd:93-125): a removed candidate waits for every listed candidate and records the smallest kept
// one as its owner; a kept candidate owns itself; not-ok candidates get INT_MAX.
constexpr int kLfTB = 256, kLfList = 16;
struct LfArgs {
    const double2 *p; const int *ok; int n; int mode; double thr;
    int self_conflict;   // conflict(p, p) holds: an exact copy of an earlier candidate is removed at once (below)
    CellIdx ci;
    int *state; unsigned epoch;
    LookBack lb;
    double2 *out; int *kept_index; int *owner; int *count;
    int *pos_of;   // nullable: per candidate, its position in out, or -1
};

template <bool OWNER>
__global__ __launch_bounds__(kLfTB) void k_lfmis(LfArgs A) {
    __shared__ int sh_vid, wsum[kLfTB / 64], sh_excl;
    __shared__ int lst[kLfList * kLfTB];   // lst[k * kLfTB + tid]: the thread's k-th listed candidate
    const int tid = threadIdx.x;
    const int vid = lb_block_id(A.lb, &sh_vid);
    const int i = vid * kLfTB + tid;
    const unsigned tag = A.epoch << 2;
    int s = 0, nl = 0, own = INT_MAX;
    bool over = false;
    double2 pi = make_double2(0.0, 0.0);
    int cx = 0, cy = 0;
    if (i < A.n) {
        if (A.ok && !A.ok[i]) {
            s = 2;
        } else {
            pi = A.p[i];
            hash_cell(A.ci.h, pi.x, pi.y, cx, cy);
            // An exact copy of an earlier candidate j is removed whatever j's fate (without OWNER): it conflicts
            // with j and with everything j conflicts with, so either j is kept or an earlier kept candidate
            // removed j and removes it too. The GVD's boundary points are facet polygon corners, each Voronoi
            // vertex ~6 times: most candidates decide here without waiting for their predecessors.
            bool dup = false;
            for (int yy = max(cy - 1, 0); yy <= min(cy + 1, A.ci.h.ny - 1) && !dup; ++yy) {
                int k0, k1;
                ci_row(A.ci, yy, cx, k0, k1);
                dup = !walk_items<8>(A.ci.items, k0, k1, [&](int j) { return A.p[j]; }, [&](int j, double2 pj) {
                    if (j >= i) return true;
                    if (!OWNER && A.self_conflict && pj.x == pi.x && pj.y == pi.y) return false;   // (dup)
                    if (conflict(pi, pj, A.mode, A.thr)) {
                        if (nl < kLfList) lst[nl * kLfTB + tid] = j;
                        else over = true;
                        ++nl;
                    }
                    return true;
                });
            }
            if (dup) s = 2;
            else if (nl == 0) { s = 1; own = i; }
        }
        if (s) st_i32(&A.state[i], (int)(tag | (unsigned)s));
    }
    // wait for the listed candidates (over: more than kLfList, re-walk the cells each time)
    unsigned spins = 0;
    while (i < A.n && s == 0) {
        bool any_kept = false, any_und = false;
        int mk = INT_MAX;
        auto look = [&](int j) {
            const unsigned w = (unsigned)ld_i32(&A.state[j]);
            if ((w & ~3u) != tag) { any_und = true; return; }
            if ((w & 3u) == 1u) { any_kept = true; mk = min(mk, j); }
        };
        if (!over) {
            for (int k = 0; k < nl && (OWNER || !any_kept); ++k) look(lst[k * kLfTB + tid]);
        } else {
            for (int yy = max(cy - 1, 0); yy <= min(cy + 1, A.ci.h.ny - 1); ++yy) {
                int k0, k1;
                ci_row(A.ci, yy, cx, k0, k1);
                for (int k = k0; k < k1; ++k) {
                    const int j = A.ci.items[k];
                    if (j < i && conflict(pi, A.p[j], A.mode, A.thr)) look(j);
                }
            }
        }
        if (OWNER) {
            if (!any_und) { s = any_kept ? 2 : 1; own = any_kept ? mk : i; }
        } else {
            if (any_kept) s = 2;
            else if (!any_und) { s = 1; own = i; }
        }
        if (s) {
            st_i32(&A.state[i], (int)(tag | (unsigned)s));
        } else if (++spins > kSpinCap) {
            atomicOr(A.lb.err, 2);
            s = 3;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (OWNER && i < A.n) A.owner[i] = own;
    // kept candidates of the block, in index order, after the kept of all earlier blocks
    const int kept = (i < A.n && s == 1) ? 1 : 0;
    int agg;
    const int r = block_excl_scan<kLfTB>(kept, wsum, &agg);
    if (tid < 64) {
        const unsigned e = lb_exclusive(A.lb, vid, (unsigned)agg);
        if (tid == 0) {
            sh_excl = (int)e;
            if (vid == (int)gridDim.x - 1) *A.count = (int)e + agg;
        }
    }
    __syncthreads();
    if (kept) {
        const int pos = sh_excl + r;
        A.out[pos] = pi;
        if (A.kept_index) A.kept_index[pos] = i;
    }
    if (A.pos_of && i < A.n) A.pos_of[i] = kept ? sh_excl + r : -1;
}

// ------------------------------------------------------------------ small problems: one workgroup each
constexpr int kSmallTB = 1024, kSmallPer = kSmallMax / kSmallTB, kSmallBuckets = 2048;
__global__ __launch_bounds__(kSmallTB) void k_dedup_small(SmallDedup A) {
    const SmallProb &P = A.prob[blockIdx.x];
    __shared__ double2 pts[kSmallMax];
    __shared__ int st[kSmallMax], items[kSmallMax], bstart[kSmallBuckets + 1], wsum[kSmallTB / 64];
    const int tid = threadIdx.x, n = P.n;
    const HashG &h = P.h;
    const int nb = h.nx * h.ny;   // <= kSmallBuckets (host)
    for (int b = tid; b <= nb; b += kSmallTB) bstart[b] = 0;
    __syncthreads();
    int bk[kSmallPer], rk[kSmallPer];
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        const int i = tid * kSmallPer + k;
        bk[k] = -1;
        if (i < n) {
            const double2 q = P.p[i];
            pts[i] = q;
            const bool ok = !P.ok || P.ok[i];
            st[i] = ok ? 0 : 2;
            if (ok) {
                int cx, cy;
                hash_cell(h, q.x, q.y, cx, cy);
                bk[k] = cy * h.nx + cx;
                rk[k] = atomicAdd(&bstart[bk[k] + 1], 1);
            }
        }
    }
    __syncthreads();
    {   // bucket starts: each thread scans its run of 2 buckets (nb <= 2048)
        const int b0 = 2 * tid + 1;
        const int c0 = b0 <= nb ? bstart[b0] : 0, c1 = b0 + 1 <= nb ? bstart[b0 + 1] : 0;
        int tot;
        const int before = block_excl_scan<kSmallTB>(c0 + c1, wsum, &tot);
        if (b0 <= nb) bstart[b0] = before + c0;
        if (b0 + 1 <= nb) bstart[b0 + 1] = before + c0 + c1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k)
        if (bk[k] >= 0) items[bstart[bk[k]] + rk[k]] = tid * kSmallPer + k;
    __syncthreads();
    // rounds over the undecided candidates (a stale LDS read only postpones a decision)
    for (int round = 0;; ++round) {
        bool und = false;
#pragma unroll
        for (int k = 0; k < kSmallPer; ++k) {
            const int i = tid * kSmallPer + k;
            if (i >= n || st[i] != 0) continue;
            const double2 q = pts[i];
            int cx, cy;
            hash_cell(h, q.x, q.y, cx, cy);
            bool kept_c = false, und_c = false;
            for (int yy = max(cy - 1, 0); yy <= min(cy + 1, h.ny - 1) && !kept_c; ++yy) {
                const int k0 = bstart[yy * h.nx + max(cx - 1, 0)], k1 = bstart[yy * h.nx + min(cx + 1, h.nx - 1) + 1];
                for (int kk = k0; kk < k1; ++kk) {
                    const int j = items[kk];
                    if (j >= i || !conflict(q, pts[j], A.mode, A.thr)) continue;
                    const int sj = st[j];
                    if (sj == 1) { kept_c = true; break; }
                    if (sj == 0) und_c = true;
                }
            }
            if (kept_c) st[i] = 2;
            else if (!und_c) st[i] = 1;
            else und = true;
        }
        if (!__syncthreads_or(und)) break;
        if (round > n + 2) {   // (cannot happen: the smallest undecided candidate decides every round)
            if (tid == 0) atomicOr(A.err, 4);
            break;
        }
    }
    // compaction in index order
    int c = 0;
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        const int i = tid * kSmallPer + k;
        c += (i < n && st[i] == 1) ? 1 : 0;
    }
    int tot;
    int pos = block_excl_scan<kSmallTB>(c, wsum, &tot);
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        const int i = tid * kSmallPer + k;
        if (i < n && st[i] == 1) P.out[pos++] = pts[i];
    }
    if (tid == 0) *P.count = tot;
}

// ------------------------------------------------------------------ host API
void greedy_dedup_async(DedupScratch &S, const double2 *cand, const int *ok, int n, int mode, double thr, const HashG &h,
                        double2 *out, int *kept_index, int *owner, int *d_count, hipStream_t s, int *pos_of) {
    if (n <= 0) {
        AOS_HIP(hipMemsetAsync(d_count, 0, sizeof(int), s));
        return;
    }
    S.cells.lb.ext_err = dedup_err(S, s);   // (one error word for all of S's launches)
    S.ci = cell_index_build(S.cells, cand, ok, n, h, s);
    const size_t cap0 = S.state.cap;
    int *state = dev<int>(S.state, n);
    if (S.state.cap != cap0) AOS_HIP(hipMemsetAsync(state, 0, S.state.cap, s));   // (epoch 0: undecided)
    if (++S.epoch >= (1u << 29)) {
        S.epoch = 1;
        AOS_HIP(hipMemsetAsync(state, 0, S.state.cap, s));
    }
    const int blocks = cdiv(n, kLfTB);
    const bool self = mode == kConflictKeyOrSq || (mode == kConflictLessEq && thr >= 0.0) || (mode == kConflictLess && thr > 0.0);
    LfArgs A{cand, ok, n, mode, thr, self ? 1 : 0, S.ci, state, S.epoch, S.lb.take(blocks, s), out, kept_index, owner, d_count,
             pos_of};
    if (owner) k_lfmis<true><<<blocks, kLfTB, 0, s>>>(A);
    else k_lfmis<false><<<blocks, kLfTB, 0, s>>>(A);
    AOS_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ read-backs without the copy engine
static bool zc_readback() {
    static const bool on = [] { const char *e = getenv("AOS_ZC_READBACK"); return !e || atoi(e) != 0; }();
    return on;
}
struct PeekArgs { const int *src[kPeekMax]; int n; };
__global__ void k_peek_host(PeekArgs P, int *h_dst) {
    if ((int)threadIdx.x < P.n) h_dst[threadIdx.x] = *P.src[threadIdx.x];
}
void peek_to_host(int *h_dst, std::initializer_list<const int *> srcs, hipStream_t s) {
    if ((int)srcs.size() > kPeekMax) throw std::runtime_error("peek_to_host: too many values");
    if (!zc_readback()) {
        int k = 0;
        for (const int *p : srcs) AOS_HIP(hipMemcpyAsync(h_dst + k++, p, sizeof(int), hipMemcpyDeviceToHost, s));
        return;
    }
    PeekArgs P{};
    for (const int *p : srcs) P.src[P.n++] = p;
    k_peek_host<<<1, 64, 0, s>>>(P, h_dst);
    AOS_HIP(hipGetLastError());
}
// 16-byte words while both ends are 16-byte aligned and the size a multiple of 16, else 4-byte words, else bytes
template <class W>
__global__ void k_copy_host(W *h_dst, const W *d_src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        h_dst[i] = d_src[i];
}
static void copy_kernel(void *h_dst, const void *d_src, size_t bytes, hipStream_t s, int max_blocks = 256) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(h_dst) | reinterpret_cast<uintptr_t>(d_src) | bytes;
    auto go = [&](auto *dst, const auto *src, size_t n) {
        const int blocks = (int)std::min<size_t>((size_t)max_blocks, (n + 255) / 256);
        k_copy_host<<<blocks, 256, 0, s>>>(dst, src, n);
    };
    if (!(a & 15)) go(static_cast<uint4 *>(h_dst), static_cast<const uint4 *>(d_src), bytes / 16);
    else if (!(a & 3)) go(static_cast<unsigned *>(h_dst), static_cast<const unsigned *>(d_src), bytes / 4);
    else go(static_cast<unsigned char *>(h_dst), static_cast<const unsigned char *>(d_src), bytes);
    AOS_HIP(hipGetLastError());
}
void copy_to_host(void *h_dst, const void *d_src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    if (zc_readback()) copy_kernel(h_dst, d_src, bytes, s);
    else AOS_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, s));
}
void copy_kernel_bulk(void *dst, const void *src, size_t bytes, int blocks, hipStream_t s) {
    if (bytes) copy_kernel(dst, src, bytes, s, blocks);
}
void copy_from_host(void *d_dst, const void *h_src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    if (zc_readback()) copy_kernel(d_dst, h_src, bytes, s);
    else AOS_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, s));
}

int *dedup_err(DedupScratch &S, hipStream_t s) { return S.lb.err_word(s); }

void dedup_check(DedupScratch &S, int err_word) {
    if (!err_word) return;
    // a stale ticket or a wait past the cap (never expected): reset the shared words, report
    S.lb.ticket.release();
    S.lb.err.release();
    S.lb.part.release();
    S.cells.lb.ticket.release();
    S.cells.lb.part.release();
    S.cells.lb.ext_err = nullptr;
    S.cells.dirty = true;
    throw std::runtime_error("greedy de-duplication: device wait failed (error word " + std::to_string(err_word) + ")");
}

int greedy_dedup(DedupScratch &S, const double2 *cand, const int *ok, int n, int mode, double thr, const HashG &h,
                 double2 *out, int *kept_index_out, hipStream_t s, int *h_scalar) {
    if (n <= 0) return 0;
    int *d = dev<int>(S.misc, 2);
    greedy_dedup_async(S, cand, ok, n, mode, thr, h, out, kept_index_out, nullptr, d, s);
    AOS_HIP(hipMemcpyAsync(h_scalar, d, sizeof(int), hipMemcpyDeviceToHost, s));
    AOS_HIP(hipMemcpyAsync(h_scalar + 1, dedup_err(S, s), sizeof(int), hipMemcpyDeviceToHost, s));
    S.sev.sync(s);
    dedup_check(S, h_scalar[1]);
    return h_scalar[0];
}

void greedy_dedup_small(DedupScratch &S, SmallDedup A, int nprob, hipStream_t s) {
    if (nprob <= 0) return;
    for (int k = 0; k < nprob; ++k)
        if (A.prob[k].n > kSmallMax || (long long)A.prob[k].h.nx * A.prob[k].h.ny > kSmallBuckets)
            throw std::logic_error("greedy_dedup_small: problem too large");
    A.err = dedup_err(S, s);
    k_dedup_small<<<nprob, kSmallTB, 0, s>>>(A);
    AOS_HIP(hipGetLastError());
}

HashG small_hash(double minx, double maxx, double miny, double maxy, double cell) {
    return make_hash_cap(minx, maxx, miny, maxy, cell, (double)kSmallBuckets);
}

}  // namespace aos
