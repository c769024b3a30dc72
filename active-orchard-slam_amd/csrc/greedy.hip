// Greedy first-come de-duplication on the GPU (see cluster_seed.h).
//
// Reference loops of the form
//   for c in candidates (in order): if no already-kept k conflicts with c: keep c
// (seed_gen:2076-2085, 1964-1974, 1460-1470; gvd:98-125; voronoi_diagram.cpp:156-204) keep exactly
// the lexicographically-first maximal independent set (LFMIS) of the conflict graph. We hash the
// candidates into cells no smaller than the conflict radius, list each candidate's EARLIER
// conflicting candidates (CSR), and decide the LFMIS in rounds over the whole grid:
// undecided c becomes kept when all listed predecessors are removed, removed once one is kept.
// Decisions are facts about the final set, so in-place updates are safe; the smallest undecided
// index always decides, so the loop terminates.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <stdexcept>

#include "cluster_seed.h"

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

__device__ __forceinline__ void hash_cell(const HashG &h, double x, double y, int &cx, int &cy) {
    double fx = (x - h.x0) * h.inv, fy = (y - h.y0) * h.inv;
    cx = !(fx > 0.0) ? 0 : (fx >= (double)(h.nx - 1) ? h.nx - 1 : (int)fx);
    cy = !(fy > 0.0) ? 0 : (fy >= (double)(h.ny - 1) ? h.ny - 1 : (int)fy);
}

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

// (also zeroes the scans' tail slots ccount[n] and f[n], instead of two memset blits)
__global__ void k_hash_keys(const double2 *p, const int *ok, int n, HashG h, int *keys, int *idx, int *tail0,
                            int *tail1) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) { *tail0 = 0; *tail1 = 0; }
    if (i >= n) return;
    int cx, cy;
    hash_cell(h, p[i].x, p[i].y, cx, cy);
    keys[i] = ok[i] ? cy * h.nx + cx : INT_MAX;
    idx[i] = i;
}

__device__ __forceinline__ int lower_bound_key(const int *keys, int n, int k) {
    int lo = 0, hi = n;
    while (lo < hi) { int m = (lo + hi) >> 1; if (keys[m] < k) lo = m + 1; else hi = m; }
    return lo;
}

__device__ __forceinline__ int lower_bound_in(const int *keys, int lo, int hi, int k) {
    while (lo < hi) { int m = (lo + hi) >> 1; if (keys[m] < k) lo = m + 1; else hi = m; }
    return lo;
}

// First sorted index of every hash row (cell ids are row-major): narrows each cell lookup of
// k_conflicts from a binary search over all n keys (~17 dependent loads) to one over one row's keys.
__global__ void k_row_starts(const int *skeys, int n, HashG h, int *rowstart) {
    const int yy = blockIdx.x * blockDim.x + threadIdx.x;
    if (yy <= h.ny) rowstart[yy] = lower_bound_key(skeys, n, yy * h.nx);
}

// coff == nullptr: count pass; else fill pass
__global__ void k_conflicts(const double2 *p, const int *ok, int n, HashG h, const int *skeys, const int *sidx,
                            const int *rowstart, int mode, double thr, const int *coff, int *ccount, int *clist,
                            long long cap) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (!ok[i]) { if (!coff) ccount[i] = 0; return; }
    int cx, cy;
    hash_cell(h, p[i].x, p[i].y, cx, cy);
    const double2 pi = p[i];
    int c = 0, w = coff ? coff[i] : 0;
    for (int yy = max(cy - 1, 0); yy <= min(cy + 1, h.ny - 1); ++yy) {
        const int hi = rowstart[yy + 1];
        const int k0 = lower_bound_in(skeys, rowstart[yy], hi, yy * h.nx + max(cx - 1, 0));
        const int k1 = lower_bound_in(skeys, k0, hi, yy * h.nx + min(cx + 1, h.nx - 1) + 1);
        for (int k = k0; k < k1; ++k) {
            int j = sidx[k];
            if (j < i && conflict(pi, p[j], mode, thr)) {
                if (coff && (long long)w + c < cap) clist[w + c] = j;   // overflow: host re-runs with the exact size
                ++c;
            }
        }
    }
    if (!coff) ccount[i] = c;
}

__global__ void k_greedy_init(const int *ok, int n, int *state) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) state[i] = ok[i] ? 0 : 2;
}
// One round over all undecided candidates, any number of workgroups. States are read with
// agent-scope loads (another workgroup may have decided a predecessor in this very round); a
// stale read only postpones a decision to a later round. undecided[0] counts candidates still
// undecided when this round looked at them: 0 means the set is complete, and the later rounds of a
// batch (prev_undecided = the previous round's counter) return at once.
__global__ void k_greedy_round(int n, const int *coff, const int *clist, int *state, int *undecided,
                               const int *prev_undecided) {
    if (prev_undecided && *prev_undecided == 0) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool und = false;
    if (i < n && __hip_atomic_load(&state[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        bool any_kept = false, any_undec = false;
        for (int k = coff[i]; k < coff[i + 1]; ++k) {
            int sj = __hip_atomic_load(&state[clist[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (sj == 1) { any_kept = true; break; }
            if (sj == 0) any_undec = true;
        }
        int ns = any_kept ? 2 : (any_undec ? 0 : 1);
        if (ns) __hip_atomic_store(&state[i], ns, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else und = true;
    }
    unsigned long long m = __ballot(und);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(undecided, (int)__popcll(m));
}

__global__ void k_kept_flags(const int *state, int n, int *f) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) f[i] = state[i] == 1;
}
// (thread 0 also gathers the batch's three read-back scalars into one slot run: one D2H copy, not three)
__global__ void k_compact(const double2 *p, const int *f, const int *pos, int n, double2 *out, int *kept_index,
                          const int *und_last, const int *n_conf, int *scalars) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) { scalars[0] = *und_last; scalars[1] = *n_conf; scalars[2] = pos[n]; }
    if (i < n && f[i]) {
        out[pos[i]] = p[i];
        if (kept_index) kept_index[pos[i]] = i;
    }
}

template <class T> static T *dev(DevBuf &b, size_t n) { return static_cast<T *>(b.ensure(sizeof(T) * std::max<size_t>(n, 1))); }

int greedy_dedup(DedupScratch &S, const double2 *cand, const int *ok, int n, int mode, double thr, const HashG &h,
                 double2 *out, int *kept_index_out, hipStream_t s, int *h_scalar) {
    if (n <= 0) return 0;
    int *keys = dev<int>(S.keys, n), *idx = dev<int>(S.idx, n), *skeys = dev<int>(S.skeys, n), *sidx = dev<int>(S.sidx, n);
    int *ccount = dev<int>(S.ccount, n + 1), *coff = dev<int>(S.coff, n + 1);
    int *f = dev<int>(S.f, n + 1), *pos = dev<int>(S.pos, n + 1);
    k_hash_keys<<<cdiv(n, 256), 256, 0, s>>>(cand, ok, n, h, keys, idx, ccount + n, f + n);
    size_t tb = 0, tb2 = 0;
    AOS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, skeys, idx, sidx, n, 0, 32, s));
    AOS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, (int *)nullptr, (int *)nullptr, n + 1, s));
    void *tmp = S.tmp.ensure(std::max(tb, tb2));
    AOS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, skeys, idx, sidx, n, 0, 32, s));
    int *rows = dev<int>(S.rows, (size_t)h.ny + 1);
    k_row_starts<<<cdiv(h.ny + 1, 256), 256, 0, s>>>(skeys, n, h, rows);
    k_conflicts<<<cdiv(n, 256), 256, 0, s>>>(cand, ok, n, h, skeys, sidx, rows, mode, thr, nullptr, ccount, nullptr, 0);
    AOS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, ccount, coff, n + 1, s));
    // Optimistic capacity for the conflict lists (no read-back of the exact total before the rounds):
    // the total comes back with the first round batch; on overflow the lists are rebuilt exactly.
    long long cap = std::max<long long>((long long)(S.clist.cap / sizeof(int)), 8LL * n);
    int *clist = dev<int>(S.clist, (size_t)cap);
    int *state = dev<int>(S.state, n);
    constexpr int kBatch = 6;
    int *und = dev<int>(S.und, kBatch + 3);   // round counters, then the three read-back scalars
    auto fill = [&]() {
        k_conflicts<<<cdiv(n, 256), 256, 0, s>>>(cand, ok, n, h, skeys, sidx, rows, mode, thr, coff, nullptr, clist, cap);
        k_greedy_init<<<cdiv(n, 256), 256, 0, s>>>(ok, n, state);
    };
    fill();
    for (int done_rounds = 0;;) {
        // a batch of rounds, then (speculatively) the compaction of the kept set, one read-back
        AOS_HIP(hipMemsetAsync(und, 0, sizeof(int) * kBatch, s));
        for (int r = 0; r < kBatch; ++r)
            k_greedy_round<<<cdiv(n, 256), 256, 0, s>>>(n, coff, clist, state, und + r, r ? und + r - 1 : nullptr);
        k_kept_flags<<<cdiv(n, 256), 256, 0, s>>>(state, n, f);
        AOS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, f, pos, n + 1, s));
        k_compact<<<cdiv(n, 256), 256, 0, s>>>(cand, f, pos, n, out, kept_index_out, und + kBatch - 1, coff + n, und + kBatch);
        AOS_HIP(hipMemcpyAsync(h_scalar, und + kBatch, 3 * sizeof(int), hipMemcpyDeviceToHost, s));
        S.sev.sync(s);
        S.n_conf = h_scalar[1];
        if ((long long)S.n_conf > cap) {   // conflict lists were truncated: rebuild at the exact size
            cap = S.n_conf;
            clist = dev<int>(S.clist, (size_t)cap);
            fill();
            done_rounds = 0;
            continue;
        }
        done_rounds += kBatch;
        if (h_scalar[0] == 0) return h_scalar[2];
        if (done_rounds > n + kBatch) throw std::runtime_error("greedy de-duplication did not converge");
    }
}

}  // namespace aos
