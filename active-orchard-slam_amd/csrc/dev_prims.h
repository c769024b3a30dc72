// Device primitives shared by the cluster, seed and GVD stages (greedy.hip defines the kernels):
//   * single-pass decoupled look-back: dynamic block ids in launch order + per-block partial words
//     tagged with the launch's epoch, so no launch needs an init kernel or a memset;
//   * a uniform-hash cell index built by counting sort (count, one single-pass scan, scatter) instead
//     of a radix sort of (cell, index) pairs: three launches, bucket b's items in items[start[b] ..
//     start[b + 1]); a 3 x 3 neighbourhood is three contiguous runs (buckets are row-major).
// Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "aos_internal.h"

namespace aos {

// ------------------------------------------------------------------ uniform hash over the plane
struct HashG { double x0, y0, inv; int nx, ny; };
// cells of side >= cell over [minx, maxx] x [miny, maxy]; points outside are clamped into the border cells
HashG make_hash(double minx, double maxx, double miny, double maxy, double cell);
// the same with the cell enlarged (never shrunk) until nx * ny <= max(4096, cells_per_item * n): a bucket
// table a counting sort can scan. Coarser cells only add candidates that the exact tests then reject.
HashG make_hash_n(double minx, double maxx, double miny, double maxy, double cell, long long n, double cells_per_item = 2.0);

__device__ __forceinline__ void hash_cell(const HashG &h, double x, double y, int &cx, int &cy) {
    const double fx = (x - h.x0) * h.inv, fy = (y - h.y0) * h.inv;
    cx = !(fx > 0.0) ? 0 : (fx >= (double)(h.nx - 1) ? h.nx - 1 : (int)fx);
    cy = !(fy > 0.0) ? 0 : (fy >= (double)(h.ny - 1) ? h.ny - 1 : (int)fy);
}

// Items of the hash's buckets: bucket b = cy * nx + cx holds items[start[b] .. start[b + 1]).
struct CellIdx {
    HashG h;
    const int *start, *items;
};
// the run of the 3 buckets (cx - 1 .. cx + 1) of row yy (clamped): [k0, k1)
__device__ __forceinline__ void ci_row(const CellIdx &c, int yy, int cx, int &k0, int &k1) {
    const int b = yy * c.h.nx;
    k0 = c.start[b + max(cx - 1, 0)];
    k1 = c.start[b + min(cx + 1, c.h.nx - 1) + 1];
}

// ------------------------------------------------------------------ look-back
constexpr unsigned kSpinCap = 1u << 21;   // a wait that outlasts this sets the error word (never expected)
struct LookBack {
    unsigned long long *part;   // per block: (tag << 32) | value, tag = epoch << 2 | flag (1 aggregate, 2 prefix)
    unsigned *ticket;           // dynamic block ids; the block that draws the last id resets it to 0
    unsigned epoch;             // of this launch (>= 1; words of other launches read as "not yet")
    int *err;                   // | 1 on a stale ticket or a wait past kSpinCap
};

__device__ __forceinline__ unsigned long long ld_u64(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u64(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_i32(const int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_i32(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// The block's id in launch order: a block only ever waits for blocks with smaller ids, which have all
// started (they drew their ids first), so the waits cannot deadlock whatever the dispatch order.
__device__ __forceinline__ int lb_block_id(const LookBack &L, int *sh) {
    if (threadIdx.x == 0) {
        const unsigned v = atomicAdd(L.ticket, 1u);
        if (v == gridDim.x - 1) __hip_atomic_store(L.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= gridDim.x) atomicOr(L.err, 1);
        *sh = (int)(v % gridDim.x);
    }
    __syncthreads();
    return *sh;
}

__device__ __forceinline__ unsigned wave_sum_u32(unsigned v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Wave 0 of block vid (all 64 lanes): publishes the block's aggregate, walks back over the
// predecessors' words 64 at a time, publishes the inclusive prefix; returns the exclusive prefix.
__device__ inline unsigned lb_exclusive(const LookBack &L, int vid, unsigned agg) {
    const int lane = threadIdx.x & 63;
    const unsigned long long tagA = (unsigned long long)((L.epoch << 2) | 1u) << 32;
    const unsigned long long tagP = (unsigned long long)((L.epoch << 2) | 2u) << 32;
    if (vid == 0) {
        if (lane == 0) st_u64(&L.part[0], tagP | agg);
        return 0;
    }
    if (lane == 0) st_u64(&L.part[vid], tagA | agg);
    unsigned excl = 0;
    int base = vid - 1;
    unsigned spins = 0;
    for (;;) {
        const int j = base - lane;
        unsigned flag = 2, val = 0;
        for (;;) {
            if (j >= 0) {
                const unsigned long long w = ld_u64(&L.part[j]);
                const unsigned tag = (unsigned)(w >> 32);
                flag = (tag >> 2) == L.epoch ? (tag & 3u) : 0u;
                val = (unsigned)w;
            }
            if (__all(flag != 0)) break;
            if (++spins > kSpinCap) {
                if (lane == 0) atomicOr(L.err, 1);
                flag = 2;
                val = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const unsigned long long pm = __ballot(flag == 2);
        if (pm) {
            const int k = __ffsll((long long)pm) - 1;
            excl += wave_sum_u32(lane <= k ? val : 0u);
            break;
        }
        excl += wave_sum_u32(val);
        base -= 64;
    }
    if (lane == 0) st_u64(&L.part[vid], tagP | (unsigned long long)(excl + agg));
    return excl;
}

// Exclusive scan of one value per thread over a block of NT threads (NT a multiple of 64); total -> *tot
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int *wsum, int *tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        const int s = wsum[k];
        before += k < w ? s : 0;
        all += s;
    }
    *tot = all;
    __syncthreads();
    return before + incl - v;
}

// ------------------------------------------------------------------ host side
// Look-back words + ticket of one stream's launches; epochs advance per launch (zeroed storage reads as
// "not yet"; the words are cleared again if the 30-bit epoch ever wraps).
struct LookBackScratch {
    DevBuf part, ticket, err;
    unsigned epoch = 0;
    int *ext_err = nullptr;         // set: report into this word instead of err
    LookBack take(int blocks, hipStream_t s);
    int *err_word(hipStream_t s);   // zeroed on allocation
};

// Single-pass exclusive scan: out[k] = in[0] + .. + in[k - 1] for k in [0, n] (out[n] = total); in is
// zeroed after it is read when zero_in (the cell index keeps its bucket counts zero between uses).
void scan_1p(LookBackScratch &lb, int *in, int *out, int n, bool zero_in, hipStream_t s);

// Cell index of the points with ok[i] != 0 (ok nullable: all) and i < *n_dev (n_dev nullable: n is exact;
// else n is an upper bound of a count the host has not read), counting sort into the hash's buckets.
struct CellScratch {
    DevBuf cnt, start, items, rank;
    LookBackScratch lb;
    bool dirty = true;   // counts not known to be zero (first use, or a build cut short)
};
CellIdx cell_index_build(CellScratch &S, const double2 *p, const int *ok, int n, const HashG &h, hipStream_t s,
                         const int *n_dev = nullptr);

}  // namespace aos
