// Device-side helpers of dev_prims.h (hash cells, cell-index rows, look-back): included by the .hip files
// only (dev_prims.h stays host-compilable for the sanitizer build). Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "dev_prims.h"
#include "dev_wave.h"

namespace aos {

__device__ __forceinline__ void hash_cell(const HashG &h, double x, double y, int &cx, int &cy) {
    const double fx = (x - h.x0) * h.inv, fy = (y - h.y0) * h.inv;
    cx = !(fx > 0.0) ? 0 : (fx >= (double)(h.nx - 1) ? h.nx - 1 : (int)fx);
    cy = !(fy > 0.0) ? 0 : (fy >= (double)(h.ny - 1) ? h.ny - 1 : (int)fy);
}

// the run of the 3 buckets (cx - 1 .. cx + 1) of row yy (clamped): [k0, k1)
__device__ __forceinline__ void ci_row(const CellIdx &c, int yy, int cx, int &k0, int &k1) {
    const int b = yy * c.h.nx;
    k0 = c.start[b + max(cx - 1, 0)];
    k1 = c.start[b + min(cx + 1, c.h.nx - 1) + 1];
}

// The items of a cell-index run [k0, k1) in batches of B whose loads are in flight together: B item indices, then
// load(j) for each (the caller's per-item reads, independent of one another), then use(j, v) in run order. A run
// walked one item at a time is a chain of two or three dependent global loads per item (round 5: the GVD
// searches spent most of their time waiting on it). use returns false to stop the walk; walk_items returns
// false when it was stopped.
template <int B, class Load, class Use>
__device__ __forceinline__ bool walk_items(const int *items, int k0, int k1, Load load, Use use) {
    for (int k = k0; k < k1; k += B) {
        int j[B];
#pragma unroll
        for (int u = 0; u < B; ++u) j[u] = k + u < k1 ? items[k + u] : -1;
        decltype(load(0)) v[B];
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (j[u] >= 0) v[u] = load(j[u]);
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (j[u] >= 0 && !use(j[u], v[u])) return false;
    }
    return true;
}

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

struct IAdd { __device__ int operator()(int a, int b) const { return a + b; } };
// (DPP row moves, dev_wave.h: the look-back's sums sit on the scans' critical path)
__device__ __forceinline__ unsigned wave_sum_u32(unsigned v) { return (unsigned)wave_reduce((int)v, 0, IAdd()); }

// Wave 0 of block vid (all 64 lanes): publishes the block's aggregate, walks back over the
// predecessors' words 64 at a time, publishes the inclusive prefix; returns the exclusive prefix. A wait
// past kSpinCap ORs errbit into *L.err.
__device__ inline unsigned lb_exclusive(const LookBack &L, int vid, unsigned agg, int errbit = 1) {
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
                if (lane == 0) atomicOr(L.err, errbit);
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
    const int incl = wave_scan_incl(v, 0, IAdd());
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

// The exclusive scan of a producer kernel's per-item values, fused into the producer (round 5: one launch and
// one pass less than producer + k_scan_1p). Block vid (lb_block_id) owns items [vid NT, (vid + 1) NT); the
// grid covers n + 1 items (the host launches lb_scan_blocks(n, NT)), every thread of every block calls this
// with its item's value (0 past n), and out[i] = v[0] + ... + v[i - 1] for i in [0, n] (out[n] = the total).
struct LbScanShared { int wsum[16], tot, excl; };
template <int NT>
__device__ __forceinline__ void lb_scan_store(const LookBack &L, int vid, int v, int n, int *out, LbScanShared &sh) {
    const int i = vid * NT + (int)threadIdx.x;
    const int before = block_excl_scan<NT>(v, sh.wsum, &sh.tot);
    if (threadIdx.x < 64) {
        const unsigned e = lb_exclusive(L, vid, (unsigned)sh.tot);
        if (threadIdx.x == 0) sh.excl = (int)e;
    }
    __syncthreads();
    if (i <= n) out[i] = sh.excl + before;
}
// The same for producers whose blocks own runs of items that are not NT long (a 2-D grid over the rows of a
// bit grid): the thread's item index i (-1: none; items increase with thread index inside a block and with
// vid across blocks), out[i] = the exclusive prefix and, from the thread holding item last, out[last + 1] =
// the total.
template <int NT>
__device__ __forceinline__ void lb_scan_store_at(const LookBack &L, int vid, int v, long long i, long long last, int *out,
                                                 LbScanShared &sh) {
    const int before = block_excl_scan<NT>(v, sh.wsum, &sh.tot);
    if (threadIdx.x < 64) {
        const unsigned e = lb_exclusive(L, vid, (unsigned)sh.tot);
        if (threadIdx.x == 0) sh.excl = (int)e;
    }
    __syncthreads();
    if (i >= 0) out[i] = sh.excl + before;
    if (i == last) out[i + 1] = sh.excl + before + v;
}

}  // namespace aos
