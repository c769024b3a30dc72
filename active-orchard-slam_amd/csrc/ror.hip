// a1-a4 RadiusOutlierRemoval + PassThrough + exclusion discs + raster (seed_gen:230-248, 452-622) as
// a two-level spatial partition for gfx950.
//
// The reference runs PCL's RadiusOutlierRemoval (kd-tree, k = minN + 1 nearest neighbours in 3-D)
// over the whole cloud, then clips and rasterises. Only points inside the clip box can reach the
// grid, and their neighbours lie within r of that box, so only that expanded ("binned") box matters.
// Here the binned box is cut into square bins of side >= r (a neighbour of p lies in p's 3 x 3 bins)
// and the bins into tiles of TB x TB bins:
//   k_rt_part<false>  count: per tile, the points whose 3 x 3 bins reach it (own tile + up to 3
//                     halo tiles). Per-workgroup LDS histograms, one global atomic per touched tile.
//   scan              tile_start = exclusive sum of the counts.
//   k_rt_part<true>   scatter: the same walk, each workgroup claims one run per touched tile with a
//                     returning atomic and writes its points there (w = 1: an own clip candidate,
//                     else 0: a neighbour only — non-candidates and halo copies).
//   k_rt_ror          one workgroup per tile: the tile's points (own + halo) are counting-sorted by
//                     bin into LDS, every own candidate counts neighbours in its 3 x 3 bins from
//                     LDS with early exit, and kept candidates set their cell in an LDS bitmap of
//                     the tile's cells that is OR-ed into the bit-packed raster at the end.
// The cloud is read twice (count, scatter) and every staged point written and read once; no
// per-point global atomic, no random gather. Results are order-free: the keep decision needs only
// "at least need points within r", and the raster is an OR.
//
// Numerics: FLANN's squared distance ((dx*dx)+dy*dy)+dz*dz in float, no FMA (-ffp-contract=off);
// this file is built with -fno-slp-vectorize (Makefile): the SLP vectorizer paired y / z of the partition
// passes' dwordx3 loads into aligned register pairs, and the moves made every load wait before use;
// dense clouds: kNN keeps iff the need-th nearest has (double)d2 <= r^2, i.e. d2 <= r2df (the
// largest float whose double is <= r^2); non-dense: radius search d2 < float(r^2). The point itself
// has d2 = 0 and is counted by the same test (not counted when r = 0 on a non-dense cloud, as FLANN's
// strict test does). Cells: generateOccupancyGrid's (int)(((double)x - origin) / (double)res).
#include <algorithm>
#include <climits>
#include <cmath>
#include <stdexcept>
#include <type_traits>

#include "aos_internal.h"
#include "dev_prims_device.h"

namespace aos {

// Exclusion discs of processPointCloud (seed_gen:487-499): x, y, radius.
__constant__ float c_excl_rt[11 * 3] = {0.646417f, 3.83918f, 1.0f,  2.0405f, 3.62485f, 1.0f,  65.3711f, 2.09755f, 1.0f,
                                        66.9094f, 2.07515f, 1.0f,  -1.61309f, 5.69933f, 1.0f, -1.97349f, 4.77329f, 1.0f,
                                        -2.11365f, 3.74464f, 1.0f, -2.26381f, 2.70848f, 1.0f, -2.66426f, 1.72738f, 1.0f,
                                        68.0229f, 2.31687f, 1.0f,  65.4647f, 2.18653f, 1.0f};


// Record layout LAY: 1 = the common PointCloud2 layout (point_step 16, x/y/z at 0/4/8): one 16 B load per
// point; 2 = the packed float3 cloud the host upload writes (step 12); 0 = any float32 x/y/z offsets
template <int LAY>
__device__ __forceinline__ void rt_load(const RorLaunch &L, uint64_t i, float &x, float &y, float &z) {
    const uint8_t *rec = L.cloud + i * (uint64_t)(LAY == 1 ? 16 : LAY == 2 ? 12 : L.step);
    if (LAY == 1) {
        const float4 v = *reinterpret_cast<const float4 *>(rec);
        x = v.x; y = v.y; z = v.z;
    } else if (LAY == 2) {
        const float *r = reinterpret_cast<const float *>(rec);
        x = r[0]; y = r[1]; z = r[2];
    } else {
        x = *reinterpret_cast<const float *>(rec + L.ox);
        y = *reinterpret_cast<const float *>(rec + L.oy);
        z = *reinterpret_cast<const float *>(rec + L.oz);
    }
}

__device__ __forceinline__ bool rt_binned(const RorLaunch &L, float x, float y, float z) {
    return isfinite(x) && isfinite(y) && isfinite(z) && x >= L.bminx && x <= L.bmaxx && y >= L.bminy &&
           y <= L.bmaxy && z >= L.bminz && z <= L.bmaxz;
}

__device__ __forceinline__ void rt_bin(const RorLaunch &L, float x, float y, int &bx, int &by) {
    bx = min(max((int)((x - L.bminx) * L.inv_cs), 0), L.nbx - 1);
    by = min(max((int)((y - L.bminy) * L.inv_cs), 0), L.nby - 1);
}

// PassThrough z, x, y (inclusive; PCL 1.12 drops non-finite) + exclusion discs, seed_gen:459-525.
__device__ __forceinline__ bool rt_candidate(const RorLaunch &L, float x, float y, float z) {
    if (z < L.cminz || z > L.cmaxz) return false;
    if (x < L.cminx || x > L.cmaxx) return false;
    if (y < L.cminy || y > L.cmaxy) return false;
    // the discs' union lies in x [-3.664, 69.023], y [0.727, 6.700] (centres +- 1): a point 0.01 or more
    // outside that box has dx^2 >= 1.02 > 1 for every disc (float rounding moves dx^2 by 1 ulp), so the
    // loop below cannot remove it
    if (x < -3.68f || x > 69.04f || y < 0.71f || y > 6.72f) return true;
#pragma unroll
    for (int e = 0; e < 11; ++e) {
        float dx = x - c_excl_rt[3 * e], dy = y - c_excl_rt[3 * e + 1];
        float dist_sq = dx * dx + dy * dy;
        float rr = c_excl_rt[3 * e + 2] * c_excl_rt[3 * e + 2];
        if (dist_sq <= rr) return false;
    }
    return true;
}

// generateOccupancyGrid's cell index (int)(a / res), a = (double)x - origin, without the f64 division in
// the common case: q = a * (1 / res) is within 3.3e-16 |q| of the rounded quotient, so its truncation is
// the quotient's unless an integer lies within that distance; q within 1e-14 |q| of an integer takes the
// exact division. (Two f64 divisions per kept candidate were ~20 % of k_rt_ror's VALU issue.)
// The exact division sits behind a wave-uniform branch: as a plain per-lane branch the compiler if-converted
// it, so every call paid the f64 division sequence (~20 f64 instructions) whatever the lanes needed.
__device__ __forceinline__ int rt_cell(double a, double res, double inv_res) {
    const double q = a * inv_res;
    const double t = trunc(q), d = fabs(q - t), tol = fabs(q) * 1e-14 + 1e-300;
    const bool exact = d < tol || d > 1.0 - tol;
    int c = (int)t;
    if (__builtin_amdgcn_ballot_w64(exact)) {   // (rare: some lane of the wave is within tol of an integer)
        const int e = (int)(a / res);
        c = exact ? e : c;
    }
    return c;
}

// dense: (double)d2 <= r2, i.e. d2 <= r2df; non-dense: d2 < r2f, i.e. d2 <= the float below r2f: both are
// d2 <= L.r2cmp (rt_configure), one compare in the inner loops
__device__ __forceinline__ bool rt_in(const RorLaunch &L, float4 p, float4 q) {
    float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
    float d2 = dx * dx;
    d2 = d2 + dy * dy;
    d2 = d2 + dz * dz;
    return d2 <= L.r2cmp;
}

// ---------------------------------------------------------------------------------------------
// Passes 1 and 3: count / scatter, a radix-sort style partition with one digit per tile. Workgroup
// w owns one contiguous chunk of the cloud. The count pass accumulates an LDS histogram over the
// chunk and stores it as row w of H (H[w * ntiles + t], a coalesced store); k_rt_colscan turns the
// columns into per-tile exclusive prefixes over the workgroups plus tile totals, one small scan of
// the totals gives the tile starts, and the scatter pass walks the same chunk again with LDS
// cursors starting at tile start + prefix. No global atomics; a tile's run from workgroup w sits
// right after workgroup w - 1's.
// block sizes: the count pass runs best at 256 threads, the scatter pass at 512 (measured,
// tools/rorbench); both walk the same per-workgroup chunks (a multiple of kRtChunkQ points)
#ifndef AOS_RT_CPER
#define AOS_RT_CPER 8
#endif
#ifndef AOS_RT_SPER
#define AOS_RT_SPER 4
#endif
#ifndef AOS_RT_CTB
#define AOS_RT_CTB 256
#endif
#ifndef AOS_RT_G
#define AOS_RT_G 512
#endif
#ifndef AOS_RT_STB   // scatter pass block size
#define AOS_RT_STB 512
#endif
#ifndef AOS_RT_COLROWS   // rows of H per k_rt_colscan block
#define AOS_RT_COLROWS 32
#endif
#ifndef AOS_RT_NT   // nontemporal cloud loads: bit 0 count pass, bit 1 scatter pass
#define AOS_RT_NT 0
#endif
constexpr int kRtCountPer = AOS_RT_CPER, kRtScatterPer = AOS_RT_SPER, kRtCountTB = AOS_RT_CTB, kRtScatterTB = AOS_RT_STB;
constexpr int kRtChunkQ = 4096;   // chunk granularity (points): a multiple of both passes' sub-chunks

// tiles whose bins a point's 3 x 3 bins touch: [tx0, tx1] x [ty0, ty1], own tile (bx / TB, by / TB)
__device__ __forceinline__ void rt_tiles(const RorLaunch &L, int bx, int by, int &tx0, int &tx1, int &ty0, int &ty1) {
    tx0 = max(bx - 1, 0) >> L.TBs; tx1 = min(bx + 1, L.nbx - 1) >> L.TBs;   // (bins are >= 0)
    ty0 = max(by - 1, 0) >> L.TBs; ty1 = min(by + 1, L.nby - 1) >> L.TBs;
}

// XCD-aware block order (cdna_hip_programming.md §5.5): consecutive blocks b = j (mod 8) run on XCD j.
__device__ __forceinline__ int rt_xcd_block(int b, int n) {
    const int q = n >> 3, r = n & 7, j = b & 7, k = b >> 3;
    return j * q + min(j, r) + k;
}

template <bool SCATTER, int LAY, int kRtTB, int kRtPer>
__global__ __launch_bounds__(kRtTB) void k_rt_part(RorLaunch L, int *H, const int *tstart, uint64_t chunk,
                                                   float4 *staged, unsigned *own_out, RtClear clr) {
    constexpr int kRtSub = kRtTB * kRtPer;
    extern __shared__ int hist[];        // [ntiles]: counts (count pass) / cursors (scatter pass)
    // chunk w: the chunks of one XCD are contiguous, so the scatter runs of chunks w and w + 1 (adjacent in
    // every tile's range) are written through the same L2 and their shared lines merge there
    const int tid = threadIdx.x, w = rt_xcd_block(blockIdx.x, gridDim.x);
    if (!SCATTER) {   // the stage's zeroed outputs (raster bits, counters, kept counts): no fill launches
        const size_t stride = (size_t)gridDim.x * kRtTB, i0 = (size_t)blockIdx.x * kRtTB + tid;
        for (size_t i = i0; i < clr.nw; i += stride) clr.w[i] = 0ull;
        for (size_t i = i0; i < (size_t)clr.nc; i += stride) clr.c[i] = 0ull;
        for (size_t i = i0; i < (size_t)clr.nk; i += stride) clr.k[i] = 0;
    }
    int *row = H + (size_t)w * L.ntiles;
    for (int t = tid; t < L.ntiles; t += kRtTB) hist[t] = SCATTER ? tstart[t] + row[t] : 0;
    __syncthreads();
    unsigned own = 0;
    const uint64_t begin = (uint64_t)w * chunk, end = min(L.n, begin + chunk);
    const unsigned cnt = begin < end ? (unsigned)(end - begin) : 0u;   // (chunks are < 2^32 points)
    // the chunk's records from a 64-bit base, then 32-bit offsets (LAY 0: the caller's point_step)
    const uint8_t *cbase = L.cloud + begin * (uint64_t)(LAY == 1 ? 16 : LAY == 2 ? 12 : L.step);
    // a record is loaded straight into the registers it is used from (float3 for the packed 12-B cloud: a
    // float4 with a validity word made the compiler wait on each load to move x, y, z into place)
    using Rec = typename std::conditional<LAY == 1, float4, float3>::type;
    auto ld = [&](unsigned i, Rec &o) {
        const uint8_t *rec = cbase + i * (unsigned)(LAY == 1 ? 16 : LAY == 2 ? 12 : L.step);
        if (LAY != 0 && (AOS_RT_NT & (SCATTER ? 2 : 1))) {
            typedef float vrec __attribute__((ext_vector_type(LAY == 1 ? 4 : 3)));
            const vrec v = __builtin_nontemporal_load(reinterpret_cast<const vrec *>(rec));
            o.x = v.x; o.y = v.y; o.z = v.z;
        } else if (LAY == 0) {
            o.x = *reinterpret_cast<const float *>(rec + L.ox);
            o.y = *reinterpret_cast<const float *>(rec + L.oy);
            o.z = *reinterpret_cast<const float *>(rec + L.oz);
        } else {
            o = *reinterpret_cast<const Rec *>(rec);
        }
    };
    // software pipelined over two register buffers that alternate (no register copies between them, so
    // the compiler does not wait on the next sub-chunk's loads to move them: round 3 found the single
    // prefetch buffer + copy waiting on 6 of its 8 loads before the current points were walked)
    // (branch-free: an index past the chunk re-reads the chunk's last point; the walk skips it)
    auto issue = [&](Rec (&buf)[kRtPer], unsigned base) {
#pragma unroll
        for (int j = 0; j < kRtPer; ++j) {
            const unsigned i = base + (unsigned)(j * kRtTB + tid);
            ld(i < cnt ? i : cnt - 1, buf[j]);
        }
    };
    auto walk = [&](const Rec (&pt)[kRtPer], unsigned base) {
#pragma unroll
        for (int j = 0; j < kRtPer; ++j) {
            const float x = pt[j].x, y = pt[j].y, z = pt[j].z;
            if (!SCATTER) {
                // count: branch-free except for the halo tiles. The first tile of the point's (1 or 2) x (1 or
                // 2) tiles gets + ok (+ 0 from a point that is past the chunk or not binned: its bins are the
                // box corner's); round 3's nested tile loops spent ~18 us of the pass on branches
                const bool ok = base + (unsigned)(j * kRtTB + tid) < cnt && rt_binned(L, x, y, z);
                own += ok ? 1u : 0u;
                int bx, by, tx0, tx1, ty0, ty1;
                rt_bin(L, ok ? x : L.bminx, ok ? y : L.bminy, bx, by);
                rt_tiles(L, bx, by, tx0, tx1, ty0, ty1);
                const int t00 = ty0 * L.ntx + tx0;
                const bool hx = tx1 > tx0, hy = ty1 > ty0;
                atomicAdd(&hist[t00], ok ? 1 : 0);
                if (ok && (hx || hy)) {
                    if (hx) atomicAdd(&hist[t00 + 1], 1);
                    if (hy) atomicAdd(&hist[t00 + L.ntx], 1);
                    if (hx && hy) atomicAdd(&hist[t00 + L.ntx + 1], 1);
                }
                continue;
            }
            if (base + (unsigned)(j * kRtTB + tid) >= cnt || !rt_binned(L, x, y, z)) continue;
            int bx, by, tx0, tx1, ty0, ty1;
            rt_bin(L, x, y, bx, by);
            rt_tiles(L, bx, by, tx0, tx1, ty0, ty1);
            const int otile = (by >> L.TBs) * L.ntx + (bx >> L.TBs);
            const int cls = rt_candidate(L, x, y, z) ? 1 : 0;
            for (int ty = ty0; ty <= ty1; ++ty)
                for (int tx = tx0; tx <= tx1; ++tx) {
                    const int t = ty * L.ntx + tx;
                    const int w = t == otile ? cls : 0;   // a halo copy is never tested there
                    const int pos = atomicAdd(&hist[t], 1);
                    if (pos < L.staged_cap) {                   // else: overflow, the frame is redone
                        const float4 v = make_float4(x, y, z, __int_as_float(w));
                        if (AOS_RT_NT & 4) {
                            typedef float v4f __attribute__((ext_vector_type(4)));
                            __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f *>(staged + pos));
                        } else {
                            staged[pos] = v;
                        }
                    } else {
                        *L.overflow = 1;
                    }
                }
        }
    };
    Rec bufA[kRtPer], bufB[kRtPer];
    if (cnt) issue(bufA, 0);
    for (unsigned base = 0; base < cnt; base += 2 * kRtSub) {
        if (base + kRtSub < cnt) issue(bufB, base + kRtSub);
        walk(bufA, base);
        if (base + kRtSub >= cnt) break;
        if (base + 2 * kRtSub < cnt) issue(bufA, base + 2 * kRtSub);
        walk(bufB, base + kRtSub);
    }
    if (!SCATTER) {
        __syncthreads();
        for (int t = tid; t < L.ntiles; t += kRtTB) row[t] = hist[t];
        // the workgroup's binned points: one plain store (k_rt_colscan sums them; round 3's per-wave global
        // atomic on one counter cost the pass ~17 us, tools/rorbench)
        own = (unsigned)wave_reduce((int)own, 0, WAdd());
        __shared__ unsigned own_w[kRtTB / 64];
        if ((tid & 63) == 0) own_w[tid >> 6] = own;
        __syncthreads();
        if (tid == 0) {
            unsigned t = 0;
            for (int k = 0; k < kRtTB / 64; ++k) t += own_w[k];
            own_out[w] = t;
        }
    }
}

// H rows -> per-tile exclusive prefixes over the workgroups (in place), the tile starts (exclusive sum of the
// tile totals, ts[ntiles] = staged total) and the binned count, in ONE launch (round 3 took four: group sums,
// group prefixes, row rewrite, tile-start scan). Block (g, b) holds rows [g kColRows, (g + 1) kColRows) of
// tiles [b kColTB, (b + 1) kColTB) in registers (thread = tile: every access is a row run), publishes its
// per-tile sums as look-back words, walks back over the row groups above it until a prefix word, rewrites its
// rows as running prefixes; the last row group's blocks then hold the tile totals and chain the tile-start
// scan over b. Blocks take ids in launch order, row-group major, so a block only waits for blocks of smaller
// ids (started before it): no deadlock whatever the dispatch order. Words carry the launch's epoch (no init).
constexpr int kColRows = AOS_RT_COLROWS, kColTB = 256;
struct ColScan {
    int *H;                  // G rows of ntiles counts -> exclusive prefixes over the rows
    int *ts;                 // [ntiles + 1] tile starts
    const unsigned *own;     // [G] binned points per count workgroup
    unsigned long long *n_own;   // [0] binned points, [2] the largest tile's record count (atomicMax)
    int ntiles, G, ng, ntb;
    LookBack L;              // part: ng x ntiles column words, then ntb tile-chain words; err bit 4 on a stuck wait
};
__global__ __launch_bounds__(kColTB) void k_rt_colscan(ColScan C) {
    __shared__ int sh_vid, wsum[kColTB / 64], sh_tot, sh_pre;
    __shared__ unsigned long long sh_own[kColTB / 64];
    const int tid = threadIdx.x;
    if (tid == 0) {
        const unsigned v = atomicAdd(C.L.ticket, 1u);
        if (v == gridDim.x - 1) __hip_atomic_store(C.L.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= gridDim.x) atomicOr(C.L.err, 4);
        sh_vid = (int)(v % gridDim.x);
    }
    __syncthreads();
    const int vid = sh_vid, g = vid / C.ntb, b = vid - g * C.ntb;
    const int t = b * kColTB + tid, r0 = g * kColRows, nr = min(C.G - r0, kColRows);
    const bool live = t < C.ntiles;
    const unsigned long long tagA = (unsigned long long)((C.L.epoch << 2) | 1u) << 32;
    const unsigned long long tagP = (unsigned long long)((C.L.epoch << 2) | 2u) << 32;
    int v[kColRows], run = 0;
    if (live) {
        int agg = 0;
#pragma unroll
        for (int r = 0; r < kColRows; ++r) {
            v[r] = r < nr ? C.H[(size_t)(r0 + r) * C.ntiles + t] : 0;
            agg += v[r];
        }
        unsigned long long *w = C.L.part + (size_t)g * C.ntiles + t;
        if (g > 0) {
            st_u64(w, tagA | (unsigned)agg);
            unsigned spins = 0;
            for (int gp = g - 1; gp >= 0; --gp) {
                unsigned long long x;
                unsigned flag;
                for (;;) {
                    x = ld_u64(C.L.part + (size_t)gp * C.ntiles + t);
                    const unsigned tag = (unsigned)(x >> 32);
                    flag = (tag >> 2) == C.L.epoch ? (tag & 3u) : 0u;
                    if (flag) break;
                    if (++spins > kSpinCap) { atomicOr(C.L.err, 4); flag = 2; x = 0; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                run += (int)(unsigned)x;
                if (flag == 2) break;
            }
        }
        st_u64(w, tagP | (unsigned)(run + agg));
#pragma unroll
        for (int r = 0; r < kColRows; ++r)
            if (r < nr) {
                C.H[(size_t)(r0 + r) * C.ntiles + t] = run;
                run += v[r];
            }
    }
    if (vid == 0) {   // the binned count: the count workgroups' own sums (no global atomic in the count pass)
        unsigned long long o = 0;
        for (int k = tid; k < C.G; k += kColTB) o += C.own[k];
        o = (unsigned long long)wave_reduce((long long)o, 0ll, WAdd());
        if ((tid & 63) == 0) sh_own[tid >> 6] = o;
        __syncthreads();
        if (tid == 0) {
            unsigned long long tot = 0;
            for (int k = 0; k < kColTB / 64; ++k) tot += sh_own[k];
            *C.n_own = tot;
        }
    }
    if (g != C.ng - 1) return;   // (uniform per block)
    // tile starts: run is now tile t's total
    const int local = block_excl_scan<kColTB>(live ? run : 0, wsum, &sh_tot);
    {   // the largest tile (a frame that cannot be redone skips the big-tile kernels when it fits the LDS cap)
        int mx = live ? run : 0;
        mx = wave_reduce(mx, 0, WMax());
        if ((tid & 63) == 0 && mx > 0) atomicMax(C.n_own + 2, (unsigned long long)mx);
    }
    if (tid < 64) {
        LookBack T = C.L;
        T.part += (size_t)C.ng * C.ntiles;
        const unsigned pre = lb_exclusive(T, b, (unsigned)sh_tot, 4);
        if (tid == 0) sh_pre = (int)pre;
    }
    __syncthreads();
    if (live) C.ts[t] = sh_pre + local;
    if (b == C.ntb - 1 && tid == 0) C.ts[C.ntiles] = sh_pre + sh_tot;
}

// ---------------------------------------------------------------------------------------------
// Pass 4: per tile, counting sort by bin in LDS, neighbour counts, raster bitmap.
#ifndef AOS_RT_THREADS
#define AOS_RT_THREADS 512
#endif
constexpr int kRorThreads = AOS_RT_THREADS, kRorCap = 2048, kRorPer = kRorCap / kRorThreads;
#ifndef AOS_RT_VARIANT   // timing experiments only (tools/rorbench): 1 = no neighbour scan, 2 = no raster,
                         // 3 = load + bin histogram only, 4 = load + counting sort only
#define AOS_RT_VARIANT 0
#endif


// record i of a neighbour list ending at k1 (a batch of 4 may run past it: those records are not counted).
// A global list (big tiles) is clamped to stay inside its allocation; a fitting tile's LDS list has 3 records
// of padding, so the batch reads at one base address with immediate offsets.
__device__ __forceinline__ float4 rt_at(const float4 *P, int i, int k1) { return P[min(i, k1 - 1)]; }
struct LdsList { const float4 *p; };
__device__ __forceinline__ float4 rt_at(LdsList P, int i, int) { return P.p[i]; }

template <class Pts>
__device__ __forceinline__ int rt_scan(const RorLaunch &L, float4 p, Pts pts, int k0, int k1, int cnt) {
    for (int k = k0; k < k1 && cnt < L.need; k += 4) {
        float4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = rt_at(pts, k + j, k1);
#pragma unroll
        for (int j = 0; j < 4; ++j) cnt += ((k + j < k1) & rt_in(L, p, q[j])) ? 1 : 0;   // (no short circuit: no branch)
    }
    return cnt;
}

// A thread examines at most kRtBudget points for its candidate; a candidate still undecided (a dense
// neighbourhood in which it finds too few neighbours: an outlier, up to ~10^4 points in a streaming
// map's big tile) goes to the workgroup's queue and is counted by a whole wave, 64 points per step.
// One lane walking such a neighbourhood alone bounded the kernel (~1 ms per scan at C4).
// Fitting tiles (round 3): the kernel was VALU-issue-bound on divergence (C2: 1.1e8 VALU
// wave-instructions for 5.6 M points; ~3 % of candidates are not kept and walk their whole 3 x 3
// neighbourhood, so nearly every wave waited on one or two long walks). The first pass now gives each
// lane 12 points; the queued candidates (~10 %) are walked one lane each with a budget of 96, packed
// together, and only the few left after that go to the waves (k_rt_ror 171 -> 150 us at C2,
// profiles/r03x_rorbench.log; 4 / 8 / 16 / 32 lanes per candidate were 238-411 us, r03t).
template <class Pts>
__device__ __forceinline__ int rt_scan_b(const RorLaunch &L, float4 p, Pts pts, int k0, int k1, int cnt, int &budget) {
    int k = k0;
    for (; k < k1 && cnt < L.need && budget > 0; k += 4, budget -= 4) {
        float4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = rt_at(pts, k + j, k1);
#pragma unroll
        for (int j = 0; j < 4; ++j) cnt += ((k + j < k1) & rt_in(L, p, q[j])) ? 1 : 0;   // (no short circuit: no branch)
    }
    if (k < k1 && cnt < L.need) budget = -1;   // cut short: undecided
    return cnt;
}
template <class Pts>
__device__ __forceinline__ int rt_wave_scan(const RorLaunch &L, float4 p, Pts pts, int k0, int k1, int cnt, int lane) {
    for (int base = k0; base < k1 && cnt < L.need; base += 64) {   // (cnt is wave-uniform)
        const int j = base + lane;
        const bool hit = (j < k1) & rt_in(L, p, rt_at(pts, min(j, k1 - 1), k1));
        cnt += (int)__popcll(__ballot(hit));
    }
    return cnt;
}

#ifndef AOS_RT_BUDGET_LDS
#define AOS_RT_BUDGET_LDS 12
#endif
#ifndef AOS_RT_BUDGET2
#define AOS_RT_BUDGET2 96
#endif
constexpr int kRtBudgetBig = 64, kRtBudgetLds = AOS_RT_BUDGET_LDS, kRtQCap = 512, kRtBudget2 = AOS_RT_BUDGET2, kRtQ2Cap = 128;

// LDS of k_rt_ror: kRorCap staged points (32 KB), the bin offsets of the largest tile (TB = 32 bins
// + ring: 34^2), the tile's raster window (kRtWinWords 64-bit words: 70 rows x 3 words at 0.1 m cells)
// and the two queues (16-bit indices): 40.8 KB, 4 workgroups per CU
constexpr int kRtMaxLocalBins = 34 * 34, kRtWinWords = 256;
// staged record w (int bits): bits 0-1 the class (0 a neighbour only, 1 an own clip candidate, 2 a
// candidate a streaming map already found kept); streaming store only: kWOld = written back by an
// earlier frame, kWCounted = a candidate below need whose count over the store is in bits kWCntShift+
constexpr int kWClass = 3, kWCounted = 4, kWOld = 8, kWCntShift = 8;

// Tiles with more than kRorCap points (a streaming map's scan footprint: up to ~10^6 points in one
// tile after a few dozen scans) do not fit LDS, and one workgroup per such tile leaves most CUs idle
// while a few walk a huge list. They are listed (k_rt_biglist) and cut into chunks of kBigChunk points
// (k_rt_bigchunks), one workgroup per chunk in grids of kBigGrid that loop over the chunks:
//   k_rt_bighist     per-chunk LDS bin histogram, added into the tile's global bin totals
//   k_rt_bigscan     per tile: bin starts (bigbins row) and bin cursors (= starts)
//   k_rt_bigscatter  per chunk: one global atomic per (chunk, non-empty bin) reserves its runs, then the
//                    chunk's points go bin-sorted into the tile's range of the scratch array
//   k_rt_ror_big     per chunk: the neighbour counts of the chunk's points, searched in the tile's
//                    bin-sorted scratch range (through the kernel boundary; see k_rt_ror for the rules)
// The order inside a bin depends on the atomics' order; the keep decision and the raster do not.
// A big tile's bins are split in two: first the points the store already held (kWOld), then this
// frame's new points. A candidate that stayed below need in an earlier frame carries its neighbour count
// over the store's points (kWCounted, count in bits kWCntShift+); points are only ever added, so its new
// count is that count plus its neighbours among the new points, found in the new halves of its 3 x 3
// bins alone. (Without it, every dirty big tile re-scanned the whole 3 x 3 neighbourhood, thousands of
// points, for each of its lasting outliers on every scan.)
// Work is split in chunks of kBigChunk points over all big tiles (choff: the chunks' prefix over the
// list), so a grid of kBigGrid workgroups stays balanced however unequal the tiles are (round 2's 16
// chunks per tile left a 10^6-point tile's 16 workgroups walking 60 k points each while the rest idled).
constexpr int kBigY = 32, kBigTB = 512, kBigBins = 2 * kRtMaxLocalBins, kBigChunk = 4096, kBigGrid = 1024;
// rt_bigbins_ints(L) ints: starts and cursors 2 x ntiles x (2 nlb + 1), list 1 + ntiles, choff ntiles + 1
struct BigBufs { int *starts, *cur, *list, *choff; };
static BigBufs big_bufs(const RorLaunch &L, int *B) {
    const size_t row = 2 * (size_t)(L.TB + 2) * (L.TB + 2) + 1, nt = (size_t)L.ntiles;
    return BigBufs{B, B + nt * row, B + 2 * nt * row, B + 2 * nt * row + 1 + nt};
}

__device__ __forceinline__ int rt_lbin(const RorLaunch &L, float4 q, int bx0, int by0, int LB) {
    int bx, by;
    rt_bin(L, q.x, q.y, bx, by);
    return (by - by0) * LB + (bx - bx0);   // in [0, LB^2): a copy lies in the tile's 3 x 3 reach
}
// big tiles: local bin b -> sub-bins 2 b (store points) and 2 b + 1 (new points)
__device__ __forceinline__ int rt_sbin(const RorLaunch &L, float4 q, int bx0, int by0, int LB) {
    return 2 * rt_lbin(L, q, bx0, by0, LB) + ((__float_as_int(q.w) & kWOld) ? 0 : 1);
}

// list[0] = number of big tiles, list[1..]: the tiles; their cursor rows zeroed, kept_tile reset. One
// thread per tile (a frame without big tiles pays one short launch; a big tile's thread zeroes its row)
__global__ __launch_bounds__(256) void k_rt_biglist(RorLaunch L, const int *tstart, BigBufs B, int *kept_tile,
                                                    const int *dirty) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= L.ntiles) return;
    const int a = tstart[t], n = tstart[t + 1] - a;
    if (!((!dirty || dirty[t + 1] != dirty[t]) && n > kRorCap && a + n <= L.staged_cap)) return;
    B.list[1 + atomicAdd(&B.list[0], 1)] = t;
    if (kept_tile) kept_tile[t] = 0;
    const int nlb1 = 2 * (L.TB + 2) * (L.TB + 2) + 1;
    int *row = B.cur + (size_t)t * nlb1;   // (rows are not 16 B aligned: plain stores)
    for (int i = 0; i < nlb1; ++i) row[i] = 0;
}

// choff[i] = chunks of the big tiles before list entry i; choff[nbig] = all chunks
__global__ __launch_bounds__(1024) void k_rt_bigchunks(const int *tstart, BigBufs B) {
    __shared__ int wsum[1024 / 64];
    const int nbig = B.list[0];
    int base = 0;
    for (int i0 = 0; i0 < nbig; i0 += 1024) {
        const int i = i0 + threadIdx.x;
        int c = 0;
        if (i < nbig) {
            const int t = B.list[1 + i];
            c = (tstart[t + 1] - tstart[t] + kBigChunk - 1) / kBigChunk;
        }
        int total;
        const int before = block_excl_scan<1024>(c, wsum, &total);   // (ends with a barrier)
        if (i < nbig) B.choff[i] = base + before;
        base += total;
    }
    if (threadIdx.x == 0) B.choff[nbig] = base;
}
__device__ __forceinline__ int big_nchunks(const BigBufs &B) { return B.choff[B.list[0]]; }
// chunk c of all big tiles -> its tile t (first record a) and the range [k0, k1) of the tile's list
__device__ __forceinline__ void big_chunk(const int *tstart, const BigBufs &B, int c, int &t, int &a, int &k0, int &k1) {
    int lo = 0, hi = B.list[0] - 1;   // the last list entry i with choff[i] <= c
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (B.choff[mid] <= c) lo = mid;
        else hi = mid - 1;
    }
    t = B.list[1 + lo];
    a = tstart[t];
    const int n = tstart[t + 1] - a;
    k0 = (c - B.choff[lo]) * kBigChunk;
    k1 = min(n, k0 + kBigChunk);
}

__global__ __launch_bounds__(kBigTB) void k_rt_bighist(RorLaunch L, const int *tstart, const float4 *staged, BigBufs B) {
    __shared__ int h[kBigBins + 1];
    const int nch = big_nchunks(B), LB = L.TB + 2, nlb = 2 * LB * LB;
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        int t, a, k0, k1;
        big_chunk(tstart, B, c, t, a, k0, k1);
        const int tx = t % L.ntx, ty = t / L.ntx;
        for (int b = threadIdx.x; b < nlb; b += kBigTB) h[b] = 0;
        __syncthreads();
        for (int k = k0 + threadIdx.x; k < k1; k += kBigTB)
            atomicAdd(&h[rt_sbin(L, staged[a + k], tx * L.TB - 1, ty * L.TB - 1, LB)], 1);
        __syncthreads();
        int *tot = B.cur + (size_t)t * (nlb + 1);
        for (int b = threadIdx.x; b < nlb; b += kBigTB)
            if (h[b]) atomicAdd(&tot[b], h[b]);
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void k_rt_bigscan(RorLaunch L, const int *tstart, BigBufs B) {
    constexpr int kSeg = (kBigBins + 1023) / 1024;
    __shared__ int wsum[1024 / 64];
    const int nbig = B.list[0], nlb = 2 * (L.TB + 2) * (L.TB + 2);
    for (int i = blockIdx.x; i < nbig; i += gridDim.x) {
        const int t = B.list[1 + i];
        int *tot = B.cur + (size_t)t * (nlb + 1), *st = B.starts + (size_t)t * (nlb + 1);
        int v[kSeg], run = 0;
#pragma unroll
        for (int j = 0; j < kSeg; ++j) {
            const int b = threadIdx.x * kSeg + j;
            v[j] = b < nlb ? tot[b] : 0;
            run += v[j];
        }
        int total;
        int before = block_excl_scan<1024>(run, wsum, &total);
#pragma unroll
        for (int j = 0; j < kSeg; ++j) {
            const int b = threadIdx.x * kSeg + j;
            if (b < nlb) { st[b] = before; tot[b] = before; }
            before += v[j];
        }
        if (threadIdx.x == 1023) st[nlb] = before;   // = the tile's point count
        __syncthreads();
    }
}

__global__ __launch_bounds__(kBigTB) void k_rt_bigscatter(RorLaunch L, const int *tstart, const float4 *staged,
                                                          float4 *scratch, BigBufs B) {
    __shared__ int h[kBigBins + 1];
    const int nch = big_nchunks(B), LB = L.TB + 2, nlb = 2 * LB * LB;
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        int t, a, k0, k1;
        big_chunk(tstart, B, c, t, a, k0, k1);
        const int tx = t % L.ntx, ty = t / L.ntx;
        const int bx0 = tx * L.TB - 1, by0 = ty * L.TB - 1;
        for (int b = threadIdx.x; b < nlb; b += kBigTB) h[b] = 0;
        __syncthreads();
        for (int k = k0 + threadIdx.x; k < k1; k += kBigTB) atomicAdd(&h[rt_sbin(L, staged[a + k], bx0, by0, LB)], 1);
        __syncthreads();
        int *cur = B.cur + (size_t)t * (nlb + 1);
        for (int b = threadIdx.x; b < nlb; b += kBigTB)
            if (h[b]) h[b] = atomicAdd(&cur[b], h[b]);   // this chunk's run in bin b
        __syncthreads();
        for (int k = k0 + threadIdx.x; k < k1; k += kBigTB) {
            const float4 v = staged[a + k];
            scratch[a + atomicAdd(&h[rt_sbin(L, v, bx0, by0, LB)], 1)] = v;
        }
        __syncthreads();
    }
}

// kept_tile (optional): the tile's count of kept owned candidates; dirty (optional): only tiles with
// dirty[t + 1] > dirty[t] are (re)counted — the streaming map's tiles that received scan points.
// BIG = false: one workgroup per tile that fits LDS (the others are left to BIG); BIG = true: workgroups
// loop over the big tiles' chunks, points searched in the scratch range.
template <bool BIG>
__global__ __launch_bounds__(kRorThreads) void k_rt_ror(RorLaunch L, const int *tstart, float4 *staged,
                                                        const float4 *scratch, uint64_t *rbits,
                                                        unsigned long long *counters, int *kept_tile,
                                                        const int *dirty, BigBufs B) {
    __shared__ float4 pts[BIG ? 1 : kRorCap + 3];   // (+ 3: rt_at's padding)
    const LdsList LP{pts};
    auto lp_get = [&](int k) { return pts[k]; };
    auto lp_put = [&](int k, float4 v) { pts[k] = v; };
    auto lp_setw = [&](int k, float w) { pts[k].w = w; };
    __shared__ int bstart[(BIG ? kBigBins : kRtMaxLocalBins) + 1];
    __shared__ unsigned long long win[kRtWinWords];
    __shared__ unsigned kept_wg;
    // candidates left to the queues: tile-local indices (< kRorCap, 16 bits) in a fitting tile
    using QIdx = typename std::conditional<BIG, int, unsigned short>::type;
    __shared__ int q_n, q2_n;
    __shared__ QIdx q_k[kRtQCap], q2_k[BIG ? 1 : kRtQ2Cap];
    const int tid = threadIdx.x;
    const int nit = BIG ? big_nchunks(B) : 1;
    for (int it = BIG ? blockIdx.x : 0; it < nit; it += BIG ? gridDim.x : 1) {
    int t, a, k0, k1;                               // the tile, its first record, the range of its runs
    if (BIG) {
        big_chunk(tstart, B, it, t, a, k0, k1);
    } else {
        t = rt_xcd_block(blockIdx.x, gridDim.x);
        a = tstart[t];
        k0 = 0;
        k1 = tstart[t + 1] - a;
    }
    const int n = tstart[t + 1] - a;
    const int tx = t % L.ntx, ty = t / L.ntx;
    if (!BIG && dirty && dirty[t + 1] == dirty[t]) return;
    if (!BIG) {
        if (n > kRorCap && a + n <= L.staged_cap) {   // a big tile: k_rt_ror<true>
            // (not launched this frame: the frame is redone with the big-tile kernels, seedgen.hip)
            if (!L.big_ok && tid == 0) atomicOr(L.overflow, 2);
            return;
        }
        if (n == 0 || a + n > L.staged_cap) {               // (an overflowed scatter: the frame is redone)
            if (kept_tile && tid == 0) kept_tile[t] = 0;
            return;
        }
    }
    if (tid == 0) { kept_wg = 0; q_n = 0; q2_n = 0; }
    const int LB = L.TB + 2;                        // local bins: the tile's bins and a ring of halo bins
    const int bx0 = tx * L.TB - 1, by0 = ty * L.TB - 1;
    const int nlb = LB * LB;
    // raster window: rows [cy0, cy0 + L.win_rows), words [cw0, cw0 + L.win_w) of the raster window bits
    const float wx_lo = L.bminx + (float)(tx * L.TB) / L.inv_cs, wy_lo = L.bminy + (float)(ty * L.TB) / L.inv_cs;
    const int cy0 = (int)floor(((double)wy_lo - L.origin_y) / (double)L.res) - 2;
    const int cx0 = (int)floor(((double)wx_lo - L.origin_x) / (double)L.res) - 2;
    const int cw0 = (int)floor((double)(cx0 - L.wx0) / 64.0);
    const bool use_win = L.win_rows > 0;
    if (use_win)
        for (int i = tid; i < L.win_rows * L.win_w; i += kRorThreads) win[i] = 0ull;
    if (BIG) {   // sub-bin offsets from k_rt_bigscan (through the kernel boundary)
        for (int i = tid; i <= 2 * nlb; i += kRorThreads) bstart[i] = B.starts[(size_t)t * (2 * nlb + 1) + i];
    } else {
        for (int i = tid; i <= nlb; i += kRorThreads) bstart[i] = 0;
    }
    __syncthreads();
    // counting sort of a fitting tile: histogram (ranks kept in registers), scan, place
    float4 q[BIG ? 1 : kRorPer];
    int rk[BIG ? 1 : kRorPer], lb[BIG ? 1 : kRorPer];
    if (!BIG) {
        // the tile's records: all loads in flight before the first use (an index past the tile re-reads its
        // last record, n >= 1 here; rk = -1 marks it)
#pragma unroll
        for (int j = 0; j < kRorPer; ++j) q[j] = staged[a + min(tid + j * kRorThreads, n - 1)];
#pragma unroll
        for (int j = 0; j < kRorPer; ++j) {
            const int k = tid + j * kRorThreads;
            lb[j] = rt_lbin(L, q[j], bx0, by0, LB);
            rk[j] = k < n ? atomicAdd(&bstart[lb[j] + 1], 1) : -1;
        }
        __syncthreads();
        if (AOS_RT_VARIANT == 3) return;   // (timing: load + histogram only)
        // exclusive bin offsets: bstart[b] = points in bins < b. Thread t sums a run of kSeg bins,
        // one block scan over the run totals, then each run is written back.
        constexpr int kSeg = (kRtMaxLocalBins + kRorThreads - 1) / kRorThreads;
        // (wave shuffles + one LDS slot per wave: 32 B of LDS where hipcub's BlockScan takes ~2 KB, which
        // kept the workgroup above the 40 KB that lets 4 of them share a CU)
        __shared__ int wsum[kRorThreads / 64];
        int v[kSeg], run = 0;
#pragma unroll
        for (int j = 0; j < kSeg; ++j) {
            const int b = tid * kSeg + j + 1;
            v[j] = b <= nlb ? bstart[b] : 0;
            run += v[j];
        }
        const int incl = wave_scan_incl(run, 0, WAdd());
        if ((tid & 63) == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        int before = incl - run;
        for (int w = 0; w < (tid >> 6); ++w) before += wsum[w];
#pragma unroll
        for (int j = 0; j < kSeg; ++j) {
            const int b = tid * kSeg + j + 1;
            before += v[j];
            if (b <= nlb) bstart[b] = before;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kRorPer; ++j)
            if (rk[j] >= 0) lp_put(bstart[lb[j]] + rk[j], q[j]);
        __syncthreads();
        if (AOS_RT_VARIANT == 4) return;   // (timing: load + counting sort only)
    }
    float4 *P = const_cast<float4 *>(scratch) + a;
    unsigned kept_n = 0;
    auto local_of = [&](float4 p, int &lx, int &ly) {   // a record's bin in the tile's local grid
        int bx, by;
        rt_bin(L, p.x, p.y, bx, by);
        lx = bx - bx0; ly = by - by0;
    };
    // w: 0 a neighbour only, 1 a candidate, 2 a candidate a streaming map already found kept (the keep
    // decision is monotone as points are added: it stays kept, its cell is already in the raster)
    const bool store = kept_tile != nullptr;
    const double res_d = (double)L.res, inv_res = 1.0 / res_d;
    auto prev_kept = [&](float4 p) {   // kept in an earlier frame: counted, not re-tested
        const int gx = rt_cell((double)p.x - L.origin_x, res_d, inv_res);
        const int gy = rt_cell((double)p.y - L.origin_y, res_d, inv_res);
        const int cx = min(max(gx, 0), L.W - 1), cy = min(max(gy, 0), L.H - 1);
        if (cx >= L.rx0 && cx < L.rx1 && cy >= L.ry0 && cy < L.ry1) ++kept_n;
    };
    auto on_kept = [&](float4 p, int k) {
        if (store) {   // remembered in the tile store (written back below)
            if (BIG) P[k].w = __int_as_float(2);   // (neighbour scans of other threads read only x, y, z)
            else lp_setw(k, __int_as_float(2));
        }
        // kept: counted iff its clamped cell is owned, rastered iff inside the grid (seed_gen:606-619)
        const int gx = rt_cell((double)p.x - L.origin_x, res_d, inv_res);
        const int gy = rt_cell((double)p.y - L.origin_y, res_d, inv_res);
        const int cx = min(max(gx, 0), L.W - 1), cy = min(max(gy, 0), L.H - 1);
        if (cx < L.rx0 || cx >= L.rx1 || cy < L.ry0 || cy >= L.ry1) return;
        ++kept_n;
        if (AOS_RT_VARIANT == 2 || gx < 0 || gx >= L.W || gy < 0 || gy >= L.H) return;
        const int bxw = gx - L.wx0, r = gy - L.wy0;
        const int wr = r - (cy0 - L.wy0), ww = (bxw >> 6) - cw0;
        const unsigned long long bit = 1ull << (bxw & 63);
        if (use_win && wr >= 0 && wr < L.win_rows && ww >= 0 && ww < L.win_w)
            atomicOr(&win[wr * L.win_w + ww], bit);
        else
            atomicOr(reinterpret_cast<unsigned long long *>(&rbits[(size_t)r * L.WWr + (bxw >> 6)]), bit);
    };
    // the neighbour ranges of a candidate, in scan order: a big tile's counted candidate -> the new halves
    // of its 3 x 3 bins (9 ranges); else its 3 bin rows, own row first
    auto range = [&](bool counted, int lx, int ly, int i, int &r0, int &r1) {
        if (counted) {
            const int b = (ly - 1 + i / 3) * LB + lx - 1 + i % 3;
            r0 = bstart[2 * b + 1]; r1 = bstart[2 * b + 2];
        } else {
            const int rb = (ly + (i == 0 ? 0 : (i == 1 ? -1 : 1))) * LB + lx - 1;
            if (BIG) { r0 = bstart[2 * rb]; r1 = bstart[2 * rb + 6]; }
            else { r0 = bstart[rb]; r1 = bstart[rb + 3]; }
        }
    };
    auto decide = [&](float4 p, int k, int cnt) {
        if (cnt >= L.need) on_kept(p, k);
        else if (store) {                       // below need: remember the full count
            const float cw = __int_as_float(1 | kWCounted | (cnt << kWCntShift));
            if (BIG) P[k].w = cw;
            else lp_setw(k, cw);
        }
    };
    for (int k = k0 + tid; k < k1; k += kRorThreads) {
        const float4 p = BIG ? P[k] : lp_get(k);
        const int w = __float_as_int(p.w), cls = w & kWClass;
        if (!cls) continue;                     // neighbour only
        if (cls == 2) { prev_kept(p); continue; }
        int lx, ly;
        local_of(p, lx, ly);
        const bool counted = BIG && (w & kWCounted);   // the store's points are counted: the new ones only
        const int nr = counted ? 9 : 3, cnt0 = AOS_RT_VARIANT == 1 ? L.need : (counted ? w >> kWCntShift : 0);
        int cnt = cnt0, budget = BIG ? kRtBudgetBig : kRtBudgetLds;
        for (int i = 0; i < nr && cnt < L.need && budget >= 0; ++i) {
            int r0, r1;
            range(counted, lx, ly, i, r0, r1);
            cnt = BIG ? rt_scan_b(L, p, P, r0, r1, cnt, budget) : rt_scan_b(L, p, LP, r0, r1, cnt, budget);
        }
        if (cnt < L.need && budget < 0) {        // undecided within the budget
            const int slot = atomicAdd(&q_n, 1);
            if (slot < kRtQCap) { q_k[slot] = (QIdx)k; continue; }
            cnt = cnt0;                          // (queue full: this thread counts it alone)
            for (int i = 0; i < nr && cnt < L.need; ++i) {
                int r0, r1;
                range(counted, lx, ly, i, r0, r1);
                cnt = BIG ? rt_scan(L, p, P, r0, r1, cnt) : rt_scan(L, p, LP, r0, r1, cnt);
            }
        }
        decide(p, k, cnt);
    }
    __syncthreads();
    {   // the queued candidates
        const int nq = min(q_n, kRtQCap), lane = tid & 63;
        if (!BIG) {
            // fitting tiles: the over-budget candidates one lane each (restarted, budget kRtBudget2), so the
            // long walks run packed together; the few still undecided after that, one wave each
            for (int i = tid; i < nq; i += kRorThreads) {
                const int k = q_k[i];
                const float4 p = lp_get(k);
                int lx, ly;
                local_of(p, lx, ly);
                int cnt = 0, budget = kRtBudget2;
                for (int r = 0; r < 3 && cnt < L.need && budget >= 0; ++r) {
                    int r0, r1;
                    range(false, lx, ly, r, r0, r1);
                    cnt = rt_scan_b(L, p, LP, r0, r1, cnt, budget);
                }
                if (cnt < L.need && budget < 0) {
                    const int slot = atomicAdd(&q2_n, 1);
                    if (slot < kRtQ2Cap) { q2_k[slot] = (QIdx)k; continue; }
                    cnt = 0;
                    for (int r = 0; r < 3 && cnt < L.need; ++r) {
                        int r0, r1;
                        range(false, lx, ly, r, r0, r1);
                        cnt = rt_scan(L, p, LP, r0, r1, cnt);
                    }
                }
                decide(p, k, cnt);
            }
            __syncthreads();
            const int nq2 = min(q2_n, kRtQ2Cap);
            for (int i = tid >> 6; i < nq2; i += kRorThreads / 64) {
                const int k = q2_k[i];
                const float4 p = lp_get(k);
                int lx, ly;
                local_of(p, lx, ly);
                int cnt = 0;
                for (int r = 0; r < 3 && cnt < L.need; ++r) {
                    int r0, r1;
                    range(false, lx, ly, r, r0, r1);
                    cnt = rt_wave_scan(L, p, LP, r0, r1, cnt, lane);
                }
                if (lane == 0) decide(p, k, cnt);
            }
        } else   // big tiles: one wave each
        for (int i = tid >> 6; i < nq; i += kRorThreads / 64) {
            const int k = q_k[i];
            const float4 p = BIG ? P[k] : lp_get(k);
            const int w = __float_as_int(p.w);
            int lx, ly;
            local_of(p, lx, ly);
            const bool counted = BIG && (w & kWCounted);
            int cnt = counted ? w >> kWCntShift : 0;
            for (int r = 0; r < (counted ? 9 : 3) && cnt < L.need; ++r) {
                int r0, r1;
                range(counted, lx, ly, r, r0, r1);
                cnt = BIG ? rt_wave_scan(L, p, P, r0, r1, cnt, lane) : rt_wave_scan(L, p, LP, r0, r1, cnt, lane);
            }
            if (lane == 0) decide(p, k, cnt);
        }
    }
    __syncthreads();
    // the store goes back bin-sorted with its kept marks and counts, every point marked as the store's: a
    // fitting tile rewrites its list, a big tile's chunk its range of the sorted scratch list
    if (store)
        for (int k = k0 + tid; k < k1; k += kRorThreads) {
            float4 v = BIG ? P[k] : lp_get(k);
            v.w = __int_as_float(__float_as_int(v.w) | kWOld);
            staged[a + k] = v;
        }
    __syncthreads();
    if (use_win)
        for (int i = tid; i < L.win_rows * L.win_w; i += kRorThreads) {
            const unsigned long long v = win[i];
            if (!v) continue;
            const int r = cy0 - L.wy0 + i / L.win_w, w = cw0 + i % L.win_w;
            if (r >= 0 && r < L.Hr && w >= 0 && w < L.WWr)
                atomicOr(reinterpret_cast<unsigned long long *>(&rbits[(size_t)r * L.WWr + w]), v);
        }
    kept_n = (unsigned)wave_reduce((int)kept_n, 0, WAdd());
    if ((tid & 63) == 0 && kept_n) {
        atomicAdd(&counters[(blockIdx.x * (kRorThreads / 64) + (tid >> 6)) & (kRorCounters - 1)],
                  (unsigned long long)kept_n);
        if (kept_tile) atomicAdd(&kept_wg, kept_n);
    }
    if (kept_tile) {
        __syncthreads();
        if (tid == 0) {
            if (BIG) atomicAdd(&kept_tile[t], (int)kept_wg);
            else kept_tile[t] = (int)kept_wg;
        }
    }
    __syncthreads();
    }
}

// Streaming map: the map's tile store (old) and the scan's partition (scan) -> the new store; per tile
// the old run, then the scan's run. tstart_new[t] = old[t] + scan[t] for t <= ntiles.
__global__ __launch_bounds__(256) void k_rt_merge(const float4 *old_st, const int *old_ts, const float4 *scan_st,
                                                  const int *scan_ts, float4 *new_st, int *new_ts, int ntiles, int cap,
                                                  int *overflow) {
    const int t = blockIdx.x;
    if (t > ntiles) return;
    const int o0 = old_ts[t], s0 = scan_ts[t], d0 = o0 + s0;
    if (threadIdx.x == 0 && blockIdx.y == 0) new_ts[t] = d0;
    if (t == ntiles) return;
    const int no = old_ts[t + 1] - o0, ns = scan_ts[t + 1] - s0;
    if ((long long)d0 + no + ns > cap) {   // the host's store size was stale: nothing is written past cap
        if (threadIdx.x == 0) *overflow = 1;
        return;
    }
    // blockIdx.y-th of gridDim.y slices of the tile's runs (a big tile's copy spreads over CUs)
    const int stride = 256 * gridDim.y;
    for (int i = blockIdx.y * 256 + threadIdx.x; i < no; i += stride) new_st[d0 + i] = old_st[o0 + i];
    for (int i = blockIdx.y * 256 + threadIdx.x; i < ns; i += stride) new_st[d0 + no + i] = scan_st[s0 + i];
}

// n_clipped of the streaming map = the sum of the tiles' kept counts (into counters[0])
__global__ __launch_bounds__(1024) void k_rt_sum_kept(const int *kept_tile, int ntiles, unsigned long long *counters) {
    __shared__ unsigned long long part[16];
    unsigned long long v = 0;
    for (int t = threadIdx.x; t < ntiles; t += 1024) v += (unsigned)kept_tile[t];
    if (threadIdx.x > 0 && threadIdx.x < kRorCounters) counters[threadIdx.x] = 0;   // (pass 4's partial adds)
    v = (unsigned long long)wave_reduce((long long)v, 0ll, WAdd());
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int i = 0; i < 16; ++i) s += part[i];
        counters[0] = s;
    }
}

// ---------------------------------------------------------------------------------------------
// est_binned: expected binned points (the previous frame's count, or a guess); it only sizes the
// tiles (TB = 32 bins, or 16 where tiles would average more than ~1400 points) — results do not
// depend on it.
void rt_configure(RorLaunch &L, int Hr, int WWr, double est_binned, int force_tb) {
    auto tiles = [&](int tb) {
        if (tb <= 0 || (tb & (tb - 1))) throw std::runtime_error("ROR tile size must be a power of two");
        L.TB = tb;
        L.TBs = __builtin_ctz((unsigned)tb);
        L.ntx = (L.nbx + tb - 1) / tb;
        L.nty = (L.nby + tb - 1) / tb;
        return (long long)L.ntx * L.nty;
    };
    if (force_tb && tiles(force_tb) <= kRtMaxTiles) {
        tiles(force_tb);
    } else {
        const double per32 = est_binned * 1.15 / (double)tiles(32);
        if (!(per32 > 1400.0 && tiles(16) <= kRtMaxTiles)) tiles(32);
    }
    if (tiles(L.TB) > kRtMaxTiles || (L.TB + 2) * (L.TB + 2) > kRtMaxLocalBins)
        throw std::runtime_error("ROR bin grid too large for the tile walk");
    L.ntiles = L.ntx * L.nty;
    L.r2cmp = L.is_dense ? L.r2df : (L.r2f > 0.0f ? std::nextafter(L.r2f, 0.0f) : -1.0f);
    L.Hr = Hr; L.WWr = WWr;
    // raster window of one tile: its cells (TB bins of 1/inv_cs) + 2 cells of slack on each side
    const double span = (double)L.TB / (double)L.inv_cs / (double)L.res;
    const int cells = (int)std::ceil(span) + 6;
    L.win_rows = cells;
    L.win_w = (cells + 63) / 64 + 1;
    if (L.win_rows * L.win_w > kRtWinWords) L.win_rows = 0;   // windows too large: OR straight into HBM
}

int rt_part_blocks(const RorLaunch &L) {
    // one contiguous chunk per workgroup; H has ntiles x G ints
    long long g = AOS_RT_G;
    const long long kRtSub = kRtChunkQ;
    while (g > 64 && (long long)L.ntiles * g > (16ll << 20)) g /= 2;
    return (int)std::max<long long>(1, std::min<long long>(g, ((long long)L.n + kRtSub - 1) / kRtSub));
}
uint64_t rt_chunk(const RorLaunch &L, int G) {
    const uint64_t c = (L.n + G - 1) / G;
    return (c + kRtChunkQ - 1) / kRtChunkQ * kRtChunkQ;
}

template <bool SCATTER, int LAY>
static void rt_part(const RorLaunch &L, int *H, const int *tstart, int G, float4 *staged, unsigned *own_out,
                    hipStream_t s, const RtClear &clr = RtClear{}) {
    constexpr int TB = SCATTER ? kRtScatterTB : kRtCountTB, PER = SCATTER ? kRtScatterPer : kRtCountPer;
    static_assert(kRtChunkQ % (TB * PER) == 0 || (TB * PER) % kRtChunkQ == 0, "chunk granularity");
    const size_t lds = sizeof(int) * (size_t)L.ntiles;
    const uint64_t stride = LAY == 1 ? 16 : LAY == 2 ? 12 : L.step;
    if (rt_chunk(L, G) * stride >= (1ull << 32))   // (k_rt_part addresses a chunk with 32-bit byte offsets)
        throw std::runtime_error("ROR partition: a workgroup's chunk of the cloud exceeds 4 GB");
    if (lds > 64 * 1024)   // the tile histogram exceeds the default dynamic-LDS limit (gfx950: 160 KB)
        AOS_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rt_part<SCATTER, LAY, TB, PER>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_rt_part<SCATTER, LAY, TB, PER><<<G, TB, lds, s>>>(L, H, tstart, rt_chunk(L, G), staged, own_out, clr);
    AOS_HIP(hipGetLastError());
}
static int rt_layout(const RorLaunch &L) {
    if (L.ox == 0 && L.oy == 4 && L.oz == 8) return L.step == 16 ? 1 : (L.step == 12 ? 2 : 0);
    return 0;
}

size_t rt_h_ints(const RorLaunch &L, int G) { return (size_t)L.ntiles * G + G; }
int rt_colscan_words(const RorLaunch &L, int G) {
    return ((G + kColRows - 1) / kColRows) * L.ntiles + (L.ntiles + kColTB - 1) / kColTB;
}

void launch_rt_count(const RorLaunch &L, int *H, int G, int *ts, unsigned long long *n_own, const LookBack &lb,
                     hipStream_t s, const RtClear &clr) {
    if (!L.n || !L.ntiles) throw std::logic_error("launch_rt_count: no points or tiles");   // (the callers check)
    unsigned *own = reinterpret_cast<unsigned *>(H + (size_t)L.ntiles * G);
    switch (rt_layout(L)) {
        case 1: rt_part<false, 1>(L, H, nullptr, G, nullptr, own, s, clr); break;
        case 2: rt_part<false, 2>(L, H, nullptr, G, nullptr, own, s, clr); break;
        default: rt_part<false, 0>(L, H, nullptr, G, nullptr, own, s, clr);
    }
    ColScan C{H, ts, own, n_own, L.ntiles, G, (G + kColRows - 1) / kColRows, (L.ntiles + kColTB - 1) / kColTB, lb};
    k_rt_colscan<<<C.ng * C.ntb, kColTB, 0, s>>>(C);
    AOS_HIP(hipGetLastError());
}

void launch_rt_scatter(const RorLaunch &L, int *H, const int *tstart, int G, float4 *staged, hipStream_t s) {
    if (!L.n) return;
    switch (rt_layout(L)) {
        case 1: rt_part<true, 1>(L, H, tstart, G, staged, nullptr, s); break;
        case 2: rt_part<true, 2>(L, H, tstart, G, staged, nullptr, s); break;
        default: rt_part<true, 0>(L, H, tstart, G, staged, nullptr, s);
    }
}

int rt_lds_tile_cap() { return kRorCap; }

size_t rt_bigbins_ints(const RorLaunch &L) {
    return 2 * (size_t)L.ntiles * (2 * (L.TB + 2) * (L.TB + 2) + 1) + 1 + L.ntiles + L.ntiles + 1;
}

void launch_rt_ror(const RorLaunch &L, const int *tstart, float4 *staged, float4 *scratch, int *bigbins,
                   uint64_t *rbits, unsigned long long *counters, int *kept_tile, const int *dirty, hipStream_t s) {
    if (!L.ntiles) return;
    const BigBufs B = big_bufs(L, bigbins);
    if (L.big_ok) {   // tiles beyond the LDS capacity: listed, chunked, sorted and counted by the big kernels
        AOS_HIP(hipMemsetAsync(B.list, 0, sizeof(int), s));
        k_rt_biglist<<<(L.ntiles + 255) / 256, 256, 0, s>>>(L, tstart, B, kept_tile, dirty);
        k_rt_bigchunks<<<1, 1024, 0, s>>>(tstart, B);
        k_rt_bighist<<<kBigGrid, kBigTB, 0, s>>>(L, tstart, staged, B);
        k_rt_bigscan<<<kBigY, 1024, 0, s>>>(L, tstart, B);
        k_rt_bigscatter<<<kBigGrid, kBigTB, 0, s>>>(L, tstart, staged, scratch, B);
    }
    k_rt_ror<false><<<L.ntiles, kRorThreads, 0, s>>>(L, tstart, staged, scratch, rbits, counters, kept_tile, dirty, B);
    if (L.big_ok)
        k_rt_ror<true><<<kBigGrid, kRorThreads, 0, s>>>(L, tstart, staged, scratch, rbits, counters, kept_tile, dirty, B);
    AOS_HIP(hipGetLastError());
}

void launch_rt_merge(const float4 *old_st, const int *old_ts, const float4 *scan_st, const int *scan_ts, float4 *new_st,
                     int *new_ts, int ntiles, int cap, int *overflow, hipStream_t s) {
    k_rt_merge<<<dim3(ntiles + 1, 8), 256, 0, s>>>(old_st, old_ts, scan_st, scan_ts, new_st, new_ts, ntiles, cap, overflow);
    AOS_HIP(hipGetLastError());
}

void launch_rt_sum_kept(const int *kept_tile, int ntiles, unsigned long long *counters, hipStream_t s) {
    k_rt_sum_kept<<<1, 1024, 0, s>>>(kept_tile, ntiles, counters);
    AOS_HIP(hipGetLastError());
}

// Reads the staged array once, so that its lines sit in the Infinity Cache when the scatter writes them.
// The scatter writes ~40 B runs per (workgroup, tile): on lines that missed the cache those partial writes
// cost it 115-124 us instead of 88 (tools/rorbench, RORBENCH_PRETOUCH; the product's staged array is evicted
// by the rest of the frame). Launched while the cloud's upload DMAs run (upload_pack), when the GPU is idle.
__global__ __launch_bounds__(256) void k_rt_touch(const float4 *p, size_t n) {
    float a = 0.f;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a += p[i].x;
    asm volatile("" ::"v"(a));   // (keeps the loads)
}
void launch_rt_touch(const float4 *p, size_t n, hipStream_t s) {
    if (!n) return;
    k_rt_touch<<<2048, 256, 0, s>>>(p, n);
    AOS_HIP(hipGetLastError());
}

}  // namespace aos
