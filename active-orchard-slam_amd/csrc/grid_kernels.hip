// Grid-stage kernels of the seed-gen hot path for gfx950 (MI355X).
//
// Numerics: built with -ffp-contract=off and correctly rounded f32/f64 div/sqrt, so every
// float/double expression below rounds exactly like the reference's x86-64 build
// (CMakeLists.txt:12: no -march, no FMA). Each kernel cites the reference lines it implements.
//
// Layout in HBM: occupancy-type grids are bit-packed, one uint64 word = 64 consecutive cells of
// a row (bit i = cell x = 64*c + i), WW = ceil(W/64) words per row, padding bits zero. Byte grids
// (int8 {0,100}) exist only for the published OccupancyGrid outputs.
#include <hipcub/hipcub.hpp>

#include <climits>
#include <stdexcept>

#include "aos_internal.h"

namespace aos {

// Exclusion discs of processPointCloud (seed_gen:487-499): x, y, radius.
__constant__ float c_excl[11 * 3] = {0.646417f, 3.83918f, 1.0f,  2.0405f, 3.62485f, 1.0f,  65.3711f, 2.09755f, 1.0f,
                                     66.9094f, 2.07515f, 1.0f,  -1.61309f, 5.69933f, 1.0f, -1.97349f, 4.77329f, 1.0f,
                                     -2.11365f, 3.74464f, 1.0f, -2.26381f, 2.70848f, 1.0f, -2.66426f, 1.72738f, 1.0f,
                                     68.0229f, 2.31687f, 1.0f,  65.4647f, 2.18653f, 1.0f};

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ void load_xyz(const RorLaunch &L, uint64_t i, float &x, float &y, float &z) {
    const uint8_t *rec = L.cloud + i * (uint64_t)L.step;
    if (L.step == 16 && L.ox == 0 && L.oy == 4 && L.oz == 8) {
        float4 v = *reinterpret_cast<const float4 *>(rec);
        x = v.x; y = v.y; z = v.z;
    } else {
        x = *reinterpret_cast<const float *>(rec + L.ox);
        y = *reinterpret_cast<const float *>(rec + L.oy);
        z = *reinterpret_cast<const float *>(rec + L.oz);
    }
}

__device__ __forceinline__ bool binned(const RorLaunch &L, float x, float y, float z) {
    return isfinite(x) && isfinite(y) && isfinite(z) && x >= L.bminx && x <= L.bmaxx && y >= L.bminy &&
           y <= L.bmaxy && z >= L.bminz && z <= L.bmaxz;
}

__device__ __forceinline__ int bin_of(const RorLaunch &L, float x, float y, int &bx, int &by) {
    bx = min(max((int)((x - L.bminx) * L.inv_cs), 0), L.nbx - 1);
    by = min(max((int)((y - L.bminy) * L.inv_cs), 0), L.nby - 1);
    return by * L.nbx + bx;
}

// PassThrough z, x, y (inclusive; PCL 1.12 drops non-finite) + exclusion discs, seed_gen:459-525.
__device__ __forceinline__ bool candidate(const RorLaunch &L, float x, float y, float z) {
    if (z < L.cminz || z > L.cmaxz) return false;
    if (x < L.cminx || x > L.cmaxx) return false;
    if (y < L.cminy || y > L.cmaxy) return false;
#pragma unroll
    for (int e = 0; e < 11; ++e) {
        float dx = x - c_excl[3 * e], dy = y - c_excl[3 * e + 1];
        float dist_sq = dx * dx + dy * dy;
        float rr = c_excl[3 * e + 2] * c_excl[3 * e + 2];
        if (dist_sq <= rr) return false;
    }
    return true;
}

// ------------------------------------------------------------------------------------------
// a1 RadiusOutlierRemoval (seed_gen:236-242) restricted to the points that can reach the grid.
// Only points inside the clip box can be rasterised; their neighbours lie within r of that box,
// so only that expanded box is binned (2-D columns of >= r, z checked exactly).
__global__ void k_ror_bin(RorLaunch L, int *bin_count, int2 *pt_binslot) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n) return;
    float x, y, z;
    load_xyz(L, i, x, y, z);
    int2 bs = make_int2(-1, 0);
    if (binned(L, x, y, z)) {
        int bx, by;
        int b = bin_of(L, x, y, bx, by);
        bs = make_int2(b, atomicAdd(&bin_count[b], 1));
    }
    pt_binslot[i] = bs;
}

__global__ void k_ror_scatter(RorLaunch L, const int *bin_start, const int2 *pt_binslot, float4 *sorted) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n) return;
    int2 bs = pt_binslot[i];
    if (bs.x < 0) return;
    float x, y, z;
    load_xyz(L, i, x, y, z);
    int cand = candidate(L, x, y, z) ? 1 : 0;
    sorted[bin_start[bs.x] + bs.y] = make_float4(x, y, z, __int_as_float(cand));
}

// Neighbour count with PCL semantics (FLANN L2_Simple: ((dx*dx)+dy*dy)+dz*dz in float):
//   dense: kNN k = need, keep iff need points have (double)d2 <= r^2;
//   !dense: radius search d2 < float(r^2), keep iff count >= need.
// Kept candidates mark their cell (generateOccupancyGrid seed_gen:606-619: double divide, trunc).
//
// The keep decision only needs "at least need points within r", so the scan order is free (own
// bin row first) and stops early.
#ifndef AOS_ROR_NOSCAN   // timing experiments only (tools/ab_variants.sh): wrong results
#define AOS_ROR_NOSCAN 0
#endif
#ifndef AOS_ROR_NOSTORE
#define AOS_ROR_NOSTORE 0
#endif
// k_ror_direct scan order: 1 row order, 2 own bin first, 3 own bin first for dense bins only
// (0 selects the LDS row sweep k_ror_sweep instead of k_ror_direct)
#ifndef AOS_ROR_DIRECT
#define AOS_ROR_DIRECT 3
#endif
constexpr int kRorDenseBin = 32;

// XCD-aware block order (cdna_hip_programming.md §5.5 T1): blocks b = j (mod 8) share an XCD's L2,
// so group j gets one contiguous range of logical blocks (neighbouring bin rows stay on one L2).
__device__ __forceinline__ int xcd_block(int b, int n) {
    const int q = n >> 3, r = n & 7, j = b & 7, k = b >> 3;
    return j * q + min(j, r) + k;
}

__device__ __forceinline__ bool ror_in(const RorLaunch &L, float4 p, float4 q) {
    float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
    float d2 = dx * dx;
    d2 = d2 + dy * dy;
    d2 = d2 + dz * dz;
    // dense: (double)d2 <= r2 is the same test as d2 <= r2df for every float d2 (incl. inf / NaN)
    return L.is_dense ? (d2 <= L.r2df) : (d2 < L.r2f);
}
template <class Ptr>
__device__ __forceinline__ int ror_scan(const RorLaunch &L, float4 p, Ptr pts, int k0, int k1, int cnt) {
    for (int k = k0; k < k1 && cnt < L.need; k += 4) {
        float4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = pts[min(k + j, k1 - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j) cnt += (k + j < k1 && ror_in(L, p, q[j])) ? 1 : 0;
    }
    return cnt;
}

// same as ror_scan on one staged LDS row (indexing the __shared__ row keeps ds_read instructions)
__device__ __forceinline__ int ror_scan_lds(const RorLaunch &L, float4 p, const float4 (&row)[512], int k0, int k1, int cnt) {
    for (int k = k0; k < k1 && cnt < L.need; k += 4) {
        float4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = row[min(k + j, k1 - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j) cnt += (k + j < k1 && ror_in(L, p, q[j])) ? 1 : 0;
    }
    return cnt;
}

// LDS-staged bins, row sweep: one workgroup per (strip of kSwSW bins) x (segment of kSwSeg bin rows).
// A candidate's neighbours lie in 3 x 3 bins; the bins of one row of a strip (plus one bin on each
// side) are one contiguous range of the bin-sorted point array, copied into LDS coalesced. It keeps
// a ring of 4 staged point rows (y-1, y, y+1 and y+2 in flight) and 5 rows of bin offsets in LDS.
// While it scans row y it has already issued the loads of row y+2's points and row y+3's offsets
// into registers, so each step costs ~max(scan, one load latency) instead of a 3-trip chain per
// workgroup. Rows with more than kSwCap points stay in global memory (scanned there).
#ifndef AOS_SW_SEG
#define AOS_SW_SEG 32
#endif
constexpr int kSwSW = 64, kSwTB = 256, kSwCap = 512, kSwSeg = AOS_SW_SEG, kSwPer = kSwCap / kSwTB;

__global__ __launch_bounds__(kSwTB) void k_ror_sweep(RorLaunch L, const int *bin_start, const float4 *sorted,
                                                     uint8_t *raster, unsigned long long *counters) {
    __shared__ float4 pts[4][kSwCap];
    __shared__ int offs[5][kSwSW + 3];
    __shared__ int staged[4];            // 1: row's points are in pts[slot]; 0: read them from global
    const int tid = threadIdx.x;
    const int nstrip = (L.nbx + kSwSW - 1) / kSwSW;
    const int blk = xcd_block(blockIdx.x, gridDim.x);
    const int strip = blk % nstrip, seg = blk / nstrip;
    const int bx0 = strip * kSwSW, bx1 = min(bx0 + kSwSW, L.nbx);
    const int xlo = max(bx0 - 1, 0), xhi = min(bx1, L.nbx - 1), nbins = xhi - xlo + 1;
    const int y0 = seg * kSwSeg, y1 = min(y0 + kSwSeg, L.nby);
    auto row_ok = [&](int yy) { return yy >= 0 && yy < L.nby; };
    auto offs_of = [&](int yy, int c) { return row_ok(yy) ? bin_start[yy * L.nbx + xlo + c] : 0; };
    // prologue: offsets of rows y0-1 .. y0+2, points of rows y0-1 .. y0+1
    for (int t = tid; t < 4 * (nbins + 1); t += kSwTB) {
        const int r = t / (nbins + 1), c = t - r * (nbins + 1), yy = y0 - 1 + r;
        offs[(yy + 5) % 5][c] = offs_of(yy, c);
    }
    __syncthreads();
    for (int r = 0; r < 3; ++r) {
        const int yy = y0 - 1 + r, o = (yy + 5) % 5, sl = (yy + 4) & 3;
        const int a = offs[o][0], n = offs[o][nbins] - a;
        if (n <= kSwCap)
            for (int t = tid; t < n; t += kSwTB) pts[sl][t] = sorted[a + t];
        if (tid == 0) staged[sl] = n <= kSwCap;
    }
    __syncthreads();
    unsigned kept_n = 0;
    for (int y = y0; y < y1; ++y) {
        // (1) issue the loads for row y+2's points and row y+3's offsets
        const int opf = (y + 2 + 5) % 5, spf = (y + 2) & 3;
        const int apf = offs[opf][0], npf = offs[opf][nbins] - apf;
        float4 q[kSwPer];
#pragma unroll
        for (int j = 0; j < kSwPer; ++j) {
            const int t = tid + j * kSwTB;
            q[j] = sorted[(t < npf && npf <= kSwCap) ? apf + t : 0];
        }
        const int onew = tid <= nbins ? offs_of(y + 3, tid) : 0;
        // (2) count neighbours of row y's candidates from the staged rows y-1, y, y+1. The own point is
        // read in a branch on the (workgroup-uniform) staged flag: a select of an LDS and a global
        // pointer would become a flat load, whose vmcnt wait would also wait for the prefetch above.
        const int ocur = (y + 5) % 5, scur = y & 3;
        const int own0 = offs[ocur][bx0 - xlo], own1 = offs[ocur][bx1 - xlo], base0 = offs[ocur][0];
        auto count_one = [&](const float4 p) {
            if (__float_as_int(p.w) == 0) return;   // not a clip candidate
            int bx, byy;
            bin_of(L, p.x, p.y, bx, byy);
            const int c0 = max(bx - 1, xlo) - xlo, c1 = min(bx + 1, xhi) - xlo + 1;
            int cnt = AOS_ROR_NOSCAN ? L.need : 0;
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const int yy = rr == 0 ? y : (rr == 1 ? y - 1 : y + 1);   // own bin row first
                if (!row_ok(yy) || cnt >= L.need) continue;
                const int o = (yy + 5) % 5, sl = (yy + 4) & 3;
                const int g0 = offs[o][c0], g1 = offs[o][c1];
                if (staged[sl]) cnt = ror_scan_lds(L, p, pts[sl], g0 - offs[o][0], g1 - offs[o][0], cnt);
                else cnt = ror_scan(L, p, sorted, g0, g1, cnt);
            }
            if (cnt >= L.need) {
                int gx = (int)(((double)p.x - L.origin_x) / (double)L.res);
                int gy = (int)(((double)p.y - L.origin_y) / (double)L.res);
                const int cx = min(max(gx, 0), L.W - 1), cy = min(max(gy, 0), L.H - 1);
                if (cx >= L.rx0 && cx < L.rx1 && cy >= L.ry0 && cy < L.ry1) {   // this tile's candidate
                    ++kept_n;
                    if (!AOS_ROR_NOSTORE && gx >= 0 && gx < L.W && gy >= 0 && gy < L.H)
                        raster[(size_t)(gy - L.wy0) * L.Wr + (gx - L.wx0)] = 1;
                }
            }
        };
        if (staged[scur]) {
            for (int k = own0 + tid; k < own1; k += kSwTB) count_one(pts[scur][k - base0]);
        } else {
            for (int k = own0 + tid; k < own1; k += kSwTB) count_one(sorted[k]);
        }
        // (3) commit the prefetched row y+2 and offsets of row y+3. Their slots held row y-2, which
        // step y no longer reads, so no barrier is needed before the writes.
        if (npf <= kSwCap) {
#pragma unroll
            for (int j = 0; j < kSwPer; ++j) {
                const int t = tid + j * kSwTB;
                if (t < npf) pts[spf][t] = q[j];
            }
        }
        if (tid <= nbins) offs[(y + 3 + 5) % 5][tid] = onew;
        if (tid == 0) staged[spf] = npf <= kSwCap;
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) kept_n += __shfl_xor(kept_n, o);
    if ((tid & 63) == 0 && kept_n)
        atomicAdd(&counters[(blk * (kSwTB / 64) + (tid >> 6)) & (kRorCounters - 1)], (unsigned long long)kept_n);   // spread: one
    // hot address would serialise ~10^5 same-address atomics in one L2 channel
}

// Kept candidate: count it if its (clamped) cell is owned, raster it if inside the grid.
__device__ __forceinline__ void ror_keep(const RorLaunch &L, float4 p, uint8_t *raster, unsigned &kept_n) {
    int gx = (int)(((double)p.x - L.origin_x) / (double)L.res);
    int gy = (int)(((double)p.y - L.origin_y) / (double)L.res);
    const int cx = min(max(gx, 0), L.W - 1), cy = min(max(gy, 0), L.H - 1);
    if (cx >= L.rx0 && cx < L.rx1 && cy >= L.ry0 && cy < L.ry1) {
        ++kept_n;
        if (!AOS_ROR_NOSTORE && gx >= 0 && gx < L.W && gy >= 0 && gy < L.H)
            raster[(size_t)(gy - L.wy0) * L.Wr + (gx - L.wx0)] = 1;
    }
}

// Direct variant: one thread per staged point, in bin order, reading the 3 x 3 neighbour bins
// straight from global memory (consecutive lanes scan nearly the same ranges, so the loads hit
// the same cache lines). No LDS, no barriers: occupancy is bounded by registers only.
__global__ __launch_bounds__(256) void k_ror_direct(RorLaunch L, const int *bin_start, const float4 *sorted,
                                                    const int *n_binned, uint8_t *raster,
                                                    unsigned long long *counters) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned kept_n = 0;
    if (i < *n_binned) {
        const float4 p = sorted[i];
        if (__float_as_int(p.w)) {
            int bx, by;
            bin_of(L, p.x, p.y, bx, by);
            const int c0 = max(bx - 1, 0), c1 = min(bx + 1, L.nbx - 1);
            int cnt = AOS_ROR_NOSCAN ? L.need : 0;
            // Scan order. Row order: the own bin row, then the rows above and below (3 bins each).
            // Own-first: the point itself (d2 = 0 passes both tests), its own bin around it, then the
            // other 8 bins; the own bin holds the likeliest neighbours, so most scans stop early.
            // Variant 3 (default) goes own-first only for a dense own bin (>= kRorDenseBin points):
            // there a row scan starts in the left bin and wades through its points, most of them > r
            // away in x (a streaming map stacks ~300 points in a canopy bin: 0.85 -> 0.34 ms). Sparse
            // bins keep the row order, which needs fewer, longer loops (C2: 0.154 ms against 0.196
            // with own-first everywhere). The keep decision does not depend on the order.
            bool own_first = AOS_ROR_DIRECT == 2;
            int b0 = 0, b1 = 0;
            if (AOS_ROR_DIRECT >= 2) {
                const int ob = by * L.nbx + bx;
                b0 = bin_start[ob];
                b1 = bin_start[ob + 1];
                own_first = own_first || b1 - b0 >= kRorDenseBin;
            }
            if (own_first) {
                cnt = 1;
                cnt = ror_scan(L, p, sorted, i + 1, b1, cnt);
                cnt = ror_scan(L, p, sorted, b0, i, cnt);
                if (cnt < L.need) cnt = ror_scan(L, p, sorted, bin_start[by * L.nbx + c0], b0, cnt);
                if (cnt < L.need) cnt = ror_scan(L, p, sorted, b1, bin_start[by * L.nbx + c1 + 1], cnt);
                for (int rr = 1; rr < 3; ++rr) {
                    const int yy = rr == 1 ? by - 1 : by + 1;
                    if (yy < 0 || yy >= L.nby || cnt >= L.need) continue;
                    cnt = ror_scan(L, p, sorted, bin_start[yy * L.nbx + c0], bin_start[yy * L.nbx + c1 + 1], cnt);
                }
            } else {
#pragma unroll
                for (int rr = 0; rr < 3; ++rr) {
                    const int yy = rr == 0 ? by : (rr == 1 ? by - 1 : by + 1);   // own bin row first
                    if (yy < 0 || yy >= L.nby || cnt >= L.need) continue;
                    cnt = ror_scan(L, p, sorted, bin_start[yy * L.nbx + c0], bin_start[yy * L.nbx + c1 + 1], cnt);
                }
            }
            if (cnt >= L.need) ror_keep(L, p, raster, kept_n);
        }
    }
    for (int o = 32; o > 0; o >>= 1) kept_n += __shfl_xor(kept_n, o);
    if ((threadIdx.x & 63) == 0 && kept_n)
        atomicAdd(&counters[(blockIdx.x * 4 + (threadIdx.x >> 6)) & (kRorCounters - 1)], (unsigned long long)kept_n);
}

// Counting sort without a per-point slot array: k_ror_count counts points per bin with
// non-returning atomics (fire and forget), the exclusive scan is written one element to the right
// (cursor[1 + b] = start of bin b), and k_ror_place claims each point's position with a returning
// atomic on that cursor. After the placement cursor[b] = start of bin b for every b <= nb, i.e.
// the cursor array IS bin_start. Order inside a bin is arbitrary, as before (the ROR decision is
// order-free).
__global__ void k_ror_count(RorLaunch L, int *bin_count) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n) return;
    float x, y, z;
    load_xyz(L, i, x, y, z);
    if (binned(L, x, y, z)) {
        int bx, by;
        atomicAdd(&bin_count[bin_of(L, x, y, bx, by)], 1);
    }
}

__global__ void k_ror_place(RorLaunch L, int *cursor, float4 *sorted) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n) return;
    float x, y, z;
    load_xyz(L, i, x, y, z);
    if (!binned(L, x, y, z)) return;
    int bx, by;
    const int pos = atomicAdd(&cursor[1 + bin_of(L, x, y, bx, by)], 1);
    sorted[pos] = make_float4(x, y, z, __int_as_float(candidate(L, x, y, z) ? 1 : 0));
}

void launch_ror_count(const RorLaunch &L, int *bin_count, hipStream_t s) {
    if (!L.n) return;
    k_ror_count<<<cdiv(L.n, 256), 256, 0, s>>>(L, bin_count);
}
void launch_ror_place(const RorLaunch &L, int *cursor, float4 *sorted, hipStream_t s) {
    if (!L.n) return;
    k_ror_place<<<cdiv(L.n, 256), 256, 0, s>>>(L, cursor, sorted);
}

void launch_ror_bin(const RorLaunch &L, int *bin_count, int2 *pt_binslot, hipStream_t s) {
    if (!L.n) return;
    k_ror_bin<<<cdiv(L.n, 256), 256, 0, s>>>(L, bin_count, pt_binslot);
}
void launch_ror_scatter(const RorLaunch &L, const int *bin_start, const int2 *pt_binslot, float4 *sorted, hipStream_t s) {
    if (!L.n) return;
    k_ror_scatter<<<cdiv(L.n, 256), 256, 0, s>>>(L, bin_start, pt_binslot, sorted);
}

void launch_ror_raster(const RorLaunch &L, const int *bin_start, const float4 *sorted, uint8_t *raster,
                       unsigned long long *counters, hipStream_t s) {
    if (AOS_ROR_DIRECT) {
        if (!L.n) return;
        k_ror_direct<<<cdiv(L.n, 256), 256, 0, s>>>(L, bin_start, sorted, bin_start + L.nbx * L.nby, raster, counters);
        return;
    }
    const long long nblk = (long long)((L.nby + kSwSeg - 1) / kSwSeg) * ((L.nbx + kSwSW - 1) / kSwSW);
    if (nblk <= 0) return;
    if (nblk > INT_MAX) throw std::runtime_error("ROR bin grid too large");
    k_ror_sweep<<<(int)nblk, kSwTB, 0, s>>>(L, bin_start, sorted, raster, counters);

}

size_t scan_temp_bytes(int n) {
    size_t t = 0;
    AOS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t, (const int *)nullptr, (int *)nullptr, n));
    return t;
}
void launch_exclusive_scan(const int *in, int *out, int n, void *temp, size_t temp_bytes, hipStream_t s) {
    AOS_HIP(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, n, s));
}

// ------------------------------------------------------------------------------------------
// Streaming ingest: a scan's records -> the map's float4 (x, y, z, 0) layout (aos_map_append).
__global__ void k_pack_xyz(const uint8_t *cloud, uint64_t n, uint32_t step, uint32_t ox, uint32_t oy, uint32_t oz,
                           float4 *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *rec = cloud + i * (uint64_t)step;
    out[i] = make_float4(*reinterpret_cast<const float *>(rec + ox), *reinterpret_cast<const float *>(rec + oy),
                         *reinterpret_cast<const float *>(rec + oz), 0.0f);
}
void launch_pack_xyz(const uint8_t *cloud, uint64_t n, uint32_t step, uint32_t ox, uint32_t oy, uint32_t oz, float4 *out,
                     hipStream_t s) {
    if (!n) return;
    k_pack_xyz<<<cdiv(n, 256), 256, 0, s>>>(cloud, n, step, ox, oy, oz, out);
}

// ------------------------------------------------------------------------------------------
// bytes (0 / non-zero) -> bits
__global__ void k_pack_bits(const uint8_t *bytes, uint64_t *bits, int W, int H, int WW) {
    int c = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (c >= WW || y >= H) return;
    const uint8_t *row = bytes + (size_t)y * W;
    uint64_t w = 0;
    int x0 = c * 64;
    if ((W & 15) == 0 && x0 + 64 <= W) {
        const uint4 *v = reinterpret_cast<const uint4 *>(row + x0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint4 u = v[q];
            uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if ((wd[k] >> (8 * b)) & 0xFF) w |= 1ull << (q * 16 + k * 4 + b);
        }
    } else {
        for (int i = 0; i < 64 && x0 + i < W; ++i)
            if (row[x0 + i]) w |= 1ull << i;
    }
    bits[(size_t)y * WW + c] = w;
}
void launch_pack_bits(const uint8_t *bytes, uint64_t *bits, int W, int H, int WW, hipStream_t s) {
    dim3 g(cdiv(WW, 64), H);
    k_pack_bits<<<g, 64, 0, s>>>(bytes, bits, W, H, WW);
}

__device__ __forceinline__ uint64_t pad_mask(int c, int WW, int W) {
    // bits of word c that lie inside the image
    int rem = W - c * 64;
    return rem >= 64 ? ~0ull : (rem <= 0 ? 0ull : ((1ull << rem) - 1));
}

// ------------------------------------------------------------------------------------------
// a5 applyInflation (seed_gen:933-967): cell = 100 iff an occupied raster cell lies within the
// integer disc dx^2 + dy^2 <= R^2 — an exact bounded squared-EDT threshold, computed as an OR
// of horizontally dilated rows: row y+dy dilated by w(dy) = floor(sqrt(R^2 - dy^2)).
struct InflTab { int w[64]; };   // w(dy), passed by value: concurrent handles share no device global
__global__ void k_inflate(const uint64_t *in, uint64_t *out, int W, int H, int WW, int R, InflTab wt) {
    int c = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (c >= WW || y >= H) return;
    uint64_t acc = 0;
    for (int dy = -R; dy <= R; ++dy) {
        int yy = y + dy;
        if (yy < 0 || yy >= H) continue;
        const uint64_t *row = in + (size_t)yy * WW;
        uint64_t b = row[c];
        uint64_t a = c > 0 ? row[c - 1] : 0ull;
        uint64_t d = c + 1 < WW ? row[c + 1] : 0ull;
        int w = wt.w[dy < 0 ? -dy : dy];
        uint64_t h = b;
        for (int s = 1; s <= w; ++s) h |= (b >> s) | (d << (64 - s)) | (b << s) | (a >> (64 - s));
        acc |= h;
    }
    out[(size_t)y * WW + c] = acc & pad_mask(c, WW, W);
}
void launch_inflate(const uint64_t *in, uint64_t *out, const FrameGeom &g, hipStream_t s) {
    InflTab wt{};
    for (int dy = 0; dy <= g.R && dy < 64; ++dy) {
        int w = 0;
        while ((w + 1) * (w + 1) + dy * dy <= g.R * g.R) ++w;
        wt.w[dy] = w;
    }
    dim3 grid(cdiv(g.WW, 64), g.H);
    k_inflate<<<grid, 64, 0, s>>>(in, out, g.W, g.H, g.WW, g.R, wt);
}

// bits -> int8 {0,100} with an optional `frame`-cell border (markBoundariesAsOccupied, seed_gen:708-757)
__global__ void k_bits_to_bytes(const uint64_t *bits, int8_t *out, int W, int H, int WW, int frame) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)W * H) return;
    int y = (int)(i / W), x = (int)(i - (size_t)y * W);
    bool v = (bits[(size_t)y * WW + (x >> 6)] >> (x & 63)) & 1ull;
    if (frame > 0 && (x < frame || y < frame || x >= W - frame || y >= H - frame)) v = true;
    out[i] = v ? 100 : 0;
}
void launch_bits_to_bytes(const uint64_t *bits, int8_t *out, const FrameGeom &g, int frame, hipStream_t s) {
    size_t n = (size_t)g.W * g.H;
    k_bits_to_bytes<<<cdiv(n, 256), 256, 0, s>>>(bits, out, g.W, g.H, g.WW, frame);
}

// ------------------------------------------------------------------------------------------
// a7 morphologyEx(MORPH_OPEN, 3x3 MORPH_ELLIPSE = cross), BORDER_CONSTANT default value:
// erosion reads 255 outside the image, dilation reads 0 (seed_gen:678-680).
__device__ __forceinline__ uint64_t ld_er(const uint64_t *in, int r, int k, int H, int WW, int W) {
    if (r < 0 || r >= H || k < 0 || k >= WW) return ~0ull;
    return in[(size_t)r * WW + k] | ~pad_mask(k, WW, W);
}
__device__ __forceinline__ uint64_t erode_at(const uint64_t *in, int r, int k, int H, int WW, int W) {
    if (r < 0 || r >= H || k < 0 || k >= WW) return 0ull;  // dilation reads 0 outside
    uint64_t c = ld_er(in, r, k, H, WW, W);
    uint64_t wv = (c << 1) | (ld_er(in, r, k - 1, H, WW, W) >> 63);
    uint64_t ev = (c >> 1) | (ld_er(in, r, k + 1, H, WW, W) << 63);
    return (c & wv & ev & ld_er(in, r - 1, k, H, WW, W) & ld_er(in, r + 1, k, H, WW, W)) & pad_mask(k, WW, W);
}
__global__ void k_open(const uint64_t *in, uint64_t *out, int W, int H, int WW) {
    int k = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
    if (k >= WW || r >= H) return;
    uint64_t e = erode_at(in, r, k, H, WW, W);
    uint64_t d = e | erode_at(in, r - 1, k, H, WW, W) | erode_at(in, r + 1, k, H, WW, W) |
                 (e << 1) | (erode_at(in, r, k - 1, H, WW, W) >> 63) | (e >> 1) | (erode_at(in, r, k + 1, H, WW, W) << 63);
    out[(size_t)r * WW + k] = d & pad_mask(k, WW, W);
}
void launch_open(const uint64_t *in, uint64_t *out, const FrameGeom &g, hipStream_t s) {
    dim3 grid(cdiv(g.WW, 64), g.H);
    k_open<<<grid, 64, 0, s>>>(in, out, g.W, g.H, g.WW);
}

// ------------------------------------------------------------------------------------------
// a7 ximgproc::thinning(THINNING_ZHANGSUEN) with temporal blocking.
// One workgroup owns a TH x TWW-word tile and loads it with a halo of HR = 2*KIT rows and one
// word (64 cells) on each side into LDS, then runs KIT full iterations (2*KIT Jacobi
// sub-iterations) in LDS: each sub-iteration invalidates one more halo row/cell from the outside
// in, so the interior stays exact. Bit-sliced logic evaluates the Zhang-Suen predicate for 64
// cells per 64-bit word:
//   A == 1       : exactly one 0->1 transition in p2,p3,...,p9,p2
//   2 <= B <= 6  : at least two set and at least two clear among p2..p9
//   m1 == m2 == 0: iter 0: p2p4p6 = p4p6p8 = 0; iter 1: p2p4p8 = p2p6p8 = 0
// Rows 0 / H-1 and columns 0 / W-1 of the image are never examined (ximgproc loops 1..n-2).
constexpr int TH = 64, TWW = 8, KIT = kThinItersPerLaunch, HR = 2 * KIT, NR = TH + 2 * HR, NC = TWW + 2;

__device__ __forceinline__ uint64_t zs_step(uint64_t n0, uint64_t n1, uint64_t n2, uint64_t c0, uint64_t c1,
                                            uint64_t c2, uint64_t s0, uint64_t s1, uint64_t s2, int sub) {
    // x0 = word to the west, x1 = this word, x2 = word to the east
    const uint64_t p2 = n1;
    const uint64_t p3 = (n1 >> 1) | (n2 << 63);   // (y-1, x+1)
    const uint64_t p4 = (c1 >> 1) | (c2 << 63);   // (y,   x+1)
    const uint64_t p5 = (s1 >> 1) | (s2 << 63);   // (y+1, x+1)
    const uint64_t p6 = s1;                       // (y+1, x)
    const uint64_t p7 = (s1 << 1) | (s0 >> 63);   // (y+1, x-1)
    const uint64_t p8 = (c1 << 1) | (c0 >> 63);   // (y,   x-1)
    const uint64_t p9 = (n1 << 1) | (n0 >> 63);   // (y-1, x-1)
    const uint64_t seq[9] = {p2, p3, p4, p5, p6, p7, p8, p9, p2};
    uint64_t one = 0, two = 0;          // transitions
    uint64_t o1 = 0, o2 = 0;            // set neighbours >= 1, >= 2
    uint64_t z1 = 0, z2 = 0;            // clear neighbours >= 1, >= 2
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint64_t t = ~seq[k] & seq[k + 1];
        two |= one & t; one |= t;
        uint64_t p = seq[k];
        o2 |= o1 & p; o1 |= p;
        uint64_t q = ~p;
        z2 |= z1 & q; z1 |= q;
    }
    uint64_t A1 = one & ~two;
    uint64_t B26 = o2 & z2;
    uint64_t m = sub == 0 ? (~(p2 & p4 & p6) & ~(p4 & p6 & p8)) : (~(p2 & p4 & p8) & ~(p2 & p6 & p8));
    return c1 & A1 & B26 & m;  // cells to delete
}

__global__ __launch_bounds__(256) void k_thin_block(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                    int W, int H, int WW, int base_iter, int *flags, ThinOwn own) {
    if (own.early_exit && base_iter >= 2 && flags[1 + base_iter - 1] == 0) return;  // converged in an earlier launch
    __shared__ uint64_t buf[2][NR][NC];
    __shared__ int chg_shared;
    const int ty0 = blockIdx.y * TH, tc0 = blockIdx.x * TWW;
    if (threadIdx.x == 0) chg_shared = 0;
    for (int idx = threadIdx.x; idx < NR * NC; idx += blockDim.x) {
        int r = idx / NC, k = idx - r * NC;
        int gy = ty0 - HR + r, gc = tc0 - 1 + k;
        buf[0][r][k] = (gy >= 0 && gy < H && gc >= 0 && gc < WW) ? in[(size_t)gy * WW + gc] : 0ull;
    }
    __syncthreads();
    int chg = 0;        // bit j: iteration base_iter + j deleted something inside this tile
    int nonempty = 0;   // after iteration 0 (only meaningful when base_iter == 0)
    int cur = 0;
    for (int s = 0; s < 2 * KIT; ++s) {
        const int sub = s & 1;
        for (int idx = threadIdx.x; idx < NR * NC; idx += blockDim.x) {
            int r = idx / NC, k = idx - r * NC;
            const int gy = ty0 - HR + r, gc = tc0 - 1 + k;
            // cells this launch reports: its tile interior, within the caller's own rectangle
            const bool mine = r >= HR && r < HR + TH && k >= 1 && k <= TWW && gy >= own.y0 && gy < own.y1 &&
                              gc >= own.c0 && gc < own.c1;
            uint64_t c1 = buf[cur][r][k];
            uint64_t nw = c1;
            if (r > 0 && r < NR - 1) {
                uint64_t c0 = k > 0 ? buf[cur][r][k - 1] : 0ull, c2 = k < NC - 1 ? buf[cur][r][k + 1] : 0ull;
                uint64_t n0 = k > 0 ? buf[cur][r - 1][k - 1] : 0ull, n1 = buf[cur][r - 1][k],
                         n2 = k < NC - 1 ? buf[cur][r - 1][k + 1] : 0ull;
                uint64_t s0 = k > 0 ? buf[cur][r + 1][k - 1] : 0ull, s1 = buf[cur][r + 1][k],
                         s2 = k < NC - 1 ? buf[cur][r + 1][k + 1] : 0ull;
                uint64_t del = zs_step(n0, n1, n2, c0, c1, c2, s0, s1, s2, sub);
                // examinable cells: 1 <= y <= H-2, 1 <= x <= W-2
                uint64_t em = 0;
                if (gy >= 1 && gy <= H - 2 && gc >= 0 && gc < WW) {
                    em = pad_mask(gc, WW, W - 1);
                    if (gc == 0) em &= ~1ull;
                }
                del &= em;
                nw = c1 & ~del;
                if (del && mine) chg |= 1 << (s >> 1);
            }
            buf[cur ^ 1][r][k] = nw;
            if (s == 1 && base_iter == 0 && nw && mine) nonempty = 1;
        }
        cur ^= 1;
        __syncthreads();
    }
    for (int idx = threadIdx.x; idx < TH * TWW; idx += blockDim.x) {
        int r = idx / TWW, k = idx - r * TWW;
        int gy = ty0 + r, gc = tc0 + k;
        if (gy < H && gc < WW) out[(size_t)gy * WW + gc] = buf[cur][HR + r][1 + k];
    }
    if (chg || nonempty) atomicOr(&chg_shared, chg | (nonempty << 30));
    __syncthreads();
    if (threadIdx.x == 0 && chg_shared) {
        int m = chg_shared;
        if (m & (1 << 30)) atomicOr(&flags[0], 1);
        for (int j = 0; j < KIT; ++j)
            if (m & (1 << j)) atomicOr(&flags[1 + base_iter + j], 1);
    }
}

void launch_thin_block(const uint64_t *in, uint64_t *out, const FrameGeom &g, int base_iter, int *flags,
                       const ThinOwn &own, hipStream_t s) {
    dim3 grid(cdiv(g.WW, TWW), cdiv(g.H, TH));
    k_thin_block<<<grid, 256, 0, s>>>(in, out, g.W, g.H, g.WW, base_iter, flags, own);
}

// a16 markPolygonBoundaryAsOccupied (seed_gen:772-825): the bbox +- 2.5 m rectangle in grid cells;
// drawLineInGrid (Bresenham, :828-870) of an axis-aligned segment is the straight run of cells.
__global__ void k_draw_rect(int8_t *grid, int W, int H, int gx0, int gy0, int gx1, int gy1) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    int xlo = min(gx0, gx1), xhi = max(gx0, gx1), ylo = min(gy0, gy1), yhi = max(gy0, gy1);
    int nx = xhi - xlo + 1, ny = yhi - ylo + 1;
    if (i < nx) {
        grid[(size_t)gy0 * W + xlo + i] = 100;
        grid[(size_t)gy1 * W + xlo + i] = 100;
    } else if (i < nx + ny) {
        int j = i - nx;
        grid[(size_t)(ylo + j) * W + gx0] = 100;
        grid[(size_t)(ylo + j) * W + gx1] = 100;
    }
}
void launch_draw_rect(int8_t *grid, const FrameGeom &g, int gx0, int gy0, int gx1, int gy1, hipStream_t s) {
    int n = abs(gx1 - gx0) + abs(gy1 - gy0) + 2;
    k_draw_rect<<<cdiv(n, 256), 256, 0, s>>>(grid, g.W, g.H, gx0, gy0, gx1, gy1);
}

}  // namespace aos
