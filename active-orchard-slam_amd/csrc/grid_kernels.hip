// Grid-stage kernels of the seed-gen hot path for gfx950 (MI355X).
//
// Numerics: built with -ffp-contract=off and correctly rounded f32/f64 div/sqrt, so every
// float/double expression below rounds exactly like the reference's x86-64 build
// (CMakeLists.txt:12: no -march, no FMA). Each kernel cites the reference lines it implements.
//
// Layout in HBM: occupancy-type grids are bit-packed, one uint64 word = 64 consecutive cells of
// a row (bit i = cell x = 64*c + i), WW = ceil(W/64) words per row, padding bits zero. Byte grids
// (int8 {0,100}) exist only for the published OccupancyGrid outputs.
#include <climits>
#include <stdexcept>

#include "aos_internal.h"

namespace aos {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// (a1-a4, ROR + clip + raster: ror.hip)

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

// Tiled streaming map (aos_tiled_map_append): the scan's records inside this rank's points box (the
// points its tile can rasterise or count as ROR neighbours, tiled.hip make_tile_plan) are appended to
// the rank's map. Their order in the map is the atomics' order: the ROR keep decision and the raster
// do not depend on point order (ror.hip).
__global__ void k_pack_xyz_box(const uint8_t *cloud, uint64_t n, uint32_t step, uint32_t ox, uint32_t oy, uint32_t oz,
                               float bx0, float by0, float bx1, float by1, float4 *out, unsigned long long *count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool keep = false;
    float4 v;
    if (i < n) {
        const uint8_t *rec = cloud + i * (uint64_t)step;
        v = make_float4(*reinterpret_cast<const float *>(rec + ox), *reinterpret_cast<const float *>(rec + oy),
                        *reinterpret_cast<const float *>(rec + oz), 0.0f);
        keep = v.x >= bx0 && v.x <= bx1 && v.y >= by0 && v.y <= by1;   // (NaN fails: never binned)
    }
    const unsigned long long m = __ballot(keep);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(count, (unsigned long long)__popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1);
    if (keep) out[base + __popcll(m & ((1ull << lane) - 1))] = v;
}
void launch_pack_xyz_box(const uint8_t *cloud, uint64_t n, uint32_t step, uint32_t ox, uint32_t oy, uint32_t oz,
                         const float box[4], float4 *out, unsigned long long *count, hipStream_t s) {
    if (!n) return;
    k_pack_xyz_box<<<cdiv(n, 256), 256, 0, s>>>(cloud, n, step, ox, oy, oz, box[0], box[1], box[2], box[3], out, count);
}

__device__ __forceinline__ uint64_t pad_mask(int c, int WW, int W) {
    // bits of word c that lie inside the image
    int rem = W - c * 64;
    return rem >= 64 ? ~0ull : (rem <= 0 ? 0ull : ((1ull << rem) - 1));
}

// ------------------------------------------------------------------------------------------
// Bits -> int8 {0, 100} bytes, one 64-cell word per thread: 64 bytes as four 16-byte stores when rows are
// 16-byte aligned (W % 16 == 0), so a wave writes 4 KB in one run (round 4's byte-per-thread kernel, with
// a 64-bit division per cell, ran at ~0.6 TB/s: 29 us per C2 grid).
__device__ __forceinline__ unsigned nib_bytes(unsigned b) {   // 4 bits -> 4 bytes of {0, 100}
    return ((b & 1u) ? 100u : 0u) | ((b & 2u) ? 100u << 8 : 0u) | ((b & 4u) ? 100u << 16 : 0u) | ((b & 8u) ? 100u << 24 : 0u);
}
__device__ __forceinline__ void store_word_bytes(int8_t *o, uint64_t v, int nb, bool vec) {
    if (vec && nb == 64) {
        uint4 *q = reinterpret_cast<uint4 *>(o);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned h = (unsigned)(v >> (16 * k));
            q[k] = make_uint4(nib_bytes(h & 15u), nib_bytes((h >> 4) & 15u), nib_bytes((h >> 8) & 15u), nib_bytes((h >> 12) & 15u));
        }
    } else {
        for (int b = 0; b < nb; ++b) o[b] = ((v >> b) & 1ull) ? 100 : 0;
    }
}
// the cells [lo, hi] of the word that starts at cell x0, as bits
__device__ __forceinline__ uint64_t run_bits(int lo, int hi, int x0) {
    const int a = max(lo - x0, 0), b = min(hi - x0, 63);
    if (a > b) return 0ull;
    return (b - a == 63 ? ~0ull : ((1ull << (b - a + 1)) - 1)) << a;
}
// The cells a published grid adds to its bits in word (x0, y): the `frame`-cell border of /occupancy_grid
// (markBoundariesAsOccupied, seed_gen:708-757) and the polygon rectangle of /skeletonized_occupancy_grid
// (markPolygonBoundaryAsOccupied, seed_gen:772-870: rows gy0 / gy1 over [xlo, xhi], columns gx0 / gx1 over
// [ylo, yhi]; r.gx0 < 0: none)
__device__ __forceinline__ uint64_t grid_extra(int x0, int y, int W, int H, int frame, const ByteRect &r) {
    uint64_t m = 0;
    if (frame > 0) m = (y < frame || y >= H - frame) ? ~0ull : (run_bits(0, frame - 1, x0) | run_bits(W - frame, W - 1, x0));
    if (r.gx0 >= 0) {
        const int xlo = min(r.gx0, r.gx1), xhi = max(r.gx0, r.gx1), ylo = min(r.gy0, r.gy1), yhi = max(r.gy0, r.gy1);
        if (y == r.gy0 || y == r.gy1) m |= run_bits(xlo, xhi, x0);
        if (y >= ylo && y <= yhi) m |= run_bits(r.gx0, r.gx0, x0) | run_bits(r.gx1, r.gx1, x0);
    }
    return m;
}

// The word-per-thread grid kernels run in blocks of 64 words x kRowBlk rows (round 6; one-row blocks before: k_open
// 8.1-9.7 -> 6.6-8.1 us per C2 launch, k_inflate and k_bits_to_bytes unchanged, profiles/r06/r06zd_kt_summary.txt)
constexpr int kRowBlk = 4;
static const dim3 kRowBlock(64, kRowBlk);
static dim3 row_grid(int WW, int H) { return dim3(cdiv(WW, 64), cdiv(H, kRowBlk)); }

// a5 applyInflation (seed_gen:933-967): cell = 100 iff an occupied raster cell lies within the
// integer disc dx^2 + dy^2 <= R^2 — an exact bounded squared-EDT threshold, computed as an OR
// of horizontally dilated rows: row y+dy dilated by w(dy) = floor(sqrt(R^2 - dy^2)).
struct InflTab { int w[64]; };   // w(dy), passed by value: concurrent handles share no device global
// (bytes != nullptr: also /occupancy_grid's bytes with the `frame` border, from the word in registers)
__global__ __launch_bounds__(64 * kRowBlk) void k_inflate(const uint64_t *in, uint64_t *out, int W, int H, int WW, int R,
                                                         InflTab wt, int8_t *bytes, int frame) {
    int c = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * kRowBlk + threadIdx.y;
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
    acc &= pad_mask(c, WW, W);
    out[(size_t)y * WW + c] = acc;
    if (bytes)
        store_word_bytes(bytes + (size_t)y * W + 64 * c, acc | grid_extra(64 * c, y, W, H, frame, ByteRect{-1, 0, 0, 0}),
                         min(64, W - 64 * c), (W & 15) == 0);
}
void launch_inflate(const uint64_t *in, uint64_t *out, const FrameGeom &g, hipStream_t s, int8_t *bytes, int frame) {
    InflTab wt{};
    for (int dy = 0; dy <= g.R && dy < 64; ++dy) {
        int w = 0;
        while ((w + 1) * (w + 1) + dy * dy <= g.R * g.R) ++w;
        wt.w[dy] = w;
    }
    k_inflate<<<row_grid(g.WW, g.H), kRowBlock, 0, s>>>(in, out, g.W, g.H, g.WW, g.R, wt, bytes, frame);
}

// bits -> int8 {0,100} with the optional frame border and rectangle (grid_extra)
__global__ __launch_bounds__(64 * kRowBlk) void k_bits_to_bytes(const uint64_t *bits, int8_t *out, int W, int H, int WW,
                                                               int frame, ByteRect r) {
    const int c = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * kRowBlk + threadIdx.y;
    if (c >= WW || y >= H) return;
    const uint64_t v = bits[(size_t)y * WW + c] | grid_extra(64 * c, y, W, H, frame, r);
    store_word_bytes(out + (size_t)y * W + 64 * c, v, min(64, W - 64 * c), (W & 15) == 0);
}
void launch_bits_to_bytes(const uint64_t *bits, int8_t *out, const FrameGeom &g, int frame, hipStream_t s, const int *rect) {
    if (reinterpret_cast<uintptr_t>(out) & 15) throw std::logic_error("launch_bits_to_bytes: output not 16-byte aligned");
    const ByteRect r = rect ? ByteRect{rect[0], rect[1], rect[2], rect[3]} : ByteRect{-1, 0, 0, 0};
    k_bits_to_bytes<<<row_grid(g.WW, g.H), kRowBlock, 0, s>>>(bits, out, g.W, g.H, g.WW, frame, r);
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
// (zero != nullptr: the thinning flags zero[0, nzero) are cleared by the blocks of row 0: no fill launch)
__global__ __launch_bounds__(64 * kRowBlk) void k_open(const uint64_t *in, uint64_t *out, int W, int H, int WW, int *zero,
                                                      int nzero) {
    int k = blockIdx.x * 64 + threadIdx.x, r = blockIdx.y * kRowBlk + threadIdx.y;
    if (zero && r == 0)
        for (int i = k; i < nzero; i += gridDim.x * 64) zero[i] = 0;
    if (k >= WW || r >= H) return;
    uint64_t e = erode_at(in, r, k, H, WW, W);
    uint64_t d = e | erode_at(in, r - 1, k, H, WW, W) | erode_at(in, r + 1, k, H, WW, W) |
                 (e << 1) | (erode_at(in, r, k - 1, H, WW, W) >> 63) | (e >> 1) | (erode_at(in, r, k + 1, H, WW, W) << 63);
    out[(size_t)r * WW + k] = d & pad_mask(k, WW, W);
}
void launch_open(const uint64_t *in, uint64_t *out, const FrameGeom &g, hipStream_t s, int *zero, int nzero) {
    k_open<<<row_grid(g.WW, g.H), kRowBlock, 0, s>>>(in, out, g.W, g.H, g.WW, zero, nzero);
}

// ------------------------------------------------------------------------------------------
// a7 ximgproc::thinning(THINNING_ZHANGSUEN) with temporal blocking.
// One workgroup owns a TH x TWW-word tile and loads it with a halo of HR = 2*KIT rows and one
// word (64 cells) on each side into LDS, then runs KIT full iterations (2*KIT Jacobi
// sub-iterations) in LDS: each sub-iteration invalidates one more halo row/cell from the outside
// in, so the interior stays exact. Bit-sliced logic evaluates the Zhang-Suen predicate for 64
// cells per 64-bit word:
//   A == 1       : exactly one 0->1 transition in p2,p3,...,p9,p2
//   2 <= B <= 6  : B = p2 + ... + p9 as four bit planes from carry-save adders (3 full adders and a
//                  half adder per word, then two carries): B >= 2 and not (B == 7 or B == 8)
//   m1 == m2 == 0: iter 0: p2p4p6 = p4p6p8 = 0; iter 1: p2p4p8 = p2p6p8 = 0
// Rows 0 / H-1 and columns 0 / W-1 of the image are never examined (ximgproc loops 1..n-2).
#ifndef AOS_THIN_TB
#define AOS_THIN_TB 1024
#endif
#ifndef AOS_THIN_TH
#define AOS_THIN_TH 128
#endif
constexpr int TH = AOS_THIN_TH, TWW = 8, KIT = kThinItersPerLaunch, HR = 2 * KIT, NR = TH + 2 * HR, NC = TWW + 2;
constexpr int kThinTB = AOS_THIN_TB;

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
    uint64_t one = 0, two = 0;          // 0 -> 1 transitions: >= 1, >= 2
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint64_t t = ~seq[k] & seq[k + 1];
        two |= one & t; one |= t;
    }
    auto fa = [](uint64_t a, uint64_t b, uint64_t c, uint64_t &s, uint64_t &cy) {
        const uint64_t x = a ^ b;
        s = x ^ c;
        cy = (a & b) | (c & x);
    };
    uint64_t sa, ca, sb, cb, b0, c4, t2, c5;
    fa(p2, p3, p4, sa, ca);
    fa(p5, p6, p7, sb, cb);
    fa(sa, sb, p8 ^ p9, b0, c4);        // bit 0 of B; carry of weight 2
    fa(ca, cb, p8 & p9, t2, c5);        // weight 2; carry of weight 4
    const uint64_t b1 = c4 ^ t2, c6 = c4 & t2;
    const uint64_t b2 = c5 ^ c6, b3 = c5 & c6;
    uint64_t A1 = one & ~two;
    uint64_t B26 = (b1 | b2 | b3) & ~(b3 | (b2 & b1 & b0));
    uint64_t m = sub == 0 ? (~(p2 & p4 & p6) & ~(p4 & p6 & p8)) : (~(p2 & p4 & p8) & ~(p2 & p6 & p8));
    return c1 & A1 & B26 & m;  // cells to delete
}

__global__ __launch_bounds__(kThinTB) void k_thin_block(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                    int W, int H, int WW, int base_iter, int *flags, ThinOwn own) {
    if (own.early_exit && base_iter >= 2 && flags[1 + base_iter - 1] == 0) return;  // converged in an earlier launch
    __shared__ uint64_t buf[2][NR][NC];
    __shared__ int chg_shared;
    const int ty0 = blockIdx.y * TH, tc0 = blockIdx.x * TWW;
    const int tile = blockIdx.y * gridDim.x + blockIdx.x;
    if (own.act_prev) {
        // No tile interior within one tile of this one deleted anything in the last two sub-iterations
        // of the previous launch: the 3 x 3 tiles are a fixed point of both sub-iterations, and a change
        // outside them travels one cell per sub-iteration, so it cannot reach this tile (>= TH rows /
        // 64 * TWW cells away) within this launch's 2 * KIT <= HR sub-iterations. Copy it through.
        bool quiet_nb = true;
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                const int by = (int)blockIdx.y + dy, bx = (int)blockIdx.x + dx;
                if (by >= 0 && by < (int)gridDim.y && bx >= 0 && bx < (int)gridDim.x && own.act_prev[by * gridDim.x + bx])
                    quiet_nb = false;
            }
        if (quiet_nb) {
            for (int idx = threadIdx.x; idx < TH * TWW; idx += blockDim.x) {
                const int r = idx / TWW, k = idx - r * TWW, gy = ty0 + r, gc = tc0 + k;
                if (gy < H && gc < WW) out[(size_t)gy * WW + gc] = in[(size_t)gy * WW + gc];
            }
            if (threadIdx.x == 0) own.act_next[tile] = 0;
            return;
        }
    }
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
    // Two consecutive sub-iterations (one of each parity) that delete nothing anywhere in the loaded
    // window leave it a fixed point of both: the remaining sub-iterations of this launch would
    // recompute the same window, so the block stops there (its later iterations delete nothing).
    int quiet = 0;
    int late_del = 0;   // this tile's interior deleted something in the launch's last two sub-iterations
    for (int s = 0; s < 2 * KIT; ++s) {
        const int sub = s & 1;
        int any_del = 0;
        // sub-iteration s is exact on rows [s + 1, NR - 1 - s) of the window (one row of the halo goes
        // stale per sub-iteration); rows outside are never read again, so they are not computed. Row 0
        // and NR - 1 (s = 0) are kept as loaded.
        const int r_lo = s == 0 ? 0 : s + 1, r_hi = s == 0 ? NR : NR - 1 - s;
        for (int idx = threadIdx.x + r_lo * NC; idx < r_hi * NC; idx += blockDim.x) {
            int r = idx / NC, k = idx - r * NC;
            const int gy = ty0 - HR + r, gc = tc0 - 1 + k;
            // cells this launch reports: its tile interior, within the caller's own rectangle
            const bool mine = r >= HR && r < HR + TH && k >= 1 && k <= TWW && gy >= own.y0 && gy < own.y1 &&
                              gc >= own.c0 && gc < own.c1;
            uint64_t c1 = buf[cur][r][k];
            uint64_t nw = c1;
            if (c1 && r > 0 && r < NR - 1) {   // (an empty word deletes nothing: whole waves skip)
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
                if (del && s >= 2 * KIT - 2 && r >= HR && r < HR + TH && k >= 1 && k <= TWW) late_del = 1;
                any_del |= del != 0;
            }
            buf[cur ^ 1][r][k] = nw;
            if (s == 1 && base_iter == 0 && nw && mine) nonempty = 1;
        }
        cur ^= 1;
        quiet = __syncthreads_or(any_del) ? 0 : quiet + 1;
        if (quiet >= 2) break;   // (block-uniform)
    }
    for (int idx = threadIdx.x; idx < TH * TWW; idx += blockDim.x) {
        int r = idx / TWW, k = idx - r * TWW;
        int gy = ty0 + r, gc = tc0 + k;
        if (gy < H && gc < WW) out[(size_t)gy * WW + gc] = buf[cur][HR + r][1 + k];
    }
    if (chg || nonempty) atomicOr(&chg_shared, chg | (nonempty << 30));
    const int late_any = __syncthreads_or(late_del);
    if (own.act_next && threadIdx.x == 0) own.act_next[tile] = late_any;
    if (threadIdx.x == 0 && chg_shared) {
        int m = chg_shared;
        if (m & (1 << 30)) atomicOr(&flags[0], 1);
        for (int j = 0; j < KIT; ++j)
            if (m & (1 << j)) atomicOr(&flags[1 + base_iter + j], 1);
    }
}

int thin_tiles(const FrameGeom &g) { return cdiv(g.WW, TWW) * cdiv(g.H, TH); }

__global__ void k_zero_ints(int *p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0;
}
void launch_zero_ints(int *p, int n, hipStream_t s) {
    if (n > 0) k_zero_ints<<<cdiv(n, 256), 256, 0, s>>>(p, n);
}

// The thinning result without a host round trip: the last launch that ran (launch j runs iff j == 0 or
// iteration j*K-1 deleted something) wrote bufs[last & 1]; it is copied into out for the later stages.
// (h_flags != nullptr: block 0 also stores the first nh flags into that pinned host buffer, the frame's
// convergence check: no copy-engine read-back)
__global__ void k_thin_pick(const int *flags, int launched, int K, const uint64_t *b0, const uint64_t *b1, uint64_t *out,
                            size_t n, int *h_flags, int nh) {
    __shared__ int last_s;
    if (h_flags && blockIdx.x == 0)
        for (int i = threadIdx.x; i < nh; i += blockDim.x) h_flags[i] = flags[i];
    if (threadIdx.x == 0) {
        int last = 0;
        for (int j = 1; j < launched; ++j) {
            if (!flags[1 + j * K - 1]) break;
            last = j;
        }
        last_s = last;
    }
    __syncthreads();
    const uint64_t *src = (last_s & 1) ? b1 : b0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) out[i] = src[i];
}
void launch_thin_pick(const int *flags, int launched, const uint64_t *b0, const uint64_t *b1, uint64_t *out, size_t n,
                      hipStream_t s, int *h_flags, int nh) {
    k_thin_pick<<<512, 256, 0, s>>>(flags, launched, KIT, b0, b1, out, n, h_flags, nh);
    AOS_HIP(hipGetLastError());
}

void launch_thin_block(const uint64_t *in, uint64_t *out, const FrameGeom &g, int base_iter, int *flags,
                       const ThinOwn &own, hipStream_t s) {
    static_assert(2 * KIT <= HR && 2 * KIT <= TH && 2 * KIT <= 64 * TWW, "the copy-through rule needs a tile >= 2 KIT cells");
    dim3 grid(cdiv(g.WW, TWW), cdiv(g.H, TH));
    k_thin_block<<<grid, kThinTB, 0, s>>>(in, out, g.W, g.H, g.WW, base_iter, flags, own);
}

}  // namespace aos
