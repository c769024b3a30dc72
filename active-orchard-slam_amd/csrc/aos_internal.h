// Internal declarations of libaos_gpu.so (MI355X / gfx950). Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "../../include/aos_gpu.h"

namespace aos {

// ------------------------------------------------------------------ errors
void set_error(const std::string &msg);
struct HipError { hipError_t e; const char *what; int line; };
#define AOS_HIP(x)                                                        \
    do {                                                                  \
        hipError_t _e = (x);                                              \
        if (_e != hipSuccess) throw ::aos::HipError{_e, #x, __LINE__};    \
    } while (0)

// Makes a device current for one scope and restores the caller's device afterwards (also on an
// exception), so a multi-GPU caller (e.g. torch with one device per thread) keeps its own device.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);   // a failure surfaces in the next HIP call
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
};

// ------------------------------------------------------------------ device buffers
// AOS_TRACE: growth of a buffer (a free + malloc, which may synchronise the device) is logged on stderr
// with its host time, against the process-wide trace clock (trace_ms)
double trace_ms();
bool trace_on();
// AOS_TRACE=1: a stage's host timeline on stderr (ms since the stage started, at each host sync)
struct HostTrace {
    const char *tag;
    const bool on = trace_on();
    const double t0 = on ? trace_ms() : 0.0;
    std::string line;
    void mark(const char *what) {
        if (!on) return;
        char b[64];
        snprintf(b, sizeof(b), " %s %.3f", what, trace_ms() - t0);
        line += b;
    }
    ~HostTrace() { if (on) fprintf(stderr, "[aos trace %s] at %.2f:%s\n", tag, t0, line.c_str()); }
};
void trace_alloc(const char *kind, size_t bytes, double t0);
// Owning, growable device allocation (freed on destruction; not copyable).
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void *ensure(size_t bytes) {
        if (bytes <= cap) return p;
        const double t0 = trace_on() ? trace_ms() : 0.0;
        if (p) AOS_HIP(hipFree(p));
        p = nullptr;
        size_t c = bytes + bytes / 8 + 256;
        AOS_HIP(hipMalloc(&p, c));
        cap = c;
        if (trace_on()) trace_alloc("device", c, t0);
        return p;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

struct PinnedBuf {
    void *p = nullptr;
    size_t cap = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf &) = delete;
    PinnedBuf &operator=(const PinnedBuf &) = delete;
    ~PinnedBuf() { release(); }
    void *ensure(size_t bytes) {
        if (bytes <= cap) return p;
        const double t0 = trace_on() ? trace_ms() : 0.0;
        if (p) AOS_HIP(hipHostFree(p));
        p = nullptr;
        size_t c = bytes + bytes / 8 + 256;
        AOS_HIP(hipHostMalloc(&p, c, hipHostMallocDefault));
        cap = c;
        if (trace_on()) trace_alloc("pinned", c, t0);
        return p;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
};

// Owning, growable pageable host allocation (64-byte aligned): host data the device reads only now and then
// (the rest of a split cloud: copied only when the polygon grows), kept out of page-locked memory.
struct HostBuf {
    void *p = nullptr;
    size_t cap = 0;
    HostBuf() = default;
    HostBuf(const HostBuf &) = delete;
    HostBuf &operator=(const HostBuf &) = delete;
    ~HostBuf() { release(); }
    void *ensure(size_t bytes) {
        if (bytes <= cap) return p;
        release();
        const size_t c = (bytes + bytes / 8 + 256 + 63) / 64 * 64;
        p = std::aligned_alloc(64, c);
        if (!p) throw std::bad_alloc();
        cap = c;
        return p;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
    void release() { std::free(p); p = nullptr; cap = 0; }
};

typedef std::vector<std::pair<double, double>> Poly;

// Geometry of one seed-gen frame (getActiveBounds + generateOccupancyGrid, seed_gen:581-600, 874-890).
struct FrameGeom {
    float minx, maxx, miny, maxy;      // polygon bbox +- 2.5 m, float
    double origin_x, origin_y;         // (double)minx, (double)miny
    float res;
    int W, H, WW;                      // WW = 64-bit words per row
    int R;                             // inflation cells
};

// ------------------------------------------------------------------ kernels (launchers)
constexpr int kRorCounters = 256;   // spread n_clipped counter slots (k_rt_ror)
struct RorLaunch {
    const uint8_t *cloud; uint64_t n; uint32_t step, ox, oy, oz; int is_dense;
    float bminx, bminy, bminz, bmaxx, bmaxy, bmaxz, inv_cs; int nbx, nby;
    float cminx, cmaxx, cminy, cmaxy, cminz, cmaxz;
    double r2; float r2f, r2df; int need;   // r2df: largest float f with (double)f <= r2
    float r2cmp;   // the keep test as one compare, d2 <= r2cmp (rt_configure: r2df, or the float below r2f)
    double origin_x, origin_y; float res; int W, H;
    // Ownership (tiled frames, tiled.hip): a kept candidate is counted iff its cell, clamped to the
    // grid, lies in [rx0, rx1) x [ry0, ry1); it is rastered (if inside the grid) into the byte window
    // whose cell (wx0, wy0) is element 0, row pitch Wr. Single-GPU frames own the whole grid.
    int rx0, ry0, rx1, ry1, wx0, wy0, Wr;
    // tile walk (ror.hip): TB x TB bins per tile, ntx x nty tiles; the raster window as bits (Hr rows
    // of WWr words, wx0 a multiple of 64); a tile's LDS raster window (win_rows x win_w words, 0: none)
    int TB, TBs, ntx, nty, ntiles, Hr, WWr, win_rows, win_w;   // TB = 1 << TBs
    int staged_cap; int *overflow;   // staged array capacity; | 1 when the scatter exceeds it, | 2 when a tile
                                     // beyond the LDS capacity was found with big_ok = 0 (the frame is redone)
    int big_ok;                      // launch the big-tile kernels (ror.hip); 0 skips their five launches
};
constexpr int kRtMaxTiles = 36000;   // tiles per frame (LDS histogram of the partition passes: 144 KB)
void rt_configure(RorLaunch &L, int Hr, int WWr, double est_binned, int force_tb = 0);
int rt_part_blocks(const RorLaunch &L);   // G: workgroups (= cloud chunks) of the partition passes
// H: rt_h_ints ints, G x ntiles (row per workgroup) + G per-workgroup binned counts. The count pass (two
// launches: count, k_rt_colscan) leaves per-tile prefixes over the workgroups in H, the tile starts in ts
// (ntiles + 1 entries, ts[ntiles] = staged total) and the binned count in *n_own; lb: a look-back of
// rt_colscan_words words whose err word gets bit 4 on a stuck wait.
struct LookBack;
size_t rt_h_ints(const RorLaunch &L, int G);
int rt_colscan_words(const RorLaunch &L, int G);
// clr: buffers the count launch zeroes before the stage's later kernels write them (no fill launches)
struct RtClear { uint64_t *w = nullptr; size_t nw = 0; unsigned long long *c = nullptr; int nc = 0; int *k = nullptr; int nk = 0; };
void launch_rt_count(const RorLaunch &L, int *H, int G, int *ts, unsigned long long *n_own, const LookBack &lb,
                     hipStream_t s, const RtClear &clr = RtClear{});
void launch_rt_scatter(const RorLaunch &L, int *H, const int *tstart, int G, float4 *staged, hipStream_t s);
// kept_tile (nullable): per-tile kept counts; dirty (nullable): a tile is counted iff dirty[t+1] > dirty[t]
// scratch: staged-sized; bigbins: rt_bigbins_ints(L) ints (tiles beyond the LDS capacity are sorted there)
size_t rt_bigbins_ints(const RorLaunch &L);
int rt_lds_tile_cap();   // records a tile may hold for k_rt_ror<false> (LDS); larger tiles take the big-tile kernels
// kept_tile != nullptr (a streaming map's store): kept candidates are marked (w = 2) in staged, which
// is rewritten bin-sorted per tile
void launch_rt_ror(const RorLaunch &L, const int *tstart, float4 *staged, float4 *scratch, int *bigbins,
                   uint64_t *rbits, unsigned long long *counters, int *kept_tile, const int *dirty, hipStream_t s);
// streaming map: merge the map's tile store with a scan's partition; n_clipped from per-tile counts
// (cap: new_st capacity in records; a merge that would exceed it writes nothing past it and sets *overflow)
void launch_rt_merge(const float4 *old_st, const int *old_ts, const float4 *scan_st, const int *scan_ts, float4 *new_st,
                     int *new_ts, int ntiles, int cap, int *overflow, hipStream_t s);
void launch_rt_sum_kept(const int *kept_tile, int ntiles, unsigned long long *counters, hipStream_t s);
// reads n staged records (brings their lines into the Infinity Cache before the scatter writes them)
void launch_rt_touch(const float4 *p, size_t n, hipStream_t s);
// PointCloud2 records (any float32 x/y/z offsets) -> float4 (x, y, z, 0)
void launch_pack_xyz(const uint8_t *cloud, uint64_t n, uint32_t step, uint32_t ox, uint32_t oy, uint32_t oz, float4 *out,
                     hipStream_t s);
// the records with x in [box[0], box[2]] and y in [box[1], box[3]] -> out[*count ...] (atomics order)
void launch_pack_xyz_box(const uint8_t *cloud, uint64_t n, uint32_t step, uint32_t ox, uint32_t oy, uint32_t oz,
                         const float box[4], float4 *out, unsigned long long *count, hipStream_t s);
// (bytes != nullptr: the inflated grid's int8 {0, 100} bytes with a `frame`-cell border in the same launch)
void launch_inflate(const uint64_t *in, uint64_t *out, const FrameGeom &g, hipStream_t s, int8_t *bytes = nullptr,
                    int frame = 0);
// rect (nullable): gx0, gy0, gx1, gy1 of markPolygonBoundaryAsOccupied's rectangle, drawn in the same launch
struct ByteRect { int gx0, gy0, gx1, gy1; };
void launch_bits_to_bytes(const uint64_t *bits, int8_t *out, const FrameGeom &g, int frame, hipStream_t s,
                          const int *rect = nullptr);
// int8 {0,100} grid (C bytes) -> ceil(C / 64) words of bits; a byte that is neither sets *err
void launch_pack_grid(const int8_t *g, size_t C, uint64_t *bits, int *err, hipStream_t s);
// (zero: nzero ints cleared in the same launch, the thinning flags)
void launch_open(const uint64_t *in, uint64_t *out, const FrameGeom &g, hipStream_t s, int *zero = nullptr, int nzero = 0);
// Zhang-Suen temporal block: KIT iterations per launch; flags[0] = non-empty after iteration 1,
// flags[1 + k] = iteration k (0-based) deleted something.
constexpr int kThinItersPerLaunch = 8;
// Cells whose deletions a launch reports in flags (rows [y0, y1), words [c0, c1) of the image it is
// given: a tile's own cells inside its halo window), and whether a launch may skip itself once an
// earlier iteration deleted nothing (single GPU only: a tile must keep pace with its neighbours).
// act_prev / act_next (optional, whole-map frames only): per tile, 1 iff its interior deleted something
// in the last two sub-iterations of the previous / this launch (thin_tiles(g) ints each); a tile whose
// 3 x 3 tile neighbourhood was quiet is a fixed point for the next KIT iterations and is copied.
struct ThinOwn { int y0, y1, c0, c1, early_exit; const int *act_prev = nullptr; int *act_next = nullptr; };
int thin_tiles(const FrameGeom &g);
void launch_thin_block(const uint64_t *in, uint64_t *out, const FrameGeom &g, int base_iter, int *flags,
                       const ThinOwn &own, hipStream_t s);
// the converged thinning buffer (from the device flags) -> out, n words (no host round trip)
// (h_flags: pinned, receives flags[0, nh) in the same launch)
void launch_thin_pick(const int *flags, int launched, const uint64_t *b0, const uint64_t *b1, uint64_t *out, size_t n,
                      hipStream_t s, int *h_flags = nullptr, int nh = 0);
void launch_zero_ints(int *p, int n, hipStream_t s);   // a kernel (no memset node in a captured graph)

// ------------------------------------------------------------------ frame helpers (seedgen.hip)
FrameGeom frame_geom(const Poly &poly, const aos_params &P);
float ror_margin(const aos_params &P);
Poly default_polygon();
int thin_iterations(const int *flags, int iters_run);

// ------------------------------------------------------------------ tiled frames (tiled.hip)
struct CommError { std::string what; };
// aos_debug_faults (test hooks): the tiled rank that reports a stuck ROR look-back (-1: none), and the
// cluster exchange's round-size cap in bytes (0: none)
extern std::atomic<int> g_debug_stuck_rank;
extern std::atomic<uint64_t> g_debug_a2a_round;
// RCCL communicator (rccl_comm.hip; aos_rccl_* in the ABI)
void rccl_unique_id(uint8_t *id);
aos_rccl *rccl_create(const uint8_t *id, int rank, int world, int device, uint64_t buf_bytes);
const aos_comm *rccl_comm(aos_rccl *r);
void rccl_destroy(aos_rccl *r);
constexpr int kMaxTiles = 16;   // per dimension
struct TilePlan {
    int tiles_x, tiles_y, rank, tx, ty;
    int G, gw;                  // halo depth: G rows / gw = G / 64 words
    int hy, hw;                 // halo in use: 0 along an untiled dimension
    int rs[kMaxTiles + 1], cs[kMaxTiles + 1];   // first row / word of each tile row / column
    int y0, y1, c0, c1;         // own rows / words
    int wy0, wy1, wc0, wc1;     // halo window, clamped to the map
    FrameGeom lg;               // the window as an image (W, H, WW; R of the map)
    long long max_border, max_own;   // words per rank: border strips / own tile, max over tiles
    float box[4];               // x/y box of the points this rank needs (xmin, ymin, xmax, ymax)
    uint64_t exchange_bytes;    // per-rank all-gather chunk
};
void free_path_state(void *p);   // path.hip

TilePlan make_tile_plan(const FrameGeom &g, float margin, int tiles_x, int tiles_y, int rank);

// Collectives enqueued on the frame's stream: the frame's kernels and its exchanges are ordered by the stream
// alone, and the host waits only where it reads a result. The library's RCCL communicator provides them
// (rccl_comm.hip); a caller's aos_comm runs through its synchronous callbacks instead. Failures throw CommError.
struct StreamColl {
    void *impl = nullptr;
    void (*all_gather)(void *impl, uint64_t bytes, hipStream_t s) = nullptr;         // as aos_comm.all_gather
    void (*gather)(void *impl, uint64_t bytes, int root, hipStream_t s) = nullptr;   // the root's recv_buf only
    void (*max_dev)(void *impl, int32_t *d, int n, hipStream_t s) = nullptr;         // device int32, in place
    void (*all_to_all)(void *impl, const uint64_t *counts, hipStream_t s) = nullptr; // as aos_comm.all_to_all
    // send_buf[0, bytes) to every rank r with peer[r] != 0 and each such rank's block into recv_buf[r * bytes, ...):
    // an all-gather restricted to a symmetric set of peers (the halo exchange: the tiles next to this one)
    void (*exchange)(void *impl, uint64_t bytes, const uint8_t *peer, hipStream_t s) = nullptr;
};
bool rccl_stream_coll(const aos_comm &cm, StreamColl &out);   // true: cm is the library's RCCL communicator

// A tiled frame's view of its communicator (tiled.hip): the stream-ordered collectives when the communicator
// has them, else the aos_comm callbacks (the stream is drained before each: they are called with it idle).
// Counts the collectives and the bytes this rank sends, and times them: host clock around a callback (a
// collective includes the wait for the slowest rank), HIP events around an enqueued one.
struct FrameComm {
    const aos_comm &c;
    StreamColl sc;
    std::vector<hipEvent_t> &ev;   // a persistent pool (the handle's): begin / end pairs of enqueued collectives
    DevBuf &red;                   // device scratch of max_flags
    int ev_used = 0;
    double ms_gather = 0.0, ms_reduce = 0.0;   // host clock
    int n_gather = 0, n_reduce = 0;
    uint64_t bytes_sent = 0, bytes_recv = 0;
    FrameComm(const aos_comm &cm, std::vector<hipEvent_t> &pool, DevBuf &scratch);
    bool ordered() const { return sc.all_gather != nullptr; }
    bool has_all_to_all() const { return ordered() ? sc.all_to_all != nullptr : c.all_to_all != nullptr; }
    void all_gather(uint64_t bytes, hipStream_t s);
    // recv_buf[r * bytes, ...) = rank r's send_buf[0, bytes) for every r with peer[r] != 0 (peer symmetric over the
    // ranks); other blocks of recv_buf undefined. An all-gather when the communicator has no point-to-point form.
    void neighbour_exchange(uint64_t bytes, const uint8_t *peer, hipStream_t s);
    // rank r's send_buf[0, bytes) -> the root's recv_buf[r * bytes, (r + 1) * bytes); the other ranks' recv_buf is
    // not written when the communicator has a personalised exchange (else it is an all-gather)
    void gather(uint64_t bytes, int root, hipStream_t s);
    void all_to_all(const uint64_t *counts, hipStream_t s);
    void max_host(int32_t *v, int n);                            // host int32, in place (no stream involved)
    void max_flags(const int *d, int32_t *h, int n, hipStream_t s);   // device ints -> their max over ranks in h (waits)
    float ms_enqueued();   // the enqueued collectives' device time so far (waits for the last one)
};

}  // namespace aos
