// Primitives shared by the cluster, seed and GVD stages (greedy.hip defines the kernels; the device-side
// helpers are in dev_prims_device.h, this header is host-compilable):
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
#include <initializer_list>

#include "aos_internal.h"

namespace aos {

// ------------------------------------------------------------------ uniform hash over the plane
struct HashG { double x0, y0, inv; int nx, ny; };
// cells of side >= cell over [minx, maxx] x [miny, maxy]; points outside are clamped into the border cells
HashG make_hash(double minx, double maxx, double miny, double maxy, double cell);
// the same with the cell enlarged (never shrunk) until nx * ny <= max(4096, cells_per_item * n): a bucket
// table a counting sort can scan. Coarser cells only add candidates that the exact tests then reject.
HashG make_hash_n(double minx, double maxx, double miny, double maxy, double cell, long long n, double cells_per_item = 2.0);

// Items of the hash's buckets: bucket b = cy * nx + cx holds items[start[b] .. start[b + 1]).
struct CellIdx {
    HashG h;
    const int *start, *items;
};
// ------------------------------------------------------------------ look-back
constexpr unsigned kSpinCap = 1u << 21;   // a wait that outlasts this sets the error word (never expected)
struct LookBack {
    unsigned long long *part;   // per block: (tag << 32) | value, tag = epoch << 2 | flag (1 aggregate, 2 prefix)
    unsigned *ticket;           // dynamic block ids; the block that draws the last id resets it to 0
    unsigned epoch;             // of this launch (>= 1; words of other launches read as "not yet")
    int *err;                   // | 1 on a stale ticket or a wait past kSpinCap
};

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

// ------------------------------------------------------------------ read-backs without the copy engine
// Small read-backs in the middle of a frame (counts, error words, cluster records, seeds) are stored into
// pinned host memory by a kernel instead of hipMemcpyAsync: a D2H copy is queued on the DMA engine behind the
// frame's 2 x 16.8 MB OccupancyGrid copies (~0.3 ms each at C2), which delayed every host wait of the
// cluster / seed stage until they had finished. h_dst: pinned host memory (PinnedBuf); the values are the
// host's once the stream has been synchronised. AOS_ZC_READBACK=0: hipMemcpyAsync instead (A/B).
constexpr int kPeekMax = 8;
void peek_to_host(int *h_dst, std::initializer_list<const int *> srcs, hipStream_t s);
void copy_to_host(void *h_dst, const void *d_src, size_t bytes, hipStream_t s);
void copy_from_host(void *d_dst, const void *h_src, size_t bytes, hipStream_t s);   // h_src pinned
// A bulk copy by a kernel of at most `blocks` workgroups (one side may be pinned host memory): the published
// grids' D2H (finish_frame), where hipMemcpyAsync now and then held the host for ~3-7 ms (AOS_TRACE)
void copy_kernel_bulk(void *dst, const void *src, size_t bytes, int blocks, hipStream_t s);

}  // namespace aos
