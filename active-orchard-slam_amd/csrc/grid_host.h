// The two published OccupancyGrids from their bit-packed device grids, expanded on
// the host. The frame's grids cross PCIe as bits (W*H/8 bytes each instead of W*H): 8x fewer bytes through the
// copy engine's blit kernels, which share the CUs (and the L2's write path to host memory) with the cluster
// stage's kernels, and host threads write the {0, 100} bytes while the cluster stage runs. Host code (no HIP
// calls): the sanitizer build runs it. Not part of the ABI.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>

#include "host_pool.h"

namespace aos {

// Rows [y0, y1) of a W x H grid of {0, 100} bytes (row pitch W) from bits (row pitch WW 64-bit words, bit x of
// row y = cell (x, y)); frame > 0: every cell within `frame` cells of the grid's edge is 100 (seed_gen:708-757).
void expand_grid_rows(const uint64_t *bits, int WW, int W, int H, int frame, int y0, int y1, int8_t *out);
// markPolygonBoundaryAsOccupied's rectangle (seed_gen:772-870): rows gy0, gy1 over [min x, max x] and columns
// gx0, gx1 over [min y, max y] set to 100 (on the device: grid_extra, grid_kernels.hip)
void draw_rect_host(int8_t *grid, int W, int H, int gx0, int gy0, int gx1, int gy1);

// One background job per frame: wait for the bits' D2H (wait()), expand both grids on `threads` host threads,
// draw the skeleton's rectangle. start() returns at once; join() waits and rethrows the job's error.
class GridExpander {
  public:
    struct Job {
        std::function<void()> wait;              // the bits are on the host once this returns
        const uint64_t *occ_bits, *skel_bits;    // inflated grid / frameless skeleton, WW words per row
        int8_t *occ, *skel;                      // W x H bytes each
        int W, H, WW, frame;
        int rect[4];                             // gx0, gy0, gx1, gy1 (rect[0] < 0: none)
        int threads;
    };
    GridExpander() = default;
    GridExpander(const GridExpander &) = delete;
    GridExpander &operator=(const GridExpander &) = delete;
    ~GridExpander();
    void start(const Job &j);
    void join();
    void drain();   // waits for a running job without its error (that job's frame has failed already)
    bool busy() const { return busy_; }

  private:
    void loop();
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    Job job_{};
    bool busy_ = false, have_ = false, quit_ = false;
    std::exception_ptr err_;
    HostPool pool_;
};

}  // namespace aos
