// Host expansion of the published OccupancyGrids from their bit-packed device grids (grid_host.h).
#include "grid_host.h"

#include <algorithm>
#include <cstring>

namespace aos {

namespace {
// LUT[b]: the 8 bytes of cells 8k .. 8k + 7 for the bit byte b (little endian: cell 8k is the low byte)
struct ByteLut {
    uint64_t v[256];
    ByteLut() {
        for (int b = 0; b < 256; ++b) {
            uint64_t w = 0;
            for (int k = 0; k < 8; ++k)
                if ((b >> k) & 1) w |= 100ull << (8 * k);
            v[b] = w;
        }
    }
};
const ByteLut &lut() {
    static const ByteLut L;
    return L;
}
}  // namespace

void expand_grid_rows(const uint64_t *bits, int WW, int W, int H, int frame, int y0, int y1, int8_t *out) {
    const uint64_t *L = lut().v;
    const int full = W / 64;   // words whose 64 cells are all inside the row
    for (int y = y0; y < y1; ++y) {
        int8_t *o = out + (size_t)y * W;
        if (frame > 0 && (y < frame || y >= H - frame)) {
            std::memset(o, 100, (size_t)W);
            continue;
        }
        const uint64_t *b = bits + (size_t)y * WW;
        for (int k = 0; k < full; ++k) {
            const uint64_t w = b[k];
            uint64_t q[8];
            for (int j = 0; j < 8; ++j) q[j] = L[(w >> (8 * j)) & 255];
            std::memcpy(o + 64 * k, q, 64);
        }
        if (full * 64 < W) {   // the row's last, partial word
            const uint64_t w = b[full];
            for (int x = 64 * full; x < W; ++x) o[x] = ((w >> (x & 63)) & 1) ? 100 : 0;
        }
        if (frame > 0) {
            const int f = std::min(frame, W);
            std::memset(o, 100, (size_t)f);
            std::memset(o + (W - f), 100, (size_t)f);
        }
    }
}

void draw_rect_host(int8_t *grid, int W, int H, int gx0, int gy0, int gx1, int gy1) {
    (void)H;
    const int xlo = std::min(gx0, gx1), xhi = std::max(gx0, gx1), ylo = std::min(gy0, gy1), yhi = std::max(gy0, gy1);
    for (int x = xlo; x <= xhi; ++x) {
        grid[(size_t)gy0 * W + x] = 100;
        grid[(size_t)gy1 * W + x] = 100;
    }
    for (int y = ylo; y <= yhi; ++y) {
        grid[(size_t)y * W + gx0] = 100;
        grid[(size_t)y * W + gx1] = 100;
    }
}

GridExpander::~GridExpander() {
    if (th_.joinable()) {
        {
            std::lock_guard<std::mutex> l(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
}

void GridExpander::start(const Job &j) {
    {   // a job left running by a failed frame: wait for it, its error belongs to that frame
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [&] { return !busy_; });
        err_ = nullptr;
    }
    if (!th_.joinable()) th_ = std::thread([this] { loop(); });
    {
        std::lock_guard<std::mutex> l(mu_);
        job_ = j;
        have_ = true;
        busy_ = true;
        err_ = nullptr;
    }
    cv_.notify_all();
}

void GridExpander::drain() {
    std::unique_lock<std::mutex> l(mu_);
    done_.wait(l, [&] { return !busy_; });
    err_ = nullptr;
}

void GridExpander::join() {
    std::unique_lock<std::mutex> l(mu_);
    done_.wait(l, [&] { return !busy_; });
    if (err_) {
        std::exception_ptr e = err_;
        err_ = nullptr;
        std::rethrow_exception(e);
    }
}

void GridExpander::loop() {
    for (;;) {
        Job j;
        {
            std::unique_lock<std::mutex> l(mu_);
            cv_.wait(l, [&] { return quit_ || have_; });
            if (quit_) return;
            have_ = false;
            j = job_;
        }
        std::exception_ptr e;
        try {
            j.wait();
            const int n = std::max(1, std::min(j.threads, 32));
            // rows in blocks of 64 (whole cache lines of the output per thread) spread over the threads
            const int blocks = (j.H + 63) / 64;
            pool_.run(n, [&](int t) {
                for (int blk = t; blk < blocks; blk += n) {
                    const int y0 = 64 * blk, y1 = std::min(j.H, y0 + 64);
                    expand_grid_rows(j.occ_bits, j.WW, j.W, j.H, j.frame, y0, y1, j.occ);
                    expand_grid_rows(j.skel_bits, j.WW, j.W, j.H, 0, y0, y1, j.skel);
                }
            });
            if (j.rect[0] >= 0) draw_rect_host(j.skel, j.W, j.H, j.rect[0], j.rect[1], j.rect[2], j.rect[3]);
        } catch (...) {
            e = std::current_exception();
        }
        {
            std::lock_guard<std::mutex> l(mu_);
            err_ = e;
            busy_ = false;
        }
        done_.notify_all();
    }
}

}  // namespace aos
