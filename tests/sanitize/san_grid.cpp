// The host expansion of the published OccupancyGrids (csrc/grid_host.cpp) vs a plain per-cell restatement of
// the device kernels k_bits_to_bytes (frame) and k_draw_rect (grid_kernels.hip), on random bit grids whose
// widths are and are not multiples of 64, through the background GridExpander (threads, a no-op wait) and
// row by row. Built with ASan + UBSan (and TSan: san_grid_tsan).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <stdexcept>
#include <algorithm>
#include <vector>

#include "grid_host.h"

using namespace aos;

static void ref_expand(const std::vector<uint64_t> &bits, int WW, int W, int H, int frame, std::vector<int8_t> &out) {
    out.assign((size_t)W * H, 0);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            bool v = (bits[(size_t)y * WW + (x >> 6)] >> (x & 63)) & 1ull;
            if (frame > 0 && (x < frame || y < frame || x >= W - frame || y >= H - frame)) v = true;
            out[(size_t)y * W + x] = v ? 100 : 0;
        }
}

int main() {
    std::mt19937_64 rng(7);
    int failed = 0, cases = 0;
    const int dims[][2] = {{64, 1}, {1, 1}, {3, 9}, {70, 11}, {128, 64}, {1546, 296}, {513, 130}, {4, 700}};
    GridExpander ex;
    for (const auto &d : dims) {
        const int W = d[0], H = d[1], WW = (W + 63) / 64;
        for (int dens = 0; dens < 3; ++dens) {
            std::vector<uint64_t> a((size_t)WW * H), b((size_t)WW * H);
            for (size_t i = 0; i < a.size(); ++i) {
                a[i] = dens == 0 ? 0 : dens == 1 ? (rng() & rng() & rng()) : rng();
                b[i] = rng() & rng();
                const int k = (int)(i % WW);   // pad bits beyond W set: they must not show
                if (64 * (k + 1) > W) {
                    const uint64_t m = ~0ull << (W - 64 * k);
                    a[i] |= m;
                    b[i] |= m;
                }
            }
            std::vector<int8_t> ro, rs, occ((size_t)W * H, 7), sk((size_t)W * H, 7);
            ref_expand(a, WW, W, H, 5, ro);
            ref_expand(b, WW, W, H, 0, rs);
            const int gx0 = std::min(2, W - 1), gy0 = std::min(1, H - 1), gx1 = W - 1, gy1 = H - 1;
            for (int x = std::min(gx0, gx1); x <= std::max(gx0, gx1); ++x) rs[(size_t)gy0 * W + x] = rs[(size_t)gy1 * W + x] = 100;
            for (int y = std::min(gy0, gy1); y <= std::max(gy0, gy1); ++y) rs[(size_t)y * W + gx0] = rs[(size_t)y * W + gx1] = 100;
            GridExpander::Job j{};
            j.wait = [] {};
            j.occ_bits = a.data(); j.skel_bits = b.data(); j.occ = occ.data(); j.skel = sk.data();
            j.W = W; j.H = H; j.WW = WW; j.frame = 5;
            j.rect[0] = gx0; j.rect[1] = gy0; j.rect[2] = gx1; j.rect[3] = gy1;
            j.threads = 1 + (int)(rng() % 8);
            ex.start(j);
            ex.join();
            ++cases;
            if (occ != ro || sk != rs) { ++failed; printf("mismatch W %d H %d dens %d\n", W, H, dens); }
            // row by row on the calling thread
            std::vector<int8_t> o2((size_t)W * H, 7);
            for (int y = 0; y < H; ++y) expand_grid_rows(a.data(), WW, W, H, 5, y, y + 1, o2.data());
            ++cases;
            if (o2 != ro) { ++failed; printf("row mismatch W %d H %d\n", W, H); }
        }
    }
    // a failing wait is reported by join() and does not poison the next job
    GridExpander::Job bad{};
    bad.wait = [] { throw std::runtime_error("copy failed"); };
    bad.W = 1; bad.H = 1; bad.WW = 1; bad.threads = 1; bad.rect[0] = -1;
    ex.start(bad);
    bool thrown = false;
    try { ex.join(); } catch (const std::runtime_error &) { thrown = true; }
    ++cases;
    if (!thrown) { ++failed; printf("error not reported\n"); }
    printf("grid expansion: %d cases, %d failed\n", cases, failed);
    return failed ? 1 : 0;
}
