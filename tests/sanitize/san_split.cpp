// ASan / UBSan check of the uploader's host gather (csrc/cloud_split.cpp): pack_split / pack_all on random
// clouds (16-byte and other layouts; points on the box faces, NaN, +-inf) against a plain restatement,
// on the AVX-512 and the scalar path, with outputs allocated exactly (points + kPackSlack) so that any
// write past the slack is a heap overflow.
#include "cloud_split.h"
#include "host_pool.h"

#include <atomic>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using namespace aos;

static int fails = 0;

static void check(uint64_t n, const PackLayout &l, std::mt19937_64 &rng, bool simd) {
    pack_set_simd(simd);
    std::vector<uint8_t> src(n * l.step + 1);
    const float box[6] = {-1.5f, 2.25f, 0.5f, 3.0f, -0.4f, 0.5f};
    std::uniform_real_distribution<float> u(-3.f, 4.f);
    for (uint64_t i = 0; i < n; ++i) {
        float v[3];
        for (int a = 0; a < 3; ++a) {
            const int r = (int)(rng() % 40);
            v[a] = r == 0 ? NAN : r == 1 ? INFINITY : r == 2 ? -INFINITY : r < 6 ? box[2 * a + (r & 1)] : u(rng);
        }
        uint8_t *rec = src.data() + i * l.step;
        for (uint32_t b = 0; b < l.step; ++b) rec[b] = (uint8_t)rng();   // other fields: noise (NaN w too)
        std::memcpy(rec + l.ox, &v[0], 4); std::memcpy(rec + l.oy, &v[1], 4); std::memcpy(rec + l.oz, &v[2], 4);
    }
    std::vector<float> ef, er;
    for (uint64_t i = 0; i < n; ++i) {
        float x, y, z;
        const uint8_t *rec = src.data() + i * l.step;
        std::memcpy(&x, rec + l.ox, 4); std::memcpy(&y, rec + l.oy, 4); std::memcpy(&z, rec + l.oz, 4);
        const bool in = x >= box[0] && x <= box[1] && y >= box[2] && y <= box[3] && z >= box[4] && z <= box[5];
        auto &o = in ? ef : er;
        o.push_back(x); o.push_back(y); o.push_back(z);
    }
    // exact sizes + slack (heap-allocated separately: ASan sees an overflow of either)
    float *front = static_cast<float *>(malloc(4 * ef.size() + kPackSlack));
    float *rest = static_cast<float *>(malloc(4 * er.size() + kPackSlack));
    uint64_t nr = ~0ull;
    const uint64_t nf = pack_split(src.data(), n, l, box, front, rest, &nr);
    auto same = [](const float *a, const std::vector<float> &b) { return b.empty() || !std::memcmp(a, b.data(), 4 * b.size()); };
    const bool ok = nf * 3 == ef.size() && nr * 3 == er.size() && same(front, ef) && same(rest, er);
    float *all = static_cast<float *>(malloc(12 * n + 4));
    pack_all(src.data(), n, l, all);
    bool ok_all = true;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *rec = src.data() + i * l.step;
        ok_all &= !std::memcmp(all + 3 * i, rec + l.ox, 4) && !std::memcmp(all + 3 * i + 1, rec + l.oy, 4) &&
                  !std::memcmp(all + 3 * i + 2, rec + l.oz, 4);
    }
    if (!ok || !ok_all) {
        printf("FAIL n=%llu step=%u simd=%d: front %llu/%zu rest %llu/%zu all %d\n", (unsigned long long)n, l.step,
               (int)pack_simd(), (unsigned long long)nf, ef.size() / 3, (unsigned long long)nr, er.size() / 3, (int)ok_all);
        ++fails;
    }
    free(front); free(rest); free(all);
}

int main() {
    std::mt19937_64 rng(11);
    const PackLayout layouts[] = {{16, 0, 4, 8}, {32, 12, 4, 20}, {12, 0, 4, 8}, {16, 4, 0, 8}};
    int cases = 0;
    for (const PackLayout &l : layouts)
        for (uint64_t n : {0ull, 1ull, 3ull, 4ull, 5ull, 7ull, 8ull, 63ull, 64ull, 1000ull, 4099ull, 100003ull})
            for (bool simd : {true, false}) { check(n, l, rng, simd); ++cases; }
    pack_set_simd(true);
    // the uploader's worker pool (host_pool.h): every index runs exactly once per job, jobs of varying width,
    // a stop and a restart in between
    {
        HostPool pool;
        std::atomic<int> hits[16];
        for (int it = 0; it < 3000; ++it) {
            const int n = 1 + it % 16;
            for (auto &h : hits) h = 0;
            pool.run(n, [&](int i) { hits[i].fetch_add(1); });
            for (int i = 0; i < 16; ++i)
                if (hits[i].load() != (i < n ? 1 : 0)) { printf("FAIL pool job %d (n %d): index %d ran %d times\n", it, n, i, hits[i].load()); ++fails; break; }
            if (it == 1500) pool.stop();
        }
        ++cases;
    }
    printf("san_split: %d cases, %d failed (AVX-512 path %s)\n", cases, fails, pack_simd() ? "on" : "not available");
    return fails ? 1 : 0;
}
