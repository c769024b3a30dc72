// ROR-stage microbenchmark (a1-a4 only): the C2 synthetic cloud, the tile walk of ror.hip compiled in,
// each pass timed with HIP events over several frames; prints the raster popcount and kept count so
// variants (-DAOS_RT_VARIANT=..., tile / LDS constants) can be checked against each other.
// Build: tools/rorbench/build.sh   Run: tools/rorbench/rorbench [grid_n] [n_points] [frames] [step: 16 | 12]
// [flush_mb: overwrite this many MB between frames, so the cloud and the staged array start cold as in a
// product frame (MALL 256 MB); 0: warm, the previous frame's lines still cached]
#include "../../active-orchard-slam_amd/csrc/ror.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" {
typedef struct orchard_cfg {
    uint64_t seed;
    uint64_t n_points;
    int32_t grid_n;
    float res;
    int32_t max_rows;
    double row_x_end;
    double outlier_frac;
} orchard_cfg;
int64_t orchard_num_trees(const orchard_cfg *c);
int64_t orchard_tree_centres(const orchard_cfg *c, double *tree_x, double *tree_y, int64_t cap);
void orchard_polygon(const orchard_cfg *c, double *poly_xy);
void orchard_generate_range(const orchard_cfg *c, const double *tree_x, const double *tree_y, int64_t n_trees,
                            uint64_t begin, uint64_t end, uint8_t *out);
}


using namespace aos;

// RORBENCH_PRETOUCH: 1 = memset the staged array, 2 = read it once, before the cloud upload (outside the timed
// stage; RORBENCH_UPLOAD=1: the cloud is re-uploaded each frame also with flush_mb > 0): does the scatter's partial-line writing run faster once the array's lines are in the Infinity Cache?
__global__ void k_touch(const float4 *p, size_t n, float *sink) {
    float a = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a += p[i].x;
    if (a == 1234.5f) *sink = a;
}

int main(int argc, char **argv) {
    const int grid_n = argc > 1 ? atoi(argv[1]) : 4096;
    const uint64_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 10000000ull;
    const int frames = argc > 3 ? atoi(argv[3]) : 10;
    const int pstep = argc > 4 ? atoi(argv[4]) : 16;   // 12: the packed float3 cloud of the host upload
    const int flush_mb = argc > 5 ? atoi(argv[5]) : 0;   // > 0: overwrite this many MB between frames (evicts MALL / L2)
    void *d_flush = nullptr;
    if (flush_mb > 0) AOS_HIP(hipMalloc(&d_flush, (size_t)flush_mb << 20));
    orchard_cfg c{3, n, grid_n, 0.1f, 0, 0.0, 0.01};
    const int64_t nt = orchard_num_trees(&c);
    std::vector<double> tx(nt), ty(nt);
    orchard_tree_centres(&c, tx.data(), ty.data(), nt);
    std::vector<uint8_t> cloud(16 * n);
    orchard_generate_range(&c, tx.data(), ty.data(), nt, 0, n, cloud.data());
    double poly[8];
    orchard_polygon(&c, poly);
    double hminx = poly[0], hmaxx = poly[0], hminy = poly[1], hmaxy = poly[1];
    for (int k = 0; k < 4; ++k) {
        hminx = std::min(hminx, poly[2 * k]); hmaxx = std::max(hmaxx, poly[2 * k]);
        hminy = std::min(hminy, poly[2 * k + 1]); hmaxy = std::max(hmaxy, poly[2 * k + 1]);
    }
    const float minx = (float)(hminx - 2.5), maxx = (float)(hmaxx + 2.5), miny = (float)(hminy - 2.5), maxy = (float)(hmaxy + 2.5);
    const float res = 0.1f;
    const int W = (int)std::ceil(std::max(0.f, maxx - minx) / res), H = (int)std::ceil(std::max(0.f, maxy - miny) / res);
    const int WW = (W + 63) / 64;
    // RORBENCH_STRIPS=K: the cloud grouped into K equal-width x strips of the clip box (stable within a strip), as a
    // host split could hand over the front (the partition's (workgroup, tile) runs become ~K x longer)
    if (const char *ks = getenv("RORBENCH_STRIPS")) {
        const int K = atoi(ks);
        if (K > 1) {
            std::vector<uint8_t> out(cloud.size());
            std::vector<uint64_t> cnt(K + 1, 0);
            auto strip = [&](uint64_t i) {
                float x; std::memcpy(&x, cloud.data() + 16 * i, 4);
                int k = (int)((x - minx) / (maxx - minx) * K);
                return k < 0 ? 0 : (k >= K ? K - 1 : k);
            };
            for (uint64_t i = 0; i < n; ++i) ++cnt[strip(i) + 1];
            for (int k = 0; k < K; ++k) cnt[k + 1] += cnt[k];
            for (uint64_t i = 0; i < n; ++i) std::memcpy(out.data() + 16 * cnt[strip(i)]++, cloud.data() + 16 * i, 16);
            cloud.swap(out);
        }
    }
    if (pstep == 12)
        for (uint64_t i = 0; i < n; ++i) std::memmove(cloud.data() + 12 * i, cloud.data() + 16 * i, 12);
    uint8_t *d_cloud;
    AOS_HIP(hipMalloc(&d_cloud, (size_t)pstep * n));
    AOS_HIP(hipMemcpy(d_cloud, cloud.data(), (size_t)pstep * n, hipMemcpyHostToDevice));
    // flush_mb < 0: the product's state instead — the cloud uploaded again from pinned host memory each frame
    uint8_t *h_pinned = nullptr;
    if (flush_mb < 0 || getenv("RORBENCH_UPLOAD")) {
        AOS_HIP(hipHostMalloc(reinterpret_cast<void **>(&h_pinned), (size_t)pstep * n, 0));
        std::memcpy(h_pinned, cloud.data(), (size_t)pstep * n);
    }

    RorLaunch L{};
    L.cloud = d_cloud; L.n = n; L.step = pstep; L.ox = 0; L.oy = 4; L.oz = 8; L.is_dense = 1;
    L.cminx = minx; L.cmaxx = maxx; L.cminy = miny; L.cmaxy = maxy; L.cminz = -0.4f; L.cmaxz = 0.5f;
    const float m = (float)(0.2 * 1.01) + 1e-4f;
    L.bminx = L.cminx - m; L.bmaxx = L.cmaxx + m; L.bminy = L.cminy - m; L.bmaxy = L.cmaxy + m;
    L.bminz = L.cminz - m; L.bmaxz = L.cmaxz + m;
    // RORBENCH_CS: another bin side (m), e.g. 1.6 for ~66 tiles: the scatter's runs per (workgroup, tile) become
    // line-sized (an experiment on the partition only: such tiles exceed the LDS tile pass, which then skips them)
    float cs_ = getenv("RORBENCH_CS") ? (float)atof(getenv("RORBENCH_CS")) : (float)(0.2 * 1.001);
    const double ext = std::max((double)L.bmaxx - L.bminx, (double)L.bmaxy - L.bminy);
    if (ext / cs_ > 8192.0) cs_ = (float)(ext / 8192.0);
    L.inv_cs = 1.0f / cs_;
    L.nbx = std::max(1, (int)((L.bmaxx - L.bminx) * L.inv_cs) + 1);
    L.nby = std::max(1, (int)((L.bmaxy - L.bminy) * L.inv_cs) + 1);
    L.r2 = 0.2 * 0.2; L.r2f = (float)L.r2; L.r2df = (float)L.r2;
    if ((double)L.r2df > L.r2) L.r2df = std::nextafter(L.r2df, 0.0f);
    L.need = 3;
    L.origin_x = minx; L.origin_y = miny; L.res = res; L.W = W; L.H = H;
    L.rx0 = 0; L.ry0 = 0; L.rx1 = W; L.ry1 = H; L.wx0 = 0; L.wy0 = 0; L.Wr = W;
    double est = 0.5 * (double)n;
    hipStream_t s;
    AOS_HIP(hipStreamCreate(&s));
    hipEvent_t e[7];
    for (auto &x : e) AOS_HIP(hipEventCreate(&x));
    int *d_H = nullptr, *d_tot = nullptr; float4 *d_staged = nullptr, *d_scr = nullptr;
    unsigned long long *d_lb = nullptr; size_t cap_lb = 0;
    const int pretouch = getenv("RORBENCH_PRETOUCH") ? atoi(getenv("RORBENCH_PRETOUCH")) : 0;
    unsigned long long *d_cnt; uint64_t *d_bits; int *d_big = nullptr; size_t cap_big = 0;
    AOS_HIP(hipMalloc(&d_cnt, 8 * (kRorCounters + 2)));
    AOS_HIP(hipMalloc(&d_bits, 8ull * WW * H));
    size_t cap_H = 0, cap_staged = 0, cap_t = 0;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int f = 0; f < frames + 2; ++f) {
        rt_configure(L, H, WW, est);
        const int G = rt_part_blocks(L);
        const int nt = L.ntiles;
        const size_t nH = (size_t)nt * G;
        if (rt_h_ints(L, G) > cap_H) { if (d_H) AOS_HIP(hipFree(d_H)); cap_H = rt_h_ints(L, G); AOS_HIP(hipMalloc(&d_H, 4 * cap_H)); }
        if ((size_t)nt + 1 > cap_t) { if (d_tot) AOS_HIP(hipFree(d_tot)); AOS_HIP(hipMalloc(&d_tot, 4 * (nt + 1))); cap_t = nt + 1; }
        int *d_ts = d_tot;
        const size_t words = rt_colscan_words(L, G);
        if (words > cap_lb) {   // look-back words (epoch-tagged: zeroed once), ticket
            if (d_lb) AOS_HIP(hipFree(d_lb));
            AOS_HIP(hipMalloc(&d_lb, 8 * words + 64)); AOS_HIP(hipMemset(d_lb, 0, 8 * words + 64)); cap_lb = words;
        }
        const LookBack lb{d_lb, reinterpret_cast<unsigned *>(d_lb + cap_lb), (unsigned)(f + 1),
                          reinterpret_cast<int *>(d_cnt + kRorCounters + 1)};
        AOS_HIP(hipMemsetAsync(d_cnt, 0, 8 * (kRorCounters + 2), s));
        AOS_HIP(hipMemsetAsync(d_bits, 0, 8ull * WW * H, s));
        if (d_flush) AOS_HIP(hipMemsetAsync(d_flush, f & 0xff, (size_t)flush_mb << 20, s));
        if (pretouch && d_staged) {   // outside the timed stage: in the product it would overlap the upload
            if (pretouch == 1) AOS_HIP(hipMemsetAsync(d_staged, 0, 16ull * cap_staged, s));
            else k_touch<<<2048, 256, 0, s>>>(d_staged, cap_staged, reinterpret_cast<float *>(d_bits));
        }
        if (h_pinned) AOS_HIP(hipMemcpyAsync(d_cloud, h_pinned, (size_t)pstep * n, hipMemcpyHostToDevice, s));
        AOS_HIP(hipEventRecord(e[0], s));
        AOS_HIP(hipEventRecord(e[2], s));
        {   // launch_rt_count with an event between its two launches (count kernel, k_rt_colscan)
            unsigned *own = reinterpret_cast<unsigned *>(d_H + nH);
            if (pstep == 12) rt_part<false, 2>(L, d_H, nullptr, G, nullptr, own, s);
            else rt_part<false, 1>(L, d_H, nullptr, G, nullptr, own, s);
            AOS_HIP(hipEventRecord(e[6], s));
            ColScan C{d_H, d_ts, own, d_cnt + kRorCounters, nt, G, (G + kColRows - 1) / kColRows, (nt + kColTB - 1) / kColTB, lb};
            k_rt_colscan<<<C.ng * C.ntb, kColTB, 0, s>>>(C);
            AOS_HIP(hipEventRecord(e[1], s));
        }
        int total = 0;
        unsigned long long own = 0;
        AOS_HIP(hipMemcpyAsync(&total, d_ts + nt, 4, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipMemcpyAsync(&own, d_cnt + kRorCounters, 8, hipMemcpyDeviceToHost, s));
        AOS_HIP(hipStreamSynchronize(s));
        est = (double)own;
        if ((size_t)total > cap_staged) {
            if (d_staged) { AOS_HIP(hipFree(d_staged)); AOS_HIP(hipFree(d_scr)); }
            AOS_HIP(hipMalloc(&d_staged, 16ull * total)); AOS_HIP(hipMalloc(&d_scr, 16ull * total)); cap_staged = total;
        }
        L.staged_cap = (int)cap_staged;
        L.overflow = reinterpret_cast<int *>(d_cnt + kRorCounters + 1);
        AOS_HIP(hipEventRecord(e[3], s));
        launch_rt_scatter(L, d_H, d_ts, G, d_staged, s);
        AOS_HIP(hipEventRecord(e[4], s));
        if (rt_bigbins_ints(L) > cap_big) { if (d_big) AOS_HIP(hipFree(d_big)); cap_big = rt_bigbins_ints(L); AOS_HIP(hipMalloc(&d_big, 4 * cap_big)); }
        launch_rt_ror(L, d_ts, d_staged, d_scr, d_big, d_bits, d_cnt, nullptr, nullptr, s);
        AOS_HIP(hipEventRecord(e[5], s));
        AOS_HIP(hipStreamSynchronize(s));
        float t[6];
        AOS_HIP(hipEventElapsedTime(&t[0], e[2], e[1]));
        AOS_HIP(hipEventElapsedTime(&t[1], e[0], e[2]));
        AOS_HIP(hipEventElapsedTime(&t[2], e[3], e[4]));
        AOS_HIP(hipEventElapsedTime(&t[3], e[4], e[5]));
        AOS_HIP(hipEventElapsedTime(&t[4], e[0], e[5]));
        AOS_HIP(hipEventElapsedTime(&t[5], e[2], e[6]));
        if (f >= 2) for (int k = 0; k < 6; ++k) acc[k] += t[k] / frames;
        if (f == frames + 1) {
            std::vector<uint64_t> bits((size_t)WW * H);
            std::vector<unsigned long long> cnt(kRorCounters);
            AOS_HIP(hipMemcpy(bits.data(), d_bits, 8 * bits.size(), hipMemcpyDeviceToHost));
            AOS_HIP(hipMemcpy(cnt.data(), d_cnt, 8 * kRorCounters, hipMemcpyDeviceToHost));
            unsigned long long pc = 0, kept = 0, hsh = 1469598103934665603ull;
            for (uint64_t w : bits) { pc += __builtin_popcountll(w); hsh = (hsh ^ w) * 1099511628211ull; }
            for (auto v : cnt) kept += v;
            unsigned long long err = 0;
            AOS_HIP(hipMemcpy(&err, d_cnt + kRorCounters + 1, 8, hipMemcpyDeviceToHost));
            printf("grid %dx%d n %llu TB %d tiles %d G %d staged %d binned %llu | raster cells %llu kept %llu hash %016llx err %llu\n", W, H,
                   (unsigned long long)n, L.TB, L.ntiles, G, total, own, pc, kept, hsh, err);
        }
    }
    const double b = 12.0 * n + (double)W * H;
    printf("(count kernel %.1f us, column scan %.1f us)\n", 1e3 * acc[5], 1e3 * (acc[0] - acc[5]));
    printf("count %.1f us  pretouch %.1f us  scatter %.1f us  tiles %.1f us  | stage %.1f us (incl. read-back gap)  "
           "§8d bytes %.0f MB -> %.3f TB/s = %.3f of 8 TB/s; count pass 12N: %.3f of peak\n",
           1e3 * acc[0], 1e3 * acc[1], 1e3 * acc[2], 1e3 * acc[3], 1e3 * acc[4], b / 1e6, b / (acc[4] * 1e-3) / 1e12,
           b / (acc[4] * 1e-3) / 8e12, 12.0 * n / (acc[0] * 1e-3) / 8e12);
    return 0;
}
