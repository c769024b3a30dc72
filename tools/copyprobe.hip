// D2H copy engine probe: a 16.8 MB (C2 OccupancyGrid) device -> pinned host copy on its own stream, alone and
// beside a short compute kernel on another stream (the cluster stage's k_fg case: the copy's blit kernels
// share the CUs). Run it under different HIP / HSA copy settings (environment) and compare:
//   copy alone, kernel alone, kernel beside the copy (µs, HIP events).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/copyprobe tools/copyprobe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// ~20 µs of streaming work over 4 MB (like k_fg over the skeleton bits + polygon tests)
__global__ void k_peek1(int *h, const int *d) { if (threadIdx.x == 0) *h = *d; }
__global__ void k_copy16(uint4 *h, const uint4 *d, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) h[i] = d[i];
}
__global__ void k_work(const unsigned long long *in, unsigned long long *out, size_t n, int reps) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long v = in[i];
    for (int r = 0; r < reps; ++r) v = v * 6364136223846793005ull + 1442695040888963407ull;
    out[i] = v;
}

extern "C" int copyprobe_main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : 16777216ull;
    const unsigned hflags = argc > 2 ? (unsigned)strtoul(argv[2], 0, 0) : 0u;   // hipHostMalloc flags
    void *d, *h;
    CK(hipMalloc(&d, bytes));
    CK(hipHostMalloc(&h, bytes, hflags));
    CK(hipMemset(d, 1, bytes));
    const size_t nw = 1 << 19;
    unsigned long long *wi, *wo;
    CK(hipMalloc(&wi, 8 * nw)); CK(hipMalloc(&wo, 8 * nw));
    CK(hipMemset(wi, 0, 8 * nw));
    // argv[3] = k: k streams are created between the copy stream and the kernel stream (HIP maps streams onto
    // GPU_MAX_HW_QUEUES hardware queues round-robin: with 4 queues, k = 3 puts both on one queue)
    const int gap = argc > 3 ? atoi(argv[3]) : 0;
    hipStream_t sc, sk, dummy[64];
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    for (int i = 0; i < gap && i < 64; ++i) CK(hipStreamCreateWithFlags(&dummy[i], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    printf("streams between the copy and the kernel stream: %d\n", gap);
    hipEvent_t c0, c1, k0, k1;
    for (hipEvent_t *e : {&c0, &c1, &k0, &k1}) CK(hipEventCreate(e));
    float tc = 0, tk = 0, tkb = 0, tcb = 0;
    const int reps = 10;
    for (int r = 0; r < reps + 2; ++r) {
        float a, b;
        CK(hipEventRecord(c0, sc));
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, sc));
        CK(hipEventRecord(c1, sc));
        CK(hipStreamSynchronize(sc));
        CK(hipEventElapsedTime(&a, c0, c1));
        CK(hipEventRecord(k0, sk));
        k_work<<<nw / 256, 256, 0, sk>>>(wi, wo, nw, 64);
        CK(hipEventRecord(k1, sk));
        CK(hipStreamSynchronize(sk));
        CK(hipEventElapsedTime(&b, k0, k1));
        if (r >= 2) { tc += a / reps; tk += b / reps; }
        // both at once: the copy first, the kernel 50 µs later
        CK(hipEventRecord(c0, sc));
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, sc));
        CK(hipEventRecord(c1, sc));
        CK(hipStreamWaitEvent(sk, c0, 0));
        CK(hipEventRecord(k0, sk));
        k_work<<<nw / 256, 256, 0, sk>>>(wi, wo, nw, 64);
        CK(hipEventRecord(k1, sk));
        CK(hipDeviceSynchronize());
        CK(hipEventElapsedTime(&a, c0, c1));
        CK(hipEventElapsedTime(&b, k0, k1));
        if (r >= 2) { tcb += a / reps; tkb += b / reps; }
    }
    // the product's pattern: the copy stream waits for an event recorded on the kernel stream after a kernel
    float tpc = 0, tpk = 0;
    for (int r = 0; r < reps + 2; ++r) {
        float a, b;
        k_work<<<nw / 256, 256, 0, sk>>>(wi, wo, nw, 64);
        CK(hipEventRecord(k0, sk));
        CK(hipStreamWaitEvent(sc, k0, 0));
        CK(hipEventRecord(c0, sc));
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, sc));
        CK(hipEventRecord(c1, sc));
        k_work<<<nw / 256, 256, 0, sk>>>(wi, wo, nw, 64);
        CK(hipEventRecord(k1, sk));
        CK(hipDeviceSynchronize());
        CK(hipEventElapsedTime(&a, c0, c1));
        CK(hipEventElapsedTime(&b, k0, k1));
        if (r >= 2) { tpc += a / reps; tpk += b / reps; }
    }
    // a 4-byte read-back on another stream while the big copy runs: hipMemcpyAsync vs a kernel storing into
    // the pinned host word (host wall-clock from issue to the end of the stream sync)
    int *hsmall; CK(hipHostMalloc(reinterpret_cast<void **>(&hsmall), 64, 0));
    double t_small = 0, t_peek = 0;
    for (int r = 0; r < reps + 2; ++r) {
        for (int mode = 0; mode < 2; ++mode) {
            CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, sc));
            const auto t0 = std::chrono::steady_clock::now();
            if (mode == 0) CK(hipMemcpyAsync(hsmall, wi, 4, hipMemcpyDeviceToHost, sk));
            else k_peek1<<<1, 64, 0, sk>>>(hsmall, reinterpret_cast<const int *>(wi));
            CK(hipStreamSynchronize(sk));
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            CK(hipDeviceSynchronize());
            if (r >= 2) (mode ? t_peek : t_small) += us / reps;
        }
    }
    // the big copy as a kernel of G workgroups storing into pinned host memory, alone and beside k_work
    for (int G : {8, 16, 32, 64, 256}) {
        float tca = 0, tcb = 0, tkb2 = 0;
        for (int r = 0; r < reps + 2; ++r) {
            float a, b;
            CK(hipEventRecord(c0, sc));
            k_copy16<<<G, 256, 0, sc>>>(static_cast<uint4 *>(h), static_cast<const uint4 *>(d), bytes / 16);
            CK(hipEventRecord(c1, sc));
            CK(hipStreamSynchronize(sc));
            CK(hipEventElapsedTime(&a, c0, c1));
            if (r >= 2) tca += a / reps;
            CK(hipEventRecord(c0, sc));
            k_copy16<<<G, 256, 0, sc>>>(static_cast<uint4 *>(h), static_cast<const uint4 *>(d), bytes / 16);
            CK(hipEventRecord(c1, sc));
            CK(hipStreamWaitEvent(sk, c0, 0));
            CK(hipEventRecord(k0, sk));
            k_work<<<nw / 256, 256, 0, sk>>>(wi, wo, nw, 64);
            CK(hipEventRecord(k1, sk));
            CK(hipDeviceSynchronize());
            CK(hipEventElapsedTime(&a, c0, c1));
            CK(hipEventElapsedTime(&b, k0, k1));
            if (r >= 2) { tcb += a / reps; tkb2 += b / reps; }
        }
        printf("kernel copy G %3d: alone %.1f us (%.1f GB/s); beside k_work: copy %.1f us, k_work %.1f us\n", G, 1e3 * tca,
               bytes / (tca * 1e-3) / 1e9, 1e3 * tcb, 1e3 * tkb2);
    }
    printf("4-byte read-back beside the big copy: hipMemcpyAsync %.1f us, peek kernel %.1f us\n", t_small, t_peek);
    printf("event-chained: copy %.1f us, kernel after the copy's start %.1f us\n", 1e3 * tpc, 1e3 * tpk);
    printf("bytes %zu hostflags 0x%x: copy alone %.1f us (%.1f GB/s), kernel alone %.1f us, both: copy %.1f us, kernel %.1f us\n",
           bytes, hflags, 1e3 * tc, bytes / (tc * 1e-3) / 1e9, 1e3 * tk, 1e3 * tcb, 1e3 * tkb);
    return 0;
}

#ifndef COPYPROBE_LIB
int main(int argc, char **argv) { return copyprobe_main(argc, argv); }
#endif
