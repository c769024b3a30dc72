// Streaming-read microbenchmark for the ROR count pass's access pattern: a packed 12-B point array (120 MB at
// 10 M points) read once per launch, cold (512 MB overwritten between launches) or warm. Each workgroup reads
// one contiguous chunk like k_rt_part. Variants: per-lane float3 (dwordx3) records, per-lane float4 (dwordx4)
// over the same bytes, workgroup counts and sizes, nontemporal loads.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/rorbench/loadbench tools/rorbench/loadbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// K: 0 = float3 per lane, 1 = float4 per lane, 2 = float4 nontemporal
// A: 0 = no counter, 1 = every wave adds its count to ONE global counter at the end (k_rt_part's n_own), 2 = one add
// per workgroup (LDS reduction first)
template <int K, int TB, int PER, int A = 0>
__global__ __launch_bounds__(TB) void k_read(const uint8_t *base, unsigned long long bytes, unsigned long long chunk,
                                             float *sink, unsigned long long *ctr) {
    const unsigned long long b0 = (unsigned long long)blockIdx.x * chunk;
    if (b0 >= bytes) return;
    const unsigned long long b1 = b0 + chunk < bytes ? b0 + chunk : bytes;
    constexpr int REC = K == 0 ? 12 : 16;
    const unsigned cnt = (unsigned)((b1 - b0) / REC);
    const uint8_t *cb = base + b0;
    float acc = 0.f;
    constexpr unsigned SUB = TB * PER;
    for (unsigned s = 0; s < cnt; s += SUB) {
        float v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            unsigned i = s + j * TB + threadIdx.x;
            i = i < cnt ? i : cnt - 1;
            if (K == 0) {
                const float3 p = *reinterpret_cast<const float3 *>(cb + (size_t)i * 12);
                v[j] = p.x + p.y + p.z;
            } else if (K == 1) {
                const float4 p = *reinterpret_cast<const float4 *>(cb + (size_t)i * 16);
                v[j] = p.x + p.y + p.z + p.w;
            } else {
                typedef float v4f __attribute__((ext_vector_type(4)));
                const v4f p = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(cb + (size_t)i * 16));
                v[j] = p.x + p.y + p.z + p.w;
            }
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) acc += v[j] > 1e30f ? 1.f : 0.f;
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
    unsigned own = (unsigned)cnt / TB + (acc != 0.f);
    for (int o = 32; o > 0; o >>= 1) own += __shfl_xor(own, o);
    if (A == 1 && (threadIdx.x & 63) == 0) atomicAdd(ctr, (unsigned long long)own);
    if (A == 2) {
        __shared__ unsigned red[TB / 64];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = own;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long t = 0;
            for (int w = 0; w < TB / 64; ++w) t += red[w];
            atomicAdd(ctr, t);
        }
    }
}

template <int K, int TB, int PER, int A = 0>
static void run(const char *name, const uint8_t *d, unsigned long long bytes, int G, float *sink, void *flush,
                size_t flush_bytes, hipStream_t s) {
    const int rec = K == 0 ? 12 : 16;
    unsigned long long chunk = (bytes + G - 1) / G;
    chunk = (chunk + rec * 256 - 1) / (rec * 256) * (rec * 256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int cold = 0; cold < 2; ++cold) {
        float tot = 0.f;
        const int reps = 10;
        for (int r = 0; r < reps + 2; ++r) {
            if (cold) CK(hipMemsetAsync(flush, r & 0xff, flush_bytes, s));
            CK(hipEventRecord(a, s));
            k_read<K, TB, PER, A><<<G, TB, 0, s>>>(d, bytes, chunk, sink, reinterpret_cast<unsigned long long *>(sink + 512));
            CK(hipEventRecord(b, s));
            CK(hipStreamSynchronize(s));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            if (r >= 2) tot += t / reps;
        }
        printf("%-14s A%d G %5d TB %4d PER %2d %s: %7.1f us  %.2f TB/s\n", name, A, G, TB, PER, cold ? "cold" : "warm",
               1e3 * tot, bytes / (tot * 1e-3) / 1e12);
    }
}

int main(int argc, char **argv) {
    const unsigned long long n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ull;
    const unsigned long long bytes = 12ull * n;
    uint8_t *d; float *sink; void *flush;
    const size_t fb = 512ull << 20;
    CK(hipMalloc(&d, bytes + 4096)); CK(hipMalloc(&sink, 4096)); CK(hipMalloc(&flush, fb));
    CK(hipMemset(d, 0, bytes + 4096));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    run<0, 256, 8>("float3", d, bytes, 512, sink, flush, fb, s);
    run<0, 256, 8, 1>("float3", d, bytes, 512, sink, flush, fb, s);
    run<0, 256, 8, 2>("float3", d, bytes, 512, sink, flush, fb, s);
    run<0, 256, 8, 1>("float3", d, bytes, 1024, sink, flush, fb, s);
    run<0, 256, 8, 2>("float3", d, bytes, 1024, sink, flush, fb, s);
    run<1, 256, 6>("float4", d, bytes, 1024, sink, flush, fb, s);
    run<2, 256, 6>("float4 nt", d, bytes, 1024, sink, flush, fb, s);
    run<2, 256, 6, 1>("float4 nt", d, bytes, 1024, sink, flush, fb, s);
    return 0;
}
