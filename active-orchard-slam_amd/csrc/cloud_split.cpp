// Host gather / split of PointCloud2 records (cloud_split.h).
#include "cloud_split.h"

#include <immintrin.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

namespace aos {

namespace {
std::atomic<int> g_simd{-1};   // -1: not decided yet

bool cpu_avx512() {
#if defined(__x86_64__)
    return __builtin_cpu_supports("avx512f");
#else
    return false;
#endif
}

inline bool std16(const PackLayout &l) { return l.step == 16 && l.ox == 0 && l.oy == 4 && l.oz == 8; }

inline void load_xyz(const uint8_t *rec, const PackLayout &l, float &x, float &y, float &z) {
    std::memcpy(&x, rec + l.ox, 4); std::memcpy(&y, rec + l.oy, 4); std::memcpy(&z, rec + l.oz, 4);
}

// branch-free scalar split of records [i0, m): each point goes to one output (3 stores either way)
uint64_t split_scalar(const uint8_t *src, uint64_t i0, uint64_t m, const PackLayout &l, const float b[6], float *front,
                      uint64_t f, float *rest, uint64_t &nr) {
    for (uint64_t i = i0; i < m; ++i) {
        float x, y, z;
        load_xyz(src + i * (uint64_t)l.step, l, x, y, z);
        const bool in = (x >= b[0]) & (x <= b[1]) & (y >= b[2]) & (y <= b[3]) & (z >= b[4]) & (z <= b[5]);
        float *w = in ? front + 3 * f : rest + 3 * nr;
        w[0] = x; w[1] = y; w[2] = z;
        f += in; nr += !in;
    }
    return f;
}

// An output stream written with nontemporal stores: points are compressed into a 4 KB staging buffer (L1) and
// leave it as whole 64-byte lines (_mm512_stream_ps), so the output's lines are never read for ownership: the
// slots and the rest buffer (120 MB at C2) are only read by the DMA engine or by a later rest copy. The first
// floats up to the destination's 64-byte boundary and the last partial line use plain stores.
// (Box A/B, tools/sdcheck/var/ntp: 8 threads over 10 M points, 1.29-1.30 ms instead of 1.56-1.60 with stores of
// whole registers at the output's end; profiles/r04y_ntp.txt.)
struct NtStream {
    static constexpr int kBuf = 1024;   // floats
    alignas(64) float buf[kBuf + 64];
    float *dst = nullptr;
    int bn = 0;
    bool aligned = false;
    void start(float *d) { dst = d; bn = 0; aligned = false; }
    __attribute__((target("avx512f"))) void flush(bool final) {
        int i = 0;
        if (!aligned) {
            int head = (int)(((64 - ((uintptr_t)dst & 63)) & 63) / 4);
            if (head > bn && !final) return;
            head = head < bn ? head : bn;
            for (; i < head; ++i) dst[i] = buf[i];
            dst += head;
            aligned = true;
        }
        if (final) {
            for (int k = 0; k < bn - i; ++k) dst[k] = buf[i + k];
            dst += bn - i;
            bn = 0;
            return;
        }
        const int full = (bn - i) & ~15;
        for (int k = 0; k < full; k += 16) _mm512_stream_ps(dst + k, _mm512_loadu_ps(buf + i + k));
        dst += full;
        i += full;
        std::memmove(buf, buf + i, sizeof(float) * (size_t)(bn - i));
        bn -= i;
    }
};
// 16-byte records, four per 512-bit register (x y z w | x y z w | ...). One compare pair gives each lane's
// test; a record is inside when its x, y, z lanes pass (w lanes forced). Its x, y, z lanes are compressed
// into the stream of its output.
__attribute__((target("avx512f,popcnt"))) uint64_t split_avx512(const uint8_t *src, uint64_t m, const float b[6],
                                                                float *front, float *rest, uint64_t &nr_out,
                                                                uint64_t &done) {
    const float ninf = -__builtin_inff(), pinf = __builtin_inff();
    const __m512 lo = _mm512_setr_ps(b[0], b[2], b[4], ninf, b[0], b[2], b[4], ninf, b[0], b[2], b[4], ninf, b[0], b[2],
                                     b[4], ninf);
    const __m512 hi = _mm512_setr_ps(b[1], b[3], b[5], pinf, b[1], b[3], b[5], pinf, b[1], b[3], b[5], pinf, b[1], b[3],
                                     b[5], pinf);
    static thread_local NtStream F, R;
    F.start(front);
    R.start(rest);
    const float *p = reinterpret_cast<const float *>(src);
    uint64_t f = 0, nr = 0;
    const uint64_t m4 = m & ~uint64_t(3);
    for (uint64_t i = 0; i < m4; i += 4) {
        const __m512 v = _mm512_loadu_ps(p + 4 * i);
        const unsigned t = (unsigned)(_mm512_cmp_ps_mask(v, lo, _CMP_GE_OQ) & _mm512_cmp_ps_mask(v, hi, _CMP_LE_OQ)) |
                           0x8888u;
        const unsigned r = t & (t >> 1) & (t >> 2) & (t >> 3) & 0x1111u;   // bit 4k: record k inside
        const unsigned k = (unsigned)_mm_popcnt_u32(r);
        _mm512_storeu_ps(F.buf + F.bn, _mm512_maskz_compress_ps((__mmask16)(r * 7u), v));
        _mm512_storeu_ps(R.buf + R.bn, _mm512_maskz_compress_ps((__mmask16)((r ^ 0x1111u) * 7u), v));
        F.bn += 3 * (int)k;
        R.bn += 3 * (int)(4 - k);
        f += k; nr += 4 - k;
        if (F.bn >= NtStream::kBuf) F.flush(false);
        if (R.bn >= NtStream::kBuf) R.flush(false);
    }
    F.flush(true);
    R.flush(true);
    _mm_sfence();   // the streamed lines are visible before the caller hands the slot to the DMA
    nr_out = nr;
    done = m4;
    return f;
}
}  // namespace

bool pack_simd() {
    int s = g_simd.load(std::memory_order_relaxed);
    if (s < 0) {
        const char *e = getenv("AOS_PACK_SIMD");
        s = (e && atoi(e) == 0) ? 0 : (cpu_avx512() ? 1 : 0);
        g_simd.store(s, std::memory_order_relaxed);
    }
    return s == 1;
}

void pack_set_simd(bool on) { g_simd.store(on && cpu_avx512() ? 1 : 0, std::memory_order_relaxed); }

void pack_all(const uint8_t *src, uint64_t m, const PackLayout &l, float *out) {
    if (std16(l)) {   // (the compiler vectorises this form)
        const float *r = reinterpret_cast<const float *>(src);
        for (uint64_t i = 0; i < m; ++i) { out[3 * i] = r[4 * i]; out[3 * i + 1] = r[4 * i + 1]; out[3 * i + 2] = r[4 * i + 2]; }
        return;
    }
    for (uint64_t i = 0; i < m; ++i) load_xyz(src + i * (uint64_t)l.step, l, out[3 * i], out[3 * i + 1], out[3 * i + 2]);
}

uint64_t pack_split(const uint8_t *src, uint64_t m, const PackLayout &l, const float box[6], float *front, float *rest,
                    uint64_t *n_rest) {
    uint64_t f = 0, nr = 0, i = 0;
    if (std16(l) && pack_simd()) f = split_avx512(src, m, box, front, rest, nr, i);
    f = split_scalar(src, i, m, l, box, front, f, rest, nr);
    *n_rest = nr;
    return f;
}

}  // namespace aos
