// Host gather of PointCloud2 records into packed float x, y, z (12 B per point): the uploader's inner loop
// (seedgen.hip upload_pack). Plain C++ (no device code); tests/sanitize/san_split.cpp checks it.
#pragma once
#include <cstddef>
#include <cstdint>

namespace aos {

struct PackLayout { uint32_t step, ox, oy, oz; };   // point_step; byte offsets of float32 x, y, z

// Both outputs of pack_split may need this many writable bytes past their last point (kept for output paths
// that store whole 64-byte registers; the AVX-512 path now writes exactly its points).
constexpr size_t kPackSlack = 64;

// All m records -> out (12 m bytes).
void pack_all(const uint8_t *src, uint64_t m, const PackLayout &l, float *out);

// Records inside box = {bminx, bmaxx, bminy, bmaxy, bminz, bmaxz} (inclusive float compares, as ror.hip's
// rt_binned: NaN never compares inside, +-inf never inside a finite box) -> front, the others -> rest, each
// in record order. Returns the front count; *n_rest = the rest count.
uint64_t pack_split(const uint8_t *src, uint64_t m, const PackLayout &l, const float box[6], float *front, float *rest,
                    uint64_t *n_rest);

// AVX-512 path for the common 16-byte layout (x, y, z at 0, 4, 8): on where the CPU has AVX-512F and
// AOS_PACK_SIMD is not 0. pack_set_simd: tests compare both paths.
bool pack_simd();
void pack_set_simd(bool on);

}  // namespace aos
