// Wave-wide reductions on DPP row moves (gfx9 DPP: row_shr:1/2/4/8, then row_bcast:15 and row_bcast:31), the wave's
// result read from lane 63. A step is a VALU move with a row permutation; __shfl_xor is an LDS permute
// (ds_bpermute) whose ~100-cycle latency every round of a reduction waits on (k_cluster_stats, round 6: its
// reductions, six permutes per 32-bit value, set ~2 us of each pass). Call with all 64 lanes active. Not part of
// the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace aos {

// lane i takes lane src(i)'s v per the DPP control; lanes without a source, or in rows left out by RM, keep old
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ int dpp_i32(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ long long dpp_i64(long long old, long long v) {
    const int lo = dpp_i32<CTRL, RM>((int)old, (int)v);
    const int hi = dpp_i32<CTRL, RM>((int)(old >> 32), (int)(v >> 32));
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dpp_f64(double old, double v) {
    return __longlong_as_double(dpp_i64<CTRL, RM>(__double_as_longlong(old), __double_as_longlong(v)));
}

__device__ __forceinline__ int lane63_i32(int v) { return __builtin_amdgcn_readlane(v, 63); }
__device__ __forceinline__ long long lane63_i64(long long v) {
    const int lo = __builtin_amdgcn_readlane((int)v, 63), hi = __builtin_amdgcn_readlane((int)(v >> 32), 63);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane63_f64(double v) { return __longlong_as_double(lane63_i64(__double_as_longlong(v))); }

// The DPP move of a value type: int, long long, double, or a struct with a member-wise dpp<CTRL, RM>(old).
template <int CTRL, int RM> __device__ __forceinline__ int dpp_move(int old, int v) { return dpp_i32<CTRL, RM>(old, v); }
template <int CTRL, int RM> __device__ __forceinline__ long long dpp_move(long long old, long long v) {
    return dpp_i64<CTRL, RM>(old, v);
}
template <int CTRL, int RM> __device__ __forceinline__ double dpp_move(double old, double v) { return dpp_f64<CTRL, RM>(old, v); }
template <int CTRL, int RM, class T> __device__ __forceinline__ T dpp_move(const T &old, const T &v) {
    return v.template dpp<CTRL, RM>(old);
}
__device__ __forceinline__ int lane63(int v) { return lane63_i32(v); }
__device__ __forceinline__ long long lane63(long long v) { return lane63_i64(v); }
__device__ __forceinline__ double lane63(double v) { return lane63_f64(v); }
template <class T> __device__ __forceinline__ T lane63(const T &v) { return v.lane63(); }

struct WAdd { template <class T> __device__ T operator()(T a, T b) const { return a + b; } };
struct WMax { template <class T> __device__ T operator()(T a, T b) const { return a > b ? a : b; } };

// The wave's reduction of v under op (associative and commutative, id its identity), the same value in every lane.
template <class T, class Op>
__device__ __forceinline__ T wave_reduce(T v, T id, Op op) {
    v = op(v, dpp_move<0x111, 0xf>(id, v));   // row_shr:1
    v = op(v, dpp_move<0x112, 0xf>(id, v));   // row_shr:2
    v = op(v, dpp_move<0x114, 0xf>(id, v));   // row_shr:4
    v = op(v, dpp_move<0x118, 0xf>(id, v));   // row_shr:8: lane 15 of each row holds the row's reduction
    v = op(v, dpp_move<0x142, 0xa>(id, v));   // row_bcast:15 into rows 1 and 3
    v = op(v, dpp_move<0x143, 0xc>(id, v));   // row_bcast:31 into rows 2 and 3: lane 63 holds the wave's
    return lane63(v);
}

// The wave's inclusive scan of v under op (lane i: v_0 op ... op v_i), and the exclusive one (lane 0: id).
template <class T, class Op>
__device__ __forceinline__ T wave_scan_incl(T v, T id, Op op) {
    v = op(v, dpp_move<0x111, 0xf>(id, v));   // row_shr:1, 2, 4, 8: inclusive inside each row of 16 lanes
    v = op(v, dpp_move<0x112, 0xf>(id, v));
    v = op(v, dpp_move<0x114, 0xf>(id, v));
    v = op(v, dpp_move<0x118, 0xf>(id, v));
    v = op(v, dpp_move<0x142, 0xa>(id, v));   // row_bcast:15: row 0's total into row 1, row 2's into row 3
    v = op(v, dpp_move<0x143, 0xc>(id, v));   // row_bcast:31: rows 0-1's total into rows 2 and 3
    return v;
}
template <class T, class Op>
__device__ __forceinline__ T wave_scan_excl(T v, T id, Op op) {
    return dpp_move<0x138, 0xf>(id, wave_scan_incl(v, id, op));   // wave_shr:1
}

}  // namespace aos
