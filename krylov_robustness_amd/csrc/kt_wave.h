// kt_wave.h -- exact lane ^ o exchanges inside a wave64 without the LDS
// crossbar.  __shfl_xor compiles to ds_bpermute_b32 (one LDS round trip per
// 32-bit half and step, issued through the LDS pipe the kernels' gathers and
// reductions also use); here o = 1, 2 are DPP quad_perm, o = 4 two DPP row
// shifts merged by bank masks (banks 0 and 2 take lane i + 4, banks 1 and 3
// lane i - 4), o = 8 DPP row_ror:8, o = 16 / 32 gfx950's
// v_permlane16/32_swap_b32 (the swap hands every lane its partner's value in
// one of its two results).  Same partner as __shfl_xor(v, o, 64) in every
// lane, so every butterfly keeps its pairs and its sums bit for bit
// (tools/wave_dpp_check.hip checks all o on random bits).
// Call in wave-uniform control flow only: the moves read the other lanes'
// registers whatever their exec bit.
#pragma once
#include <hip/hip_runtime.h>

namespace kt {

#ifndef KT_SHFL_DPP
#define KT_SHFL_DPP 1
#endif

__device__ __forceinline__ unsigned xor_lane_u32(unsigned v, int o) {
    switch (o) {
        case 1:
            return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        case 2:
            return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
        case 4: {
            const int t = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x104, 0xF, 0x5, false);  // row_shl:4, banks 0, 2
            return (unsigned)__builtin_amdgcn_update_dpp(t, (int)v, 0x114, 0xF, 0xA, false);     // row_shr:4, banks 1, 3
        }
        case 8:
            return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
        case 16: {
            const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return (__lane_id() & 16) ? r[0] : r[1];
        }
        default: {  // 32
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return (__lane_id() & 32) ? r[0] : r[1];
        }
    }
}

__device__ __forceinline__ double shfl_xor_d(double v, int o) {
#if KT_SHFL_DPP
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = xor_lane_u32((unsigned)b, o), hi = xor_lane_u32((unsigned)(b >> 32), o);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
#else
    return __shfl_xor(v, o, 64);
#endif
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
#if KT_SHFL_DPP
    const unsigned lo = xor_lane_u32((unsigned)v, o), hi = xor_lane_u32((unsigned)(v >> 32), o);
    return ((unsigned long long)hi << 32) | lo;
#else
    return __shfl_xor(v, o, 64);
#endif
}

__device__ __forceinline__ int shfl_xor_i(int v, int o) {
#if KT_SHFL_DPP
    return (int)xor_lane_u32((unsigned)v, o);
#else
    return __shfl_xor(v, o, 64);
#endif
}

__device__ __forceinline__ double shfl_xor(double v, int o) { return shfl_xor_d(v, o); }
__device__ __forceinline__ unsigned long long shfl_xor(unsigned long long v, int o) { return shfl_xor_u64(v, o); }
__device__ __forceinline__ int shfl_xor(int v, int o) { return shfl_xor_i(v, o); }

}  // namespace kt
