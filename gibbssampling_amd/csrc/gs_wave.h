// gs_wave.h — wavefront (64-lane) primitives for gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace gs {

// LDS hand-off inside one wavefront: its LDS operations execute in order, so a
// counter wait plus a scheduling barrier suffices (no workgroup barrier).
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// DPP move of a double (two 32-bit halves); lanes without a source read +0.0.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWMASK, 0xf, true);
    hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, ROWMASK, 0xf, true);
    return __hiloint2double(hi, lo);
}

// Inclusive prefix sum over the 64 lanes with DPP row shifts and row broadcasts
// (VALU latency only; no LDS crossbar).  Rounding differs from a sequential sum;
// callers that need the reference's sequential sums certify against a bound.
__device__ __forceinline__ double wave_incl_scan_f64(double x) {
    x = x + dpp_f64<0x111, 0xf>(x);  // row_shr:1
    x = x + dpp_f64<0x112, 0xf>(x);  // row_shr:2
    x = x + dpp_f64<0x114, 0xf>(x);  // row_shr:4
    x = x + dpp_f64<0x118, 0xf>(x);  // row_shr:8
    x = x + dpp_f64<0x142, 0xa>(x);  // row_bcast:15 into rows 1, 3
    x = x + dpp_f64<0x143, 0xc>(x);  // row_bcast:31 into rows 2, 3
    return x;
}

__device__ __forceinline__ double lane_read_f64(double x, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum_f64(double x) {
    return lane_read_f64(wave_incl_scan_f64(x), 63);
}

__device__ __forceinline__ int popc64(unsigned long long m) { return __popcll(m); }

}  // namespace gs
