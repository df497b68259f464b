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

// x / d for x < 2^16 by a multiply with magic = 0xffffffff / d + 1.  d = 1 has no
// 32-bit magic (it would wrap to 0): its quotient is x.
__device__ __forceinline__ uint32_t magic_magic(uint32_t d) { return 0xffffffffu / d + 1u; }
__device__ __forceinline__ int magic_div(uint32_t x, uint32_t d, uint32_t magic) {
    return d == 1 ? (int)x : (int)__umulhi(x, magic);
}

// v with its bytes at index >= nb cleared (nb >= 16 keeps all)
__device__ __forceinline__ uint4 keep_bytes(uint4 v, int nb) {
    auto m = [nb](int d) -> uint32_t {
        const int k = nb - 4 * d;
        return k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : (1u << (8 * k)) - 1u);
    };
    return make_uint4(v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3));
}

__device__ __forceinline__ int wave_sum_i32(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, true);
    return __builtin_amdgcn_readlane(v, 63);
}

// Inclusive prefix sum of an int over the 64 lanes (DPP; lanes without a source
// read 0), per lane.
__device__ __forceinline__ int wave_incl_scan_i32(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, true);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, true);  // row_bcast:31
    return v;
}

// Maximum of a non-negative float over the 64 lanes (integer order of the bit
// patterns; DPP lanes without a source read 0).
__device__ __forceinline__ float wave_max_nonneg_f32(float x) {
    int v = __float_as_int(x);
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, true));
    return __int_as_float(__builtin_amdgcn_readlane(v, 63));
}

// Maximum of an unsigned 64-bit key over the 64 lanes (DPP row shifts / row
// broadcasts; lanes without a source read 0, the identity), wave-uniform.
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long x) {
#define GS_MAX_STEP(CTRL, RM)                                                                \
    {                                                                                        \
        const int lo_ = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, RM, 0xf, true); \
        const int hi_ = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, RM, 0xf, \
                                                    true);                                  \
        const unsigned long long y_ = ((unsigned long long)(uint32_t)hi_ << 32) | (uint32_t)lo_; \
        x = y_ > x ? y_ : x;                                                                 \
    }
    GS_MAX_STEP(0x111, 0xf)  // row_shr:1
    GS_MAX_STEP(0x112, 0xf)  // row_shr:2
    GS_MAX_STEP(0x114, 0xf)  // row_shr:4
    GS_MAX_STEP(0x118, 0xf)  // row_shr:8
    GS_MAX_STEP(0x142, 0xa)  // row_bcast:15 into rows 1, 3
    GS_MAX_STEP(0x143, 0xc)  // row_bcast:31 into rows 2, 3
#undef GS_MAX_STEP
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, 63);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}

// Minimum of an int over the 64 lanes, wave-uniform (identity INT_MAX).
__device__ __forceinline__ int wave_min_i32(int v) {
    constexpr int kMax = 0x7fffffff;
    v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x111, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x112, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x114, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x118, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x142, 0xa, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}

// Order-preserving unsigned key of a binary64 value: x < y <=> key(x) < key(y) for
// numbers (-0.0 is folded onto +0.0); NaN maps to 0, below every number (F#
// generic comparison ranks NaN lowest).
__device__ __forceinline__ unsigned long long order_key(double v) {
    if (v != v) return 0ull;
    const unsigned long long b = (unsigned long long)__double_as_longlong(v + 0.0);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// log2 of a positive binary64 value to float accuracy: exponent from v_frexp,
// v_log_f32 on the mantissa rounded to binary32.  |error| <= kLog2AbsErr +
// |result| * 2^-24 (the transcendental's share is checked by gs_fastmath_check).
// 0 -> -inf, +inf -> +inf, NaN/negative -> NaN.
__device__ __forceinline__ float flog2(double v) {
    if (!(v > 0.0)) return v == 0.0 ? -INFINITY : __builtin_nanf("");
    if (v == INFINITY) return INFINITY;
    const int ex = __builtin_amdgcn_frexp_exp(v);
    const float m = (float)__builtin_amdgcn_frexp_mant(v);
    return (float)ex + __builtin_amdgcn_logf(m);
}

// 2^x for |x| < 1000 as binary64 (no binary32 under/overflow): v_exp_f32 on
// the fractional part, exact power of two by v_ldexp_f64.
__device__ __forceinline__ double fexp2(float x) {
    const float fl = floorf(x);
    return ldexp((double)__builtin_amdgcn_exp2f(x - fl), (int)fl);
}

}  // namespace gs
