// gs_pick.h — segmented wavefront primitives and the certified roulette pick
// (.fs:746-754), shared by the sweep kernels (gs_sweep.hip, gs_sweep_dna.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "gs_common.h"
#include "gs_wave.h"

namespace gs {

// ---- segmented wavefront primitives: groups of GL in {16, 32, 64} lanes -------
// Every one of them must run with all 64 lanes active.
__device__ __forceinline__ int bperm_i32(int v, int src) {
    return __builtin_amdgcn_ds_bpermute(src << 2, v);
}
__device__ __forceinline__ double bperm_f64(double x, int src) {
    return __hiloint2double(bperm_i32(__double2hiint(x), src), bperm_i32(__double2loint(x), src));
}
__device__ __forceinline__ int64_t bperm_i64(int64_t x, int src) {
    const uint32_t lo = (uint32_t)bperm_i32((int)(uint32_t)x, src);
    const uint32_t hi = (uint32_t)bperm_i32((int)(uint32_t)((uint64_t)x >> 32), src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Inclusive prefix sum inside each group (DPP row shifts; row broadcasts only
// within a group).
template <int GL>
__device__ __forceinline__ double seg_scan_f64(double x) {
    x = x + dpp_f64<0x111, 0xf>(x);
    x = x + dpp_f64<0x112, 0xf>(x);
    x = x + dpp_f64<0x114, 0xf>(x);
    x = x + dpp_f64<0x118, 0xf>(x);
    if constexpr (GL >= 32) x = x + dpp_f64<0x142, 0xa>(x);  // row_bcast:15 into rows 1, 3
    if constexpr (GL == 64) x = x + dpp_f64<0x143, 0xc>(x);  // row_bcast:31 into rows 2, 3
    return x;
}

template <int GL>
__device__ __forceinline__ int seg_scan_i32(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
    if constexpr (GL >= 32) v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, true);
    if constexpr (GL == 64) v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, true);
    return v;
}

// the same in wrapping unsigned arithmetic (modular sums, e.g. fixed-point prefixes)
template <int GL>
__device__ __forceinline__ uint32_t seg_scan_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
    if constexpr (GL >= 32) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, true);
    if constexpr (GL == 64) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, true);
    return v;
}

// inclusive running maximum of non-negative ints (float bit patterns order alike)
template <int GL>
__device__ __forceinline__ int seg_scan_max_i32(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));
    if constexpr (GL >= 32) v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, true));
    if constexpr (GL == 64) v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, true));
    return v;
}

// the value of the group's last lane, in every lane of the group (GL = 16, one DPP row a
// group: DPP row_newbcast:15, control 0x15F on gfx950 -- tools/probe/dpp_newbcast.hip --
// one VALU a dword and no LDS round trip; a disabled source lane gives 0, as the
// bpermute's would)
template <int GL>
__device__ __forceinline__ int seg_last_i32(int v, int lane) {
    if constexpr (GL == 64)
        return __builtin_amdgcn_readlane(v, 63);
    else if constexpr (GL == 16)
        return __builtin_amdgcn_update_dpp(0, v, 0x15F, 0xf, 0xf, false);
    else
        return bperm_i32(v, lane | (GL - 1));
}
template <int GL>
__device__ __forceinline__ double seg_last_f64(double x, int lane) {
    if constexpr (GL == 64)
        return lane_read_f64(x, 63);
    else if constexpr (GL == 16)
        return __hiloint2double(seg_last_i32<16>(__double2hiint(x), lane), seg_last_i32<16>(__double2loint(x), lane));
    else
        return bperm_f64(x, lane | (GL - 1));
}

// the group's ballot, bit i = group lane i
template <int GL>
__device__ __forceinline__ unsigned long long seg_ballot(bool p, int lane) {
    const unsigned long long m = __ballot(p);
    if constexpr (GL == 64)
        return m;
    else
        return (m >> (lane & ~(GL - 1))) & ((1ull << GL) - 1ull);
}

__device__ __forceinline__ int wave_max_i32(int v) {
    return __builtin_amdgcn_readlane(seg_scan_max_i32<64>(v), 63);
}

// Certified roulette pick (.fs:746-754), per group.  Group lane l scored windows
// [l*R, l*R + nv_l) into sG (background weights) and sM (motif weights, lcat
// categories); ev(k, g, m) re-evaluates window k exactly as the scan did (m =
// -inf: not a category).  Weights are non-negative and each is within its share
// of eabs (the summed absolute error bound) of the reference's.  Groups with
// !on do not pick (returns -5).  Returns 0 (background category pk), 1 (motif
// category pk), or < 0 when the pick is not certified (the caller falls back):
// -1 total not separated from its error bound, -2 no candidate lane, -3 u
// within the bound of a deciding CDF boundary, -4 u between two lanes' blocks.
// All 64 lanes must be active.
template <int GL, class Eval>
__device__ int certified_pick(const Eval &ev, bool on, int K, int R, int lane, double u,
                              double sG, double sM, int lcat, int npass, double eabs_g,
                              double eabs_m_per, double eabs_m_rel, int &pk) {
    const int li = lane & (GL - 1), gbase = lane & ~(GL - 1);
    const double inclG = seg_scan_f64<GL>(sG);
    const double inclM = seg_scan_f64<GL>(sM);
    const double totG = seg_last_f64<GL>(inclG, lane), totM = seg_last_f64<GL>(inclM, lane);
    const double total = totG + totM;
    const double eabs = totG * eabs_g + (double)npass * eabs_m_per + totM * eabs_m_rel;
    int res = on ? 1 : -5;  // 1: still deciding
    if (res == 1 && (!(total > 4.0 * eabs) || !(total < INFINITY))) res = -1;  // also NaN, <= 0
    // rounding of the reference's sequential sums and of ours (wavefront scans,
    // one division each), relative to the total; SA = total (weights >= 0)
    const double ncat = (double)(K + npass + 2);
    // 1 / total by v_rcp_f64 and two Newton steps.  v_rcp_f64 is specified to about
    // 2^-23 relative; each step squares the relative error e (to e^2 plus the two
    // FMAs' roundings, 2^-52), so two give < 2^-46^2 + 2^-52 ~ 2^-52 whatever the
    // first guess within 2^-23: far below the 2^-48 added (the prefix ratios it
    // scales are all <= 1 + delta).  The approximation term eabs/T (1 + (T + eabs)/(T -
    // eabs)) is bounded with it by eabs r (2 + 2.67 eabs r) (T > 4 eabs), widened by 2^-40
    double inv = __builtin_amdgcn_rcp(total);
    inv = fma(inv, fma(-total, inv, 1.0), inv);
    inv = fma(inv, fma(-total, inv, 1.0), inv);
    const double er = eabs * inv;
    const double delta = (8.0 * ncat + 64.0) * 0x1.0p-53 + 0x1.0p-48 +
                         er * (2.0 + 2.67 * er) * (1.0 + 0x1.0p-40);
    const int nv = min(max(K - li * R, 0), R);
    const bool phaseG = !(u > totG * inv + delta);
    // lane level: the first lane whose block range may contain u
    const double lo = phaseG ? (inclG - sG) * inv : (totG + (inclM - sM)) * inv;
    const double hi = phaseG ? inclG * inv : (totG + inclM) * inv;
    const bool cand =
        res == 1 && (phaseG ? nv > 0 : lcat > 0) && u >= lo - delta && u <= hi + delta;
    const unsigned long long b = seg_ballot<GL>(cand, lane);
    if (res == 1 && !b) res = -2;
    const int f = b ? __ffsll((long long)b) - 1 : 0;
    double base;
    int nf;
    if constexpr (GL == 64) {
        base = lane_read_f64(lo, f);
        nf = __builtin_amdgcn_readlane(nv, f);
    } else {
        base = bperm_f64(lo, gbase + f);
        nf = bperm_i32(nv, gbase + f);
    }
    // window level inside lane f's block, GL windows at a time
    const int nfmax = wave_max_i32(res == 1 ? nf : 0);
    for (int c0 = 0; c0 < nfmax; c0 += GL) {
        const int t = c0 + li;
        double w = 0.0;
        bool is_cat = false;
        if (res == 1 && t < nf) {
            double g, m;
            ev(f * R + t, g, m);
            const double x = phaseG ? g : m;
            is_cat = phaseG || x != -INFINITY;
            if (is_cat) w = x * inv;
        }
        const double incl = seg_scan_f64<GL>(w);
        const double l0 = base + (incl - w), h0 = base + incl;
        const bool no = !is_cat || u < l0 - delta || u > h0 + delta;
        const bool yes = !no && u >= l0 + delta && u <= h0 - delta;
        const unsigned long long bb = seg_ballot<GL>(res == 1 && !no, lane);
        const int first = bb ? __ffsll((long long)bb) - 1 : 0;
        const int y = GL == 64 ? __builtin_amdgcn_readlane((int)yes, first)
                               : bperm_i32((int)yes, gbase + first);
        if (res == 1 && bb) {
            if (y) {
                pk = f * R + c0 + first;
                res = phaseG ? 10 : 11;
            } else {
                res = -3;
            }
        }
        base = base + seg_last_f64<GL>(incl, lane);
    }
    if (res == 1) res = -4;
    return res >= 10 ? res - 10 : res;
}

}  // namespace gs
