// gs_sweep.hip — fused Gibbs sweep kernel for gfx950 (MI355X).
//
// One workgroup = one 64-lane wavefront; workgroups grid-stride over this rank's
// sequences.  Per sequence n (MotifSampler.findBestMotifIndicesByWithStartPositions,
// .fs:935-970, motifAmount = 1):
//   1. stage the encoded sequence into LDS with 16-byte loads, build its symbol
//      histogram (CompositeVector, .fs:60-62);
//   2. hold-one-out background counts and PCV from the global aggregates
//      (createFCVWithout/fuseFrequencyVectors/increaseInPlaceFCVOf/
//      createNormalizedPCVOfFCV, .fs:945-954) — integer-exact;
//   3. hold-one-out PFM -> PPM -> PWM (.fs:955-965), staged in LDS as [j][symbol];
//   4. every W-mer window scored (.fs:759-777): S_k (PWM product) and G_k
//      (background product), left folds in binary64 exactly as the reference;
//      log2 cut-off test (.fs:735-738);
//   5. roulette pick (.fs:746-754): wavefront prefix sums give a certified pick;
//      when u falls within the rounding bound of a boundary, one lane redoes the
//      reference's sequential sums exactly;
//   6. the picked segment is folded into per-workgroup aggregates of the NEW
//      snapshot, flushed to XCD-replicated global accumulators once per workgroup:
//      they are the next sweep's count matrix / background totals.
//
// Compiled with -ffp-contract=off: no FMA contraction, so products and quotients
// round exactly as the reference's IEEE binary64 operations.
#include <hip/hip_runtime.h>

#include "gs_common.h"

using namespace gs;

namespace {

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ __forceinline__ double wave_incl_scan(double x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        double y = __shfl_up(x, d, 64);
        if (lane >= d) x = x + y;
    }
    return x;
}

__device__ __forceinline__ void raise_error(const SweepArgs &a, int code, int64_t gidx) {
    atomicCAS(a.err_code, 0, code);
    atomicMin(a.err_index, (unsigned long long)gidx);
}

// Certified search over one 64-category chunk.  Returns 1 = picked lane *f,
// 2 = uncertain (fallback), 0 = every category certainly false (continue).
__device__ __forceinline__ int chunk_pick(double w, bool present, double u, double delta,
                                          double &carry, int lane, int *f) {
    double incl = wave_incl_scan(w, lane);
    double excl = __shfl_up(incl, 1, 64);
    if (lane == 0) excl = 0.0;
    double acc = carry + excl;
    double hi = acc + w;
    bool cf = (u < acc - delta) || (u > hi + delta);
    bool ct = (u >= acc + delta) && (u <= hi - delta);
    unsigned long long m = __ballot(present && !cf);
    carry = carry + __shfl(incl, 63, 64);
    if (m == 0ull) return 0;
    int first = __ffsll((long long)m) - 1;
    unsigned long long tm = __ballot(ct);
    *f = first;
    return ((tm >> first) & 1ull) ? 1 : 2;
}

}  // namespace

extern "C" __global__ void __launch_bounds__(64) gs_sweep_kernel(SweepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x;
    if (__hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;

    const int A = a.A, W = a.W, AW = A * W;
    double *pcv = (double *)(lds + a.o_pcv);        // [128] by encoded byte
    double *pwm = (double *)(lds + a.o_pwm);        // [W][A+1]
    double *Gs = (double *)(lds + a.o_G);           // [Kmax]
    double *Ms = (double *)(lds + a.o_M);           // [Kmax]
    unsigned long long *mask = (unsigned long long *)(lds + a.o_mask);
    int64_t *T = (int64_t *)(lds + a.o_T);          // [A]
    int64_t *aggM = (int64_t *)(lds + a.o_aggM);    // [A]
    int32_t *cg = (int32_t *)(lds + a.o_cg);        // [A*W]
    int32_t *aggC = (int32_t *)(lds + a.o_aggC);    // [A*W]
    int32_t *comp = (int32_t *)(lds + a.o_comp);    // [128]
    int32_t *misc = (int32_t *)(lds + a.o_misc);
    uint8_t *sseq = (uint8_t *)(lds + a.o_seq);

    // ---- prologue: aggregates of the snapshot (sum of the replicas) ----
    for (int c = lane; c < a.cells; c += 64) {
        int64_t s = 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r) s += a.agg_in ? a.agg_in[(int64_t)r * a.stride + c] : 0;
        if (c < AW) {
            cg[c] = (int32_t)s;
            aggC[c] = 0;
        } else {
            T[c - AW] = s;  // composition total for now, T below
            aggM[c - AW] = 0;
        }
    }
    if (blockIdx.x == 0 && a.agg_zero)
        for (int i = lane; i < kRepl * a.stride; i += 64) a.agg_zero[i] = 0;
    __syncthreads();
    if (a.mode == 0) {
        for (int x = lane; x < A; x += 64) {
            int64_t s = T[x];
            for (int j = 0; j < W; ++j) s -= cg[x * W + j];
            T[x] = s;
        }
    }
    __syncthreads();

    for (int n = blockIdx.x; n < a.n_local; n += gridDim.x) {
        const int L = a.len[n];
        const int K = L - W + 1;
        const uint8_t *g = a.seq + a.doff[n];
        for (int i = lane * 16; i < L; i += 64 * 16)
            *(uint4 *)(sseq + i) = *(const uint4 *)(g + i);
        comp[lane] = 0;
        comp[lane + 64] = 0;
        __syncthreads();
        for (int i = lane; i < L; i += 64) atomicAdd(&comp[sseq[i]], 1);
        __syncthreads();

        const int p = a.pos_in[n];
        const int64_t gidx = a.global_offset + n;
        int newp = p;
        if (a.mode == 0) {
            // ---- hold-one-out background (integer exact) ----
            int64_t bgc = 0;
            int32_t ca = 0;
            if (lane < A) {
                int segc = 0;
                if (p >= 0)
                    for (int j = 0; j < W; ++j) segc += (sseq[p + j] == lane);
                ca = comp[lane];
                bgc = T[lane] + (p >= 0 ? (int64_t)segc : (int64_t)ca);
            }
            int64_t alpha_tot = wave_sum_i64((int64_t)ca);
            int64_t tot = wave_sum_i64(bgc) + ((int64_t)L - alpha_tot);
            if (tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
                if (lane == 0) raise_error(a, 3, gidx);
                continue;
            }
            const double sbg = (double)tot + a.apc;
            if (lane < A) pcv[lane] = ((double)bgc + a.pc) / sbg;  // .fs:119
            if (lane < kSlots) pcv[kNonAlpha + lane] = (double)comp[kNonAlpha + lane];  // raw (Q3)
            __syncthreads();
            // ---- PWM = PPM / PCV (.fs:257-260, .fs:286) ----
            const int A1 = A + 1;
            for (int c = lane; c < W * A1; c += 64) {
                int j = c / A1, e = c - j * A1;
                double v = 0.0;
                if (e < A) {
                    int cnt = cg[e * W + j] - ((p >= 0 && sseq[p + j] == e) ? 1 : 0);
                    double ppm = ((double)cnt + a.pc) / a.den;
                    v = ppm / pcv[e];
                }
                pwm[c] = v;
            }
            __syncthreads();
            // ---- score every window (.fs:759-782) ----
            double sumG = 0.0, sumM = 0.0, sumAbs = 0.0;
            int npass = 0;
            for (int k0 = 0; k0 < K; k0 += 64) {
                const int k = k0 + lane;
                const bool valid = k < K;
                double S = 1.0, G = 1.0;
                if (valid) {
                    for (int j = 0; j < W; ++j) {
                        const int e = sseq[k + j];
                        S = S * pwm[j * A1 + (e < A ? e : A)];
                        G = G * pcv[e];
                    }
                }
                bool pass = false;
                double M = 0.0;
                if (valid && S >= a.thr_lo) {
                    double l2 = log(S * 1.0) / kLn2;
                    if (l2 > a.cutoff) {
                        pass = true;
                        M = l2;
                    }
                }
                if (valid) {
                    Gs[k] = G;
                    Ms[k] = M;
                    sumG += G;
                    sumM += M;
                    sumAbs += fabs(G) + fabs(M);
                }
                unsigned long long pm = __ballot(pass);
                if (lane == 0) mask[k0 >> 6] = pm;
                npass += pass ? 1 : 0;
            }
            sumG = wave_sum(sumG);
            sumM = wave_sum(sumM);
            sumAbs = wave_sum(sumAbs);
            npass = (int)wave_sum_i64((int64_t)npass);
            __syncthreads();
            const double total = sumG + sumM;
            const double ncat = (double)(K + npass + 2);
            const double delta = 8.0 * ncat * 0x1.0p-53 * (sumAbs / fabs(total));
            const double u = a.u_in ? a.u_in[n] : uniform(a.seed, a.stream, (uint64_t)gidx);

            // ---- certified roulette (.fs:746-754) ----
            int kind = -1, pk = -1;  // kind 0 = background category, 1 = motif category
            int state = 0;           // 0 searching, 1 picked, 2 fallback
            double carry = 0.0;
            const double gfrac = sumG / total;
            if (u > gfrac + 2.0 * delta) {
                carry = gfrac;
            } else {
                for (int k0 = 0; k0 < K && state == 0; k0 += 64) {
                    const int k = k0 + lane;
                    const bool present = k < K;
                    const double w = present ? Gs[k] / total : 0.0;
                    int f;
                    int r = chunk_pick(w, present, u, delta, carry, lane, &f);
                    if (r == 1) {
                        state = 1;
                        kind = 0;
                        pk = k0 + f;
                    } else if (r == 2) {
                        state = 2;
                    }
                }
            }
            if (state == 0 && npass > 0) {
                for (int k0 = 0; k0 < K && state == 0; k0 += 64) {
                    const int k = k0 + lane;
                    const bool present = k < K && ((mask[k0 >> 6] >> lane) & 1ull);
                    const double w = present ? Ms[k] / total : 0.0;
                    int f;
                    int r = chunk_pick(w, present, u, delta, carry, lane, &f);
                    if (r == 1) {
                        state = 1;
                        kind = 1;
                        pk = k0 + f;
                    } else if (r == 2) {
                        state = 2;
                    }
                }
            }
            if (state == 2) {
                // exact sequential restatement, one lane
                if (lane == 0) {
                    atomicAdd(a.fallbacks, 1ull);
                    double s = 0.0;
                    for (int k = 0; k < K; ++k) s = s + Gs[k];
                    for (int k = 0; k < K; ++k)
                        if ((mask[k >> 6] >> (k & 63)) & 1ull) s = s + Ms[k];
                    double acc = 0.0;
                    int rk = -1, rp = -1;
                    for (int k = 0; k < K && rk < 0; ++k) {
                        double w = Gs[k] / s;
                        if (acc <= u && u <= acc + w) {
                            rk = 0;
                            rp = k;
                        }
                        acc = acc + w;
                    }
                    for (int k = 0; k < K && rk < 0; ++k) {
                        if (!((mask[k >> 6] >> (k & 63)) & 1ull)) continue;
                        double w = Ms[k] / s;
                        if (acc <= u && u <= acc + w) {
                            rk = 1;
                            rp = k;
                        }
                        acc = acc + w;
                    }
                    misc[0] = rk;
                    misc[1] = rp;
                }
                __syncthreads();
                kind = misc[0];
                pk = misc[1];
                __syncthreads();
            }
            if (kind < 0) {  // every category certainly (or exactly) missed: list overrun
                if (lane == 0) raise_error(a, 2, gidx);
                continue;
            }
            newp = kind == 0 ? -1 : pk;
            if (lane == 0) {
                a.pos_out[n] = newp;
                a.pwms_out[n] = kind == 0 ? Gs[pk] : Ms[pk];
            }
        }
        // ---- fold the chosen segment into the next snapshot's aggregates ----
        if (newp >= 0) {
            for (int c = lane; c < AW; c += 64) {
                int x = c / W, j = c - x * W;
                aggC[c] += (sseq[newp + j] == x) ? 1 : 0;
            }
            if (lane < A) aggM[lane] += comp[lane];
        }
        __syncthreads();
    }
    // ---- flush per-workgroup aggregates into replica blockIdx % kRepl ----
    int64_t *dst = a.agg_out + (int64_t)(blockIdx.x % kRepl) * a.stride;
    for (int c = lane; c < a.cells; c += 64) {
        int64_t v = c < AW ? (int64_t)aggC[c] : aggM[c - AW];
        if (v != 0) atomicAdd((unsigned long long *)&dst[c], (unsigned long long)v);
    }
}

// Host-side launch helpers (the C-ABI translation unit stays free of kernel code).
hipError_t gs_sweep_occupancy(int *blocks_per_cu, size_t lds_bytes) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, gs_sweep_kernel, 64,
                                                        lds_bytes);
}
hipError_t gs_sweep_launch(const SweepArgs &a, int grid, size_t lds_bytes, hipStream_t stream) {
    hipLaunchKernelGGL(gs_sweep_kernel, dim3(grid), dim3(64), lds_bytes, stream, a);
    return hipGetLastError();
}
