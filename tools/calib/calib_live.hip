// FETCH_SIZE / WRITE_SIZE calibration for the live-chain sweep kernel's global access
// pattern (gs_sweep_live.hip; MI355X_MICROARCH.md § HBM: "calibrate on a known byte
// count in your own access pattern").  One lane per target, 64 targets a wavefront,
// exactly the kernel's loads and stores outside LDS:
//   - the descriptors len[n] (4 B), pos_in[n] (4 B), pkoff[n] (8 B);
//   - the own segment: two 4-byte words of the packed sequence at pkoff + p / 16;
//   - the packed words as the scan streams them: 16-byte loads (4-byte aligned) at
//     pkoff + 4 q for q = 0 .. nch (nch = ceil((L - W + 1 + 14) / 64)), which run one
//     chunk past the sequence into the next one's words;
//   - the outputs pos_out[n] (4 B) and pwms_out[n] (8 B).
// Sequences are packed 16 symbols a word, each padded to a multiple of 4 words, as
// gs_set_sequences lays them out.  Known HBM bytes per launch: reads N (16 + 16 ceil(L
// / 64)), writes N 12.
//   calib_live <N> <L> <W> <launches>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ void calib_live_target(const uint32_t *pk, const int64_t *pkoff, const int *len,
                                                  const int *pos, int t, int W, int *pos_out, double *pwms_out) {
    const int L = len[t], p = pos[t];
    const int64_t wo = pkoff[t];
    uint32_t acc = 0;
    if (p >= 0) acc ^= pk[wo + (p >> 4)] ^ pk[wo + (p >> 4) + 1];
    const int nch = (L - W + 1 + 14 + 63) >> 6;
    for (int q = 0; q <= nch; ++q) {
        uint4 v;
        __builtin_memcpy(&v, pk + wo + 4 * q, 16);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    pos_out[t] = (int)(acc & 0xff);
    pwms_out[t] = (double)acc;
}

// one lane a target over the whole grid (the round-3 calibration)
__global__ void __launch_bounds__(256) calib_live_kernel(const uint32_t *pk, const int64_t *pkoff, const int *len,
                                                         const int *pos, int n, int W, int *pos_out,
                                                         double *pwms_out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    calib_live_target(pk, pkoff, len, pos, t, W, pos_out, pwms_out);
}

// the live kernel's launch shape since its work counters (round 5): a grid of `grid`
// workgroups of wpb wavefronts, a wavefront's first tile (64 targets) its rank, each
// next one from a device counter (one atomic a tile, as the kernel's pools)
__global__ void __launch_bounds__(512) calib_live_ctr_kernel(const uint32_t *pk, const int64_t *pkoff, const int *len,
                                                             const int *pos, int n, int W, int *pos_out,
                                                             double *pwms_out, unsigned int *ctr) {
    const int lane = threadIdx.x & 63;
    const int nwaves = gridDim.x * (blockDim.x >> 6);
    const int ntiles = (n + 63) / 64;
    int tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    while (tile < ntiles) {
        int nx = 0;
        if (lane == 0) nx = (int)atomicAdd(ctr, 1u) + nwaves;
        const int t = tile * 64 + lane;
        if (t < n) calib_live_target(pk, pkoff, len, pos, t, W, pos_out, pwms_out);
        tile = __shfl(nx, 0, 64);
    }
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1000000;
    const int L = argc > 2 ? atoi(argv[2]) : 200;
    const int W = argc > 3 ? atoi(argv[3]) : 12;
    const int launches = argc > 4 ? atoi(argv[4]) : 10;
    const int wpb = argc > 5 ? atoi(argv[5]) : 0;   // > 0: the work-counter launch shape
    const int grid_arg = argc > 6 ? atoi(argv[6]) : 0;
    const int words = (L + 15) / 16, padded = (words + 3) / 4 * 4;
    std::vector<int64_t> off(n);
    std::vector<int> len(n, L), pos(n);
    for (int i = 0; i < n; ++i) {
        off[i] = (int64_t)i * padded;
        pos[i] = (int)((i * 2654435761u) % (unsigned)(L - W + 1));
    }
    const size_t nw = (size_t)n * padded + 64;
    std::vector<uint32_t> pk(nw);
    for (size_t i = 0; i < nw; ++i) pk[i] = (uint32_t)(i * 2654435761u);
    uint32_t *dpk;
    int64_t *doff;
    int *dlen, *dpos, *dpo;
    double *dpw;
    if (hipMalloc(&dpk, nw * 4) || hipMalloc(&doff, (size_t)n * 8) || hipMalloc(&dlen, (size_t)n * 4) ||
        hipMalloc(&dpos, (size_t)n * 4) || hipMalloc(&dpo, (size_t)n * 4) || hipMalloc(&dpw, (size_t)n * 8))
        return 1;
    if (hipMemcpy(dpk, pk.data(), nw * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(doff, off.data(), (size_t)n * 8, hipMemcpyHostToDevice) ||
        hipMemcpy(dlen, len.data(), (size_t)n * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(dpos, pos.data(), (size_t)n * 4, hipMemcpyHostToDevice))
        return 1;
    unsigned int *dctr = nullptr;
    if (hipMalloc(&dctr, 4)) return 1;
    for (int i = 0; i < launches; ++i) {
        if (wpb > 0) {
            // (the counter zeroed between launches: its atomics are the kernel's own, the
            // memset is not counted against the kernel)
            if (hipMemsetAsync(dctr, 0, 4, 0)) return 1;
            hipLaunchKernelGGL(calib_live_ctr_kernel, dim3(grid_arg), dim3(64 * wpb), 0, 0, dpk, doff, dlen, dpos, n,
                               W, dpo, dpw, dctr);
        } else {
            hipLaunchKernelGGL(calib_live_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dpk, doff, dlen, dpos, n, W,
                               dpo, dpw);
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"n\": %d, \"L\": %d, \"W\": %d, \"waves_per_block\": %d, \"grid\": %d, "
           "\"bytes_read_per_launch\": %lld, \"bytes_written_per_launch\": %lld}\n",
           n, L, W, wpb, grid_arg, (long long)n * (16 + 4LL * padded), (long long)n * 12);
    (void)hipFree(dctr);
    (void)hipFree(dpk);
    (void)hipFree(doff);
    (void)hipFree(dlen);
    (void)hipFree(dpos);
    (void)hipFree(dpo);
    (void)hipFree(dpw);
    return 0;
}
