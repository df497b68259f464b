// FETCH_SIZE / WRITE_SIZE calibration for the general sweep kernel's global access
// pattern (gs_sweep.hip; MI355X_MICROARCH.md § HBM: "calibrate on a known byte count
// in your own access pattern").  GL lanes per sequence, 64 / GL sequences a wavefront,
// 4 wavefronts a workgroup, contiguous sequence ranges per wavefront, exactly the
// kernel's loads and stores outside LDS:
//   - the batch descriptors len[n] (4 B), doff[n] (8 B), pos_in[n] (4 B), one lane a
//     sequence (the group's first descriptors again, by lanes 0..G-1: cached);
//   - the sequence (pair codes): one 16-byte load per group lane, L bytes padded to 16;
//   - the composition comp[n][E+1] (int32), one group lane an entry;
//   - the snapshot's 8 aggregate replicas (cells int64 each), every workgroup;
//   - the outputs pos_out[n] (4 B) and pwms_out[n] (8 B), and one atomic add a cell
//     into replica blockIdx % 8.
// Known HBM bytes per launch: reads N (16 + 16 ceil(L / 16) + 4 (E + 1)) + 8 * 8 cells,
// writes N 12 + 8 * 8 cells.
//   calib_sweep <N> <L> <GL> <E> <cells> <launches>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(1024) calib_sweep_kernel(const uint8_t *seq, const int64_t *doff, const int *len,
                                                          const int *pos, const int *comp, const int64_t *agg,
                                                          int n, int GL, int CS, int cells, int *pos_out,
                                                          double *pwms_out, int64_t *agg_out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const int G = 64 / GL, gi = lane / GL, li = lane & (GL - 1);
    const int nwaves = gridDim.x * wpb, gw = blockIdx.x * wpb + w;
    const int q = n / nwaves, r = n % nwaves;
    const int n0 = gw * q + min(gw, r), cnt = q + (gw < r ? 1 : 0);
    uint32_t acc = 0;
    // the snapshot's replicas
    for (int c = threadIdx.x; c < cells; c += blockDim.x) {
        int64_t s = 0;
        for (int rr = 0; rr < 8; ++rr) s += agg[(int64_t)rr * cells + c];
        acc ^= (uint32_t)s;
    }
    // batch descriptors, one lane a sequence
    int bl = 0, bp = -1;
    int64_t bo = 0;
    if (lane < cnt) {
        bl = len[n0 + lane];
        bo = doff[n0 + lane];
        bp = pos[n0 + lane];
    }
    for (int it = 0; it * G < cnt; ++it) {
        const int s = it * G + gi;
        const int L = __shfl(bl, s & 63, 64);
        const int64_t o = __shfl(bo, s & 63, 64);
        if (s < cnt) {
            if (li * 16 < L) {
                const uint4 v = *(const uint4 *)(seq + o + li * 16);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
            if (li < CS) acc ^= (uint32_t)comp[(int64_t)(n0 + s) * CS + li];
        }
    }
    acc ^= (uint32_t)bp;
    for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
    if (lane < cnt) {
        pos_out[n0 + lane] = (int)(acc & 0xff);
        pwms_out[n0 + lane] = (double)acc;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < cells; c += blockDim.x)
        atomicAdd((unsigned long long *)&agg_out[(int64_t)(blockIdx.x % 8) * cells + c], (unsigned long long)(acc & 1));
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 10000;
    const int L = argc > 2 ? atoi(argv[2]) : 200;
    const int GL = argc > 3 ? atoi(argv[3]) : 16;
    const int E = argc > 4 ? atoi(argv[4]) : 4;
    const int cells = argc > 5 ? atoi(argv[5]) : 52;
    const int launches = argc > 6 ? atoi(argv[6]) : 10;
    // the kernel's launch shape: wavefronts a workgroup and workgroups (0: one wavefront
    // per 64/GL sequences) -- config 5's sweep runs 12 x 256 (round 5 on)
    const int wpb = argc > 7 ? atoi(argv[7]) : 4;
    const int grid_arg = argc > 8 ? atoi(argv[8]) : 0;
    const int CS = E + 1;
    const int64_t stride = (L + 15) / 16 * 16;
    std::vector<int64_t> off(n);
    std::vector<int> len(n, L), pos(n), comp((size_t)n * CS, 1);
    for (int i = 0; i < n; ++i) {
        off[i] = (int64_t)i * stride;
        pos[i] = (int)((i * 2654435761u) % 100u);
    }
    const size_t nb = (size_t)n * stride + 64;
    std::vector<uint8_t> sq(nb);
    for (size_t i = 0; i < nb; ++i) sq[i] = (uint8_t)(i * 2654435761u >> 24);
    std::vector<int64_t> agg((size_t)8 * cells, 1);
    uint8_t *dsq;
    int64_t *doff, *dagg, *dago;
    int *dlen, *dpos, *dcomp, *dpo;
    double *dpw;
    if (hipMalloc(&dsq, nb) || hipMalloc(&doff, (size_t)n * 8) || hipMalloc(&dlen, (size_t)n * 4) ||
        hipMalloc(&dpos, (size_t)n * 4) || hipMalloc(&dcomp, (size_t)n * CS * 4) || hipMalloc(&dpo, (size_t)n * 4) ||
        hipMalloc(&dpw, (size_t)n * 8) || hipMalloc(&dagg, agg.size() * 8) || hipMalloc(&dago, agg.size() * 8))
        return 1;
    if (hipMemcpy(dsq, sq.data(), nb, hipMemcpyHostToDevice) ||
        hipMemcpy(doff, off.data(), (size_t)n * 8, hipMemcpyHostToDevice) ||
        hipMemcpy(dlen, len.data(), (size_t)n * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(dpos, pos.data(), (size_t)n * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(dcomp, comp.data(), (size_t)n * CS * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(dagg, agg.data(), agg.size() * 8, hipMemcpyHostToDevice) || hipMemset(dago, 0, agg.size() * 8))
        return 1;
    // the sweep kernel's grid: one wavefront per 64/GL sequences, 4 a workgroup
    const int waves = (n + 64 / GL - 1) / (64 / GL);
    const int grid = grid_arg > 0 ? grid_arg : (waves + wpb - 1) / wpb;
    for (int i = 0; i < launches; ++i)
        hipLaunchKernelGGL(calib_sweep_kernel, dim3(grid), dim3(64 * wpb), 0, 0, dsq, doff, dlen, dpos, dcomp, dagg, n, GL,
                           CS, cells, dpo, dpw, dago);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"n\": %d, \"L\": %d, \"GL\": %d, \"E\": %d, \"waves_per_block\": %d, \"grid\": %d, "
           "\"bytes_read_per_launch\": %lld, \"bytes_written_per_launch\": %lld}\n",
           n, L, GL, E, wpb, grid, (long long)n * (16 + stride + 4LL * CS) + 64LL * cells, (long long)n * 12 + 64LL * cells);
    (void)hipFree(dsq);
    (void)hipFree(doff);
    (void)hipFree(dlen);
    (void)hipFree(dpos);
    (void)hipFree(dcomp);
    (void)hipFree(dpo);
    (void)hipFree(dpw);
    (void)hipFree(dagg);
    (void)hipFree(dago);
    return 0;
}
