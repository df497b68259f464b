// FETCH_SIZE / WRITE_SIZE calibration for the long-sequence sweep kernel's global
// access pattern (gs_sweep_long.hip; MI355X_MICROARCH.md § HBM: "calibrate on a known
// byte count in your own access pattern").  One 16-lane row a target, four targets a
// wavefront iteration, the kernel's loads and stores outside LDS exactly:
//   - the descriptors len[n] (4 B), pos_in[n] (4 B), pkoff[n] (8 B), read by all 16
//     lanes of the row (one address);
//   - lane q's 16-byte load (4-byte aligned) from the word of its first window x0 =
//     q (K / 16) + min(q, K % 16): the 16 loads of a row cover the sequence's words;
//   - the outputs pos_out[n] (4 B) and pwms_out[n] (8 B), by the row's lane 0.
// Wavefronts take batches of four targets at a stride of the grid's wavefronts (the
// kernel hands them out by counters: the same set of addresses per launch).  Sequences
// are packed 16 symbols a word, each padded to a multiple of 4 words, as
// gs_set_sequences lays them out.  Known HBM bytes per launch: reads N (16 + 16
// ceil(L / 64)), writes N 12.
//   calib_long <N> <L> <W> <launches> [waves]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(256) calib_long_kernel(const uint32_t *pk, const int64_t *pkoff, const int *len,
                                                         const int *pos, int n, int W, int *pos_out,
                                                         double *pwms_out) {
    const int lane = threadIdx.x & 63, t = lane >> 4, q = lane & 15;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    const int nb = (n + 3) / 4;
    for (int b = wave; b < nb; b += nwaves) {
        const int s = 4 * b + t;
        if (s >= n) continue;
        const int L = len[s], p = pos[s];
        const int64_t wo = pkoff[s];
        uint32_t acc = (uint32_t)p;
        const int K = L - W + 1;
        const int x0 = q * (K >> 4) + min(q, K & 15);
        uint4 v;
        __builtin_memcpy(&v, pk + wo + (x0 >> 4), 16);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
        // (the row's sum, so that every lane's load is live)
        for (int m = 1; m < 16; m <<= 1) acc ^= (uint32_t)__shfl_xor((int)acc, m, 64);
        if (q == 0) {
            pos_out[s] = (int)(acc & 0xff);
            pwms_out[s] = (double)acc;
        }
    }
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 100000;
    const int L = argc > 2 ? atoi(argv[2]) : 500;
    const int W = argc > 3 ? atoi(argv[3]) : 15;
    const int launches = argc > 4 ? atoi(argv[4]) : 10;
    const int waves = argc > 5 ? atoi(argv[5]) : 3072;  // the kernel's grid at config 3
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
    const int blocks = (waves + 3) / 4;
    for (int i = 0; i < launches; ++i)
        hipLaunchKernelGGL(calib_long_kernel, dim3(blocks), dim3(256), 0, 0, dpk, doff, dlen, dpos, n, W, dpo, dpw);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"n\": %d, \"L\": %d, \"W\": %d, \"waves\": %d, \"bytes_read_per_launch\": %lld, "
           "\"bytes_written_per_launch\": %lld}\n",
           n, L, W, blocks * 4, (long long)n * (16 + 4LL * padded), (long long)n * 12);
    (void)hipFree(dpk);
    (void)hipFree(doff);
    (void)hipFree(dlen);
    (void)hipFree(dpos);
    (void)hipFree(dpo);
    (void)hipFree(dpw);
    return 0;
}
