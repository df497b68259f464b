// FETCH_SIZE calibration for the sweep kernel's read pattern (MI355X_MICROARCH.md
// § HBM: "calibrate on a known byte count in your own access pattern").
// Lane groups of 16 lanes each read one sequence of L bytes laid out at a 16-byte
// aligned stride with uint4 loads (lane li reads bytes [16 li, 16 li + 16) while
// 16 li < L), as gs_sweep_kernel stages its sequences; one int per group is written.
//   calib_read <N> <L> <launches>   -> prints the known bytes read per launch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(256) calib_read_kernel(const unsigned char *seq, int n, int L,
                                                         int stride, unsigned *out) {
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int s = wave * 4 + g;
    unsigned acc = 0;
    if (s < n && li * 16 < L) {
        const uint4 v = *(const uint4 *)(seq + (size_t)s * stride + li * 16);
        acc = v.x ^ v.y ^ v.z ^ v.w;
    }
    for (int d = 8; d >= 1; d >>= 1) acc ^= __shfl_xor(acc, d, 16);
    if (s < n && li == 0) out[s] = acc;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 10000;
    const int L = argc > 2 ? atoi(argv[2]) : 200;
    const int launches = argc > 3 ? atoi(argv[3]) : 20;
    const int stride = (L + 15) / 16 * 16;
    unsigned char *d = nullptr;
    unsigned *o = nullptr;
    if (hipMalloc(&d, (size_t)n * stride + 64) != hipSuccess || hipMalloc(&o, (size_t)n * 4) != hipSuccess)
        return 1;
    std::vector<unsigned char> h((size_t)n * stride + 64);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned char)(i * 2654435761u >> 24);
    if (hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess) return 1;
    const int waves = (n + 3) / 4, blocks = (waves + 3) / 4;
    for (int i = 0; i < launches; ++i) {
        hipLaunchKernelGGL(calib_read_kernel, dim3(blocks), dim3(256), 0, 0, d, n, L, stride, o);
        // a large buffer between launches would evict; this pattern, like the sweep,
        // re-reads a small resident set
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const long long lines16 = (long long)n * ((L + 15) / 16) * 16;
    printf("{\"n\": %d, \"L\": %d, \"bytes_read_per_launch\": %lld, \"bytes_written_per_launch\": %lld}\n",
           n, L, lines16, (long long)n * 4);
    (void)hipFree(d);
    (void)hipFree(o);
    return 0;
}
