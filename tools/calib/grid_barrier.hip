// Launch-chain vs persistent-kernel cost of the sweep's synchronisation skeleton:
// per sweep, every workgroup sums the 8 XCD replicas of the aggregates, adds its
// own contribution to its XCD's replica, and the next sweep may start only when
// all workgroups are done.  (a) one launch per sweep, (b) one launch for all
// sweeps with a grid barrier (device-scope counter, bounded spin).
//
//   grid_barrier <workgroups> <sweeps>      prints µs per sweep for (a) and (b)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kRepl = 8, kCells = 56, kThreads = 256;

__device__ void skeleton(const long long *in, long long *out, long long *zero, long long *lds) {
    const int tid = threadIdx.x;
    for (int c = tid; c < kCells; c += kThreads) {
        long long s = 0;
        for (int r = 0; r < kRepl; ++r) s += in[r * kCells + c];
        lds[c] = s;
    }
    if (blockIdx.x == 0)
        for (int i = tid; i < kRepl * kCells; i += kThreads) zero[i] = 0;
    __syncthreads();
    long long *dst = out + (blockIdx.x % kRepl) * kCells;
    for (int c = tid; c < kCells; c += kThreads) atomicAdd((unsigned long long *)&dst[c], 1ull + (lds[c] & 1));
}

__global__ void __launch_bounds__(kThreads) step_kernel(long long *bufs, int t) {
    __shared__ long long lds[kCells];
    long long *b[3] = {bufs, bufs + kRepl * kCells, bufs + 2 * kRepl * kCells};
    skeleton(b[t % 3], b[(t + 1) % 3], b[(t + 2) % 3], lds);
}

__global__ void __launch_bounds__(kThreads) persist_kernel(long long *bufs, int sweeps,
                                                           unsigned int *ctr, int *timeout) {
    __shared__ long long lds[kCells];
    long long *b[3] = {bufs, bufs + kRepl * kCells, bufs + 2 * kRepl * kCells};
    for (int t = 0; t < sweeps; ++t) {
        skeleton(b[t % 3], b[(t + 1) % 3], b[(t + 2) % 3], lds);
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();  // release this workgroup's replica updates
            atomicAdd(ctr, 1u);
            const unsigned int goal = gridDim.x * (unsigned)(t + 1);
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < goal) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t0 > 50000000ull) {  // 0.5 s at 100 MHz: give up
                    atomicExch(timeout, 1);
                    break;
                }
            }
        }
        __syncthreads();
        if (__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char **argv) {
    int grid = argc > 1 ? atoi(argv[1]) : 512, sweeps = argc > 2 ? atoi(argv[2]) : 200;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)persist_kernel, kThreads, 0));
    if (grid > per_cu * prop.multiProcessorCount) {
        fprintf(stderr, "grid %d exceeds co-resident %d x %d\n", grid, per_cu, prop.multiProcessorCount);
        return 1;
    }
    long long *bufs;
    unsigned int *ctr;
    int *to;
    CK(hipMalloc(&bufs, 3 * kRepl * kCells * 8));
    CK(hipMalloc(&ctr, 4));
    CK(hipMalloc(&to, 4));
    CK(hipMemset(bufs, 0, 3 * kRepl * kCells * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms_a = 0, ms_b = 0;
    for (int rep = 0; rep < 3; ++rep) {
        for (int t = 0; t < 10; ++t) hipLaunchKernelGGL(step_kernel, grid, kThreads, 0, 0, bufs, t);
        CK(hipEventRecord(e0));
        for (int t = 0; t < sweeps; ++t) hipLaunchKernelGGL(step_kernel, grid, kThreads, 0, 0, bufs, t);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_a, e0, e1));
        CK(hipMemset(ctr, 0, 4));
        CK(hipMemset(to, 0, 4));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(persist_kernel, grid, kThreads, 0, 0, bufs, sweeps, ctr, to);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_b, e0, e1));
        int h_to = 0;
        CK(hipMemcpy(&h_to, to, 4, hipMemcpyDeviceToHost));
        printf("{\"grid\": %d, \"sweeps\": %d, \"launch_chain_us\": %.3f, \"persistent_us\": %.3f, \"timeout\": %d}\n",
               grid, sweeps, 1000.0 * ms_a / sweeps, 1000.0 * ms_b / sweeps, h_to);
        if (h_to) return 2;
    }
    return 0;
}
