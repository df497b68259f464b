// Probe: DPP control 0x15F on gfx950 (row_newbcast:15): every lane of a 16-lane row gets
// lane 15 of its row (the long kernel's row totals without ds_bpermute).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *out) {
    const int lane = threadIdx.x;
    const int v = lane * 3 + 1;
    out[lane] = __builtin_amdgcn_update_dpp(0, v, 0x15F, 0xF, 0xF, false);
}
int main() {
    int *d; hipMalloc(&d, 256);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[64]; hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; ++i) { int want = ((i & ~15) + 15) * 3 + 1; if (h[i] != want) { ++bad; printf("lane %d got %d want %d\n", i, h[i], want); } }
    printf("row_share:15 %s\n", bad ? "MISMATCH" : "ok");
    return bad != 0;
}
