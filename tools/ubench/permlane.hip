// Semantics check of v_permlane32_swap_b32 on gfx950 (prints lanes 0, 1, 32, 33).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned *out) {
    const unsigned l = threadIdx.x;
    unsigned x = 1000 + l, y = 2000 + l;
    auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    out[2 * l] = r[0];
    out[2 * l + 1] = r[1];
}
int main() {
    unsigned *d, h[128];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: x' = %u  y' = %u\n", l, h[2 * l], h[2 * l + 1]);
    return 0;
}
