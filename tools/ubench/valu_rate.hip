// tools/ubench/valu_rate.hip -- VALU issue rate per SIMD on gfx950 for the
// instruction kinds the DCT kernels use (scalar vs packed fp32, fp64, int16x2).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP8(x) x x x x x x x x
template <int KIND>
__global__ void k(float *out, int iters, unsigned long long *clk) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3;
    float b = 1.0001f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) {  // v_fma_f32
            REP8(asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (KIND == 1) {  // v_pk_fma_f32 (2 lanes of fp32 per instruction)
            REP8(asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"((double)b));)
        } else if (KIND == 2) {  // v_fma_f64
            REP8(asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"((double)b));)
        } else if (KIND == 3) {  // v_pk_add_u16
            REP8(asm volatile("v_pk_add_u16 %0, %0, %8\n v_pk_add_u16 %1, %1, %8\n v_pk_add_u16 %2, %2, %8\n v_pk_add_u16 %3, %3, %8\n v_pk_add_u16 %4, %4, %8\n v_pk_add_u16 %5, %5, %8\n v_pk_add_u16 %6, %6, %8\n v_pk_add_u16 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (KIND == 4) {  // v_add_f32 with a literal
            REP8(asm volatile("v_add_f32 %0, 0x3f800001, %0\n v_add_f32 %1, 0x3f800001, %1\n v_add_f32 %2, 0x3f800001, %2\n v_add_f32 %3, 0x3f800001, %3\n v_add_f32 %4, 0x3f800001, %4\n v_add_f32 %5, 0x3f800001, %5\n v_add_f32 %6, 0x3f800001, %6\n v_add_f32 %7, 0x3f800001, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
        } else {  // v_cvt_f32_ubyte1
            REP8(asm volatile("v_cvt_f32_ubyte1 %0, %0\n v_cvt_f32_ubyte1 %1, %1\n v_cvt_f32_ubyte1 %2, %2\n v_cvt_f32_ubyte1 %3, %3\n v_cvt_f32_ubyte1 %4, %4\n v_cvt_f32_ubyte1 %5, %5\n v_cvt_f32_ubyte1 %6, %6\n v_cvt_f32_ubyte1 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(d0 + d1 + d2 + d3);
}

int main() {
    float *out; unsigned long long *clk, hclk[2];
    hipMalloc(&out, 256 * 32 * 64 * sizeof(float) * 4);
    hipMalloc(&clk, 16);
    const char *names[] = {"v_fma_f32", "v_pk_fma_f32", "v_fma_f64", "v_pk_add_u16", "v_add_f32 lit", "v_cvt_f32_ubyte1"};
    const int per_iter[] = {64, 32, 32, 64, 64, 64};
    const int iters = 2000;
    for (int kind = 0; kind < 6; ++kind)
        for (int wps = 1; wps <= 4; wps *= 2) {  // waves per SIMD
            int blocks = 256 * wps;  // 256-thread blocks (4 waves = one per SIMD)
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                switch (kind) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, clk); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, clk); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, clk); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, clk); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters, clk); break;
                    default: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, iters, clk); break;
                }
                hipEventRecord(e1); hipEventSynchronize(e1);
            }
            float ms; hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
            double ghz = (double)hclk[0] / (hclk[1] / 100e6) / 1e9;
            double instr_per_simd = (double)iters * per_iter[kind] * wps;  // each SIMD runs wps waves
            double cycles = ms * 1e-3 * ghz * 1e9;
            printf("%-18s waves/SIMD=%d  %.3f ms  clk %.2f GHz  cycles per wave-instr per SIMD: %.2f\n", names[kind], wps, ms, ghz, cycles / instr_per_simd);
        }
    return 0;
}
