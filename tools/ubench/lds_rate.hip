// LDS instruction throughput per CU on gfx950, for the Huffman kernel's mix:
// conflict-free dword ops (lane l -> dword l of a 256-B row, rows varying), 4-wave
// workgroups, 3 resident per CU (as huffman_bits_kernel), every wave issuing the
// same op back to back.  Reports wave-instructions per CU per clock (s_memtime).
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result tools/ubench/lds_rate.hip -o tools/ubench/lds_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kRows = 64, kIters = 4096;
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int OP>
__global__ __launch_bounds__(256) void lds_op(unsigned *out, unsigned long long *clk) {
    __shared__ unsigned ctr[kRows * 64 * 4 / 4 + 4096];  // 16 KiB of rows + padding to 3 WGs per CU
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kRows * 64; i += 256) ctr[i] = 0;
    __syncthreads();
    unsigned acc = 0, inc = 1u << (8 * wv), keep = ~(0xFFu << (8 * wv));
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            unsigned *p = &ctr[((r * 4 + (i & 3)) & (kRows - 1)) * 64 + lane];
            if (OP == 0) __hip_atomic_fetch_add(p, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            if (OP == 1) acc += __hip_atomic_fetch_and(p, keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned *)p;
            if (OP == 2) asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(acc + r) : "memory");
            if (OP == 3) {
                unsigned x;
                asm volatile("ds_read_b32 %0, %1" : "=v"(x) : "v"(a) : "memory");
                acc ^= x;
            }
            if (OP == 4) acc += __hip_atomic_fetch_add(p, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            // 8- and 16-byte ops: lane l -> bytes 8l / 16l of a 512 / 1024-B row (conflict-free)
            const unsigned a8 = (unsigned)(((r * 4 + (i & 3)) & 15) * 1024 + lane * 8);
            const unsigned a16 = (unsigned)(((r * 4 + (i & 3)) & 15) * 1024 + lane * 16);
            if (OP == 5) asm volatile("ds_write_b64 %0, %1" ::"v"(a8), "v"(v2u{acc, (unsigned)r}) : "memory");
            if (OP == 6) asm volatile("ds_write_b128 %0, %1" ::"v"(a16), "v"(v4u{acc, (unsigned)r, acc, (unsigned)r}) : "memory");
            if (OP == 7) {
                v2u x;
                asm volatile("ds_read_b64 %0, %1" : "=v"(x) : "v"(a8) : "memory");
                acc ^= x[0];
            }
            if (OP == 8) {
                v4u x;
                asm volatile("ds_read_b128 %0, %1" : "=v"(x) : "v"(a16) : "memory");
                acc ^= x[0];
            }
        }
        if (OP == 3 || OP >= 7) __builtin_amdgcn_s_waitcnt(0xC07F);  // the asm reads' results (acc ^= x above is not ordered)
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = acc + ctr[lane];
}

template <int OP>
static void run(const char *name, int cus) {
    const int grid = cus * 3;
    unsigned *out;
    unsigned long long *clk;
    hipMalloc(&out, grid * 256 * 4);
    hipMalloc(&clk, grid * 8);
    hipLaunchKernelGGL(lds_op<OP>, dim3(grid), dim3(256), 0, 0, out, clk);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(lds_op<OP>, dim3(grid), dim3(256), 0, 0, out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double winst = (double)grid * 4 * kIters * 16;  // wave-instructions
    // s_memtime counts at 100 MHz on gfx9 parts; report per-CU rate against the event time
    printf("%-22s %8.3f ms  %.3f wave-instr per CU per ns  (%.2f ns each per CU)\n", name, ms,
           winst / cus / (ms * 1e6), (ms * 1e6) / (winst / cus));
    hipFree(out);
    hipFree(clk);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d, 3 workgroups x 4 waves per CU, %d x 16 ops per wave\n", cus, kIters);
    run<0>("ds_add_u32", cus);
    run<1>("ds_and_rtn_b32", cus);
    run<2>("ds_write_b32", cus);
    run<3>("ds_read_b32", cus);
    run<4>("ds_add_rtn_u32", cus);
    run<5>("ds_write_b64", cus);
    run<6>("ds_write_b128", cus);
    run<7>("ds_read_b64", cus);
    run<8>("ds_read_b128", cus);
    return 0;
}
