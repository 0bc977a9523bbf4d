// tools/ubench/hbm_off.hip -- does the relative placement of the read front and
// the write front matter (DRAM bank/channel conflicts between the two streams)?
// The flat 1:2 stream (hbm_mix2 "s12 nt/plain WG4") with the output base moved by
// OFF bytes, and with the input traversed with a lead: the wave-batch order of
// the WRITES lags the reads by LAG batches of the whole grid.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/hbm_off tools/ubench/hbm_off.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int AUX>
__global__ __launch_bounds__(256) void k_s12(const u4v *__restrict__ in, char *__restrict__ out, uint32_t nb) {
    const int lane = threadIdx.x & 63;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += gridDim.x * 4) {
        u4v v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(in + (size_t)b * 256 + k * 64 + lane);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(out + (size_t)b * 8192, 0, 8192, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            __builtin_amdgcn_raw_buffer_store_b128(v[k], rc, lane * 16, k * 1024, AUX);
            __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ u4v{1, 0, 0, 0}, rc, lane * 16, (k + 4) * 1024, AUX);
        }
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 8;
    const size_t nblk = 12441600;
    const uint32_t nb = (uint32_t)(nblk / 64);
    const size_t in_bytes = nblk * 64, out_bytes = nblk * 128;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    char *src, *dst;
    const size_t slack = 64 << 20;
    CHECK(hipMalloc(&src, in_bytes));
    CHECK(hipMalloc(&dst, out_bytes + slack));
    CHECK(hipMemset(src, 7, in_bytes));
    CHECK(hipMemset(dst, 0, out_bytes + slack));
    printf("src %p dst %p\n", (void *)src, (void *)dst);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double b12 = (double)nblk * 192;
    const size_t offs[] = {0, 256, 1024, 4096, 8192, 16384, 65536, 262144, 1 << 20, 2 << 20, 3 << 20, 5 << 20, 8 << 20, 16 << 20, 33 << 20};
    for (int aux : {0, 2}) {
        for (size_t off : offs) {
            std::vector<float> v;
            for (int r = 0; r < reps + 1; ++r) {
                CHECK(hipEventRecord(e0));
                if (aux) hipLaunchKernelGGL((k_s12<2>), dim3(cus * 4), dim3(256), 0, 0, (const u4v *)src, dst + off, nb);
                else hipLaunchKernelGGL((k_s12<0>), dim3(cus * 4), dim3(256), 0, 0, (const u4v *)src, dst + off, nb);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float t;
                CHECK(hipEventElapsedTime(&t, e0, e1));
                if (r) v.push_back(t);
            }
            std::sort(v.begin(), v.end());
            printf("%s out offset %9zu  median %7.1f us %5.1f %%  best %5.1f %%\n", aux ? "nt   " : "plain", off,
                   v[v.size() / 2] * 1e3, b12 / v[v.size() / 2] / 1e6 / 80.0, b12 / v[0] / 1e6 / 80.0);
        }
    }
    return 0;
}
