"""Generate tools/ubench/intrate.hip: issue cost of integer VALU encodings on gfx950
(VOP2 e32 vs VOP3 e64 forms, selects, compares, bitfield ops) -- 8 independent
chains per wave, 4 waves/SIMD, s_memtime around the loop.
    python tools/ubench/gen_intrate.py && hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -o tools/ubench/intrate tools/ubench/intrate.hip"""
OPS = {
    "v_add_u32_e32":      "v_add_u32_e32 {d}, {a}, {d}",
    "v_sub_u32_e32":      "v_sub_u32_e32 {d}, {a}, {d}",
    "v_and_b32_e32":      "v_and_b32_e32 {d}, {a}, {d}",
    "v_or_b32_e32":       "v_or_b32_e32 {d}, {a}, {d}",
    "v_min_u32_e32":      "v_min_u32_e32 {d}, {a}, {d}",
    "v_max_u32_e32":      "v_max_u32_e32 {d}, {a}, {d}",
    "v_lshlrev_b32_e32":  "v_lshlrev_b32_e32 {d}, {a}, {d}",
    "v_lshrrev_b32_e32":  "v_lshrrev_b32_e32 {d}, {a}, {d}",
    "v_mul_u32_u24_e32":  "v_mul_u32_u24_e32 {d}, {a}, {d}",
    "v_cndmask_b32_e32":  "v_cndmask_b32_e32 {d}, {a}, {d}, vcc",
    "v_cndmask_b32_e64":  "v_cndmask_b32_e64 {d}, {a}, {d}, s[20:21]",
    "v_cmp_ne_u32_e32":   "v_cmp_ne_u32_e32 vcc, {a}, {d}",
    "v_cmp_ne_u32_e64":   "v_cmp_ne_u32_e64 s[20:21], {a}, {d}",
    "v_bfe_u32":          "v_bfe_u32 {d}, {d}, {a}, 1",
    "v_add3_u32":         "v_add3_u32 {d}, {a}, {d}, {a}",
    "v_lshl_add_u32":     "v_lshl_add_u32 {d}, {a}, 1, {d}",
    "v_and_or_b32":       "v_and_or_b32 {d}, {a}, {d}, {a}",
    "v_mad_u32_u24":      "v_mad_u32_u24 {d}, {a}, {d}, {a}",
    "v_perm_b32":         "v_perm_b32 {d}, {a}, {d}, {a}",
    "v_pk_add_u16":       "v_pk_add_u16 {d}, {a}, {d}",
    "v_pk_min_u16":       "v_pk_min_u16 {d}, {a}, {d}",
    "v_add_u32_e64":      "v_add_u32_e64 {d}, {a}, {d}",
    "v_min_u32_e64":      "v_min_u32_e64 {d}, {a}, {d}",
    "v_sad_u32":          "v_sad_u32 {d}, {a}, {d}, {a}",
    "v_med3_u32":         "v_med3_u32 {d}, {a}, {d}, {a}",
    "v_ffbl_b32":         "v_ffbl_b32_e32 {d}, {d}",
    "v_bcnt_u32_b32":     "v_bcnt_u32_b32 {d}, {d}, {a}",
    "v_subrev_u32_e32":   "v_subrev_u32_e32 {d}, {a}, {d}",
}
out = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <string.h>']
for i, (name, fmt) in enumerate(OPS.items()):
    chains = []
    for c in range(8):
        chains.append(fmt.format(d=f"%{c}", a=f"%{(c + 1) % 8}"))
    body = "\\n".join(chains)
    asm = (f'asm volatile("{body}" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) '
           f':: "vcc", "s20", "s21");')
    out.append(f'''__global__ __launch_bounds__(256) void k{i}(unsigned *out, int iters, unsigned long long *clk) {{
  unsigned a0=threadIdx.x,a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7;
  unsigned long long t0=__builtin_amdgcn_s_memtime();
  for (int i=0;i<iters;++i) {{ {asm} {asm} {asm} {asm} }}
  unsigned long long t1=__builtin_amdgcn_s_memtime();
  if (threadIdx.x==0) clk[blockIdx.x]=t1-t0;
  out[blockIdx.x*256+threadIdx.x]=a0^a1^a2^a3^a4^a5^a6^a7;
}}''')
names = list(OPS)
out.append('typedef void (*K)(unsigned*,int,unsigned long long*);')
out.append('K ks[] = {' + ','.join(f'k{i}' for i in range(len(names))) + '};')
out.append('const char *nm[] = {' + ','.join(f'"{n}"' for n in names) + '};')
out.append(f'''int main() {{
  int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
  int cus = p.multiProcessorCount, grid = cus * 4;  /* 16 waves per CU: 4 per SIMD */
  unsigned *o; unsigned long long *c; hipMalloc(&o, grid*256*4); hipMalloc(&c, grid*8);
  unsigned long long *h = (unsigned long long*)malloc(grid*8);
  const int iters = 2000, per = 32 * iters;  /* wave-instructions per wave */
  for (int k = 0; k < {len(names)}; ++k) {{
    for (int rep = 0; rep < 2; ++rep) {{
      hipLaunchKernelGGL(ks[k], dim3(grid), dim3(256), 0, 0, o, iters, c);
      hipDeviceSynchronize();
    }}
    hipMemcpy(h, c, grid*8, hipMemcpyDeviceToHost);
    double m = 0; for (int i = 0; i < grid; ++i) m += h[i]; m /= grid;
    /* s_memtime counts at the shader clock; 4 waves share a SIMD */
    printf("%-20s %6.2f cycles per wave-instruction per SIMD\\n", nm[k], m / per / 4.0);
  }}
  return 0;
}}''')
open("tools/ubench/intrate.hip", "w").write("\n".join(out) + "\n")
