// Diagnostic: issue throughput (cycles per wave-instruction) of candidate VALU ops on gfx950,
// 8 independent chains per wave, 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define REP8(x) x x x x x x x x
#define TP(name, decl, body, use)                                                              \
__global__ __launch_bounds__(256) void t_##name(unsigned *io, long long *cyc) {               \
    unsigned u0 = io[threadIdx.x], u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4,        \
             u5 = u0 + 5, u6 = u0 + 6, u7 = u0 + 7; decl;                                      \
    long long t0 = __builtin_amdgcn_s_memtime();                                              \
    for (int r = 0; r < 64; r++) { REP8(body) }                                               \
    long long t1 = __builtin_amdgcn_s_memtime();                                              \
    io[threadIdx.x] = use; if (threadIdx.x == 0) *cyc = t1 - t0; }
TP(dot2c, , asm volatile("v_dot2c_i32_i16 %0, %8, %8\n v_dot2c_i32_i16 %1, %8, %8\n v_dot2c_i32_i16 %2, %8, %8\n v_dot2c_i32_i16 %3, %8, %8\n v_dot2c_i32_i16 %4, %8, %8\n v_dot2c_i32_i16 %5, %8, %8\n v_dot2c_i32_i16 %6, %8, %8\n v_dot2c_i32_i16 %7, %8, %8" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(u0));, u0+u1+u2+u3+u4+u5+u6+u7)
TP(mad_i64_i32, unsigned long long a0 = u0; unsigned long long a1 = u1; unsigned long long a2 = u2; unsigned long long a3 = u3; unsigned long long a4 = u4; unsigned long long a5 = u5; unsigned long long a6 = u6; unsigned long long a7 = u7,
   asm volatile("v_mad_i64_i32 %0, vcc, %8, %8, %0\n v_mad_i64_i32 %1, vcc, %8, %8, %1\n v_mad_i64_i32 %2, vcc, %8, %8, %2\n v_mad_i64_i32 %3, vcc, %8, %8, %3\n v_mad_i64_i32 %4, vcc, %8, %8, %4\n v_mad_i64_i32 %5, vcc, %8, %8, %5\n v_mad_i64_i32 %6, vcc, %8, %8, %6\n v_mad_i64_i32 %7, vcc, %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(u0) : "vcc");,
   (unsigned)(a0+a1+a2+a3+a4+a5+a6+a7))
TP(add_f64, double d0 = u0; double d1 = u1; double d2 = u2; double d3 = u3; double d4 = u4; double d5 = u5; double d6 = u6; double d7 = u7,
   asm volatile("v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "v"(d0));,
   (unsigned)(d0+d1+d2+d3+d4+d5+d6+d7))
TP(fract_f64, double d0 = u0; double d1 = u1; double d2 = u2; double d3 = u3; double d4 = u4; double d5 = u5; double d6 = u6; double d7 = u7,
   asm volatile("v_fract_f64 %0, %0\n v_fract_f64 %1, %1\n v_fract_f64 %2, %2\n v_fract_f64 %3, %3\n v_fract_f64 %4, %4\n v_fract_f64 %5, %5\n v_fract_f64 %6, %6\n v_fract_f64 %7, %7" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));,
   (unsigned)(d0+d1+d2+d3+d4+d5+d6+d7))
TP(cvt_i32_f64, double d0 = u0; int e0; int e1; int e2; int e3; int e4; int e5; int e6; int e7,
   asm volatile("v_cvt_i32_f64 %0, %8\n v_cvt_i32_f64 %1, %8\n v_cvt_i32_f64 %2, %8\n v_cvt_i32_f64 %3, %8\n v_cvt_i32_f64 %4, %8\n v_cvt_i32_f64 %5, %8\n v_cvt_i32_f64 %6, %8\n v_cvt_i32_f64 %7, %8" : "=v"(e0), "=v"(e1), "=v"(e2), "=v"(e3), "=v"(e4), "=v"(e5), "=v"(e6), "=v"(e7) : "v"(d0)); u0 += e0+e1+e2+e3+e4+e5+e6+e7;,
   u0)
TP(ldexp_f64, double d0 = u0; double d1 = u1; double d2 = u2; double d3 = u3; double d4 = u4; double d5 = u5; double d6 = u6; double d7 = u7,
   asm volatile("v_ldexp_f64 %0, %0, 1\n v_ldexp_f64 %1, %1, 1\n v_ldexp_f64 %2, %2, 1\n v_ldexp_f64 %3, %3, 1\n v_ldexp_f64 %4, %4, 1\n v_ldexp_f64 %5, %5, 1\n v_ldexp_f64 %6, %6, 1\n v_ldexp_f64 %7, %7, 1" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));,
   (unsigned)(d0+d1+d2+d3+d4+d5+d6+d7))
TP(add_u32, , asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(u0));, u0+u1+u2+u3+u4+u5+u6+u7)

TP(fma_f64, double d0 = u0; double d1 = u1; double d2 = u2; double d3 = u3; double d4 = u4; double d5 = u5; double d6 = u6; double d7 = u7,
   asm volatile("v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n v_fma_f64 %3, %3, %8, %8\n v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "v"(d0));,
   (unsigned)(d0+d1+d2+d3+d4+d5+d6+d7))
TP(add_f64_s, double d0 = u0; double d1 = u1; double d2 = u2; double d3 = u3; double d4 = u4; double d5 = u5; double d6 = u6; double d7 = u7; double sc = __builtin_amdgcn_readfirstlane(u0),
   asm volatile("v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "s"(sc));,
   (unsigned)(d0+d1+d2+d3+d4+d5+d6+d7))
TP(bfe_u32, , asm volatile("v_bfe_u32 %0, %0, %8, 1\n v_bfe_u32 %1, %1, %8, 1\n v_bfe_u32 %2, %2, %8, 1\n v_bfe_u32 %3, %3, %8, 1\n v_bfe_u32 %4, %4, %8, 1\n v_bfe_u32 %5, %5, %8, 1\n v_bfe_u32 %6, %6, %8, 1\n v_bfe_u32 %7, %7, %8, 1" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(u0));, u0+u1+u2+u3+u4+u5+u6+u7)
TP(lshl_add_u64, unsigned long long a0 = u0; unsigned long long a1 = u1; unsigned long long a2 = u2; unsigned long long a3 = u3; unsigned long long a4 = u4; unsigned long long a5 = u5; unsigned long long a6 = u6; unsigned long long a7 = u7,
   asm volatile("v_lshl_add_u64 %0, %0, 0, %8\n v_lshl_add_u64 %1, %1, 0, %8\n v_lshl_add_u64 %2, %2, 0, %8\n v_lshl_add_u64 %3, %3, 0, %8\n v_lshl_add_u64 %4, %4, 0, %8\n v_lshl_add_u64 %5, %5, 0, %8\n v_lshl_add_u64 %6, %6, 0, %8\n v_lshl_add_u64 %7, %7, 0, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(a0));,
   (unsigned)(a0+a1+a2+a3+a4+a5+a6+a7))
TP(cvt_u32_f64, double d0 = u0; unsigned e0; unsigned e1; unsigned e2; unsigned e3; unsigned e4; unsigned e5; unsigned e6; unsigned e7,
   asm volatile("v_cvt_u32_f64 %0, %8\n v_cvt_u32_f64 %1, %8\n v_cvt_u32_f64 %2, %8\n v_cvt_u32_f64 %3, %8\n v_cvt_u32_f64 %4, %8\n v_cvt_u32_f64 %5, %8\n v_cvt_u32_f64 %6, %8\n v_cvt_u32_f64 %7, %8" : "=v"(e0), "=v"(e1), "=v"(e2), "=v"(e3), "=v"(e4), "=v"(e5), "=v"(e6), "=v"(e7) : "v"(d0)); u0 += e0+e1+e2+e3+e4+e5+e6+e7;,
   u0)
TP(mix_f64_int, double d0 = u0; double d1 = u1; double d2 = u2; double d3 = u3,
   asm volatile("v_add_f64 %0, %0, %8\n v_add_u32 %4, %4, %9\n v_add_f64 %1, %1, %8\n v_add_u32 %5, %5, %9\n v_add_f64 %2, %2, %8\n v_add_u32 %6, %6, %9\n v_add_f64 %3, %3, %8\n v_add_u32 %7, %7, %9" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(d0), "v"(u0));,
   (unsigned)(d0+d1+d2+d3)+u4+u5+u6+u7)

#define RUN(name) { hipLaunchKernelGGL(t_##name, 1024, 256, 0, 0, io, cyc); hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b); \
  hipEventRecord(a); hipLaunchKernelGGL(t_##name, 1024, 256, 0, 0, io, cyc); hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); \
  /* 1024 WGs x 4 waves = 4096 waves = 4/SIMD; each wave issues 64*8*8 = 4096 instrs */ \
  printf("%-12s %.2f cycles/wave-instr per SIMD (at 2.4 GHz)\n", #name, ms * 1e-3 * 2.4e9 / (4.0 * 4096)); }
int main() {
    unsigned *io; long long *cyc;
    (void)hipMalloc(&io, 256 * 4); (void)hipMalloc(&cyc, 8); (void)hipMemset(io, 1, 1024);
    RUN(add_u32) RUN(add_f64) RUN(fract_f64) RUN(ldexp_f64) RUN(cvt_i32_f64) RUN(dot2c) RUN(mad_i64_i32) RUN(fma_f64) RUN(add_f64_s) RUN(bfe_u32) RUN(lshl_add_u64) RUN(cvt_u32_f64) RUN(mix_f64_int)
    return 0;
}
