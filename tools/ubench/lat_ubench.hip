// Diagnostic: dependent-chain latency (cycles) of single VALU ops on gfx950, one wave alone,
// measured with s_memtime around 256 dependent instructions (inline asm keeps the chain intact).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP16(x) x x x x x x x x x x x x x x x x
#define CHAIN(name, setup, body)                                                              \
__global__ void k_##name(double *io, long long *cyc) {                                       \
    double d = io[threadIdx.x]; unsigned u = (unsigned)threadIdx.x; int e = 3;               \
    setup;                                                                                   \
    long long t0 = __builtin_amdgcn_s_memtime();                                              \
    REP16(REP16(body))                                                                       \
    long long t1 = __builtin_amdgcn_s_memtime();                                              \
    io[threadIdx.x] = d + u + e; if (threadIdx.x == 0) *cyc = t1 - t0; }

CHAIN(add_f64, , asm volatile("v_add_f64 %0, %0, %0" : "+v"(d));)
CHAIN(fma_f64, , asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d));)
CHAIN(mul_f64, , asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d));)
CHAIN(ldexp_f64, , asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d) : "v"(e));)
CHAIN(floor_f64, , asm volatile("v_floor_f64 %0, %0" : "+v"(d));)
CHAIN(fract_f64, , asm volatile("v_fract_f64 %0, %0" : "+v"(d));)
CHAIN(rndne_f64, , asm volatile("v_rndne_f64 %0, %0" : "+v"(d));)
CHAIN(frexp_exp, , asm volatile("v_frexp_exp_i32_f64 %0, %1\n v_cvt_f64_i32 %1, %0" : "+v"(e), "+v"(d));)
CHAIN(cvt_i32_f64, , asm volatile("v_cvt_i32_f64 %0, %1\n v_cvt_f64_i32 %1, %0" : "+v"(e), "+v"(d));)
CHAIN(add_u32, , asm volatile("v_add_u32 %0, %0, %0" : "+v"(u));)
CHAIN(and_or_b32, , asm volatile("v_and_or_b32 %0, %0, %0, %0" : "+v"(u));)
CHAIN(lshl_add_u32, , asm volatile("v_lshl_add_u32 %0, %0, 2, %0" : "+v"(u));)
CHAIN(dot2c, , asm volatile("v_dot2c_i32_i16 %0, %0, %0" : "+v"(u));)
CHAIN(mad_i64_i32, unsigned long long a64 = u, asm volatile("v_mad_i64_i32 %0, vcc, %1, %1, %0" : "+v"(a64) : "v"(u) : "vcc"); u += (unsigned)a64;)
CHAIN(cmp_cnd_u32, , asm volatile("v_cmp_lt_u32 vcc, %0, 5\n v_cndmask_b32 %0, %0, 0, vcc" : "+v"(u) :: "vcc");)

#define RUN(name, n) { hipLaunchKernelGGL(k_##name, 1, 64, 0, 0, io, cyc); hipLaunchKernelGGL(k_##name, 1, 64, 0, 0, io, cyc); \
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost); printf("%-14s %6.1f cycles/op (s_memtime units)\n", #name, c / (256.0 * n)); }

int main() {
    double *io; long long *cyc;
    (void)hipMalloc(&io, 64 * sizeof(double)); (void)hipMalloc(&cyc, 8);
    double h[64]; for (int i = 0; i < 64; i++) h[i] = 1.0 + i * 1e-3;
    (void)hipMemcpy(io, h, sizeof h, hipMemcpyHostToDevice);
    RUN(add_f64, 1) RUN(fma_f64, 1) RUN(mul_f64, 1) RUN(ldexp_f64, 1) RUN(floor_f64, 1) RUN(fract_f64, 1)
    RUN(rndne_f64, 1) RUN(frexp_exp, 2) RUN(cvt_i32_f64, 2) RUN(add_u32, 1) RUN(and_or_b32, 1)
    RUN(lshl_add_u32, 1) RUN(dot2c, 1) RUN(mad_i64_i32, 2) RUN(cmp_cnd_u32, 2)
    return 0;
}
