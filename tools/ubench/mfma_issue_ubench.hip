// Diagnostic: what an MFMA costs the VALU stream it is interleaved with, for the two shapes the
// fast path can accumulate on: v_mfma_f32_4x4x4_16b_f16 (one per two channel-steps per lane) and
// v_mfma_f32_16x16x32_f16 (one per four channel-steps: 8 f16 of B per lane).  Each body issues
// V VALU adds (8 independent chains) and M MFMAs rotating over 8 independent accumulators, so no
// MFMA waits on its own previous result.  Reported: SIMD cycles per body (wall time x 2.4 GHz /
// (waves per SIMD x bodies per wave)) at 2, 4 and 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef float f4_t __attribute__((ext_vector_type(4)));
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));

#define ADD(i) "v_add_u32 %" #i ", %" #i ", %24\n"
#define ADD8 ADD(0) ADD(1) ADD(2) ADD(3) ADD(4) ADD(5) ADD(6) ADD(7)
/* operand numbering: 0-7 u[], 8-15 acc[], 16-17 a4/b4 (h4), 18-19 a8/b8 (h8), 20-23 spare, 24 sc */
#define M4(c) "v_mfma_f32_4x4x4_16b_f16 %" #c ", %16, %17, %" #c "\n"
#define M16(c) "v_mfma_f32_16x16x32_f16 %" #c ", %18, %19, %" #c "\n"

#define KERN(name, body)                                                                       \
__global__ __launch_bounds__(256) void k_##name(uint32_t *io, long long *cyc) {               \
    uint32_t u[8]; f4_t acc[8];                                                               \
    const uint32_t s0 = io[threadIdx.x];                                                      \
    _Pragma("unroll") for (int i = 0; i < 8; i++) { u[i] = s0 + i;                            \
        acc[i] = f4_t{(float)(s0 & 7), 1.f, 2.f, (float)i}; }                                 \
    h4_t a4 = {(_Float16)1, (_Float16)2, (_Float16)(s0 & 3), (_Float16)0};                    \
    h4_t b4 = {(_Float16)3, (_Float16)(s0 & 1), (_Float16)1, (_Float16)2};                    \
    h8_t a8, b8;                                                                              \
    _Pragma("unroll") for (int i = 0; i < 8; i++) { a8[i] = (_Float16)(i + (s0 & 1));         \
        b8[i] = (_Float16)(3 - i); }                                                          \
    const uint32_t sc = __builtin_amdgcn_readfirstlane(s0 * 3u + 1u);                         \
    for (int r = 0; r < 1024; r++) {                                                          \
        asm volatile(body                                                                     \
            : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]),         \
              "+v"(u[6]), "+v"(u[7]), "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), \
              "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7])                          \
            : "v"(a4), "v"(b4), "v"(a8), "v"(b8), "v"(0), "v"(0), "v"(0), "v"(0), "v"(sc));   \
    }                                                                                         \
    uint32_t s = 0;                                                                           \
    _Pragma("unroll") for (int i = 0; i < 8; i++) s += u[i] + (uint32_t)(acc[i][0] + acc[i][3]); \
    io[threadIdx.x] = s;                                                                      \
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = 0; }

/* 16 adds per body, with 0 / 2 / 4 / 8 4x4x4 MFMAs or 0 / 1 / 2 / 4 16x16x32 MFMAs */
KERN(v16, ADD8 ADD8)
KERN(v16_m4x2, ADD8 M4(8) ADD8 M4(9))
KERN(v16_m4x4, ADD(0) ADD(1) ADD(2) ADD(3) M4(8) ADD(4) ADD(5) ADD(6) ADD(7) M4(9)
               ADD(0) ADD(1) ADD(2) ADD(3) M4(10) ADD(4) ADD(5) ADD(6) ADD(7) M4(11))
KERN(v16_m4x8, ADD(0) ADD(1) M4(8) ADD(2) ADD(3) M4(9) ADD(4) ADD(5) M4(10) ADD(6) ADD(7) M4(11)
               ADD(0) ADD(1) M4(12) ADD(2) ADD(3) M4(13) ADD(4) ADD(5) M4(14) ADD(6) ADD(7) M4(15))
KERN(v16_m16x1, ADD8 M16(8) ADD8)
KERN(v16_m16x2, ADD8 M16(8) ADD8 M16(9))
KERN(v16_m16x4, ADD(0) ADD(1) ADD(2) ADD(3) M16(8) ADD(4) ADD(5) ADD(6) ADD(7) M16(9)
                ADD(0) ADD(1) ADD(2) ADD(3) M16(10) ADD(4) ADD(5) ADD(6) ADD(7) M16(11))
KERN(m4x8_only, M4(8) M4(9) M4(10) M4(11) M4(12) M4(13) M4(14) M4(15))
KERN(m16x8_only, M16(8) M16(9) M16(10) M16(11) M16(12) M16(13) M16(14) M16(15))

typedef void (*kfn)(uint32_t *, long long *);
static void run(const char *name, kfn f)
{
    static uint32_t *io = nullptr; static long long *cyc = nullptr;
    if (!io) { (void)hipMalloc(&io, 256 * 4); (void)hipMalloc(&cyc, 8); (void)hipMemset(io, 1, 1024); }
    printf("%-12s", name);
    for (int w = 2; w <= 8; w *= 2) {
        const int grid = 256 * w;                         /* w workgroups of 4 waves per CU */
        hipLaunchKernelGGL(f, grid, 256, 0, 0, io, cyc);
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        for (int r = 0; r < 8; r++) hipLaunchKernelGGL(f, grid, 256, 0, 0, io, cyc);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 8;
        printf("  w%d %7.2f", w, ms * 1e-3 * 2.4e9 / (w * 1024.0));
        (void)hipEventDestroy(a); (void)hipEventDestroy(b);
    }
    printf("   cycles per body\n");
}
#define RUN(n) run(#n, k_##n);
int main()
{
    printf("SIMD cycles per loop body (16 VALU adds + M MFMAs, 8 accumulators), wall @2.4 GHz\n");
    RUN(v16) RUN(v16_m4x2) RUN(v16_m4x4) RUN(v16_m4x8) RUN(v16_m16x1) RUN(v16_m16x2)
    RUN(v16_m16x4) RUN(m4x8_only) RUN(m16x8_only)
    return 0;
}
