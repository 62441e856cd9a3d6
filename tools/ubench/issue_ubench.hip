// Diagnostic: VALU issue cost (SIMD cycles per wave-instruction) of the candidate ops for the
// fast-path render loop, at 1, 2, 4 and 8 waves per SIMD, plus whole candidate loop bodies.
// Each wave runs 64 x 8 independent instructions (8 chains).  Cycles = wall time x 2.4 GHz
// (MI355X peak clock) / (waves per SIMD x instructions per wave); the s_memtime column is the
// same from the wave's own clock (absolute, for the clock actually reached).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP8(x) x x x x x x x x
#define K8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)

// one kernel per op: u[8] 32-bit and d[8] 64-bit registers, all live
#define KERN(name, body)                                                                       \
__global__ __launch_bounds__(256) void k_##name(uint32_t *io, long long *cyc) {               \
    uint32_t u[8]; uint64_t d[8]; float f[8][2];                                              \
    const uint32_t s0 = io[threadIdx.x];                                                      \
    _Pragma("unroll") for (int i = 0; i < 8; i++) {                                           \
        u[i] = s0 + i; d[i] = ((uint64_t)s0 << 20) + i; f[i][0] = (float)(s0 + i); f[i][1] = 1.f; }  \
    const uint32_t sc = __builtin_amdgcn_readfirstlane(s0 * 3u + 1u);                         \
    long long t0 = __builtin_amdgcn_s_memtime();                                              \
    for (int r = 0; r < 2048; r++) { body }                                                     \
    long long t1 = __builtin_amdgcn_s_memtime();                                              \
    uint32_t acc = 0;                                                                         \
    _Pragma("unroll") for (int i = 0; i < 8; i++) acc += u[i] + (uint32_t)d[i] + (uint32_t)(d[i] >> 32) + (uint32_t)f[i][0] + (uint32_t)f[i][1]; \
    io[threadIdx.x] = acc;                                                                    \
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0; }

#define V(i) "v"(u[i])
#define OP_U(ins) \
    asm volatile(ins " %0, %0, %8\n" ins " %1, %1, %8\n" ins " %2, %2, %8\n" ins " %3, %3, %8\n" \
                 ins " %4, %4, %8\n" ins " %5, %5, %8\n" ins " %6, %6, %8\n" ins " %7, %7, %8"   \
                 : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]),       \
                   "+v"(u[6]), "+v"(u[7]) : "v"(sc));
#define OP_U3(ins, c) \
    asm volatile(ins " %0, %0, %8, " c "\n" ins " %1, %1, %8, " c "\n" ins " %2, %2, %8, " c "\n" \
                 ins " %3, %3, %8, " c "\n" ins " %4, %4, %8, " c "\n" ins " %5, %5, %8, " c "\n" \
                 ins " %6, %6, %8, " c "\n" ins " %7, %7, %8, " c                                \
                 : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]),       \
                   "+v"(u[6]), "+v"(u[7]) : "v"(sc));

KERN(add_u32, OP_U("v_add_u32"))
KERN(and_b32, OP_U("v_and_b32"))
KERN(xor_b32, OP_U("v_xor_b32"))
KERN(lshrrev_b32, OP_U("v_lshrrev_b32"))
KERN(mul_u32_u24, OP_U("v_mul_u32_u24"))
KERN(add_f32, OP_U("v_add_f32"))
KERN(alignbit, OP_U3("v_alignbit_b32", "21"))
KERN(bfe_u32, OP_U3("v_bfe_u32", "1"))
KERN(and_or, OP_U3("v_and_or_b32", "%8"))
KERN(lshl_add_u32, OP_U3("v_lshl_add_u32", "3"))
KERN(perm_b32, OP_U3("v_perm_b32", "%8"))
KERN(add3_u32, OP_U3("v_add3_u32", "%8"))
KERN(lshl_add_u64,
     asm volatile("v_lshl_add_u64 %0, %0, 0, %8\n v_lshl_add_u64 %1, %1, 0, %8\n v_lshl_add_u64 %2, %2, 0, %8\n v_lshl_add_u64 %3, %3, 0, %8\n v_lshl_add_u64 %4, %4, 0, %8\n v_lshl_add_u64 %5, %5, 0, %8\n v_lshl_add_u64 %6, %6, 0, %8\n v_lshl_add_u64 %7, %7, 0, %8"
                  : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]) : "v"(d[0]));)
KERN(add_co_pair,
     asm volatile("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %9, vcc\n v_add_co_u32 %2, vcc, %2, %8\n v_addc_co_u32 %3, vcc, %3, %9, vcc\n v_add_co_u32 %4, vcc, %4, %8\n v_addc_co_u32 %5, vcc, %5, %9, vcc\n v_add_co_u32 %6, vcc, %6, %8\n v_addc_co_u32 %7, vcc, %7, %9, vcc"
                  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(sc), "v"(u[0]) : "vcc");)
KERN(lshrrev_b64,
     asm volatile("v_lshrrev_b64 %0, %8, %0\n v_lshrrev_b64 %1, %8, %1\n v_lshrrev_b64 %2, %8, %2\n v_lshrrev_b64 %3, %8, %3\n v_lshrrev_b64 %4, %8, %4\n v_lshrrev_b64 %5, %8, %5\n v_lshrrev_b64 %6, %8, %6\n v_lshrrev_b64 %7, %8, %7"
                  : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]) : "v"(u[0]));)
KERN(mad_i64_i32,
     asm volatile("v_mad_i64_i32 %0, vcc, %8, %8, %0\n v_mad_i64_i32 %1, vcc, %8, %8, %1\n v_mad_i64_i32 %2, vcc, %8, %8, %2\n v_mad_i64_i32 %3, vcc, %8, %8, %3\n v_mad_i64_i32 %4, vcc, %8, %8, %4\n v_mad_i64_i32 %5, vcc, %8, %8, %5\n v_mad_i64_i32 %6, vcc, %8, %8, %6\n v_mad_i64_i32 %7, vcc, %8, %8, %7"
                  : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]) : "v"(u[0]) : "vcc");)
KERN(mad_u32_u24,
     asm volatile("v_mad_u32_u24 %0, %8, %8, %0\n v_mad_u32_u24 %1, %8, %8, %1\n v_mad_u32_u24 %2, %8, %8, %2\n v_mad_u32_u24 %3, %8, %8, %3\n v_mad_u32_u24 %4, %8, %8, %4\n v_mad_u32_u24 %5, %8, %8, %5\n v_mad_u32_u24 %6, %8, %8, %6\n v_mad_u32_u24 %7, %8, %8, %7"
                  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(sc));)
KERN(pk_add_f32,
     asm volatile("v_pk_add_f32 %0, %0, %8\n v_pk_add_f32 %1, %1, %8\n v_pk_add_f32 %2, %2, %8\n v_pk_add_f32 %3, %3, %8\n v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %5, %5, %8\n v_pk_add_f32 %6, %6, %8\n v_pk_add_f32 %7, %7, %8"
                  : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]) : "v"(d[0]));)
KERN(dot2_i32_i16,
     asm volatile("v_dot2_i32_i16 %0, %8, %8, %0\n v_dot2_i32_i16 %1, %8, %8, %1\n v_dot2_i32_i16 %2, %8, %8, %2\n v_dot2_i32_i16 %3, %8, %8, %3\n v_dot2_i32_i16 %4, %8, %8, %4\n v_dot2_i32_i16 %5, %8, %8, %5\n v_dot2_i32_i16 %6, %8, %8, %6\n v_dot2_i32_i16 %7, %8, %8, %7"
                  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(sc));)
KERN(cndmask,
     asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(sc) : "vcc");)
// a VOP2 and a 64-bit op alternating (do different op classes overlap?)
KERN(mix_add_mad,
     asm volatile("v_add_u32 %0, %0, %10\n v_mad_i64_i32 %4, vcc, %10, %10, %4\n v_add_u32 %1, %1, %10\n v_mad_i64_i32 %5, vcc, %10, %10, %5\n v_add_u32 %2, %2, %10\n v_mad_i64_i32 %6, vcc, %10, %10, %6\n v_add_u32 %3, %3, %10\n v_mad_i64_i32 %7, vcc, %10, %10, %7"
                  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]) : "v"(u[4]), "v"(u[5]), "v"(sc) : "vcc");)


// round 3 candidates: a 32-bit window shift taking the chip from byte 3 of a 32-bit code
// accumulator (SDWA), shifts with the value in an SGPR, VOP2 carry adds, dot2c, MFMA issue cost
#define OP_S(fmt) \
    asm volatile(fmt(0) "\n" fmt(1) "\n" fmt(2) "\n" fmt(3) "\n" fmt(4) "\n" fmt(5) "\n" fmt(6) "\n" fmt(7) \
                 : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]),       \
                   "+v"(u[6]), "+v"(u[7]) : "s"(sc));
#define F_LSHR_E64(i) "v_lshrrev_b32_e64 %" #i ", %" #i ", %8"
#define F_LSHR_SDWA(i) "v_lshrrev_b32_sdwa %" #i ", %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
#define F_ADD_SDWA(i) "v_add_u32_sdwa %" #i ", %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
#define F_ADDCO(i) "v_add_co_u32 %" #i ", vcc, %8, %" #i
#define F_DOT2C(i) "v_dot2c_f32_f16 %" #i ", %8, %" #i
#define F_ALIGN_S(i) "v_alignbit_b32 %" #i ", %8, %" #i ", 21"
KERN(lshr_e64_s, OP_S(F_LSHR_E64))
KERN(lshr_sdwa_s, OP_S(F_LSHR_SDWA))
KERN(add_sdwa_s, OP_S(F_ADD_SDWA))
KERN(add_co_vop2, asm volatile(F_ADDCO(0) "\n" F_ADDCO(1) "\n" F_ADDCO(2) "\n" F_ADDCO(3) "\n" F_ADDCO(4) "\n" F_ADDCO(5) "\n" F_ADDCO(6) "\n" F_ADDCO(7)
                          : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "s"(sc) : "vcc");)
KERN(dot2c_f32_f16, asm volatile(F_DOT2C(0) "\n" F_DOT2C(1) "\n" F_DOT2C(2) "\n" F_DOT2C(3) "\n" F_DOT2C(4) "\n" F_DOT2C(5) "\n" F_DOT2C(6) "\n" F_DOT2C(7)
                            : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(sc));)
KERN(alignbit_s, OP_S(F_ALIGN_S))
KERN(lshrrev_b64_s,
     asm volatile("v_lshrrev_b64 %0, %8, %16\n v_lshrrev_b64 %1, %9, %16\n v_lshrrev_b64 %2, %10, %16\n v_lshrrev_b64 %3, %11, %16\n v_lshrrev_b64 %4, %12, %16\n v_lshrrev_b64 %5, %13, %16\n v_lshrrev_b64 %6, %14, %16\n v_lshrrev_b64 %7, %15, %16"
                  : "=v"(d[0]), "=v"(d[1]), "=v"(d[2]), "=v"(d[3]), "=v"(d[4]), "=v"(d[5]), "=v"(d[6]), "=v"(d[7])
                  : "v"(u[0]), "v"(u[1]), "v"(u[2]), "v"(u[3]), "v"(u[4]), "v"(u[5]), "v"(u[6]), "v"(u[7]), "s"((uint64_t)sc * 7u));
     _Pragma("unroll") for (int i = 0; i < 8; i++) u[i] ^= (uint32_t)d[i];)
KERN(mov_b64,
     asm volatile("v_mov_b64 %0, %8\n v_mov_b64 %1, %8\n v_mov_b64 %2, %8\n v_mov_b64 %3, %8\n v_mov_b64 %4, %8\n v_mov_b64 %5, %8\n v_mov_b64 %6, %8\n v_mov_b64 %7, %8"
                  : "=v"(d[0]), "=v"(d[1]), "=v"(d[2]), "=v"(d[3]), "=v"(d[4]), "=v"(d[5]), "=v"(d[6]), "=v"(d[7]) : "s"((uint64_t)sc * 5u));)
// 8 VOP2 adds plus 2 independent MFMA 4x4x4 (16 blocks) per group: the MFMAs' issue cost over add_u32
typedef float f4_t __attribute__((ext_vector_type(4)));
#define MFMA_BODY \
     f4_t a0 = {f[0][0], f[0][1], f[1][0], f[1][1]}; f4_t a1 = {f[2][0], f[2][1], f[3][0], f[3][1]}; \
     asm volatile("v_add_u32 %0, %0, %12\n v_mfma_f32_4x4x4_16b_f16 %8, %10, %11, %8\n v_add_u32 %1, %1, %12\n v_add_u32 %2, %2, %12\n v_add_u32 %3, %3, %12\n v_mfma_f32_4x4x4_16b_f16 %9, %11, %10, %9\n v_add_u32 %4, %4, %12\n v_add_u32 %5, %5, %12\n v_add_u32 %6, %6, %12\n v_add_u32 %7, %7, %12" \
                  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]), "+v"(a0), "+v"(a1) \
                  : "v"(d[0]), "v"(d[1]), "v"(sc)); \
     f[0][0] = a0[0] + a1[3]; f[1][1] = a0[2] + a1[1];
KERN(mix_add_mfma4, MFMA_BODY)

typedef void (*kfn)(uint32_t *, long long *);
static void run(const char *name, kfn f)
{
    static uint32_t *io = nullptr; static long long *cyc = nullptr;
    if (!io) { (void)hipMalloc(&io, 256 * 4); (void)hipMalloc(&cyc, 8); (void)hipMemset(io, 1, 1024); }
    printf("%-14s", name);
    for (int w = 1; w <= 8; w *= 2) {
        const int grid = 256 * w;                         /* w workgroups of 4 waves per CU */
        hipLaunchKernelGGL(f, grid, 256, 0, 0, io, cyc);
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        for (int r = 0; r < 4; r++) hipLaunchKernelGGL(f, grid, 256, 0, 0, io, cyc);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 4;
        long long c = 0; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        const double instr = 2048.0 * 8.0;                 /* per wave */
        printf("  w%d %5.2f (%5.2f)", w, ms * 1e-3 * 2.4e9 / (w * instr), (double)c / instr / w);
        (void)hipEventDestroy(a); (void)hipEventDestroy(b);
    }
    printf("\n");
}
#define RUN(n) run(#n, k_##n);
int main()
{
    printf("cycles per wave-instruction per SIMD at w waves/SIMD: wall@2.4GHz (s_memtime/w)\n");
    RUN(add_u32) RUN(and_b32) RUN(xor_b32) RUN(lshrrev_b32) RUN(mul_u32_u24) RUN(add_f32)
    RUN(alignbit) RUN(bfe_u32) RUN(and_or) RUN(lshl_add_u32) RUN(perm_b32) RUN(add3_u32)
    RUN(lshl_add_u64) RUN(add_co_pair) RUN(lshrrev_b64) RUN(mad_i64_i32) RUN(mad_u32_u24)
    RUN(pk_add_f32) RUN(dot2_i32_i16) RUN(cndmask) RUN(mix_add_mad)
    RUN(lshr_e64_s) RUN(lshr_sdwa_s) RUN(add_sdwa_s) RUN(add_co_vop2) RUN(dot2c_f32_f16)
    RUN(alignbit_s) RUN(lshrrev_b64_s) RUN(mov_b64) RUN(mix_add_mfma4)
    return 0;
}
