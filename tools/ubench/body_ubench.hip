// Diagnostic: cost of candidate fast-path loop bodies (SIMD cycles per wave per channel-sample)
// in the real kernel's shape: 16 packed I/Q int64 accumulators per lane, a uniform channel loop
// over 12 channels with line parameters in SGPRs, 16 unrolled 64-sample steps, LDS LUT reads and
// 64-bit scalar chip windows.  Variants:
//   cur   : X,Z 64-bit lines (2^-64 cycle, 2^-50 chip), chip = Z>>50, t = W>>chip,
//           y = (t<<31) + X_hi, addr = (y>>21)&0x7FC, 512-entry LUT     (round-1 kernel)
//   alb   : X 32-bit (2^-32 cycle), Z 64-bit with 32 fraction bits (hi word = chip), t = W>>Z_hi,
//           addr = alignbit(t, X, 21) & 0xFFC into a 1024-entry LUT (second half negated)
//   cnd   : as alb but the chip sign selects the signed gain with v_cndmask (sign mask from
//           v_cmp on t), LUT address from X alone
//   sdw   : X 32-bit, code C 32-bit 8.24 (byte 3 = chip mod 256), one rotated 32-bit window per
//           step in an SGPR (scalar running byte offset, 2 SALU per step), t = W >> byte3(C) by
//           SDWA, addr = alignbit(t, X, 21) & M with M, dX, dC, g in VGPRs (all-VGPR VOP2 forms)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define NSTEP 16
/* scalar buffer load with an SGPR byte offset (SMEM), seen by the compiler's lgkmcnt tracking */
typedef int gss_v4i __attribute__((ext_vector_type(4)));
extern "C" __device__ int gss_s_buffer_load_i32(gss_v4i, int, int)
    __asm("llvm.amdgcn.s.buffer.load.i32");
__device__ inline gss_v4i gss_rsrc(const void *p, uint32_t bytes)
{
    const uint64_t a = (uint64_t)p;
    gss_v4i r = {(int)(uint32_t)a, (int)(uint32_t)(a >> 32) & 0xFFFF, (int)bytes, 0x00020000};
    return r;
}
#define NCH 12

template <int V>
__global__ __launch_bounds__(256) void body(const uint64_t *__restrict__ tab, const uint64_t *prm,
                                            int64_t *out, int chunks)
{
    __shared__ int32_t lut[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) lut[i] = (i * 2654435761u) >> 8;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int64_t acc[NSTEP];
#pragma unroll
    for (int s = 0; s < NSTEP; s++) acc[s] = 0;
    for (int c = 0; c < chunks; c++) {
        for (int k = 0; k < NCH; k++) {
            const uint64_t xs = prm[4 * k + 0] + c, zs = prm[4 * k + 1];
            const uint64_t x0 = prm[4 * k + 2] * c, z0 = prm[4 * k + 3] + (uint64_t)c * 977;
            const int g = (int)(prm[4 * k] & 127) + 1;
            const uint64_t *T = tab + (k & 31) * 3136;
            if (V == 0) {
                uint64_t X = x0 + lane * xs, Z = z0 + lane * zs;
                const uint64_t dX = xs << 6, dZ = zs << 6;
                const uint32_t Zh = (uint32_t)(Z >> 32), dZh = (uint32_t)((dZ << 1) >> 32);
#pragma unroll
                for (int s = 0; s < NSTEP; s += 2) {
                    const uint64_t W = T[((Zh + (uint32_t)(s / 2) * dZh) >> 18) & 2047];
#pragma unroll
                    for (int ss = 0; ss < 2; ss++) {
                        const uint32_t ci = (uint32_t)(Z >> 50);
                        const uint32_t t = (uint32_t)(W >> (ci & 63));
                        const uint32_t y = (t << 31) + (uint32_t)(X >> 32);
                        const int32_t e = *(const int32_t *)((const char *)lut + ((y >> 21) & 0x7FCu));
                        acc[s + ss] += (int64_t)g * e;
                        X += dX; Z += dZ;
                    }
                }
            } else if (V == 3) {
                uint32_t X = (uint32_t)((x0 + lane * xs) >> 32);
                uint32_t C = (uint32_t)((z0 + lane * zs) >> 26);
                uint32_t dX = (uint32_t)((xs << 6) >> 32), dC = (uint32_t)((zs << 6) >> 26);
                uint32_t M = 0xFFCu;
                int gv = g;
                asm volatile("" : "+v"(dX), "+v"(dC), "+v"(M), "+v"(gv));
                const gss_v4i rs = gss_rsrc(T, 3136 * 8);
                uint32_t Qb = (uint32_t)__builtin_amdgcn_readfirstlane(C >> 20) & 0x3ffcu;
                const uint32_t dq = __builtin_amdgcn_readfirstlane((uint32_t)((zs << 6) >> 46));
                uint32_t W[NSTEP];
#pragma unroll
                for (int s = 0; s < NSTEP; s++) {
                    W[s] = (uint32_t)gss_s_buffer_load_i32(rs, (int)Qb, 0);
                    Qb += dq;
                }
#pragma unroll
                for (int s = 0; s < NSTEP; s++) {
                    uint32_t t;
                    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD "
                        "src0_sel:BYTE_3 src1_sel:DWORD" : "=v"(t) : "v"(C), "s"(W[s]));
                    const uint32_t a = __builtin_amdgcn_alignbit(t, X, 21) & M;
                    const int32_t e = *(const int32_t *)((const char *)lut + a);
                    acc[s] += (int64_t)gv * e;
                    X += dX; C += dC;
                }
            } else {
                uint32_t X = (uint32_t)((x0 + lane * xs) >> 32);
                uint64_t Z = (z0 + lane * zs) >> 18;
                const uint32_t dX = (uint32_t)((xs << 6) >> 32);
                const uint64_t dZ = (zs << 6) >> 18;
                const uint32_t Zh = (uint32_t)(__builtin_amdgcn_readfirstlane((uint32_t)(Z >> 32)));
                const uint32_t dZh = (uint32_t)((dZ << 1) >> 32);
#pragma unroll
                for (int s = 0; s < NSTEP; s += 2) {
                    const uint64_t W = T[(Zh + (uint32_t)(s / 2) * dZh) & 2047];
#pragma unroll
                    for (int ss = 0; ss < 2; ss++) {
                        const uint32_t zh = (uint32_t)(Z >> 32);
                        if (V == 1) {
                            const uint32_t t = (uint32_t)(W >> (zh & 63));
                            const uint32_t a = __builtin_amdgcn_alignbit(t, X, 21) & 0xFFCu;
                            const int32_t e = *(const int32_t *)((const char *)lut + a);
                            acc[s + ss] += (int64_t)g * e;
                        } else {
                            const uint32_t t = (uint32_t)(W >> (zh & 63));
                            const int32_t e = *(const int32_t *)((const char *)lut + ((X >> 21) & 0x7FCu));
                            const int gs = (t & 1) ? -g : g;
                            acc[s + ss] += (int64_t)gs * e;
                        }
                        X += dX; Z += dZ;
                    }
                }
            }
        }
    }
    int64_t r = 0;
#pragma unroll
    for (int s = 0; s < NSTEP; s++) r ^= acc[s];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main()
{
    uint64_t *tab, *prm; int64_t *out;
    (void)hipMalloc(&tab, 32 * 3136 * 8); (void)hipMemset(tab, 0x5a, 32 * 3136 * 8);
    uint64_t hp[4 * NCH];
    for (int k = 0; k < NCH; k++) {
        hp[4 * k] = 0x0002f3a1c0000000ull + k * 12345; hp[4 * k + 1] = 0x0000631234567890ull + k;
        hp[4 * k + 2] = 0x123456789abcdefull * (k + 1); hp[4 * k + 3] = (uint64_t)k << 52;
    }
    (void)hipMalloc(&prm, sizeof hp); (void)hipMemcpy(prm, hp, sizeof hp, hipMemcpyHostToDevice);
    const int grid = 256 * 8 * 4;       /* 8 waves/SIMD resident x 4 rounds */
    (void)hipMalloc(&out, (size_t)grid * 256 * 8);
    const int chunks = 32;
    const char *names[] = {"cur", "alb", "cnd", "sdw"};
    for (int v = 0; v < 4; v++) {
        void (*f)(const uint64_t *, const uint64_t *, int64_t *, int) =
            v == 0 ? body<0> : v == 1 ? body<1> : v == 2 ? body<2> : body<3>;
        hipLaunchKernelGGL(f, grid, 256, 0, 0, tab, prm, out, chunks);
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        for (int r = 0; r < 3; r++) hipLaunchKernelGGL(f, grid, 256, 0, 0, tab, prm, out, chunks);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 3;
        const double wave_cs = (double)grid * 4 * chunks * NCH * NSTEP;   /* wave-channel-samples */
        printf("%-4s %.3f ms  %.2f SIMD-cycles per wave-channel-sample (2.4 GHz), %.2f (2.0 GHz)\n",
               names[v], ms, ms * 1e-3 * 2.4e9 * 1024 / wave_cs, ms * 1e-3 * 2.0e9 * 1024 / wave_cs);
    }
    return 0;
}
