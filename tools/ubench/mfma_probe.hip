// Operand layout, exactness and issue cost of v_mfma_f32_4x4x4_16b_f16 on gfx950, for the
// fast path's MFMA accumulation (LIN_MFMA in gss_synth.hip).
//   layout: with A = row-distinct and B = column-distinct integers, checks the assumed mapping
//           lane 4b+i holds A_b[i][0..3], lane 4b+j holds B_b[0..3][j] and C_b[0..3][j];
//   exact:  integer f16 operands |a| <= 2048, |b| <= 250 summed into f32 near 1.5*2^23 stay exact;
//   cost:   loops of (4 VALU + 0.5 MFMA) against (5 VALU) per lane-step, cycles per wave-step.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/mfma_probe.hip -o tools/ubench/mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float float4_ __attribute__((ext_vector_type(4)));

__global__ void layout(const float *a, const float *b, float *c)
{
    const int l = threadIdx.x;
    half4 A, B;
    for (int k = 0; k < 4; k++) {
        A[k] = (_Float16)a[l * 4 + k];
        B[k] = (_Float16)b[l * 4 + k];
    }
    float4_ C = {0, 0, 0, 0};
    C = __builtin_amdgcn_mfma_f32_4x4x4f16(A, B, C, 0, 0, 0);
    for (int r = 0; r < 4; r++)
        c[l * 4 + r] = C[r];
}

// the render loop's shape: per step an LDS LUT read at an address from the phase word, then
// (MFMA=0) v_mad_i64_i32 into a packed accumulator or (MFMA=1) one MFMA per two steps
template <int MFMA>
__global__ __launch_bounds__(256) void loop(uint32_t *out, int iters, uint64_t D)
{
    __shared__ uint32_t lut[1024];
    for (int i = threadIdx.x; i < 1024; i += 256)
        lut[i] = i * 0x00010001u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    /* lanes on consecutive samples: 0.001 cycle (0.5 cell) and 0.39 chip per sample */
    const uint64_t S1 = (4294967ull << 32) | 6543360u;
    uint64_t P = (uint64_t)lane * S1 + (uint64_t)blockIdx.x * 0x9E3779B97F4A7C15ull;
    uint32_t W = 0x5A5A1234u * (lane | 1), M = 0xFFCu;
    asm volatile("" : "+v"(M), "+v"(W));
    int64_t acc[16];
    float4_ cq[8];
    for (int s = 0; s < 16; s++) acc[s] = 0;
    for (int s = 0; s < 8; s++) cq[s] = float4_{0, 0, 0, 0};
    half4 A = {(_Float16)(lane & 3), (_Float16)1, (_Float16)0, (_Float16)2};
    int g = lane + 3;
    for (int it = 0; it < iters; it++) {
        uint32_t e[16];
#pragma unroll
        for (int s = 0; s < 16; s++) {
            uint32_t t;
            asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 "
                "src1_sel:DWORD" : "=v"(t) : "v"((uint32_t)P), "v"(W));
            const uint32_t a = __builtin_amdgcn_alignbit(t, (uint32_t)(P >> 32), 21) & M;
            e[s] = *(const uint32_t *)((const char *)lut + a);
            if (!MFMA) {
                acc[s] += (int64_t)g * (int64_t)(int32_t)e[s];
            } else if (s & 1) {
                half4 B;
                uint32_t bb[2] = {e[s - 1], e[s]};
                memcpy(&B, bb, 8);
                cq[s / 2] = __builtin_amdgcn_mfma_f32_4x4x4f16(A, B, cq[s / 2], 0, 0, 0);
            }
            P += D;
            asm volatile("" : "+v"(P));       /* one 64-bit add per step, as the kernel */
        }
    }
    uint32_t x = 0;
    for (int s = 0; s < 16; s++) x ^= (uint32_t)acc[s];
    for (int s = 0; s < 8; s++) x ^= __float_as_uint(cq[s][0] + cq[s][1] + cq[s][2] + cq[s][3]);
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

int main()
{
    // ---- layout ----
    float ha[256], hb[256], hc[256];
    for (int l = 0; l < 64; l++)
        for (int k = 0; k < 4; k++) {
            ha[l * 4 + k] = (float)((l % 4) * 4 + k + 1) * ((l / 4) % 2 ? -1 : 1);   // A_b[i][k]
            hb[l * 4 + k] = (float)(k * 37 + (l % 4) * 5 + (l / 4));                  // B_b[k][j]
        }
    float *da, *db, *dc;
    hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dc, sizeof hc);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    layout<<<1, 64>>>(da, db, dc);
    hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < 16; b++)
        for (int j = 0; j < 4; j++)
            for (int i = 0; i < 4; i++) {
                float want = 0;
                for (int k = 0; k < 4; k++)
                    want += ha[(4 * b + i) * 4 + k] * hb[(4 * b + j) * 4 + k];
                float got = hc[(4 * b + j) * 4 + i];
                if (got != want && bad++ < 5)
                    printf("layout mismatch b%d i%d j%d: got %g want %g\n", b, i, j, got, want);
            }
    printf("layout %s (lane 4b+i: A row i; lane 4b+j: B column j, C column j rows 0..3)\n",
           bad ? "WRONG" : "OK");
    // ---- exactness: 1.5*2^23 + 64 plus 16 channels of +-2048 x +-250 ----
    {
        float a2[256], b2[256];
        for (int l = 0; l < 64; l++)
            for (int k = 0; k < 4; k++) {
                a2[l * 4 + k] = (float)(((l * 7 + k * 13) % 4097) - 2048);
                b2[l * 4 + k] = (float)(((l * 11 + k * 29) % 501) - 250);
            }
        hipMemcpy(da, a2, sizeof a2, hipMemcpyHostToDevice);
        hipMemcpy(db, b2, sizeof b2, hipMemcpyHostToDevice);
        layout<<<1, 64>>>(da, db, dc);
        hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
        int bad2 = 0;
        for (int b = 0; b < 16; b++)
            for (int j = 0; j < 4; j++)
                for (int i = 0; i < 4; i++) {
                    long long want = 0;
                    for (int k = 0; k < 4; k++)
                        want += (long long)a2[(4 * b + i) * 4 + k] * (long long)b2[(4 * b + j) * 4 + k];
                    if ((long long)hc[(4 * b + j) * 4 + i] != want) bad2++;
                }
        printf("exact integer products/sums: %s\n", bad2 ? "NO" : "yes");
    }
    // ---- cost ----
    uint32_t *dout;
    const int grid = 256 * 16, iters = 256;
    hipMalloc(&dout, (size_t)grid * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++)
        for (int m = 0; m < 2; m++) {
            hipEventRecord(e0);
            if (m) loop<1><<<grid, 256>>>(dout, iters, 64 * ((4294967ull << 32) | 6543360u));
            else loop<0><<<grid, 256>>>(dout, iters, 64 * ((4294967ull << 32) | 6543360u));
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double wave_steps = (double)grid * 4 * iters * 16;
            printf("%s: %.3f ms, %.2f cycles/wave-step per SIMD at 2.4 GHz\n",
                   m ? "mfma (4 VALU + LDS + 0.5 mfma)" : "mad  (5 VALU + LDS)", ms,
                   ms * 1e-3 * 2.4e9 * 1024 / wave_steps);
        }
    return 0;
}
