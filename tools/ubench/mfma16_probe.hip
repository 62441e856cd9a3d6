// Operand layout and exactness of v_mfma_f32_16x16x32_f16 on gfx950, for the fast path's
// channel-pair accumulation (gss_synth.hip, LIN_MFMA 2).
//   layout: random small integer A, B placed by the assumed map (lane l holds A[l&15][8(l>>4)+j]
//           and B[8(l>>4)+j][l&15], j = 0..7; C[4(l>>4)+r][l&15], r = 0..3), checked against a
//           host matmul of the same matrices;
//   exact:  the kernel's own use -- per lane B = two channels' (cos, sin) f16 words of two steps,
//           A = the pair's gains on the lanes 20q + r, C starting at 1.5 2^23 + 64 -- over many
//           accumulations with |gain| <= 2048 and |LUT| <= 250, against int64 sums.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/mfma16_probe.hip -o tools/ubench/mfma16_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float4_ __attribute__((ext_vector_type(4)));

__global__ void layout(const float *a, const float *b, const float *c0, float *c)
{
    const int l = threadIdx.x;
    half8 A, B;
    for (int j = 0; j < 8; j++) {
        A[j] = (_Float16)a[(l & 15) * 32 + 8 * (l >> 4) + j];      /* A[row][k] row-major 16x32 */
        B[j] = (_Float16)b[(8 * (l >> 4) + j) * 16 + (l & 15)];     /* B[k][col] row-major 32x16 */
    }
    float4_ C;
    for (int r = 0; r < 4; r++)
        C[r] = c0[(4 * (l >> 4) + r) * 16 + (l & 15)];
    C = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, C, 0, 0, 0);
    for (int r = 0; r < 4; r++)
        c[(4 * (l >> 4) + r) * 16 + (l & 15)] = C[r];
}

/* the render kernel's accumulation: lane l's outputs (I_s, Q_s, I_s+1, Q_s+1) from its own two
   channels' words; iters pairs of (ga, gb, words) per lane, sums checked on the host */
__global__ void pairs(const int16_t *ga, const int16_t *gb, const int16_t *lut, int iters,
                      float *out)
{
    const int l = threadIdx.x, q = l >> 4, r = l & 3;
    const bool act = ((l & 15) >> 2) == q;
    float4_ C = {12582976.0f, 12582976.0f, 12582976.0f, 12582976.0f};
    for (int it = 0; it < iters; it++) {
        half8 A;
        for (int j = 0; j < 8; j++)
            A[j] = (_Float16)0;
        if (act) {
            A[r] = (_Float16)ga[it];
            A[4 + r] = (_Float16)gb[it];
        }
        half8 B;
        for (int j = 0; j < 8; j++)
            B[j] = (_Float16)lut[(it * 64 + l) * 8 + j];
        C = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, C, 0, 0, 0);
    }
    for (int k = 0; k < 4; k++)
        out[l * 4 + k] = C[k];
}

static float h16(float x) { return (float)(_Float16)x; }

int main()
{
    /* ---- layout ---- */
    float a[16 * 32], b[32 * 16], c0[256], c[256], want[256];
    srand(1);
    for (int i = 0; i < 512; i++) {
        a[i] = h16((float)(rand() % 17 - 8));
        b[i] = h16((float)(rand() % 13 - 6));
    }
    for (int i = 0; i < 256; i++)
        c0[i] = (float)(rand() % 100);
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) {
            double s = c0[i * 16 + j];
            for (int k = 0; k < 32; k++)
                s += (double)a[i * 32 + k] * b[k * 16 + j];
            want[i * 16 + j] = (float)s;
        }
    float *da, *db, *dc0, *dc;
    (void)hipMalloc(&da, sizeof a); (void)hipMalloc(&db, sizeof b);
    (void)hipMalloc(&dc0, sizeof c0); (void)hipMalloc(&dc, sizeof c);
    (void)hipMemcpy(da, a, sizeof a, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b, sizeof b, hipMemcpyHostToDevice);
    (void)hipMemcpy(dc0, c0, sizeof c0, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(layout, 1, 64, 0, 0, da, db, dc0, dc);
    (void)hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; i++)
        bad += c[i] != want[i];
    printf("layout 16x16x32 f16: %d of 256 outputs differ from the assumed map\n", bad);

    /* ---- exactness in the kernel's pattern ---- */
    const int iters = 4096;
    int16_t *ga = (int16_t *)malloc(iters * 2), *gb = (int16_t *)malloc(iters * 2);
    int16_t *lut = (int16_t *)malloc((size_t)iters * 64 * 8 * 2);
    for (int i = 0; i < iters; i++) {
        /* gains of either sign up to 2048 (gain differences of a data-bit flip), small ones too */
        ga[i] = (int16_t)((rand() % 4097) - 2048) / ((i % 16) ? 16 : 1);
        gb[i] = (int16_t)((rand() % 4097) - 2048) / ((i % 16 == 7) ? 1 : 16);
    }
    for (size_t i = 0; i < (size_t)iters * 64 * 8; i++)
        lut[i] = (int16_t)((rand() % 501) - 250);
    int16_t *dga, *dgb, *dlut;
    float *dout, out[256];
    (void)hipMalloc(&dga, iters * 2); (void)hipMalloc(&dgb, iters * 2);
    (void)hipMalloc(&dlut, (size_t)iters * 64 * 8 * 2); (void)hipMalloc(&dout, sizeof out);
    (void)hipMemcpy(dga, ga, iters * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dgb, gb, iters * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dlut, lut, (size_t)iters * 64 * 8 * 2, hipMemcpyHostToDevice);
    /* partial sums must stay in (-2^23, 2^23) around the bias: check in chunks of 16 iters */
    int worst = 0, nbad = 0, checked = 0;
    for (int n = 16; n <= iters; n *= 4) {
        hipLaunchKernelGGL(pairs, 1, 64, 0, 0, dga, dgb, dlut, n, dout);
        (void)hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; l++)
            for (int k = 0; k < 4; k++) {
                int64_t s = 64, peak = 0;
                for (int it = 0; it < n; it++) {
                    s += (int64_t)ga[it] * lut[(it * 64 + l) * 8 + k] +
                         (int64_t)gb[it] * lut[(it * 64 + l) * 8 + 4 + k];
                    peak = llabs(s) > peak ? llabs(s) : peak;
                }
                if (peak >= (1 << 22))
                    continue;                       /* outside the exact domain: not checked */
                checked++;
                const int64_t got = (int64_t)out[l * 4 + k] - 12582912;
                if (got != s) {
                    nbad++;
                    worst = llabs(got - s) > worst ? (int)llabs(got - s) : worst;
                }
            }
    }
    printf("exactness (pairs, bias 1.5*2^23+64): %d of %d checked outputs inexact, worst %d\n",
           nbad, checked, worst);
    return bad || nbad;
}
