/* Test-only harness: renders blocks from the certified integer lines (gss_lin_t) with scalar C,
   exactly the arithmetic the GPU fast path (gss_lin_kernel) performs: LUT cell = high 9 bits of
   x0 + p*xs (mod 2^64), chip = floor((z0 + p*zs) / 2^50) mod 1023, signed gain from the
   schedule, the patched samples.  tests/test_linearize.py compares its bytes with the scalar oracle of the reference
   loop (oracle/synth_oracle.c) on every block gss_linearize certifies. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../../include/gpssim_amd.h"

typedef unsigned __int128 u128;

static int ca_chip(const uint32_t *bits, int i) { return (int)((bits[i >> 5] >> (i & 31)) & 1u); }

int lc_render(const gss_chan_blk_t *blk, const int32_t *nch, const gss_lin_t *lin,
              const int32_t *fast, const uint32_t *ca_bits, const int32_t *sinT,
              const int32_t *cosT, int nblk, int n, int fmt, uint8_t *out)
{
    const size_t bb = fmt == 16 ? (size_t)n * 4 : fmt == 8 ? (size_t)n * 2 : (size_t)n / 4;
    int16_t *iq = malloc(sizeof(int16_t) * 2 * (size_t)n);
    int rendered = 0;
    for (int b = 0; b < nblk; b++) {
        if (!fast[b])
            continue;
        rendered++;
        for (int p = 0; p < n; p++) {
            int i_acc = 64, q_acc = 64;
            for (int k = 0; k < nch[b]; k++) {
                const gss_lin_t *l = &lin[(size_t)b * GSS_MAXCH + k];
                const gss_chan_blk_t *c = &blk[(size_t)b * GSS_MAXCH + k];
                const uint64_t x = l->x0 + (uint64_t)p * l->xs;
                int ti = (int)(x >> 55);
                const u128 z = (u128)l->z0 + (u128)p * l->zs;
                int chip = (int)((uint64_t)(z >> 50) % GSS_CA_LEN);
                for (int j = 0; j < GSS_NPATCH; j++)
                    if (l->ppos[j] == p) {                     /* the exact cell / chip */
                        if (l->pval[j] >> 16)
                            chip = l->pval[j] & 0xFFFF;
                        else
                            ti = l->pval[j] & 0xFFFF;
                    }
                const int ca = ca_chip(ca_bits + (size_t)c->ca_tbl * GSS_CA_WORDS, chip) * 2 - 1;
                int g = l->gval[0];
                for (int i = 1; i < GSS_NGC; i++)
                    if (l->gpos[i] <= p)
                        g = l->gval[i];
                i_acc += g * ca * cosT[ti];
                q_acc += g * ca * sinT[ti];
            }
            iq[2 * p] = (int16_t)(i_acc >> 7);
            iq[2 * p + 1] = (int16_t)(q_acc >> 7);
        }
        uint8_t *dst = out + (size_t)b * bb;
        if (fmt == 16) {
            memcpy(dst, iq, sizeof(int16_t) * 2 * (size_t)n);
        } else if (fmt == 8) {
            for (int i = 0; i < 2 * n; i++)
                ((int8_t *)dst)[i] = (int8_t)(iq[i] >> 4);
        } else {
            memset(dst, 0, bb);
            for (int i = 0; i < 2 * n; i++)
                dst[i / 8] |= (uint8_t)((iq[i] > 0) << (7 - i % 8));
        }
    }
    free(iq);
    return rendered;
}
