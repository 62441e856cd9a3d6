/* Test-only harness: renders blocks from the certified integer lines (gss_lin_t) with scalar C,
   exactly the arithmetic the GPU fast path (gss_lin_kernel) performs: the kernel's LUT cell and
   chip at each sample (gss_lin_kernel_at, csrc/common/gss_lin.h: chunk anchors plus
   32-bit steps), the signed gain from the schedule, the packed I/Q accumulator
   (64 + 2^21) + 2^22 (64 + ...) and the patch corrections.  tests/test_linearize.py compares its
   bytes with the scalar oracle of the reference loop (oracle/synth_oracle.c) on every block
   gss_linearize certifies. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../../include/gpssim_amd.h"
#include "../../gps-sdr-sim_amd/csrc/common/gss_lin.h"

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
            int64_t acc = 64 + (1 << 21) + ((int64_t)64 << 22);
            for (int k = 0; k < nch[b]; k++) {
                const gss_lin_t *l = &lin[(size_t)b * GSS_MAXCH + k];
                const gss_chan_blk_t *c = &blk[(size_t)b * GSS_MAXCH + k];
                const gss_lin_kc kk = gss_lin_kernel_at(l->x0, l->xs, l->z0, l->zs, p);
                const int ti = kk.cell, chip = kk.chip;
                const int ca = ca_chip(ca_bits + (size_t)c->ca_tbl * GSS_CA_WORDS, chip) * 2 - 1;
                int g = l->gval[0];
                for (int i = 1; i < GSS_NGC; i++)
                    if (l->gpos[i] <= p)
                        g = l->gval[i];
                acc += (int64_t)(g * ca) * ((int64_t)cosT[ti] + ((int64_t)sinT[ti] << 22));
                for (int j = 0; j < GSS_NPATCH; j++)
                    if (l->ppos[j] == p)
                        acc += l->pdelta[j];
            }
            /* the kernel's epilogue: I field (sum I + 64 + 2^21) in bits 0..21, Q above */
            const int64_t fi = (acc & ((1 << 22) - 1)) - (1 << 21);
            iq[2 * p] = (int16_t)(fi >> 7);
            iq[2 * p + 1] = (int16_t)(acc >> 29);
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
