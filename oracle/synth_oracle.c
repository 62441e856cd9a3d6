/*
 * synth_oracle.c — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this; the product path (libgpssim_amd.so) never does.
 *
 * A literal, scalar restatement of the reference per-sample loop:
 *   gpssim.c:2190-2256  per sample, per active channel: LUT carrier × C/A chip × nav bit × gain,
 *                       integer-accumulated; code/carrier phase advance with wraps and the
 *                       chip/bit/word counters
 *   gpssim.c:2257-2263  (acc+64)>>7 → short
 *   gpssim.c:2266-2288  SC01 bit packing (MSB first), SC08 (>>4), SC16 raw
 * Carrier tables (gpssim.c:15-83) are rebuilt from round(250 sin(2π(k+½)/512)) with the one
 * quarter-wave exception (k=35 → 105); tests/test_oracle.py pins them against a fixture taken
 * from the reference source.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "synth_oracle.h"

void oracle_lut(int *sin512, int *cos512)
{
    int q[128];
    for (int k = 0; k < 128; k++)
        q[k] = (int)lround(250.0 * sin(2.0 * 3.14159265358979323846 * (k + 0.5) / 512.0));
    q[35] = 105;
    for (int k = 0; k < 512; k++) {
        int h = k & 255;
        int v = h < 128 ? q[h] : q[255 - h];
        sin512[k] = k < 256 ? v : -v;
    }
    for (int k = 0; k < 512; k++)
        cos512[k] = sin512[(k + 128) & 511];
}

size_t oracle_block_bytes(int n, int fmt)
{
    return fmt == 16 ? (size_t)n * 4 : fmt == 8 ? (size_t)n * 2 : fmt == 1 ? (size_t)n / 4 : 0;
}

typedef struct {
    int prn_tbl, gain;
    double carr, fcd, code, fcod;
    int icode, ibit, iword, dataBit, codeCA;
    const uint32_t *ca, *dwrd;
} och;

static int ca_chip(const uint32_t *bits, int i) { return (int)((bits[i >> 5] >> (i & 31)) & 1u); }

int oracle_synth(const gss_chan_blk_t *blk, const int32_t *nch, const uint32_t *ca_bits,
                 const uint32_t *nav, int nblk, int n, int fmt, void *out, double *carr_end)
{
    static int sinT[512], cosT[512];
    static int init = 0;
    if (!init) { oracle_lut(sinT, cosT); init = 1; }
    int status = 0;
    short *iq = (short *)malloc(sizeof(short) * 2 * (size_t)n);
    unsigned char *o = (unsigned char *)out;
    size_t bb = oracle_block_bytes(n, fmt);

    for (int b = 0; b < nblk; b++) {
        och ch[GSS_MAXCH];
        int nc = nch[b];
        for (int k = 0; k < nc; k++) {
            const gss_chan_blk_t *p = &blk[(size_t)b * GSS_MAXCH + k];
            och *c = &ch[k];
            c->carr = p->carr0;
            c->fcd = p->carr_step;
            c->code = p->code0;
            c->fcod = p->code_step;
            c->icode = p->icode; c->ibit = p->ibit; c->iword = p->iword;
            c->gain = p->gain;
            c->ca = ca_bits + (size_t)p->ca_tbl * GSS_CA_WORDS;
            c->dwrd = nav + (size_t)p->nav_tbl * GSS_NAV_WORDS;
            /* computeCodePhase's codeCA / dataBit (gpssim.c:1344-1345) */
            c->codeCA = ca_chip(c->ca, (int)c->code) * 2 - 1;
            if (c->iword > 59) { status = GSS_E_RANGE; c->iword = 59; }
            c->dataBit = (int)((c->dwrd[c->iword] >> (29 - c->ibit)) & 0x1u) * 2 - 1;
        }
        for (int isamp = 0; isamp < n; isamp++) {
            int i_acc = 0, q_acc = 0;
            for (int k = 0; k < nc; k++) {
                och *c = &ch[k];
                int iTable = (int)floor(c->carr * 512.0);
                int ip = c->dataBit * c->codeCA * cosT[iTable & 511] * c->gain;
                int qp = c->dataBit * c->codeCA * sinT[iTable & 511] * c->gain;
                i_acc += ip;
                q_acc += qp;
                c->code += c->fcod;
                if (c->code >= 1023) {
                    c->code -= 1023;
                    c->icode++;
                    if (c->icode >= 20) {
                        c->icode = 0;
                        c->ibit++;
                        if (c->ibit >= 30) {
                            c->ibit = 0;
                            c->iword++;
                        }
                        if (c->iword > 59) { status = GSS_E_RANGE; c->iword = 59; }
                        c->dataBit = (int)((c->dwrd[c->iword] >> (29 - c->ibit)) & 0x1u) * 2 - 1;
                    }
                }
                c->codeCA = ca_chip(c->ca, (int)c->code) * 2 - 1;
                c->carr += c->fcd;
                if (c->carr >= 1.0)
                    c->carr -= 1.0;
                else if (c->carr < 0.0)
                    c->carr += 1.0;
            }
            i_acc = (i_acc + 64) >> 7;
            q_acc = (q_acc + 64) >> 7;
            iq[isamp * 2] = (short)i_acc;
            iq[isamp * 2 + 1] = (short)q_acc;
        }
        unsigned char *dst = o + (size_t)b * bb;
        if (fmt == 1) {
            for (int i = 0; i < 2 * n; i++) {
                if (i % 8 == 0) dst[i / 8] = 0;
                dst[i / 8] |= (unsigned char)((iq[i] > 0 ? 1 : 0) << (7 - i % 8));
            }
        } else if (fmt == 8) {
            for (int i = 0; i < 2 * n; i++)
                ((signed char *)dst)[i] = (signed char)(iq[i] >> 4);
        } else {
            memcpy(dst, iq, sizeof(short) * 2 * (size_t)n);
        }
        for (int k = 0; k < nc; k++) {
            if (carr_end) carr_end[(size_t)b * GSS_MAXCH + k] = ch[k].carr;
        }
    }
    free(iq);
    return status;
}


/* Brute-force reference recurrences (one double step per sample, gpssim.c:2212-2250), used by
   the tests to check the product's jump-ahead walk. */
double oracle_carr_brute(double x, double s, int64_t n)
{
    for (int64_t i = 0; i < n; i++) {
        x += s;
        if (x >= 1.0)
            x -= 1.0;
        else if (x < 0.0)
            x += 1.0;
    }
    return x;
}

/* the brute-force carrier chain sampled at ascending sample indices at[0..m) */
void oracle_carr_trace(double x, double s, const int64_t *at, int m, double *out)
{
    int64_t pos = 0;
    for (int j = 0; j < m; j++) {
        x = oracle_carr_brute(x, s, at[j] - pos);
        pos = at[j];
        out[j] = x;
    }
}

double oracle_code_brute(double c, double s, int64_t n, int32_t *icode, int32_t *ibit,
                         int32_t *iword)
{
    for (int64_t i = 0; i < n; i++) {
        c += s;
        if (c >= 1023) {
            c -= 1023;
            if (++*icode >= 20) {
                *icode = 0;
                if (++*ibit >= 30) {
                    *ibit = 0;
                    ++*iword;
                }
            }
        }
    }
    return c;
}
