/*
 * gss_integ.c — the drop-in a gps-sdr-sim maintainer adds next to gpssim.c.
 *
 * gpssim.c keeps everything around its sample loop: ranges, gains, computeCodePhase, nav words,
 * channel allocation (gpssim.c:2156-2188, 2290-2353).  Two calls replace the loop and its
 * pack/fwrite epilogue (gpssim.c:2190-2288):
 *     gss_integ_block(chan, gain, iq_buff_size, data_format, delt, grx.sec, fp);  per block
 *     gss_integ_flush(fp);                                                        after the loop
 * Blocks are collected into batches of GSS_INTEG_K and rendered by libgpssim_amd.so
 * (gss_synth_host: certified fast path, exact path for the rest).  A batch is flushed at the
 * reference's 30 s update (igrx % 300 == 0, gpssim.c:2294-2296): that update rewrites dwrd and
 * may reallocate channels right after the block, so no batch spans it.
 * The carrier phase is the only state the reference loop carries into the next block
 * (gpssim.c:2245-2250); gss_carr_advance_ck advances it exactly, without running the loop, and
 * records the block's GSS_NCK carrier checkpoints for the GPU.
 * Both carrier builds of the reference are handled (gpssim.h:4): with FLOAT_CARR_PHASE the
 * double carr_phase is advanced by gss_carr_advance_ck; without it chan[i].carr_phase is the
 * uint32 chain of 2^-25 cycle steps carr_phasestep (gpssim.c:1625, 2176, 2202, 2252), which the
 * rows carry as exact multiples of 2^-25 (carr0 = (carr_phase mod 2^25) / 2^25, carr_step =
 * carr_phasestep / 2^25, the library's --carrier=int convention) and which is advanced here by
 * the same integer additions the loop would make.
 * Compiled together with the maintainer's gpssim.c/gpssim.h (channel_t, MAX_CHAN, CA_SEQ_LEN);
 * tools/integration/build_integ.py does that against a /tmp copy of the reference.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gpssim.h"
#include "gpssim_amd.h"

#ifndef GSS_INTEG_K
#define GSS_INTEG_K 100                       /* blocks per GPU call */
#endif

static struct {
    gss_dev *dev;
    gss_chan_blk_t blk[GSS_INTEG_K * GSS_MAXCH];
    double ck[GSS_INTEG_K * GSS_MAXCH * GSS_NCK];
    int32_t nch[GSS_INTEG_K];
    uint32_t ca[MAX_SAT][GSS_CA_WORDS];       /* packed chan[i].ca, bit j%32 of word j/32 */
    int ca_done[MAX_SAT];
    uint32_t nav[GSS_INTEG_K * GSS_MAXCH][GSS_NAV_WORDS];
    int kb, n, fmt;
    void *out;
} g;

static void fail(void)
{
    fprintf(stderr, "ERROR: %s\n", gss_last_error());
    exit(1);
}

void gss_integ_flush(FILE *fp)
{
    if (g.kb == 0)
        return;
    if (gss_synth_host(g.dev, g.blk, g.nch, g.ck, &g.ca[0][0], MAX_SAT, &g.nav[0][0],
                       g.kb * GSS_MAXCH, g.kb, g.n, g.fmt, g.out, NULL))
        fail();
    fwrite(g.out, 1, gss_block_bytes(g.n, g.fmt) * (size_t)g.kb, fp);   /* gpssim.c:2276-2287 */
    g.kb = 0;
}

void gss_integ_block(channel_t *chan, const int *gain, int iq_buff_size, int data_format,
                     double delt, double grx_sec, FILE *fp)
{
    if (!g.dev) {
        if (gss_dev_open(&g.dev, 0))
            fail();
        g.n = iq_buff_size;
        g.fmt = data_format;
        g.out = malloc(gss_block_bytes(iq_buff_size, data_format) * GSS_INTEG_K);
        if (!g.out) {
            fprintf(stderr, "ERROR: Failed to allocate the output batch.\n");
            exit(1);
        }
    }
    int c = 0;
    for (int i = 0; i < MAX_CHAN; i++) {
        if (chan[i].prn == 0)
            continue;
        const int row = g.kb * GSS_MAXCH + c;
        gss_chan_blk_t *p = &g.blk[row];
        const int sv = chan[i].prn - 1;
        if (!g.ca_done[sv]) {
            memset(g.ca[sv], 0, sizeof g.ca[sv]);
            for (int j = 0; j < CA_SEQ_LEN; j++)
                g.ca[sv][j >> 5] |= (uint32_t)(chan[i].ca[j] & 1) << (j & 31);
            g.ca_done[sv] = 1;
        }
        for (int w = 0; w < N_DWRD; w++)
            g.nav[row][w] = (uint32_t)chan[i].dwrd[w];
#ifdef FLOAT_CARR_PHASE
        p->carr0 = chan[i].carr_phase;
        p->carr_step = chan[i].f_carr * delt;        /* the loop's own products */
#else
        p->carr0 = (double)(chan[i].carr_phase & 0x1FFFFFFu) / 33554432.0;
        p->carr_step = (double)chan[i].carr_phasestep / 33554432.0;
#endif
        p->code0 = chan[i].code_phase;
        p->code_step = chan[i].f_code * delt;
        p->icode = chan[i].icode;
        p->ibit = chan[i].ibit;
        p->iword = chan[i].iword;
        p->gain = gain[i];
        p->ca_tbl = sv;
        p->nav_tbl = row;
        /* the carrier the reference loop would leave behind, exactly */
#ifdef FLOAT_CARR_PHASE
        chan[i].carr_phase = gss_carr_advance_ck(chan[i].carr_phase, p->carr_step, iq_buff_size,
                                                 &g.ck[(size_t)row * GSS_NCK]);
#else
        for (int j = 0; j < GSS_NCK; j++) {      /* phase at sample (j n) / GSS_NCK */
            const unsigned int at = chan[i].carr_phase +
                (unsigned int)chan[i].carr_phasestep * (unsigned int)(((long long)j * iq_buff_size) / GSS_NCK);
            g.ck[(size_t)row * GSS_NCK + j] = (double)(at & 0x1FFFFFFu) / 33554432.0;
        }
        chan[i].carr_phase += (unsigned int)chan[i].carr_phasestep * (unsigned int)iq_buff_size;
#endif
        c++;
    }
    for (int k = c; k < GSS_MAXCH; k++)
        memset(&g.blk[g.kb * GSS_MAXCH + k], 0, sizeof g.blk[0]);
    g.nch[g.kb++] = c;
    /* the reference's 30 s nav/allocation update follows this block: no batch spans it */
    if (g.kb == GSS_INTEG_K || (int)(grx_sec * 10.0 + 0.5) % 300 == 0)
        gss_integ_flush(fp);
}
