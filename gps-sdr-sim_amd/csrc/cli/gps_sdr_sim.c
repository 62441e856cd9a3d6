/*
 * gps_sdr_sim.c — the command-line program: reference option surface (-e/-u/-g/-c/-l/-t/-T/-d/
 * -o/-s/-b/-i/-v), reference stderr messages, byte-identical gpssim.bin.  The per-sample work
 * runs on the GPU (gss_synth_host); this driver only moves batches of blocks between the host
 * control plane (gss_scn_next) and the sink (fwrite to file or stdout), gpssim.c:2101-2111,
 * 2276-2287.  There is no CPU fallback: without a GPU it exits with an error.
 * Env: GSS_DEVICE (ordinal, default 0), GSS_BATCH (blocks per launch, default 100),
 *      GSS_THREADS (planner threads, default 8).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "gpssim_amd.h"
#include "cli_args.h"

int main(int argc, char **argv)
{
    gss_cli_t cli;
    if (gss_cli_parse(argc, argv, &cli))
        return 1;
    gss_scn *scn = NULL;
    if (gss_scn_open(&scn, &cli.opt)) {
        fprintf(stderr, "%s\n", gss_last_error());
        return 1;
    }
    gss_scn_info_t info;
    gss_scn_info(scn, &info);

    gss_dev *dev = NULL;
    int ordinal = getenv("GSS_DEVICE") ? atoi(getenv("GSS_DEVICE")) : 0;
    if (gss_dev_open(&dev, ordinal)) {
        fprintf(stderr, "ERROR: %s\n", gss_last_error());
        return 1;
    }
    FILE *fp = stdout;
    if (strcmp("-", cli.out_file)) {
        fp = fopen(cli.out_file, "wb");
        if (fp == NULL) {
            fprintf(stderr, "ERROR: Failed to open output file.\n");
            return 1;
        }
    }
    int batch = getenv("GSS_BATCH") ? atoi(getenv("GSS_BATCH")) : 100;
    int threads = getenv("GSS_THREADS") ? atoi(getenv("GSS_THREADS")) : 8;
    if (batch < 1) batch = 1;
    uint32_t ca[32 * GSS_CA_WORDS];
    gss_ca_table(ca);
    size_t bb = gss_block_bytes(info.n_per_blk, info.data_format);
    gss_chan_blk_t *blk = malloc(sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)batch);
    int32_t *nch = malloc(sizeof(int32_t) * (size_t)batch);
    unsigned char *out = malloc(bb * (size_t)batch);
    double *ck = malloc(sizeof(double) * GSS_MAXCH * GSS_NCK * (size_t)batch);
    if (!blk || !nch || !out || !ck) {
        fprintf(stderr, "ERROR: Failed to allocate I/Q buffer.\n");
        return 1;
    }
    clock_t t0 = clock();
    for (;;) {
        int nb = 0;
        if (gss_scn_next(scn, batch, blk, nch, ck, &nb, threads)) {
            fprintf(stderr, "\nERROR: %s\n", gss_last_error());
            return 1;
        }
        if (nb == 0)
            break;
        const uint32_t *nav;
        int nnav;
        gss_scn_nav_table(scn, &nav, &nnav);
        if (gss_synth_host(dev, blk, nch, ck, ca, 32, nav, nnav, nb, info.n_per_blk,
                           info.data_format, out, NULL)) {
            fprintf(stderr, "\nERROR: %s\n", gss_last_error());
            return 1;
        }
        if (fwrite(out, 1, bb * (size_t)nb, fp) != bb * (size_t)nb) {
            fprintf(stderr, "\nERROR: write failed.\n");
            return 1;
        }
    }
    clock_t t1 = clock();
    fprintf(stderr, "\nDone!\n");
    if (fp != stdout)
        fclose(fp);
    fprintf(stderr, "Process time = %.1f [sec]\n", (double)(t1 - t0) / CLOCKS_PER_SEC);
    gss_dev_close(dev);
    gss_scn_close(scn);
    free(blk); free(nch); free(out); free(ck);
    return 0;
}
