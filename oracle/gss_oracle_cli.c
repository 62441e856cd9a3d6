/*
 * gss_oracle_cli.c — TEST INFRASTRUCTURE ONLY.  The all-CPU restatement of gps-sdr-sim:
 * the repo's host control plane (gss_scn_*, product code) feeding the scalar oracle sample loop
 * (synth_oracle.c) instead of the GPU.  Same command line as the reference.  Used (a) to pin the
 * host plane + oracle against the reference's golden sha256 (tests/test_oracle.py) and (b) as
 * bench.py's "port" CPU baseline when the reference binary is unavailable.
 * Extra env: GSS_THREADS (planner threads, default 8), GSS_BATCH (blocks per batch).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "synth_oracle.h"
#include "../gps-sdr-sim_amd/csrc/cli/cli_args.h"

int main(int argc, char **argv)
{
    gss_cli_t cli;
    if (gss_cli_parse(argc, argv, &cli))
        return 1;
    gss_scn *scn = NULL;
    int rc = gss_scn_open(&scn, &cli.opt);
    if (rc) {
        fprintf(stderr, "%s\n", gss_last_error());
        return 1;
    }
    gss_scn_info_t info;
    gss_scn_info(scn, &info);
    FILE *fp = strcmp(cli.out_file, "-") ? fopen(cli.out_file, "wb") : stdout;
    if (fp == NULL) {
        fprintf(stderr, "ERROR: Failed to open output file.\n");
        return 1;
    }
    int threads = getenv("GSS_THREADS") ? atoi(getenv("GSS_THREADS")) : 8;
    int batch = getenv("GSS_BATCH") ? atoi(getenv("GSS_BATCH")) : 50;
    uint32_t ca[32 * GSS_CA_WORDS];
    gss_ca_table(ca);
    gss_chan_blk_t *blk = malloc(sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)batch);
    int32_t *nch = malloc(sizeof(int32_t) * (size_t)batch);
    size_t bb = oracle_block_bytes(info.n_per_blk, info.data_format);
    unsigned char *out = malloc(bb * (size_t)batch);
    clock_t t0 = clock();
    for (;;) {
        int nb = 0;
        rc = gss_scn_next(scn, batch, blk, nch, NULL, &nb, threads);
        if (rc) {
            fprintf(stderr, "%s\n", gss_last_error());
            return 1;
        }
        if (nb == 0)
            break;
        const uint32_t *nav;
        int nnav;
        gss_scn_nav_table(scn, &nav, &nnav);
        oracle_synth(blk, nch, ca, nav, nb, info.n_per_blk, info.data_format, out, NULL);
        fwrite(out, 1, bb * (size_t)nb, fp);
    }
    clock_t t1 = clock();
    fprintf(stderr, "\nDone!\n");
    if (fp != stdout)
        fclose(fp);
    fprintf(stderr, "Process time = %.1f [sec]\n", (double)(t1 - t0) / CLOCKS_PER_SEC);
    gss_scn_close(scn);
    free(blk); free(nch); free(out);
    return 0;
}
