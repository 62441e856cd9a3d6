/*
 * run_harness.c — gss_run's host threads without a GPU, for the sanitizers (tools/sanitize.sh).
 *
 * gss_run (csrc/hip/gss_run.hip) splits the planning of a run over three threads besides its main
 * one, each with its own worker pool (pool.c, gss_pool_select): a rows thread that owns the
 * scenario and produces deferred rows (gss_scn_next_deferred), a planner thread that runs the
 * carrier chain from speculative walks (gss_carr_chain_starts -> walks -> gss_carr_chain_spec)
 * and a prover thread (gss_linearize).  This harness runs the same host functions in the same
 * arrangement -- bounded queues between the threads, the walks by gss_spec_host instead of the
 * GPU -- and checks the rows against one serial gss_scn_next pass of the same scenario (the
 * host chain), byte for byte.  Built with -fsanitize=thread and with -fsanitize=address,undefined
 * over the host plane's own sources; any report fails the run.
 *
 * usage: run_harness NAV_FILE [seconds] [batch] [fmt]
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gpssim_amd.h"

void gss_pool_select(int id);               /* pool.c */

typedef struct {
    gss_chan_blk_t *blk;
    int32_t *nch;
    gss_chain_t *chain;
    uint32_t *nav;                          /* the nav table when the batch was produced */
    int n_nav, nb;
    gss_lin_t *lin;
    int32_t *fast;
    int hits;
} batch_t;

typedef struct {                            /* a bounded FIFO of batches (NULL: end) */
    pthread_mutex_t mu;
    pthread_cond_t cv;
    batch_t *q[4];
    int head, n;
} queue_t;

static void q_init(queue_t *q)
{
    pthread_mutex_init(&q->mu, NULL);
    pthread_cond_init(&q->cv, NULL);
    q->head = q->n = 0;
}

static void q_push(queue_t *q, batch_t *b)
{
    pthread_mutex_lock(&q->mu);
    while (q->n == 4)
        pthread_cond_wait(&q->cv, &q->mu);
    q->q[(q->head + q->n++) % 4] = b;
    pthread_cond_broadcast(&q->cv);
    pthread_mutex_unlock(&q->mu);
}

static batch_t *q_pop(queue_t *q)
{
    pthread_mutex_lock(&q->mu);
    while (q->n == 0)
        pthread_cond_wait(&q->cv, &q->mu);
    batch_t *b = q->q[q->head];
    q->head = (q->head + 1) % 4;
    q->n--;
    pthread_cond_broadcast(&q->cv);
    pthread_mutex_unlock(&q->mu);
    return b;
}

typedef struct {
    gss_scn *scn;
    int batch, n_per_blk, threads;
    double carr[GSS_MAXCH];
    uint32_t ca[32 * GSS_CA_WORDS];
    queue_t rows_q, plan_q, done_q;
    int err;
} run_t;

static void *rows_thread(void *arg)
{
    run_t *r = (run_t *)arg;
    gss_pool_select(1);
    for (;;) {
        batch_t *b = calloc(1, sizeof *b);
        b->blk = calloc((size_t)r->batch * GSS_MAXCH, sizeof *b->blk);
        b->nch = calloc((size_t)r->batch, sizeof *b->nch);
        b->chain = calloc((size_t)r->batch * GSS_MAXCH, sizeof *b->chain);
        if (gss_scn_next_deferred(r->scn, r->batch, b->blk, b->nch, b->chain, &b->nb,
                                  r->threads)) {
            fprintf(stderr, "rows: %s\n", gss_last_error());
            r->err = 1;
            b->nb = 0;
        }
        if (b->nb == 0) {
            free(b->blk); free(b->nch); free(b->chain); free(b);
            q_push(&r->rows_q, NULL);
            return NULL;
        }
        const uint32_t *rows;
        gss_scn_nav_table(r->scn, &rows, &b->n_nav);  /* a copy for the prover */
        b->nav = malloc((size_t)b->n_nav * GSS_NAV_WORDS * sizeof *b->nav);
        memcpy(b->nav, rows, (size_t)b->n_nav * GSS_NAV_WORDS * sizeof *b->nav);
        q_push(&r->rows_q, b);
    }
}

static void *planner_thread(void *arg)
{
    run_t *r = (run_t *)arg;
    gss_pool_select(0);
    for (;;) {
        batch_t *b = q_pop(&r->rows_q);
        if (!b) {
            q_push(&r->plan_q, NULL);
            return NULL;
        }
        const int nrow = b->nb * GSS_MAXCH;
        gss_spec_in_t *in = calloc((size_t)nrow, sizeof *in);
        gss_spec_t *spec = calloc((size_t)nrow, sizeof *spec);
        if (gss_carr_chain_starts(r->carr, b->blk, b->nch, b->chain, b->nb, r->n_per_blk, in) ||
            gss_spec_host(in, nrow, r->n_per_blk, spec, r->threads) ||
            gss_carr_chain_spec(r->carr, b->blk, b->nch, b->chain, b->nb, r->n_per_blk, in, spec,
                                r->threads, &b->hits)) {
            fprintf(stderr, "planner: %s\n", gss_last_error());
            r->err = 1;
        }
        free(in);
        free(spec);
        q_push(&r->plan_q, b);
    }
}

static void *prover_thread(void *arg)
{
    run_t *r = (run_t *)arg;
    gss_pool_select(2);
    for (;;) {
        batch_t *b = q_pop(&r->plan_q);
        if (!b) {
            q_push(&r->done_q, NULL);
            return NULL;
        }
        b->lin = calloc((size_t)b->nb * GSS_MAXCH, sizeof *b->lin);
        b->fast = calloc((size_t)b->nb, sizeof *b->fast);
        if (gss_linearize(b->blk, b->nch, b->nb, r->n_per_blk, r->ca, 32, b->nav, b->n_nav,
                          b->lin, b->fast, r->threads)) {
            fprintf(stderr, "prover: %s\n", gss_last_error());
            r->err = 1;
        }
        q_push(&r->done_q, b);
    }
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s NAV_FILE [seconds] [batch] [fmt]\n", argv[0]);
        return 2;
    }
    gss_opts_t o;
    memset(&o, 0, sizeof o);
    o.nav_file = argv[1];
    o.has_llh = 1;
    o.llh[0] = 30.286502; o.llh[1] = 120.032669; o.llh[2] = 100.0;
    o.samp_freq = 2.6e6;
    o.data_format = argc > 4 ? atoi(argv[4]) : 1;
    o.duration = argc > 2 ? atof(argv[2]) : 300.0;
    o.quiet = 1;
    run_t r;
    memset(&r, 0, sizeof r);
    r.batch = argc > 3 ? atoi(argv[3]) : 512;
    r.threads = 4;
    gss_scn *ref = NULL;
    if (gss_scn_open(&r.scn, &o) || gss_scn_open(&ref, &o)) {
        fprintf(stderr, "open: %s\n", gss_last_error());
        return 1;
    }
    gss_scn_info_t info;
    gss_scn_info(r.scn, &info);
    r.n_per_blk = info.n_per_blk;
    gss_ca_table(r.ca);
    gss_scn_carrier(r.scn, r.carr);            /* block 0: every slot starts with a reset */
    q_init(&r.rows_q); q_init(&r.plan_q); q_init(&r.done_q);
    pthread_t th[3];
    pthread_create(&th[0], NULL, rows_thread, &r);
    pthread_create(&th[1], NULL, planner_thread, &r);
    pthread_create(&th[2], NULL, prover_thread, &r);

    /* main: the serial reference beside the pipeline, batch for batch */
    gss_chan_blk_t *want = calloc((size_t)r.batch * GSS_MAXCH, sizeof *want);
    int32_t *wn = calloc((size_t)r.batch, sizeof *wn);
    long blocks = 0, rows = 0, hits = 0, fast = 0, bad = 0;
    for (;;) {
        batch_t *b = q_pop(&r.done_q);
        if (!b)
            break;
        int nw = 0;
        if (gss_scn_next(ref, b->nb, want, wn, NULL, &nw, r.threads) || nw != b->nb) {
            fprintf(stderr, "reference: %s\n", gss_last_error());
            return 1;
        }
        for (int i = 0; i < b->nb; i++) {
            rows += b->nch[i];
            fast += b->fast[i];
            if (wn[i] != b->nch[i] ||
                memcmp(&want[(size_t)i * GSS_MAXCH], &b->blk[(size_t)i * GSS_MAXCH],
                       sizeof(gss_chan_blk_t) * (size_t)b->nch[i]))
                bad++;
        }
        blocks += b->nb;
        hits += b->hits;
        free(b->blk); free(b->nch); free(b->chain); free(b->nav); free(b->lin); free(b->fast);
        free(b);
    }
    for (int i = 0; i < 3; i++)
        pthread_join(th[i], NULL);
    free(want);
    free(wn);
    gss_scn_close(r.scn);
    gss_scn_close(ref);
    printf("run_harness: %ld blocks, %ld rows (%ld translated), %ld certified, %ld differ from "
           "the serial chain\n", blocks, rows, hits, fast, bad);
    return (r.err || bad || blocks != info.n_blocks) ? 1 : 0;
}
