/*
 * pool.c — the host plane's worker threads, created once and reused.
 *
 * gss_run plans a batch every few milliseconds (rows, carrier chain, proofs: three parallel
 * sections per batch); creating and joining 16 threads for each costs 0.1-1.7 ms, a large share
 * of a 16-block batch at 20 MS/s.  gss_pool_run(nthreads, nparts, fn, arg) runs fn(arg, part)
 * for part = 0 .. nparts-1 on the caller plus up to nthreads-1 pooled workers, which take parts
 * dynamically (an atomic counter), so uneven parts balance themselves.  One job at a time per
 * pool: a second caller waits for the first job to finish (jobs never nest).  Three pools, chosen
 * per calling thread (gss_pool_select): gss_run's rows and proof threads have their own.
 * fork(): the workers do not exist in a child, so a pthread_atfork handler (registered at the
 * first job) takes every pool's locks before the fork, releases them in the parent and resets
 * the pools in the child (no workers, fresh locks): the child's first job grows its own.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include "gss_host.h"

#define POOL_MAX 64
#define POOL_N 3                         /* 0: the default; 1, 2: gss_run's rows, proofs */

typedef struct {
    pthread_mutex_t run_mu;              /* one job at a time */
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    int n_workers;                       /* started (never exit)                        */
    uint64_t generation;                 /* bumped per job                              */
    int job_workers;                     /* workers 0 .. job_workers-1 take part        */
    int active;                          /* workers still in the current job            */
    gss_task_fn job_fn;
    void *job_arg;
    int job_nparts;
    int next_part;                       /* taken with __atomic_fetch_add               */
} pool_t;

#define POOL_INIT {PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, \
                   PTHREAD_COND_INITIALIZER, 0, 0, 0, 0, NULL, NULL, 0, 0}
static pool_t pools[POOL_N] = {POOL_INIT, POOL_INIT, POOL_INIT};
static __thread int tl_pool;             /* the calling thread's pool (gss_pool_select) */

/* fork: no job runs across it (prepare takes each pool's job lock, then its state lock) */
static void fork_prepare(void)
{
    for (int i = 0; i < POOL_N; i++) {
        pthread_mutex_lock(&pools[i].run_mu);
        pthread_mutex_lock(&pools[i].mu);
    }
}

static void fork_parent(void)
{
    for (int i = POOL_N - 1; i >= 0; i--) {
        pthread_mutex_unlock(&pools[i].mu);
        pthread_mutex_unlock(&pools[i].run_mu);
    }
}

static void fork_child(void)             /* only the forking thread exists here */
{
    for (int i = 0; i < POOL_N; i++) {
        pool_t *P = &pools[i];
        pthread_mutex_init(&P->run_mu, NULL);
        pthread_mutex_init(&P->mu, NULL);
        pthread_cond_init(&P->go, NULL);
        pthread_cond_init(&P->done, NULL);
        P->n_workers = 0;
        P->job_workers = 0;
        P->active = 0;
    }
}

static pthread_once_t atfork_once = PTHREAD_ONCE_INIT;
static void atfork_register(void) { pthread_atfork(fork_prepare, fork_parent, fork_child); }

/* Route this thread's gss_pool_run jobs to pool id (0 default): gss_run's rows and proof threads
   take their own workers, so that their range passes and proofs run beside the planner's chain
   instead of queueing behind it. */
void gss_pool_select(int id)
{
    tl_pool = id >= 0 && id < POOL_N ? id : 0;
}

typedef struct {
    pool_t *p;
    int id;
} worker_arg;

static void take_parts(pool_t *P, gss_task_fn fn, void *arg, int nparts)
{
    for (;;) {
        const int p = __atomic_fetch_add(&P->next_part, 1, __ATOMIC_RELAXED);
        if (p >= nparts)
            return;
        fn(arg, p);
    }
}

static void *worker(void *arg)
{
    pool_t *P = ((worker_arg *)arg)->p;
    const int id = ((worker_arg *)arg)->id;
    free(arg);
    uint64_t seen = 0;
    pthread_mutex_lock(&P->mu);
    for (;;) {
        while (P->generation == seen || id >= P->job_workers) {
            if (P->generation != seen)           /* a job this worker sits out */
                seen = P->generation;
            pthread_cond_wait(&P->go, &P->mu);
        }
        seen = P->generation;
        gss_task_fn fn = P->job_fn;
        void *a = P->job_arg;
        const int np = P->job_nparts;
        pthread_mutex_unlock(&P->mu);
        take_parts(P, fn, a, np);
        pthread_mutex_lock(&P->mu);
        if (--P->active == 0)
            pthread_cond_signal(&P->done);
    }
    return NULL;
}

int gss_pool_run(int nthreads, int nparts, gss_task_fn fn, void *arg)
{
    if (nparts <= 0)
        return 0;
    if (nthreads > nparts)
        nthreads = nparts;
    if (nthreads > POOL_MAX + 1)
        nthreads = POOL_MAX + 1;
    if (nthreads <= 1) {
        for (int p = 0; p < nparts; p++)
            fn(arg, p);
        return 0;
    }
    pthread_once(&atfork_once, atfork_register);
    pool_t *P = &pools[tl_pool];
    pthread_mutex_lock(&P->run_mu);
    pthread_mutex_lock(&P->mu);
    while (P->n_workers < nthreads - 1) {        /* grow the pool on first use */
        pthread_t t;
        pthread_attr_t at;
        worker_arg *wa = malloc(sizeof *wa);
        if (wa == NULL)
            break;
        wa->p = P;
        wa->id = P->n_workers;
        pthread_attr_init(&at);
        pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
        const int ok = pthread_create(&t, &at, worker, wa) == 0;
        pthread_attr_destroy(&at);
        if (!ok) {
            free(wa);
            break;
        }
        P->n_workers++;
    }
    const int w = nthreads - 1 < P->n_workers ? nthreads - 1 : P->n_workers;
    P->job_fn = fn;
    P->job_arg = arg;
    P->job_nparts = nparts;
    P->job_workers = w;
    P->active = w;
    __atomic_store_n(&P->next_part, 0, __ATOMIC_RELAXED);
    P->generation++;
    pthread_cond_broadcast(&P->go);
    pthread_mutex_unlock(&P->mu);
    take_parts(P, fn, arg, nparts);              /* the caller works too */
    pthread_mutex_lock(&P->mu);
    while (P->active > 0)
        pthread_cond_wait(&P->done, &P->mu);
    pthread_mutex_unlock(&P->mu);
    pthread_mutex_unlock(&P->run_mu);
    return 0;
}
