/*
 * pool.c — the host plane's worker threads, created once and reused.
 *
 * gss_run plans a batch every few milliseconds (rows, carrier chain, proofs: three parallel
 * sections per batch); creating and joining 16 threads for each costs 0.1-1.7 ms, a large share
 * of a 16-block batch at 20 MS/s.  gss_pool_run(nthreads, nparts, fn, arg) runs fn(arg, part)
 * for part = 0 .. nparts-1 on the caller plus up to nthreads-1 pooled workers, which take parts
 * dynamically (an atomic counter), so uneven parts balance themselves.  One job at a time: a
 * second caller waits for the first job to finish (jobs never nest).
 */
#include <pthread.h>
#include <stdint.h>
#include "gss_host.h"

#define POOL_MAX 64

static pthread_mutex_t run_mu = PTHREAD_MUTEX_INITIALIZER;     /* one job at a time */
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t go = PTHREAD_COND_INITIALIZER, done = PTHREAD_COND_INITIALIZER;
static int n_workers;                    /* started (never exit)                        */
static uint64_t generation;              /* bumped per job                              */
static int job_workers;                  /* workers 0 .. job_workers-1 take part        */
static int active;                       /* workers still in the current job            */
static gss_task_fn job_fn;
static void *job_arg;
static int job_nparts;
static int next_part;                    /* taken with __atomic_fetch_add               */

static void take_parts(gss_task_fn fn, void *arg, int nparts)
{
    for (;;) {
        const int p = __atomic_fetch_add(&next_part, 1, __ATOMIC_RELAXED);
        if (p >= nparts)
            return;
        fn(arg, p);
    }
}

static void *worker(void *arg)
{
    const int id = (int)(intptr_t)arg;
    uint64_t seen = 0;
    pthread_mutex_lock(&mu);
    for (;;) {
        while (generation == seen || id >= job_workers) {
            if (generation != seen)               /* a job this worker sits out */
                seen = generation;
            pthread_cond_wait(&go, &mu);
        }
        seen = generation;
        gss_task_fn fn = job_fn;
        void *a = job_arg;
        const int np = job_nparts;
        pthread_mutex_unlock(&mu);
        take_parts(fn, a, np);
        pthread_mutex_lock(&mu);
        if (--active == 0)
            pthread_cond_signal(&done);
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
    pthread_mutex_lock(&run_mu);
    pthread_mutex_lock(&mu);
    while (n_workers < nthreads - 1) {        /* grow the pool on first use */
        pthread_t t;
        pthread_attr_t at;
        pthread_attr_init(&at);
        pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
        const int ok = pthread_create(&t, &at, worker, (void *)(intptr_t)n_workers) == 0;
        pthread_attr_destroy(&at);
        if (!ok)
            break;
        n_workers++;
    }
    const int w = nthreads - 1 < n_workers ? nthreads - 1 : n_workers;
    job_fn = fn;
    job_arg = arg;
    job_nparts = nparts;
    job_workers = w;
    active = w;
    __atomic_store_n(&next_part, 0, __ATOMIC_RELAXED);
    generation++;
    pthread_cond_broadcast(&go);
    pthread_mutex_unlock(&mu);
    take_parts(fn, arg, nparts);              /* the caller works too */
    pthread_mutex_lock(&mu);
    while (active > 0)
        pthread_cond_wait(&done, &mu);
    pthread_mutex_unlock(&mu);
    pthread_mutex_unlock(&run_mu);
    return 0;
}
