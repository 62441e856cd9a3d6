/*
 * gss_run.hip — the streaming driver: whole run (or a block range of it) from the host control
 * plane to the caller's byte sink, every stage overlapped.  Replaces the reference's block loop
 * (gpssim.c:2154-2353: refresh, sample loop, fwrite at 2276/2283/2287, 30 s updates).
 *
 *   planner thread   gss_scn_next into pinned slot buffers (+ the sources of the nav rows new
 *                    since the previous slot), then gss_linearize: the fast path's certified
 *                    lines and patches.  With the fast path (float carrier) the carrier chain
 *                    is run ahead on the GPU: the rows come without carriers
 *                    (gss_scn_next_deferred), every block's walk runs from a guess of its start
 *                    on the planner's own stream (gss_spec_device), and the serial chain on the
 *                    host takes one partial cycle per block (gss_carr_chain_spec; exact either
 *                    way, gss_phase.h); the next batch's walks run while this slot is proved.
 *                    With a carrier hand-off (gss_run_ex) the whole range's chain is run ahead
 *                    the same way, in chunks, once the carriers arrive.  GSS_RUN_SPEC=0: the
 *                    host walks every block (gss_scn_next, gss_carr_chain)
 *   main thread      per slot: async H2D; the 30 s producer builds the new nav rows of the
 *                    run's device nav table (gss_nav_rows_device; the C/A table likewise, once
 *                    per run: gss_ca_table_device); gss_synth_lin_device on the compute stream
 *                    (certified blocks on the integer fast path, the rest on Stage A + B; with
 *                    GSS_PATH=walk gss_synth_device renders every block), then async D2H into a
 *                    pinned output buffer on the copy stream (after an event); while the next
 *                    slot renders, hands the previous slot's bytes to the sink in run order
 *
 * Slots cycle planner -> main -> sink -> planner; a slot's buffers belong to exactly one side at
 * a time (state under a mutex).  Shipped defaults (GSS_RUN_NCOPY = 1, GSS_RUN_DEPTH = 2): one
 * compute stream and one copy stream, NSLOT = DEPTH + 2 = 4 slots; DEPTH slots are submitted
 * before the oldest is handed to the sink, so the copy engine always has the next slot's D2H
 * queued behind the current one (DEPTH 1 left it idle while the next slot uploaded and
 * rendered: 12.5 vs 13.4 GS/s, profiles/round3/ablate_r3n.log).  NCOPY = 2 alternates slots over
 * two copy streams (two DMA engines on the link; measured slower, same log).  A slot's device
 * output buffer is rewritten only after its own D2H (event).
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>
#include "gpssim_amd.h"

extern "C" int gss_fail(int code, const char *fmt, ...);
extern "C" void gss_pool_select(int id);             /* pool.c */
/* n bytes from src to dst by a copy kernel on st: pinned host or device memory on either side
   (gss_producers.hip; not exported) */
int run_copy_launch(void *dst, const void *src, size_t n, hipStream_t st);

#define RUN_TRY(x)                                                                           \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess)                                                                \
            return gss_fail(GSS_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_),      \
                            __FILE__, __LINE__);                                             \
    } while (0)

namespace {

/* GSS_RUN_TRACE=1: per-slot timestamps on stderr (planner start/end, submit, drain wait/end) */
static double tnow()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}
static int trace_on()
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("GSS_RUN_TRACE");
        on = e && e[0] == '1';
    }
    return on;
}

#ifndef GSS_RUN_NCOPY
#define GSS_RUN_NCOPY 1
#endif
#ifndef GSS_RUN_DEPTH
#define GSS_RUN_DEPTH 2                                /* profiles/round3/ablate_r3n.log */
#endif
constexpr int NCOPY = GSS_RUN_NCOPY;                   /* copy streams (DMA engines) */
constexpr int DEPTH = GSS_RUN_DEPTH;                   /* slots submitted, not yet drained */
#ifndef GSS_RUN_AHEAD
#define GSS_RUN_AHEAD 2
#endif
constexpr int NSLOT = DEPTH + GSS_RUN_AHEAD;           /* + slots planned / proven ahead */
constexpr size_t SLOT_OUT_MAX = (size_t)256 << 20;     /* pinned output bytes per slot */

enum { FREE, PROVING, PLANNED };                  /* PROVING: rows planned, proofs pending */

/* The slots' output buffers (pinned host + device, ~133 MB each at the defaults) outlive a run:
   page-locking them costs tens of ms, so a later gss_run in the same process (a service, or a
   rank's next window) takes them from this pool instead.  Bounded by POOL_MAX_BYTES (the sizes
   of the buffers themselves); a buffer is reused only for a request of at least half its size,
   and gss_dev_close frees a device's buffers (gss_run_pool_drain). */
namespace {
struct PoolBuf { void *p; size_t n; int dev; bool host; };
std::mutex pool_mu;
std::vector<PoolBuf> pool;
size_t pool_bytes = 0;
constexpr size_t POOL_MAX_BYTES = (size_t)2 << 30;
}  // namespace

/* a buffer of at least n bytes; *got = its actual size, which pool_put must be given back */
static hipError_t pool_get(void **p, size_t n, bool host, int dev, size_t *got)
{
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        for (size_t i = 0; i < pool.size(); i++) {
            const PoolBuf &b = pool[i];
            if (b.host == host && b.dev == dev && b.n >= n && b.n <= 2 * n) {
                *p = b.p;
                *got = b.n;
                pool_bytes -= b.n;
                pool.erase(pool.begin() + (long)i);
                return hipSuccess;
            }
        }
    }
    *got = n;
    return host ? hipHostMalloc(p, n, hipHostMallocDefault) : hipMalloc(p, n);
}

static void pool_put(void *p, size_t n, bool host, int dev)
{
    if (!p)
        return;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        if (pool_bytes + n <= POOL_MAX_BYTES) {
            pool.push_back({p, n, dev, host});
            pool_bytes += n;
            return;
        }
    }
    (void)(host ? hipHostFree(p) : hipFree(p));
}

/* The run's other buffers and its streams outlive it the same way (a run creates a dozen
   streams and pins ~75 MB of rows, lines and walk buffers at 2,048-block slots: most of a short
   run's start-up): pin_alloc / dev_alloc take from the buffer pool and record the
   size they got, so that pin_free / dev_free (any pointer, null included) give it back;
   stream_get / stream_put keep idle non-blocking streams per device and priority. */
namespace {
std::unordered_map<void *, PoolBuf> pool_out;          /* pooled buffers in use, by pointer */
struct PoolStream { hipStream_t s; int dev; int hi; };
std::vector<PoolStream> spool;                         /* idle streams */
std::vector<PoolStream> spool_out;                     /* pooled streams in use */
}  // namespace

static hipError_t pooled_alloc(void **p, size_t n, bool host)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    size_t got = 0;
    *p = nullptr;
    const hipError_t e = pool_get(p, n, host, dev, &got);
    if (e == hipSuccess && *p) {
        std::lock_guard<std::mutex> lk(pool_mu);
        pool_out[*p] = {*p, got, dev, host};
    }
    return e;
}

static void pooled_free(void *p)
{
    if (!p)
        return;
    PoolBuf b;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        const auto it = pool_out.find(p);
        if (it == pool_out.end())
            return;                                    /* not a pooled buffer */
        b = it->second;
        pool_out.erase(it);
    }
    pool_put(b.p, b.n, b.host, b.dev);
}

static hipError_t pin_alloc(void **p, size_t n) { return pooled_alloc(p, n, true); }
static hipError_t dev_alloc(void **p, size_t n) { return pooled_alloc(p, n, false); }
static void pin_free(void *p) { pooled_free(p); }
static void dev_free(void *p) { pooled_free(p); }

/* a non-blocking stream of the current device (hi: the highest priority) */
static hipError_t stream_get(hipStream_t *s, bool hi)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        for (size_t i = 0; i < spool.size(); i++)
            if (spool[i].dev == dev && spool[i].hi == (int)hi) {
                *s = spool[i].s;
                spool_out.push_back(spool[i]);
                spool.erase(spool.begin() + (long)i);
                return hipSuccess;
            }
    }
    hipError_t e;
    if (hi) {
        int lo_pri = 0, hi_pri = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri);
        e = hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi_pri);
    } else {
        e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    }
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(pool_mu);
        spool_out.push_back({*s, dev, (int)hi});
    }
    return e;
}

/* back to the pool when it came from stream_get (the caller has synchronised it), else
   destroyed (the CU-masked streams) */
static void stream_put(hipStream_t s)
{
    if (!s)
        return;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        for (size_t i = 0; i < spool_out.size(); i++)
            if (spool_out[i].s == s) {
                if (spool.size() < 64) {
                    spool.push_back(spool_out[i]);
                    spool_out.erase(spool_out.begin() + (long)i);
                    return;
                }
                spool_out.erase(spool_out.begin() + (long)i);
                break;
            }
    }
    (void)hipStreamDestroy(s);
}

/* free the pooled buffers of device `dev` (gss_dev_close; -1: every device) */
/* The streams a run takes (compute, copy and nav at normal priority; the walks' and one proof
   stream per slot at the highest), made into the pool when the device opens (gss_dev_open):
   creating a high-priority stream costs ~4 ms in a fresh process, and GPU-proof runs take five
   more than host-proof runs (23 ms of a 0.7 s configs[3] run, profiles/round5/e2e/README.md) */
extern "C" void gss_run_pool_prewarm(int dev)
{
    int have[2] = {0, 0};
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        for (const PoolStream &p : spool)
            if (p.dev == dev)
                have[p.hi ? 1 : 0]++;
    }
    int lo_pri = 0, hi_pri = 0;
    if (hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri) != hipSuccess)
        return;
    const int want[2] = {2 + NCOPY, 1 + NSLOT};
    for (int hi = 0; hi < 2; hi++)
        for (; have[hi] < want[hi]; have[hi]++) {
            hipStream_t s = nullptr;
            if ((hi ? hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi_pri)
                    : hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess)
                return;
            std::lock_guard<std::mutex> lk(pool_mu);
            spool.push_back({s, dev, hi});
        }
}

extern "C" void gss_run_pool_drain(int dev)
{
    std::vector<PoolBuf> out;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        for (size_t i = 0; i < pool.size();) {
            if (dev < 0 || pool[i].dev == dev) {
                out.push_back(pool[i]);
                pool_bytes -= pool[i].n;
                pool.erase(pool.begin() + (long)i);
            } else {
                i++;
            }
        }
    }
    std::vector<PoolStream> sout;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        for (size_t i = 0; i < spool.size();) {
            if (dev < 0 || spool[i].dev == dev) {
                sout.push_back(spool[i]);
                spool.erase(spool.begin() + (long)i);
            } else {
                i++;
            }
        }
    }
    for (const PoolBuf &b : out)
        (void)(b.host ? hipHostFree(b.p) : hipFree(b.p));
    for (const PoolStream &q : sout)
        (void)hipStreamDestroy(q.s);
}

struct Slot {
    /* planner side (pinned host memory) */
    gss_chan_blk_t *blk = nullptr;
    int32_t *nch = nullptr;
    double *ck = nullptr;
    gss_nav_src_t *nav = nullptr;    /* sources of the nav rows new with this slot (pinned)  */
    int nav_cap = 0, n_nav = 0;      /* ... capacity, count                                   */
    int nav_first = 0;               /* global row index of the first of them                 */
    gss_lin_t *lin = nullptr;        /* certified lines [nb][GSS_MAXCH] (fast path)      */
    int32_t *fast = nullptr;         /* fast[nb], then the exact-path block list [n_fb] */
    gss_carr_anchor_t *anch = nullptr;   /* the chain's anchors [nb][GSS_MAXCH] (proofs)   */
    int has_anch = 0;                /* ... filled for this use of the slot               */
    int sb_idx = -1;                 /* records mode: the walk batch it came from (its device
                                        walks are the GPU proofs' anchors)                  */
    int n_fb = 0;
    int verdicts = 0;                /* GPU proofs: the exact-path blocks went with the render
                                        (submit_proven), no redo in drain                     */
    int nb = 0, nch_max = 1;
    int64_t first = 0;               /* run index of the slot's first block */
    const uint32_t *lin_nav = nullptr;   /* the nav table its proofs read (prover thread)  */
    int lin_n_nav = 0;
    int end = 0, err = 0;            /* last slot / planner error code      */
    int state = FREE;
    /* main side */
    uint8_t *d_in = nullptr;
    size_t d_in_cap = 0;
    uint8_t *d_out = nullptr, *h_out = nullptr;
    size_t h_out_bytes = 0, d_out_bytes = 0;   /* their sizes (pool_get / pool_put)        */
    int32_t *d_status = nullptr, *h_status = nullptr;
    hipEvent_t rendered = nullptr;   /* compute stream: the slot's kernels are done      */
    hipEvent_t done = nullptr;       /* copy stream: the slot's bytes are in h_out        */
    hipEvent_t tq = nullptr;         /* GSS_RUN_TRACE: the compute stream reached the slot */
    hipEvent_t tk = nullptr;         /* ... its inputs are uploaded (kernels next)        */
    hipEvent_t tc = nullptr;         /* ... the copy stream reached its download          */
    /* GPU proofs, launched by the planner (proof_ahead) */
    hipStream_t pst = nullptr;       /* the slot's proof stream                          */
    hipEvent_t navd = nullptr;       /* its nav rows are built (the planner's nav stream) */
    hipEvent_t proved = nullptr;     /* its rows are on the device and proven            */
    int gpu_proven = 0;              /* this use of the slot is proven on the GPU         */
};

struct Run {
    gss_scn *scn;
    int batch, threads, n_per_blk, use_lin, carrier_int;
    int proof_mode = 0;              /* 0: host proofs, 1: all on the GPU, 2: every other slot */
    int gpu_proof = 0;               /* any proofs on the GPU (gss_proof.hip), run ahead by the
                                        planner on each slot's own stream (proof_ahead)        */
    hipStream_t nav_st = nullptr;    /* ... the planner's stream for the slots' nav rows      */
    hipEvent_t t_base = nullptr;     /* GSS_RUN_TRACE: the GPU clock's origin (compute stream) */
    hipEvent_t ca_ready = nullptr;   /* GPU proofs: the device C/A table is built (compute stream) */
    int upload_dev = 1;              /* uploads by kernel (h2d); GSS_RUN_UPLOAD=dma: copy engine */
    const uint32_t *d_ca = nullptr;  /* the run's device C/A table                            */
    int force_exact;                 /* GSS_RUN_FORCE_EXACT=k: every k-th block to the exact
                                        path (tests of the mixed batch), 0 = off */
    int late_verdicts = 0;           /* GSS_RUN_LATE_VERDICTS=1 (tests): submit_proven treats every
                                        GPU proof as still running, so rejected blocks always take
                                        the redo path in drain (redo_rejected)            */
    int64_t first, last;             /* [first, last) block range of the run */
    int64_t start = 0;               /* the handle's next block when the run began (an earlier
                                        run, a seek): the planner's and rows thread's cursor   */
    const gss_run_opts_t *opts;      /* carrier hand-off (gss_run_ex), or null */
    /* with opts->carr_in: the whole range planned up front (rows, carriers, checkpoints) */
    std::vector<gss_chan_blk_t> pre_blk;
    std::vector<int32_t> pre_nch;
    std::vector<double> pre_ck;
    int64_t pre_n = 0, pre_at = 0;
    std::mutex mu;
    std::condition_variable cv;
    int abort = 0;
    uint32_t ca[32 * GSS_CA_WORDS];  /* C/A chips (gss_ca_table) for the proofs' patch terms */
    int nav_planned = 0;             /* nav rows whose sources a slot has taken (planner)      */
    uint32_t *d_nav = nullptr;       /* the run's nav table on the device, built by the GPU   */
    size_t d_nav_cap = 0;            /* producer (gss_nav_rows_device); rows                   */
    /* the carrier chain run ahead (planner thread): two batches, so that the GPU walks of the
       next one run while this slot's proofs do */
    struct SpecBatch {
        std::vector<gss_chan_blk_t> blk;
        std::vector<int32_t> nch;
        std::vector<gss_chain_t> chain;
        gss_spec_in_t *h_in = nullptr;        /* pinned host, read and written by the lanes */
        gss_spec_t *h_spec = nullptr;
        /* records mode (r.rec): the walks and guesses stay on the device (d_in, d_spec) and
           only each row's record comes back (h_rec, pinned) */
        gss_spec_in_t *d_in = nullptr;
        gss_spec_t *d_spec = nullptr;
        gss_spec_rec_t *h_rec = nullptr;
        hipEvent_t consumed = nullptr;        /* a slot's GPU proof has read d_in / d_spec */
        int consumed_pending = 0;
        double carr[GSS_MAXCH];                              /* exact, at its first block */
        int nb = 0, launched = 0;
        double tg = 0.0, tk = 0.0;                           /* trace: guess start, launch end */
        hipEvent_t walked = nullptr;          /* spec stream: this batch's walks are done      */
    } sb[3];
    int sb_cur = 0;
    int sb_head = 0, n_fly = 0, fly_end = 0;   /* rows_ahead: walks in flight (FIFO from
                                                  sb_head), and whether the rows have ended */
    /* the rows produced ahead on their own thread (chain run ahead, no hand-off): during the run
       the scenario belongs to that thread; it hands over each batch's rows with the nav rows and
       sources new with it, and the planner keeps the slot carriers and host copies of the nav
       table (the proofs read it) */
    struct RowBatch {
        std::vector<gss_chan_blk_t> blk;
        std::vector<int32_t> nch;
        std::vector<gss_chain_t> chain;
        std::vector<gss_nav_src_t> nav_src;
        std::vector<uint32_t> nav_rows;
        int64_t first = 0;
        int nb = 0, end = 0, err = 0, ready = 0;
        double t0 = 0.0, t1 = 0.0;                           /* trace: production start, end */
    } rb[2];
    int rows_ahead = 0, rb_take = 0, rows_done = 0;
    int prover = 0;                  /* proofs on their own thread (rows_ahead, fast path): the
                                        planner hands slots over PROVING */
    double carr[GSS_MAXCH];          /* rows_ahead: the slot carriers at the planner's next batch */
    std::vector<gss_nav_src_t> nav_src_h;
    std::vector<uint32_t> nav_rows_h;
    gss_dev *dev = nullptr;
    int spec = 0;                    /* per batch (gss_run), or over the range (hand-off)      */
    int rec = 0;                     /* per batch: records, not walks, back from the GPU
                                        (gss_spec_records_device; GSS_RUN_REC=0: the walks)    */
    int dev_anch = 0;                /* records mode: GPU proofs take their anchors from the
                                        batch's device walks (GSS_RUN_DEV_ANCHORS=1).  Off: the
                                        configs[4] run measured 43.2-43.4 GB/s with them against
                                        43.8-44.8 without (profiles/round5/e2e/probe_r5s)      */
    hipStream_t spec_st = nullptr;
    uint64_t *spec_warm = nullptr;   /* device scratch of the walks' first launch (one row) */
    int64_t spec_rows = 0, spec_hits = 0;
    Slot slot[NSLOT];
};

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
/* the walks' warm-up scratch (one row): in, its device copy, the walk, the record */
constexpr size_t WARM_IN = (sizeof(gss_spec_in_t) + 255) & ~(size_t)255;
constexpr size_t WARM_SPEC = (sizeof(gss_spec_t) + 255) & ~(size_t)255;
constexpr size_t WARM_BYTES = 2 * WARM_IN + WARM_SPEC + 128;
static_assert(sizeof(gss_spec_rec_t) <= 128, "the record fits its warm-up slot");

/* The carrier checkpoints feed only the exact path's Stage A, i.e. the blocks the proofs do not
   certify (none of the 2,999 of the bench run).  With the fast path the chain is therefore
   walked without them (a third cheaper: no partial-cycle walks to the 8 checkpoint positions)
   and they are computed afterwards for the uncertified blocks only, from each row's carr0 by
   the same exact walk.  The integer-carrier chain records them for free and keeps doing so. */
static bool lazy_ck(const Run &r) { return r.use_lin && !r.carrier_int; }

/* Uploads of the slots' inputs (rows, lines, checkpoints, nav sources: ~10 MB per 2048-block
   slot) by a kernel reading the pinned host buffers directly, not by the copy engine
   (run_copy_launch, gss_producers.hip): an engine copy queues behind the download of the slot
   before (the same engine, FIFO), so each slot's render started only once the previous slot's
   bytes were out, and the downloads ran at 0.78 of the link (tools/d2h_overlap.py: a 10 MB
   upload issued during a 133 MB download finishes with it, 2.09 ms instead of 0.20).  The
   kernel's reads go host-to-device, the downloads device-to-host: the two directions of the
   link overlap. */
static int dev_copy(void *dst, const void *src, size_t n, hipStream_t st)
{
    return run_copy_launch(dst, src, n, st);
}

/* host buffer (pinned) to device, stream-ordered on st */
static int h2d(const Run &r, void *dst, const void *src, size_t n, hipStream_t st)
{
    if (n == 0 || r.upload_dev)
        return dev_copy(dst, src, n, st);
    return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st) == hipSuccess
               ? 0 : gss_fail(GSS_E_HIP, "upload of %zu B", n);
}
#define RUN_H2D(dst, src, n, st)                                                          \
    do {                                                                                  \
        int rc_ = h2d(r, (dst), (src), (n), (st));                                        \
        if (rc_) return rc_;                                                              \
    } while (0)

}  // namespace
int run_proof_launch(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                     const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                     const gss_carr_anchor_t *anch, const gss_spec_in_t *sin,
                     const gss_spec_t *sspec, gss_lin_t *lin, int32_t *fast, int64_t first,
                     int force_exact, hipStream_t st);            /* gss_proof.hip */
namespace {

static void fill_fb_ck(const Run &r, Slot &sl)
{
    if (r.force_exact > 0) {
        for (int i = 0; i < sl.nb; i++)
            if ((sl.first + i) % r.force_exact == 0)
                sl.fast[i] = 0;
        int nf = 0;
        for (int i = 0; i < sl.nb; i++)
            if (!sl.fast[i])
                sl.fast[sl.nb + nf++] = i;
        sl.n_fb = nf;
    }
    if (!lazy_ck(r))
        return;
    for (int i = 0; i < sl.n_fb; i++) {
        const int b = sl.fast[sl.nb + i];
        for (int k = 0; k < sl.nch[b]; k++) {
            const size_t e = (size_t)b * GSS_MAXCH + k;
            (void)gss_carr_advance_ck(sl.blk[e].carr0, sl.blk[e].carr_step, r.n_per_blk,
                                      sl.ck + e * GSS_NCK);
        }
    }
}

/* The up-front range's chain run ahead on the GPU, in chunks of 4,096 blocks: each chunk's
   guesses from the exact carriers at its start, its walks, then its chain (exact). */
int chain_upfront_spec(Run &r, double *carr, const gss_chain_t *chain)
{
    constexpr int CH = 4096;
    const size_t rows_max = (size_t)CH * GSS_MAXCH;
    gss_spec_in_t *h_in = nullptr;                     /* pinned: the lanes use them directly */
    gss_spec_t *h_spec = nullptr;
    int rc = 0;
    if (pin_alloc((void **)&h_in, sizeof(gss_spec_in_t) * rows_max) !=
            hipSuccess ||
        pin_alloc((void **)&h_spec, sizeof(gss_spec_t) * rows_max) !=
            hipSuccess)
        rc = gss_fail(GSS_E_NOMEM, "carrier-chain buffers (%zu rows)", rows_max);
    int64_t hits = 0, n_rows = 0;
    for (int64_t b0 = 0; !rc && b0 < r.pre_n; b0 += CH) {
        const int nb = r.pre_n - b0 < CH ? (int)(r.pre_n - b0) : CH;
        const int nrow = nb * GSS_MAXCH;
        gss_chan_blk_t *blk = &r.pre_blk[(size_t)b0 * GSS_MAXCH];
        const int32_t *nch = &r.pre_nch[(size_t)b0];
        const gss_chain_t *ch = chain + (size_t)b0 * GSS_MAXCH;
        rc = gss_carr_chain_starts(carr, blk, nch, ch, nb, r.n_per_blk, h_in);
        if (rc) break;
        if ((rc = gss_spec_device(r.dev, h_in, nrow, r.n_per_blk, h_spec, r.spec_st)) != 0 ||
            hipStreamSynchronize(r.spec_st) != hipSuccess) {
            if (!rc) rc = gss_fail(GSS_E_HIP, "carrier-chain walks");
            break;
        }
        int hit = 0;
        rc = gss_carr_chain_spec(carr, blk, nch, ch, nb, r.n_per_blk, h_in, h_spec, r.threads,
                                 &hit);
        hits += hit;
        for (int i = 0; i < nb; i++)
            n_rows += nch[i];
    }
    if (trace_on())
        fprintf(stderr, "trace spec upfront rows %lld hits %lld\n", (long long)n_rows,
                (long long)hits);
    pin_free(h_in); pin_free(h_spec);
    return rc;
}

/* The walks' records of every row of the up-front range, CH blocks per launch, from starts per
   row (g: [pre_n][GSS_MAXCH]) or, without them, from the lines out of carr (the first pass) */
int upfront_records(Run &r, const gss_chain_t *chain, const double *carr, const double *g,
                    std::vector<gss_spec_rec_t> &rec)
{
    constexpr int CH = 4096;
    const size_t rows_max = (size_t)CH * GSS_MAXCH;
    gss_spec_in_t *h_in = nullptr, *d_in = nullptr;
    gss_spec_t *d_spec = nullptr;
    gss_spec_rec_t *h_rec = nullptr;
    int rc = 0;
    if (pin_alloc((void **)&h_in, sizeof(gss_spec_in_t) * rows_max) != hipSuccess ||
        pin_alloc((void **)&h_rec, sizeof(gss_spec_rec_t) * rows_max) != hipSuccess ||
        dev_alloc((void **)&d_in, sizeof(gss_spec_in_t) * rows_max) != hipSuccess ||
        dev_alloc((void **)&d_spec, sizeof(gss_spec_t) * rows_max) != hipSuccess)
        rc = gss_fail(GSS_E_NOMEM, "carrier-chain buffers (%zu rows)", rows_max);
    rec.resize((size_t)r.pre_n * GSS_MAXCH);
    double c[GSS_MAXCH];
    memcpy(c, carr, sizeof c);
    for (int64_t b0 = 0; !rc && b0 < r.pre_n; b0 += CH) {
        const int nb = r.pre_n - b0 < CH ? (int)(r.pre_n - b0) : CH;
        const int nrow = nb * GSS_MAXCH;
        const gss_chan_blk_t *blk = &r.pre_blk[(size_t)b0 * GSS_MAXCH];
        const int32_t *nch = &r.pre_nch[(size_t)b0];
        const gss_chain_t *ch = chain + (size_t)b0 * GSS_MAXCH;
        rc = gss_carr_chain_starts(c, blk, nch, ch, nb, r.n_per_blk, h_in);   /* k, s, pad */
        if (rc) break;
        if (g) {                                       /* the given starts instead of lines */
            for (int i = 0; i < nrow; i++)
                if (h_in[i].k == 0)
                    h_in[i].g = g[(size_t)b0 * GSS_MAXCH + i];
        } else {
            (void)gss_carr_line_end(c, blk, nch, ch, nb, r.n_per_blk, c);
        }
        if ((rc = gss_spec_records_device(r.dev, h_in, nrow, r.n_per_blk, d_in, d_spec, h_rec,
                                          r.spec_st)) != 0 ||
            hipStreamSynchronize(r.spec_st) != hipSuccess) {
            if (!rc) rc = gss_fail(GSS_E_HIP, "carrier-chain records");
            break;
        }
        memcpy(&rec[(size_t)b0 * GSS_MAXCH], h_rec, sizeof(gss_spec_rec_t) * (size_t)nrow);
    }
    pin_free(h_in); pin_free(h_rec); dev_free(d_in); dev_free(d_spec);
    return rc;
}

/* The up-front chain speculated across ranks (opts->carr_predict; shard.chain_speculated's
   steps): the range's map by the lines -> a predicted start -> walks and records from it -> the
   exact chain from that start and its map -> a second, ~1e-13 prediction -> the rows whose
   carrier depends on the start walked again from the first chain's carriers moved by the
   correction -> carr_in -> the records' chain (a compare and two adds per row where the
   links hold) -> carr_out.  Exact whatever the predictions. */
int chain_upfront_speculated(Run &r, const gss_chain_t *chain, const double *start0,
                             double *carr)
{
    const int64_t nb = r.pre_n;
    const size_t rows = (size_t)nb * GSS_MAXCH;
    const double t0 = tnow();
    int reset[GSS_MAXCH] = {0};
    for (int64_t b = 0; b < nb; b++)
        for (int k = 0; k < r.pre_nch[(size_t)b] && k < GSS_MAXCH; k++) {
            const gss_chain_t &c = chain[(size_t)b * GSS_MAXCH + k];
            if (c.reset && c.slot >= 0 && c.slot < GSS_MAXCH)
                reset[c.slot] = 1;
        }
    const bool exact0 = r.first == 0;                   /* the run's own start: no prediction */
    double zero[GSS_MAXCH] = {0}, end[GSS_MAXCH], map[3 * GSS_MAXCH], x0[GSS_MAXCH],
        x1[GSS_MAXCH];
    int rc = gss_carr_line_end(zero, r.pre_blk.data(), r.pre_nch.data(), chain, (int)nb,
                               r.n_per_blk, end);
    auto make_map = [&](const double *from, const double *to) {
        for (int i = 0; i < GSS_MAXCH; i++) {
            map[i] = exact0 ? start0[i] : 0.0;
            const double a = to[i] - from[i];
            map[GSS_MAXCH + i] = reset[i] ? to[i] : a - floor(a);
            map[2 * GSS_MAXCH + i] = reset[i] ? 1.0 : 0.0;
        }
    };
    make_map(zero, end);
    if (!rc && r.opts->carr_predict(r.opts->carr_user, 0, map, x0))
        rc = gss_fail(GSS_E_IO, "carrier prediction (round 0) failed at block %lld",
                      (long long)r.first);
    if (rc)
        return rc;
    if (exact0)
        memcpy(x0, start0, sizeof x0);
    std::vector<gss_spec_rec_t> rec;
    rc = upfront_records(r, chain, x0, nullptr, rec);
    if (rc)
        return rc;
    std::vector<gss_chan_blk_t> first(r.pre_blk);      /* the chain from the predicted start */
    double e0[GSS_MAXCH];
    memcpy(e0, x0, sizeof e0);
    int hit = 0;
    rc = gss_carr_chain_records(e0, first.data(), r.pre_nch.data(), chain, (int)nb, r.n_per_blk,
                                rec.data(), r.threads, &hit);
    if (rc)
        return rc;
    make_map(x0, e0);
    if (r.opts->carr_predict(r.opts->carr_user, 1, map, x1))
        return gss_fail(GSS_E_IO, "carrier prediction (round 1) failed at block %lld",
                        (long long)r.first);
    if (exact0)
        memcpy(x1, x0, sizeof x1);
    double d[GSS_MAXCH];
    bool moved = false;
    for (int i = 0; i < GSS_MAXCH; i++) {
        const double v = x1[i] - x0[i] + 0.5;
        d[i] = (v - floor(v)) - 0.5;
        moved = moved || (d[i] != 0.0 && !reset[i]);
    }
    int64_t rewalked = 0;
    if (moved) {                                       /* the start-dependent rows, corrected */
        std::vector<double> g(rows);
        int seen_reset[GSS_MAXCH] = {0};
        for (int64_t b = 0; b < nb; b++)
            for (int k = 0; k < GSS_MAXCH; k++) {
                const size_t e = (size_t)b * GSS_MAXCH + k;
                g[e] = first[e].carr0;
                if (k >= r.pre_nch[(size_t)b])
                    continue;
                const int sl = chain[e].slot;
                if (sl < 0 || sl >= GSS_MAXCH)
                    continue;
                if (chain[e].reset)
                    seen_reset[sl] = 1;
                if (!seen_reset[sl]) {
                    const double v = first[e].carr0 + d[sl];
                    g[e] = v - floor(v);
                    rewalked++;
                }
            }
        rc = upfront_records(r, chain, x1, g.data(), rec);
        if (rc)
            return rc;
    }
    const double t1 = tnow();
    if (r.opts->carr_in(r.opts->carr_user, carr))
        return gss_fail(GSS_E_IO, "carrier hand-off (in) failed at block %lld",
                        (long long)r.first);
    const double t2 = tnow();
    rc = gss_carr_chain_records(carr, r.pre_blk.data(), r.pre_nch.data(), chain, (int)nb,
                                r.n_per_blk, rec.data(), r.threads, &hit);
    if (trace_on())
        fprintf(stderr, "trace spec speculated rows %zu hits %d rewalked %lld pre %.6f wait %.6f "
                "handoff %.6f\n", rows, hit, (long long)rewalked, t1 - t0, t2 - t1, tnow() - t2);
    return rc;
}

/* gss_run_ex with a carrier hand-off: seek to the range, produce its rows, take the slot
   carriers at its first block from carr_in, walk the chain, give the end state to carr_out. */
int plan_range_upfront(Run &r)
{
    int rc = gss_scn_seek(r.scn, r.first, r.threads);
    if (rc)
        return rc;
    /* the speculated chain: with a prediction callback and the walks on the GPU */
    const bool speculate = r.opts->carr_predict && r.spec && r.rec;
    /* a prediction callback this rank will not use (GSS_RUN_SPEC=0, GSS_RUN_REC=0, the exact
       path): round -1 tells the ranks after it not to wait for its maps */
    if (r.opts->carr_predict && !speculate &&
        r.opts->carr_predict(r.opts->carr_user, -1, nullptr, nullptr))
        return gss_fail(GSS_E_IO, "carrier hand-off: publishing the no-speculation marker");
    double start0[GSS_MAXCH] = {0};
    if (speculate && r.first == 0 && (rc = gss_scn_carrier(r.scn, start0)) != 0)
        return rc;
    std::vector<gss_chain_t> chain;
    const int step = 4096;
    for (;;) {
        const int64_t want = r.last - r.first - r.pre_n;
        if (want <= 0)
            break;
        const int ask = want < step ? (int)want : step;
        r.pre_blk.resize((size_t)(r.pre_n + ask) * GSS_MAXCH);
        r.pre_nch.resize((size_t)(r.pre_n + ask));
        chain.resize((size_t)(r.pre_n + ask) * GSS_MAXCH);
        int nb = 0;
        rc = gss_scn_next_deferred(r.scn, ask, &r.pre_blk[(size_t)r.pre_n * GSS_MAXCH],
                                   &r.pre_nch[(size_t)r.pre_n],
                                   &chain[(size_t)r.pre_n * GSS_MAXCH], &nb, r.threads);
        if (rc)
            return rc;
        r.pre_n += nb;
        if (nb < ask)
            break;                                     /* end of the run */
    }
    double carr[GSS_MAXCH];
    if (!lazy_ck(r))
        r.pre_ck.resize((size_t)r.pre_n * GSS_MAXCH * GSS_NCK);
    if (speculate) {
        rc = chain_upfront_speculated(r, chain.data(), start0, carr);
        if (rc)
            return rc;
        if (r.opts->carr_out && r.opts->carr_out(r.opts->carr_user, carr))
            return gss_fail(GSS_E_IO, "carrier hand-off (out) failed after block %lld",
                            (long long)(r.first + r.pre_n - 1));
        return 0;
    }
    if (r.opts->carr_in(r.opts->carr_user, carr))
        return gss_fail(GSS_E_IO, "carrier hand-off (in) failed at block %lld",
                        (long long)r.first);
    if (r.spec)                                        /* the chain run ahead on the GPU */
        rc = chain_upfront_spec(r, carr, chain.data());
    else
        rc = gss_carr_chain(carr, r.pre_blk.data(), r.pre_nch.data(), chain.data(),
                            (int)r.pre_n, r.n_per_blk, r.carrier_int,
                            lazy_ck(r) ? nullptr : r.pre_ck.data(), r.threads);
    if (rc)
        return rc;
    if (r.opts->carr_out && r.opts->carr_out(r.opts->carr_user, carr))
        return gss_fail(GSS_E_IO, "carrier hand-off (out) failed after block %lld",
                        (long long)(r.first + r.pre_n - 1));
    return 0;
}

/* The nav rows new since the previous slot, as sources for the GPU producer: rows
   [r.nav_planned, upto) of the scenario's table (rows are appended in run order). */
int take_nav_sources(Run &r, Slot &sl, int upto)
{
    const gss_nav_src_t *src = nullptr;
    int n_all = 0;
    if (r.rows_ahead) {
        src = r.nav_src_h.data();
        n_all = (int)r.nav_src_h.size();
    } else {
        gss_scn_nav_sources(r.scn, &src, &n_all);
    }
    if (upto > n_all)
        upto = n_all;
    const int n = upto > r.nav_planned ? upto - r.nav_planned : 0;
    if (n > sl.nav_cap) {
        pin_free(sl.nav);
        sl.nav = nullptr;
        sl.nav_cap = 0;
        const int cap = n * 2 + 16;
        if (pin_alloc((void **)&sl.nav, sizeof(gss_nav_src_t) * (size_t)cap) != hipSuccess)
            return gss_fail(GSS_E_NOMEM, "pinned nav sources");
        sl.nav_cap = cap;
    }
    if (n > 0)
        memcpy(sl.nav, src + r.nav_planned, sizeof(gss_nav_src_t) * (size_t)n);
    /* the chains' next links within the slot's rows, from their prev links: the rows thread's
       copies (nav_src_h) were taken when each row was new, before its successor existed, and
       gss_nav_kernel reaches every row but a chain's head through them */
    for (int i = 0; i < n; i++)
        sl.nav[i].next = -1;
    for (int i = 0; i < n; i++) {
        const int pv = sl.nav[i].prev;
        if (pv >= r.nav_planned && pv < r.nav_planned + i)
            sl.nav[pv - r.nav_planned].next = r.nav_planned + i;
    }
    sl.nav_first = r.nav_planned;
    sl.n_nav = n;
    r.nav_planned += n;
    return 0;
}

/* the slot's batch from the up-front plan (rows keep their global nav indices) */
int take_upfront(Run &r, Slot &sl, int *nb_out)
{
    const int64_t left = r.pre_n - r.pre_at;
    const int nb = left < r.batch ? (int)left : r.batch;
    *nb_out = nb;
    if (nb <= 0)
        return 0;
    const size_t rows = (size_t)nb * GSS_MAXCH;
    memcpy(sl.blk, &r.pre_blk[(size_t)r.pre_at * GSS_MAXCH], rows * sizeof(gss_chan_blk_t));
    memcpy(sl.nch, &r.pre_nch[(size_t)r.pre_at], (size_t)nb * sizeof(int32_t));
    if (!lazy_ck(r))
        memcpy(sl.ck, &r.pre_ck[(size_t)r.pre_at * GSS_MAXCH * GSS_NCK],
               rows * GSS_NCK * sizeof(double));
    int hi = -1;
    for (int b = 0; b < nb; b++)
        for (int k = 0; k < sl.nch[b]; k++) {
            const int t = sl.blk[(size_t)b * GSS_MAXCH + k].nav_tbl;
            hi = t > hi ? t : hi;
        }
    const int rc = take_nav_sources(r, sl, hi + 1);
    if (rc)
        return rc;
    sl.first = r.first + r.pre_at;
    r.pre_at += nb;
    return 0;
}

/* The carrier chain run ahead on the GPU (see the header), in two steps per batch:
   spec_launch produces the batch's rows (carriers deferred) and its guesses and queues the GPU
   walks; spec_finish waits for them, walks the chain (exact) and hands the rows over.  The
   planner launches batch k+1 right after finishing batch k, so that k+1's walks run on the GPU
   while k's proofs run on the host. */
/* next_ask's batches in run order, produced ahead of the planner (rows_ahead): the scenario's
   rows with their carriers deferred, and the nav rows and sources new with each batch */
int next_ask(const Run &r, int64_t cursor);

void rows_thread(Run *r)
{
    {
        const char *e = getenv("GSS_RUN_ROWS_POOL");   /* 0: share the planner's workers */
        gss_pool_select(e && e[0] == '0' ? 0 : 1);
    }
    int64_t cursor = r->start;
    int nav_done = 0;
    for (int i = 0;; i++) {
        Run::RowBatch &q = r->rb[i & 1];
        {
            std::unique_lock<std::mutex> lk(r->mu);
            r->cv.wait(lk, [&] { return r->abort || !q.ready; });
            if (r->abort)
                break;
        }
        const int ask = next_ask(*r, cursor);
        if (ask <= 0)
            break;                                     /* the planner asks no further */
        q.t0 = trace_on() ? tnow() : 0.0;
        int nb = 0;
        int rc = gss_scn_next_deferred(r->scn, ask, q.blk.data(), q.nch.data(), q.chain.data(),
                                       &nb, r->threads);
        const gss_nav_src_t *src = nullptr;
        const uint32_t *rows = nullptr;
        int n_src = 0, n_rows = 0;
        if (!rc)
            rc = gss_scn_nav_sources(r->scn, &src, &n_src);
        if (!rc)
            rc = gss_scn_nav_table(r->scn, &rows, &n_rows);
        if (!rc && (n_src != n_rows || n_src < nav_done))
            rc = gss_fail(GSS_E_STATE, "nav table and sources out of step");
        if (!rc) {
            q.nav_src.assign(src + nav_done, src + n_src);
            q.nav_rows.assign(rows + (size_t)nav_done * GSS_NAV_WORDS,
                              rows + (size_t)n_rows * GSS_NAV_WORDS);
            nav_done = n_src;
        }
        q.first = cursor;
        q.nb = nb;
        q.err = rc;
        q.end = rc || nb == 0;
        cursor += nb;
        q.t1 = trace_on() ? tnow() : 0.0;
        {
            std::lock_guard<std::mutex> lk(r->mu);
            q.ready = 1;
        }
        r->cv.notify_all();
        if (q.end)
            break;
    }
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->rows_done = 1;
    }
    r->cv.notify_all();
}

/* the next batch of rows_ahead into b (vectors swapped, no copy); its nav rows and sources onto
   the planner's copies */
int take_rows(Run &r, Run::SpecBatch &b, int *nb_out)
{
    *nb_out = 0;
    Run::RowBatch &q = r.rb[r.rb_take];
    const double tw = trace_on() ? tnow() : 0.0;
    {
        std::unique_lock<std::mutex> lk(r.mu);
        r.cv.wait(lk, [&] { return r.abort || q.ready || r.rows_done; });
        if (!q.ready)
            return gss_fail(GSS_E_STATE, r.abort ? "run aborted" : "rows ended before the run");
    }
    if (q.err)
        return q.err;
    std::swap(b.blk, q.blk);
    std::swap(b.nch, q.nch);
    std::swap(b.chain, q.chain);
    if (r.nav_rows_h.size() + q.nav_rows.size() > r.nav_rows_h.capacity()) {
        /* beyond the reservation (not expected): the prover reads the table, so grow it only
           with no slot in its hands */
        std::unique_lock<std::mutex> lk(r.mu);
        r.cv.wait(lk, [&] {
            for (const Slot &x : r.slot)
                if (x.state == PROVING)
                    return r.abort != 0;
            return true;
        });
        if (r.abort)
            return gss_fail(GSS_E_STATE, "run aborted");
    }
    r.nav_src_h.insert(r.nav_src_h.end(), q.nav_src.begin(), q.nav_src.end());
    r.nav_rows_h.insert(r.nav_rows_h.end(), q.nav_rows.begin(), q.nav_rows.end());
    *nb_out = q.nb;
    if (trace_on())
        fprintf(stderr, "trace rows nb %d produced %.6f %.6f wait %.6f\n", q.nb, q.t0, q.t1,
                tnow() - tw);
    {
        std::lock_guard<std::mutex> lk(r.mu);
        q.ready = 0;
    }
    r.cv.notify_all();
    r.rb_take ^= 1;
    return 0;
}

int spec_launch(Run &r, Run::SpecBatch &b, int ask)
{
    b.nb = 0;
    b.launched = 1;
    int rc = 0, nb = 0;
    if (r.rows_ahead) {
        /* the finished batches' exact carriers, carried by the lines through the batch still in
           flight (if any): a prediction, ~3e-10 cycle off, which only the guesses use */
        memcpy(b.carr, r.carr, sizeof b.carr);
        for (int f = 0; f < r.n_fly; f++) {
            const Run::SpecBatch &p = r.sb[(r.sb_head + f) % 3];
            if (p.nb > 0)
                (void)gss_carr_line_end(b.carr, p.blk.data(), p.nch.data(), p.chain.data(), p.nb,
                                        r.n_per_blk, b.carr);
        }
        rc = take_rows(r, b, &nb);
    } else {
        rc = gss_scn_carrier(r.scn, b.carr);
        if (!rc)
            rc = gss_scn_next_deferred(r.scn, ask, b.blk.data(), b.nch.data(), b.chain.data(),
                                       &nb, r.threads);
    }
    if (rc || nb == 0)
        return rc;
    b.nb = nb;
    const int nrow = nb * GSS_MAXCH;
    b.tg = trace_on() ? tnow() : 0.0;
    rc = gss_carr_chain_starts(b.carr, b.blk.data(), b.nch.data(), b.chain.data(), nb,
                               r.n_per_blk, b.h_in);           /* the walkers guess the rest */
    if (rc)
        return rc;
    /* the lanes read their rows from, and write their walks to, the pinned host buffers
       directly (a few hundred bytes each): no copy engine in the loop (it queues behind the
       slots' downloads).  Staging them through device memory by copy kernels (one pass of
       16-byte copies each way) measured the same: the downloads beside them run at ~0.8 of the
       link either way, the walks' own traffic (~14 MB per 2048-block slot back to the host,
       with the 10 MB of uploads) sharing its device-to-host direction */
    if (b.consumed_pending) {            /* a GPU proof still reads the batch's device walks */
        RUN_TRY(hipStreamWaitEvent(r.spec_st, b.consumed, 0));
        b.consumed_pending = 0;
    }
    rc = r.rec ? gss_spec_records_device(r.dev, b.h_in, nrow, r.n_per_blk, b.d_in, b.d_spec,
                                         b.h_rec, r.spec_st)
               : gss_spec_device(r.dev, b.h_in, nrow, r.n_per_blk, b.h_spec, r.spec_st);
    if (rc)
        return rc;
    RUN_TRY(hipEventRecord(b.walked, r.spec_st));    /* not the stream: later batches queue */
    b.tk = trace_on() ? tnow() : 0.0;
    return 0;
}

/* the batch's chain; anch (NULL: none): its anchors for the slot's proofs */
int spec_finish(Run &r, Run::SpecBatch &b, gss_chan_blk_t *blk, int32_t *nch, int *nb_out,
                gss_carr_anchor_t *anch)
{
    b.launched = 0;
    *nb_out = 0;
    const int nb = b.nb;
    b.nb = 0;
    if (nb == 0)
        return 0;
    const double tw = trace_on() ? tnow() : 0.0;
    RUN_TRY(hipEventSynchronize(b.walked));
    const double t0 = trace_on() ? tnow() : 0.0;
    double carr[GSS_MAXCH];                          /* exact: the batches before are done */
    memcpy(carr, r.rows_ahead ? r.carr : b.carr, sizeof carr);
    int hit = 0;
    int rc = r.rec ? gss_carr_chain_records(carr, b.blk.data(), b.nch.data(), b.chain.data(), nb,
                                            r.n_per_blk, b.h_rec, r.threads, &hit)
                   : gss_carr_chain_anchored(carr, b.blk.data(), b.nch.data(), b.chain.data(),
                                             nb, r.n_per_blk, b.h_in, b.h_spec, r.threads, &hit,
                                             anch);
    if (rc)
        return rc;
    if (r.rows_ahead)
        memcpy(r.carr, carr, sizeof carr);             /* the scenario is the rows thread's */
    else
        rc = gss_scn_set_carrier(r.scn, carr);
    if (rc)
        return rc;
    memcpy(blk, b.blk.data(), sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)nb);
    memcpy(nch, b.nch.data(), sizeof(int32_t) * (size_t)nb);
    int rows = 0;
    for (int i = 0; i < nb; i++)
        rows += nch[i];
    r.spec_rows += rows;
    r.spec_hits += hit;
    if (trace_on())
        fprintf(stderr, "trace spec nb %d rows %d hits %d guess %.6f gpu_wait %.6f chain %.6f\n",
                nb, rows, hit, b.tk - b.tg, t0 - tw, tnow() - t0);
    *nb_out = nb;
    return 0;
}

/* the next batch's size from the cursor: stops exactly at the range start and at its end */
int next_ask(const Run &r, int64_t cursor)
{
    const int64_t want = r.last - cursor;
    if (want <= 0)
        return 0;
    int ask = want < r.batch ? (int)want : r.batch;
    if (cursor < r.first && r.first - cursor < ask)
        ask = (int)(r.first - cursor);
    return ask;
}

/* Fill slot k's pinned buffers with the next batch inside [first, last); without a carrier
   hand-off, blocks before `first` are planned (the carrier chain is serial) and dropped. */
int plan_into(Run &r, Slot &sl, int64_t *cursor)
{
    sl.has_anch = 0;
    sl.sb_idx = -1;
    if (r.opts && r.opts->carr_in) {
        int nb = 0;
        int rc = take_upfront(r, sl, &nb);
        if (rc)
            return rc;
        if (nb == 0) {
            sl.nb = 0;
            sl.end = 1;
            return 0;
        }
        sl.nb = nb;
        int m = 1;
        for (int i = 0; i < nb; i++)
            m = sl.nch[i] > m ? sl.nch[i] : m;
        sl.nch_max = m;
        sl.n_fb = 0;
        if (r.use_lin && !sl.gpu_proven) {
            const uint32_t *rows = nullptr;
            int n_rows = 0;
            gss_scn_nav_table(r.scn, &rows, &n_rows);
            rc = gss_linearize(sl.blk, sl.nch, nb, r.n_per_blk, r.ca, 32, rows, n_rows,
                               sl.lin, sl.fast, r.threads);
            if (rc)
                return rc;
            int nf = 0;
            for (int i = 0; i < nb; i++)
                if (!sl.fast[i])
                    sl.fast[nb + nf++] = i;
            sl.n_fb = nf;
            fill_fb_ck(r, sl);
        }
        return 0;
    }
    for (;;) {
        const int ask = next_ask(r, *cursor);
        int nb = 0;
        int rc = 0;
        if (r.rows_ahead) {
            /* two batches' walks in flight: the oldest is finished (its chain, exact) while the
               next one's walks run on the GPU; the batch after that is launched first */
            while (!rc && r.n_fly < 2 && !r.fly_end) {
                int64_t lc = *cursor;
                for (int f = 0; f < r.n_fly; f++)
                    lc += r.sb[(r.sb_head + f) % 3].nb;
                const int a = next_ask(r, lc);
                if (a <= 0)
                    break;
                Run::SpecBatch &b = r.sb[(r.sb_head + r.n_fly) % 3];
                rc = spec_launch(r, b, a);
                r.n_fly++;
                if (!rc && b.nb == 0)
                    r.fly_end = 1;                     /* the scenario's end */
            }
            if (!rc && r.n_fly > 0) {
                rc = spec_finish(r, r.sb[r.sb_head], sl.blk, sl.nch, &nb, sl.anch);
                sl.sb_idx = r.sb_head;
                r.sb_head = (r.sb_head + 1) % 3;
                r.n_fly--;
            }
        } else if (r.spec) {
            Run::SpecBatch &b = r.sb[r.sb_cur];
            if (!b.launched && ask > 0)
                rc = spec_launch(r, b, ask);
            if (!rc && b.launched) {                   /* else the range is done: nb stays 0 */
                rc = spec_finish(r, b, sl.blk, sl.nch, &nb, sl.anch);
                sl.sb_idx = r.sb_cur;                  /* the walks this slot's anchors are in */
            }
            if (!rc && nb > 0) {                       /* the next batch's walks, on the GPU now */
                const int ask2 = next_ask(r, *cursor + nb);
                r.sb_cur ^= 1;
                if (ask2 > 0)
                    rc = spec_launch(r, r.sb[r.sb_cur], ask2);
            }
        } else if (ask > 0) {
            /* before the range only the carrier chain matters: no checkpoints recorded */
            rc = gss_scn_next(r.scn, ask, sl.blk, sl.nch,
                              (*cursor < r.first || lazy_ck(r)) ? nullptr : sl.ck, &nb, r.threads);
        }
        if (rc)
            return rc;
        if (nb == 0) {
            sl.nb = 0;
            sl.end = 1;
            return 0;
        }
        int64_t b0 = *cursor;
        *cursor += nb;
        if (b0 < r.first)
            continue;                                  /* before the range: planned, dropped */
        sl.first = b0;
        sl.nb = nb;
        sl.has_anch = sl.anch != nullptr && r.spec && !r.rec;
        int m = 1;
        for (int i = 0; i < nb; i++)
            m = sl.nch[i] > m ? sl.nch[i] : m;
        sl.nch_max = m;
        const uint32_t *rows = nullptr;
        int n_rows = 0;
        if (r.rows_ahead) {
            rows = r.nav_rows_h.data();
            n_rows = (int)(r.nav_rows_h.size() / GSS_NAV_WORDS);
        } else {
            gss_scn_nav_table(r.scn, &rows, &n_rows);
        }
        rc = take_nav_sources(r, sl, n_rows);          /* the GPU builds the new rows */
        if (rc)
            return rc;
        if (r.prover) {                                /* the proofs, on the prover thread */
            sl.lin_nav = rows;
            sl.lin_n_nav = n_rows;
            return 0;
        }
        sl.n_fb = 0;
        if (r.use_lin && !sl.gpu_proven) {             /* the proofs, on the planner thread */
            if (trace_on())
                fprintf(stderr, "trace scn_done %.6f\n", tnow());
            rc = gss_linearize_ex(sl.blk, sl.nch, nb, r.n_per_blk, r.ca, 32, rows, n_rows,
                                  sl.has_anch ? sl.anch : nullptr, sl.lin, sl.fast, r.threads);
            if (rc)
                return rc;
            int nf = 0;
            for (int i = 0; i < nb; i++)
                if (!sl.fast[i])
                    sl.fast[nb + nf++] = i;
            sl.n_fb = nf;
            fill_fb_ck(r, sl);
        }
        return 0;
    }
}

int proof_ahead(Run &r, Slot &sl);

void planner(Run *r)
{
    int64_t cursor = r->start;
    int up_rc = (r->opts && r->opts->carr_in) ? plan_range_upfront(*r) : 0;
    for (int i = 0;; i++) {
        Slot &sl = r->slot[i % NSLOT];
        {
            std::unique_lock<std::mutex> lk(r->mu);
            r->cv.wait(lk, [&] { return r->abort || sl.state == FREE; });
            if (r->abort)
                return;
        }
        const double t0 = trace_on() ? tnow() : 0.0;
        sl.gpu_proven = r->use_lin && (r->proof_mode == 1 || (r->proof_mode == 2 && (i & 1)));
        int rc = up_rc ? up_rc : plan_into(*r, sl, &cursor);
        if (!rc && !sl.end && r->gpu_proof)
            rc = proof_ahead(*r, sl);
        if (trace_on())
            fprintf(stderr, "trace plan slot %d nb %d %.6f %.6f\n", i % NSLOT, sl.nb, t0, tnow());
        {
            std::lock_guard<std::mutex> lk(r->mu);
            if (rc) {
                sl.err = rc;
                sl.end = 1;
            }
            sl.state = r->prover ? PROVING : PLANNED;
        }
        r->cv.notify_all();
        if (sl.end)
            return;
    }
}

/* The slots' proofs in slot order (r.prover): gss_linearize on this thread's own worker pool,
   the exact-path block list and its checkpoints, then the slot goes to the main thread. */
void prover(Run *r)
{
    gss_pool_select(2);
    for (int i = 0;; i++) {
        Slot &sl = r->slot[i % NSLOT];
        {
            std::unique_lock<std::mutex> lk(r->mu);
            r->cv.wait(lk, [&] { return r->abort || sl.state == PROVING; });
            if (r->abort)
                return;
        }
        const double t0 = trace_on() ? tnow() : 0.0;
        if (!sl.end && !sl.err && !sl.gpu_proven) {
            int rc = gss_linearize_ex(sl.blk, sl.nch, sl.nb, r->n_per_blk, r->ca, 32, sl.lin_nav,
                                      sl.lin_n_nav, sl.has_anch ? sl.anch : nullptr, sl.lin,
                                      sl.fast, r->threads);
            if (rc) {
                sl.err = rc;
                sl.end = 1;
            } else {
                int nf = 0;
                for (int b = 0; b < sl.nb; b++)
                    if (!sl.fast[b])
                        sl.fast[sl.nb + nf++] = b;
                sl.n_fb = nf;
                fill_fb_ck(*r, sl);
            }
        }
        if (trace_on())
            fprintf(stderr, "trace prove slot %d nb %d %.6f %.6f\n", i % NSLOT, sl.nb, t0, tnow());
        const int end = sl.end;
        {
            std::lock_guard<std::mutex> lk(r->mu);
            sl.state = PLANNED;
        }
        r->cv.notify_all();
        if (end)
            return;
    }
}

/* Nav-table rows a run can end with: the handle's rows so far (earlier runs, seeks, the
   allocation) plus, per 30 s update the run can cross, the re-generated frame of every active
   channel and a fresh one for every channel allocation, at most 2 GSS_MAXCH (scenario.c:
   update_30s, allocate_channels) -- the reservations of the tables that must not move during
   the run (the prover's host copy, the device table with GPU proofs) */
size_t nav_rows_bound(const gss_scn *s, const gss_scn_info_t &info)
{
    const uint32_t *rows = nullptr;
    int n = 0;
    if (gss_scn_nav_table(s, &rows, &n) != 0 || n < 0)
        n = 0;
    return (size_t)n + ((size_t)info.n_blocks / 300 + 2) * 2 * GSS_MAXCH;
}

/* the device nav table holds at least `rows` rows (grown on the compute stream's order) */
int nav_reserve(Run &r, size_t rows, hipStream_t st)
{
    if (rows <= r.d_nav_cap)
        return 0;
    size_t cap = r.d_nav_cap ? 2 * r.d_nav_cap : 4096;
    while (cap < rows)
        cap *= 2;
    uint32_t *p = nullptr;
    RUN_TRY(dev_alloc((void **)&p, sizeof(uint32_t) * GSS_NAV_WORDS * cap));
    if (r.d_nav) {
        RUN_TRY(hipStreamSynchronize(st));             /* earlier slots' kernels read it */
        RUN_TRY(hipMemcpy(p, r.d_nav, sizeof(uint32_t) * GSS_NAV_WORDS * r.d_nav_cap,
                          hipMemcpyDeviceToDevice));
        dev_free(r.d_nav);
    }
    r.d_nav = p;
    r.d_nav_cap = cap;
    return 0;
}

/* a slot's inputs on the device, one allocation (sl.d_in) */
struct SlotDev {
    gss_chan_blk_t *blk;
    int32_t *nch;
    double *ck;
    gss_nav_src_t *src;
    gss_lin_t *lin;
    int32_t *fast;                   /* fast[nb], then the exact-path block list */
    gss_carr_anchor_t *anch;         /* the chain's anchors (GPU proofs), or null */
    size_t need;
};

SlotDev slot_dev(const Slot &sl)
{
    const size_t s_blk = sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)sl.nb;
    const size_t s_nch = sizeof(int32_t) * (size_t)sl.nb;
    const size_t s_ck = sizeof(double) * GSS_MAXCH * GSS_NCK * (size_t)sl.nb;
    const size_t s_nav = sizeof(gss_nav_src_t) * (size_t)(sl.n_nav > 0 ? sl.n_nav : 1);
    const size_t s_lin = sl.lin ? sizeof(gss_lin_t) * GSS_MAXCH * (size_t)sl.nb : 0;
    const size_t s_fast = sl.lin ? sizeof(int32_t) * 2 * (size_t)sl.nb : 0;
    const int anch = sl.has_anch && sl.gpu_proven;
    const size_t s_anch = anch ? sizeof(gss_carr_anchor_t) * GSS_MAXCH * (size_t)sl.nb : 0;
    SlotDev v;
    v.need = al256(s_blk) + al256(s_nch) + al256(s_ck) + al256(s_nav) + al256(s_lin) +
             al256(s_fast) + al256(s_anch);
    uint8_t *p = sl.d_in;
    v.blk = (gss_chan_blk_t *)p;
    v.nch = (int32_t *)(p + al256(s_blk));
    v.ck = (double *)(p + al256(s_blk) + al256(s_nch));
    v.src = (gss_nav_src_t *)(p + al256(s_blk) + al256(s_nch) + al256(s_ck));
    v.lin = (gss_lin_t *)((uint8_t *)v.src + al256(s_nav));
    v.fast = (int32_t *)((uint8_t *)v.lin + al256(s_lin));
    v.anch = anch ? (gss_carr_anchor_t *)((uint8_t *)v.fast + al256(s_fast)) : nullptr;
    return v;
}

/* GPU proofs, run ahead (planner thread, right after the slot is planned): the slot's rows go
   to its device buffer on its own stream, its new nav rows are built on the planner's nav
   stream (in slot order: a row may continue the one before it), and the proof kernel runs as
   soon as both are there, so that several slots' proofs overlap the downloads of the slots
   before them instead of waiting on the render stream.  The device nav table was reserved for
   the whole run at set-up, so it never moves under the renders. */
int proof_ahead(Run &r, Slot &sl)
{
    /* the nav rows of every slot come from here when any slot is proven on the GPU (a row may
       continue one that an earlier slot brought); the proof only for the slots that take it */
    const size_t need = slot_dev(sl).need;
    if (need > sl.d_in_cap) {                          /* the slot is FREE: nothing reads it */
        dev_free(sl.d_in);
        sl.d_in = nullptr;
        sl.d_in_cap = 0;
        RUN_TRY(dev_alloc((void **)&sl.d_in, need));
        sl.d_in_cap = need;
    }
    const SlotDev v = slot_dev(sl);
    const int n_rows = sl.nav_first + sl.n_nav;
    if ((size_t)n_rows > r.d_nav_cap)
        return gss_fail(GSS_E_RANGE, "nav rows %d past the run's reservation %zu", n_rows,
                        r.d_nav_cap);
    if (sl.n_nav > 0) {
        RUN_H2D(v.src, sl.nav, sizeof(gss_nav_src_t) * (size_t)sl.n_nav, r.nav_st);
        int rc = gss_nav_rows_device(r.dev, v.src, sl.nav_first, sl.n_nav, r.d_nav, r.nav_st);
        if (rc)
            return rc;
    }
    RUN_TRY(hipEventRecord(sl.navd, r.nav_st));
    if (!sl.gpu_proven)
        return 0;
    RUN_H2D(v.blk, sl.blk, sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)sl.nb, sl.pst);
    RUN_H2D(v.nch, sl.nch, sizeof(int32_t) * (size_t)sl.nb, sl.pst);
    if (!lazy_ck(r))               /* (with lazy checkpoints only a rejected block needs them) */
        RUN_H2D(v.ck, sl.ck, sizeof(double) * GSS_MAXCH * GSS_NCK * (size_t)sl.nb, sl.pst);
    if (v.anch)
        RUN_H2D(v.anch, sl.anch, sizeof(gss_carr_anchor_t) * GSS_MAXCH * (size_t)sl.nb, sl.pst);
    RUN_TRY(hipStreamWaitEvent(sl.pst, sl.navd, 0));
    Run::SpecBatch *sb = r.rec && r.dev_anch && sl.sb_idx >= 0 && !v.anch ? &r.sb[sl.sb_idx]
                                                                          : nullptr;
    int rc = run_proof_launch(v.blk, v.nch, sl.nb, r.n_per_blk, r.d_ca, 32, r.d_nav,
                              n_rows > 0 ? n_rows : 1, v.anch, sb ? sb->d_in : nullptr,
                              sb ? sb->d_spec : nullptr, v.lin, v.fast, sl.first, r.force_exact,
                              sl.pst);
    if (rc)
        return rc;
    if (sb) {                                /* the batch's next walks wait for this proof */
        RUN_TRY(hipEventRecord(sb->consumed, sl.pst));
        sb->consumed_pending = 1;
    }
    /* the verdicts to the host at once: when the proof is done by the slot's submission, its
       rejected blocks take the exact path in the same render (submit_proven) */
    RUN_TRY(hipMemcpyAsync(sl.fast, v.fast, sizeof(int32_t) * (size_t)sl.nb,
                           hipMemcpyDeviceToHost, sl.pst));
    RUN_TRY(hipEventRecord(sl.proved, sl.pst));
    return 0;
}

/* submit for a slot proven by proof_ahead: render (every block as certified; the rejected ones
   are redone in drain), then the bytes, the status and the proofs' verdicts to the host */
int submit_proven(gss_dev *d, Run &r, Slot &sl, int n_per_blk, int fmt, size_t bb,
                  hipStream_t st, hipStream_t cp)
{
    const SlotDev v = slot_dev(sl);
    const int n_rows = sl.nav_first + sl.n_nav;
    RUN_TRY(hipStreamWaitEvent(st, sl.proved, 0));
    /* the proof done (it ran ahead): its verdicts are on the host, and the blocks it rejected
       (rare) render on the exact path beside the certified ones, as with host proofs; else the
       verdicts come back with the bytes and drain redoes the rejected blocks */
    int nf = 0;
    sl.verdicts = 0;
    const hipError_t q = r.late_verdicts ? hipErrorNotReady : hipEventQuery(sl.proved);
    if (q == hipSuccess) {
        for (int b = 0; b < sl.nb; b++)
            if (!sl.fast[b])
                sl.fast[sl.nb + nf++] = b;
        sl.n_fb = nf;
        if (nf > 0) {
            if (lazy_ck(r))
                for (int i = 0; i < nf; i++) {
                    const int b = sl.fast[sl.nb + i];
                    for (int k = 0; k < sl.nch[b]; k++) {
                        const size_t e = (size_t)b * GSS_MAXCH + k;
                        (void)gss_carr_advance_ck(sl.blk[e].carr0, sl.blk[e].carr_step,
                                                  r.n_per_blk, sl.ck + e * GSS_NCK);
                    }
                }
            RUN_H2D(v.ck, sl.ck, sizeof(double) * GSS_MAXCH * GSS_NCK * (size_t)sl.nb, st);
            RUN_H2D(v.fast + sl.nb, sl.fast + sl.nb, sizeof(int32_t) * (size_t)nf, st);
        }
        sl.verdicts = 1;
    } else if (q != hipErrorNotReady) {
        return gss_fail(GSS_E_HIP, "proof event query: %s", hipGetErrorString(q));
    }
    RUN_TRY(hipMemsetAsync(sl.d_status, 0, sizeof(int32_t), st));
    int rc = gss_synth_lin_device(d, v.blk, v.nch, sl.nch_max, v.lin, v.fast, v.fast + sl.nb, nf,
                                  v.ck, r.d_ca, 32, r.d_nav, n_rows > 0 ? n_rows : 1, sl.nb,
                                  n_per_blk, fmt, sl.d_out, sl.d_status, st);
    if (rc)
        return rc;
    RUN_TRY(hipEventRecord(sl.rendered, st));
    RUN_TRY(hipStreamWaitEvent(cp, sl.rendered, 0));
    if (sl.tc)
        RUN_TRY(hipEventRecord(sl.tc, cp));
    RUN_TRY(hipMemcpyAsync(sl.h_out, sl.d_out, bb * (size_t)sl.nb, hipMemcpyDeviceToHost, cp));
    RUN_TRY(hipMemcpyAsync(sl.h_status, sl.d_status, sizeof(int32_t), hipMemcpyDeviceToHost, cp));
    RUN_TRY(hipMemcpyAsync(sl.fast, v.fast, sizeof(int32_t) * (size_t)sl.nb,
                           hipMemcpyDeviceToHost, cp));
    RUN_TRY(hipEventRecord(sl.done, cp));
    return 0;
}

int submit(gss_dev *d, Run &r, Slot &sl, const uint32_t *d_ca, int n_per_blk, int fmt,
           size_t bb, hipStream_t st, hipStream_t cp)
{
    /* the slot's previous D2H must have read d_out before the kernels rewrite it */
    RUN_TRY(hipStreamWaitEvent(st, sl.done, 0));
    if (sl.tq)
        RUN_TRY(hipEventRecord(sl.tq, st));
    if (sl.lin && sl.gpu_proven)
        return submit_proven(d, r, sl, n_per_blk, fmt, bb, st, cp);
    const size_t need = slot_dev(sl).need;
    if (need > sl.d_in_cap) {
        RUN_TRY(hipStreamSynchronize(st));
        dev_free(sl.d_in);
        sl.d_in = nullptr;
        sl.d_in_cap = 0;
        RUN_TRY(dev_alloc((void **)&sl.d_in, need));
        sl.d_in_cap = need;
    }
    const double tq0 = trace_on() ? tnow() : 0.0;
    const SlotDev v = slot_dev(sl);
    gss_chan_blk_t *d_blk = v.blk;
    int32_t *d_nch = v.nch;
    double *d_ck = v.ck;
    gss_nav_src_t *d_src = v.src;
    gss_lin_t *d_lin = v.lin;
    int32_t *d_fast = v.fast;
    const size_t s_blk = sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)sl.nb;
    const size_t s_lin = sizeof(gss_lin_t) * GSS_MAXCH * (size_t)sl.nb;
    RUN_H2D(d_blk, sl.blk, s_blk, st);
    RUN_H2D(d_nch, sl.nch, sizeof(int32_t) * (size_t)sl.nb, st);
    RUN_H2D(d_ck, sl.ck, sizeof(double) * GSS_MAXCH * GSS_NCK * (size_t)sl.nb, st);
    /* the 30 s producer: this slot's new nav rows built on the device (gss_producers.hip); with
       GPU proofs in the run the planner has built them already (proof_ahead) */
    const int n_rows = sl.nav_first + sl.n_nav;
    int rc = r.gpu_proof ? 0 : nav_reserve(r, (size_t)(n_rows > 0 ? n_rows : 1), st);
    if (rc)
        return rc;
    if (r.gpu_proof) {
        RUN_TRY(hipStreamWaitEvent(st, sl.navd, 0));
    } else if (sl.n_nav > 0) {
        RUN_H2D(d_src, sl.nav, sizeof(gss_nav_src_t) * (size_t)sl.n_nav, st);
        rc = gss_nav_rows_device(d, d_src, sl.nav_first, sl.n_nav, r.d_nav, st);
        if (rc)
            return rc;
    }
    const uint32_t *d_nav = r.d_nav;
    const double tq1 = trace_on() ? tnow() : 0.0;
    RUN_TRY(hipMemsetAsync(sl.d_status, 0, sizeof(int32_t), st));
    if (sl.lin) {
        RUN_H2D(d_lin, sl.lin, s_lin, st);
        RUN_H2D(d_fast, sl.fast, sizeof(int32_t) * (size_t)(sl.nb + sl.n_fb), st);
        if (sl.tk)
            RUN_TRY(hipEventRecord(sl.tk, st));
        rc = gss_synth_lin_device(d, d_blk, d_nch, sl.nch_max, d_lin, d_fast, d_fast + sl.nb,
                                  sl.n_fb, d_ck, d_ca, 32, d_nav, n_rows, sl.nb, n_per_blk,
                                  fmt, sl.d_out, sl.d_status, st);
    } else {
        rc = gss_synth_device(d, d_blk, d_nch, sl.nch_max, d_ck, d_ca, 32, d_nav, n_rows,
                              sl.nb, n_per_blk, fmt, sl.d_out, nullptr, sl.d_status, st);
    }
    if (rc)
        return rc;
    const double tq2 = trace_on() ? tnow() : 0.0;
    RUN_TRY(hipEventRecord(sl.rendered, st));
    RUN_TRY(hipStreamWaitEvent(cp, sl.rendered, 0));
    if (sl.tc)
        RUN_TRY(hipEventRecord(sl.tc, cp));
    RUN_TRY(hipMemcpyAsync(sl.h_out, sl.d_out, bb * (size_t)sl.nb, hipMemcpyDeviceToHost, cp));
    RUN_TRY(hipMemcpyAsync(sl.h_status, sl.d_status, sizeof(int32_t), hipMemcpyDeviceToHost, cp));
    RUN_TRY(hipEventRecord(sl.done, cp));
    if (trace_on())
        fprintf(stderr, "trace submit_parts start %.6f h2d %.6f render %.6f out %.6f\n", tq0, tq1, tq2,
                tnow());
    return 0;
}

/* GPU proofs: the blocks they rejected (fast[b] == 0, rare: none in the bench runs) rendered
   again on the exact path alone (their checkpoints from the rows' exact carriers; the fast
   flags zeroed on the device, so that the fast kernel renders nothing), and only their bytes
   copied to the host again; synchronous */
int redo_rejected(gss_dev *d, Run &r, Slot &sl, const uint32_t *d_ca, int n_rows, int n_per_blk,
                  int fmt, size_t bb, hipStream_t st)
{
    int nf = 0;
    for (int b = 0; b < sl.nb; b++)
        if (!sl.fast[b])
            sl.fast[sl.nb + nf++] = b;
    if (nf == 0)
        return 0;
    sl.n_fb = nf;
    if (lazy_ck(r))
        for (int i = 0; i < nf; i++) {
            const int b = sl.fast[sl.nb + i];
            for (int k = 0; k < sl.nch[b]; k++) {
                const size_t e = (size_t)b * GSS_MAXCH + k;
                (void)gss_carr_advance_ck(sl.blk[e].carr0, sl.blk[e].carr_step, r.n_per_blk,
                                          sl.ck + e * GSS_NCK);
            }
        }
    const SlotDev v = slot_dev(sl);
    RUN_H2D(v.ck, sl.ck, sizeof(double) * GSS_MAXCH * GSS_NCK * (size_t)sl.nb, st);
    RUN_TRY(hipMemsetAsync(v.fast, 0, sizeof(int32_t) * (size_t)sl.nb, st));
    RUN_H2D(v.fast + sl.nb, sl.fast + sl.nb, sizeof(int32_t) * (size_t)nf, st);
    RUN_TRY(hipMemsetAsync(sl.d_status, 0, sizeof(int32_t), st));
    int rc = gss_synth_lin_device(d, v.blk, v.nch, sl.nch_max, v.lin, v.fast, v.fast + sl.nb, nf,
                                  v.ck, d_ca, 32, r.d_nav, n_rows, sl.nb, n_per_blk, fmt,
                                  sl.d_out, sl.d_status, st);
    if (rc)
        return rc;
    for (int i = 0; i < nf;) {                        /* runs of consecutive rejected blocks */
        const int b0 = sl.fast[sl.nb + i];
        int j = i + 1;
        while (j < nf && sl.fast[sl.nb + j] == b0 + (j - i))
            j++;
        RUN_TRY(hipMemcpyAsync(sl.h_out + bb * (size_t)b0, sl.d_out + bb * (size_t)b0,
                               bb * (size_t)(j - i), hipMemcpyDeviceToHost, st));
        i = j;
    }
    RUN_TRY(hipMemcpyAsync(sl.h_status, sl.d_status, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    RUN_TRY(hipStreamSynchronize(st));
    for (int i = 0; i < nf; i++)                      /* (the verdicts stay on the host copy) */
        sl.fast[sl.fast[sl.nb + i]] = 0;
    if (trace_on())
        fprintf(stderr, "trace redo first %lld blocks %d\n", (long long)sl.first, nf);
    return 0;
}

int drain(gss_dev *d, Run &r, Slot &sl, const uint32_t *d_ca, int n_per_blk, int fmt,
          size_t bb, hipStream_t st, gss_sink_fn sink, void *user)
{
    const double t0 = trace_on() ? tnow() : 0.0;
    RUN_TRY(hipEventSynchronize(sl.done));
    const double t1 = trace_on() ? tnow() : 0.0;
    if (sl.lin && sl.gpu_proven && !sl.verdicts && !*sl.h_status) {
        int rc = redo_rejected(d, r, sl, d_ca, sl.nav_first + sl.n_nav, n_per_blk, fmt, bb, st);
        if (rc)
            return rc;
    }
    if (*sl.h_status)
        return gss_fail(GSS_E_RANGE, "nav word index ran past dwrd[59]");
    if (sink(user, sl.h_out, bb * (size_t)sl.nb, sl.first, sl.nb))
        return gss_fail(GSS_E_IO, "sink failed at block %lld", (long long)sl.first);
    if (trace_on()) {
        fprintf(stderr, "trace drain first %lld wait %.6f %.6f sink_end %.6f\n",
                (long long)sl.first, t0, t1, tnow());
        float a = 0, k = 0, b = 0, c = 0, q = 0;       /* GPU clock: ms since the run's base */
        if (sl.tq && r.t_base && hipEventElapsedTime(&a, r.t_base, sl.tq) == hipSuccess &&
            hipEventElapsedTime(&b, r.t_base, sl.rendered) == hipSuccess &&
            hipEventElapsedTime(&c, r.t_base, sl.done) == hipSuccess) {
            if (!sl.lin || sl.gpu_proven || hipEventElapsedTime(&k, r.t_base, sl.tk) != hipSuccess)
                k = a;
            if (hipEventElapsedTime(&q, r.t_base, sl.tc) != hipSuccess)
                q = b;
            fprintf(stderr, "trace gpu first %lld start %.3f kernels %.3f rendered %.3f done %.3f "
                    "copy %.3f\n", (long long)sl.first, a, k, b, c, q);
        }
    }
    {
        std::lock_guard<std::mutex> lk(r.mu);
        sl.state = FREE;
    }
    r.cv.notify_all();
    return 0;
}

/* GSS_RUN_SPEC_CUS=N (measurement): the walks' stream on N of the device's CUs, spread over
   them (every (ncu / N)-th), and with GSS_RUN_RENDER_REST=1 the render stream on the others */
int spec_cus()
{
    const char *e = getenv("GSS_RUN_SPEC_CUS");
    return e && *e ? atoi(e) : 0;
}

hipError_t cu_mask_stream(hipStream_t *st, int n_sel, bool rest)
{
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0 || n_sel <= 0 || n_sel >= ncu)
        return hipErrorInvalidValue;
    const int every = ncu / n_sel;
    std::vector<uint32_t> m((size_t)(ncu + 31) / 32, 0u);
    for (int i = 0; i < ncu; i++)
        if ((i % every == 0) != rest)
            m[(size_t)i / 32] |= 1u << (i % 32);
    return hipExtStreamCreateWithCUMask(st, (uint32_t)m.size(), m.data());
}

bool make_streams(hipStream_t *cp)
{
    for (int k = 0; k < NCOPY; k++)
        if (stream_get(&cp[k], false) != hipSuccess)
            return false;
    return true;
}

int run_main(gss_dev *d, Run &r, int n_per_blk, int fmt, size_t bb, gss_sink_fn sink,
             void *user, hipStream_t st, hipStream_t *cp, const uint32_t *d_ca)
{
    int pending[DEPTH], np = 0, head = 0;              /* submitted, not yet drained (FIFO) */
    for (int i = 0;; i++) {
        Slot &sl = r.slot[i % NSLOT];
        {
            std::unique_lock<std::mutex> lk(r.mu);
            r.cv.wait(lk, [&] { return sl.state == PLANNED; });
        }
        if (sl.end) {
            int rc = 0;
            for (; np > 0 && rc == 0; np--, head = (head + 1) % DEPTH)
                rc = drain(d, r, r.slot[pending[head]], d_ca, n_per_blk, fmt, bb, st, sink, user);
            return sl.err ? sl.err : rc;
        }
        if (np == DEPTH) {                             /* oldest slot out to the sink */
            int rc = drain(d, r, r.slot[pending[head]], d_ca, n_per_blk, fmt, bb, st, sink, user);
            if (rc)
                return rc;
            head = (head + 1) % DEPTH;
            np--;
        }
        const double ts0 = trace_on() ? tnow() : 0.0;
        int rc = submit(d, r, sl, d_ca, n_per_blk, fmt, bb, st, cp[i % NCOPY]);
        if (trace_on())
            fprintf(stderr, "trace submit slot %d %.6f %.6f\n", i % NSLOT, ts0, tnow());
        if (rc)
            return rc;
        pending[(head + np) % DEPTH] = i % NSLOT;
        np++;
    }
}

}  // namespace

extern "C" int gss_run(gss_dev *d, gss_scn *s, int64_t first_block, int64_t n_blocks, int batch,
                       int threads, gss_sink_fn sink, void *user)
{
    return gss_run_ex(d, s, first_block, n_blocks, batch, threads, sink, user, nullptr);
}

extern "C" int gss_run_ex(gss_dev *d, gss_scn *s, int64_t first_block, int64_t n_blocks,
                          int batch, int threads, gss_sink_fn sink, void *user,
                          const gss_run_opts_t *opts)
{
    if (!d || !s || !sink || first_block < 0)
        return gss_fail(GSS_E_ARG, "invalid run arguments");
    const double t_enter = trace_on() ? tnow() : 0.0;
    gss_scn_info_t info;
    int rc = gss_scn_info(s, &info);
    if (rc) return rc;
    const size_t bb = gss_block_bytes(info.n_per_blk, info.data_format);
    if (bb == 0)
        return gss_fail(GSS_E_ARG, "invalid format %d for %d samples/block", info.data_format,
                        info.n_per_blk);
    Run r;
    r.scn = s;
    r.opts = opts;
    r.carrier_int = info.carrier_int;
    r.threads = threads > 0 ? threads : 1;
    r.n_per_blk = info.n_per_blk;
    {
        const char *path = getenv("GSS_PATH");        /* "walk": the exact path for every block */
        r.use_lin = !(path && strcmp(path, "walk") == 0);
        const char *fe = getenv("GSS_RUN_FORCE_EXACT");
        r.force_exact = fe && *fe ? atoi(fe) : 0;
        const char *lv = getenv("GSS_RUN_LATE_VERDICTS");
        r.late_verdicts = lv && *lv == '1';
        const char *up = getenv("GSS_RUN_UPLOAD");
        r.upload_dev = !(up && strcmp(up, "dma") == 0);
    }
    r.batch = batch > 0 ? batch : 100;
    if ((size_t)r.batch * bb > SLOT_OUT_MAX)
        r.batch = (int)(SLOT_OUT_MAX / bb) > 0 ? (int)(SLOT_OUT_MAX / bb) : 1;
    r.first = first_block;
    r.last = n_blocks < 0 ? INT64_MAX : first_block + n_blocks;
    /* the handle may have produced blocks already (an earlier run or seek): the run continues
       from there; blocks before first_block are planned (the carrier chain) and dropped */
    r.start = info.next_block;
    if (first_block < r.start)
        return gss_fail(GSS_E_STATE, "run from block %lld, but the scenario is at block %lld",
                        (long long)first_block, (long long)r.start);

    int ordinal = 0;
    RUN_TRY(hipGetDevice(&ordinal));
    hipStream_t st = nullptr, cp[NCOPY] = {};
    uint32_t *d_ca = nullptr;
    int err = 0;
    auto cleanup = [&]() {
        if (st) (void)hipStreamSynchronize(st);
        for (hipStream_t c : cp)
            if (c) (void)hipStreamSynchronize(c);
        if (r.nav_st) (void)hipStreamSynchronize(r.nav_st);
        for (Slot &sl : r.slot)                        /* proofs run ahead, not yet rendered */
            if (sl.pst) (void)hipStreamSynchronize(sl.pst);
        for (Slot &sl : r.slot) {
            pin_free(sl.blk); pin_free(sl.nch); pin_free(sl.ck);
            pin_free(sl.nav); pin_free(sl.h_status);
            pool_put(sl.h_out, sl.h_out_bytes, true, ordinal);
            pool_put(sl.d_out, sl.d_out_bytes, false, ordinal);
            pin_free(sl.lin); pin_free(sl.fast); pin_free(sl.anch);
            dev_free(sl.d_in); dev_free(sl.d_status);
            if (sl.done) (void)hipEventDestroy(sl.done);
            if (sl.rendered) (void)hipEventDestroy(sl.rendered);
            if (sl.tq) (void)hipEventDestroy(sl.tq);
            if (sl.tk) (void)hipEventDestroy(sl.tk);
            if (sl.tc) (void)hipEventDestroy(sl.tc);
        }
        for (Slot &sl : r.slot) {
            stream_put(sl.pst);
            if (sl.navd) (void)hipEventDestroy(sl.navd);
            if (sl.proved) (void)hipEventDestroy(sl.proved);
        }
        stream_put(r.nav_st);
        dev_free(d_ca);
        dev_free(r.d_nav);
        if (r.spec_st) (void)hipStreamSynchronize(r.spec_st);
        for (Run::SpecBatch &b : r.sb) {
            pin_free(b.h_in); pin_free(b.h_spec); pin_free(b.h_rec);
            dev_free(b.d_in); dev_free(b.d_spec);
            if (b.walked) (void)hipEventDestroy(b.walked);
            if (b.consumed) (void)hipEventDestroy(b.consumed);
        }
        dev_free(r.spec_warm);
        stream_put(r.spec_st);
        if (trace_on() && r.spec_rows)
            fprintf(stderr, "trace spec total rows %lld hits %lld\n", (long long)r.spec_rows,
                    (long long)r.spec_hits);
        stream_put(st);
        for (hipStream_t c : cp)
            stream_put(c);
        if (r.t_base) (void)hipEventDestroy(r.t_base);
        if (r.ca_ready) (void)hipEventDestroy(r.ca_ready);
    };
    /* buffers */
    {
        gss_ca_table(r.ca);                            /* the proofs' copy, on the host */
        if (dev_alloc((void **)&d_ca, sizeof r.ca) != hipSuccess ||
            (spec_cus() > 0 && getenv("GSS_RUN_RENDER_REST")
                 ? cu_mask_stream(&st, spec_cus(), true)
                 : stream_get(&st, false)) != hipSuccess ||
            !make_streams(cp) ||
            (trace_on() && (hipEventCreate(&r.t_base) != hipSuccess ||
                            hipEventRecord(r.t_base, st) != hipSuccess)))
            err = gss_fail(GSS_E_HIP, "run setup failed");
        /* the kernels' copy built on the device by the 30 s producer (gss_producers.hip) */
        if (!err)
            err = gss_ca_table_device(d, d_ca, st);
        const size_t nb = (size_t)r.batch;
        for (Slot &sl : r.slot) {
            if (err) break;
            if (pin_alloc((void **)&sl.blk, sizeof(gss_chan_blk_t) * GSS_MAXCH * nb) != hipSuccess ||
                pin_alloc((void **)&sl.nch, sizeof(int32_t) * nb) !=
                    hipSuccess ||
                pin_alloc((void **)&sl.ck, sizeof(double) * GSS_MAXCH * GSS_NCK * nb) != hipSuccess ||
                pool_get((void **)&sl.h_out, bb * nb, true, ordinal, &sl.h_out_bytes) !=
                    hipSuccess ||
                pin_alloc((void **)&sl.h_status, sizeof(int32_t)) !=
                    hipSuccess ||
                pool_get((void **)&sl.d_out, bb * nb, false, ordinal, &sl.d_out_bytes) !=
                    hipSuccess ||
                dev_alloc((void **)&sl.d_status, sizeof(int32_t)) != hipSuccess ||
                hipEventCreateWithFlags(&sl.done, trace_on() ? hipEventDefault
                                                             : hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&sl.rendered, trace_on() ? hipEventDefault
                                                                 : hipEventDisableTiming) !=
                    hipSuccess ||
                (trace_on() && (hipEventCreate(&sl.tq) != hipSuccess ||
                                hipEventCreate(&sl.tk) != hipSuccess ||
                                hipEventCreate(&sl.tc) != hipSuccess)))
                err = gss_fail(GSS_E_NOMEM, "run buffers (%zu B per slot)", bb * nb);
            if (!err && r.use_lin &&
                (pin_alloc((void **)&sl.lin, sizeof(gss_lin_t) * GSS_MAXCH * nb) != hipSuccess ||
                 pin_alloc((void **)&sl.fast, sizeof(int32_t) * 2 * nb) != hipSuccess))
                err = gss_fail(GSS_E_NOMEM, "run lines (%zu B per slot)",
                               sizeof(gss_lin_t) * GSS_MAXCH * nb);
        }
        const double t_slots = trace_on() ? tnow() : 0.0;
        /* the chain run ahead: fast path, float carrier (per batch, or over the up-front range
           of a hand-off) */
        {
            const char *e = getenv("GSS_RUN_SPEC");
            r.spec = lazy_ck(r) && !(e && e[0] == '0');
            const char *er = getenv("GSS_RUN_REC");
            r.rec = r.spec && !(opts && opts->carr_in && !opts->carr_predict) &&
                    !(er && er[0] == '0');
            const char *ed = getenv("GSS_RUN_DEV_ANCHORS");
            r.dev_anch = ed && ed[0] == '1';
        }
        if (!err && r.spec) {
            const size_t rows = nb * GSS_MAXCH;
            r.dev = d;
            /* high priority: the walks wait for free CUs behind the render kernels otherwise */
            if ((spec_cus() > 0
                     ? cu_mask_stream(&r.spec_st, spec_cus(), false)
                     : stream_get(&r.spec_st, true)) !=
                    hipSuccess ||
                dev_alloc((void **)&r.spec_warm, WARM_BYTES) != hipSuccess)
                err = gss_fail(GSS_E_HIP, "run carrier-chain stream");
            for (Run::SpecBatch &b : r.sb) {
                if (err) break;
                b.blk.resize(rows);
                b.nch.resize(nb);
                b.chain.resize(rows);
                if (hipEventCreateWithFlags(&b.walked, hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&b.consumed, hipEventDisableTiming) != hipSuccess ||
                    pin_alloc((void **)&b.h_in, sizeof(gss_spec_in_t) * rows) != hipSuccess ||
                    (r.rec ? dev_alloc((void **)&b.d_in, sizeof(gss_spec_in_t) * rows) !=
                                     hipSuccess ||
                                 dev_alloc((void **)&b.d_spec, sizeof(gss_spec_t) * rows) !=
                                     hipSuccess ||
                                 pin_alloc((void **)&b.h_rec, sizeof(gss_spec_rec_t) * rows) != hipSuccess
                           : pin_alloc((void **)&b.h_spec, sizeof(gss_spec_t) * rows) != hipSuccess))
                    err = gss_fail(GSS_E_NOMEM, "run carrier-chain buffers (%zu rows)", rows);
            }
            /* the chain's anchors for the proofs' carrier walks (GSS_RUN_ANCHORS=0: none) */
            const char *ea = getenv("GSS_RUN_ANCHORS");
            if (r.use_lin && !(opts && opts->carr_in) && !(ea && ea[0] == '0'))
                for (Slot &sl : r.slot) {
                    if (err) break;
                    if (pin_alloc((void **)&sl.anch, sizeof(gss_carr_anchor_t) * rows) != hipSuccess)
                        err = gss_fail(GSS_E_NOMEM, "run anchors (%zu rows)", rows);
                }
        }
        /* the rows and prover threads where the planner is the limit: slots of >= 1024 blocks
           (-b 1 at 2.6 MS/s: 2,048).  The D2H-bound formats gain nothing from them, and inside
           bench.py's process the extra threads cost the -b 16 leg a third of its download rate
           (profiles/round3/e2e_planner/bench_*_r3af.log); GSS_RUN_ROWS_AHEAD=1 / 0 forces */
        {
            const char *e = getenv("GSS_RUN_ROWS_AHEAD");
            const bool want = e && *e ? e[0] != '0' : r.batch >= 1024;
            r.rows_ahead = r.spec && !(opts && opts->carr_in) && want;
        }
        {
            /* GSS_RUN_PROOF=gpu: the proofs on the GPU, run ahead by the planner (proof_ahead);
               host: on the host threads; split: every other slot on the GPU.  The default (auto)
               proves on the GPU only the planner-bound runs (rows ahead: slots of >= 1024
               blocks, the -b 1 runs) with the walks' records (no walks on the host): there the
               host's CPUs are the limit and the proofs take them off it (configs[4] e2e 0.85-0.86
               against 0.80-0.82 of the D2H ceiling, profiles/round5/e2e/b_*_r5q).  Elsewhere the
               two are even since the proof kernel spreads a small slot's channels over waves
               (configs[3]: 0.695-0.702 s against 0.695-0.705, the headline and configs[2] within
               noise; profiles/round5/e2e/r6e, e2e_modes_r6i.log), and host proofs keep the
               GPU's queues to the render and the copies */
            const char *e = getenv("GSS_RUN_PROOF");
            const int gpu_auto = r.rows_ahead && r.rec ? 1 : 0;
            r.proof_mode = !r.use_lin ? 0 : !e || !*e || strcmp(e, "auto") == 0 ? gpu_auto :
                           strcmp(e, "gpu") == 0 ? 1 : strcmp(e, "split") == 0 ? 2 : 0;
            r.gpu_proof = r.proof_mode != 0;
        }
        r.prover = r.rows_ahead && r.use_lin && r.proof_mode != 1;
        {
            const char *e = getenv("GSS_RUN_PROVER");
            if (e && e[0] == '0')
                r.prover = 0;
        }
        if (!err && r.rows_ahead) {
            /* the nav table's host copy never moves while the prover reads it (take_rows
               still grows it safely if the bound were passed) */
            r.nav_rows_h.reserve(nav_rows_bound(s, info) * GSS_NAV_WORDS);
            for (Run::RowBatch &q : r.rb) {
                q.blk.resize(nb * GSS_MAXCH);
                q.nch.resize(nb);
                q.chain.resize(nb * GSS_MAXCH);
            }
            err = gss_scn_carrier(s, r.carr);
        }
        const double t_rows = trace_on() ? tnow() : 0.0;
        if (!err)
            err = gss_dev_reserve(d, r.batch, info.n_per_blk);
        const double t_reserve = trace_on() ? tnow() : 0.0;
        if (trace_on())
            fprintf(stderr, "trace setup_parts slots %.6f spec_rows %.6f reserve %.6f\n",
                    t_slots - t_enter, t_rows - t_slots, t_reserve - t_rows);
        if (!err && r.gpu_proof) {
            /* proofs run ahead on the slots' own streams (proof_ahead); the device nav table
               reserved for the whole run (nav_rows_bound) */
            r.dev = d;
            r.d_ca = d_ca;
            if (stream_get(&r.nav_st, false) != hipSuccess)
                err = gss_fail(GSS_E_HIP, "run nav stream");
            for (Slot &sl : r.slot) {
                if (err) break;
                if (stream_get(&sl.pst, true) != hipSuccess ||
                    hipEventCreateWithFlags(&sl.navd, hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&sl.proved, hipEventDisableTiming) != hipSuccess)
                    err = gss_fail(GSS_E_HIP, "run proof streams");
            }
            const double t_pst = trace_on() ? tnow() : 0.0;
            if (!err)
                err = nav_reserve(r, nav_rows_bound(s, info), st);
            /* the C/A table (built on st above) before any proof stream reads it: an event the
               proof streams wait for (a host wait here held the start-up for the table's first
               kernel, ~20 ms in a fresh process) */
            if (!err && (hipEventCreateWithFlags(&r.ca_ready, hipEventDisableTiming) != hipSuccess ||
                         hipEventRecord(r.ca_ready, st) != hipSuccess))
                err = gss_fail(GSS_E_HIP, "run set-up");
            for (Slot &sl : r.slot)
                if (!err && hipStreamWaitEvent(sl.pst, r.ca_ready, 0) != hipSuccess)
                    err = gss_fail(GSS_E_HIP, "run set-up");
            if (trace_on())
                fprintf(stderr, "trace setup_proofs streams %.6f nav_ca %.6f\n", t_pst - t_reserve,
                        tnow() - t_pst);
        }
    }
    if (err) {
        cleanup();
        return err;
    }
    if (trace_on())
        fprintf(stderr, "trace setup enter %.6f ready %.6f\n", t_enter, tnow());
    std::thread th([&r, ordinal] {
        (void)hipSetDevice(ordinal);                   /* pinned reallocations */
        planner(&r);
    });
    std::thread th_rows, th_prove;
    if (r.rows_ahead)
        th_rows = std::thread(rows_thread, &r);
    if (r.prover)
        th_prove = std::thread(prover, &r);
    if (r.spec) {
        /* the walks' first launch costs ~1 ms (the kernel's first use): here, on one zero row,
           while the planner produces its first rows, instead of inside its first batch */
        uint8_t *w = (uint8_t *)r.spec_warm;
        (void)hipMemsetAsync(r.spec_warm, 0, WARM_BYTES, r.spec_st);
        (void)gss_spec_device(d, (gss_spec_in_t *)w, 1, info.n_per_blk,
                              (gss_spec_t *)(w + 2 * WARM_IN), r.spec_st);
        if (r.rec) {
            (void)hipMemsetAsync(r.spec_warm, 0, WARM_BYTES, r.spec_st);
            (void)gss_spec_records_device(d, (gss_spec_in_t *)w, 1, info.n_per_blk,
                                          (gss_spec_in_t *)(w + WARM_IN),
                                          (gss_spec_t *)(w + 2 * WARM_IN),
                                          (gss_spec_rec_t *)(w + 2 * WARM_IN + WARM_SPEC),
                                          r.spec_st);
        }
    }
    err = run_main(d, r, info.n_per_blk, info.data_format, bb, sink, user, st, cp, d_ca);
    {
        std::lock_guard<std::mutex> lk(r.mu);
        r.abort = 1;
    }
    r.cv.notify_all();
    th.join();
    if (th_rows.joinable())
        th_rows.join();
    if (th_prove.joinable())
        th_prove.join();
    if (r.rows_ahead && !err)                          /* the scenario's carriers: run's end */
        err = gss_scn_set_carrier(s, r.carr);
    cleanup();
    return err;
}

/* Threads besides the planner and main ones (round 3):
 *   rows thread      (chain ahead, no hand-off, slots of >= 1024 blocks unless GSS_RUN_ROWS_AHEAD
 *                    says otherwise) owns the scenario during the run: next_ask's
 *                    batches (gss_scn_next_deferred) with the nav rows and sources new with each,
 *                    a batch ahead of the planner, on its own worker pool; the planner then keeps
 *                    the slot carriers and host copies of the nav table (GSS_RUN_ROWS_AHEAD=0:
 *                    rows on the planner thread; GSS_RUN_ROWS_POOL=0: the planner's pool)
 *   prover thread    (rows ahead, fast path) the slots' proofs in slot order on its own worker
 *                    pool: the planner hands a slot over PROVING, the prover marks it PLANNED
 *                    for the main thread (GSS_RUN_PROVER=0: proofs on the planner thread)
 */
