/*
 * gss_producers.hip — the 30 s producers on the GPU: the C/A chip table
 * (codegen, gpssim.c:132-171) and the LNAV frame rows with parity (generateNavMsg,
 * gpssim.c:1467-1547; computeChecksum 693-756) that the render kernels read, built on the device
 * from the host plane's compact sources (gss_nav_src_t).  The arithmetic is gss_nav.h, shared
 * with the host checker gss_nav_rows_host.  gss_run builds its device nav table with them.
 * Also the planner's carrier chain walked ahead: gss_spec_kernel runs each
 * block's walk from a guess of its start (gss_phase.h, speculative block walk), one lane per row,
 * so that the serial chain on the host (gss_carr_chain_spec) takes one partial cycle per block.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gpssim_amd.h"
#include "../common/gss_nav.h"
#include "../common/gss_phase.h"

extern "C" int gss_fail(int code, const char *fmt, ...);
extern "C" int gss_dev_ordinal(const gss_dev *d);

/* one workgroup of 64 lanes: lane 0 runs the two 10-stage registers (1023 steps), then the wave
   forms each PRN's chips 64 at a time and packs them with a ballot */
__global__ __launch_bounds__(64) void gss_ca_kernel(uint32_t *__restrict__ out)
{
    __shared__ uint32_t g1[GSS_CA_WORDS], g2[GSS_CA_WORDS];
    const int lane = threadIdx.x;
    if (lane == 0)
        gss_g1g2(g1, g2);
    __syncthreads();
    for (int prn = 1; prn <= 32; prn++)
        for (int c0 = 0; c0 < 32 * GSS_CA_WORDS; c0 += 64) {
            const int i = c0 + lane;
            const uint32_t bit = i < GSS_CA_LEN ? gss_ca_chip(g1, g2, prn, i) : 0u;
            const uint64_t m = __builtin_amdgcn_ballot_w64(bit != 0);
            if (lane < 2)
                out[(size_t)(prn - 1) * GSS_CA_WORDS + c0 / 32 + lane] =
                    (uint32_t)(m >> (32 * lane));
        }
}

/* rows [first, first + n): a lane per row whose predecessor is not among them (a chain head)
   builds its row and then the rows that continue it, in order */
__global__ void gss_nav_kernel(const gss_nav_src_t *__restrict__ src, int first, int n,
                               uint32_t *__restrict__ rows)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    if (src[i].prev >= first)
        return;                                   /* built by its chain's head */
    for (int r = first + i, guard = 0; r >= first && r < first + n && guard < n; guard++) {
        const gss_nav_src_t *q = &src[r - first];
        gss_nav_frame(q, gss_nav_head(q, rows), rows + (size_t)r * GSS_NAV_WORDS);
        r = q->next;
    }
}

extern "C" int gss_ca_table_device(gss_dev *d, uint32_t *out, void *stream)
{
    if (!d || !out)
        return gss_fail(GSS_E_ARG, "invalid C/A table arguments");
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_ca_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "C/A kernel: %s", hipGetErrorString(e));
}

extern "C" int gss_nav_rows_device(gss_dev *d, const gss_nav_src_t *src, int first, int n,
                                   uint32_t *rows, void *stream)
{
    if (!d || (n > 0 && (!src || !rows)) || first < 0 || n < 0)
        return gss_fail(GSS_E_ARG, "invalid nav-row arguments");
    if (n == 0)
        return 0;
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_nav_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                       (hipStream_t)stream, src, first, n, rows);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "nav kernel: %s", hipGetErrorString(e));
}

/* one lane per segment of a row (gss_spec_seg_walk).  Rows laid out [nblk][GSS_MAXCH] are taken
   channel-major, so that a wave's lanes walk the segments of consecutive blocks of one channel:
   close steps, nearly the same cycles and binades (uniform control flow) instead of 16 different
   Dopplers per wave.
   The rows and walks may live in pinned host memory (gss_spec_device from gss_run's host-walk
   modes), so the workgroup (64 / GSS_SPEC_K rows x GSS_SPEC_K segments: 2 x 32) stages them in
   LDS: each row read once across the link in 8-byte words instead of by each of its lanes, and
   the walks written back whole (16-byte stores) instead of field by field -- the walks' link
   traffic had slowed the slot downloads beside them by a tenth (tools/d2h_overlap.py).
   Segments past a row's k are written as zeros. */
constexpr int SPEC_ROWS = 64 / GSS_SPEC_K;               /* rows per workgroup */
static_assert(sizeof(gss_spec_in_t) % 8 == 0 && sizeof(gss_spec_t) % 16 == 0, "row sizes");

__device__ inline int spec_row_of(int u, int nrow)
{
    const int nb = nrow / GSS_MAXCH;
    return nrow % GSS_MAXCH ? u : (u % nb) * GSS_MAXCH + u / nb;
}

/* ---- the walks from a cycle cache shared by a row's lanes, misses walked in rounds ------------
 * A row's GSS_SPEC_K lanes walk the same carrier step s, so a cycle one lane walks (from post-wrap
 * w, with the interval [w + clo, w + chi] of starts it translates exactly: gss_walk_margins_cc's
 * argument) serves every lane of the row whose cycle starts inside it: end = w' + (v0 - w0), the
 * segment's interval narrowed to the entry's (conservative, so the chain's fix-up stays exact).
 * On SIMT lanes a miss must not stall the wave once per lane (the per-lane caches of round 6 ran
 * 12 % slower for that reason), so a lane whose cycle is not in the cache waits, the others go on
 * from the cache, and the waiting lanes walk their cycles together, one round for all of them,
 * once half the active lanes wait (or none can go on); their cycles then enter the cache.
 * Descending cycles are cached whole (head, the real steps below T and the wrap), not only their
 * heads: every step's rounding is a translation inside the intersection of the steps' margins.
 * The cache: SC_N entries per row in LDS (start interval [lo, hi], end offset dv = v0 - w0, steps
 * L) and SC_NB buckets over the row's post-wrap range (|s| wide) of the last two entries that
 * cover each; a lookup reads one bucket and tests at most two entries.  A stale bucket slot only
 * misses (an entry is used only when its own interval holds the start).  Host model of the
 * schedule (miss rounds 4-5 per wave against 11-12 cycle walks, headline rows): DESIGN.md §7.1.
 * The intervals differ from the host walk's (gss_spec_seg_walk) by the cache's `safe` shrink and
 * the entries' own margins: the tests compare ends, wraps and p1/w1 bit for bit and require the
 * device intervals inside the host's; GSS_SPEC_SHARED=0 builds the plain per-lane walk. */
#ifndef GSS_SPEC_SHARED
#define GSS_SPEC_SHARED 1
#endif
#ifndef SC_N
#define SC_N 64                                       /* cache entries per row */
#endif
#define SC_NB 64                                      /* buckets per row */
#ifndef SC_TH4
#define SC_TH4 2                                      /* a miss round once SC_TH4/4 wait */
#endif
#define SC_GUARD (1 << 20)                            /* rounds; never reached (then: no interval) */

/* one whole cycle from post-wrap value *x (at most left steps), its start margins in [*clo, *chi];
   *wr: it ended on a wrap (a whole cycle, cacheable) */
__device__ inline int64_t sc_cycle(double *x, double s, int64_t left, double *clo, double *chi,
                                   int *wr)
{
    if (s > 0.0)
        return gss_asc_to_wrap(x, s, 1.0, left, wr, clo, chi);
    const double T = gss_pow2(gss_exp2i(-s) + 2);
    const double dunit = gss_pow2(-53);
    int st = 0;
    double v = *x;
    int64_t t = gss_desc_head(&v, s, T, left, &st, clo, chi);
    *wr = 0;
    if (st) {
        while (t < left) {                            /* below T: real steps to the wrap */
            gss_margin_step(v, s, dunit, clo, chi);
            const double r = v + s;
            t++;
            if (r < 0.0) {
                const double lim = -r - 2.0 * dunit;
                if (lim < *chi) *chi = lim;
                gss_margin_step(r, 1.0, dunit, clo, chi);
                v = r + 1.0;
                *wr = 1;
                break;
            }
            if (-r > *clo) *clo = -r;
            v = r;
        }
    }
    *x = v;
    return t;
}

struct spec_cc {                                      /* one row's cache (LDS) */
    double lo[SC_N], hi[SC_N], dv[SC_N];
    int32_t L[SC_N];
    uint16_t bk[SC_NB];                               /* two entry indices + 1 (0: empty) */
    int32_t next;
};

__device__ inline int sc_bucket(double w, double base, double scale)
{
    const double f = (w - base) * scale;
    return f <= 0.0 ? 0 : f >= (double)(SC_NB - 1) ? SC_NB - 1 : (int)f;
}

/* a lane's results, written to the row's walk after the cache is done with (the two share LDS) */
struct sc_res {
    gss_spec_seg_t sg;
    int64_t p1;
    double w1;
};

/* the segment walk of gss_spec_seg_walk, its cycles through the row's cache; every lane of the
   wave calls it (walk: this lane has segment j to walk, from the row's start guess g (j = 0) or
   its guessed start Pj, Wj, to stop; its fields come back in *res) */
__device__ void sc_seg_walk(double g, double s, int64_t Pj, double Wj, int64_t stop, int j,
                            int64_t n, sc_res *res, bool walk, spec_cc *cc)
{
    gss_spec_seg_t *sg = &res->sg;
    bool act = false;
    double x = 0.0;
    int64_t left = 0;
    if (walk) {
        int64_t pos = 0;
        sg->dlo = 1.0;                                /* an empty interval until walked */
        sg->dhi = 0.0;
        sg->wrap_end = 0;
        if (j == 0) {
            x = g;
            int wr = 0;
            const int64_t t = s != 0.0 ? gss_carr_to_wrap(&x, s, stop, &wr) : stop;
            res->p1 = wr ? t : n;
            res->w1 = x;
            sg->end = x;
            act = wr && t < stop;
            pos = t;
        } else {
            x = Wj;
            pos = Pj;
            sg->end = x;
            act = s != 0.0 && pos < stop;
        }
        left = stop - pos;
#ifdef SC_SKIP
        act = false;                                  /* measurement: the kernel without walks */
#endif
    }
    const bool walked = act;                          /* the segment's interval is walked */
    const double as = s < 0.0 ? -s : s;
    const double base = s > 0.0 ? 0.0 : 1.0 - as;
    const double scale = as > 0.0 ? (double)SC_NB / as : 0.0;
    const double safe = 4.0 * gss_pow2(-52);
    double dlo = -GSS_BIG, dhi = GSS_BIG;
    int last = 0;
    bool blocked = false;
    for (int round = 0;; round++) {
        const uint64_t am = __builtin_amdgcn_ballot_w64(act);
        if (!am)
            break;
        if (round >= SC_GUARD) {                      /* (never) no interval: the host walks it */
            if (act) {
                dlo = 1.0;
                dhi = 0.0;
            }
            break;
        }
        bool hit = false;
        if (act && !blocked) {
            /* both slots' entries read at once (one LDS round trip after the bucket's) */
            const uint32_t wd = cc->bk[sc_bucket(x, base, scale)];
            const int i0 = (int)(wd & 0xFFu) - 1, i1 = (int)((wd >> 8) & 0xFFu) - 1;
            const int a0 = i0 < 0 ? 0 : i0, a1 = i1 < 0 ? 0 : i1;
            const double lo0 = cc->lo[a0], hi0 = cc->hi[a0], dv0 = cc->dv[a0];
            const double lo1 = cc->lo[a1], hi1 = cc->hi[a1], dv1 = cc->dv[a1];
            const int32_t L0 = cc->L[a0], L1 = cc->L[a1];
            const bool ok0 = i0 >= 0 && x >= lo0 && x <= hi0 && L0 <= left;
            const bool ok1 = i1 >= 0 && x >= lo1 && x <= hi1 && L1 <= left;
            if (ok0 || ok1) {
                const double lo = (ok0 ? lo0 : lo1) - x, hi = (ok0 ? hi0 : hi1) - x;
                if (lo > dlo) dlo = lo;
                if (hi < dhi) dhi = hi;
                x = x + (ok0 ? dv0 : dv1);
                left -= ok0 ? L0 : L1;
                last = 1;
                hit = true;
            }
            blocked = !hit;
            if (left <= 0)
                act = false;
        }
        const uint64_t bm = __builtin_amdgcn_ballot_w64(act && blocked);
        const uint64_t hm = __builtin_amdgcn_ballot_w64(hit);
        if (!bm || (hm && 4 * __builtin_popcountll(bm) < SC_TH4 * __builtin_popcountll(am)))
            continue;
        /* a miss round: every waiting lane walks its cycle and enters it */
        if (act && blocked) {
            const double w = x;
            double clo = -GSS_BIG, chi = GSS_BIG;
            int wr = 0;
            const int64_t t = sc_cycle(&x, s, left, &clo, &chi, &wr);
            left -= t;
            if (clo > dlo) dlo = clo;
            if (chi < dhi) dhi = chi;
            last = wr;
            blocked = false;
            if (left <= 0)
                act = false;
            if (wr && clo <= 0.0 && chi >= 0.0 && t <= INT32_MAX) {
                const int i = atomicAdd(&cc->next, 1) % SC_N;
                double lo = w + clo + safe, hi = w + chi - safe;
                if (lo > w) lo = w;                   /* the walked start itself is valid */
                if (hi < w) hi = w;
                cc->lo[i] = lo;
                cc->hi[i] = hi;
                cc->dv[i] = x - w;
                cc->L[i] = (int32_t)t;
                const int b1 = sc_bucket(lo, base, scale), b2 = sc_bucket(hi, base, scale);
                for (int b = b1; b <= b2; b++)        /* (racing lanes may drop a slot: a miss) */
                    cc->bk[b] = (uint16_t)((cc->bk[b] << 8) | (uint32_t)(i + 1));
            }
        }
        __syncthreads();                              /* one wave: the entries before the lookups */
    }
    if (walked) {
        sg->end = x;
        sg->dlo = dlo;
        sg->dhi = dhi;
        sg->wrap_end = last;
    }
}

/* in: the rows (read); back: where the rows go back with the walkers' guesses (in itself for
   gss_spec_device, only the rows guessed here; the device copy for gss_spec_records_device, every
   row).  heads: read only each row's start, step, k and pad (the walkers guess the rest) */
__global__ __launch_bounds__(64) void gss_spec_kernel(const gss_spec_in_t *in,
                                                      gss_spec_in_t *back, int nrow, int n,
                                                      gss_spec_t *__restrict__ spec, int heads)
{
    __shared__ gss_spec_in_t s_in[SPEC_ROWS];
#if GSS_SPEC_SHARED
    __shared__ union {                                  /* the caches, then the walks */
        spec_cc cc[SPEC_ROWS];
        gss_spec_t out[SPEC_ROWS];
    } s_u;
    gss_spec_t *s_out = s_u.out;
#else
    __shared__ gss_spec_t s_out[SPEC_ROWS];
#endif
    __shared__ int s_guessed[SPEC_ROWS];
    constexpr int WI = sizeof(gss_spec_in_t) / 8, WO = sizeof(gss_spec_t) / 16;
    const int lane = threadIdx.x, r = lane / GSS_SPEC_K, j = lane % GSS_SPEC_K;
    const int u0 = blockIdx.x * SPEC_ROWS;
    const int wr = heads ? 3 : WI;                       /* g, s, (k, pad): 3 words */
    for (int q = lane; q < SPEC_ROWS * WI; q += 64) {    /* the rows in, 8 bytes a lane */
        const int rr = q / WI, w = q % WI;
        if (u0 + rr < nrow)
            ((uint64_t *)&s_in[rr])[w] =
                w < wr ? ((const uint64_t *)&in[spec_row_of(u0 + rr, nrow)])[w] : 0;
    }
#if !GSS_SPEC_SHARED
    for (int q = lane; q < SPEC_ROWS * WO; q += 64)      /* the walks zeroed */
        ((uint4 *)s_out)[q] = make_uint4(0, 0, 0, 0);
#endif
    __syncthreads();
    const bool live = u0 + r < nrow;
#if GSS_SPEC_SHARED
    /* the row's guesses (gss_spec_guess_row) made in parallel, lane j the j-th, and its walk
       fields read from LDS: no lane holds a copy of the row (which went to scratch) */
    const double g = s_in[r].g, s = s_in[r].s;
    const bool guess = live && s_in[r].k == 0;
    __syncthreads();                                     /* every lane has read k */
    if (guess) {
        int64_t m = 0, p = 0;
        double w = 0.0;
        const int64_t kk = gss_spec_guess_kk(g, s, n, &m);
        int ok = 0;
        if (j >= 1 && j < kk)
            ok = gss_spec_guess_one(g, s, m, kk, j, &p, &w);
        const int64_t pp = __shfl_up(p, 1, GSS_SPEC_K);  /* guess j - 1's position */
        const int64_t prev = j == 1 ? 0 : pp;
        const bool bad = j >= 1 && (j >= kk || !ok || p <= prev || p >= n);
        const uint64_t rm = GSS_SPEC_K == 64 ? ~0ull : ((1ull << GSS_SPEC_K) - 1);
        const uint64_t rb = (__builtin_amdgcn_ballot_w64(bad) >> (r * GSS_SPEC_K)) & rm;
        const int k = rb ? __builtin_ctzll(rb) : GSS_SPEC_K;    /* the first guess that fails */
        if (j >= 1 && j < k) {
            s_in[r].P[j] = p;
            s_in[r].W[j] = w;
        }
        if (j == 0)
            s_in[r].k = k;
    }
    if (j == 0)
        s_guessed[r] = guess;
    for (int q = lane; q < SPEC_ROWS * SC_NB; q += 64)
        s_u.cc[q / SC_NB].bk[q % SC_NB] = 0;
    if (lane < SPEC_ROWS)
        s_u.cc[lane].next = 0;
    __syncthreads();
    const int kr = s_in[r].k, k = kr < 1 ? 1 : (kr > GSS_SPEC_K ? GSS_SPEC_K : kr);
    const bool walk = live && j < kr;
    sc_res res;
    sc_seg_walk(g, s, s_in[r].P[j], s_in[r].W[j], j + 1 < k ? s_in[r].P[j + 1] : (int64_t)n, j,
                n, &res, walk, &s_u.cc[r]);
    __syncthreads();                                     /* the caches are done with */
    for (int q = lane; q < SPEC_ROWS * WO; q += 64)      /* the walks zeroed */
        ((uint4 *)s_out)[q] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (walk) {
        s_out[r].seg[j] = res.sg;
        if (j == 0) {
            s_out[r].p1 = res.p1;
            s_out[r].w1 = res.w1;
        }
    }
#else
    gss_spec_in_t row = s_in[r];
    const bool guess = live && row.k == 0;
    if (guess) {
        /* segment starts not guessed yet (gss_carr_chain_starts): every lane of the row makes
           the same guesses; its first lane writes them back for the host's chain */
        gss_spec_guess_row(row.g, row.s, n, &row);
    }
    __syncthreads();                                     /* every lane has read s_in[r] */
    if (j == 0) {
        s_guessed[r] = guess;
        if (guess)
            s_in[r] = row;
    }
    if (live && j < row.k)
        gss_spec_seg_walk(&row, j, n, &s_out[r]);
#endif
    __syncthreads();
    for (int q = lane; q < SPEC_ROWS * WO; q += 64) {    /* the walks out, 16 bytes a lane */
        const int rr = q / WO, w = q % WO;
        if (u0 + rr < nrow)
            ((uint4 *)&spec[spec_row_of(u0 + rr, nrow)])[w] = ((const uint4 *)&s_out[rr])[w];
    }
    for (int q = lane; q < SPEC_ROWS * WI; q += 64) {    /* the walkers' guesses back */
        const int rr = q / WI, w = q % WI;
        if (u0 + rr < nrow && (s_guessed[rr] || back != in))
            ((uint64_t *)&back[spec_row_of(u0 + rr, nrow)])[w] = ((const uint64_t *)&s_in[rr])[w];
    }
}

/* Each row's record (gss_phase.h gss_spec_record) from the walks in device memory: one lane per
   row, the link from the previous row of its slot (in[].pad); the records staged in LDS and
   written to host-visible memory in 16-byte stores (72 B per row instead of the walk's 272 and
   the guesses' 152) */
constexpr int REC_ROWS = 64;
static_assert(sizeof(gss_spec_rec_t) == 72, "record size");

__global__ __launch_bounds__(REC_ROWS) void gss_spec_rec_kernel(
    const gss_spec_in_t *__restrict__ in, const gss_spec_t *__restrict__ spec, int nrow, int n,
    gss_spec_rec_t *__restrict__ rec)
{
    __shared__ gss_spec_rec_t s_rec[REC_ROWS];
    const int lane = threadIdx.x;
    const int u0 = blockIdx.x * REC_ROWS, i = u0 + lane;
    if (i < nrow) {
        const int p = in[i].pad;
        const bool ok = p >= 0 && p < i;
        gss_spec_record(&in[i], &spec[i], ok ? &in[p] : nullptr, ok ? &spec[p] : nullptr, n,
                        &s_rec[lane]);
        if (s_rec[lane].ok & 2)
            s_rec[lane].ok |= (i - p) << 2;         /* the row the link was built against */
    }
    __syncthreads();
    constexpr int W = sizeof(gss_spec_rec_t) * REC_ROWS / 16;
    const int rows = nrow - u0 < REC_ROWS ? nrow - u0 : REC_ROWS;
    const int words = rows * (int)sizeof(gss_spec_rec_t) / 8;   /* 9 words a row */
    if (rows == REC_ROWS) {
        for (int q = lane; q < W; q += REC_ROWS)
            ((uint4 *)&rec[u0])[q] = ((const uint4 *)s_rec)[q];
    } else {
        for (int q = lane; q < words; q += REC_ROWS)
            ((uint64_t *)&rec[u0])[q] = ((const uint64_t *)s_rec)[q];
    }
}

extern "C" int gss_spec_records_device(gss_dev *d, const gss_spec_in_t *in, int nrow,
                                       int n_per_blk, gss_spec_in_t *d_in, gss_spec_t *d_spec,
                                       gss_spec_rec_t *rec, void *stream)
{
    if (!d || nrow < 0 || n_per_blk <= 0 ||
        (nrow > 0 && (!in || !d_in || !d_spec || !rec)) || ((uintptr_t)in & 7) ||
        ((uintptr_t)d_in & 7) || ((uintptr_t)d_spec & 15) || ((uintptr_t)rec & 15) ||
        (const void *)in == (const void *)d_in)
        return gss_fail(GSS_E_ARG, "invalid speculative-record arguments (rows 8-byte, walks "
                        "and records 16-byte aligned, in and d_in apart)");
    if (nrow == 0)
        return 0;
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_spec_kernel, dim3((unsigned)((nrow + SPEC_ROWS - 1) / SPEC_ROWS)),
                       dim3(64), 0, (hipStream_t)stream, in, d_in, nrow, n_per_blk, d_spec, 1);
    hipLaunchKernelGGL(gss_spec_rec_kernel, dim3((unsigned)((nrow + REC_ROWS - 1) / REC_ROWS)),
                       dim3(REC_ROWS), 0, (hipStream_t)stream, d_in, d_spec, nrow, n_per_blk,
                       rec);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "record kernels: %s", hipGetErrorString(e));
}

extern "C" int gss_spec_device(gss_dev *d, gss_spec_in_t *in, int nrow, int n_per_blk,
                               gss_spec_t *spec, void *stream)
{
    if (!d || nrow < 0 || n_per_blk <= 0 || (nrow > 0 && (!in || !spec)) ||
        ((uintptr_t)in & 7) || ((uintptr_t)spec & 15))
        return gss_fail(GSS_E_ARG, "invalid speculative-walk arguments (rows 8-byte, walks "
                        "16-byte aligned)");
    if (nrow == 0)
        return 0;
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_spec_kernel, dim3((unsigned)((nrow + SPEC_ROWS - 1) / SPEC_ROWS)),
                       dim3(64), 0,
                       (hipStream_t)stream, in, in, nrow, n_per_blk, spec, 0);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "spec kernel: %s", hipGetErrorString(e));
}

/* gss_run's uploads of its slots' inputs (gss_run.hip, dev_copy): 16-byte vector loads, four in
   flight per lane; the tail bytes (and unaligned buffers) byte by byte */
__global__ __launch_bounds__(256) void upload_kernel(const uint4 *__restrict__ src,
                                                     uint4 *__restrict__ dst, size_t n16,
                                                     int tail)
{
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride],
                    d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride)
        dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < tail)
        ((uint8_t *)(dst + n16))[threadIdx.x] = ((const uint8_t *)(src + n16))[threadIdx.x];
}

__global__ __launch_bounds__(256) void upload_bytes_kernel(const uint8_t *__restrict__ src,
                                                           uint8_t *__restrict__ dst, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        dst[i] = src[i];
}

/* n bytes from src to dst by a kernel on st: pinned host (hipHostMalloc) or device memory on
   either side (gss_run's uploads; not exported) */
int run_copy_launch(void *dst, const void *src, size_t n, hipStream_t st)
{
    if (n == 0)
        return 0;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
        const size_t n16 = n >> 4;
        const size_t g = (n16 + 1023) / 1024;
        hipLaunchKernelGGL(upload_kernel, dim3((unsigned)(g < 1 ? 1 : g > 2048 ? 2048 : g)),
                           dim3(256), 0, st, (const uint4 *)src, (uint4 *)dst, n16,
                           (int)(n & 15));
    } else {
        const size_t g = (n + 255) / 256;
        hipLaunchKernelGGL(upload_bytes_kernel, dim3((unsigned)(g > 2048 ? 2048 : g)), dim3(256),
                           0, st, (const uint8_t *)src, (uint8_t *)dst, n);
    }
    return hipGetLastError() == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "copy kernel launch");
}
