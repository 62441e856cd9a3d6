/*
 * linearize.c — certified integer lines for the sample loop's two double recurrences: the host
 * side of the GPU fast path (gss_lin_kernel).
 *
 * The reference steps, per sample and channel (gpssim.c:2212-2250),
 *     code += f_code*delt  (wrap at 1023, counters icode/ibit/iword, new data bit every 20 wraps)
 *     carr += f_carr*delt  (wrap into [0,1))
 * and reads LUT[floor(512 carr)] and ca[floor(code)].  For one block this file takes the
 * fixed-point lines of the block's own start values and steps,
 *     carrier  X(p) = rnd(carr0 2^64) + p rnd(carr_step 2^64)  mod 2^64,  LUT cell X >> 55
 *     code     Z(p) = rnd(code0 2^50) + p rnd(code_step 2^50),            chip (Z >> 50) mod 1023
 * The kernel renders from chunk anchors of these lines plus 32-bit steps (gss_lin.h: the
 * kernel's cell and chip at sample p are gss_lin_kernel_at, within
 * GSS_LIN_KDEV_* of the lines).  This file proves, with exact integer arithmetic, at which samples
 * the kernel could read another LUT cell or chip sign than the reference's doubles, decides those
 * samples exactly and, where the kernel's term differs, stores the difference as a patch
 * (gss_lin_t ppos/pdelta) that the kernel adds to that sample's accumulator.
 *
 * Proof, per chain and block of n samples:
 *   1. Each reference step is one IEEE addition (error <= 2^-53 cycle for sums below 2, <= 2^-44
 *      chip below 1024) plus a wrap that is exact (carr -= 1 and code -= 1023, Sterbenz) or
 *      rounded once (carr += 1, <= 2^-54).  So the unwrapped exact value moves by the step plus
 *      less than 2^12 units of 2^-64 cycle (2^7 units of 2^-50 chip) per sample, and the line by
 *      the step plus at most half a unit: |line - exact| <= D1 = 2 + n (err + 1) over the block,
 *      about 2^-34 cycle and 2^-25 chip for a 0.1 s block at 2.6 MS/s.  |kernel - line| <= D2
 *      (GSS_LIN_KDEV_*: about 2^-30 cycle and 2^-21 chip).
 *   2. The exact value, the line and the kernel can fall into different cells only where the line
 *      lies within D = D1 + D2 of a cell boundary (a multiple of B = 2^55, resp. 2^50):
 *      (line(p) + D) mod B < 2 D.  These samples are enumerated exactly, each as the first p after
 *      the previous one whose residue falls below 2 D: first_below, a Euclid-like descent in
 *      O(log B) steps.  At 2.6 MS/s about one carrier chain in two has one.
 *   3. The exact value at each of them comes from the cycle-cached walks of gss_phase.h, the
 *      kernel's from gss_lin.h; where the signed LUT term differs it becomes a patch.
 *   4. Code wraps are chip boundaries too: the k-th wrap falls where the line crosses
 *      1023 k 2^50, one sample earlier or later only where step 3 found the exact value on the
 *      other side.  The counters and the signed gain (gpssim.c:2186, 2219-2237) follow; the
 *      kernel applies the gain by sample position, so a patch only ever corrects cell and chip.
 * A channel with more than LIN_MAXHIT ambiguous samples or GSS_NPATCH patches, or failing a
 * precondition of the kernel (below), sends its block to the exact walking path (Stage A +
 * Stage B); gss_linearize reports that per block.  Cost: O(log B) per chain plus the rare walks.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "gss_host.h"
#include "../common/gss_proof.h"        /* the per-channel proof (shared with the GPU) */

/* ---- exact modular minimum --------------------------------------------------------------- */
/* min over 0 <= p < n of (a + p*s) mod m, for 0 <= a, s < m, n >= 1.  Each round replaces the
 * modulus by s <= m/2 (increasing sawtooth: its minima are the values just after each wrap) or by
 * m - s < m/2 (decreasing sawtooth: the values just before each wrap, plus the last one). */
u128 gss_minmod(u128 n, u128 m, u128 a, u128 s)
{
    u128 best = a;
    for (;;) {
        if (a < best) best = a;
        if (s == 0 || n <= 1)
            return best;
        if (2 * s <= m) {
            u128 k = (a + (n - 1) * s) / m;          /* wraps within [0, n) */
            if (k == 0)
                return best;
            u128 ms = m % s;
            u128 na = (a % s + s - ms) % s;          /* (a - m) mod s: value after wrap 1 */
            u128 ns = (s - ms) % s;                  /* (-m) mod s: step between wraps */
            n = k; m = s; a = na; s = ns;
        } else {
            u128 d = m - s;
            u128 last = (a + (n - 1) * s) % m;       /* end of the final (partial) run */
            if (last < best) best = last;
            u128 nd = n * d;
            if (nd <= a)
                return best;
            u128 k = (nd - a + m - 1) / m;           /* complete descending runs */
            u128 na = a % d, ns = m % d;             /* run j ends at (a + j m) mod d */
            n = k; m = d; a = na; s = ns;
        }
    }
}

u128 gss_maxmod(u128 n, u128 m, u128 a, u128 s)
{
    return m - 1 - gss_minmod(n, m, m - 1 - a, (m - s) % m);
}

#ifdef GSS_PF_STATS
/* measurement builds: how deep the proofs' descents go (gss_pf_stats reads and clears) */
static long pf_depth_hist[GSS_PF_EUCLID_MAX + 2];
void gss_pf_depth_note(int d) { __atomic_add_fetch(&pf_depth_hist[d], 1, __ATOMIC_RELAXED); }
void gss_pf_stats(long *out)
{
    for (int i = 0; i < GSS_PF_EUCLID_MAX + 2; i++)
        out[i] = __atomic_exchange_n(&pf_depth_hist[i], 0, __ATOMIC_RELAXED);
}
#endif

/* exported for tests: first_below, and min and max of (a + p s) mod m over [0, n) */
uint64_t gss_first_below(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t w)
{
    if (m == 0 || m >= ((uint64_t)1 << 62) || w == 0 || w > m)
        return UINT64_MAX;
    return first_below(n, m, a % m, s % m, w);
}

/* exported for tests: the proof's hit enumeration (hits_mod), by the three gaps or (scan) one
   descent per hit */
int gss_hits_mod(uint64_t n, uint64_t lgB, uint64_t a0, uint64_t st, uint64_t w, int64_t *hit,
                 int cap, int scan)
{
    if (lgB < 1 || lgB > 55 || n == 0 || w == 0 || w >= ((uint64_t)1 << lgB) / 2 || !hit ||
        cap < 0)
        return -2;
    const uint64_t B = (uint64_t)1 << lgB;
    if (n > INT32_MAX)
        return -2;
    int32_t *h32 = malloc(sizeof(int32_t) * (size_t)(cap > 0 ? cap : 1));
    if (!h32)
        return -2;
    const int nh = hits_mod(n, B, a0 & (B - 1), st & (B - 1), w, h32, cap, scan);
    for (int i = 0; i < nh; i++)
        hit[i] = h32[i];
    free(h32);
    return nh;
}

/* (64-bit operands) */
void gss_minmax_mod(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t *mn, uint64_t *mx)
{
    *mn = (uint64_t)gss_minmod(n, m, a % m, s % m);
    *mx = (uint64_t)gss_maxmod(n, m, a % m, s % m);
}

/* the LUT the proof compares terms with (gss_lut), filled once by pthread_once before any worker
   reads it */
static int32_t lut_sinT[512], lut_cosT[512];
static pthread_once_t lut_once = PTHREAD_ONCE_INIT;

static void lut_fill(void) { gss_lut(lut_sinT, lut_cosT); }

typedef struct {
    const gss_chan_blk_t *blk;
    const int32_t *nch;
    const uint32_t *nav, *ca;
    int n_nav, n_ca, n_per_blk, b_lo, b_hi;
    gss_lin_t *lin;
    int32_t *fast;
    const gss_carr_anchor_t *anch;
} lin_job;

static void *lin_run(void *arg)
{
    lin_job *j = arg;
    for (int b = j->b_lo; b < j->b_hi; b++) {
        int ok = 1, gsum = 0;
        const int nc = j->nch[b];
        for (int k = 0; k < GSS_MAXCH; k++) {
            gss_lin_t *l = &j->lin[(size_t)b * GSS_MAXCH + k];
            memset(l, 0, sizeof *l);
            for (int i = 0; i < GSS_NGC; i++)
                l->gpos[i] = INT32_MAX;
            for (int i = 0; i < GSS_NPATCH; i++)
                l->ppos[i] = INT32_MAX;
        }
        if (nc < 0 || nc > GSS_MAXCH)
            ok = 0;
        for (int k = 0; ok && k < nc; k++) {
            const gss_chan_blk_t *p = &j->blk[(size_t)b * GSS_MAXCH + k];
            gsum += p->gain < 0 ? -p->gain : p->gain;
            if (p->nav_tbl < 0 || p->nav_tbl >= j->n_nav || p->ca_tbl < 0 ||
                p->ca_tbl >= j->n_ca) {
                ok = 0;
                break;
            }
            ok = lin_channel(p, j->n_per_blk, j->nav + (size_t)p->nav_tbl * GSS_NAV_WORDS,
                             j->ca + (size_t)p->ca_tbl * GSS_CA_WORDS, lut_cosT, lut_sinT,
                             j->anch ? &j->anch[(size_t)b * GSS_MAXCH + k] : NULL, NULL, NULL,
                             &j->lin[(size_t)b * GSS_MAXCH + k]);
            if (p->gain > 1024 || p->gain < -1024)    /* an exact f16 MFMA operand, and so is
                                                         its doubled data-bit difference */
                ok = 0;
        }
        /* the kernel's sums: the packed int64 I/Q accumulator (LIN_MFMA=0) needs
           250*sum|gain| + 64 < 2^21; the MFMA build's f32 sums from 1.5 2^23 need < 2^22 */
        if (gsum > 8000)
            ok = 0;
        j->fast[b] = ok;
    }
    return NULL;
}

static void lin_part(void *arg, int b)
{
    lin_job j = *(const lin_job *)arg;
    j.b_lo = b;
    j.b_hi = b + 1;
    (void)lin_run(&j);
}

int gss_linearize(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                  const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                  gss_lin_t *lin, int32_t *fast, int threads)
{
    return gss_linearize_ex(blk, nch, nblk, n_per_blk, ca_bits, n_ca, nav, n_nav, NULL, lin, fast,
                            threads);
}

int gss_linearize_ex(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                     const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                     const gss_carr_anchor_t *anch, gss_lin_t *lin, int32_t *fast, int threads)
{
    if (!blk || !nch || !lin || !fast || nblk < 0 || n_per_blk <= 0 || (n_nav > 0 && !nav) ||
        (n_ca > 0 && !ca_bits) || n_ca < 0)
        return gss_fail(GSS_E_ARG, "invalid linearize arguments");
    if (nblk == 0)
        return 0;
    pthread_once(&lut_once, lut_fill);                /* before any worker thread starts */
    const lin_job all = {blk, nch, nav, ca_bits, n_nav, n_ca, n_per_blk, 0, nblk, lin, fast, anch};
    /* one part per block on the pooled workers (blocks differ in their ambiguous samples) */
    gss_pool_run(threads, nblk, lin_part, (void *)&all);
    return 0;
}
