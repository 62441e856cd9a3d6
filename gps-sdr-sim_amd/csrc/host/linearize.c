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
#include "../common/gss_phase.h"
#include "../common/gss_lin.h"

typedef unsigned __int128 u128;
typedef __int128 i128;

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

/* ---- exact first hit ------------------------------------------------------------------------- */
/* Smallest x in [0, lim] with lo <= (s x) mod m <= hi, for 1 <= lo <= hi < m < 2^62 and s < m;
 * UINT64_MAX if there is none.  Every candidate is >= ceil(lo/s); if s x reaches [lo, hi] before
 * its first wrap, that is x.  Otherwise [lo, hi] holds no multiple of s (so hi - lo < s), and x
 * exists for wrap count y iff some multiple of s lies in [lo + m y, hi + m y], i.e. (m y) mod s
 * lies in [s - hi mod s, s - lo mod s]: the same question for (m mod s, s), Euclid's descent, with
 * x = ceil((lo + m y) / s) of the least y.  x <= lim needs y <= lim s / m: the descent stops as
 * soon as that bound (an overestimate in double, so nothing is cut wrongly) is out of reach. */
static uint64_t first_in(uint64_t s, uint64_t m, uint64_t lo, uint64_t hi, uint64_t lim)
{
    if (s == 0)
        return UINT64_MAX;
    const uint64_t x = (lo + s - 1) / s;
    if (x > lim)
        return UINT64_MAX;
    if (s * x <= hi)                                 /* s x <= lo + s - 1 < 2^63 */
        return x;
    const uint64_t lr = lo % s, hr = hi % s;         /* 1 <= lr <= hr < s (no multiple inside) */
    const double yd = (double)lim * (double)s / (double)m + 2.0;
    const uint64_t ylim = yd < 0x1p52 ? (uint64_t)yd : UINT64_MAX;
    const uint64_t y = first_in(m % s, s, s - hr, s - lr, ylim);
    if (y == UINT64_MAX)
        return UINT64_MAX;
    const u128 v = ((u128)lo + (u128)m * y + s - 1) / s;
    return v <= lim ? (uint64_t)v : UINT64_MAX;
}

/* Smallest p in [0, n) with (a + p s) mod m < w (0 <= a, s < m < 2^62, 0 < w <= m), or n. */
static uint64_t first_below(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t w)
{
    if (n == 0)
        return 0;
    if (a < w)
        return 0;
    /* (a + p s) mod m < w  <=>  (s p) mod m in [m - a, m - a + w - 1], a range below m as a >= w */
    const uint64_t p = first_in(s, m, m - a, m - a + w - 1, n - 1);
    return p < n ? p : n;
}

/* exported for tests: first_below, and min and max of (a + p s) mod m over [0, n) */
uint64_t gss_first_below(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t w)
{
    if (m == 0 || m >= ((uint64_t)1 << 62) || w == 0 || w > m)
        return UINT64_MAX;
    return first_below(n, m, a % m, s % m, w);
}

/* (64-bit operands) */
void gss_minmax_mod(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t *mn, uint64_t *mx)
{
    *mn = (uint64_t)gss_minmod(n, m, a % m, s % m);
    *mx = (uint64_t)gss_maxmod(n, m, a % m, s % m);
}

/* ---- fixed point ----------------------------------------------------------------------------- */
/* x * 2^k rounded to nearest (ties away); *inexact set if rounding happened.  |x| < 2^60. */
static i128 to_fix(double x, int k, int *inexact)
{
    int e;
    double fr = frexp(x, &e);                        /* x = fr * 2^e, 0.5 <= |fr| < 1 */
    int64_t m = (int64_t)ldexp(fr, 53);              /* exact: x = m * 2^(e-53) */
    int sh = e - 53 + k;
    if (x == 0.0)
        return 0;
    if (sh >= 0)
        return (i128)m * ((i128)1 << sh);            /* no left shift of a negative value */
    if (sh < -62) {
        *inexact = 1;
        return 0;
    }
    int64_t am = m < 0 ? -m : m;
    int64_t q = am >> -sh, r = am - (q << -sh);
    if (r != 0) {
        *inexact = 1;
        if (r >= ((int64_t)1 << (-sh - 1)))
            q++;
    }
    return m < 0 ? -(i128)q : (i128)q;
}

/* Step 2: the samples p in [1, n) where the line L0 + p S comes within delta of a cell boundary
   (a multiple of 2^lgB).  Writes up to cap of them in ascending order to hit[]; returns their
   number, or -1 if there are more (or delta is not small against B).  Each hit is the next
   sample whose residue falls below 2 delta (first_below: O(log B) per hit). */
static int ambiguous(i128 L0, i128 S, i128 delta, int lgB, int64_t n, int64_t *hit, int cap)
{
    const uint64_t B = (uint64_t)1 << lgB;           /* lgB <= 55 */
    if (delta >= (i128)(B / 4))
        return -1;
    if (delta <= 0)
        return 0;                                    /* nothing within a zero distance */
    const uint64_t st = (uint64_t)(((S % (i128)B) + (i128)B) % (i128)B);
    /* r(p) in [0, delta) or [B - delta, B)  <=>  (r(p) + delta) mod B < 2 delta */
    const uint64_t a0 = (uint64_t)((((L0 % (i128)B) + (i128)B) % (i128)B + delta) % (i128)B);
    const uint64_t w = 2 * (uint64_t)delta;
    int nh = 0;
    int64_t p0 = 1;
    while (p0 < n) {
        const uint64_t a = (uint64_t)(((u128)a0 + (u128)p0 * st) % B);
        const uint64_t m = (uint64_t)(n - p0);
        const uint64_t i = first_below(m, B, a, st, w);
        if (i >= m)
            break;
        if (nh == cap)
            return -1;
        hit[nh++] = p0 + (int64_t)i;
        p0 += (int64_t)i + 1;
    }
    return nh;
}

/* ---- one block ------------------------------------------------------------------------------ */
#define LIN_CARR_LGB 55          /* 2^55 units of 2^-64 cycle = one of the 512 LUT cells */
#define LIN_CODE_LGB 50          /* 2^50 units of 2^-50 chip = one chip */
#define LIN_CARR_ERR ((i128)1 << 12)    /* one step's rounding (bound), units of 2^-64 cycle */
#define LIN_CODE_ERR ((i128)1 << 7)     /* one step's rounding (bound), units of 2^-50 chip  */
#define LIN_MAXHIT 64            /* ambiguous samples examined per chain */

static int signed_gain(int gain, const uint32_t *nav, int iword, int ibit)
{
    return ((nav[iword] >> (29 - ibit)) & 1u) ? gain : -gain;
}

static int find_hit(const int64_t *hit, int nh, int64_t q)
{
    for (int i = 0; i < nh; i++)
        if (hit[i] == q)
            return i;
    return -1;
}

/* code wraps between the block start and state c, from the counters */
static int64_t wraps_of(const gss_code_state *c, const gss_chan_blk_t *p)
{
    return ((int64_t)(c->iword - p->iword) * 30 + (c->ibit - p->ibit)) * 20 +
           (c->icode - p->icode);
}

/* cos + 2^22 sin of LUT cell c (the kernel's packed I/Q term, gpssim.c:15-83); the tables are
   filled once, by pthread_once, before any worker reads them */
static int32_t lut_sinT[512], lut_cosT[512];
static pthread_once_t lut_once = PTHREAD_ONCE_INIT;

static void lut_fill(void) { gss_lut(lut_sinT, lut_cosT); }

static int64_t lut_packed(int c)
{
    return (int64_t)lut_cosT[c] + (int64_t)lut_sinT[c] * ((int64_t)1 << 22);
}

static int ca_sign(const uint32_t *ca, int chip)          /* codeCA (gpssim.c:2220) */
{
    return ((ca[chip >> 5] >> (chip & 31)) & 1u) ? 1 : -1;
}

/* 1 if the line value v lies within d of a multiple of 2^lgB */
static int near_boundary(i128 v, i128 d, int lgB)
{
    const i128 B = (i128)1 << lgB;
    return (((v + d) % B) + B) % B < 2 * d;
}

/* merge two ascending sample lists and {0}: ascending, no duplicates */
static int merge_hits(const int64_t *a, int na, const int64_t *b, int nb, int64_t *out)
{
    int i = 0, j = 0, n = 0;
    out[n++] = 0;
    while (i < na || j < nb) {
        int64_t v = (j >= nb || (i < na && a[i] <= b[j])) ? a[i++] : b[j++];
        if (v != out[n - 1])
            out[n++] = v;
    }
    return n;
}

/* 1 if certified (lin filled), 0 if this channel needs the exact path */
static int lin_channel(const gss_chan_blk_t *p, int n, const uint32_t *nav, const uint32_t *ca,
                       gss_lin_t *lin)
{
    int inexact = 0;
    int64_t hx[LIN_MAXHIT], hz[LIN_MAXHIT], hq[2 * LIN_MAXHIT + 1];
    gss_code_state at_hz[LIN_MAXHIT];

    /* ---- the two lines and the samples where they decide nothing (gpssim.c:2212-2250) ---- */
    const double x0 = p->carr0, s = p->carr_step;
    if (!(x0 >= 0.0 && x0 < 1.0) || !(s > -0.5 && s < 0.5))
        return 0;
    const i128 X0 = to_fix(x0, 64, &inexact), XS = to_fix(s, 64, &inexact);
    const i128 DX1 = 2 + (i128)n * (LIN_CARR_ERR + 1);           /* line vs reference */
    const double c0 = p->code0, cs = p->code_step;
    if (!(c0 >= 0.0 && c0 < GSS_CA_SEQ_LEN_D) || !(cs > 0.0 && cs < 1.0))
        return 0;
    const int64_t ZS = (int64_t)to_fix(cs, 50, &inexact);
    /* An exact chain: the integer-carrier variant's rows (--carrier=int, gpssim.c:2252) are
       multiples of 2^-25 cycle, so every IEEE step and wrap of the reference is exact and the
       line IS the reference.  The kernel then rounds nothing either (xs is a multiple of 2^39,
       gss_lin.h): its carrier word is the line's, a multiple of 2^7, plus the code word's
       carries, fewer than 2^7 (KDEV below 2^39 units of 2^-64): no sample can change cell. */
    int ix = 0;
    (void)to_fix(x0, 25, &ix);
    (void)to_fix(s, 25, &ix);
    const int exact_carr = !ix && GSS_LIN_KDEV_CARR((uint64_t)ZS) < ((uint64_t)1 << 39);
    const int nhx = exact_carr ? 0 : ambiguous(X0, XS, DX1 + GSS_LIN_KDEV_CARR((uint64_t)ZS),
                                               LIN_CARR_LGB, n, hx, LIN_MAXHIT);
    if (nhx < 0)
        return 0;
    if (p->iword < 0 || p->iword >= GSS_NAV_WORDS || p->ibit < 0 || p->ibit >= 30 ||
        p->icode < 0 || p->icode >= 20)
        return 0;
    const int64_t Z0 = (int64_t)to_fix(c0, 50, &inexact);
    const int64_t per = (int64_t)GSS_CA_LEN << LIN_CODE_LGB;
    /* the kernel reads one 32-chip window per 64-sample step, starting up to 2 chips below
       lane 0's chip: from the LDS window pass (GSS_LIN_WIN_OK) or the chunk window table
       (gss_lin_win16_ok); both hold, so that either build of the kernel may render the block */
    if (ZS <= 0 || Z0 >= per || !GSS_LIN_WIN_OK((uint64_t)ZS) ||
        !gss_lin_win16_ok((uint64_t)ZS, n))
        return 0;
    const int nhz = ambiguous(Z0, ZS, 2 + (i128)n * (LIN_CODE_ERR + 1) + GSS_LIN_KDEV_CODE,
                              LIN_CODE_LGB, n, hz, LIN_MAXHIT);
    if (nhz < 0)
        return 0;
    lin->x0 = (uint64_t)X0;
    lin->xs = (uint64_t)XS;
    lin->z0 = (uint64_t)Z0;
    lin->zs = (uint64_t)ZS;

    /* exact code state at the code's ambiguous samples */
    gss_code_state st = {c0, p->icode, p->ibit, p->iword};
    int64_t at = 0;
    for (int i = 0; i < nhz; i++) {
        gss_code_walk_cc(&st, cs, hz[i] - at);
        at = hz[i];
        at_hz[i] = st;
    }

    /* ---- code wraps, data bits and the signed-gain schedule ---- */
    int ng = 0;
    int g = signed_gain(p->gain, nav, p->iword, p->ibit);
    lin->gpos[ng] = 0;
    lin->gval[ng++] = g;
    gss_code_state cnt = {0.0, p->icode, p->ibit, p->iword};
    /* the line's k-th wrap is the first q with Z0 + q ZS >= k per: q = ceil((k per - Z0) / ZS). */
    /* Only the wraps that start a data bit matter: wrap 20 - icode, then every 20th (icode counts
       0..19, gss_code_count_wrap).  The ones between decide nothing, and a later wrap lies >= 1023
       samples further on (code_step < 1), so the loop ends where the per-wrap loop would. */
    for (int64_t k = 20 - p->icode;; k += 20) {
        const i128 num = (i128)k * per - Z0;             /* > 0: k >= 1, Z0 < per */
        int64_t q = (int64_t)(num / ZS) + (num % ZS > 0);
        if (q - 1 >= n)
            break;
        int j = find_hit(hz, nhz, q - 1);
        if (j >= 0 && wraps_of(&at_hz[j], p) >= k)
            q--;                                 /* the exact value wrapped one sample earlier */
        else if ((j = find_hit(hz, nhz, q)) >= 0 && wraps_of(&at_hz[j], p) < k)
            q++;                                 /* ... or one sample later */
        if (q >= n)
            break;
        cnt.icode = 19;                          /* the 19 wraps since the last data bit */
        gss_code_count_wrap(&cnt);               /* a new data bit */
        if (cnt.iword >= GSS_NAV_WORDS)
            return 0;                            /* dwrd[60]: the exact path reports it */
        const int g2 = signed_gain(p->gain, nav, cnt.iword, cnt.ibit);
        if (g2 != g) {
            /* the kernel takes at most one change per 4096-sample wave segment (they are
               >= 20 code periods = 20 ms apart in any real run) */
            if (ng == GSS_NGC || (ng > 1 && q - lin->gpos[ng - 1] < 4096))
                return 0;
            lin->gpos[ng] = (int32_t)q;
            lin->gval[ng++] = g2;
            g = g2;
        }
    }
    for (int i = ng; i < GSS_NGC; i++) {
        lin->gpos[i] = INT32_MAX;
        lin->gval[i] = g;
    }

    /* ---- patches: the exact term where the kernel's differs ---- */
    const int nq = merge_hits(hx, nhx, hz, nhz, hq);
    double x = x0;
    int64_t xat = 0;
    int np = 0, gi = 0;
    for (int i = 0; i < nq; i++) {
        const int64_t q = hq[i];
        int cell, chip;
        if (q == 0) {
            cell = (int)floor(x0 * 512.0);
        } else if (near_boundary(X0 + (i128)q * XS, DX1, LIN_CARR_LGB)) {
            x = gss_carr_walk_cc(x, s, q - xat);     /* the reference may differ from the line */
            xat = q;
            cell = (int)floor(x * 512.0);
            if (cell > 511)      /* carr += 1.0 rounded to 1.0: the reference reads cosTable512[512]
                                    (SURVEY A.7); the exact path renders it */
                return 0;
        } else {                                 /* proven: exact = line */
            cell = (int)((uint64_t)(X0 + (i128)q * XS) >> LIN_CARR_LGB);
        }
        int j;
        if (q == 0)
            chip = (int)floor(c0);
        else if ((j = find_hit(hz, nhz, q)) >= 0)
            chip = (int)floor(at_hz[j].ph);
        else
            chip = (int)(((Z0 + (i128)q * ZS) >> LIN_CODE_LGB) % GSS_CA_LEN);
        const gss_lin_kc kk = gss_lin_kernel_at((uint64_t)X0, (uint64_t)XS, (uint64_t)Z0,
                                                 (uint64_t)ZS, q);
        const int kcell = kk.cell, kchip = kk.chip;
        const int64_t te = ca_sign(ca, chip) * lut_packed(cell);
        const int64_t tk = ca_sign(ca, kchip) * lut_packed(kcell);
        if (te == tk)
            continue;
        while (gi + 1 < GSS_NGC && lin->gpos[gi + 1] <= q)
            gi++;
        if (np == GSS_NPATCH)
            return 0;
        lin->ppos[np] = (int32_t)q;
        lin->pdelta[np++] = (int64_t)lin->gval[gi] * (te - tk);
    }
    (void)inexact;
    return 1;
}

typedef struct {
    const gss_chan_blk_t *blk;
    const int32_t *nch;
    const uint32_t *nav, *ca;
    int n_nav, n_ca, n_per_blk, b_lo, b_hi;
    gss_lin_t *lin;
    int32_t *fast;
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
                             j->ca + (size_t)p->ca_tbl * GSS_CA_WORDS,
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
    if (!blk || !nch || !lin || !fast || nblk < 0 || n_per_blk <= 0 || (n_nav > 0 && !nav) ||
        (n_ca > 0 && !ca_bits) || n_ca < 0)
        return gss_fail(GSS_E_ARG, "invalid linearize arguments");
    if (nblk == 0)
        return 0;
    pthread_once(&lut_once, lut_fill);                /* before any worker thread starts */
    const lin_job all = {blk, nch, nav, ca_bits, n_nav, n_ca, n_per_blk, 0, nblk, lin, fast};
    /* one part per block on the pooled workers (blocks differ in their ambiguous samples) */
    gss_pool_run(threads, nblk, lin_part, (void *)&all);
    return 0;
}
