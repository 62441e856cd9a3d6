/*
 * linearize.c — certified integer linearisation of the sample loop's two double recurrences.
 *
 * The reference steps, per sample and channel (gpssim.c:2212-2250),
 *     code += f_code*delt  (wrap at 1023, counters icode/ibit/iword, new data bit every 20 wraps)
 *     carr += f_carr*delt  (wrap into [0,1))
 * and reads LUT[floor(512 carr)] and ca[floor(code)].  Every step is one IEEE rounding, so the
 * exact trajectory differs from the real line x0 + p*s by a deterministic, slowly varying error.
 * For one 0.1 s block this file finds a 64-bit integer line L(p) = L0 + p*S and proves, with exact
 * integer arithmetic, that floor(L(p) / B) equals floor(exact(p) / B) for every sample p of the
 * block (B = 2^55 in carrier units of 2^-64 cycle: the 512 LUT cells; B = 2^50 in code units of
 * 2^-50 chip: the chips, and so also the 1023-chip wraps).  The GPU fast path (gss_lin_kernel)
 * then needs only 64-bit integer adds per sample.
 *
 * Proof, per chain:
 *   1. The exact chain is walked wrap by wrap (gss_phase.h cycle-cached walks, the same ones the
 *      planner uses), giving the exact unwrapped value U at p = 0, at every wrap and at p = n.
 *   2. S = round((U(n) - U(0)) / n); e(p) = U(p) - L(p) is known exactly at those points.
 *   3. Between two known points e changes by at most g per sample, g = |s*2^k - S| + (bound of
 *      one step's rounding error: 2^-53 cycle = 2^11 units for the carrier, 2^-44 chip = 2^6
 *      units for the code; the bounds used are doubled).  So |e| <= (|e_a| + |e_b| + (p_b-p_a) g)/2
 *      on [p_a, p_b]; Delta is the maximum over the block.
 *   4. min_p (L(p) mod B) >= Delta and max_p (L(p) mod B) <= B-1-Delta over p in [0, n), both
 *      computed exactly (gss_minmod: Euclid-like, O(log B)).  Then no cell boundary lies between
 *      L(p) and the exact value, for any p.
 * A channel that fails (or any other precondition below) sends its block to the exact walking
 * path (Stage A + Stage B); gss_linearize reports that per block.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "gss_host.h"
#include "../common/gss_phase.h"

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

/* exported for tests (64-bit operands): min and max of (a + p s) mod m over [0, n) */
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
        return (i128)m << sh;
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

static i128 iabs128(i128 v) { return v < 0 ? -v : v; }

static i128 round_div(i128 num, int64_t den)        /* den > 0, nearest */
{
    i128 h = den / 2;
    return num >= 0 ? (num + h) / den : -((-num + h) / den);
}

/* known exact points of one chain: sample index and unwrapped fixed-point value */
typedef struct {
    int64_t *p;
    i128 *u;
    int n, cap;
} pts_t;

static int pts_push(pts_t *t, int64_t p, i128 u)
{
    if (t->n == t->cap) {
        int nc = t->cap ? 2 * t->cap : 64;
        int64_t *np = realloc(t->p, sizeof(int64_t) * nc);
        if (!np) return -1;
        t->p = np;
        i128 *nu = realloc(t->u, sizeof(i128) * nc);
        if (!nu) return -1;
        t->u = nu;
        t->cap = nc;
    }
    t->p[t->n] = p;
    t->u[t->n] = u;
    t->n++;
    return 0;
}

/* Steps 2-4 for a chain with known points t (first at p=0, last at p=n): slope, Delta, and the
   certificate against cells of size 2^lgB.  step_err: bound of one step's rounding error in
   units; s_fix: the step s in units (rounded).  Returns 1 if certified. */
static int certify(const pts_t *t, int64_t n, i128 s_fix, i128 step_err, int lgB, i128 *L0,
                   i128 *S, i128 *delta_out)
{
    const i128 u0 = t->u[0];
    const i128 sl = round_div(t->u[t->n - 1] - u0, n);
    const i128 g = iabs128(s_fix - sl) + 1 + step_err;
    i128 delta = 0;
    i128 e_prev = 0;
    for (int i = 0; i < t->n; i++) {
        const i128 e = t->u[i] - (u0 + (i128)t->p[i] * sl);
        if (i > 0) {
            const i128 b = (iabs128(e_prev) + iabs128(e) + (i128)(t->p[i] - t->p[i - 1]) * g + 1) / 2;
            if (b > delta) delta = b;
        }
        e_prev = e;
    }
    delta += 4;                                      /* fixed-point roundings of the points */
    *L0 = u0;
    *S = sl;
    *delta_out = delta;
    const u128 B = (u128)1 << lgB;
    if (delta >= (i128)(B / 4))
        return 0;
    /* samples 1 .. n-1 (sample 0 is L(0) = the start value rounded: the caller checks it) */
    if (n < 2)
        return 1;
    const u128 st = (u128)(((sl % (i128)B) + (i128)B) % (i128)B);
    const u128 a = ((u128)(((u0 % (i128)B) + (i128)B) % (i128)B) + st) % B;
    const u128 mn = gss_minmod((u128)(n - 1), B, a, st);
    const u128 mx = gss_maxmod((u128)(n - 1), B, a, st);
    if (getenv("GSS_LIN_DEBUG"))
        fprintf(stderr, "certify lgB=%d pts=%d delta=2^%.1f g=2^%.1f min=2^%.1f B-1-max=2^%.1f\n",
                lgB, t->n, log2((double)delta), log2((double)g), log2((double)mn + 1),
                log2((double)(B - 1 - mx) + 1));
    return mn >= (u128)delta && mx + (u128)delta <= B - 1;
}

/* ---- one block ------------------------------------------------------------------------------ */
#define LIN_CARR_LGB 55          /* 2^55 units of 2^-64 cycle = one of the 512 LUT cells */
#define LIN_CODE_LGB 50          /* 2^50 units of 2^-50 chip = one chip */
#define LIN_CARR_ERR ((i128)1 << 12)
#define LIN_CODE_ERR ((i128)1 << 7)

typedef struct {
    pts_t pc, pz;
} lin_ws;

static int signed_gain(int gain, const uint32_t *nav, int iword, int ibit)
{
    return ((nav[iword] >> (29 - ibit)) & 1u) ? gain : -gain;
}

/* 1 if certified (lin filled), 0 if this channel needs the exact path, <0 on allocation error */
static int lin_channel(const gss_chan_blk_t *p, int n, const uint32_t *nav, lin_ws *ws,
                       gss_lin_t *lin)
{
    int inexact = 0;
    /* ---- carrier (gpssim.c:2245-2250) ---- */
    const double x0 = p->carr0, s = p->carr_step;
    if (!(x0 >= 0.0 && x0 < 1.0) || !(s > -0.5 && s < 0.5))
        return 0;
    pts_t *t = &ws->pc;
    t->n = 0;
    gss_carr_it it;
    gss_carr_it_init(&it, x0, s, n);
    int64_t w = 0;
    if (pts_push(t, 0, to_fix(x0, 64, &inexact))) return -1;
    while (gss_carr_next_wrap(&it)) {
        w += s > 0.0 ? 1 : -1;
        if (pts_push(t, it.pos, to_fix(it.x, 64, &inexact) + ((i128)w << 64))) return -1;
    }
    if (it.pos != n) return 0;
    if (pts_push(t, n, to_fix(it.x, 64, &inexact) + ((i128)w << 64))) return -1;
    i128 L0, S, dl;
    if (!certify(t, n, to_fix(s, 64, &inexact), LIN_CARR_ERR, LIN_CARR_LGB, &L0, &S, &dl))
        return 0;
    if (L0 < 0 || L0 >= ((i128)1 << 64) || (int)(L0 >> LIN_CARR_LGB) != (int)floor(x0 * 512.0))
        return 0;                                /* sample 0: the rounded start's own cell */
    lin->x0 = (uint64_t)L0;
    lin->xs = (uint64_t)S;

    /* ---- code with its counters (gpssim.c:2212-2237) ---- */
    const double c0 = p->code0, cs = p->code_step;
    if (!(c0 >= 0.0 && c0 < GSS_CA_SEQ_LEN_D) || !(cs > 0.0 && cs < 1.0))
        return 0;
    if (p->iword < 0 || p->iword >= GSS_NAV_WORDS || p->ibit < 0 || p->ibit >= 30 ||
        p->icode < 0 || p->icode >= 20)
        return 0;
    t = &ws->pz;
    t->n = 0;
    gss_code_state st0 = {c0, p->icode, p->ibit, p->iword};
    gss_code_it ic;
    gss_code_it_init(&ic, st0, cs, n);
    const i128 per = (i128)GSS_CA_LEN << LIN_CODE_LGB;
    if (pts_push(t, 0, to_fix(c0, 50, &inexact))) return -1;
    int ng = 0;
    int g = signed_gain(p->gain, nav, p->iword, p->ibit);
    lin->gpos[ng] = 0;
    lin->gval[ng++] = g;
    int64_t nw = 0;
    int prev_ibit = p->ibit, prev_iword = p->iword;
    while (gss_code_next_wrap(&ic)) {
        nw++;
        if (pts_push(t, ic.pos, to_fix(ic.c.ph, 50, &inexact) + nw * per)) return -1;
        if (ic.c.ibit != prev_ibit || ic.c.iword != prev_iword) {     /* a new data bit */
            prev_ibit = ic.c.ibit;
            prev_iword = ic.c.iword;
            if (ic.c.iword >= GSS_NAV_WORDS)
                return 0;                       /* dwrd[60]: the exact path reports it */
            const int g2 = signed_gain(p->gain, nav, ic.c.iword, ic.c.ibit);
            if (g2 != g) {
                /* the kernel takes at most one change per 4096-sample wave segment (they are
                   >= 20 code periods = 20 ms apart in any real run) */
                if (ng == GSS_NGC || (ng > 1 && ic.pos - lin->gpos[ng - 1] < 4096)) return 0;
                lin->gpos[ng] = (int32_t)ic.pos;
                lin->gval[ng++] = g2;
                g = g2;
            }
        }
    }
    if (ic.pos != n) return 0;
    if (pts_push(t, n, to_fix(ic.c.ph, 50, &inexact) + nw * per)) return -1;
    if (!certify(t, n, to_fix(cs, 50, &inexact), LIN_CODE_ERR, LIN_CODE_LGB, &L0, &S, &dl))
        return 0;
    if (L0 < 0 || (int64_t)(L0 >> LIN_CODE_LGB) != (int64_t)floor(c0))
        return 0;                                /* sample 0: the rounded start's own chip */
    /* the kernel reads a 64-chip window per two 64-sample steps: 127 steps + 2 chips <= 64 */
    if (S * 127 + ((i128)2 << LIN_CODE_LGB) > ((i128)64 << LIN_CODE_LGB))
        return 0;
    lin->z0 = (uint64_t)L0;
    lin->zs = (uint64_t)S;
    for (int i = ng; i < GSS_NGC; i++) {
        lin->gpos[i] = INT32_MAX;
        lin->gval[i] = g;
    }
    return 1;
}

typedef struct {
    const gss_chan_blk_t *blk;
    const int32_t *nch;
    const uint32_t *nav;
    int n_nav, n_per_blk, b_lo, b_hi;
    gss_lin_t *lin;
    int32_t *fast;
    int err;
} lin_job;

static void *lin_run(void *arg)
{
    lin_job *j = arg;
    lin_ws ws;
    memset(&ws, 0, sizeof ws);
    for (int b = j->b_lo; b < j->b_hi && !j->err; b++) {
        int ok = 1, gsum = 0;
        const int nc = j->nch[b];
        for (int k = 0; k < GSS_MAXCH; k++) {
            gss_lin_t *l = &j->lin[(size_t)b * GSS_MAXCH + k];
            memset(l, 0, sizeof *l);
            for (int i = 0; i < GSS_NGC; i++)
                l->gpos[i] = INT32_MAX;
        }
        if (nc < 0 || nc > GSS_MAXCH)
            ok = 0;
        for (int k = 0; ok && k < nc; k++) {
            const gss_chan_blk_t *p = &j->blk[(size_t)b * GSS_MAXCH + k];
            gsum += p->gain < 0 ? -p->gain : p->gain;
            if (p->nav_tbl < 0 || p->nav_tbl >= j->n_nav) {
                ok = 0;
                break;
            }
            int r = lin_channel(p, j->n_per_blk, j->nav + (size_t)p->nav_tbl * GSS_NAV_WORDS,
                                &ws, &j->lin[(size_t)b * GSS_MAXCH + k]);
            if (r < 0) {
                j->err = GSS_E_NOMEM;
                break;
            }
            ok = r;
        }
        /* the packed I/Q accumulator (gss_lin_kernel) needs 250*sum|gain| + 64 < 2^21 */
        if (gsum > 8000)
            ok = 0;
        j->fast[b] = ok;
    }
    free(ws.pc.p); free(ws.pc.u); free(ws.pz.p); free(ws.pz.u);
    return NULL;
}

int gss_linearize(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                  const uint32_t *nav, int n_nav, gss_lin_t *lin, int32_t *fast, int threads)
{
    if (!blk || !nch || !lin || !fast || nblk < 0 || n_per_blk <= 0 || (n_nav > 0 && !nav))
        return gss_fail(GSS_E_ARG, "invalid linearize arguments");
    if (nblk == 0)
        return 0;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if (threads > nblk) threads = nblk;
    pthread_t tid[64];
    lin_job job[64];
    int started[64] = {0};
    const int per = (nblk + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        int lo = t * per, hi = lo + per > nblk ? nblk : lo + per;
        job[t] = (lin_job){blk, nch, nav, n_nav, n_per_blk, lo, hi, lin, fast, 0};
        if (lo >= hi)
            continue;
        if (threads == 1 || pthread_create(&tid[t], NULL, lin_run, &job[t]) != 0)
            lin_run(&job[t]);
        else
            started[t] = 1;
    }
    int err = 0;
    for (int t = 0; t < threads; t++) {
        if (started[t])
            pthread_join(tid[t], NULL);
        if (job[t].err)
            err = job[t].err;
    }
    return err ? gss_fail(err, "out of memory in gss_linearize") : 0;
}
