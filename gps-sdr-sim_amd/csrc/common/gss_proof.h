/*
 * gss_proof.h — the fast path's proof for one channel of one block (lin_channel), shared bit for
 * bit by the host (csrc/host/linearize.c: gss_linearize) and the GPU (csrc/hip/gss_proof.hip:
 * gss_linearize_device).  The method is linearize.c's header comment; this file holds its
 * arithmetic: the exact first-hit descent (first_in, first_below), the ambiguous-sample
 * enumeration, the code-wrap and signed-gain schedule and the patches.  Everything here is exact
 * integer arithmetic plus the IEEE walks of gss_phase.h (no contraction: -ffp-contract=off on
 * both sides), so both builds produce the same gss_lin_t rows.
 * Device constraints kept for the host too: no recursion (first_in descends iteratively, at most
 * GSS_PF_EUCLID_MAX levels; deeper gives the channel up) and no 128-bit division (gss_pf_udiv).
 */
#ifndef GSS_PROOF_H
#define GSS_PROOF_H

#include <math.h>
#include <stdint.h>
#include <string.h>
#include "gpssim_amd.h"
#include "gss_phase.h"
#include "gss_lin.h"

#if defined(__HIPCC__)
#define GSS_PF static __host__ __device__ inline
#else
#define GSS_PF static inline
#endif

typedef unsigned __int128 u128;
typedef __int128 i128;

/* floor(a / b) for b > 0 and a quotient below 2^64: a 64-bit division when a fits 64 bits; for a
   quotient below 2^53 a double estimate (a's two halves converted apart: relative error below
   2^-51, so off by at most two here) corrected by exact products; above, an exact shift-subtract
   long division (no caller reaches it: the proofs' quotients stay far below 2^53).  No 128-bit
   division (none on the GPU, a slow library call on the host). */
GSS_PF uint64_t gss_pf_udiv(u128 a, uint64_t b)
{
    const uint64_t hi = (uint64_t)(a >> 64), lo = (uint64_t)a;
    if (hi == 0)
        return lo / b;
    if (a < ((u128)b << 53)) {
        uint64_t q = (uint64_t)(((double)hi * 0x1p64 + (double)lo) / (double)b);
        while ((u128)q * b > a)
            q--;
        while ((u128)(q + 1) * b <= a)
            q++;
        return q;
    }
    u128 r = 0;                                      /* r < 2^65 throughout */
    uint64_t q = 0;
    for (int i = 127; i >= 0; i--) {
        r = (r << 1) | (uint64_t)((a >> i) & 1u);
        if (r >= b) {
            r -= b;
            if (i < 64)
                q |= (uint64_t)1 << i;
        }
    }
    return q;
}

#ifndef GSS_PF_EUCLID_MAX
#define GSS_PF_EUCLID_MAX 32       /* descent levels kept (a deeper one gives up: uncertified).
                                      The deepest descent of every test scenario (static and
                                      circle 2.6 MS/s, 20 MS/s, -b 1; ~2.5 M descents) is 21
                                      levels (GSS_PF_STATS builds); 32 keeps a
                                      margin at 768 B of stack per lane instead of 1.5 KB */
#endif
#ifdef GSS_PF_STATS
void gss_pf_depth_note(int d);     /* linearize.c: a histogram of descent depths */
#endif
#define GSS_PF_GIVE_UP (UINT64_MAX - 1)
GSS_PF uint64_t first_in(uint64_t s, uint64_t m, uint64_t lo, uint64_t hi, uint64_t lim)
{
    /* the descent, level by level (iterative: the GPU proof has no call stack to spare); each
       level that needs the next one's answer keeps (s, m, lo, lim) for the way back up */
    /* (a level's modulus is the level above's step: m_{d+1} = s_d, so only m_0 is kept) */
    uint64_t fs[GSS_PF_EUCLID_MAX], flo[GSS_PF_EUCLID_MAX], flim[GSS_PF_EUCLID_MAX];
    const uint64_t m0 = m;
    int d = 0;
    uint64_t r;
    for (;;) {
        if (s == 0) {
            r = UINT64_MAX;
            break;
        }
        const uint64_t x = (lo + s - 1) / s;
        if (x > lim) {
            r = UINT64_MAX;
            break;
        }
        if (s * x <= hi) {                               /* s x <= lo + s - 1 < 2^63 */
            r = x;
            break;
        }
        if (d == GSS_PF_EUCLID_MAX)
            return GSS_PF_GIVE_UP;
#ifdef GSS_PF_STATS                                  /* (host measurement builds only) */
        gss_pf_depth_note(d + 1);
#endif
        /* no multiple of s in [lo, hi]: both lie in ((x - 1) s, x s), so their residues are
           one product away (no further division; 1 <= lr <= hr < s) */
        const uint64_t base = s * (x - 1), lr = lo - base, hr = hi - base;
        const double yd = (double)lim * (double)s / (double)m + 2.0;
        const uint64_t ylim = yd < 0x1p52 ? (uint64_t)yd : UINT64_MAX;
        fs[d] = s; flo[d] = lo; flim[d] = lim;
        d++;
        const uint64_t ns = m % s;
        m = s;
        lo = s - hr;
        hi = s - lr;
        s = ns;
        lim = ylim;
    }
    while (d > 0) {                                      /* y = r: x = ceil((lo + m y) / s) */
        d--;
        if (r == UINT64_MAX)
            return UINT64_MAX;
        const uint64_t md = d ? fs[d - 1] : m0;
        const u128 num = (u128)flo[d] + (u128)md * r + fs[d] - 1;
        /* v <= lim  <=>  num < (lim + 1) s; only then divide (the quotient fits) */
        r = num < ((u128)flim[d] + 1) * fs[d] ? gss_pf_udiv(num, fs[d]) : UINT64_MAX;
    }
    return r;
}

/* Smallest p in [0, n) with (a + p s) mod m < w (0 <= a, s < m < 2^62, 0 < w <= m), or n. */
GSS_PF uint64_t first_below(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t w)
{
    if (n == 0)
        return 0;
    if (a < w)
        return 0;
    /* (a + p s) mod m < w  <=>  (s p) mod m in [m - a, m - a + w - 1], a range below m as a >= w */
    const uint64_t p = first_in(s, m, m - a, m - a + w - 1, n - 1);
    if (p == GSS_PF_GIVE_UP)
        return GSS_PF_GIVE_UP;
    return p < n ? p : n;
}

/* ---- fixed point ----------------------------------------------------------------------------- */
/* x * 2^k rounded to nearest (ties away); *inexact set if rounding happened.  |x| < 2^60. */
GSS_PF i128 to_fix(double x, int k, int *inexact)
{
    int e;
    int64_t m;                                       /* exact: x = m * 2^(e-53) */
    uint64_t bits;
    memcpy(&bits, &x, sizeof bits);
    const int E = (int)((bits >> 52) & 0x7FF);
    if (E != 0 && E != 0x7FF) {                      /* normal: the fields directly */
        const int64_t M = (int64_t)((bits & (((uint64_t)1 << 52) - 1)) | ((uint64_t)1 << 52));
        m = (bits >> 63) ? -M : M;
        e = E - 1022;                                /* frexp's: x = (M / 2^53) * 2^e */
    } else {
        const double fr = frexp(x, &e);              /* x = fr * 2^e, 0.5 <= |fr| < 1 */
        m = (int64_t)ldexp(fr, 53);
    }
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

/* The samples p in [1, n) with (a0 + p st) mod B < w (B a power of two, w < B / 2), ascending,
   up to cap of them in hit[]; their number, or -1 if there are more or a descent gives up.
   scan: each hit found by its own descent from the one before (first_below: O(log B) each).
   Otherwise the descents find the first hit and the two gaps of the window's first returns:
   by the three-gap theorem (Slater) a point x of [0, w) comes back to it after ga steps (moving
   by da = ga st mod B) if x + da < w, after gb steps (moving back by db = B - gb st mod B) if
   x >= db, and after ga + gb steps otherwise, ga and gb the first p >= 1 with p st mod B in
   [0, w) resp. (B - w, B) -- no two returns come sooner, and the three ranges split [0, w)
   since da + db >= w.  Every further hit is then O(1).  Gaps past the range are not needed:
   a return through one lies past it too.  The switch from the scan to the gaps comes after
   gap_at hits (below). */
#ifndef GSS_PF_GAPS
#define GSS_PF_GAPS 0            /* (measurement builds: 1 gaps from the first hit, 2 never)       */
#endif
GSS_PF int hits_mod(uint64_t n, uint64_t B, uint64_t a0, uint64_t st, uint64_t w, int32_t *hit,
                    int cap, int scan)
{
    const uint64_t M = B - 1;
    /* the two gap descents pay once a few hits follow: from the first hit where the window
       expects two or more in the range (n w / B), after the third where it expects fewer (most
       such ranges have none or one, which the scan finds in one or two descents) */
    const int gap_at = GSS_PF_GAPS == 1 ? 1 : GSS_PF_GAPS == 2 ? -1 :
                       (double)n * (double)w >= 2.0 * (double)B ? 1 : 3;
    int nh = 0;
    int64_t p0 = 1;
    while (p0 < (int64_t)n) {
        const uint64_t a = (a0 + (uint64_t)p0 * st) & M;            /* mod 2^64, then mod B */
        const uint64_t m = n - (uint64_t)p0;
        const uint64_t i = first_below(m, B, a, st, w);
        if (i == GSS_PF_GIVE_UP)
            return -1;
        if (i >= m)
            break;
        if (nh == cap)
            return -1;
        hit[nh++] = (int32_t)(p0 + (int64_t)i);
        p0 += (int64_t)i + 1;
        if (scan || nh != gap_at)
            continue;
        /* the gaps, for returns that stay inside the range */
        const int64_t p = hit[nh - 1];
        const uint64_t lim = n - 1 - (uint64_t)p;
        if (lim == 0)
            break;
        const uint64_t s1 = st & M;
        const uint64_t ia = first_below(lim, B, s1, s1, w);          /* (1 + i) st mod B < w */
        const uint64_t ib = s1 ? first_in(s1, B, B - w + 1, B - 1, lim) : UINT64_MAX;
        if (ia == GSS_PF_GIVE_UP || ib == GSS_PF_GIVE_UP)
            continue;                                 /* the scan from here on */
        const int has_a = ia < lim, has_b = ib >= 1 && ib <= lim;
        const uint64_t ga = ia + 1, gb = ib;
        const uint64_t da = has_a ? (ga * s1) & M : 0, db = has_b ? B - ((gb * s1) & M) : 0;
        uint64_t x = (a0 + (uint64_t)p * st) & M, q = (uint64_t)p;
        for (;;) {
            if (has_a && x + da < w) {
                q += ga;
                x += da;
            } else if (has_b && x >= db) {
                q += gb;
                x -= db;
            } else if (has_a && has_b) {
                q += ga + gb;
                x = x + da - db;
            } else {
                break;                                /* the next return lies past the range */
            }
            if (q >= n)
                break;
            if (nh == cap)
                return -1;
            hit[nh++] = (int32_t)q;
        }
        return nh;
    }
    return nh;
}

/* Step 2: the samples p in [1, n) where the line L0 + p S comes within delta of a cell boundary
   (a multiple of 2^lgB).  Writes up to cap of them in ascending order to hit[]; returns their
   number, or -1 if there are more (or delta is not small against B). */
GSS_PF int ambiguous(i128 L0, i128 S, i128 delta, int lgB, int64_t n, int32_t *hit, int cap)
{
    const uint64_t B = (uint64_t)1 << lgB;           /* lgB <= 55 */
    if (delta >= (i128)(B / 4))
        return -1;
    if (delta <= 0)
        return 0;                                    /* nothing within a zero distance */
    /* residues mod the power of two B: the low lgB bits of the two's complement value */
    const uint64_t st = (uint64_t)S & (B - 1);
    /* r(p) in [0, delta) or [B - delta, B)  <=>  (r(p) + delta) mod B < 2 delta */
    const uint64_t a0 = ((uint64_t)L0 + (uint64_t)delta) & (B - 1);
    const uint64_t w = 2 * (uint64_t)delta;
    return hits_mod((uint64_t)n, B, a0, st, w, hit, cap, 0);
}

/* ---- one block ------------------------------------------------------------------------------ */
#define LIN_CARR_LGB 55          /* 2^55 units of 2^-64 cycle = one of the 512 LUT cells */
#define LIN_CODE_LGB 50          /* 2^50 units of 2^-50 chip = one chip */
#define LIN_CARR_ERR ((i128)1 << 12)    /* one step's rounding (bound), units of 2^-64 cycle */
#define LIN_CODE_ERR ((i128)1 << 7)     /* one step's rounding (bound), units of 2^-50 chip  */
#define LIN_MAXHIT 64            /* ambiguous samples examined per chain */

GSS_PF int signed_gain(int gain, const uint32_t *nav, int iword, int ibit)
{
    return ((nav[iword] >> (29 - ibit)) & 1u) ? gain : -gain;
}

GSS_PF int find_hit(const int32_t *hit, int nh, int64_t q)
{
    for (int i = 0; i < nh; i++)
        if (hit[i] == q)
            return i;
    return -1;
}

/* code wraps between the block start and state c, from the counters */
GSS_PF int64_t wraps_of(const gss_code_state *c, const gss_chan_blk_t *p)
{
    return ((int64_t)(c->iword - p->iword) * 30 + (c->ibit - p->ibit)) * 20 +
           (c->icode - p->icode);
}

/* what the proof keeps of the exact code state at an ambiguous code sample: its chip and its
   wraps since the block start (8 B instead of a 24-B gss_code_state per sample) */
typedef struct gss_pf_code {
    int32_t chip, wraps;
} gss_pf_code;

/* cos + 2^22 sin of LUT cell c (the kernel's packed I/Q term, gpssim.c:15-83), from the tables of
   gss_lut */
GSS_PF int64_t lut_packed(const int32_t *lcos, const int32_t *lsin, int c)
{
    return (int64_t)lcos[c] + (int64_t)lsin[c] * ((int64_t)1 << 22);
}

GSS_PF int ca_sign(const uint32_t *ca, int chip)          /* codeCA (gpssim.c:2220) */
{
    return ((ca[chip >> 5] >> (chip & 31)) & 1u) ? 1 : -1;
}

/* 1 if the line value v lies within d of a multiple of 2^lgB */
GSS_PF int near_boundary(i128 v, i128 d, int lgB)
{
    const uint64_t B = (uint64_t)1 << lgB;           /* (v + d) mod B: the low lgB bits */
    return (i128)(((uint64_t)v + (uint64_t)d) & (B - 1)) < 2 * d;
}

/* ---- one channel's proof in three parts ----------------------------------------------------
 * lin_carrier  the carrier line, its ambiguous samples and the exact LUT cell at each of them
 *              (exact walks from the chain's anchors where the reference may differ from it);
 * lin_code     the code line, its ambiguous samples and the exact chip at each, the code wraps'
 *              data bits and the signed-gain schedule;
 * lin_patches  sample 0 and every ambiguous sample of either line in ascending order: the exact
 *              term against the kernel's, a patch where they differ.
 * The first two are independent: the GPU proves them on two lanes at once (gss_proof.hip), the
 * host in order (lin_channel).  A failing channel's row is reset to its initial state
 * (lin_row_reset) on both, so the rows match byte for byte whichever part failed first. */
typedef struct gss_pf_side {          /* one line's ambiguous samples and the exact values there */
    int32_t n;                        /* their number                                         */
    int32_t q[LIN_MAXHIT];            /* samples, ascending                                  */
    int32_t v[LIN_MAXHIT];            /* the exact LUT cell (carrier) or chip (code) there    */
} gss_pf_side;

GSS_PF void lin_row_reset(gss_lin_t *l)
{
    memset(l, 0, sizeof *l);
    for (int i = 0; i < GSS_NGC; i++)
        l->gpos[i] = INT32_MAX;
    for (int i = 0; i < GSS_NPATCH; i++)
        l->ppos[i] = INT32_MAX;
}

/* the carrier part (1: done, 0: the channel needs the exact path).  an (NULL: none): the chain's
   exact carrier values inside the block (gss_carr_anchor_t), where the carrier walks to the
   ambiguous samples start instead of at the block start; or, without them, sin / sspec (NULL:
   none): the row's speculative walk, from which the anchors are made the first time a walk is
   needed (gss_spec_anchors; gss_run's GPU proofs over the walks it keeps on the device).  The
   rows are the same either way. */
GSS_PF int lin_carrier(const gss_chan_blk_t *p, int n, const gss_carr_anchor_t *an,
                       const gss_spec_in_t *sin, const gss_spec_t *sspec, gss_pf_side *cx,
                       gss_lin_t *lin)
{
    gss_carr_anchor_t la;
    int inexact = 0;
    cx->n = 0;
    /* ---- the line and the samples where it decides nothing (gpssim.c:2245-2250) ---- */
    const double x0 = p->carr0, s = p->carr_step, cs = p->code_step;
    if (!(x0 >= 0.0 && x0 < 1.0) || !(s > -0.5 && s < 0.5) || n <= 0 || n > INT32_MAX / 2 ||
        !(cs > 0.0 && cs < 1.0))
        return 0;
    const i128 X0 = to_fix(x0, 64, &inexact), XS = to_fix(s, 64, &inexact);
    const i128 DX1 = 2 + (i128)n * (LIN_CARR_ERR + 1);           /* line vs reference */
    const int64_t ZS = (int64_t)to_fix(cs, 50, &inexact);       /* (the kernel's deviation) */
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
                                               LIN_CARR_LGB, n, cx->q, LIN_MAXHIT);
    if (nhx < 0)
        return 0;
    lin->x0 = (uint64_t)X0;
    lin->xs = (uint64_t)XS;
    /* ---- the exact cell at each: the line's where it is farther than DX1 from a cell boundary
       (the reference lies within DX1 of it), else an exact walk from the last anchor or the
       last walk before it ---- */
    double x = x0;
    int64_t xat = 0;
    for (int i = 0; i < nhx; i++) {
        const int64_t q = cx->q[i];
        int cell;
        if (near_boundary(X0 + (i128)q * XS, DX1, LIN_CARR_LGB)) {
            if (!an && sin && sspec && sin->s == s) {  /* the anchors, once, from the walk */
                gss_spec_anchors(x0, n, sin, sspec, la.pos, la.val);
                an = &la;
            }
            if (an)                                  /* from the last anchor past the walk */
                for (int a = GSS_SPEC_K - 1; a >= 1; a--)
                    if (an->pos[a] > xat && an->pos[a] <= q) {
                        x = an->val[a];
                        xat = an->pos[a];
                        break;
                    }
#ifndef GSS_PF_NOWALK                                /* (measurement builds: no walks) */
            x = gss_carr_walk_cc(x, s, q - xat);     /* the reference may differ from the line */
#endif
            xat = q;
            cell = (int)floor(x * 512.0);
            if (cell > 511)      /* carr += 1.0 rounded to 1.0: the reference reads cosTable512[512]
                                    (SURVEY A.7); the exact path renders it */
                return 0;
        } else {                                 /* proven: exact = line */
            cell = (int)((uint64_t)(X0 + (i128)q * XS) >> LIN_CARR_LGB);
        }
        cx->v[i] = cell;
    }
    cx->n = nhx;
    (void)inexact;
    return 1;
}

/* the code part (1: done, 0: the exact path) */
GSS_PF int lin_code(const gss_chan_blk_t *p, int n, const uint32_t *nav, gss_pf_side *cz,
                    gss_lin_t *lin)
{
    int inexact = 0;
    int32_t wr_hz[LIN_MAXHIT];                       /* code wraps at each ambiguous sample */
    const int32_t *hz = cz->q;
    cz->n = 0;
    const double c0 = p->code0, cs = p->code_step;
    if (n <= 0 || n > INT32_MAX / 2 || !(c0 >= 0.0 && c0 < GSS_CA_SEQ_LEN_D) ||
        !(cs > 0.0 && cs < 1.0))
        return 0;
    const int64_t ZS = (int64_t)to_fix(cs, 50, &inexact);
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
    const i128 DZ1 = 2 + (i128)n * (LIN_CODE_ERR + 1);            /* line vs reference */
    const int nhz = ambiguous(Z0, ZS, DZ1 + GSS_LIN_KDEV_CODE, LIN_CODE_LGB, n, cz->q,
                              LIN_MAXHIT);
    if (nhz < 0)
        return 0;
    lin->z0 = (uint64_t)Z0;
    lin->zs = (uint64_t)ZS;

    /* exact code state at the code's ambiguous samples (the samples where the KERNEL's chip may
       differ from the line's).  The reference's value lies within DZ1 of the line, so where the
       line is farther than that from every chip boundary the reference has the line's chip and
       the line's number of wraps: its state follows from the line, and only the samples whose
       line is within DZ1 of a boundary take the exact walk (from the last walked state) */
    gss_code_state st = {c0, p->icode, p->ibit, p->iword};
    int64_t at = 0;
    for (int i = 0; i < nhz; i++) {
        const i128 zq = (i128)Z0 + (i128)hz[i] * ZS;
        if (near_boundary(zq, DZ1, LIN_CODE_LGB)) {
#ifndef GSS_PF_NOWALK
            gss_code_walk_cc(&st, cs, hz[i] - at);
#endif
            at = hz[i];
            cz->v[i] = (int32_t)floor(st.ph);
            wr_hz[i] = (int32_t)wraps_of(&st, p);
        } else {
            /* the line's chip and wraps (from chip 0 of the block) */
            const int64_t chips = (int64_t)(zq >> LIN_CODE_LGB);
            cz->v[i] = (int32_t)(chips % GSS_CA_LEN);
            wr_hz[i] = (int32_t)(chips / GSS_CA_LEN);
        }
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
        const uint64_t qd = gss_pf_udiv((u128)num, (uint64_t)ZS);
        int64_t q = (int64_t)qd + ((u128)qd * (uint64_t)ZS < (u128)num);
        if (q - 1 >= n)
            break;
        int j = find_hit(hz, nhz, q - 1);
        if (j >= 0 && wr_hz[j] >= k)
            q--;                                 /* the exact value wrapped one sample earlier */
        else if ((j = find_hit(hz, nhz, q)) >= 0 && wr_hz[j] < k)
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
    cz->n = nhz;
    (void)inexact;
    return 1;
}

/* the patches, after both parts: the exact term where the kernel's differs, at sample 0 and
   every ambiguous sample of either line in ascending order (the two lists merged as read) */
GSS_PF int lin_patches(const gss_chan_blk_t *p, int n, const uint32_t *ca, const int32_t *lcos,
                       const int32_t *lsin, const gss_pf_side *cx, const gss_pf_side *cz,
                       gss_lin_t *lin)
{
    int inexact = 0;
    const double x0 = p->carr0, c0 = p->code0;
    const i128 X0 = to_fix(x0, 64, &inexact), XS = to_fix(p->carr_step, 64, &inexact);
    const int64_t Z0 = (int64_t)to_fix(c0, 50, &inexact);
    const int64_t ZS = (int64_t)to_fix(p->code_step, 50, &inexact);
    const int nhx = cx->n, nhz = cz->n;
    int np = 0, gi = 0;
    int hxi = 0, hzi = 0;
    (void)n;
    for (int64_t q = 0; q >= 0;) {
        int cell, chip;
        if (q == 0)
            cell = (int)floor(x0 * 512.0);
        else if (hxi < nhx && cx->q[hxi] == q)       /* (hxi: the first carrier hit not below q) */
            cell = cx->v[hxi];
        else
            cell = (int)((uint64_t)(X0 + (i128)q * XS) >> LIN_CARR_LGB);
        if (q == 0)
            chip = (int)floor(c0);
        else if (hzi < nhz && cz->q[hzi] == q)
            chip = cz->v[hzi];
        else
            chip = (int)((uint64_t)((Z0 + (i128)q * ZS) >> LIN_CODE_LGB) % GSS_CA_LEN);
        const gss_lin_kc kk = gss_lin_kernel_at((uint64_t)X0, (uint64_t)XS, (uint64_t)Z0,
                                                 (uint64_t)ZS, q);
        const int kcell = kk.cell, kchip = kk.chip;
        const int64_t te = ca_sign(ca, chip) * lut_packed(lcos, lsin, cell);
        const int64_t tk = ca_sign(ca, kchip) * lut_packed(lcos, lsin, kcell);
        if (te != tk) {
            while (gi + 1 < GSS_NGC && lin->gpos[gi + 1] <= q)
                gi++;
            if (np == GSS_NPATCH)
                return 0;
            lin->ppos[np] = (int32_t)q;
            lin->pdelta[np++] = (int64_t)lin->gval[gi] * (te - tk);
        }
        /* the next sample of the merged lists past q (-1: none) */
        while (hxi < nhx && cx->q[hxi] <= q)
            hxi++;
        while (hzi < nhz && cz->q[hzi] <= q)
            hzi++;
        q = hxi < nhx ? (hzi < nhz && cz->q[hzi] < cx->q[hxi] ? cz->q[hzi] : cx->q[hxi])
                      : hzi < nhz ? cz->q[hzi] : -1;
    }
    (void)inexact;
    return 1;
}

/* 1 if certified (lin filled), 0 if this channel needs the exact path (lin reset): the three
   parts in order (lin_carrier's anchors: as there) */
GSS_PF int lin_channel(const gss_chan_blk_t *p, int n, const uint32_t *nav, const uint32_t *ca,
                       const int32_t *lcos, const int32_t *lsin, const gss_carr_anchor_t *an,
                       const gss_spec_in_t *sin, const gss_spec_t *sspec, gss_lin_t *lin)
{
    gss_pf_side cx, cz;
    const int ok = lin_carrier(p, n, an, sin, sspec, &cx, lin) && lin_code(p, n, nav, &cz, lin) &&
                   lin_patches(p, n, ca, lcos, lsin, &cx, &cz, lin);
    if (!ok)
        lin_row_reset(lin);
    return ok;
}


#endif /* GSS_PROOF_H */
