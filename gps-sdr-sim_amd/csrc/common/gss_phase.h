/*
 * gss_phase.h — exact restatement of the sample loop's two double recurrences, shared by the
 * host planner (gcc) and the HIP kernels (hipcc).  Everything here must reproduce every IEEE
 * double rounding of the reference loop, so: no FMA contraction (built with -ffp-contract=off),
 * no fast-math, and only operations whose result is either the reference's own operation or
 * provably exact.
 *
 * Reference recurrences (gpssim.c):
 *   carrier  2245-2250   carr += f_carr*delt;  if (carr>=1) carr-=1; else if (carr<0) carr+=1;
 *   code     2212-2237   code += f_code*delt;  if (code>=1023) { code-=1023; icode++ → 20 →
 *                        ibit++ → 30 → iword++ }
 *
 * Jump-ahead ("binade walk").  While a value v stays inside one binade [2^e, 2^(e+1)) its lattice
 * is u = 2^(e-52) and fl(v+s) = v + round(s/u)*u, with round-half-even resolving to an even
 * multiple once v sits on an even lattice point.  So a run of J steps inside a binade is v+J*K*u,
 * computed exactly with integers.  Steps that change binade, and the wraps, are taken as real
 * double steps.  gss_jump() returns the longest run that is provably a pure lattice translation;
 * SURVEY.md §7(4) option B, verified against brute force in tests/test_phase_walk.py.
 */
#ifndef GSS_PHASE_H
#define GSS_PHASE_H

#include <stdint.h>

#if defined(__HIPCC__)
#define GSS_HD __host__ __device__ inline
#else
#define GSS_HD static inline
#endif

#define GSS_CA_SEQ_LEN_D 1023.0   /* CA_SEQ_LEN as compared in gpssim.c:2214 */

typedef union { double d; uint64_t u; } gss_bits64;

GSS_HD double gss_pow2(int k)   /* exact 2^k for -1022 <= k <= 1023 */
{
    gss_bits64 b;
    b.u = (uint64_t)(k + 1023) << 52;
    return b.d;
}

/* One reference carrier step (gpssim.c:2245-2250). */
GSS_HD double gss_carr_step1(double x, double s)
{
    x = x + s;
    if (x >= 1.0)
        x -= 1.0;
    else if (x < 0.0)
        x += 1.0;
    return x;
}

/* Code phase with its counters (gpssim.c:2212-2237). */
typedef struct gss_code_state {
    double  ph;
    int32_t icode, ibit, iword;
} gss_code_state;

GSS_HD void gss_code_step1(gss_code_state *c, double cs)
{
    c->ph = c->ph + cs;
    if (c->ph >= GSS_CA_SEQ_LEN_D) {
        c->ph -= GSS_CA_SEQ_LEN_D;
        c->icode++;
        if (c->icode >= 20) {
            c->icode = 0;
            c->ibit++;
            if (c->ibit >= 30) {
                c->ibit = 0;
                c->iword++;
            }
        }
    }
}

/*
 * Longest run of steps from v (step s != 0) that are exact lattice translations.
 *   W  : wrap threshold for ascending chains (1.0 carrier, 1023.0 code); the run never produces
 *        a value >= W.  Descending chains wrap only below 0, which no positive binade reaches.
 * Returns J >= 0 and sets *D to the per-step increment (J*D exact).  J == INT64_MAX means the
 * value is stationary (|s| < u/2): every further step returns v.
 */
GSS_HD int64_t gss_jump(double v, double s, double W, double *D)
{
    gss_bits64 b;
    b.d = v;
    if (b.u >> 63) return 0;                      /* negative or -0 */
    int E = (int)((b.u >> 52) & 0x7FF);
    if (E < 64 || E == 0x7FF) return 0;          /* zero / tiny / non-finite: take real steps */
    int64_t m = (int64_t)((b.u & 0xFFFFFFFFFFFFFull) | (1ull << 52));   /* v = m*u */
    double u = gss_pow2(E - 1075);
    double inv_u = gss_pow2(1075 - E);
    double as = s < 0.0 ? -s : s;
    double sig = as * inv_u;                      /* |s|/u, exact (power-of-two scaling) */
    if (!(sig < 4503599627370496.0)) return 0;    /* >= 2^52: every step leaves the binade */
    double sfl = (double)(int64_t)sig;            /* floor (sig >= 0) */
    int64_t k = (int64_t)sfl;
    double frac = sig - sfl;                      /* exact */
    int64_t K;
    if (frac < 0.5)
        K = k;
    else if (frac > 0.5)
        K = k + 1;
    else {                                        /* tie: stable only from an even lattice point */
        if (m & 1) return 0;
        K = (k & 1) ? k + 1 : k;
    }
    if (K == 0) { *D = 0.0; return INT64_MAX; }
    int64_t lim;
    if (s > 0.0) {
        int64_t tau = (1ll << 53) - m;            /* (2^(e+1) - v)/u */
        lim = tau - k - 1;                        /* j*K + sig < tau  <=>  j*K <= tau-floor(sig)-1 */
        double top = gss_pow2(E - 1022);          /* 2^(e+1) */
        if (W <= top) {                           /* wrap threshold inside this binade */
            int64_t omega = (int64_t)((W - v) * inv_u);
            int64_t lim2 = omega - K - 1;         /* v + (j+1)*K*u < W */
            if (lim2 < lim) lim = lim2;
        }
    } else {
        int64_t beta = m - (1ll << 52);           /* (v - 2^e)/u */
        int64_t kc = frac > 0.0 ? k + 1 : k;      /* ceil(|s|/u) */
        lim = beta - kc;                          /* j*K + |sig| <= beta */
    }
    if (lim < 0) return 0;
    *D = (s > 0.0 ? (double)K : -(double)K) * u;
    return lim / K + 1;
}

/* Advance the carrier recurrence by n steps, exactly. */
GSS_HD double gss_carr_walk(double x, double s, int64_t n)
{
    while (n > 0) {
        double D;
        int64_t J = gss_jump(x, s, 1.0, &D);
        if (J > 0) {
            if (J == INT64_MAX) return x;
            if (J > n) J = n;
            x = x + (double)J * D;               /* J*K <= 2^52: product and sum exact */
            n -= J;
            if (n == 0) break;
        }
        x = gss_carr_step1(x, s);
        n--;
    }
    return x;
}

/* Advance the code recurrence (with counters) by n steps, exactly. */
GSS_HD void gss_code_walk(gss_code_state *c, double cs, int64_t n)
{
    while (n > 0) {
        double D;
        int64_t J = gss_jump(c->ph, cs, GSS_CA_SEQ_LEN_D, &D);
        if (J > 0) {
            if (J == INT64_MAX) return;
            if (J > n) J = n;
            c->ph = c->ph + (double)J * D;
            n -= J;
            if (n == 0) break;
        }
        gss_code_step1(c, cs);
        n--;
    }
}

#endif /* GSS_PHASE_H */
