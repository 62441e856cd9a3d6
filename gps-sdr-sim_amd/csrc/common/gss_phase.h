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
#if defined(__HIP_DEVICE_COMPILE__)
    /* no 64-bit integer divider on the GPU: floor(lim / K) from the hardware reciprocal refined
       by one Newton step (relative error ~2^-50: the estimate is off by at most a few), then
       fixed up exactly in f64 -- lim, K < 2^53 and the residual lim - q K is an integer of
       magnitude below 2^53, so one fma gives it exactly (no IEEE division sequence and no
       64-bit integer multiplies on this hot path of every exact walk) */
    const double Kd = (double)K, ld = (double)lim;
    double r = __builtin_amdgcn_rcp(Kd);
    r = __builtin_fma(__builtin_fma(-Kd, r, 1.0), r, r);
    double q = __builtin_floor(ld * r);
    double res = __builtin_fma(-q, Kd, ld);
    while (res < 0.0) {
        q -= 1.0;
        res += Kd;
    }
    while (res >= Kd) {
        q += 1.0;
        res -= Kd;
    }
    return (int64_t)q + 1;
#else
    return lim / K + 1;
#endif
}

/* ---- the same jump in f64 only (GPU form: no 64-bit integer multiply/divide) ------------------
 * All quantities are integers below 2^54 held in doubles, so every operation below is exact
 * except the one division, whose floor is corrected with an exact fma residual.  Same contract
 * as gss_jump(), but returns J capped at nmax (a double holding an integer) and *dv = ±J*K*u,
 * the exact total displacement.  A stationary value (K == 0) returns nmax with *dv = 0. */
#if defined(__HIP_DEVICE_COMPILE__)
#define GSS_FREXP_EXP(v)   __builtin_amdgcn_frexp_exp(v)
#define GSS_LDEXP(v, e)    __builtin_amdgcn_ldexp((v), (e))
#define GSS_FLOOR(v)       __builtin_floor(v)
#define GSS_RINT(v)        __builtin_rint(v)
#define GSS_FMA(a, b, c)   __builtin_fma((a), (b), (c))
#else
#include <math.h>
GSS_HD int gss_frexp_exp_h(double v) { int e; (void)frexp(v, &e); return e; }
#define GSS_FREXP_EXP(v)   gss_frexp_exp_h(v)
#define GSS_LDEXP(v, e)    ldexp((v), (e))
#define GSS_FLOOR(v)       floor(v)
#define GSS_RINT(v)        rint(v)                /* default rounding: nearest-even */
#define GSS_FMA(a, b, c)   fma((a), (b), (c))
#endif

GSS_HD double gss_jumpf(double v, double s, double W, double nmax, double *dv)
{
    if (!(v >= 0x1p-900)) return 0.0;             /* zero, negative, tiny, NaN: real steps */
    int ex = GSS_FREXP_EXP(v);                    /* binade [2^(ex-1), 2^ex), lattice 2^(ex-53) */
    double m = GSS_LDEXP(v, 53 - ex);             /* v/u in [2^52, 2^53) */
    double as = s < 0.0 ? -s : s;
    double sig = GSS_LDEXP(as, 53 - ex);          /* |s|/u */
    if (!(sig < 0x1p52)) return 0.0;
    double k = GSS_FLOOR(sig);
    double frac = sig - k;
    double K = GSS_RINT(sig);                     /* round-half-even = fl()'s rule from even m */
    if (frac == 0.5) {
        double h = m * 0.5;
        if (h != GSS_FLOOR(h)) return 0.0;        /* tie from an odd lattice point */
    }
    if (K == 0.0) { *dv = 0.0; return nmax; }
    double lim;
    if (s > 0.0) {
        lim = ((0x1p53 - m) - k) - 1.0;           /* result stays below 2^ex */
        if (W <= GSS_LDEXP(1.0, ex)) {            /* and below the wrap threshold */
            double l2 = (GSS_LDEXP(W - v, 53 - ex) - K) - 1.0;
            if (l2 < lim) lim = l2;
        }
    } else {
        lim = (m - 0x1p52) - (frac > 0.0 ? k + 1.0 : k);   /* result stays >= 2^(ex-1) */
    }
    if (lim < 0.0) return 0.0;
    double q = GSS_FLOOR(lim / K);                /* correctly rounded: floor is q or q+1 */
    if (GSS_FMA(-q, K, lim) < 0.0) q -= 1.0;
    double J = q + 1.0;
    if (J > nmax) J = nmax;
    double d = GSS_LDEXP(J * K, ex - 53);         /* J*K <= 2^53: exact */
    *dv = s > 0.0 ? d : -d;
    return J;
}

/* n steps (n an integer held in a double) of x += s with the reference's wrap at W
   (>= W: -W, else < 0: +W; carrier W = 1, code W = 1023).  *nwrap counts wraps. */
GSS_HD double gss_walkf(double x, double s, double W, double n, int *nwrap)
{
    if (s == 0.0)
        return x;
    while (n > 0.0) {
        double dv;
        double J = gss_jumpf(x, s, W, n, &dv);
        if (J > 0.0) {
            x = x + dv;
            n -= J;
            if (n == 0.0) break;
        }
        x = x + s;
        n -= 1.0;
        if (x >= W) { x -= W; (*nwrap)++; }
        else if (x < 0.0) { x += W; (*nwrap)++; }
    }
    return x;
}

/* Walk from *x until just after the next wrap, at most *left steps.  Returns 1 on a wrap
   (*x = post-wrap value), 0 when *left runs out (*x = value reached); *left is decremented by
   the steps taken. */
GSS_HD int gss_to_wrapf(double *x, double s, double W, double *left)
{
    double v = *x, n = *left;
    int wr = 0;
    if (s == 0.0) {
        n = 0.0;
    } else {
        while (n > 0.0) {
            double dv;
            double J = gss_jumpf(v, s, W, n, &dv);
            if (J > 0.0) {
                v = v + dv;
                n -= J;
                if (n == 0.0) break;
            }
            v = v + s;
            n -= 1.0;
            if (v >= W) { v -= W; wr = 1; break; }
            if (v < 0.0) { v += W; wr = 1; break; }
        }
    }
    *x = v;
    *left = n;
    return wr;
}

/* ---- branch-free form of one walk iteration (GPU lanes: no divergent control flow) -----------
 * One iteration = the longest exact lattice jump from v (possibly empty, gss_jumpf's rules),
 * then one real reference step with its wrap, if steps remain.  Every lane executes the same
 * instruction sequence; decisions are selects.  Lane constants: as = |s|, rs = 1/|s| (any
 * rounding), W the wrap threshold and exW = ceil(log2 W) (frexp convention: the wrap limit
 * applies in the binade [2^(ex-1), 2^ex) iff ex >= exW; 0 for the carrier, 10 for the code).
 * Returns 1 if the real step wrapped.
 *
 * Exactness of each line: every double below holds an integer < 2^54 or a lattice value, so all
 * adds are exact; q0 is within one of floor(lim/K) for K >= 2^26 (see gss_jumpf) and the fma
 * residual lim - q0*K is exact; v + J*K*u is the lattice point J steps on, exact via one fma. */
GSS_HD int gss_iter_bfx(double *pv, double s, double as, double rs, double W, int exW,
                        double *pleft, double *pJ, double *pDs)
{
    const double v = *pv;
    const double left = *pleft;
    const int ex = GSS_FREXP_EXP(v);
    const int sh = 53 - ex;
    const double m = GSS_LDEXP(v, sh);                 /* v/u */
    const double sig = GSS_LDEXP(as, sh);              /* |s|/u */
    const double urs = GSS_LDEXP(rs, ex - 53);         /* u/|s| */
    const double k = GSS_FLOOR(sig);
    const double K = GSS_RINT(sig);                    /* round-half-even, fl()'s rule */
    const double frac = sig - k;
    const double h = m * 0.5;
    const int odd_tie = (frac == 0.5) & (h != GSS_FLOOR(h));
    /* ascending: stay below 2^ex, and below W in W's binade */
    double lim = ((0x1p53 - 1.0) - k) - m;
    const double l2 = (GSS_LDEXP(W - v, sh) - 1.0) - K;
    lim = ((ex >= exW) & (l2 < lim)) ? l2 : lim;
    /* descending: stay >= 2^(ex-1) */
    const double lim_d = (m - 0x1p52) - (frac > 0.0 ? k + 1.0 : k);
    lim = s > 0.0 ? lim : lim_d;
    const int live = (v >= 0x1p-900) & (sig < 0x1p52) & !odd_tie;
    const int stat = live & (K == 0.0);                /* stationary: no step moves v */
    const int ok = live & (K != 0.0) & (lim >= 0.0);
    double J;
    if (K >= 0x1p26) {
        const double q0 = GSS_FLOOR(lim * urs);
        const double r0 = GSS_FMA(-q0, K, lim);
        J = r0 < 0.0 ? q0 : (r0 >= K ? q0 + 2.0 : q0 + 1.0);
    } else {                                           /* tiny steps: exact division */
        const double Ks = K != 0.0 ? K : 1.0;
        double q = GSS_FLOOR(lim / Ks);
        q = GSS_FMA(-q, Ks, lim) < 0.0 ? q - 1.0 : q;
        J = q + 1.0;
    }
    J = J > left ? left : J;
    J = ok ? J : (stat ? left : 0.0);
    const double Ds = GSS_LDEXP(s > 0.0 ? K : -K, ex - 53);   /* signed K*u: one step's move */
    const double v1 = GSS_FMA(J, Ds, v);
    const double left1 = left - J;
    *pJ = J;
    *pDs = Ds;
    const int step = left1 > 0.0;
    const double r = v1 + s;
    const int hi = r >= W, lo = r < 0.0;
    const double rw = hi ? r - W : (lo ? r + W : r);
    *pv = step ? rw : v1;
    *pleft = step ? left1 - 1.0 : left1;
    return step & (hi | lo);
}

GSS_HD int gss_iter_bf(double *pv, double s, double as, double rs, double W, int exW,
                       double *pleft)
{
    double J, Ds;
    return gss_iter_bfx(pv, s, as, rs, W, exW, pleft, &J, &Ds);
}

/* exW for a wrap threshold W (>= 1): smallest ex with W <= 2^ex */
GSS_HD int gss_exw(double W)
{
    int e = GSS_FREXP_EXP(W);                          /* W in [2^(e-1), 2^e) */
    return GSS_LDEXP(1.0, e - 1) == W ? e - 1 : e;
}

/* ---- direction-specialised trips (fewer instructions; the GPU Stage A hot loop) --------------
 * Same contract as gss_iter_bfx for one chain kind:
 *   GSS_TRIP_CARR_ASC  carrier, s > 0 (W = 1: the wrap limit is the binade top of [0.5, 1))
 *   GSS_TRIP_CARR_DESC carrier, s < 0 (wraps below 0 with carr += 1, rounded)
 *   GSS_TRIP_CODE      code phase, s > 0, W = 1023 inside the binade [512, 1024)
 * Scale factors come from the exponent field: with E the biased exponent of v (v in
 * [2^(E-1023), 2^(E-1022)), lattice u = 2^(E-1075)), 1/u and u are built as doubles from E, and
 * m = v/u = 2^52 + mantissa is v with its exponent field replaced by 1075.  The tie parity of m
 * is the mantissa's last bit.  Requires v >= 2^-900 for a jump (smaller v: real steps only). */
#define GSS_TRIP_CARR_ASC  0
#define GSS_TRIP_CARR_DESC 1
#define GSS_TRIP_CODE      2

GSS_HD double gss_d_from_hi(uint32_t hi, uint32_t lo)
{
    gss_bits64 b;
    b.u = ((uint64_t)hi << 32) | lo;
    return b.d;
}

GSS_HD int gss_trip(int kind, double *pv, double s, double rs, double *pleft, double *pJ,
                    double *pDs)
{
    const double v = *pv;
    const double left = *pleft;
    gss_bits64 vb;
    vb.d = v;
    const uint32_t hi = (uint32_t)(vb.u >> 32), lo = (uint32_t)vb.u;
    const uint32_t X = hi & 0x7FF00000u;                       /* E << 20 */
    const double P = gss_d_from_hi(0x83200000u - X, 0u);       /* 2^(1075-E) = 1/u */
    const double Pi = gss_d_from_hi(X - 0x03400000u, 0u);      /* 2^(E-1075) = u   */
    const double m = gss_d_from_hi((hi & 0x000FFFFFu) | 0x43300000u, lo);   /* v/u */
    const double as = kind == GSS_TRIP_CARR_DESC ? -s : s;
    const double sig = as * P;
    const double k = GSS_FLOOR(sig);
    const double K = GSS_RINT(sig);
    const double frac = sig - k;
    const int odd_tie = (frac == 0.5) & (int)(lo & 1u);
    double lim;
    if (kind == GSS_TRIP_CARR_DESC) {
        lim = (m - 0x1p52) - (frac > 0.0 ? k + 1.0 : k);       /* stay >= 2^(ex-1) */
    } else {
        lim = ((0x1p53 - 1.0) - k) - m;                        /* stay < 2^ex */
        if (kind == GSS_TRIP_CARR_ASC) {
            /* top binade [0.5,1): a result rounding up to 1.0 would wrap: (j+1)K < 2^53 - m */
            lim = X == (1022u << 20) ? lim - (K - k) : lim;
        } else {
            const double l2 = ((GSS_CA_SEQ_LEN_D - v) * P - 1.0) - K;    /* v + (j+1)Ku < 1023 */
            lim = ((X >= (1032u << 20)) & (l2 < lim)) ? l2 : lim;
        }
    }
    const int live = (v >= 0x1p-900) & (sig < 0x1p52) & !odd_tie & (lim >= 0.0);
    double J;
    if (K >= 0x1p26) {
        const double q0 = GSS_FLOOR(lim * (rs * Pi));          /* lim*u/|s| */
        const double r0 = GSS_FMA(-q0, K, lim);
        J = (q0 + 1.0) + ((r0 >= K ? 1.0 : 0.0) + (r0 < 0.0 ? -1.0 : 0.0));
        J = live ? (J < left ? J : left) : 0.0;
    } else if (K == 0.0) {                                      /* stationary */
        J = ((v >= 0x1p-900) & (sig < 0x1p52) & !odd_tie) ? left : 0.0;
    } else {                                                    /* tiny steps: exact division */
        double q = GSS_FLOOR(lim / K);
        q = GSS_FMA(-q, K, lim) < 0.0 ? q - 1.0 : q;
        J = live ? (q + 1.0 < left ? q + 1.0 : left) : 0.0;
    }
    const double Ds = kind == GSS_TRIP_CARR_DESC ? -(K * Pi) : K * Pi;   /* one step's move */
    const double v1 = GSS_FMA(J, Ds, v);
    const double left1 = left - J;
    const double r = v1 + s;                                    /* the real step */
    double r2;
    int wr;
    if (kind == GSS_TRIP_CARR_DESC) {
        wr = r < 0.0;
        r2 = r + (wr ? 1.0 : 0.0);                              /* carr += 1.0 (rounded) */
    } else {
        const double W = kind == GSS_TRIP_CODE ? GSS_CA_SEQ_LEN_D : 1.0;
        wr = r >= W;
        r2 = r - (wr ? W : 0.0);                                /* exact */
    }
    const int step = left1 > 0.0;
    *pv = step ? r2 : v1;
    *pleft = step ? left1 - 1.0 : 0.0;
    *pJ = J;
    *pDs = Ds;
    return step & wr;
}

#ifndef GSS_CARR_MACRO
#define GSS_CARR_MACRO 8         /* real carrier steps near a wrap (gss_seg_states) */
#endif
/* one reference carrier step (gpssim.c:2245-2250): on the GPU v_fract_f64 of the sum, which is
   exactly carr-1 / carr+1 for sums in [0,2) / (-1,1) */
#if defined(__HIP_DEVICE_COMPILE__)
#define GSS_CARR_STEP(v, s) __builtin_amdgcn_fract((v) + (s))
#else
#define GSS_CARR_STEP(v, s) gss_carr_step1((v), (s))
#endif

/* Exact states at the segment starts n0 = j*seg_r in [pos0, pos1) of one chain (j < nseg),
 * walking from v at position pos0 (Stage A of the GPU path: out_x[j] = phase at n0, out_c[j] =
 * code counters icode|ibit<<8|iword<<16 at n0 for the code chain; arrays indexed by the absolute
 * segment j).  A trip covers positions (pb, pa]: a lattice jump of J steps from vb (state at
 * pb + i is vb + i*Ds, exact) and one real step to pa.  At most one segment start usually falls
 * in a trip; more (long jumps at tiny Dopplers) take a loop.  kind: GSS_TRIP_* (the carrier kind
 * must match the sign of st; st == 0 means no motion).  Returns the value at pos1 if want_end,
 * else the value where the walk stopped (after the last segment start in range). */
GSS_HD double gss_seg_states(int kind, double v, double st, uint32_t cnt, int pos0, int pos1,
                             int nseg, int seg_r, int want_end, double *out_x, uint32_t *out_c)
{
    const int code = kind == GSS_TRIP_CODE;
    const double rs = 1.0 / (st < 0.0 ? -st : st);
    const double p0 = (double)pos0, total = (double)(pos1 - pos0), R = (double)seg_r;
    int seg = (pos0 + seg_r - 1) / seg_r;               /* first segment start >= pos0 */
    int seg_hi = (pos1 + seg_r - 1) / seg_r;            /* segment starts < pos1 */
    if (seg_hi > nseg)
        seg_hi = nseg;
    double left = st == 0.0 ? 0.0 : total;             /* no motion: no wraps */
    double n0 = (double)seg * R - p0;                   /* next segment start, relative */
    if (seg < seg_hi && n0 == 0.0) {                    /* a segment starts at pos0 */
        out_x[seg] = v;
        if (code)
            out_c[seg] = cnt;
        seg++;
        n0 += R;
    }
    if (left == 0.0)
        for (; seg < seg_hi; seg++) {
            out_x[seg] = v;
            if (code)
                out_c[seg] = cnt;
        }
    while (left > 0.0 && (seg < seg_hi || want_end)) {
        const double vb = v, pb = total - left;
        double J, Ds;
        const int wr = gss_trip(kind, &v, st, rs, &left, &J, &Ds);
        const double pa = total - left;
        const uint32_t cnt_b = cnt;
        if (code & wr) {                                /* gpssim.c:2216-2236 */
            uint32_t icode = (cnt & 0xFFu) + 1u, ibit = (cnt >> 8) & 0xFFu, iword = cnt >> 16;
            const uint32_t nb = icode >= 20u;
            icode = nb ? 0u : icode;
            ibit += nb;
            const uint32_t nw = ibit >= 30u;
            ibit = nw ? 0u : ibit;
            iword += nw;
            cnt = icode | (ibit << 8) | (iword << 16);
        }
        if (seg + 1 < seg_hi && n0 + R <= pa) {         /* rare: two or more starts */
            for (; seg + 1 < seg_hi && n0 + R <= pa; seg++, n0 += R) {
                out_x[seg] = n0 <= pb + J ? GSS_FMA(n0 - pb, Ds, vb) : v;
                if (code)
                    out_c[seg] = n0 == pa ? cnt : cnt_b;
            }
        }
        if (seg < seg_hi && n0 <= pa) {
            out_x[seg] = n0 <= pb + J ? GSS_FMA(n0 - pb, Ds, vb) : v;
            if (code)
                out_c[seg] = n0 == pa ? cnt : cnt_b;
            seg++;
            n0 += R;
        }
        if (!code) {
            /* Carrier phases near 0 sit in tiny binades whose trips cover 1-4 samples each: right
               after an ascending wrap (v < |s|), and in the last GSS_CARR_MACRO samples before a
               descending wrap.  Take GSS_CARR_MACRO real steps there instead (the reference's
               own step, wrap included), when no segment start and not the end fall inside. */
            const double as = st < 0.0 ? -st : st;
            double vm = v;
            for (int i = 0; i < GSS_CARR_MACRO; i++)
                vm = GSS_CARR_STEP(vm, st);
            const double lo = kind == GSS_TRIP_CARR_ASC ? as : (double)GSS_CARR_MACRO * as;
            const int mac = (v < lo) & (left > (double)GSS_CARR_MACRO) &
                            ((seg >= seg_hi) | (n0 > pa + (double)GSS_CARR_MACRO));
            v = mac ? vm : v;
            left = mac ? left - (double)GSS_CARR_MACRO : left;
        }
    }
    return v;
}

#ifndef GSS_CODE_MACRO
#define GSS_CODE_MACRO 10        /* real steps right after a code wrap (gss_code_seg_states_bf) */
#endif

/* "Some lane of the wave" on the GPU (uniform loop control); the chain itself on the host. */
#if defined(__HIP_DEVICE_COMPILE__)
#define GSS_ANY(c) (__builtin_amdgcn_ballot_w64(c) != 0)
#else
#define GSS_ANY(c) (c)
#endif

/* The code chain of gss_seg_states (GSS_TRIP_CODE, pos0 = 0, pos1 = n, no end value) without
 * divergent branches, for the GPU Stage A where code chains are few and long and so bound by the
 * latency of one wave's instruction stream, not by issue.  Every trip is gss_trip's K >= 2^26 form
 * as straight-line selects (with st >= 2^-16 the lattice index K = rne(st/u) is >= 2^27 in every
 * binade below 1024); a finished chain makes empty trips (J = 0, no step) until its wave is done.
 * The first segment start in a trip is stored unconditionally, to row slot `dummy` (>= nseg) when
 * there is none; a trip that crosses more starts (top-binade jumps longer than seg_r, high
 * sample rates) takes a uniform loop.  st == 0 (padding channel): every start gets (v, cnt). */
GSS_HD void gss_code_seg_states_bf(double v, double st, uint32_t cnt, int n, int nseg, int seg_r,
                                   int dummy, double *out_x, uint32_t *out_c)
{
    const double rs = st > 0.0 ? 1.0 / st : 0.0, R = (double)seg_r, total = (double)n;
    double left = st > 0.0 ? total : 0.0;
    int seg = 0;
    double n0 = 0.0;
    if (left == 0.0) {
        for (; seg < nseg; seg++) {
            out_x[seg] = v;
            out_c[seg] = cnt;
        }
    } else if (nseg > 0) {
        out_x[0] = v;
        out_c[0] = cnt;
        seg = 1;
        n0 = R;
    }
    for (;;) {
        const double vb = v, pb = total - left;
        const uint32_t cnt_b = cnt;
        gss_bits64 bits;
        bits.d = v;
        const uint32_t hi = (uint32_t)(bits.u >> 32), lo = (uint32_t)bits.u;
        const uint32_t X = hi & 0x7FF00000u;                       /* E << 20 */
        const double P = gss_d_from_hi(0x83200000u - X, 0u);       /* 1/u */
        const double Pi = gss_d_from_hi(X - 0x03400000u, 0u);      /* u   */
        const double m = gss_d_from_hi((hi & 0x000FFFFFu) | 0x43300000u, lo);
        const double sig = st * P;
        const double k = GSS_FLOOR(sig);
        const double K = GSS_RINT(sig);
        const int odd_tie = ((sig - k) == 0.5) & (int)(lo & 1u);
        const double lim0 = ((0x1p53 - 1.0) - k) - m;               /* stay < 2^ex */
        const double l2 = ((GSS_CA_SEQ_LEN_D - v) * P - 1.0) - K;   /* v + (j+1)Ku < 1023 */
        const double lim = ((X >= (1032u << 20)) & (l2 < lim0)) ? l2 : lim0;
        const int live = (v >= 0x1p-900) & (sig < 0x1p52) & !odd_tie & (lim >= 0.0);
        const double q0 = GSS_FLOOR(lim * (rs * Pi));
        const double r0 = GSS_FMA(-q0, K, lim);
        double J = (q0 + 1.0) + ((r0 >= K ? 1.0 : 0.0) + (r0 < 0.0 ? -1.0 : 0.0));
        J = live ? (J < left ? J : left) : 0.0;
        const double Ds = K * Pi;
        const double v1 = GSS_FMA(J, Ds, v);
        const double left1 = left - J;
        const double r = v1 + st;                                   /* the real step */
        const int wr = r >= GSS_CA_SEQ_LEN_D;
        const double r2 = wr ? r - GSS_CA_SEQ_LEN_D : r;
        const int step = left1 > 0.0;
        v = step ? r2 : v1;
        left = step ? left1 - 1.0 : 0.0;
        {                                                           /* gpssim.c:2216-2236 */
            uint32_t icode = (cnt & 0xFFu) + 1u, ibit = (cnt >> 8) & 0xFFu, iword = cnt >> 16;
            const uint32_t nb = icode >= 20u;
            icode = nb ? 0u : icode;
            ibit += nb;
            const uint32_t nw = ibit >= 30u;
            ibit = nw ? 0u : ibit;
            iword += nw;
            cnt = (step & wr) ? (icode | (ibit << 8) | (iword << 16)) : cnt;
        }
        const double pa = total - left;
        {
            const int e1 = (seg < nseg) & (n0 <= pa);
            const int idx = e1 ? seg : dummy;
            out_x[idx] = n0 <= pb + J ? GSS_FMA(n0 - pb, Ds, vb) : v;
            out_c[idx] = n0 == pa ? cnt : cnt_b;
            seg += e1;
            n0 += e1 ? R : 0.0;
        }
        if (GSS_ANY((seg < nseg) & (n0 <= pa))) {                  /* rare: more starts */
            while ((seg < nseg) & (n0 <= pa)) {
                out_x[seg] = n0 <= pb + J ? GSS_FMA(n0 - pb, Ds, vb) : v;
                out_c[seg] = n0 == pa ? cnt : cnt_b;
                seg++;
                n0 += R;
            }
        }
        {
            /* After a wrap (v < st) the next binades are tiny: five trips cover the first ~10
               samples.  Take GSS_CODE_MACRO real steps instead, when neither a segment start,
               the block end nor a wrap (the steps rise monotonically) falls inside. */
            double vm = v;
            for (int i = 0; i < GSS_CODE_MACRO; i++)
                vm = vm + st;
            const int mac = (v < st) & (vm < GSS_CA_SEQ_LEN_D) &
                            (left > (double)GSS_CODE_MACRO) &
                            ((seg >= nseg) | (n0 > pa + (double)GSS_CODE_MACRO));
            v = mac ? vm : v;
            left = mac ? left - (double)GSS_CODE_MACRO : left;
        }
        if (!GSS_ANY((left > 0.0) & (seg < nseg)))
            break;
    }
}

/* n steps with gss_iter_bf; returns the value, *nwrap counts wraps. */
GSS_HD double gss_walk_bf(double x, double s, double W, double n, int *nwrap)
{
    const double as = s < 0.0 ? -s : s;
    if (s == 0.0)
        return x;
    const double rs = 1.0 / as;
    const int exw = gss_exw(W);
    while (n > 0.0)
        *nwrap += gss_iter_bf(&x, s, as, rs, W, exw, &n);
    return x;
}

/* Advance the carrier recurrence by n steps, exactly. */
GSS_HD double gss_carr_walk(double x, double s, int64_t n)
{
    if (s == 0.0)                                /* x + 0 == x: nothing moves */
        return x;
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
    if (cs == 0.0 && c->ph < GSS_CA_SEQ_LEN_D)   /* stationary below the wrap */
        return;
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


/* =========================================================================================
 * Cycle-granular exact walk with a cycle-map cache.
 *
 * Between two wraps ("a cycle") the chain starts from a post-wrap value w that sits on a coarse
 * lattice (2^-52 for the ascending carrier, 2^-43 for the code phase, 2^-53 for the descending
 * carrier).  Every lattice the cycle passes through is at least as fine, so translating w by a
 * multiple δ of that coarse unit translates the whole trajectory by δ — provided every step's
 * exact sum stays in the same binade (same rounding lattice, same tie parity) and every wrap
 * decision is unchanged.  gss_cycle_walk() walks one cycle with the jump walk and records the
 * δ-interval for which that holds (the "margins"); later cycles whose start falls inside a cached
 * interval are taken in O(1): w' = w + dx after L steps.  Verified against brute force in
 * tests/test_phase_walk.py.
 * ========================================================================================= */

typedef struct gss_cyc {
    double lo, hi;        /* valid start values (inclusive)                                     */
    double w0, v0;        /* the walked start and its end value: end(w) = v0 + (w - w0), where
                             w - w0 is exact (same coarse lattice) and so is the sum (the result
                             is representable).  A stored difference v0 - w0 would round.      */
    int64_t L;            /* steps                                                              */
    int succ;             /* the entry the cycle after this one used last time (-1: none)       */
} gss_cyc;

#ifndef GSS_CC_N
#define GSS_CC_N 16
#endif
typedef struct gss_cyc_cache {
    gss_cyc e[GSS_CC_N];
    int n, next;
    int enabled;
    int last;             /* entry of the previous cycle (-1: none / not cached) */
} gss_cyc_cache;

/* exponent of a positive normal double: v in [2^e, 2^(e+1)) */
GSS_HD int gss_exp2i(double v)
{
    gss_bits64 b;
    b.d = v;
    return (int)((b.u >> 52) & 0x7FF) - 1023;
}

/* Margins of one exact step v -> fl(v+s) (ascending or descending), folded into [dlo, dhi]:
   the exact sum t = v + s must stay in its binade under translation by δ (δ a multiple of
   dunit).  An exact tie is translation-invariant only while dunit is an even multiple of the
   result lattice (round-half-even then sees the same parity); otherwise no translation. */
GSS_HD void gss_margin_step(double v, double s, double dunit, double *dlo, double *dhi)
{
    double r = v + s;
    double bb = r - v;
    double err = (v - (r - bb)) + (s - bb);            /* TwoSum: t = r + err exactly */
    double ar = r < 0.0 ? -r : r, aerr = r < 0.0 ? -err : err;   /* work with |t| */
    if (ar == 0.0) { *dlo = 0.0; *dhi = 0.0; return; }
    int e = gss_exp2i(ar);
    double p = gss_pow2(e);
    if (ar == p && aerr < 0.0) { e -= 1; p = gss_pow2(e); }
    /* an exact round-half-even tie depends on the parity of the result: not translatable */
    double half_ulp = gss_pow2(e - 53);
    if ((aerr == half_ulp || aerr == -half_ulp) && 4.0 * half_ulp > dunit) {
        *dlo = 0.0;
        *dhi = 0.0;
        return;
    }
    double below = (ar - p) + aerr;                    /* |t| - 2^e  >= 0 */
    double above = (2.0 * p - ar) - aerr;              /* 2^(e+1) - |t| > 0 */
    /* translating v by δ moves t by δ; in |t| terms the sign flips for negative t */
    double lo = r < 0.0 ? -above : -below, hi = r < 0.0 ? below : above;
    if (lo > *dlo) *dlo = lo;
    if (hi < *dhi) *dhi = hi;
}

/* A conservative gss_margin_step for the steps inside a carrier jump (W = 1: v and fl(v + s) in
   the same binade [2^e, 2^(e+1)), e <= -1).  The exact sum t = v + s lies within half an ulp of
   r = fl(v + s), so the distances of r to the binade's ends less one ulp bound t's from inside;
   no tie rule is needed there (a translation by 2^-52 is an even multiple of the lattice
   2^(e-52), so round-half-even sees the same parity).  Narrower than the exact interval by at
   most two ulps. */
GSS_HD void gss_margin_step_carr(double v, double s, double *dlo, double *dhi)
{
    const double r = v + s;
    const int e = gss_exp2i(r);
    const double p = gss_pow2(e), ulp = gss_pow2(e - 52);
    const double lo = ulp - (r - p);                   /* -(t - 2^e), rounded outward */
    const double hi = (2.0 * p - r) - ulp;             /* 2^(e+1) - t, rounded inward */
    if (lo > *dlo) *dlo = lo;
    if (hi < *dhi) *dhi = hi;
}

/* Walk ascending (s > 0) from w until the first wrap at threshold W (carrier W=1, code 1023)
   or n steps.  Returns steps taken; *x = value reached (post-wrap if *wrapped).  If margins is
   non-NULL, accumulates the admissible translation interval [*dlo, *dhi] of w. */
GSS_HD int64_t gss_asc_to_wrap(double *x, double s, double W, int64_t n, int *wrapped,
                               double *dlo, double *dhi)
{
    double v = *x;
    int64_t taken = 0;
    const double dunit = gss_pow2(gss_exp2i(W) - 52);      /* lattice of post-wrap values */
    *wrapped = 0;
    while (taken < n) {
        double D;
        int64_t J = gss_jump(v, s, W, &D);
        if (J > 0) {
            if (J == INT64_MAX) { if (dlo) { *dlo = 0.0; *dhi = 0.0; } taken = n; break; }
            if (J > n - taken) J = n - taken;
            if (dlo && W == 1.0) {                       /* carrier: the cheap bound */
                gss_margin_step_carr(v, s, dlo, dhi);
                gss_margin_step_carr(v + (double)(J - 1) * D, s, dlo, dhi);
                double top = v + (double)J * D;
                double lim = (W - top) - 2.0 * gss_pow2(gss_exp2i(W) - 52);
                if (lim < *dhi) *dhi = lim;
            } else if (dlo) {
                gss_margin_step(v, s, dunit, dlo, dhi);
                double vl = v + (double)(J - 1) * D;
                gss_margin_step(vl, s, dunit, dlo, dhi);
                double top = v + (double)J * D;         /* largest non-wrap result: r + δ < W */
                double lim = (W - top) - 2.0 * gss_pow2(gss_exp2i(W) - 52);
                if (lim < *dhi) *dhi = lim;
            }
            v = v + (double)J * D;
            taken += J;
            if (taken == n) break;
        }
        double r = v + s;
        if (dlo) {                /* the carrier's non-wrapping steps take the cheap bound too:
                                     a binade crossing below 1 rounds to a lattice that 2^-52
                                     still divides evenly; the wrap step keeps the exact rule */
            if (W == 1.0 && r < 1.0)
                gss_margin_step_carr(v, s, dlo, dhi);
            else
                gss_margin_step(v, s, dunit, dlo, dhi);
        }
        taken++;
        if (r >= W) {                                    /* wrap step: r + δ >= W */
            if (dlo) {
                double lim = W - r;
                if (lim > *dlo) *dlo = lim;
            }
            v = r - W;
            *wrapped = 1;
            break;
        }
        if (dlo) {
            double lim = (W - r) - 2.0 * gss_pow2(gss_exp2i(W) - 52);
            if (lim < *dhi) *dhi = lim;
        }
        v = r;
    }
    *x = v;
    return taken;
}

/* Descending carrier (s < 0), head of a cycle: from w walk down until the first value below T
   (T = 2^(e_s+2) > 2|s|, so no wrap can happen in the head) or n steps; margins as above.
   Returns steps taken; *stopped = 1 if a value < T was reached. */
GSS_HD int64_t gss_desc_head(double *x, double s, double T, int64_t n, int *stopped,
                             double *dlo, double *dhi)
{
    double v = *x;
    int64_t taken = 0;
    *stopped = 0;
    while (taken < n) {
        if (v < T) { *stopped = 1; break; }
        double D;
        int64_t J = gss_jump(v, s, 1.0, &D);
        if (J > 0) {
            if (J == INT64_MAX) { if (dlo) { *dlo = 0.0; *dhi = 0.0; } taken = n; break; }
            if (J > n - taken) J = n - taken;
            if (dlo) {
                gss_margin_step(v, s, gss_pow2(-53), dlo, dhi);
                gss_margin_step(v + (double)(J - 1) * D, s, gss_pow2(-53), dlo, dhi);
            }
            v = v + (double)J * D;                  /* stays >= 2^e >= T */
            taken += J;
            if (taken == n) break;
            continue;
        }
        if (dlo) gss_margin_step(v, s, gss_pow2(-53), dlo, dhi);
        v = v + s;                                  /* v >= T > 2|s|: no wrap */
        taken++;
    }
    if (taken == n && v < T) *stopped = 1;
    *x = v;
    return taken;
}

#define GSS_BIG 1.0e300

/* The orbit of cycle starts visits the entries in a nearly fixed order (the cycle map is a
   translation per entry), so the successor of the previous cycle's entry is tried first. */
GSS_HD const gss_cyc *gss_cc_find(gss_cyc_cache *cc, double w, int64_t nmax)
{
    const int p = cc->last >= 0 ? cc->e[cc->last].succ : -1;
    int hit = -1;
    if (p >= 0 && w >= cc->e[p].lo && w <= cc->e[p].hi && cc->e[p].L <= nmax) {
        hit = p;
    } else {
        for (int i = 0; i < cc->n; i++)
            if (w >= cc->e[i].lo && w <= cc->e[i].hi && cc->e[i].L <= nmax) {
                hit = i;
                break;
            }
    }
    if (hit >= 0 && cc->last >= 0)
        cc->e[cc->last].succ = hit;
    cc->last = hit;
    return hit >= 0 ? &cc->e[hit] : 0;
}

GSS_HD void gss_cc_put(gss_cyc_cache *cc, double w, double dlo, double dhi, double safe,
                       double v_end, int64_t L)
{
    if (!(dlo <= 0.0 && dhi >= 0.0)) return;
    const int i = cc->next;
    gss_cyc *e = &cc->e[i];
    e->lo = w + dlo + safe;
    e->hi = w + dhi - safe;
    if (e->lo > w) e->lo = w;                  /* the walked start itself is always valid */
    if (e->hi < w) e->hi = w;
    e->w0 = w;
    e->v0 = v_end;
    e->L = L;
    e->succ = -1;
    if (cc->last >= 0 && cc->last != i)
        cc->e[cc->last].succ = i;
    cc->last = i;
    cc->next = (cc->next + 1) % GSS_CC_N;
    if (cc->n < GSS_CC_N) cc->n++;
}

/* The entry the last cycle used, copied out of the cache (on the GPU the cache lives in scratch,
   a probe is two or three dependent loads): a code walk's cycles take the same entry as the
   cycle before 85 % of the time, so the walks test this copy first (any entry that holds the
   start gives the exact end, so which one a walk takes changes nothing but its speed). */
typedef struct gss_cyc_mru {
    double lo, hi, w0, v0;
    int64_t L;             /* 0: none */
} gss_cyc_mru;

GSS_HD void gss_mru_set(gss_cyc_mru *m, const gss_cyc *e)
{
    m->lo = e->lo;
    m->hi = e->hi;
    m->w0 = e->w0;
    m->v0 = e->v0;
    m->L = e->L;
}

/* the cycle from w by the copy, if it holds w (1) */
GSS_HD int gss_mru_take(const gss_cyc_mru *m, double *w, int64_t nmax, int64_t *L)
{
    if (m->L > 0 && *w >= m->lo && *w <= m->hi && m->L <= nmax) {
        *w = m->v0 + (*w - m->w0);
        *L = m->L;
        return 1;
    }
    return 0;
}

/* ---- carrier iterator: exact, cycle by cycle ---------------------------------------------- */
typedef struct gss_carr_it {
    double x, s, T;
    int64_t pos, left;     /* samples done / remaining */
    int mid;               /* x is not a post-wrap value (block start) */
    gss_cyc_mru mru;
    gss_cyc_cache cc;
} gss_carr_it;

GSS_HD void gss_carr_it_init(gss_carr_it *it, double x, double s, int64_t n)
{
    it->x = x;
    it->s = s;
    it->pos = 0;
    it->left = n;
    it->mid = 1;
    it->cc.n = 0;
    it->cc.next = 0;
    it->cc.last = -1;
    it->cc.enabled = (s != 0.0);
    it->mru.L = 0;
    double as = s < 0.0 ? -s : s;
    it->T = as > 0.0 ? gss_pow2(gss_exp2i(as) + 2) : 0.0;
}

/* Plain (uncached) walk to the next wrap. */
GSS_HD int gss_carr_plain_to_wrap(gss_carr_it *it)
{
    int wr = 0;
    int64_t taken;
    if (it->s > 0.0) {
        taken = gss_asc_to_wrap(&it->x, it->s, 1.0, it->left, &wr, 0, 0);
    } else {
        double v = it->x;
        taken = 0;
        while (taken < it->left) {
            double D;
            int64_t J = gss_jump(v, it->s, 1.0, &D);
            if (J > 0) {
                if (J == INT64_MAX) { taken = it->left; break; }
                if (J > it->left - taken) J = it->left - taken;
                v = v + (double)J * D;
                taken += J;
                if (taken == it->left) break;
            }
            double r = v + it->s;
            taken++;
            if (r >= 1.0) { v = r - 1.0; wr = 1; break; }     /* reference order: >=1 first */
            if (r < 0.0) { v = r + 1.0; wr = 1; break; }
            v = r;
        }
        it->x = v;
    }
    it->pos += taken;
    it->left -= taken;
    return wr;
}

/* Advance to just after the next wrap (returns 1, x = post-wrap value, pos = its sample index)
   or to the end of the range (returns 0, x = final value). */
GSS_HD int gss_carr_next_wrap(gss_carr_it *it)
{
    if (it->left <= 0) return 0;
    if (it->mid || !it->cc.enabled) {
        it->mid = 0;
        return gss_carr_plain_to_wrap(it);
    }
    const double safe = 4.0 * gss_pow2(-52);
    int64_t L = 0;
    if (it->s > 0.0) {
        if (gss_mru_take(&it->mru, &it->x, it->left, &L)) {
            it->pos += L;
            it->left -= L;
            return 1;
        }
        const gss_cyc *e = gss_cc_find(&it->cc, it->x, it->left);
        if (e) {
            gss_mru_set(&it->mru, e);
            it->x = e->v0 + (it->x - e->w0);
            it->pos += e->L;
            it->left -= e->L;
            return 1;
        }
        double w = it->x, dlo = -GSS_BIG, dhi = GSS_BIG;
        int wr = 0;
        int64_t taken = gss_asc_to_wrap(&it->x, it->s, 1.0, it->left, &wr, &dlo, &dhi);
        it->pos += taken;
        it->left -= taken;
        if (wr && dlo <= 0.0 && dhi >= 0.0) {
            gss_cc_put(&it->cc, w, dlo, dhi, safe, it->x, taken);
            gss_mru_set(&it->mru, &it->cc.e[it->cc.last]);
        }
        return wr;
    }
    /* descending: cached head down to T, then real steps to the wrap */
    if (gss_mru_take(&it->mru, &it->x, it->left, &L)) {
        it->pos += L;
        it->left -= L;
    } else {
        const gss_cyc *e = gss_cc_find(&it->cc, it->x, it->left);
        if (e) {
            gss_mru_set(&it->mru, e);
            it->x = e->v0 + (it->x - e->w0);
            it->pos += e->L;
            it->left -= e->L;
        } else {
            double w = it->x, dlo = -GSS_BIG, dhi = GSS_BIG;
            int st = 0;
            int64_t taken = gss_desc_head(&it->x, it->s, it->T, it->left, &st, &dlo, &dhi);
            it->pos += taken;
            it->left -= taken;
            if (!st) return 0;
            if (dlo <= 0.0 && dhi >= 0.0) {
                gss_cc_put(&it->cc, w, dlo, dhi, safe, it->x, taken);
                gss_mru_set(&it->mru, &it->cc.e[it->cc.last]);
            }
        }
    }
    while (it->left > 0) {
        double r = it->x + it->s;
        it->pos++;
        it->left--;
        if (r < 0.0) { it->x = r + 1.0; return 1; }
        it->x = r;
    }
    return 0;
}

/* Exact advance of the carrier by n samples using the cycle cache. */
GSS_HD double gss_carr_walk_cc(double x, double s, int64_t n)
{
    gss_carr_it it;
    gss_carr_it_init(&it, x, s, n);
    while (gss_carr_next_wrap(&it)) {
    }
    return it.x;
}

/* ---- speculative block walk: the planner's carrier chain off the serial path -------------------
 * The chain (gpssim.c:2245-2250, carried across blocks) is serial: a block's start is the previous
 * block's exact end.  But every cycle after a wrap starts on the post-wrap lattice (2^-52
 * ascending, 2^-53 descending), and a walk from there is a translation of the walk from a nearby
 * lattice point, exactly, inside an interval the margins give (the cycle cache's argument,
 * applied to whole stretches of cycles).  So a block's walk can run ahead of the chain, in
 * parallel over blocks and over GSS_SPEC_K segments of each block (on the GPU: gss_run), from
 * guesses: the start from the slot's line (accurate to ~1e-12 per block), and the segment starts
 * at wraps the line predicts (position P[j] and post-wrap value W[j], gss_carr_chain_guess):
 *   gss_spec_seg_walk  segment 0: the guess g -> its first wrap (p1, w1) exactly, then on to P[1]
 *                      with margins; segment j: from W[j] at P[j] to P[j+1] (the block end for the
 *                      last) with margins: end(start + d) = end + d for every lattice multiple d
 *                      in [dlo, dhi], and whether the segment ended on a wrap
 *   gss_spec_fix       the true start x -> its first wrap exactly (one partial cycle); if that wrap
 *                      is at p1, d = w1(x) - w1 is carried through the segments while it stays in
 *                      their intervals; where a check fails (or with no wrap in the block) the
 *                      cycle-cached walk goes on from the last exact value.
 * Exact in every case; tests/test_phase_walk.py and test_host_plane.py check against brute force
 * and the serial chain. */
#ifndef GSS_SPEC_T_DEFINED             /* = include/gpssim_amd.h */
#define GSS_SPEC_T_DEFINED
#ifndef GSS_SPEC_K
#define GSS_SPEC_K 32                   /* segments per block (8 before round 6: the GPU walks
                                          then took 1.19 ms per headline window, 0.88 with 16;
                                          with the row-shared cycle cache 0.65 with 16, 0.55
                                          with 32, 0.61 with 64: profiles/round6/spec_k/s6z) */
#endif
typedef struct gss_spec_in {           /* a row's guesses (host, gss_carr_chain_guess)          */
    double g, s;                       /* start guess, carr_step (0: padding row)               */
    int32_t k, pad;                    /* segments (1..GSS_SPEC_K)                              */
    int64_t P[GSS_SPEC_K];             /* segment j >= 1 starts at sample P[j], a predicted wrap */
    double W[GSS_SPEC_K];              /* ... with post-wrap value W[j]                         */
} gss_spec_in_t;                       /* 24 + 16 GSS_SPEC_K bytes */
typedef struct gss_spec_seg {
    double end, dlo, dhi;              /* end value, admissible translations of the start       */
    int64_t wrap_end;                  /* 1: the segment's last step wrapped                    */
} gss_spec_seg_t;
typedef struct gss_spec {              /* a row's speculative walk (GPU or host)                */
    int64_t p1;                        /* samples to the guess's first wrap (n: none)           */
    double w1;                         /* its post-wrap value                                   */
    gss_spec_seg_t seg[GSS_SPEC_K];
} gss_spec_t;                          /* 16 + 32 GSS_SPEC_K bytes */
#endif

/* Exactly to the first wrap or n steps (the reference's order: ">= 1" before "< 0"). */
GSS_HD int64_t gss_carr_to_wrap(double *x, double s, int64_t n, int *wr)
{
    if (s > 0.0)
        return gss_asc_to_wrap(x, s, 1.0, n, wr, 0, 0);
    double v = *x;
    int64_t taken = 0;
    *wr = 0;
    while (taken < n) {
        double D;
        int64_t J = gss_jump(v, s, 1.0, &D);
        if (J > 0) {
            if (J == INT64_MAX) { taken = n; break; }
            if (J > n - taken) J = n - taken;
            v = v + (double)J * D;
            taken += J;
            if (taken == n) break;
        }
        const double r = v + s;
        taken++;
        if (r >= 1.0) { v = r - 1.0; *wr = 1; break; }
        if (r < 0.0) { v = r + 1.0; *wr = 1; break; }
        v = r;
    }
    *x = v;
    return taken;
}

/* From a post-wrap value, n steps recording the admissible translations of the start; *wrap_end
   = the last step wrapped.  Ascending: gss_asc_to_wrap's margins.  Descending: the head down to T
   by gss_desc_head, then every real step below T, the wrap add and the wrap decisions with their
   own margins. */
GSS_HD double gss_walk_margins(double x, double s, int64_t n, double *dlo, double *dhi,
                               int *wrap_end)
{
    int64_t left = n;
    int last = 0;
    if (s > 0.0) {
        while (left > 0) {
            int wr = 0;
            left -= gss_asc_to_wrap(&x, s, 1.0, left, &wr, dlo, dhi);
            last = wr;
        }
        *wrap_end = last;
        return x;
    }
    const double T = gss_pow2(gss_exp2i(-s) + 2);
    const double dunit = gss_pow2(-53);
    while (left > 0) {
        int st = 0;
        last = 0;
        left -= gss_desc_head(&x, s, T, left, &st, dlo, dhi);
        if (!st || left <= 0)
            break;
        while (left > 0) {                      /* below T: real steps to the wrap */
            gss_margin_step(x, s, dunit, dlo, dhi);
            const double r = x + s;
            left--;
            if (r < 0.0) {                      /* r + d < 0 as well, and the rounded r + 1 */
                const double lim = -r - 2.0 * dunit;
                if (lim < *dhi) *dhi = lim;
                gss_margin_step(r, 1.0, dunit, dlo, dhi);
                x = r + 1.0;
                last = 1;
                break;
            }
            if (-r > *dlo) *dlo = -r;           /* r + d >= 0: no wrap under translation */
            x = r;
        }
    }
    *wrap_end = last;
    return x;
}

/* gss_walk_margins over whole cycles from the cycle cache (GSS_SPEC_CC: the speculative walks'
   default).  A cycle whose start w lies in a cached entry's interval [lo, hi] (its own margins,
   shrunk by `safe`, gss_cc_put) is a translation of the cached walk: end = v0 + (w - w0), and
   every start translation d keeping w + d in [lo, hi] keeps it one, so the segment's interval
   narrows to [lo - w, hi - w] (a subset of what the steps' own margins allow: conservative,
   so the chain's fix-up stays exact).  A miss walks the cycle with margins and caches it.
   Descending: the head down to T is cached the same way; the few real steps below T keep their
   per-step margins.  Cuts a segment's walk from ~13 binade jumps per carrier cycle to one cache
   probe for most cycles: 2.3x faster on one host core, but 12 % SLOWER on the GPU (gss_spec_kernel
   1.36-1.42 against 1.21-1.23 ms per headline window, profiles/round6/spec_cache/): each lane
   misses its cold cache at its own cycles, so nearly every cycle some lane of the wave walks it
   in full while the others wait, and the probes go through scratch.  Off by default (the host
   walk, gss_spec_host); -DGSS_SPEC_CC=1 builds it (test_phase_walk.py checks it).  The GPU walks
   instead share one cache per row in LDS and walk their misses in rounds (gss_producers.hip,
   sc_seg_walk). */
#ifndef GSS_SPEC_CC
#define GSS_SPEC_CC 0
#endif
GSS_HD double gss_walk_margins_cc(double x, double s, int64_t n, double *dlo, double *dhi,
                                  int *wrap_end, gss_cyc_cache *cc)
{
    int64_t left = n;
    int last = 0;
    const double safe = 4.0 * gss_pow2(-52);
    cc->n = 0;
    cc->next = 0;
    cc->last = -1;
    cc->enabled = 1;
    if (s > 0.0) {
        while (left > 0) {
            const double w = x;
            const gss_cyc *e = gss_cc_find(cc, w, left);
            if (e) {
                const double lo = e->lo - w, hi = e->hi - w;
                if (lo > *dlo) *dlo = lo;
                if (hi < *dhi) *dhi = hi;
                x = e->v0 + (w - e->w0);
                left -= e->L;
                last = 1;
                continue;
            }
            double clo = -GSS_BIG, chi = GSS_BIG;
            int wr = 0;
            const int64_t taken = gss_asc_to_wrap(&x, s, 1.0, left, &wr, &clo, &chi);
            left -= taken;
            last = wr;
            if (clo > *dlo) *dlo = clo;
            if (chi < *dhi) *dhi = chi;
            if (wr) gss_cc_put(cc, w, clo, chi, safe, x, taken);
        }
        *wrap_end = last;
        return x;
    }
    const double T = gss_pow2(gss_exp2i(-s) + 2);
    const double dunit = gss_pow2(-53);
    while (left > 0) {
        last = 0;
        const double w = x;
        const gss_cyc *e = gss_cc_find(cc, w, left);
        if (e) {
            const double lo = e->lo - w, hi = e->hi - w;
            if (lo > *dlo) *dlo = lo;
            if (hi < *dhi) *dhi = hi;
            x = e->v0 + (w - e->w0);
            left -= e->L;
        } else {
            double clo = -GSS_BIG, chi = GSS_BIG;
            int st = 0;
            const int64_t taken = gss_desc_head(&x, s, T, left, &st, &clo, &chi);
            left -= taken;
            if (clo > *dlo) *dlo = clo;
            if (chi < *dhi) *dhi = chi;
            if (!st || left <= 0)
                break;
            gss_cc_put(cc, w, clo, chi, safe, x, taken);
        }
        while (left > 0) {                      /* below T: real steps to the wrap */
            gss_margin_step(x, s, dunit, dlo, dhi);
            const double r = x + s;
            left--;
            if (r < 0.0) {                      /* r + d < 0 as well, and the rounded r + 1 */
                const double lim = -r - 2.0 * dunit;
                if (lim < *dhi) *dhi = lim;
                gss_margin_step(r, 1.0, dunit, dlo, dhi);
                x = r + 1.0;
                last = 1;
                break;
            }
            if (-r > *dlo) *dlo = -r;           /* r + d >= 0: no wrap under translation */
            x = r;
        }
    }
    *wrap_end = last;
    return x;
}

/* The line of a slot predicts where a block's walk wraps: ascending, wrap q at step
   ceil((q - g)/s) with post-wrap value g + p s - q; descending, wrap q at step
   floor((g + q - 1)/|s|) + 1 with value g + p s + q.  Segment starts: GSS_SPEC_K - 1 wraps spread
   over the block's wraps after its first (gss_carr_chain_guess on the host, or the walkers
   themselves for rows left with k = 0).  Doubles suffice (errors ~1e-13 against translation
   intervals ~1e-8; guesses only: any mismatch is caught by the fix-up). */
/* the wraps m in the block the line predicts and the guesses kk to make (0: none, k = 1) */
GSS_HD int64_t gss_spec_guess_kk(double g0, double s, int64_t n, int64_t *m)
{
    if (s == 0.0)
        return 0;
    const double e = g0 + (double)n * s;                 /* the line at the block end */
    const double mw = s > 0.0 ? floor(e) : floor(1.0 - e);   /* wraps in the block */
    if (!(mw >= 2.0))
        return 0;
    *m = mw > 1e9 ? (int64_t)1e9 : (int64_t)mw;
    return *m < GSS_SPEC_K ? *m : GSS_SPEC_K;
}

/* guess j (1 <= j < kk): the predicted wrap's position *p and post-wrap value *w; 0 if the value
   is off the unit interval (the guesses end before it).  The caller also ends them where p is
   not past the guess before it or not inside the block. */
GSS_HD int gss_spec_guess_one(double g0, double s, int64_t m, int64_t kk, int64_t j, int64_t *p,
                              double *w)
{
    const double as = s > 0.0 ? s : -s;
    const double unit = s > 0.0 ? 0x1p-52 : 0x1p-53;
    const int64_t q = 1 + (j * (m - 1) + kk - 1) / kk;          /* wrap index, >= 2 */
    *p = s > 0.0 ? (int64_t)ceil(((double)q - g0) / as)
                 : (int64_t)floor((g0 + (double)q - 1.0) / as) + 1;
    const double v = (g0 + (double)*p * s) + (s > 0.0 ? -(double)q : (double)q);
    *w = rint(v / unit) * unit;
    return *w >= 0.0 && *w < 1.0;
}

GSS_HD void gss_spec_guess_row(double g, double s, int64_t n, gss_spec_in_t *in)
{
    const double g0 = g;
    in->g = g0;
    in->s = s;
    in->k = 1;
    /* in->pad: the caller's (the previous row of the slot, gss_carr_chain_starts) */
    int64_t m = 0;
    const int64_t kk = gss_spec_guess_kk(g0, s, n, &m);
    int k = 1;
    int64_t prev = 0;
    for (int64_t j = 1; j < kk; j++) {
        int64_t p;
        double w;
        const int ok = gss_spec_guess_one(g0, s, m, kk, j, &p, &w);
        if (p <= prev || p >= n || !ok)
            break;
        in->P[k] = p;
        in->W[k] = w;
        prev = p;
        k++;
    }
    in->k = k;
}

/* Segment j of a row's walk (n samples per block). */
GSS_HD void gss_spec_seg_walk(const gss_spec_in_t *in, int j, int64_t n, gss_spec_t *o)
{
    const double s = in->s;
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    gss_spec_seg_t *sg = &o->seg[j];
    const int64_t stop = j + 1 < k ? in->P[j + 1] : n;
    double x;
    int64_t pos;
    sg->dlo = 1.0;                              /* an empty interval until walked */
    sg->dhi = 0.0;
    sg->wrap_end = 0;
    if (j == 0) {
        x = in->g;
        int wr = 0;
        const int64_t t = s != 0.0 ? gss_carr_to_wrap(&x, s, stop, &wr) : stop;
        o->p1 = wr ? t : n;
        o->w1 = x;
        sg->end = x;
        if (!wr || t >= stop)
            return;                             /* no wrap before the segment's end */
        pos = t;
    } else {
        x = in->W[j];
        pos = in->P[j];
        sg->end = x;
        if (s == 0.0 || pos >= stop)
            return;
    }
    double dlo = -GSS_BIG, dhi = GSS_BIG;
    int we = 0;
#if GSS_SPEC_CC
    gss_cyc_cache cc;
    x = gss_walk_margins_cc(x, s, stop - pos, &dlo, &dhi, &we, &cc);
#else
    x = gss_walk_margins(x, s, stop - pos, &dlo, &dhi, &we);
#endif
    sg->end = x;
    sg->dlo = dlo;
    sg->dhi = dhi;
    sg->wrap_end = we;
}

/* The exact walk from v at sample pos to the block end, through the segment starts P[j] (j >= j0)
   past pos: with av != NULL, av[j] = the exact value at P[j] (the chain's anchors). */
GSS_HD double gss_spec_walk_rest(double v, int64_t pos, int64_t n, const gss_spec_in_t *in, int k,
                                 int j0, double *av)
{
    const double s = in->s;
    if (av) {
        for (int j = j0 < 1 ? 1 : j0; j < k; j++) {
            if (in->P[j] <= pos)
                continue;
            v = gss_carr_walk_cc(v, s, in->P[j] - pos);
            pos = in->P[j];
            av[j] = v;
        }
    }
    return gss_carr_walk_cc(v, s, n - pos);
}

/* From the row's exact post-wrap value v at its first wrap (pos = o->p1): the segments'
   translations while they hold, then the exact walk.  *hit = 1 where every segment translated;
   *dlast = the translation of the last segment (the row's end is its end + *dlast); av (NULL:
   none) gets the exact value at every segment start P[j], j >= 1 (gss_spec_walk_rest). */
GSS_HD double gss_spec_fix_at(double v, int64_t n, const gss_spec_in_t *in, const gss_spec_t *o,
                              int *hit, double *dlast, double *av)
{
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    int64_t pos = o->p1;
    double d = v - o->w1;                       /* exact: both on the post-wrap lattice */
    int j = 0;
    *hit = 0;
    for (; j < k; j++) {
        const gss_spec_seg_t *sg = &o->seg[j];
        if (!(d >= sg->dlo && d <= sg->dhi))
            break;                              /* v is still the exact value at pos */
        v = sg->end + d;
        pos = j + 1 < k ? in->P[j + 1] : n;
        if (j + 1 < k) {
            if (av)
                av[j + 1] = v;
            if (!sg->wrap_end) { j++; break; }   /* exact at pos, but not post-wrap */
            d = v - in->W[j + 1];
        }
    }
    if (j == k && pos == n) {
        *hit = 1;
        *dlast = d;
        return v;
    }
    return gss_spec_walk_rest(v, pos, n, in, k, j + 1, av);
}

/* The block's exact end from its true start x and the row's speculative walk: x to its first
   wrap exactly (one partial cycle), then gss_spec_fix_at where that wrap is the guess's. */
GSS_HD double gss_spec_fix_d(double x, int64_t n, const gss_spec_in_t *in, const gss_spec_t *o,
                             int *hit, double *dlast, double *av)
{
    const double s = in->s;
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    *hit = 0;
    double v = x;
    int wr = 0;
    const int64_t t = gss_carr_to_wrap(&v, s, n, &wr);
    if (!wr || t >= n) {                        /* no wrap: v is the end, walked exactly */
        if (av && s != 0.0) {                   /* (anchors: walked again, to each P[j]) */
            return gss_spec_walk_rest(x, 0, n, in, k, 1, av);
        }
        return v;
    }
    if (t == o->p1)
        return gss_spec_fix_at(v, n, in, o, hit, dlast, av);
    return gss_spec_walk_rest(v, t, n, in, k, 1, av);
}

/* A row's anchors from its exact start x and its walk: pos[0] = 0, val[0] = x, and at every
   segment start P[j] the fix-up passed or walked, the exact carrier there (pos -1: none). */
GSS_HD void gss_spec_anchors(double x, int64_t n, const gss_spec_in_t *in, const gss_spec_t *o,
                             int32_t *pos, double *val)
{
    double av[GSS_SPEC_K];
    for (int j = 0; j < GSS_SPEC_K; j++)
        av[j] = -1.0;                                /* a carrier value is never negative */
    int hit = 0;
    double d = 0.0;
    (void)gss_spec_fix_d(x, n, in, o, &hit, &d, av);
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    pos[0] = 0;
    val[0] = x;
    for (int j = 1; j < GSS_SPEC_K; j++) {
        const int ok = j < k && av[j] >= 0.0 && in->P[j] > 0 && in->P[j] < n;
        pos[j] = ok ? (int32_t)in->P[j] : -1;
        val[j] = ok ? av[j] : 0.0;
    }
}

GSS_HD double gss_spec_fix(double x, int64_t n, const gss_spec_in_t *in, const gss_spec_t *o,
                           int *hit)
{
    double d;
    return gss_spec_fix_d(x, n, in, o, hit, &d, 0);
}

/* gss_carr_to_wrap with the admissible translations [*dlo, *dhi] of the start (lattice 2^-52
   ascending, 2^-53 descending: the chain's translations), for a start anywhere in [0, 1): the
   link from a row's speculative end to the next row's first wrap (gss_spec_links). */
GSS_HD int64_t gss_carr_to_wrap_margins(double *x, double s, int64_t n, int *wr, double *dlo,
                                        double *dhi)
{
    *wr = 0;
    if (s > 0.0)
        return gss_asc_to_wrap(x, s, 1.0, n, wr, dlo, dhi);
    const double T = gss_pow2(gss_exp2i(-s) + 2);
    const double dunit = gss_pow2(-53);
    double v = *x;
    int st = 0;
    int64_t taken = gss_desc_head(&v, s, T, n, &st, dlo, dhi);
    while (st && taken < n) {                   /* below T: real steps to the wrap */
        gss_margin_step(v, s, dunit, dlo, dhi);
        const double r = v + s;
        taken++;
        if (r < 0.0) {
            const double lim = -r - 2.0 * dunit;
            if (lim < *dhi) *dhi = lim;
            gss_margin_step(r, 1.0, dunit, dlo, dhi);
            v = r + 1.0;
            *wr = 1;
            break;
        }
        if (-r > *dlo) *dlo = -r;
        v = r;
    }
    *x = v;
    return taken;
}

/* ---- a row's walk folded into one record (gss_spec_records*, gss_carr_chain_records) ----------
 * gss_spec_fix_at's checks, d_j in [dlo_j, dhi_j] with d_0 = d + c and d_j+1 = d_j + (end_j -
 * W_j+1), are one interval on d: [lo_j - c_j, hi_j - c_j] over j, rounded inward (the c_j are
 * sums of post-wrap lattice values, exact in double; so is every translation the chain then
 * forms).  0 where no translation can carry the row (an empty interval, or a segment that does
 * not end on a wrap before the last). */
#ifndef GSS_SPEC_REC_DEFINED
#define GSS_SPEC_REC_DEFINED
typedef struct gss_spec_rec {          /* a row's speculative walk folded (GPU or host)            */
    double w1;                         /* post-wrap value at the guess's first wrap                */
    double slo, shi, sdd;              /* self: d0 = (true post-wrap value at p1) - w1 in [slo,
                                          shi] -> the row's last translation is d0 + sdd ...     */
    double end;                        /* ... and its end is end + (d0 + sdd)                      */
    double llo, lhi, ldd;              /* link: the previous row of the slot translated by d in
                                          [llo, lhi] -> this one's last translation is d + ldd    */
    int32_t p1;                        /* samples to the guess's first wrap                        */
    int32_t ok;                        /* bit 0: self record, bit 1: link record                   */
} gss_spec_rec_t;                      /* 72 bytes */
#endif

GSS_HD int gss_spec_fold(const gss_spec_in_t *in, const gss_spec_t *o, double c, double lo,
                         double hi, double *olo, double *ohi, double *odd)
{
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    for (int j = 0; j < k; j++) {
        const gss_spec_seg_t *sg = &o->seg[j];
        if (!(sg->dlo <= sg->dhi))
            return 0;
        const double l = nextafter(sg->dlo - c, GSS_BIG), h = nextafter(sg->dhi - c, -GSS_BIG);
        if (l > lo) lo = l;
        if (h < hi) hi = h;
        if (j + 1 < k) {
            if (!sg->wrap_end)
                return 0;                        /* the walk goes on exactly: no record */
            c += sg->end - in->W[j + 1];
        }
    }
    if (!(lo <= hi))
        return 0;
    *olo = lo;
    *ohi = hi;
    *odd = c;
    return 1;
}

/* The link part: the row entered from y, the previous row's last segment end (that row
   translated by d starts this one at y + d): its partial cycle walked from y with margins. */
GSS_HD int gss_spec_link_fold(double y, const gss_spec_in_t *in, const gss_spec_t *o, int64_t n,
                              double *olo, double *ohi, double *odd)
{
    double a = -GSS_BIG, b = GSS_BIG;
    int wr = 0;
    double x = y;
    const int64_t t = gss_carr_to_wrap_margins(&x, in->s, n, &wr, &a, &b);
    if (!wr || t >= n || t != o->p1 || !(a <= b))
        return 0;
    return gss_spec_fold(in, o, x - o->w1, a, b, olo, ohi, odd);
}

/* Row e's record; prev (NULL: none) the previous row of its slot within the batch. */
GSS_HD void gss_spec_record(const gss_spec_in_t *in, const gss_spec_t *o,
                            const gss_spec_in_t *pin, const gss_spec_t *po, int64_t n,
                            gss_spec_rec_t *r)
{
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    r->w1 = o->w1;
    r->p1 = (int32_t)(o->p1 < n ? o->p1 : n);
    r->end = o->seg[k - 1].end;
    r->slo = 1.0; r->shi = 0.0; r->sdd = 0.0;
    r->llo = 1.0; r->lhi = 0.0; r->ldd = 0.0;
    r->ok = 0;
    if (in->s == 0.0 || o->p1 >= n)
        return;
    if (gss_spec_fold(in, o, 0.0, -GSS_BIG, GSS_BIG, &r->slo, &r->shi, &r->sdd))
        r->ok |= 1;
    if (pin && po && pin->s != 0.0) {
        const int kp = pin->k < 1 ? 1 : (pin->k > GSS_SPEC_K ? GSS_SPEC_K : pin->k);
        if (gss_spec_link_fold(po->seg[kp - 1].end, in, o, n, &r->llo, &r->lhi, &r->ldd))
            r->ok |= 2;
    }
}

/* ---- code iterator ---------------------------------------------------------------------- */
typedef struct gss_code_it {
    gss_code_state c;
    double cs;
    int64_t pos, left;
    int mid;
    gss_cyc_mru mru;
    gss_cyc_cache cc;
} gss_code_it;

GSS_HD void gss_code_it_init(gss_code_it *it, gss_code_state c, double cs, int64_t n)
{
    it->c = c;
    it->cs = cs;
    it->pos = 0;
    it->left = n;
    it->mid = 1;
    it->cc.n = 0;
    it->cc.next = 0;
    it->cc.last = -1;
    it->cc.enabled = (cs > 0.0);
    it->mru.L = 0;
}

GSS_HD void gss_code_count_wrap(gss_code_state *c)
{
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

GSS_HD int gss_code_next_wrap(gss_code_it *it)
{
    if (it->left <= 0) return 0;
    const double W = GSS_CA_SEQ_LEN_D;
    int wr = 0;
    if (it->mid || !it->cc.enabled) {
        it->mid = 0;
        int64_t taken = gss_asc_to_wrap(&it->c.ph, it->cs, W, it->left, &wr, 0, 0);
        it->pos += taken;
        it->left -= taken;
        if (wr) gss_code_count_wrap(&it->c);
        return wr;
    }
    int64_t L = 0;
    if (gss_mru_take(&it->mru, &it->c.ph, it->left, &L)) {
        it->pos += L;
        it->left -= L;
        gss_code_count_wrap(&it->c);
        return 1;
    }
    const gss_cyc *e = gss_cc_find(&it->cc, it->c.ph, it->left);
    if (e) {
        gss_mru_set(&it->mru, e);
        it->c.ph = e->v0 + (it->c.ph - e->w0);
        it->pos += e->L;
        it->left -= e->L;
        gss_code_count_wrap(&it->c);
        return 1;
    }
    double w = it->c.ph, dlo = -GSS_BIG, dhi = GSS_BIG;
    int64_t taken = gss_asc_to_wrap(&it->c.ph, it->cs, W, it->left, &wr, &dlo, &dhi);
    it->pos += taken;
    it->left -= taken;
    if (wr) {
        if (dlo <= 0.0 && dhi >= 0.0) {
            gss_cc_put(&it->cc, w, dlo, dhi, 4.0 * gss_pow2(-43), it->c.ph, taken);
            gss_mru_set(&it->mru, &it->cc.e[it->cc.last]);
        }
        gss_code_count_wrap(&it->c);
    }
    return wr;
}

GSS_HD void gss_code_walk_cc(gss_code_state *c, double cs, int64_t n)
{
    gss_code_it it;
    gss_code_it_init(&it, *c, cs, n);
    while (gss_code_next_wrap(&it)) {
    }
    *c = it.c;
}
/* Carrier checkpoints the host planner records while it walks a block (the walk it must do
 * anyway to get the next block's carr_phase): ck[j] = exact carrier at sample gss_ck_pos(j, n),
 * j < GSS_NCK (ck[0] = x).  The GPU then walks each block's carrier as GSS_NCK independent
 * sub-chains.  Cycle-cached wrap-by-wrap walk; each checkpoint is a plain walk of less than one
 * cycle from the last wrap before it.  Returns the value at n (the next block's carr0). */
#ifndef GSS_NCK
#define GSS_NCK 8                     /* = GSS_NCK in include/gpssim_amd.h */
#endif
GSS_HD int gss_ck_pos(int j, int n) { return (int)(((int64_t)j * n) / GSS_NCK); }

GSS_HD double gss_carr_walk_ck(double x, double s, int n, double *ck)
{
    gss_carr_it it;
    gss_carr_it_init(&it, x, s, n);
    int j = 1;
    ck[0] = x;
    int64_t last_pos = 0;
    double last_x = x;
    while (gss_carr_next_wrap(&it)) {
        for (; j < GSS_NCK && gss_ck_pos(j, n) < it.pos; j++)
            ck[j] = gss_carr_walk(last_x, s, gss_ck_pos(j, n) - last_pos);
        last_pos = it.pos;
        last_x = it.x;
    }
    for (; j < GSS_NCK; j++)
        ck[j] = gss_carr_walk(last_x, s, gss_ck_pos(j, n) - last_pos);
    return it.x;
}

#endif /* GSS_PHASE_H */
