/* Test-only harness: exposes the product's shared phase arithmetic (gss_phase.h) — both the
   plain binade walk used by Stage-B lanes and the cycle-cached walk used by Stage A and the host
   planner — so tests/test_phase_walk.py can check them against the brute-force oracle. */
#include "../../gps-sdr-sim_amd/csrc/common/gss_phase.h"

double wc_carr_plain(double x, double s, int64_t n) { return gss_carr_walk(x, s, n); }
double wc_carr_cached(double x, double s, int64_t n) { return gss_carr_walk_cc(x, s, n); }

double wc_code(int cached, double c, double s, int64_t n, int32_t *ic, int32_t *ib, int32_t *iw)
{
    gss_code_state st = {c, *ic, *ib, *iw};
    if (cached)
        gss_code_walk_cc(&st, s, n);
    else
        gss_code_walk(&st, s, n);
    *ic = st.icode;
    *ib = st.ibit;
    *iw = st.iword;
    return st.ph;
}

/* anchors exactly as Stage A emits them, for one chain: positions and values of the last wrap
   at or before every segment start */
int wc_carr_anchors(double x0, double s, int64_t n, int seg_r, int nseg, int32_t *an, double *ax)
{
    gss_carr_it it;
    gss_carr_it_init(&it, x0, s, n);
    int seg = 0;
    int32_t a = 0;
    double v = x0;
    for (;;) {
        int wr = gss_carr_next_wrap(&it);
        int64_t nw = wr ? it.pos : n;
        while (seg < nseg && (int64_t)seg * seg_r < nw) {
            an[seg] = a;
            ax[seg] = v;
            seg++;
        }
        if (!wr || seg >= nseg)
            break;
        a = (int32_t)it.pos;
        v = it.x;
    }
    return seg;
}

/* ---- f64-only forms used by the GPU kernels (gss_jumpf / gss_walkf / gss_to_wrapf) ---- */
double wc_carr_f(double x, double s, int64_t n, int32_t *nwrap)
{
    int w = 0;
    double r = gss_walkf(x, s, 1.0, (double)n, &w);
    *nwrap = w;
    return r;
}

/* code chain advanced wrap by wrap, exactly as the Stage-A code lanes do */
double wc_code_f(double c, double s, int64_t n, int32_t *ic, int32_t *ib, int32_t *iw)
{
    gss_code_state st = {c, *ic, *ib, *iw};
    double left = (double)n;
    while (left > 0.0 && gss_to_wrapf(&st.ph, s, GSS_CA_SEQ_LEN_D, &left))
        gss_code_count_wrap(&st);
    *ic = st.icode;
    *ib = st.ibit;
    *iw = st.iword;
    return st.ph;
}

/* Stage A (carrier chain) + Stage B lane start, f64 forms: for every segment start n0 = seg*R the
   exact carrier value, walked from the last wrap at or before n0.  Returns the number of Stage-B
   walks that (wrongly) crossed a wrap; 0 expected. */
int wc_carr_seg_starts_f(double x0, double s, int64_t n, int seg_r, int nseg, double *out)
{
    double left = (double)n, v = x0, ax = x0;
    int64_t an = 0, pos = 0;
    int seg = 0, bad = 0;
    for (;;) {
        double l0 = left;
        int wr = gss_to_wrapf(&v, s, 1.0, &left);
        pos += (int64_t)(l0 - left);
        int64_t nw = wr ? pos : n;
        while (seg < nseg && (int64_t)seg * seg_r < nw) {
            int w = 0;
            out[seg] = gss_walkf(ax, s, 1.0, (double)((int64_t)seg * seg_r - an), &w);
            bad += w;
            seg++;
        }
        if (!wr || seg >= nseg)
            break;
        an = pos;
        ax = v;
    }
    return bad;
}

/* ---- branch-free lane form (gss_iter_bf / gss_walk_bf): what the GPU lanes execute ---- */
double wc_carr_bf(double x, double s, int64_t n, int32_t *nwrap)
{
    int w = 0;
    double r = gss_walk_bf(x, s, 1.0, (double)n, &w);
    *nwrap = w;
    return r;
}

double wc_code_bf(double c, double s, int64_t n, int32_t *ic, int32_t *ib, int32_t *iw)
{
    gss_code_state st = {c, *ic, *ib, *iw};
    double left = (double)n, as = s < 0.0 ? -s : s, rs = 1.0 / as;
    if (s != 0.0)
        while (left > 0.0)
            if (gss_iter_bf(&st.ph, s, as, rs, GSS_CA_SEQ_LEN_D, gss_exw(GSS_CA_SEQ_LEN_D), &left))
                gss_code_count_wrap(&st);
    *ic = st.icode;
    *ib = st.ibit;
    *iw = st.iword;
    return st.ph;
}

/* Stage A (GPU form, gss_seg_states): exact phase (and code counters) at every segment start
   in [pos0, pos1) */
double wc_seg_states(double v, double s, int code, uint32_t cnt, int pos0, int pos1, int seg_r,
                     int nseg, int want_end, double *out_x, uint32_t *out_c)
{
    int kind = code ? GSS_TRIP_CODE : (s < 0.0 ? GSS_TRIP_CARR_DESC : GSS_TRIP_CARR_ASC);
    return gss_seg_states(kind, v, s, cnt, pos0, pos1, nseg, seg_r, want_end, out_x, out_c);
}

/* branch-free code chain (GPU Stage A code waves) */
void wc_code_seg_bf(double v, double s, uint32_t cnt, int n, int seg_r, int nseg, int dummy,
                    double *out_x, uint32_t *out_c)
{
    gss_code_seg_states_bf(v, s, cnt, n, nseg, seg_r, dummy, out_x, out_c);
}

/* host planner carrier checkpoints */
double wc_carr_walk_ck(double x, double s, int n, double *ck) { return gss_carr_walk_ck(x, s, n, ck); }
int wc_nck(void) { return GSS_NCK; }

/* carrier walk by specialised trips (both directions) */
double wc_carr_trip(double x, double s, int64_t n)
{
    int kind = s < 0.0 ? GSS_TRIP_CARR_DESC : GSS_TRIP_CARR_ASC;
    double left = (double)n, rs = 1.0 / (s < 0.0 ? -s : s), J, Ds;
    if (s == 0.0)
        return x;
    while (left > 0.0)
        gss_trip(kind, &x, s, rs, &left, &J, &Ds);
    return x;
}

/* the speculative segment walk's margins, plain (gss_walk_margins) or from the cycle cache
   (gss_walk_margins_cc, GSS_SPEC_CC builds): end value, admissible start translations, wrap */
double wc_margins(double x, double s, int64_t n, int use_cc, double *dlo, double *dhi, int *we)
{
    *dlo = -GSS_BIG;
    *dhi = GSS_BIG;
    if (use_cc) {
        gss_cyc_cache cc;
        return gss_walk_margins_cc(x, s, n, dlo, dhi, we, &cc);
    }
    return gss_walk_margins(x, s, n, dlo, dhi, we);
}
