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
