/*
 * gnss_time.c — GPS week/second arithmetic.  Each function restates one reference routine and
 * keeps its exact double operation order (the rounded 1 ms grid of incGpsTime feeds every
 * block epoch, so a single different rounding shifts the whole run).
 */
#include <math.h>
#include "gss_host.h"

/* date2gps, gpssim.c:177-200.  Days since the GPS epoch (1980-01-06), then week/second split. */
void gt_from_date(const dtime_t *t, gtime_t *g)
{
    static const int cum_days[12] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334};
    int years = t->y - 1980;
    int leap = years / 4 + 1;
    if ((years % 4) == 0 && t->m <= 2)
        leap--;
    int days = years * 365 + cum_days[t->m - 1] + t->d + leap - 6;
    g->week = days / 7;
    g->sec = (double)(days % 7) * K_SEC_DAY + t->hh * K_SEC_HOUR + t->mm * K_SEC_MIN + t->sec;
}

/* gps2date, gpssim.c:202-219 (Julian-day based calendar conversion). */
void gt_to_date(const gtime_t *g, dtime_t *t)
{
    int jd = (int)(7 * g->week + floor(g->sec / 86400.0) + 2444245.0) + 1537;
    int yy = (int)((jd - 122.1) / 365.25);
    int dd = 365 * yy + yy / 4;
    int mo = (int)((jd - dd) / 30.6001);

    t->d = jd - dd - (int)(30.6001 * mo);
    t->m = mo - 1 - 12 * (mo / 14);
    t->y = yy - 4715 - ((7 + t->m) / 10);
    t->hh = ((int)(g->sec / 3600.0)) % 24;
    t->mm = ((int)(g->sec / 60.0)) % 60;
    t->sec = g->sec - 60.0 * floor(g->sec / 60.0);
}

/* subGpsTime, gpssim.c:779-787. */
double gt_diff(gtime_t g1, gtime_t g0)
{
    double dt = g1.sec - g0.sec;
    dt += (double)(g1.week - g0.week) * K_SEC_WEEK;
    return dt;
}

/* incGpsTime, gpssim.c:789-811: add, snap to the 1 ms grid, renormalise the week. */
gtime_t gt_add(gtime_t g0, double dt)
{
    gtime_t r;
    r.week = g0.week;
    r.sec = g0.sec + dt;
    r.sec = round(r.sec * 1000.0) / 1000.0;
    while (r.sec >= K_SEC_WEEK) {
        r.sec -= K_SEC_WEEK;
        r.week++;
    }
    while (r.sec < 0.0) {
        r.sec += K_SEC_WEEK;
        r.week--;
    }
    return r;
}
