/*
 * gnss_orbit.c — broadcast-ephemeris orbit, Klobuchar ionosphere and pseudorange.
 * Restates satpos (gpssim.c:379-484), ionosphericDelay (1170-1245), computeRange (1253-1310)
 * and checkSatVisibility (1549-1570) with the reference's operation order.
 */
#include <math.h>
#include "gss_host.h"

/* Wrap a time difference into [-half week, +half week] (gpssim.c:410-413, 475-478). */
static double week_wrap(double tk)
{
    if (tk > K_SEC_HALF_WEEK)
        tk -= K_SEC_WEEK;
    else if (tk < -K_SEC_HALF_WEEK)
        tk += K_SEC_WEEK;
    return tk;
}

/* satpos: SV position/velocity (ECEF) and clock [s, s/s] at time g. */
void sv_state(const eph_t *e, gtime_t g, double *pos, double *vel, double *clk)
{
    double tk = week_wrap(g.sec - e->toe.sec);

    /* Kepler's equation by Newton iteration to 1e-14 */
    double mk = e->m0 + e->n * tk;
    double ek = mk, ek_prev = ek + 1.0;
    double one_m_ecos = 0.0;
    while (fabs(ek - ek_prev) > 1.0E-14) {
        ek_prev = ek;
        one_m_ecos = 1.0 - e->ecc * cos(ek_prev);
        ek = ek + (mk - ek_prev + e->ecc * sin(ek_prev)) / one_m_ecos;
    }
    double sek = sin(ek), cek = cos(ek);
    double ekdot = e->n / one_m_ecos;
    double rel = -4.442807633E-10 * e->ecc * e->sqrta * sek;

    /* argument of latitude, radius, inclination with second-harmonic corrections */
    double pk = atan2(e->sq1e2 * sek, cek - e->ecc) + e->aop;
    double pkdot = e->sq1e2 * ekdot / one_m_ecos;
    double s2pk = sin(2.0 * pk), c2pk = cos(2.0 * pk);

    double uk = pk + e->cus * s2pk + e->cuc * c2pk;
    double suk = sin(uk), cuk = cos(uk);
    double ukdot = pkdot * (1.0 + 2.0 * (e->cus * c2pk - e->cuc * s2pk));

    double rk = e->A * one_m_ecos + e->crc * c2pk + e->crs * s2pk;
    double rkdot = e->A * e->ecc * sek * ekdot + 2.0 * pkdot * (e->crs * c2pk - e->crc * s2pk);

    double ik = e->inc0 + e->idot * tk + e->cic * c2pk + e->cis * s2pk;
    double sik = sin(ik), cik = cos(ik);
    double ikdot = e->idot + 2.0 * pkdot * (e->cis * c2pk - e->cic * s2pk);

    /* position in the orbital plane, then rotate by the corrected node longitude */
    double xp = rk * cuk, yp = rk * suk;
    double xpdot = rkdot * cuk - yp * ukdot;
    double ypdot = rkdot * suk + xp * ukdot;

    double ok = e->omg0 + tk * e->omgkdot - K_OMEGA_E * e->toe.sec;
    double sok = sin(ok), cok = cos(ok);

    pos[0] = xp * cok - yp * cik * sok;
    pos[1] = xp * sok + yp * cik * cok;
    pos[2] = yp * sik;

    double tmp = ypdot * cik - yp * sik * ikdot;
    vel[0] = -e->omgkdot * pos[1] + xpdot * cok - tmp * sok;
    vel[1] = e->omgkdot * pos[0] + xpdot * sok + tmp * cok;
    vel[2] = yp * cik * ikdot + ypdot * sik;

    /* clock polynomial + relativistic term - group delay */
    tk = week_wrap(g.sec - e->toc.sec);
    clk[0] = e->af0 + tk * (e->af1 + tk * e->af2) + rel - e->tgd;
    clk[1] = e->af1 + 2.0 * tk * e->af2;
}

/* ionosphericDelay: Klobuchar model in semi-circles [m]. */
double iono_delay(const iono_t *io, gtime_t g, const double *llh, const double *azel)
{
    if (io->enable == 0)
        return 0.0;

    double E = azel[1] / K_PI;
    double phi_u = llh[0] / K_PI;
    double lam_u = llh[1] / K_PI;
    double F = 1.0 + 16.0 * pow((0.53 - E), 3.0);          /* obliquity */

    if (io->vflg == 0)
        return F * 5.0e-9 * K_C;

    double psi = 0.0137 / (E + 0.11) - 0.022;
    double phi_i = phi_u + psi * cos(azel[0]);
    if (phi_i > 0.416)
        phi_i = 0.416;
    else if (phi_i < -0.416)
        phi_i = -0.416;
    double lam_i = lam_u + psi * sin(azel[0]) / cos(phi_i * K_PI);
    double phi_m = phi_i + 0.064 * cos((lam_i - 1.617) * K_PI);
    double phi_m2 = phi_m * phi_m;
    double phi_m3 = phi_m2 * phi_m;

    double amp = io->alpha0 + io->alpha1 * phi_m + io->alpha2 * phi_m2 + io->alpha3 * phi_m3;
    if (amp < 0.0)
        amp = 0.0;
    double per = io->beta0 + io->beta1 * phi_m + io->beta2 * phi_m2 + io->beta3 * phi_m3;
    if (per < 72000.0)
        per = 72000.0;

    double t = K_SEC_DAY / 2.0 * lam_i + g.sec;            /* local time */
    while (t >= K_SEC_DAY)
        t -= K_SEC_DAY;
    while (t < 0)
        t += K_SEC_DAY;

    double X = 2.0 * K_PI * (t - 50400.0) / per;
    if (fabs(X) < 1.57) {
        double X2 = X * X, X4 = X2 * X2;
        return F * (5.0e-9 + amp * (1.0 - X2 / 2.0 + X4 / 24.0)) * K_C;
    }
    return F * 5.0e-9 * K_C;
}

/* computeRange: light-time + Sagnac corrected pseudorange, rate, az/el and iono delay.  llh and
   tmat are the receiver's geodetic position and local frame (ecef_to_llh, enu_matrix of xyz): the
   reference recomputes them per call (gpssim.c:1277-1279); they depend on xyz alone, so callers
   with many satellites per receiver position pass them in (sv_range_at). */
void sv_range_at(rng_t *rho, const eph_t *e, const iono_t *io, gtime_t g, const double *xyz,
                 const double *llh, double tmat[3][3])
{
    double pos[3], vel[3], clk[2], los[3], neu[3];

    sv_state(e, g, pos, vel, clk);
    for (int i = 0; i < 3; i++)
        los[i] = pos[i] - xyz[i];
    double tau = vnorm3(los) / K_C;

    for (int i = 0; i < 3; i++)                 /* back-propagate to transmission time */
        pos[i] -= vel[i] * tau;
    double xr = pos[0] + pos[1] * K_OMEGA_E * tau;   /* earth rotation during flight */
    double yr = pos[1] - pos[0] * K_OMEGA_E * tau;
    pos[0] = xr;
    pos[1] = yr;

    for (int i = 0; i < 3; i++)
        los[i] = pos[i] - xyz[i];
    double range = vnorm3(los);
    rho->d = range;
    rho->range = range - K_C * clk[0];
    rho->rate = vdot3(vel, los) / range;
    rho->g = g;

    ecef_to_neu(los, tmat, neu);
    neu_to_azel(rho->azel, neu);

    rho->iono_delay = iono_delay(io, g, llh, rho->azel);
    rho->range += rho->iono_delay;
}

void sv_range(rng_t *rho, const eph_t *e, const iono_t *io, gtime_t g, const double *xyz)
{
    double llh[3], tmat[3][3];
    ecef_to_llh(xyz, llh);
    enu_matrix(llh, tmat);
    sv_range_at(rho, e, io, g, xyz, llh, tmat);
}

/* checkSatVisibility: 1 visible, 0 below mask, -1 no valid ephemeris. */
int sv_visible(const eph_t *e, gtime_t g, const double *xyz, double elv_mask, double *azel)
{
    double llh[3], neu[3], pos[3], vel[3], clk[3], los[3], tmat[3][3];

    if (e->vflg != 1)
        return -1;
    ecef_to_llh(xyz, llh);
    enu_matrix(llh, tmat);
    sv_state(e, g, pos, vel, clk);
    for (int i = 0; i < 3; i++)
        los[i] = pos[i] - xyz[i];
    ecef_to_neu(los, tmat, neu);
    neu_to_azel(azel, neu);
    return (azel[1] * K_R2D > elv_mask) ? 1 : 0;
}
