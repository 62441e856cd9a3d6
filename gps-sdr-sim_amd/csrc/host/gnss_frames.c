/*
 * gnss_frames.c — WGS-84 frame conversions and 3-vector helpers (gpssim.c:100-126, 225-370).
 * Expression order follows the reference so that every intermediate rounds identically.
 */
#include <math.h>
#include "gss_host.h"

double vnorm3(const double *x)                               /* normVect, gpssim.c:113 */
{
    return sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
}

double vdot3(const double *a, const double *b)               /* dotProd, gpssim.c:123 */
{
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

/* xyz2llh, gpssim.c:225-273: fixed-point iteration on the ellipsoidal height correction. */
void ecef_to_llh(const double *xyz, double *llh)
{
    const double a = K_WGS84_A, e = K_WGS84_E, eps = 1.0e-3;
    const double e2 = e * e;

    if (vnorm3(xyz) < eps) {            /* degenerate: earth centre */
        llh[0] = 0.0;
        llh[1] = 0.0;
        llh[2] = -a;
        return;
    }
    double x = xyz[0], y = xyz[1], z = xyz[2];
    double r2 = x * x + y * y;
    double dz = e2 * z, zp, nh, sl, nrad;
    for (;;) {
        zp = z + dz;
        nh = sqrt(r2 + zp * zp);
        sl = zp / nh;
        nrad = a / sqrt(1.0 - e2 * sl * sl);
        double dz_next = nrad * e2 * sl;
        if (fabs(dz - dz_next) < eps)
            break;
        dz = dz_next;
    }
    llh[0] = atan2(zp, sqrt(r2));
    llh[1] = atan2(y, x);
    llh[2] = nh - nrad;
}

/* llh2xyz, gpssim.c:279-311. */
void llh_to_ecef(const double *llh, double *xyz)
{
    const double a = K_WGS84_A, e = K_WGS84_E;
    const double e2 = e * e;
    double clat = cos(llh[0]), slat = sin(llh[0]);
    double clon = cos(llh[1]), slon = sin(llh[1]);
    double es = e * slat;
    double nrad = a / sqrt(1.0 - es * es);
    double rn = (nrad + llh[2]) * clat;

    xyz[0] = rn * clon;
    xyz[1] = rn * slon;
    xyz[2] = ((1.0 - e2) * nrad + llh[2]) * slat;
}

/* ltcmat, gpssim.c:317-338: rows are north, east, up. */
void enu_matrix(const double *llh, double t[3][3])
{
    double slat = sin(llh[0]), clat = cos(llh[0]);
    double slon = sin(llh[1]), clon = cos(llh[1]);

    t[0][0] = -slat * clon;  t[0][1] = -slat * slon;  t[0][2] = clat;
    t[1][0] = -slon;         t[1][1] = clon;          t[1][2] = 0.0;
    t[2][0] = clat * clon;   t[2][1] = clat * slon;   t[2][2] = slat;
}

/* ecef2neu, gpssim.c:345-352. */
void ecef_to_neu(const double *xyz, double t[3][3], double *neu)
{
    for (int r = 0; r < 3; r++)
        neu[r] = t[r][0] * xyz[0] + t[r][1] * xyz[1] + t[r][2] * xyz[2];
}

/* neu2azel, gpssim.c:358-370. */
void neu_to_azel(double *azel, const double *neu)
{
    azel[0] = atan2(neu[1], neu[0]);
    if (azel[0] < 0.0)
        azel[0] += (2.0 * K_PI);
    double ne = sqrt(neu[0] * neu[0] + neu[1] * neu[1]);
    azel[1] = atan2(neu[2], ne);
}
