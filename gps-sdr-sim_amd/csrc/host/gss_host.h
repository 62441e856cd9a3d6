/*
 * gss_host.h — internal types and constants of the host control plane.
 *
 * The numeric constants below must be the reference's decimal literals (gpssim.h:43-74), not
 * "better" values: e.g. POW2_M29 written as 1.862645149230957e-9 parses to a double one ulp away
 * from 2^-29, and PI is 3.1415926535898, not M_PI.  Every output bit depends on them.
 */
#ifndef GSS_HOST_H
#define GSS_HOST_H

#include <stdint.h>
#include <stdio.h>
#include "gpssim_amd.h"

/* ---- constants (gpssim.h:10-79) ---------------------------------------------------------- */
#define K_MAX_LINE          100          /* MAX_CHAR  */
#define K_MAX_SAT           32
#define K_MAX_CHAN          GSS_MAXCH
#define K_STATIC_MAX_DUR    86400
#define K_N_SBF             5
#define K_N_DWRD_SBF        10
#define K_N_DWRD            GSS_NAV_WORDS
#define K_CA_LEN            GSS_CA_LEN
#define K_CARR_INT_ONE      33554432.0      /* 512*65536: one cycle of the integer carrier */
#define K_EPH_SETS          13           /* EPHEM_ARRAY_SIZE */

#define K_SEC_WEEK          604800.0
#define K_SEC_HALF_WEEK     302400.0
#define K_SEC_DAY           86400.0
#define K_SEC_HOUR          3600.0
#define K_SEC_MIN           60.0

#define K_P2_M5   0.03125
#define K_P2_M19  1.907348632812500e-6
#define K_P2_M29  1.862645149230957e-9
#define K_P2_M31  4.656612873077393e-10
#define K_P2_M33  1.164153218269348e-10
#define K_P2_M43  1.136868377216160e-13
#define K_P2_M55  2.775557561562891e-17
#define K_P2_M50  8.881784197001252e-016
#define K_P2_M30  9.313225746154785e-010
#define K_P2_M27  7.450580596923828e-009
#define K_P2_M24  5.960464477539063e-008

#define K_GM          3.986005e14
#define K_OMEGA_E     7.2921151467e-5
#define K_PI          3.1415926535898
#define K_WGS84_A     6378137.0
#define K_WGS84_E     0.0818191908426
#define K_R2D         57.2957795131
#define K_C           2.99792458e8
#define K_LAMBDA_L1   0.190293672798365
#define K_CODE_FREQ   (1.023e6)
#define K_CARR_TO_CODE (1.0/1540.0)

/* ---- types -------------------------------------------------------------------------------- */
typedef struct { int week; double sec; } gtime_t;                      /* gpstime_t  */
typedef struct { int y, m, d, hh, mm; double sec; } dtime_t;           /* datetime_t */

typedef struct {                     /* one broadcast ephemeris (ephem_t, gpssim.h:102-136)     */
    int vflg;
    dtime_t t;
    gtime_t toc, toe;
    int iodc, iode;
    double deltan, cuc, cus, cic, cis, crc, crs, ecc, sqrta, m0, omg0, inc0, aop, omgdot, idot;
    double af0, af1, af2, tgd;
    int svhlth, codeL2;
    double n, sq1e2, A, omgkdot;     /* derived (gpssim.c:1156-1159) */
} eph_t;

typedef struct {                     /* ionoutc_t (gpssim.h:138-147) */
    int enable, vflg;
    double alpha0, alpha1, alpha2, alpha3, beta0, beta1, beta2, beta3, A0, A1;
    int dtls, tot, wnt, dtlsf, dn, wnlsf;
} iono_t;

typedef struct {                     /* range_t (gpssim.h:149-157) */
    gtime_t g;
    double range, rate, d, azel[2], iono_delay;
} rng_t;

typedef struct {                     /* the fields of channel_t (gpssim.h:160-183) we keep      */
    int prn;
    uint32_t ca_bits[GSS_CA_WORDS];
    int8_t ca[K_CA_LEN];             /* 0/1 chips */
    double f_carr, f_code;
    double carr_phase;               /* FLOAT_CARR_PHASE: value at allocation (planner carries) */
    double code_phase;
    gtime_t g0;
    uint32_t sbf[K_N_SBF][K_N_DWRD_SBF];
    uint32_t dwrd[K_N_DWRD];
    int iword, ibit, icode;
    double azel[2];
    rng_t rho0;
    int nav_row;                     /* row of the nav table holding the current dwrd          */
    gss_nav_src_t fsrc;              /* the current frame as a GPU producer source (nav_frame)  */
    int frame_init;                  /* the current frame was built from sbf[4] (allocation)    */
    int frame_seq;                   /* frames built so far on this channel                      */
    int last_row, last_row_seq;      /* the channel's last pushed row and its frame_seq          */
    int carr_fresh;                  /* carr_phase was (re)initialised since the last block     */
} chan_t;

/* ---- gnss_time.c -------------------------------------------------------------------------- */
void   gt_from_date(const dtime_t *t, gtime_t *g);           /* date2gps  gpssim.c:177 */
void   gt_to_date(const gtime_t *g, dtime_t *t);             /* gps2date  gpssim.c:202 */
double gt_diff(gtime_t g1, gtime_t g0);                      /* subGpsTime gpssim.c:779 */
gtime_t gt_add(gtime_t g0, double dt);                       /* incGpsTime gpssim.c:789 */

/* ---- gnss_frames.c ------------------------------------------------------------------------ */
void   ecef_to_llh(const double *xyz, double *llh);          /* xyz2llh gpssim.c:225 */
void   llh_to_ecef(const double *llh, double *xyz);          /* llh2xyz gpssim.c:279 */
void   enu_matrix(const double *llh, double t[3][3]);        /* ltcmat  gpssim.c:317 */
void   ecef_to_neu(const double *xyz, double t[3][3], double *neu);  /* gpssim.c:345 */
void   neu_to_azel(double *azel, const double *neu);         /* gpssim.c:358 */
double vnorm3(const double *x);
double vdot3(const double *a, const double *b);

/* ---- gnss_orbit.c ------------------------------------------------------------------------- */
void   sv_state(const eph_t *eph, gtime_t g, double *pos, double *vel, double *clk); /* satpos */
double iono_delay(const iono_t *io, gtime_t g, const double *llh, const double *azel);
void   sv_range(rng_t *rho, const eph_t *eph, const iono_t *io, gtime_t g, const double *xyz);
void   sv_range_at(rng_t *rho, const eph_t *eph, const iono_t *io, gtime_t g, const double *xyz,
                   const double *llh, double tmat[3][3]);   /* llh, tmat of xyz given */
int    sv_visible(const eph_t *eph, gtime_t g, const double *xyz, double elv_mask, double *azel);

/* ---- gnss_navmsg.c ------------------------------------------------------------------------ */
void   ca_generate(int8_t *ca, int prn);                     /* codegen gpssim.c:132 */
void   ca_pack(const int8_t *ca, uint32_t *bits);
void   nav_subframes(const eph_t *eph, const iono_t *io, uint32_t sbf[5][K_N_DWRD_SBF]);
uint32_t nav_parity(uint32_t source, int nib);               /* computeChecksum gpssim.c:693 */
void   nav_frame(gtime_t g, chan_t *ch, int init);           /* generateNavMsg gpssim.c:1467 */

/* ---- gnss_inputs.c ------------------------------------------------------------------------ */
int    rinex_read(eph_t eph[][K_MAX_SAT], iono_t *io, const char *fname);
int    motion_read_csv(double (*xyz)[3], int cap, const char *fname);
int    motion_read_nmea(double (*xyz)[3], int cap, const char *fname);

/* ---- pool.c ------------------------------------------------------------------------------- */
typedef void (*gss_task_fn)(void *arg, int part);
int    gss_pool_run(int nthreads, int nparts, gss_task_fn fn, void *arg);
void   gss_pool_select(int id);     /* this thread's pool: 0 default; 1, 2 gss_run's rows, proofs */

/* ---- errors ------------------------------------------------------------------------------- */
int    gss_fail(int code, const char *fmt, ...);
extern double gss_ant_pat_db[37];

#endif
