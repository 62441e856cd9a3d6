/*
 * gnss_inputs.c — RINEX v2 navigation, user-motion CSV and NMEA GGA readers.
 * Restates readRinexNavAll (gpssim.c:818-1168), readUserMotion (1358-1384) and readNmeaGGA
 * (1386-1465).  Fields are fixed-column; like the reference we read lines into one reused
 * 100-byte buffer with fgets, so a short line sees the same bytes the reference would.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "gss_host.h"

/* Copy `len` bytes at line+off into a NUL-terminated field (strncpy semantics), converting the
   Fortran 'D' exponent to 'E' (replaceExpDesignator, gpssim.c:763-777). */
static const char *field(char *dst, const char *line, int off, int len, int fortran_exp)
{
    strncpy(dst, line + off, (size_t)len);
    dst[len] = 0;
    if (fortran_exp)
        for (int i = 0; i < len; i++)
            if (dst[i] == 'D')
                dst[i] = 'E';
    return dst;
}

static double fnum(char *tmp, const char *line, int off)    /* one 19-column D19.12 value */
{
    return atof(field(tmp, line, off, 19, 1));
}

int rinex_read(eph_t eph[][K_MAX_SAT], iono_t *io, const char *fname)
{
    char line[K_MAX_LINE], tmp[20];
    FILE *fp = fopen(fname, "rt");
    if (fp == NULL)
        return -1;

    for (int k = 0; k < K_EPH_SETS; k++)
        for (int sv = 0; sv < K_MAX_SAT; sv++)
            eph[k][sv].vflg = 0;

    /* header: ION ALPHA / ION BETA / DELTA-UTC / LEAP SECONDS (labels at column 60) */
    int have = 0;
    while (fgets(line, K_MAX_LINE, fp) != NULL) {
        const char *lab = line + 60;
        if (strncmp(lab, "END OF HEADER", 13) == 0)
            break;
        if (strncmp(lab, "ION ALPHA", 9) == 0) {
            io->alpha0 = atof(field(tmp, line, 2, 12, 1));
            io->alpha1 = atof(field(tmp, line, 14, 12, 1));
            io->alpha2 = atof(field(tmp, line, 26, 12, 1));
            io->alpha3 = atof(field(tmp, line, 38, 12, 1));
            have |= 1;
        } else if (strncmp(lab, "ION BETA", 8) == 0) {
            io->beta0 = atof(field(tmp, line, 2, 12, 1));
            io->beta1 = atof(field(tmp, line, 14, 12, 1));
            io->beta2 = atof(field(tmp, line, 26, 12, 1));
            io->beta3 = atof(field(tmp, line, 38, 12, 1));
            have |= 2;
        } else if (strncmp(lab, "DELTA-UTC", 9) == 0) {
            io->A0 = fnum(tmp, line, 3);
            io->A1 = fnum(tmp, line, 22);
            io->tot = atoi(field(tmp, line, 41, 9, 0));
            io->wnt = atoi(field(tmp, line, 50, 9, 0));
            if (io->tot % 4096 == 0)
                have |= 4;
        } else if (strncmp(lab, "LEAP SECONDS", 12) == 0) {
            io->dtls = atoi(field(tmp, line, 0, 6, 0));
            have |= 8;
        }
    }
    io->vflg = (have == 0xF) ? 1 : 0;

    /* 8-line ephemeris records; a new set starts when toc moves > 1 h past the set's first toc */
    gtime_t set_t0 = {-1, 0.0};
    int set = 0;
    while (fgets(line, K_MAX_LINE, fp) != NULL) {
        dtime_t t;
        gtime_t g;
        int sv = atoi(field(tmp, line, 0, 2, 0)) - 1;
        t.y = atoi(field(tmp, line, 3, 2, 0)) + 2000;
        t.m = atoi(field(tmp, line, 6, 2, 0));
        t.d = atoi(field(tmp, line, 9, 2, 0));
        t.hh = atoi(field(tmp, line, 12, 2, 0));
        t.mm = atoi(field(tmp, line, 15, 2, 0));
        t.sec = atof(field(tmp, line, 18, 2, 0));   /* reference keeps 2 of the 4 columns */
        gt_from_date(&t, &g);

        if (set_t0.week == -1)
            set_t0 = g;
        if (gt_diff(g, set_t0) > K_SEC_HOUR) {
            set_t0 = g;
            if (++set >= K_EPH_SETS)
                break;
        }
        /* a PRN outside 1..32 would index out of bounds in the reference; park it in a scratch
           record instead (never valid) */
        static eph_t scratch;
        eph_t *e = (sv >= 0 && sv < K_MAX_SAT) ? &eph[set][sv] : &scratch;

        e->t = t;
        e->toc = g;
        e->af0 = fnum(tmp, line, 22);
        e->af1 = fnum(tmp, line, 41);
        e->af2 = fnum(tmp, line, 60);

        if (fgets(line, K_MAX_LINE, fp) == NULL) break;      /* BROADCAST ORBIT 1 */
        e->iode = (int)fnum(tmp, line, 3);
        e->crs = fnum(tmp, line, 22);
        e->deltan = fnum(tmp, line, 41);
        e->m0 = fnum(tmp, line, 60);

        if (fgets(line, K_MAX_LINE, fp) == NULL) break;      /* 2 */
        e->cuc = fnum(tmp, line, 3);
        e->ecc = fnum(tmp, line, 22);
        e->cus = fnum(tmp, line, 41);
        e->sqrta = fnum(tmp, line, 60);

        if (fgets(line, K_MAX_LINE, fp) == NULL) break;      /* 3 */
        e->toe.sec = fnum(tmp, line, 3);
        e->cic = fnum(tmp, line, 22);
        e->omg0 = fnum(tmp, line, 41);
        e->cis = fnum(tmp, line, 60);

        if (fgets(line, K_MAX_LINE, fp) == NULL) break;      /* 4 */
        e->inc0 = fnum(tmp, line, 3);
        e->crc = fnum(tmp, line, 22);
        e->aop = fnum(tmp, line, 41);
        e->omgdot = fnum(tmp, line, 60);

        if (fgets(line, K_MAX_LINE, fp) == NULL) break;      /* 5 */
        e->idot = fnum(tmp, line, 3);
        e->codeL2 = (int)fnum(tmp, line, 22);
        e->toe.week = (int)fnum(tmp, line, 41);

        if (fgets(line, K_MAX_LINE, fp) == NULL) break;      /* 6 */
        e->svhlth = (int)fnum(tmp, line, 22);
        if (e->svhlth > 0 && e->svhlth < 32)
            e->svhlth += 32;                                /* set the summary MSB */
        e->tgd = fnum(tmp, line, 41);
        e->iodc = (int)fnum(tmp, line, 60);

        if (fgets(line, K_MAX_LINE, fp) == NULL) break;      /* 7 */
        e->vflg = (e == &scratch) ? 0 : 1;

        e->A = e->sqrta * e->sqrta;
        e->n = sqrt(K_GM / (e->A * e->A * e->A)) + e->deltan;
        e->sq1e2 = sqrt(1.0 - e->ecc * e->ecc);
        e->omgkdot = e->omgdot - K_OMEGA_E;
    }
    fclose(fp);
    if (set_t0.week >= 0)
        set += 1;
    return set;
}

/* readUserMotion: "t,x,y,z" at 10 Hz.  A line sscanf cannot start on ends the file; a partly
   parsed line keeps the previous values for the missing fields, as in the reference. */
int motion_read_csv(double (*xyz)[3], int cap, const char *fname)
{
    char line[K_MAX_LINE];
    double t, x = 0, y = 0, z = 0;
    FILE *fp = fopen(fname, "rt");
    if (fp == NULL)
        return -1;
    int n;
    for (n = 0; n < cap; n++) {
        if (fgets(line, K_MAX_LINE, fp) == NULL)
            break;
        if (sscanf(line, "%lf,%lf,%lf,%lf", &t, &x, &y, &z) == EOF)
            break;
        xyz[n][0] = x;
        xyz[n][1] = y;
        xyz[n][2] = z;
    }
    fclose(fp);
    return n;
}

/* readNmeaGGA: $xxGGA sentences → ECEF via llh2xyz (geoid height added to altitude). */
int motion_read_nmea(double (*xyz)[3], int cap, const char *fname)
{
    char line[K_MAX_LINE], tmp[8];
    FILE *fp = fopen(fname, "rt");
    if (fp == NULL)
        return -1;
    int n = 0;
    while (fgets(line, K_MAX_LINE, fp) != NULL) {
        char *tok = strtok(line, ",");
        if (tok == NULL || strncmp(tok + 3, "GGA", 3) != 0)
            continue;
        double llh[3], pos[3];
        tok = strtok(NULL, ",");                       /* UTC time */
        tok = strtok(NULL, ",");                       /* ddmm.mmmm */
        strncpy(tmp, tok, 2); tmp[2] = 0;
        llh[0] = atof(tmp) + atof(tok + 2) / 60.0;
        tok = strtok(NULL, ",");
        if (tok[0] == 'S')
            llh[0] *= -1.0;
        llh[0] /= K_R2D;
        tok = strtok(NULL, ",");                       /* dddmm.mmmm */
        strncpy(tmp, tok, 3); tmp[3] = 0;
        llh[1] = atof(tmp) + atof(tok + 3) / 60.0;
        tok = strtok(NULL, ",");
        if (tok[0] == 'W')
            llh[1] *= -1.0;
        llh[1] /= K_R2D;
        strtok(NULL, ",");                             /* fix quality */
        strtok(NULL, ",");                             /* satellites */
        strtok(NULL, ",");                             /* HDOP */
        tok = strtok(NULL, ",");                       /* altitude MSL */
        llh[2] = atof(tok);
        strtok(NULL, ",");                             /* "M" */
        tok = strtok(NULL, ",");                       /* geoid separation */
        llh[2] += atof(tok);
        llh_to_ecef(llh, pos);
        xyz[n][0] = pos[0];
        xyz[n][1] = pos[1];
        xyz[n][2] = pos[2];
        if (++n >= cap)
            break;
    }
    fclose(fp);
    return n;
}
