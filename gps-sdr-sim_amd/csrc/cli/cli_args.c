/*
 * cli_args.c — option surface of the reference (getopt string "e:u:g:c:l:o:s:b:T:t:d:iv",
 * gpssim.c:1756-1852), same validation messages and the same last-option-wins behaviour.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include "cli_args.h"

#define USER_MOTION_SIZE_DEFAULT 3000
#define STATIC_MAX_DURATION 86400

void gss_cli_usage(void)
{
    fprintf(stderr,
            "Usage: gps-sdr-sim [options]\n"
            "Options:\n"
            "  -e <gps_nav>     RINEX navigation file for GPS ephemerides (required)\n"
            "  -u <user_motion> User motion file (dynamic mode)\n"
            "  -g <nmea_gga>    NMEA GGA stream (dynamic mode)\n"
            "  -c <location>    ECEF X,Y,Z in meters (static mode) e.g. 3967283.154,1022538.181,4872414.484\n"
            "  -l <location>    Lat,Lon,Hgt (static mode) e.g. 35.681298,139.766247,10.0\n"
            "  -t <date,time>   Scenario start time YYYY/MM/DD,hh:mm:ss\n"
            "  -T <date,time>   Overwrite TOC and TOE to scenario start time\n"
            "  -d <duration>    Duration [sec] (dynamic mode max: %.0f, static mode max: %d)\n"
            "  -o <output>      I/Q sampling data file (default: gpssim.bin)\n"
            "  -s <frequency>   Sampling frequency [Hz] (default: 2600000)\n"
            "  -b <iq_bits>     I/Q data format [1/8/16] (default: 16)\n"
            "  -i               Disable ionospheric delay for spacecraft scenario\n"
            "  -v               Show details about simulated channels\n",
            ((double)USER_MOTION_SIZE_DEFAULT) / 10.0, STATIC_MAX_DURATION);
}

static void set_start(gss_cli_t *c, int y, int m, int d, int hh, int mm, double sec)
{
    c->opt.has_start = 1;
    c->opt.start[0] = y; c->opt.start[1] = m; c->opt.start[2] = d;
    c->opt.start[3] = hh; c->opt.start[4] = mm;
    c->opt.start_sec = sec;
}

int gss_cli_parse(int argc, char **argv, gss_cli_t *c)
{
    memset(c, 0, sizeof *c);
    strcpy(c->out_file, "gpssim.bin");
    c->opt.samp_freq = 2.6e6;
    c->opt.data_format = GSS_FMT_SC16;
    c->opt.duration = -1.0;                   /* → USER_MOTION_SIZE/10 */
    c->opt.user_motion_size = USER_MOTION_SIZE_DEFAULT;
    const char *ums = getenv("GSS_USER_MOTION_SIZE");   /* the reference's -DUSER_MOTION_SIZE */
    if (ums && atoi(ums) > 0)
        c->opt.user_motion_size = atoi(ums);

    /* --carrier=float|int (an extension: the reference chooses at compile time, gpssim.h:4) is
       taken out before the reference's getopt loop sees the arguments */
    char *av[argc + 1];
    int ac = 0;
    for (int i = 0; i < argc; i++) {
        if (i > 0 && strncmp(argv[i], "--carrier=", 10) == 0) {
            if (strcmp(argv[i] + 10, "int") == 0)
                c->opt.carrier_int = 1;
            else if (strcmp(argv[i] + 10, "float") == 0)
                c->opt.carrier_int = 0;
            else {
                fprintf(stderr, "ERROR: Invalid carrier mode (float or int).\n");
                return 1;
            }
            continue;
        }
        av[ac++] = argv[i];
    }
    av[ac] = NULL;
    argc = ac;
    argv = av;

    if (argc < 3) {
        gss_cli_usage();
        return 1;
    }
    int r, has_d = 0;
    /* 0, not 1: glibc then re-initialises all of getopt's state.  With 1 it keeps its pointer
       into the previous call's argv, which a library caller (the Python binding) has freed, and
       reads it as more options. */
    optind = 0;
    while ((r = getopt(argc, argv, "e:u:g:c:l:o:s:b:T:t:d:iv")) != -1) {
        switch (r) {
        case 'e':
            snprintf(c->nav_file, sizeof c->nav_file, "%s", optarg);
            break;
        case 'u':
            snprintf(c->motion_file, sizeof c->motion_file, "%s", optarg);
            c->opt.nmea = 0;
            break;
        case 'g':
            snprintf(c->motion_file, sizeof c->motion_file, "%s", optarg);
            c->opt.nmea = 1;
            break;
        case 'c':
            c->opt.has_xyz = 1;
            c->opt.has_llh = 0;
            sscanf(optarg, "%lf,%lf,%lf", &c->opt.xyz[0], &c->opt.xyz[1], &c->opt.xyz[2]);
            break;
        case 'l':
            c->opt.has_llh = 1;
            c->opt.has_xyz = 0;
            sscanf(optarg, "%lf,%lf,%lf", &c->opt.llh[0], &c->opt.llh[1], &c->opt.llh[2]);
            break;
        case 'o':
            snprintf(c->out_file, sizeof c->out_file, "%s", optarg);
            break;
        case 's':
            c->opt.samp_freq = atof(optarg);
            if (c->opt.samp_freq < 1.0e6) {
                fprintf(stderr, "ERROR: Invalid sampling frequency.\n");
                return 1;
            }
            break;
        case 'b':
            c->opt.data_format = atoi(optarg);
            if (c->opt.data_format != 1 && c->opt.data_format != 8 && c->opt.data_format != 16) {
                fprintf(stderr, "ERROR: Invalid I/Q data format.\n");
                return 1;
            }
            break;
        case 'T':
            c->opt.time_overwrite = 1;
            if (strncmp(optarg, "now", 3) == 0) {
                time_t now;
                time(&now);
                struct tm *gmt = gmtime(&now);
                set_start(c, gmt->tm_year + 1900, gmt->tm_mon + 1, gmt->tm_mday, gmt->tm_hour,
                          gmt->tm_min, (double)gmt->tm_sec);
                break;
            }
            /* fall through: -T with a date parses like -t (gpssim.c:1804-1835) */
        case 't': {
            int y = 0, m = 0, d = 0, hh = 0, mm = 0;
            double sec = 0.0;
            sscanf(optarg, "%d/%d/%d,%d:%d:%lf", &y, &m, &d, &hh, &mm, &sec);
            if (y <= 1980 || m < 1 || m > 12 || d < 1 || d > 31 || hh < 0 || hh > 23 || mm < 0 ||
                mm > 59 || sec < 0.0 || sec >= 60.0) {
                fprintf(stderr, "ERROR: Invalid date and time.\n");
                return 1;
            }
            set_start(c, y, m, d, hh, mm, floor(sec));
            break;
        }
        case 'd':
            c->opt.duration = atof(optarg);
            has_d = 1;
            break;
        case 'i':
            c->opt.iono_disable = 1;
            break;
        case 'v':
            c->opt.verbose = 1;
            break;
        case ':':
        case '?':
            gss_cli_usage();
            return 1;
        default:
            break;
        }
    }
    c->opt.nav_file = c->nav_file;
    c->opt.motion_file = c->motion_file[0] ? c->motion_file : NULL;
    if (has_d && c->opt.duration < 0.0) {
        fprintf(stderr, "ERROR: Invalid duration.\n");
        return 1;
    }
    return 0;
}
