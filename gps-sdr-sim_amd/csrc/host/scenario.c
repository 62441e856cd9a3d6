/*
 * scenario.c — the host control plane: main() of gpssim.c minus the per-sample loop.
 *
 *   gss_scn_open  ≙ gpssim.c:1738-2152  (options → inputs → start time → ephemeris set →
 *                                        first channel allocation → antenna pattern)
 *   gss_scn_next  ≙ gpssim.c:2154-2188  (per-block refresh: range, code phase, gain)
 *                 + gpssim.c:2290-2352  (30 s nav/ephemeris/allocation update, time step)
 *                 + the carrier-phase chain the sample loop carries across blocks
 *                   (gpssim.c:2245-2250), produced exactly by the planner below.
 *
 * The sample loop itself is not here: its inputs are emitted as gss_chan_blk_t rows and the
 * GPU synthesises them (gss_synth_*).
 */
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "gss_host.h"
#include "../common/gss_nav.h"
#include "../common/gss_phase.h"

/* Receiver antenna attenuation [dB] vs boresight angle 0:5:180 deg (gpssim.c:86-91). */
double gss_ant_pat_db[37] = {
     0.00,  0.00,  0.22,  0.44,  0.67,  1.11,  1.56,  2.00,  2.44,  2.89,  3.56,  4.22,
     4.89,  5.56,  6.22,  6.89,  7.56,  8.22,  8.89,  9.78, 10.67, 11.56, 12.44, 13.33,
    14.44, 15.56, 16.67, 17.78, 18.89, 20.00, 21.33, 22.67, 24.00, 25.56, 27.33, 29.33,
    31.56};

/* ---- error reporting ---------------------------------------------------------------------- */
static __thread char g_err[512];

int gss_fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

const char *gss_last_error(void) { return g_err; }

static double wall_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ---- scenario state ------------------------------------------------------------------------ */
struct gss_scn {
    gss_opts_t opt;
    int quiet;
    eph_t eph[K_EPH_SETS + 1][K_MAX_SAT];   /* +1: the reference reads eph[ieph+1] at ieph=12 */
    int neph, ieph;
    iono_t io;
    double (*xyz)[3];
    int numd, static_mode;
    int n_per_blk;
    double samp_freq, delt;
    gtime_t g0, grx;
    chan_t chan[K_MAX_CHAN];
    int alloc_sat[K_MAX_SAT];
    double ant_pat[37];
    int iumd;                               /* next block index, 1..numd-1 (gpssim.c:2154) */
    uint32_t *nav_rows;
    gss_nav_src_t *nav_src;          /* row r's source for the GPU producer (gss_nav.h)         */
    int n_nav, cap_nav;
    double carr[K_MAX_CHAN];                /* planner: carrier at the next block start per slot */
    int carr_known;                         /* 0 after gss_scn_seek or gss_scn_next_deferred
                                               until gss_scn_set_carrier                      */
    double plan_sec;
    int64_t rows_out;                       /* blocks whose rows this handle has produced */
    /* per-batch carrier-chain bookkeeping of gss_scn_next (gss_scn_next_deferred's is the
       caller's) */
    int batch_cap;
    gss_chain_t *chain;                     /* [b][k] */
    /* ranges of the blocks up to the next 30 s update, computed in parallel (range_pass) */
    rng_t *rg;                              /* [j][slot] */
    int rg_cap;
};

static void msg(const gss_scn *s, const char *fmt, ...)
{
    if (s->quiet)
        return;
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
}

/* Append a copy of ch->dwrd to the nav table and point the channel at it.  The row's source
   (gss_nav_src_t) continues the channel's previous row when that row holds the frame before this
   one, is rebuilt from sbf[4] for a fresh allocation, and carries its first ten words otherwise
   (frames built during a seek are not rows). */
static int nav_push(gss_scn *s, chan_t *ch)
{
    if (s->n_nav == s->cap_nav) {
        int cap = s->cap_nav ? 2 * s->cap_nav : 256;
        uint32_t *p = realloc(s->nav_rows, (size_t)cap * GSS_NAV_WORDS * sizeof(uint32_t));
        if (p == NULL)
            return gss_fail(GSS_E_NOMEM, "out of memory (nav table)");
        s->nav_rows = p;
        gss_nav_src_t *q = realloc(s->nav_src, (size_t)cap * sizeof(gss_nav_src_t));
        if (q == NULL)
            return gss_fail(GSS_E_NOMEM, "out of memory (nav sources)");
        s->nav_src = q;
        s->cap_nav = cap;
    }
    const int r = s->n_nav;
    memcpy(s->nav_rows + (size_t)r * GSS_NAV_WORDS, ch->dwrd, sizeof ch->dwrd);
    gss_nav_src_t *src = &s->nav_src[r];
    *src = ch->fsrc;
    src->next = -1;
    memset(src->head, 0, sizeof src->head);
    if (ch->frame_init) {
        src->prev = GSS_NAV_HEAD_INIT;
    } else if (ch->last_row >= 0 && ch->last_row_seq == ch->frame_seq - 1) {
        src->prev = ch->last_row;
        s->nav_src[ch->last_row].next = r;
    } else {
        src->prev = GSS_NAV_HEAD_GIVEN;
        memcpy(src->head, ch->dwrd, sizeof src->head);
    }
    ch->last_row = r;
    ch->last_row_seq = ch->frame_seq;
    ch->nav_row = s->n_nav++;
    return 0;
}

/* allocateChannel, gpssim.c:1572-1648: (de)allocate visible satellites into free slots. */
static int allocate_channels(gss_scn *s, const eph_t *eset, gtime_t grx, const double *xyz)
{
    int nsat = 0;
    const double origin[3] = {0.0, 0.0, 0.0};

    for (int sv = 0; sv < K_MAX_SAT; sv++) {
        double azel[2];
        if (sv_visible(&eset[sv], grx, xyz, 0.0, azel) == 1) {
            nsat++;
            if (s->alloc_sat[sv] != -1)
                continue;
            int i;
            for (i = 0; i < K_MAX_CHAN; i++) {
                chan_t *ch = &s->chan[i];
                if (ch->prn != 0)
                    continue;
                rng_t rho;
                ch->prn = sv + 1;
                ch->azel[0] = azel[0];
                ch->azel[1] = azel[1];
                ca_generate(ch->ca, ch->prn);
                ca_pack(ch->ca, ch->ca_bits);
                nav_subframes(&eset[sv], &s->io, ch->sbf);
                nav_frame(grx, ch, 1);
                int rc = nav_push(s, ch);
                if (rc)
                    return rc;
                sv_range(&rho, &eset[sv], &s->io, grx, xyz);
                ch->rho0 = rho;
                /* initial carrier phase from the range difference to the geocentre
                   (gpssim.c:1615-1622, FLOAT_CARR_PHASE branch) */
                double r_xyz = rho.range;
                sv_range(&rho, &eset[sv], &s->io, grx, origin);
                double r_ref = rho.range;
                double ph = (2.0 * r_ref - r_xyz) / K_LAMBDA_L1;
                ch->carr_phase = ph - floor(ph);
                if (s->opt.carrier_int)   /* #else branch: (unsigned int)(512*65536*phase) */
                    ch->carr_phase = (double)(unsigned int)(512.0 * 65536.0 * ch->carr_phase) /
                                     K_CARR_INT_ONE;
                ch->carr_fresh = 1;
                break;
            }
            if (i < K_MAX_CHAN)
                s->alloc_sat[sv] = i;
        } else if (s->alloc_sat[sv] >= 0) {
            s->chan[s->alloc_sat[sv]].prn = 0;
            s->alloc_sat[sv] = -1;
        }
    }
    return nsat;
}

static void print_channels(const gss_scn *s)
{
    for (int i = 0; i < K_MAX_CHAN; i++) {
        const chan_t *c = &s->chan[i];
        if (c->prn > 0)
            msg(s, "%02d %6.1f %5.1f %11.1f %5.1f\n", c->prn, c->azel[0] * K_R2D,
                c->azel[1] * K_R2D, c->rho0.d, c->rho0.iono_delay);
    }
}

int gss_scn_open(gss_scn **out, const gss_opts_t *opt)
{
    *out = NULL;
    gss_scn *s = calloc(1, sizeof *s);
    if (s == NULL)
        return gss_fail(GSS_E_NOMEM, "out of memory");
    s->opt = *opt;
    s->quiet = opt->quiet;
    int ums = opt->user_motion_size > 0 ? opt->user_motion_size : 3000;
    int rc = GSS_E_INPUT;

    /* ---- options (gpssim.c:1739-1881) ---- */
    if (opt->nav_file == NULL || opt->nav_file[0] == 0) {
        rc = gss_fail(GSS_E_ARG, "ERROR: GPS ephemeris file is not specified.");
        goto fail;
    }
    double fs = opt->samp_freq > 0 ? opt->samp_freq : 2.6e6;
    if (fs < 1.0e6) {
        rc = gss_fail(GSS_E_ARG, "ERROR: Invalid sampling frequency.");
        goto fail;
    }
    int fmt = opt->data_format ? opt->data_format : GSS_FMT_SC16;
    if (fmt != GSS_FMT_SC01 && fmt != GSS_FMT_SC08 && fmt != GSS_FMT_SC16) {
        rc = gss_fail(GSS_E_ARG, "ERROR: Invalid I/Q data format.");
        goto fail;
    }
    s->opt.data_format = fmt;
    s->io.enable = opt->iono_disable ? 0 : 1;
    /* -c/-l select static mode; so does the absence of a motion file (gpssim.c:1860-1867) */
    s->static_mode = opt->has_xyz || opt->has_llh || opt->motion_file == NULL ||
                     opt->motion_file[0] == 0;
    double duration = opt->duration >= 0.0 ? opt->duration : (double)ums / 10.0;
    if (duration < 0.0 || (duration > ((double)ums) / 10.0 && !s->static_mode) ||
        (duration > K_STATIC_MAX_DUR && s->static_mode)) {
        rc = gss_fail(GSS_E_ARG, "ERROR: Invalid duration.");
        goto fail;
    }
    int iduration = (int)(duration * 10.0 + 0.5);

    fs = floor(fs / 10.0);
    s->n_per_blk = (int)fs;
    fs *= 10.0;
    s->samp_freq = fs;
    s->delt = 1.0 / fs;
    if (fmt == GSS_FMT_SC01 && (s->n_per_blk % 4) != 0) {
        /* the reference overflows its 1-bit buffer here */
        rc = gss_fail(GSS_E_ARG, "ERROR: -b 1 needs samples per 0.1 s divisible by 4.");
        goto fail;
    }

    /* ---- receiver position (gpssim.c:1887-1917) ---- */
    if (!s->static_mode) {
        s->xyz = calloc((size_t)ums, sizeof *s->xyz);
        if (s->xyz == NULL) { rc = gss_fail(GSS_E_NOMEM, "out of memory"); goto fail; }
        int numd = opt->nmea ? motion_read_nmea(s->xyz, ums, opt->motion_file)
                             : motion_read_csv(s->xyz, ums, opt->motion_file);
        if (numd == -1) {
            rc = gss_fail(GSS_E_IO, "ERROR: Failed to open user motion / NMEA GGA file.");
            goto fail;
        }
        if (numd == 0) {
            rc = gss_fail(GSS_E_INPUT, "ERROR: Failed to read user motion / NMEA GGA data.");
            goto fail;
        }
        s->numd = numd > iduration ? iduration : numd;
    } else {
        s->xyz = calloc(1, sizeof *s->xyz);
        if (s->xyz == NULL) { rc = gss_fail(GSS_E_NOMEM, "out of memory"); goto fail; }
        if (opt->has_xyz) {
            memcpy(s->xyz[0], opt->xyz, sizeof s->xyz[0]);
        } else if (opt->has_llh) {
            double llh[3] = {opt->llh[0] / K_R2D, opt->llh[1] / K_R2D, opt->llh[2]};
            llh_to_ecef(llh, s->xyz[0]);
        }
        /* else: the reference's default (Tokyo) never reaches llh2xyz
           and its observed behaviour is an earth-centre receiver: xyz stays {0,0,0}. */
        msg(s, "Using static location mode.\n");
        s->numd = iduration;
    }

    /* ---- ephemerides (gpssim.c:1926-1948) ---- */
    s->neph = rinex_read(s->eph, &s->io, opt->nav_file);
    if (s->neph == 0) { rc = gss_fail(GSS_E_INPUT, "ERROR: No ephemeris available."); goto fail; }
    if (s->neph == -1) { rc = gss_fail(GSS_E_IO, "ERROR: ephemeris file not found."); goto fail; }
    if (opt->verbose && s->io.vflg) {
        msg(s, "  %12.3e %12.3e %12.3e %12.3e\n", s->io.alpha0, s->io.alpha1, s->io.alpha2,
            s->io.alpha3);
        msg(s, "  %12.3e %12.3e %12.3e %12.3e\n", s->io.beta0, s->io.beta1, s->io.beta2,
            s->io.beta3);
        msg(s, "   %19.11e %19.11e  %9d %9d\n", s->io.A0, s->io.A1, s->io.tot, s->io.wnt);
        msg(s, "%6d\n", s->io.dtls);
    }

    /* ---- scenario start time (gpssim.c:1950-2039) ---- */
    gtime_t gmin = {0, 0}, gmax = {0, 0};
    dtime_t tmin = {0}, tmax = {0};
    for (int sv = 0; sv < K_MAX_SAT; sv++)
        if (s->eph[0][sv].vflg == 1) { gmin = s->eph[0][sv].toc; tmin = s->eph[0][sv].t; break; }
    for (int sv = 0; sv < K_MAX_SAT; sv++)
        if (s->eph[s->neph - 1][sv].vflg == 1) {
            gmax = s->eph[s->neph - 1][sv].toc;
            tmax = s->eph[s->neph - 1][sv].t;
            break;
        }
    dtime_t t0;
    gtime_t g0;
    if (opt->has_start) {
        t0.y = opt->start[0]; t0.m = opt->start[1]; t0.d = opt->start[2];
        t0.hh = opt->start[3]; t0.mm = opt->start[4]; t0.sec = opt->start_sec;
        gt_from_date(&t0, &g0);
        if (opt->time_overwrite) {
            /* move every TOC/TOE by the offset between the scenario start (2 h aligned)
               and the file's first TOC (gpssim.c:1980-2014) */
            gtime_t gt;
            gt.week = g0.week;
            gt.sec = (double)(((int)(g0.sec)) / 7200) * 7200.0;
            double dsec = gt_diff(gt, gmin);
            s->io.wnt = gt.week;
            s->io.tot = (int)gt.sec;
            for (int sv = 0; sv < K_MAX_SAT; sv++)
                for (int i = 0; i < s->neph; i++) {
                    eph_t *e = &s->eph[i][sv];
                    if (e->vflg != 1)
                        continue;
                    gtime_t gn = gt_add(e->toc, dsec);
                    dtime_t tn;
                    gt_to_date(&gn, &tn);
                    e->toc = gn;
                    e->t = tn;
                    e->toe = gt_add(e->toe, dsec);
                }
        } else if (gt_diff(g0, gmin) < 0.0 || gt_diff(gmax, g0) < 0.0) {
            msg(s, "ERROR: Invalid start time.\n");
            msg(s, "tmin = %4d/%02d/%02d,%02d:%02d:%02.0f (%d:%.0f)\n", tmin.y, tmin.m, tmin.d,
                tmin.hh, tmin.mm, tmin.sec, gmin.week, gmin.sec);
            msg(s, "tmax = %4d/%02d/%02d,%02d:%02d:%02.0f (%d:%.0f)\n", tmax.y, tmax.m, tmax.d,
                tmax.hh, tmax.mm, tmax.sec, gmax.week, gmax.sec);
            rc = gss_fail(GSS_E_INPUT, "ERROR: Invalid start time.");
            goto fail;
        }
    } else {
        g0 = gmin;
        t0 = tmin;
    }
    s->g0 = g0;
    msg(s, "Start time = %4d/%02d/%02d,%02d:%02d:%02.0f (%d:%.0f)\n", t0.y, t0.m, t0.d, t0.hh,
        t0.mm, t0.sec, g0.week, g0.sec);
    msg(s, "Duration = %.1f [sec]\n", ((double)s->numd) / 10.0);

    /* ---- current ephemeris set: first set with a TOC within ±1 h (gpssim.c:2042-2067) ---- */
    s->ieph = -1;
    for (int i = 0; i < s->neph && s->ieph < 0; i++)
        for (int sv = 0; sv < K_MAX_SAT; sv++)
            if (s->eph[i][sv].vflg == 1) {
                double dt = gt_diff(g0, s->eph[i][sv].toc);
                if (dt >= -K_SEC_HOUR && dt < K_SEC_HOUR) {
                    s->ieph = i;
                    break;
                }
            }
    if (s->ieph == -1) {
        rc = gss_fail(GSS_E_INPUT, "ERROR: No current set of ephemerides has been found.");
        goto fail;
    }

    /* ---- channels (gpssim.c:2117-2143) ---- */
    for (int i = 0; i < K_MAX_CHAN; i++) {
        s->chan[i].prn = 0;
        s->chan[i].last_row = -1;
    }
    for (int sv = 0; sv < K_MAX_SAT; sv++)
        s->alloc_sat[sv] = -1;
    s->grx = gt_add(g0, 0.0);
    rc = allocate_channels(s, s->eph[s->ieph], s->grx, s->xyz[0]);
    if (rc < 0)
        goto fail;
    print_channels(s);
    for (int i = 0; i < 37; i++)
        s->ant_pat[i] = pow(10.0, -gss_ant_pat_db[i] / 20.0);

    s->grx = gt_add(s->grx, 0.1);
    s->iumd = 1;
    s->carr_known = 1;              /* every slot's chain starts with a reset at block 0 */
    *out = s;
    return 0;
fail:
    gss_scn_close(s);
    return rc;
}

int gss_scn_info(const gss_scn *s, gss_scn_info_t *info)
{
    if (s == NULL || info == NULL)
        return gss_fail(GSS_E_ARG, "null argument");
    info->n_per_blk = s->n_per_blk;
    info->n_blocks = s->numd > 1 ? s->numd - 1 : 0;
    info->data_format = s->opt.data_format;
    info->samp_freq = s->samp_freq;
    info->delt = s->delt;
    info->week = s->g0.week;
    info->sec = s->g0.sec;
    info->next_block = s->iumd - 1;
    info->rows_out = s->rows_out;
    info->carrier_int = s->opt.carrier_int;
    return 0;
}

/* ---- exact carrier planner ------------------------------------------------------------------
 * One chain per channel slot; a slot's chain restarts whenever allocateChannel re-initialises
 * its carr_phase.  Slots are independent, so the planner runs one slot per thread. */
/* The integer carrier (FLOAT_CARR_PHASE undefined): carr_phase += carr_phasestep per sample in
   a uint32 whose bits 16..24 index the LUT (gpssim.c:2202, 2252), i.e. a chain mod 2^25.  Rows
   carry it as multiples of 2^-25 cycle; n steps from x is (x + n step) mod 1, exactly. */
static double carr_int_walk(double x, double step, int n, double *ck)
{
    const uint32_t xi = (uint32_t)(x * K_CARR_INT_ONE);
    const int64_t si = (int64_t)(step * K_CARR_INT_ONE);
    if (ck)
        for (int j = 0; j < GSS_NCK; j++)
            ck[j] = (double)((xi + (uint32_t)(si * gss_ck_pos(j, n))) & 0x1FFFFFFu) /
                    K_CARR_INT_ONE;
    return (double)((xi + (uint32_t)(si * n)) & 0x1FFFFFFu) / K_CARR_INT_ONE;
}

typedef struct {
    double *carr;
    gss_chan_blk_t *blk;
    const int32_t *nch;
    const gss_chain_t *chain;
    double *ck;
    int nblk, n_per_blk, carrier_int, slot_lo, slot_hi;
} plan_job;

static void *plan_slots(void *arg)
{
    plan_job *j = arg;
    for (int slot = j->slot_lo; slot < j->slot_hi; slot++) {
        double x = j->carr[slot];
        for (int b = 0; b < j->nblk; b++) {
            for (int k = 0; k < j->nch[b]; k++) {
                size_t e = (size_t)b * GSS_MAXCH + k;
                if (j->chain[e].slot != slot)
                    continue;
                if (j->chain[e].reset)
                    x = j->chain[e].init;
                j->blk[e].carr0 = x;
                if (j->carrier_int)        /* exact integer chain, checkpoints included */
                    x = carr_int_walk(x, j->blk[e].carr_step, j->n_per_blk,
                                      j->ck ? j->ck + e * GSS_NCK : NULL);
                else if (j->ck) /* same walk, recording the sub-block checkpoints on the way */
                    x = gss_carr_walk_ck(x, j->blk[e].carr_step, j->n_per_blk,
                                         j->ck + e * GSS_NCK);
                else
                    x = gss_carr_walk_cc(x, j->blk[e].carr_step, j->n_per_blk);
                break;
            }
        }
        j->carr[slot] = x;
    }
    return NULL;
}

static void plan_slot_part(void *arg, int slot)
{
    plan_job j = *(const plan_job *)arg;
    j.slot_lo = slot;
    j.slot_hi = slot + 1;
    (void)plan_slots(&j);
}

/* The carrier chain (gpssim.c:2245-2250, carried across blocks) over nblk consecutive blocks:
   one chain per channel slot, restarted where allocateChannel re-initialised it; slots are
   independent, so one slot per thread. */
int gss_carr_chain(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                   const gss_chain_t *chain, int nblk, int n_per_blk, int carrier_int,
                   double *carr_ck, int threads)
{
    if (carr == NULL || (nblk > 0 && (blk == NULL || nch == NULL || chain == NULL)) ||
        nblk < 0 || n_per_blk <= 0)
        return gss_fail(GSS_E_ARG, "invalid carrier-chain arguments");
    const plan_job all = {carr, blk, nch, chain, carr_ck, nblk, n_per_blk, carrier_int, 0,
                          K_MAX_CHAN};
    gss_pool_run(threads, K_MAX_CHAN, plan_slot_part, (void *)&all);   /* one part per slot */
    return 0;
}

/* ---- the chain with the block walks run ahead (gss_phase.h, speculative block walk) ---------- */
typedef struct {
    const gss_chan_blk_t *blk;
    int n_per_blk;
    gss_spec_in_t *in;
} guess_job;

static void guess_part(void *arg, int b)
{
    const guess_job *j = arg;
    for (int k = 0; k < GSS_MAXCH; k++) {
        gss_spec_in_t *r = &j->in[(size_t)b * GSS_MAXCH + k];
        if (r->k == 0)
            gss_spec_guess_row(r->g, r->s, j->n_per_blk, r);
    }
}

/* the starts, serially: the line of each slot from its exact start (in double: the drift over a
   batch, ~1e-13 per block, stays far inside the translation intervals); k = 0 on live rows (their
   segment starts not guessed yet), 1 on padding rows; pad = the index of the previous row of the
   same slot chain in the batch (-1: the slot's first row here, or a re-initialisation), which the
   records' links read (gss_spec_records*) */
static void chain_starts(const double *carr, const gss_chan_blk_t *blk, const int32_t *nch,
                         const gss_chain_t *chain, int nblk, int n_per_blk, gss_spec_in_t *in)
{
    double run[K_MAX_CHAN];
    int32_t last[K_MAX_CHAN];
    for (int i = 0; i < K_MAX_CHAN; i++) {
        run[i] = carr[i];
        last[i] = -1;
    }
    for (int b = 0; b < nblk; b++)
        for (int k = 0; k < GSS_MAXCH; k++) {
            const size_t e = (size_t)b * GSS_MAXCH + k;
            const int slot = k < nch[b] ? chain[e].slot : -1;
            in[e].k = 1;
            in[e].pad = -1;
            in[e].s = 0.0;
            in[e].g = 0.0;
            if (slot < 0 || slot >= K_MAX_CHAN)
                continue;
            if (chain[e].reset) {
                run[slot] = chain[e].init;
                last[slot] = -1;
            }
            in[e].pad = last[slot];
            last[slot] = (int32_t)e;
            const double g = run[slot];
            in[e].g = g >= 0.0 && g < 1.0 ? g : 0.0;
            in[e].s = blk[e].carr_step;
            in[e].k = 0;
            const double v = g + (double)n_per_blk * blk[e].carr_step;
            run[slot] = v - floor(v);
        }
}

/* The slots' carriers after the batch, predicted by the same lines (a start for the batch after
   it while its own chain is still pending: ~3e-10 cycle off after 2,048 blocks, far inside the
   translation intervals) */
int gss_carr_line_end(const double *carr, const gss_chan_blk_t *blk, const int32_t *nch,
                      const gss_chain_t *chain, int nblk, int n_per_blk, double *carr_end)
{
    if (carr == NULL || carr_end == NULL || nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (blk == NULL || nch == NULL || chain == NULL)))
        return gss_fail(GSS_E_ARG, "invalid carrier-line arguments");
    double run[K_MAX_CHAN];
    for (int i = 0; i < K_MAX_CHAN; i++)
        run[i] = carr[i];
    for (int b = 0; b < nblk; b++)
        for (int k = 0; k < nch[b] && k < GSS_MAXCH; k++) {
            const size_t e = (size_t)b * GSS_MAXCH + k;
            const int slot = chain[e].slot;
            if (slot < 0 || slot >= K_MAX_CHAN)
                continue;
            if (chain[e].reset)
                run[slot] = chain[e].init;
            const double v = run[slot] + (double)n_per_blk * blk[e].carr_step;
            run[slot] = v - floor(v);
        }
    for (int i = 0; i < K_MAX_CHAN; i++)
        carr_end[i] = run[i];
    return 0;
}

int gss_carr_chain_starts(const double *carr, const gss_chan_blk_t *blk, const int32_t *nch,
                          const gss_chain_t *chain, int nblk, int n_per_blk, gss_spec_in_t *in)
{
    if (carr == NULL || in == NULL || nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (blk == NULL || nch == NULL || chain == NULL)))
        return gss_fail(GSS_E_ARG, "invalid carrier-guess arguments");
    chain_starts(carr, blk, nch, chain, nblk, n_per_blk, in);
    return 0;
}

int gss_carr_chain_guess(const double *carr, const gss_chan_blk_t *blk, const int32_t *nch,
                         const gss_chain_t *chain, int nblk, int n_per_blk, gss_spec_in_t *in)
{
    if (carr == NULL || in == NULL || nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (blk == NULL || nch == NULL || chain == NULL)))
        return gss_fail(GSS_E_ARG, "invalid carrier-guess arguments");
    chain_starts(carr, blk, nch, chain, nblk, n_per_blk, in);
    /* the segment starts, in parallel over blocks */
    const guess_job j = {blk, n_per_blk, in};
    gss_pool_run(8, nblk, guess_part, (void *)&j);
    return 0;
}

typedef struct {
    gss_spec_in_t *in;
    int nrow, n_per_blk;
    gss_spec_t *spec;
} spec_host_job;

static void spec_host_part(void *arg, int part)
{
    const spec_host_job *j = arg;
    for (int i = part * 16; i < j->nrow && i < part * 16 + 16; i++) {
        if (j->in[i].k == 0)                     /* segment starts not guessed yet */
            gss_spec_guess_row(j->in[i].g, j->in[i].s, j->n_per_blk, &j->in[i]);
        for (int g = 0; g < j->in[i].k && g < GSS_SPEC_K; g++)
            gss_spec_seg_walk(&j->in[i], g, j->n_per_blk, &j->spec[i]);
    }
}

int gss_spec_host(gss_spec_in_t *in, int nrow, int n_per_blk, gss_spec_t *spec, int threads)
{
    if (nrow < 0 || n_per_blk <= 0 || (nrow > 0 && (in == NULL || spec == NULL)))
        return gss_fail(GSS_E_ARG, "invalid speculative-walk arguments");
    const spec_host_job j = {in, nrow, n_per_blk, spec};
    gss_pool_run(threads, (nrow + 15) / 16, spec_host_part, (void *)&j);
    return 0;
}

typedef struct {
    double *carr;
    gss_chan_blk_t *blk;
    const int32_t *nch;
    const gss_chain_t *chain;
    const gss_spec_in_t *in;
    const gss_spec_t *spec;
    gss_carr_anchor_t *anch;
    int nblk, n_per_blk;
    int hits[K_MAX_CHAN];
} spec_chain_job;

/* one row's end from its true start x; with a != NULL its anchors: the start, and the exact value
   at every segment start the fix-up passed or walked */
static double fix_row(double x, int n, const gss_spec_in_t *in, const gss_spec_t *o, int *hit,
                      double *d, gss_carr_anchor_t *a)
{
    if (a == NULL)
        return gss_spec_fix_d(x, n, in, o, hit, d, NULL);
    double av[GSS_SPEC_K];
    for (int j = 0; j < GSS_SPEC_K; j++)
        av[j] = -1.0;                                /* a carrier value is never negative */
    const double end = gss_spec_fix_d(x, n, in, o, hit, d, av);
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    a->pos[0] = 0;
    a->val[0] = x;
    for (int j = 1; j < GSS_SPEC_K; j++) {
        const int ok = j < k && av[j] >= 0.0 && in->P[j] > 0 && in->P[j] < n;
        a->pos[j] = ok ? (int32_t)in->P[j] : -1;
        a->val[j] = ok ? av[j] : 0.0;
    }
    return end;
}

static void spec_slot_part(void *arg, int slot)
{
    spec_chain_job *j = arg;
    double x = j->carr[slot], d = 0.0;
    int hits = 0;
    for (int b = 0; b < j->nblk; b++)
        for (int k = 0; k < j->nch[b]; k++) {
            const size_t e = (size_t)b * GSS_MAXCH + k;
            if (j->chain[e].slot != slot)
                continue;
            if (j->chain[e].reset)
                x = j->chain[e].init;
            j->blk[e].carr0 = x;
            int hit = 0;
            x = fix_row(x, j->n_per_blk, &j->in[e], &j->spec[e], &hit, &d,
                        j->anch ? &j->anch[e] : NULL);
            hits += hit;
            break;
        }
    j->carr[slot] = x;
    j->hits[slot] = hits;
}

static void anchors_none(gss_carr_anchor_t *anch, const int32_t *nch, int nblk)
{
    for (int b = 0; b < nblk; b++)
        for (int k = 0; k < GSS_MAXCH; k++) {
            gss_carr_anchor_t *a = &anch[(size_t)b * GSS_MAXCH + k];
            for (int j = 0; j < GSS_SPEC_K; j++) {
                a->pos[j] = -1;
                a->val[j] = 0.0;
            }
        }
    (void)nch;
}

int gss_carr_chain_anchored(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                            const gss_chain_t *chain, int nblk, int n_per_blk,
                            const gss_spec_in_t *in, const gss_spec_t *spec, int threads,
                            int *n_hit, gss_carr_anchor_t *anch)
{
    if (carr == NULL || nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (blk == NULL || nch == NULL || chain == NULL || in == NULL || spec == NULL)))
        return gss_fail(GSS_E_ARG, "invalid carrier-chain arguments");
    if (anch)
        anchors_none(anch, nch, nblk);                /* padding rows: none */
    spec_chain_job j = {carr, blk, nch, chain, in, spec, anch, nblk, n_per_blk, {0}};
    gss_pool_run(threads, K_MAX_CHAN, spec_slot_part, (void *)&j);   /* one part per slot */
    if (n_hit) {
        int h = 0;
        for (int i = 0; i < K_MAX_CHAN; i++)
            h += j.hits[i];
        *n_hit = h;
    }
    return 0;
}

int gss_carr_chain_spec(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                        const gss_chain_t *chain, int nblk, int n_per_blk,
                        const gss_spec_in_t *in, const gss_spec_t *spec, int threads,
                        int *n_hit)
{
    return gss_carr_chain_anchored(carr, blk, nch, chain, nblk, n_per_blk, in, spec, threads,
                                   n_hit, NULL);
}

/* anchors of rows whose carr0 the chain has set (any chain): in parallel over blocks */
typedef struct {
    const gss_chan_blk_t *blk;
    const int32_t *nch;
    const gss_spec_in_t *in;
    const gss_spec_t *spec;
    gss_carr_anchor_t *anch;
    int n_per_blk;
} anchor_job;

static void anchor_part(void *arg, int b)
{
    const anchor_job *j = arg;
    for (int k = 0; k < j->nch[b] && k < GSS_MAXCH; k++) {
        const size_t e = (size_t)b * GSS_MAXCH + k;
        gss_spec_anchors(j->blk[e].carr0, j->n_per_blk, &j->in[e], &j->spec[e],
                         j->anch[e].pos, j->anch[e].val);
    }
}

int gss_carr_anchors(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                     const gss_spec_in_t *in, const gss_spec_t *spec, gss_carr_anchor_t *anch,
                     int threads)
{
    if (nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (blk == NULL || nch == NULL || in == NULL || spec == NULL || anch == NULL)))
        return gss_fail(GSS_E_ARG, "invalid carrier-anchor arguments");
    anchors_none(anch, nch, nblk);
    const anchor_job j = {blk, nch, in, spec, anch, n_per_blk};
    gss_pool_run(threads, nblk, anchor_part, (void *)&j);
    return 0;
}

/* ---- links between a slot's consecutive rows (gss_spec_links / gss_carr_chain_linked) --------
 * Where row e' of a slot translated by d (its end = its last segment's end + d), the next row e of
 * the slot starts at y + d, y = that segment's end: known before the chain runs.  So e's partial
 * cycle to its first wrap is walked from y ahead of time with the admissible translations of y,
 * and e's whole walk folds into one record: e translates iff d is in [lo, hi], and then its own
 * last translation is d + dd and its end is end + (d + dd).  Exact: every translation the record
 * chains (d_0 = d + (w1' - w1), d_j+1 = d_j + (end_j - W_j+1)) is a sum of post-wrap lattice
 * values (multiples of 2^-52 ascending, 2^-53 descending, below 2 in magnitude), so the double
 * arithmetic carries it exactly, and the bounds lo_j - c_j are rounded inward. */
typedef struct {
    const int32_t *nch;
    const gss_chain_t *chain;
    const gss_spec_in_t *in;
    const gss_spec_t *spec;
    gss_spec_link_t *link;
    int nblk, n_per_blk;
} link_job;

/* the record of row e entered from y (the previous row's last segment end); 0: none */
static int link_row(double y, const gss_spec_in_t *in, const gss_spec_t *o, int64_t n,
                    gss_spec_link_t *L)
{
    double lo, hi, dd;
    if (!gss_spec_link_fold(y, in, o, n, &lo, &hi, &dd))
        return 0;
    L->lo = lo;
    L->hi = hi;
    L->dd = dd;
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    L->end = o->seg[k - 1].end;
    return 1;
}

static void link_slot_part(void *arg, int slot)
{
    const link_job *j = arg;
    int64_t prev = -1;
    for (int b = 0; b < j->nblk; b++)
        for (int k = 0; k < j->nch[b]; k++) {
            const size_t e = (size_t)b * GSS_MAXCH + k;
            if (j->chain[e].slot != slot)
                continue;
            gss_spec_link_t *L = &j->link[e];
            L->lo = 1.0;                          /* an empty interval: no record */
            L->hi = 0.0;
            L->dd = L->end = 0.0;
            if (prev >= 0 && !j->chain[e].reset && j->in[e].s != 0.0 && j->in[prev].s != 0.0) {
                const gss_spec_in_t *pi = &j->in[prev];
                const int kp = pi->k < 1 ? 1 : (pi->k > GSS_SPEC_K ? GSS_SPEC_K : pi->k);
                if (!link_row(j->spec[prev].seg[kp - 1].end, &j->in[e], &j->spec[e],
                              j->n_per_blk, L)) {
                    L->lo = 1.0;
                    L->hi = 0.0;
                }
            }
            prev = (int64_t)e;
            break;
        }
}

int gss_spec_links(const int32_t *nch, const gss_chain_t *chain, int nblk, int n_per_blk,
                   const gss_spec_in_t *in, const gss_spec_t *spec, gss_spec_link_t *link,
                   int threads)
{
    if (nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (nch == NULL || chain == NULL || in == NULL || spec == NULL || link == NULL)))
        return gss_fail(GSS_E_ARG, "invalid spec-link arguments");
    for (size_t e = 0; e < (size_t)nblk * GSS_MAXCH; e++) {
        link[e].lo = 1.0;
        link[e].hi = 0.0;
        link[e].dd = link[e].end = 0.0;
    }
    const link_job j = {nch, chain, in, spec, link, nblk, n_per_blk};
    gss_pool_run(threads, K_MAX_CHAN, link_slot_part, (void *)&j);      /* one part per slot */
    return 0;
}

typedef struct {
    double *carr;
    gss_chan_blk_t *blk;
    const int32_t *nch;
    const gss_chain_t *chain;
    const gss_spec_in_t *in;
    const gss_spec_t *spec;
    const gss_spec_link_t *link;
    int nblk, n_per_blk;
    int hits[K_MAX_CHAN];
} linked_job;

static void linked_slot_part(void *arg, int slot)
{
    linked_job *j = arg;
    double x = j->carr[slot], d = 0.0;
    int hits = 0, held = 0;
    for (int b = 0; b < j->nblk; b++)
        for (int k = 0; k < j->nch[b]; k++) {
            const size_t e = (size_t)b * GSS_MAXCH + k;
            if (j->chain[e].slot != slot)
                continue;
            if (j->chain[e].reset) {
                x = j->chain[e].init;
                held = 0;
            }
            j->blk[e].carr0 = x;
            const gss_spec_link_t *L = &j->link[e];
            int hit = 0;
            if (held && d >= L->lo && d <= L->hi) {
                d += L->dd;
                x = L->end + d;
                hit = 1;
            } else {
                x = gss_spec_fix_d(x, j->n_per_blk, &j->in[e], &j->spec[e], &hit, &d, NULL);
            }
            held = hit;
            hits += hit;
            break;
        }
    j->carr[slot] = x;
    j->hits[slot] = hits;
}

int gss_carr_chain_linked(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                          const gss_chain_t *chain, int nblk, int n_per_blk,
                          const gss_spec_in_t *in, const gss_spec_t *spec,
                          const gss_spec_link_t *link, int threads, int *n_hit)
{
    if (carr == NULL || nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (blk == NULL || nch == NULL || chain == NULL || in == NULL || spec == NULL ||
                      link == NULL)))
        return gss_fail(GSS_E_ARG, "invalid carrier-chain arguments");
    linked_job j = {carr, blk, nch, chain, in, spec, link, nblk, n_per_blk, {0}};
    gss_pool_run(threads, K_MAX_CHAN, linked_slot_part, (void *)&j);
    if (n_hit) {
        int h = 0;
        for (int i = 0; i < K_MAX_CHAN; i++)
            h += j.hits[i];
        *n_hit = h;
    }
    return 0;
}

/* ---- records: each row's walk folded (gss_phase.h gss_spec_record), the chain from them ------- */
typedef struct {
    const gss_spec_in_t *in;
    const gss_spec_t *spec;
    gss_spec_rec_t *rec;
    int nrow, n_per_blk;
} rec_job;

static void rec_part(void *arg, int part)
{
    const rec_job *j = arg;
    for (int i = part * 64; i < j->nrow && i < part * 64 + 64; i++) {
        const int p = j->in[i].pad;
        const int ok = p >= 0 && p < i;
        gss_spec_record(&j->in[i], &j->spec[i], ok ? &j->in[p] : NULL, ok ? &j->spec[p] : NULL,
                        j->n_per_blk, &j->rec[i]);
        if (j->rec[i].ok & 2)
            j->rec[i].ok |= (i - p) << 2;            /* the row the link was built against */
    }
}

int gss_spec_records(const gss_spec_in_t *in, const gss_spec_t *spec, int nrow, int n_per_blk,
                     gss_spec_rec_t *rec, int threads)
{
    if (nrow < 0 || n_per_blk <= 0 || (nrow > 0 && (in == NULL || spec == NULL || rec == NULL)))
        return gss_fail(GSS_E_ARG, "invalid spec-record arguments");
    const rec_job j = {in, spec, rec, nrow, n_per_blk};
    gss_pool_run(threads, (nrow + 63) / 64, rec_part, (void *)&j);
    return 0;
}

typedef struct {
    double *carr;
    gss_chan_blk_t *blk;
    const int32_t *nch;
    const gss_chain_t *chain;
    const gss_spec_rec_t *rec;
    int nblk, n_per_blk;
    int hits[K_MAX_CHAN];
} rec_chain_job;

static void rec_slot_part(void *arg, int slot)
{
    rec_chain_job *j = arg;
    const int64_t n = j->n_per_blk;
    double x = j->carr[slot], d = 0.0;
    int hits = 0, held = 0;
    size_t e_prev = 0;                               /* the slot's previous row (held: valid) */
    for (int b = 0; b < j->nblk; b++)
        for (int k = 0; k < j->nch[b]; k++) {
            const size_t e = (size_t)b * GSS_MAXCH + k;
            if (j->chain[e].slot != slot)
                continue;
            if (j->chain[e].reset) {
                x = j->chain[e].init;
                held = 0;
            }
            j->blk[e].carr0 = x;
            const gss_spec_rec_t *R = &j->rec[e];
            /* a link record holds only if it was built against this slot's previous row
               (ok bits 2.., the row distance; rows from elsewhere, e.g. zero-filled pads, fail
               the check and walk) */
            const int linked = held && (R->ok & 2) && (size_t)(R->ok >> 2) == e - e_prev;
            e_prev = e;
            if (linked && d >= R->llo && d <= R->lhi) {
                d += R->ldd;                         /* the link: no walk at all */
                x = R->end + d;
                hits++;
                break;
            }
            const double s = j->blk[e].carr_step;
            double v = x;
            int wr = 0;
            const int64_t t = gss_carr_to_wrap(&v, s, n, &wr);
            held = 0;
            if (!wr || t >= n) {
                x = v;                               /* no wrap: walked exactly */
            } else if ((R->ok & 1) && t == R->p1 && v - R->w1 >= R->slo && v - R->w1 <= R->shi) {
                d = (v - R->w1) + R->sdd;            /* the row's own record */
                x = R->end + d;
                held = 1;
                hits++;
            } else {
                x = gss_carr_walk_cc(v, s, n - t);   /* a translation fails: the exact walk */
            }
            break;
        }
    j->carr[slot] = x;
    j->hits[slot] = hits;
}

int gss_carr_chain_records(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                           const gss_chain_t *chain, int nblk, int n_per_blk,
                           const gss_spec_rec_t *rec, int threads, int *n_hit)
{
    if (carr == NULL || nblk < 0 || n_per_blk <= 0 ||
        (nblk > 0 && (blk == NULL || nch == NULL || chain == NULL || rec == NULL)))
        return gss_fail(GSS_E_ARG, "invalid carrier-chain arguments");
    rec_chain_job j = {carr, blk, nch, chain, rec, nblk, n_per_blk, {0}};
    gss_pool_run(threads, K_MAX_CHAN, rec_slot_part, (void *)&j);
    if (n_hit) {
        int h = 0;
        for (int i = 0; i < K_MAX_CHAN; i++)
            h += j.hits[i];
        *n_hit = h;
    }
    return 0;
}

/* ---- per-block ranges in parallel --------------------------------------------------------------
 * The per-block refresh (gpssim.c:2156-2188) needs computeRange for every active channel of
 * every block, and block b only uses its own range and block b-1's.  Between two 30 s updates the
 * channel set, the ephemeris set and the receiver positions are fixed, so the ranges of a run of
 * blocks up to the next update are independent: threads compute them (range_pass), then the
 * blocks' refreshes, again in parallel (next_rows). */
typedef struct {
    const gss_scn *s;
    const gtime_t *g;                       /* [j] receiver time of block j of the run */
    int j0, nj, jstep;
    int iumd0;
} range_job;

static void *range_worker(void *arg)
{
    range_job *r = arg;
    const gss_scn *s = r->s;
    for (int j = r->j0; j < r->nj; j += r->jstep) {
        const double *xyz = s->static_mode ? s->xyz[0] : s->xyz[r->iumd0 + j];
        double llh[3], tmat[3][3];                   /* the receiver's frame, once per block */
        ecef_to_llh(xyz, llh);
        enu_matrix(llh, tmat);
        for (int i = 0; i < K_MAX_CHAN; i++) {
            const chan_t *ch = &s->chan[i];
            if (ch->prn > 0)
                sv_range_at(&s->rg[(size_t)j * K_MAX_CHAN + i], &s->eph[s->ieph][ch->prn - 1],
                            &s->io, r->g[j], xyz, llh, tmat);
        }
    }
    return NULL;
}

static void range_part(void *arg, int j)
{
    range_job r = *(const range_job *)arg;
    r.j0 = j;
    r.nj = j + 1;
    (void)range_worker(&r);
}

/* blocks of the run from the current one that share its channel set (the last is the one after
   which the 30 s update runs), at most max_j; their ranges into s->rg */
static int range_pass(gss_scn *s, int max_j, int threads)
{
    gtime_t gbuf[300 + 1];
    int nj = 0;
    gtime_t g = s->grx;
    while (nj < max_j && nj < 300 && s->iumd + nj < s->numd) {
        gbuf[nj++] = g;
        if ((int)(g.sec * 10.0 + 0.5) % 300 == 0)
            break;
        g = gt_add(g, 0.1);
    }
    if (nj > s->rg_cap) {
        free(s->rg);
        s->rg = malloc((size_t)nj * K_MAX_CHAN * sizeof(rng_t));
        if (s->rg == NULL) {
            s->rg_cap = 0;
            return gss_fail(GSS_E_NOMEM, "out of memory");
        }
        s->rg_cap = nj;
    }
    const range_job all = {s, gbuf, 0, nj, 1, s->iumd};
    gss_pool_run(threads, nj, range_part, (void *)&all);      /* one part per block */
    return nj;
}

/* The 30 s update after the block at s->grx (gpssim.c:2294-2345): nav message, ephemeris set,
   allocation.  push_nav: append the new dwrd to the nav table (not while seeking). */
static int update_30s(gss_scn *s, const double *xyz, int push_nav)
{
    for (int i = 0; i < K_MAX_CHAN; i++)
        if (s->chan[i].prn > 0) {
            nav_frame(s->grx, &s->chan[i], 0);
            if (push_nav) {
                int rc = nav_push(s, &s->chan[i]);
                if (rc)
                    return rc;
            }
        }
    /* step to the next ephemeris set when its TOC is < 1 h away; only the first valid SV of that
       set is tested (gpssim.c:2307-2326).  New subframes reach dwrd at the next 30 s update. */
    for (int sv = 0; sv < K_MAX_SAT; sv++) {
        if (s->eph[s->ieph + 1][sv].vflg == 1) {
            double dt = gt_diff(s->eph[s->ieph + 1][sv].toc, s->grx);
            if (dt < K_SEC_HOUR) {
                s->ieph++;
                for (int i = 0; i < K_MAX_CHAN; i++)
                    if (s->chan[i].prn != 0)
                        nav_subframes(&s->eph[s->ieph][s->chan[i].prn - 1], &s->io,
                                      s->chan[i].sbf);
            }
            break;
        }
    }
    int rc = allocate_channels(s, s->eph[s->ieph], s->grx, xyz);
    if (rc < 0)
        return rc;
    if (push_nav && s->opt.verbose) {
        msg(s, "\n");
        print_channels(s);
    }
    return 0;
}

/* The per-block refresh of one channel (gpssim.c:2156-2188) from its range at the block (rho)
   and at the block before (rho_prev): the row, and in *c the channel state the serial loop of
   the reference leaves behind (azel, Doppler, code state, rho0). */
typedef struct {
    double azel[2], f_carr, f_code, code_phase;
    int iword, ibit, icode;
} refresh_state;

static void refresh_row(const gss_scn *s, const chan_t *ch, const rng_t *rho_prev,
                        const rng_t *rho_p, gss_chan_blk_t *p, refresh_state *st)
{
    const rng_t rho = *rho_p;                  /* sv_range at the block's time (range_pass) */
    st->azel[0] = rho.azel[0];
    st->azel[1] = rho.azel[1];

    /* computeCodePhase(chan, rho, 0.1), gpssim.c:1317-1351 */
    double rhorate = (rho.range - rho_prev->range) / 0.1;
    st->f_carr = -rhorate / K_LAMBDA_L1;
    st->f_code = K_CODE_FREQ + st->f_carr * K_CARR_TO_CODE;
    double ms = ((gt_diff(rho_prev->g, ch->g0) + 6.0) - rho_prev->range / K_C) * 1000.0;
    int ims = (int)ms;
    st->code_phase = (ms - (double)ims) * K_CA_LEN;
    st->iword = ims / 600;
    ims -= st->iword * 600;
    st->ibit = ims / 20;
    ims -= st->ibit * 20;
    st->icode = ims;

    /* gain: path loss × antenna pattern, scaled 2^7 (gpssim.c:2179-2186) */
    double path_loss = 20200000.0 / rho.d;
    int ibs = (int)((90.0 - rho.azel[1] * K_R2D) / 5.0);
    double ant_gain = s->ant_pat[ibs];
    int gain = (int)(path_loss * ant_gain * 128.0);

    p->carr0 = 0.0;                            /* filled by the carrier chain */
    p->carr_step = st->f_carr * s->delt;
    if (s->opt.carrier_int)                    /* carr_phasestep (gpssim.c:2175-2177) */
        p->carr_step = (double)(int)round(512.0 * 65536.0 * st->f_carr * s->delt) /
                       K_CARR_INT_ONE;
    p->code0 = st->code_phase;
    p->code_step = st->f_code * s->delt;
    p->icode = st->icode;
    p->ibit = st->ibit;
    p->iword = st->iword;
    p->gain = gain;
    p->ca_tbl = ch->prn - 1;
    p->nav_tbl = ch->nav_row;
}

/* the rows of a range pass's blocks in parallel: block j's refresh needs only its range and
   block j - 1's (the pass's first block: the channel's rho0 before the pass), and the channel set
   is fixed between two 30 s updates, which end a pass */
typedef struct {
    const gss_scn *s;
    gss_chan_blk_t *blk;
    int32_t *nch;
    gss_chain_t *chain;
    double *carr_ck;
    const rng_t *rho_start;                    /* [K_MAX_CHAN] rho0 before the pass */
    const int *fresh;                          /* [K_MAX_CHAN] carr_fresh before the pass */
} refresh_job;

static void refresh_part(void *arg, int j)
{
    const refresh_job *r = (const refresh_job *)arg;
    const gss_scn *s = r->s;
    gss_chan_blk_t *row = r->blk + (size_t)j * GSS_MAXCH;
    gss_chain_t *cr = r->chain + (size_t)j * GSS_MAXCH;
    const rng_t *rg = s->rg + (size_t)j * K_MAX_CHAN;
    int k = 0;
    for (int i = 0; i < K_MAX_CHAN; i++) {
        const chan_t *ch = &s->chan[i];
        if (ch->prn <= 0)
            continue;
        refresh_state st;
        refresh_row(s, ch, j ? &rg[i - K_MAX_CHAN] : &r->rho_start[i], &rg[i], &row[k], &st);
        gss_chain_t *c = &cr[k];
        memset(c, 0, sizeof *c);
        c->slot = (int8_t)i;
        c->reset = (uint8_t)(j == 0 ? r->fresh[i] : 0);
        c->init = ch->carr_phase;
        k++;
    }
    for (int q = k; q < GSS_MAXCH; q++) {
        memset(&row[q], 0, sizeof row[q]);
        memset(&cr[q], 0, sizeof cr[q]);
        cr[q].slot = -1;
    }
    if (r->carr_ck)                            /* padding rows: defined (zero) checkpoints */
        memset(r->carr_ck + ((size_t)j * GSS_MAXCH + k) * GSS_NCK, 0,
               sizeof(double) * GSS_NCK * (GSS_MAXCH - k));
    r->nch[j] = k;
}

/* Rows of the next blocks without their carrier phase (carr0 = 0): the per-block refresh and the
   30 s updates of gpssim.c:2154-2352; chain[] records which slot chain each row continues.
   Per range pass (the blocks up to the next 30 s update): the ranges, then the rows, each in
   parallel over the pass's blocks; the channel state is then left as the reference's serial
   loop leaves it (its last block's refresh), and the 30 s update runs after the pass. */
static int next_rows(gss_scn *s, int max_blocks, gss_chan_blk_t *blk, int32_t *nch,
                     gss_chain_t *chain, double *carr_ck, int *n_out, int threads)
{
    int nb = 0;
    while (nb < max_blocks && s->iumd < s->numd) {
        const int nr = range_pass(s, max_blocks - nb, threads);
        if (nr < 0)
            return nr;
        if (nr == 0)
            break;
        rng_t rho_start[K_MAX_CHAN];
        int fresh[K_MAX_CHAN];
        for (int i = 0; i < K_MAX_CHAN; i++) {
            rho_start[i] = s->chan[i].rho0;
            fresh[i] = s->chan[i].carr_fresh;
        }
        const refresh_job rj = {s, blk + (size_t)nb * GSS_MAXCH, nch + nb,
                                chain + (size_t)nb * GSS_MAXCH,
                                carr_ck ? carr_ck + (size_t)nb * GSS_MAXCH * GSS_NCK : NULL,
                                rho_start, fresh};
        gss_pool_run(threads, nr, refresh_part, (void *)&rj);
        /* the channel state after the pass's last block, as the serial loop leaves it */
        const rng_t *last = s->rg + (size_t)(nr - 1) * K_MAX_CHAN;
        for (int i = 0; i < K_MAX_CHAN; i++) {
            chan_t *ch = &s->chan[i];
            if (ch->prn <= 0)
                continue;
            gss_chan_blk_t scratch;
            refresh_state st;
            refresh_row(s, ch, nr > 1 ? &last[i - K_MAX_CHAN] : &rho_start[i], &last[i], &scratch,
                        &st);
            ch->azel[0] = st.azel[0];
            ch->azel[1] = st.azel[1];
            ch->f_carr = st.f_carr;
            ch->f_code = st.f_code;
            ch->code_phase = st.code_phase;
            ch->iword = st.iword;
            ch->ibit = st.ibit;
            ch->icode = st.icode;
            ch->rho0 = last[i];
            ch->carr_fresh = 0;
        }
        for (int j = 0; j < nr; j++) {
            const double *xyz = s->static_mode ? s->xyz[0] : s->xyz[s->iumd];
            /* ---- 30 s update: nav message, ephemeris set, allocation (gpssim.c:2294-2345);
               range_pass ends a pass at it, so only its last block can reach one ---- */
            int igrx = (int)(s->grx.sec * 10.0 + 0.5);
            if (igrx % 300 == 0) {
                if (j != nr - 1)
                    return gss_fail(GSS_E_STATE, "30 s update inside a range pass");
                int rc = update_30s(s, xyz, 1);
                if (rc)
                    return rc;
            }
            s->grx = gt_add(s->grx, 0.1);
            msg(s, "\rTime into run = %4.1f", gt_diff(s->grx, s->g0));
            s->iumd++;
        }
        nb += nr;
    }
    s->rows_out += nb;
    *n_out = nb;
    return 0;
}

int gss_scn_next_deferred(gss_scn *s, int max_blocks, gss_chan_blk_t *blk, int32_t *nch,
                          gss_chain_t *chain, int *n_out, int threads)
{
    *n_out = 0;
    if (s == NULL || blk == NULL || nch == NULL || chain == NULL || max_blocks <= 0)
        return gss_fail(GSS_E_ARG, "invalid argument");
    double t_start = wall_now();
    int rc = next_rows(s, max_blocks, blk, nch, chain, NULL, n_out, threads);
    s->plan_sec += wall_now() - t_start;
    /* the slot carriers (s->carr) still belong to the first of these blocks: gss_scn_next
       refuses to run on them until the chain's end arrives by gss_scn_set_carrier (a run that
       stops early therefore leaves the handle marked, not silently stale) */
    if (*n_out > 0)
        s->carr_known = 0;
    return rc;
}

int gss_scn_next(gss_scn *s, int max_blocks, gss_chan_blk_t *blk, int32_t *nch, double *carr_ck,
                 int *n_out, int threads)
{
    *n_out = 0;
    if (s == NULL || blk == NULL || nch == NULL || max_blocks <= 0)
        return gss_fail(GSS_E_ARG, "invalid argument");
    if (!s->carr_known)
        return gss_fail(GSS_E_STATE, "carrier phases unknown after gss_scn_seek: "
                        "gss_scn_set_carrier first, or use gss_scn_next_deferred");
    double t_start = wall_now();
    if (max_blocks > s->batch_cap) {
        free(s->chain);
        s->chain = malloc((size_t)max_blocks * GSS_MAXCH * sizeof(gss_chain_t));
        if (!s->chain) {
            s->batch_cap = 0;
            return gss_fail(GSS_E_NOMEM, "out of memory");
        }
        s->batch_cap = max_blocks;
    }
    int nb = 0;
    int rc = next_rows(s, max_blocks, blk, nch, s->chain, carr_ck, &nb, threads);
    if (rc == 0)
        rc = gss_carr_chain(s->carr, blk, nch, s->chain, nb, s->n_per_blk, s->opt.carrier_int,
                            carr_ck, threads);
    s->plan_sec += wall_now() - t_start;
    *n_out = rc ? 0 : nb;
    return rc;
}

/* Jump to run block `block` without producing the blocks before it: only the 30 s updates are
   replayed (nav frames, ephemeris steps, allocation: all independent of the per-block refresh),
   plus, for the block just before the target, the ranges that computeCodePhase of the target
   block needs as rho0 (gpssim.c:1324-1348).  The slots' carrier phases are then unknown. */
int gss_scn_seek(gss_scn *s, int64_t block, int threads)
{
    (void)threads;
    if (s == NULL || block < 0)
        return gss_fail(GSS_E_ARG, "invalid seek");
    const int64_t target = block + 1;                 /* iumd of the first block to produce */
    if (target < s->iumd)
        return gss_fail(GSS_E_STATE, "seek backwards (at block %d, asked %lld)", s->iumd - 1,
                        (long long)block);
    if (target > s->numd)
        return gss_fail(GSS_E_ARG, "seek past the end (%d blocks)", s->numd - 1);
    if (target == s->iumd)
        return 0;
    double t_start = wall_now();
    while (s->iumd < target) {
        const double *xyz = s->static_mode ? s->xyz[0] : s->xyz[s->iumd];
        for (int i = 0; i < K_MAX_CHAN; i++) {
            chan_t *ch = &s->chan[i];
            if (ch->prn <= 0)
                continue;
            ch->carr_fresh = 0;              /* the chain started in a skipped block */
            if (s->iumd == target - 1) {     /* rho0 of the target block: this block's range */
                rng_t rho;
                sv_range(&rho, &s->eph[s->ieph][ch->prn - 1], &s->io, s->grx, xyz);
                ch->rho0 = rho;
                ch->azel[0] = rho.azel[0];
                ch->azel[1] = rho.azel[1];
            }
        }
        int igrx = (int)(s->grx.sec * 10.0 + 0.5);
        if (igrx % 300 == 0) {
            int rc = update_30s(s, xyz, 0);
            if (rc)
                return rc;
        }
        s->grx = gt_add(s->grx, 0.1);
        s->iumd++;
    }
    /* the active channels' current words as rows of this handle's nav table */
    for (int i = 0; i < K_MAX_CHAN; i++)
        if (s->chan[i].prn > 0) {
            int rc = nav_push(s, &s->chan[i]);
            if (rc)
                return rc;
        }
    s->carr_known = 0;
    s->plan_sec += wall_now() - t_start;
    return 0;
}

int gss_scn_carrier(const gss_scn *s, double *carr)
{
    if (s == NULL || carr == NULL)
        return gss_fail(GSS_E_ARG, "null argument");
    memcpy(carr, s->carr, sizeof s->carr);
    return 0;
}

int gss_scn_set_carrier(gss_scn *s, const double *carr)
{
    if (s == NULL || carr == NULL)
        return gss_fail(GSS_E_ARG, "null argument");
    memcpy(s->carr, carr, sizeof s->carr);
    s->carr_known = 1;
    return 0;
}

int gss_scn_nav_sources(const gss_scn *s, const gss_nav_src_t **src, int *n_rows)
{
    if (s == NULL || src == NULL || n_rows == NULL)
        return gss_fail(GSS_E_ARG, "invalid nav-source query");
    *src = s->nav_src;
    *n_rows = s->n_nav;
    return 0;
}

int gss_nav_rows_host(const gss_nav_src_t *src, int first, int n, uint32_t *rows)
{
    if ((n > 0 && (src == NULL || rows == NULL)) || first < 0 || n < 0)
        return gss_fail(GSS_E_ARG, "invalid nav-row arguments");
    for (int i = 0; i < n; i++) {
        const gss_nav_src_t *q = &src[i];
        if (q->prev >= first + i || q->prev < GSS_NAV_HEAD_GIVEN)
            return gss_fail(GSS_E_ARG, "nav source %d: prev %d out of order", first + i, q->prev);
        gss_nav_frame(q, gss_nav_head(q, rows), rows + (size_t)(first + i) * GSS_NAV_WORDS);
    }
    return 0;
}

int gss_scn_nav_table(const gss_scn *s, const uint32_t **rows, int *n_rows)
{
    if (s == NULL)
        return gss_fail(GSS_E_ARG, "null scenario");
    *rows = s->nav_rows;
    *n_rows = s->n_nav;
    return 0;
}

double gss_scn_plan_seconds(const gss_scn *s) { return s ? s->plan_sec : 0.0; }

int gss_scn_close(gss_scn *s)
{
    if (s == NULL)
        return 0;
    free(s->xyz);
    free(s->nav_rows);
    free(s->nav_src);
    free(s->chain);
    free(s->rg);
    free(s);
    return 0;
}

/* ---- small exported helpers ----------------------------------------------------------------- */
int gss_ca_table(uint32_t *out)
{
    int8_t ca[K_CA_LEN];
    for (int prn = 1; prn <= 32; prn++) {
        ca_generate(ca, prn);
        ca_pack(ca, out + (size_t)(prn - 1) * GSS_CA_WORDS);
    }
    return 0;
}

double gss_carr_advance(double carr, double step, int64_t n)
{
    return gss_carr_walk_cc(carr, step, n);
}

double gss_carr_advance_ck(double carr, double step, int n, double *ck)
{
    return gss_carr_walk_ck(carr, step, n, ck);
}

double gss_code_advance(double code, double step, int64_t n, int32_t *icode, int32_t *ibit,
                        int32_t *iword)
{
    gss_code_state c = {code, *icode, *ibit, *iword};
    gss_code_walk_cc(&c, step, n);
    *icode = c.icode;
    *ibit = c.ibit;
    *iword = c.iword;
    return c.ph;
}

/* Carrier tables (gpssim.c:15-83): round(250 sin(2π(k+½)/512)) on a quarter wave, except the
   reference's entry 35 (and its mirrors) which is 105, not 106; the rest follows from
   sin(π-x)=sin x, sin(x+π)=-sin x and cos x = sin(x+π/2). */
int gss_lut(int32_t *sin512, int32_t *cos512)
{
    int32_t q[128];
    for (int k = 0; k < 128; k++)
        q[k] = (int32_t)lround(250.0 * sin(2.0 * 3.14159265358979323846 * (k + 0.5) / 512.0));
    q[35] = 105;
    for (int k = 0; k < 512; k++) {
        int h = k & 255;
        int32_t v = h < 128 ? q[h] : q[255 - h];
        sin512[k] = k < 256 ? v : -v;
    }
    for (int k = 0; k < 512; k++)
        cos512[k] = sin512[(k + 128) & 511];
    return 0;
}

const char *gss_version(void) { return "gpssim_amd 0.1 (gfx950)"; }

/* the bytes the reference writes per block (gpssim.c:2276, 2283, 2287): 4, 2 or 1/4 per sample;
   0 for an invalid format or a -b 1 block of samples not a multiple of 4 */
size_t gss_block_bytes(int n, int fmt)
{
    if (n <= 0) return 0;
    switch (fmt) {
    case GSS_FMT_SC16: return (size_t)n * 4;
    case GSS_FMT_SC08: return (size_t)n * 2;
    case GSS_FMT_SC01: return (n % 4) ? 0 : (size_t)n / 4;
    default: return 0;
    }
}

