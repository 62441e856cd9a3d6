/*
 * gps_sdr_sim.c — the command-line program: reference option surface (-e/-u/-g/-c/-l/-t/-T/-d/
 * -o/-s/-b/-i/-v), reference stderr messages, byte-identical gpssim.bin.  The whole block loop
 * runs in gss_run (host planner thread, GPU stages, pinned downloads); this driver only supplies
 * the sink (fwrite to file or stdout), gpssim.c:2101-2111, 2276-2287.  There is no CPU
 * fallback: without a GPU it exits with an error.
 * Multi-GPU: launched N times with RANK / WORLD_SIZE / LOCAL_RANK set (e.g. `torchrun
 * --no-python --nproc-per-node N gps-sdr-sim ... -o FILE`), process r synthesises the contiguous
 * block range [B r/N, B (r+1)/N) on GPU LOCAL_RANK and pwrite()s it at its byte offset of FILE
 * (every rank ftruncate()s FILE to the run's size first, safe in any order): the same file as
 * one process writes, with no collective.  Planned once per node: rank r seeks to
 * its first block and plans only its own range; the 16 slot carriers at its first block (the one
 * state the sample loop carries across blocks, gpssim.c:2245-2250) come from rank r-1 through a
 * hand-off file next to FILE, FILE.gss-carr-<run id>-<block>, written atomically (tmp + rename)
 * and removed by its reader.  The run id is torchrun's TORCHELASTIC_RUN_ID (or GSS_RUN_ID);
 * without one every rank plans the blocks before its range itself.  torchrun's default run id
 * is the same for every launch ("none"), so a file left by an interrupted earlier run can sit
 * at the same path: the payload carries a fingerprint of everything the carriers depend on (the
 * scenario options, the bytes of the navigation and motion files, the world size and the
 * boundary block), and a reader ignores a file whose fingerprint differs and waits for its own.
 * With a run id the chain is also speculated across the ranks (gss_run_opts_t.carr_predict): each
 * rank publishes its map of the slot carriers in two rounds of FILE.gss-map-* files and walks its
 * range before its carriers arrive (GSS_HANDOFF_SPEC=0: off).
 * Env: GSS_DEVICE (ordinal; default LOCAL_RANK or 0), GSS_BATCH (blocks per launch, default
 *      128), GSS_THREADS (planner threads, default the CPU share: cgroup cpu.max, else the online
 *      CPUs, at most 16), GSS_HANDOFF_TIMEOUT (seconds a rank waits
 *      for its carriers, default 3600).
 */
#include <fcntl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include "gpssim_amd.h"
#include "cli_args.h"

static int write_sink(void *user, const void *bytes, size_t n, int64_t first_block, int nblocks)
{
    (void)first_block; (void)nblocks;
    return fwrite(bytes, 1, n, (FILE *)user) == n ? 0 : 1;
}

typedef struct { int fd; size_t block_bytes; } pwrite_ctx;

static int pwrite_sink(void *user, const void *bytes, size_t n, int64_t first_block, int nblocks)
{
    (void)nblocks;
    const pwrite_ctx *c = (const pwrite_ctx *)user;
    off_t off = (off_t)first_block * (off_t)c->block_bytes;
    const char *p = (const char *)bytes;
    while (n > 0) {
        ssize_t w = pwrite(c->fd, p, n, off);
        if (w <= 0)
            return 1;
        p += w;
        off += w;
        n -= (size_t)w;
    }
    return 0;
}

static int env_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

/* planner threads: the CPUs' worth of time this process may use (cgroup v2 cpu.max quota, else
   the online CPUs), 1..16 (16 channel slots; more buys the chain nothing) */
static int default_threads(void)
{
    long n = sysconf(_SC_NPROCESSORS_ONLN);
    FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r");
    if (f) {
        char q[32] = {0};
        long period = 0;
        if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
            n = atol(q) / period;
        fclose(f);
    }
    return n < 1 ? 1 : n > 16 ? 16 : (int)n;
}

/* The carrier hand-off between ranks (plan once per node): a 16-double file per boundary, and,
   for the chain speculated across ranks (gss_run_opts_t.carr_predict), each rank's map of the
   slot carriers per round, FILE.gss-map-<run id>-<round>-<first block>, read by the ranks after
   it and removed by the last rank once its own carriers have arrived (every rank has read the
   maps by then: each reads them before it waits for its carriers). */
typedef struct {
    gss_scn *scn;
    char in_path[600], out_path[600];      /* empty: none (rank 0 / last rank) */
    uint64_t fp_in, fp_out;                /* fingerprints: scenario + boundary block */
    double timeout_s;
    /* speculation */
    const char *out_file, *run_id;
    int rank, world;
    int64_t n_blocks;
    uint64_t fp;                           /* the scenario's fingerprint */
} handoff_ctx;

static int64_t rank_first(const handoff_ctx *h, int r) { return h->n_blocks * r / h->world; }

#define HANDOFF_MAGIC 0x67737364u          /* "gssd": magic, fingerprint, 16 carriers */

/* FNV-1a 64 */
static uint64_t fnv(uint64_t h, const void *p, size_t n)
{
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; i++)
        h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

static void map_path(const handoff_ctx *h, int round, int r, char *out, size_t n)
{
    snprintf(out, n, "%s.gss-map-%s-%d-%lld", h->out_file, h->run_id, round,
             (long long)rank_first(h, r));
}

static uint64_t map_fp(const handoff_ctx *h, int round, int r)
{
    const int64_t first = rank_first(h, r);
    return fnv(fnv(h->fp ^ 0x6d6170u, &round, sizeof round), &first, sizeof first);
}

static uint64_t fnv_file(uint64_t h, const char *path)
{
    if (!path || !*path)
        return fnv(h, "-", 1);
    FILE *f = fopen(path, "rb");
    if (!f)
        return fnv(h, path, strlen(path));
    unsigned char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0)
        h = fnv(h, buf, n);
    fclose(f);
    return h;
}

/* the scenario's identity: every option that shapes the carriers, and the input files' bytes */
static uint64_t scenario_fingerprint(const gss_cli_t *cli, int world)
{
    const gss_opts_t *o = &cli->opt;
    uint64_t h = 0xcbf29ce484222325ull;
    h = fnv_file(h, cli->nav_file);
    h = fnv_file(h, cli->motion_file[0] ? cli->motion_file : NULL);
#define FP(x) h = fnv(h, &(x), sizeof(x))
    FP(o->nmea); FP(o->has_xyz); FP(o->xyz); FP(o->has_llh); FP(o->llh); FP(o->samp_freq);
    FP(o->data_format); FP(o->duration); FP(o->has_start); FP(o->time_overwrite); FP(o->start);
    FP(o->start_sec); FP(o->iono_disable); FP(o->user_motion_size); FP(o->carrier_int);
    FP(world);
#undef FP
    return h;
}

static int handoff_in(void *user, double *carr)
{
    const handoff_ctx *h = (const handoff_ctx *)user;
    if (!h->in_path[0])                    /* rank 0: every slot starts with a reset */
        return gss_scn_carrier(h->scn, carr);
    struct timespec nap = {0, 1000000};
    double waited = 0.0;
    for (;;) {
        FILE *f = fopen(h->in_path, "rb");
        if (f) {
            uint32_t magic = 0;
            uint64_t fp = 0;
            const int ok = fread(&magic, sizeof magic, 1, f) == 1 &&
                           fread(&fp, sizeof fp, 1, f) == 1 &&
                           fread(carr, sizeof(double), GSS_MAXCH, f) == GSS_MAXCH;
            fclose(f);
            if (ok && magic == HANDOFF_MAGIC && fp == h->fp_in) {
                unlink(h->in_path);
                if (h->rank == h->world - 1 && h->run_id)   /* every rank has read the maps */
                    for (int round = 0; round < 2; round++)
                        for (int r = 0; r + 1 < h->world; r++) {
                            char path[640];
                            map_path(h, round, r, path, sizeof path);
                            unlink(path);
                        }
                return 0;
            }
            /* another run's (or a torn) file: not ours, wait for rank r-1 to replace it */
        }
        if (waited > h->timeout_s)
            return 1;
        nanosleep(&nap, NULL);
        waited += 1e-3;
    }
}

#define MAP_MAGIC 0x6773736du              /* "gssm": magic, fingerprint, 48 doubles */
#define NOSPEC_MAGIC 0x6773736eu           /* "gssn": the rank does not speculate      */

static int write_map(const handoff_ctx *h, int round, uint32_t magic, const double *map)
{
    char path[640], tmp[660];
    static const double zero[3 * GSS_MAXCH];
    map_path(h, round, h->rank, path, sizeof path);
    snprintf(tmp, sizeof tmp, "%s.tmp", path);
    FILE *f = fopen(tmp, "wb");
    if (!f)
        return 1;
    const uint64_t fp = map_fp(h, round, h->rank);
    int ok = fwrite(&magic, sizeof magic, 1, f) == 1 && fwrite(&fp, sizeof fp, 1, f) == 1 &&
             fwrite(map ? map : zero, sizeof(double), 3 * GSS_MAXCH, f) == 3 * GSS_MAXCH;
    ok = (fclose(f) == 0) && ok;
    return (ok && rename(tmp, path) == 0) ? 0 : 1;
}

/* publish this rank's map of `round`, then compose the maps of the ranks before it; round -1:
   this rank does not speculate -- markers in place of both rounds' maps, so a rank after it
   that does fails at once (gss_run_opts_t.carr_predict) */
static int handoff_predict(void *user, int round, const double *map, double *start)
{
    const handoff_ctx *h = (const handoff_ctx *)user;
    char path[640];
    if (round < 0) {
        if (h->rank + 1 < h->world)
            for (int q = 0; q < 2; q++)
                if (write_map(h, q, NOSPEC_MAGIC, NULL))
                    return 1;
        return 0;
    }
    /* the last rank's map has no reader */
    if (h->rank + 1 < h->world && write_map(h, round, MAP_MAGIC, map))
        return 1;
    double x[GSS_MAXCH];
    memcpy(x, map, sizeof x);                           /* rank 0: its own start */
    for (int r = 0; r < h->rank; r++) {
        double m[3 * GSS_MAXCH];
        map_path(h, round, r, path, sizeof path);
        struct timespec nap = {0, 1000000};
        double waited = 0.0;
        for (;;) {
            FILE *f = fopen(path, "rb");
            if (f) {
                uint32_t magic = 0;
                uint64_t fp = 0;
                const int ok = fread(&magic, sizeof magic, 1, f) == 1 &&
                               fread(&fp, sizeof fp, 1, f) == 1 &&
                               fread(m, sizeof(double), 3 * GSS_MAXCH, f) == 3 * GSS_MAXCH;
                fclose(f);
                if (ok && magic == NOSPEC_MAGIC && fp == map_fp(h, round, r)) {
                    fprintf(stderr, "ERROR: rank %d does not speculate the carrier chain but "
                            "rank %d does: give every rank the same GSS_HANDOFF_SPEC, "
                            "GSS_RUN_SPEC, GSS_RUN_REC and GSS_PATH.\n", r, h->rank);
                    return 1;
                }
                if (ok && magic == MAP_MAGIC && fp == map_fp(h, round, r))
                    break;
            }
            if (waited > h->timeout_s)
                return 1;
            nanosleep(&nap, NULL);
            waited += 1e-3;
        }
        if (r == 0)
            memcpy(x, m, sizeof x);                     /* the run's initial carriers */
        for (int i = 0; i < GSS_MAXCH; i++) {
            const double add = m[GSS_MAXCH + i], v = x[i] + add;
            x[i] = m[2 * GSS_MAXCH + i] != 0.0 ? add : v - floor(v);
        }
    }
    memcpy(start, x, sizeof x);
    return 0;
}

static int handoff_out(void *user, const double *carr)
{
    const handoff_ctx *h = (const handoff_ctx *)user;
    if (!h->out_path[0])
        return 0;
    char tmp[640];
    snprintf(tmp, sizeof tmp, "%s.tmp", h->out_path);
    FILE *f = fopen(tmp, "wb");
    if (!f)
        return 1;
    const uint32_t magic = HANDOFF_MAGIC;
    int ok = fwrite(&magic, sizeof magic, 1, f) == 1 &&
             fwrite(&h->fp_out, sizeof h->fp_out, 1, f) == 1 &&
             fwrite(carr, sizeof(double), GSS_MAXCH, f) == GSS_MAXCH;
    ok = (fclose(f) == 0) && ok;
    return (ok && rename(tmp, h->out_path) == 0) ? 0 : 1;
}

/* One process of a multi-GPU run: its block range, pwrite()n at its offset of the output file. */
static int run_rank(const gss_cli_t *cli, gss_scn *scn, const gss_scn_info_t *info, int rank,
                    int world)
{
    if (!strcmp("-", cli->out_file)) {
        fprintf(stderr, "ERROR: a multi-process run needs an output file (-o FILE).\n");
        return 1;
    }
    gss_dev *dev = NULL;
    if (gss_dev_open(&dev, env_int("GSS_DEVICE", env_int("LOCAL_RANK", 0)))) {
        fprintf(stderr, "ERROR: %s\n", gss_last_error());
        return 1;
    }
    const int64_t nb = info->n_blocks;
    const int64_t first = nb * rank / world, last = nb * (rank + 1) / world;
    pwrite_ctx c = {-1, gss_block_bytes(info->n_per_blk, info->data_format)};
    c.fd = open(cli->out_file, O_WRONLY | O_CREAT, 0644);
    if (c.fd < 0 || ftruncate(c.fd, (off_t)nb * (off_t)c.block_bytes)) {
        fprintf(stderr, "ERROR: Failed to open output file.\n");
        return 1;
    }
    const char *run_id = getenv("TORCHELASTIC_RUN_ID");
    if (!run_id || !*run_id)
        run_id = getenv("GSS_RUN_ID");
    handoff_ctx h;
    memset(&h, 0, sizeof h);
    h.scn = scn;
    h.timeout_s = env_int("GSS_HANDOFF_TIMEOUT", 3600);
    const uint64_t fp = scenario_fingerprint(cli, world);
    h.fp_in = fnv(fp, &first, sizeof first);
    h.fp_out = fnv(fp, &last, sizeof last);
    h.fp = fp;
    h.out_file = cli->out_file;
    h.run_id = run_id;
    h.rank = rank;
    h.world = world;
    h.n_blocks = nb;
    /* GSS_HANDOFF_SPEC=0: the carriers first, then the chain (no speculation; every rank of a
       run must agree) */
    const int spec = env_int("GSS_HANDOFF_SPEC", 1);
    gss_run_opts_t ro = {handoff_in, handoff_out, &h, spec ? handoff_predict : NULL};
    if (run_id && *run_id) {
        if (rank > 0)
            snprintf(h.in_path, sizeof h.in_path, "%s.gss-carr-%s-%lld", cli->out_file, run_id,
                     (long long)first);
        if (rank + 1 < world)
            snprintf(h.out_path, sizeof h.out_path, "%s.gss-carr-%s-%lld", cli->out_file,
                     run_id, (long long)last);
        /* not speculating here: the markers tell a rank after this one that does (the library
           writes them through the callback when its own settings rule speculation out) */
        if (!spec && handoff_predict(&h, -1, NULL, NULL)) {
            fprintf(stderr, "ERROR: rank %d: carrier hand-off files.\n", rank);
            return 1;
        }
    }
    if (gss_run_ex(dev, scn, first, last - first, env_int("GSS_BATCH", 128),
                   env_int("GSS_THREADS", default_threads()), pwrite_sink, &c,
                   run_id && *run_id ? &ro : NULL)) {
        fprintf(stderr, "\nERROR: rank %d: %s\n", rank, gss_last_error());
        return 1;
    }
    if (close(c.fd)) {
        fprintf(stderr, "ERROR: rank %d: write failed.\n", rank);
        return 1;
    }
    if (rank == 0)
        fprintf(stderr, "\nDone!\n");
    gss_dev_close(dev);
    gss_scn_close(scn);
    return 0;
}

int main(int argc, char **argv)
{
    gss_cli_t cli;
    if (gss_cli_parse(argc, argv, &cli))
        return 1;
    gss_scn *scn = NULL;
    if (gss_scn_open(&scn, &cli.opt)) {
        fprintf(stderr, "%s\n", gss_last_error());
        return 1;
    }
    gss_scn_info_t info;
    gss_scn_info(scn, &info);

    const int world = env_int("WORLD_SIZE", 1), rank = env_int("RANK", 0);
    if (world < 1 || rank < 0 || rank >= world) {
        fprintf(stderr, "ERROR: invalid RANK %d / WORLD_SIZE %d.\n", rank, world);
        return 1;
    }
    if (world > 1)
        return run_rank(&cli, scn, &info, rank, world);

    gss_dev *dev = NULL;
    int ordinal = env_int("GSS_DEVICE", 0);
    if (gss_dev_open(&dev, ordinal)) {
        fprintf(stderr, "ERROR: %s\n", gss_last_error());
        return 1;
    }
    FILE *fp = stdout;
    if (strcmp("-", cli.out_file)) {
        fp = fopen(cli.out_file, "wb");
        if (fp == NULL) {
            fprintf(stderr, "ERROR: Failed to open output file.\n");
            return 1;
        }
    }
    int batch = env_int("GSS_BATCH", 128);
    int threads = env_int("GSS_THREADS", default_threads());
    if (batch < 1) batch = 1;
    clock_t t0 = clock();
    /* planning, upload, both kernel stages, download and fwrite overlap inside gss_run; the
       sink sees each batch's bytes in run order (gpssim.c:2276/2283/2287) */
    if (gss_run(dev, scn, 0, -1, batch, threads, write_sink, fp)) {
        fprintf(stderr, "\nERROR: %s\n", gss_last_error());
        return 1;
    }
    clock_t t1 = clock();
    fprintf(stderr, "\nDone!\n");
    if (fp != stdout)
        fclose(fp);
    fprintf(stderr, "Process time = %.1f [sec]\n", (double)(t1 - t0) / CLOCKS_PER_SEC);
    gss_dev_close(dev);
    gss_scn_close(scn);
    return 0;
}
