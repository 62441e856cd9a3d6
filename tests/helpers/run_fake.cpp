/*
 * run_fake.cpp — gss_run itself (csrc/hip/gss_run.hip: its planner, rows and prover threads, slot
 * state machine, output-buffer pool, uploads, streams and events) on the CPU, for the sanitizers
 * (tools/sanitize.sh: -fsanitize=thread, -fsanitize=address,undefined).  gss_run.hip is built
 * unchanged against the fake HIP runtime of tests/helpers/fake_hip (streams drained by their own
 * threads), with the device functions of tests/helpers/fake_dev.cpp (host walks, host proofs, a
 * render that writes each block's fingerprint).  Every byte the sink receives is checked
 * against rows produced independently by a serial gss_scn_next pass over a fresh scenario (the
 * host carrier chain), in every mode of the run:
 *   default (chain run ahead, rows ahead for large batches, host proofs), GSS_RUN_SPEC=0,
 *   GSS_RUN_ROWS_AHEAD=1 / 0 with GSS_RUN_PROVER=0 / 1, GSS_RUN_PROOF=gpu / split,
 *   GSS_RUN_FORCE_EXACT (blocks on the exact path, lazy checkpoints), GSS_RUN_UPLOAD=dma,
 *   GSS_RUN_REC=0 (the walks back instead of records; the chain's anchors for the proofs),
 *   a range from a mid-run block, two runs on one handle, the carrier hand-off of gss_run_ex
 *   (two ranks in sequence), and a sink that stops the run.
 * Test infrastructure only (no GPU, nothing of it ships).
 *
 * usage: run_fake NAV_FILE [seconds] [batch] [fmt]
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "gpssim_amd.h"
#include "fake_dev.h"

extern "C" void gss_run_pool_drain(int dev);      /* gss_run.hip: the pooled slot buffers */

static const char *g_nav;
static double g_secs = 70.0;
static int g_fmt = 1;
static std::vector<uint64_t> g_want;            /* per block: its fingerprint */

static gss_scn *open_scn()
{
    gss_opts_t o;
    memset(&o, 0, sizeof o);
    o.nav_file = g_nav;
    o.has_llh = 1;
    o.llh[0] = 30.286502;
    o.llh[1] = 120.032669;
    o.llh[2] = 100.0;
    o.samp_freq = 2.6e6;
    o.data_format = g_fmt;
    o.duration = g_secs;
    o.quiet = 1;
    gss_scn *s = nullptr;
    if (gss_scn_open(&s, &o)) {
        fprintf(stderr, "scenario: %s\n", gss_last_error());
        exit(2);
    }
    return s;
}

/* the reference fingerprints: one serial pass with the host chain */
static void reference()
{
    gss_scn *s = open_scn();
    std::vector<gss_chan_blk_t> blk;
    std::vector<int32_t> nch;
    for (;;) {
        const int ask = 256;
        const size_t at = nch.size();
        blk.resize((at + ask) * GSS_MAXCH);
        nch.resize(at + ask);
        int nb = 0;
        if (gss_scn_next(s, ask, &blk[at * GSS_MAXCH], &nch[at], nullptr, &nb, 4)) {
            fprintf(stderr, "reference rows: %s\n", gss_last_error());
            exit(2);
        }
        nch.resize(at + nb);
        blk.resize((at + nb) * GSS_MAXCH);
        if (nb < ask)
            break;
    }
    const uint32_t *rows = nullptr;
    int n_rows = 0;
    gss_scn_nav_table(s, &rows, &n_rows);
    g_want.resize(nch.size());
    for (size_t b = 0; b < nch.size(); b++)
        if (fake_block_print(&blk[b * GSS_MAXCH], nch[b], rows, n_rows, &g_want[b])) {
            fprintf(stderr, "reference row outside the nav table\n");
            exit(2);
        }
    gss_scn_close(s);
}

struct Sink {
    size_t bb;
    int64_t next;                 /* the block the sink expects next */
    int64_t stop_at = -1;         /* return non-zero at this block (the stop test) */
    long bad = 0, blocks = 0;
};

static int sink(void *user, const void *bytes, size_t n, int64_t first, int nb)
{
    Sink *k = (Sink *)user;
    if (first != k->next || n != k->bb * (size_t)nb) {
        fprintf(stderr, "sink: blocks %lld+%d (%zu B), expected block %lld\n", (long long)first,
                nb, n, (long long)k->next);
        k->bad++;
    }
    std::vector<uint8_t> want(k->bb);
    for (int i = 0; i < nb; i++) {
        const int64_t b = first + i;
        if (b < 0 || b >= (int64_t)g_want.size()) {
            k->bad++;
            continue;
        }
        fake_fill(want.data(), k->bb, g_want[b]);
        if (memcmp(want.data(), (const uint8_t *)bytes + k->bb * (size_t)i, k->bb) != 0) {
            if (k->bad < 5)
                fprintf(stderr, "sink: block %lld differs\n", (long long)b);
            k->bad++;
        }
        k->blocks++;
    }
    k->next = first + nb;
    return k->stop_at >= first && k->stop_at < first + nb;
}

struct Mode {
    const char *name;
    std::vector<std::pair<const char *, const char *>> env;
};

static const char *ENV_KEYS[] = {"GSS_RUN_SPEC", "GSS_RUN_ROWS_AHEAD", "GSS_RUN_PROVER",
                                 "GSS_RUN_PROOF", "GSS_RUN_FORCE_EXACT", "GSS_RUN_UPLOAD",
                                 "GSS_RUN_ROWS_POOL", "GSS_RUN_REC", "GSS_RUN_ANCHORS",
                                 "GSS_RUN_DEV_ANCHORS", "GSS_RUN_LATE_VERDICTS"};

static void set_env(const Mode &m)
{
    for (const char *k : ENV_KEYS)
        unsetenv(k);
    for (auto &kv : m.env)
        setenv(kv.first, kv.second, 1);
}

static int fails = 0;

static void check(const char *what, int rc, const Sink &k, int64_t first, int64_t want_blocks)
{
    const bool ok = rc == 0 && k.bad == 0 && k.blocks == want_blocks &&
                    k.next == first + want_blocks;
    printf("%-44s rc %d blocks %ld bad %ld %s\n", what, rc, k.blocks, k.bad, ok ? "ok" : "FAIL");
    if (!ok) {
        if (rc)
            printf("  error: %s\n", gss_last_error());
        fails++;
    }
}

struct Baton {
    double carr[GSS_MAXCH];
    int set = 0;
    gss_scn *first = nullptr;     /* rank 0: its carriers are its scenario's own */
    /* the chain speculated across ranks (carr_predict): the ranks' published maps per round */
    int rank = 0;
    double maps[4][2][3 * GSS_MAXCH];
    int calls = 0;
};
/* what the ranks' collective (shard.compose_start, or the CLI's map files) would return: the
   composition of the maps of the ranks before this one, started from rank 0's initial carriers */
static int carr_predict(void *u, int round, const double *map, double *out)
{
    Baton *b = (Baton *)u;
    if (round < 0 || round > 1 || b->rank < 0 || b->rank > 3)
        return 1;
    memcpy(b->maps[b->rank][round], map, sizeof b->maps[0][0]);
    b->calls++;
    double x[GSS_MAXCH];
    memcpy(x, b->maps[0][round], sizeof x);
    for (int r = 0; r < b->rank; r++)
        for (int i = 0; i < GSS_MAXCH; i++) {
            const double add = b->maps[r][round][GSS_MAXCH + i];
            const double v = x[i] + add;
            x[i] = b->maps[r][round][2 * GSS_MAXCH + i] != 0.0 ? add : v - floor(v);
        }
    memcpy(out, x, sizeof x);
    return 0;
}
static int carr_out(void *u, const double *c)
{
    Baton *b = (Baton *)u;
    memcpy(b->carr, c, sizeof b->carr);
    b->set = 1;
    return 0;
}
static int carr_in(void *u, double *c)
{
    Baton *b = (Baton *)u;
    if (b->first)
        return gss_scn_carrier(b->first, c);
    if (!b->set)
        return 1;
    memcpy(c, b->carr, sizeof b->carr);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: run_fake NAV_FILE [seconds] [batch] [fmt]\n");
        return 2;
    }
    g_nav = argv[1];
    if (argc > 2) g_secs = atof(argv[2]);
    const int batch = argc > 3 ? atoi(argv[3]) : 64;
    if (argc > 4) g_fmt = atoi(argv[4]);
    reference();
    const int64_t nblk = (int64_t)g_want.size();
    gss_scn_info_t info;
    {
        gss_scn *s = open_scn();
        gss_scn_info(s, &info);
        gss_scn_close(s);
    }
    const size_t bb = gss_block_bytes(info.n_per_blk, g_fmt);
    printf("reference: %lld blocks of %d samples, -b %d (%zu B per block), batch %d\n",
           (long long)nblk, info.n_per_blk, g_fmt, bb, batch);
    gss_dev *d = fake_dev_open();

    const std::vector<Mode> modes = {
        {"default", {}},
        {"host chain (GSS_RUN_SPEC=0)", {{"GSS_RUN_SPEC", "0"}}},
        {"rows ahead, device proofs (auto)", {{"GSS_RUN_ROWS_AHEAD", "1"}}},
        {"rows ahead, device proofs, anchors from the device walks",
         {{"GSS_RUN_ROWS_AHEAD", "1"}, {"GSS_RUN_DEV_ANCHORS", "1"}}},
        {"rows ahead, prover thread", {{"GSS_RUN_ROWS_AHEAD", "1"}, {"GSS_RUN_PROOF", "host"}}},
        {"rows ahead, proofs on the planner",
         {{"GSS_RUN_ROWS_AHEAD", "1"}, {"GSS_RUN_PROVER", "0"}, {"GSS_RUN_PROOF", "host"}}},
        {"rows ahead, shared worker pool",
         {{"GSS_RUN_ROWS_AHEAD", "1"}, {"GSS_RUN_ROWS_POOL", "0"}, {"GSS_RUN_PROOF", "host"}}},
        {"rows on the planner", {{"GSS_RUN_ROWS_AHEAD", "0"}}},
        {"device proofs (GSS_RUN_PROOF=gpu)", {{"GSS_RUN_PROOF", "gpu"}}},
        {"device proofs, rows ahead", {{"GSS_RUN_PROOF", "gpu"}, {"GSS_RUN_ROWS_AHEAD", "1"}}},
        {"split proofs", {{"GSS_RUN_PROOF", "split"}, {"GSS_RUN_ROWS_AHEAD", "1"}}},
        {"every 7th block exact", {{"GSS_RUN_FORCE_EXACT", "7"}}},
        {"every 5th exact, device proofs", {{"GSS_RUN_FORCE_EXACT", "5"}, {"GSS_RUN_PROOF", "gpu"}}},
        {"every 5th exact, device proofs, late verdicts (redo in drain)",
         {{"GSS_RUN_FORCE_EXACT", "5"}, {"GSS_RUN_PROOF", "gpu"}, {"GSS_RUN_LATE_VERDICTS", "1"}}},
        {"every 3rd exact, rows ahead", {{"GSS_RUN_FORCE_EXACT", "3"}, {"GSS_RUN_ROWS_AHEAD", "1"}}},
        {"every 3rd exact, rows ahead, host proofs",
         {{"GSS_RUN_FORCE_EXACT", "3"}, {"GSS_RUN_ROWS_AHEAD", "1"}, {"GSS_RUN_PROOF", "host"}}},
        {"uploads by the copy engine", {{"GSS_RUN_UPLOAD", "dma"}}},
        {"walks back, anchors (GSS_RUN_REC=0)", {{"GSS_RUN_REC", "0"}}},
        {"walks back, anchors, rows ahead, device proofs",
         {{"GSS_RUN_REC", "0"}, {"GSS_RUN_ROWS_AHEAD", "1"}, {"GSS_RUN_PROOF", "gpu"}}},
        {"walks back, no anchors", {{"GSS_RUN_REC", "0"}, {"GSS_RUN_ANCHORS", "0"}}},
    };
    /* RUN_FAKE_QUICK=1 (the CPU suite's sanitizer test): every third mode, the whole-run and
       the two runs on one handle kept; the full list is tools/sanitize.sh's default */
    const char *quick_env = getenv("RUN_FAKE_QUICK");
    const bool quick = quick_env && quick_env[0] == '1';
    int mi = 0;
    for (const Mode &m : modes) {
        if (quick && (mi++ % 3) != 0)
            continue;
        set_env(m);
        {
            gss_scn *s = open_scn();
            Sink k{bb, 0};
            const int rc = gss_run(d, s, 0, -1, batch, 4, sink, &k);
            check((std::string(m.name) + ": whole run").c_str(), rc, k, 0, nblk);
            gss_scn_close(s);
        }
        {
            gss_scn *s = open_scn();
            const int64_t f = nblk / 3 + 1, n = nblk / 2;
            Sink k{bb, f};
            const int rc = gss_run(d, s, f, n, batch / 2 + 1, 3, sink, &k);
            check((std::string(m.name) + ": mid-run range").c_str(), rc, k, f, n);
            gss_scn_close(s);
        }
    }
    set_env(modes[0]);
    {   /* two runs on one handle, the second continuing the first */
        gss_scn *s = open_scn();
        const int64_t mid = nblk / 2 + 3;
        Sink k{bb, 0};
        int rc = gss_run(d, s, 0, mid, batch, 4, sink, &k);
        if (!rc)
            rc = gss_run(d, s, mid, -1, batch, 4, sink, &k);
        check("two runs on one handle", rc, k, 0, nblk);
        gss_scn_close(s);
    }
    for (const char *proof : {"", "gpu"}) {   /* two ranks in sequence, carriers handed over */
        if (*proof)
            setenv("GSS_RUN_PROOF", proof, 1);
        const int64_t mid = nblk / 2 - 5;
        Baton baton;
        gss_run_opts_t o0 = {carr_in, carr_out, &baton}, o1 = {carr_in, nullptr, &baton};
        gss_scn *s0 = open_scn();
        baton.first = s0;
        Sink k0{bb, 0};
        int rc = gss_run_ex(d, s0, 0, mid, batch, 4, sink, &k0, &o0);
        baton.first = nullptr;
        gss_scn_close(s0);
        gss_scn *s1 = open_scn();
        Sink k1{bb, mid};
        if (!rc)
            rc = gss_run_ex(d, s1, mid, -1, batch, 4, sink, &k1, &o1);
        gss_scn_close(s1);
        k0.blocks += k1.blocks;
        k0.bad += k1.bad;
        k0.next = k1.next;
        check(*proof ? "hand-off, two ranks, device proofs" : "hand-off, two ranks", rc, k0, 0,
              nblk);
        unsetenv("GSS_RUN_PROOF");
    }
    for (const char *proof : {"", "gpu"}) {   /* three ranks, the chain speculated across them */
        if (*proof)
            setenv("GSS_RUN_PROOF", proof, 1);
        const int64_t b1 = nblk / 3 + 7, b2 = 2 * nblk / 3 - 3;
        Baton baton;
        gss_run_opts_t o = {carr_in, carr_out, &baton, carr_predict};
        Sink all{bb, 0};
        int rc = 0;
        const int64_t firsts[3] = {0, b1, b2}, counts[3] = {b1, b2 - b1, -1};
        for (int r = 0; r < 3 && !rc; r++) {
            gss_scn *s = open_scn();
            baton.rank = r;
            baton.first = r == 0 ? s : nullptr;
            Sink k{bb, firsts[r]};
            gss_run_opts_t oo = o;
            if (r == 2)
                oo.carr_out = nullptr;
            rc = gss_run_ex(d, s, firsts[r], counts[r], batch, 4, sink, &k, &oo);
            gss_scn_close(s);
            all.blocks += k.blocks;
            all.bad += k.bad;
            all.next = k.next;
        }
        if (!rc && baton.calls != 6)
            rc = 1;                                     /* two rounds per rank */
        check(*proof ? "speculated hand-off, 3 ranks, device proofs" : "speculated hand-off, 3 ranks",
              rc, all, 0, nblk);
        unsetenv("GSS_RUN_PROOF");
    }
    {   /* the sink stops the run: an error, no hang, no leak */
        gss_scn *s = open_scn();
        Sink k{bb, 0};
        k.stop_at = nblk / 2;
        const int rc = gss_run(d, s, 0, -1, batch, 4, sink, &k);
        const bool ok = rc == GSS_E_IO && k.bad == 0;
        printf("%-44s rc %d blocks %ld %s\n", "sink stops the run", rc, k.blocks,
               ok ? "ok" : "FAIL");
        fails += !ok;
        gss_scn_close(s);
    }
    gss_run_pool_drain(-1);
    fake_dev_close(d);
    printf("%s\n", fails ? "FAILED" : "all modes ok");
    return fails ? 1 : 0;
}
