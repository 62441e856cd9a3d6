/*
 * fake_dev.cpp — the device side of gss_run on the CPU (tools/sanitize.sh; test infrastructure
 * only).  Each function gss_run.hip calls on the GPU is queued on its stream of the fake HIP
 * runtime (fake_hip/) and run there by host code:
 *   gss_ca_table_device / gss_nav_rows_device   the host producers (gss_ca_table, gss_nav_rows_host)
 *   gss_spec_device                             the walks on the host (gss_spec_host)
 *   gss_spec_records_device                     walks and records on the host (gss_spec_records)
 *   run_proof_launch                            the proofs on the host (gss_linearize; the GPU proof
 *                                               writes the same rows, tests/test_gpu_proof.py)
 *   run_copy_launch                             memcpy
 *   gss_synth_lin_device / gss_synth_device     a "render" that fills each block with a fingerprint
 *                                               of what the kernels would read for it: its rows
 *                                               (exact carriers included) and the words of the nav
 *                                               rows they point at; on the exact path it also checks
 *                                               the carrier checkpoints against an exact walk
 * so the harness (run_fake.cpp) can check every byte the sink receives against rows produced
 * independently, while the run's real threads, slots, pools and streams do their work.
 */
#include <hip/hip_runtime.h>
#include <string.h>
#include "gpssim_amd.h"
#include "fake_dev.h"

struct gss_dev {
    int ordinal;
};

extern "C" gss_dev *fake_dev_open(void)
{
    gss_dev *d = new gss_dev();
    d->ordinal = 0;
    return d;
}
extern "C" void fake_dev_close(gss_dev *d) { delete d; }
extern "C" int gss_dev_ordinal(const gss_dev *d) { return d->ordinal; }
extern "C" int gss_dev_reserve(gss_dev *d, int max_blocks, int n_per_blk)
{
    (void)d;
    return max_blocks > 0 && n_per_blk > 0 ? 0 : GSS_E_ARG;
}

extern "C" int gss_ca_table_device(gss_dev *d, uint32_t *out, void *stream)
{
    (void)d;
    fake_enqueue((hipStream_t)stream, [out] { gss_ca_table(out); });
    return 0;
}

extern "C" int gss_nav_rows_device(gss_dev *d, const gss_nav_src_t *src, int first, int n,
                                   uint32_t *rows, void *stream)
{
    (void)d;
    fake_enqueue((hipStream_t)stream, [=] { (void)gss_nav_rows_host(src, first, n, rows); });
    return 0;
}

extern "C" int gss_spec_device(gss_dev *d, gss_spec_in_t *in, int nrow, int n_per_blk,
                               gss_spec_t *spec, void *stream)
{
    (void)d;
    fake_enqueue((hipStream_t)stream, [=] { (void)gss_spec_host(in, nrow, n_per_blk, spec, 1); });
    return 0;
}

extern "C" int gss_spec_records_device(gss_dev *d, const gss_spec_in_t *in, int nrow,
                                       int n_per_blk, gss_spec_in_t *d_in, gss_spec_t *d_spec,
                                       gss_spec_rec_t *rec, void *stream)
{
    if (!d || nrow < 0 || (nrow > 0 && (!in || !d_in || !d_spec || !rec)))
        return GSS_E_ARG;
    fake_enqueue((hipStream_t)stream, [=] {
        for (int i = 0; i < nrow; i++) {              /* the heads only, as the kernel reads */
            gss_spec_in_t r{};
            r.g = in[i].g;
            r.s = in[i].s;
            r.k = in[i].k;
            r.pad = in[i].pad;
            d_in[i] = r;
        }
        (void)gss_spec_host(d_in, nrow, n_per_blk, d_spec, 1);
        (void)gss_spec_records(d_in, d_spec, nrow, n_per_blk, rec, 1);
    });
    return 0;
}

int run_proof_launch(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                     const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                     const gss_carr_anchor_t *anch, const gss_spec_in_t *sin,
                     const gss_spec_t *sspec, gss_lin_t *lin, int32_t *fast, int64_t first,
                     int force_exact, hipStream_t st)
{
    if (nblk <= 0)
        return 0;
    fake_enqueue(st, [=] {
        /* the walks the anchors would come from are read here (their lifetime is what the run
           must keep: a reused batch must wait for this proof), then the host proof */
        volatile double sink = 0.0;
        if (sin && sspec)
            for (int i = 0; i < nblk * GSS_MAXCH; i++)
                sink = sink + sin[i].g + sspec[i].w1;
        (void)sink;
        (void)gss_linearize_ex(blk, nch, nblk, n_per_blk, ca_bits, n_ca, nav, n_nav, anch, lin,
                               fast, 1);
        if (force_exact > 0)
            for (int b = 0; b < nblk; b++)
                if ((first + b) % force_exact == 0)
                    fast[b] = 0;
    });
    return 0;
}

int run_copy_launch(void *dst, const void *src, size_t n, hipStream_t st)
{
    if (n)
        fake_enqueue(st, [=] { memcpy(dst, src, n); });
    return 0;
}

/* the fingerprint of block b's inputs (shared with the harness, fake_dev.h) */
static void render(const gss_chan_blk_t *blk, const int32_t *nch, const uint32_t *nav, int n_nav,
                   const double *carr_ck, const int32_t *fb, int n_fb, int nblk, int n_per_blk,
                   int fmt, uint8_t *out, int32_t *status)
{
    const size_t bb = gss_block_bytes(n_per_blk, fmt);
    for (int b = 0; b < nblk; b++) {
        uint64_t h;
        if (fake_block_print(blk + (size_t)b * GSS_MAXCH, nch[b], nav, n_nav, &h)) {
            __atomic_fetch_or(status, 4, __ATOMIC_RELAXED);
            h = 0;
        }
        fake_fill(out + bb * (size_t)b, bb, h);
    }
    /* the exact path's blocks: their checkpoints must be the exact walk's */
    for (int i = 0; carr_ck && i < n_fb; i++) {
        const int b = fb ? fb[i] : i;
        for (int k = 0; k < nch[b]; k++) {
            const gss_chan_blk_t *p = blk + (size_t)b * GSS_MAXCH + k;
            double ck[GSS_NCK];
            (void)gss_carr_advance_ck(p->carr0, p->carr_step, n_per_blk, ck);
            if (memcmp(ck, carr_ck + ((size_t)b * GSS_MAXCH + k) * GSS_NCK, sizeof ck) != 0)
                fake_fill(out + bb * (size_t)b, bb, 0xBADC0FFEEull);
        }
    }
}

extern "C" int gss_synth_lin_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                                    int nch_max, const gss_lin_t *lin, const int32_t *fast,
                                    const int32_t *fb_list, int n_fb, const double *carr_ck,
                                    const uint32_t *ca_bits, int n_ca, const uint32_t *nav,
                                    int n_nav, int nblk, int n_per_blk, int fmt, void *out,
                                    int32_t *status, void *stream)
{
    (void)d; (void)nch_max; (void)ca_bits; (void)n_ca;
    if (!blk || !nch || !lin || !fast || !out || nblk <= 0 || (n_fb > 0 && !fb_list))
        return GSS_E_ARG;
    fake_enqueue((hipStream_t)stream, [=] {
        /* (blocks the fast flags reject and the list omits are the device proofs' rejects,
           rendered again by gss_run's redo; every block gets its fingerprint here) */
        render(blk, nch, nav, n_nav, n_fb ? carr_ck : nullptr, fb_list, n_fb, nblk, n_per_blk, fmt,
               (uint8_t *)out, status);
    });
    return 0;
}

extern "C" int gss_synth_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                                int nch_max, const double *carr_ck, const uint32_t *ca_bits,
                                int n_ca, const uint32_t *nav, int n_nav, int nblk, int n_per_blk,
                                int fmt, void *out, double *carr_end, int32_t *status,
                                void *stream)
{
    (void)d; (void)nch_max; (void)ca_bits; (void)n_ca; (void)carr_end;
    fake_enqueue((hipStream_t)stream, [=] {
        render(blk, nch, nav, n_nav, carr_ck, nullptr, nblk, nblk, n_per_blk, fmt, (uint8_t *)out,
               status);
    });
    return 0;
}
