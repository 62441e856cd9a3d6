/*
 * gss_proof.hip — the fast path's proofs on the GPU (gss_linearize_device): the same per-channel
 * proof as the host's gss_linearize (csrc/common/gss_proof.h, compiled for both), one lane per
 * (block, channel), sixteen blocks per workgroup.  gss_run uses it so that the 24 h -b 1 run's
 * proofs (60 % of its host CPU time: 15-17 µs per block on one core) leave the host; the rows it
 * writes are byte for byte the host's (tests/test_gpu_proof.py).
 *
 * Per block the host proves channels in order and stops at the first that fails; here all
 * channels run at once, so the rows after a block's first failing channel are reset to the
 * host's initial state afterwards (they are never rendered: the block goes to the exact path).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <mutex>
#include "gpssim_amd.h"
#include "../common/gss_proof.h"

extern "C" int gss_fail(int code, const char *fmt, ...);
extern "C" int gss_dev_ordinal(const gss_dev *d);

namespace {

struct proof_lut {                     /* gss_lut's tables as a kernel argument (|v| <= 250) */
    int16_t c[512], s[512];
};

const proof_lut &host_lut()
{
    static proof_lut L;
    static std::once_flag once;
    std::call_once(once, [] {
        int32_t s[512], c[512];
        gss_lut(s, c);
        for (int i = 0; i < 512; i++) {
            L.s[i] = (int16_t)s[i];
            L.c[i] = (int16_t)c[i];
        }
    });
    return L;
}

}  // namespace

/* (outside the anonymous namespace, so that profiles name the kernel: rocprofv3 prints
   "(anonymous namespace)::..." for the others) */
__device__ static void lin_row_init(gss_lin_t *l)
{
    lin_row_reset(l);
}

/* One block per workgroup, as two halves of 16 * STRIDE threads: the first half proves the
   channels' carrier lines (lin_carrier: its descents and the exact walks from the anchors), the
   second their code lines and gain schedules (lin_code), thread STRIDE k of a half for channel
   k; after a barrier the first half merges the two into the patches (lin_patches).  A lane's
   proof is a long dependent chain (descents, exact walks: latency, not throughput: VALU issue
   0.22), so the two independent parts run on different waves at the same time (on one wave
   they would diverge and run one after the other).  A small launch spreads a half over more
   waves (STRIDE 16 / 32: 4 / 8 waves of a few live lanes) so that the SIMDs interleave them; a
   large one (STRIDE 4) still gives each half one wave per block (proof_stride). */
/* waves per SIMD the register budget aims at: the compiler's own (131 VGPRs: 3 waves) left the
   headline window's 2,999 workgroups in two rounds; 5 (96 VGPRs, 96 B more scratch) proves it in
   0.45 ms against 0.48, 4 and 6 in between (profiles/round6/proof/ab_pw_s6v.txt); 0: the
   compiler's budget */
#ifndef PF_WAVES_PER_EU
#define PF_WAVES_PER_EU 5
#endif
#if PF_WAVES_PER_EU
#define PF_OCC __attribute__((amdgpu_waves_per_eu(PF_WAVES_PER_EU)))
#else
#define PF_OCC
#endif
template <int STRIDE>
__global__ __launch_bounds__(2 * GSS_MAXCH * STRIDE) PF_OCC void gss_proof_kernel(
    const gss_chan_blk_t *__restrict__ blk, const int32_t *__restrict__ nch, int nblk,
    int n_per_blk, const uint32_t *__restrict__ ca, int n_ca, const uint32_t *__restrict__ nav,
    int n_nav, proof_lut lut, const gss_carr_anchor_t *__restrict__ anch,
    const gss_spec_in_t *__restrict__ sin, const gss_spec_t *__restrict__ sspec,
    gss_lin_t *__restrict__ lin, int32_t *__restrict__ fast, int64_t first, int force_exact)
{
    static_assert(GSS_MAXCH * STRIDE % 64 == 0, "each half whole waves");
    constexpr int HALF = GSS_MAXCH * STRIDE;
    __shared__ int32_t lcos[512], lsin[512];
    __shared__ int fail_k[GSS_MAXCH];
    __shared__ int gabs[GSS_MAXCH];
    __shared__ int part_ok[GSS_MAXCH][2];
    __shared__ gss_pf_side s_cz[GSS_MAXCH];              /* the code parts, for the first half */
    gss_pf_side cx;                                      /* a first-half thread's carrier part */
    for (int i = threadIdx.x; i < 512; i += blockDim.x) {
        lcos[i] = lut.c[i];
        lsin[i] = lut.s[i];
    }
    const int role = threadIdx.x / HALF, t = threadIdx.x % HALF, b = blockIdx.x;
    const int k = t / STRIDE;
    const bool slot = t % STRIDE == 0;                   /* the thread of channel slot k */
    const bool lead = role == 0 && slot;
    gss_lin_t *l = lin + (size_t)b * GSS_MAXCH + k;
    const int nc = b < nblk ? nch[b] : 0;
    const bool live = b < nblk && nc >= 0 && nc <= GSS_MAXCH && k < nc;
    const gss_chan_blk_t *p = blk + (size_t)b * GSS_MAXCH + k;
    const bool tables_ok = live && p->nav_tbl >= 0 && p->nav_tbl < n_nav && p->ca_tbl >= 0 &&
                           p->ca_tbl < n_ca;
    if (lead && b < nblk)
        lin_row_init(l);
    __syncthreads();                                      /* (the row reset before both parts) */
    if (slot) {
        int ok = 0;
#ifdef PF_SKIP                                           /* measurement builds: one half only */
        if (role == PF_SKIP - 1) {
            part_ok[k][role] = 0;
        } else
#endif
        if (tables_ok) {
            if (role == 0)
                ok = lin_carrier(p, n_per_blk, anch ? anch + (size_t)b * GSS_MAXCH + k : nullptr,
                                 sin ? sin + (size_t)b * GSS_MAXCH + k : nullptr,
                                 sspec ? sspec + (size_t)b * GSS_MAXCH + k : nullptr, &cx, l);
            else
                ok = lin_code(p, n_per_blk, nav + (size_t)p->nav_tbl * GSS_NAV_WORDS, &s_cz[k],
                              l);
        }
        part_ok[k][role] = ok;
    }
    __syncthreads();                                      /* both parts' sides and row fields */
    int failed = 0, g = 0;
    if (lead && b < nblk) {
        if (nc < 0 || nc > GSS_MAXCH) {
            failed = k == 0;                            /* the block fails before any channel */
        } else if (k < nc) {
            g = p->gain < 0 ? -p->gain : p->gain;
            int ok = tables_ok && part_ok[k][0] && part_ok[k][1] &&
                     lin_patches(p, n_per_blk, ca + (size_t)p->ca_tbl * GSS_CA_WORDS, lcos, lsin,
                                 &cx, &s_cz[k], l);
            if (!ok)
                lin_row_reset(l);                       /* as lin_channel on the host */
            if (p->gain > 1024 || p->gain < -1024)
                ok = 0;
            failed = !ok;
        }
    }
    if (lead) {
        fail_k[k] = failed ? k : GSS_MAXCH;
        gabs[k] = g;
    }
    __syncthreads();
    /* the block's first failing channel and its gain sum (the host's loop order) */
    int kf = GSS_MAXCH, gsum = 0;
    for (int jj = 0; jj < GSS_MAXCH; jj++) {
        const int f = fail_k[jj];
        kf = f < kf ? f : kf;
    }
    for (int jj = 0; jj < GSS_MAXCH && jj <= kf; jj++)
        gsum += gabs[jj];
    if (lead && b < nblk) {
        if (k > kf)
            lin_row_init(l);                            /* the host never reached this channel */
        if (k == 0) {
            int ok = kf == GSS_MAXCH && gsum <= 8000;
            if (force_exact > 0 && (first + b) % force_exact == 0)
                ok = 0;
            fast[b] = ok;
        }
    }
}

/* threads per channel slot and half (waves: nblk STRIDE / 2) for a launch of nblk blocks: the
   widest spread the chip still holds about at once (256 CUs x 4 SIMDs x 4-8 waves of this
   kernel); GSS_PROOF_STRIDE = 4, 16 or 32 forces one (measurements, tests) */
static int proof_stride(int nblk)
{
    const char *e = getenv("GSS_PROOF_STRIDE");        /* (read per launch: tests switch it) */
    const int forced = e ? atoi(e) : 0;
    if (forced == 4 || forced == 16 || forced == 32)
        return forced;
    const long waves_cap = 8192;
    for (int s = 32; s >= 16; s /= 2)
        if ((long)nblk * s / 2 <= waves_cap)
            return s;
    return 4;
}

/* gss_run's launch (force_exact: its test hook; sin / sspec: the batch's walks on the device,
   the anchors' source in records mode); not exported (exports.map) */
int run_proof_launch(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                     const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                     const gss_carr_anchor_t *anch, const gss_spec_in_t *sin,
                     const gss_spec_t *sspec, gss_lin_t *lin, int32_t *fast, int64_t first,
                     int force_exact, hipStream_t st)
{
    if (nblk <= 0)
        return 0;
#define PF_LAUNCH(S)                                                                             \
    hipLaunchKernelGGL(gss_proof_kernel<S>, dim3((unsigned)nblk), dim3(2 * GSS_MAXCH * (S)), 0, \
                       st,                                                                      \
                       blk, nch, nblk, n_per_blk, ca_bits, n_ca, nav, n_nav, host_lut(), anch,  \
                       sin, sspec, lin, fast, first, force_exact)
    switch (proof_stride(nblk)) {
    case 32: PF_LAUNCH(32); break;
    case 16: PF_LAUNCH(16); break;
    default: PF_LAUNCH(4); break;
    }
#undef PF_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "proof kernel launch");
}

extern "C" int gss_linearize_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                                    int nblk, int n_per_blk, const uint32_t *ca_bits, int n_ca,
                                    const uint32_t *nav, int n_nav, gss_lin_t *lin, int32_t *fast,
                                    void *stream)
{
    return gss_linearize_device_ex(d, blk, nch, nblk, n_per_blk, ca_bits, n_ca, nav, n_nav, NULL,
                                   lin, fast, stream);
}

extern "C" int gss_linearize_device_ex(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                                       int nblk, int n_per_blk, const uint32_t *ca_bits, int n_ca,
                                       const uint32_t *nav, int n_nav,
                                       const gss_carr_anchor_t *anch, gss_lin_t *lin,
                                       int32_t *fast, void *stream)
{
    if (!d || !blk || !nch || !lin || !fast || nblk < 0 || n_per_blk <= 0 ||
        (n_nav > 0 && !nav) || (n_ca > 0 && !ca_bits) || n_ca < 0)
        return gss_fail(GSS_E_ARG, "invalid linearize_device arguments");
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice");
    return run_proof_launch(blk, nch, nblk, n_per_blk, ca_bits, n_ca, nav, n_nav, anch, nullptr,
                            nullptr, lin, fast, 0, 0, (hipStream_t)stream);
}
