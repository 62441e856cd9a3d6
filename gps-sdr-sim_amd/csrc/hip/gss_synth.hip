/*
 * gss_synth.hip — the hot path on gfx950: GPS L1 C/A baseband synthesis of whole 0.1 s blocks.
 *
 * Replaces the reference per-sample loop (gpssim.c:2190-2264) and its quantise/pack epilogue
 * (gpssim.c:2257-2288).  Bit-exact: the two double recurrences per channel (carrier, code) are
 * evaluated with the same IEEE double additions as the reference (-ffp-contract=off; the
 * checkpoint stage jumps over provably exact lattice runs, see common/gss_phase.h).
 *
 * Stage A  gss_ckpt_kernel      one lane per (block, channel): walks the block's carrier and code
 *                               chains exactly, writing the state every R samples (checkpoints).
 * Stage B  gss_synth_kernel     one lane per R-sample segment of a block, all channels:
 *                               LDS tables (per-channel LUT × gain, C/A chips in both polarities,
 *                               nav words), exact recurrences, integer accumulation, (acc+64)>>7,
 *                               SC16/SC08/SC01 packing, 16-byte stores.
 * Integer/byte work only: no MFMA.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "gpssim_amd.h"
#include "../common/gss_phase.h"

#define SEG_R          1024   /* samples per Stage-B lane (checkpoint spacing) */
#define SYNTH_THREADS  256
#define CKPT_THREADS   64

/* ---------------------------------------------------------------------------------------- */
/* Carrier LUT (gpssim.c:15-83): quarter wave round(250 sin(2π(k+½)/512)), entry 35 = 105.   */
/* Generated on the host once (gss_lut) and passed as a kernel argument table.               */
/* ---------------------------------------------------------------------------------------- */
struct lut_arg { int16_t sin512[512]; int16_t cos512[512]; };

/* ======================================================================================== */
/* Stage A: checkpoints                                                                     */
/* ======================================================================================== */
__global__ __launch_bounds__(CKPT_THREADS) void gss_ckpt_kernel(
    const gss_chan_blk_t *__restrict__ blk, const int32_t *__restrict__ nch, int nblk,
    int n_per_blk, int nseg, int nchp, double *__restrict__ ck_carr,
    double *__restrict__ ck_code, uint32_t *__restrict__ ck_ctr, double2 *__restrict__ steps,
    double *__restrict__ carr_end)
{
    int gid = blockIdx.x * CKPT_THREADS + threadIdx.x;
    int b = gid / GSS_MAXCH, k = gid % GSS_MAXCH;
    if (b >= nblk || k >= nchp)
        return;
    size_t row = ((size_t)b * GSS_MAXCH + k) * (size_t)nseg;
    if (k >= nch[b]) {                       /* padding channel: constant, never wraps */
        steps[(size_t)b * GSS_MAXCH + k] = make_double2(0.0, 0.0);
        for (int s = 0; s < nseg; s++) {
            ck_carr[row + s] = 0.0;
            ck_code[row + s] = 0.0;
            ck_ctr[row + s] = 0u;
        }
        return;
    }
    const gss_chan_blk_t p = blk[(size_t)b * GSS_MAXCH + k];
    /* Stage B keeps the carrier as Y = 512*carr: fl(Y + 512 s) == 512 fl(carr + s) exactly */
    steps[(size_t)b * GSS_MAXCH + k] = make_double2(p.carr_step * 512.0, p.code_step);
    double x = p.carr0;
    gss_code_state c;
    c.ph = p.code0;
    c.icode = p.icode;
    c.ibit = p.ibit;
    c.iword = p.iword;
    for (int s = 0; s < nseg; s++) {
        ck_carr[row + s] = x;
        ck_code[row + s] = c.ph;
        ck_ctr[row + s] = (uint32_t)c.icode | ((uint32_t)c.ibit << 8) | ((uint32_t)c.iword << 16);
        int len = n_per_blk - s * SEG_R;
        if (len > SEG_R) len = SEG_R;
        x = gss_carr_walk(x, p.carr_step, len);
        gss_code_walk(&c, p.code_step, len);
    }
    if (carr_end)
        carr_end[(size_t)b * GSS_MAXCH + k] = x;
}

/* ======================================================================================== */
/* Stage B: synthesis                                                                       */
/* ======================================================================================== */
template <int FMT> struct fmt_traits;
template <> struct fmt_traits<16> { static constexpr int SPV = 4; };   /* samples per 16 B */
template <> struct fmt_traits<8>  { static constexpr int SPV = 8; };
template <> struct fmt_traits<1>  { static constexpr int SPV = 64; };

__device__ __forceinline__ uint32_t hi32(double v) { return (uint32_t)__double2hiint(v); }

/* (acc+64)>>7 → int16 pair, from the packed 64-bit accumulator  I + Q*2^32 */
__device__ __forceinline__ void quantise(uint64_t acc, int &i16, int &q16)
{
    int32_t isum = (int32_t)(uint32_t)acc;
    int32_t qsum = (int32_t)((int64_t)(acc - (uint64_t)(int64_t)isum) >> 32);
    i16 = (int)(int16_t)((isum + 64) >> 7);
    q16 = (int)(int16_t)((qsum + 64) >> 7);
}

/* One output sample: all channels' contributions, then the exact state advance.
   Reference: gpssim.c:2195-2256 (per channel) and 2257-2259 (rounding). */
template <int NCH>
__device__ __forceinline__ void one_sample(double *Y, double *C, uint32_t *ctr, uint32_t *cab,
                                           const uint64_t *s_lut, const uint32_t *s_ca,
                                           const uint32_t *s_nav, const double2 *ustep,
                                           int &bad, int &i16, int &q16)
{
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        /* LUT[floor(512 carr)] × chip sign × data sign × gain (gpssim.c:2200-2209); the sign
           flips the LUT index by half a cycle: LUT[(i+256)%512] == -LUT[i]. */
        int ci = (int)C[k];
        uint32_t cw = *(const uint32_t *)((const uint8_t *)(s_ca + k * 2 * GSS_CA_WORDS) +
                                          cab[k] + ((ci >> 5) << 2));
        uint32_t neg = (cw >> (ci & 31)) & 1u;
        int ti = (int)Y[k];
        acc += s_lut[k * 512 + ((ti + (int)(neg << 8)) & 511)];

        /* carrier advance + wrap (gpssim.c:2245-2250) in Y = 512*carr units.  The test is on
           the value, like the reference: hi32(Y) >= hi32(512.0) holds exactly when Y >= 512
           or Y < 0 (sign bit); then Y -= 512 or Y += 512. */
        Y[k] = Y[k] + ustep[k].x;
        if (hi32(Y[k]) >= 0x40800000u)
            Y[k] = Y[k] + (Y[k] < 0.0 ? 512.0 : -512.0);

        /* code advance + chip/bit/word counters (gpssim.c:2212-2237) */
        C[k] = C[k] + ustep[k].y;
        if (C[k] >= 1023.0) {
            C[k] -= 1023.0;
            uint32_t c = ctr[k];
            int icode = (int)(c & 0xFF) + 1, ibit = (c >> 8) & 0xFF, iword = c >> 16;
            if (icode >= 20) {
                icode = 0;
                if (++ibit >= 30) { ibit = 0; iword++; }
                if (iword > 59) { bad = 1; iword = 59; }
                cab[k] = ((s_nav[k * 64 + iword] >> (29 - ibit)) & 1u) * (GSS_CA_WORDS * 4);
            }
            ctr[k] = (uint32_t)icode | ((uint32_t)ibit << 8) | ((uint32_t)iword << 16);
        }
    }
    quantise(acc, i16, q16);
}

/* Place one quantised sample into the 16-byte output vector (gpssim.c:2266-2287). */
template <int FMT>
__device__ __forceinline__ void pack_sample(uint32_t *word, int sidx, int i16, int q16)
{
    if (FMT == 16) {
        word[sidx] = (uint32_t)(uint16_t)i16 | ((uint32_t)(uint16_t)q16 << 16);
    } else if (FMT == 8) {                     /* iq_buff >> 4 → signed char */
        uint32_t pair = (uint32_t)(uint8_t)(int8_t)(i16 >> 4) |
                        ((uint32_t)(uint8_t)(int8_t)(q16 >> 4) << 8);
        word[sidx >> 1] |= pair << (16 * (sidx & 1));
    } else {                                   /* byte = {I0 Q0 I1 Q1 I2 Q2 I3 Q3}, MSB first */
        int byte = sidx >> 2, pos = 7 - 2 * (sidx & 3);
        uint32_t bits = ((uint32_t)(i16 > 0) << pos) | ((uint32_t)(q16 > 0) << (pos - 1));
        word[byte >> 2] |= bits << (8 * (byte & 3));
    }
}

/* 16 output bytes: one dwordx4 store when the address allows it (block bases are multiples of
   the block size, which need not be a multiple of 16, e.g. -b 1 blocks of 65000 B). */
__device__ __forceinline__ void store16(uint8_t *p, const uint32_t *w)
{
    uintptr_t a = (uintptr_t)p;
    if ((a & 15) == 0) {
        *(uint4 *)p = make_uint4(w[0], w[1], w[2], w[3]);
    } else if ((a & 3) == 0) {
        for (int i = 0; i < 4; i++)
            ((uint32_t *)p)[i] = w[i];
    } else {
        for (int i = 0; i < 16; i++)
            p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

template <int NCH, int FMT>
__global__ __launch_bounds__(SYNTH_THREADS, 2) void gss_synth_kernel(
    const gss_chan_blk_t *__restrict__ blk, const int32_t *__restrict__ nch,
    const uint32_t *__restrict__ ca_bits, const uint32_t *__restrict__ nav,
    const double *__restrict__ ck_carr, const double *__restrict__ ck_code,
    const uint32_t *__restrict__ ck_ctr, const double2 *__restrict__ steps, lut_arg lut,
    int n_per_blk, int nseg, int wg_per_blk, uint8_t *__restrict__ out, size_t block_bytes,
    int32_t *__restrict__ status)
{
    constexpr int SPV = fmt_traits<FMT>::SPV;
    __shared__ uint64_t s_lut[NCH][512];          /* (cos*gain) + (sin*gain)<<32            */
    __shared__ uint32_t s_ca[NCH][2][GSS_CA_WORDS]; /* [pol]: neg-sign bit per chip           */
    __shared__ uint32_t s_nav[NCH][64];

    const int b = blockIdx.x / wg_per_blk;
    const int w = blockIdx.x % wg_per_blk;
    const int tid = threadIdx.x;
    const int nc = nch[b];
    const gss_chan_blk_t *prow = blk + (size_t)b * GSS_MAXCH;

    /* ---- LDS tables for this block ---- */
    for (int i = tid; i < NCH * 512; i += SYNTH_THREADS) {
        int k = i >> 9, j = i & 511;
        int32_t g = k < nc ? prow[k].gain : 0;
        int64_t I = (int64_t)lut.cos512[j] * g, Q = (int64_t)lut.sin512[j] * g;
        s_lut[k][j] = (uint64_t)I + ((uint64_t)Q << 32);
    }
    for (int i = tid; i < NCH * GSS_CA_WORDS; i += SYNTH_THREADS) {
        int k = i / GSS_CA_WORDS, j = i % GSS_CA_WORDS;
        uint32_t v = k < nc ? ca_bits[(size_t)prow[k].ca_tbl * GSS_CA_WORDS + j] : 0u;
        /* sign = dataBit*codeCA is negative iff chip != data bit:
           pol 0 (data bit 0): neg = chip;  pol 1 (data bit 1): neg = !chip */
        s_ca[k][0][j] = v;
        s_ca[k][1][j] = ~v;
    }
    for (int i = tid; i < NCH * 64; i += SYNTH_THREADS) {
        int k = i >> 6, j = i & 63;
        s_nav[k][j] = (k < nc && j < GSS_NAV_WORDS)
                          ? nav[(size_t)prow[k].nav_tbl * GSS_NAV_WORDS + j] : 0u;
    }
    __syncthreads();
    const double2 *ustep = steps + (size_t)b * GSS_MAXCH;   /* block-uniform: scalar loads */

    const int seg = w * SYNTH_THREADS + tid;
    if (seg >= nseg)
        return;
    int len = n_per_blk - seg * SEG_R;
    if (len > SEG_R) len = SEG_R;

    /* ---- per-lane channel state from the checkpoints ---- */
    double Y[NCH], C[NCH];
    uint32_t ctr[NCH], cab[NCH];
    int bad = 0;
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        size_t r = ((size_t)b * GSS_MAXCH + k) * (size_t)nseg + seg;
        Y[k] = ck_carr[r] * 512.0;
        C[k] = ck_code[r];
        ctr[k] = ck_ctr[r];
        int ibit = (ctr[k] >> 8) & 0xFF, iword = ctr[k] >> 16;
        if (iword > 59) { bad = 1; iword = 59; }
        uint32_t d = (s_nav[k][iword] >> (29 - ibit)) & 1u;
        cab[k] = d * (GSS_CA_WORDS * 4);              /* byte offset of the polarity table */
    }

    uint8_t *dst = out + (size_t)b * block_bytes;
    size_t byte0 = FMT == 16 ? (size_t)seg * SEG_R * 4 : FMT == 8 ? (size_t)seg * SEG_R * 2
                                                       : (size_t)seg * SEG_R / 4;
    uint8_t *vdst = dst + byte0;
    const int nfull = len / SPV;

    for (int v = 0; v < nfull; v++) {
        uint32_t word[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int sidx = 0; sidx < SPV; sidx++) {
            int i16, q16;
            one_sample<NCH>(Y, C, ctr, cab, &s_lut[0][0], &s_ca[0][0][0], &s_nav[0][0], ustep,
                            bad, i16, q16);
            pack_sample<FMT>(word, sidx, i16, q16);
        }
        store16(vdst + 16 * v, word);
    }
    const int remain = len - nfull * SPV;           /* ragged tail of the block's last segment */
    if (remain > 0) {
        uint32_t word[4] = {0u, 0u, 0u, 0u};
        for (int sidx = 0; sidx < remain; sidx++) {
            int i16, q16;
            one_sample<NCH>(Y, C, ctr, cab, &s_lut[0][0], &s_ca[0][0][0], &s_nav[0][0], ustep,
                            bad, i16, q16);
            pack_sample<FMT>(word, sidx, i16, q16);
        }
        int nbytes = FMT == 16 ? remain * 4 : FMT == 8 ? remain * 2 : remain / 4;
        uint8_t *bp = vdst + 16 * nfull;
        for (int i = 0; i < nbytes; i++)
            bp[i] = (uint8_t)(word[i >> 2] >> (8 * (i & 3)));
    }
    if (bad && status)
        atomicOr(status, 1);
}

/* ======================================================================================== */
/* C ABI                                                                                    */
/* ======================================================================================== */
struct gss_dev {
    int ordinal;
    double *ck_carr = nullptr, *ck_code = nullptr;
    uint32_t *ck_ctr = nullptr;
    size_t ck_cap = 0;                   /* entries */
    double2 *steps = nullptr;
    size_t steps_cap = 0;                /* blocks */
    static constexpr int RING = 256;
    hipEvent_t ev[RING][3];
    int n_ev = 0;                        /* launches recorded since the last reset */
    lut_arg lut;
    /* host-call staging */
    void *h_in = nullptr; size_t h_in_cap = 0;
    void *d_out = nullptr; size_t d_out_cap = 0;
    double *d_cend = nullptr; size_t d_cend_cap = 0;
    int32_t *d_status = nullptr;
};

extern "C" int gss_fail(int code, const char *fmt, ...);

#define HIP_TRY(x)                                                                           \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess)                                                                \
            return gss_fail(GSS_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_),      \
                            __FILE__, __LINE__);                                             \
    } while (0)

extern "C" size_t gss_block_bytes(int n, int fmt)
{
    if (n <= 0) return 0;
    switch (fmt) {
    case GSS_FMT_SC16: return (size_t)n * 4;
    case GSS_FMT_SC08: return (size_t)n * 2;
    case GSS_FMT_SC01: return (n % 4) ? 0 : (size_t)n / 4;
    default: return 0;
    }
}

extern "C" int gss_dev_open(gss_dev **out, int ordinal)
{
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return gss_fail(GSS_E_NODEV, "no HIP device visible");
    if (ordinal < 0 || ordinal >= count)
        return gss_fail(GSS_E_ARG, "device ordinal %d out of range (%d devices)", ordinal, count);
    HIP_TRY(hipSetDevice(ordinal));
    gss_dev *d = new gss_dev();
    d->ordinal = ordinal;
    for (int r = 0; r < gss_dev::RING; r++)
        for (int i = 0; i < 3; i++)
            HIP_TRY(hipEventCreate(&d->ev[r][i]));
    int32_t s[512], c[512];
    gss_lut(s, c);
    for (int i = 0; i < 512; i++) {
        d->lut.sin512[i] = (int16_t)s[i];
        d->lut.cos512[i] = (int16_t)c[i];
    }
    HIP_TRY(hipMalloc(&d->d_status, sizeof(int32_t)));
    *out = d;
    return 0;
}

extern "C" int gss_dev_close(gss_dev *d)
{
    if (!d) return 0;
    (void)hipSetDevice(d->ordinal);
    void *bufs[] = {d->ck_carr, d->ck_code, d->ck_ctr, d->steps, d->h_in, d->d_out, d->d_cend,
                    d->d_status};
    for (void *p : bufs)
        (void)hipFree(p);
    for (int r = 0; r < gss_dev::RING; r++)
        for (int i = 0; i < 3; i++)
            (void)hipEventDestroy(d->ev[r][i]);
    delete d;
    return 0;
}

static int nseg_of(int n) { return (n + SEG_R - 1) / SEG_R; }

extern "C" int gss_dev_reserve(gss_dev *d, int max_blocks, int n_per_blk)
{
    if (!d || max_blocks <= 0 || n_per_blk <= 0)
        return gss_fail(GSS_E_ARG, "invalid reserve arguments");
    HIP_TRY(hipSetDevice(d->ordinal));
    if ((size_t)max_blocks > d->steps_cap) {
        (void)hipFree(d->steps);
        d->steps = nullptr;
        d->steps_cap = 0;
        HIP_TRY(hipMalloc(&d->steps, sizeof(double2) * GSS_MAXCH * (size_t)max_blocks));
        d->steps_cap = (size_t)max_blocks;
    }
    size_t need = (size_t)max_blocks * GSS_MAXCH * (size_t)nseg_of(n_per_blk);
    if (need <= d->ck_cap)
        return 0;
    (void)hipFree(d->ck_carr); (void)hipFree(d->ck_code); (void)hipFree(d->ck_ctr);
    d->ck_carr = d->ck_code = nullptr; d->ck_ctr = nullptr; d->ck_cap = 0;
    HIP_TRY(hipMalloc(&d->ck_carr, need * sizeof(double)));
    HIP_TRY(hipMalloc(&d->ck_code, need * sizeof(double)));
    HIP_TRY(hipMalloc(&d->ck_ctr, need * sizeof(uint32_t)));
    d->ck_cap = need;
    return 0;
}

typedef void (*synth_fn)(const gss_chan_blk_t *, const int32_t *, const uint32_t *,
                         const uint32_t *, const double *, const double *, const uint32_t *,
                         const double2 *, lut_arg, int, int, int, uint8_t *, size_t, int32_t *);

template <int FMT> static synth_fn pick_nch(int nchp)
{
    switch (nchp) {
#define C(N) case N: return gss_synth_kernel<N, FMT>;
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15) C(16)
#undef C
    default: return nullptr;
    }
}

static synth_fn pick_kernel(int fmt, int nchp)
{
    switch (fmt) {
    case 16: return pick_nch<16>(nchp);
    case 8: return pick_nch<8>(nchp);
    case 1: return pick_nch<1>(nchp);
    default: return nullptr;
    }
}

extern "C" int gss_synth_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                                int nch_max, const uint32_t *ca_bits, int n_ca, const uint32_t *nav,
                                int n_nav, int nblk, int n_per_blk, int fmt, void *out,
                                double *carr_end, int32_t *status, void *stream)
{
    (void)n_ca; (void)n_nav;
    if (!d || !blk || !nch || !ca_bits || !out || nblk <= 0 || n_per_blk <= 0)
        return gss_fail(GSS_E_ARG, "invalid synth arguments");
    size_t bb = gss_block_bytes(n_per_blk, fmt);
    if (bb == 0)
        return gss_fail(GSS_E_ARG, "invalid format %d for %d samples/block", fmt, n_per_blk);
    HIP_TRY(hipSetDevice(d->ordinal));
    int rc = gss_dev_reserve(d, nblk, n_per_blk);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    int nseg = nseg_of(n_per_blk);
    int nchp = nch_max < 1 ? 1 : nch_max;         /* kernel instance; fewer channels padded */
    if (nchp > GSS_MAXCH)
        return gss_fail(GSS_E_ARG, "nch_max %d > %d", nch_max, GSS_MAXCH);
    synth_fn fn = pick_kernel(fmt, nchp);
    if (!fn)
        return gss_fail(GSS_E_ARG, "no kernel for fmt=%d nch=%d", fmt, nchp);

    int ck_blocks = (nblk * GSS_MAXCH + CKPT_THREADS - 1) / CKPT_THREADS;
    hipEvent_t *ev = d->ev[d->n_ev % gss_dev::RING];
    d->n_ev++;
    HIP_TRY(hipEventRecord(ev[0], st));
    hipLaunchKernelGGL(gss_ckpt_kernel, dim3(ck_blocks), dim3(CKPT_THREADS), 0, st, blk, nch,
                       nblk, n_per_blk, nseg, nchp, d->ck_carr, d->ck_code, d->ck_ctr,
                       d->steps, carr_end);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[1], st));
    int wg_per_blk = (nseg + SYNTH_THREADS - 1) / SYNTH_THREADS;
    hipLaunchKernelGGL(fn, dim3(nblk * wg_per_blk), dim3(SYNTH_THREADS), 0, st, blk, nch,
                       ca_bits, nav, d->ck_carr, d->ck_code, d->ck_ctr, d->steps, d->lut,
                       n_per_blk, nseg, wg_per_blk, (uint8_t *)out, bb, status);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[2], st));
    return 0;
}

extern "C" int gss_dev_timing(gss_dev *d, int reset, int *n, float *ckpt_ms, float *synth_ms)
{
    if (!d) return gss_fail(GSS_E_ARG, "null device");
    if (reset) {
        d->n_ev = 0;
        return 0;
    }
    int cnt = d->n_ev < gss_dev::RING ? d->n_ev : gss_dev::RING;
    double a = 0.0, b = 0.0;
    if (cnt > 0) {
        HIP_TRY(hipEventSynchronize(d->ev[(d->n_ev - 1) % gss_dev::RING][2]));
        for (int i = 0; i < cnt; i++) {
            hipEvent_t *e = d->ev[(d->n_ev - 1 - i) % gss_dev::RING];
            float t0 = 0.f, t1 = 0.f;
            HIP_TRY(hipEventElapsedTime(&t0, e[0], e[1]));
            HIP_TRY(hipEventElapsedTime(&t1, e[1], e[2]));
            a += t0;
            b += t1;
        }
        a /= cnt;
        b /= cnt;
    }
    if (n) *n = cnt;
    if (ckpt_ms) *ckpt_ms = (float)a;
    if (synth_ms) *synth_ms = (float)b;
    return 0;
}

template <class T> static int grow(T **p, size_t *cap, size_t need)
{
    if (need <= *cap) return 0;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc((void **)p, need));
    *cap = need;
    return 0;
}

extern "C" int gss_synth_host(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                              const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                              int nblk, int n_per_blk, int fmt, void *out, double *carr_end)
{
    if (!d || !blk || !nch || !ca_bits || !out || nblk <= 0 || n_ca <= 0)
        return gss_fail(GSS_E_ARG, "invalid synth arguments");
    size_t bb = gss_block_bytes(n_per_blk, fmt);
    if (bb == 0)
        return gss_fail(GSS_E_ARG, "invalid format %d for %d samples/block", fmt, n_per_blk);
    HIP_TRY(hipSetDevice(d->ordinal));
    int maxc = 1;
    for (int b = 0; b < nblk; b++) {
        if (nch[b] < 0 || nch[b] > GSS_MAXCH)
            return gss_fail(GSS_E_ARG, "nch[%d]=%d out of range", b, nch[b]);
        if (nch[b] > maxc) maxc = nch[b];
        for (int k = 0; k < nch[b]; k++) {
            const gss_chan_blk_t *p = &blk[(size_t)b * GSS_MAXCH + k];
            if (p->ca_tbl < 0 || p->ca_tbl >= n_ca || p->nav_tbl < 0 || p->nav_tbl >= n_nav ||
                p->ibit < 0 || p->ibit >= 30 || p->icode < 0 || p->icode >= 20 || p->iword < 0 ||
                p->iword >= GSS_NAV_WORDS || !(p->code0 >= 0.0 && p->code0 < 1023.0) ||
                !(p->carr0 >= 0.0 && p->carr0 <= 1.0))
                return gss_fail(GSS_E_ARG, "block %d channel %d: parameter out of range", b, k);
        }
    }
    size_t sz_blk = sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)nblk;
    size_t sz_nch = sizeof(int32_t) * (size_t)nblk;
    size_t sz_ca = sizeof(uint32_t) * GSS_CA_WORDS * (size_t)n_ca;
    size_t sz_nav = sizeof(uint32_t) * GSS_NAV_WORDS * (size_t)(n_nav > 0 ? n_nav : 1);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t tot = al(sz_blk) + al(sz_nch) + al(sz_ca) + al(sz_nav);
    int rc = grow((uint8_t **)&d->h_in, &d->h_in_cap, tot);
    if (rc) return rc;
    uint8_t *base = (uint8_t *)d->h_in;
    gss_chan_blk_t *d_blk = (gss_chan_blk_t *)base;
    int32_t *d_nch = (int32_t *)(base + al(sz_blk));
    uint32_t *d_ca = (uint32_t *)(base + al(sz_blk) + al(sz_nch));
    uint32_t *d_nav = (uint32_t *)(base + al(sz_blk) + al(sz_nch) + al(sz_ca));
    HIP_TRY(hipMemcpy(d_blk, blk, sz_blk, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_nch, nch, sz_nch, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_ca, ca_bits, sz_ca, hipMemcpyHostToDevice));
    if (n_nav > 0)
        HIP_TRY(hipMemcpy(d_nav, nav, sz_nav, hipMemcpyHostToDevice));
    else
        HIP_TRY(hipMemset(d_nav, 0, sz_nav));
    rc = grow((uint8_t **)&d->d_out, &d->d_out_cap, bb * (size_t)nblk);
    if (rc) return rc;
    double *d_cend = nullptr;
    if (carr_end) {
        rc = grow(&d->d_cend, &d->d_cend_cap, sizeof(double) * GSS_MAXCH * (size_t)nblk);
        if (rc) return rc;
        d_cend = d->d_cend;
    }
    HIP_TRY(hipMemset(d->d_status, 0, sizeof(int32_t)));
    rc = gss_synth_device(d, d_blk, d_nch, maxc, d_ca, n_ca, d_nav, n_nav, nblk, n_per_blk, fmt,
                          d->d_out, d_cend, d->d_status, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, d->d_out, bb * (size_t)nblk, hipMemcpyDeviceToHost));
    if (carr_end)
        HIP_TRY(hipMemcpy(carr_end, d_cend, sizeof(double) * GSS_MAXCH * (size_t)nblk,
                          hipMemcpyDeviceToHost));
    int32_t st = 0;
    HIP_TRY(hipMemcpy(&st, d->d_status, sizeof st, hipMemcpyDeviceToHost));
    if (st)
        return gss_fail(GSS_E_RANGE, "nav word index ran past dwrd[59]");
    return 0;
}
