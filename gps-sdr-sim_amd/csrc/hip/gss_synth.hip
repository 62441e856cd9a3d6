/*
 * gss_synth.hip — the hot path on gfx950: GPS L1 C/A baseband synthesis of whole 0.1 s blocks.
 *
 * Replaces the reference per-sample loop (gpssim.c:2190-2264) and its quantise/pack epilogue
 * (gpssim.c:2257-2288).  Bit-exact: every channel's carrier and code phase are the reference's
 * serial IEEE double recurrences (built with -ffp-contract=off); the only shortcuts are provably
 * exact lattice translations (common/gss_phase.h).
 *
 * Stage A  gss_anchor_kernel    one lane per (block, channel, chain); waves are channel-major
 *                               (64 consecutive blocks, one chain kind), walking the block with
 *                               direction-specialised branch-free f64 lattice trips (gss_trip)
 *                               and recording the exact phase (and code counters) at every
 *                               R-sample segment start (gss_seg_states).
 * Stage B  gss_synth_kernel     one lane per R-sample segment of a block, all channels.  Each lane
 *                               first walks every channel from its anchor to the segment start
 *                               (≤ one cycle, no wrap), then runs the per-sample recurrences:
 *                               carrier via v_fract_f64, chip sign from a byte table, data-bit
 *                               sign folded into the gain, LUT[floor(512 carr)] x gain summed
 *                               over channels with v_dot2 on packed int16, (acc+64)>>7,
 *                               SC16/SC08/SC01 packing.  Output is staged per lane in LDS
 *                               (128 B) and stored by the wave as whole 128-B lines.
 * gss_lin_kernel (the fast path, below) renders the blocks the host proof certifies: integer
 * phase lines, LDS LUT reads, and the gain x LUT sums on the matrix cores.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "gpssim_amd.h"
#include "../common/gss_phase.h"
#include "../common/gss_lin.h"

#define SYNTH_THREADS  256
#define SYNTH_WAVES    (SYNTH_THREADS / 64)
#define ANCHOR_THREADS 64                /* one wave per workgroup: a wave is one chain kind  */
#define CHUNK_BYTES    128               /* output bytes per lane per staged chunk: a line */
#define CHUNK_PIECES   (CHUNK_BYTES / 16)
#define LUT_N          1024              /* index ti + 256*neg <= 767; padded to a power of 2 */

struct lut_arg { int16_t sin512[512]; int16_t cos512[512]; };

/* ======================================================================================== */
/* Stage A: anchors                                                                         */
/* ======================================================================================== */
/* Stage A walks one chain per lane.  Waves are channel-major: a wave holds one chain kind of one
   channel slot for 64 consecutive blocks, so the carrier's Doppler sign, and with it the
   specialised trip (gss_trip: ascending / descending carrier, code), is wave-uniform except
   across a zero crossing.  The trip is issue-bound (~9-cycle dependent f64 latency but ~50-100
   VALU per trip, measured in tools/ubench/), so one chain per lane beats interleaving two.  The
   walk is gss_seg_states: the exact state at every segment start, interpolated on the lattice
   jump that crosses it. */
__global__ __launch_bounds__(ANCHOR_THREADS) void gss_anchor_kernel(
    const gss_chan_blk_t *__restrict__ blk, const int32_t *__restrict__ nch,
    const double *__restrict__ carr_ck, int nblk, int nchp, int n_per_blk, int nseg, int nsegp,
    int seg_r, double *__restrict__ seg_carr, double *__restrict__ seg_code,
    uint32_t *__restrict__ seg_cnt, double *__restrict__ carr_end,
    const int32_t *__restrict__ blist)
{
    /* blist (optional): the batch's blocks this launch handles (the fast path's leftovers);
       anchor rows are indexed by the position in the list, everything else by the block */
    /* wave index space: [longest chains first] code waves nchp x nbw (one lane per block) and
       carrier waves nchp x nbwc (one lane per block sub-chain: GSS_NCK of them per block when
       the planner's checkpoints are given, else one) */
    const int nsub = carr_ck ? GSS_NCK : 1;
    const int nbw = (nblk + ANCHOR_THREADS - 1) / ANCHOR_THREADS;
    const int nbwc = (nblk * nsub + ANCHOR_THREADS - 1) / ANCHOR_THREADS;
    int wid = blockIdx.x;
    bool code;
    if (carr_ck) {
        code = wid < nchp * nbw;
        if (!code) wid -= nchp * nbw;
    } else {
        code = wid >= nchp * nbwc;
        if (code) wid -= nchp * nbwc;
    }
    const int per = code ? nbw : nbwc;
    const int k = wid / per;
    const int idx = (wid - k * per) * ANCHOR_THREADS + threadIdx.x;
    const int sub = code ? 1 : nsub;                       /* lanes per block */
    const int b = idx / sub, j = idx - b * sub;
    if (k >= nchp || b >= nblk)
        return;
    const int rb = blist ? blist[b] : b;                  /* the block itself */
    const size_t bk = (size_t)rb * GSS_MAXCH + k;
    const size_t row = ((size_t)b * GSS_MAXCH + k) * (size_t)nsegp;
    const bool real = k < nch[rb];
    /* padding channels of the kernel instance: no motion (Stage B gives them no gain) */
    gss_chan_blk_t p = blk[bk];
    if (!real) {
        p.carr0 = p.carr_step = p.code0 = p.code_step = 0.0;
        p.icode = p.ibit = p.iword = 0;
    }
    if (code) {
        const uint32_t cnt = (uint32_t)p.icode | ((uint32_t)p.ibit << 8) |
                             ((uint32_t)p.iword << 16);
        /* code chains (one per block) are the long pole of the kernel and few: latency-bound, so
           the branch-free walk; a code step below 2^-16 (not a GNSS sample rate) takes the
           general walk.  Slot nseg of the row is the walk's dummy store target. */
        if (!GSS_ANY(p.code_step != 0.0 && p.code_step < 0x1p-16))
            gss_code_seg_states_bf(p.code0, p.code_step, cnt, n_per_blk, nseg, seg_r, nseg,
                                   seg_code + row, seg_cnt + row);
        else
            gss_seg_states(GSS_TRIP_CODE, p.code0, p.code_step, cnt, 0, n_per_blk, nseg, seg_r, 0,
                           seg_code + row, seg_cnt + row);
        return;
    }
    const int pos0 = carr_ck ? gss_ck_pos(j, n_per_blk) : 0;
    const int pos1 = j + 1 < nsub ? gss_ck_pos(j + 1, n_per_blk) : n_per_blk;
    const double v0 = carr_ck && real ? carr_ck[bk * GSS_NCK + j] : p.carr0;
    const bool want_end = carr_end != nullptr && real && j == nsub - 1;
    const bool desc = p.carr_step < 0.0;
    const uint64_t nd = __builtin_amdgcn_ballot_w64(desc);
    double e;
    if (nd == 0)                                           /* the usual case: uniform sign */
        e = gss_seg_states(GSS_TRIP_CARR_ASC, v0, p.carr_step, 0u, pos0, pos1, nseg, seg_r,
                           want_end, seg_carr + row, nullptr);
    else if (nd == __builtin_amdgcn_ballot_w64(true))
        e = gss_seg_states(GSS_TRIP_CARR_DESC, v0, p.carr_step, 0u, pos0, pos1, nseg, seg_r,
                           want_end, seg_carr + row, nullptr);
    else if (desc)                                         /* mixed wave: both paths, in turn */
        e = gss_seg_states(GSS_TRIP_CARR_DESC, v0, p.carr_step, 0u, pos0, pos1, nseg, seg_r,
                           want_end, seg_carr + row, nullptr);
    else
        e = gss_seg_states(GSS_TRIP_CARR_ASC, v0, p.carr_step, 0u, pos0, pos1, nseg, seg_r,
                           want_end, seg_carr + row, nullptr);
    if (want_end)
        carr_end[bk] = e;
}

/* ======================================================================================== */
/* Stage B: synthesis                                                                       */
/* ======================================================================================== */
template <int FMT> struct fmt_traits;
template <> struct fmt_traits<16> { static constexpr int SPC = CHUNK_BYTES / 4; }; /* samples/chunk */
template <> struct fmt_traits<8>  { static constexpr int SPC = CHUNK_BYTES / 2; };
template <> struct fmt_traits<1>  { static constexpr int SPC = CHUNK_BYTES * 4; };

/* floor(512 carr) and floor(C) for four channels with one v_add_f64 each: in round-toward-
   zero mode, carr + 2^43 lands on the lattice 2^-9 of [2^43, 2^43+1) at 2^43 + floor(512 carr)/512,
   so its low word is floor(512 carr) (carr in [0,1)); C + 2^52 has lattice 1, low word floor(C)
   (C in [0,1024)).  The MODE switch (double rounding field, bits 3:2) and the adds sit in one asm
   block so that no other floating-point instruction runs in the modified mode. */
__device__ __forceinline__ void floors4(double c0, double c1, double c2, double c3, double k0,
                                        double k1, double k2, double k3, uint32_t *ti,
                                        uint32_t *ci)
{
    double y0, y1, y2, y3, z0, z1, z2, z3;
    const double M9 = 0x1p43, M52 = 0x1p52;
    asm volatile(
        "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3\n\t"
        "s_nop 3\n\t"
        "v_add_f64 %0, %8, %16\n\t"
        "v_add_f64 %1, %9, %16\n\t"
        "v_add_f64 %2, %10, %16\n\t"
        "v_add_f64 %3, %11, %16\n\t"
        "v_add_f64 %4, %12, %17\n\t"
        "v_add_f64 %5, %13, %17\n\t"
        "v_add_f64 %6, %14, %17\n\t"
        "v_add_f64 %7, %15, %17\n\t"
        "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 0\n\t"
        "s_nop 3"
        : "=&v"(y0), "=&v"(y1), "=&v"(y2), "=&v"(y3), "=&v"(z0), "=&v"(z1), "=&v"(z2), "=&v"(z3)
        : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "v"(k0), "v"(k1), "v"(k2), "v"(k3), "s"(M9),
          "s"(M52));
    ti[0] = (uint32_t)__double2loint(y0); ti[1] = (uint32_t)__double2loint(y1);
    ti[2] = (uint32_t)__double2loint(y2); ti[3] = (uint32_t)__double2loint(y3);
    ci[0] = (uint32_t)__double2loint(z0); ci[1] = (uint32_t)__double2loint(z1);
    ci[2] = (uint32_t)__double2loint(z2); ci[3] = (uint32_t)__double2loint(z3);
}

/* 16 bytes to global memory: one dwordx4 store when aligned (block bases are multiples of the
   block size, e.g. 65000 B at -b 1, so not always). */
__device__ __forceinline__ void store16(uint8_t *p, uint4 v)
{
    uintptr_t a = (uintptr_t)p;
    if ((a & 15) == 0) {
        *(uint4 *)p = v;
    } else if ((a & 3) == 0) {
        ((uint32_t *)p)[0] = v.x; ((uint32_t *)p)[1] = v.y;
        ((uint32_t *)p)[2] = v.z; ((uint32_t *)p)[3] = v.w;
    } else {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int i = 0; i < 16; i++)
            p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* data-bit sign folded into the gain: I + 2^22 Q += (dataBit*gain) * (codeCA*(cos + 2^22 sin)) */
__device__ __forceinline__ int signed_gain(int gain, uint32_t bit) { return bit ? gain : -gain; }

/* Chip signs come from a per-lane 32-chip register window per channel, refreshed every P
   samples from a bit-packed, cyclically extended chip table in LDS (CBITS_W words per channel:
   bit j = codeCA(j mod 1023) < 0, j < 32 CBITS_W).  The window taken at extended chip index
   `base` is rotated: bit p holds the chip j in [base, base+32) with j = p (mod 32), so the sign
   of chip floor(C) is v_bfe_u32(win, floor(C), 1) (the offset is taken mod 32) with no
   per-lane base.  The code phase advances <= ks_max chips per sample, so P = floor(29/ks_max)
   samples (>= 1) never leave the window.  The lazy code wrap keeps the extended index
   continuous: floor(C) = 1023.. reads the extension, and the wrap (C -= 1023, i.e. +1 mod 32)
   rotates the window left by one. */
#ifndef SYNTH_OCC
#define SYNTH_OCC(nch) ((nch) <= 12 ? 3 : 2)   /* waves per SIMD the register budget targets */
#endif
#define CBITS_W 68                         /* covers extended indices < 2176 (C < 1023 + ks)  */

template <int NCH, int FMT>
__global__ __launch_bounds__(SYNTH_THREADS) __attribute__((amdgpu_waves_per_eu(SYNTH_OCC(NCH)))) void gss_synth_kernel(
    const gss_chan_blk_t *__restrict__ blk, const int32_t *__restrict__ nch,
    const uint32_t *__restrict__ ca_bits, const uint32_t *__restrict__ nav,
    const double *__restrict__ seg_carr, const double *__restrict__ seg_code,
    const uint32_t *__restrict__ seg_cnt, lut_arg lut, int n_per_blk, int nseg, int nsegp,
    int seg_r, int wg_per_blk, uint8_t *__restrict__ out, size_t block_bytes, int32_t *__restrict__ status,
    const int32_t *__restrict__ blist)
{
    constexpr int SPC = fmt_traits<FMT>::SPC;
    constexpr int NCH4 = (NCH + 3) & ~3;
    constexpr int BPS4 = FMT == 16 ? 16 : FMT == 8 ? 8 : 1;      /* 4 x bytes per sample */
    __shared__ int32_t s_lut[LUT_N];                      /* cos + 2^22 sin, index mod 512   */
    __shared__ uint32_t s_cbits[NCH][CBITS_W];            /* extended chip-sign bits         */
    __shared__ uint32_t s_nav[NCH][64];
    __shared__ uint16_t s_st[NCH][SYNTH_THREADS];         /* code counters, touched on wraps only:
                                                             icode | ibit<<5 | iword<<10 */
    __shared__ uint32_t s_stage[SYNTH_WAVES][64 * CHUNK_BYTES / 4];

    const int bc = blockIdx.x / wg_per_blk;                /* anchor row (list position)   */
    const int b = blist ? blist[bc] : bc;                  /* the block                    */
    const int w = blockIdx.x % wg_per_blk;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int nc = nch[b];
    const gss_chan_blk_t *prow = blk + (size_t)b * GSS_MAXCH;

    /* ---- LDS tables for this block ---- */
    for (int i = tid; i < LUT_N; i += SYNTH_THREADS) {
        int j = i & 511;                                  /* LUT[i+256] = -LUT[i] (mod 512) */
        s_lut[i] = (int32_t)lut.cos512[j] + (int32_t)lut.sin512[j] * (1 << 22);
    }
    for (int i = tid; i < NCH * CBITS_W; i += SYNTH_THREADS) {
        int k = i / CBITS_W, wd = i % CBITS_W;
        uint32_t v = 0;
        if (k < nc) {
            const uint32_t *cb = ca_bits + (size_t)prow[k].ca_tbl * GSS_CA_WORDS;
            int j = (32 * wd) % 1023;
            for (int q = 0; q < 32; q++) {
                v |= (((cb[j >> 5] >> (j & 31)) & 1u) ^ 1u) << q;
                j = j == 1022 ? 0 : j + 1;
            }
        }
        s_cbits[k][wd] = v;
    }
    for (int i = tid; i < NCH * 64; i += SYNTH_THREADS) {
        int k = i >> 6, j = i & 63;
        s_nav[k][j] = (k < nc && j < GSS_NAV_WORDS)
                          ? nav[(size_t)prow[k].nav_tbl * GSS_NAV_WORDS + j] : 0u;
    }
    __syncthreads();

    const int seg = w * SYNTH_THREADS + tid;
    const bool active = seg < nseg;
    const int n0 = seg * seg_r;
    int len = active ? n_per_blk - n0 : 0;
    if (len > seg_r) len = seg_r;
    const int segc = active ? seg : nseg - 1;           /* inactive lanes: any valid anchor */

    /* block-uniform channel steps (scalar registers); padding channels: no motion, no gain.
       Gains are re-read (scalar loads) where a data bit changes, to spare scalar registers. */
    double cs[NCH], ks[NCH];
    double ks_max = 0.0;
    int gsum = 0;
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        const bool real = k < nc;
        cs[k] = real ? prow[k].carr_step : 0.0;
        ks[k] = real ? prow[k].code_step : 0.0;
        ks_max = fmax(ks_max, ks[k]);
        const int gk = real ? prow[k].gain : 0;
        gsum += gk < 0 ? -gk : gk;
    }
    /* window refresh period (see CBITS_W) */
    const int P = ks_max < 29.0 / 65536.0 ? 65536 : max(1, (int)(29.0 / ks_max));
    /* the packed int64 accumulator needs |sum I + 64| < 2^21: 250 * sum|gain| + 64 (the
       reference's gains are <= 129 per channel); larger gains take the int32 path */
    const bool big = gsum > 8000;

    /* ---- exact per-lane start state (Stage A), every channel of the instance ---- */
    double carr[NCH], C[NCH];
    int g[NCH];                   /* gain with the data-bit sign */
    uint32_t win[NCH];            /* rotated chip-sign window (see CBITS_W) */
    int bad = 0;
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        const size_t r = ((size_t)bc * GSS_MAXCH + k) * (size_t)nsegp + segc;
        carr[k] = seg_carr[r];
        C[k] = seg_code[r];
        uint32_t c = seg_cnt[r];
        int ibit = (c >> 8) & 0xFF, iw = c >> 16;
        if (iw > 59) { bad |= 1; iw = 59; c = (c & 0xFFFFu) | (59u << 16); }
        s_st[k][tid] = (uint16_t)((c & 0x1Fu) | (((c >> 8) & 0x1Fu) << 5) | ((c >> 16) << 10));
        g[k] = signed_gain(k < nc ? prow[k].gain : 0, (s_nav[k][iw] >> (29 - ibit)) & 1u);
        win[k] = 0;
    }

    uint8_t *dst = out + (size_t)b * block_bytes + (size_t)n0 * BPS4 / 4;
    uint32_t *stg = s_stage[wave];
    uint32_t *mine = stg + lane * (CHUNK_BYTES / 4);
    const int nchunk = len / SPC;                       /* full chunks of this lane */
    int lane_chunks = (len + SPC - 1) / SPC;
    for (int off = 32; off > 0; off >>= 1)
        lane_chunks = max(lane_chunks, __shfl_xor(lane_chunks, off));
    /* wave-uniform trip counts (chunks and samples): lanes past their own end keep computing
       (harmlessly, nothing is stored) so that no loop-carried state sits under divergent
       control flow */
    const int wave_chunks = __builtin_amdgcn_readfirstlane(lane_chunks);
    int left = 0;                                       /* samples until the next refresh */

    for (int ch = 0; ch < wave_chunks; ch++) {
        const bool full = ch < nchunk;
        const int nsamp = full ? SPC : (ch == nchunk ? len - nchunk * SPC : 0);
        uint32_t bits = 0;
#pragma unroll 1
        for (int sidx = 0; sidx < SPC; sidx++) {
            /* floor(512 carr) and floor(C) of the current state, four channels per mode switch */
            uint32_t ti[NCH4], ci[NCH4];
#pragma unroll
            for (int k0 = 0; k0 < NCH; k0 += 4)
                floors4(carr[k0], carr[min(k0 + 1, NCH - 1)], carr[min(k0 + 2, NCH - 1)],
                        carr[min(k0 + 3, NCH - 1)], C[k0], C[min(k0 + 1, NCH - 1)],
                        C[min(k0 + 2, NCH - 1)], C[min(k0 + 3, NCH - 1)], &ti[k0], &ci[k0]);
            if (left == 0) {                          /* uniform: new chip windows at floor(C) */
#pragma unroll
                for (int k = 0; k < NCH; k++) {
                    const uint32_t base = ci[k];
                    const uint32_t *row = &s_cbits[k][base >> 5];
                    const uint32_t hi_mask = 0xFFFFFFFFu << (base & 31u);   /* v_bfi */
                    win[k] = (row[0] & hi_mask) | (row[1] & ~hi_mask);
                }
                left = P;
            }
            left--;
            /* chip sign (1 = codeCA -1) of every channel, before the wrap below rotates win */
            uint32_t t[NCH];
#pragma unroll
            for (int k = 0; k < NCH; k++) {
                t[k] = __builtin_amdgcn_ubfe(win[k], ci[k], 1);
                asm volatile("" : "+v"(t[k]));   /* keep above the branch: no copies of win */
            }
            /* the code phase of the previous step may have reached 1023 (gpssim.c:2214): apply
               that wrap now, before this step's add; floor(C) >= 1023 reads the table's cyclic
               extension.  Rare (once per ~2600 samples per channel): a uniform branch per
               channel, selects inside, so no loop-carried state sits under divergent control
               flow. */
            uint32_t cmax = ci[0];
#pragma unroll
            for (int k = 1; k < NCH; k++)
                cmax = max(cmax, ci[k]);                      /* v_max3_u32 */
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(cmax >= 1023u) != 0, 0)) {
#pragma unroll
                for (int k = 0; k < NCH; k++) {
                    const bool wk = ci[k] >= 1023u;
                    if (__builtin_amdgcn_ballot_w64(wk)) {    /* gpssim.c:2214-2237 */
                        C[k] = wk ? C[k] - GSS_CA_SEQ_LEN_D : C[k];
                        win[k] = wk ? __builtin_amdgcn_alignbit(win[k], win[k], 31) : win[k];
                        const uint32_t c = s_st[k][tid];
                        int icode = (int)(c & 0x1F) + 1, ibit = (c >> 5) & 0x1F,
                            iword = (int)(c >> 10);
                        const bool nbit = icode >= 20;
                        if (nbit) {
                            icode = 0;
                            if (++ibit >= 30) { ibit = 0; iword++; }
                            if (iword > 59) { bad |= (wk && sidx < nsamp) ? 1 : 0; iword = 59; }
                        }
                        const uint32_t c2 = (uint32_t)icode | ((uint32_t)ibit << 5) |
                                            ((uint32_t)iword << 10);
                        if (wk)
                            s_st[k][tid] = (uint16_t)c2;
                        if (__builtin_amdgcn_ballot_w64(wk && nbit)) {
                            const int ng = signed_gain(prow[k].gain * (k < nc ? 1 : 0),
                                                       (s_nav[k][iword] >> (29 - ibit)) & 1u);
                            g[k] = (wk && nbit) ? ng : g[k];
                        }
                    }
                }
            }
            /* LUT[floor(512 carr)] x codeCA (gpssim.c:2200-2209) */
            int32_t e[NCH];
#pragma unroll
            for (int k = 0; k < NCH; k++)
                e[k] = s_lut[ti[k] + (t[k] << 8)];
            int acc_i, acc_q;
            if (__builtin_expect(!big, 1)) {
                /* I and Q of all channels in one int64: acc = (sum I + 64) + 2^22 (sum Q + 64)
                   (gpssim.c:2200-2210, the +64 of 2257) */
                int64_t acc = 64 + ((int64_t)64 << 22);
#pragma unroll
                for (int k = 0; k < NCH; k++)
                    acc += (int64_t)g[k] * (int64_t)e[k];          /* v_mad_i64_i32 */
                const uint32_t alo = (uint32_t)acc;
                acc_i = ((int)(alo << 10)) >> 10;                  /* sext22 */
                acc_q = (int)(acc >> 22) + (int)((alo >> 21) & 1u);
            } else {
                /* large gains: separate (wrapping) int32 sums, as the reference's int math */
                uint32_t ai = 64, aq = 64;
#pragma unroll
                for (int k = 0; k < NCH; k++) {
                    const int cv = (int)((uint32_t)e[k] << 10) >> 10;
                    const int sv = (e[k] - cv) >> 22;
                    ai += (uint32_t)g[k] * (uint32_t)cv;
                    aq += (uint32_t)g[k] * (uint32_t)sv;
                }
                acc_i = (int)ai;
                acc_q = (int)aq;
            }
#pragma unroll
            for (int k = 0; k < NCH; k++) {
                /* carrier (gpssim.c:2245-2250): carr+s is in [0,2) ascending or (-1,1)
                   descending, where v_fract_f64 returns exactly the reference's carr-1 / carr+1
                   (x - floor(x), one IEEE rounding) */
                carr[k] = __builtin_amdgcn_fract(carr[k] + cs[k]);
                C[k] = C[k] + ks[k];                          /* code (gpssim.c:2212) */
            }
            /* gpssim.c:2257-2263: (acc+64)>>7 (arithmetic), then (short).  Written
               unconditionally: samples past this lane's end land in staging bytes that are never
               copied out. */
            int i16 = (int)(int16_t)(acc_i >> 7);
            int q16 = (int)(int16_t)(acc_q >> 7);
            if (FMT == 16) {
                mine[sidx] = (uint32_t)(uint16_t)i16 | ((uint32_t)(uint16_t)q16 << 16);
            } else if (FMT == 8) {                    /* iq_buff >> 4 → signed char */
                ((uint16_t *)mine)[sidx] = (uint16_t)((uint32_t)(uint8_t)(int8_t)(i16 >> 4) |
                                           ((uint32_t)(uint8_t)(int8_t)(q16 >> 4) << 8));
            } else {                                  /* {I0 Q0 I1 Q1 ...} MSB first */
                bits = (bits << 2) | ((uint32_t)(i16 > 0) << 1) | (uint32_t)(q16 > 0);
                if ((sidx & 15) == 15) {
                    /* a tail word keeps its first nb samples and zero padding */
                    int nb = nsamp - (sidx & ~15);
                    uint32_t w32 = nb >= 16 ? bits : nb > 0 ? (bits >> 2 * (16 - nb)) << 2 * (16 - nb) : 0u;
                    mine[sidx >> 4] = __builtin_bswap32(w32);
                    bits = 0;
                }
            }
        }
        const bool any_full = __any(full);
        if (any_full) {
            /* the wave stores whole 128-B chunks of 8 lanes per instruction: lane j stores
               16-B piece j%8 of source lane 8 i + j/8 */
            wave_sync_lds();
            for (int i = 0; i < CHUNK_PIECES; i++) {
                int src = (64 / CHUNK_PIECES) * i + lane / CHUNK_PIECES, piece = lane % CHUNK_PIECES;
                int src_full = __shfl(full ? 1 : 0, src);
                if (src_full) {
                    uint8_t *sdst = dst + (ptrdiff_t)(src - lane) * ((ptrdiff_t)seg_r * BPS4 / 4) +
                                    (size_t)ch * CHUNK_BYTES + piece * 16;
                    const uint32_t *sp = stg + src * (CHUNK_BYTES / 4) + piece * 4;
                    store16(sdst, make_uint4(sp[0], sp[1], sp[2], sp[3]));
                }
            }
            wave_sync_lds();
        }
        if (!full && nsamp > 0) {                     /* ragged tail: this lane's own bytes */
            int nbytes = nsamp * BPS4 / 4;
            uint8_t *bp = dst + (size_t)ch * CHUNK_BYTES;
            const uint8_t *sp = (const uint8_t *)mine;
            for (int i = 0; i < nbytes; i++)
                bp[i] = sp[i];
        }
    }
    if (bad && status)
        atomicOr(status, bad);
}

/* ======================================================================================== */
/* Fast path: certified integer lines (csrc/host/linearize.c; render model common/gss_lin.h)  */
/* ======================================================================================== */
/* For a certified block, sample p of channel k reads the LUT cell and chip that gss_lin.h
   defines from the block's two integer lines (gss_lin_t), with the signed gain of the schedule
   and, at the rare patched samples, a correction to the exact term: no floating point and no
   walk.  Lanes are consecutive samples: one wave step renders 64 consecutive samples, so the LUT
   reads of a wave hit a few neighbouring cells and the output leaves as one contiguous 256-B
   (-b 16) store per step.
   A workgroup of 4 waves renders 4 consecutive 4096-sample segments of one block; a wave
   renders its segment in 4 chunks of LIN_CH = 16 steps of 64 samples.  Per chunk the wave's
   lanes first write every channel's record in parallel (lin_ct in LDS: the chunk base, the step,
   the gain operands, the window-table rows to load next); then, two channels at a time, each
   lane forms its anchors P (code in the low word, carrier in the high word, gss_lin.h) with one
   64-bit add of the chunk base to its entry of the workgroup's lane table (LDS), and per
   64-sample step and channel
       t = W_s >> byte3(P.lo)  chip sign at bit 0, from the step's window        v_lshrrev_b32_sdwa
       a = alignbit(t, P.hi, 21) & M   LUT byte address: cell (carrier bits 23..31) at bits
                                    2..10, chip sign at bit 11 (second half of the LUT negated)
       e = LUT[a]              (cos, sin) as an f16 pair                          ds_read_b32
       P += D                  carrier and code together                          v_lshl_add_u64
   and per two steps and two channels one v_mfma_f32_16x16x32_f16 accumulates gain x (cos, sin)
   into the four I/Q sums of the lane's two samples: 4 VALU + 1 LDS + 1/4 MFMA per
   channel-sample.  The code is a 32-bit word beside the carrier (a carry out of the code word
   adds 2^-32 cycle to the carrier, which the render model counts).
   Chip windows: the window of extended chip E holds the 32 chips from E on, rotated (bit e mod 32
   = sign of chip e mod 1023, 1 = negative), so that any lane whose chip e lies in [E, E + 32)
   takes its sign with a shift by e mod 32 = byte 3 of the code word mod 32.  Step s of a chunk
   whose code base has chip E uses entry [row][E][s] of the chunk window table (gss_tw16_kernel,
   per C/A row one 64-byte row of the 16 steps' windows per start chip, 5.2 MB, rebuilt per call
   because the sample rate sets the window advance); the window then starts at most two chips
   below lane 0's chip and every lane's chip of the step lies inside it when 63 zs + 3 chips <= 31
   (GSS_LIN_WIN_OK, checked by the proof, gss_lin_win16_ok).
   The rows are loaded into SGPRs by an s_load_dwordx16 the compiler does not see, into 16
   registers it never allocates (the kernel is limited to LIN_SW_SGPRS by amdgpu_num_sgpr; the
   buffers s[68:83] and s[84:99] sit above that), issued one pair ahead (while the pair before
   renders; the last pair of a chunk loads the next chunk's first); at the pair's start an
   explicit s_waitcnt and s_mov_b64s hand the windows to ordinary SGPRs, which the chip-sign shift
   takes directly.  Hidden from the compiler, a load in flight leaves the LDS waits counted (a
   pending load only makes one of them wait for one more LDS read), so the LUT reads stay
   pipelined (1.62-1.64 ms per 300 s launch against 1.76 for windows built in LDS, round 4;
   compiler-visible scalar loads share lgkmcnt with the LUT reads and cost +16 %, round 3).
   Accumulation on the matrix cores: channels in pairs on v_mfma_f32_16x16x32_f16.  Lane l holds
   B[8 (l>>4) + j][l & 15] (j = 0..7) and C[4 (l>>4) + r][l & 15] (r = 0..3), so a lane's four
   outputs depend only on its own eight B values when A row 4q + r is zero outside K columns
   8q .. 8q+7 (tools/ubench/mfma16_probe.hip checks the map and the exact sums on gfx950).  B is
   the lane's four LUT words -- channel a at steps s, s+1, channel b at steps s, s+1 -- and A puts
   g_a at column 8q + r and g_b at 8q + 4 + r of row 4q + r: the lanes 20q + r hold those two
   gains (elements r and 4 + r), every other lane zeros.  A lone last channel, and the rare
   gain-change reruns, take one v_mfma_f32_4x4x4_16b_f16 per channel and two steps instead: lane
   4b + i holds row i of block b's A (the gain at slot i) and lane 4b + j column j of B (its own
   two LUT words: K = cos_s, sin_s, cos_s+1, sin_s+1) and of C (I_s, Q_s, I_s+1, Q_s+1)
   (tools/ubench/mfma_probe.hip).
   Exactness: the LUT values (|v| <= 250) and the doubled gains (|2 g| <= 2048, their data-bit
   differences <= 4096 and even; the proof admits |g| <= 1024, sum |g| <= 8000) are exact f16
   integers, products are exact in f32, and the accumulators start at 1.5 2^23 + 128, so that
   each sum holds 2 (sum + 64), an even integer below 2^23 in magnitude: exact in any order, and
   its IEEE bits 0x4B400000 + 2 (sum + 64) put (sum + 64) >> 7 + 2^14 in bits 8..23.  The -b 16
   sample word is then one byte permutation of the I and Q bits and one packed 16-bit add of
   0xC000; -b 8 takes bits 12..; -b 1 compares with 0x4B400000 + 256. */
#define LIN_THREADS 256
#define LIN_WAVES   (LIN_THREADS / 64)
#define LIN_STEPS   (GSS_LIN_SEG / 64)     /* 64-sample steps per wave segment: 4096 samples    */
#define LIN_CH      GSS_LIN_CH             /* steps per chunk (one accumulator each)            */
#define CBW_PRE     2                      /* a window starts at most this far below chip 0      */
#define CBW_CHIPS   3072                   /* window starts per row: E0 <= 1023 plus a segment's
                                              reach (4160 samples * 0.46 chip) plus a window     */
#define CAB_W       ((CBW_CHIPS + 96) / 32)    /* sign words per row: chips -32 .. CBW_CHIPS + 63 */
static_assert(LIN_STEPS % LIN_CH == 0 && (LIN_CH & (LIN_CH - 1)) == 0, "whole chunks");
#define LIN_SW_SGPRS 68                    /* hidden window buffers: s[68:83] and s[84:99]       */
typedef _Float16 lin_half4 __attribute__((ext_vector_type(4)));
typedef _Float16 lin_half8 __attribute__((ext_vector_type(8)));
typedef float lin_f4 __attribute__((ext_vector_type(4)));
#define LIN_GS    2                        /* the gain scale on the matrix cores                 */
#define LIN_MAGF  (12582912.0f + 64.0f * LIN_GS)   /* 1.5 2^23 + 64 LIN_GS                       */
#define LIN_MAGB  0x4B400000u              /* IEEE bits of 1.5 2^23                              */

/* per (block, segment wave, chunk, channel): the chunk's render parameters, built by the wave's
   lanes in parallel (vector loads and VALU) and read back by the render loop with broadcast LDS
   reads, so that the scalar unit (one per CU, shared by its four SIMDs) does no per-channel
   work */
struct alignas(16) lin_ct {
    uint64_t B;                  /* the chunk's base (gss_lin.h)                                */
    uint64_t D;                  /* the 64-sample step dC : dX                                  */
    int32_t g;                   /* (unused)                                                    */
    int32_t gd;                  /* gain change inside the chunk (g1 - g0), from sample pos1 on */
    int32_t pos1;
    uint32_t flags;              /* 1: a gain change inside the chunk, 2: patched samples       */
    uint32_t q0, dq, tab;        /* (dq, tab: the channel's window step and C/A row)            */
    uint32_t wa;                 /* byte offset of the chunk's window-table row                 */
    uint32_t na, nb;             /* the rows to load while the pair (k, k + 1) renders -- the
                                    next pair's, the lone last channel's (twice) or the next
                                    chunk's first pair's (lin_sw_pair); one 8-byte read         */
    uint32_t wn;                 /* the next chunk's row                                        */
    uint32_t g2;                 /* the gain as an f16 pair                                     */
    uint32_t A[5][2];            /* A[i]: the 4x4x4 MFMA's gain operand of lane 4b + i (the gain
                                    at f16 slot i); A[4] zeros.  The pair MFMA's operand half of
                                    each lane is A[its class] (lin_pair_cls)                    */
};
/* the broadcast reads of the record assume these alignments (a misaligned ds_read_b128 is split
   by the hardware and cost the round-4 LDS-window build 3x) */
static_assert(offsetof(lin_ct, A) % 8 == 0, "lin_ct.A: 8-byte reads");

/* per (block, channel): the render constants of gss_lin.h (written by gss_linseg_kernel) */
struct lin_chan {
    uint64_t xs, zs;             /* the lines' per-sample steps                                 */
    uint64_t d;                  /* the 64-sample step dX : dC of P (gss_lin_dx : gss_lin_dz)    */
    uint32_t dq;                 /* window offset advance per step, 1/16 chip, rounded down      */
    uint32_t tab;                /* the channel's C/A table row                                  */
};
/* per (block, channel, wave segment of 64*LIN_STEPS samples): the lines at the segment start,
   so that the render kernel needs no 128-bit arithmetic and no schedule search */
struct lin_seg {
    uint64_t x;                  /* X(n0) + gss_lin_xa(xs): the first chunk's carrier anchor base */
    uint64_t z;                  /* ((E0 << 50) | fraction) + gss_lin_za(zs): the first chunk's
                                    code anchor base, E0 = gss_lin_e0(chip at the segment start) */
    int32_t g01;                 /* signed gain at the start (low 16) and after pos1 (high 16)   */
    int32_t pos1;                /* sample of the first gain change in the segment, or INT32_MAX */
    uint32_t npatch;             /* patched samples of the channel inside the segment            */
    uint32_t pad;
};

__global__ void gss_linseg_kernel(const gss_lin_t *__restrict__ lin,
                                  const gss_chan_blk_t *__restrict__ blk,
                                  const int32_t *__restrict__ nch, const int32_t *__restrict__ fast,
                                  int nblk, int nseg, lin_seg *__restrict__ seg_out,
                                  lin_chan *__restrict__ chan_out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblk * GSS_MAXCH * nseg)
        return;
    const int sg = i % nseg, bk = i / nseg, b = bk / GSS_MAXCH, k = bk % GSS_MAXCH;
    if (!fast[b] || k >= nch[b])
        return;
    const gss_lin_t *L = lin + bk;
    const uint64_t xa = gss_lin_xa(L->xs);
    if (sg == 0) {
        lin_chan c;
        c.xs = L->xs;
        c.zs = L->zs;
        c.d = ((uint64_t)gss_lin_dx(L->xs) << 32) | gss_lin_dz(L->zs);
        c.dq = (uint32_t)((L->zs * 64u) >> 46);
        c.tab = (uint32_t)blk[bk].ca_tbl;
        chan_out[bk] = c;
    }
    const uint64_t n0 = (uint64_t)sg * (64 * LIN_STEPS);
    const uint64_t lo = L->z0 + n0 * L->zs;
    const uint64_t hi = __umul64hi(n0, L->zs) + (lo < L->z0 ? 1u : 0u);
    const uint32_t E0 = gss_lin_e0((hi << 14) | (lo >> 50));
    lin_seg r;
    r.z = (((uint64_t)E0 << 50) | (lo & ((1ull << 50) - 1))) + gss_lin_za(L->zs);
    r.x = L->x0 + n0 * L->xs + xa;
    int q = 0;
    while (q + 1 < GSS_NGC && L->gpos[q + 1] <= (int)n0)
        q++;
    const int g0 = L->gval[q];
    const bool more = q + 1 < GSS_NGC && L->gpos[q + 1] < (int)n0 + 64 * LIN_STEPS;
    const int g1 = more ? L->gval[q + 1] : g0;
    r.g01 = (int32_t)(((uint32_t)g0 & 0xFFFFu) | ((uint32_t)g1 << 16));
    r.pos1 = more ? L->gpos[q + 1] : INT32_MAX;
    int np = 0;
    for (int j = 0; j < GSS_NPATCH; j++)
        np += L->ppos[j] >= (int)n0 && L->ppos[j] < (int)n0 + 64 * LIN_STEPS;
    r.npatch = (uint32_t)np;
    r.pad = 0;
    seg_out[i] = r;
}

/* per C/A row, the chip-sign bit-stream extended cyclically: bit j of the row = sign of extended
   chip j - 32 (chip (j - 32) mod 1023, 1 = codeCA -1) */
__global__ void gss_cab_kernel(const uint32_t *__restrict__ ca_bits, int n_ca,
                               uint32_t *__restrict__ cab)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_ca * CAB_W)
        return;
    const int row = i / CAB_W, j0 = (i - row * CAB_W) * 32 - 32;
    const uint32_t *cb = ca_bits + (size_t)row * GSS_CA_WORDS;
    uint32_t w = 0;
    for (int q = 0; q < 32; q++) {
        const int e = j0 + q, chip = ((e % GSS_CA_LEN) + GSS_CA_LEN) % GSS_CA_LEN;
        w |= (((cb[chip >> 5] >> (chip & 31)) & 1u) ^ 1u) << q;
    }
    cab[i] = w;
}

/* the chunk window table (gss_lin.h): entry [row][E][s] = the 32 chips from extended chip
   e = E + ((s w) >> 4) - GSS_LIN_CBW_PRE on of row's bit-stream, rotated left by e mod 32 (bit
   (c mod 32) = chip c's sign), the word the LDS window pass builds; w = gss_lin_wstep16.  The
   start is clamped to the bit-stream, which a certified channel never reaches. */
__global__ void gss_tw16_kernel(const uint32_t *__restrict__ cab, int n_ca, uint32_t w,
                                uint32_t *__restrict__ tw)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_ca * GSS_LIN_TWE * LIN_CH)
        return;
    const int row = i / (GSS_LIN_TWE * LIN_CH), r = i - row * (GSS_LIN_TWE * LIN_CH);
    const int E = r / LIN_CH, st = r % LIN_CH;
    const uint32_t j = min((uint32_t)(E + (int)(((uint32_t)st * w) >> 4) - GSS_LIN_CBW_PRE + 32),
                           (uint32_t)(32 * CAB_W - 64));       /* bit index: chip j - 32 */
    const uint32_t *c = cab + (size_t)row * CAB_W;
    const uint32_t lin = __builtin_amdgcn_alignbit(c[(j >> 5) + 1], c[j >> 5], j & 31);
    tw[i] = __builtin_amdgcn_alignbit(lin, lin, (32u - j) & 31u);
}

/* a channel's chunk windows: the row of its chunk in the chunk window table (wave-uniform) */
struct lin_wsrc {
    const uint32_t *W;
};

/* all LIN_CH windows of a chunk by compiler-visible scalar loads (the rare gain-change reruns),
   waited for before the steps (the scalar and LDS loads share one counter, so a window load left
   in flight would turn every LUT read's wait into a full drain) */
__device__ __forceinline__ void lin_wissue(const lin_wsrc &w, uint32_t (&ws)[LIN_CH])
{
#pragma unroll
    for (int s = 0; s < LIN_CH; s++)
        ws[s] = w.W[s];                               /* uniform: one s_load_dwordx16 for all 16 */
}

/* ... and the fence that needs them all (one wait, after every load of the chunk is issued) */
__device__ __forceinline__ void lin_wfence(const uint32_t (&ws)[LIN_CH])
{
    static_assert(LIN_CH == 16, "the fence below names 16 windows");
    asm volatile("" :: "s"(ws[0]), "s"(ws[1]), "s"(ws[2]), "s"(ws[3]), "s"(ws[4]), "s"(ws[5]),
                 "s"(ws[6]), "s"(ws[7]), "s"(ws[8]), "s"(ws[9]), "s"(ws[10]), "s"(ws[11]),
                 "s"(ws[12]), "s"(ws[13]), "s"(ws[14]), "s"(ws[15]));
}

__device__ __forceinline__ lin_wsrc lin_wsrc_of(const lin_ct &t, const uint32_t *__restrict__ tw)
{
    const uint32_t off = __builtin_amdgcn_readfirstlane(t.wa);
    return lin_wsrc{(const uint32_t *)__builtin_assume_aligned(
        (const char *)tw + off, 64)};
}

#define LIN_SW_CLOBB "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", \
                     "s95", "s96", "s97", "s98", "s99"
#define LIN_SW_CLOBA "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", \
                     "s79", "s80", "s81", "s82", "s83"
/* channel row off (a byte offset, any lane's copy) into the hidden buffer s[84:99]; with pairs a
   second row into s[68:83] (the clobbers put them in the kernel's SGPR count; the compiler
   allocates none of them).  clang warns that registers above the amdgpu_num_sgpr limit "may not
   be preserved across the asm statement": nothing but these statements names them (the limit
   keeps the allocator, spills and the ABI below s68), which the GPU tests of this build check
   byte for byte, so the warning is silenced here only. */
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lin_sw_load(const uint32_t *__restrict__ tw, uint32_t off)
{
    const uint32_t *p = (const uint32_t *)((const char *)tw +
                                           (uint32_t)__builtin_amdgcn_readfirstlane(off));
    asm volatile("s_load_dwordx16 s[84:99], %0, 0x0" : : "s"(p) : LIN_SW_CLOBB);
}
__device__ __forceinline__ void lin_sw_load2(const uint32_t *__restrict__ tw, uint32_t off_a,
                                             uint32_t off_b)
{
    const uint32_t *pa = (const uint32_t *)((const char *)tw +
                                            (uint32_t)__builtin_amdgcn_readfirstlane(off_a));
    const uint32_t *pb = (const uint32_t *)((const char *)tw +
                                            (uint32_t)__builtin_amdgcn_readfirstlane(off_b));
    asm volatile("s_load_dwordx16 s[68:83], %0, 0x0\n\ts_load_dwordx16 s[84:99], %1, 0x0"
                 : : "s"(pa), "s"(pb) : LIN_SW_CLOBA, LIN_SW_CLOBB);
}
#pragma clang diagnostic pop
/* wait for the loads (and every LDS read) and copy a hidden buffer into 16 SGPRs the compiler
   owns: the steps then schedule like any SGPR operand, and the buffer is free for the next
   load */
#define LIN_SW_TAKE(BUF, W)                                                                       \
    asm volatile("s_waitcnt lgkmcnt(0)\n\t"                                                      \
                 "s_mov_b64 %0, s[" #BUF "+0:" #BUF "+1]\n\ts_mov_b64 %1, s[" #BUF "+2:" #BUF "+3]\n\t" \
                 "s_mov_b64 %2, s[" #BUF "+4:" #BUF "+5]\n\ts_mov_b64 %3, s[" #BUF "+6:" #BUF "+7]\n\t" \
                 "s_mov_b64 %4, s[" #BUF "+8:" #BUF "+9]\n\ts_mov_b64 %5, s[" #BUF "+10:" #BUF "+11]\n\t" \
                 "s_mov_b64 %6, s[" #BUF "+12:" #BUF "+13]\n\ts_mov_b64 %7, s[" #BUF "+14:" #BUF "+15]" \
                 : "=s"(W[0]), "=s"(W[1]), "=s"(W[2]), "=s"(W[3]), "=s"(W[4]), "=s"(W[5]),      \
                   "=s"(W[6]), "=s"(W[7]))
__device__ __forceinline__ void lin_sw_split(const uint64_t (&w)[8], uint32_t (&ws)[LIN_CH])
{
    static_assert(LIN_CH == 16, "16 windows");
#pragma unroll
    for (int i = 0; i < 8; i++) {
        ws[2 * i] = (uint32_t)w[i];
        ws[2 * i + 1] = (uint32_t)(w[i] >> 32);
    }
}
__device__ __forceinline__ void lin_sw_take(uint32_t (&ws)[LIN_CH])          /* s[84:99] */
{
    uint64_t w[8];
    LIN_SW_TAKE(84, w);
    lin_sw_split(w, ws);
}
__device__ __forceinline__ void lin_sw_take_a(uint32_t (&ws)[LIN_CH])        /* s[68:83] */
{
    uint64_t w[8];
    LIN_SW_TAKE(68, w);
    lin_sw_split(w, ws);
}

/* one channel's LIN_CH steps on one v_mfma_f32_4x4x4_16b_f16 per two steps: the lane's anchor P
   (carrier : code, high : low word, gss_lin.h), its 64-sample step D, the steps' windows W, the
   LUT mask M and the gain operand A (lin_gain_operand); with LANE_GAIN (a gain-change rerun) the
   LUT words of samples before pos1 are zeroed and A carries the gain difference */
template <bool LANE_GAIN, bool FIRST = false>
__device__ __forceinline__ void lin_channel_chunk_m(lin_f4 (&cq)[LIN_CH / 2], lin_f4 c0, uint64_t P,
                                                    uint64_t D, lin_wsrc W, uint32_t M,
                                                    lin_half4 A, int pos1, int p0,
                                                    const int32_t *__restrict__ s_lut)
{
    uint32_t e0 = 0;
    uint32_t sw[LIN_CH];
    lin_wissue(W, sw);
    lin_wfence(sw);
#pragma unroll
    for (int s = 0; s < LIN_CH; s++) {
        const uint32_t ws = sw[s];
        uint32_t t;
        asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 "
            "src1_sel:DWORD" : "=v"(t) : "v"((uint32_t)P), "s"(ws));                  /* bit 0: sign */
        const uint32_t a = __builtin_amdgcn_alignbit(t, (uint32_t)(P >> 32), 21) & M;
        uint32_t e = *(const uint32_t *)((const char *)s_lut + a);
        if (LANE_GAIN)
            e = p0 + s * 64 >= pos1 ? e : 0u;
        if (s & 1) {
            const uint2 bb = make_uint2(e0, e);
            cq[s / 2] = __builtin_amdgcn_mfma_f32_4x4x4f16(A, __builtin_bit_cast(lin_half4, bb),
                                                          FIRST ? c0 : cq[s / 2], 0, 0, 0);
        } else {
            e0 = e;
        }
        P += D;
    }
}

/* the lone last channel k of a chunk: its 16 steps from windows ws (SGPRs), one 4x4x4 MFMA per
   two steps */
__device__ __forceinline__ void lin_sw_steps(lin_f4 (&cq)[LIN_CH / 2], const lin_ct &t, int k,
                                             int lane, const uint64_t *s_lane, uint32_t M,
                                             const int32_t *__restrict__ s_lut,
                                             const uint32_t (&ws)[LIN_CH])
{
    uint64_t P = s_lane[k * 64 + lane] + t.B;
    const uint64_t D = t.D;
    const lin_half4 A = __builtin_bit_cast(lin_half4, *(const uint2 *)t.A[lane & 3]);
    uint32_t e0 = 0;
#pragma unroll
    for (int s = 0; s < LIN_CH; s++) {
        uint32_t tt;
        asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 "
            "src1_sel:DWORD" : "=v"(tt) : "v"((uint32_t)P), "s"(ws[s]));      /* bit 0: sign */
        const uint32_t a = __builtin_amdgcn_alignbit(tt, (uint32_t)(P >> 32), 21) & M;
        const uint32_t e = *(const uint32_t *)((const char *)s_lut + a);
        if (s & 1) {
            const uint2 bb = make_uint2(e0, e);
            cq[s / 2] = __builtin_amdgcn_mfma_f32_4x4x4f16(A, __builtin_bit_cast(lin_half4, bb),
                                                          cq[s / 2], 0, 0, 0);
        } else {
            e0 = e;
        }
        P += D;
    }
}

/* the lane's row of lin_ct.A for the pair MFMA's gain operand: r = lane mod 4 on lanes 20q + r
   (q, r = 0..3), which hold g_a at element r and g_b at 4 + r; 4 (zeros) elsewhere */
__device__ __forceinline__ uint32_t lin_pair_cls(int lane)
{
    const int q = lane >> 4, r = lane & 3;
    return ((lane & 15) >> 2) == q ? (uint32_t)r : 4u;
}

/* channels k0, k0 + 1 from the hidden buffers s[68:83], s[84:99] (loaded while the pair before
   rendered); the next pair's rows (or the lone last channel's) load meanwhile.  FIRST: the
   chunk's first pair, whose MFMAs take the bias c0 as C (no initialisation moves) */
template <bool FIRST>
__device__ __forceinline__ void lin_sw_pair(lin_f4 (&cq)[LIN_CH / 2], lin_f4 c0, const lin_ct *T, int k0,
                                            int nc, int lane, const uint64_t *s_lane, uint32_t M,
                                            const int32_t *__restrict__ s_lut,
                                            const uint32_t *__restrict__ tw, uint32_t cls,
                                            bool more)
{
    const lin_ct &ta = T[k0], &tb = T[k0 + 1];
    uint64_t Pa = s_lane[k0 * 64 + lane] + ta.B, Pb = s_lane[(k0 + 1) * 64 + lane] + tb.B;
    const uint64_t Da = ta.D, Db = tb.D;
    const uint2 ga = *(const uint2 *)ta.A[cls], gb = *(const uint2 *)tb.A[cls];
    const lin_half8 A = __builtin_bit_cast(lin_half8, make_uint4(ga.x, ga.y, gb.x, gb.y));
    /* the rows to load while this pair renders (the record's na, nb): the next pair's (or the
       lone last channel's), or after the last pair the next chunk's first pair (more: there is a
       next chunk) */
    uint32_t na = ta.na, nb = ta.nb;
    asm volatile("" : "+v"(na), "+v"(nb));       /* read with the record, before the wait below */
    uint32_t wsa[LIN_CH], wsb[LIN_CH];
    lin_sw_take_a(wsa);
    lin_sw_take(wsb);
    if (k0 + 2 < nc || more)
        lin_sw_load2(tw, na, nb);
    uint32_t ea0 = 0, eb0 = 0;
#pragma unroll
    for (int s = 0; s < LIN_CH; s++) {
        uint32_t ta_, tb_;
        asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 "
            "src1_sel:DWORD" : "=v"(ta_) : "v"((uint32_t)Pa), "s"(wsa[s]));
        asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 "
            "src1_sel:DWORD" : "=v"(tb_) : "v"((uint32_t)Pb), "s"(wsb[s]));
        const uint32_t aa = __builtin_amdgcn_alignbit(ta_, (uint32_t)(Pa >> 32), 21) & M;
        const uint32_t ab = __builtin_amdgcn_alignbit(tb_, (uint32_t)(Pb >> 32), 21) & M;
        const uint32_t ea = *(const uint32_t *)((const char *)s_lut + aa);
        const uint32_t eb = *(const uint32_t *)((const char *)s_lut + ab);
        if (s & 1) {
            const uint4 bb = make_uint4(ea0, ea, eb0, eb);
            cq[s / 2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, __builtin_bit_cast(lin_half8, bb),
                                                              FIRST ? c0 : cq[s / 2], 0, 0, 0);
        } else {
            ea0 = ea;
            eb0 = eb;
        }
        Pa += Da;
        Pb += Db;
    }
}

/* the MFMA gain operand of this lane (g at slot lane mod 4, f16 bits gh) */
__device__ __forceinline__ lin_half4 lin_gain_operand(uint32_t gh, int lane)
{
    const uint32_t x = gh << ((lane & 1) * 16);
    const uint2 v = (lane & 2) ? make_uint2(0u, x) : make_uint2(x, 0u);
    return __builtin_bit_cast(lin_half4, v);
}

__device__ __forceinline__ uint32_t lin_f16_bits(int g)
{
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(float)g);
}

/* output stores: the stream is written once and never read back by this kernel, while each
   XCD's L2 must keep the chip-window table warm: non-temporal */
__device__ __forceinline__ void lin_put(uint32_t *p, uint32_t v)
{
    __builtin_nontemporal_store(v, p);
}

/* v_writelane_b32: a wave-uniform value into one lane (no clang builtin in this toolchain) */
extern "C" __device__ int gss_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");

/* Per step s of a chunk, from the accumulators: the -b 16 sample word (I16 | Q16 << 16), the
   -b 8 halfword (I8 | Q8 << 8) and the -b 1 signs (I16 > 0, Q16 > 0), gpssim.c:2257-2287.  The
   IEEE bits of 1.5 2^23 + 2 (sum + 64) are 0x4B400000 + 2 (sum + 64), so (sum + 64) >> n is the
   word shifted by n + 1, offset by 0x4B400000 >> (n + 1). */
__device__ __forceinline__ uint32_t lin_ib(const lin_f4 (&cq)[LIN_CH / 2], int s)
{
    return __float_as_uint(cq[s / 2][2 * (s & 1)]);
}
__device__ __forceinline__ uint32_t lin_qb(const lin_f4 (&cq)[LIN_CH / 2], int s)
{
    return __float_as_uint(cq[s / 2][2 * (s & 1) + 1]);
}
__device__ __forceinline__ uint32_t lin_w16(const lin_f4 (&cq)[LIN_CH / 2], int s)
{
    /* bytes 1, 2 of the I bits (low half) and of the Q bits (high half): 2^14 + (sum + 64) >> 7
       each, then + 0xC000 per half = (sum + 64) >> 7 mod 2^16 */
    const uint32_t pq = __builtin_amdgcn_perm(lin_qb(cq, s), lin_ib(cq, s), 0x06050201u);
    uint32_t r;
    asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(pq), "s"(0xC000C000u));
    return r;
}
__device__ __forceinline__ uint32_t lin_w8(const lin_f4 (&cq)[LIN_CH / 2], int s)
{
    /* the Q byte is shifted straight into place by an SDWA shift that preserves the rest of the
       destination: two shifts, no perm */
    constexpr uint32_t sh = 12u;
    uint32_t d = lin_ib(cq, s) >> sh;                 /* bytes 2, 3: not stored */
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "
        "src1_sel:DWORD" : "+v"(d) : "v"(sh), "v"(lin_qb(cq, s)));
    return d;
}
__device__ __forceinline__ bool lin_ipos(const lin_f4 (&cq)[LIN_CH / 2], int s)
{
    return lin_ib(cq, s) >= LIN_MAGB + 128u * LIN_GS;
}
__device__ __forceinline__ bool lin_qpos(const lin_f4 (&cq)[LIN_CH / 2], int s)
{
    return lin_qb(cq, s) >= LIN_MAGB + 128u * LIN_GS;
}

template <int FMT, bool TAIL>
__device__ __forceinline__ void lin_store(const lin_f4 (&acc)[LIN_CH / 2], uint8_t *__restrict__ ob,
                                          int nb0, int lane, int n_per_blk)
{
    /* the -b 1 epilogue hands lane 4 s + j the 16 samples 64 s + 16 j .. + 15: 4 LIN_CH lanes */
    static_assert(FMT != 1 || LIN_CH == 16, "-b 1 packing assumes 16-step chunks");
    uint32_t pk[LIN_CH];
    pk[0] = 0;
#pragma unroll
    for (int s = 0; s < LIN_CH; s++) {
        const int nb = nb0 + s * 64, p = nb + lane;
        const bool in = !TAIL || p < n_per_blk;
        if (FMT == 16) {
            /* packed first, stored after the loop: distinct data registers, so a store never
               holds up the next pack (a VMEM store reads its data VGPR after issue) */
            pk[s] = lin_w16(acc, s);
        } else if (FMT == 8) {                            /* iq_buff >> 4 → signed char */
            const uint32_t v = lin_w8(acc, s);
            if (!TAIL)                            /* SGPR base, 32-bit lane offset, as -b 16 */
                asm volatile("global_store_short %0, %1, %2 offset:%3"
                             : : "v"((uint32_t)lane * 2u), "v"(v),
                               "s"((uint16_t *)ob + nb0 + (s >> 4) * 2048), "i"((s & 15) * 128)
                             : "memory");
            else if (in)
                ((uint16_t *)ob)[p] = (uint16_t)v;
        } else {                                          /* {I0 Q0 I1 Q1 ...} MSB first */
            /* I16 > 0 <=> sum I + 64 >= 128 <=> the I word >= 0x4B400000 + 256, the same for
               Q (gpssim.c:2266-2276: bit = iq_buff[] > 0) */
            const uint64_t mi = __builtin_amdgcn_ballot_w64(lin_ipos(acc, s));
            const uint64_t mq = __builtin_amdgcn_ballot_w64(lin_qpos(acc, s));
            /* lane 4s + j collects the I (low half) and Q (high half) sign bits of samples
               64 s + 16 j .. + 15: scalar packs, one lane write each */
            const uint32_t ilo = (uint32_t)mi, ihi = (uint32_t)(mi >> 32);
            const uint32_t qlo = (uint32_t)mq, qhi = (uint32_t)(mq >> 32);
            pk[0] = (uint32_t)gss_writelane((int)((ilo & 0xFFFFu) | (qlo << 16)), 4 * s, (int)pk[0]);
            pk[0] = (uint32_t)gss_writelane((int)((ilo >> 16) | (qlo & 0xFFFF0000u)), 4 * s + 1, (int)pk[0]);
            pk[0] = (uint32_t)gss_writelane((int)((ihi & 0xFFFFu) | (qhi << 16)), 4 * s + 2, (int)pk[0]);
            pk[0] = (uint32_t)gss_writelane((int)((ihi >> 16) | (qhi & 0xFFFF0000u)), 4 * s + 3, (int)pk[0]);
            (void)in;
        }
    }
    if (FMT == 1) {
        /* each lane now holds 16 samples' I bits (low) and Q bits (high): interleave them into the
           reference's bytes (sample 4b + m: I at bit 7 - 2m, Q at bit 6 - 2m) and store the
           chunk's 256 bytes with one dword per lane */
        uint32_t vi = pk[0] & 0xFFFFu, vq = pk[0] >> 16;
        vi = (vi | (vi << 8)) & 0x00FF00FFu; vq = (vq | (vq << 8)) & 0x00FF00FFu;
        vi = (vi | (vi << 4)) & 0x0F0F0F0Fu; vq = (vq | (vq << 4)) & 0x0F0F0F0Fu;
        vi = (vi | (vi << 2)) & 0x33333333u; vq = (vq | (vq << 2)) & 0x33333333u;
        vi = (vi | (vi << 1)) & 0x55555555u; vq = (vq | (vq << 1)) & 0x55555555u;
        const uint32_t x = (vi << 1) | vq;                  /* bit 2k + 1 = I_k, bit 2k = Q_k */
        const uint32_t y = ((x & 0x03030303u) << 6) | ((x & 0x0C0C0C0Cu) << 2) |
                           ((x >> 2) & 0x0C0C0C0Cu) | ((x >> 6) & 0x03030303u);
        uint8_t *dst = ob + nb0 / 4 + 4 * lane;
        const int first = nb0 + 16 * lane;                  /* this lane's first sample */
        const bool whole = !TAIL || first + 16 <= n_per_blk;
        if (whole && ((uintptr_t)(ob + nb0 / 4) & 3u) == 0) {
            lin_put((uint32_t *)dst, y);
        } else {
            for (int b = 0; b < 4; b++)                     /* ragged tail or unaligned block */
                if (first + 4 * b < n_per_blk)
                    dst[b] = (uint8_t)(y >> (8 * b));
        }
    }
    if (FMT == 16) {
        __builtin_amdgcn_sched_barrier(0);
        if (!TAIL) {
            /* uniform base in SGPRs, 32-bit lane offset: no 64-bit address VGPRs per store */
            uint32_t *base = (uint32_t *)ob + nb0;
            const uint32_t off = (uint32_t)lane * 4u;
#pragma unroll
            for (int s = 0; s < LIN_CH; s++)
                asm volatile("global_store_dword %0, %1, %2 offset:%3 nt"  /* 13-bit offset */
                             : : "v"(off), "v"(pk[s]), "s"(base + (s >> 4) * 1024),
                               "i"((s & 15) * 256) : "memory");
        } else {
#pragma unroll
            for (int s = 0; s < LIN_CH; s++) {
                const int p = nb0 + s * 64 + lane;
                if (!TAIL || p < n_per_blk)
                    lin_put(((uint32_t *)ob) + p, pk[s]);
            }
        }
    }
}

/* The chunk holds samples where the render arithmetic does not give the exact term (gss_lin_t
   ppos/pdelta, rare): add the correction to that lane and step, the packed delta dI + 2^22 dQ
   split into its two exact integers and added in f32 (exact: integers below 2^24) */
__device__ __forceinline__ void lin_patch_fix(lin_f4 (&cq)[LIN_CH / 2],
                                              const gss_lin_t *__restrict__ Lk, int nb0, int lane)
{
    for (int j = 0; j < GSS_NPATCH; j++) {
        const int pp = Lk->ppos[j];                   /* ascending, unused = INT32_MAX */
        if (pp >= nb0 + 64 * LIN_CH)
            break;
        if (pp < nb0)
            continue;
        const int q = pp - nb0;
        const int64_t d = lane == (q & 63) ? Lk->pdelta[j] : 0;
        const int di = (int)((uint32_t)d << 10) >> 10;
        const float fi = (float)(di * LIN_GS), fq = (float)((int)((d - di) >> 22) * LIN_GS);
        /* every accumulator takes fi (fq) times a wave-uniform 0 or 1: in-place multiply-adds
           (exact), no branches and no selects that would keep two copies of the set live */
        const int sq = __builtin_amdgcn_readfirstlane(q >> 6);
#pragma unroll
        for (int s = 0; s < LIN_CH; s++) {
            const float m = s == sq ? 1.0f : 0.0f;
            cq[s / 2][2 * (s & 1)] = __builtin_fmaf(m, fi, cq[s / 2][2 * (s & 1)]);
            cq[s / 2][2 * (s & 1) + 1] = __builtin_fmaf(m, fq, cq[s / 2][2 * (s & 1) + 1]);
        }
    }
}


/* workgroups per CU the register budget aims at: the window loads pipeline deeper at 5-6 waves
   per SIMD (8 would spill; 3, 4 and 5 measured the same, round 4) */
#define LIN_MINB 4
template <int FMT>
__global__ __launch_bounds__(LIN_THREADS, LIN_MINB) __attribute__((amdgpu_num_sgpr(LIN_SW_SGPRS)))
void gss_lin_kernel(
    const gss_lin_t *__restrict__ lin, const lin_seg *__restrict__ segs,
    const lin_chan *__restrict__ chans, const int32_t *__restrict__ nch,
    const int32_t *__restrict__ fast, const uint32_t *__restrict__ cab,
    const uint32_t *__restrict__ tw, lut_arg lut, int n_per_blk, int nseg, int wg_per_blk,
    uint8_t *__restrict__ out, size_t block_bytes)
{
    __shared__ int32_t s_lut[1024];                       /* (cos, sin) f16; [512+i] = -[i] */
    __shared__ uint64_t s_lane[GSS_MAXCH * 64];           /* lane offsets L(l) per channel    */
    __shared__ lin_ct s_ct[LIN_WAVES][GSS_MAXCH];         /* the current chunk, per wave      */
    const int b = blockIdx.x / wg_per_blk;
    const int w = blockIdx.x - b * wg_per_blk;
    if (!fast[b])
        return;                                           /* the exact path renders it */
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);    /* wave-uniform: scalar */
    for (int i = tid; i < 512; i += LIN_THREADS) {
        const uint32_t v = lin_f16_bits(lut.cos512[i]) | (lin_f16_bits(lut.sin512[i]) << 16);
        s_lut[i] = (int32_t)v;
        s_lut[512 + i] = (int32_t)(v ^ 0x80008000u);
    }
    const lin_chan *CH = chans + (size_t)b * GSS_MAXCH;
    const int nc = nch[b];
    for (int i = tid; i < nc * 64; i += LIN_THREADS)
        s_lane[i] = gss_lin_lane(CH[i >> 6].xs, CH[i >> 6].zs, (uint32_t)(i & 63));
    (void)cab;
    __syncthreads();
    uint32_t M = 0xFFCu;                                  /* LUT address mask, in a VGPR */
    asm volatile("" : "+v"(M));
    const uint32_t cls = lin_pair_cls(lane);              /* the pair MFMA's gain operand row */
    lin_f4 c0 = lin_f4{LIN_MAGF, LIN_MAGF, LIN_MAGF, LIN_MAGF};   /* the accumulators' bias */
    asm volatile("" : "+v"(c0));
    const int sg = w * LIN_WAVES + wave;
    const int n0 = sg * (64 * LIN_STEPS);
    if (n0 >= n_per_blk)
        return;
    const gss_lin_t *L = lin + (size_t)b * GSS_MAXCH;
    const lin_seg *S = segs + (size_t)b * GSS_MAXCH * nseg + sg;
    lin_ct *T = s_ct[wave];
    uint8_t *ob = out + (size_t)b * block_bytes;
    bool sw_ahead = false;                 /* the chunk's first pair is already loading */
    /* ---- lane k: channel k's rows, the same for every chunk of the wave: loaded once, the
       record's constant fields written once, the lines advanced by one chunk per chunk ---- */
    uint64_t xb = 0, zb = 0, xs10 = 0, zs10 = 0;       /* chunk bases, per-chunk advances     */
    int32_t pos1 = INT32_MAX;
    uint32_t pflag = 0, gh0 = 0, gh1 = 0;
    uint32_t trow = 0, wa_next = 0;                    /* table row base, this chunk's row     */
    int g_after = -1;                                  /* the gain the record holds (none yet) */
    if (lane < nc) {
        const lin_chan ck = CH[lane];
        const lin_seg sk = S[(size_t)lane * nseg];
        xb = sk.x;
        zb = sk.z;
        xs10 = ck.xs << 10;
        zs10 = ck.zs << 10;
        static_assert(64 * LIN_CH == 1024, "one chunk = 2^10 samples");
        pos1 = sk.pos1;
        pflag = sk.npatch != 0 ? 2u : 0u;
        const int g0 = (int)(int16_t)(sk.g01 & 0xFFFF), g1 = sk.g01 >> 16;
        gh0 = lin_f16_bits(g0 * LIN_GS);
        gh1 = lin_f16_bits(g1 * LIN_GS);
        lin_ct &t = T[lane];
        t.D = ck.d;
        t.gd = g1 - g0;
        t.pos1 = sk.pos1;
        t.dq = ck.dq;
        t.tab = ck.tab;
        t.A[4][0] = 0;
        t.A[4][1] = 0;
        /* a chunk's row of the window table: its C/A row and code base chip E (clamped to the
           table; gss_lin_win16_ok keeps a certified channel inside it) */
        trow = ck.tab * GSS_LIN_TWE;
        wa_next = (trow + min((uint32_t)(zb >> 50), (uint32_t)(GSS_LIN_TWE - 1))) *
                  (uint32_t)(LIN_CH * sizeof(uint32_t));
    }

    const int nc_blk = nc;
    for (int c = 0; c < LIN_STEPS / LIN_CH; c++) {
        /* the channel count made opaque per chunk: its conditions (nc > 1, lane + 2 < nc, ...)
           are recomputed by the scalar unit and one compare each, instead of being hoisted out
           of the loop, spilled to VGPR lanes and read back with 12 v_readlane per chunk */
        int nc = nc_blk;
        asm volatile("" : "+s"(nc));
        const int nb0 = n0 + c * (64 * LIN_CH);           /* first sample of the chunk */
        if (nb0 >= n_per_blk)
            break;
        /* ---- the chunk's parameters, lane k for channel k: computed on every lane (the
           lanes past nc hold zero rows and flags, their values unused), stored by the first nc
           (no phi moves for the lanes outside) ---- */
        const bool after = pos1 <= nb0;                    /* the data bit changed before it */
        const bool chg = pos1 < nb0 + 64 * LIN_CH;         /* ... or changes inside it      */
        const uint32_t my_flags = (chg && !after ? 1u : 0u) | pflag;
        const uint64_t zn = zb + zs10;                     /* the next chunk's code base */
        const uint32_t my_wa = wa_next;
        const uint32_t my_wn = (trow + min((uint32_t)(zn >> 50), (uint32_t)(GSS_LIN_TWE - 1))) *
                               (uint32_t)(LIN_CH * sizeof(uint32_t));
        if (lane < nc) {
            lin_ct &t = T[lane];
            /* the chunk's base B (gss_lin.h): the segment's lines plus c chunks */
            t.B = (xb & ~0xFFFFFFFFull) | (uint32_t)(zb >> GSS_LIN_CSH);
            t.flags = my_flags;
            t.wa = my_wa;
            t.wn = my_wn;
            if ((int)after != g_after) {                   /* the gain the chunk starts with */
                g_after = (int)after;
                const uint32_t gh = after ? gh1 : gh0;
                t.A[0][0] = gh;         t.A[0][1] = 0;     /* lane 4b + i's gain operand */
                t.A[1][0] = gh << 16;   t.A[1][1] = 0;
                t.A[2][0] = 0;          t.A[2][1] = gh;
                t.A[3][0] = 0;          t.A[3][1] = gh << 16;
                t.g2 = gh | (gh << 16);
            }
        }
        wa_next = my_wn;
        xb += xs10;
        zb = zn;
        /* the channels with a gain change or patches in this chunk (wave-uniform) */
        /* the first two channels' rows of this chunk and the next (scalar: readlane) */
        const uint32_t wa0 = (uint32_t)__builtin_amdgcn_readlane((int)my_wa, 0);
        const uint32_t wa1r = (uint32_t)__builtin_amdgcn_readlane((int)my_wa, 1);
        const uint32_t wn0 = (uint32_t)__builtin_amdgcn_readlane((int)my_wn, 0);
        const uint32_t wn1r = (uint32_t)__builtin_amdgcn_readlane((int)my_wn, 1);
        const uint32_t wa1 = nc > 1 ? wa1r : wa0, wn1 = nc > 1 ? wn1r : wn0;
        {
            /* the rows each pair (k, k + 1) loads ahead (gather from lanes k + 2, k + 3, 0, 1:
               once per chunk in parallel, instead of selects per pair); the channels are lanes
               0..15, one DPP row: lane k takes lane k + 2's / k + 3's by a row shift (row_shl),
               the first pair's by readlane -- no LDS permutes */
            const uint32_t wa2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)my_wa, 0x102, 0xF,
                                                                       0xF, true);
            const uint32_t wa3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)my_wa, 0x103, 0xF,
                                                                       0xF, true);
            if (lane < nc) {
                const bool in2 = lane + 2 < nc, in3 = lane + 3 < nc;
                T[lane].na = in2 ? wa2 : wn0;
                T[lane].nb = in3 ? wa3 : in2 ? wa2 : wn1;
            }
        }
        const uint64_t fmask = __builtin_amdgcn_ballot_w64(my_flags != 0);
        wave_sync_lds();
        lin_f4 acc[LIN_CH / 2];
        /* the first pair's rows: loaded during the chunk before, or now */
        if (nc > 0 && !sw_ahead)
            lin_sw_load2(tw, wa0, wa1);
        const bool more = c + 1 < LIN_STEPS / LIN_CH && nb0 + 64 * LIN_CH < n_per_blk;
        int k0 = 0;
        if (nc >= 2) {                                    /* the first pair sets acc = bias + ... */
            lin_sw_pair<true>(acc, c0, T, 0, nc, lane, s_lane, M, s_lut, tw, cls, more);
            k0 = 2;
        } else {
            /* (the copies pinned inside this branch: hoisted, they cost 32 moves every chunk) */
#pragma unroll
            for (int s = 0; s < LIN_CH / 2; s++) {
                lin_f4 v = c0;
                asm volatile("" : "+v"(v));
                acc[s] = v;
            }
        }
        /* unrolled: each pair's record and lane-table addresses are immediate offsets */
#pragma unroll
        for (int p = 1; p < GSS_MAXCH / 2; p++) {
            if (2 * p + 1 >= nc)
                break;
            lin_sw_pair<false>(acc, c0, T, 2 * p, nc, lane, s_lane, M, s_lut, tw, cls, more);
            k0 = 2 * p + 2;
        }
        if (k0 < nc) {                                    /* the lone last channel: s[68:83] */
            uint32_t ws[LIN_CH], wb[LIN_CH];
            lin_sw_take_a(ws);
            lin_sw_take(wb);                              /* (its duplicate, unused) */
            (void)wb;
            if (more)                                     /* the next chunk's first pair */
                lin_sw_load2(tw, wn0, wn1);
            lin_sw_steps(acc, T[k0], k0, lane, s_lane, M, s_lut, ws);
            k0 = nc;
        }
        sw_ahead = nc > 0 && more;
        for (int k = k0; k < nc; k++) {                   /* (none left: k0 == nc) */
            const lin_ct &t = T[k];
            const uint64_t B = t.B, D = t.D;
            const uint2 a2 = *(const uint2 *)t.A[lane & 3];
            lin_channel_chunk_m<false>(acc, c0, s_lane[k * 64 + lane] + B, D, lin_wsrc_of(t, tw), M,
                                       __builtin_bit_cast(lin_half4, a2), 0, 0, s_lut);
        }
        /* gain changes and patches (rare): only the channels whose flags are set */
        for (uint64_t fm = fmask; fm; fm &= fm - 1) {
            const int k = __builtin_amdgcn_readfirstlane((int)__builtin_ctzll(fm));
            const lin_ct &t = T[k];
            const uint64_t B = t.B, D = t.D;
            const uint32_t fl = __builtin_amdgcn_readfirstlane(t.flags);
            if (__builtin_expect(fl & 1u, 0)) {
                uint32_t l2 = (uint32_t)lane;
                asm volatile("" : "+v"(l2));
                lin_channel_chunk_m<true>(acc, c0, s_lane[k * 64 + l2] + B, D, lin_wsrc_of(t, tw), M,
                                          lin_gain_operand(lin_f16_bits(t.gd * LIN_GS), (int)l2), t.pos1,
                                          nb0 + (int)l2, s_lut);
            }
            if (__builtin_expect(fl & 2u, 0))
                lin_patch_fix(acc, L + k, nb0, lane);
        }
        wave_sync_lds();                                  /* T is rewritten by the next chunk */
        if (nb0 + 64 * LIN_CH <= n_per_blk)
            lin_store<FMT, false>(acc, ob, nb0, lane, n_per_blk);
        else
            lin_store<FMT, true>(acc, ob, nb0, lane, n_per_blk);
    }
}


/* ======================================================================================== */
/* C ABI                                                                                    */
/* ======================================================================================== */
struct gss_dev {
    int ordinal;
    int seg_r = 1024;                    /* samples per Stage-B lane (env GSS_SEG_R)   */
    struct anchor_set {                  /* segment-start states [blocks][16][nsegp]     */
        double *carr = nullptr, *code = nullptr;
        uint32_t *cnt = nullptr;
        size_t cap = 0;
    } set[2];                            /* two sets: Stage A of batch k+1 beside B of k  */
    static constexpr int RING = 256;
    hipEvent_t ev_a[RING][2], ev_b[RING][2];   /* start/end of each stage launch          */
    hipEvent_t ev_l[RING][2];                  /* ... and of each fast-path launch         */
    int n_a = 0, n_b = 0, n_l = 0;
    lut_arg lut;
    void *h_in = nullptr; size_t h_in_cap = 0;
    void *d_out = nullptr; size_t d_out_cap = 0;
    double *d_cend = nullptr; size_t d_cend_cap = 0;
    uint32_t *d_cbw = nullptr; size_t d_cbw_cap = 0;   /* chip-sign bit-streams (gss_cab_kernel) */
    void *d_seg = nullptr; size_t d_seg_cap = 0;       /* lin_seg rows (gss_linseg_kernel)   */
    int32_t *d_status = nullptr;
    /* the exact path's leftovers of a fast-path call run on their own stream beside the fast
       kernel (a few latency-bound blocks would otherwise serialise after it) */
    hipStream_t aux = nullptr;
    hipEvent_t ev_in = nullptr, ev_fb = nullptr;
};

extern "C" int gss_fail(int code, const char *fmt, ...);

#define HIP_TRY(x)                                                                           \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess)                                                                \
            return gss_fail(GSS_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_),      \
                            __FILE__, __LINE__);                                             \
    } while (0)

#define GSS_STR2(x) #x
#define GSS_STR(x) GSS_STR2(x)
/* the device ordinal of an open handle (gss_producers.hip, gss_run.hip) */
extern "C" int gss_dev_ordinal(const gss_dev *d) { return d->ordinal; }

extern "C" const char *gss_build_info(void)
{
    return "lin_mfma=2 lin_ch=" GSS_STR(LIN_CH) " lin_swin=3 spec_k=" GSS_STR(GSS_SPEC_K)
           " arch=gfx950";
}


extern "C" void gss_run_pool_prewarm(int dev);    /* gss_run.hip */

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
    const char *r = getenv("GSS_SEG_R");
    if (r && atoi(r) >= 256 && atoi(r) % 256 == 0)
        d->seg_r = atoi(r);
    for (int i = 0; i < gss_dev::RING; i++)
        for (int j = 0; j < 2; j++) {
            HIP_TRY(hipEventCreate(&d->ev_a[i][j]));
            HIP_TRY(hipEventCreate(&d->ev_b[i][j]));
            HIP_TRY(hipEventCreate(&d->ev_l[i][j]));
        }
    int32_t s[512], c[512];
    gss_lut(s, c);
    for (int i = 0; i < 512; i++) {
        d->lut.sin512[i] = (int16_t)s[i];
        d->lut.cos512[i] = (int16_t)c[i];
    }
    HIP_TRY(hipMalloc(&d->d_status, sizeof(int32_t)));
    int prio_lo = 0, prio_hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIP_TRY(hipStreamCreateWithPriority(&d->aux, hipStreamNonBlocking, prio_hi));
    HIP_TRY(hipEventCreateWithFlags(&d->ev_in, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d->ev_fb, hipEventDisableTiming));
    gss_run_pool_prewarm(ordinal);                   /* gss_run's streams, made once here */
    *out = d;
    return 0;
}

extern "C" void gss_run_pool_drain(int dev);      /* gss_run.hip */

extern "C" int gss_dev_close(gss_dev *d)
{
    if (!d) return 0;
    (void)hipSetDevice(d->ordinal);
    gss_run_pool_drain(d->ordinal);                  /* gss_run's pooled slot buffers */
    for (auto &a : d->set) {
        (void)hipFree(a.carr);
        (void)hipFree(a.code);
        (void)hipFree(a.cnt);
    }
    if (d->aux) (void)hipStreamDestroy(d->aux);
    if (d->ev_in) (void)hipEventDestroy(d->ev_in);
    if (d->ev_fb) (void)hipEventDestroy(d->ev_fb);
    void *bufs[] = {d->h_in, d->d_out, d->d_cend, d->d_cbw, d->d_seg, d->d_status};
    for (void *p : bufs)
        (void)hipFree(p);
    for (int i = 0; i < gss_dev::RING; i++)
        for (int j = 0; j < 2; j++) {
            (void)hipEventDestroy(d->ev_a[i][j]);
            (void)hipEventDestroy(d->ev_b[i][j]);
            (void)hipEventDestroy(d->ev_l[i][j]);
        }
    delete d;
    return 0;
}

static int nseg_of(int n, int r) { return (n + r - 1) / r; }
/* anchor row stride: the segment starts and one dummy slot (gss_code_seg_states_bf) */
static int nsegp_of(int n, int r) { return (nseg_of(n, r) + 1 + 31) & ~31; }

static int reserve_set(gss_dev *d, int set, int max_blocks, int n_per_blk, int R)
{
    gss_dev::anchor_set &a = d->set[set];
    size_t need = (size_t)max_blocks * GSS_MAXCH * (size_t)nsegp_of(n_per_blk, R);
    if (need <= a.cap)
        return 0;
    (void)hipFree(a.carr);
    (void)hipFree(a.code);
    (void)hipFree(a.cnt);
    a.carr = a.code = nullptr;
    a.cnt = nullptr;
    a.cap = 0;
    HIP_TRY(hipMalloc(&a.carr, need * sizeof(double)));
    HIP_TRY(hipMalloc(&a.code, need * sizeof(double)));
    HIP_TRY(hipMalloc(&a.cnt, need * sizeof(uint32_t)));
    a.cap = need;
    return 0;
}

extern "C" int gss_dev_reserve(gss_dev *d, int max_blocks, int n_per_blk)
{
    if (!d || max_blocks <= 0 || n_per_blk <= 0)
        return gss_fail(GSS_E_ARG, "invalid reserve arguments");
    HIP_TRY(hipSetDevice(d->ordinal));
    for (int set = 0; set < 2; set++) {
        int rc = reserve_set(d, set, max_blocks, n_per_blk, d->seg_r);
        if (rc) return rc;
    }
    return 0;
}

typedef void (*synth_fn)(const gss_chan_blk_t *, const int32_t *, const uint32_t *,
                         const uint32_t *, const double *, const double *, const uint32_t *,
                         lut_arg, int, int, int, int, int, uint8_t *, size_t, int32_t *,
                         const int32_t *);

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

/* Stage A over nblk blocks, or over the nblk blocks listed in blist (device) when non-null */
static int anchor_launch(gss_dev *d, int set, const gss_chan_blk_t *blk, const int32_t *nch,
                         int nch_max, const double *carr_ck, int nblk, int n_per_blk,
                         double *carr_end, const int32_t *blist, int R, void *stream)
{
    if (!d || !blk || !nch || nblk <= 0 || n_per_blk <= 0 || set < 0 || set > 1)
        return gss_fail(GSS_E_ARG, "invalid anchor arguments");
    if (nch_max > GSS_MAXCH)
        return gss_fail(GSS_E_ARG, "nch_max %d > %d", nch_max, GSS_MAXCH);
    HIP_TRY(hipSetDevice(d->ordinal));
    int rc = reserve_set(d, set, nblk, n_per_blk, R);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int nseg = nseg_of(n_per_blk, R), nsegp = nsegp_of(n_per_blk, R);
    const int nchp = nch_max < 1 ? 1 : nch_max;
    const gss_dev::anchor_set &a = d->set[set];
    /* channel-major waves; code chains one lane per block (first: they are the long pole),
       carrier chains one lane per block sub-chain (GSS_NCK per block with checkpoints) */
    const int a_blocks = nchp * ((nblk + ANCHOR_THREADS - 1) / ANCHOR_THREADS) +
                         nchp * ((nblk * (carr_ck ? GSS_NCK : 1) + ANCHOR_THREADS - 1) /
                                 ANCHOR_THREADS);
    hipEvent_t *ev = d->ev_a[d->n_a % gss_dev::RING];
    d->n_a++;
    HIP_TRY(hipEventRecord(ev[0], st));
    hipLaunchKernelGGL(gss_anchor_kernel, dim3(a_blocks), dim3(ANCHOR_THREADS), 0, st, blk, nch,
                       carr_ck, nblk, nchp, n_per_blk, nseg, nsegp, R, a.carr, a.code, a.cnt,
                       carr_end, blist);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[1], st));
    return 0;
}

extern "C" int gss_anchor_device(gss_dev *d, int set, const gss_chan_blk_t *blk,
                                 const int32_t *nch, int nch_max, const double *carr_ck,
                                 int nblk, int n_per_blk, double *carr_end, void *stream)
{
    return anchor_launch(d, set, blk, nch, nch_max, carr_ck, nblk, n_per_blk, carr_end, nullptr,
                         d->seg_r, stream);
}

/* Stage B over nblk blocks, or over the nblk blocks listed in blist (device) when non-null */
static int render_launch(gss_dev *d, int set, const gss_chan_blk_t *blk, const int32_t *nch,
                         int nch_max, const uint32_t *ca_bits, const uint32_t *nav, int nblk,
                         int n_per_blk, int fmt, void *out, int32_t *status,
                         const int32_t *blist, int R, void *stream)
{
    if (!d || !blk || !nch || !ca_bits || !out || nblk <= 0 || n_per_blk <= 0 || set < 0 ||
        set > 1)
        return gss_fail(GSS_E_ARG, "invalid render arguments");
    const size_t bb = gss_block_bytes(n_per_blk, fmt);
    if (bb == 0)
        return gss_fail(GSS_E_ARG, "invalid format %d for %d samples/block", fmt, n_per_blk);
    const int nseg = nseg_of(n_per_blk, R), nsegp = nsegp_of(n_per_blk, R);
    const gss_dev::anchor_set &a = d->set[set];
    if ((size_t)nblk * GSS_MAXCH * (size_t)nsegp > a.cap)
        return gss_fail(GSS_E_STATE, "anchor set %d holds no Stage A output of this size", set);
    const int nchp = nch_max < 1 ? 1 : nch_max;
    if (nchp > GSS_MAXCH)
        return gss_fail(GSS_E_ARG, "nch_max %d > %d", nch_max, GSS_MAXCH);
    synth_fn fn = pick_kernel(fmt, nchp);
    if (!fn)
        return gss_fail(GSS_E_ARG, "no kernel for fmt=%d nch=%d", fmt, nchp);
    HIP_TRY(hipSetDevice(d->ordinal));
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t *ev = d->ev_b[d->n_b % gss_dev::RING];
    d->n_b++;
    const int wg_per_blk = (nseg + SYNTH_THREADS - 1) / SYNTH_THREADS;
    HIP_TRY(hipEventRecord(ev[0], st));
    hipLaunchKernelGGL(fn, dim3(nblk * wg_per_blk), dim3(SYNTH_THREADS), 0, st, blk, nch, ca_bits,
                       nav, a.carr, a.code, a.cnt, d->lut, n_per_blk, nseg, nsegp, R, wg_per_blk,
                       (uint8_t *)out, bb, status, blist);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[1], st));
    return 0;
}

extern "C" int gss_render_device(gss_dev *d, int set, const gss_chan_blk_t *blk,
                                 const int32_t *nch, int nch_max, const uint32_t *ca_bits,
                                 int n_ca, const uint32_t *nav, int n_nav, int nblk,
                                 int n_per_blk, int fmt, void *out, int32_t *status, void *stream)
{
    (void)n_ca; (void)n_nav;
    return render_launch(d, set, blk, nch, nch_max, ca_bits, nav, nblk, n_per_blk, fmt, out,
                         status, nullptr, d->seg_r, stream);
}

/* ---- fast path -------------------------------------------------------------------------- */
typedef void (*lin_fn)(const gss_lin_t *, const lin_seg *, const lin_chan *, const int32_t *,
                       const int32_t *, const uint32_t *, const uint32_t *, lut_arg, int, int,
                       int, uint8_t *, size_t);

static lin_fn pick_lin(int fmt)
{
    switch (fmt) {
    case 16: return gss_lin_kernel<16>;
    case 8: return gss_lin_kernel<8>;
    case 1: return gss_lin_kernel<1>;
    default: return nullptr;
    }
}

extern "C" int gss_synth_lin_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                                    int nch_max, const gss_lin_t *lin, const int32_t *fast,
                                    const int32_t *fb_list, int n_fb, const double *carr_ck,
                                    const uint32_t *ca_bits, int n_ca, const uint32_t *nav,
                                    int n_nav, int nblk, int n_per_blk, int fmt, void *out,
                                    int32_t *status, void *stream)
{
    (void)n_nav;
    if (!d || !blk || !nch || !lin || !fast || !ca_bits || !out || nblk <= 0 || n_per_blk <= 0 ||
        n_ca <= 0 || n_fb < 0 || n_fb > nblk || (n_fb > 0 && !fb_list))
        return gss_fail(GSS_E_ARG, "invalid synth_lin arguments");
    const size_t bb = gss_block_bytes(n_per_blk, fmt);
    if (bb == 0)
        return gss_fail(GSS_E_ARG, "invalid format %d for %d samples/block", fmt, n_per_blk);
    const int nchp = nch_max < 1 ? 1 : nch_max;
    if (nchp > GSS_MAXCH)
        return gss_fail(GSS_E_ARG, "nch_max %d > %d", nch_max, GSS_MAXCH);
    lin_fn fn = pick_lin(fmt);
    if (!fn)
        return gss_fail(GSS_E_ARG, "no fast kernel for fmt=%d nch=%d", fmt, nchp);
    HIP_TRY(hipSetDevice(d->ordinal));
    hipStream_t st = (hipStream_t)stream;
    /* chip-sign bit-streams of every C/A table row (32 x 99 x 4 B) and, after them, the chunk
       window table (32 x 2560 x 64 B); rebuilt per call (the sample rate sets its window
       advance): a few µs */
    const size_t ncbw = (size_t)n_ca * CAB_W, ntw = (size_t)n_ca * GSS_LIN_TWE * LIN_CH;
    const size_t tw_off = (ncbw + 63) & ~(size_t)63;
    if ((tw_off + ntw) * sizeof(uint32_t) > d->d_cbw_cap) {
        (void)hipFree(d->d_cbw);
        d->d_cbw = nullptr;
        d->d_cbw_cap = 0;
        HIP_TRY(hipMalloc(&d->d_cbw, (tw_off + ntw) * sizeof(uint32_t)));
        d->d_cbw_cap = (tw_off + ntw) * sizeof(uint32_t);
    }
    hipLaunchKernelGGL(gss_cab_kernel, dim3((unsigned)((ncbw + 255) / 256)), dim3(256), 0, st,
                       ca_bits, n_ca, d->d_cbw);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(gss_tw16_kernel, dim3((unsigned)((ntw + 255) / 256)), dim3(256), 0, st,
                       (const uint32_t *)d->d_cbw, n_ca, gss_lin_wstep16(n_per_blk),
                       d->d_cbw + tw_off);
    HIP_TRY(hipGetLastError());
    const int segs = (n_per_blk + 64 * LIN_STEPS - 1) / (64 * LIN_STEPS);
    const int wg_per_blk = (segs + LIN_WAVES - 1) / LIN_WAVES;
    const size_t nsegrows = (size_t)nblk * GSS_MAXCH * segs;
    const size_t seg_bytes = nsegrows * sizeof(lin_seg);
    const size_t need_rows = seg_bytes + (size_t)nblk * GSS_MAXCH * sizeof(lin_chan);
    if (need_rows > d->d_seg_cap) {
        (void)hipFree(d->d_seg);
        d->d_seg = nullptr;
        d->d_seg_cap = 0;
        HIP_TRY(hipMalloc(&d->d_seg, need_rows));
        d->d_seg_cap = need_rows;
    }
    lin_seg *d_segs = (lin_seg *)d->d_seg;
    lin_chan *d_chans = (lin_chan *)((char *)d->d_seg + seg_bytes);
    hipLaunchKernelGGL(gss_linseg_kernel, dim3((unsigned)((nsegrows + 255) / 256)), dim3(256), 0,
                       st, lin, blk, nch, fast, nblk, segs, d_segs, d_chans);
    HIP_TRY(hipGetLastError());
    if (n_fb > 0) {          /* the exact path for the uncertified blocks, on the aux stream */
        HIP_TRY(hipEventRecord(d->ev_in, st));
        HIP_TRY(hipStreamWaitEvent(d->aux, d->ev_in, 0));
        /* short Stage-B segments (256 samples): few blocks, so latency matters, not work */
        const int R = 256;
        int rc = anchor_launch(d, 0, blk, nch, nch_max, carr_ck, n_fb, n_per_blk, nullptr,
                               fb_list, R, d->aux);
        if (rc) return rc;
        rc = render_launch(d, 0, blk, nch, nch_max, ca_bits, nav, n_fb, n_per_blk, fmt, out,
                           status, fb_list, R, d->aux);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(d->ev_fb, d->aux));
    }
    hipEvent_t *ev = d->ev_l[d->n_l % gss_dev::RING];
    d->n_l++;
    HIP_TRY(hipEventRecord(ev[0], st));
    hipLaunchKernelGGL(fn, dim3((unsigned)nblk * wg_per_blk), dim3(LIN_THREADS), 0, st, lin,
                       (const lin_seg *)d_segs, (const lin_chan *)d_chans, nch, fast, d->d_cbw,
                       d->d_cbw + tw_off, d->lut, n_per_blk, segs, wg_per_blk, (uint8_t *)out, bb);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[1], st));
    if (n_fb > 0)                                 /* the call completes when both are done */
        HIP_TRY(hipStreamWaitEvent(st, d->ev_fb, 0));
    return 0;
}

extern "C" int gss_synth_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                                int nch_max, const double *carr_ck, const uint32_t *ca_bits,
                                int n_ca,
                                const uint32_t *nav, int n_nav, int nblk, int n_per_blk, int fmt,
                                void *out, double *carr_end, int32_t *status, void *stream)
{
    if (!d || !blk || !nch || !ca_bits || !out || nblk <= 0 || n_per_blk <= 0)
        return gss_fail(GSS_E_ARG, "invalid synth arguments");
    if (gss_block_bytes(n_per_blk, fmt) == 0)
        return gss_fail(GSS_E_ARG, "invalid format %d for %d samples/block", fmt, n_per_blk);
    int rc = gss_anchor_device(d, 0, blk, nch, nch_max, carr_ck, nblk, n_per_blk, carr_end,
                               stream);
    if (rc) return rc;
    return gss_render_device(d, 0, blk, nch, nch_max, ca_bits, n_ca, nav, n_nav, nblk, n_per_blk,
                             fmt, out, status, stream);
}

/* average [ms] of the last min(n, RING) launches of one stage's event ring */
static int ring_avg(hipEvent_t (*ev)[2], int n, double *avg)
{
    const int cnt = n < gss_dev::RING ? n : gss_dev::RING;
    double acc = 0.0;
    if (cnt > 0) {
        HIP_TRY(hipEventSynchronize(ev[(n - 1) % gss_dev::RING][1]));
        for (int i = 0; i < cnt; i++) {
            hipEvent_t *e = ev[(n - 1 - i) % gss_dev::RING];
            float t = 0.f;
            HIP_TRY(hipEventElapsedTime(&t, e[0], e[1]));
            acc += t;
        }
        acc /= cnt;
    }
    *avg = acc;
    return 0;
}

extern "C" int gss_dev_timing(gss_dev *d, int reset, int *n, float *ckpt_ms, float *synth_ms)
{
    if (!d) return gss_fail(GSS_E_ARG, "null device");
    if (reset) {
        d->n_a = d->n_b = d->n_l = 0;
        return 0;
    }
    double a = 0.0, b = 0.0;
    int rc = ring_avg(d->ev_a, d->n_a, &a);
    if (rc) return rc;
    rc = ring_avg(d->ev_b, d->n_b, &b);
    if (rc) return rc;
    if (n) *n = d->n_b < gss_dev::RING ? d->n_b : gss_dev::RING;
    if (ckpt_ms) *ckpt_ms = (float)a;
    if (synth_ms) *synth_ms = (float)b;
    return 0;
}

extern "C" int gss_dev_timing_lin(gss_dev *d, int *n, float *lin_ms)
{
    if (!d) return gss_fail(GSS_E_ARG, "null device");
    double l = 0.0;
    int rc = ring_avg(d->ev_l, d->n_l, &l);
    if (rc) return rc;
    if (n) *n = d->n_l < gss_dev::RING ? d->n_l : gss_dev::RING;
    if (lin_ms) *lin_ms = (float)l;
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
                              const double *carr_ck, const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                              int nblk, int n_per_blk, int fmt, void *out, double *carr_end)
{
    if (!d || !blk || !nch || !ca_bits || !out || nblk <= 0 || n_ca <= 0)
        return gss_fail(GSS_E_ARG, "invalid synth arguments");
    size_t bb = gss_block_bytes(n_per_blk, fmt);
    if (bb == 0)
        return gss_fail(GSS_E_ARG, "invalid format %d for %d samples/block", fmt, n_per_blk);
    if (n_per_blk > (1 << 30))
        return gss_fail(GSS_E_ARG, "block too large");
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
                !(p->carr0 >= 0.0 && p->carr0 <= 1.0) ||
                !(p->code_step > 0.0 && p->code_step < 1023.0) ||
                !(p->carr_step > -1.0 && p->carr_step < 1.0))
                return gss_fail(GSS_E_ARG, "block %d channel %d: parameter out of range", b, k);
            if (carr_ck)
                for (int j = 0; j < GSS_NCK; j++) {
                    double c = carr_ck[((size_t)b * GSS_MAXCH + k) * GSS_NCK + j];
                    if (!(c >= 0.0 && c <= 1.0))
                        return gss_fail(GSS_E_ARG, "block %d channel %d: checkpoint %d out of "
                                        "range", b, k, j);
                }
        }
    }
    size_t sz_blk = sizeof(gss_chan_blk_t) * GSS_MAXCH * (size_t)nblk;
    size_t sz_nch = sizeof(int32_t) * (size_t)nblk;
    size_t sz_ca = sizeof(uint32_t) * GSS_CA_WORDS * (size_t)n_ca;
    size_t sz_nav = sizeof(uint32_t) * GSS_NAV_WORDS * (size_t)(n_nav > 0 ? n_nav : 1);
    size_t sz_ck = carr_ck ? sizeof(double) * GSS_MAXCH * GSS_NCK * (size_t)nblk : 0;
    /* the certified fast path unless the caller wants carrier end phases (exact path only) */
    const char *path = getenv("GSS_PATH");
    const bool use_lin = carr_end == nullptr && !(path && strcmp(path, "walk") == 0);
    size_t sz_lin = use_lin ? sizeof(gss_lin_t) * GSS_MAXCH * (size_t)nblk : 0;
    size_t sz_fast = use_lin ? sizeof(int32_t) * 2 * (size_t)nblk : 0;   /* fast[] + list */
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t tot = al(sz_blk) + al(sz_nch) + al(sz_ca) + al(sz_nav) + al(sz_ck) + al(sz_lin) +
                 al(sz_fast);
    int rc = grow((uint8_t **)&d->h_in, &d->h_in_cap, tot);
    if (rc) return rc;
    if (use_lin) {
        gss_lin_t *h_lin = (gss_lin_t *)malloc(sz_lin);
        int32_t *h_fast = (int32_t *)malloc(sz_fast);
        if (!h_lin || !h_fast) {
            free(h_lin);
            free(h_fast);
            return gss_fail(GSS_E_NOMEM, "out of memory");
        }
        rc = gss_linearize(blk, nch, nblk, n_per_blk, ca_bits, n_ca, nav, n_nav, h_lin, h_fast, 8);
        int n_fb = 0;
        for (int b = 0; b < nblk; b++)
            if (!h_fast[b])
                h_fast[nblk + n_fb++] = b;
        uint8_t *lb = (uint8_t *)d->h_in + al(sz_blk) + al(sz_nch) + al(sz_ca) + al(sz_nav) +
                      al(sz_ck);
        gss_lin_t *d_lin = (gss_lin_t *)lb;
        int32_t *d_fast = (int32_t *)(lb + al(sz_lin));
        if (rc == 0 && hipMemcpy(d_lin, h_lin, sz_lin, hipMemcpyHostToDevice) != hipSuccess)
            rc = gss_fail(GSS_E_HIP, "upload of the fast-path lines failed");
        if (rc == 0 && hipMemcpy(d_fast, h_fast, sz_fast, hipMemcpyHostToDevice) != hipSuccess)
            rc = gss_fail(GSS_E_HIP, "upload of the fast-path lines failed");
        free(h_lin);
        free(h_fast);
        if (rc) return rc;
        uint8_t *base = (uint8_t *)d->h_in;
        gss_chan_blk_t *d_blk = (gss_chan_blk_t *)base;
        int32_t *d_nch = (int32_t *)(base + al(sz_blk));
        uint32_t *d_ca = (uint32_t *)(base + al(sz_blk) + al(sz_nch));
        uint32_t *d_nav = (uint32_t *)(base + al(sz_blk) + al(sz_nch) + al(sz_ca));
        double *d_ck = carr_ck ? (double *)(base + al(sz_blk) + al(sz_nch) + al(sz_ca) +
                                            al(sz_nav)) : nullptr;
        if (carr_ck)
            HIP_TRY(hipMemcpy(d_ck, carr_ck, sz_ck, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_blk, blk, sz_blk, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_nch, nch, sz_nch, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_ca, ca_bits, sz_ca, hipMemcpyHostToDevice));
        if (n_nav > 0)
            HIP_TRY(hipMemcpy(d_nav, nav, sz_nav, hipMemcpyHostToDevice));
        else
            HIP_TRY(hipMemset(d_nav, 0, sz_nav));
        rc = grow((uint8_t **)&d->d_out, &d->d_out_cap, bb * (size_t)nblk);
        if (rc) return rc;
        HIP_TRY(hipMemset(d->d_status, 0, sizeof(int32_t)));
        rc = gss_synth_lin_device(d, d_blk, d_nch, maxc, d_lin, d_fast, d_fast + nblk, n_fb, d_ck,
                                  d_ca, n_ca, d_nav, n_nav, nblk, n_per_blk, fmt, d->d_out,
                                  d->d_status, nullptr);
        if (rc) return rc;
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(out, d->d_out, bb * (size_t)nblk, hipMemcpyDeviceToHost));
        int32_t stv = 0;
        HIP_TRY(hipMemcpy(&stv, d->d_status, sizeof stv, hipMemcpyDeviceToHost));
        if (stv)
            return gss_fail(GSS_E_RANGE, "nav word index ran past dwrd[59]");
        return 0;
    }
    uint8_t *base = (uint8_t *)d->h_in;
    gss_chan_blk_t *d_blk = (gss_chan_blk_t *)base;
    int32_t *d_nch = (int32_t *)(base + al(sz_blk));
    uint32_t *d_ca = (uint32_t *)(base + al(sz_blk) + al(sz_nch));
    uint32_t *d_nav = (uint32_t *)(base + al(sz_blk) + al(sz_nch) + al(sz_ca));
    double *d_ck = carr_ck ? (double *)(base + al(sz_blk) + al(sz_nch) + al(sz_ca) + al(sz_nav))
                           : nullptr;
    if (carr_ck)
        HIP_TRY(hipMemcpy(d_ck, carr_ck, sz_ck, hipMemcpyHostToDevice));
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
    rc = gss_synth_device(d, d_blk, d_nch, maxc, d_ck, d_ca, n_ca, d_nav, n_nav, nblk, n_per_blk,
                          fmt,
                          d->d_out, d_cend, d->d_status, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, d->d_out, bb * (size_t)nblk, hipMemcpyDeviceToHost));
    if (carr_end)
        HIP_TRY(hipMemcpy(carr_end, d_cend, sizeof(double) * GSS_MAXCH * (size_t)nblk,
                          hipMemcpyDeviceToHost));
    int32_t stv = 0;
    HIP_TRY(hipMemcpy(&stv, d->d_status, sizeof stv, hipMemcpyDeviceToHost));
    if (stv)
        return gss_fail(GSS_E_RANGE, "nav word index ran past dwrd[59]");
    return 0;
}
