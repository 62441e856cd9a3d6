/*
 * gss_lin.h — the fast path's render arithmetic, restated once for the three places that must
 * agree on it bit for bit: the GPU kernel (gss_lin_kernel, csrc/hip/gss_synth.hip), the host
 * proof that certifies blocks for it (csrc/host/linearize.c) and the CPU checker of the tests
 * (tests/helpers/lin_check.c).
 *
 * A block's channel is described by two 64-bit integer lines (gss_lin_t): the carrier
 * X(p) = x0 + p*xs mod 2^64 [2^-64 cycle] and the code Z(p) = z0 + p*zs [2^-50 chip, unwrapped]
 * (linearize.c proves how close they stay to the reference's double recurrences,
 * gpssim.c:2212-2250).  The kernel does not evaluate them at every sample.  Samples are grouped
 * in chunks of GSS_LIN_CHUNK (block-relative, aligned), a chunk in GSS_LIN_CH steps of 64 (lane l
 * of step s renders sample p = c + 64 s + l), and each lane keeps code and carrier in ONE 64-bit
 * register P (code in the low word, 8.24 fixed point with byte 3 = chip mod 256; carrier in the
 * high word, 2^-32 cycle) that advances by one 64-bit add per step:
 *   anchor   P(c, l) = B(c) + L(l)  mod 2^64, from the chunk's base and the lane's offset
 *              B = hi32(X(c) + A) : lo32((Z(c) + Ac) >> 26)
 *              L = hi32(l xs + 2^31) : lo32((l zs) >> 26)
 *   step     P += dX : dC,   dX = hi32(64 xs + 2^31) [2^-32 cycle],
 *                            dC = (64 zs + 2^25) >> 26 [2^-24 chip]
 *            A = 2^31 - (GSS_LIN_CH - 1) e / 2 and Ac = 2^25 - (GSS_LIN_CH - 1) ec / 2 centre
 *            the steps' errors e = dX 2^32 - 64 xs and ec = dC 2^26 - 64 zs.
 *   Z(c) is the code line reduced at its wave segment's start (GSS_LIN_SEG samples, aligned)
 *   to the chip there mod 1023 (1023 for chip 0: gss_lin_e0), plus the fraction.
 *   LUT cell = high word >> 23, where every carry out of the low word (at the anchor add and at
 *   each step, one per 256 chips) adds 2^-32 cycle to the carrier; chip = (unwrapped low word
 *   >> 24) mod 1023.
 * Each rounding is at most one unit (half a unit where rounded to nearest) and the carries only
 * add, so the carrier is within (GSS_LIN_CH/2 + 3) 2^31 + (2 + (GSS_LIN_CH - 1) dC / 2^32) 2^32
 * and the code within (GSS_LIN_CH/2 + 3) 2^25 of the lines (GSS_LIN_KDEV_*, 2^-64 cycle and 2^-50 chip); the
 * proof adds these to its own line-versus-reference bound.
 * The kernel reads each step's chip sign from a 32-chip window (gss_lin_kernel): every lane's
 * chip of one step must lie in it, which linearize.c checks as 63 zs + 3 chips <= 31
 * (GSS_LIN_WIN_OK).
 */
#ifndef GSS_LIN_H
#define GSS_LIN_H

#include <stdint.h>

#ifndef GSS_LIN_CH
#define GSS_LIN_CH     16                      /* 64-sample steps per chunk                   */
#endif
#define GSS_LIN_CHUNK  (64 * GSS_LIN_CH)       /* samples per chunk (block-relative, aligned) */
#define GSS_LIN_SEG    4096                    /* samples per wave segment: the code line is
                                                  taken mod 1023 chips at each segment start   */

#if defined(__HIPCC__)
#define GSS_LIN_FN static __host__ __device__ inline
#else
#define GSS_LIN_FN static inline
#endif

#define GSS_LIN_CSH    26                      /* code line (2^-50 chip) >> 26 = 8.24 chips   */

/* per-step increments and the carrier's anchor offset */
GSS_LIN_FN uint32_t gss_lin_dx(uint64_t xs) { return (uint32_t)((xs * 64u + (1ull << 31)) >> 32); }
GSS_LIN_FN uint32_t gss_lin_dz(uint64_t zs)
{
    return (uint32_t)((zs * 64u + (1ull << (GSS_LIN_CSH - 1))) >> GSS_LIN_CSH);
}
GSS_LIN_FN uint64_t gss_lin_xa(uint64_t xs)
{
    const int64_t e = (int64_t)(((uint64_t)gss_lin_dx(xs) << 32) - xs * 64u);
    return (1ull << 31) - (uint64_t)((e * (GSS_LIN_CH - 1)) / 2);
}
/* the code's anchor offset Ac (rounding and centring), added to Z(c) before >> 26 */
GSS_LIN_FN uint64_t gss_lin_za(uint64_t zs)
{
    const int64_t ec = (int64_t)(((uint64_t)gss_lin_dz(zs) << GSS_LIN_CSH) - zs * 64u);
    return (1ull << (GSS_LIN_CSH - 1)) - (uint64_t)((ec * (GSS_LIN_CH - 1)) / 2);
}

/* the chip the code line is reduced to at a segment start: the chip there mod 1023, taken as 1023
   for chip 0 so that the (possibly negative) anchor offset keeps the reduced line positive */
GSS_LIN_FN uint32_t gss_lin_e0(uint64_t chips)
{
    const uint32_t e = (uint32_t)(chips % 1023u);
    return e ? e : 1023u;
}

/* worst-case distance of the kernel's values from the lines, in line units (2^-64 cycle,
   2^-50 chip) */
/* carrier: roundings plus the carries of the code word, at most one at the anchor and one per
   2^32 of code advance over the chunk's steps (zs: the code line's step, 2^-50 chip per sample) */
#define GSS_LIN_KDEV_CARR(zs)                                                                      \
    ((((uint64_t)GSS_LIN_CH / 2 + 3) << 31) +                                                     \
     ((2 + (((uint64_t)gss_lin_dz(zs) * (GSS_LIN_CH - 1)) >> 32)) << 32))
#define GSS_LIN_KDEV_CODE (((uint64_t)GSS_LIN_CH / 2 + 3) << (GSS_LIN_CSH - 1))
/* the 32-chip step window holds every lane's chip (zs in 2^-50 chip per sample, < 1 chip) */
#define GSS_LIN_WIN_OK(zs) ((zs) * 63u + (3ull << 50) <= (31ull << 50))

/* The chunk window table (gss_tw16_kernel, gss_lin_kernel): row r (a C/A table row) and chunk
   start chip E hold the 16 steps' 32-chip windows of a chunk whose code base zb has
   zb >> 50 = E; step s's window starts at extended chip E + ((s w) >> 4) - GSS_LIN_CBW_PRE, w =
   gss_lin_wstep16(n_per_blk) the nominal chip advance per 64-sample step in 1/16 chip (1.023 MHz
   over the sample rate).  One table serves every channel of a launch: a channel's true advance
   differs from w by its code Doppler (parts in 10^6) and the rounding of w, which
   gss_lin_win16_ok checks against the window's slack, per channel and block. */
#define GSS_LIN_TWE     2560                   /* chunk start chips per table row            */
#define GSS_LIN_CBW_PRE 2                      /* a window starts this far below E + (s w>>4) */
GSS_LIN_FN uint32_t gss_lin_wstep16(int n_per_blk)
{
    return (uint32_t)((104755200ull + (uint64_t)n_per_blk / 2) / (uint64_t)n_per_blk);
}
/* every lane's chip of every step lies in the step's table window, and every chunk's E is inside
   the table, for a channel of code step zs (2^-50 chip per sample) whose code line is reduced to
   at most chip 1024 at each wave segment start (gss_lin_e0) */
GSS_LIN_FN int gss_lin_win16_ok(uint64_t zs, int n_per_blk)
{
    const int64_t U = (int64_t)1 << 50, z = (int64_t)zs;
    /* the kernel's code within KDEV of its anchored line, plus the anchor's centring offset and
       a margin (all below 2^-23 chip) */
    const int64_t kd = (int64_t)GSS_LIN_KDEV_CODE + ((int64_t)1 << 27);
    const uint32_t w = gss_lin_wstep16(n_per_blk);
    if (zs == 0 || zs >= (uint64_t)U)
        return 0;
    for (int s = 0; s < GSS_LIN_CH; s++) {
        const int64_t f = (int64_t)(((uint64_t)s * w) >> 4) - GSS_LIN_CBW_PRE;
        if (64 * s * z - kd < f * U)                          /* lane 0 at or above the start */
            return 0;
        if (U + (64 * s + 63) * z + kd > (f + 32) * U)        /* lane 63 below the end        */
            return 0;
    }
    /* the last chunk of a segment starts 3 chunks after a base at most 1024 chips */
    return 1025 * U + (int64_t)(GSS_LIN_SEG - GSS_LIN_CHUNK) * z + kd < (int64_t)GSS_LIN_TWE * U;
}

/* the lane offset L(l) of gss_lin.h: carrier word (high) and code word (low) */
GSS_LIN_FN uint64_t gss_lin_lane(uint64_t xs, uint64_t zs, uint32_t l)
{
    const uint32_t lx = (uint32_t)(((uint64_t)l * xs + (1ull << 31)) >> 32);
    const uint32_t lz = (uint32_t)(((uint64_t)l * zs) >> GSS_LIN_CSH);
    return ((uint64_t)lx << 32) | lz;
}

/* the kernel's LUT cell and chip at block sample p (128-bit code line; the proof's, on the host
   and in gss_linearize_device) */
typedef struct {
    int cell, chip;
} gss_lin_kc;

GSS_LIN_FN gss_lin_kc gss_lin_kernel_at(uint64_t x0, uint64_t xs, uint64_t z0, uint64_t zs,
                                         int64_t p)
{
    const int64_t c = p & ~(int64_t)(GSS_LIN_CHUNK - 1);
    const int64_t l = p & 63, s = (p - c) >> 6;
    const uint64_t lane = gss_lin_lane(xs, zs, (uint32_t)l);
    /* code: the low word, unwrapped (no carries in), from the line reduced at the segment start */
    const int64_t n0 = p & ~(int64_t)(GSS_LIN_SEG - 1);
    const unsigned __int128 zn = (unsigned __int128)z0 + (unsigned __int128)(uint64_t)n0 * zs;
    const int64_t chips = (int64_t)(zn >> 50), e0 = gss_lin_e0((uint64_t)chips);
    const __int128 z = (__int128)z0 + (__int128)c * (__int128)zs -
                      (__int128)(chips - e0) * ((__int128)1 << 50);
    const unsigned __int128 zk = (unsigned __int128)((z + (int64_t)gss_lin_za(zs)) >> GSS_LIN_CSH);
    const uint64_t za = (uint64_t)(uint32_t)zk + (uint32_t)lane;       /* anchor add, carry */
    const uint64_t zw = (uint64_t)(uint32_t)za + (uint64_t)s * gss_lin_dz(zs);   /* low word */
    const unsigned __int128 kz = zk + (uint32_t)lane + (unsigned __int128)(uint64_t)s *
                                 gss_lin_dz(zs);
    /* carrier: the high word plus the low word's carries */
    const uint32_t xb = (uint32_t)((x0 + (uint64_t)c * xs + gss_lin_xa(xs)) >> 32);
    const uint32_t xk = xb + (uint32_t)(lane >> 32) + (uint32_t)(za >> 32) +
                        (uint32_t)s * gss_lin_dx(xs) + (uint32_t)(zw >> 32);
    gss_lin_kc r;
    r.cell = (int)(xk >> 23);
    r.chip = (int)((uint64_t)(kz >> 24) % 1023u);
    return r;
}

#endif /* GSS_LIN_H */
