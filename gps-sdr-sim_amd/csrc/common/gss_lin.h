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
 * of step s renders sample p = c + 64 s + l), and each lane keeps carrier and code in ONE 64-bit
 * register P (carrier in the low word, 2^-32 cycle; code in the high word, 8.24 fixed point with
 * byte 3 = chip mod 256) that advances by one 64-bit add per step:
 *   anchor   P(c, l) = B(c) + L(l)  mod 2^64, from the chunk's base and the lane's offset
 *              B = lo32((Z(c) + 2^25) >> 26) : hi32(X(c) + A)
 *              L = lo32((l zs) >> 26)        : hi32(l xs + 2^31)
 *   step     P += dC : dX,   dX = hi32(64 xs + 2^31) [2^-32 cycle],
 *                            dC = (64 zs + 2^25) >> 26 [2^-24 chip]
 *            A = 2^31 - (GSS_LIN_CH - 1) e / 2 centres the carrier steps' error
 *            e = dX 2^32 - 64 xs.
 *   LUT cell = low word >> 23;  chip = (unwrapped high word >> 24) mod 1023, where every carry
 *   out of the low word (at the anchor add and at each step) adds 2^-24 chip to the code.
 * Each rounding is at most one unit and the carries only add, so the carrier is within
 * (GSS_LIN_CH/2 + 3) 2^31 and the code within 3 GSS_LIN_CH 2^25 of the lines (GSS_LIN_KDEV_*,
 * 2^-64 cycle and 2^-50 chip); the proof adds these to its own line-versus-reference bound.
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

/* worst-case distance of the kernel's values from the lines, in line units (2^-64 cycle,
   2^-50 chip) */
#define GSS_LIN_KDEV_CARR (((uint64_t)GSS_LIN_CH / 2 + 3) << 31)
#define GSS_LIN_KDEV_CODE ((uint64_t)(3 * GSS_LIN_CH) << (GSS_LIN_CSH - 1))
/* the 32-chip step window holds every lane's chip (zs in 2^-50 chip per sample, < 1 chip) */
#define GSS_LIN_WIN_OK(zs) ((zs) * 63u + (3ull << 50) <= (31ull << 50))

/* the lane offset L(l) of gss_lin.h: code word (high) and carrier word (low) */
GSS_LIN_FN uint64_t gss_lin_lane(uint64_t xs, uint64_t zs, uint32_t l)
{
    const uint32_t lx = (uint32_t)(((uint64_t)l * xs + (1ull << 31)) >> 32);
    const uint32_t lz = (uint32_t)(((uint64_t)l * zs) >> GSS_LIN_CSH);
    return ((uint64_t)lz << 32) | lx;
}

#if !defined(__HIP_DEVICE_COMPILE__)
/* the kernel's LUT cell and chip at block sample p (host side: 128-bit code line) */
typedef struct {
    int cell, chip;
} gss_lin_kc;

GSS_LIN_FN gss_lin_kc gss_lin_kernel_at(uint64_t x0, uint64_t xs, uint64_t z0, uint64_t zs,
                                         int64_t p)
{
    const int64_t c = p & ~(int64_t)(GSS_LIN_CHUNK - 1);
    const int64_t l = p & 63, s = (p - c) >> 6;
    const uint64_t lane = gss_lin_lane(xs, zs, (uint32_t)l);
    const uint32_t xb = (uint32_t)((x0 + (uint64_t)c * xs + gss_lin_xa(xs)) >> 32);
    const uint64_t xa = (uint64_t)xb + (uint32_t)lane;         /* anchor add, with its carry */
    const uint64_t xk = (uint64_t)(uint32_t)xa + (uint64_t)s * gss_lin_dx(xs);
    const unsigned __int128 z = (unsigned __int128)z0 + (unsigned __int128)(uint64_t)c * zs;
    const unsigned __int128 k = ((z + (1u << (GSS_LIN_CSH - 1))) >> GSS_LIN_CSH) +
                                (lane >> 32) + (xa >> 32) +
                                (unsigned __int128)(uint64_t)s * gss_lin_dz(zs) + (xk >> 32);
    gss_lin_kc r;
    r.cell = (int)((uint32_t)xk >> 23);
    r.chip = (int)((uint64_t)(k >> 24) % 1023u);
    return r;
}
#endif

#endif /* GSS_LIN_H */
