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
 * of step s renders sample chunk + 64 s + l), and per chunk and lane the kernel takes one anchor
 * from the lines, then adds 32-bit (carrier) or 32.32 fixed-point (code) steps:
 *   carrier  K(p) = hi32(X(c + l) + A) + s * dX  mod 2^32,  dX = hi32(64 xs + 2^31)  [2^-32 cycle]
 *            A = 2^31 - (GSS_LIN_CH - 1) e / 2 centres the steps' error e = dX 2^32 - 64 xs
 *            LUT cell = K(p) >> 23
 *   code     C(p) = ((Z(c + l) + 2^17) >> 18) + s * dZ,   dZ = (64 zs + 2^17) >> 18
 *                                                                      [2^-32 chip, unwrapped]
 *            chip = (C(p) >> 32) mod 1023
 * (p = c + 64 s + l).  Each rounding is at most half a unit, so
 * |K 2^32 - X| <= 2^31 + |s - (GSS_LIN_CH - 1)/2| 2^31 and |C 2^18 - Z| <= 2^17 (1 + s):
 * GSS_LIN_KDEV_* bound these, and the proof adds them to its own line-versus-reference bound.
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

/* per-step increments and the carrier's anchor offset */
GSS_LIN_FN uint32_t gss_lin_dx(uint64_t xs) { return (uint32_t)((xs * 64u + (1ull << 31)) >> 32); }
GSS_LIN_FN uint64_t gss_lin_dz(uint64_t zs) { return (zs * 64u + (1ull << 17)) >> 18; }
GSS_LIN_FN uint64_t gss_lin_xa(uint64_t xs)
{
    const int64_t e = (int64_t)(((uint64_t)gss_lin_dx(xs) << 32) - xs * 64u);
    return (1ull << 31) - (uint64_t)((e * (GSS_LIN_CH - 1)) / 2);
}

/* worst-case distance of the kernel's values from the lines, in line units (2^-64 cycle,
   2^-50 chip) */
#define GSS_LIN_KDEV_CARR (((uint64_t)GSS_LIN_CH / 2 + 1) << 31)
#define GSS_LIN_KDEV_CODE ((uint64_t)GSS_LIN_CH << 17)

#if !defined(__HIP_DEVICE_COMPILE__)
/* the kernel's carrier LUT cell and chip at block sample p (host side: 128-bit code line) */
GSS_LIN_FN int gss_lin_kcell(uint64_t x0, uint64_t xs, int64_t p)
{
    const int64_t c = p & ~(int64_t)(GSS_LIN_CHUNK - 1);
    const int64_t l = p & 63, s = (p - c) >> 6;
    const uint64_t a = x0 + (uint64_t)(c + l) * xs + gss_lin_xa(xs);
    const uint32_t k = (uint32_t)(a >> 32) + (uint32_t)s * gss_lin_dx(xs);
    return (int)(k >> 23);
}

GSS_LIN_FN int gss_lin_kchip(uint64_t z0, uint64_t zs, int64_t p)
{
    const int64_t c = p & ~(int64_t)(GSS_LIN_CHUNK - 1);
    const int64_t l = p & 63, s = (p - c) >> 6;
    const unsigned __int128 z = (unsigned __int128)z0 + (unsigned __int128)(uint64_t)(c + l) * zs;
    const unsigned __int128 k = ((z + (1u << 17)) >> 18) + (unsigned __int128)(uint64_t)s *
                                gss_lin_dz(zs);
    return (int)((uint64_t)(k >> 32) % 1023u);
}
#endif

#endif /* GSS_LIN_H */
