/*
 * gss_nav.h — the 30 s producers as host/device functions: the C/A Gold code
 * chips (codegen, gpssim.c:132-171) and one LNAV frame's 30-bit words with parity
 * (generateNavMsg gpssim.c:1467-1547, computeChecksum 693-756).  The same code runs in the GPU
 * producers (csrc/hip/gss_producers.hip) and in the host checker gss_nav_rows_host, and must
 * reproduce the host plane's gnss_navmsg.c word for word (tests/test_producers.py).
 */
#ifndef GSS_NAV_H
#define GSS_NAV_H

#include <stdint.h>
#include "gpssim_amd.h"

#if defined(__HIPCC__)
#define GSS_NAV_HD __host__ __device__ inline
#else
#define GSS_NAV_HD static inline
#endif

/* ---- C/A code --------------------------------------------------------------------------------
 * G1 = 1 + x^3 + x^10, G2 = 1 + x^2 + x^3 + x^6 + x^8 + x^9 + x^10, both registers all ones at
 * the epoch (the reference's -1 state).  Bit j of a 10-bit register is stage j+1; the output is
 * stage 10.  Chip i of PRN p = G1(i) xor G2(i + 1023 - delay(p)), 1 = codeCA -1. */
#define GSS_G2_DELAYS                                                                       \
    {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258,                 \
     469, 470, 471, 472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862}

/* the G1 and G2 output bits for chips 0..1022, packed like the table rows */
GSS_NAV_HD void gss_g1g2(uint32_t *g1, uint32_t *g2)
{
    uint32_t r1 = 0x3FFu, r2 = 0x3FFu;
    for (int w = 0; w < GSS_CA_WORDS; w++)
        g1[w] = g2[w] = 0;
    for (int i = 0; i < GSS_CA_LEN; i++) {
        g1[i >> 5] |= ((r1 >> 9) & 1u) << (i & 31);
        g2[i >> 5] |= ((r2 >> 9) & 1u) << (i & 31);
        const uint32_t f1 = ((r1 >> 2) ^ (r1 >> 9)) & 1u;
        const uint32_t f2 = ((r2 >> 1) ^ (r2 >> 2) ^ (r2 >> 5) ^ (r2 >> 7) ^ (r2 >> 8) ^
                             (r2 >> 9)) & 1u;
        r1 = ((r1 << 1) | f1) & 0x3FFu;
        r2 = ((r2 << 1) | f2) & 0x3FFu;
    }
}

GSS_NAV_HD uint32_t gss_bit(const uint32_t *b, int i) { return (b[i >> 5] >> (i & 31)) & 1u; }

/* chip i (0..1022) of PRN p (1..32) from the packed G1/G2 sequences */
GSS_NAV_HD uint32_t gss_ca_chip(const uint32_t *g1, const uint32_t *g2, int prn, int i)
{
    const short delay[32] = GSS_G2_DELAYS;
    int j = i + GSS_CA_LEN - delay[prn - 1];
    if (j >= GSS_CA_LEN)
        j -= GSS_CA_LEN;
    return gss_bit(g1, i) ^ gss_bit(g2, j);
}

/* ---- LNAV parity (IS-GPS-200 eq. 20-XIV) ---------------------------------------------------- */
GSS_NAV_HD uint32_t gss_par(uint32_t v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__popc(v) & 1u;
#else
    return (uint32_t)__builtin_popcount(v) & 1u;
#endif
}

/* the word `source` (data bits 29..6; the previous word's D29 and D30 bits in bits 31 and 30)
   with its six parity bits; nib: words 2 and 10, whose bits 23/24 are solved for zero parity */
GSS_NAV_HD uint32_t gss_nav_parity(uint32_t source, int nib)
{
    const uint32_t m0 = 0x3B1F3480u, m1 = 0x1D8F9A40u, m2 = 0x2EC7CD00u, m3 = 0x1763E680u,
                   m4 = 0x2BB1F340u, m5 = 0x0B7A89C0u;
    uint32_t d = source & 0x3FFFFFC0u;
    const uint32_t d29 = (source >> 31) & 1u, d30 = (source >> 30) & 1u;
    if (nib) {
        if ((d30 + gss_par(m4 & d)) & 1u)
            d ^= 1u << 6;
        if ((d29 + gss_par(m5 & d)) & 1u)
            d ^= 1u << 7;
    }
    uint32_t D = d30 ? d ^ 0x3FFFFFC0u : d;
    D |= ((d29 + gss_par(m0 & d)) & 1u) << 5;
    D |= ((d30 + gss_par(m1 & d)) & 1u) << 4;
    D |= ((d29 + gss_par(m2 & d)) & 1u) << 3;
    D |= ((d30 + gss_par(m3 & d)) & 1u) << 2;
    D |= ((d30 + gss_par(m4 & d)) & 1u) << 1;
    D |= ((d29 + gss_par(m5 & d)) & 1u);
    return D & 0x3FFFFFFFu;
}

/* One frame row (chan_t.dwrd after generateNavMsg): words 0..9 from `head` (the previous frame's
   subframe 5) or, with head == 0, rebuilt from sbf[4] and this tow (a newly allocated channel);
   words 10..59 the frame's five subframes with TOW counts tow+1 .. tow+5 and the week in
   subframe 1 word 3. */
GSS_NAV_HD void gss_nav_frame(const gss_nav_src_t *src, const uint32_t *head, uint32_t *dwrd)
{
    uint32_t tow = src->tow, prev = 0;
    for (int i = 0; i < 10; i++) {
        if (head) {
            dwrd[i] = head[i];
        } else {
            uint32_t wd = src->sbf[4][i];
            if (i == 1)
                wd |= (tow & 0x1FFFFu) << 13;
            wd |= (prev << 30) & 0xC0000000u;
            dwrd[i] = gss_nav_parity(wd, i == 1 || i == 9);
        }
        prev = dwrd[i];
    }
    for (int s = 0; s < 5; s++) {
        tow++;
        for (int i = 0; i < 10; i++) {
            uint32_t wd = src->sbf[s][i];
            if (s == 0 && i == 2)
                wd |= (src->wn & 0x3FFu) << 20;
            if (i == 1)
                wd |= (tow & 0x1FFFFu) << 13;
            wd |= (prev << 30) & 0xC0000000u;
            prev = gss_nav_parity(wd, i == 1 || i == 9);
            dwrd[10 * (s + 1) + i] = prev;
        }
    }
}

/* the head of row r: the rows table when it continues row prev, its own words when given */
GSS_NAV_HD const uint32_t *gss_nav_head(const gss_nav_src_t *src, const uint32_t *rows)
{
    if (src->prev >= 0)
        return rows + (size_t)src->prev * GSS_NAV_WORDS + 50;
    return src->prev == GSS_NAV_HEAD_GIVEN ? src->head : (const uint32_t *)0;
}

#endif
