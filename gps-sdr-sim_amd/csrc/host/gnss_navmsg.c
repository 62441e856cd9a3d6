/*
 * gnss_navmsg.c — C/A Gold codes and the LNAV message (subframes 1-5, TOW/WN, parity).
 * Restates codegen (gpssim.c:132-171), eph2sbf (490-665), countBits/computeChecksum
 * (671-756) and generateNavMsg (1467-1547).  The 30-bit words end up in chan_t.dwrd, the table
 * the kernel reads one data bit at a time.
 */
#include <math.h>
#include <string.h>
#include "gss_host.h"

/* ---- C/A code: G1 = 1+x^3+x^10, G2 = 1+x^2+x^3+x^6+x^8+x^9+x^10, PRN-specific G2 delay --- */
static const short g2_delay[32] = {
      5,   6,   7,   8,  17,  18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258,
    469, 470, 471, 472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862};

void ca_generate(int8_t *ca, int prn)
{
    /* registers hold +1/-1 ("0"/"1"), taps multiply (XOR in the ±1 domain) */
    int8_t g1[K_CA_LEN], g2[K_CA_LEN];
    int r1[10], r2[10];
    if (prn < 1 || prn > 32)
        return;
    for (int i = 0; i < 10; i++)
        r1[i] = r2[i] = -1;
    for (int i = 0; i < K_CA_LEN; i++) {
        g1[i] = (int8_t)r1[9];
        g2[i] = (int8_t)r2[9];
        int fb1 = r1[2] * r1[9];
        int fb2 = r2[1] * r2[2] * r2[5] * r2[7] * r2[8] * r2[9];
        memmove(&r1[1], &r1[0], 9 * sizeof(int));
        memmove(&r2[1], &r2[0], 9 * sizeof(int));
        r1[0] = fb1;
        r2[0] = fb2;
    }
    int off = K_CA_LEN - g2_delay[prn - 1];
    for (int i = 0; i < K_CA_LEN; i++)
        ca[i] = (int8_t)((1 - g1[i] * g2[(i + off) % K_CA_LEN]) / 2);
}

void ca_pack(const int8_t *ca, uint32_t *bits)
{
    memset(bits, 0, GSS_CA_WORDS * sizeof(uint32_t));
    for (int i = 0; i < K_CA_LEN; i++)
        if (ca[i])
            bits[i >> 5] |= 1u << (i & 31);
}

/* ---- ephemeris → subframe words (data bits only; parity added by nav_frame) -------------- */
void nav_subframes(const eph_t *eph, const iono_t *io, uint32_t sbf[5][K_N_DWRD_SBF])
{
    /* scaled integer fields, conversions exactly as gpssim.c:536-584 */
    uint64_t wn = 0;                          /* transmission WN inserted later (gpssim.c:534) */
    uint64_t toe = (uint64_t)(eph->toe.sec / 16.0);
    uint64_t toc = (uint64_t)(eph->toc.sec / 16.0);
    uint64_t iode = (uint64_t)(eph->iode);
    uint64_t iodc = (uint64_t)(eph->iodc);
    int64_t deltan = (int64_t)(eph->deltan / K_P2_M43 / K_PI);
    int64_t cuc = (int64_t)(eph->cuc / K_P2_M29);
    int64_t cus = (int64_t)(eph->cus / K_P2_M29);
    int64_t cic = (int64_t)(eph->cic / K_P2_M29);
    int64_t cis = (int64_t)(eph->cis / K_P2_M29);
    int64_t crc = (int64_t)(eph->crc / K_P2_M5);
    int64_t crs = (int64_t)(eph->crs / K_P2_M5);
    uint64_t ecc = (uint64_t)(eph->ecc / K_P2_M33);
    uint64_t sqrta = (uint64_t)(eph->sqrta / K_P2_M19);
    int64_t m0 = (int64_t)(eph->m0 / K_P2_M31 / K_PI);
    int64_t omg0 = (int64_t)(eph->omg0 / K_P2_M31 / K_PI);
    int64_t inc0 = (int64_t)(eph->inc0 / K_P2_M31 / K_PI);
    int64_t aop = (int64_t)(eph->aop / K_P2_M31 / K_PI);
    int64_t omgdot = (int64_t)(eph->omgdot / K_P2_M43 / K_PI);
    int64_t idot = (int64_t)(eph->idot / K_P2_M43 / K_PI);
    int64_t af0 = (int64_t)(eph->af0 / K_P2_M31);
    int64_t af1 = (int64_t)(eph->af1 / K_P2_M43);
    int64_t af2 = (int64_t)(eph->af2 / K_P2_M55);
    int64_t tgd = (int64_t)(eph->tgd / K_P2_M31);
    uint64_t svhlth = (uint64_t)(eph->svhlth);
    uint64_t codeL2 = (uint64_t)(eph->codeL2);
    const uint64_t ura = 0, data_id = 1, sv4_p25 = 63, sv5_p25 = 51, sv4_p18 = 56;

    uint64_t wna = (uint64_t)(eph->toe.week % 256);
    uint64_t toa = (uint64_t)(eph->toe.sec / 4096.0);

    int64_t a0 = (int64_t)round(io->alpha0 / K_P2_M30);
    int64_t a1 = (int64_t)round(io->alpha1 / K_P2_M27);
    int64_t a2 = (int64_t)round(io->alpha2 / K_P2_M24);
    int64_t a3 = (int64_t)round(io->alpha3 / K_P2_M24);
    int64_t b0 = (int64_t)round(io->beta0 / 2048.0);
    int64_t b1 = (int64_t)round(io->beta1 / 16384.0);
    int64_t b2 = (int64_t)round(io->beta2 / 65536.0);
    int64_t b3 = (int64_t)round(io->beta3 / 65536.0);
    int64_t A0 = (int64_t)round(io->A0 / K_P2_M30);
    int64_t A1 = (int64_t)round(io->A1 / K_P2_M50);
    int64_t dtls = (int64_t)(io->dtls);
    uint64_t tot = (uint64_t)(io->tot / 4096);
    uint64_t wnt = (uint64_t)(io->wnt % 256);
    const uint64_t wnlsf = 1929 % 256, dn = 7;   /* scheduled leap second, gpssim.c:582-584 */
    const int64_t dtlsf = 18;

#define F(v, mask, sh) ((((uint64_t)(v)) & (mask)) << (sh))
    const uint64_t TLM = 0x8B0000ull << 6;
    uint64_t w[5][10];

    /* subframe 1: clock */
    w[0][0] = TLM;  w[0][1] = 0x1ull << 8;
    w[0][2] = F(wn, 0x3FF, 20) | F(codeL2, 0x3, 18) | F(ura, 0xF, 14) | F(svhlth, 0x3F, 8)
            | F(iodc >> 8, 0x3, 6);
    w[0][3] = 0; w[0][4] = 0; w[0][5] = 0;
    w[0][6] = F(tgd, 0xFF, 6);
    w[0][7] = F(iodc, 0xFF, 22) | F(toc, 0xFFFF, 6);
    w[0][8] = F(af2, 0xFF, 22) | F(af1, 0xFFFF, 6);
    w[0][9] = F(af0, 0x3FFFFF, 8);

    /* subframe 2: ephemeris I */
    w[1][0] = TLM;  w[1][1] = 0x2ull << 8;
    w[1][2] = F(iode, 0xFF, 22) | F(crs, 0xFFFF, 6);
    w[1][3] = F(deltan, 0xFFFF, 14) | F(m0 >> 24, 0xFF, 6);
    w[1][4] = F(m0, 0xFFFFFF, 6);
    w[1][5] = F(cuc, 0xFFFF, 14) | F(ecc >> 24, 0xFF, 6);
    w[1][6] = F(ecc, 0xFFFFFF, 6);
    w[1][7] = F(cus, 0xFFFF, 14) | F(sqrta >> 24, 0xFF, 6);
    w[1][8] = F(sqrta, 0xFFFFFF, 6);
    w[1][9] = F(toe, 0xFFFF, 14);

    /* subframe 3: ephemeris II */
    w[2][0] = TLM;  w[2][1] = 0x3ull << 8;
    w[2][2] = F(cic, 0xFFFF, 14) | F(omg0 >> 24, 0xFF, 6);
    w[2][3] = F(omg0, 0xFFFFFF, 6);
    w[2][4] = F(cis, 0xFFFF, 14) | F(inc0 >> 24, 0xFF, 6);
    w[2][5] = F(inc0, 0xFFFFFF, 6);
    w[2][6] = F(crc, 0xFFFF, 14) | F(aop >> 24, 0xFF, 6);
    w[2][7] = F(aop, 0xFFFFFF, 6);
    w[2][8] = F(omgdot, 0xFFFFFF, 6);
    w[2][9] = F(iode, 0xFF, 22) | F(idot, 0x3FFF, 8);

    /* subframe 4: page 18 (iono/UTC) when the header carried them, else page 25 */
    w[3][0] = TLM;  w[3][1] = 0x4ull << 8;
    if (io->vflg) {
        w[3][2] = (data_id << 28) | (sv4_p18 << 22) | F(a0, 0xFF, 14) | F(a1, 0xFF, 6);
        w[3][3] = F(a2, 0xFF, 22) | F(a3, 0xFF, 14) | F(b0, 0xFF, 6);
        w[3][4] = F(b1, 0xFF, 22) | F(b2, 0xFF, 14) | F(b3, 0xFF, 6);
        w[3][5] = F(A1, 0xFFFFFF, 6);
        w[3][6] = F(A0 >> 8, 0xFFFFFF, 6);
        w[3][7] = F(A0, 0xFF, 22) | F(tot, 0xFF, 14) | F(wnt, 0xFF, 6);
        w[3][8] = F(dtls, 0xFF, 22) | F(wnlsf, 0xFF, 14) | F(dn, 0xFF, 6);
        w[3][9] = F(dtlsf, 0xFF, 22);
    } else {
        w[3][2] = (data_id << 28) | (sv4_p25 << 22);
        for (int i = 3; i < 10; i++) w[3][i] = 0;
    }

    /* subframe 5: page 25 (almanac reference) */
    w[4][0] = TLM;  w[4][1] = 0x5ull << 8;
    w[4][2] = (data_id << 28) | (sv5_p25 << 22) | F(toa, 0xFF, 14) | F(wna, 0xFF, 6);
    for (int i = 3; i < 10; i++) w[4][i] = 0;
#undef F

    for (int s = 0; s < 5; s++)
        for (int i = 0; i < 10; i++)
            sbf[s][i] = (uint32_t)w[s][i];
}

/* ---- GPS parity (IS-GPS-200 eq. 20-XIV), computeChecksum gpssim.c:693-756 ---------------- */
static unsigned parity32(uint32_t v)
{
    return (unsigned)__builtin_popcount(v) & 1u;
}

uint32_t nav_parity(uint32_t source, int nib)
{
    static const uint32_t mask[6] = {0x3B1F3480u, 0x1D8F9A40u, 0x2EC7CD00u,
                                     0x1763E680u, 0x2BB1F340u, 0x0B7A89C0u};
    uint32_t d = source & 0x3FFFFFC0u;
    unsigned d29 = (source >> 31) & 1u;       /* D29* of the previous word */
    unsigned d30 = (source >> 30) & 1u;       /* D30* of the previous word */

    if (nib) {                                /* words 2 and 10: solve bits 23/24 for zero parity */
        if ((d30 + parity32(mask[4] & d)) & 1u)
            d ^= 1u << 6;
        if ((d29 + parity32(mask[5] & d)) & 1u)
            d ^= 1u << 7;
    }
    uint32_t D = d;
    if (d30)
        D ^= 0x3FFFFFC0u;
    D |= ((d29 + parity32(mask[0] & d)) & 1u) << 5;
    D |= ((d30 + parity32(mask[1] & d)) & 1u) << 4;
    D |= ((d29 + parity32(mask[2] & d)) & 1u) << 3;
    D |= ((d30 + parity32(mask[3] & d)) & 1u) << 2;
    D |= ((d30 + parity32(mask[4] & d)) & 1u) << 1;
    D |= ((d29 + parity32(mask[5] & d)) & 1u);
    return D & 0x3FFFFFFFu;
}

/* ---- generateNavMsg, gpssim.c:1467-1547 ---------------------------------------------------
 * dwrd[0..9]   : subframe 5 of the previous frame (init: rebuilt from sbf[4] with this TOW)
 * dwrd[10..59] : subframes 1..5 of the frame starting at the 30 s-aligned epoch g0        */
void nav_frame(gtime_t g, chan_t *ch, int init)
{
    gtime_t g0;
    g0.week = g.week;
    g0.sec = (double)(((unsigned long)(g.sec + 0.5)) / 30UL) * 30.0;
    ch->g0 = g0;

    uint32_t wn = (uint32_t)(g0.week % 1024);
    uint32_t tow = (uint32_t)(((unsigned long)g0.sec) / 6UL);
    uint32_t prev = 0;
    /* the frame as a source for the GPU producer (gss_nav.h): the same data words, TOW, week */
    memcpy(ch->fsrc.sbf, ch->sbf, sizeof ch->fsrc.sbf);
    ch->fsrc.tow = tow;
    ch->fsrc.wn = wn;
    ch->frame_init = init == 1;
    ch->frame_seq++;

    if (init == 1) {
        for (int i = 0; i < K_N_DWRD_SBF; i++) {
            uint32_t wd = ch->sbf[4][i];
            if (i == 1)
                wd |= (tow & 0x1FFFFu) << 13;
            wd |= (prev << 30) & 0xC0000000u;
            ch->dwrd[i] = nav_parity(wd, (i == 1) || (i == 9));
            prev = ch->dwrd[i];
        }
    } else {
        for (int i = 0; i < K_N_DWRD_SBF; i++) {
            ch->dwrd[i] = ch->dwrd[K_N_DWRD_SBF * K_N_SBF + i];
            prev = ch->dwrd[i];
        }
    }

    for (int s = 0; s < K_N_SBF; s++) {
        tow++;
        for (int i = 0; i < K_N_DWRD_SBF; i++) {
            uint32_t wd = ch->sbf[s][i];
            if (s == 0 && i == 2)
                wd |= (wn & 0x3FFu) << 20;
            if (i == 1)
                wd |= (tow & 0x1FFFFu) << 13;
            wd |= (prev << 30) & 0xC0000000u;
            uint32_t out = nav_parity(wd, (i == 1) || (i == 9));
            ch->dwrd[(s + 1) * K_N_DWRD_SBF + i] = out;
            prev = out;
        }
    }
}
