/* fake_dev.cpp's block fingerprint, shared with the harness (test infrastructure only) */
#ifndef FAKE_DEV_H
#define FAKE_DEV_H
#include <stdint.h>
#include <string.h>
#include "gpssim_amd.h"
#ifdef __cplusplus
extern "C" {
#endif
struct gss_dev;
struct gss_dev *fake_dev_open(void);
void fake_dev_close(struct gss_dev *d);

static inline uint64_t fake_mix(uint64_t h, uint64_t v)
{
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 29);
}

/* what a block's render reads: its channel rows and their nav rows' words; 1 if a row points
   outside the nav table */
static inline int fake_block_print(const gss_chan_blk_t *p, int nch, const uint32_t *nav,
                                   int n_nav, uint64_t *out)
{
    uint64_t h = fake_mix(0, (uint64_t)nch);
    for (int k = 0; k < nch; k++, p++) {
        uint64_t v[4];
        memcpy(&v[0], &p->carr0, 8);
        memcpy(&v[1], &p->carr_step, 8);
        memcpy(&v[2], &p->code0, 8);
        memcpy(&v[3], &p->code_step, 8);
        for (int i = 0; i < 4; i++)
            h = fake_mix(h, v[i]);
        h = fake_mix(h, ((uint64_t)(uint32_t)p->icode << 32) | (uint32_t)p->ibit);
        h = fake_mix(h, ((uint64_t)(uint32_t)p->iword << 32) | (uint32_t)p->gain);
        h = fake_mix(h, (uint64_t)(uint32_t)p->ca_tbl);
        if (p->nav_tbl < 0 || p->nav_tbl >= n_nav)
            return 1;
        for (int w = 0; w < GSS_NAV_WORDS; w++)
            h = fake_mix(h, nav[(size_t)p->nav_tbl * GSS_NAV_WORDS + w]);
    }
    *out = h;
    return 0;
}

static inline void fake_fill(uint8_t *o, size_t n, uint64_t h)
{
    for (size_t i = 0; i < n; i++)
        o[i] = (uint8_t)(h >> (8 * (i & 7)));
}
#ifdef __cplusplus
}
#endif
#endif
