/*
 * synth_oracle.h — TEST INFRASTRUCTURE ONLY (never linked into the product).
 * Scalar CPU restatement of the reference sample loop and quantise/pack epilogue
 * (gpssim.c:2190-2288), driven by the same per-block parameters as gss_synth_*.
 */
#ifndef SYNTH_ORACLE_H
#define SYNTH_ORACLE_H
#include <stdint.h>
#include "../include/gpssim_amd.h"
#ifdef __cplusplus
extern "C" {
#endif
/* out: nblk*gss block bytes; carr_end optional [nblk][16]; returns 0, or GSS_E_RANGE if a
   nav-word index ran past 59 (the reference reads out of bounds there). */
int oracle_synth(const gss_chan_blk_t *blk, const int32_t *nch, const uint32_t *ca_bits,
                 const uint32_t *nav, int nblk, int n_per_blk, int fmt, void *out,
                 double *carr_end);
size_t oracle_block_bytes(int n_per_blk, int fmt);
double oracle_carr_brute(double x, double s, int64_t n);
void oracle_carr_trace(double x, double s, const int64_t *at, int m, double *out);
double oracle_code_brute(double c, double s, int64_t n, int32_t *icode, int32_t *ibit,
                         int32_t *iword);
void oracle_lut(int *sin512, int *cos512);
#ifdef __cplusplus
}
#endif
#endif
