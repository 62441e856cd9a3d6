// Diagnostic microbenchmark (not product code): Stage-A anchor walk variants on realistic
// synthetic chains (2999 blocks x 12 channels, |f| up to 3.2 kHz at 2.6 MS/s, code step ~0.3935).
//   MODE 0: trips only (no emission)            MODE 1: emission decisions, anchors to LDS only
//   MODE 2: emission with direct global stores  (ONE=1: one chain kind per wave, else both/lane)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include "../../gps-sdr-sim_amd/csrc/common/gss_phase.h"

struct P { double carr0, cstep, code0, kstep; };

template <int MODE, bool CODE>
__device__ __forceinline__ void trip_emit(double &v, double &left, double st, double as, double rs,
        double W, int exW, double total, int &seg, int32_t &an, double &ax, int nseg, int seg_r,
        int32_t *an_out, double *ax_out, size_t row, double *lds, int lane)
{
    const int wr = gss_iter_bf(&v, st, as, rs, W, exW, &left);
    if (MODE == 0) { seg += wr; return; }
    const int32_t pos = (int32_t)(total - left);
    const bool fin = seg < nseg && seg * seg_r <= pos;
    const bool use_new = wr && seg * seg_r >= pos;
    if (fin) {
        if (MODE == 2) {
            an_out[row + seg] = use_new ? pos : an;
            ax_out[row + seg] = use_new ? v : ax;
        } else {
            lds[lane * 17 + (seg & 15)] = use_new ? v : ax;
        }
    }
    seg += fin ? 1 : 0;
    an = wr ? pos : an;
    ax = wr ? v : ax;
}

template <int MODE, bool ONE>
__global__ __launch_bounds__(64) void anc_k(const P *p, int npairs, int nseg, int seg_r, double total,
                                            int32_t *an_out, double *ax_out, double *sink)
{
    __shared__ double lds[64 * 17 * 2];
    const int lane = threadIdx.x;
    int pair, chain;
    if (ONE) { chain = blockIdx.x & 1; pair = (blockIdx.x >> 1) * 64 + lane; }
    else { chain = 2; pair = blockIdx.x * 64 + lane; }
    if (pair >= npairs) return;
    const P q = p[pair];
    double vc = q.carr0, lc = total, axc = vc; int segc = 0; int32_t anc = 0;
    double vk = q.code0, lk = total, axk = vk; int segk = 0; int32_t ank = 0;
    const double cas = fabs(q.cstep), crs = 1.0 / cas, kas = q.kstep, krs = 1.0 / kas;
    const size_t rowc = (size_t)pair * 2 * nseg, rowk = rowc + nseg;
    if (chain == 0 || chain == 2) {
        if (chain == 2) {
            while (lc > 0.0 || lk > 0.0) {
                trip_emit<MODE, false>(vc, lc, q.cstep, cas, crs, 1.0, 0, total, segc, anc, axc, nseg,
                                       seg_r, an_out, ax_out, rowc, lds, lane);
                trip_emit<MODE, true>(vk, lk, q.kstep, kas, krs, 1023.0, 10, total, segk, ank, axk, nseg,
                                      seg_r, an_out, ax_out, rowk, lds + 64 * 17, lane);
            }
        } else {
            while (lc > 0.0)
                trip_emit<MODE, false>(vc, lc, q.cstep, cas, crs, 1.0, 0, total, segc, anc, axc, nseg,
                                       seg_r, an_out, ax_out, rowc, lds, lane);
        }
    } else {
        while (lk > 0.0)
            trip_emit<MODE, true>(vk, lk, q.kstep, kas, krs, 1023.0, 10, total, segk, ank, axk, nseg,
                                  seg_r, an_out, ax_out, rowk, lds, lane);
    }
    sink[pair] = vc + vk + segc + segk + lds[lane];
}

template <int MODE, bool ONE>
static float run(const P *d, int npairs, int nseg, int32_t *an, double *ax, double *sink)
{
    int grid = ONE ? 2 * ((npairs + 63) / 64) : (npairs + 63) / 64;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((anc_k<MODE, ONE>), grid, 64, 0, 0, d, npairs, nseg, 1024, 260000.0, an, ax, sink);
    hipEventRecord(e0);
    hipLaunchKernelGGL((anc_k<MODE, ONE>), grid, 64, 0, 0, d, npairs, nseg, 1024, 260000.0, an, ax, sink);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main()
{
    const int nblk = 2999, nch = 12, npairs = nblk * nch, nseg = 254;
    P *h = (P *)malloc(sizeof(P) * npairs);
    srand(1);
    double fch[12];
    for (int k = 0; k < nch; k++) fch[k] = -3200.0 + 6400.0 * (k + 0.5) / nch;   /* spread dopplers */
    for (int i = 0; i < npairs; i++) {
        int k = i % nch;
        double f = fch[k] + (rand() / (double)RAND_MAX - 0.5) * 10.0;
        h[i].carr0 = rand() / (RAND_MAX + 1.0);
        h[i].cstep = f / 2.6e6;
        h[i].code0 = 1023.0 * rand() / (RAND_MAX + 1.0);
        h[i].kstep = (1.023e6 + f / 1540.0) / 2.6e6;
    }
    P *d; int32_t *an; double *ax, *sink;
    (void)hipMalloc(&d, sizeof(P) * npairs);
    (void)hipMemcpy(d, h, sizeof(P) * npairs, hipMemcpyHostToDevice);
    (void)hipMalloc(&an, sizeof(int32_t) * npairs * 2 * nseg);
    (void)hipMalloc(&ax, sizeof(double) * npairs * 2 * nseg);
    (void)hipMalloc(&sink, sizeof(double) * npairs);
    printf("one-chain-per-wave: trips only %.3f ms | lds %.3f ms | global %.3f ms\n",
           run<0, true>(d, npairs, nseg, an, ax, sink), run<1, true>(d, npairs, nseg, an, ax, sink),
           run<2, true>(d, npairs, nseg, an, ax, sink));
    printf("both-chains-per-lane: trips only %.3f ms | lds %.3f ms | global %.3f ms\n",
           run<0, false>(d, npairs, nseg, an, ax, sink), run<1, false>(d, npairs, nseg, an, ax, sink),
           run<2, false>(d, npairs, nseg, an, ax, sink));
    return 0;
}
