// Diagnostic microbenchmark (not product code): the Stage-A code chain (gss_seg_states with
// GSS_TRIP_CODE) on realistic synthetic blocks (2.6 MS/s, 260000 samples/block, code step ~0.3935).
// Varies the number of chains to tell a serial-latency-bound walk (time independent of the count)
// from a throughput-bound one, and compares the general walk with gss_code_seg_states_bf.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../gps-sdr-sim_amd/csrc/common/gss_phase.h"

struct P { double code0, kstep; };

template <int ILP>
__global__ __launch_bounds__(64) void code_k(const P *p, int nchain, int n, int nseg, int nsegp,
                                             int seg_r, double *ox, uint32_t *oc)
{
    constexpr int L = ILP == 9 ? 1 : ILP;          /* ILP 9: the branch-free walk, one chain */
    const int i0 = (blockIdx.x * 64 + threadIdx.x) * L;
#pragma unroll
    for (int c = 0; c < L; c++) {
        const int i = i0 + c;
        if (i < nchain) {
            if (ILP == 9)
                gss_code_seg_states_bf(p[i].code0, p[i].kstep, 0u, n, nseg, seg_r, nseg,
                                       ox + (size_t)i * nsegp, oc + (size_t)i * nsegp);
            else
                gss_seg_states(GSS_TRIP_CODE, p[i].code0, p[i].kstep, 0u, 0, n, nseg, seg_r, 0,
                               ox + (size_t)i * nsegp, oc + (size_t)i * nsegp);
        }
    }
}

template <int ILP> static float run(const P *d, int nchain, int n, int nseg, int nsegp, double *ox,
                                    uint32_t *oc)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    constexpr int L = ILP == 9 ? 1 : ILP;
    int grid = (nchain + 64 * L - 1) / (64 * L);
    hipLaunchKernelGGL(code_k<ILP>, dim3(grid), dim3(64), 0, 0, d, nchain, n, nseg, nsegp, 1024, ox, oc);
    (void)hipEventRecord(a);
    for (int r = 0; r < 3; r++)
        hipLaunchKernelGGL(code_k<ILP>, dim3(grid), dim3(64), 0, 0, d, nchain, n, nseg, nsegp, 1024, ox, oc);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 3;
}

int main()
{
    const int nmax = 2999 * 12, n = 260000, nseg = 254, nsegp = 256;
    P *h = (P *)malloc(sizeof(P) * nmax);
    srand(1);
    for (int i = 0; i < nmax; i++) {
        double f = -3200.0 + 6400.0 * rand() / (double)RAND_MAX;
        h[i].code0 = 1023.0 * rand() / (RAND_MAX + 1.0);
        h[i].kstep = (1.023e6 + f / 1540.0) / 2.6e6;
    }
    P *d; double *ox; uint32_t *oc;
    (void)hipMalloc(&d, sizeof(P) * nmax);
    (void)hipMemcpy(d, h, sizeof(P) * nmax, hipMemcpyHostToDevice);
    (void)hipMalloc(&ox, sizeof(double) * nmax * nsegp);
    (void)hipMalloc(&oc, sizeof(uint32_t) * nmax * nsegp);
    for (int nc : {64, 4096, 16384, nmax})
        printf("chains %6d: general %.3f ms  branch-free %.3f ms\n", nc,
               run<1>(d, nc, n, nseg, nsegp, ox, oc), run<9>(d, nc, n, nseg, nsegp, ox, oc));
    return 0;
}
