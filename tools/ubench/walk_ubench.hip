// Microbenchmark: cost of one gss_iter_bf trip on gfx950 at various waves/SIMD, with and
// without anchor-style scattered stores.  Diagnostic only (not part of the product).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../gps-sdr-sim_amd/csrc/common/gss_phase.h"

__global__ void walk_k(const double *s_in, double *out, int trips, int store_every, double *sink,
                       int nseg)
{
    int gid = blockIdx.x * blockDim.x + threadIdx.x;
    double s = s_in[gid & 1023];
    double as = s < 0 ? -s : s, rs = 1.0 / as;
    double v = 0.123456789 + 1e-3 * (gid & 63), left = 1e12;
    int nw = 0, seg = 0;
    for (int t = 0; t < trips; t++) {
        nw += gss_iter_bf(&v, s, as, rs, 1.0, &left);
        if (store_every && (t % store_every) == 0 && seg < nseg) {
            sink[(size_t)gid * nseg + seg] = v;
            seg++;
        }
    }
    out[gid] = v + nw;
}

__global__ void chain_k(double *out, int n)
{
    double a = out[threadIdx.x], b = 1.0000001;
    for (int i = 0; i < n; i++) a = a * b + 1e-9;   // dependent f64 fma chain (contracted)
    out[threadIdx.x] = a;
}

int main()
{
    const int trips = 4000;
    double *s, *out, *sink;
    hipMalloc(&s, 1024 * sizeof(double));
    double hs[1024];
    for (int i = 0; i < 1024; i++) hs[i] = (i & 1 ? -1 : 1) * (500.0 + 3.0 * i) / 2.6e6;
    hipMemcpy(s, hs, sizeof hs, hipMemcpyHostToDevice);
    hipMalloc(&out, 65536 * 64 * sizeof(double));
    const int nseg = 254;
    hipMalloc(&sink, (size_t)8192 * 64 * nseg * sizeof(double));   /* max lanes x nseg */
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float ms;
    // dependent fma chain latency, one wave
    hipLaunchKernelGGL(chain_k, 1, 64, 0, 0, out, 100000);
    hipEventRecord(e0); hipLaunchKernelGGL(chain_k, 1, 64, 0, 0, out, 1000000); hipEventRecord(e1);
    hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("dependent f64 fma chain: %.2f ns per op (1 wave)\n", ms * 1e6 / 1e6);
    {   /* the real Stage-A grid: 1126 one-wave workgroups, 3436 trips */
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(walk_k, 1126, 64, 0, 0, s, out, 3436, 0, sink, nseg);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            printf("grid 1126x64, 3436 trips: %.3f ms (%.0f cyc/trip)\n", ms, ms * 1e-3 * 2.4e9 / 3436);
            hipEventRecord(e0);
            hipLaunchKernelGGL(walk_k, 563, 128, 0, 0, s, out, 3436, 0, sink, nseg);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            printf("grid 563x128, 3436 trips: %.3f ms (%.0f cyc/trip)\n", ms, ms * 1e-3 * 2.4e9 / 3436);
        }
    }
    int waves_list[] = {256, 512, 1024, 2048};
    int st_list[] = {0};
    for (int st : st_list)
        for (int wv : waves_list) {
            hipLaunchKernelGGL(walk_k, wv, 64, 0, 0, s, out, 100, st, sink, nseg);
            hipEventRecord(e0);
            hipLaunchKernelGGL(walk_k, wv, 64, 0, 0, s, out, trips, st, sink, nseg);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            printf("waves %5d (%.1f/SIMD) stores/%2d trips: %.3f ms = %.0f ns/trip/wave-slot, %.1f cyc@2.4GHz per trip\n",
                   wv, wv / 1024.0, st, ms, ms * 1e6 / trips, ms * 1e-3 * 2.4e9 / trips);
        }
    return 0;
}
