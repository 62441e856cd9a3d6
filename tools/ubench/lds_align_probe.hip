// Probe: what ds_read_b32 returns for an LDS byte address that is not a multiple of 4 on gfx950
// (auto-aligned down to the dword, or the unaligned 4 bytes).  Decides whether the fast path may
// skip masking the two low address bits.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void probe(unsigned *out)
{
    __shared__ unsigned s[64];
    s[threadIdx.x] = 0x11111111u * (threadIdx.x & 15) + (threadIdx.x << 28);
    __syncthreads();
    unsigned a = 4 * 5 + (threadIdx.x & 3), v;
    asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    out[64 + threadIdx.x] = s[(threadIdx.x + 1) & 63];
    out[threadIdx.x] = v;
}
int main()
{
    unsigned *d, h[64];
    (void)hipMalloc(&d, 512);
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, d);
    (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    printf("word5=%08x word6=%08x | offset+0: %08x +1: %08x +2: %08x +3: %08x\n",
           0x11111111u * 5 + (5u << 28), 0x11111111u * 6 + (6u << 28), h[0], h[1], h[2], h[3]);
    return 0;
}
