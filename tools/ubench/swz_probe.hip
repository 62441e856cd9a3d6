// Probe: a swizzled buffer resource (SWIZZLE_EN, ADD_TID_ENABLE, INDEX_STRIDE 64, ELEMENT_SIZE 4)
// so that one buffer_store_dwordx4 writes dword d of lane l at base + off*64 + d*256 + l*4, i.e.
// four consecutive 64-sample steps of the fast path's lane-per-sample layout in one instruction.
// The buffer is bounds-checked (num_records), so a wrong descriptor drops writes, never strays.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_swz(uint32_t *buf, uint32_t nbytes, uint32_t w3, uint32_t sdiv)
{
    const uint64_t base = (uint64_t)buf;
    v4i rs;
    rs.x = (int)(uint32_t)base;
    rs.y = (int)((uint32_t)(base >> 32) & 0xFFFFu) | (int)(1u << 31);   /* SWIZZLE_EN, stride 0 */
    rs.z = (int)nbytes;                                                    /* num_records */
    rs.w = (int)w3;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    v4i d0 = {(int)(0x1000u * wave + 0 * 64 + lane), (int)(0x1000u * wave + 1 * 64 + lane),
              (int)(0x1000u * wave + 2 * 64 + lane), (int)(0x1000u * wave + 3 * 64 + lane)};
    v4i d1 = {(int)(0x1000u * wave + 4 * 64 + lane), (int)(0x1000u * wave + 5 * 64 + lane),
              (int)(0x1000u * wave + 6 * 64 + lane), (int)(0x1000u * wave + 7 * 64 + lane)};
    /* soffset = the wave's 2 KB (8 steps x 256 B); offsets within it 0 and 16 (x64 = 1 KB) */
    const uint32_t soff = wave * 2048u / sdiv;   /* 1: soffset added after the swizzle */
    asm volatile("buffer_store_dwordx4 %0, off, %1, %2 offset:0 nt\n"
                 "buffer_store_dwordx4 %3, off, %1, %2 offset:16 nt"
                 : : "v"(d0), "s"(rs), "s"(soff), "v"(d1) : "memory");
}

int main()
{
    const int waves = 4, nbytes = waves * 2048;
    uint32_t *d;
    hipMalloc(&d, nbytes + 4096);
    uint32_t h[(nbytes + 4096) / 4];
    /* word3 candidates: DATA_FORMAT 32 (4 << 15), ELEMENT_SIZE 4 B (1 << 19), INDEX_STRIDE 64
       (3 << 21), ADD_TID_ENABLE (1 << 23) */
    const uint32_t w3s[] = {(4u << 15) | (1u << 19) | (3u << 21) | (1u << 23)};
    for (uint32_t sdiv : {1u, 64u})
    for (uint32_t w3 : w3s) {
        hipMemset(d, 0xFF, nbytes + 4096);
        hipLaunchKernelGGL(k_swz, 1, 64 * waves, 0, 0, d, (uint32_t)nbytes, w3, sdiv);
        hipError_t e = hipDeviceSynchronize();
        hipMemcpy(h, d, nbytes + 4096, hipMemcpyDeviceToHost);
        int ok = 0, bad = 0, first_bad = -1;
        for (int i = 0; i < nbytes / 4; i++) {
            const uint32_t want = 0x1000u * (i / 512) + (i % 512);   /* wave, step*64 + lane */
            if (h[i] == want) ok++; else { bad++; if (first_bad < 0) first_bad = i; }
        }
        int beyond = 0;
        for (int i = nbytes / 4; i < (nbytes + 4096) / 4; i++) beyond += h[i] != 0xFFFFFFFFu;
        printf("sdiv %u w3 %08x: err %s ok %d bad %d first_bad %d (got %08x) beyond %d\n", sdiv, w3,
               hipGetErrorString(e), ok, bad, first_bad, first_bad >= 0 ? h[first_bad] : 0, beyond);
        for (int i = 0; i < 8; i++) printf("%08x ", h[i]);
        printf("\n");
    }
    return 0;
}
