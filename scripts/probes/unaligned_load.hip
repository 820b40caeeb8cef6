// Probe: do 16-byte global loads at byte-misaligned addresses return the
// bytes at that address on gfx950 (ROCm's default memory alignment mode)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(const uint8_t *buf, uint4 *out, uint4 *ref)
{
    const int t = threadIdx.x;                 // byte offset 0..63
    const uint8_t *p = buf + 1000 + t;
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    out[t] = v;
    uint32_t w[4];
    for (int d = 0; d < 4; d++)
        w[d] = p[4 * d] | (p[4 * d + 1] << 8) | (p[4 * d + 2] << 16) | ((uint32_t)p[4 * d + 3] << 24);
    ref[t] = make_uint4(w[0], w[1], w[2], w[3]);
}

int main()
{
    uint8_t h[4096];
    for (int i = 0; i < 4096; i++) h[i] = (uint8_t)(i * 131 + 7);
    uint8_t *d; uint4 *o, *r;
    hipMalloc(&d, 4096); hipMalloc(&o, 64 * 16); hipMalloc(&r, 64 * 16);
    hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    k<<<1, 64>>>(d, o, r);
    hipError_t e = hipDeviceSynchronize();
    uint4 ho[64], hr[64];
    hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
    hipMemcpy(hr, r, sizeof hr, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < 64; t++)
        if (ho[t].x != hr[t].x || ho[t].y != hr[t].y || ho[t].z != hr[t].z || ho[t].w != hr[t].w) {
            if (bad < 4) printf("offset %d: got %08x %08x want %08x %08x\n", t, ho[t].x, ho[t].y, hr[t].x, hr[t].y);
            bad++;
        }
    printf("sync=%s mismatches=%d of 64\n", hipGetErrorString(e), bad);
    return bad ? 1 : 0;
}
