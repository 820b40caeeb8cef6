// Microbenchmark: the dependent-chain cost of the two
// byte-serial signature recurrences on one gfx950 lane, with the library's
// own device code and the data in registers (no memory traffic):
//   md5   one my_md5 block (fdfs_md5.hpp md5_compress: 64 dependent steps)
//   elf4  ELFHash_ex, the asm 4-VALU-per-byte form of sig_hash_kernel's steps
//   elfc  ELFHash_ex, the 3-op chain form of its big-file lanes
// at W = 1..4 waves per SIMD.  Cycles come from s_memtime (the shader clock)
// and time from s_memrealtime (100 MHz), so each line carries the clock the
// SIMDs actually ran at.  Per lane: cycles per block / byte (the chain's
// latency at W = 1); per SIMD: bytes per cycle (its throughput at W).
// Build: hipcc -O3 --offload-arch=gfx950 -I../../fastdfs_amd/csrc chain_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "fdfs_device.hpp"
#include "fdfs_md5.hpp"

using namespace fdfs;

struct Stamp {
    unsigned long long c0, c1, t0, t1;
};

__global__ void k_md5(int iters, uint32_t *out, Stamp *st)
{
    uint32_t s[4] = {0x67452301u ^ threadIdx.x, 0xefcdab89u, 0x98badcfeu, 0x10325476u ^ blockIdx.x};
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        m[k] = (threadIdx.x * 0x9E3779B9u) ^ (k * 0x85EBCA6Bu) ^ blockIdx.x;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        md5_compress(s, m);
        m[i & 15] ^= s[0];  // keeps the blocks distinct without lengthening the chain
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
    if (threadIdx.x == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

template <bool CHAIN>
__global__ void k_elf(int iters, uint32_t *out, Stamp *st)
{
    uint32_t e = threadIdx.x, y = 0;
    uint32_t w0 = threadIdx.x * 0x9E3779B9u, w1 = w0 ^ 0x85EBCA6Bu, w2 = w0 + 0xC2B2AE35u, w3 = ~w0;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {  // 16 bytes per iteration
        if (CHAIN) {
            elf_word4_chain<true, false>(w0, e);
            elf_word4_chain<true, false>(w1, e);
            elf_word4_chain<true, false>(w2, e);
            elf_word4_chain_y<true>(w3, e, y);
        } else {
            elf_vec16y<true>(make_uint4(w0, w1, w2, w3), e, y);
        }
        w0 += e;  // data that depends on the chain: nothing hoists
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = e ^ y;
    if (threadIdx.x == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    Stamp *st, *hst;
    const int maxb = ncu * 4 * 4;
    hipMalloc(&out, sizeof(uint32_t) * 64 * maxb);
    hipMalloc(&st, sizeof(Stamp) * maxb);
    hst = new Stamp[maxb];
    printf("{\"cus\": %d, \"runs\": [\n", ncu);
    bool first = true;
    for (const char *name : {"md5", "elf4", "elfc"}) {
        const bool md5 = name[0] == 'm';
        const int iters = md5 ? 4000 : 40000;
        const double bytes_per_iter = md5 ? 64.0 : 16.0;
        for (int w = 1; w <= 4; w++) {
            const int blocks = ncu * 4 * w;  // 64-thread blocks, dealt round-robin: w waves per SIMD
            for (int rep = 0; rep < 2; rep++) {  // the first launch warms up
                if (md5)
                    hipLaunchKernelGGL(k_md5, dim3(blocks), dim3(64), 0, 0, iters, out, st);
                else if (name[3] == 'c')
                    hipLaunchKernelGGL(k_elf<true>, dim3(blocks), dim3(64), 0, 0, iters, out, st);
                else
                    hipLaunchKernelGGL(k_elf<false>, dim3(blocks), dim3(64), 0, 0, iters, out, st);
                hipDeviceSynchronize();
            }
            hipMemcpy(hst, st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost);
            double cyc = 0, ns = 0;
            for (int b = 0; b < blocks; b++) {
                cyc += (double)(hst[b].c1 - hst[b].c0);
                ns += (double)(hst[b].t1 - hst[b].t0) * 10.0;  // 100 MHz
            }
            cyc /= blocks;
            ns /= blocks;
            const double per_lane = cyc / (iters * bytes_per_iter);  // cycles per byte on one lane
            printf("%s{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_byte_lane\": %.4f, "
                   "\"cycles_per_step_lane\": %.2f, \"bytes_per_step\": %d, \"simd_bytes_per_cycle\": %.3f, "
                   "\"clock_ghz\": %.3f}",
                   first ? "" : ",\n", name, w, per_lane, cyc / iters, (int)bytes_per_iter, 64.0 * w / per_lane,
                   cyc / ns);
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
