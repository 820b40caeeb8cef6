// Microbenchmark: sig_hash_kernel's big-file ELF chain phase on data in HBM
// (config 4 --method hash: 8 files, one wave, lanes 0-7 each streaming its own
// file).  Is the chain phase held up by its loads (lookahead NS - 1 steps of
// 128 B), by the clock, or by neither?  Per run: shader cycles per byte per
// lane (s_memtime) and the clock (s_memrealtime).
//   regs   the chain on register data (no loads): chain_ubench's elfc
//   ns2    two 128-byte load sets (one step of lookahead), the shipped form
//   ns4    four sets (three steps of lookahead)
// Build: hipcc -O3 --offload-arch=gfx950 -I../../fastdfs_amd/csrc chain_mem_ubench.hip -o chain_mem_ubench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "fdfs_device.hpp"

using namespace fdfs;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Stamp {
    unsigned long long c0, c1, t0, t1;
};

constexpr uint64_t kFile = 256ull << 20;  // bytes per lane
constexpr int kLanes = 8;

template <int NS>
__global__ __launch_bounds__(64) void k_chain(const uint8_t *src, uint64_t bytes, uint32_t *out, Stamp *st)
{
    constexpr int SV = 8;
    const int lane = threadIdx.x & 63;
    const bool act = lane < kLanes;
    const uint8_t *p = src + (act ? lane : 0) * kFile;
    const uint32_t nsteps = (uint32_t)(bytes / (16 * SV));
    uint32_t e = 0, y = 0;
    u32x4 RS[NS][SV];
    auto issue = [&](u32x4 (&R)[SV], uint32_t stp) {
        const uint8_t *ln = p + (uint64_t)(stp < nsteps ? stp : 0) * 16 * SV;
#pragma unroll
        for (int q = 0; q < SV; q++)
            asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(R[q]) : "v"(ln), "i"(16 * q) : "memory");
    };
    auto wait_older = [&](u32x4 (&R)[SV]) {
        asm volatile("s_waitcnt vmcnt(%8)"
                     : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]), "+v"(R[4]), "+v"(R[5]), "+v"(R[6]), "+v"(R[7])
                     : "i"(SV * (NS - 1))
                     : "memory");
    };
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k = 0; k < NS - 1; k++)
        issue(RS[k], k);
    for (uint32_t s = 0; s < nsteps; s += NS) {
#pragma unroll
        for (int k = 0; k < NS; k++) {
            issue(RS[(k + NS - 1) % NS], s + k + NS - 1);
            wait_older(RS[k]);
#pragma unroll
            for (int q = 0; q < SV; q++) {
                elf_word4_chain<true, false>(RS[k][q][0], e);
                elf_word4_chain<true, false>(RS[k][q][1], e);
                elf_word4_chain<true, false>(RS[k][q][2], e);
                elf_word4_chain_y<true>(RS[k][q][3], e, y);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NS; k++)
        asm volatile("s_waitcnt vmcnt(0)"
                     : "+v"(RS[k][0]), "+v"(RS[k][1]), "+v"(RS[k][2]), "+v"(RS[k][3]), "+v"(RS[k][4]), "+v"(RS[k][5]),
                       "+v"(RS[k][6]), "+v"(RS[k][7])::"memory");
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + lane] = e ^ y;
    if (lane == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

__global__ void k_regs(const uint8_t *, uint64_t bytes, uint32_t *out, Stamp *st)
{
    uint32_t e = threadIdx.x, y = 0;
    uint32_t w0 = threadIdx.x * 0x9E3779B9u, w1 = w0 ^ 0x85EBCA6Bu, w2 = w0 + 0xC2B2AE35u, w3 = ~w0;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (uint64_t i = 0; i < bytes / 16; i++) {
        elf_word4_chain<true, false>(w0, e);
        elf_word4_chain<true, false>(w1, e);
        elf_word4_chain<true, false>(w2, e);
        elf_word4_chain_y<true>(w3, e, y);
        w0 += e;
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = e ^ y;
    if (threadIdx.x == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

int main()
{
    uint8_t *src;
    uint32_t *out;
    Stamp *st, hst;
    hipMalloc(&src, kFile * kLanes);
    hipMemset(src, 0x5A, kFile * kLanes);
    hipMalloc(&out, 64 * sizeof(uint32_t));
    hipMalloc(&st, sizeof(Stamp));
    const uint64_t bytes = 64ull << 20;  // per lane per run
    printf("{\"runs\": [\n");
    bool first = true;
    for (const char *name : {"regs", "ns2", "ns4", "ns2", "regs"}) {
        for (int rep = 0; rep < 2; rep++) {
            if (name[0] == 'r')
                hipLaunchKernelGGL(k_regs, dim3(1), dim3(64), 0, 0, src, bytes, out, st);
            else if (name[2] == '2')
                hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, src, bytes, out, st);
            else
                hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), 0, 0, src, bytes, out, st);
            const hipError_t err = hipDeviceSynchronize();
            if (err != hipSuccess) {  // stop at the first failure: nothing more runs on the GPU
                printf("\n]}\nerror %s in %s\n", hipGetErrorString(err), name);
                return 2;
            }
        }
        hipMemcpy(&hst, st, sizeof(Stamp), hipMemcpyDeviceToHost);
        const double cyc = (double)(hst.c1 - hst.c0), ns = (double)(hst.t1 - hst.t0) * 10.0;
        printf("%s{\"kernel\": \"%s\", \"cycles_per_byte_lane\": %.4f, \"clock_ghz\": %.3f, \"mb_per_s_lane\": %.1f}",
               first ? "" : ",\n", name, cyc / bytes, cyc / ns, bytes / ns * 1e3);
        first = false;
    }
    printf("\n]}\n");
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
