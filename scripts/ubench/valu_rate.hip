// Microbenchmark: issue rate (8 independent chains per lane, many waves) and
// dependent latency (1 chain, 1 wave per SIMD) of the integer VALU ops the
// signature kernels use, on gfx950.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define OPS(X) X(dot4, "v_dot4_u32_u8 %0, %0, %1, %0") \
               X(bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96") \
               X(perm, "v_perm_b32 %0, %0, %1, %0") \
               X(lshladd, "v_lshl_add_u32 %0, %0, 4, %1") \
               X(add3, "v_add3_u32 %0, %0, %1, %0") \
               X(mullo, "v_mul_lo_u32 %0, %0, %1") \
               X(alignbit, "v_alignbit_b32 %0, %0, %1, 7") \
               X(add, "v_add_u32 %0, %0, %1") \
               X(ashr, "v_ashrrev_i32 %0, 3, %0")

#define KDEF(name, ins)                                                          \
__global__ void k_##name(uint32_t *out, int iters, int chains)                   \
{                                                                                \
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u; \
    if (chains == 8) {                                                           \
        for (int i = 0; i < iters; i++) {                                        \
            asm volatile(ins : "+v"(a0) : "v"(k)); asm volatile(ins : "+v"(a1) : "v"(k)); \
            asm volatile(ins : "+v"(a2) : "v"(k)); asm volatile(ins : "+v"(a3) : "v"(k)); \
            asm volatile(ins : "+v"(a4) : "v"(k)); asm volatile(ins : "+v"(a5) : "v"(k)); \
            asm volatile(ins : "+v"(a6) : "v"(k)); asm volatile(ins : "+v"(a7) : "v"(k)); \
        }                                                                        \
    } else {                                                                     \
        for (int i = 0; i < iters; i++) {                                        \
            asm volatile(ins : "+v"(a0) : "v"(k)); asm volatile(ins : "+v"(a0) : "v"(k)); \
            asm volatile(ins : "+v"(a0) : "v"(k)); asm volatile(ins : "+v"(a0) : "v"(k)); \
            asm volatile(ins : "+v"(a0) : "v"(k)); asm volatile(ins : "+v"(a0) : "v"(k)); \
            asm volatile(ins : "+v"(a0) : "v"(k)); asm volatile(ins : "+v"(a0) : "v"(k)); \
        }                                                                        \
    }                                                                            \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
}
OPS(KDEF)

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    uint32_t *out;
    hipMalloc(&out, sizeof(uint32_t) * 4096 * 1024 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    printf("CUs %d, clock %d kHz; cycles at that clock per wave-instruction per SIMD\n", ncu, clk);
#define RUN(name, ins)                                                                         \
    for (int wps : {1, 2, 4, 8}) {                                                             \
        for (int ch : {1, 8}) {                                                                \
            int blocks = ncu * 4 * wps; /* 64-thread blocks: wps waves per SIMD */               \
            hipLaunchKernelGGL(k_##name, dim3(blocks), dim3(64), 0, 0, out, 100, ch);          \
            hipEventRecord(e0);                                                                \
            hipLaunchKernelGGL(k_##name, dim3(blocks), dim3(64), 0, 0, out, iters, ch);        \
            hipEventRecord(e1);                                                                \
            hipEventSynchronize(e1);                                                           \
            float ms;                                                                          \
            hipEventElapsedTime(&ms, e0, e1);                                                  \
            double instr_per_simd = (double)iters * 8 * wps;                                   \
            double cyc = ms * 1e-3 * clk * 1e3 / instr_per_simd;                               \
            printf("%-9s waves/SIMD %d chains %d: %.2f cyc/instr/SIMD, %.2f cyc/instr/wave\n", \
                   #name, wps, ch, cyc, cyc * wps);                                            \
        }                                                                                      \
    }
    OPS(RUN)
    return 0;
}
