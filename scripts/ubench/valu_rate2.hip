#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k_add_vop2(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_add_lit(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a7) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_xor_vop2(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a7) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_xor_e64(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a7) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_add_e64(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a7) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_bitop3(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a0) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a1) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a2) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a3) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a4) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a5) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a6) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a7) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a0) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a1) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a2) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a3) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a4) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a5) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a6) : "v"(k)); asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_lshladd(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a0) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a1) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a2) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a3) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a4) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a5) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a6) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a7) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a0) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a1) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a2) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a3) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a4) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a5) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a6) : "v"(k)); asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_bfe(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a0) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a1) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a2) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a3) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a4) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a5) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a6) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a7) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a0) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a1) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a2) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a3) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a4) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a5) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a6) : "v"(k)); asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_add_sdwa(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a7) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a0) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a1) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a2) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a3) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a4) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a5) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a6) : "v"(k)); asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_mul24(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a7) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a0) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a1) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a2) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a3) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a4) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a5) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a6) : "v"(k)); asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_dot4(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a0) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a1) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a2) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a3) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a4) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a5) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a6) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a7) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a0) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a1) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a2) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a3) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a4) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a5) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a6) : "v"(k)); asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_perm(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, k = blockIdx.x | 0x01010101u;
    for (int i = 0; i < iters; i++) {
        asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a0) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a1) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a2) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a3) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a4) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a5) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a6) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a7) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a0) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a1) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a2) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a3) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a4) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a5) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a6) : "v"(k)); asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(a7) : "v"(k));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
int main()
{
    int ncu = 0, clk = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    uint32_t *out;
    (void)hipMalloc(&out, sizeof(uint32_t) * 4096 * 1024 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 20000;
#define RUN(K, NAME)                                                                      \
    for (int wps : {2, 4, 8}) {                                                           \
        int blocks = ncu * 4 * wps;                                                       \
        hipLaunchKernelGGL(K, dim3(blocks), dim3(64), 0, 0, out, 100);                    \
        (void)hipEventRecord(e0);                                                         \
        hipLaunchKernelGGL(K, dim3(blocks), dim3(64), 0, 0, out, iters);                  \
        (void)hipEventRecord(e1);                                                         \
        (void)hipEventSynchronize(e1);                                                    \
        float ms;                                                                         \
        (void)hipEventElapsedTime(&ms, e0, e1);                                           \
        double cyc = ms * 1e-3 * clk * 1e3 / ((double)iters * 16 * wps);                  \
        printf("%-9s waves/SIMD %d: %.2f cyc/instr/SIMD\n", NAME, wps, cyc);              \
    }
RUN(k_add_vop2, "add_vop2");
RUN(k_add_lit, "add_lit");
RUN(k_xor_vop2, "xor_vop2");
RUN(k_xor_e64, "xor_e64");
RUN(k_add_e64, "add_e64");
RUN(k_bitop3, "bitop3");
RUN(k_lshladd, "lshladd");
RUN(k_bfe, "bfe");
RUN(k_add_sdwa, "add_sdwa");
RUN(k_mul24, "mul24");
RUN(k_dot4, "dot4");
RUN(k_perm, "perm");
    return 0;
}