// Pure HBM read rate on one MI355X (calibration for crc_seg_kernel, DESIGN
// 4.1): 8 GiB read once per launch, every 16-byte vector XOR-folded (one
// result word per thread, so no load is dead), timed with HIP events over
// 5 launches after 2 warm-ups.  Variants:
//   grid  : B blocks x T threads, grid-stride over 4 KiB blocks of the
//           buffer, each wave reading U blocks ahead (U x 4 loads of 16 B
//           per lane in flight);
//   nt    : the same loads non-temporal;
//   glds  : global_load_lds_dwordx4 into a per-wave LDS ring of R slots of
//           SLOT bytes (lane-linear), folded from LDS after a counted vmcnt
//           (inline asm, so R - 1 slots stay in flight).
// hipcc --offload-arch=gfx950 -O3 read_bw.hip -o read_bw && ./read_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(512) void k_reg(const uint4 *__restrict__ v, uint64_t nblk, uint32_t *out)
{
    const int lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint32_t acc = 0;
    // wave w owns a contiguous range of 4 KiB blocks (like crc_seg_kernel's segments)
    const uint64_t b0 = nblk * w / nw, b1 = nblk * (w + 1) / nw;
    for (uint64_t b = b0; b < b1; b += U) {
        uint4 r[U][4];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint64_t bb = b + u < b1 ? b + u : b1 - 1;
                const uint4 *p = v + bb * 256 + 4 * lane + q;
                if constexpr (NT) {
                    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                    const v4 t = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p));
                    r[u][q] = make_uint4(t.x, t.y, t.z, t.w);
                } else {
                    r[u][q] = *p;
                }
            }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                acc ^= r[u][q].x ^ r[u][q].y ^ r[u][q].z ^ r[u][q].w;
    }
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// glds: each wave streams its range through an R-slot ring of SLOT bytes in LDS
template <int R, int AUX, int SLOT = 4096>
__global__ __launch_bounds__(1024) void k_glds(const uint4 *__restrict__ v, uint64_t nblk, uint32_t *out)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t ring[];
    constexpr int NI = SLOT / 1024;  // glds instructions per slot
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *my = ring + (size_t)wv * R * SLOT;
    const uint64_t nsl = nblk * (4096 / SLOT);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t b0 = nsl * w / nw, b1 = nsl * (w + 1) / nw;
    uint32_t acc = 0;
    // inline asm: with __builtin_amdgcn_global_load_lds hipcc waits for
    // every outstanding LDS-DMA load before each LDS read (vmcnt(0)), which
    // leaves one slot in flight whatever R is
    auto issue = [&](uint64_t b, int slot) {
        const uint64_t bb = b < b1 ? b : b1 - 1;
#pragma unroll
        for (int q = 0; q < NI; q++) {
            const uint4 *p = v + bb * (SLOT / 16) + q * 64 + lane;
            const uint32_t dst = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(my + slot * SLOT + q * 1024);
            if (AUX)
                asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" : : "v"(p), "{m0}"(dst) : "memory");
            else
                asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(p), "{m0}"(dst) : "memory");
        }
    };
#pragma unroll
    for (int s = 0; s < R - 1; s++)
        issue(b0 + s, s);
    int slot = 0;
    for (uint64_t b = b0; b < b1; b++) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's last reads are done
        issue(b + R - 1, (slot + R - 1) % R);
        // the oldest of R slots in flight has landed once (R - 1) * NI remain
        if constexpr ((R - 1) * NI == 4)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if constexpr ((R - 1) * NI == 8)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if constexpr ((R - 1) * NI == 12)
            asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else if constexpr ((R - 1) * NI == 2)
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if constexpr ((R - 1) * NI == 6)
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint4 *s = reinterpret_cast<const uint4 *>(my + slot * SLOT);
#pragma unroll
        for (int q = 0; q < NI; q++) {
            const uint4 x = s[q * 64 + lane];
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
        }
        slot = (slot + 1) % R;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename F>
static float timeit(F f)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    f();
    hipEventRecord(a);
    for (int i = 0; i < 5; i++)
        f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main()
{
    const uint64_t bytes = 8ull << 30, nblk = bytes / 4096;
    uint4 *v;
    uint32_t *out;
    CK(hipMalloc(&v, bytes));
    CK(hipMemset(v, 1, bytes));
    CK(hipMalloc(&out, 64 << 20));
    int ncu = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess)
        ncu = p.multiProcessorCount;
    auto rep = [&](const char *name, float ms) { printf("%-36s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9); };
    char nm[128];
    for (int bpc : {2, 4, 8})
        for (int T : {256, 512}) {
            const int grid = ncu * bpc * 512 / T;
            snprintf(nm, sizeof nm, "reg U1 T%d blk/CU %d", T, grid / ncu);
            rep(nm, timeit([&] { k_reg<1, false><<<grid, T>>>(v, nblk, out); }));
            snprintf(nm, sizeof nm, "reg U2 T%d blk/CU %d", T, grid / ncu);
            rep(nm, timeit([&] { k_reg<2, false><<<grid, T>>>(v, nblk, out); }));
            snprintf(nm, sizeof nm, "reg U4 T%d blk/CU %d", T, grid / ncu);
            rep(nm, timeit([&] { k_reg<4, false><<<grid, T>>>(v, nblk, out); }));
            snprintf(nm, sizeof nm, "reg U2 nt T%d blk/CU %d", T, grid / ncu);
            rep(nm, timeit([&] { k_reg<2, true><<<grid, T>>>(v, nblk, out); }));
        }
    // G workgroups per CU sharing W waves (each its ring in dynamic LDS), slots of S
    auto glds = [&](const char *tag, int waves, int G, int R, int S, int aux, auto kern) {
        const size_t lds = (size_t)(waves / G) * R * S;
        snprintf(nm, sizeof nm, "glds %s %2d waves/CU in %d WG R%d x %d B (%zu KB/WG)", tag, waves, G, R, S, lds >> 10);
        rep(nm, timeit([&] { kern<<<ncu * G, 64 * (waves / G), lds>>>(v, nblk, out); }));
    };
    glds("nt", 8, 1, 2, 4096, 2, k_glds<2, 2, 4096>);
    glds("nt", 8, 1, 3, 4096, 2, k_glds<3, 2, 4096>);
    glds("nt", 8, 1, 4, 4096, 2, k_glds<4, 2, 4096>);
    glds("nt", 8, 2, 2, 4096, 2, k_glds<2, 2, 4096>);
    glds("nt", 8, 2, 3, 4096, 2, k_glds<3, 2, 4096>);
    glds("nt", 8, 2, 4, 4096, 2, k_glds<4, 2, 4096>);
    glds("nt", 12, 1, 2, 4096, 2, k_glds<2, 2, 4096>);
    glds("nt", 12, 1, 3, 4096, 2, k_glds<3, 2, 4096>);
    glds("nt", 16, 2, 2, 4096, 2, k_glds<2, 2, 4096>);
    glds("nt", 16, 4, 2, 4096, 2, k_glds<2, 2, 4096>);
    glds("nt", 4, 1, 4, 4096, 2, k_glds<4, 2, 4096>);
    glds("def", 8, 1, 3, 4096, 0, k_glds<3, 0, 4096>);
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
