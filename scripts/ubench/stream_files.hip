// How fast can a wave stream 64 files at once, as a function of the
// contiguous bytes fetched per file per round?  Config-2 layout: 1M files
// of U[4 KiB, 64 KiB] packed at 16 B, waves take 64 files in descending size
// order (so a wave's files are scattered over the 34.8 GB buffer).  Each
// round a wave loads CH bytes of each of its 64 files with coalesced
// 16-byte lane loads (CH/16 lanes per file) and XORs them (no LDS).
// Mode L (per-lane): each lane reads its own file, 8 x 16 B per step.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

template <int CH>
__global__ __launch_bounds__(256) void k_coal(const uint8_t *base, const uint64_t *offs,
                                              const uint32_t *sizes, const uint32_t *order,
                                              uint32_t n, uint32_t *out)
{
    constexpr int PER = CH / 16, FPI = 64 / PER, NLD = 64 / FPI;
    const int lane = threadIdx.x & 63;
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w * 64 >= n) return;
    const int piece = lane % PER, fsub = lane / PER;
    const uint32_t myf = order[min(w * 64 + lane, n - 1)];
    const uint32_t mysz = sizes[myf];
    uint32_t mx = mysz;
    for (int o = 32; o; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    const uint64_t myoff = offs[myf];
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t r = 0; r * CH < mx; r++) {
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            const int src = k * FPI + fsub;
            const uint64_t o = __shfl(myoff, src);
            const uint32_t sz = __shfl(mysz, src);
            const uint32_t pos = r * CH + piece * 16;
            if (pos + 16 <= sz) {
                const uint4 v = *reinterpret_cast<const uint4 *>(base + o + pos);
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
        }
    }
    out[w * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}


// coal64 + a per-lane MALL/L2 warm-up: every PFR rounds each lane touches
// the 4 lines of its own file's window PFD rounds ahead (one dword per
// 128-byte line, result discarded), so DRAM sees 512-byte bursts per file.
template <int CH, int PFR, int PFD>
__global__ __launch_bounds__(256) void k_coal_pf(const uint8_t *base, const uint64_t *offs,
                                                 const uint32_t *sizes, const uint32_t *order,
                                                 uint32_t n, uint32_t *out)
{
    constexpr int PER = CH / 16, FPI = 64 / PER, NLD = 64 / FPI;
    const int lane = threadIdx.x & 63;
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w * 64 >= n) return;
    const int piece = lane % PER, fsub = lane / PER;
    const uint32_t myf = order[min(w * 64 + lane, n - 1)];
    const uint32_t mysz = sizes[myf];
    uint32_t mx = mysz;
    for (int o = 32; o; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    const uint64_t myoff = offs[myf];
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint32_t dummy = 0;
    for (uint32_t r = 0; r * CH < mx; r++) {
        if (r % PFR == 0) {
            const uint32_t wpos = (r + PFD) * CH;
#pragma unroll
            for (int q = 0; q < (PFR * CH) / 128; q++) {
                const uint32_t pos = wpos + q * 128;
                const uint8_t *a = base + myoff + (pos < mysz ? pos : 0);
                // one register, live for the whole kernel, takes every result
                asm volatile("global_load_dword %0, %1, off" : "+v"(dummy) : "v"(a) : "memory");
            }
        }
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            const int src = k * FPI + fsub;
            const uint64_t o = __shfl(myoff, src);
            const uint32_t sz = __shfl(mysz, src);
            const uint32_t pos = r * CH + piece * 16;
            if (pos + 16 <= sz) {
                const uint4 v = *reinterpret_cast<const uint4 *>(base + o + pos);
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(dummy));
    out[w * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w ^ dummy;
}

__global__ __launch_bounds__(256) void k_lane(const uint8_t *base, const uint64_t *offs,
                                              const uint32_t *sizes, const uint32_t *order,
                                              uint32_t n, uint32_t *out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t f = order[i];
    const uint4 *v = reinterpret_cast<const uint4 *>(base + offs[f]);
    const uint32_t nv = sizes[f] / 16;
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint32_t j = 0;
    for (; j + 8 <= nv; j += 8) {
        uint4 a[8];
#pragma unroll
        for (int q = 0; q < 8; q++) a[q] = v[j + q];
#pragma unroll
        for (int q = 0; q < 8; q++) { acc.x ^= a[q].x; acc.y ^= a[q].y; acc.z ^= a[q].z; acc.w ^= a[q].w; }
    }
    out[i] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// Mode glds (round 6): the 64 files' 128-byte rounds through a
// per-wave LDS ring of R slots of 8 KiB by LDS-DMA (global_load_lds_dwordx4,
// counted vmcnt waits in inline asm, no load registers): instruction q loads
// files 8q .. 8q + 7, lanes 8j + i the pieces of file 8q + j (one 128-byte
// line per 8 lanes), the piece order rotated by the file (f >> 1) so that
// the 64 lanes' ds_read_b128 of one piece index are conflict-free; each lane
// then reads its own file's 8 pieces from LDS and XORs them.
template <int R, bool NT>
__global__ __launch_bounds__(256) void k_glds(const uint8_t *base, const uint64_t *offs, const uint32_t *sizes,
                                              const uint32_t *order, uint32_t n, uint32_t *out)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t ring[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *my = ring + (size_t)wv * R * 8192;
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w * 64 >= n)
        return;
    const uint32_t myf = order[min(w * 64 + lane, n - 1)];
    const uint32_t mysz = sizes[myf];
    uint32_t mx = mysz;
    for (int o = 32; o; o >>= 1)
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    const uint64_t myoff = offs[myf];
    const int i = lane & 7, j = lane >> 3;
    uint64_t fo[8];
    uint32_t fs[8], pc[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int f = 8 * q + j;
        fo[q] = __shfl(myoff, f);
        fs[q] = __shfl(mysz, f);
        pc[q] = ((i + (f >> 1)) & 7) * 16;  // the piece this lane loads for file f
    }
    const uint32_t rounds = (mx + 127) / 128;
    auto issue = [&](uint32_t r, int slot) {
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t pos = r * 128 + pc[q];
            const uint8_t *p = base + fo[q] + (pos + 16 <= fs[q] ? pos : 0);
            const uint32_t dst = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(my + slot * 8192 + q * 1024);
            if (NT)
                asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" : : "v"(p), "{m0}"(dst) : "memory");
            else
                asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(p), "{m0}"(dst) : "memory");
        }
    };
#pragma unroll
    for (int s = 0; s < R - 1; s++)
        issue(s, s);
    uint4 acc = make_uint4(0, 0, 0, 0);
    int slot = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(r + R - 1, (slot + R - 1) % R);
        if constexpr (R == 2)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if constexpr (R == 3)
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
        const uint8_t *row = my + slot * 8192 + lane * 128;
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const uint4 x = *reinterpret_cast<const uint4 *>(row + ((v - (lane >> 1)) & 7) * 16);
            acc.x ^= x.x; acc.y ^= x.y; acc.z ^= x.z; acc.w ^= x.w;
        }
        slot = (slot + 1) % R;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[w * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main()
{
    setvbuf(stdout, NULL, _IONBF, 0);
    const uint32_t n = 1000000;
    std::vector<uint32_t> sizes(n), order(n);
    std::vector<uint64_t> offs(n);
    uint64_t x = 1, tot = 0;
    for (uint32_t i = 0; i < n; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        sizes[i] = 4096 + (uint32_t)((x >> 33) % 61441);
        offs[i] = tot;
        tot += (sizes[i] + 15) / 16 * 16;
        order[i] = i;
    }
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return sizes[a] > sizes[b]; });
    uint8_t *d_base; uint64_t *d_offs; uint32_t *d_sizes, *d_order, *d_out;
    if (hipMalloc(&d_base, tot) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(d_base, 0x5a, tot);
    (void)hipMalloc(&d_offs, n * 8); (void)hipMalloc(&d_sizes, n * 4); (void)hipMalloc(&d_order, n * 4);
    (void)hipMalloc(&d_out, n * 4 + 256);
    (void)hipMemcpy(d_offs, offs.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_sizes, sizes.data(), n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_order, order.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    printf("%u files, %.2f GB\n", n, tot / 1e9);
    auto run = [&](const char *name, auto launch) {
        launch(); (void)hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; it++) {
            (void)hipEventRecord(e0); launch(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1); best = std::min(best, ms);
        }
        printf("%-10s %.3f ms  %.0f GB/s  %s\n", name, best, tot / (best * 1e-3) / 1e9, hipGetErrorString(hipGetLastError()));
    };
    const unsigned g = (n + 255) / 256;
    run("lane", [&] { hipLaunchKernelGGL(k_lane, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("coal64", [&] { hipLaunchKernelGGL(k_coal<64>, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("coal128", [&] { hipLaunchKernelGGL(k_coal<128>, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("coal256", [&] { hipLaunchKernelGGL(k_coal<256>, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("coal512", [&] { hipLaunchKernelGGL(k_coal<512>, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("c64pf8x4", [&] { hipLaunchKernelGGL((k_coal_pf<64, 8, 8>), dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("c64pf8x16", [&] { hipLaunchKernelGGL((k_coal_pf<64, 8, 16>), dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("c64pf16x16", [&] { hipLaunchKernelGGL((k_coal_pf<64, 16, 16>), dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("c128pf8x8", [&] { hipLaunchKernelGGL((k_coal_pf<128, 8, 8>), dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("glds R2", [&] { hipLaunchKernelGGL((k_glds<2, false>), dim3(g), dim3(256), 4 * 2 * 8192, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("glds R2 nt", [&] { hipLaunchKernelGGL((k_glds<2, true>), dim3(g), dim3(256), 4 * 2 * 8192, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("glds R3 nt", [&] { hipLaunchKernelGGL((k_glds<3, true>), dim3(g), dim3(256), 4 * 3 * 8192, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("glds R4 nt", [&] { hipLaunchKernelGGL((k_glds<4, true>), dim3(g), dim3(256), 4 * 4 * 8192, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("coal1024", [&] { hipLaunchKernelGGL(k_coal<1024>, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    // identity order (a wave's 64 files adjacent in memory)
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    (void)hipMemcpy(d_order, order.data(), n * 4, hipMemcpyHostToDevice);
    run("lane-adj", [&] { hipLaunchKernelGGL(k_lane, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("coal64-adj", [&] { hipLaunchKernelGGL(k_coal<64>, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    run("coal256-adj", [&] { hipLaunchKernelGGL(k_coal<256>, dim3(g), dim3(256), 0, 0, d_base, d_offs, d_sizes, d_order, n, d_out); });
    return 0;
}
