// Where do the two waves of a 128-thread workgroup land?  md5_pair_kernel's
// shape (128 threads, ~36 KB of LDS, four workgroups per CU, a persistent
// grid of 4 x CUs) records each wave's HW_ID (SIMD, CU, shader array, SE,
// XCC) through an ordinary vector store; the host then counts, per SIMD, how
// many wave-0 (MD5) and wave-1 (loader) waves it holds at once.
//
// hipcc --offload-arch=gfx950 -O2 -o scripts/probes/simd_probe scripts/probes/simd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(128) void where(uint32_t *out, uint32_t *xcc, int spin)
{
    __shared__ uint32_t pad[36 * 256];  // 36 KB: four workgroups per CU
    pad[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
    const uint32_t xid = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID
    // keep every workgroup resident while the others start
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin)
        ;
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = blockIdx.x * 2 + (threadIdx.x >> 6);
        out[w] = hw + pad[(threadIdx.x + 1) & 127] * 0;
        xcc[w] = xid;
    }
}

int main()
{
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = 4 * ncu, nwave = 2 * grid;
    uint32_t *d = nullptr, *x = nullptr;
    if (hipMalloc(&d, nwave * 4) != hipSuccess || hipMalloc(&x, nwave * 4) != hipSuccess)
        return 1;
    where<<<grid, 128>>>(d, x, 200000);  // 2 ms at 100 MHz
    if (hipDeviceSynchronize() != hipSuccess)
        return 2;
    std::vector<uint32_t> h(nwave), hx(nwave);
    (void)hipMemcpy(h.data(), d, nwave * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hx.data(), x, nwave * 4, hipMemcpyDeviceToHost);
    // gfx9 HW_ID: wave_id [3:0], simd_id [5:4], pipe [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, std::pair<int, int>> per_simd;  // (xcc, se, sh, cu, simd)
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, int> simd_of_wave0;
    int same = 0, pairs = 0;
    for (int b = 0; b < grid; b++) {
        uint32_t s[2];
        for (int k = 0; k < 2; k++) {
            const uint32_t v = h[2 * b + k];
            const uint32_t simd = (v >> 4) & 3, cu = (v >> 8) & 15, sh = (v >> 12) & 1, se = (v >> 13) & 7;
            const auto key = std::make_tuple(hx[2 * b + k] & 15, se, sh * 16 + cu, simd);
            (k ? per_simd[key].second : per_simd[key].first)++;
            s[k] = (hx[2 * b + k] & 15) << 16 | se << 8 | (sh * 16 + cu) << 2 | simd;
        }
        pairs++;
        same += s[0] == s[1];
    }
    std::map<std::pair<int, int>, int> hist;  // (wave-0 count, wave-1 count) per SIMD -> SIMDs
    for (auto &kv : per_simd)
        hist[kv.second]++;
    printf("workgroups %d (4 per CU over %d CUs), both waves on one SIMD: %d of %d\n", grid, ncu, same, pairs);
    printf("SIMDs by (MD5-role waves, loader-role waves) held:\n");
    for (auto &kv : hist)
        printf("  (%d, %d): %d SIMDs\n", kv.first.first, kv.first.second, kv.second);
    printf("workgroups on CU (xcc 0, se 0, cu 0), all (wave: simd/wave-slot):\n");
    for (int b = 0; b < grid; b++) {
        uint32_t v0 = h[2 * b], v1 = h[2 * b + 1];
        if ((hx[2 * b] & 15) || ((v0 >> 13) & 7) || ((v0 >> 8) & 15) || ((v0 >> 12) & 1))
            continue;
        printf("  wg %d: w0 %u/%u  w1 %u/%u\n", b, (v0 >> 4) & 3, v0 & 15, (v1 >> 4) & 3, v1 & 15);
    }
    std::map<std::pair<int, int>, int> slot_simd;  // (wave index in WG, simd - simd of wave 0) histogram
    for (int b = 0; b < grid; b++)
        slot_simd[{(int)(h[2 * b] & 15), (int)(((h[2 * b + 1] >> 4) - (h[2 * b] >> 4)) & 3)}]++;
    printf("(wave-slot of wave 0, simd(w1) - simd(w0) mod 4): workgroups\n");
    for (auto &kv : slot_simd)
        printf("  (%d, %d): %d\n", kv.first.first, kv.first.second, kv.second);
    return 0;
}
