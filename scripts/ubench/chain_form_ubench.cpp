// Microbenchmark: the library's two single-chain forms on the same MD5 chains
// (fdfs_md5.hip, included whole): md5_chain_wg (a workgroup per file, the
// chain wave beside a helper wave that makes the K + m sums) and
// md5_chain_wave (a wave per file feeding its own LDS ring), with 1, 2 or 4
// chain waves per workgroup.  One file of 8 MiB per chain, as many chains
// as CUs; time per launch from HIP events (the same for every chain), so
// the per-chain rate is bytes / time.  Which placement makes the self-fed
// wave slower than the helper form in the product (profiles/r06/chain_wave_ab.txt)?
// Build: hipcc -O3 --offload-arch=gfx950 -x hip -I../../fastdfs_amd/csrc chain_form_ubench.cpp -o chain_form_ubench
#include "../../fastdfs_amd/csrc/fdfs_md5.hip"

#include <cstdio>
#include <cstdlib>

using namespace fdfs;

constexpr uint64_t kFileBytes = 8ull << 20;

__global__ __launch_bounds__(128) void k_wg(const uint8_t *src, uint8_t *sig)
{
    __shared__ __attribute__((aligned(16))) uint32_t ring[16 * 256];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    md5_chain_wg(src + blockIdx.x * kFileBytes, kFileBytes, blockIdx.x, wv, reinterpret_cast<uint4 *>(ring), sig,
                 nullptr, nullptr);
}

template <int W>
__global__ __launch_bounds__(64 * W) void k_wave(const uint8_t *src, uint8_t *sig)
{
    __shared__ __attribute__((aligned(16))) uint32_t ring[W * 1024];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t f = blockIdx.x * W + wv;
    md5_chain_wave(src + f * kFileBytes, kFileBytes, f, reinterpret_cast<uint4 *>(ring) + wv * 256, sig, nullptr,
                   nullptr);
}

int main(int argc, char **argv)
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int nfiles = argc > 1 ? atoi(argv[1]) : ncu;  // chains (a multiple of 4)
    uint8_t *src, *sig;
    hipMalloc(&src, kFileBytes * nfiles);
    hipMalloc(&sig, 24 * nfiles);
    hipMemset(src, 0x5A, kFileBytes * nfiles);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d, \"chains\": %d, \"file_bytes\": %llu, \"runs\": [\n", ncu, nfiles,
           (unsigned long long)kFileBytes);
    const char *names[] = {"wg_helper", "wave_x1", "wave_x2", "wave_x4", "wg_helper"};
    for (int v = 0; v < 5; v++) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0, 0);
            if (v == 0 || v == 4)
                hipLaunchKernelGGL(k_wg, dim3(nfiles), dim3(128), 0, 0, src, sig);
            else if (v == 1)
                hipLaunchKernelGGL(k_wave<1>, dim3(nfiles), dim3(64), 0, 0, src, sig);
            else if (v == 2)
                hipLaunchKernelGGL(k_wave<2>, dim3(nfiles / 2), dim3(128), 0, 0, src, sig);
            else
                hipLaunchKernelGGL(k_wave<4>, dim3(nfiles / 4), dim3(256), 0, 0, src, sig);
            hipEventRecord(e1, 0);
            const hipError_t err = hipEventSynchronize(e1);
            if (err != hipSuccess) {
                printf("\n]}\nerror %s\n", hipGetErrorString(err));
                return 2;
            }
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("%s{\"form\": \"%s\", \"ms\": %.3f, \"mb_per_s_per_chain\": %.1f, \"cycles_per_byte_at_2.4GHz\": %.3f}",
               v ? ",\n" : "", names[v], best, kFileBytes / (best * 1e3), best * 1e-3 * 2.4e9 / kFileBytes);
    }
    printf("\n]}\n");
    return 0;
}
