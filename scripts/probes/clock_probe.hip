// Shader clock under load: one wave spins for `ms` of wall time (s_memrealtime,
// 100 MHz) and counts shader cycles (s_memtime) over the same interval; the
// host prints the ratio as MHz, `samples` times with `gap_ms` between them.
// Run beside a bench process to see the clock the chip holds under that load.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

__global__ void clock_kernel(unsigned long long ticks, unsigned long long *out)
{
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r = r0;
    while (r - r0 < ticks)
        r = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r - r0;
    }
}

int main(int argc, char **argv)
{
    const int samples = argc > 1 ? atoi(argv[1]) : 20;
    const int gap_ms = argc > 2 ? atoi(argv[2]) : 500;
    const int ms = argc > 3 ? atoi(argv[3]) : 20;
    unsigned long long *d, h[2];
    if (hipMalloc(&d, 16) != hipSuccess)
        return 1;
    for (int i = 0; i < samples; i++) {
        clock_kernel<<<1, 64>>>((unsigned long long)ms * 100000ull, d);
        if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess)
            return 1;
        printf("sample %d: %.0f MHz\n", i, (double)h[0] / ((double)h[1] / 100.0));
        fflush(stdout);
        usleep(gap_ms * 1000);
    }
    (void)hipFree(d);
    return 0;
}
