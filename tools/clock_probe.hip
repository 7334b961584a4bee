// clock_probe.hip -- DIAGNOSTIC ONLY (not part of libmchecksum): samples the
// shader clock while other kernels run.  One wave, lane 0: every `period`
// ticks of the constant 100 MHz real-time counter it records
// (shader-clock counter, real-time counter).  The ratio of their increments
// is the SCLK over that interval (tools/clock_series.py).  The sampler uses
// no LDS and one wave, so it co-resides with a persistent 1024-thread
// workgroup on one CU and perturbs the measured kernel by ~1/256.
// Exit: after `n` samples, or when the real-time counter passed `limit`
// ticks since the start, whichever comes first -- every path ends.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(64) void clock_sampler(unsigned long long *buf, uint32_t n, uint32_t period,
                                                    unsigned long long limit) {
    if (threadIdx.x != 0) return;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long next = r0;
    for (uint32_t i = 0; i < n; i++) {
        unsigned long long r;
        do {
            __builtin_amdgcn_s_sleep(2);
            r = __builtin_amdgcn_s_memrealtime();
        } while (r < next && r - r0 < limit);
        const unsigned long long c = __builtin_amdgcn_s_memtime();
        buf[2 * i] = c;
        buf[2 * i + 1] = r;
        if (r - r0 >= limit) return;  // the host zero-fills buf: unused samples stay 0
        next = r + period;
    }
}

extern "C" int mck_clock_sampler(void *buf, uint32_t n, uint32_t period, unsigned long long limit, void *stream) {
    hipLaunchKernelGGL(clock_sampler, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long *)buf, n, period,
                       limit);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
