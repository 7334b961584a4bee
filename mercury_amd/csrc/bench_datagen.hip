// bench_datagen.hip -- device-side synthetic payload bytes for the tests and
// bench.py (libmchecksum_bench.so; not part of the mchecksum ABI).
//
// Bytes are little-endian 64-bit words splitmix64(seed ^ (first_word + i))
// (SURVEY.md 8(d)), generated where they are checksummed so no 4 GiB H2D copy
// is needed; the CPU oracle regenerates the identical bytes on the host.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_kernel(uint64_t *dst, uint64_t nwords, uint64_t seed, uint64_t first) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    // two words (16 B) per thread per iteration
    for (uint64_t i = tid; 2 * i + 1 < nwords; i += nthr) {
        ulonglong2 v;
        v.x = splitmix64(seed ^ (first + 2 * i));
        v.y = splitmix64(seed ^ (first + 2 * i + 1));
        reinterpret_cast<ulonglong2 *>(dst)[i] = v;
    }
    if (tid == 0 && (nwords & 1)) dst[nwords - 1] = splitmix64(seed ^ (first + nwords - 1));
}

__global__ void tail_kernel(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t first) {
    const uint64_t nw = nbytes / 8;
    const uint64_t w = splitmix64(seed ^ (first + nw));
    for (uint64_t b = 0; b < (nbytes & 7); b++) dst[8 * nw + b] = (uint8_t)(w >> (8 * b));
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int mck_bench_fill_splitmix(void *dev, uint64_t nbytes,
                                                                               uint64_t seed, uint64_t first_word,
                                                                               void *stream) {
    if (!dev && nbytes) return -1;
    if (((uintptr_t)dev & 15) != 0) return -1;
    const uint64_t nwords = nbytes / 8;
    hipStream_t s = (hipStream_t)stream;
    if (nwords) {
        uint64_t blocks = (nwords / 2 + 255) / 256;
        if (blocks > 8192) blocks = 8192;
        if (!blocks) blocks = 1;
        hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (uint64_t *)dev, nwords, seed,
                           first_word);
    }
    if (nbytes & 7) hipLaunchKernelGGL(tail_kernel, dim3(1), dim3(1), 0, s, (uint8_t *)dev, nbytes, seed, first_word);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Test utility (tests/test_gpu_slots.py): hold a stream until the host
// releases it.  One wave polls a word of host memory (mck_bench_host_alloc:
// coherent, mapped into the device) until it reads non-zero, or until
// max_ticks of the 100 MHz real-time counter have passed -- then *expired = 1
// (the test fails rather than the stream staying blocked).  Unlike a sleep
// kernel, the hold ends exactly when the test says so.
namespace {
__global__ __launch_bounds__(64) void gate_kernel(const uint32_t *flag, uint32_t *expired, uint64_t max_ticks) {
    const uint64_t t0 = wall_clock64();
    for (;;) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
        if (wall_clock64() - t0 > max_ticks) {
            if (threadIdx.x == 0) __hip_atomic_store(expired, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(32);
    }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) void *mck_bench_host_alloc(uint64_t nbytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, nbytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
    memset(p, 0, nbytes);
    return p;
}

extern "C" __attribute__((visibility("default"))) int mck_bench_host_free(void *p) {
    return hipHostFree(p) == hipSuccess ? 0 : -1;
}

extern "C" __attribute__((visibility("default"))) int mck_bench_gate(const uint32_t *flag, uint32_t *expired,
                                                                     double max_seconds, void *stream) {
    if (!flag || !expired || !(max_seconds > 0) || max_seconds > 60) return -1;
    void *df = nullptr, *de = nullptr;
    if (hipHostGetDevicePointer(&df, const_cast<uint32_t *>(flag), 0) != hipSuccess ||
        hipHostGetDevicePointer(&de, expired, 0) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint32_t *)df, (uint32_t *)de,
                       (uint64_t)(max_seconds * 1e8));
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
