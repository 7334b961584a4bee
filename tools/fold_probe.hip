// fold_probe.hip -- DIAGNOSTIC ONLY: the CRC-64 step fold itself (f64x from
// crc_gpu_device.h: 12 ds_read_b64 lookups, 14 address ops, the 13-input XOR
// tree) on register data -- no HBM stream -- at the occupancies the batch
// kernels can use: CH independent 64-bit states per lane, one 1024-thread
// workgroup per CU (4 waves/SIMD) or two (8 waves/SIMD).  Tables hold random
// words (timing only).  Reports shader cycles per 8-byte word per CU and per
// lookup per CU.  Every launch ends after its fixed loop.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "crc_gpu_device.h"

namespace {
constexpr int kSteps = 512;

template <int CH, int MINB>
__global__ __launch_bounds__(1024, MINB) void fold(uint64_t *sink, unsigned long long *stamps, uint64_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kL64Main];
    for (uint32_t i = threadIdx.x; i < kL64Main / 8; i += 1024)
        reinterpret_cast<uint64_t *>(lds)[i] = (i + seed) * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const uint32_t lc = (threadIdx.x & 31u) << 3;
    Lane64 ln = lane64(lc);
    uint64_t x[CH];
#pragma unroll
    for (int k = 0; k < CH; k++) x[k] = seed * (k + 1) + threadIdx.x * 0x5851F42D4C957F2Dull;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kSteps; it++) {
#pragma unroll
        for (int k = 0; k < CH; k++) x[k] = f64x(lds, x[k], x[k] >> 7, ln);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < CH; k++) r ^= x[k];
    sink[blockIdx.x * 1024 + threadIdx.x] = r;
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t w = blockIdx.x * 16 + threadIdx.x / 64;
        stamps[2 * w] = t0;
        stamps[2 * w + 1] = t1;
    }
}

template <int CH, int MINB>
void run(int cus, uint64_t *sink, unsigned long long *stamps) {
    const int grid = cus * MINB, waves = grid * 16;
    std::vector<unsigned long long> h(2 * waves);
    double best = 1e30;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL((fold<CH, MINB>), dim3(grid), dim3(1024), 0, 0, sink, stamps, 11u + rep);
        if (hipDeviceSynchronize() != hipSuccess) return;
        (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
        double sum = 0;
        for (int w = 0; w < waves; w++) sum += (double)(h[2 * w + 1] - h[2 * w]);
        const double dur = sum / waves;
        const double words_per_cu = (double)(waves / cus) * CH * kSteps;  // wave-words
        best = dur / words_per_cu < best ? dur / words_per_cu : best;
    }
    printf("  %d state(s)/lane, %d WG/CU (%d waves/SIMD): %.1f cycles per wave-word per CU = %.2f per lookup; "
           "%.1f B/clk/CU\n", CH, MINB, 4 * MINB, best, best / 12, 512.0 / best);
}
}  // namespace

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint64_t *sink = nullptr;
    unsigned long long *stamps = nullptr;
    (void)hipMalloc(&sink, (size_t)cus * 2048 * 8);
    (void)hipMalloc(&stamps, (size_t)cus * 32 * 16);
    printf("CRC-64 fold f64x on register data, %d CUs (C3's kernel: 2 states/lane, 1 WG/CU, ~29.9 cycles per wave-word per CU with HBM):\n", cus);
    run<1, 1>(cus, sink, stamps);
    run<2, 1>(cus, sink, stamps);
    run<4, 1>(cus, sink, stamps);
    run<1, 2>(cus, sink, stamps);
    run<2, 2>(cus, sink, stamps);
    (void)hipFree(sink);
    (void)hipFree(stamps);
    return 0;
}
