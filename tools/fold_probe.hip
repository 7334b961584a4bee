// fold_probe.hip -- DIAGNOSTIC ONLY: the CRC-64 step fold itself (f64x from
// crc_gpu_device.h: 12 ds_read_b64 lookups, 14 address ops, the 13-input XOR
// tree) on register data -- no HBM stream -- at the occupancies the batch
// kernels can use: CH independent 64-bit states per lane, one 1024-thread
// workgroup per CU (4 waves/SIMD) or two (8 waves/SIMD).  Tables hold random
// words (timing only).  Reports shader cycles per 8-byte word per CU and per
// lookup per CU.  Every launch ends after its fixed loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "crc_gpu_device.h"

namespace {
constexpr int kSteps = 512;

template <int CH, int MINB>
__global__ __launch_bounds__(1024, 4 * MINB) void fold(uint64_t *sink, unsigned long long *stamps, uint64_t seed) {
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

// The same fold fed by an HBM stream, as in the batch kernel's aligned loop:
// each wave reads its own contiguous region with a 4-deep ring of 16-B
// non-temporal loads per lane (one 1 KiB wave-load per step), 2 states per
// lane (lo / hi 8 bytes), the data word folded in by the XOR tree.
template <int MINB, int R>
__global__ __launch_bounds__(1024, 4 * MINB) void stream_fold(const uint4 *data, uint64_t words_per_wave, uint64_t *sink,
                                                           unsigned long long *stamps) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kL64Main];
    for (uint32_t i = threadIdx.x; i < kL64Main / 8; i += 1024)
        reinterpret_cast<uint64_t *>(lds)[i] = (i + 7) * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 16 + threadIdx.x / 64;
    Lane64 ln = lane64((lane & 31u) << 3);
    gbyte_t p = global_ptr(reinterpret_cast<const uint8_t *>(data + (uint64_t)wave * words_per_wave * 64 + lane), false);
    const uint64_t K = words_per_wave;
    uint4 ring[R];
#pragma unroll
    for (int u = 0; u < R; u++) ring[u] = ldg16<true>(p + u * 1024);
    uint64_t x0 = lo64(ring[0]), x1 = hi64(ring[0]);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint64_t k = R; k < K; k += R) {
        p += R * 1024;
#pragma unroll
        for (int u = 0; u < R; u++) {
            ring[u] = ldg16<true>(p + u * 1024);
            const uint4 nx = ring[(u + 1) % R];
            x0 = f64x(lds, x0, lo64(nx), ln);
            x1 = f64x(lds, x1, hi64(nx), ln);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 1024 + threadIdx.x] = x0 ^ x1;
    if ((threadIdx.x & 63u) == 0) {
        stamps[2 * wave] = t0;
        stamps[2 * wave + 1] = t1;
    }
}

// One state per lane: 8 bytes per lane and step (512 B per wave-load), the
// shape a two-workgroup-per-CU CRC-64 loop would take to fit 64 VGPRs.
typedef const __attribute__((address_space(1))) uint64_t *g64_t;
template <int MINB, int R>
__global__ __launch_bounds__(1024, 4 * MINB) void stream_fold1(const uint64_t *data, uint64_t steps_per_wave,
                                                            uint64_t *sink, unsigned long long *stamps) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kL64Main];
    for (uint32_t i = threadIdx.x; i < kL64Main / 8; i += 1024)
        reinterpret_cast<uint64_t *>(lds)[i] = (i + 7) * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 16 + threadIdx.x / 64;
    Lane64 ln = lane64((lane & 31u) << 3);
    g64_t p = (g64_t)(data + (uint64_t)wave * steps_per_wave * 64 + lane);
    const uint64_t K = steps_per_wave;
    uint64_t ring[R];
#pragma unroll
    for (int u = 0; u < R; u++) ring[u] = __builtin_nontemporal_load(p + u * 64);
    uint64_t x = ring[0];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint64_t k = R; k < K; k += R) {
        p += R * 64;
#pragma unroll
        for (int u = 0; u < R; u++) {
            ring[u] = __builtin_nontemporal_load(p + u * 64);
            x = f64x(lds, x, ring[(u + 1) % R], ln);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 1024 + threadIdx.x] = x;
    if ((threadIdx.x & 63u) == 0) {
        stamps[2 * wave] = t0;
        stamps[2 * wave + 1] = t1;
    }
}

// Steady state, interleaved: `rounds` rounds of `series` back-to-back 4 GiB
// launches per variant (one event pair per series), variants in turn, so
// every variant sees the same power-controller state; the median per-launch
// time and the in-kernel shader clock (s_memtime cycles over the event time)
// of each variant.
template <int MINB, int R>
float series_stream(int cus, const uint4 *data, uint64_t *sink, unsigned long long *stamps, int series, double *ghz) {
    const int grid = cus * MINB, waves = grid * 16;
    const uint64_t wpw = (4ull << 30) / 1024 / waves / R * R;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < series; i++)
        hipLaunchKernelGGL((stream_fold<MINB, R>), dim3(grid), dim3(1024), 0, 0, data, wpw, sink, stamps);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(2 * waves);
    (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int w = 0; w < waves; w++) sum += (double)(h[2 * w + 1] - h[2 * w]);
    *ghz = sum / waves / (ms / series * 1e6);  // cycles of a wave's loop per ns of launch (lower bound)
    return ms / series;
}
template <int MINB, int R>
float series_stream1(int cus, const uint64_t *data, uint64_t *sink, unsigned long long *stamps, int series, double *ghz) {
    const int grid = cus * MINB, waves = grid * 16;
    const uint64_t spw = (4ull << 30) / 512 / waves / R * R;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < series; i++)
        hipLaunchKernelGGL((stream_fold1<MINB, R>), dim3(grid), dim3(1024), 0, 0, data, spw, sink, stamps);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(2 * waves);
    (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int w = 0; w < waves; w++) sum += (double)(h[2 * w + 1] - h[2 * w]);
    *ghz = sum / waves / (ms / series * 1e6);
    return ms / series;
}

template <int MINB, int R>
void run_stream(int cus, const uint4 *data, uint64_t *sink, unsigned long long *stamps) {
    const int grid = cus * MINB, waves = grid * 16;
    const uint64_t bytes = 4ull << 30;
    const uint64_t wpw = bytes / 1024 / waves / R * R;  // wave-steps per wave
    std::vector<unsigned long long> h(2 * waves);
    double best = 1e30, best_ms = 0;
    for (int rep = 0; rep < 4; rep++) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL((stream_fold<MINB, R>), dim3(grid), dim3(1024), 0, 0, data, wpw, sink, stamps);
        (void)hipEventRecord(e1, 0);
        if (hipDeviceSynchronize() != hipSuccess) return;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
        double sum = 0;
        for (int w = 0; w < waves; w++) sum += (double)(h[2 * w + 1] - h[2 * w]);
        const double dur = sum / waves;
        const double cyc = dur / ((double)(waves / cus) * 2 * wpw);  // per wave-word per CU
        if (cyc < best) {
            best = cyc;
            best_ms = ms;
        }
    }
    const double gb = (double)waves * wpw * 1024 / 1e9;
    printf("  HBM-fed, ring %d, %d WG/CU (%d waves/SIMD): %.1f cycles per wave-word per CU; %.3f ms for %.2f GB = %.2f TB/s\n",
           R, MINB, 4 * MINB, best, best_ms, gb, gb / best_ms);
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
    uint4 *data = nullptr;
    (void)hipMalloc(&data, (4ull << 30) + 65536);
    (void)hipMemset(data, 0x5A, (4ull << 30) + 65536);
    run_stream<1, 4>(cus, data, sink, stamps);
    run_stream<1, 8>(cus, data, sink, stamps);
    run_stream<2, 4>(cus, data, sink, stamps);
    run_stream<1, 4>(cus, data, sink, stamps);
    run_stream<2, 4>(cus, data, sink, stamps);
    // steady-state series, variants interleaved
    {
        const char *names[] = {"2 states, 1 WG/CU, ring 4 (C3's shape)", "2 states, 2 WG/CU, ring 4",
                               "1 state (8 B/lane), 2 WG/CU, ring 8", "1 state (8 B/lane), 2 WG/CU, ring 4",
                               "1 state (8 B/lane), 1 WG/CU, ring 8"};
        std::vector<std::vector<float>> t(5);
        std::vector<std::vector<double>> g(5);
        for (int r = 0; r < 7; r++)
            for (int v = 0; v < 5; v++) {
                double ghz = 0;
                float ms = v == 0   ? series_stream<1, 4>(cus, data, sink, stamps, 20, &ghz)
                           : v == 1 ? series_stream<2, 4>(cus, data, sink, stamps, 20, &ghz)
                           : v == 2 ? series_stream1<2, 8>(cus, reinterpret_cast<const uint64_t *>(data), sink, stamps, 20, &ghz)
                           : v == 3 ? series_stream1<2, 4>(cus, reinterpret_cast<const uint64_t *>(data), sink, stamps, 20, &ghz)
                                    : series_stream1<1, 8>(cus, reinterpret_cast<const uint64_t *>(data), sink, stamps, 20, &ghz);
                if (r > 0) {  // round 0 warms up
                    t[v].push_back(ms);
                    g[v].push_back(ghz);
                }
            }
        printf("steady state, 20 launches per series, 6 interleaved rounds (median ms per 4 GiB launch; loop GHz):\n");
        for (int v = 0; v < 5; v++) {
            std::vector<float> a = t[v];
            std::sort(a.begin(), a.end());
            std::vector<double> b = g[v];
            std::sort(b.begin(), b.end());
            printf("  %-40s %.4f ms = %.2f TB/s; loop clock %.2f GHz\n", names[v], a[a.size() / 2],
                   4.294967296 / a[a.size() / 2], b[b.size() / 2]);
        }
    }
    (void)hipFree(data);
    (void)hipFree(sink);
    (void)hipFree(stamps);
    return 0;
}
