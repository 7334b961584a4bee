// lds_chain_probe.hip -- DIAGNOSTIC ONLY: is the CRC-64 fold loop bound by the
// latency of its dependent lookup chains or by throughput?  Each lane runs CH
// independent chains of the fold's lookup pattern -- an SDWA address from the
// chain value, ds_read_b64 from a 32x-replicated table, XOR of the result back
// into the chain -- with one 1024-thread workgroup per CU (4 waves/SIMD) or
// two 512-thread ones... (WG = threads per workgroup, WPC = workgroups per CU).
// cycles per lookup per CU = wave duration * waves per CU ... reported as
// shader cycles per lookup per CU (lower is better; the LDS array's own
// bound for ds_read_b64 is 2).  Every launch ends after its fixed loop.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

namespace {
constexpr int kIters = 1024;

template <int CH, int BLOCK, int MINB>
__global__ __launch_bounds__(BLOCK, MINB) void chains(uint32_t *sink, unsigned long long *stamps, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 1024];
    for (uint32_t i = threadIdx.x; i < 64 * 1024 / 4; i += BLOCK) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u + seed;
    __syncthreads();
    uint32_t a[CH], ad[CH];
    const uint32_t lc = (threadIdx.x & 31u) << 3;
#pragma unroll
    for (int k = 0; k < CH; k++) {
        a[k] = seed * 2654435761u + k * 40503u + threadIdx.x * 977u;
        ad[k] = lc;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
        uint64_t v[CH];
#pragma unroll
        for (int k = 0; k < CH; k++) {
            asm volatile("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_2"
                         : "+v"(ad[k]) : "s"(0x3Fu), "v"(a[k]));
            v[k] = *reinterpret_cast<const uint64_t *>(lds + ad[k] + (k & 3) * 16384);
        }
#pragma unroll
        for (int k = 0; k < CH; k++) a[k] ^= (uint32_t)v[k] ^ (uint32_t)(v[k] >> 32);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < CH; k++) x ^= a[k];
    sink[blockIdx.x * BLOCK + threadIdx.x] = x;
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t w = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64;
        stamps[2 * w] = t0;
        stamps[2 * w + 1] = t1;
    }
}

template <int CH, int BLOCK, int MINB = 1>
void run(int cus, int wpc, uint32_t *sink, unsigned long long *stamps) {
    const int grid = cus * wpc, waves = grid * (BLOCK / 64);
    std::vector<unsigned long long> h(2 * waves);
    double best = 1e30;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL((chains<CH, BLOCK, MINB>), dim3(grid), dim3(BLOCK), 0, 0, sink, stamps, 7u + rep);
        if (hipDeviceSynchronize() != hipSuccess) return;
        (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
        unsigned long long lo = ~0ull, hi = 0;
        for (int w = 0; w < waves; w++) {
            lo = h[2 * w] < lo ? h[2 * w] : lo;
            hi = h[2 * w + 1] > hi ? h[2 * w + 1] : hi;
        }
        // (stamps of different CUs share one clock domain per XCD; the span over
        // all waves bounds the CU's duration from above)
        double sum = 0;
        for (int w = 0; w < waves; w++) sum += (double)(h[2 * w + 1] - h[2 * w]);
        const double dur = sum / waves;
        const double lookups_per_cu = (double)(waves / cus) * 64 / 64 * CH * kIters;  // wave-instructions
        best = dur / lookups_per_cu < best ? dur / lookups_per_cu : best;
    }
    printf("  %2d chains/lane  %4d threads x %d WG/CU (%2d waves/SIMD): %.2f cycles per lookup per CU\n", CH, BLOCK,
           wpc, BLOCK / 64 * wpc / 4, best);
}
}  // namespace

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *sink = nullptr;
    unsigned long long *stamps = nullptr;
    (void)hipMalloc(&sink, (size_t)cus * 2048 * 4);
    (void)hipMalloc(&stamps, (size_t)cus * 32 * 16);
    printf("CRC-64 lookup chains (SDWA address -> ds_read_b64 -> XOR), %d CUs:\n", cus);
    run<2, 1024>(cus, 1, sink, stamps);
    run<4, 1024>(cus, 1, sink, stamps);
    run<8, 1024>(cus, 1, sink, stamps);
    run<16, 1024>(cus, 1, sink, stamps);
    run<24, 1024>(cus, 1, sink, stamps);
    run<2, 1024, 2>(cus, 2, sink, stamps);  // 64 KiB LDS each: 2 per CU = 128 KiB, 8 waves/SIMD
    run<4, 1024, 2>(cus, 2, sink, stamps);
    run<8, 1024, 2>(cus, 2, sink, stamps);
    run<16, 1024, 2>(cus, 2, sink, stamps);
    (void)hipFree(sink);
    (void)hipFree(stamps);
    return 0;
}
