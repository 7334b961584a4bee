// valu_probe.hip -- DIAGNOSTIC ONLY (not part of libmchecksum): issue cost of
// the vector instructions the CRC fold loops are made of, on gfx950, with the
// loops' occupancy (one 1024-thread workgroup per CU: 4 waves per SIMD).
//
// Each lane runs 8 independent chains of one instruction kind (inline asm, so
// the exact encoding is measured), 2048 iterations; every wave stamps the
// shader clock (s_memtime) around its loop.  cycles per instruction per SIMD
// = wave duration / (4 waves x 8 chains x iterations).  Kinds: VOP2 XOR,
// VOP3 bitop3, SDWA AND into a byte (as the CRC-64 address formation), v_perm,
// v_bfi, a VOP2 shift, and ds_read_b64 (LDS, conflict-free, with one VOP2
// XOR each to consume the data), and the CRC-64 word mix (1 SDWA + 1 ds_read
// + 1 bitop3).  Every launch ends after its fixed loop: no waits.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

namespace {

constexpr int kChains = 8;
constexpr int kIters = 2048;

template <int OP>
__device__ __forceinline__ void op(uint32_t &a, uint32_t b, uint32_t c, const uint8_t *lds) {
    if constexpr (OP == 0) {
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    } else if constexpr (OP == 1) {
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (OP == 2) {
        asm volatile("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_2"
                     : "+v"(a) : "s"(0x3Fu), "v"(b));
    } else if constexpr (OP == 3) {
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (OP == 4) {
        asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a) : "s"(0x07070707u), "v"(b));
    } else if constexpr (OP == 5) {
        asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a));
    }
}

// OP 6 / 7: one iteration over all chains (LDS loads through C++, so the
// compiler places the lgkmcnt waits: all reads issued, then consumed)
template <int OP>
__device__ __forceinline__ void iter_lds(uint32_t (&a)[kChains], uint32_t b, uint32_t c, const uint8_t *lds) {
    uint64_t v[kChains];
    if constexpr (OP == 6) {
#pragma unroll
        for (int k = 0; k < kChains; k++) v[k] = *reinterpret_cast<const uint64_t *>(lds + c + k * 256);
#pragma unroll
        for (int k = 0; k < kChains; k++) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"((uint32_t)v[k]));
    } else {
        // CRC-64 per lookup: 1 SDWA address + 1 ds_read_b64 + 2 bitop3 (the two
        // 32-bit halves of a 64-bit XOR tree input, 3 inputs each)
#pragma unroll
        for (int k = 0; k < kChains; k++) {
            uint32_t ad = c;
            asm volatile("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_2"
                         : "+v"(ad) : "s"(0x3Fu), "v"(a[k]));
            v[k] = *reinterpret_cast<const uint64_t *>(lds + ad + k * 16384 % 65536);
        }
#pragma unroll
        for (int k = 0; k < kChains; k += 2) {
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[k]) : "v"((uint32_t)v[k]), "v"((uint32_t)v[k + 1]));
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[k + 1]) : "v"((uint32_t)(v[k] >> 32)), "v"((uint32_t)(v[k + 1] >> 32)));
        }
    }
}

template <int OP>
__global__ __launch_bounds__(1024, 1) void probe(uint32_t *sink, unsigned long long *stamps, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 1024];
    for (uint32_t i = threadIdx.x; i < 64 * 1024 / 4; i += 1024) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t a[kChains];
    const uint32_t b = seed ^ (threadIdx.x * 8u), c = (threadIdx.x & 31u) << 3;
#pragma unroll
    for (int k = 0; k < kChains; k++) a[k] = seed + k * 77u + threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
        if constexpr (OP >= 6) {
            iter_lds<OP>(a, b, c, lds);
        } else {
#pragma unroll
            for (int k = 0; k < kChains; k++) op<OP>(a[k], b, c, lds);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < kChains; k++) x ^= a[k];
    sink[blockIdx.x * 1024 + threadIdx.x] = x;
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t w = blockIdx.x * 16 + threadIdx.x / 64;
        stamps[2 * w] = t0;
        stamps[2 * w + 1] = t1;
    }
}

template <int OP>
double run(int cus, uint32_t *sink, unsigned long long *stamps) {
    std::vector<unsigned long long> h(2 * 16 * cus);
    double best = 1e30;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(probe<OP>, dim3(cus), dim3(1024), 0, 0, sink, stamps, 12345u + rep);
        if (hipDeviceSynchronize() != hipSuccess) return -1;
        (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
        double sum = 0;
        for (int w = 0; w < 16 * cus; w++) sum += (double)(h[2 * w + 1] - h[2 * w]);
        const double per_wave = sum / (16 * cus);
        // 4 waves share a SIMD; OP 7 counts one lookup (4 instructions) per chain
        const double cyc = per_wave / (4.0 * kChains * kIters);
        best = cyc < best ? cyc : best;
    }
    return best;
}

}  // namespace

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *sink = nullptr;
    unsigned long long *stamps = nullptr;
    (void)hipMalloc(&sink, (size_t)cus * 1024 * 4);
    (void)hipMalloc(&stamps, (size_t)cus * 16 * 16);
    const char *names[] = {"v_xor_b32 (VOP2)", "v_bitop3_b32 (VOP3)", "v_and_b32_sdwa (byte)", "v_perm_b32",
                           "v_bfi_b32", "v_lshrrev_b32 (VOP2)", "ds_read_b64 + v_xor (waited)",
                           "CRC-64 lookup: sdwa+ds_read_b64+0.5x2 bitop3"};
    double r[8];
    r[0] = run<0>(cus, sink, stamps);
    r[1] = run<1>(cus, sink, stamps);
    r[2] = run<2>(cus, sink, stamps);
    r[3] = run<3>(cus, sink, stamps);
    r[4] = run<4>(cus, sink, stamps);
    r[5] = run<5>(cus, sink, stamps);
    r[6] = run<6>(cus, sink, stamps);
    r[7] = run<7>(cus, sink, stamps);
    printf("shader cycles per wave-instruction per SIMD (4 waves/SIMD, %d CUs, %d chains x %d iterations):\n", cus,
           kChains, kIters);
    for (int i = 0; i < 8; i++) printf("  %-44s %.2f\n", names[i], r[i]);
    (void)hipFree(sink);
    (void)hipFree(stamps);
    return 0;
}
