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
    } else if constexpr (OP == 12) {  // the f5 address form: byte & 0xF8, rest of the dword zeroed
        asm volatile("v_and_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                     : "+v"(a) : "s"(0xF8u));
    } else if constexpr (OP == 13) {  // VOP2 AND with the mask in an SGPR
        asm volatile("v_and_b32 %0, %1, %0" : "+v"(a) : "s"(0xF8F8u));
    } else if constexpr (OP == 14) {
        asm volatile("v_bfe_u32 %0, %0, 11, 5" : "+v"(a));
    } else if constexpr (OP == 15) {  // (a & mask) | c as one bitop3 (S0 & S1 | S2 = 0xEA), mask in an SGPR
        asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xea" : "+v"(a) : "s"(0x3F00u), "v"(c));
    } else if constexpr (OP == 16) {
        asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a) : "v"(b));
    } else if constexpr (OP == 17) {
        asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "s"(0x3F00u), "v"(c));
    } else if constexpr (OP == 18) {
        asm volatile("v_alignbit_b32 %0, %0, %1, 5" : "+v"(a) : "v"(b));
    } else if constexpr (OP == 19) {  // bfi as a bitop3 (S0 ? S1 : S2 = 0xCA), mask in an SGPR
        asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca" : "+v"(a) : "s"(0x07070707u), "v"(b));
    } else if constexpr (OP == 20) {
        asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(a) : "v"(c));
    } else if constexpr (OP == 21) {  // v_perm with a constant selector in an SGPR
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(c), "s"(0x0C020400u));
    } else if constexpr (OP == 22) {  // SDWA AND into byte 1 (PRESERVE), the mask in a VGPR
        asm volatile("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_2"
                     : "+v"(a) : "v"(c), "v"(b));
    } else if constexpr (OP == 23) {  // SDWA AND (PAD), the mask in a VGPR
        asm volatile("v_and_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                     : "+v"(a) : "v"(c));
    } else if constexpr (OP == 24) {  // VOP2 AND, VGPR mask
        asm volatile("v_and_b32 %0, %1, %0" : "+v"(a) : "v"(c));
    } else if constexpr (OP == 25) {  // VOP2 XOR with an SGPR operand
        asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a) : "s"(0x1234u));
    } else if constexpr (OP == 26) {  // bitop3 as bfi, mask in a VGPR
        asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca" : "+v"(a) : "v"(c), "v"(b));
    } else if constexpr (OP == 27) {  // VOP2 AND with an inline constant
        asm volatile("v_and_b32 %0, 63, %0" : "+v"(a));
    } else if constexpr (OP == 28) {  // VOP2 shift left, inline
        asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a));
    } else if constexpr (OP == 29) {  // v_or_b32 VGPR
        asm volatile("v_or_b32 %0, %1, %0" : "+v"(a) : "v"(c));
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

// OP 8..11: LDS read throughput alone -- 16 reads per iteration (asm, fixed
// conflict-free lane addresses: lane copy (lane % 32) * 8 plus a table
// offset), one lgkmcnt(0) wait, then 2 VOP2 XORs to keep the data live.
// 8: ds_read_b64 within 16 KiB; 9: ds_read_b64 over 128 KiB (a base register
// per 32 KiB); 10: ds_read_b128 (16 copies, 16 B each); 11: ds_read_b32.
template <int OP>
__device__ __forceinline__ void iter_lds_only(uint32_t (&a)[kChains], uint32_t c) {
    uint32_t acc0 = 0, acc1 = 0;
    if constexpr (OP == 8 || OP == 9) {
        uint64_t v[16];
        const uint32_t b0 = c, b1 = c + (OP == 9 ? 32768u : 0u), b2 = c + (OP == 9 ? 65536u : 0u),
                       b3 = c + (OP == 9 ? 98304u : 0u);
#define RD(i, base, off) asm volatile("ds_read_b64 %0, %1 offset:" #off : "=v"(v[i]) : "v"(base))
        RD(0, b0, 0); RD(1, b0, 2048); RD(2, b0, 4096); RD(3, b0, 6144);
        RD(4, b1, 8192); RD(5, b1, 10240); RD(6, b1, 12288); RD(7, b1, 14336);
        RD(8, b2, 256); RD(9, b2, 2304); RD(10, b2, 4352); RD(11, b2, 6400);
        RD(12, b3, 8448); RD(13, b3, 10496); RD(14, b3, 12544); RD(15, b3, 14592);
#undef RD
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < 16; i++) { acc0 ^= (uint32_t)v[i]; acc1 ^= (uint32_t)(v[i] >> 32); }
    } else if constexpr (OP == 10) {
        uint4 v[16];
        const uint32_t b = (c >> 3) << 4;  // 16 lanes' copies per 256 B row
#define RD(i, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(v[i]) : "v"(b))
        RD(0, 0); RD(1, 2048); RD(2, 4096); RD(3, 6144); RD(4, 8192); RD(5, 10240); RD(6, 12288); RD(7, 14336);
        RD(8, 512); RD(9, 2560); RD(10, 4608); RD(11, 6656); RD(12, 8704); RD(13, 10752); RD(14, 12800); RD(15, 14848);
#undef RD
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < 16; i++) { acc0 ^= v[i].x ^ v[i].z; acc1 ^= v[i].y ^ v[i].w; }
    } else {
        uint32_t v[16];
        const uint32_t b = c >> 1;  // 32 lanes' 4-B copies per 128 B
#define RD(i, off) asm volatile("ds_read_b32 %0, %1 offset:" #off : "=v"(v[i]) : "v"(b))
        RD(0, 0); RD(1, 2048); RD(2, 4096); RD(3, 6144); RD(4, 8192); RD(5, 10240); RD(6, 12288); RD(7, 14336);
        RD(8, 256); RD(9, 2304); RD(10, 4352); RD(11, 6400); RD(12, 8448); RD(13, 10496); RD(14, 12544); RD(15, 14592);
#undef RD
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < 16; i++) acc0 ^= v[i];
    }
    a[0] ^= acc0;
    a[1] ^= acc1;
}

template <int OP>
__global__ __launch_bounds__(1024, 1) void probe(uint32_t *sink, unsigned long long *stamps, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[(OP == 9 ? 144 : 64) * 1024];
    for (uint32_t i = threadIdx.x; i < sizeof(lds) / 4; i += 1024) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t a[kChains];
    const uint32_t b = seed ^ (threadIdx.x * 8u), c = (threadIdx.x & 31u) << 3;
#pragma unroll
    for (int k = 0; k < kChains; k++) a[k] = seed + k * 77u + threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
        if constexpr (OP >= 8 && OP <= 11) {
            iter_lds_only<OP>(a, c);
        } else if constexpr (OP == 6 || OP == 7) {
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
        // 4 waves share a SIMD; OP 7 counts one lookup (3 instructions) per
        // chain; OP 8..11 one LDS read (of 16 per iteration)
        const double cyc = per_wave / (4.0 * (OP >= 8 && OP <= 11 ? 16 : kChains) * kIters);
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
                           "CRC-64 lookup: sdwa+ds_read_b64+0.5x2 bitop3", "ds_read_b64 (16 KiB), 16 in flight",
                           "ds_read_b64 (128 KiB), 16 in flight", "ds_read_b128, 16 in flight",
                           "ds_read_b32, 16 in flight", "v_and_b32_sdwa (byte, UNUSED_PAD)",
                           "v_and_b32 (VOP2, SGPR mask)", "v_bfe_u32", "v_bitop3 (x & m) | c, SGPR mask",
                           "v_lshl_or_b32", "v_and_or_b32 (SGPR mask)", "v_alignbit_b32",
                           "v_bitop3 as bfi (SGPR mask)", "v_lshl_add_u32", "v_perm_b32 (SGPR selector)",
                           "v_and_b32_sdwa PRESERVE, VGPR mask", "v_and_b32_sdwa PAD, VGPR mask",
                           "v_and_b32 (VOP2, VGPR mask)", "v_xor_b32 (VOP2, SGPR operand)",
                           "v_bitop3 as bfi, VGPR mask", "v_and_b32 (VOP2, inline 63)", "v_lshlrev_b32 (VOP2)",
                           "v_or_b32 (VOP2, VGPR)"};
    double r[30];
    r[0] = run<0>(cus, sink, stamps);
    r[1] = run<1>(cus, sink, stamps);
    r[2] = run<2>(cus, sink, stamps);
    r[3] = run<3>(cus, sink, stamps);
    r[4] = run<4>(cus, sink, stamps);
    r[5] = run<5>(cus, sink, stamps);
    r[6] = run<6>(cus, sink, stamps);
    r[7] = run<7>(cus, sink, stamps);
    r[8] = run<8>(cus, sink, stamps);
    r[9] = run<9>(cus, sink, stamps);
    r[10] = run<10>(cus, sink, stamps);
    r[11] = run<11>(cus, sink, stamps);
    r[12] = run<12>(cus, sink, stamps);
    r[13] = run<13>(cus, sink, stamps);
    r[14] = run<14>(cus, sink, stamps);
    r[15] = run<15>(cus, sink, stamps);
    r[16] = run<16>(cus, sink, stamps);
    r[17] = run<17>(cus, sink, stamps);
    r[18] = run<18>(cus, sink, stamps);
    r[19] = run<19>(cus, sink, stamps);
    r[20] = run<20>(cus, sink, stamps);
    r[21] = run<21>(cus, sink, stamps);
    r[22] = run<22>(cus, sink, stamps);
    r[23] = run<23>(cus, sink, stamps);
    r[24] = run<24>(cus, sink, stamps);
    r[25] = run<25>(cus, sink, stamps);
    r[26] = run<26>(cus, sink, stamps);
    r[27] = run<27>(cus, sink, stamps);
    r[28] = run<28>(cus, sink, stamps);
    r[29] = run<29>(cus, sink, stamps);
    printf("shader cycles per wave-instruction per SIMD (4 waves/SIMD, %d CUs, %d chains x %d iterations):\n", cus,
           kChains, kIters);
    printf("(per SIMD; the CU's LDS serves 4 SIMDs: divide the LDS rows by 4 for cycles per read per CU)\n");
    for (int i = 0; i < 30; i++) printf("  %-44s %.2f\n", names[i], r[i]);
    (void)hipFree(sink);
    (void)hipFree(stamps);
    return 0;
}
