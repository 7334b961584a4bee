// mchecksum_gpu_ext.hip -- MI355X batch entry points next to the payload CRC
// (declared in include/mchecksum_gpu.h):
//
//  * mchecksum_gpu_checksum_segments -- the CRC of scatter-gather objects: a
//    bulk handle's segments (HG_Bulk_create(count, buf_ptrs, buf_sizes),
//    src/mercury_bulk.h:55,79) registered as device memory (hg_bulk_attr
//    mem_type HG_MEM_TYPE_ROCM, src/mercury_types.h:38,44-47), hashed as the
//    concatenation of its segments in order.  Mercury never checksums bulk
//    data today (src/mercury_core_types.h:68-69); this is what a receiver
//    would call to check a device-resident bulk transfer in one launch.
//  * mchecksum_gpu_verify_core_headers -- the CRC16 check of Mercury core
//    headers (hg_core_header_request_proc / _response_proc,
//    src/mercury_core_header.c:175-289) for a batch of received messages that
//    already sit in device memory.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "crc_gpu_device.h"
#include "gpu_host.h"
#include "mchecksum_gpu.h"
#include "mchecksum_models.h"

namespace {

// ------------------------------------------------------------ segments ----
//
// Object j = the concatenation of segments [first[j], first[j+1]).  By
// linearity (register form, crc_gpu_layout.h):
//   CRC(object) = Z^N(init) ^ XOR_c Z^(after_c)(L(chunk_c)) ^ xorout
// where chunks of at most kChunk bytes tile every segment, L is the CRC with
// zero init and no finalisation, N is the object's byte count and after_c the
// number of object bytes that follow chunk c.  Two launches after zeroing the
// output: one workgroup scans the segment lengths into byte and chunk prefix
// sums (caller's workspace); then persistent waves stride over chunks, compute
// L on 64 lanes with the payload kernels' step loop, shift it by after_c (at
// most 12 table-operator applications, base-16 digits) and XOR it into
// out[j] with an atomic -- XOR commutes, so the value is deterministic.  The
// same launch adds each object's Z^N(init) ^ xorout term.
//
// 256 KiB chunks: enough of them to fill the chip from a single GiB-sized
// segment, while the shift (a few us of dependent scalar loads) stays a few
// percent of a chunk's scan time.  A chunk that ends its object needs no shift.
constexpr uint64_t kChunk = 256u << 10;

struct SegArgs {
    const uint64_t *addr, *len;
    uint64_t nseg;
    const uint64_t *first;
    uint64_t nobj;
    const uint64_t *P, *C;  // workspace: byte / chunk exclusive prefix sums, nseg + 1 each
    void *out;
    const void *pack, *shift;
};

// Exclusive prefix sums of segment bytes (P) and chunk counts (C) -- one
// 1024-thread workgroup, 8 consecutive segments per thread per tile.
__global__ __launch_bounds__(1024) void seg_scan_kernel(const uint64_t *len, uint64_t nseg, uint64_t *P, uint64_t *C) {
    __shared__ uint64_t wp[16], wc[16];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint64_t carry_p = 0, carry_c = 0;
    for (uint64_t base = 0; base < nseg; base += 8192) {
        uint64_t lp[8], lc[8], sp = 0, sc = 0;
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const uint64_t i = base + t * 8u + e;
            const uint64_t l = i < nseg ? len[i] : 0;
            lp[e] = sp;
            lc[e] = sc;
            sp += l;
            sc += (l + kChunk - 1) / kChunk;
        }
        // inclusive wave scan of the thread sums
        uint64_t ip = sp, ic = sc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t op = __shfl_up(ip, d, 64), oc = __shfl_up(ic, d, 64);
            if (lane >= (uint32_t)d) {
                ip += op;
                ic += oc;
            }
        }
        if (lane == 63) {
            wp[w] = ip;
            wc[w] = ic;
        }
        __syncthreads();
        uint64_t bp = 0, bc = 0, tp = 0, tc = 0;  // waves before mine, tile total
        for (uint32_t v = 0; v < 16; v++) {
            if (v < w) {
                bp += wp[v];
                bc += wc[v];
            }
            tp += wp[v];
            tc += wc[v];
        }
        const uint64_t ep = carry_p + bp + ip - sp, ec = carry_c + bc + ic - sc;  // exclusive, this thread
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const uint64_t i = base + t * 8u + e;
            if (i < nseg) {
                P[i] = ep + lp[e];
                C[i] = ec + lc[e];
            }
        }
        carry_p += tp;
        carry_c += tc;
        __syncthreads();
    }
    if (t == 0) {
        P[nseg] = carry_p;
        C[nseg] = carry_c;
    }
}

// Z^n(x) from the base-16 digit tables; n and x are wave-uniform on the chunk
// path, so the table words come through the scalar cache.
__device__ __forceinline__ uint32_t shift32(const crc32_shift_pack_t *sp, uint32_t x, uint64_t n) {
    for (int k = 0; n; k++, n >>= 4) {
        const uint32_t d = (uint32_t)(n & 15u);
        if (d) {
            const uint32_t *t = &sp->op[k][d - 1][0][0];
            uint32_t r = 0;
#pragma unroll
            for (int h = 0; h < 8; h++) r ^= t[h * 16 + ((x >> (4 * h)) & 15u)];
            x = r;
        }
    }
    return x;
}

__device__ __forceinline__ uint64_t shift64(const crc64_shift_pack_t *sp, uint64_t x, uint64_t n) {
    for (int k = 0; n; k++, n >>= 4) {
        const uint32_t d = (uint32_t)(n & 15u);
        if (d) {
            const uint64_t *t = &sp->op[k][d - 1][0][0];
            uint64_t r = 0;
#pragma unroll
            for (int h = 0; h < 16; h++) r ^= t[h * 16 + ((x >> (4 * h)) & 15u)];
            x = r;
        }
    }
    return x;
}

// (readfirstlane returns int: cast through uint32_t so nothing sign-extends)
__device__ __forceinline__ uint32_t uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform(uint64_t v) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return (uint64_t)hi << 32 | lo;
}

// A wave's contiguous range of chunks [c, c1), walked in order.  The segment
// and object indices only advance, so a chunk costs a few cached scalar loads
// instead of two binary searches (~30 dependent loads); chunks are at most
// 256 KiB, so equal chunk counts are near-equal bytes.
struct ChunkWalk {
    const SegArgs *a;
    uint64_t c, c1, s, j;

    __device__ ChunkWalk(const SegArgs &args, uint32_t wave, uint32_t nw, uint64_t nchunks) : a(&args) {
        c = nchunks * wave / nw;
        c1 = nchunks * (wave + 1) / nw;
        s = c < c1 ? lower_bound_u64(a->C, a->nseg + 1, c + 1) - 1 : 0;
        j = c < c1 && s >= a->first[0] ? lower_bound_u64(a->first, a->nobj + 1, s + 1) - 1 : 0;
    }

    // Next chunk: its bytes [addr, addr + n) and, when its segment belongs to
    // an object (*in), the object and the object bytes that follow it.
    __device__ bool next(uint64_t *addr, uint64_t *n, bool *in, uint64_t *obj, uint64_t *after) {
        if (c >= c1) return false;
        while (a->C[s + 1] <= c) s++;  // skips empty segments
        const uint64_t off = (c - a->C[s]) * kChunk, L = a->len[s];
        *addr = a->addr[s] + off;
        *n = L - off < kChunk ? L - off : kChunk;
        *in = s >= a->first[0] && s < a->first[a->nobj];
        if (*in) {
            while (a->first[j + 1] <= s) j++;
            *obj = j;
            *after = a->P[a->first[j + 1]] - (a->P[s] + off + *n);
        }
        c++;
        return true;
    }
};

// PART 0: every chunk + the object terms (CRC-32C: 140 KiB of LDS, one
// workgroup per CU either way).  CRC-64 splits the chunks by shape: PART 1
// takes the aligned ones with two workgroups per CU (8 waves/SIMD: the
// VALU/LDS-bound loop needs them, and <= 64 VGPRs only fits the aligned
// loop), PART 2 the ragged ones and the object terms.
// (keyed W * 4 + PART: a comma inside __launch_bounds__ splits the macro)
template <int KEY>
constexpr int kSegWavesPerEU = KEY == 64 * 4 + 1 ? 8 : 1;

template <int W, int PART>
__global__ __launch_bounds__(1024, kSegWavesPerEU<W * 4 + PART>) void seg_kernel(SegArgs a) {
    constexpr int kWPB = 1024 / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWPB + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * kWPB;
    const uint64_t nchunks = a.C[a.nseg];
    if constexpr (W == 32) {
        __shared__ __attribute__((aligned(16))) uint8_t lds_raw[kL32Bytes];
        const crc32_gpu_pack_t *pk = reinterpret_cast<const crc32_gpu_pack_t *>(a.pack);
        const crc32_shift_pack_t *sp = reinterpret_cast<const crc32_shift_pack_t *>(a.shift);
        fill_lds32<false, 1024>(lds_raw, pk);
        __syncthreads();
        const Tab32<false> lds{lds_raw};
        const uint32_t lc0 = (lane & 31u) << 2, lc1 = lc0 | 0x10000u;
        uint32_t *out = reinterpret_cast<uint32_t *>(a.out);
        ChunkWalk walk(a, wave, nw, nchunks);
        uint64_t p, n, j, after;
        bool in;
        while (walk.next(&p, &n, &in, &j, &after)) {
            if (!in) continue;
            const uint8_t *q = reinterpret_cast<const uint8_t *>(p);
            // whole 1 KiB steps from a 16-B aligned start (the usual bulk
            // segment) take the aligned loop: no edge masks, no pad operator
            uint32_t x = p % 16 == 0 && n % 1024 == 0
                             ? payload32_aligned<6, false>(lds, q, n >> 10, lane, lc0, lc1, 0u)
                             : payload32_g64<false, Tab32<false>, true>(lds, pk, q, n, lane, lc0, lc1);
            x = shift32(sp, uniform(x), after);
            if (lane == 0) atomicXor(out + j, x);
        }
        for (uint64_t j = (uint64_t)blockIdx.x * 1024 + threadIdx.x; j < a.nobj; j += (uint64_t)gridDim.x * 1024) {
            const uint64_t N = a.P[a.first[j + 1]] - a.P[a.first[j]];
            atomicXor(out + j, shift32(sp, pk->init, N) ^ pk->xorout);
        }
    } else {
        __shared__ __attribute__((aligned(16))) uint8_t lds[kL64Bytes];
        const crc64_gpu_pack_t *pk = reinterpret_cast<const crc64_gpu_pack_t *>(a.pack);
        const crc64_shift_pack_t *sp = reinterpret_cast<const crc64_shift_pack_t *>(a.shift);
        fill_lds64<1024, false>(lds, pk);
        __syncthreads();
        const uint32_t lc = (lane & 31u) << 3;
        unsigned long long *out = reinterpret_cast<unsigned long long *>(a.out);
        ChunkWalk walk(a, wave, nw, nchunks);
        uint64_t p, n, j, after;
        bool in;
        while (walk.next(&p, &n, &in, &j, &after)) {
            if (!in) continue;
            const uint8_t *q = reinterpret_cast<const uint8_t *>(p);
            const bool aligned = p % 16 == 0 && n % 1024 == 0;
            if (aligned != (PART == 1)) continue;
            uint64_t x;
            if constexpr (PART == 1)
                x = payload64_aligned<6, false, false>(lds, pk, q, (uint32_t)(n >> 10), lane, lc, 0ull);
            else
                x = payload64_g64<false, true>(lds, pk, q, n, lane, lc);
            x = shift64(sp, uniform(x), after);
            if (lane == 0) atomicXor(out + j, (unsigned long long)x);
        }
        if constexpr (PART == 1) return;
        for (uint64_t j = (uint64_t)blockIdx.x * 1024 + threadIdx.x; j < a.nobj; j += (uint64_t)gridDim.x * 1024) {
            const uint64_t N = a.P[a.first[j + 1]] - a.P[a.first[j]];
            atomicXor(out + j, (unsigned long long)(shift64(sp, pk->init, N) ^ pk->xorout));
        }
    }
}

// --------------------------------------------------------- core headers ----
//
// Wire layout (hg_core_header_*_proc, src/mercury_core_header.c:175-289; the
// structs are 16 bytes, src/mercury_core_header.h:23-40, and a buffer shorter
// than that is rejected, :183-184 / :240-242):
//   request : hg u8 | protocol u8 | id u64 big-endian | flags u8 | cookie u8 | hash u16 BE at 12
//   response: ret_code i8 | flags u8 | cookie u16 BE | hash u16 BE at 4
// The CRC runs over the HOST-order field values as the proc code feeds them to
// mchecksum_update (HG_CORE_HEADER_CHECKSUM_UPDATE, :48-55): request
// hg, protocol, id (8 little-endian bytes), flags, cookie = 12 bytes; response
// ret_code, flags, cookie (2 little-endian bytes) = 4 bytes.
constexpr uint32_t kHdrSize = 16;

struct HdrArgs {
    const uint8_t *buf;
    const uint64_t *off;
    uint64_t count;
    uint8_t *status;
    uint32_t *mism;
    const uint16_t *table;  // byte table of the 16-bit model
    uint32_t kind, reflected, init, xorout;
};

__global__ __launch_bounds__(256) void core_header_kernel(HdrArgs a) {
    __shared__ uint16_t T[256];
    T[threadIdx.x] = a.table[threadIdx.x];
    __syncthreads();
    for (uint64_t m = (uint64_t)blockIdx.x * 256 + threadIdx.x; m < a.count; m += (uint64_t)gridDim.x * 256) {
        const uint64_t o = a.off[m];
        const bool whole = a.off[m + 1] - o >= kHdrSize;
        const uint8_t *h = a.buf + o;
        uint8_t img[12];
        uint32_t n, wire = 0;
        if (!whole) {
            n = 0;
        } else if (a.kind == MCHECKSUM_GPU_CORE_HEADER_REQUEST) {
            img[0] = h[0];
            img[1] = h[1];
#pragma unroll
            for (int b = 0; b < 8; b++) img[2 + b] = h[9 - b];  // big-endian on the wire, host LE image
            img[10] = h[10];
            img[11] = h[11];
            wire = (uint32_t)h[12] << 8 | h[13];
            n = 12;
        } else {
            img[0] = h[0];
            img[1] = h[1];
            img[2] = h[3];
            img[3] = h[2];
            wire = (uint32_t)h[4] << 8 | h[5];
            n = 4;
        }
        uint32_t r = a.init;
        if (a.reflected) {
            for (uint32_t i = 0; i < n; i++) r = (r >> 8) ^ T[(r ^ img[i]) & 0xFFu];
        } else {
            for (uint32_t i = 0; i < n; i++) r = ((r << 8) ^ T[((r >> 8) ^ img[i]) & 0xFFu]) & 0xFFFFu;
        }
        const bool bad = !whole || ((r ^ a.xorout) & 0xFFFFu) != wire;
        if (a.status) a.status[m] = bad ? 1 : 0;
        if (bad && a.mism) atomicAdd(a.mism, 1u);
    }
}

}  // namespace

// ------------------------------------------------------------ host side ----

namespace mck {

// Per-device, per-model extension tables (shift pack for 32/64-bit models,
// byte table for 16-bit ones), built and uploaded once under g_mu.
static int get_ext(DevCtx *c, int idx, const void **out) {
    if (c->ext[idx]) {
        *out = c->ext[idx];
        return 0;
    }
    const mck_model_t &m = mck_models[idx];
    size_t bytes = 0;
    void *host = nullptr;
    int rc = -1;
    if (m.width == 16) {
        bytes = 256 * sizeof(uint16_t);
        uint16_t *t = (uint16_t *)calloc(256, sizeof(uint16_t));
        host = t;
        if (t) {
            const uint32_t rp = (uint32_t)mck_reflect(m.poly, 16);
            for (uint32_t i = 0; i < 256; i++) {
                uint32_t r;
                if (m.reflected) {
                    r = i;
                    for (int k = 0; k < 8; k++) r = r & 1u ? (r >> 1) ^ rp : r >> 1;
                } else {
                    r = i << 8;
                    for (int k = 0; k < 8; k++) r = (r & 0x8000u ? (r << 1) ^ (uint32_t)m.poly : r << 1) & 0xFFFFu;
                }
                t[i] = (uint16_t)r;
            }
            rc = 0;
        }
    } else {
        crc_rmodel_t rm;
        rm.width = m.width;
        rm.rpoly = mck_reflect(m.poly, m.width);
        rm.rinit = mck_reflect(m.init, m.width);
        rm.xorout = m.xorout;
        bytes = m.width == 32 ? sizeof(crc32_shift_pack_t) : sizeof(crc64_shift_pack_t);
        host = calloc(1, bytes);
        if (host)
            rc = m.width == 32 ? crc32_shift_pack_build(&rm, (crc32_shift_pack_t *)host)
                               : crc64_shift_pack_build(&rm, (crc64_shift_pack_t *)host);
    }
    if (rc != 0) {
        free(host);
        return set_err(MCHECKSUM_GPU_EINVAL, "table build failed for %s", m.name);
    }
    void *d = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e == hipSuccess) e = hipMemcpy(d, host, bytes, hipMemcpyHostToDevice);
    free(host);
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        return hip_err(e, "table upload");
    }
    c->ext[idx] = d;
    *out = d;
    return 0;
}

}  // namespace mck

using namespace mck;

extern "C" {

size_t mchecksum_gpu_segments_work_size(size_t nseg) { return 2 * sizeof(uint64_t) * (nseg + 1); }

int mchecksum_gpu_checksum_segments(const char *hash_method, const uint64_t *dev_seg_addr,
                                    const uint64_t *dev_seg_len, size_t nseg, const uint64_t *dev_obj_first,
                                    size_t nobj, void *dev_work, size_t work_size, void *dev_out, void *stream) {
    if (!dev_obj_first || (nobj && !dev_out) || (nseg && (!dev_seg_addr || !dev_seg_len)) || !dev_work)
        return set_err(MCHECKSUM_GPU_EINVAL, "NULL pointer argument");
    if (work_size < mchecksum_gpu_segments_work_size(nseg) || (uintptr_t)dev_work % 8)
        return set_err(MCHECKSUM_GPU_EINVAL, "workspace smaller than mchecksum_gpu_segments_work_size() or unaligned");
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    int width = 0;
    DevCtx *c = nullptr;
    const void *pack = nullptr, *shift = nullptr;
    int rc = prologue(hash_method, CRC_GPU_MAX_LOG2G, &width, &c, &pack);
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        rc = get_ext(c, mck_model_index(hash_method), &shift);
    }
    if (rc) return rc;
    if (nobj == 0) return MCHECKSUM_GPU_OK;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(dev_out, 0, nobj * (size_t)(width / 8), s);
    if (e != hipSuccess) return hip_err(e, "hipMemsetAsync");
    SegArgs a{};
    a.addr = dev_seg_addr;
    a.len = dev_seg_len;
    a.nseg = nseg;
    a.first = dev_obj_first;
    a.nobj = nobj;
    a.P = (const uint64_t *)dev_work;
    a.C = (const uint64_t *)dev_work + (nseg + 1);
    a.out = dev_out;
    a.pack = pack;
    a.shift = shift;
    hipLaunchKernelGGL(seg_scan_kernel, dim3(1), dim3(1024), 0, s, dev_seg_len, (uint64_t)nseg, (uint64_t *)a.P,
                       (uint64_t *)a.C);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_err(e, "segment scan launch");
    if (width == 32) {
        hipLaunchKernelGGL((seg_kernel<32, 0>), dim3(c->cus), dim3(1024), 0, s, a);
    } else {
        hipLaunchKernelGGL((seg_kernel<64, 1>), dim3(2 * c->cus), dim3(1024), 0, s, a);
        e = hipGetLastError();
        if (e != hipSuccess) return hip_err(e, "segment kernel launch");
        hipLaunchKernelGGL((seg_kernel<64, 2>), dim3(c->cus), dim3(1024), 0, s, a);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return hip_err(e, "segment kernel launch");
    return MCHECKSUM_GPU_OK;
}

int mchecksum_gpu_verify_core_headers(const char *hash_method, int kind, const void *dev_buf,
                                      const uint64_t *dev_msg_offsets, size_t count, uint8_t *dev_status,
                                      uint32_t *dev_mismatches, void *stream) {
    if ((count && !dev_buf) || !dev_msg_offsets) return set_err(MCHECKSUM_GPU_EINVAL, "NULL pointer argument");
    if (kind != MCHECKSUM_GPU_CORE_HEADER_REQUEST && kind != MCHECKSUM_GPU_CORE_HEADER_RESPONSE)
        return set_err(MCHECKSUM_GPU_EINVAL, "unknown core header kind %d", kind);
    const int idx = mck_model_index(hash_method);
    if (idx < 0)
        return set_err(MCHECKSUM_GPU_EMETHOD, "unknown hash method \"%s\"", hash_method ? hash_method : "(null)");
    const mck_model_t &m = mck_models[idx];
    if (m.width != 16)
        return set_err(MCHECKSUM_GPU_EMETHOD, "core headers carry a 16-bit hash: \"%s\" is not a crc16 model",
                       hash_method);
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    DevCtx *c = nullptr;
    const void *table = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        int rc = device_ctx(&c);
        if (rc) return rc;
        rc = get_ext(c, idx, &table);
        if (rc) return rc;
    }
    if (count == 0) return MCHECKSUM_GPU_OK;
    HdrArgs a{};
    a.buf = (const uint8_t *)dev_buf;
    a.off = dev_msg_offsets;
    a.count = count;
    a.status = dev_status;
    a.mism = dev_mismatches;
    a.table = (const uint16_t *)table;
    a.kind = (uint32_t)kind;
    a.reflected = (uint32_t)m.reflected;
    a.init = (uint32_t)(m.reflected ? mck_reflect(m.init, 16) : m.init);
    a.xorout = (uint32_t)m.xorout;
    uint64_t blocks = (count + 255) / 256;
    if (blocks > (uint64_t)c->cus * 8) blocks = (uint64_t)c->cus * 8;
    hipLaunchKernelGGL(core_header_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_err(e, "core header kernel launch");
    return MCHECKSUM_GPU_OK;
}

}  // extern "C"
