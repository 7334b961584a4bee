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
//  * mchecksum_gpu_checksum_xdr -- the proc checksum of messages serialized in
//    XDR mode (HG_HAS_XDR, src/mercury_proc.h:110-122,147-160), where the
//    buffer holds big-endian, 4-byte-rounded XDR but the checksum covers the
//    host-order field values: a per-field schema says how to undo the XDR.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <type_traits>

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
// number of object bytes that follow chunk c.  Short scan launches write the
// segment lengths' byte and chunk prefix sums (caller's workspace) and preset
// out[j] = init ^ xorout (the CRC of an empty object); then persistent waves
// take chunks, compute L on 64 lanes with the payload kernels' step loop,
// shift it by after_c (at most 12 table-operator applications, base-16
// digits) and XOR it into out[j] with an atomic -- XOR commutes, so the value
// is deterministic.  The chunk that starts its object (object offset 0) runs
// its step loop from the register `init` instead of 0 (R(init, M) =
// R(0, M ^ init): init rides in its first W/8 bytes, or Z^n(init) is added
// for a chunk shorter than that) and XORs init once more, cancelling the
// preset's: Z^after(Z^n(init)) = Z^N(init), so the object term costs nothing
// (round 3 added it in a launch of its own: ~6 us per call, plus a kernel
// boundary).
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
    const unsigned long long *ragged;  // workspace: non-zero if any chunk needs the ragged loop
    // workspace: per segment s, {its object j (kNoObj outside [first[0],
    // first[nobj])), first[j], first[j + 1], the object's head segment (its
    // first non-empty one; kNoObj when the scan block could not tell)} (4
    // words: one scalar load in the queue pass), and the segment of each chunk
    // while the chunks fit map_cap
    const uint64_t *obj;
    const uint32_t *map;
    uint64_t map_cap;
    void *out;
    const void *pack, *shift;
    // work-queue slot of the chunk passes (crc_gpu_device.h, WgQueue; nullptr:
    // static split) and the caller's fail-closed word
    unsigned long long *queue;
    uint32_t *err_word;
    // the scan's fault report of this call (ScanArgs): claim == scan_key(epoch,
    // *gen - 1) means the scan gave up, so the chunk pass hashes nothing
    const uint64_t *fault_claim, *gen;
    uint64_t epoch;
};

// Exclusive prefix sums of segment bytes (P) and chunk counts (C), each
// segment's object, the chunk -> segment map and the ragged flag, in ONE
// launch over scan blocks of kScanBlk segments (round 4; one workgroup
// streams only ~20 GB/s, so a single-workgroup scan of 32768 segments took
// 48 us).  A block scans its own segments, publishes its aggregate, and finds
// its offset by a decoupled look-back over the blocks before it: one wave
// reads 64 predecessors' descriptors at once and sums aggregates back to the
// nearest published inclusive prefix, then publishes its own inclusive prefix.
// Descriptors carry the call's epoch (a process-wide counter from a random
// seed), so a workspace left by an earlier call needs no clearing.  The wait
// depends only on blocks dispatched before this one (a kernel's workgroups
// are dispatched in order and run to completion), and is bounded: a give-up
// is counted as a queue fault and reported on the caller's error word.
// The totals also flag segments whose chunks cannot all take the aligned loop
// (start not 16-B aligned or length not a multiple of 1 KiB).  The same
// launch presets out[j] = init ^ xorout.  Round 3 ran this as a block-reduce
// launch and a block-offset launch (4.8 + 8.5 us at 32768 segments, beside a
// kernel boundary), round 2 as three.  (1 or 2 segments per scan thread --
// 4x / 2x the scan blocks -- measured +-0.1% on the bench's 32768-segment
// lists, profiles/r05/scan_per/.)
constexpr uint32_t kScanThreads = 256, kScanPer = 4, kScanBlk = kScanThreads * kScanPer;
constexpr uint32_t kDescWords = 8;  // per scan block: flag, aggregate (p, c, r), inclusive (p, c, r), pad

__device__ __forceinline__ uint64_t seg_chunks(uint64_t l) { return (l + kChunk - 1) / kChunk; }

// Block-wide inclusive scan of (p, c) over the first 256 threads (a wider
// block's other threads only take part in the barrier); returns the block
// totals through *tp, *tc.
__device__ __forceinline__ void block_scan2(uint64_t &p, uint64_t &c, uint64_t *tp, uint64_t *tc) {
    __shared__ uint64_t wp[4], wc[4];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    if (w < kScanThreads / 64) {
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t op = __shfl_up(p, d, 64), oc = __shfl_up(c, d, 64);
            if (lane >= (uint32_t)d) {
                p += op;
                c += oc;
            }
        }
        if (lane == 63) {
            wp[w] = p;
            wc[w] = c;
        }
    }
    __syncthreads();
    if (w >= kScanThreads / 64) return;
    uint64_t bp = 0, bc = 0, sp = 0, sc = 0;
#pragma unroll
    for (uint32_t v = 0; v < kScanThreads / 64; v++) {
        if (v < w) {
            bp += wp[v];
            bc += wc[v];
        }
        sp += wp[v];
        sc += wc[v];
    }
    p += bp;
    c += bc;
    *tp = sp;
    *tc = sc;
}

constexpr uint64_t kNoObj = ~0ull;

// One wave: the largest index j < n with a[j] <= key (a sorted ascending,
// a[0] <= key), by 64-ary narrowing: each round probes 64 evenly spaced
// entries at once (3 rounds of loads for n = 8193 instead of 13 dependent ones).
__device__ __forceinline__ uint64_t wave_last_le(const uint64_t *a, uint64_t n, uint64_t key, uint32_t lane) {
    uint64_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t idx = lo + (uint64_t)lane * step;
        const unsigned long long m = __ballot(idx < hi && a[idx] <= key);
        const uint64_t L = 63u - (uint32_t)__builtin_clzll(m);  // lane 0 (a[lo] <= key) is always set
        lo += L * step;
        hi = lo + step < hi ? lo + step : hi;
    }
    return lo;
}

// (readfirstlane returns int: cast through uint32_t so nothing sign-extends)
__device__ __forceinline__ uint32_t uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform(uint64_t v) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Wave 0 of block b: publish (tp, tc, tr), look back, publish the inclusive
// prefix; returns the exclusive prefix (bytes, chunks, ragged) in every lane.
// false: the bounded wait gave up (fault counted).
__device__ __forceinline__ bool seg_lookback(uint64_t *desc, uint64_t b, uint64_t epoch, uint64_t tp, uint64_t tc,
                                             uint64_t tr, uint32_t lane, uint64_t *ep, uint64_t *ec, uint64_t *er,
                                             uint64_t fault_block) {
    uint64_t *me = desc + kDescWords * b;
#if MCK_QFAULT_TEST
    // injected stall (MCHECKSUM_GPU_QFAULT_MODE=scanstall): this block never
    // publishes, so every later block waits out its deadline
    const bool mute = (g_mck_qfault_mode & 2u) && b == fault_block;
#else
    constexpr bool mute = false;
#endif
    if (lane == 0 && !mute) {
        st_relaxed(me + 1, tp);
        st_relaxed(me + 2, tc);
        st_relaxed(me + 3, tr);
        if (b == 0) {
            st_relaxed(me + 4, tp);
            st_relaxed(me + 5, tc);
            st_relaxed(me + 6, tr);
        }
        __hip_atomic_store(me, epoch * 4 + (b == 0 ? 2u : 1u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t sp = 0, sc = 0, sr = 0;
    bool ok = true;
    if (b > 0) {
        int64_t k = (int64_t)b - 1;  // window: blocks k, k - 1, ..., k - 63 (lane order)
        Deadline dl;  // 1 s of real time (crc_gpu_device.h)
        for (;;) {
#if MCK_QFAULT_TEST
            if (b == fault_block && g_mck_qfault_mode == 0u) {  // injected give-up (test builds, MCHECKSUM_GPU_QFAULT_SCAN)
                if (lane == 0) queue_fault(11, b, 0);
                ok = false;
                break;
            }
#else
            (void)fault_block;
#endif
            const int64_t idx = k - (int64_t)lane;
            const uint64_t f = idx >= 0 ? ld_relaxed(desc + kDescWords * (uint64_t)idx) : epoch * 4 + 2;
            const uint32_t state = (f >> 2) == epoch ? (uint32_t)(f & 3u) : 0u;
            const unsigned long long incl = __ballot(state == 2), none = __ballot(state == 0);
            const uint32_t S = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;  // nearest inclusive prefix
            const unsigned long long below = S >= 64 ? ~0ull : ((1ull << S) - 1);
            if (none & below) {  // a nearer block has not published yet
                __builtin_amdgcn_s_sleep(1);
                if (dl.passed()) {
                    if (lane == 0) queue_fault(10, b, (uint64_t)k);
                    ok = false;
                    break;
                }
                continue;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            uint64_t vp = 0, vc = 0, vr = 0;
            if (idx >= 0 && lane <= S) {
                const uint64_t *d = desc + kDescWords * (uint64_t)idx + (lane == S ? 4 : 1);
                vp = ld_relaxed(d);
                vc = ld_relaxed(d + 1);
                vr = ld_relaxed(d + 2);
            }
            sp += wave_sum(vp);
            sc += wave_sum(vc);
            sr |= wave_sum(vr);
            if (S < 64) break;
            k -= 64;
        }
        if (lane == 0 && !mute) {
            st_relaxed(me + 4, sp + tp);
            st_relaxed(me + 5, sc + tc);
            st_relaxed(me + 6, sr | tr);
            __hip_atomic_store(me, epoch * 4 + 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    *ep = sp;
    *ec = sc;
    *er = sr ? 1u : 0u;
    return ok;
}

// Each segment's object (obj, the queue pass's map) without a per-segment
// search: waves 1 and 2 find the objects of the block's first and last
// segments (wave_last_le over first[]); a thread per object in between writes
// the object's index and bounds over its segments in LDS rows of the block
// (empty objects write nothing, so a segment gets the last object whose range
// starts at or before it), and every thread then reads its own segments'
// entries.  Round 3 ran a binary search over all of first[] in global memory
// per segment: ~14 dependent loads, 15 of the pass's 17 us at 32768 segments.
// The scan's arguments.
struct ScanArgs {
    const uint64_t *len, *addr;
    uint64_t nseg;
    uint64_t *desc;
    uint64_t epoch;
    uint64_t *P, *C;
    unsigned long long *ragged;
    const uint64_t *first;
    uint64_t nobj;
    uint64_t *obj;
    uint32_t *map;
    uint64_t map_cap;
    void *out;
    uint32_t width;
    uint64_t preset;
    uint32_t *err_word;
    uint64_t *fault_claim;  // workspace word: the call's key once a fault was reported
    uint64_t *gen;          // workspace word: calls scanned in this workspace (the key's second half)
    uint64_t fault_block;
};
// A call's key: its epoch and the workspace's call count.  A graph replays
// its captured epoch, so the epoch alone cannot tell two replays apart
// (ADVICE r5); the count moves on every scan, captured or not.
__device__ __forceinline__ uint64_t scan_key(uint64_t epoch, uint64_t gen) {
    return epoch ^ (gen * 0x9E3779B97F4A7C15ull) ^ 0xD1B54A32D192ED03ull;
}
// A call's scan-side give-ups (a look-back in any scan block) add 1 to the
// error word between them, as the header promises per call: the first to
// swap the call's key into the claim word reports, the rest see it already
// there -- and the chunk pass, seeing it, hashes nothing (fail closed, and
// no second deadline in the same call).
__device__ __forceinline__ void report_scan_fault(const ScanArgs &sa, uint64_t gen) {
    const uint64_t key = scan_key(sa.epoch, gen);
    const uint64_t was = __hip_atomic_exchange(sa.fault_claim, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (was != key && sa.err_word) atomicAdd(sa.err_word, 1u);
}
// LDS scratch of one scan block: the object rows of its segments (4 x u64 +
// u32 each) and a few broadcast words
constexpr uint32_t kScanScratch = kScanBlk * (4 * 8 + 4) + 64;

// Scan block b of nb (kScanThreads threads).
__device__ __forceinline__ void scan_block(const ScanArgs &sa, uint64_t b, uint64_t nb, uint8_t *scratch) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const bool act = tid < kScanThreads;
    const uint64_t nseg = sa.nseg, nobj = sa.nobj;
    const uint64_t s0 = b * kScanBlk, s1 = s0 + kScanBlk < nseg ? s0 + kScanBlk : nseg;
    uint64_t *row = reinterpret_cast<uint64_t *>(scratch);
    uint64_t *row_f0 = row + kScanBlk, *row_f1 = row_f0 + kScanBlk;  // the object's first[j], first[j + 1]
    uint64_t *row_hs = row_f1 + kScanBlk;                             // the object's head segment
    uint32_t *row_ne = reinterpret_cast<uint32_t *>(row_hs + kScanBlk);  // 1: the segment is not empty
    uint64_t *bc = reinterpret_cast<uint64_t *>(row_ne + kScanBlk);     // jb, je, ex[3]
    uint32_t *rag = reinterpret_cast<uint32_t *>(bc + 5);
    // every object starts as the CRC of the empty message (the chunk passes XOR into it)
    if (act)
        for (uint64_t j = b * kScanThreads + tid; j < nobj; j += nb * kScanThreads) {
            if (sa.width == 64) reinterpret_cast<uint64_t *>(sa.out)[j] = sa.preset;
            else reinterpret_cast<uint32_t *>(sa.out)[j] = (uint32_t)sa.preset;
        }
    uint64_t l[kScanPer], p = 0, c = 0, r = 0;
#pragma unroll
    for (uint32_t e = 0; e < kScanPer; e++) {
        const uint64_t i = s0 + tid * kScanPer + e;
        l[e] = act && i < nseg ? sa.len[i] : 0;
        p += l[e];
        c += seg_chunks(l[e]);
        r |= act && i < nseg && l[e] && (l[e] % 1024 != 0 || sa.addr[i] % 16 != 0);
    }
    // the objects touching this block (queue pass only)
    const uint64_t f0 = sa.first[0], f1 = sa.first[nobj];
    const uint64_t lo_s = s0 > f0 ? s0 : f0, hi_s = s1 < f1 ? s1 : f1;
    if (sa.obj && lo_s < hi_s) {
        if (w == 1) {
            const uint64_t jb = wave_last_le(sa.first, nobj + 1, lo_s, lane);
            if (lane == 0) bc[0] = jb;
        } else if (w == 2) {
            const uint64_t je = wave_last_le(sa.first, nobj + 1, hi_s - 1, lane);
            if (lane == 0) bc[1] = je;
        }
    }
    const uint64_t p0 = p, c0 = c;
    uint64_t tp = 0, tc = 0;
    block_scan2(p, c, &tp, &tc);
    if (tid == 0) *rag = 0;
    __syncthreads();
    if (act && __any(r != 0) && lane == 0) atomicOr(rag, 1u);
    __syncthreads();
    uint64_t *ex = bc + 2;
    if (w == 0) {
        // the workspace's call count, read before this block publishes: the
        // last block bumps it only after its look-back saw every block's
        // descriptor, so all blocks of the call read the same count
        const uint64_t gen = uniform(ld_relaxed(sa.gen));
        uint64_t ep, ec, er;
        const bool ok = seg_lookback(sa.desc, b, sa.epoch, tp, tc, *rag, lane, &ep, &ec, &er, sa.fault_block);
        if (lane == 0) {
            ex[0] = ep;
            ex[1] = ec;
            ex[2] = er;
            if (!ok) report_scan_fault(sa, gen);  // fail closed: the scan is not trustworthy
            if (b + 1 == nb) st_relaxed(sa.gen, gen + 1);
        }
    }
    __syncthreads();
    if (b + 1 == nb && tid == 0) {
        sa.P[nseg] = ex[0] + tp;
        sa.C[nseg] = ex[1] + tc;
        *sa.ragged = ex[2] | *rag;
    }
    uint64_t ep = ex[0] + p - p0, ec = ex[1] + c - c0;
    if (sa.obj) {
        if (act) {
            for (uint32_t t = tid; t < kScanBlk; t += kScanThreads) row[t] = kNoObj;
#pragma unroll
            for (uint32_t e = 0; e < kScanPer; e++) row_ne[tid * kScanPer + e] = l[e] != 0;
        }
        __syncthreads();
        if (act && lo_s < hi_s) {
            const uint64_t jb = bc[0], je = bc[1];
            for (uint64_t k = jb + tid; k <= je; k += kScanThreads) {
                const uint64_t a0 = sa.first[k], a1 = sa.first[k + 1];
                const uint64_t lo = a0 > lo_s ? a0 : lo_s, hi = a1 < hi_s ? a1 : hi_s;
                // the head segment is known here when the object starts in this
                // block and one of its segments here is not empty; otherwise
                // (kNoObj) the chunk pass compares byte offsets instead
                uint64_t hs = kNoObj;
                if (a0 >= s0)
                    for (uint64_t i = lo; i < hi; i++)
                        if (row_ne[i - s0]) {
                            hs = i;
                            break;
                        }
                for (uint64_t i = lo; i < hi; i++) {
                    row[i - s0] = k;
                    row_f0[i - s0] = a0;
                    row_f1[i - s0] = a1;
                    row_hs[i - s0] = hs;
                }
            }
        }
        __syncthreads();
    }
    if (!act) return;
#pragma unroll
    for (uint32_t e = 0; e < kScanPer; e++) {
        const uint64_t i = s0 + tid * kScanPer + e;
        if (i < nseg) {
            sa.P[i] = ep;
            sa.C[i] = ec;
            if (sa.obj) {
                const uint64_t t = i - s0;
                sa.obj[4 * i] = row[t];
                if (row[t] != kNoObj) {
                    sa.obj[4 * i + 1] = row_f0[t];
                    sa.obj[4 * i + 2] = row_f1[t];
                    sa.obj[4 * i + 3] = row_hs[t];
                }
            }
            // chunk -> segment map, while it fits (the chunk passes check the
            // total against map_cap and search C otherwise)
            const uint64_t ce = ec + seg_chunks(l[e]);
            if (ce <= sa.map_cap)
                for (uint64_t k = ec; k < ce; k++) sa.map[k] = (uint32_t)i;
        }
        ep += l[e];
        ec += seg_chunks(l[e]);
    }
}

__global__ __launch_bounds__(kScanThreads) void seg_scan(ScanArgs sa) {
    __shared__ __attribute__((aligned(16))) uint8_t scratch[kScanScratch];
    scan_block(sa, blockIdx.x, gridDim.x, scratch);
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
    // an object (*in), the object, the object bytes that follow it (*end -
    // *stop, as seg_locate) and whether it starts the object (*head).
    __device__ bool next(uint64_t *addr, uint64_t *n, bool *in, uint64_t *obj, uint64_t *end, uint64_t *stop,
                         bool *head) {
        if (c >= c1) return false;
        while (s < a->nseg && a->C[s + 1] <= c) s++;  // skips empty segments
        const uint64_t cs = s < a->nseg ? a->C[s] : ~0ull, L = s < a->nseg ? a->len[s] : 0;
        const uint64_t off = (c - cs) * kChunk;
        if (cs > c || off >= L) {  // maps of a failed scan (reported): skip, never read out of bounds
            *in = false;
            c++;
            return true;
        }
        *addr = a->addr[s] + off;
        *n = L - off < kChunk ? L - off : kChunk;
        *in = s >= a->first[0] && s < a->first[a->nobj];
        if (*in) {
            while (j + 1 < a->nobj && a->first[j + 1] <= s) j++;
            *obj = j;
            *end = a->P[a->first[j + 1]];
            *stop = a->P[s] + off + *n;
            *head = a->P[s] + off == a->P[a->first[j]];
        }
        c++;
        return true;
    }
};

// Work-queue chunk pass (CRC-64).  Chunks are the queue's units, so a wave
// holds chunks from anywhere in the list and needs each one's segment and
// object without walking: the scan writes both maps (SegArgs::obj, ::map), so
// a chunk costs three dependent scalar loads.  A list with more chunks than
// the map holds (segments far above 1 MiB on average) searches C instead.
// The first build searched C and first[] for every chunk (a guess plus a
// gallop): its search loops pushed the 64-VGPR CRC-64 pass into 54 SGPR / 10
// VGPR spills and it measured 5% slower than the static ranges
// (profiles/r02/ab_seg_queue.log).
//
// Chunk c (< nchunks): its bytes [addr, addr + n) and, when its segment
// belongs to an object (*in), the object, the object bytes after it (*end -
// *stop) and whether it starts the object (*head).  c is wave-uniform, so
// every load is scalar: the map, then the segment's words and its 4-word
// object record.  The object's end offset (*end) is a third dependent load,
// but the payload loop does not wait for it -- the caller subtracts only
// after the loop (round 4: the head test from the record's head segment
// instead of the object's start offset, a second third-round load).  Only a
// chunk whose object's head the scan block could not place compares byte
// offsets.  Locate latency is not what limits the pass: two rounds instead
// of three measured within noise, and so did a one-round locate of bench.py's
// seg layout from the chunk index alone; the same layout with a constant
// chunk length measured +1.6-2.5% -- the compile-time trip count gave the
// payload loop whole-ring code (payload64_even, crc_gpu_device.h), now taken
// for every chunk of whole rings (profiles/r04/ab_seg_locate_bound.log,
// ab_seg_cheats.log, ab_seg_full.log, ab_seg_head.log, ab_seg_even.log).
__device__ __forceinline__ void seg_locate(const SegArgs &a, uint64_t c, uint64_t nchunks, uint64_t *addr,
                                           uint64_t *n, bool *in, uint64_t *obj, uint64_t *end, uint64_t *stop,
                                           bool *head) {
    const uint64_t s = nchunks <= a.map_cap ? (uint64_t)a.map[c] : lower_bound_u64(a.C, a.nseg + 1, c + 1) - 1;
    // (a scan whose look-back gave up -- reported on the error word -- leaves
    // maps that may not fit: such a chunk is skipped, never read out of bounds)
    const uint64_t cs = s < a.nseg ? a.C[s] : ~0ull, L = s < a.nseg ? a.len[s] : 0;
    const uint64_t off = (c - cs) * kChunk;
    if (cs > c || off >= L) {
        *in = false;
        return;
    }
    *addr = a.addr[s] + off;
    *n = L - off < kChunk ? L - off : kChunk;
    const uint64_t *o4 = a.obj + 4 * s;  // {j, first[j], first[j + 1], head segment}
    const uint64_t j = o4[0];
    *in = j != kNoObj;
    if (*in) {
        *obj = j;
        const uint64_t at = a.P[s] + off;
        *end = a.P[o4[2]];
        *stop = at + *n;
        const uint64_t hs = o4[3];
        *head = hs != kNoObj ? hs == s && off == 0 : at == a.P[o4[1]];
    }
}

// The chunk passes, one launch after the scan: one 1024-thread workgroup per
// CU either way.  CRC-32C (140 KiB of LDS tables): each wave walks a static
// contiguous range of chunks (ChunkWalk).  CRC-64 (round 4, "merged"): every
// chunk from the work queue, the ragged loop beside the aligned one in 128
// VGPRs and every operator in LDS.  (Round 3 split the CRC-64 chunks by
// shape: the aligned ones at two workgroups per CU, the ragged ones in a
// launch of their own -- ~7 us per call even when it found none.  Round 5
// tried scanning inside the chunk pass for lists of one scan block: one
// launch per call, but slower per call -- the other workgroups wait on block
// 0's scan with an agent-scope acquire -- and not kept: HISTORY.md.)
constexpr uint64_t kSegNtBytes = 512ull << 20;

template <int W>
__global__ __launch_bounds__(1024, 1) void seg_kernel(SegArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_tab[W == 32 ? kL32Bytes : kL64Bytes];
    constexpr int kWPB = 1024 / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWPB + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * kWPB;
    const uint64_t nchunks = uniform(a.C[a.nseg]);
    // the CRC-64 pass takes chunks from the work queue (the host passes a
    // slot; without one, for_each_unit strides statically)
    constexpr bool kQueue = W == 64;
    __shared__ WgQueue wgq;
    if (kQueue && threadIdx.x == 0) wg_queue_init(&wgq, a.queue, nchunks);
    // the scan of this call gave up (reported on the error word): hash nothing
    // -- after the queue's init, which readies the slot's other bank
    if (uniform(ld_relaxed(a.fault_claim)) == scan_key(a.epoch, uniform(ld_relaxed(a.gen)) - 1)) return;
    // CRC-32C: calls body(addr, n, j, end, stop, head) for every chunk of
    // this wave's static range that belongs to an object.
    auto chunks = [&](auto &&body) -> bool {
        ChunkWalk walk(a, wave, nw, nchunks);
        uint64_t p, n, j = 0, end = 0, stop = 0;
        bool in, head = false;
        while (walk.next(&p, &n, &in, &j, &end, &stop, &head))
            if (in) body(p, n, j, end, stop, head);
        return false;
    };
    if constexpr (W == 32) {
        uint8_t *lds_raw = lds_tab;
        const crc32_gpu_pack_t *pk = reinterpret_cast<const crc32_gpu_pack_t *>(a.pack);
        const crc32_shift_pack_t *sp = reinterpret_cast<const crc32_shift_pack_t *>(a.shift);
        fill_lds32<false, 1024>(lds_raw, pk);
        __syncthreads();
        const Tab32<false> lds{lds_raw};
        const uint32_t lc0 = (lane & 31u) << 2, lc1 = lc0 | 0x10000u;
        uint32_t *out = reinterpret_cast<uint32_t *>(a.out);
        const bool nt = uniform(a.P[a.nseg]) >= kSegNtBytes;  // as for CRC-64 below
        const uint32_t init = pk->init;
        const bool faulted = chunks([&](uint64_t p, uint64_t n, uint64_t j, uint64_t end, uint64_t stop, bool head) {
            const uint8_t *q = reinterpret_cast<const uint8_t *>(p);
            // whole rings of 1 KiB steps from a 16-B aligned start (the usual
            // bulk segment) take the aligned loop: no edge masks, no pad operator
            const bool aligned = p % 16 == 0 && n % (1024u * kRing) == 0 && n != 0;
            // the object's first chunk starts from the register init (in its
            // first 4 bytes; Z^n(init) for a shorter chunk)
            const uint32_t reg = head && n >= 4 ? init : 0u;
            uint32_t x = aligned && nt    ? payload32_aligned<6, true>(lds, q, n >> 10, lane, lc0, lc1, reg)
                         : aligned        ? payload32_aligned<6, false>(lds, q, n >> 10, lane, lc0, lc1, reg)
                                          : payload32_g64<false, Tab32<false>, true>(lds, pk, q, n, lane, lc0, lc1, reg);
            x = uniform(x);
            if (head && n < 4) x ^= pk->zinit[n];
            x = shift32(sp, x, end - stop);  // (the object bytes after the chunk)
            if (lane == 0) atomicXor(out + j, head ? x ^ init : x);  // ^ init: cancels the preset's
        });
        if (faulted && lane == 0 && a.err_word) atomicAdd(a.err_word, 1u);
    } else {
        uint8_t *lds = lds_tab;
        const crc64_gpu_pack_t *pk = reinterpret_cast<const crc64_gpu_pack_t *>(a.pack);
        const crc64_shift_pack_t *sp = reinterpret_cast<const crc64_shift_pack_t *>(a.shift);
        fill_lds64<1024, kOpsLds>(lds, pk);
        __syncthreads();
        const uint32_t lc = (lane & 31u) << 3;
        unsigned long long *out = reinterpret_cast<unsigned long long *>(a.out);
        // Non-temporal payload loads once the batch is far larger than the
        // Infinity Cache, as for fixed batches.  Here the size is only known on
        // the device (the segment scan's total), so the choice is a uniform
        // branch per chunk: +3% on `seg` (duplicating the whole walk under one
        // branch measured the same and spills more).
        const bool nt = uniform(a.P[a.nseg]) >= kSegNtBytes;
        const uint64_t init = pk->init;
        // Pipelined (round 6, as the split CRC-64 pieces): a chunk of whole
        // rings from an aligned start (every chunk of a list of 16-B aligned
        // KiB-multiple segments) runs from a ring its predecessor loaded --
        // the wave takes the next chunk and issues its first loads as soon as
        // the current step loop ends, before the current chunk's lane combine,
        // Z^n shift and output XOR.  Other chunks run on their own.
        struct Chunk {
            uint64_t p = 0, n = 0, j = 0, end = 0, stop = 0;
            bool in = false, head = false, even = false;
        };
        auto locate = [&](uint64_t c, Chunk *k) {
            seg_locate(a, c, nchunks, &k->p, &k->n, &k->in, &k->j, &k->end, &k->stop, &k->head);
            k->even = k->in && k->p % 16 == 0 && k->n % (1024u * kRing64) == 0 && k->n >= 2048u * kRing64;
        };
        auto issue = [&](uint4 (&ring)[kRing64], const Chunk &k) {
            if (nt) ring64_load<true>(ring, reinterpret_cast<const uint8_t *>(k.p), lane);
            else ring64_load<false>(ring, reinterpret_cast<const uint8_t *>(k.p), lane);
        };
        UnitTaker<ChunkPlan> tk(&wgq, a.queue, nchunks, wave, nw, false, ChunkPlan(nchunks));
        Lane64 ln = lane64(lc);
        uint4 ring[kRing64];
        uint64_t c = 0;
        Chunk cur;
        bool have = tk.take_unit(&c);
        if (have) locate(c, &cur);
        if (have && cur.even) issue(ring, cur);
        while (have) {
            const uint8_t *q = reinterpret_cast<const uint8_t *>(cur.p);
            // the object's first chunk starts from the register init (in its
            // first 8 bytes; Z^n(init) for a shorter, ragged chunk)
            const uint64_t reg = cur.head && cur.n >= 8 ? init : 0ull;
            uint64_t x = 0, x0 = 0, x1 = 0;
            const bool aligned = cur.p % 16 == 0 && cur.n % 1024 == 0;
            if (cur.even) {
                if (nt) fold64_ring<true>(lds, ring, q, (uint32_t)(cur.n >> 10), lane, ln, reg, &x0, &x1);
                else fold64_ring<false>(lds, ring, q, (uint32_t)(cur.n >> 10), lane, ln, reg, &x0, &x1);
            } else if (cur.in && aligned) {
                x = payload64_aligned<6, false, kOpsLds>(lds, pk, q, (uint32_t)(cur.n >> 10), lane, lc, reg);
            } else if (cur.in) {
                x = payload64_g64<false, true>(lds, pk, q, cur.n, lane, lc, reg);
            }
            uint64_t cn = 0;
            Chunk nxt;
            const bool next = tk.take_unit(&cn);
            if (next) locate(cn, &nxt);
            if (next && nxt.even) issue(ring, nxt);  // in flight during the combine below
            if (cur.in) {
                if (cur.even) x = combine64<6, kOpsLds>(lds, pk, x0, x1, lane);
                x = uniform(x);
                if (!aligned && cur.head && cur.n < 8) x ^= pk->zinit[cur.n];
                x = shift64(sp, x, cur.end - cur.stop);  // (the object bytes after the chunk)
                if (lane == 0) atomicXor(out + cur.j, (unsigned long long)(cur.head ? x ^ init : x));  // ^ init: cancels the preset's
            }
            cur = nxt;
            have = next;
        }
        const bool faulted = tk.finish(wave);
        if (faulted && lane == 0 && a.err_word) atomicAdd(a.err_word, 1u);
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
    uint32_t nbad = 0;
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
        nbad += bad;
    }
    add_mismatches(a.mism, nbad);  // once per workgroup (crc_gpu_device.h)
}

// ------------------------------------------------------------------ XDR ----
//
// Under HG_HAS_XDR every typed field goes through xdr_<type>: RNDUP(sizeof)
// bytes on the wire -- a 1-, 2- or 4-byte integer as one big-endian 32-bit
// word (sign-extended for the signed types), an 8-byte integer as two
// big-endian words, high first -- while HG_PROC_CHECKSUM_UPDATE hashes the
// sizeof(type) bytes of the HOST variable (src/mercury_proc.h:110-122).  Byte
// arrays go through xdr_opaque: the bytes, then zero pad to a multiple of 4,
// with only the bytes hashed (:147-160).  hg_proc_save_ptr/restore_ptr regions
// (bulk handles, src/mercury_proc_bulk.c:91-125) are raw at their exact size
// (src/mercury_proc.c:277-335).  So a whole-buffer CRC is wrong in XDR mode;
// this kernel walks a per-message field schema instead.  The hashed stream of
// a little-endian host is, per field: the low `size` bytes of the decoded
// integer in little-endian order, or the raw bytes of an opaque/raw field.
//
// One wave per message, the schema walk wave-uniform (the schema rides in the
// kernel arguments).  The register L of the hashed stream starts at the
// model's initial value and is built field by field: an integer updates it
// byte by byte from an LDS byte table; an opaque or raw field of n bytes is
// cut into 64 lane ranges hashed byte by byte, each shifted past the bytes
// after it (Z^k from the base-16 digit tables) and XOR-reduced over the
// wave, then L <- Z^n(L) ^ that.  CRC = L ^ xorout.
//
// Large batches (the throughput layout, round 3) run the same walk in
// persistent 1024-thread workgroups that also hold the payload kernels' LDS
// tables: an opaque or raw field of >= kXdrFastMin bytes is hashed by the
// payload step loop (coalesced 1 KiB steps, payload32_g64 / payload64_g64 in
// RAW form: zero init, no finalisation) instead of 64 byte-serial lane
// ranges, and messages come from the work queue (crc_gpu_device.h).  The
// step loop starts from the running register itself (it rides in the field's
// first bytes, R(L, M) = R(0, M ^ L)), so such a field needs no Z^n shift:
// an iovec message (hg_perf_proc_iovec, Testing/perf/hg/mercury_perf.c:897-923:
// a u32 length, then the bytes) costs its 4-byte table walk plus what the
// same payload costs through the offsets kernel -- no dependent chain of
// digit-table loads per message (round 3: two Z^n shifts per message before).
constexpr uint32_t kXdrMaxFields = 64;
constexpr uint64_t kXdrFastMin = 256;

struct XdrArgs {
    const uint8_t *buf;
    const uint64_t *off;
    uint64_t count;
    void *out;
    uint8_t *status;
    const void *shift;
    const void *pack;                // throughput kernel: the model's G = 64 table pack
    unsigned long long *queue;       // throughput kernel: work-queue slot (nullptr: static split)
    uint32_t *err_word;              // throughput kernel: fail-closed report
    uint64_t rpoly, init, xorout;
    uint32_t nf;
    uint32_t kind[kXdrMaxFields], size[kXdrMaxFields];
};

template <int W>
using xdr_reg_t = typename std::conditional<W == 32, uint32_t, uint64_t>::type;

template <int W>
__device__ __forceinline__ xdr_reg_t<W> xdr_shift(const void *sp, xdr_reg_t<W> x, uint64_t n) {
    if constexpr (W == 32) return shift32(reinterpret_cast<const crc32_shift_pack_t *>(sp), x, n);
    else return shift64(reinterpret_cast<const crc64_shift_pack_t *>(sp), x, n);
}

// Byte table of the register form (Z^1 of the low byte) for entry t < 256.
template <int W>
__device__ __forceinline__ xdr_reg_t<W> xdr_tab_entry(uint64_t rpoly, uint32_t t) {
    using R = xdr_reg_t<W>;
    R r = (R)t;
    for (int k = 0; k < 8; k++) r = (r & 1u) ? (r >> 1) ^ (R)rpoly : r >> 1;
    return r;
}

// One message (one wave, wave-uniform walk): writes out[m] and status[m].
// fast(p, len, &L) may hash an opaque/raw field of len bytes at p itself,
// continuing the running register L (returning true); otherwise 64 lane
// ranges are hashed byte by byte and combined into L.
template <int W, class Fast>
__device__ __forceinline__ void xdr_message(const XdrArgs &a, uint64_t m, const xdr_reg_t<W> *tab, uint32_t lane,
                                            Fast &&fast) {
    using R = xdr_reg_t<W>;
    uint64_t pos = a.off[m];
    const uint64_t end = a.off[m + 1];
    R acc = (R)a.init;
    uint64_t last = 0;
    bool bad = end < pos;
    for (uint32_t f = 0; f < a.nf && !bad; f++) {
        const uint32_t kind = a.kind[f], sz = a.size[f];
        if (kind == MCHECKSUM_XDR_SKIP_IF_ZERO) {
            if (last == 0) f += sz;
            continue;
        }
        if (kind == MCHECKSUM_XDR_INT) {
            const uint32_t slot = sz <= 4 ? 4u : 8u;
            if (end - pos < slot) {
                bad = true;
                break;
            }
            uint64_t v = 0;
            for (uint32_t b = 0; b < slot; b++) v = v << 8 | a.buf[pos + b];
            for (uint32_t b = 0; b < sz; b++) acc = (acc >> 8) ^ tab[(uint32_t)(acc ^ (R)(v >> (8 * b))) & 0xFFu];
            last = sz == 8 ? v : v & ((1ull << (8 * sz)) - 1);
            pos += slot;
            continue;
        }
        const bool raw = kind == MCHECKSUM_XDR_RAW || kind == MCHECKSUM_XDR_RAW_LEN;
        const uint64_t len = (kind == MCHECKSUM_XDR_OPAQUE_LEN || kind == MCHECKSUM_XDR_RAW_LEN) ? last : sz;
        if (len > end - pos || (!raw && ((len + 3) & ~3ull) > end - pos)) {
            bad = true;
            break;
        }
        if (!fast(a.buf + pos, len, &acc)) {
            R p = 0;
            const uint64_t chunk = (len + 63) / 64;
            const uint64_t lo = lane * chunk < len ? lane * chunk : len, hi = lo + chunk < len ? lo + chunk : len;
            for (uint64_t i = lo; i < hi; i++) p = (p >> 8) ^ tab[(uint32_t)(p ^ a.buf[pos + i]) & 0xFFu];
            p = xdr_shift<W>(a.shift, p, len - hi);
#pragma unroll
            for (int k = 1; k < 64; k <<= 1) p ^= __shfl_xor(p, k, 64);
            acc = xdr_shift<W>(a.shift, acc, len) ^ p;
        }
        pos += raw ? len : (len + 3) & ~3ull;
    }
    if (lane == 0) {
        const R crc = bad ? (R)0 : acc ^ (R)a.xorout;
        reinterpret_cast<R *>(a.out)[m] = crc;
        if (a.status) a.status[m] = bad ? 1 : 0;
    }
}

// Latency layout (small batches): 256-thread workgroups, a byte table only.
template <int W>
__global__ __launch_bounds__(256) void xdr_kernel(XdrArgs a) {
    using R = xdr_reg_t<W>;
    __shared__ R tab[256];
    tab[threadIdx.x] = xdr_tab_entry<W>(a.rpoly, threadIdx.x);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t m = uniform((uint32_t)(blockIdx.x * 4 + (threadIdx.x >> 6))); m < a.count; m += nw)
        xdr_message<W>(a, m, tab, lane, [](const uint8_t *, uint64_t, R *) { return false; });
}

// Throughput layout (large batches): persistent 1024-thread workgroups with the
// payload step loop's LDS tables (CRC-32C: the replicated byte tables, one
// workgroup per CU; CRC-64: the 12-lookup tables with combine operators in
// global memory) and the byte table after them; messages from the work queue.
template <int W>
constexpr uint32_t kXdrMainLds = W == 32 ? kL32Bytes : kL64Main;

template <int W, bool NT>
__global__ __launch_bounds__(1024, 1) void xdr_fast_kernel(XdrArgs a) {
    using R = xdr_reg_t<W>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kXdrMainLds<W> + 256 * sizeof(R)];
    __shared__ WgQueue wgq;
    R *tab = reinterpret_cast<R *>(lds + kXdrMainLds<W>);
    if (threadIdx.x == 0) wg_queue_init(&wgq, a.queue, a.count);
    if constexpr (W == 32) fill_lds32<false, 1024>(lds, reinterpret_cast<const crc32_gpu_pack_t *>(a.pack));
    else fill_lds64<1024, kOpsGlobal>(lds, reinterpret_cast<const crc64_gpu_pack_t *>(a.pack));
    if (threadIdx.x < 256) tab[threadIdx.x] = xdr_tab_entry<W>(a.rpoly, threadIdx.x);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 16u + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * 16u;
    const uint32_t lc0 = (lane & 31u) << 2, lc1 = lc0 | 0x10000u, lc64 = (lane & 31u) << 3;
    auto fast = [&](const uint8_t *p, uint64_t len, R *reg) -> bool {
        if (len < kXdrFastMin || len >= (1ull << 31)) return false;
        if constexpr (W == 32)
            *reg = payload32_g64<NT, Tab32<false>, true>(Tab32<false>{lds}, reinterpret_cast<const crc32_gpu_pack_t *>(a.pack),
                                                         p, len, lane, lc0, lc1, *reg);
        else
            *reg = payload64_g64<NT, true, kOpsGlobal>(lds, reinterpret_cast<const crc64_gpu_pack_t *>(a.pack), p, len,
                                                       lane, lc64, *reg);
        return true;
    };
    const bool faulted = for_each_unit<true>(&wgq, a.queue, a.count, wave, nw,
                                             [&](uint64_t m) { xdr_message<W>(a, m, tab, lane, fast); });
    if (faulted) {  // fail closed: the caller's error word, and every status flagged
        if (lane == 0 && a.err_word) atomicAdd(a.err_word, 1u);
        if (a.status)
            for (uint64_t m = lane; m < a.count; m += 64) a.status[m] = 1;
    }
}

}  // namespace

// ------------------------------------------------------------ host side ----

namespace mck {

// Per-device, per-model extension tables (shift pack for 32/64-bit models,
// byte table for 16-bit ones), built and uploaded once (under g_mu), then
// read without a lock.
int get_ext(DevCtx *c, int idx, const void **out) {
    if (void *p = c->ext[idx].load(std::memory_order_acquire)) {
        *out = p;
        return 0;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (void *p = c->ext[idx].load(std::memory_order_relaxed)) {
        *out = p;
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
        const crc_rmodel_t rm = gpu_rmodel(idx);
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
    c->ext[idx].store(d, std::memory_order_release);
    *out = d;
    return 0;
}

long long ext_queue_faults() {
    unsigned int n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_mck_queue_faults), sizeof(n), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return n;
}

}  // namespace mck

using namespace mck;

extern "C" {

// P, C (nseg + 1 each), the ragged flag, the scan's fault claim, the workspace's
// call count, a spare word, the look-back descriptor of
// each scan block (kDescWords), each segment's object and its bounds in
// first[] and its head segment (4 nseg), then the chunk -> segment map (u32 entries:
// 4 per segment + 64 Ki, i.e. lists averaging up to ~1 MiB per segment, or
// one huge segment up to 16 GiB; none past 2^32 segments).  More than 2^40
// segments (far beyond device memory) is rejected, so the size cannot wrap:
// SIZE_MAX then makes any allocation of it fail.
constexpr uint64_t kMaxSegs = 1ull << 40;
uint64_t seg_map_cap(uint64_t nseg) { return nseg < (1ull << 32) ? 4 * nseg + 65536 : 0; }
// Test builds (MCK_QFAULT_TEST): MCHECKSUM_GPU_QFAULT_SCAN=b makes scan block
// b give up its look-back -- or, with MCHECKSUM_GPU_QFAULT_MODE=scanstall,
// never publish its descriptor (tests/test_gpu_fail_closed.py); ~0 = none.
uint64_t scan_fault_block() {
    return MCK_QFAULT_TEST ? mck_settings()->qfault_scan : ~0ull;
}
// scan blocks of a list (one at least: the scan launch writes the totals)
uint64_t seg_blocks(uint64_t nseg) { return nseg ? (nseg + kScanBlk - 1) / kScanBlk : 1; }
uint64_t seg_words(uint64_t nseg) { return 2 * (nseg + 1) + 4 + kDescWords * seg_blocks(nseg) + 4 * nseg; }
// The scan's look-back epochs: a process-wide counter from a random seed, so a
// workspace's descriptors from any earlier call (this process or, through
// reused memory, another) never match the current call's.
uint64_t scan_epoch() {
    static std::atomic<uint64_t> ctr{[] {
        uint64_t seed = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 0x9E3779B97F4A7C15ull;
        try {
            std::random_device rd;
            seed ^= (uint64_t)rd() << 32 ^ rd();
        } catch (...) {  // no entropy source: the clock alone (never throw through the C ABI)
        }
        return (seed & ((1ull << 60) - 1)) | 1ull;
    }()};
    return ctr.fetch_add(1, std::memory_order_relaxed) & ((1ull << 61) - 1);
}
size_t mchecksum_gpu_segments_work_size(size_t nseg) {
    if ((uint64_t)nseg > kMaxSegs) return SIZE_MAX;
    return sizeof(uint64_t) * seg_words(nseg) + sizeof(uint32_t) * seg_map_cap(nseg);
}

int mchecksum_gpu_checksum_segments(const char *hash_method, const uint64_t *dev_seg_addr,
                                    const uint64_t *dev_seg_len, size_t nseg, const uint64_t *dev_obj_first,
                                    size_t nobj, void *dev_work, size_t work_size, void *dev_out, void *stream) {
    if (!dev_obj_first || (nobj && !dev_out) || (nseg && (!dev_seg_addr || !dev_seg_len)) || !dev_work)
        return set_err(MCHECKSUM_GPU_EINVAL, "NULL pointer argument");
    if ((uint64_t)nseg > kMaxSegs) return set_err(MCHECKSUM_GPU_EINVAL, "more than 2^40 segments in one call");
    if (work_size < mchecksum_gpu_segments_work_size(nseg) || (uintptr_t)dev_work % 8)
        return set_err(MCHECKSUM_GPU_EINVAL, "workspace smaller than mchecksum_gpu_segments_work_size() or unaligned");
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    int width = 0;
    DevCtx *c = nullptr;
    const void *pack = nullptr, *shift = nullptr;
    int rc = prologue(hash_method, CRC_GPU_MAX_LOG2G, &width, &c, &pack);
    if (rc) return rc;
    rc = get_ext(c, mck_model_index(hash_method), &shift);
    if (rc) return rc;
    if (nobj == 0) return MCHECKSUM_GPU_OK;
    hipStream_t s = (hipStream_t)stream;
    SegArgs a{};
    a.addr = dev_seg_addr;
    a.len = dev_seg_len;
    a.nseg = nseg;
    a.first = dev_obj_first;
    a.nobj = nobj;
    a.P = (const uint64_t *)dev_work;
    a.C = (const uint64_t *)dev_work + (nseg + 1);
    a.ragged = (const unsigned long long *)dev_work + 2 * (nseg + 1);
    const uint64_t nb = seg_blocks(nseg);
    uint64_t *desc = (uint64_t *)dev_work + 2 * (nseg + 1) + 4;
    a.obj = desc + kDescWords * nb;
    a.map = reinterpret_cast<const uint32_t *>((const uint64_t *)dev_work + seg_words(nseg));
    // only the CRC-64 queue pass reads the map; MCHECKSUM_GPU_SEG_MAP_CAP caps
    // the part of it used (tests: 0 forces the search over C)
    a.map_cap = width == 64 ? seg_map_cap(nseg) : 0;
    {
        const uint64_t v = mck_settings()->gpu_seg_map_cap;
        a.map_cap = v < a.map_cap ? v : a.map_cap;
    }
    a.out = dev_out;
    a.pack = pack;
    a.shift = shift;
    a.err_word = error_word();
    a.fault_claim = (const uint64_t *)dev_work + 2 * (nseg + 1) + 1;
    a.gen = (const uint64_t *)dev_work + 2 * (nseg + 1) + 2;
    // every object starts as the CRC of the empty message, init ^ xorout in
    // the kernels' register form (MSB-first models: byte-reversed, swapped
    // back with the outputs below)
    const crc_rmodel_t rm = gpu_rmodel(mck_model_index(hash_method));
    const uint64_t preset = rm.rinit ^ rm.xorout;
    ScanArgs sa{};
    sa.len = dev_seg_len;
    sa.addr = dev_seg_addr;
    sa.nseg = nseg;
    sa.desc = desc;
    sa.epoch = a.epoch = scan_epoch();
    sa.P = (uint64_t *)a.P;
    sa.C = (uint64_t *)a.C;
    sa.ragged = (unsigned long long *)a.ragged;
    sa.first = dev_obj_first;
    sa.nobj = nobj;
    sa.obj = width == 64 ? (uint64_t *)a.obj : nullptr;
    sa.map = (uint32_t *)a.map;
    sa.map_cap = a.map_cap;
    sa.out = dev_out;
    sa.width = (uint32_t)width;
    sa.preset = preset;
    sa.err_word = a.err_word;
    sa.fault_claim = (uint64_t *)a.fault_claim;
    sa.gen = (uint64_t *)a.gen;
    sa.fault_block = scan_fault_block();
    hipError_t e = launch_kernel(seg_scan, dim3((unsigned)nb), dim3(kScanThreads), s, nullptr, sa);
    if (e != hipSuccess) return hip_err(e, "segment scan launch");
    if (width == 32) {
        e = launch_kernel(seg_kernel<32>, dim3(c->cus), dim3(1024), s, nullptr, a);
        if (e != hipSuccess) return hip_err(e, "segment kernel launch");
    } else {
        SlotRef sr = queue_slot(c, stream);
        a.queue = sr.q;
        e = launch_kernel(seg_kernel<64>, dim3(c->cus), dim3(1024), s, sr.done, a);
        if (e != hipSuccess) {
            slot_unissue(c, sr);
            return hip_err(e, "segment kernel launch");
        }
        slot_issued(sr);
    }
    // MSB-first model: the kernels' values are the CRCs byte-swapped (crc_gpu_layout.h)
    if (gpu_msb(mck_model_index(hash_method))) return swap_outputs(dev_out, nobj, width, stream);
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
    if (int rc = device_ctx(&c)) return rc;
    if (int rc = get_ext(c, idx, &table)) return rc;
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
    const hipError_t e = launch_kernel(core_header_kernel, dim3((unsigned)blocks), dim3(256), (hipStream_t)stream, nullptr, a);
    if (e != hipSuccess) return hip_err(e, "core header kernel launch");
    return MCHECKSUM_GPU_OK;
}

int mchecksum_gpu_checksum_xdr(const char *hash_method, const mchecksum_xdr_field_t *fields, size_t nfields,
                               const void *dev_buf, const uint64_t *dev_msg_offsets, size_t count, void *dev_out,
                               uint8_t *dev_status, void *stream) {
    if ((nfields && !fields) || !dev_msg_offsets || (count && (!dev_buf || !dev_out)))
        return set_err(MCHECKSUM_GPU_EINVAL, "NULL pointer argument");
    if (nfields > kXdrMaxFields) return set_err(MCHECKSUM_GPU_EINVAL, "more than %u schema fields", kXdrMaxFields);
    XdrArgs a{};
    for (size_t f = 0; f < nfields; f++) {
        const uint32_t k = fields[f].kind, z = fields[f].size;
        const bool ok = (k == MCHECKSUM_XDR_INT && (z == 1 || z == 2 || z == 4 || z == 8)) ||
                        k == MCHECKSUM_XDR_OPAQUE || k == MCHECKSUM_XDR_RAW || k == MCHECKSUM_XDR_OPAQUE_LEN ||
                        k == MCHECKSUM_XDR_RAW_LEN || (k == MCHECKSUM_XDR_SKIP_IF_ZERO && z <= nfields - f - 1);
        if (!ok) return set_err(MCHECKSUM_GPU_EINVAL, "schema field %zu: bad kind %u / size %u", f, k, z);
        a.kind[f] = k;
        a.size[f] = z;
    }
    int width = 0;
    const int idx = gpu_model(hash_method, &width);
    if (idx == -1) return set_err(MCHECKSUM_GPU_EMETHOD, "unknown hash method \"%s\"", hash_method ? hash_method : "(null)");
    if (idx < 0 || gpu_msb(idx))
        return set_err(MCHECKSUM_GPU_EMETHOD, "method \"%s\" has no XDR kernel (reflected 32/64-bit only)", hash_method);
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    DevCtx *c = nullptr;
    const void *shift = nullptr;
    if (int rc = device_ctx(&c)) return rc;
    if (int rc = get_ext(c, idx, &shift)) return rc;
    if (count == 0) return MCHECKSUM_GPU_OK;
    // throughput layout for batches past a receive queue's worth of RPCs
    // (MCHECKSUM_GPU_XDR_FAST=0/1 overrides)
    const int fset = mck_settings()->gpu_xdr_fast;
    const bool fast = fset >= 0 ? fset == 1 : count > 1024;
    if (fast) {
        int w2 = 0;
        const void *pack = nullptr;
        int rc = prologue(hash_method, CRC_GPU_MAX_LOG2G, &w2, &c, &pack);
        if (rc) return rc;
        a.pack = pack;
    }
    const mck_model_t &m = mck_models[idx];
    a.buf = (const uint8_t *)dev_buf;
    a.off = dev_msg_offsets;
    a.count = count;
    a.out = dev_out;
    a.status = dev_status;
    a.shift = shift;
    a.rpoly = mck_reflect(m.poly, m.width);
    a.init = mck_reflect(m.init, m.width);
    a.xorout = m.xorout;
    a.nf = (uint32_t)nfields;
    if (fast) {
        // non-temporal loads for batches far past the Infinity Cache, sized
        // by count as for offsets batches (MCHECKSUM_GPU_NT=0/1 overrides)
        const int nset = mck_settings()->gpu_nt;
        const bool nt = nset >= 0 ? nset == 1 : count >= 8192;
        a.err_word = error_word();
        uint64_t blocks = (count + 15) / 16;
        if (blocks > (uint64_t)c->cus) blocks = (uint64_t)c->cus;
        SlotRef sr = queue_slot(c, stream);
        a.queue = sr.q;
        auto k = width == 32 ? (nt ? xdr_fast_kernel<32, true> : xdr_fast_kernel<32, false>)
                             : (nt ? xdr_fast_kernel<64, true> : xdr_fast_kernel<64, false>);
        const hipError_t e = launch_kernel(k, dim3((unsigned)blocks), dim3(1024), (hipStream_t)stream, sr.done, a);
        if (e != hipSuccess) {
            slot_unissue(c, sr);
            return hip_err(e, "XDR kernel launch");
        }
        slot_issued(sr);
        return MCHECKSUM_GPU_OK;
    }
    uint64_t blocks = (count + 3) / 4;
    if (blocks > (uint64_t)c->cus * 8) blocks = (uint64_t)c->cus * 8;
    const hipError_t e = launch_kernel(width == 32 ? xdr_kernel<32> : xdr_kernel<64>, dim3((unsigned)blocks), dim3(256),
                                       (hipStream_t)stream, nullptr, a);
    if (e != hipSuccess) return hip_err(e, "XDR kernel launch");
    return MCHECKSUM_GPU_OK;
}

}  // extern "C"
