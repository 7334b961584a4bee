// crc_gpu_device.h -- device side of the MI355X (gfx950) batch CRC kernels:
// the table-driven step loops, sub-stream combine trees and the persistent
// batch kernels.  Included by the translation units that launch them
// (mchecksum_gpu.hip: fixed / offsets / verify batches; mchecksum_gpu_ext.hip:
// scatter-gather segments and core headers).  Algebra: crc_gpu_layout.h.
#ifndef CRC_GPU_DEVICE_H
#define CRC_GPU_DEVICE_H

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "crc_gpu_layout.h"
#include "crc_gpu_mask.h"

namespace {

// Tuning constants are the measured best (their A/Bs: DESIGN.md and
// HISTORY.md; losing alternatives are not kept in the source).
constexpr int kBlock = 1024;  // 16 waves: 4 per SIMD
constexpr int kRing = 4;      // dwordx4 pieces in flight per lane
// Offsets batches (one payload per wave, ~32 KiB average) want a deeper ring:
// 8 measured +4% over 4 on C4, while 8 costs 1-5% on the aligned batches.
constexpr int kRingOff = 8;

// CRC-32C LDS map: [0,128K) main byte tables x32 copies; then op nibble
// tables; then the two-level combine operators (crc_gpu_layout.h lv, 8 KiB).
constexpr uint32_t kL32Main = 131072;
constexpr uint32_t kL32Lv = kL32Main + CRC32_NOPS_MAX * 512;
constexpr uint32_t kL32Bytes = kL32Lv + 2 * 8 * 16 * 8 * 4;
// Light layout for small batches: the 4 byte tables unreplicated (4 KiB, so
// the per-workgroup LDS fill is 16 KiB instead of 140 KiB) and 256-thread
// workgroups spread over every CU; lookups may bank-conflict, which a small
// batch never notices.
constexpr uint32_t kL32LightMain = 4096;
constexpr uint32_t kL32LightBytes = kL32LightMain + CRC32_NOPS_MAX * 512;
constexpr int kLightBlock = 256;

// CRC-32C table access policy: Tab32<false> = 32x-replicated conflict-free
// layout (throughput), Tab32<true> = light layout (latency of small batches).
template <bool LIGHT>
struct Tab32 {
    const uint8_t *lds;
};
// CRC-64 LDS map.  A 64-bit word is looked up in 12 tables (pack f5 / f6,
// crc_gpu_layout.h): bits 3..7 of each of its 8 bytes index a 32-entry table
// at 8-B stride -- one 256-B row, entry v on bank pair v, so distinct entries
// never share a bank and equal ones broadcast: conflict-free without lane
// copies, and the address is (byte & 0xF8) itself --, and bits 0..2 of bytes i
// and i + 4, gathered into one 6-bit index by one shift + bit-select for all
// four, index a 64-entry table replicated 32x (entry v at v*256 B + lane copy
// (lane % 32)*8: 16 KiB per table).  Then the combine operators (16 nibble
// tables, 2 KiB each).  (Round 1's 16-lookup nibble form needed a third more
// LDS reads; 11 lookups over 7-bit tables, a wide-row map with cheaper address
// ops and two workgroups per CU all measured slower: HISTORY.md.)
constexpr uint32_t kL64P5 = 0;
constexpr uint32_t kL64P6 = 8 * 256;
constexpr uint32_t kL64Main = kL64P6 + 4 * 16384;
constexpr uint32_t kL64Bytes = kL64Main + CRC64_NOPS_MAX * 2048;
// Where the CRC-64 combine operators live: all in LDS (one 1024-thread
// workgroup per CU: the aligned batches and the merged segment pass), all in
// global memory (the XDR throughput kernel), or the six butterflies
// Z^-(16*2^k) in LDS and Z^-8 and the tail operators -- the two ends of the
// offsets path's dependent chain -- in global memory (the offsets path: two
// workgroups per CU at 79.9 KiB each, +6-8% on C4-layout CRC-64 over either
// pure form, profiles/r01/ab20_crc64_offsets_mix.log).
enum OpsMode : int { kOpsLds = 0, kOpsGlobal = 1, kOpsMix = 2 };

// Launch shape per kernel.  CRC-32C: one 1024-thread workgroup per CU (the
// replicated tables take 140 KiB), or the light layout's 256-thread
// workgroups, 8 per CU.  CRC-64 aligned and generic fixed batches: one
// 1024-thread workgroup per CU with every operator in LDS (round 4: C3 -2.6%
// in time against two workgroups per CU with the operators in global memory,
// profiles/r04/ab_c3_onewg.log).  CRC-64 offsets batches: two workgroups per
// CU, the mixed operator placement and a 4-deep ring so the loop fits 64
// VGPRs (a ring of 8 at two workgroups spills: -42%).
template <int W, int MODE, bool LIGHT = false, int LG = -1>
struct Shape {
    static constexpr bool two = W == 64 && MODE == 2;
    static constexpr int block = LIGHT ? kLightBlock : kBlock;
    static constexpr int blocks_per_cu = LIGHT ? 8 : two ? 2 : 1;
    static constexpr int ops_mode = two ? kOpsMix : kOpsLds;
    static constexpr uint32_t lds64_bytes = two ? kL64Main + 6 * 2048 : kL64Bytes;
};
constexpr int kRingOff64 = 4;
// single-argument aliases keyed MODE * 16 + LOG2G (a comma inside
// __launch_bounds__ splits the macro)
template <int KEY>
constexpr int kBlk64 = Shape<64, KEY / 16, false, KEY % 16>::block;
template <int KEY>
constexpr int kWpe64 = Shape<64, KEY / 16, false, KEY % 16>::blocks_per_cu * Shape<64, KEY / 16, false, KEY % 16>::block / 256;

enum Mode : int { kFixedAligned = 0, kFixedGeneric = 1, kOffsets = 2 };

struct BatchArgs {
    const uint8_t *base;
    const uint64_t *offsets;
    uint64_t stride, len, count;
    void *out;
    const void *expected;
    uint8_t *status;
    uint32_t *mismatches;
    const void *pack;
    // message mode (verify_messages): payload i = [offsets[i] + pay_off,
    // offsets[i+1]), expected CRC = big-endian u32 at offsets[i] + hash_off
    uint32_t msg, pay_off, hash_off;
    // work-queue slot (WgQueue below), exclusive to this launch's stream;
    // nullptr = static assignment
    unsigned long long *queue;
    // optional caller word (mchecksum_gpu_set_error_word): +1 when this launch
    // could not hash every payload (fail-closed report for checksum modes)
    uint32_t *err_word;
    // split CRC-64 pieces (crc64_batch_kernel<..., SPLIT>): each payload is
    // 2^split_log2 pieces of kSplitBytes, recombined with the Z^n shift pack
    const void *shift;
    uint32_t split_log2;
    // MSB-first model on a verify call: the kernel's value is the CRC
    // byte-swapped (crc_gpu_layout.h), so swap before comparing
    uint32_t bswap;
    // split CRC-64: 1 = every queue chunk holds whole payloads (SplitPlan::whole),
    // so the pieces combine in the workgroup's LDS and out[] needs no zeroing
    uint32_t split_lds;
};
// Piece size of a split payload: 256 KiB = 256 steps of the G = 64 loop.
// (A/B, round 4: 128 KiB pieces +2.9%, 512 KiB +6.8% on C3 time, profiles/r04/ab_split_piece.log)
constexpr uint64_t kSplitBytes = 256u << 10;
// Payloads per queue chunk whose pieces a workgroup can combine in LDS, and
// the accumulator sets (chunks with pieces in flight) it keeps.
constexpr uint32_t kSplitAcc = 16;
constexpr uint32_t kAccSets = 32;

// ------------------------------------------------------------ work queue --
// Dynamic distribution of payloads over waves.  With a static assignment the
// waves of one 4 GiB launch finish between 566 and 642 us (p10..max; the XCDs
// stream at different rates, profiles/r01/tail_trace.json), so the slowest
// wave sets the launch time.  Per-wave tickets from global counters do not
// work: device-scope atomics on one address retire ~1 per 45 ns on MI355X,
// so 8 per-XCD counters fed one ticket per payload group throttled C2 2.6x.
//
// Two levels instead.  Units [0, n) form chunks (ChunkPlan below); the chunk
// ids are dealt round-robin to 8 sub-queues (one per XCD by blockIdx % 8, the
// dispatch order), each a global counter on its own 256-B line.  A workgroup
// takes whole chunks (one device-scope atomic per chunk, stealing from the
// next sub-queue once its own is drained) and its waves take the chunk's
// units one at a time through an LDS counter.  The wave that takes the slot a
// quarter chunk before the end fetches the NEXT chunk -- after reading its own
// chunk id, so fetches run in chunk order and the first "no more chunks" is
// final -- and the fetch's latency hides under the rest of the chunk.  Chunk
// ids pass through a small LDS ring whose entries are recycled only after all
// readers of the previous occupant have read it (the host hands each launch a
// slot of its stream's own, mchecksum_gpu.hip).  tests/test_queue_model.py
// runs the same protocol on the CPU under random interleavings.
//
// Two banks per slot (round 3).  Launch s on a slot counts in bank s & 1 (the
// host passes that bank) and, from its first workgroup at entry, zeroes the
// protocol lines of the OTHER bank, which the slot's next launch will use --
// launches on a slot never overlap, so nobody is using that bank.  Round 2
// instead had the launch's last group zero its own bank at exit, behind a
// hierarchical exit count (LDS per workgroup, a line per group, one per
// slot): three dependent device-scope atomics, the zeroing and a wait after
// the last wave's last payload, on every launch's critical path.  Round 3
// kept one non-returning add per workgroup on a completion line, summed by the
// host (a device round trip) before it gave a slot to another stream; round 4
// records a HIP event at each slot launch's completion instead
// (hipExtLaunchKernel's stop event, queried without blocking, queue_slot), so
// a workgroup's exit touches no slot line.
// Bank layout (one counter per 256-B line, 8 KiB per bank, 16 KiB-aligned
// slots): [0, 8) sub-queue tickets, [8] fault flag of the launch (claimed by
// its first faulting wave, which reports), [9] abort flag (set by any wave
// whose bounded wait gave up; every later wait of the launch then gives up at
// once, so one call spends at most one deadline however many stalls it meets)
// -- all zeroed by the previous launch on the slot.
//
// Exclusivity.  A slot serves one launch at a time: the host hands the queue
// only to eager launches, each on a slot of its stream's own (launches on one
// stream never overlap).  Launches it cannot give an exclusive slot -- graph
// captures (every replay reuses the captured arguments, and two execs of one
// capture may replay at once) and streams past the per-stream table -- get
// no slot and take the static split (units wave, wave + #waves, ...).  (Round
// 2 had such launches claim a shared slot with a tag; a launch whose early
// workgroups found the slot busy and later ones found it free never released
// it, and its next replay -- same tag -- ran on stale counters and skipped
// units: one wrong batch in 400 concurrent replays.  The XOR-accumulating
// kernels (split CRC-64 pieces, scatter-gather chunks) also cannot tolerate
// the units such mixed launches hashed twice.)
constexpr uint32_t kQSub = 8;
constexpr uint32_t kQStride = 32;  // u64 words between counters
constexpr uint32_t kQFault = kQSub;
constexpr uint32_t kQAbort = kQSub + 1;
constexpr uint32_t kQBankLines = kQAbort + 1;  // protocol lines, zeroed before the bank's next use
constexpr uint64_t kQBankBytes = 8192;
constexpr uint32_t kQBankWords = (uint32_t)(kQBankBytes / 8);
constexpr uint32_t kQSlotWords = 2 * kQBankWords;  // slots 2 * kQBankBytes aligned: bank ^ kQBankBytes = the other
static_assert(kQBankLines * kQStride <= kQBankWords, "bank overflow");
// Chunk size: a power of two, about a quarter of a workgroup's fair share
// of units, between 1 and 32 (C4: 32 units; a 5000-payload batch: 4).
// Fixed 16 starved half the workgroups of C3's 8192 units at 2 WGs per CU; 32
// beat 16 on the large batches.  The next chunk is fetched when a quarter of
// the current one is left to take: early enough to hide the fetch (~1.3 us
// mean), late enough that a workgroup holds little unstarted work when the
// queue runs dry.
constexpr uint32_t kWgChunkMaxLog2 = 5;
// Which batches take the queue (profiles/r01/ab12_work_queue.log, medians
// vs the static split): variable-length (offsets) batches, +4% C4 and +8%
// C4-layout CRC-64 over the byte-balanced static split, and the large
// (non-temporal, >= 512 MiB) aligned CRC-32C batches, +2.3% on the headline.
// Smaller fixed batches and CRC-64 fixed batches keep the static stride:
// there the queue's fixed costs outweigh the balance (C2 -11% warm, -14%
// with cold lines, profiles/r06/ab_c2cold.log; 2 KiB -16% and 8/16 KiB
// +-0.3% at the round-6 lane counts, profiles/r06/ab_c2dyn.log; C3 -5%).
__host__ __device__ constexpr bool dyn_policy(int width, int mode, bool nt, bool light) {
    return !light && (mode == 2 || (width == 32 && nt && mode == 0));  // 2 = kOffsets
}
__device__ __forceinline__ uint32_t chunk_log2(uint64_t n) {
    const uint64_t share = n / (4ull * gridDim.x);
    uint32_t l = 0;
    while (l < kWgChunkMaxLog2 && (2ull << l) <= share) l++;
    return l;
}

// Chunk plan: ids [0, nbig) are full chunks of 2^cl units; the last
// (about one full chunk per workgroup of) units go out as eighth chunks, ids
// [nbig, nch), so a workgroup that fetches late holds little unstarted work
// when the queue runs dry.  The highest ids are handed out last (every
// sub-queue counts up), so the small chunks form the tail.
// Tail chunks are 2^-kQTailShift of a full one, over the last full chunk per
// workgroup.  Eighths since round 4 (quarters before): never slower in two
// one-process A/Bs, headline -0.4% / -0.6%, C3 -0.7%, seg -0.7%, C4 +-0 in
// time (profiles/r04/ab_qtail.log, ab_round4_knobs.log: "t3"); single-unit
// tail chunks lost 2.3% on C4 (one fetch per unit), two full chunks per
// workgroup of tail +0.5% on the headline.
constexpr uint32_t kQTailShift = 3;
struct ChunkPlan {
    uint32_t cl, sl;    // log2 of the full / tail chunk size
    uint64_t nbig, nch, big_end;
    __device__ __forceinline__ explicit ChunkPlan(uint64_t n) {
        cl = chunk_log2(n);
        sl = cl >= kQTailShift ? cl - kQTailShift : cl;
        const uint64_t tail = (uint64_t)gridDim.x << cl;
        nbig = n > tail ? (n - tail) >> cl : 0;
        big_end = nbig << cl;
        nch = nbig + ((n - big_end + (1ull << sl) - 1) >> sl);
    }
    // first unit and size of chunk id
    __device__ __forceinline__ uint64_t start(uint64_t id) const {
        return id < nbig ? id << cl : big_end + ((id - nbig) << sl);
    }
    __device__ __forceinline__ uint32_t size(uint64_t id) const { return id < nbig ? 1u << cl : 1u << sl; }
};
// Split CRC-64: the queue plan of a split launch -- ChunkPlan's layout over
// count << psl units, unit u = piece (u & (2^psl - 1)) of payload u >> psl.
// (Late round 5 also tried the tail's payloads in 2-4x finer pieces: the
// per-wave end spread fell from 111 to 42 us, but every piece pays its own
// combine and Z^n shift, and C3 lost 0.5%: HISTORY.md.)
struct SplitPlan {
    uint32_t cl, sl;       // log2 of the full / tail chunk size (units)
    uint32_t psl;          // log2 pieces per payload
    uint64_t nbig, nch, big_end, n;
    __host__ __device__ SplitPlan(uint64_t count, uint32_t psl_, uint32_t grid) : psl(psl_) {
        n = count << psl;
        const uint64_t share = n / (4ull * grid);
        cl = 0;
        while (cl < kWgChunkMaxLog2 && (2ull << cl) <= share) cl++;
        sl = cl >= kQTailShift ? cl - kQTailShift : cl;
        const uint64_t tail = (uint64_t)grid << cl;
        nbig = n > tail ? (n - tail) >> cl : 0;
        big_end = nbig << cl;
        nch = nbig + ((n - big_end + (1ull << sl) - 1) >> sl);
    }
    __host__ __device__ uint64_t start(uint64_t id) const { return id < nbig ? id << cl : big_end + ((id - nbig) << sl); }
    __host__ __device__ uint32_t size(uint64_t id) const { return id < nbig ? 1u << cl : 1u << sl; }
    // unit u: piece *q of payload *p
    __host__ __device__ void unit(uint64_t u, uint64_t *p, uint32_t *q) const {
        *p = u >> psl;
        *q = (uint32_t)u & ((1u << psl) - 1u);
    }
    // every chunk holds whole payloads, at most kSplitAcc of them (the
    // in-workgroup combine, split_lds)
    __host__ __device__ bool whole() const {
        return psl >= 1 && (1u << psl) <= (1u << sl) && (1u << cl) / (1u << psl) <= kSplitAcc;
    }
};

constexpr uint32_t kWgRing = 8;    // LDS ring of published chunk ids
constexpr uint64_t kNoChunk = 0xFFFFFFFFull;

struct WgQueue {
    unsigned int slot;     // next (chunk, unit) slot of this workgroup
    unsigned int drained;  // sub-queues (counted from home) found empty
    unsigned int busy;     // 1: no slot for this launch -> static split
    unsigned int reads[kWgRing];
    unsigned long long entry[kWgRing];  // (chunk seq << 32) | global chunk id
};

// (readfirstlane returns int: widen each half as uint32_t, or a low half with
// bit 31 set would sign-extend over the high half)
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return (uint64_t)hi << 32 | lo;
}

template <class T>
__device__ __forceinline__ T lds_ld(T *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <class T>
__device__ __forceinline__ void lds_st(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Every wait in the queue protocol is bounded in time: a wait still unmet
// after kWaitTicks of the constant 100 MHz real-time counter (1 s; or a wave
// that takes more slots than the launch has) counts a fault in
// g_mck_queue_faults (read by mchecksum_gpu_queue_faults()) and leaves the
// loop, so a protocol failure shows up as a fault count and a failed call
// instead of a wedged GPU.  Diagnostic builds (-DMCK_TRACE=1) also record
// where (g_mck_qdiag).
__device__ unsigned int g_mck_queue_faults;
#if MCK_TRACE
__device__ unsigned long long g_mck_qdiag[4 * 64];
__device__ unsigned int g_mck_qdiag_n;
// per wave: fetches, fetch ticks (sum), fetch ticks (max), entry-wait ticks
__device__ unsigned long long g_mck_qwave[6 * 16384];
// per unit (u < 2^17): completion time | (blockIdx % 8) << 60 (tools/unit_timeline.py)
__device__ unsigned long long g_mck_unit_end[1u << 17];
#endif
__device__ __noinline__ void queue_fault(uint32_t kind, uint64_t a, uint64_t b) {
    atomicAdd(&g_mck_queue_faults, 1u);
#if MCK_TRACE
    const unsigned int i = atomicAdd(&g_mck_qdiag_n, 1u);
    if (i < 64) {
        g_mck_qdiag[4 * i] = kind;
        g_mck_qdiag[4 * i + 1] = blockIdx.x * 64ull + (threadIdx.x >> 6);
        g_mck_qdiag[4 * i + 2] = a;
        g_mck_qdiag[4 * i + 3] = b;
    }
#else
    (void)kind;
    (void)a;
    (void)b;
#endif
}
// A wait's deadline, on wall_clock64() -- the 100 MHz real-time counter,
// independent of the shader clock and of how slow each poll gets under
// contention (round 4's reverted in-kernel zeroing hung with 8192 waves
// polling one line: an iteration count had bounded nothing).  The counter is
// read on every 16th poll only (the polls stay tight: the ring-entry wait sits
// on the path of every unit taken) and the first read starts the clock.
//  * Preemption: a gap of more than kGapTicks between two reads (16 polls
//    take microseconds) means the wave was switched out -- CWSR, when other
//    processes share the GPU -- and that time does not count, so a healthy
//    launch resumed after a long preemption does not fail closed at once.
//  * Abort: the launch's abort flag (kQAbort; nullptr for waits outside the
//    queue) is read with the counter; once any wait of the launch has given
//    up, every other one gives up at its next read, so a call meets at most
//    one deadline however many stalls it has.
#ifndef MCK_WAIT_TICKS
#define MCK_WAIT_TICKS 100000000ull  // 1 s at 100 MHz
#endif
constexpr uint64_t kWaitTicks = MCK_WAIT_TICKS;
constexpr uint64_t kGapTicks = 5000000ull;  // 50 ms
struct Deadline {
    const unsigned long long *abort = nullptr;
    uint64_t t0 = 0, last = 0;
    uint32_t polls = 0;
    __device__ explicit Deadline(const unsigned long long *abort_word = nullptr) : abort(abort_word) {}
    // true once this wait has lasted kWaitTicks, or the launch aborted (call once per poll)
    __device__ __forceinline__ bool passed() {
        if ((++polls & 15u) != 1u) return false;
        const uint64_t now = wall_clock64();
        if (polls == 1u) {
            t0 = last = now;
            return abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (now - last > kGapTicks) t0 += now - last;  // switched out: not waiting time
        last = now;
        return now - t0 > kWaitTicks || (abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
};
// The launch's abort flag in its bank (queue non-null), set by a wave whose wait gave up.
__device__ __forceinline__ unsigned long long *abort_word(unsigned long long *q) { return q + kQAbort * kQStride; }
__device__ __forceinline__ void raise_abort(unsigned long long *q) {
    if (q) __hip_atomic_store(abort_word(q), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#define MCK_WAIT_GUARD(dl, kind, A_, B_) \
    if ((dl).passed()) {                 \
        queue_fault(kind, A_, B_);       \
        break;                           \
    }

#if MCK_QFAULT_TEST
// Test builds: which failure the qfault library injects (set from
// MCHECKSUM_GPU_QFAULT_MODE before every launch, gpu_host.h): 0 = a wave gives
// up one unit without waiting (workgroup 3, the first unit of its second
// chunk; in the segment scan, block MCHECKSUM_GPU_QFAULT_SCAN gives up its
// look-back); 1 = "stall": workgroup 3 never publishes its third chunk, so its
// waves wait out the deadline; 2 = "scanstall": segment-scan block
// MCHECKSUM_GPU_QFAULT_SCAN never publishes its look-back descriptor, so its
// successors wait out theirs; 3 = "stall+scanstall": both in one call.
__device__ unsigned int g_mck_qfault_mode;
#endif

// Steal order: thieves of one home start at different victims.  On since
// round 3: never slower in four one-process A/Bs over rounds 3-4 (headline
// +0.1 to +0.2%, C4 +0.14 to +0.55%; profiles/r03/ab_steal_rot*.log,
// profiles/r04/ab_qmask.log) -- gains inside the run-to-run band, kept because
// the rotation is free (one index formula, a bijection over the other seven
// sub-queues, run by the CPU model in tests/test_queue_model.py).  A drained-
// state mask read before stealing (one load per fetch instead of an atomic on
// each drained sub-queue) measured -0.1% / -0.5% and is gone.
// One lane: the next global chunk id for this workgroup, or kNoChunk.
__device__ uint64_t wg_fetch(WgQueue *L, unsigned long long *q, uint64_t nch) {
    const uint32_t home = blockIdx.x % kQSub;
    uint32_t d = lds_ld(&L->drained);
    while (d < kQSub) {
        // thieves of one home start at different victims (a rotation of the
        // other seven by workgroup), so a drained XCD's 32 workgroups do not
        // all queue on the next sub-queue's counter at the end of the batch
        const uint32_t k = d == 0 ? home : (home + 1 + (d - 1 + (blockIdx.x / kQSub) % (kQSub - 1)) % (kQSub - 1)) % kQSub;
        // sub-queue k owns chunks k, k + 8, k + 16, ...: every XCD streams
        // from the same moving window of the batch (contiguous per-XCD ranges
        // -- 8 windows far apart -- measured 8% slower on the headline batch)
        const uint64_t t = atomicAdd(q + k * kQStride, 1ull);
        if (k + t * kQSub < nch) return k + t * kQSub;
        atomicMax(&L->drained, d + 1);
        const uint32_t seen = lds_ld(&L->drained);
        d = seen > d + 1 ? seen : d + 1;
    }
    return kNoChunk;
}

// One lane: make chunk `seq` of this workgroup known in the ring.  Returns
// false when the wait for the ring entry's readers gave up (fault counted,
// the launch's abort flag raised).
__device__ bool wg_publish(WgQueue *L, unsigned long long *q, uint32_t seq, uint64_t id, uint32_t cl) {
    const uint32_t r = seq % kWgRing;
    bool ok = true;
    Deadline dl(abort_word(q));
    if (seq >= kWgRing)
        while (lds_ld(&L->reads[r]) != (1u << cl)) {
            __builtin_amdgcn_s_sleep(1);
            if (dl.passed()) {
                queue_fault(1, seq, lds_ld(&L->reads[r]));
                raise_abort(q);
                ok = false;
                break;
            }
        }
    lds_st(&L->reads[r], 0u);
    lds_st(&L->entry[r], (unsigned long long)seq << 32 | id);
    return ok;
}

// Thread 0, before the kernel's first barrier: reset the LDS state and
// publish the first chunk (its fetch overlaps the LDS table fill); workgroup
// 0 first zeroes the other bank's protocol lines for the slot's next launch
// (the fetch's returning atomic waits for those adds to be performed: vmcnt
// also counts non-returning atomics on gfx9-family parts).  Without a slot
// (see "Exclusivity") the workgroup takes the static split (busy = 1).
//
// Split in two for kernels whose waves start on a static first unit
// (for_each_unit<DYN, true>): wg_queue_reset (LDS only) before the barrier,
// wg_queue_start after it -- the fetch's round trip then no longer sits in
// front of thread 0's wave's table fill (waves look for a chunk only after
// their first unit; until the publish they wait on the ring entry).
__device__ __attribute__((unused)) void wg_queue_reset(WgQueue *L, unsigned long long *q) {
    L->slot = 0;
    L->drained = 0;
    L->busy = q == nullptr;
    for (uint32_t r = 0; r < kWgRing; r++) {
        L->reads[r] = 0;
        L->entry[r] = ~0ull;
    }
}
template <class Plan>
__device__ __attribute__((unused)) void wg_queue_start_plan(WgQueue *L, unsigned long long *q, const Plan &plan) {
    if (!q) return;
    if (blockIdx.x == 0) {
        unsigned long long *o = reinterpret_cast<unsigned long long *>(reinterpret_cast<uintptr_t>(q) ^ kQBankBytes);
#pragma unroll
        for (uint32_t j = 0; j < kQBankLines; j++) atomicExch(o + j * kQStride, 0ull);
    }
    (void)wg_publish(L, q, 0, wg_fetch(L, q, plan.nch), plan.cl);
}
__device__ __attribute__((unused)) void wg_queue_start(WgQueue *L, unsigned long long *q, uint64_t n) {
    if (!q) return;
    wg_queue_start_plan(L, q, ChunkPlan(n));
}
__device__ __attribute__((unused)) void wg_queue_init(WgQueue *L, unsigned long long *q, uint64_t n) {
    wg_queue_reset(L, q);
    wg_queue_start(L, q, n);
}
template <class Plan>
__device__ __attribute__((unused)) void wg_queue_init_plan(WgQueue *L, unsigned long long *q, const Plan &plan) {
    wg_queue_reset(L, q);
    wg_queue_start_plan(L, q, plan);
}


template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const T o = __shfl_xor(v, k, 64);
        v = o > v ? o : v;
    }
    return v;
}

// Calls body(u) for this wave's units: through the work queue (DYN: the
// throughput kernels, wg_queue_init has run) or u = wave, wave + nw, ... (the
// light layout's small batches, and DYN launches without a slot).
//
// Fail closed.  Every wait of the queue protocol is bounded; a wave whose wait
// gives up leaves the loop, and the units it would still have taken may then
// never be hashed.  for_each_unit returns true in the FIRST such wave of the
// launch (one fault flag per slot), which must then run fail_closed(): it
// reports the launch as failed, so unhashed bytes never read as verified.
// -DMCK_QFAULT_TEST=1 (test builds only) forces one give-up per launch.
#ifndef MCK_QFAULT_TEST
#define MCK_QFAULT_TEST 0
#endif
//
// FIRST: the caller has already run each wave's first unit, `wave` itself
// (known at kernel entry, so its loads can go out before the LDS fill); the
// static cursor starts at wave + nw and the queue deals units [q0, n),
// q0 = min(n, nw) -- wg_queue_init gets n - q0 (first_static_units).
__device__ __forceinline__ uint64_t first_static_units(uint64_t n, uint32_t nw) { return n < nw ? n : nw; }

// One wave's side of the queue protocol: take() takes the wave's next slot
// (LDS counter), waits for its chunk in the ring, does the slot's fetch duty
// and names the unit.  Without a slot (busy) it walks the static split.
template <class Plan>
struct UnitTaker {
    WgQueue *L;
    unsigned long long *queue;
    uint64_t n, q0, su, nch, max_iters, iters = 0;
    uint32_t nw, cl, cu, lead, flt = 0;  // flt (lane 0): a wait of this wave gave up
    uint32_t seq = 0;                     // the workgroup's chunk sequence number of the last slot taken
    bool l0;
    Plan plan;
#if MCK_TRACE
    unsigned long long qs_n = 0, qs_sum = 0, qs_max = 0, qs_wait = 0, qs_busy = 0, qs_units = 0;
#endif
    __device__ __forceinline__ UnitTaker(WgQueue *L_, unsigned long long *q, uint64_t n_, uint32_t wave, uint32_t nw_,
                                         bool first, const Plan &p)
        : L(L_), queue(q), n(n_), q0(first ? first_static_units(n_, nw_) : 0),
          su(first ? (uint64_t)wave + nw_ : wave), nch(p.nch), nw(nw_), cl(p.cl), cu(1u << p.cl),
          lead(cu > 4 ? cu / 4 : 1), l0((threadIdx.x & 63u) == 0), plan(p) {
        max_iters = (uint64_t)cu * nch + 4ull * cu + 64;
    }
    // The wave's next slot: false when the wave is done (the queue ran dry,
    // or a wait gave up); else *u = its unit, or n for a tail chunk's slot
    // past the chunk's size.  (busy is re-read from LDS every call -- an
    // atomic load the compiler cannot hoist: one call site of the payload loop
    // for both splits; a second inlined copy made the offsets kernels spill.)
    __device__ __forceinline__ bool take(uint64_t *u) {
        if (__builtin_amdgcn_readfirstlane(lds_ld(&L->busy))) {
            if (su >= n) return false;
            *u = su;
            su += nw;
            return true;
        }
        uint64_t e = 0;
        uint32_t t = 0;
        if (++iters > max_iters) {  // more slots than the launch has: protocol fault
            if (l0) {
                queue_fault(3, iters, 0);
                flt = 1;
            }
            return false;
        }
        if (l0) {
            t = atomicAdd(&L->slot, 1u);
            const uint32_t seq = t >> cl, r = seq % kWgRing;
            Deadline dl(abort_word(queue));
#if MCK_TRACE
            const unsigned long long w0 = wall_clock64();
            unsigned long long f0 = 0;
#endif
            while (((e = lds_ld(&L->entry[r])) >> 32) != seq) {
                __builtin_amdgcn_s_sleep(1);
                MCK_WAIT_GUARD(dl, 2, seq, e)
            }
#if MCK_TRACE
            qs_wait += wall_clock64() - w0;
#endif
            if ((e >> 32) != seq) {  // gave up (fault counted)
                raise_abort(queue);
                e = kNoChunk;
                flt = 1;
            }
            atomicAdd(&L->reads[r], 1u);
            // One taker per chunk (slot cu - lead) fetches the next chunk --
            // after its own chunk is known, so fetches run in chunk order and
            // the first kNoChunk is final.
            if ((t & (cu - 1)) == cu - lead) {
#if MCK_TRACE
                f0 = wall_clock64();
#endif
#if MCK_QFAULT_TEST
                // injected stall: workgroup 3 neither fetches nor publishes
                // its third chunk (no chunk is lost: the other workgroups take
                // every unit), so each of its waves waits out the deadline on
                // that ring entry
                const bool stall = (g_mck_qfault_mode & 1u) && blockIdx.x == 3 && seq == 1;
#else
                constexpr bool stall = false;
#endif
                const uint64_t nid = (e & 0xFFFFFFFFull) == kNoChunk || stall ? kNoChunk : wg_fetch(L, queue, nch);
#if MCK_TRACE
                const unsigned long long df = wall_clock64() - f0;
                qs_n++;
                qs_sum += df;
                qs_max = df > qs_max ? df : qs_max;
#endif
                if (!stall && !wg_publish(L, queue, seq + 1, nid, cl)) flt = 1;
            }
#if MCK_QFAULT_TEST
            // injected give-up: workgroup 3 drops the first unit of its second
            // chunk (after its reads/publish duties, so the rest of the launch
            // runs on)
            if (g_mck_qfault_mode == 0u && blockIdx.x == 3 && seq == 1 && (t & (cu - 1)) == 0 && !flt) {
                queue_fault(9, seq, t);
                e = kNoChunk;
                flt = 1;
            }
#endif
        }
        t = __builtin_amdgcn_readfirstlane(t);
        seq = t >> cl;
        const uint64_t id = uniform64(e) & 0xFFFFFFFFull;
        if (id == kNoChunk) return false;
        // every chunk spans cu slots; a tail chunk's slots past its size are skipped
        const uint32_t k = t & (cu - 1);
        *u = k < plan.size(id) ? q0 + plan.start(id) + k : n;
        return true;
    }
    // The wave's next unit, past any empty slots: false when it is done.
    __device__ __forceinline__ bool take_unit(uint64_t *u) {
        while (take(u))
            if (*u < n) return true;
        return false;
    }
    // After the wave's last take: true in the FIRST wave of the launch whose
    // wait gave up (it claims the bank's fault flag and must run fail_closed).
    __device__ __forceinline__ bool finish(uint32_t wave) {
#if MCK_TRACE
        if (l0 && wave < 16384u) {
            g_mck_qwave[4 * wave] = qs_n;
            g_mck_qwave[4 * wave + 1] = qs_sum;
            g_mck_qwave[4 * wave + 2] = qs_max;
            g_mck_qwave[4 * wave + 3] = qs_wait;
            g_mck_qwave[4 * 16384 + 2 * wave] = qs_units;
            g_mck_qwave[4 * 16384 + 2 * wave + 1] = qs_busy;
        }
#else
        (void)wave;
#endif
        if (__builtin_amdgcn_readfirstlane(lds_ld(&L->busy))) return false;  // no slot
        uint32_t first = 0;
        if (l0 && flt) first = atomicCAS(queue + kQFault * kQStride, 0ull, 1ull) == 0ull;
        return __builtin_amdgcn_readfirstlane(first) != 0;
    }
};

template <bool DYN, bool FIRST = false, class Plan = ChunkPlan, class F>
__device__ __forceinline__ bool for_each_unit(WgQueue *L, unsigned long long *queue, uint64_t n, uint32_t wave,
                                              uint32_t nw, F &&body, const Plan *given = nullptr) {
    if constexpr (DYN) {
        const Plan plan = [&] {
            if constexpr (std::is_same_v<Plan, ChunkPlan>) return given ? *given : ChunkPlan(n - (FIRST ? first_static_units(n, nw) : 0));
            else return *given;
        }();
        UnitTaker<Plan> tk(L, queue, n, wave, nw, FIRST, plan);
        uint64_t u;
        while (tk.take(&u)) {
#if MCK_TRACE
            const unsigned long long b0 = wall_clock64();
#endif
            if (u < n) body(u);
#if MCK_TRACE
            tk.qs_busy += wall_clock64() - b0;
            tk.qs_units += u < n;
            if (tk.l0 && u < n && u < (1ull << 17)) g_mck_unit_end[u] = wall_clock64() | (unsigned long long)(blockIdx.x % kQSub) << 60;
#endif
        }
        return tk.finish(wave);
    } else {
        for (uint64_t u = FIRST ? (uint64_t)wave + nw : wave; u < n; u += nw) body(u);
        return false;
    }
}

// Run by the wave for_each_unit picked after a give-up (wave-uniform): the
// launch did not hash every payload, so it must not read as clean.  The
// caller's error word (if set) gets +1; a verify launch adds `count` to the
// mismatch counter and marks every payload's status 1 -- payloads that are
// hashed after this sweep overwrite theirs with the true result, so each
// status ends as the correct value or 1 ("flagged"), never a stale 0.
template <bool VERIFY>
__device__ __forceinline__ void fail_closed(const BatchArgs &a) {
    const uint32_t lane = threadIdx.x & 63u;
    if (lane == 0) {
        if (a.err_word) atomicAdd(a.err_word, 1u);
        if (VERIFY && a.mismatches) atomicAdd(a.mismatches, (uint32_t)a.count);
    }
    if (VERIFY && a.status)
        for (uint64_t p = lane; p < a.count; p += 64) a.status[p] = 1;
}

// Network-order u32 at an arbitrary byte address (the HG header's payload
// hash, src/mercury_header.c:111-112 writes it with htonl).
__device__ __forceinline__ uint32_t load_be32(const uint8_t *q) {
    return (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | (uint32_t)q[3];
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Payload bytes are read exactly once.  Non-temporal loads keep a batch far
// larger than the 256 MiB Infinity Cache from churning the caches: +13% on the
// 4 GiB headline batch (profiles/r01/ab1.log); a small batch replayed
// back to back is faster with the default policy (it partly hits the cache).
template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint4 *p) {
    if constexpr (NT) {
        const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

__device__ __forceinline__ uint32_t lds32(const uint8_t *lds, uint32_t a) {
    return *reinterpret_cast<const uint32_t *>(lds + a);
}
__device__ __forceinline__ uint64_t lds64(const uint8_t *lds, uint32_t a) {
    return *reinterpret_cast<const uint64_t *>(lds + a);
}

// ---------------------------------------------------------------- CRC-32C --

// a ^ b ^ c in one VALU op: gfx950's v_bitop3_b32 with truth table 0x96
// (there is no v_xor3_b32 on CDNA; hipcc does not form bitop3 from ^ chains).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Z^(16G)(x): main[p][byte_p(x)], tables p=0,1 in LDS region 0 (lc0), p=2,3
// in region 1 (lc1 has +64 KiB in its byte 2); odd p at +128 B.  One step of
// a sub-stream costs 4 v_perm + 2 v_bitop3 (+1 XOR with the data word) per
// 4 bytes.  (Folding the next word into this XOR tree instead -- a look-ahead
// pipeline -- measured 7% slower on the headline batch, profiles/r01/ab3.log.)
__device__ __forceinline__ uint32_t f32s(Tab32<false> t, uint32_t x, uint32_t lc0, uint32_t lc1) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, lc0, 0x0C020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(x, lc0, 0x0C020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(x, lc1, 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(x, lc1, 0x0C020700u);
    return xor3(lds32(t.lds, a0), lds32(t.lds, a1 + 128), lds32(t.lds, a2)) ^ lds32(t.lds, a3 + 128);
}

__device__ __forceinline__ uint32_t f32s(Tab32<true> t, uint32_t x, uint32_t, uint32_t) {
    const uint32_t a0 = (x << 2) & 0x3FCu, a1 = (x >> 6) & 0x3FCu, a2 = (x >> 14) & 0x3FCu, a3 = (x >> 22) & 0x3FCu;
    return xor3(lds32(t.lds, a0), lds32(t.lds, a1 + 1024), lds32(t.lds, a2 + 2048)) ^ lds32(t.lds, a3 + 3072);
}

// Z^(16G)(x) ^ extra: the fourth lookup and the next data word share one bitop3.
__device__ __forceinline__ uint32_t f32sx(Tab32<false> t, uint32_t x, uint32_t extra, uint32_t lc0, uint32_t lc1) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, lc0, 0x0C020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(x, lc0, 0x0C020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(x, lc1, 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(x, lc1, 0x0C020700u);
    return xor3(xor3(lds32(t.lds, a0), lds32(t.lds, a1 + 128), lds32(t.lds, a2)), lds32(t.lds, a3 + 128), extra);
}
__device__ __forceinline__ uint32_t f32sx(Tab32<true> t, uint32_t x, uint32_t extra, uint32_t lc0, uint32_t lc1) {
    return f32s(t, x, lc0, lc1) ^ extra;
}

template <bool LIGHT>
__device__ __forceinline__ uint32_t op32(Tab32<LIGHT> tab, uint32_t o, uint32_t x) {
    const uint32_t base = (LIGHT ? kL32LightMain : kL32Main) + o * 512;
    uint32_t t[8];
#pragma unroll
    for (int h = 0; h < 8; h++) t[h] = lds32(tab.lds, base + h * 64 + (((x >> (4 * h)) & 15u) << 2));
    return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// Lane-dependent operator i of level l of the two-level combine (LDS map
// above; interleaved so that lanes with different i hit different banks).
__device__ __forceinline__ uint32_t oplv32(Tab32<false> tab, uint32_t l, uint32_t i, uint32_t x) {
    const uint32_t base = kL32Lv + l * 4096 + i * 4;
    uint32_t t[8];
#pragma unroll
    for (int h = 0; h < 8; h++) t[h] = lds32(tab.lds, base + h * 512 + (((x >> (4 * h)) & 15u) << 5));
    return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// XOR_q Z^(-4q)(S_q) in the lane, then over the G lanes of the group.  For
// G = 64 on the throughput layout: lane l = 8a + b applies
// Z^(-16b), the 8 lanes of each a XOR-reduce (shuffles only), the groups
// apply Z^(-128a) and XOR-reduce -- two table operators on the lane's path
// instead of six butterfly levels of one each.
template <int LOG2G, class TAB>
__device__ __forceinline__ uint32_t combine32(TAB lds, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                              uint32_t gl) {
    uint32_t x = s0 ^ op32(lds, 0, s1);
    const uint32_t y = s2 ^ op32(lds, 0, s3);
    x ^= op32(lds, 1, y);
    if constexpr (LOG2G == 6 && std::is_same<TAB, Tab32<false>>::value) {
        x = oplv32(lds, 0, gl & 7u, x);
        x ^= __shfl_xor(x, 1, 64);
        x ^= __shfl_xor(x, 2, 64);
        x ^= __shfl_xor(x, 4, 64);
        x = oplv32(lds, 1, gl >> 3, x);
        x ^= __shfl_xor(x, 8, 64);
        x ^= __shfl_xor(x, 16, 64);
        x ^= __shfl_xor(x, 32, 64);
        return x;
    }
#pragma unroll
    for (int k = 0; k < LOG2G; k++) {
        const uint32_t other = __shfl_xor(x, 1 << k, 64);
        const bool bit = (gl >> k) & 1u;
        const uint32_t lo = bit ? other : x, hi = bit ? x : other;
        x = lo ^ op32(lds, 2 + k, hi);
    }
    return x;
}

// LDS fill in 16-byte granules: a replicated entry's 4 neighbouring copies are
// one ds_write_b128 of the same value (8 per thread at 1024 threads instead of
// 32 dword loads + writes); the operator tables are copied as uint4.  The
// throughput layout issues every load of the fill (8 table entries, one
// operator granule, one combine-operator granule per thread) before its first
// write, so the fill costs one global round trip instead of three (round 2 ran
// the three copies one after another, each behind its own wait).
// `issue` runs between the fill's loads and its LDS writes (the kernel's
// first-payload prefetch: issued after the table loads, it does not delay
// their writes).
struct NoIssue {
    __device__ void operator()() const {}
};
template <bool LIGHT, int BLOCK, class F = NoIssue>
__device__ void fill_lds32(uint8_t *lds, const crc32_gpu_pack_t *pk, F &&issue = F{}) {
    uint4 *l4 = reinterpret_cast<uint4 *>(lds);
    const uint4 *ops = reinterpret_cast<const uint4 *>(&pk->ops[0][0][0]);
    const uint32_t nops = pk->nops * 32u;
    if constexpr (LIGHT) {
        // all loads (one main-table granule, up to three operator granules per
        // thread) before the first write: one global round trip, not two
        static_assert(BLOCK == 256 && CRC32_NOPS_MAX * 32 <= 3 * BLOCK, "fill granules per thread");
        issue();
        const uint4 *m = reinterpret_cast<const uint4 *>(&pk->main[0][0]);
        const uint32_t t = threadIdx.x;
        const uint4 mv = m[t];
        auto op_at = [&](uint32_t q) { return ops[q < CRC32_NOPS_MAX * 32u ? q : 0u]; };
        uint4 o0 = op_at(t), o1 = op_at(t + BLOCK), o2 = op_at(t + 2 * BLOCK);
        // (pinned after all four loads are out: the compiler sank each
        // operator load into its predicated store, one round trip apiece)
        asm volatile("" : "+v"(o0.x), "+v"(o0.y), "+v"(o0.z), "+v"(o0.w), "+v"(o1.x), "+v"(o1.y), "+v"(o1.z),
                     "+v"(o1.w), "+v"(o2.x), "+v"(o2.y), "+v"(o2.z), "+v"(o2.w));
        l4[t] = mv;
        if (t < nops) l4[kL32LightMain / 16 + t] = o0;
        if (t + BLOCK < nops) l4[kL32LightMain / 16 + t + BLOCK] = o1;
        if (t + 2 * BLOCK < nops) l4[kL32LightMain / 16 + t + 2 * BLOCK] = o2;
    } else {
        static_assert(BLOCK == 1024 && CRC32_NOPS_MAX * 32 <= BLOCK, "one operator granule per thread");
        const uint32_t t = threadIdx.x;
        const uint4 *lv = reinterpret_cast<const uint4 *>(&pk->lv[0][0][0][0]);  // two-level combine operators
        // loads in range of the pack's arrays whatever nops is (so none waits
        // for the scalar load of nops), stores predicated
        const uint32_t tc = t < CRC32_NOPS_MAX * 32u ? t : 0u, tl = t & 511u;
        uint4 o = ops[tc];
        const uint4 w = lv[tl];
        uint32_t v[8];
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) {
            const uint32_t d = (t + i * BLOCK) << 2;
            const uint32_t region = d >> 14, e = (d >> 6) & 255u, half = (d >> 5) & 1u;
            v[i] = pk->main[2 * region + half][e];
        }
        // keep the operator load up here with the others (the compiler would
        // sink it into the predicated store below, behind a second round trip)
        asm volatile("" : "+v"(o.x), "+v"(o.y), "+v"(o.z), "+v"(o.w));
        issue();
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) l4[t + i * BLOCK] = make_uint4(v[i], v[i], v[i], v[i]);
        if (t < nops) l4[kL32Main / 16 + t] = o;
        if (t < 512u) l4[kL32Lv / 16 + t] = w;
    }
}

// Ring slot j % kRing holds the piece of step j, loaded kRing steps ahead.
//
// Aligned fixed-size payload: base 16-B aligned, len = K * 16G, no masking,
// no pad bytes (tail op is the identity and is skipped).
// Global-address-space views: loads through them are global_load (never
// flat_load, which would also count against lgkmcnt and make every LDS wait
// wait for HBM), and a wave-uniform base in SGPRs gives the saddr form.
typedef const __attribute__((address_space(1))) uint8_t *gbyte_t;
typedef const __attribute__((address_space(1))) u32x4_t *gvec_t;
__device__ __forceinline__ gbyte_t global_ptr(const uint8_t *p, bool uniform) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    return (gbyte_t)(uniform ? uniform64(v) : v);
}
template <bool NT>
__device__ __forceinline__ uint4 ldg16(gbyte_t p) {
    const gvec_t q = (gvec_t)p;
    u32x4_t v;
    if constexpr (NT) v = __builtin_nontemporal_load(q);
    else v = *q;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Aligned step loop without per-step tests: K is a multiple of kRing and
// >= kRing (launch_fixed's aligned test), so every load of the steady loop is
// in range and the last kRing steps run without loads.  The load pointer
// advances by kRing steps per iteration (for G = 64 a wave-uniform SGPR pair:
// saddr loads with the lane offset in one VGPR and the slot in the immediate).
// Each slot's data word is folded into the state before the slot is reloaded,
// so the ring needs no register copies.
// The first kRing steps of a payload (every one in range: K >= kRing).
template <int LOG2G, bool NT>
__device__ __forceinline__ void ring32_load(uint4 (&ring)[kRing], const uint8_t *p, uint32_t gl) {
    constexpr uint32_t S = 16u << LOG2G;
    const gbyte_t lb = global_ptr(p, LOG2G == 6);
#pragma unroll
    for (uint32_t u = 0; u < kRing; u++) ring[u] = ldg16<NT>(lb + (16u * gl + u * S));
}

// loaded: ring already holds the payload's first kRing steps (ring32_load,
// issued by the kernel before its LDS fill for the wave's first payload).
template <int LOG2G, bool NT, class TAB>
__device__ __forceinline__ uint32_t payload32_aligned(TAB lds, const uint8_t *p, uint64_t K64, uint32_t gl,
                                                      uint32_t lc0, uint32_t lc1, uint32_t init,
                                                      uint4 (&ring)[kRing], bool loaded) {
    constexpr uint32_t G = 1u << LOG2G;
    constexpr uint32_t R = kRing;
    constexpr uint32_t S = 16u * G;  // bytes per step
    const uint32_t K = (uint32_t)K64;
    gbyte_t lb = global_ptr(p, LOG2G == 6);
    const uint32_t lo = 16u * gl;
    if (!loaded) ring32_load<LOG2G, NT>(ring, p, gl);
    lb += R * S;
    uint32_t x0 = gl == 0 ? init : 0u, x1 = 0, x2 = 0, x3 = 0;
    // look-ahead: y holds state ^ (data of the step about to run), and the
    // next step's data word rides in the table-XOR tree (2 v_bitop3, no XOR)
    uint32_t y0 = x0 ^ ring[0].x, y1 = ring[0].y, y2 = ring[0].z, y3 = ring[0].w;
    for (uint32_t k = R; k < K; k += R) {
#pragma unroll
        for (uint32_t u = 0; u < R; u++) {
            ring[u] = ldg16<NT>(lb + (lo + u * S));
            const uint4 nx = ring[(u + 1) % R];
            y0 = f32sx(lds, y0, nx.x, lc0, lc1);
            y1 = f32sx(lds, y1, nx.y, lc0, lc1);
            y2 = f32sx(lds, y2, nx.z, lc0, lc1);
            y3 = f32sx(lds, y3, nx.w, lc0, lc1);
        }
        lb += R * S;
    }
#pragma unroll
    for (uint32_t u = 0; u + 1 < R; u++) {
        const uint4 nx = ring[u + 1];
        y0 = f32sx(lds, y0, nx.x, lc0, lc1);
        y1 = f32sx(lds, y1, nx.y, lc0, lc1);
        y2 = f32sx(lds, y2, nx.z, lc0, lc1);
        y3 = f32sx(lds, y3, nx.w, lc0, lc1);
    }
    x0 = f32s(lds, y0, lc0, lc1);
    x1 = f32s(lds, y1, lc0, lc1);
    x2 = f32s(lds, y2, lc0, lc1);
    x3 = f32s(lds, y3, lc0, lc1);
    return combine32<LOG2G>(lds, x0, x1, x2, x3, gl);
}
template <int LOG2G, bool NT, class TAB>
__device__ __forceinline__ uint32_t payload32_aligned(TAB lds, const uint8_t *p, uint64_t K, uint32_t gl,
                                                      uint32_t lc0, uint32_t lc1, uint32_t init) {
    uint4 ring[kRing];
    return payload32_aligned<LOG2G, NT>(lds, p, K, gl, lc0, lc1, init, ring, false);
}

// Any alignment, any length (0 included).  Per-lane window; the wave loops to
// the largest step count of its groups.
template <int LOG2G, bool NT, class TAB>
__device__ __forceinline__ uint32_t payload32_generic(TAB lds, const crc32_gpu_pack_t *pk,
                                                      const uint8_t *p, uint64_t len, uint32_t gl, uint32_t lc0,
                                                      uint32_t lc1) {
    constexpr int G = 1 << LOG2G;
    constexpr int64_t step = 16 * G;
    const uint32_t init = pk->init;
    const uint64_t sa = reinterpret_cast<uint64_t>(p), ea = sa + len;
    const uint64_t a0 = sa & ~15ull, a1 = (ea + 15) & ~15ull;
    const int64_t W = (int64_t)(a1 - a0);
    const int64_t K = (W + step - 1) >> (4 + LOG2G);
    const int64_t r0 = W - K * step;
    const int64_t hs = (int64_t)(sa - a0), he = (int64_t)(ea - a0);
    const int64_t ilen = (int64_t)len;
    const int64_t kmax = LOG2G == 6 ? K : wave_max(K);
    const int64_t lane_off = 16 * (int64_t)gl;

    const gbyte_t g0 = global_ptr(reinterpret_cast<const uint8_t *>(a0), false);
    auto fetch = [&](int64_t k) -> uint4 {
        const int64_t pc = r0 + k * step + lane_off;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < K && pc >= 0) v = ldg16<NT>(g0 + (uint64_t)pc);
        return v;
    };
    // edge handling (crc_gpu_mask.h) for the piece of step k < K
    auto prep = [&](int64_t k, uint4 v) -> uint4 {
        const int64_t pc = r0 + k * step + lane_off;
        if (!mck_piece_clean(pc, hs, he, 4)) {
            const int64_t lo = pc - hs;
            v.x = mck_mask32(v.x, lo, ilen, init);
            v.y = mck_mask32(v.y, lo + 4, ilen, init);
            v.z = mck_mask32(v.z, lo + 8, ilen, init);
            v.w = mck_mask32(v.w, lo + 12, ilen, init);
        }
        return v;
    };

    uint4 ring[kRing];
#pragma unroll
    for (int u = 0; u < kRing; u++) ring[u] = fetch(u);
    uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;
    for (int64_t k = 0; k < kmax; k += kRing) {
#pragma unroll
        for (int u = 0; u < kRing; u++) {
            const int64_t j = k + u;
            const uint4 raw = ring[u];
            ring[u] = fetch(j + kRing);
            if (j < K) {
                const uint4 w = prep(j, raw);
                x0 = f32s(lds, x0 ^ w.x, lc0, lc1);
                x1 = f32s(lds, x1 ^ w.y, lc0, lc1);
                x2 = f32s(lds, x2 ^ w.z, lc0, lc1);
                x3 = f32s(lds, x3 ^ w.w, lc0, lc1);
            }
        }
    }
    uint32_t x = combine32<LOG2G>(lds, x0, x1, x2, x3, gl);
    x = op32(lds, 2 + LOG2G + (uint32_t)(a1 - ea), x);
    if (len < 4) x ^= pk->zinit[len];
    return x;
}

// Step grid of the one-payload-per-wave loops (payload32_g64 / payload64_g64):
// the window of 1 KiB steps ENDS on a 128-B line boundary past the payload
// (16 B before round 3), so every step reads exactly 8 whole
// lines.  With non-temporal loads a line that two steps straddle is fetched
// twice: on C4's byte-packed payloads that was 1.7% of extra HBM requests
// (TCC_EA0_RDREQ: 6.83e7 vs 6.74e7 with NT off, profiles/r03/tcc_c4_nt*.txt;
// NT off costs 11%).  Reads stay inside the last byte's 128-B line, hence
// its page.  The up-to-127 pad bytes are removed by Z^-t, t = 16q + r: the
// tail table Z^-r and the butterfly operators Z^-(16*2^k) for the bits of q.
constexpr uint64_t kGridAlign = 128;

template <class TAB>
__device__ __forceinline__ uint32_t tail32(TAB lds, uint32_t t, uint32_t x) {
    x = op32(lds, 2 + 6 + (t & 15u), x);
#pragma unroll
    for (uint32_t k = 0; k < 3; k++)
        if ((t >> (4 + k)) & 1u) x = op32(lds, 2 + k, x);
    return x;
}

// One payload per wave (G = 64): the window geometry is wave-uniform, so the
// payload base stays in SGPRs, each lane carries a 32-bit offset (saddr-form
// global loads), and "does this step touch an edge?" is a scalar test -- only
// the first/last steps pay for per-lane masking.  Payloads < 2 GiB.
// RAW: no finalisation and the register starts at `reg` (default 0: the
// linear part L(M) of the CRC, used to combine the pieces of a scatter-gather
// object, mchecksum_gpu_ext.hip); a non-zero `reg` continues a running
// register (the XDR walker's fields) and needs len >= 4, since it rides in
// the first four payload bytes (R(reg, M) = R(0, M ^ reg)).
template <bool NT, class TAB, bool RAW = false>
__device__ __forceinline__ uint32_t payload32_g64(TAB lds, const crc32_gpu_pack_t *pk, const uint8_t *p,
                                                  uint64_t len, uint32_t gl, uint32_t lc0, uint32_t lc1,
                                                  uint32_t reg = 0u) {
    const uint32_t init = RAW ? reg : pk->init;
    const uint64_t sa = reinterpret_cast<uint64_t>(p), ea = sa + len;
    const uint64_t a0 = sa & ~15ull, a1 = (ea + kGridAlign - 1) & ~(kGridAlign - 1);
    const uint32_t W = (uint32_t)(a1 - a0);
    const uint32_t K = (W + 1023u) >> 10;
    const uint32_t lead = K * 1024u - W;                 // window starts `lead` bytes into step 0
    const gbyte_t wb = global_ptr(reinterpret_cast<const uint8_t *>(a0 - lead), true);  // step grid origin
    const uint32_t qs = lead + (uint32_t)(sa - a0);      // payload [qs, qe) relative to wb
    const uint32_t qe = lead + (uint32_t)(ea - a0);
    const int32_t ilen = (int32_t)len;
    const uint32_t lo_lane = 16u * gl;
    // steps [kc0, kc1) are clean for every lane
    const uint32_t kc0 = (qs + 4u + 1023u) >> 10;
    const uint32_t kc1 = qe >= 1024u ? (qe - 1024u) / 1024u + 1u : 0u;
    constexpr uint32_t R = kRingOff;

    uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;
    auto fold = [&](uint32_t kk, uint4 v) {
        if (kk < kc0 || kk >= kc1) {  // wave-uniform: an edge step
            const int32_t lo = (int32_t)(kk * 1024u + lo_lane) - (int32_t)qs;
            v.x = mck_mask32(v.x, lo, ilen, init);
            v.y = mck_mask32(v.y, lo + 4, ilen, init);
            v.z = mck_mask32(v.z, lo + 8, ilen, init);
            v.w = mck_mask32(v.w, lo + 12, ilen, init);
        }
        x0 = f32s(lds, x0 ^ v.x, lc0, lc1);
        x1 = f32s(lds, x1 ^ v.y, lc0, lc1);
        x2 = f32s(lds, x2 ^ v.z, lc0, lc1);
        x3 = f32s(lds, x3 ^ v.w, lc0, lc1);
    };
    // Loads go through global (address-space 1) pointers -- flat loads would
    // also count against lgkmcnt, so every LDS wait of the fold would wait for
    // the ring's HBM loads too -- and only step 0 tests lanes (the ones before
    // the window start read nothing); the steady loop loads unconditionally.
    uint4 ring[R];
    ring[0] = K > 0 && lo_lane >= lead ? ldg16<NT>(wb + lo_lane) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t u = 1; u < R; u++) ring[u] = u < K ? ldg16<NT>(wb + (u * 1024u + lo_lane)) : make_uint4(0, 0, 0, 0);
    uint32_t k = 0;
    for (; k + 2 * R <= K; k += R) {
#pragma unroll
        for (uint32_t u = 0; u < R; u++) {
            const uint4 v = ring[u];
            ring[u] = ldg16<NT>(wb + ((k + u + R) * 1024u + lo_lane));
            fold(k + u, v);
        }
    }
    for (; k < K; k += R) {
#pragma unroll
        for (uint32_t u = 0; u < R; u++) {
            const uint4 v = ring[u];
            if (k + u + R < K) ring[u] = ldg16<NT>(wb + ((k + u + R) * 1024u + lo_lane));
            if (k + u < K) fold(k + u, v);
        }
    }
    uint32_t x = combine32<6>(lds, x0, x1, x2, x3, gl);
    x = tail32(lds, (uint32_t)(a1 - ea), x);
    if (!RAW && len < 4) x ^= pk->zinit[len];
    return x;
}

// Byte-balanced static partition of an offsets batch: wave w owns payloads
// whose start offset lies in [off0 + total*w/nw, off0 + total*(w+1)/nw).
__device__ __forceinline__ uint64_t lower_bound_u64(const uint64_t *a, uint64_t n, uint64_t key) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void wave_range(const uint64_t *off, uint64_t count, uint32_t wave, uint32_t nw,
                                           uint64_t *first, uint64_t *last) {
    const uint64_t o0 = off[0], total = off[count] - o0;
    const uint64_t q = total / nw, r = total % nw;
    const uint64_t lo = o0 + q * wave + (r * wave) / nw;
    const uint64_t hi = o0 + q * (wave + 1) + (r * (wave + 1)) / nw;
    *first = wave == 0 ? 0 : lower_bound_u64(off, count, lo);
    *last = wave + 1 == nw ? count : lower_bound_u64(off, count, hi);
}

// Diagnostic build (-DMCK_TRACE=1, tools/tail_trace.py): per-wave clock
// stamps (kernel entry, after the LDS fill, exit) of the last launch.
#ifndef MCK_TRACE
#define MCK_TRACE 0
#endif
#if MCK_TRACE
constexpr int kTraceWaves = 16384;
__device__ unsigned long long g_mck_trace[3 * kTraceWaves];
// the XCD each wave ran on (hardware register XCC_ID), stamped at entry
__device__ unsigned int g_mck_trace_xcc[kTraceWaves];
// the shader-clock counter (clock64) at entry and exit: with the wall stamps
// the clock each XCD ran at over the wave's life (tools/xcd_clock.py)
__device__ unsigned long long g_mck_trace_clk[2 * kTraceWaves];
__device__ __forceinline__ unsigned int xcc_id() {
    unsigned int r;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(r));
    return r & 15u;
}
#define MCK_STAMP(w, k)                                                                   \
    do {                                                                                  \
        if ((threadIdx.x & 63u) == 0 && (w) < kTraceWaves) {                              \
            g_mck_trace[3 * (w) + (k)] = wall_clock64();                                  \
            if ((k) == 0) g_mck_trace_xcc[(w)] = xcc_id();                                \
            if ((k) != 1) g_mck_trace_clk[2 * (w) + ((k) >> 1)] = clock64();              \
        }                                                                                 \
    } while (0)
#else
#define MCK_STAMP(w, k) do { } while (0)
#endif

// A verify launch counts its mismatches per lane (nbad) and adds them to the
// caller's counter once per WORKGROUP at its end.  Device-scope atomics on one
// word serialize: one per bad payload (or per wave) made 4096 bad 4 KiB
// messages a 58 us kernel against 19 us when they all matched
// (tools/lat_offsets.py), so a corrupted buffer cost three times a good one.
// Every thread of the workgroup calls this, once.
__device__ __forceinline__ void add_mismatches(uint32_t *ctr, uint32_t nbad) {
    __shared__ uint32_t wg_bad;
    if (threadIdx.x == 0) wg_bad = 0;
    __syncthreads();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) nbad += __shfl_xor(nbad, d, 64);
    if ((threadIdx.x & 63u) == 0 && nbad) atomicAdd(&wg_bad, nbad);
    __syncthreads();
    if (threadIdx.x == 0 && wg_bad && ctr) atomicAdd(ctr, wg_bad);
}

template <typename T, bool VERIFY>
__device__ __forceinline__ void emit(const BatchArgs &a, uint64_t p, T v, uint32_t &nbad) {
    if (VERIFY) {
        if (a.bswap) {
            if constexpr (sizeof(T) == 8) v = (T)__builtin_bswap64((uint64_t)v);
            else v = (T)__builtin_bswap32((uint32_t)v);
        }
        const bool bad = reinterpret_cast<const T *>(a.expected)[p] != v;
        if (a.status) a.status[p] = bad ? 1 : 0;
        nbad += bad;
    } else {
        reinterpret_cast<T *>(a.out)[p] = v;
    }
}

template <bool LIGHT>
constexpr int kBlk32 = LIGHT ? kLightBlock : kBlock;

template <int LOG2G, int MODE, bool VERIFY, bool NT, bool LIGHT = false>
__global__ __launch_bounds__(kBlk32<LIGHT>, 1) void crc32c_batch_kernel(BatchArgs a) {
    constexpr int kWavesPerBlock = kBlk32<LIGHT> / 64;
    __shared__ __attribute__((aligned(16))) uint8_t lds_raw[LIGHT ? kL32LightBytes : kL32Bytes];
    const crc32_gpu_pack_t *pk = reinterpret_cast<const crc32_gpu_pack_t *>(a.pack);
    MCK_STAMP(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6), 0);
    constexpr int PPW = 64 >> LOG2G;
    const uint64_t units = MODE == kOffsets ? a.count : (a.count + PPW - 1) / PPW;
    __shared__ WgQueue wgq;
    constexpr bool DYN = dyn_policy(32, MODE, NT, LIGHT);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & ((1u << LOG2G) - 1u), grp = lane >> LOG2G;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    // Aligned batches on the static split (C2): the loads of the wave's first
    // payload go out inside the LDS table fill, so their HBM round trip
    // overlaps the fill's.  The queue path (the headline) keeps its first unit
    // dynamic: a static first unit there measured 1% slower (round 3); the
    // light layout gained nothing from it.
    constexpr bool PRE = MODE == kFixedAligned && !LIGHT && !DYN;
    // model words read once, ahead of any store (scalar loads; read after the
    // barrier they became a vector load per payload whose wait, merged with
    // the ring's at the prefetch branch, cost a vmcnt(0) per payload)
    const uint32_t init = pk->init, xorout = pk->xorout;
    uint4 ring0[kRing];
    const bool pre = PRE && wave < units;
    if (DYN && threadIdx.x == 0) wg_queue_init(&wgq, a.queue, units);
    fill_lds32<LIGHT, kBlk32<LIGHT>>(lds_raw, pk, [&] {
        // Throughput layout: unconditional (a wave without a first unit reads
        // the last payload's first steps) -- loads under a branch leave the
        // waitcnt pass a merge point, where it falls back to vmcnt(0) for the
        // fill's writes.  Light layout (small batches: most of its 8192 waves
        // may have no unit): only waves with a first unit load, and before the
        // fill's loads (fill_lds32 runs `issue` first there), so the fill's
        // waits count the same on both paths.
        if constexpr (PRE) {
            const uint64_t p = (uint64_t)wave * PPW + grp;
            if (!LIGHT || pre) ring32_load<LOG2G, NT>(ring0, a.base + (p < a.count ? p : a.count - 1) * a.stride, gl);
        }
    });
    __syncthreads();
    MCK_STAMP(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6), 1);
    const Tab32<LIGHT> lds{lds_raw};

    const uint32_t lc0 = (lane & 31u) << 2, lc1 = lc0 | 0x10000u;
    uint32_t nbad = 0;  // verify: this lane's mismatches (add_mismatches)

    if (MODE == kOffsets) {
        auto one = [&](uint64_t p) {
            const uint64_t m0 = a.offsets[p], m1 = a.offsets[p + 1];
            // message mode: a message shorter than its headers fails verification
            const bool short_msg = a.msg && m1 - m0 < a.pay_off;
            const uint64_t o = a.msg ? (short_msg ? m1 : m0 + a.pay_off) : m0;
            const uint64_t n = m1 - o;
            const uint32_t x = n < (1ull << 31) ? payload32_g64<NT>(lds, pk, a.base + o, n, gl, lc0, lc1)
                                                : payload32_generic<LOG2G, NT>(lds, pk, a.base + o, n, gl, lc0, lc1);
            if (gl == 0) {
                if (VERIFY && a.msg) {
                    const bool bad = short_msg || load_be32(a.base + m0 + a.hash_off) != (x ^ xorout);
                    if (a.status) a.status[p] = bad ? 1 : 0;
                    nbad += bad;
                } else {
                    emit<uint32_t, VERIFY>(a, p, x ^ xorout, nbad);
                }
            }
        };
        if constexpr (!LIGHT) {
            if (for_each_unit<true>(&wgq, a.queue, units, wave, nw, one)) fail_closed<VERIFY>(a);
        } else {  // static: a byte-balanced contiguous range per wave
            uint64_t first, last;
            wave_range(a.offsets, a.count, wave, nw, &first, &last);
            for (uint64_t p = first; p < last; p++) one(p);
        }
        if constexpr (VERIFY) add_mismatches(a.mismatches, nbad);
        MCK_STAMP(wave, 2);
        return;
    }
    auto unit = [&](uint64_t u, bool loaded) {
        const uint64_t p = u * PPW + grp;
        const bool act = p < a.count;
        const uint64_t pc = act ? p : a.count - 1;
        uint32_t x;
        if (MODE == kFixedAligned)
            x = payload32_aligned<LOG2G, NT>(lds, a.base + pc * a.stride, a.len >> (4 + LOG2G), gl, lc0, lc1, init, ring0,
                                             loaded);
        else
            x = payload32_generic<LOG2G, NT>(lds, pk, a.base + pc * a.stride, a.len, gl, lc0, lc1);
        if (act && gl == 0) emit<uint32_t, VERIFY>(a, p, x ^ xorout, nbad);
    };
    // The prefetched first unit runs in a copy of the payload loop of its own:
    // one copy behind a loaded/not-loaded branch leaves the prefetch loads
    // pending at the loop head in the waitcnt pass's view, and it then waited
    // vmcnt(0) -- the previous payload's CRC store included -- at every payload.
    if (PRE && pre) unit(wave, true);
    const bool faulted = for_each_unit<DYN, PRE>(&wgq, a.queue, units, wave, nw, [&](uint64_t u) { unit(u, false); });
    if (faulted) fail_closed<VERIFY>(a);
    if constexpr (VERIFY) add_mismatches(a.mismatches, nbad);
    MCK_STAMP(wave, 2);
}

// Z^n(x) from the base-16 digit tables; n and x are wave-uniform on the chunk
// paths (mchecksum_gpu_ext.hip) and the split CRC-64 pieces below, so the table words come through the scalar cache.
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

// ----------------------------------------------------------------- CRC-64 --

__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
    return (uint64_t)xor3((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32 |
           xor3((uint32_t)a, (uint32_t)b, (uint32_t)c);
}

// XOR of 16 table words and one more value: 8 bitop3 per 32-bit half.
__device__ __forceinline__ uint64_t xor17(const uint64_t *r, uint64_t extra) {
    const uint64_t a = xor3_64(r[0], r[1], r[2]), b = xor3_64(r[3], r[4], r[5]), c = xor3_64(r[6], r[7], r[8]);
    const uint64_t d = xor3_64(r[9], r[10], r[11]), e = xor3_64(r[12], r[13], r[14]);
    return xor3_64(xor3_64(r[15], extra, a), xor3_64(b, c, d), e);
}

// Per-lane lookup address registers of f64x: the lane-copy offset in byte 0
// of four persistent registers, whose byte 1 the pair index is written into
// by one v_and_b32_sdwa each (dst_unused:UNUSED_PRESERVE keeps byte 0), so a
// replicated lookup costs one VALU op and no separate masking.
struct Lane64 {
    uint32_t lc;
    uint32_t al[4];
};
__device__ __forceinline__ Lane64 lane64(uint32_t lc) { return Lane64{lc, {lc, lc, lc, lc}}; }

// (byte B of x) & 0xF8: a 5-bit field scaled by 8, its own f5 address;
// (byte B of t) & 0x3F into byte 1 of the lane-copy register a.
#define MCK_SDWA_P6(B)                                                                              \
    __device__ __forceinline__ uint32_t sdwa_f8_##B(uint32_t x) {                                   \
        uint32_t r;                                                                                 \
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "         \
            "src1_sel:BYTE_" #B : "=v"(r) : "s"(0xF8u), "v"(x));                                    \
        return r;                                                                                   \
    }                                                                                               \
    __device__ __forceinline__ void sdwa_p6_##B(uint32_t &a, uint32_t t) {                          \
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "   \
            "src1_sel:BYTE_" #B : "+v"(a) : "s"(0x3Fu), "v"(t));                                    \
    }
MCK_SDWA_P6(0)
MCK_SDWA_P6(1)
MCK_SDWA_P6(2)
MCK_SDWA_P6(3)
#undef MCK_SDWA_P6
// Byte i of the result: bits 0..2 of byte i of the low half xl and, above
// them, bits 0..4 of byte i of the high half xh -- the 6-bit index of pair
// table i (bytes i and i + 4 of the word; sdwa_p6 keeps 6 bits).  One shift
// and one v_bfi_b32 (mask in an SGPR; VOP3 takes no literal on gfx9) for all
// four pair indexes: round 1 paired bytes (2i, 2i+1) within a half, which took
// a shift and a bit-select per half (28 -> 26 VALU ops per 8-byte word on a
// VALU-bound loop).  The C form (x & m) | (y & ~m) compiled to v_and +
// v_and_or: one op more.  (Round 5: the bit-select as a v_bitop3 with its mask
// in a VGPR, which the probe issues faster, measured +-0 in the loop.)
__device__ __forceinline__ uint32_t gather6(uint32_t xl, uint32_t xh) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x07070707u), "v"(xl), "v"(xh << 3));
    return r;
}
__device__ __forceinline__ uint64_t xor13(const uint64_t *r, uint64_t extra) {
    const uint64_t a = xor3_64(r[0], r[1], r[2]), b = xor3_64(r[3], r[4], r[5]), c = xor3_64(r[6], r[7], r[8]);
    return xor3_64(a, b, xor3_64(c, xor3_64(r[9], r[10], r[11]), extra));
}
// Z^(16G)(x) ^ next from the 12 tables f5/f6 (LDS map above): 12 address
// ops, 2 for the gather, 12 v_bitop3 for the XOR tree (the next data word
// rides in its 13th input).
__device__ __forceinline__ uint64_t f64x(const uint8_t *lds, uint64_t x, uint64_t next, Lane64 &ln) {
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    // byte i of t: bits 0..2 of bytes i and i + 4 of the word (bit-select)
    const uint32_t t = gather6(xl, xh);
    uint64_t r[12];
    r[0] = lds64(lds, sdwa_f8_0(xl) + kL64P5 + 0 * 256);
    r[1] = lds64(lds, sdwa_f8_1(xl) + kL64P5 + 1 * 256);
    r[2] = lds64(lds, sdwa_f8_2(xl) + kL64P5 + 2 * 256);
    r[3] = lds64(lds, sdwa_f8_3(xl) + kL64P5 + 3 * 256);
    r[4] = lds64(lds, sdwa_f8_0(xh) + kL64P5 + 4 * 256);
    r[5] = lds64(lds, sdwa_f8_1(xh) + kL64P5 + 5 * 256);
    r[6] = lds64(lds, sdwa_f8_2(xh) + kL64P5 + 6 * 256);
    r[7] = lds64(lds, sdwa_f8_3(xh) + kL64P5 + 7 * 256);
    sdwa_p6_0(ln.al[0], t);
    r[8] = lds64(lds, ln.al[0] + kL64P6 + 0 * 16384);
    sdwa_p6_1(ln.al[1], t);
    r[9] = lds64(lds, ln.al[1] + kL64P6 + 1 * 16384);
    sdwa_p6_2(ln.al[2], t);
    r[10] = lds64(lds, ln.al[2] + kL64P6 + 2 * 16384);
    sdwa_p6_3(ln.al[3], t);
    r[11] = lds64(lds, ln.al[3] + kL64P6 + 3 * 16384);
    return xor13(r, next);
}

template <bool OG>
__device__ __forceinline__ uint64_t op64(const uint8_t *lds, const crc64_gpu_pack_t *pk, uint32_t o, uint64_t x) {
    uint64_t r[16];
    if constexpr (OG) {
        const uint64_t *t = &pk->ops[o][0][0];
#pragma unroll
        for (int h = 0; h < 16; h++) r[h] = t[h * 16 + ((x >> (4 * h)) & 15u)];
    } else {
        const uint32_t base = kL64Main + o * 2048;
#pragma unroll
        for (int h = 0; h < 16; h++) r[h] = lds64(lds, base + h * 128 + (uint32_t)(((x >> (4 * h)) & 15u) << 3));
    }
    return xor17(r, 0);
}

template <int OM>
__device__ __forceinline__ uint64_t opm64(const uint8_t *lds, const crc64_gpu_pack_t *pk, uint32_t o, uint64_t x) {
    if constexpr (OM == kOpsMix) {
        if (o >= 1 && o <= 6) return op64<false>(lds, pk, o - 1, x);  // butterflies at kL64Main
        return op64<true>(lds, pk, o, x);
    } else {
        return op64<OM == kOpsGlobal>(lds, pk, o, x);
    }
}

template <int LOG2G, int OM>
__device__ __forceinline__ uint64_t combine64(const uint8_t *lds, const crc64_gpu_pack_t *pk, uint64_t s0, uint64_t s1,
                                              uint32_t gl) {
    uint64_t x = s0 ^ opm64<OM>(lds, pk, 0, s1);
#pragma unroll
    for (int k = 0; k < LOG2G; k++) {
        const uint64_t other = __shfl_xor(x, 1 << k, 64);
        const bool bit = (gl >> k) & 1u;
        const uint64_t lo = bit ? other : x, hi = bit ? x : other;
        x = lo ^ opm64<OM>(lds, pk, 1 + k, hi);
    }
    return x;
}

// The same sum as a halving reduction (lane 0 of each group of G lanes): at
// distance d = G/2, ..., 2, 1 the lanes below d add Z^-(16d) of the state d
// lanes up, so level d's lookups run on d lanes where the butterfly's ran on
// all G, and lane 0 ends with the sum (payload64_g64 then runs its tail
// operators on lane 0 alone).  C4-layout CRC-64 +3.1% / +2.4%
// (profiles/r06/ab_c4_64_combine.log, ab_lane0.log: the combine and tail were
// 14% of that kernel's time; running the tail on the wave-uniform value
// through the scalar cache instead cost 9%).  The C3 split pieces and the
// segment chunk pass measured +-0 / -0.9% with it and keep the butterfly;
// payload64_g64 uses it only in the offsets kernels (kOpsMix).
template <int LOG2G, int OM>
__device__ __forceinline__ uint64_t combine64_lane0(const uint8_t *lds, const crc64_gpu_pack_t *pk, uint64_t s0,
                                                    uint64_t s1, uint32_t gl) {
    uint64_t x = s0 ^ opm64<OM>(lds, pk, 0, s1);
#pragma unroll
    for (int k = LOG2G - 1; k >= 0; k--) {
        const uint32_t d = 1u << k;
        const uint64_t hi = __shfl_down(x, d, 64);
        if (gl < d) x ^= opm64<OM>(lds, pk, 1 + k, hi);
    }
    return x;
}

template <int BLOCK, int OM>
__device__ void fill_lds64(uint8_t *lds, const crc64_gpu_pack_t *pk) {
    uint64_t *l = reinterpret_cast<uint64_t *>(lds);
    uint4 *l4 = reinterpret_cast<uint4 *>(lds);
    // f6: entry v of table i at i*16 KiB + v*256 B, 32 copies (two per 16-B write)
    for (uint32_t q = threadIdx.x; q < 4096u; q += BLOCK) {
        const uint64_t v = pk->f6[q >> 10][(q >> 4) & 63u];
        l4[kL64P6 / 16 + q] = make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)v, (uint32_t)(v >> 32));
    }
    for (uint32_t d = threadIdx.x; d < 256u; d += BLOCK) l[kL64P5 / 8 + d] = pk->f5[d >> 5][d & 31u];
    if constexpr (OM == kOpsLds) {
        const uint4 *ops = reinterpret_cast<const uint4 *>(&pk->ops[0][0][0]);
        const uint32_t nops = pk->nops * 128u;
        for (uint32_t q = threadIdx.x; q < nops; q += BLOCK) l4[kL64Main / 16 + q] = ops[q];
    } else if constexpr (OM == kOpsMix) {  // ops 1..6 (needs G = 64: nops >= 7)
        const uint4 *ops = reinterpret_cast<const uint4 *>(&pk->ops[1][0][0]);
        for (uint32_t q = threadIdx.x; q < 6u * 128u; q += BLOCK) l4[kL64Main / 16 + q] = ops[q];
    }
}

__device__ __forceinline__ uint64_t lo64(uint4 v) { return (uint64_t)v.y << 32 | v.x; }
__device__ __forceinline__ uint64_t hi64(uint4 v) { return (uint64_t)v.w << 32 | v.z; }

// Aligned CRC-64 loop: a 4-deep ring of dwordx4 loads per lane, two 64-bit
// sub-streams per lane.  Whole rings (K a multiple of the ring, K >= 2
// rings) take payload64_even: no load or step is conditional, so the waitcnt
// pass sees one load per step and waits vmcnt(R - 1) throughout.  In the
// merged segment kernel the general loop -- conditional ring fill and tail --
// kept only one or two loads in flight (vmcnt(1) in its steady loop,
// vmcnt(0) after the fill): +2.5% on seg for the even form
// (profiles/r04/ab_seg_even.log).
constexpr int kRing64 = 4;
template <int LOG2G, bool NT, int OM>
__device__ __forceinline__ uint64_t payload64_even(const uint8_t *lds, const crc64_gpu_pack_t *pk, const uint8_t *p,
                                                   uint32_t K, uint32_t gl, uint32_t lc, uint64_t init) {
    constexpr int G = 1 << LOG2G;
    constexpr int R = kRing64;
    Lane64 ln = lane64(lc);
    gbyte_t src = global_ptr(p, LOG2G == 6) + 16u * gl;
    uint4 ring[R];
#pragma unroll
    for (int u = 0; u < R; u++) ring[u] = ldg16<NT>(src + u * (16u * G));
    // x holds state ^ (the data word of the step about to run)
    uint64_t x0 = (gl == 0 ? init : 0ull) ^ lo64(ring[0]), x1 = hi64(ring[0]);
    for (uint32_t k = R; k < K; k += R) {
        src += R * (16u * G);
#pragma unroll
        for (int u = 0; u < R; u++) {
            ring[u] = ldg16<NT>(src + u * (16u * G));
            const uint4 nx = ring[(u + 1) % R];
            x0 = f64x(lds, x0, lo64(nx), ln);
            x1 = f64x(lds, x1, hi64(nx), ln);
        }
    }
#pragma unroll
    for (int u = 0; u < R; u++) {
        const uint4 nx = u + 1 < R ? ring[u + 1] : make_uint4(0, 0, 0, 0);
        x0 = f64x(lds, x0, lo64(nx), ln);
        x1 = f64x(lds, x1, hi64(nx), ln);
    }
    return combine64<LOG2G, OM>(lds, pk, x0, x1, gl);
}

// The split pieces' loop (G = 64, K a multiple of the ring and >= 2 rings):
// ring64_load issues a piece's first kRing64 steps -- early, while the
// previous piece still combines -- and fold64_ring runs the piece from them,
// leaving the two sub-stream registers uncombined.
template <bool NT>
__device__ __forceinline__ void ring64_load(uint4 (&ring)[kRing64], const uint8_t *p, uint32_t gl) {
    const gbyte_t src = global_ptr(p, true) + 16u * gl;
#pragma unroll
    for (int u = 0; u < kRing64; u++) ring[u] = ldg16<NT>(src + u * 1024u);
}
template <bool NT>
__device__ __forceinline__ void fold64_ring(const uint8_t *lds, uint4 (&ring)[kRing64], const uint8_t *p, uint32_t K,
                                            uint32_t gl, Lane64 &ln, uint64_t init, uint64_t *s0, uint64_t *s1) {
    constexpr int R = kRing64;
    gbyte_t src = global_ptr(p, true) + 16u * gl;
    uint64_t x0 = (gl == 0 ? init : 0ull) ^ lo64(ring[0]), x1 = hi64(ring[0]);
    for (uint32_t k = R; k < K; k += R) {
        src += R * 1024u;
#pragma unroll
        for (int u = 0; u < R; u++) {
            ring[u] = ldg16<NT>(src + u * 1024u);
            const uint4 nx = ring[(u + 1) % R];
            x0 = f64x(lds, x0, lo64(nx), ln);
            x1 = f64x(lds, x1, hi64(nx), ln);
        }
    }
#pragma unroll
    for (int u = 0; u < R; u++) {
        const uint4 nx = u + 1 < R ? ring[u + 1] : make_uint4(0, 0, 0, 0);
        x0 = f64x(lds, x0, lo64(nx), ln);
        x1 = f64x(lds, x1, hi64(nx), ln);
    }
    *s0 = x0;
    *s1 = x1;
}

template <int LOG2G, bool NT, int OM>
__device__ __forceinline__ uint64_t payload64_aligned(const uint8_t *lds, const crc64_gpu_pack_t *pk, const uint8_t *p,
                                                      uint32_t K, uint32_t gl, uint32_t lc, uint64_t init) {
    constexpr int G = 1 << LOG2G;
    constexpr int R = kRing64;
    if (K % R == 0 && K >= 2 * R) return payload64_even<LOG2G, NT, OM>(lds, pk, p, K, gl, lc, init);
    Lane64 ln = lane64(lc);
    // global (address-space 1) loads: a flat load would also hold up every LDS wait
    const gbyte_t src = global_ptr(p, LOG2G == 6) + 16u * gl;
    auto ldk = [&](uint32_t k) { return ldg16<NT>(src + (uint64_t)k * (16u * G)); };
    uint4 ring[R];
#pragma unroll
    for (int u = 0; u < R; u++) ring[u] = (uint32_t)u < K ? ldk(u) : make_uint4(0, 0, 0, 0);
    // x holds state ^ (the data word of the step about to run)
    uint64_t x0 = (gl == 0 ? init : 0ull) ^ lo64(ring[0]), x1 = hi64(ring[0]);
    uint32_t k = 0;
    for (; k + 2 * R <= K; k += R) {  // every load and look-ahead in range
#pragma unroll
        for (int u = 0; u < R; u++) {
            ring[u] = ldk(k + u + R);
            const uint4 nx = ring[(u + 1) % R];
            x0 = f64x(lds, x0, lo64(nx), ln);
            x1 = f64x(lds, x1, hi64(nx), ln);
        }
    }
    for (; k < K; k += R) {
#pragma unroll
        for (int u = 0; u < R; u++) {
            if (k + u + R < K) ring[u] = ldk(k + u + R);
            if (k + u < K) {
                const uint4 nx = k + u + 1 < K ? ring[(u + 1) % R] : make_uint4(0, 0, 0, 0);
                x0 = f64x(lds, x0, lo64(nx), ln);
                x1 = f64x(lds, x1, hi64(nx), ln);
            }
        }
    }
    return combine64<LOG2G, OM>(lds, pk, x0, x1, gl);
}

template <int LOG2G, bool NT, int OM = kOpsLds>
__device__ __forceinline__ uint64_t payload64_generic(const uint8_t *lds, const crc64_gpu_pack_t *pk,
                                                      const uint8_t *p, uint64_t len, uint32_t gl, uint32_t lc) {
    constexpr int G = 1 << LOG2G;
    constexpr int64_t step = 16 * G;
    const uint64_t init = pk->init;
    const uint64_t sa = reinterpret_cast<uint64_t>(p), ea = sa + len;
    const uint64_t a0 = sa & ~15ull, a1 = (ea + 15) & ~15ull;
    const int64_t W = (int64_t)(a1 - a0);
    const int64_t K = (W + step - 1) >> (4 + LOG2G);
    const int64_t r0 = W - K * step;
    const int64_t hs = (int64_t)(sa - a0), he = (int64_t)(ea - a0);
    const int64_t ilen = (int64_t)len;
    const int64_t kmax = LOG2G == 6 ? K : wave_max(K);
    const int64_t lane_off = 16 * (int64_t)gl;

    const gbyte_t g0 = global_ptr(reinterpret_cast<const uint8_t *>(a0), false);
    auto fetch = [&](int64_t k) -> uint4 {
        const int64_t pc = r0 + k * step + lane_off;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < K && pc >= 0) v = ldg16<NT>(g0 + (uint64_t)pc);
        return v;
    };
    // edge handling (crc_gpu_mask.h) for the piece of step k < K
    auto prep = [&](int64_t k, uint4 v, uint64_t *w0, uint64_t *w1) {
        const int64_t pc = r0 + k * step + lane_off;
        *w0 = lo64(v);
        *w1 = hi64(v);
        if (!mck_piece_clean(pc, hs, he, 8)) {
            const int64_t lo = pc - hs;
            *w0 = mck_mask64(*w0, lo, ilen, init);
            *w1 = mck_mask64(*w1, lo + 8, ilen, init);
        }
    };

    uint4 ring[kRing];
#pragma unroll
    for (int u = 0; u < kRing; u++) ring[u] = fetch(u);
    uint64_t x0 = 0, x1 = 0;
    Lane64 ln = lane64(lc);
    for (int64_t k = 0; k < kmax; k += kRing) {
#pragma unroll
        for (int u = 0; u < kRing; u++) {
            const int64_t j = k + u;
            const uint4 raw = ring[u];
            ring[u] = fetch(j + kRing);
            if (j < K) {
                uint64_t w0, w1;
                prep(j, raw, &w0, &w1);
                x0 = f64x(lds, x0 ^ w0, 0, ln);
                x1 = f64x(lds, x1 ^ w1, 0, ln);
            }
        }
    }
    uint64_t x = combine64<LOG2G, OM>(lds, pk, x0, x1, gl);
    x = opm64<OM>(lds, pk, 1 + LOG2G + (uint32_t)(a1 - ea), x);
    if (len < 8) x ^= pk->zinit[len];
    return x;
}

template <int OM>
__device__ __forceinline__ uint64_t tail64(const uint8_t *lds, const crc64_gpu_pack_t *pk, uint32_t t, uint64_t x) {
    x = opm64<OM>(lds, pk, 1 + 6 + (t & 15u), x);
#pragma unroll
    for (uint32_t k = 0; k < 3; k++)
        if ((t >> (4 + k)) & 1u) x = opm64<OM>(lds, pk, 1 + k, x);
    return x;
}

// CRC-64 counterpart of payload32_g64 (a non-zero RAW `reg` needs len >= 8).
template <bool NT, bool RAW = false, int OM = kOpsLds>
__device__ __forceinline__ uint64_t payload64_g64(const uint8_t *lds, const crc64_gpu_pack_t *pk, const uint8_t *p,
                                                  uint64_t len, uint32_t gl, uint32_t lc, uint64_t reg = 0ull) {
    const uint64_t init = RAW ? reg : pk->init;
    const uint64_t sa = reinterpret_cast<uint64_t>(p), ea = sa + len;
    const uint64_t a0 = sa & ~15ull, a1 = (ea + kGridAlign - 1) & ~(kGridAlign - 1);
    const uint32_t W = (uint32_t)(a1 - a0);
    const uint32_t K = (W + 1023u) >> 10;
    const uint32_t lead = K * 1024u - W;
    const gbyte_t wb = global_ptr(reinterpret_cast<const uint8_t *>(a0 - lead), true);
    const uint32_t qs = lead + (uint32_t)(sa - a0);
    const uint32_t qe = lead + (uint32_t)(ea - a0);
    const int32_t ilen = (int32_t)len;
    const uint32_t lo_lane = 16u * gl;
    const uint32_t kc0 = (qs + 8u + 1023u) >> 10;
    const uint32_t kc1 = qe >= 1024u ? (qe - 1024u) / 1024u + 1u : 0u;
    constexpr uint32_t R = kRingOff64;

    uint64_t x0 = 0, x1 = 0;
    Lane64 ln = lane64(lc);
    auto fold = [&](uint32_t kk, uint4 v) {
        uint64_t w0 = lo64(v), w1 = hi64(v);
        if (kk < kc0 || kk >= kc1) {  // wave-uniform: an edge step
            const int32_t lo = (int32_t)(kk * 1024u + lo_lane) - (int32_t)qs;
            w0 = mck_mask64(w0, lo, ilen, init);
            w1 = mck_mask64(w1, lo + 8, ilen, init);
        }
        x0 = f64x(lds, x0 ^ w0, 0, ln);
        x1 = f64x(lds, x1 ^ w1, 0, ln);
    };
    uint4 ring[R];
    ring[0] = K > 0 && lo_lane >= lead ? ldg16<NT>(wb + lo_lane) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t u = 1; u < R; u++) ring[u] = u < K ? ldg16<NT>(wb + (u * 1024u + lo_lane)) : make_uint4(0, 0, 0, 0);
    uint32_t k = 0;
    for (; k + 2 * R <= K; k += R) {
#pragma unroll
        for (uint32_t u = 0; u < R; u++) {
            const uint4 v = ring[u];
            ring[u] = ldg16<NT>(wb + ((k + u + R) * 1024u + lo_lane));
            fold(k + u, v);
        }
    }
    for (; k < K; k += R) {
#pragma unroll
        for (uint32_t u = 0; u < R; u++) {
            const uint4 v = ring[u];
            if (k + u + R < K) ring[u] = ldg16<NT>(wb + ((k + u + R) * 1024u + lo_lane));
            if (k + u < K) fold(k + u, v);
        }
    }
    uint64_t x;
    if constexpr (OM == kOpsMix) {  // the offsets batches (see combine64_lane0)
        x = combine64_lane0<6, OM>(lds, pk, x0, x1, gl);
        if (gl == 0) x = tail64<OM>(lds, pk, (uint32_t)(a1 - ea), x);
        x = uniform64(x);
    } else {  // the segment and XDR kernels: the halving form there cost the
              // segment chunk pass 6.8% (register allocation of its other paths,
              // profiles/r06/ab_seg_lane0.log)
        x = combine64<6, OM>(lds, pk, x0, x1, gl);
        x = tail64<OM>(lds, pk, (uint32_t)(a1 - ea), x);
    }
    if (!RAW && len < 8) x ^= pk->zinit[len];
    return x;
}

// SPLIT (aligned batches of large payloads, G = 64): a unit is one
// kSplitBytes piece q of payload p, so the work queue balances pieces instead
// of whole 1 MiB payloads (one per wave at C3's shape: the slowest XCD set the
// launch time).  By linearity the payload's register is the XOR over pieces of
// Z^(bytes after piece q)(L_q), L_0 carrying the initial value; each piece
// adds its term (and piece 0 the final XOR) to out[p] with a 64-bit atomic
// XOR, into an output the host zeroed before the launch.
template <int LOG2G, int MODE, bool VERIFY, bool NT, bool SPLIT = false>
__global__ __launch_bounds__(kBlk64<MODE * 16 + LOG2G>, kWpe64<MODE * 16 + LOG2G>) void crc64_batch_kernel(BatchArgs a) {
    using S = Shape<64, MODE, false, LOG2G>;
    constexpr int kWPB = S::block / 64;
    __shared__ __attribute__((aligned(16))) uint8_t lds[S::lds64_bytes];
    const crc64_gpu_pack_t *pk = reinterpret_cast<const crc64_gpu_pack_t *>(a.pack);
    constexpr int PPW = 64 >> LOG2G;
    // split launches: the plan with the finer tail pieces (SplitPlan)
    const SplitPlan splan(SPLIT ? a.count : 0, SPLIT ? a.split_log2 : 1u, gridDim.x);
    const uint64_t units = MODE == kOffsets ? a.count : SPLIT ? splan.n : (a.count + PPW - 1) / PPW;
    __shared__ WgQueue wgq;
    constexpr bool DYN = dyn_policy(64, MODE, NT, false) || SPLIT;
    MCK_STAMP(blockIdx.x * kWPB + (threadIdx.x >> 6), 0);
    if (DYN && threadIdx.x == 0) {
        if constexpr (SPLIT) wg_queue_init_plan(&wgq, a.queue, splan);
        else wg_queue_init(&wgq, a.queue, units);
    }
    // split pieces combined in the workgroup (SPLIT, split_lds): per set
    // (chunk sequence number % kAccSets) and payload (% kSplitAcc) the XOR of
    // the pieces' terms, their count and the owning chunk (sequence + 1; 0 free)
    __shared__ unsigned long long sacc[SPLIT ? kAccSets * kSplitAcc : 1];
    __shared__ unsigned int scnt[SPLIT ? kAccSets * kSplitAcc : 1];
    __shared__ unsigned int stag[SPLIT ? kAccSets * kSplitAcc : 1];
    if (SPLIT && threadIdx.x < kAccSets * kSplitAcc) {
        sacc[threadIdx.x] = 0;
        scnt[threadIdx.x] = 0;
        stag[threadIdx.x] = 0;
    }
    fill_lds64<S::block, S::ops_mode>(lds, pk);
    __syncthreads();
    MCK_STAMP(blockIdx.x * kWPB + (threadIdx.x >> 6), 1);

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & ((1u << LOG2G) - 1u), grp = lane >> LOG2G;
    const uint32_t lc = (lane & 31u) << 3;
    const uint64_t xorout = pk->xorout;
    const uint32_t nw = gridDim.x * kWPB;
    uint32_t nbad = 0;  // verify: this lane's mismatches (add_mismatches)
    // A static split with fewer units than waves numbers the waves across
    // workgroups first, so a small batch spreads over CUs (the host then
    // launches one workgroup per unit) instead of filling one CU's LDS
    // pipe: 64 x 4 KiB took 18.4 us packed into one workgroup.
    const bool spread = !DYN && units < nw;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(spread ? (threadIdx.x >> 6) * gridDim.x + blockIdx.x
                                                                : blockIdx.x * kWPB + (threadIdx.x >> 6));

    if (MODE == kOffsets) {
        auto one = [&](uint64_t p) {
            const uint64_t o = a.offsets[p];
            const uint64_t n = a.offsets[p + 1] - o;
            const uint64_t x = n < (1ull << 31) ? payload64_g64<NT, false, S::ops_mode>(lds, pk, a.base + o, n, gl, lc)
                                                : payload64_generic<LOG2G, NT, S::ops_mode>(lds, pk, a.base + o, n, gl, lc);
            if (gl == 0) emit<uint64_t, VERIFY>(a, p, x ^ xorout, nbad);
        };
        if (for_each_unit<true>(&wgq, a.queue, units, wave, nw, one)) fail_closed<VERIFY>(a);
        if constexpr (VERIFY) add_mismatches(a.mismatches, nbad);
        return;
    }
    if constexpr (SPLIT) {
        static_assert(LOG2G == 6 && MODE == kFixedAligned && !VERIFY, "split pieces: aligned G = 64 checksums");
        const crc64_shift_pack_t *sp = reinterpret_cast<const crc64_shift_pack_t *>(a.shift);
        unsigned long long *out = reinterpret_cast<unsigned long long *>(a.out);
        // In-workgroup combine (split_lds, a slot launch whose queue chunks hold
        // whole payloads): per ring entry and payload, the XOR of the pieces'
        // terms and their count; the last piece stores the CRC -- no zeroing
        // launch and no global atomics.  Otherwise (graph captures: static
        // split) each piece XORs its term into the out[] the host zeroed.
        // (The host's check is repeated here: a mismatch is a fault, never a
        // silently wrong value.)
        const bool in_wg = a.split_lds && a.queue && splan.whole();
        if (a.split_lds && !in_wg) {  // host and device disagree: fail closed, reported once per launch
            if (blockIdx.x == 0 && threadIdx.x < 64) {
                if (threadIdx.x == 0) queue_fault(13, units, a.split_log2);
                fail_closed<false>(a);
            }
            return;
        }
        // Pipelined (round 6): a wave takes its NEXT piece as soon as the
        // current one's step loop ends and issues that piece's first loads,
        // so their HBM round trip overlaps the current piece's lane combine,
        // Z^n shift and accumulation (before, each 256 KiB piece waited one
        // HBM latency at its start, after its predecessor's combine).  A
        // taken piece's ring read counts at once (no deferred reader), so the
        // accumulators are keyed by the chunk's sequence number instead of
        // its ring entry: set seq % kAccSets, owner tag seq + 1.  A piece
        // whose entry an older chunk still holds waits for it (bounded; the
        // older chunk's pieces are all taken and never wait on this one); a
        // newer owner means one wave held every taken piece of its chunk while
        // the workgroup's other waves finished kAccSets - 1 whole chunks (most
        // of a launch at a 256 KiB piece per wave and chunk) -- a fault, never
        // a value.
        const uint32_t pieces = 1u << splan.psl;
        const uint64_t bytes = a.len >> splan.psl;  // kSplitBytes
        const uint32_t K = (uint32_t)(bytes >> 10);
        auto src_of = [&](uint64_t u, uint64_t *p, uint32_t *q) {
            splan.unit(u, p, q);
            return a.base + *p * a.stride + (uint64_t)*q * bytes;
        };
        UnitTaker<SplitPlan> tk(&wgq, a.queue, units, wave, nw, false, splan);
        Lane64 ln = lane64(lc);
        uint4 ring[kRing64];
        uint64_t u, p = 0;
        uint32_t q = 0;
        bool have = tk.take_unit(&u);
        uint32_t seq = tk.seq;
        const uint8_t *src = have ? src_of(u, &p, &q) : a.base;
        if (have) ring64_load<NT>(ring, src, gl);
        while (have) {
            uint64_t x0, x1;
            fold64_ring<NT>(lds, ring, src, K, gl, ln, q == 0 ? pk->init : 0ull, &x0, &x1);
            uint64_t un = 0, pn = 0;
            uint32_t qn = 0;
            const bool next = tk.take_unit(&un);
            const uint32_t seqn = tk.seq;
            const uint8_t *srcn = next ? src_of(un, &pn, &qn) : src;
            if (next) ring64_load<NT>(ring, srcn, gl);  // in flight during the combine below
            const uint64_t x = combine64<6, kOpsLds>(lds, pk, x0, x1, gl);
            if (gl == 0) {
                const uint64_t t = shift64(sp, x, (uint64_t)(pieces - 1 - q) * bytes) ^ (q == 0 ? xorout : 0ull);
                if (in_wg) {
                    const uint32_t ai = (seq % kAccSets) * kSplitAcc + (uint32_t)(p & (kSplitAcc - 1));
                    const uint32_t me = seq + 1;
                    Deadline dl(abort_word(a.queue));
                    bool own = false;
                    for (;;) {
                        const uint32_t tg = lds_ld(&stag[ai]);
                        if (tg == me) {
                            own = true;
                            break;
                        }
                        if (tg == 0u) {
                            unsigned int expect = 0u;
                            if (__hip_atomic_compare_exchange_strong(&stag[ai], &expect, me, __ATOMIC_ACQ_REL,
                                                                     __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                                own = true;
                                break;
                            }
                            continue;
                        }
                        if (tg > me) {  // a newer chunk on this entry: fail closed
                            queue_fault(16, seq, tg);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        if (dl.passed()) {  // the older chunk never finished
                            queue_fault(17, seq, tg);
                            raise_abort(a.queue);
                            break;
                        }
                    }
                    if (own) {
                        // (one wave's LDS atomics are performed in order: a
                        // piece's XOR lands before its count, the last piece's
                        // reset before the entry's release)
                        __hip_atomic_fetch_xor(&sacc[ai], (unsigned long long)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        const uint32_t seen = __hip_atomic_fetch_add(&scnt[ai], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (seen == pieces - 1) {
                            out[p] = __hip_atomic_exchange(&sacc[ai], 0ull, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                            __hip_atomic_store(&scnt[ai], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            __hip_atomic_store(&stag[ai], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                    } else {
                        tk.flt = 1;
                    }
                } else {
                    atomicXor(out + p, (unsigned long long)t);
                }
            }
            have = next;
            u = un;
            p = pn;
            q = qn;
            seq = seqn;
            src = srcn;
        }
        const bool faulted = tk.finish(wave);
        if (faulted) fail_closed<false>(a);
        MCK_STAMP(blockIdx.x * kWPB + (threadIdx.x >> 6), 2);
        return;
    }
    const bool faulted = for_each_unit<DYN>(&wgq, a.queue, units, wave, nw, [&](uint64_t u) {
        const uint64_t p = u * PPW + grp;
        const bool act = p < a.count;
        const uint64_t pc = act ? p : a.count - 1;
        uint64_t x;
        if constexpr (MODE == kFixedAligned)
            x = payload64_aligned<LOG2G, NT, S::ops_mode>(lds, pk, a.base + pc * a.stride, (uint32_t)(a.len >> (4 + LOG2G)), gl, lc, pk->init);
        else
            x = payload64_generic<LOG2G, NT>(lds, pk, a.base + pc * a.stride, a.len, gl, lc);
        if (act && gl == 0) emit<uint64_t, VERIFY>(a, p, x ^ xorout, nbad);
    });
    if (faulted) fail_closed<VERIFY>(a);
    if constexpr (VERIFY) add_mismatches(a.mismatches, nbad);
    MCK_STAMP(blockIdx.x * kWPB + (threadIdx.x >> 6), 2);
}

}  // namespace

#endif  // CRC_GPU_DEVICE_H
