// mchecksum_gpu.hip -- MI355X (gfx950) batch CRC kernels behind the C ABI in
// include/mchecksum_gpu.h.
//
// What is computed.  For each payload i, the value mchecksum_get() returns
// after mchecksum_update(payload_i) -- the CRC Mercury stores in the HG header
// for a serialized proc buffer (src/mercury_proc.c:358-406,
// src/mercury.c:699-707, src/mercury_header.c:111-112).
//
// How (algebra in crc_gpu_layout.h; validated by tests/native/kernel_emulator):
//  * A payload is covered by a 16-byte-aligned window whose END is aligned to
//    the step grid; G lanes (one group) cover one step of 16*G bytes, each lane
//    one coalesced dwordx4 (so a G = 64 wave reads 1 KiB per instruction).
//  * Every W-bit word slot of a lane is an independent sub-stream with a
//    uniform stride of 16*G bytes, so "advance by the stride" is folded into
//    the lookup tables: s <- F(s ^ w) costs 4 byte lookups (CRC-32C) or 16
//    nibble lookups (CRC-64) and no shift/multiply.
//  * Lookup tables live in LDS, laid out so that every ds_read_b32/b64 is
//    conflict-free: CRC-32C byte tables and CRC-64 low-nibble tables are
//    replicated 32x (lane l reads copy l % 32), CRC-64 high-nibble tables sit
//    at a 16-B entry stride.  One VALU op forms each lookup address (v_perm_b32
//    or v_and_b32_sdwa: the byte or nibble as entry, the lane copy in the low
//    byte).
//  * Sub-streams are combined by a tree (in-lane, then xor-shuffles across the
//    group) whose level operators Z^-(2^k * W/8) are nibble tables in LDS;
//    Z^-t removes the t pad bytes after the payload end.
//  * Persistent grid: one 1024-thread workgroup per CU for CRC-32C (the
//    replicated tables take 128 KiB of the 160 KiB LDS), two for CRC-64.  Waves
//    take payloads from a device-side work queue (large aligned CRC-32C and
//    all offsets batches) or by a static stride (crc_gpu_device.h, dyn_policy).
//    Batches <= 16 MiB take a light layout: unreplicated tables, 256-thread
//    workgroups on every CU.
// No MFMA: this is HBM-bound byte scanning; the roofline is HBM read bandwidth.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>

#include "crc_gpu_device.h"
#include "gpu_host.h"
#include "mchecksum_gpu.h"
#include "mchecksum_models.h"

namespace mck {
// ------------------------------------------------------------ host side ----

thread_local char t_err[256] = "";
// mchecksum_gpu_set_error_word(): device word bumped by a launch that could
// not hash every payload (per host thread; nullptr = none)
thread_local uint32_t *t_err_word = nullptr;

int set_err(int rc, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t_err, sizeof(t_err), fmt, ap);
    va_end(ap);
    return rc;
}

int hip_err(hipError_t e, const char *what) {
    snprintf(t_err, sizeof(t_err), "%s: %s", what, hipGetErrorString(e));
    return MCHECKSUM_GPU_EHIP;
}

std::mutex g_mu;
DevCtx g_dev[kMaxDev];

// Method -> (model index, width) for GPU-capable (32/64-bit) models.
int gpu_model(const char *method, int *width) {
    const int idx = mck_model_index(method);
    if (idx < 0) return -1;
    const mck_model_t &m = mck_models[idx];
    if (m.width != 32 && m.width != 64) return -2;
    *width = m.width;
    return idx;
}

bool gpu_msb(int idx) { return !mck_models[idx].reflected; }

// A reflected model as is; an MSB-first model as the reflected model of the
// same polynomial over bit-reversed bytes, conjugated by R (crc_gpu_layout.h):
// rinit / xorout reflected, then R-mapped.
crc_rmodel_t gpu_rmodel(int idx) {
    const mck_model_t &m = mck_models[idx];
    crc_rmodel_t rm{};
    rm.width = m.width;
    rm.rpoly = mck_reflect(m.poly, m.width);
    rm.msb = !m.reflected;
    rm.rinit = rm.msb ? crc_rev_bytes(m.width, mck_reflect(m.init, m.width)) : mck_reflect(m.init, m.width);
    rm.xorout = rm.msb ? crc_rev_bytes(m.width, mck_reflect(m.xorout, m.width)) : m.xorout;
    return rm;
}

__global__ __launch_bounds__(256) void bswap_kernel(void *out, uint64_t n, int width) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        if (width == 64) {
            unsigned long long *p = reinterpret_cast<unsigned long long *>(out) + i;
            *p = __builtin_bswap64(*p);
        } else {
            uint32_t *p = reinterpret_cast<uint32_t *>(out) + i;
            *p = __builtin_bswap32(*p);
        }
    }
}

int swap_outputs(void *dev_out, uint64_t count, int width, void *stream) {
    if (!count) return MCHECKSUM_GPU_OK;
    uint64_t blocks = (count + 255) / 256;
    blocks = blocks > 1024 ? 1024 : blocks;
    const hipError_t e =
        launch_kernel(bswap_kernel, dim3((unsigned)blocks), dim3(256), (hipStream_t)stream, nullptr, dev_out, count, width);
    if (e != hipSuccess) return hip_err(e, "output byte swap");
    return MCHECKSUM_GPU_OK;
}

int device_ctx(DevCtx **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_err(e, "hipGetDevice");
    if (dev < 0 || dev >= kMaxDev) return set_err(MCHECKSUM_GPU_ENODEV, "device id %d out of range", dev);
    DevCtx &c = g_dev[dev];
    if (c.init.load(std::memory_order_acquire)) {
        *out = &c;
        return 0;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (!c.init.load(std::memory_order_relaxed)) {
        int cus = 0;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return hip_err(e, "hipDeviceGetAttribute");
        c.cus = cus > 0 ? cus : 1;
        // tests only: a smaller slot pool (MCHECKSUM_GPU_QUEUE_SLOTS=n), so a
        // test can hold every slot in flight
        const uint32_t qs = mck_settings()->gpu_queue_slots;
        if (qs >= 1 && qs < kQueueSlots) c.nslots = qs;
        // slots aligned to two banks, so a bank's partner is its address ^ kQBankBytes
        const size_t slot_bytes = (size_t)kQSlotWords * sizeof(unsigned long long);
        const size_t qbytes = (size_t)kQueueSlots * slot_bytes + slot_bytes;
        e = hipMalloc(&c.queue_mem, qbytes);
        if (e == hipSuccess) e = hipMemset(c.queue_mem, 0, qbytes);
        if (e == hipSuccess)
            c.queue = reinterpret_cast<unsigned long long *>((reinterpret_cast<uintptr_t>(c.queue_mem) + slot_bytes - 1) /
                                                             slot_bytes * slot_bytes);
        if (e != hipSuccess) {
            if (c.queue_mem) (void)hipFree(c.queue_mem);
            c.queue_mem = nullptr;
            c.queue = nullptr;
            return hip_err(e, "work-queue allocation");
        }
        c.init.store(true, std::memory_order_release);
    }
    *out = &c;
    return 0;
}

// Returns the device table pack for (model, log2g), building it on first use.
int get_pack(DevCtx *c, int idx, int log2g, const void **pack) {
    if (void *p = c->pack[idx][log2g].load(std::memory_order_acquire)) {
        *pack = p;
        return 0;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (void *p = c->pack[idx][log2g].load(std::memory_order_relaxed)) {
        *pack = p;
        return 0;
    }
    const mck_model_t &m = mck_models[idx];
    const crc_rmodel_t rm = gpu_rmodel(idx);
    void *host = nullptr;
    size_t bytes = 0;
    int rc;
    if (m.width == 32) {
        bytes = sizeof(crc32_gpu_pack_t);
        host = calloc(1, bytes);
        rc = host ? crc32_gpu_pack_build(&rm, log2g, (crc32_gpu_pack_t *)host) : -1;
    } else {
        bytes = sizeof(crc64_gpu_pack_t);
        host = calloc(1, bytes);
        rc = host ? crc64_gpu_pack_build(&rm, log2g, (crc64_gpu_pack_t *)host) : -1;
    }
    if (rc != 0) {
        free(host);
        return set_err(MCHECKSUM_GPU_EINVAL, "table build failed for %s (G = %d)", m.name, 1 << log2g);
    }
    void *d = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e == hipSuccess) e = hipMemcpy(d, host, bytes, hipMemcpyHostToDevice);
    free(host);
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        return hip_err(e, "table upload");
    }
    c->pack[idx][log2g].store(d, std::memory_order_release);
    *pack = d;
    return 0;
}

// Whether slot i is idle: handed to no launch that has not yet been enqueued,
// and its latest launch is done with it -- its `done` event, recorded by that
// launch's completion (launch_kernel's stop event), queried without blocking:
// not a device round trip, so it may run under the pool lock.  A
// never-recorded event reads as complete.  (Late round 5 had the launch's
// last workgroup store a completion word to host-mapped memory instead:
// correct, +-0 without a profiler, not kept.)
bool slot_idle(const DevCtx *c, uint32_t i) {
    const SlotState &s = c->slot[i];
    if (s.pending.load(std::memory_order_acquire)) return false;
    const hipError_t e = hipEventQuery(s.done);
    if (e == hipSuccess) return true;
    if (e != hipErrorNotReady) (void)hipGetLastError();
    return false;
}

// In-flight slots looked at per queue_slot call: a couple while the pool has
// idle slots (so the most recently used lines, warm in L2, are reused first),
// more when it is empty.
constexpr uint32_t kReapSome = 2, kReapMax = 8;

SlotRef queue_slot(DevCtx *c, void *stream) {
    SlotRef r;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &st) != hipSuccess) {
        (void)hipGetLastError();
        st = hipStreamCaptureStatusNone;
    }
    std::lock_guard<std::mutex> lk(c->pool_mu);
    // A captured launch replays with these arguments, possibly on two graph
    // execs at once: no slot can be exclusive to it, so it takes the static
    // split (crc_gpu_device.h, "Exclusivity").
    if (st != hipStreamCaptureStatusNone) {
        c->n_noslot++;
        return r;
    }
    if (c->idle.empty() && c->in_flight.empty())  // first use on this device: every slot idle, slot 0 on top
        for (uint32_t k = c->nslots; k-- > 0;) c->idle.push_back(k);
    // Reap: look at the oldest in-flight slots; those whose launches have
    // completed return to the pool, busy ones go to the back of the FIFO
    // (left at the head, a few long-blocked launches -- a stream
    // waiting on an event -- were looked at by every call while completed
    // slots behind them were never reaped, and every launch fell back to the
    // static split once the idle stack ran out).
    const uint32_t limit = c->idle.empty() ? kReapMax : kReapSome;
    const size_t nlook = c->in_flight.size() < limit ? c->in_flight.size() : limit;
    uint32_t busy = 0;
    for (size_t k = 0; k < nlook; k++) {
        const uint32_t i = c->in_flight.front();
        c->in_flight.pop_front();
        if (slot_idle(c, i)) {
            c->idle.push_back(i);
            c->n_reaped++;
        } else {
            c->in_flight.push_back(i);
            busy++;
        }
    }
    if (c->idle.empty()) {  // the oldest launches are all still running: static split
        c->n_busy_skip += busy;
        c->n_noslot++;
        return r;
    }
    const uint32_t i = c->idle.back();
    SlotState &s = c->slot[i];
    if (!s.done && hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        s.done = nullptr;
        c->n_noslot++;
        return r;
    }
    c->idle.pop_back();
    c->in_flight.push_back(i);
    c->n_busy_skip += busy;
    c->n_slot++;
    s.pending.store(true, std::memory_order_relaxed);
    r.q = c->queue + (size_t)i * kQSlotWords + (s.seq & 1u) * kQBankWords;
    s.seq++;
    r.idx = (int)i;
    r.done = s.done;
    r.st = &s;
    return r;
}

// The launch holding r is enqueued and its completion event recorded: the
// slot now reads busy until that launch completes.
void slot_issued(SlotRef &r) {
    if (r.st) r.st->pending.store(false, std::memory_order_release);
}

// The launch call failed, so the kernel was not enqueued (launch_kernel
// reports the call's own status): the bank it was given is still clean, and
// the slot goes straight back to the pool.
void slot_unissue(DevCtx *c, SlotRef &r) {
    if (r.idx < 0) return;
    std::lock_guard<std::mutex> lk(c->pool_mu);
    SlotState &s = c->slot[r.idx];
    s.seq--;
    for (auto it = c->in_flight.end(); it != c->in_flight.begin();) {
        if (*--it == (uint32_t)r.idx) {
            c->in_flight.erase(it);
            break;
        }
    }
    c->idle.push_back((uint32_t)r.idx);
    c->n_slot--;
    c->n_noslot++;
    s.pending.store(false, std::memory_order_release);
    r.idx = -1;
    r.st = nullptr;
}

uint32_t *error_word() { return t_err_word; }

typedef void (*kern_t)(BatchArgs);

__global__ __launch_bounds__(256) void zero_u64_kernel(unsigned long long *p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) p[i] = 0;
}

struct KLaunch {
    kern_t k;
    int block, blocks_per_cu;
};

// MCHECKSUM_GPU_LOG2G=g: 2^g lanes per payload for every fixed batch (A/B)
bool lg_forced() { return mck_settings()->gpu_log2g >= 0; }

int choose_log2g(size_t len, int width) {
    if (lg_forced()) return mck_settings()->gpu_log2g;
    // CRC-32, 1 KiB to under 8 KiB: 16 steps per payload -- 4 lanes at 1 KiB,
    // 8 at 2 KiB, 16 at 4 KiB.  Round 6 timed these shapes on cold lines
    // (4 copies of each batch read in turn, so no launch re-reads what the
    // last one left in the 256 MiB Infinity Cache; tools/ab_variants.py
    // --rotate 4, profiles/r06/ab_lgcold.log): C2's 4 KiB at 16 lanes 50.5 us
    // against 61.6 at 4 (+22%), 2 KiB at 8 lanes +3%; round 4 had chosen 4
    // lanes throughout from back-to-back replays of one batch, which the
    // cache served (-1.9% for 16 lanes there).  From 8 KiB about 32 steps
    // per payload (8 KiB: 16 lanes, 16 KiB: 32 -- both still the best cold),
    // 64 lanes from 32 KiB (the headline).
    if (width == 32 && len >= 1024) {
        if (len < 8192) {
            int lg = 2;
            while (lg < 4 && ((size_t)512 << lg) <= len) lg++;
            return lg;
        }
        int lg = 0;
        while (lg < CRC_GPU_MAX_LOG2G && ((size_t)512 << (lg + 1)) <= len) lg++;
        return lg;
    }
    // CRC-64 (profiles/r04/ab_crc64_log2g.log): about 128 steps per payload,
    // 4 lanes at least -- 4 KiB: 4 lanes -6.9%, 16 KiB: 8 lanes -6.7%, 64 KiB:
    // 32 lanes -3.5% against the >= 16-step rule's 16 / 64 / 64.
    if (width == 64 && len >= 1024) {
        int lg = 2;
        while (lg < CRC_GPU_MAX_LOG2G && ((size_t)2048 << (lg + 1)) <= len) lg++;
        return lg;
    }
    // Otherwise aim for >= 16 steps per payload, at most 64 lanes per payload.
    const size_t target = len / 256;
    int lg = 0;
    while (lg < CRC_GPU_MAX_LOG2G && ((size_t)1 << (lg + 1)) <= target) lg++;
    return lg;
}

template <int W, int LOG2G, int MODE, bool VERIFY, bool NT = false, bool LIGHT = false>
KLaunch kernel_ptr() {
    using S = Shape<W, MODE, LIGHT, LOG2G>;
    if constexpr (W == 32) return {crc32c_batch_kernel<LOG2G, MODE, VERIFY, NT, LIGHT>, S::block, S::blocks_per_cu};
    else return {crc64_batch_kernel<LOG2G, MODE, VERIFY, NT>, S::block, S::blocks_per_cu};
}

template <int W, int LOG2G>
KLaunch pick_fixed_lg(bool aligned, bool nt, bool light) {
    if constexpr (W == 32) {
        if (light)
            return aligned ? kernel_ptr<W, LOG2G, kFixedAligned, false, false, true>()
                           : kernel_ptr<W, LOG2G, kFixedGeneric, false, false, true>();
    }
    if (!aligned) return kernel_ptr<W, LOG2G, kFixedGeneric, false>();
    return nt ? kernel_ptr<W, LOG2G, kFixedAligned, false, true>() : kernel_ptr<W, LOG2G, kFixedAligned, false>();
}

template <int W>
KLaunch pick_fixed(int log2g, bool aligned, bool nt, bool light) {
    switch (log2g) {
        case 0: return pick_fixed_lg<W, 0>(aligned, nt, light);
        case 1: return pick_fixed_lg<W, 1>(aligned, nt, light);
        case 2: return pick_fixed_lg<W, 2>(aligned, nt, light);
        case 3: return pick_fixed_lg<W, 3>(aligned, nt, light);
        case 4: return pick_fixed_lg<W, 4>(aligned, nt, light);
        case 5: return pick_fixed_lg<W, 5>(aligned, nt, light);
        default: return pick_fixed_lg<W, 6>(aligned, nt, light);
    }
}

// Non-temporal payload loads when the batch is far larger than the 256 MiB
// Infinity Cache (MCHECKSUM_GPU_NT=0/1 overrides).
// Small batches (<= 16 MiB) take the light CRC-32C layout (16 KiB LDS fill, 256-thread
// workgroups over every CU, 64 lanes per payload): the full layout's 140 KiB
// fill and 1024-thread workgroups cost ~6-12 us per call there
// (profiles/r01/latency.json).  MCHECKSUM_GPU_LIGHT=0/1 overrides.
constexpr uint64_t kLightMaxBytes = 16ull << 20;  // crossover ~24 MiB (latency.json)
bool use_light(uint64_t batch_bytes, bool known) {
    if (mck_settings()->gpu_light >= 0) return mck_settings()->gpu_light == 1;
    return known && batch_bytes <= kLightMaxBytes;
}

// Lanes per payload for the light layout: as many as keep K >= kRing whole steps.
int light_log2g(size_t len) {
    if (lg_forced()) return mck_settings()->gpu_log2g;
    int lg = CRC_GPU_MAX_LOG2G;
    while (lg > 0 && ((size_t)16 << lg) * kRing > len) lg--;
    return lg;
}

bool use_nt(uint64_t batch_bytes) {
    if (mck_settings()->gpu_nt >= 0) return mck_settings()->gpu_nt == 1;
    return batch_bytes >= (512ull << 20);
}

// Launch a batch kernel; a slot launch records the slot's completion event.
// A failed launch call is taken back from its slot (slot_unissue).
int launch(DevCtx *c, const KLaunch &kl, const BatchArgs &a, unsigned blocks, void *stream, SlotRef &sr) {
    const hipError_t e = launch_kernel(kl.k, dim3(blocks), dim3(kl.block), (hipStream_t)stream, sr.done, a);
    if (e != hipSuccess) {
        slot_unissue(c, sr);
        return hip_err(e, "kernel launch");
    }
    slot_issued(sr);
    return MCHECKSUM_GPU_OK;
}

unsigned grid_for(const DevCtx *c, uint64_t waves_needed, const KLaunch &kl) {
    const uint64_t wpb = (uint64_t)kl.block / 64;
    uint64_t blocks = (waves_needed + wpb - 1) / wpb;
    if (blocks > (uint64_t)c->cus * kl.blocks_per_cu) blocks = (uint64_t)c->cus * kl.blocks_per_cu;
    return blocks ? (unsigned)blocks : 1u;
}

// The table pack for another lanes-per-payload choice (cached per device).
int repack(DevCtx *c, const char *method, int log2g, const void **pack) {
    int width = 0;
    const int idx = gpu_model(method, &width);
    return get_pack(c, idx, log2g, pack);
}

int prologue(const char *method, int log2g, int *width, DevCtx **c, const void **pack) {
    int idx = gpu_model(method, width);
    if (idx == -1) return set_err(MCHECKSUM_GPU_EMETHOD, "unknown hash method \"%s\"", method ? method : "(null)");
    if (idx < 0) return set_err(MCHECKSUM_GPU_EMETHOD, "method \"%s\" has no GPU kernel (32/64-bit only)", method);
    int rc = device_ctx(c);
    if (rc) return rc;
    return get_pack(*c, idx, log2g, pack);
}

// The work queue counts chunk ids and per-workgroup slots in 32 bits
// (crc_gpu_device.h, WgQueue): 2^31 payloads per call keeps both in range.
constexpr uint64_t kMaxUnits = 1ull << 31;

int do_offsets(const char *method, const void *base, const uint64_t *offsets, size_t count, void *out,
               const void *expected, uint8_t *status, uint32_t *mism, void *stream, bool verify,
               bool msg = false, size_t pay_off = 0, size_t hash_off = 0) {
    // an empty batch needs no buffers (not even the one-entry offsets table)
    if (count && (!base || !offsets || (!verify && !out) || (verify && !msg && !expected)))
        return set_err(MCHECKSUM_GPU_EINVAL, "NULL pointer argument");
    if (msg && (hash_off + 4 > pay_off || pay_off > (1u << 30)))
        return set_err(MCHECKSUM_GPU_EINVAL, "hash_offset + 4 must not exceed payload_offset");
    if ((uint64_t)count > kMaxUnits) return set_err(MCHECKSUM_GPU_EINVAL, "more than 2^31 payloads in one call");
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    int width = 0;
    DevCtx *c = nullptr;
    const void *pack = nullptr;
    int rc = prologue(method, CRC_GPU_MAX_LOG2G, &width, &c, &pack);
    if (rc) return rc;
    if (count == 0) return MCHECKSUM_GPU_OK;
    BatchArgs a{};
    a.base = (const uint8_t *)base;
    a.offsets = offsets;
    a.count = count;
    a.out = out;
    a.expected = expected;
    a.status = status;
    a.mismatches = mism;
    a.pack = pack;
    a.msg = msg ? 1u : 0u;
    a.pay_off = (uint32_t)pay_off;
    a.hash_off = (uint32_t)hash_off;
    a.queue = nullptr;
    a.err_word = t_err_word;
    if (msg && width != 32)
        return set_err(MCHECKSUM_GPU_EMETHOD, "message verify carries a 32-bit header hash: crc32c only");
    const int midx = gpu_model(method, &width);
    a.bswap = verify && gpu_msb(midx) ? 1u : 0u;  // checksum calls swap after the launch
    KLaunch k;
    // The offsets table stays on the device, so size the batch by its count:
    // 8192+ payloads of the C4 mix are ~270 MB and up.
    const bool nt = use_nt(count >= 8192 ? (1ull << 40) : 0);
    // small offsets batches (<= 1024 payloads: a receive queue's worth of RPCs)
    // take the light layout
    const bool light = width == 32 && use_light(count <= 1024 ? 0 : ~0ull, true);
    if (width == 32 && light)
        k = verify ? kernel_ptr<32, 6, kOffsets, true, false, true>() : kernel_ptr<32, 6, kOffsets, false, false, true>();
    else if (width == 32)
        k = verify ? (nt ? kernel_ptr<32, 6, kOffsets, true, true>() : kernel_ptr<32, 6, kOffsets, true>())
                   : (nt ? kernel_ptr<32, 6, kOffsets, false, true>() : kernel_ptr<32, 6, kOffsets, false>());
    else
        k = verify ? (nt ? kernel_ptr<64, 6, kOffsets, true, true>() : kernel_ptr<64, 6, kOffsets, true>())
                   : (nt ? kernel_ptr<64, 6, kOffsets, false, true>() : kernel_ptr<64, 6, kOffsets, false>());
    SlotRef sr;
    const unsigned grid = grid_for(c, count, k);
    if (dyn_policy(width, kOffsets, nt, light)) sr = queue_slot(c, stream);
    a.queue = sr.q;
    rc = launch(c, k, a, grid, stream, sr);
    if (rc == MCHECKSUM_GPU_OK && gpu_msb(midx) && !verify) rc = swap_outputs(out, count, width, stream);
    return rc;
}

// Large aligned CRC-64 payloads go to the work queue as kSplitBytes pieces
// (crc64_batch_kernel<..., SPLIT>) once the batch is big enough for the
// non-temporal path; MCHECKSUM_GPU_SPLIT=0/1 overrides.
bool use_split(int width, int lg, bool aligned, bool nt, size_t len, size_t stride) {
    const int forced = mck_settings()->gpu_split;
    if (forced == 0) return false;
    const bool shape = width == 64 && lg == CRC_GPU_MAX_LOG2G && aligned && len % kSplitBytes == 0 &&
                       len / kSplitBytes >= 2 && len / kSplitBytes <= 64 && ((len / kSplitBytes) & (len / kSplitBytes - 1)) == 0 &&
                       stride % 16 == 0;
    if (forced == 1) return shape;
    return shape && nt;
}

// MCHECKSUM_GPU_SPLIT_LDS=0: split CRC-64 pieces always combine through the
// zeroed output (tests, A/B).
bool use_split_lds() { return mck_settings()->gpu_split_lds != 0; }

int launch_fixed(DevCtx *c, int idx, const void *pack, int width, int lg, const void *dev_base, size_t stride,
                 size_t len, size_t count, void *dev_out, void *stream, bool light) {
    const uint64_t step = 16ull << lg;
    // The aligned path needs whole steps and K = len/step a multiple of the
    // load ring depth; everything else takes the generic path.
    const bool aligned = ((uintptr_t)dev_base % 16 == 0) && (stride % 16 == 0 || count == 1) &&
                         len >= step * kRing && (len % (step * kRing) == 0) && (len >> (4 + lg)) < (1ull << 31) && !mck_settings()->gpu_force_generic;
    BatchArgs a{};
    a.base = (const uint8_t *)dev_base;
    a.stride = stride;
    a.len = len;
    a.count = count;
    a.out = dev_out;
    a.pack = pack;
    a.err_word = t_err_word;
    const bool nt = !light && use_nt((uint64_t)len * count);
    uint32_t sl = 0;
    while ((kSplitBytes << sl) < len && sl < 63) sl++;
    if (use_split(width, lg, aligned, nt, len, count > 1 ? stride : 16) && ((uint64_t)count << sl) <= kMaxUnits) {
        const void *shift = nullptr;
        if (int rc = get_ext(c, idx, &shift)) return rc;
        a.shift = shift;
        a.split_log2 = sl;
        using S6 = Shape<64, kFixedAligned, false, 6>;
        const KLaunch k = nt ? KLaunch{crc64_batch_kernel<6, kFixedAligned, false, true, true>, S6::block, S6::blocks_per_cu}
                             : KLaunch{crc64_batch_kernel<6, kFixedAligned, false, false, true>, S6::block, S6::blocks_per_cu};
        const unsigned grid = grid_for(c, (uint64_t)count << sl, k);
        SlotRef sr = queue_slot(c, stream);
        a.queue = sr.q;
        // With a slot and queue chunks of whole payloads the pieces combine in
        // their workgroup (crc_gpu_device.h, split_lds).  Otherwise they XOR
        // their terms into out[]: zero it first, in stream order, with a kernel
        // -- a hipMemsetAsync captured into a graph did not order against the
        // kernel node on replays after the first (the pieces landed in a
        // half-zeroed output: tests/test_gpu_queue.py, concurrent replays).
        a.split_lds = sr.q && use_split_lds() && SplitPlan(count, sl, grid).whole() ? 1u : 0u;
        if (!a.split_lds) {
            uint64_t zb = (count + 255) / 256;
            zb = zb > 1024 ? 1024 : zb;
            const hipError_t e = launch_kernel(zero_u64_kernel, dim3((unsigned)zb), dim3(256), (hipStream_t)stream, nullptr,
                                               reinterpret_cast<unsigned long long *>(dev_out), (uint64_t)count);
            if (e != hipSuccess) {
                slot_unissue(c, sr);
                return hip_err(e, "output zeroing");
            }
        }
        int rc = launch(c, k, a, grid, stream, sr);
        if (rc == MCHECKSUM_GPU_OK && gpu_msb(idx)) rc = swap_outputs(dev_out, count, width, stream);
        return rc;
    }
    const KLaunch k = width == 32 ? pick_fixed<32>(lg, aligned, nt, light) : pick_fixed<64>(lg, aligned, nt, false);
    const uint64_t ppw = 64u >> lg;
    const bool dyn = dyn_policy(width, aligned ? kFixedAligned : kFixedGeneric, nt, light);
    const uint64_t units = (count + ppw - 1) / ppw;
    unsigned blocks = grid_for(c, units, k);
    // CRC-64 static split with fewer units than one full workgroup per CU:
    // one workgroup per unit, at most one per CU (each pays a 66 KiB LDS
    // fill); the kernel then numbers waves across workgroups first
    if (width == 64 && !dyn && units < (uint64_t)c->cus * (uint64_t)(k.block / 64))
        blocks = (unsigned)(units < (uint64_t)c->cus ? (units ? units : 1) : c->cus);
    SlotRef sr;
    if (dyn) {
        sr = queue_slot(c, stream);
        a.queue = sr.q;
    }
    int rc = launch(c, k, a, blocks, stream, sr);
    if (rc == MCHECKSUM_GPU_OK && gpu_msb(idx)) rc = swap_outputs(dev_out, count, width, stream);
    return rc;
}

}  // namespace mck

using namespace mck;

extern "C" {

int mchecksum_gpu_available(void) {
    // The device count cannot change for the life of the process: ask HIP
    // once (every batch call checks this first; ~1 us saved per call).
    static std::atomic<int> cached{-1};
    int v = cached.load(std::memory_order_relaxed);
    if (v >= 0) return v;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    v = n > 0 ? 1 : 0;
    cached.store(v, std::memory_order_relaxed);
    return v;
}

int mchecksum_gpu_prepare(const char *hash_method) {
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    const int idx = mck_model_index(hash_method);
    if (idx < 0) return set_err(MCHECKSUM_GPU_EMETHOD, "unknown hash method \"%s\"", hash_method ? hash_method : "(null)");
    DevCtx *c = nullptr;
    if (mck_models[idx].width != 16) {  // payload kernels: a table pack per lanes-per-payload width
        for (int lg = 0; lg <= CRC_GPU_MAX_LOG2G; lg++) {
            int width = 0;
            const void *pack = nullptr;
            int rc = prologue(hash_method, lg, &width, &c, &pack);
            if (rc) return rc;
        }
    }
    // ... and the extension tables every entry point may need (Z^n shift pack:
    // split CRC-64 pieces, segments, XDR; CRC-16 byte table: core headers),
    // so that no call captured into a graph uploads anything
    int rc = device_ctx(&c);
    if (rc) return rc;
    const void *ext = nullptr;
    return get_ext(c, idx, &ext);
}

int mchecksum_gpu_lanes_per_payload(const char *hash_method, size_t len) {
    int width = 0;
    if (gpu_model(hash_method, &width) < 0) return -1;
    return 1 << choose_log2g(len, width);
}

int mchecksum_gpu_checksum_fixed(const char *hash_method, const void *dev_base, size_t stride, size_t len,
                                 size_t count, void *dev_out, void *stream) {
    if (count && (!dev_base || !dev_out)) return set_err(MCHECKSUM_GPU_EINVAL, "NULL pointer argument");
    if (count > 1 && stride < len) return set_err(MCHECKSUM_GPU_EINVAL, "stride smaller than len");
    if ((uint64_t)count > kMaxUnits) return set_err(MCHECKSUM_GPU_EINVAL, "more than 2^31 payloads in one call");
    // the batch must fit the address space: stride * (count - 1) + len
    if (count > 1 && (uint64_t)stride > (UINT64_MAX - (uint64_t)len) / (count - 1))
        return set_err(MCHECKSUM_GPU_EINVAL, "stride * (count - 1) + len overflows");
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    int width = 0;
    if (gpu_model(hash_method, &width) >= 0 && width == 32 && use_light((uint64_t)len * count, true)) {
        int lg = light_log2g(len);
        DevCtx *c = nullptr;
        const void *pack = nullptr;
        int rc = prologue(hash_method, lg, &width, &c, &pack);
        if (rc) return rc;
        if (count == 0) return MCHECKSUM_GPU_OK;
        // light layout: no more lanes per payload than give every CU about
        // four waves (4096 x 4 KiB: 16 lanes -12% against 64; 1024 x 4 KiB
        // keeps 64, profiles/r04/ab_small_knobs.log)
        const int lg0 = lg;
        if (!lg_forced())
            while (lg > 0 && ((uint64_t)count << (lg - 1)) >= (uint64_t)c->cus * 4 * 64) lg--;
        if (lg != lg0 && (rc = repack(c, hash_method, lg, &pack))) return rc;
        return launch_fixed(c, gpu_model(hash_method, &width), pack, width, lg, dev_base, stride, len, count, dev_out,
                            stream, true);
    }
    int lg = choose_log2g(len, width);
    DevCtx *c = nullptr;
    const void *pack = nullptr;
    int rc = prologue(hash_method, lg, &width, &c, &pack);
    if (rc) return rc;
    if (count == 0) return MCHECKSUM_GPU_OK;
    // a batch too small for the chosen payloads per wave to occupy every wave
    // slot (16 per CU) gets more lanes per payload: 8192 x 4 KiB at 4 lanes
    // ran 2x slower than at 64 (profiles/r04/ab_small_knobs.log)
    const int lg0 = lg;
    if (!lg_forced())
        while (lg < CRC_GPU_MAX_LOG2G && ((count + (64u >> lg) - 1) >> (6 - lg)) < (uint64_t)c->cus * 16) lg++;
    // (the pack for another width only: repack)
    if (lg != lg0 && (rc = repack(c, hash_method, lg, &pack))) return rc;
    return launch_fixed(c, gpu_model(hash_method, &width), pack, width, lg, dev_base, stride, len, count, dev_out,
                        stream, false);
}

int mchecksum_gpu_checksum_offsets(const char *hash_method, const void *dev_base, const uint64_t *dev_offsets,
                                   size_t count, void *dev_out, void *stream) {
    return do_offsets(hash_method, dev_base, dev_offsets, count, dev_out, nullptr, nullptr, nullptr, stream, false);
}

int mchecksum_gpu_verify_offsets(const char *hash_method, const void *dev_base, const uint64_t *dev_offsets,
                                 size_t count, const void *dev_expected, uint8_t *dev_status,
                                 uint32_t *dev_mismatches, void *stream) {
    return do_offsets(hash_method, dev_base, dev_offsets, count, nullptr, dev_expected, dev_status,
                      dev_mismatches, stream, true);
}

int mchecksum_gpu_verify_messages(const char *hash_method, const void *dev_buf, const uint64_t *dev_msg_offsets,
                                  size_t count, size_t payload_offset, size_t hash_offset, uint8_t *dev_status,
                                  uint32_t *dev_mismatches, void *stream) {
    return do_offsets(hash_method, dev_buf, dev_msg_offsets, count, nullptr, nullptr, dev_status, dev_mismatches,
                      stream, true, true, payload_offset, hash_offset);
}

const char *mchecksum_gpu_last_error(void) { return t_err; }

void mchecksum_gpu_reload_settings(void) { mck_settings_reload(); }

int mchecksum_gpu_set_error_word(uint32_t *dev_word) {
    t_err_word = dev_word;
    return MCHECKSUM_GPU_OK;
}

long long mchecksum_gpu_queue_faults(void) {
    if (!mchecksum_gpu_available()) return -1;
    unsigned int n = 0;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_mck_queue_faults), sizeof(n), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    // mchecksum_gpu_ext.hip's kernels (the segment chunk queue) count into
    // their own translation unit's copy of the counter
    const long long ext = ext_queue_faults();
    if (ext < 0) return -1;
    return (long long)n + ext;
}

int mchecksum_gpu_queue_stats(long long *stats, size_t n) {
    if (!stats) return set_err(MCHECKSUM_GPU_EINVAL, "NULL pointer argument");
    if (!mchecksum_gpu_available()) return set_err(MCHECKSUM_GPU_ENODEV, "no HIP device");
    DevCtx *c = nullptr;
    int rc = device_ctx(&c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->pool_mu);
    const long long v[MCHECKSUM_GPU_QSTAT_COUNT] = {c->n_slot, c->n_noslot, c->n_reaped, c->n_busy_skip,
                                                    (long long)c->in_flight.size()};
    for (size_t i = 0; i < n && i < MCHECKSUM_GPU_QSTAT_COUNT; i++) stats[i] = v[i];
    return MCHECKSUM_GPU_OK;
}

#if MCK_TRACE
// Diagnostic builds only: copy the per-wave stamps of the last launch.
MCHECKSUM_PUBLIC int mck_debug_trace_read(void *host, size_t bytes) {
    if (bytes > sizeof(g_mck_trace)) bytes = sizeof(g_mck_trace);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mck_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
// ... the per-wave work-queue timings of the last launch ...
MCHECKSUM_PUBLIC int mck_debug_qwave_read(void *host, size_t bytes) {
    if (bytes > sizeof(g_mck_qwave)) bytes = sizeof(g_mck_qwave);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mck_qwave), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
// ... the per-unit completion stamps of the last launch ...
MCHECKSUM_PUBLIC int mck_debug_units_read(void *host, size_t bytes) {
    if (bytes > sizeof(g_mck_unit_end)) bytes = sizeof(g_mck_unit_end);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mck_unit_end), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
// ... the XCD of each wave of the last launch ...
MCHECKSUM_PUBLIC int mck_debug_trace_xcc_read(void *host, size_t bytes) {
    if (bytes > sizeof(g_mck_trace_xcc)) bytes = sizeof(g_mck_trace_xcc);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mck_trace_xcc), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
// ... the shader-clock stamps (entry, exit) of each wave of the last launch ...
MCHECKSUM_PUBLIC int mck_debug_trace_clk_read(void *host, size_t bytes) {
    if (bytes > sizeof(g_mck_trace_clk)) bytes = sizeof(g_mck_trace_clk);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mck_trace_clk), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
// ... and the work-queue fault records (count, then 4 words per record).
MCHECKSUM_PUBLIC int mck_debug_qdiag_read(unsigned int *n, unsigned long long *rec) {
    if (hipMemcpyFromSymbol(n, HIP_SYMBOL(g_mck_qdiag_n), sizeof(*n), 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(rec, HIP_SYMBOL(g_mck_qdiag), sizeof(g_mck_qdiag), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

}  // extern "C"
