// gpu_host.h -- host-side plumbing shared by the batch-kernel translation
// units (mchecksum_gpu.hip, mchecksum_gpu_ext.hip): per-device table packs,
// error text, launch helpers.  Internal (hidden visibility), not part of the ABI.
#ifndef MCK_GPU_HOST_H
#define MCK_GPU_HOST_H

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <vector>

#include "crc_gpu_device.h"
#include "mchecksum_models.h"

namespace mck {

constexpr int kMaxDev = 64;

constexpr uint32_t kStreamSlots = 2048;
constexpr uint32_t kQueueSlots = kStreamSlots;

// One slot: the work-queue counters (kQSlotWords words in DevCtx::queue),
// held by one launch at a time, from queue_slot() until that launch's
// completion.
struct SlotState {
    uint64_t seq = 0;            // launches enqueued on the slot: launch s counts in bank s & 1
    // recorded by the completion of the slot's latest launch (hipExtLaunchKernel stop event)
    hipEvent_t done = nullptr;
    std::atomic<bool> pending{false};  // handed out, launch not yet enqueued (its event not yet recorded)
};

// Locking: a call takes no lock on its common path.  The context, table packs
// and extension tables are created once under g_mu and published through
// atomics (double-checked); the slot pool has a mutex of its own per device,
// held for the few host-side steps of queue_slot / slot_unissue.
struct DevCtx {
    std::atomic<bool> init{false};
    int cus = 0;
    std::atomic<void *> pack[MCK_NMODELS][CRC_GPU_MAX_LOG2G + 1] = {};
    std::atomic<void *> ext[MCK_NMODELS] = {};  // mchecksum_gpu_ext.hip's per-model tables
    std::mutex pool_mu;                         // the slot pool below
    // Work-queue slots of the batch kernels (WgQueue, crc_gpu_device.h):
    // kQueueSlots zeroed counter sets of two banks each: launch s on a slot
    // uses bank s & 1 and zeroes the other for launch s + 1.  A slot serves one
    // launch at a time: every eager queue launch takes an idle slot from the
    // pool and holds it until its completion records the slot's `done` event
    // (queried without blocking when the slot is reaped back into the pool).
    // No stream owns a slot, so nothing depends on stream handles, their
    // reuse after hipStreamDestroy, or host threads sharing a stream.
    // Graph-captured launches, and launches that find no idle slot, get none
    // and take the plain static split (crc_gpu_device.h, "Exclusivity").
    unsigned long long *queue = nullptr;        // 2 * kQBankBytes-aligned view of queue_mem
    void *queue_mem = nullptr;
    SlotState slot[kQueueSlots];
    uint32_t nslots = kQueueSlots;              // slots in the pool (MCHECKSUM_GPU_QUEUE_SLOTS lowers it for tests)
    std::vector<uint32_t> idle;                 // slots known idle; the most recently reaped on top (pool_mu)
    std::deque<uint32_t> in_flight;             // slots handed out, oldest first (pool_mu)
    // diagnostics (mchecksum_gpu_queue_stats)
    long long n_slot = 0, n_noslot = 0, n_reaped = 0, n_busy_skip = 0;
};

// A launch's slot bank (counters), the slot's index and its completion event.
// The launch must record `done` (launch_kernel's `stop`) and then call
// slot_issued(), or slot_unissue() if the launch call failed.
struct SlotRef {
    unsigned long long *q = nullptr;
    int idx = -1;
    hipEvent_t done = nullptr;
    SlotState *st = nullptr;
};

// Enqueue kernel k on stream s and return THIS launch's status: hipLaunchKernel
// / hipExtLaunchKernel report whether the launch was enqueued, where
// hipGetLastError() would also return an earlier call's sticky error (and a
// slot launch read as failed would be taken back while its kernel runs).
// stop: an event the kernel's completion records (slot launches only; they are
// never captured into graphs).  Arguments are converted to the kernel's
// parameter types before their addresses are taken.
template <class T>
struct Param {
    using type = T;
};
#if MCK_QFAULT_TEST
// Test builds: the injected failure of the next launch (g_mck_qfault_mode,
// crc_gpu_device.h; each translation unit has its own copy) from
// MCHECKSUM_GPU_QFAULT_MODE ("stall" = 1, "scanstall" = 2, "stall+scanstall"
// = 3, else the give-up = 0), in stream order.
static inline void qfault_mode_to_device(hipStream_t s) {
    static unsigned int modes[4] = {0u, 1u, 2u, 3u};  // static: the async copy's source must outlive the call
    const int k = mck_settings()->qfault_mode & 3;
    const unsigned int *m = &modes[k];
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mck_qfault_mode), m, sizeof(*m), 0, hipMemcpyHostToDevice, s);
}
#endif
template <class... P>
hipError_t launch_kernel(void (*k)(P...), dim3 grid, dim3 block, hipStream_t s, hipEvent_t stop,
                         typename Param<P>::type... args) {
    void *argv[] = {static_cast<void *>(&args)...};
#if MCK_QFAULT_TEST
    qfault_mode_to_device(s);
#endif
    if (stop) return hipExtLaunchKernel(reinterpret_cast<const void *>(k), grid, block, argv, 0, s, nullptr, stop, 0);
    return hipLaunchKernel(reinterpret_cast<const void *>(k), grid, block, argv, 0, s);
}

extern std::mutex g_mu;  // creation of contexts and tables only

// Record a formatted error for mchecksum_gpu_last_error(); returns rc.
int set_err(int rc, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_err(hipError_t e, const char *what);
// Method -> model index for GPU batch kernels (32/64-bit): -1 unknown, -2 no kernel.
int gpu_model(const char *method, int *width);
// The kernels' form of catalogue model idx (MSB-first models in the byte-
// reversed register domain, crc_gpu_layout.h), and whether it is MSB-first:
// then the host byte-swaps the outputs after the launch (swap_outputs).
crc_rmodel_t gpu_rmodel(int idx);
bool gpu_msb(int idx);
int swap_outputs(void *dev_out, uint64_t count, int width, void *stream);
// Current device's context, created on first use (takes g_mu then only).
int device_ctx(DevCtx **out);
// Model + device context + table pack for lanes-per-payload 2^log2g (g_mu on creation only).
int prologue(const char *method, int log2g, int *width, DevCtx **c, const void **pack);
// Per-device, per-model extension tables (mchecksum_gpu_ext.hip): the
// Z^n shift pack of a 32/64-bit model, the byte table of a 16-bit one
// (g_mu on creation only).
int get_ext(DevCtx *c, int idx, const void **out);
// Work-queue slot bank for one launch of a throughput (non-light) batch
// kernel on `stream`, exclusive to that launch until it completes; empty
// (static split) for a launch being captured into a graph or when no slot is
// idle.  A launch given a slot passes r.done as launch_kernel's `stop` event,
// then calls slot_issued() -- or slot_unissue() if the launch call failed.
SlotRef queue_slot(DevCtx *c, void *stream);
void slot_issued(SlotRef &r);
void slot_unissue(DevCtx *c, SlotRef &r);
// Queue-fault count of mchecksum_gpu_ext.hip's kernels (their own copy of
// g_mck_queue_faults) on the current device; -1 on error.
long long ext_queue_faults();
// This host thread's fail-closed report word (mchecksum_gpu_set_error_word), or nullptr.
uint32_t *error_word();

}  // namespace mck

#endif  // MCK_GPU_HOST_H
