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
    // MCK_SLOT_DONE: the launch itself stores the slot's completed-launch count
    // to DevCtx::slot_done[slot] (crc_gpu_device.h, "Completion"), so the slot
    // is idle once that word reaches seq.  Otherwise: an event recorded by the
    // completion of the slot's latest launch (hipExtLaunchKernel stop event).
    hipEvent_t done = nullptr;
    std::atomic<bool> pending{false};  // handed out, launch not yet enqueued (its event not yet recorded)
};

struct DevCtx {
    bool init = false;
    int cus = 0;
    void *pack[MCK_NMODELS][CRC_GPU_MAX_LOG2G + 1] = {};
    void *ext[MCK_NMODELS] = {};  // mchecksum_gpu_ext.hip's per-model tables
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
    unsigned long long *slot_done = nullptr;    // host-mapped, one word per slot (MCK_SLOT_DONE)
    SlotState slot[kQueueSlots];
    uint32_t nslots = kQueueSlots;              // slots in the pool (MCHECKSUM_GPU_QUEUE_SLOTS lowers it for tests)
    std::vector<uint32_t> idle;                 // slots known idle; the most recently reaped on top (guarded by g_mu)
    std::deque<uint32_t> in_flight;             // slots handed out, oldest first (guarded by g_mu)
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
// MCHECKSUM_GPU_QFAULT_MODE ("stall" = 1, "scanstall" = 2, else the give-up
// = 0), in stream order.
static inline void qfault_mode_to_device(hipStream_t s) {
    const char *env = getenv("MCHECKSUM_GPU_QFAULT_MODE");
    static unsigned int modes[3] = {0u, 1u, 2u};  // static: the async copy's source must outlive the call
    const int k = !env ? 0 : strcmp(env, "stall") == 0 ? 1 : strcmp(env, "scanstall") == 0 ? 2 : 0;
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

extern std::mutex g_mu;

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
// Current device's context (caller holds g_mu).
int device_ctx(DevCtx **out);
// Model + device context + table pack for lanes-per-payload 2^log2g (takes g_mu).
int prologue(const char *method, int log2g, int *width, DevCtx **c, const void **pack);
// Per-device, per-model extension tables (mchecksum_gpu_ext.hip): the
// Z^n shift pack of a 32/64-bit model, the byte table of a 16-bit one
// (caller holds g_mu).
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
// Set a translation unit's copy of the slot pool base and completion words
// (g_mck_qbase, g_mck_slot_done) on the current device.
hipError_t ext_set_slot_globals(unsigned long long *qbase, unsigned long long *done_dev);
// This host thread's fail-closed report word (mchecksum_gpu_set_error_word), or nullptr.
uint32_t *error_word();

}  // namespace mck

#endif  // MCK_GPU_HOST_H
