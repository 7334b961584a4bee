// gpu_host.h -- host-side plumbing shared by the batch-kernel translation
// units (mchecksum_gpu.hip, mchecksum_gpu_ext.hip): per-device table packs,
// error text, launch helpers.  Internal (hidden visibility), not part of the ABI.
#ifndef MCK_GPU_HOST_H
#define MCK_GPU_HOST_H

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <unordered_map>

#include "crc_gpu_device.h"
#include "mchecksum_models.h"

namespace mck {

constexpr int kMaxDev = 64;

constexpr uint32_t kStreamSlots = 2048;
constexpr uint32_t kQueueSlots = kStreamSlots;

// One slot: the work-queue counters (kQSlotWords words in DevCtx::queue),
// owned by one stream at a time.
struct SlotState {
    uintptr_t sid = 0;  // owning stream (handle)
    uint64_t issued_wgs = 0;     // workgroups of the launches handed this slot (each counts its completion, kQDone)
    uint64_t seq = 0;            // launches enqueued on the slot: launch s counts in bank s & 1 (guarded by its launch lock)
    uint64_t last_use = 0;       // LRU tick
    bool owned = false;
};

struct DevCtx {
    bool init = false;
    int cus = 0;
    void *pack[MCK_NMODELS][CRC_GPU_MAX_LOG2G + 1] = {};
    void *ext[MCK_NMODELS] = {};  // mchecksum_gpu_ext.hip's per-model tables
    // Work-queue slots of the batch kernels (WgQueue, crc_gpu_device.h):
    // kQueueSlots zeroed counter sets of two banks each (crc_gpu_device.h):
    // launch s on a slot uses bank s & 1 and zeroes the other for launch s + 1.
    // Eager launches use a slot of their stream's own (keyed by the handle);
    // launches on one stream never overlap.  When all slots are owned, the
    // least recently used slot whose issued workgroups have all completed
    // (kQDone) changes owner.
    // Graph-captured launches, and streams that find no idle slot, get none
    // and take the plain static split (crc_gpu_device.h, "Exclusivity").
    unsigned long long *queue = nullptr;        // 2 * kQBankBytes-aligned view of queue_mem
    void *queue_mem = nullptr;
    SlotState slot[kQueueSlots];               // guarded by g_mu
    std::unordered_map<uintptr_t, uint32_t> sid_slot;  // guarded by g_mu
    uint32_t nslots = 0;                        // slots handed out so far
    uint64_t tick = 0;
    hipStream_t probe = nullptr;                // private stream: reads kQDone words
    unsigned long long *probe_host = nullptr;   // pinned copy of one slot for those reads
    // Launch locks (slot i: launch_mu[i % kLaunchLocks]), held from the bank
    // choice through the kernel's enqueue: two host threads launching on one
    // stream then enqueue in bank order, so the device alternates the banks.
    static constexpr uint32_t kLaunchLocks = 64;
    std::mutex launch_mu[kLaunchLocks];
    // diagnostics (mchecksum_gpu_queue_stats)
    long long n_slot = 0, n_noslot = 0, n_reclaim = 0, n_busy_skip = 0;
};

// A launch's slot bank (counters), the slot's index and the launch's grid;
// holds the slot's launch lock until the launch is enqueued (end of scope)
// or taken back (slot_unissue).
struct SlotRef {
    unsigned long long *q = nullptr;
    int idx = -1;
    uint32_t grid = 0;
    std::unique_lock<std::mutex> lk;
};

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
// Work-queue slot bank for one launch of `grid` workgroups of a throughput
// (non-light) batch kernel on `stream`, exclusive to that stream; empty
// (static split) for a launch being captured into a graph or a stream that
// finds no idle slot.  Every workgroup of a launch given a slot must count
// itself done on it (slot_exit): if the launch fails to start,
// slot_unissue() takes the launch back.  Keep the SlotRef alive until the
// kernel is enqueued: it holds the slot's launch lock.
SlotRef queue_slot(DevCtx *c, void *stream, uint32_t grid);
void slot_unissue(DevCtx *c, SlotRef &r);
// Queue-fault count of mchecksum_gpu_ext.hip's kernels (their own copy of
// g_mck_queue_faults) on the current device; -1 on error.
long long ext_queue_faults();
// This host thread's fail-closed report word (mchecksum_gpu_set_error_word), or nullptr.
uint32_t *error_word();

}  // namespace mck

#endif  // MCK_GPU_HOST_H
