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

struct DevCtx {
    bool init = false;
    int cus = 0;
    void *pack[MCK_NMODELS][CRC_GPU_MAX_LOG2G + 1] = {};
    void *ext[MCK_NMODELS] = {};  // mchecksum_gpu_ext.hip's per-model tables
    // Work-queue slots of the batch kernels (WgQueue, crc_gpu_device.h):
    // kQueueSlots zeroed counter sets; a launch's last group re-zeroes its slot.
    // Eager launches use a slot of their stream's own (the first kStreamSlots
    // streams seen on the device; launches on one stream never overlap).  A
    // launch captured into a hipGraph keeps its slot for every replay: those
    // come round-robin from kCapturedSlots; streams past the table share
    // kOverflowSlots by hash.  Both of those claim the slot on the device
    // (BatchArgs::own) and a launch that finds it owned by another running
    // launch takes the static split (crc_gpu_device.h, "Ownership"), so a
    // collision costs speed, never correctness.
    unsigned long long *queue = nullptr;
    uint32_t queue_captured = 0;
    std::unordered_map<void *, uint32_t> stream_slot;  // guarded by g_mu
};
constexpr uint32_t kStreamSlots = 2048;
constexpr uint32_t kCapturedSlots = 1024;
constexpr uint32_t kOverflowSlots = 1024;
constexpr uint32_t kQueueSlots = kStreamSlots + kCapturedSlots + kOverflowSlots;

extern std::mutex g_mu;

// Record a formatted error for mchecksum_gpu_last_error(); returns rc.
int set_err(int rc, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_err(hipError_t e, const char *what);
// Method -> model index for GPU batch kernels (reflected 32/64-bit): -1 unknown, -2 no kernel.
int gpu_model(const char *method, int *width);
// Current device's context (caller holds g_mu).
int device_ctx(DevCtx **out);
// Model + device context + table pack for lanes-per-payload 2^log2g (takes g_mu).
int prologue(const char *method, int log2g, int *width, DevCtx **c, const void **pack);
// Per-device, per-model extension tables (mchecksum_gpu_ext.hip): the
// Z^n shift pack of a 32/64-bit model, the byte table of a 16-bit one
// (caller holds g_mu).
int get_ext(DevCtx *c, int idx, const void **out);
// Work-queue slot for one launch of a throughput (non-light) batch kernel on
// `stream`; *own = 1 when the launch must claim it on the device.
unsigned long long *queue_slot(DevCtx *c, void *stream, uint32_t *own);

}  // namespace mck

#endif  // MCK_GPU_HOST_H
