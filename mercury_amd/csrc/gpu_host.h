// gpu_host.h -- host-side plumbing shared by the batch-kernel translation
// units (mchecksum_gpu.hip, mchecksum_gpu_ext.hip): per-device table packs,
// error text, launch helpers.  Internal (hidden visibility), not part of the ABI.
#ifndef MCK_GPU_HOST_H
#define MCK_GPU_HOST_H

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>

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
    // kQueueSlots zeroed counter sets; a launch's last wave re-zeroes its slot.
    // Eager launches take the next slot of a ring of kEagerSlots, so launches
    // that run at the same time (different streams) get different slots unless
    // more than kEagerSlots are in flight at once.  A launch captured into a
    // hipGraph keeps its slot for every replay, so it gets one of its own from
    // the remaining kCapturedSlots, never handed out again.
    unsigned long long *queue = nullptr;
    uint32_t queue_next = 0;
    uint32_t queue_captured = 0;
};
constexpr uint32_t kQueueSlots = 4096;
constexpr uint32_t kCapturedSlots = 1024;
constexpr uint32_t kEagerSlots = kQueueSlots - kCapturedSlots;

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
// Work-queue slot for one launch of a throughput (non-light) batch kernel on
// `stream`; nullptr (error recorded) once a device's captured slots run out.
unsigned long long *queue_slot(DevCtx *c, void *stream);

}  // namespace mck

#endif  // MCK_GPU_HOST_H
