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
    // streams seen on the device; launches on one stream never overlap).
    // Graph-captured launches and streams past the table get none and take
    // the static split (crc_gpu_device.h, "Exclusivity").
    unsigned long long *queue = nullptr;
    std::unordered_map<void *, uint32_t> stream_slot;  // guarded by g_mu
};
constexpr uint32_t kStreamSlots = 2048;
constexpr uint32_t kQueueSlots = kStreamSlots;

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
// Work-queue slot for one launch of a throughput (non-light) batch kernel on
// `stream`, exclusive to that stream; nullptr (static split) for a launch
// being captured into a graph or a stream past the table.
unsigned long long *queue_slot(DevCtx *c, void *stream);
// This host thread's fail-closed report word (mchecksum_gpu_set_error_word), or nullptr.
uint32_t *error_word();

}  // namespace mck

#endif  // MCK_GPU_HOST_H
