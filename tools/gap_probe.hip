// gap_probe.hip -- the launch boundary of a headline-shaped streaming kernel
// (one 1024-thread workgroup per CU, 140 KiB of LDS, non-temporal 16-B loads
// over 4 GiB), on one stream, by how the launch is made:
//   plain     hipLaunchKernel
//   ext_stop  hipExtLaunchKernel with a stop event (the work-queue slot
//             launches' completion evidence, mchecksum_gpu.hip queue_slot)
//   ext_stop2 the same, alternating two events
//   ext_stop32 the same, 32 events in turn (the slot pool's pattern)
//   rec       hipLaunchKernel, then hipEventRecord
//   ext_nofence  ext_stop with an event made with hipEventDisableSystemFence
//   ext_devrel   ext_stop with an event made with hipEventReleaseToDevice
// Prints the event-timed device time per launch; run it under rocprofv3
// --kernel-trace to read the gaps between dispatches (tools/overlap_probe.py
// --analyze KERNEL_TRACE.csv --kernel read_nt).
// Build: hipcc -O3 --offload-arch=gfx950 tools/gap_probe.hip -o build/gap_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int kLdsWords = 140 * 1024 / 4;

__global__ __launch_bounds__(1024) void read_nt(const uint4 *p, uint64_t n, uint32_t *sink) {
    __shared__ uint32_t lds[kLdsWords];
    for (int i = threadIdx.x; i < kLdsWords; i += 1024) lds[i] = i;
    __syncthreads();
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 1024) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(p + i);
        const uint4 v = make_uint4(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1),
                                   __builtin_nontemporal_load(q + 2), __builtin_nontemporal_load(q + 3));
        acc ^= lds[(v.x ^ v.y ^ v.z ^ v.w) % kLdsWords];
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads alive
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t n = (4ull << 30) / 16;
    uint4 *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, n * 16));
    CK(hipMemset(buf, 1, n * 16));
    CK(hipMalloc(&sink, 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t t0, t1, ev[32], evnf, evdr;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int k = 0; k < 32; k++) CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evnf, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&evdr, hipEventDisableTiming | hipEventReleaseToDevice));
    void *args[] = {&buf, (void *)&n, &sink};
    const char *names[] = {"plain", "ext_stop", "ext_stop2", "ext_stop32", "rec", "ext_nofence", "ext_devrel"};
    const int L = 20;
    for (int rep = 0; rep < 2; rep++) {
        for (int mode = 0; mode < 7; mode++) {
            for (int w = 0; w < 10; w++) hipLaunchKernelGGL(read_nt, dim3(cus), dim3(1024), 0, s, buf, n, sink);
            CK(hipEventRecord(t0, s));
            for (int i = 0; i < L; i++) {
                if (mode == 0 || mode == 4) {
                    hipLaunchKernelGGL(read_nt, dim3(cus), dim3(1024), 0, s, buf, n, sink);
                    if (mode == 4) CK(hipEventRecord(ev[i & 31], s));
                } else {
                    CK(hipExtLaunchKernel((const void *)read_nt, dim3(cus), dim3(1024), args, 0, s, nullptr,
                                          mode == 5 ? evnf : mode == 6 ? evdr : ev[mode == 2 ? i & 1 : mode == 3 ? i & 31 : 0], 0));
                }
            }
            CK(hipEventRecord(t1, s));
            CK(hipStreamSynchronize(s));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            printf("{\"rep\": %d, \"mode\": \"%s\", \"device_us_per_launch\": %.2f}\n", rep, names[mode], ms * 1e3 / L);
        }
    }
    return 0;
}
